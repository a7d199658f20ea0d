#!/bin/bash
# Kernel traces of the config-4 (S3D, 256 clips) and config-5 (ResVitKan, 512
# crops) sub-measurements plus per-layer event timings (tools/rvk_layers.py).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_cfg45${PROF_TAG}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 python3 -u $R/tools/rvk_layers.py --model s3d --B 256 > $OUT/s3d_layers.txt 2>&1 || { tail -5 $OUT/s3d_layers.txt; exit 1; }
tail -1 $OUT/s3d_layers.txt
timeout -k 10 200 python3 -u $R/tools/rvk_layers.py --model rvk --B 512 > $OUT/rvk_layers.txt 2>&1 || { tail -5 $OUT/rvk_layers.txt; exit 1; }
tail -1 $OUT/rvk_layers.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/s3d -o run -- python3 $R/bench.py --only s3d --steps 5 --warmup 2 > $OUT/s3d_bench.log 2>&1 || exit $?
echo s3d trace ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rvk -o run -- python3 $R/bench.py --only resvitkan --steps 5 --warmup 2 > $OUT/rvk_bench.log 2>&1 || exit $?
echo rvk trace ok

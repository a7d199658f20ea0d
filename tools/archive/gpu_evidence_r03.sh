#!/bin/bash
# Round-3 evidence pass (TAG, default f): every GPU test, the default bench line, smoke, the
# CViT kernel trace and the config-4/5 traces + per-layer timings.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rA > gpurun_out/pytest_gpu.log 2>&1 || { tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
echo bench ok
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
OUT=$R/gpurun_out/prof_r03${TAG:-f}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp16-line --no-video --no-s3d --no-resvitkan --no-repbn8 > $OUT/trace_bench.log 2>&1 || exit $?
echo cvit trace ok
PROF_TAG=${TAG:-f} bash $R/tools/profile_cfg45_r03.sh

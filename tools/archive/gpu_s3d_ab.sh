#!/bin/bash
# S3D changes: the pool / S3D GPU tests, then config 4 (and 5) same-box A/B of the
# working tree's library against libfac_cvit_base.so, alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 300 --timeout-method thread -k "pool or s3d" > gpurun_out/pytest_s3d.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/pytest_s3d.log | head; tail -3 gpurun_out/pytest_s3d.log; exit 1; }
tail -1 gpurun_out/pytest_s3d.log
for v in base new base new; do
  if [ $v = base ]; then export FAC_CVIT_LIB=$R/fac_fake_amd/libfac_cvit_base.so; else unset FAC_CVIT_LIB; fi
  for w in ${WORKLOADS:-s3d}; do
    timeout -k 10 300 python -u bench.py --only $w --steps 10 --warmup 3 > gpurun_out/ab_${w}_$v.log 2>&1 || { tail -5 gpurun_out/ab_${w}_$v.log; exit 1; }
    echo "$w $v $(tail -1 gpurun_out/ab_${w}_$v.log | cut -c1-330)"
  done
done

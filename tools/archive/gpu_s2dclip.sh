#!/bin/bash
# S3D's first conv with the space-to-depth packing folded in (fac_conv_s2d4_clip):
# its bit-equality test + every S3D test, then config 4 against libfac_cvit_base.so.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 300 --timeout-method thread -k "s2d4 or s3d" > gpurun_out/pytest_s2dc.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pytest_s2dc.log | head -20; tail -3 gpurun_out/pytest_s2dc.log; exit 1; }
tail -1 gpurun_out/pytest_s2dc.log
for rep in 1 2; do for v in base new; do
  if [ $v = base ]; then export FAC_CVIT_LIB=$R/fac_fake_amd/libfac_cvit_base.so; else unset FAC_CVIT_LIB; fi
  timeout -k 10 300 python -u bench.py --only s3d --steps 10 --warmup 3 > gpurun_out/ab_s3d_$v.log 2>&1 || { tail -5 gpurun_out/ab_s3d_$v.log; exit 1; }
  python -c "import json; l=json.loads(open('gpurun_out/ab_s3d_$v.log').read().strip().splitlines()[-1]); r=l.get('conv_pool_layer_roofline',{}); print('s3d $v', l['value'], l['ms_per_step'], r.get('fraction_of_step'), r.get('roofline_ms'))"
done; done

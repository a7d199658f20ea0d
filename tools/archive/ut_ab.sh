#!/bin/bash
# convnd_igemm uniform-tap gather: GPU op tests, then ResVitKan / S3D bench with FAC_CONV_UT=0/1 (twice)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_ut_tests.log 2>&1 || { tail -30 gpurun_out/r03_ut_tests.log; exit 1; }
tail -1 gpurun_out/r03_ut_tests.log
for rep in 1 2; do for ut in 0 1; do for w in resvitkan s3d; do
  FAC_CONV_UT=$ut timeout -k 10 200 python -u bench.py --only $w --steps 10 --warmup 3 > gpurun_out/r03_ut_$w.log 2>&1 || { tail -5 gpurun_out/r03_ut_$w.log; exit 1; }
  python -c "import json; l=json.loads(open('gpurun_out/r03_ut_$w.log').read().strip().splitlines()[-1]); print('ut=$ut $w', l['value'], l['ms_per_step'], l['conv_pool_layer_roofline']['fraction_of_step'])"
done; done; done

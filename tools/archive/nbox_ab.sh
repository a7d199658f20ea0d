#!/bin/bash
# two-box conv3x3 workgroups: GPU parity tests with FAC_CONV_NBOX=2, then the headline bench arms
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
FAC_CONV_NBOX=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/nbox_tests.log 2>&1 || { tail -30 gpurun_out/nbox_tests.log; exit 1; }
tail -1 gpurun_out/nbox_tests.log
for rep in 1 2; do for a in 1 2; do
  FAC_CONV_NBOX=$a timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp16-line --no-video --no-s3d --no-resvitkan --no-repbn8 > gpurun_out/nbox_b.log 2>&1 || { tail -5 gpurun_out/nbox_b.log; exit 1; }
  python -c "import json; l=json.loads(open('gpurun_out/nbox_b.log').read().strip().splitlines()[-1]); print('nbox=$a', l['value'], l['ms_per_step'], {k: v for k, v in l['stage_ms'].items() if k in ('conv7','conv8','conv9','conv10','conv11','conv12','conv13')})"
done; done

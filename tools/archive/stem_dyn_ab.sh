#!/bin/bash
# Stem phase stamps (static schedule), then the CViT bench with stem_dynamic 0 / 1, same box, twice;
# fused-stem parity tests first.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "fused_stem or conv1_fused or golden or b256 or real_crops or graph or pipelined" > gpurun_out/stemdyn_tests.log 2>&1 || { tail -30 gpurun_out/stemdyn_tests.log; exit 1; }
tail -1 gpurun_out/stemdyn_tests.log
timeout -k 5 60 tools/ubench/bin/stem_ubench_base | grep -E "stem224|wg 0|fetch:|conv2 / conv3" | head -4
for rep in 1 2; do for v in 1 0; do
  timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-fp16-line --no-video --no-s3d --no-resvitkan --no-repbn8 --no-cpu-baseline --opt stem_dynamic=$v > gpurun_out/stemdyn_$v.log 2>&1 || { tail -5 gpurun_out/stemdyn_$v.log; exit 1; }
  python -c "import json,sys; l=json.loads(open('gpurun_out/stemdyn_$v.log').read().strip().splitlines()[-1]); print('dyn$v', l['value'], l['ms_per_step'], l['roofline']['launch_ms'], l['roofline']['launch_ms_sync_profile'], l['roofline']['frac'], l['parity']['max_abs_dprob'])"
done; done

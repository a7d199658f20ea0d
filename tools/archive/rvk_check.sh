#!/bin/bash
# ResVitKan GPU parity tests (+ the op tests), per-layer timings (512 crops) and the config-5 bench line.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
T=${TAG:-x}
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread > gpurun_out/rvkc_tests_$T.log 2>&1 || { tail -30 gpurun_out/rvkc_tests_$T.log; exit 1; }
tail -1 gpurun_out/rvkc_tests_$T.log
timeout -k 10 200 python3 -u tools/rvk_layers.py --model rvk --B 512 > gpurun_out/rvkc_layers_$T.txt 2>&1 || { tail -5 gpurun_out/rvkc_layers_$T.txt; exit 1; }
grep -E "^1x1x1/11 (64->256|256->128|128->512|512->128|256->1024|64->64|256->64) " gpurun_out/rvkc_layers_$T.txt | sort | uniq -c | head; tail -1 gpurun_out/rvkc_layers_$T.txt
timeout -k 10 200 python -u bench.py --only resvitkan --steps 10 --warmup 3 > gpurun_out/rvkc_bench_$T.log 2>&1 || { tail -5 gpurun_out/rvkc_bench_$T.log; exit 1; }
python -c "import json; l=json.loads(open('gpurun_out/rvkc_bench_$T.log').read().strip().splitlines()[-1]); print('rvk', l['value'], l['ms_per_step'], l['conv_pool_layer_roofline']['fraction_of_step'])"

# branch-free pack_input_s2d: op tests, then the config-5 trace's pack_input_s2d mean (was 517 us at 3072 crops)
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py tests/test_gpu_parity.py > gpurun_out/pack_pytest.log 2>&1 || { tail -30 gpurun_out/pack_pytest.log; exit 1; }
tail -2 gpurun_out/pack_pytest.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/packtr -o run -- python3 bench.py --only resvitkan --steps 5 --warmup 2 > gpurun_out/packtr.log 2>&1
grep -h "pack_input_s2d\|conv_s2d4_mp" gpurun_out/packtr/run_kernel_stats.csv | cut -c1-200
tail -1 gpurun_out/packtr.log | cut -c1-300

timeout -k 10 600 python -u -m pytest tests/test_repbn8.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_rb8.log 2>&1; rc=$?; tail -5 gpurun_out/t_rb8.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --only repbn8 --steps 10 --warmup 3 > gpurun_out/b_rb8.log 2>&1; rc=$?; tail -2 gpurun_out/b_rb8.log; exit $rc

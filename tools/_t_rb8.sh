timeout -k 10 600 python -u -m pytest tests/test_repbn8.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/t_rb8.log 2>&1; rc=$?; tail -15 gpurun_out/t_rb8.log; exit $rc

#!/bin/bash
# GPU-box script: parity tests, then (if nothing crashed) a short bench.
mkdir -p gpurun_out
rocminfo 2>/dev/null | grep -m2 -E "gfx9" > gpurun_out/arch.txt
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -rA > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/pytest_gpu.log
if [ $rc -le 1 ]; then
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
  brc=$?
  echo "bench rc=$brc"
  tail -3 gpurun_out/bench.log
  exit $brc
fi
exit $rc

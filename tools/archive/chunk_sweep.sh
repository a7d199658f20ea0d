mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1 || { echo "tests failed rc=$?"; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for c in 0 32 64 128; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --stem-chunk $c > gpurun_out/chunk_$c.log 2>&1 || exit $?
  echo "chunk $c: $(tail -1 gpurun_out/chunk_$c.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stage_ms"]; print(d["value"], d["ms_per_step"], [round(s[k],3) for k in ("conv1","conv4","conv5","conv6","conv7","conv8","conv9")])')"
done

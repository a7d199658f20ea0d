#!/bin/bash
# ResVitKan throughput vs the ResNet stem's crop chunk (bench.py --only resvitkan)
for ch in 256 128 64 32; do
  timeout -k 10 300 python bench.py --only resvitkan --steps 10 --warmup 3 --stem-chunk $ch > gpurun_out/rvk_$ch.log 2>&1 || { tail -5 gpurun_out/rvk_$ch.log; exit 1; }
  tail -1 gpurun_out/rvk_$ch.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($ch, d['value'], d['ms_per_step'])"
done

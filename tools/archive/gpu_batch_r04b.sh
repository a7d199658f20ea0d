# late round-4 per-GPU batch sweep, larger batches (configs 4/5), two alternations
set -e
mkdir -p gpurun_out
rm -f gpurun_out/batch_r04b.txt
for rep in 1 2; do
for b in 768 1024 1536; do
  timeout -k 10 240 python -u bench.py --only s3d --steps 10 --warmup 3 --s3d-batch $b > gpurun_out/s3d_b$b.txt 2>&1
  tail -1 gpurun_out/s3d_b$b.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('config4',d); print('s3d $b', c.get('value'), c.get('conv_pool_layer_roofline',{}).get('fraction_of_step'))" >> gpurun_out/batch_r04b.txt
done
for b in 1536 2048 3072; do
  timeout -k 10 240 python -u bench.py --only resvitkan --steps 8 --warmup 3 --rvk-batch $b > gpurun_out/rvk_b$b.txt 2>&1
  tail -1 gpurun_out/rvk_b$b.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('config5',d); print('rvk $b', c.get('value'), c.get('conv_pool_layer_roofline',{}).get('fraction_of_step'))" >> gpurun_out/batch_r04b.txt
done
done
cat gpurun_out/batch_r04b.txt

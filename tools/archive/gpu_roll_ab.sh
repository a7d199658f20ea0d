# maxpool3_roll for the 4x7x7 Inception pools: pool / S3D GPU tests, per-call
# timing, then config-4 A/B of pool_roll (0 = maxpool3_s1) in one box
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py \
  -k "pool or s3d" > gpurun_out/roll_pytest.log 2>&1 || { tail -30 gpurun_out/roll_pytest.log; exit 1; }
tail -2 gpurun_out/roll_pytest.log
timeout -k 10 200 python -u tools/pool_roll_ab.py --B 384 --arms 0,1 > gpurun_out/pool_roll2.txt 2>&1
cat gpurun_out/pool_roll2.txt
rm -f gpurun_out/s3d_roll_ab.txt
for v in 0 1 0 1 0 1; do
  timeout -k 10 240 python -u bench.py --only s3d --steps 20 --warmup 5 --opt pool_roll=$v > gpurun_out/s3d_roll_$v.txt 2>&1
  tail -1 gpurun_out/s3d_roll_$v.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('config4',d); print('$v', c.get('value'), c.get('conv_pool_layer_roofline',{}).get('fraction_of_step'))" >> gpurun_out/s3d_roll_ab.txt
done
cat gpurun_out/s3d_roll_ab.txt

# convnd_pt column segments (S3D merged heads at 14x14): conv / S3D GPU tests,
# then config-4 A/B of nd_pt_wide (0 = igemm) in one box, three alternations
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py \
  -k "conv_nd or s3d or split" > gpurun_out/ndpt2_pytest.log 2>&1 || { tail -30 gpurun_out/ndpt2_pytest.log; exit 1; }
tail -3 gpurun_out/ndpt2_pytest.log
rm -f gpurun_out/s3d_pt_ab2.txt
for v in 0 1024 0 1024 0 1024; do
  timeout -k 10 240 python -u bench.py --only s3d --steps 20 --warmup 5 --opt nd_pt_wide=$v > gpurun_out/s3d_pt_$v.txt 2>&1
  tail -1 gpurun_out/s3d_pt_$v.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('config4',d); print('$v', c.get('value'), c.get('conv_pool_layer_roofline',{}).get('fraction_of_step'))" >> gpurun_out/s3d_pt_ab2.txt
done
cat gpurun_out/s3d_pt_ab2.txt

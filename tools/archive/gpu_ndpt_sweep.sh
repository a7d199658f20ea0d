# config-4 (S3D) clips/s against the nd_pt_wide row-tile threshold, two alternations, one box
set -e
mkdir -p gpurun_out
rm -f gpurun_out/s3d_pt_sweep.txt
for rep in 1 2; do
for v in 0 1 64 128 256 512; do
  timeout -k 10 240 python -u bench.py --only s3d --steps 20 --warmup 5 --opt nd_pt_wide=$v > gpurun_out/s3d_pt_$v.txt 2>&1
  tail -1 gpurun_out/s3d_pt_$v.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('config4',d); print('$v', c.get('value'), c.get('conv_pool_layer_roofline',{}).get('fraction_of_step'))" >> gpurun_out/s3d_pt_sweep.txt
done
done
for v in 0 256; do
  timeout -k 10 240 python -u bench.py --only resvitkan --steps 20 --warmup 5 --opt nd_pt_wide=$v > gpurun_out/rvk_pt_$v.txt 2>&1
  tail -1 gpurun_out/rvk_pt_$v.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('config5',d); print('rvk $v', c.get('value'), c.get('conv_pool_layer_roofline',{}).get('fraction_of_step'))" >> gpurun_out/s3d_pt_sweep.txt
done
cat gpurun_out/s3d_pt_sweep.txt

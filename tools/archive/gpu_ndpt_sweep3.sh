# config 4 at the default batch against the nd_pt_wide row-tile threshold (256 / 64 / 32), two alternations
set -e
mkdir -p gpurun_out
rm -f gpurun_out/s3d_pt_sweep3.txt
for rep in 1 2; do
for v in 256 64 32; do
  timeout -k 10 240 python -u bench.py --only s3d --steps 8 --warmup 3 --opt nd_pt_wide=$v > gpurun_out/s3d_ptw_$v.txt 2>&1
  tail -1 gpurun_out/s3d_ptw_$v.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('config4',d); print('$v', c.get('value'), c.get('conv_pool_layer_roofline',{}).get('fraction_of_step'))" >> gpurun_out/s3d_pt_sweep3.txt
done
done
cat gpurun_out/s3d_pt_sweep3.txt

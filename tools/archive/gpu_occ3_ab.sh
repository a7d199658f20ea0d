# convnd_igemm 3-per-CU tile for narrow convs (nd_occ3 0 / 4 / 8): config-4 A/B at the default batch
set -e
mkdir -p gpurun_out
rm -f gpurun_out/s3d_occ3_ab.txt
for v in 0 4 8 0 4 8; do
  timeout -k 10 240 python -u bench.py --only s3d --steps 10 --warmup 3 --opt nd_occ3=$v > gpurun_out/s3d_occ3_$v.txt 2>&1
  tail -1 gpurun_out/s3d_occ3_$v.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('config4',d); print('$v', c.get('value'), c.get('conv_pool_layer_roofline',{}).get('fraction_of_step'))" >> gpurun_out/s3d_occ3_ab.txt
done
cat gpurun_out/s3d_occ3_ab.txt

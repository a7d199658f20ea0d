# config 2 (pipelined CViT) against the fused stem's persistent workgroup count (stem_nwg; 0 = one per CU)
set -e
mkdir -p gpurun_out
rm -f gpurun_out/stemnwg_ab.txt
for rep in 1 2; do
for v in 0 240 224 208; do
  timeout -k 10 240 python -u bench.py --no-video --no-resvitkan --no-s3d --no-repbn8 --no-fp16-line --no-cpu-baseline --opt stem_nwg=$v > gpurun_out/stemnwg_$v.txt 2>&1
  tail -1 gpurun_out/stemnwg_$v.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], d['roofline']['launch_ms'])" >> gpurun_out/stemnwg_ab.txt
done
done
cat gpurun_out/stemnwg_ab.txt

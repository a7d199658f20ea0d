#!/bin/bash
# Same-box A/B of a fac_set_option knob: per-layer bit-equality + time
# (tools/db_ab.py), then the bench line per arm.
#   KEY=conv_tr ARMS=0,1 LAYERS=3,4,5 bash tools/gpu_ab.sh
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
KEY=${KEY:-conv_tr}; ARMS=${ARMS:-0,1}; LAYERS=${LAYERS:-3,4,5,6,7,8,13,14,15,16}
timeout -k 10 300 python -u tools/db_ab.py --dtype ${DT:-bf16} --key $KEY --arms $ARMS --layers $LAYERS > gpurun_out/ab_$KEY.log 2>&1 || { tail -20 gpurun_out/ab_$KEY.log; exit 1; }
cat gpurun_out/ab_$KEY.log
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp16-line --no-video --no-resvitkan --no-s3d --no-repbn8"
for rep in 1 2; do for arm in ${ARMS//,/ }; do
  timeout -k 10 300 $B --opt $KEY=$arm > gpurun_out/b_${KEY}_$arm.log 2>&1 || { tail -5 gpurun_out/b_${KEY}_$arm.log; exit 1; }
  echo "$KEY=$arm: $(tail -1 gpurun_out/b_${KEY}_$arm.log | cut -c90-160)"
done; done

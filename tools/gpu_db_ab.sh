#!/bin/bash
# Same-box A/B of conv3x3_db (fac_set_option "conv_db") against conv3x3_bn_relu:
# per-layer bit-equality + time (tools/db_ab.py), then the bench line per arm.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/db_ab.py --dtype bf16 --arms 0,7,11 --layers 6,7,8,9,10,11,12,13,14,15,16 > gpurun_out/db_ab_bf16.log 2>&1 || { tail -20 gpurun_out/db_ab_bf16.log; exit 1; }
cat gpurun_out/db_ab_bf16.log
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp16-line --no-video --no-resvitkan --no-s3d --no-repbn8"
for arm in 0 ${DB_ARMS:-7 11}; do
  timeout -k 10 300 $B --opt conv_db=$arm > gpurun_out/b$arm.log 2>&1 || { tail -5 gpurun_out/b$arm.log; exit 1; }
  echo "arm $arm: $(tail -1 gpurun_out/b$arm.log | cut -c1-200)"
done

#!/bin/bash
# conv4-6 chunk-planar activations: parity tests, same-box A/B of the arms, FETCH_SIZE per 112^2 kernel
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
R=$(pwd)
mkdir -p gpurun_out
ARMS="conv112_cpl=0;conv112_cpl=1" DTYPES="fp16 bf16" REPS=${REPS:-2} TESTK="conv112 or each_conv or b256_config2 or c1_single or b32_all or few_crop or stem_chunking or pipelined" bash tools/ab_bench.sh || exit 1
export TMPDIR=/tmp
for v in 0 1; do
  (cd /tmp && timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/cpl_fetch_$v -o run -- python3 $R/bench.py --steps 5 --warmup 2 --dtype bf16 --no-cpu-baseline --no-fp16-line --no-video --no-s3d --no-resvitkan --no-repbn8 --opt conv112_cpl=$v > $R/gpurun_out/cpl_fetch_$v.log 2>&1) || { tail -5 gpurun_out/cpl_fetch_$v.log; exit 1; }
done
python - <<'PY'
import csv, glob, collections
for v in (0, 1):
    f = glob.glob(f'gpurun_out/cpl_fetch_{v}/**/*counter_collection.csv', recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        n = r.get('Kernel_Name', '')
        if 'conv3x3_bn_relu' in n and '16, 16, 64' in n and r.get('Counter_Name') == 'FETCH_SIZE':
            acc[n.split('(')[0]].append(float(r['Counter_Value']))
    for n, xs in acc.items():
        print('conv112_cpl=%d %-95s n=%d FETCH_SIZE mean (raw KiB) %.0f' % (v, n[:95], len(xs), sum(xs) / len(xs)))
PY

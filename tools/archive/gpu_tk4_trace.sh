#!/bin/bash
# kernel traces of eager S3D forwards with the (3,1,1) convs on the 4-frame (tk2_zw4=7) / 2-frame (0) waves
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in 7 0; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/tk4tr_$v -o run -- python3 tools/s3d_eager.py --B ${B:-384} --u8 --opt tk2_zw4=$v > gpurun_out/tk4tr_$v.log 2>&1 || { tail -5 gpurun_out/tk4tr_$v.log; exit 1; }
done
python - <<'PY'
import sqlite3, glob
for v in (7, 0):
    db = glob.glob(f'gpurun_out/tk4tr_{v}/**/*.db', recursive=True)[0]
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), avg(duration) from kernels where name like '%conv_tk2%' group by name").fetchall()
    tot = c.execute("select sum(duration) from kernels").fetchone()[0]
    print('tk2_zw4=%d total %.3f ms' % (v, tot / 1e6))
    for r in rows:
        print('   %-90s %4d %8.1f us' % (r[0][:90], r[1], r[2] / 1e3))
PY

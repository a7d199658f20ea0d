#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "s3d" > gpurun_out/b0_pytest.log 2>&1 || { tail -30 gpurun_out/b0_pytest.log; exit 1; }
tail -1 gpurun_out/b0_pytest.log
B=384 bash tools/gpu_s3d_trace.sh || exit 1
python - <<'PY'
import sqlite3
for arm in ('fused','two'):
    c=sqlite3.connect(f'gpurun_out/s3dtr_{arm}/run_results.db')
    rows=c.execute("select name, count(*), avg(duration) from kernels where name like '%s3d_base0%' or name like '%conv_s2d4%' or name like '%conv_tk2<fac::BF16, 2, 7%' group by name").fetchall()
    tot=c.execute("select sum(duration) from kernels").fetchone()[0]
    print(arm, 'total ms %.3f' % (tot/1e6), ['%s %d %.1f us' % (r[0][:40], r[1], r[2]/1e3) for r in rows])
PY
hipcc --offload-arch=gfx950 -O3 -std=c++17 -DB0_STAMPS -I fac_fake_amd/csrc -I include -o gpurun_out/b0_ubench tools/ubench/b0_ubench.hip > gpurun_out/b0_build.log 2>&1 || { tail -5 gpurun_out/b0_build.log; exit 1; }
timeout -k 10 120 gpurun_out/b0_ubench

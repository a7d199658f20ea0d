#!/bin/bash
# Round-end evidence on one GPU box: every GPU test, the default bench line,
# smoke, then rocprofv3 traces of the config-4/5/RepBn8 sub-measurements.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rA > gpurun_out/pytest_gpu.log 2>&1 || { tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
export TMPDIR=/tmp
cd /tmp
for w in resvitkan s3d repbn8; do
  mkdir -p $R/gpurun_out/prof_$w
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$w/trace -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --only $w > $R/gpurun_out/prof_$w/trace_bench.log 2>&1 || exit $?
  echo $w ok
done

#!/bin/bash
# Round-6 evidence pass (second session, after the S3D / ResVitKan fusions): every GPU test, smoke, the default bench line, the
# reference-mode latency breakdown (PROFILE=1: then the headline profile
# passes, PMC=1: and the configs-4/5 PMC passes).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rA > gpurun_out/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -20; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-300
timeout -k 10 240 python -u tools/ref_latency.py > gpurun_out/ref_latency.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ref_latency.txt | tail -4
if [ -n "$PROFILE" ]; then PROF_TAG=${PROF_TAG:-a} bash tools/profile_r06.sh || exit 1; fi
if [ -n "$PMC" ]; then PROF_TAG=${PROF_TAG:-a} bash tools/pmc_cfg45.sh || exit 1; fi
echo pass ok

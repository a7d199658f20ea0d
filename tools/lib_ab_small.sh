#!/bin/bash
# Same-box A/B of the in-tree library against PREV (FAC_CVIT_LIB) on the B-crop
# graph forward (tools/small_b_trace.py --graph), alternating, REPS rounds.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
if [ -n "$TESTK" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$TESTK" > gpurun_out/labs_pytest.log 2>&1 || { tail -30 gpurun_out/labs_pytest.log; exit 1; }
  tail -1 gpurun_out/labs_pytest.log
fi
for rep in $(seq 1 ${REPS:-3}); do
  for arm in prev cur; do
    if [ $arm = prev ]; then export FAC_CVIT_LIB=$PREV; else unset FAC_CVIT_LIB; fi
    for b in ${BS:-29}; do
      echo -n "$arm "; timeout -k 10 120 python -u tools/small_b_trace.py --graph --batch $b --reps 300 --warmup 200 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
    done
  done
done
unset FAC_CVIT_LIB

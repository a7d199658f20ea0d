#!/bin/bash
# Round 6: packed conv epilogue (bit-identity + per-layer times vs the
# round-5 lib), and the few-row GEMMs' hot/cold weight-stream times.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "isolated or golden or small14 or ring9 or few_crop" > gpurun_out/b_pytest.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/b_pytest.log | head -20; tail -5 gpurun_out/b_pytest.log; exit 1; }
tail -1 gpurun_out/b_pytest.log
timeout -k 10 200 python -u tools/gemm_l2.py --dtype fp16 > gpurun_out/gemm_l2.txt 2>&1 || { tail -5 gpurun_out/gemm_l2.txt; exit 1; }
grep -v "^{" gpurun_out/gemm_l2.txt | grep -v amdgpu
for rep in 1 2; do
for arm in prev cur; do
  if [ $arm = prev ]; then export FAC_CVIT_LIB=ab/libfac_cvit_r05.so; else unset FAC_CVIT_LIB; fi
  timeout -k 10 200 python -u tools/conv_sweep.py --dtype fp16 --tag "$arm" > gpurun_out/ep_${arm}.txt 2>&1 || { tail -5 gpurun_out/ep_${arm}.txt; exit 1; }
  tail -1 gpurun_out/ep_${arm}.txt
done; done
unset FAC_CVIT_LIB

#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/blas_probe.py 1024 2>&1 | grep -v amdgpu.ids | tee gpurun_out/blas_probe.log

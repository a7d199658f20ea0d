#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
for l in 0 1 2 3; do timeout -k 10 60 tools/ubench/bin/nd_ubench $l > gpurun_out/nd_$l.log 2>&1 || { tail -5 gpurun_out/nd_$l.log; exit 1; }; done
cat gpurun_out/nd_0.log gpurun_out/nd_1.log | grep -v amdgpu.ids

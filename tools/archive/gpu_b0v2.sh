#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
PREV=ab/libfac_cvit_head.so ONLY=s3d REPS=${REPS:-2} TESTK=s3d bash tools/lib_ab.sh || exit 1
hipcc --offload-arch=gfx950 -O3 -std=c++17 -DB0_STAMPS -I fac_fake_amd/csrc -I include -o gpurun_out/b0_ubench tools/ubench/b0_ubench.hip > gpurun_out/b0_build.log 2>&1 || { tail -5 gpurun_out/b0_build.log; exit 1; }
timeout -k 10 120 gpurun_out/b0_ubench

#!/bin/bash
# kernel traces of eager S3D forwards (uint8 clips), base.0 fused vs two launches
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for arm in fused two; do
  extra=""; [ $arm = two ] && extra="--no-fuse"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/s3dtr_$arm -o run -- python3 tools/s3d_eager.py --B ${B:-384} --u8 $extra > gpurun_out/s3dtr_$arm.log 2>&1 || { tail -5 gpurun_out/s3dtr_$arm.log; exit 1; }
done
echo ok

# uint8 S3D clips (fac_conv_s2d4_clip_u8): s2d / S3D GPU tests, then fp32 vs uint8 input A/B
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py \
  -k "s2d4 or s3d" > gpurun_out/u8_pytest.log 2>&1 || { tail -30 gpurun_out/u8_pytest.log; exit 1; }
tail -2 gpurun_out/u8_pytest.log
timeout -k 10 300 python -u tools/s3d_input_ab.py --B 384 > gpurun_out/s3d_u8_ab.txt 2>&1
cat gpurun_out/s3d_u8_ab.txt

mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -m gpu -x -k "fused_stem224 or c1_single or b256" > gpurun_out/ab_test.log 2>&1; echo "testA rc=$?"
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/benchA.log 2>&1; echo "benchA rc=$?"
FAC_CVIT_LIB=$PWD/fac_fake_amd/libfac_cvit_B.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/benchB.log 2>&1; echo "benchB rc=$?"

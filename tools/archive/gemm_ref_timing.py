"""Reference timing of torch.matmul (hipBLASLt) on the ResNet-50 1x1-conv GEMM
shapes of ResVitKan at B=256 (M = pixels, N = Cout, K = Cin), bf16: what a
library GEMM reaches on these shapes, for comparison with fac_conv_nd.
GPU box only."""
import torch

shapes = [(802816, 256, 64), (802816, 64, 256), (802816, 128, 256), (200704, 512, 128), (200704, 128, 512),
          (200704, 256, 512), (50176, 1024, 256), (50176, 256, 1024), (50176, 512, 1024), (12544, 2048, 512),
          (12544, 512, 2048), (12544, 2048, 1024)]
dev = torch.device("cuda:0")
for M, N, K in shapes:
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        c = a @ w.t()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(10):
        e0.record()
        c = a @ w.t()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ms = sorted(ts)[5]
    print(f"M {M:7d} N {N:5d} K {K:5d}: {ms * 1e3:7.1f} us  {2 * M * N * K / ms / 1e9:7.1f} TF/s  "
          f"{2 * (M * K + N * K + M * N) / ms / 1e6:6.0f} GB/s", flush=True)

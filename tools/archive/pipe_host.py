"""Host-side view of the pipelined bench loop: how long each
fac_forward_nhwc_u8_pipelined call blocks the host, and how far ahead of the
GPU the host runs (GPU box: python tools/pipe_host.py)."""
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from fac_fake_amd.weights import make_crops, make_state_dict  # noqa: E402
from fac_fake_amd import _lib  # noqa: E402
from fac_fake_amd.cvit import CViT  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    B = 256
    lib = _lib.load()
    model = CViT(dtype="bf16")
    model.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in make_state_dict(0).items()})
    model.to(dev)
    model.reserve(B, dev)
    ctx = model._ctx
    crops = torch.from_numpy(make_crops(B, seed=3)).to(dev)
    pidx = (torch.arange(B, device=dev) % 32).to(torch.int32)
    lgs = [torch.empty(B, 2, dtype=torch.float32, device=dev) for _ in range(2)]
    score = torch.empty((), dtype=torch.float32, device=dev)
    stream = torch.cuda.Stream(dev)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    for rep in range(2):
        host = []
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        ev[0].record(stream)
        for k in range(n):
            a = time.perf_counter()
            _lib.check(lib.fac_forward_nhwc_u8_pipelined(ctx, crops.data_ptr(), B, pidx.data_ptr(), lgs[k & 1].data_ptr(),
                                                         None, score.data_ptr(), stream.cuda_stream), ctx, "pipelined")
            host.append(time.perf_counter() - a)
            ev[k + 1].record(stream)  # end of batch k's conv stack on the main stream
        t_enq = time.perf_counter() - t0
        _lib.check(lib.fac_pipeline_join(ctx, 0, stream.cuda_stream), ctx, "join")
        torch.cuda.synchronize(dev)
        total = time.perf_counter() - t0
        conv = [ev[k].elapsed_time(ev[k + 1]) for k in range(n)]
        print(f"rep {rep}: {n} steps {total * 1e3:.2f} ms ({total / n * 1e3:.3f} ms/step), host enqueue "
              f"{t_enq * 1e3:.2f} ms; per call host ms mean {np.mean(host) * 1e3:.3f} max {np.max(host) * 1e3:.3f}; "
              f"main-stream step ms: {' '.join(f'{c:.2f}' for c in conv[:12])}", flush=True)


if __name__ == "__main__":
    main()

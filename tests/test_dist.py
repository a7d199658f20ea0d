"""Multi-rank path on CPU (gloo, world_size 2 and 3): frame sharding + the one
logit all-gather reproduce the single-process video score bit-for-bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, logits, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fac_fake_amd.prediction import pre_process_prediction, pred_sig
        from fac_fake_amd.sharding import gather_logits, shard_bounds
        n = logits.shape[0]
        lo, hi = shard_bounds(n, world, rank)
        local = torch.from_numpy(logits[lo:hi].copy())     # this rank's per-crop logits
        full = gather_logits(local, n)
        score = float(pre_process_prediction(pred_sig(full))) if n else 0.5
        q.put((rank, full.numpy(), score))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 40), (2, 3), (3, 300), (2, 1)])
def test_sharded_gather_matches_single_process(golden, world, n):
    from oracle import postproc
    base = golden("golden_chunks.npz")["logits"].astype(np.float32)
    logits = np.resize(base, (n, 2)).astype(np.float32)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, logits, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = postproc.video_score(logits)
    for rank, full, score in res:
        assert np.array_equal(full, logits)
        assert score == pytest.approx(want, abs=1e-7)

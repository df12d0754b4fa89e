"""IT-column sharding of the static matrix on CPU ranks (gloo, world size 2
and 3, uneven word slices): the all-gather / SUM / MIN combination of gpusched.feasibility.combine over
synthetic shard results equals the unsharded matrix (the GPU side is
tests/test_gpu_parity.py::test_feasibility_shards_combine_to_whole)."""
import os
import socket

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

from gpusched.feasibility import combine, word_range


def _whole(seed=5, P=40, T=2, W=7, N=7 * 64 - 5):
    rng = np.random.default_rng(seed)
    rows = rng.integers(0, 2**63, size=(P, T, W), dtype=np.int64).view(np.uint64)
    rows[:, :, -1] &= np.uint64((1 << (N - 64 * (W - 1))) - 1)
    name_rank = rng.permutation(N).astype(np.uint32)
    price = rng.integers(0, 1000, size=N)
    keys = np.full((P, T), 2**64 - 1, dtype=np.uint64)
    nfo = np.zeros((P, T), dtype=np.uint32)
    return rows, name_rank, price, keys, nfo


def _shard(rows, name_rank, price, r, world):
    P, T, W = rows.shape
    wb, we = word_range(W, r, world)
    part = np.zeros_like(rows)
    part[:, :, wb:we] = rows[:, :, wb:we]
    keys = np.full((P, T), 2**64 - 1, dtype=np.uint64)
    nfo = np.zeros((P, T), dtype=np.uint32)
    for p in range(P):
        for t in range(T):
            its = [w * 64 + b for w in range(wb, we) for b in range(64) if (int(part[p, t, w]) >> b) & 1]
            nfo[p, t] = len(its)
            if its:
                keys[p, t] = min((int(price[i]) << 32) | int(name_rank[i]) for i in its)
    return part, nfo, keys


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rows, name_rank, price, _, _ = _whole()
        part, nfo, keys = _shard(rows, name_rank, price, rank, world)
        out = combine(part, nfo, keys, name_rank, rank, world, dist)
        q.put((rank, {k: v.tolist() for k, v in out.items()}))
    finally:
        dist.destroy_process_group()


import pytest  # noqa: E402


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_feasibility_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p_ in procs:
        p_.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p_ in procs:
        p_.join(timeout=60)
        assert p_.exitcode == 0
    rows, name_rank, price, _, _ = _whole()
    full, nfo, keys = _shard(rows, name_rank, price, 0, 1)
    want = combine(full, nfo, keys, name_rank, 0, 1, None)
    for r in range(world):
        for k in ("rows", "n_feasible_offerings", "cheapest", "cheapest_key"):
            assert np.array_equal(np.asarray(res[r][k], dtype=want[k].dtype), want[k]), (r, k)

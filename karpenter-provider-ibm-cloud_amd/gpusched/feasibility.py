"""The static pod x offering feasibility matrix sharded by instance-type
columns over GPUs (BASELINE north_star: "offering columns per
GPU with an RCCL all-reduce (min-price/index) over xGMI").

Rank r evaluates instance-type words [W*r/N, W*(r+1)/N) with
gs_feasibility_shard; the shards combine exactly:
  rows        integer SUM all-reduce (each word is non-zero on one rank only,
              so the sum is the bitwise OR),
  offerings   SUM all-reduce,
  cheapest    MIN all-reduce of the OrderByPrice key (price_rank << 32 |
              name_rank), mapped back to the type through its name rank.
"""
import numpy as np

NONE_KEY = np.iinfo(np.int64).max


def word_range(words, rank, world):
    return words * rank // world, words * (rank + 1) // world


def combine(rows, nfo, keys, name_rank, rank, world, dist, device=None):
    """all-reduce one rank's shard result into the full matrix (every rank)"""
    keys = np.where(keys == np.uint64(2**64 - 1), NONE_KEY, keys.astype(np.int64))
    if world > 1:
        import torch
        t_rows = torch.from_numpy(rows.view(np.int64).copy())
        t_nfo = torch.from_numpy(nfo.astype(np.int64))
        t_key = torch.from_numpy(keys.copy())
        if device is not None:
            t_rows, t_nfo, t_key = t_rows.to(device), t_nfo.to(device), t_key.to(device)
        dist.all_reduce(t_rows, op=dist.ReduceOp.SUM)
        dist.all_reduce(t_nfo, op=dist.ReduceOp.SUM)
        dist.all_reduce(t_key, op=dist.ReduceOp.MIN)
        rows = t_rows.cpu().numpy().view(np.uint64)
        nfo = t_nfo.cpu().numpy().astype(np.uint32)
        keys = t_key.cpu().numpy()
    it_of_rank = np.empty(len(name_rank), dtype=np.int64)
    it_of_rank[name_rank] = np.arange(len(name_rank))
    cheapest = np.where(keys == NONE_KEY, -1, it_of_rank[(keys & 0xFFFFFFFF) % max(len(name_rank), 1)])
    return {"rows": rows, "n_feasible_offerings": nfo, "cheapest": cheapest.astype(np.int32), "cheapest_key": keys}


def sharded_feasibility(solver, words, rank, world, dist=None, device=None):
    """the full static matrix on every rank from one IT-column shard per rank"""
    wb, we = word_range(words, rank, world)
    f, res = solver.feasibility_shard(wb, we)
    out = combine(f["rows"], f["n_feasible_offerings"], f["cheapest_key"], f["it_name_rank"], rank, world, dist, device)
    out["t_kernel_ms"] = res.t_kernel_ms
    return out

"""The static pod x offering feasibility matrix sharded by instance-type
columns over GPUs (BASELINE north_star: "offering columns per
GPU with an RCCL all-reduce (min-price/index) over xGMI").

Rank r evaluates instance-type words [W*r/N, W*(r+1)/N) with
gs_feasibility_shard(_device); the shards combine exactly:
  rows        ALL-GATHER of each rank's own word slice (disjoint columns,
              padded to ceil(W/N) words), written into place,
  offerings   SUM all-reduce,
  cheapest    MIN all-reduce of the OrderByPrice key (price_rank << 32 |
              name_rank; INT64_MAX = none), mapped back to the type through
              its name rank.
`device_combine` runs the collectives on the library's HBM buffers (RCCL over
xGMI, no host round trip); `combine` is the same algebra on host arrays (gloo
on CPU ranks, and the pod-level result of gs_feasibility_shard).  One process
driving several GPUs uses the library's own sharded context instead
(gs_config.n_shards, csrc/multi.cpp).
"""
import numpy as np

NONE_KEY = np.iinfo(np.int64).max


def word_range(words, rank, world):
    return words * rank // world, words * (rank + 1) // world


def cheapest_from_keys(keys, name_rank):
    name_rank = np.asarray(name_rank)
    it_of_rank = np.empty(len(name_rank), dtype=np.int64)
    it_of_rank[name_rank] = np.arange(len(name_rank))
    low = (keys & 0xFFFFFFFF) % max(len(name_rank), 1)
    return np.where(keys == NONE_KEY, -1, it_of_rank[low]).astype(np.int32)


def _gather_slices(rows2d, words, rank, world, dist):
    """rows2d: torch int64 [n, >= words]; every rank's word slice all-gathered
    into place (each rank sends only its own columns)"""
    import torch
    S = -(-words // world)  # widest slice
    wb, we = word_range(words, rank, world)
    mine = torch.zeros((rows2d.shape[0], S), dtype=torch.int64, device=rows2d.device)
    mine[:, :we - wb] = rows2d[:, wb:we]
    parts = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine)
    for r in range(world):
        b, e = word_range(words, r, world)
        rows2d[:, b:e] = parts[r][:, :e - b]


def combine(rows, nfo, keys, name_rank, rank, world, dist, device=None):
    """combine one rank's shard result into the full matrix (every rank)"""
    keys = np.asarray(keys).astype(np.int64)
    if world > 1:
        import torch
        P, T, W = rows.shape
        t_rows = torch.from_numpy(rows.view(np.int64).reshape(P * T, W).copy())
        t_nfo = torch.from_numpy(nfo.astype(np.int64))
        t_key = torch.from_numpy(keys.copy())
        if device is not None:
            t_rows, t_nfo, t_key = t_rows.to(device), t_nfo.to(device), t_key.to(device)
        _gather_slices(t_rows, W, rank, world, dist)
        dist.all_reduce(t_nfo, op=dist.ReduceOp.SUM)
        dist.all_reduce(t_key, op=dist.ReduceOp.MIN)
        rows = t_rows.cpu().numpy().view(np.uint64).reshape(P, T, W)
        nfo = t_nfo.cpu().numpy().astype(np.uint32)
        keys = t_key.cpu().numpy()
    return {"rows": rows, "n_feasible_offerings": nfo, "cheapest": cheapest_from_keys(keys, name_rank),
            "cheapest_key": keys}


class _DeviceArray:
    """zero-copy view of a library-owned HBM buffer for torch (__cuda_array_interface__)"""

    def __init__(self, ptr, n, typestr):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (int(ptr), False),
                                         "strides": None, "version": 2}


def device_views(res, device):
    """torch tensors over a gs_feas_device result: rows (int64 bits), offerings (int32), keys (int64)"""
    import torch
    VT = res.n_variants * res.n_templates
    rows = torch.as_tensor(_DeviceArray(res.rows, VT * res.row_stride, "<i8"), device=device)
    nfo = torch.as_tensor(_DeviceArray(res.n_feasible_offerings, VT, "<i4"), device=device)
    key = torch.as_tensor(_DeviceArray(res.cheapest_key, VT, "<i8"), device=device)
    return rows, nfo, key


def device_combine(res, dist, device):
    """the collectives in place on the library's buffers (RCCL): all-gather
    of the disjoint word slices, SUM of offering counts, MIN of keys"""
    rows, nfo, key = device_views(res, device)
    world, rank = dist.get_world_size(), dist.get_rank()
    VT, S = res.n_variants * res.n_templates, res.row_stride
    _gather_slices(rows.view(VT, S), res.words, rank, world, dist)
    dist.all_reduce(nfo, op=dist.ReduceOp.SUM)
    dist.all_reduce(key, op=dist.ReduceOp.MIN)
    return rows, nfo, key


def expand_to_pods(res, rows, nfo, key, n_nodepools):
    """variant-level device result -> the gs_feas_result layout [pod][nodepool] on host"""
    V, T, S, W = res.n_variants, res.n_templates, res.row_stride, res.words
    rows = rows.cpu().numpy().view(np.uint64).reshape(V, T, S)[:, :, :W]
    nfo = nfo.cpu().numpy().view(np.uint32).reshape(V, T)
    key = key.cpu().numpy().reshape(V, T)
    vop = np.ctypeslib.as_array(res.variant_of_pod, (res.n_pods,)).astype(np.int64) if res.n_pods else \
        np.zeros(0, dtype=np.int64)
    tnp = np.ctypeslib.as_array(res.template_nodepool, (T,)).astype(np.int64) if T else np.zeros(0, dtype=np.int64)
    name_rank = np.ctypeslib.as_array(res.it_name_rank, (res.n_its,)).copy() if res.n_its else np.zeros(0, np.uint32)
    P = res.n_pods
    o_rows = np.zeros((P, n_nodepools, W), dtype=np.uint64)
    o_nfo = np.zeros((P, n_nodepools), dtype=np.uint32)
    o_key = np.full((P, n_nodepools), NONE_KEY, dtype=np.int64)
    for t in range(T):
        o_rows[:, tnp[t]] = rows[vop, t]
        o_nfo[:, tnp[t]] = nfo[vop, t]
        o_key[:, tnp[t]] = key[vop, t]
    return {"rows": o_rows, "n_feasible_offerings": o_nfo, "cheapest": cheapest_from_keys(o_key, name_rank),
            "cheapest_key": o_key}


def sharded_feasibility(solver, words, rank, world, dist=None, device=None):
    """the full static matrix on every rank from one IT-column shard per rank"""
    wb, we = word_range(words, rank, world)
    f, res = solver.feasibility_shard(wb, we)
    out = combine(f["rows"], f["n_feasible_offerings"], f["cheapest_key"], f["it_name_rank"], rank, world, dist, device)
    out["t_kernel_ms"] = res.t_kernel_ms
    return out

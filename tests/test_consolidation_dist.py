"""Multi-rank consolidation on CPU (gloo, world_size 2): simulations sharded
round-robin over ranks, commands all-gathered, policy replayed by the
product's host-only gs_consolidation_choose.  The per-rank evaluator here is
the oracle restricted to the rank's shard (the GPU path is exercised by
tests/test_consolidation.py::test_gpu_consolidation_sharded_union_equals_whole)."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from gpusched import abi, synth
from gpusched.consolidation import sharded_consolidation
from oracle import pyoracle


def _oracle_shard(cin):
    st, cmds, _, _ = pyoracle.consolidate(cin)
    assert st == abi.GS_OK
    r, w = cin.struct.shard_index, cin.struct.shard_count
    if w:
        for i, c in enumerate(cmds):
            if i % w != r:
                cmds[i] = {"decision": abi.DECISION_SKIPPED, "reason": 0, "n_new_claims": 0, "n_failed_pods": 0,
                           "n_candidates": c["n_candidates"], "nodepool": None, "spot_only": 0, "options": [],
                           "option_prices": [], "candidate_price": 0.0}
    return cmds


def _worker(rank, world, port, mode, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p = synth.random_consolidation(3, n_nodes=14, n_pending=1)
        out = sharded_consolidation(_oracle_shard, p, list(range(14)), mode, rank, world, dist)
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("mode", [abi.CONSOLIDATE_SINGLE, abi.CONSOLIDATE_MULTI])
def test_sharded_consolidation_gloo_world2(mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, mode, q)) for r in range(2)]
    for p_ in procs:
        p_.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p_ in procs:
        p_.join(timeout=60)
        assert p_.exitcode == 0
    p = synth.random_consolidation(3, n_nodes=14, n_pending=1)
    from gpusched.consolidation import ConsolidationInput
    st, cmds, chosen, multi = pyoracle.consolidate(ConsolidationInput(p, list(range(14)), mode=mode))
    assert res[0] == res[1] == (cmds, chosen, multi)

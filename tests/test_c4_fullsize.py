"""BASELINE configs[3] at full size (VERDICT r5 Weak 2 / Next 2): the
simulation kernel's command lists for every SingleNodeConsolidation candidate
of the c4 / c4_mixed / c4_e2e sweeps (5,000 state nodes each) and for all 100
MultiNodeConsolidation prefixes candidates[0:j+2] of the c4 and c4_e2e
clusters, against the oracle's digests committed in
tests/golden/c4_consolidation.json (tests/golden/make_c4_golden.py: the
oracle's naive re-Solve of every reduced problem on a process pool).

The sweeps run in both workgroup shapes of the simulation kernel: all 5,000
simulations in one launch take the narrow 128-thread shape (ffd.hip
FB_SIM_NARROW, >= 4 simulations per CU), and 5 shards of 1,000 take the
wide 256-thread shape; the MultiNode prefixes (few, large simulations) run
wide.  c4, c4_e2e and both prefix sweeps are all Delete (every candidate's
pods fit on the kept nodes), so their command records are identical and
the digests coincide; c4_mixed holds Delete, Replace and NoOp."""
import hashlib
import json
import os
import sys

import pytest

from gpusched import abi
from gpusched.consolidation import ConsolidationInput

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_c4_golden as G  # noqa: E402

GOLDEN = json.load(open(os.path.join(HERE, "golden", "c4_consolidation.json")))


def test_golden_covers_every_sweep():
    assert set(GOLDEN) == set(G.SWEEPS)
    for name, g in GOLDEN.items():
        assert g["n_commands"] == (G.N_NODES if G.SWEEPS[name][2] == "single" else G.N_PREFIXES)
        assert sum(g["decisions"].values()) == g["n_commands"]
    assert len(GOLDEN["c4_mixed_single"]["decisions"]) == 3  # Delete, Replace and NoOp


def _digest(cmds):
    return hashlib.sha256(json.dumps(cmds, sort_keys=True, separators=(",", ":")).encode()).hexdigest()


@pytest.fixture(scope="module")
def solver():
    from gpusched.lib import Solver
    s = Solver(0)
    yield s
    s.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c4_single", "c4_mixed_single", "c4_e2e_single"])
def test_gpu_single_node_sweep_full_size(solver, name):
    p = G.cluster(name)
    cands = list(range(G.N_NODES))
    narrow, _, _, _ = solver.consolidate(ConsolidationInput(p, cands, mode=abi.CONSOLIDATE_SINGLE))
    assert len(narrow) == G.N_NODES
    assert _digest(narrow) == GOLDEN[name]["sha256"]
    wide = [None] * G.N_NODES
    for r in range(5):
        part = solver.consolidate(ConsolidationInput(p, cands, mode=abi.CONSOLIDATE_SINGLE, shard=(r, 5)))[0]
        for i in range(r, G.N_NODES, 5):
            wide[i] = part[i]
    assert _digest(wide) == GOLDEN[name]["sha256"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c4_multi", "c4_e2e_multi"])
def test_gpu_multi_node_prefixes_full_size(solver, name):
    p = G.cluster(name)
    multi, _, _, _ = solver.consolidate(ConsolidationInput(p, list(range(G.N_NODES)), mode=abi.CONSOLIDATE_MULTI))
    assert len(multi) == G.N_PREFIXES
    assert _digest(multi) == GOLDEN[name]["sha256"]

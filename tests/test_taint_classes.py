"""Taint vocabularies past 64 distinct taints (VERDICT r3 "What's missing" 3).

The device keeps taints as 64-bit masks.  The encoder maps each distinct taint
to its class of equal toleration pattern (the spec variants that tolerate it):
Taints.ToleratesPod holds iff every taint of the NodePool / node is tolerated,
so taints in one class are interchangeable and the masks carry one bit per
class.  Up to 64 classes are accepted; the raw taint count is not limited.
The oracle has no such encoding and no limit, so it checks the classes: CPU
tests pin acceptance and refusal, GPU tests require the HIP Solve (wave and
block kernels) to equal the oracle bit for bit.
"""
import numpy as np
import pytest

from gpusched import abi, lib, synth
from gpusched.problem import ProblemBuilder
from oracle import pyoracle

Z = "topology.kubernetes.io/zone"


def many_taints(seed, n_nodes=90, n_pods=60, distinct_tol=4, np_taints=True):
    """existing nodes each carrying its own team taint (90+ distinct taints),
    NodePools with taints of their own; pods tolerate every team taint, one
    team's taint, or none"""
    rng = np.random.default_rng(seed)
    b = ProblemBuilder()
    its = synth.build_catalog(b, synth.FAKE_PROFILES, synth.FAKE_ZONES, spot=False,
                              prices=synth.price_table(synth.FAKE_PROFILES))
    b.add_nodepool("open", weight=0)
    if np_taints:
        b.add_nodepool("gpu", weight=10, taints=[("nvidia.com/gpu", "true", "NoSchedule")])
        b.add_nodepool("batch", weight=5, taints=[("batch", "x", "NoSchedule"), ("batch-pref", "y", "PreferNoSchedule")])
    for k in range(n_nodes):
        it = its[int(rng.integers(0, len(its)))]
        labels = {r[0]: r[2][0] for r in it.requirements}
        labels[Z] = str(rng.choice(synth.FAKE_ZONES))
        labels["karpenter.sh/capacity-type"] = "on-demand"
        labels["kubernetes.io/hostname"] = f"n{k}"
        taints = [("team", f"t{k}", "NoSchedule")]
        if rng.random() < 0.3:
            taints.append(("zone-maint", f"m{k % 7}", "NoExecute"))
        b.add_node(f"n{k}", labels, {"cpu": int(rng.choice([2000, 4000])), "memory": 8 << 30, "pods": 20_000},
                   taints=taints)
    teams = [int(t) for t in rng.choice(n_nodes, size=distinct_tol, replace=False)]
    for i in range(n_pods):
        r = rng.random()
        if r < 0.3:
            tols = [("team", "Exists", "", ""), ("zone-maint", "Exists", "", "")]
        elif r < 0.6:
            tols = [("team", "Equal", f"t{teams[int(rng.integers(0, len(teams)))]}", "NoSchedule")]
        elif r < 0.75:
            tols = [("nvidia.com/gpu", "Exists", "", "NoSchedule")]
        elif r < 0.85:
            tols = [("batch", "Equal", "x", "")]
        else:
            tols = []
        b.add_pod(f"p{i}", 1_700_000_000_000_000_000 + i, {"cpu": int(rng.choice([250, 500, 1000])),
                                                            "memory": 1 << 30, "pods": 1000}, tolerations=tols)
    return b.build()


def test_more_than_64_taints_accepted():
    p = many_taints(0)
    st, res, _ = pyoracle.solve(p)
    assert st == abi.GS_OK and res["claims"]
    assert lib.validate(p)[0] == abi.GS_OK


def test_more_than_64_taint_classes_refused():
    # 70 pods, pod i tolerating only node i's team taint: 70 toleration
    # patterns over 80 taints (71 classes with the untolerated rest)
    b = ProblemBuilder()
    synth.build_catalog(b, synth.FAKE_PROFILES, synth.FAKE_ZONES, spot=False,
                        prices=synth.price_table(synth.FAKE_PROFILES))
    b.add_nodepool("open")
    for k in range(80):
        b.add_node(f"n{k}", {Z: synth.FAKE_ZONES[k % len(synth.FAKE_ZONES)], "kubernetes.io/hostname": f"n{k}"},
                   {"cpu": 4000, "memory": 8 << 30, "pods": 20_000}, taints=[("team", f"t{k}", "NoSchedule")])
    for i in range(70):
        b.add_pod(f"p{i}", i, {"cpu": 500, "memory": 1 << 30, "pods": 1000},
                  tolerations=[("team", "Equal", f"t{i}", "NoSchedule")])
    p = b.build()
    st, res, _ = pyoracle.solve(p)
    assert st == abi.GS_OK and len(res["claims"]) == 0  # each pod lands on its own node
    s, msg = lib.validate(p)
    assert s == abi.GS_E_UNSUPPORTED and "taint classes" in msg


@pytest.mark.parametrize("seed", range(6))
def test_oracle_and_encoder_accept(seed):
    p = many_taints(10 + seed)
    assert pyoracle.solve(p)[0] == abi.GS_OK
    assert lib.validate(p)[0] == abi.GS_OK


@pytest.fixture(scope="module", params=["wave", "block"])
def solver(request):
    from gpusched.lib import Solver
    s = Solver(0, {"wave": 0, "block": abi.GS_CFG_BLOCK_SOLVE}[request.param])
    yield s
    s.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(12))
def test_gpu_many_taints(solver, seed):
    from test_gpu_parity import _diff
    p = many_taints(100 + seed, n_pods=int(np.random.default_rng(seed).integers(20, 120)))
    st, want, _ = pyoracle.solve(p)
    assert st == abi.GS_OK
    got, _ = solver.solve(p)
    d = _diff(got, want)
    assert d is None, d

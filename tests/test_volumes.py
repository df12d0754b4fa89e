"""CSI attach limits on existing nodes (<U> karpenter
scheduling.VolumeUsage.ExceedsLimits in ExistingNode.CanAdd: the union of the
node's and the pod's volumes per driver must stay within the CSINode
allocatable count; NodeClaims carry no limit).

CPU known-answer tests pin the oracle on hand-derived cases; GPU tests
require both Solve kernels to equal the oracle bit for bit on random
problems.  Upstream semantics are recalled, not vendored: parity unpinned
(DESIGN.md §1).
"""
import pytest

from gpusched import abi, lib, synth
from gpusched.problem import ProblemBuilder
from oracle import pyoracle

Z = "topology.kubernetes.io/zone"
H = "kubernetes.io/hostname"
EBS = "ebs.csi"


def _base(limits=({EBS: 1}, {})):
    b = ProblemBuilder()
    synth.build_catalog(b, synth.FAKE_PROFILES, synth.FAKE_ZONES, spot=False,
                        prices=synth.price_table(synth.FAKE_PROFILES))
    b.add_nodepool("default", requirements=[(Z, "In", synth.FAKE_ZONES)])
    for k, lim in enumerate(limits):
        b.add_node(f"n{k}", {Z: synth.FAKE_ZONES[0], H: f"n{k}"}, {"cpu": 8000, "memory": 32 << 30, "pods": 110_000},
                   volume_limits=lim)
    return b


def _pod(b, name, vols):
    b.add_pod(name, 0, {"cpu": 500, "memory": 1 << 30, "pods": 1000}, volumes=vols)


def _solve(b):
    st, res, _ = pyoracle.solve(b.build())
    assert st == abi.GS_OK
    return res


def test_new_volume_over_the_limit_skips_the_node():
    b = _base()
    b.add_bound_pod(0, "b0", 0, {"cpu": 100}, volumes=[(EBS, "pv-0")])
    _pod(b, "p0", [(EBS, "pv-1")])  # n0 would hold 2 > 1
    _pod(b, "p1", [(EBS, "pv-0")])  # shares pv-0: the union stays 1
    _pod(b, "p2", [])                # no volume: the union is the node's own (1)
    res = _solve(b)
    assert res["nodes"] == [[1, 2], [0]] and not res["claims"]


def test_node_already_over_its_limit_takes_no_pod():
    b = _base(limits=({EBS: 1},))
    b.add_bound_pod(0, "b0", 0, {"cpu": 100}, volumes=[(EBS, "pv-0"), (EBS, "pv-1")])
    _pod(b, "p0", [])
    res = _solve(b)
    assert res["nodes"] == [[]] and [c["pods"] for c in res["claims"]] == [[0]]


def test_limit_fills_then_nodeclaims_take_the_rest():
    b = _base(limits=({EBS: 2},))
    for i in range(4):
        _pod(b, f"p{i}", [(EBS, f"pv-{i}")])
    res = _solve(b)
    assert res["nodes"] == [[0, 1]] and [c["pods"] for c in res["claims"]] == [[2, 3]]


def test_other_drivers_are_unlimited():
    b = _base(limits=({EBS: 0},))
    _pod(b, "p0", [("nfs.csi", "share")])
    _pod(b, "p1", [(EBS, "pv-0")])
    res = _solve(b)
    assert res["nodes"] == [[0]] and [c["pods"] for c in res["claims"]] == [[1]]


def test_refusals():
    b = _base()
    for i in range(5):
        b.add_pod(f"p{i}", 0, {"cpu": 1}, volumes=[(f"drv{i}", "v")])
    assert lib.validate(b.build())[0] == abi.GS_E_UNSUPPORTED  # more than 4 drivers
    b = _base()
    b.add_pod("x", 0, {"cpu": 1}, flags=abi.POD_VOLUMES)
    assert lib.validate(b.build())[0] == abi.GS_E_UNSUPPORTED


@pytest.mark.parametrize("seed", range(40))
def test_oracle_and_encoder_accept_random_volumes(seed):
    p = synth.random_volumes(seed)
    assert pyoracle.solve(p)[0] == abi.GS_OK
    st, msg = lib.validate(p)
    assert st == abi.GS_OK, msg


# ------------------------------------------------------------------ GPU parity
@pytest.fixture(scope="module", params=["wave", "block", "hbm"])
def solver(request):
    from gpusched.lib import Solver
    s = Solver(0, {"wave": 0, "block": abi.GS_CFG_BLOCK_SOLVE, "hbm": abi.GS_CFG_CLAIMS_HBM}[request.param])
    yield s
    s.close()


def _check(solver, p):
    from test_gpu_parity import _diff
    st, want, _ = pyoracle.solve(p)
    assert st == abi.GS_OK
    got, _ = solver.solve(p)
    d = _diff(got, want)
    assert d is None, d


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(100))
def test_gpu_volumes_random(solver, seed):
    _check(solver, synth.random_volumes(seed))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_gpu_volumes_random_many_pods(solver, seed):
    _check(solver, synth.random_volumes(300 + seed, n_pods=300))

"""Existing nodes that lack a label a pod constrains (VERDICT r4 Missing 1,
next-round item 4).

<U> ExistingNode.CanAdd checks Requirements.Compatible(node requirements, pod
requirements) without AllowUndefinedWellKnownLabels: a key the node lacks is
fine for a pod's NotIn / DoesNotExist and refuses every other operator.  Add
then keeps the intersection as the node's requirement, so the node gains
state on that key: after a NotIn pod the node holds NotIn[...] and admits a
later In pod whose values avoid it; after a DoesNotExist pod it admits no In
pod.  Nodes karpenter did not launch lack the karpenter-ibm.sh/* labels
(reference pkg/apis/v1alpha1/labels.go:37-45), so this is common.

The device keeps a node's instance-type / zone / capacity-type label as one
value id; such keys get a free slot ("shadow") carrying the nodes' full
requirement state when some node lacks them.  CPU tests pin the rules on the
oracle; GPU tests require both Solve kernels and the simulation kernel to
equal the oracle on the known answers and on random clusters.
"""
import pytest

from gpusched import abi, lib, synth
from gpusched.problem import ProblemBuilder
from oracle import pyoracle

Z = "topology.kubernetes.io/zone"
H = "kubernetes.io/hostname"
FAM = "karpenter-ibm.sh/instance-family"
SIZE = "karpenter-ibm.sh/instance-size"
CT = "karpenter.sh/capacity-type"


def bare_node(pods, node_labels=None):
    """one roomy node with only zone and hostname labels (no instance-type
    keys); pods: (cpu, required terms) in queue order (cpu descending)"""
    b = ProblemBuilder()
    synth.build_catalog(b, synth.FAKE_PROFILES, synth.FAKE_ZONES, spot=True,
                        prices=synth.price_table(synth.FAKE_PROFILES))
    b.add_nodepool("np")
    labels = {Z: synth.FAKE_ZONES[0], H: "n0"}
    labels.update(node_labels or {})
    b.add_node("n0", labels, {"cpu": 16000, "memory": 64 << 30, "pods": 100_000})
    for i, (cpu, terms) in enumerate(pods):
        b.add_pod(f"p{i}", 1_700_000_000_000_000_000, {"cpu": cpu, "memory": 1 << 30, "pods": 1000},
                  required_terms=terms)
    return b.build()


# (id, pods, node labels, pods expected on the node (by index))
KATS = [
    ("notin_on_absent_key", [(1000, [[(FAM, "NotIn", ["gx2"])]])], None, [0]),
    ("dne_on_absent_key", [(1000, [[(SIZE, "DoesNotExist", [])]])], None, [0]),
    ("in_on_absent_key_refused", [(1000, [[(FAM, "In", ["bx2"])]])], None, []),
    ("exists_on_absent_key_refused", [(1000, [[(FAM, "Exists", [])]])], None, []),
    ("notin_then_in_admitted", [(2000, [[(FAM, "NotIn", ["gx2"])]]), (1000, [[(FAM, "In", ["bx2"])]])], None, [0, 1]),
    ("notin_then_excluded_in_refused", [(2000, [[(FAM, "NotIn", ["bx2"])]]), (1000, [[(FAM, "In", ["bx2"])]])],
     None, [0]),
    ("notin_then_exists_admitted", [(2000, [[(FAM, "NotIn", ["gx2"])]]), (1000, [[(FAM, "Exists", [])]])], None, [0, 1]),
    ("dne_then_in_refused", [(2000, [[(SIZE, "DoesNotExist", [])]]), (1000, [[(SIZE, "In", ["2x8"])]])], None, [0]),
    ("dne_then_notin_admitted", [(2000, [[(SIZE, "DoesNotExist", [])]]), (1000, [[(SIZE, "NotIn", ["2x8"])]])],
     None, [0, 1]),
    ("capacity_type_notin_absent", [(1000, [[(CT, "NotIn", ["spot"])]])], None, [0]),
    ("capacity_type_in_absent_refused", [(1000, [[(CT, "In", ["on-demand"])]])], None, []),
    ("labelled_node_notin_excludes", [(1000, [[(FAM, "NotIn", ["bx2"])]])], {FAM: "bx2"}, []),
    ("labelled_node_in_admits", [(1000, [[(FAM, "In", ["bx2"])]])], {FAM: "bx2"}, [0]),
    ("in_and_in_empty_is_dne", [(1000, [[(FAM, "In", ["bx2"]), (FAM, "In", ["cx2"])]])], None, [0]),
]


@pytest.mark.parametrize("k", range(len(KATS)), ids=[x[0] for x in KATS])
def test_oracle_absent_label_rules(k):
    _, pods, labels, on_node = KATS[k]
    p = bare_node(pods, labels)
    st, res, _ = pyoracle.solve(p)
    assert st == abi.GS_OK
    assert res["nodes"] == [on_node]
    assert lib.validate(p)[0] == abi.GS_OK


@pytest.mark.parametrize("seed", range(40))
def test_random_partial_labels_accepted(seed):
    p = synth.random_problem(9000 + seed, n_pods=30, partial_labels=True)
    assert pyoracle.solve(p)[0] == abi.GS_OK
    st, msg = lib.validate(p)
    assert st == abi.GS_OK, msg


# ------------------------------------------------------------------- GPU parity
@pytest.fixture(scope="module", params=["wave", "block"])
def solver(request):
    from gpusched.lib import Solver
    s = Solver(0, {"wave": 0, "block": abi.GS_CFG_BLOCK_SOLVE}[request.param])
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
@pytest.mark.parametrize("k", range(len(KATS)), ids=[x[0] for x in KATS])
def test_gpu_absent_label_rules(solver, k):
    _, pods, labels, _ = KATS[k]
    _check(solver, bare_node(pods, labels))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(40))
def test_gpu_random_partial_labels(solver, seed):
    _check(solver, synth.random_problem(9000 + seed, n_pods=30 + 5 * (seed % 7), partial_labels=True,
                                        inflight=bool(seed % 2)))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(16))
@pytest.mark.parametrize("mode", [abi.CONSOLIDATE_SINGLE, abi.CONSOLIDATE_MULTI])
def test_gpu_consolidation_partial_labels(seed, mode):
    from gpusched.lib import Solver
    from test_consolidation import check
    s = Solver(0)
    try:
        check(s, synth.random_consolidation(9100 + seed, n_nodes=16, n_pending=int(seed % 3), partial_labels=True,
                                            inflight=bool(seed % 2)), mode)
    finally:
        s.close()

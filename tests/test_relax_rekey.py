"""Topology.Update re-keying after a relaxation (VERDICT r5 Weak 1 / Next 1).

<U> Scheduler.Solve calls Topology.Update(pod) after every Preferences.Relax
that changed the pod: the pod leaves every group, and its remaining
constraints are keyed again.  A spread group's TopologyGroup.Hash covers the
node filter (MakeTopologyNodeFilter: the node selector AND each required
node-affinity term, by key, and the pod's tolerations), so two relaxations
move a spread owner to another hash: dropping a required node-affinity term
(removeRequiredNodeAffinityTerm, more than one term) and adding the
PreferNoSchedule toleration (toleratePreferNoScheduleTaints, when a NodePool
carries such a taint).  A hash seen before is that group; a new one is a
group created at that moment, whose countDomains counts the cluster's bound
pods only -- none of this Solve's earlier placements -- and, on the hostname
key, none of the in-flight NodeClaims registered before it (a Record makes a
NodeClaim its domain).

The oracle restates this (oracle/solve.cpp topo_update); the product encodes
such groups as lazy groups that the kernels activate at the Relax
(encode.cpp pod_phase_b2, ffd_common.hpp topo_relaxed / topo_mark_unknown).
Parity against upstream itself stays unpinned (no Go toolchain here).
"""
import pytest

from gpusched import abi, lib, synth
from gpusched.problem import ProblemBuilder
from oracle import pyoracle

Z = "topology.kubernetes.io/zone"
H = "kubernetes.io/hostname"
PNS = ("dedicated", "x", "PreferNoSchedule")
BIG = {"cpu": 5000, "memory": 1 << 30, "pods": 1000}  # one per NodeClaim (8 vCPU at most)
SMALL = {"cpu": 500, "memory": 1 << 30, "pods": 1000}


def _catalog():
    b = ProblemBuilder()
    synth.build_catalog(b, synth.FAKE_PROFILES, synth.FAKE_ZONES, spot=False,
                        prices=synth.price_table(synth.FAKE_PROFILES))
    return b


def _placements(res):
    """(pods, nodepool index, zone) per NodeClaim"""
    out = []
    for c in res["claims"]:
        z = [ln.split("|")[2] for ln in c["requirements"].split("\n") if ln.startswith(Z + "|")]
        out.append((c["pods"], c["nodepool"], z[0] if z else None))
    return out


def pns_case():
    """NodePool a (weight 10) offers us-south-1 only; NodePool b offers every
    zone with a PreferNoSchedule taint.  p1 and p2 fail (a's zone is full for
    their spread, b is not tolerated), relax into the toleration and so into a
    new group that has not counted p0: p1 takes us-south-1 again."""
    b = _catalog()
    b.add_nodepool("a", weight=10, requirements=[(Z, "In", synth.FAKE_ZONES[:1])])
    b.add_nodepool("b", requirements=[(Z, "In", synth.FAKE_ZONES)], taints=[PNS])
    sp = {"key": Z, "max_skew": 1, "selector": {"labels": {"app": "web"}}}
    for i in range(3):
        b.add_pod(f"p{i}", i, BIG, labels={"app": "web"}, spreads=[sp])
    return b.build()


def term_case():
    """four spread pods fill the zones 2/1/1; a fifth pod's first required
    term names a zone no NodePool offers, so it relaxes to its second term:
    a new filter (one term instead of two), a new group with no counts, and
    the pod takes us-south-1 where the old group would have sent it to
    us-south-2"""
    b = _catalog()
    b.add_nodepool("default", requirements=[(Z, "In", synth.FAKE_ZONES)])
    sp = {"key": Z, "max_skew": 1, "selector": {"labels": {"app": "web"}}}
    for i in range(4):
        b.add_pod(f"q{i}", i, BIG, labels={"app": "web"}, spreads=[sp])
    b.add_pod("p", 9, BIG, labels={"app": "web"}, spreads=[sp],
              required_terms=[[(Z, "In", ["us-south-9"])], [(Z, "In", synth.FAKE_ZONES)]])
    return b.build()


def hostname_case():
    """every NodePool carries a PreferNoSchedule taint the q pods tolerate;
    the p pods (hostname spread, maxSkew 3) relax into the toleration, so
    their spread is a new hostname group: the NodeClaim the q pods opened is
    no domain of it until q2 is recorded there"""
    b = _catalog()
    b.add_nodepool("a", requirements=[(Z, "In", synth.FAKE_ZONES)], taints=[PNS])
    tol = [("", "Exists", "", "PreferNoSchedule")]
    sp = {"key": H, "max_skew": 3, "selector": {"labels": {"app": "web"}}}
    order = [("q0", 0, True), ("q1", 1, True), ("p0", 2, False), ("p1", 3, False), ("q2", 4, True),
             ("p2", 5, False)]
    for uid, ts, is_q in order:
        b.add_pod(uid, ts, SMALL, labels={"app": "web"}, tolerations=tol if is_q else [],
                  spreads=[] if is_q else [sp])
    return b.build()


def hostname_unknown_case():
    """as hostname_case without q2: the q pods' NodeClaim never becomes a
    domain of the new group, so the p pods open their own NodeClaim"""
    b = _catalog()
    b.add_nodepool("a", requirements=[(Z, "In", synth.FAKE_ZONES)], taints=[PNS])
    tol = [("", "Exists", "", "PreferNoSchedule")]
    sp = {"key": H, "max_skew": 3, "selector": {"labels": {"app": "web"}}}
    for uid, ts, is_q in [("q0", 0, True), ("q1", 1, True), ("p0", 2, False), ("p1", 3, False)]:
        b.add_pod(uid, ts, SMALL, labels={"app": "web"}, tolerations=tol if is_q else [],
                  spreads=[] if is_q else [sp])
    return b.build()


KATS = {"pns": pns_case, "term": term_case, "hostname": hostname_case, "hostname_unknown": hostname_unknown_case}


def test_pns_relaxation_creates_a_group_without_earlier_counts():
    st, res, _ = pyoracle.solve(pns_case())
    assert st == abi.GS_OK and not res["errors"]
    assert pyoracle.last_groups_created() == 1
    # p0 and p1 on NodePool a in us-south-1 (the new group saw none of p0), p2
    # on NodePool b in us-south-2; keeping the old group would give
    # us-south-1 / -2 / -3
    assert _placements(res) == [([0], 0, "us-south-1"), ([1], 0, "us-south-1"), ([2], 1, "us-south-2")]
    assert lib.validate(pns_case()) == (abi.GS_OK, "")


def test_required_term_drop_creates_a_group_without_earlier_counts():
    st, res, _ = pyoracle.solve(term_case())
    assert st == abi.GS_OK and not res["errors"]
    assert pyoracle.last_groups_created() == 1
    zones = [z for pods, _, z in _placements(res) for _ in pods]
    # q0..q3: us-south-1, -2, -3, -1; p: us-south-1 (the old group: us-south-2)
    assert zones == ["us-south-1", "us-south-2", "us-south-3", "us-south-1", "us-south-1"]
    assert lib.validate(term_case()) == (abi.GS_OK, "")


def test_new_hostname_group_knows_only_later_nodeclaims():
    st, res, _ = pyoracle.solve(hostname_unknown_case())
    assert st == abi.GS_OK and not res["errors"]
    assert pyoracle.last_groups_created() == 1
    # keeping the old group (counts 2 on the q NodeClaim, maxSkew 3) would
    # put p0 beside q0 and q1
    assert [pods for pods, _, _ in _placements(res)] == [[0, 1], [2, 3]]
    st, res, _ = pyoracle.solve(hostname_case())
    assert st == abi.GS_OK and not res["errors"]
    # q2 (counted by the new group) makes the q NodeClaim its domain with
    # count 1, so p0 and p1 join it (counts 2, 3) and p2 opens a NodeClaim;
    # the old group (count 3 there after q2) gives [[0, 1, 4], [2, 3, 5]]
    assert [pods for pods, _, _ in _placements(res)] == [[0, 1, 4, 2, 3], [5]]
    for f in (hostname_case, hostname_unknown_case):
        assert lib.validate(f()) == (abi.GS_OK, "")


def min_domains_case():
    """pods with different minDomains relax into one new zone group: the pod
    that relaxes first (p1, minDomains 5 > 3 zones, so the group's minimum
    stays 0) creates it, and the later owners (p2 without minDomains) use its
    minDomains -- an order the kernels learn at the Relax itself"""
    b = _catalog()
    b.add_nodepool("a", weight=10, requirements=[(Z, "In", synth.FAKE_ZONES[:1])])
    b.add_nodepool("b", requirements=[(Z, "In", synth.FAKE_ZONES)], taints=[PNS])
    for i, mind in enumerate((None, 5, None, 5)):
        sp = {"key": Z, "max_skew": 1, "selector": {"labels": {"app": "web"}}}
        if mind:
            sp["min_domains"] = mind
        b.add_pod(f"p{i}", i, BIG, labels={"app": "web"}, spreads=[sp])
    return b.build()


KATS["min_domains"] = min_domains_case


def test_lazy_group_takes_its_creators_min_domains():
    st, res, _ = pyoracle.solve(min_domains_case())
    assert st == abi.GS_OK
    assert pyoracle.last_groups_created() == 1
    assert lib.validate(min_domains_case()) == (abi.GS_OK, "")


@pytest.mark.parametrize("seed", range(80))
def test_random_relax_oracle_runs(seed):
    assert pyoracle.solve(synth.random_relax(seed))[0] == abi.GS_OK


def test_random_relax_rekeys_and_is_accepted():
    """the relax-heavy problems exercise the re-keying (most create a group
    mid-Solve) and the product accepts most of them (a floor, so a tighter
    refusal rule cannot shrink the GPU coverage to nothing)"""
    rekeyed = accepted = 0
    for seed in range(80):
        p = synth.random_relax(seed)
        pyoracle.solve(p)
        rekeyed += pyoracle.last_groups_created() > 0
        st, msg = lib.validate(p)
        assert st == abi.GS_OK, msg
        accepted += 1
    assert rekeyed >= 50, rekeyed


def test_consolidation_pns_clusters_accepted():
    for seed in range(24):
        assert lib.validate(synth.random_consolidation_general(seed, pns=True)) == (abi.GS_OK, "")


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
@pytest.mark.parametrize("name", sorted(KATS))
def test_gpu_rekey_kats(solver, name):
    _check(solver, KATS[name]())


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(80))
def test_gpu_random_relax(solver, seed):
    _check(solver, synth.random_relax(seed))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
def test_gpu_random_relax_many_pods(solver, seed):
    _check(solver, synth.random_relax(500 + seed, n_pods=300))


@pytest.fixture(scope="module")
def csolver():
    from gpusched.lib import Solver
    s = Solver(0)
    yield s
    s.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(24))
@pytest.mark.parametrize("mode", [abi.CONSOLIDATE_SINGLE, abi.CONSOLIDATE_MULTI])
def test_gpu_consolidation_pns(csolver, seed, mode):
    """consolidation simulations on clusters whose NodePools carry a
    PreferNoSchedule taint: the rescheduled pods relax into the toleration and
    re-key their spreads in each simulation's own Topology"""
    from test_consolidation_general import check
    check(csolver, synth.random_consolidation_general(seed, pns=True), mode)

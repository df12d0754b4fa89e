"""Topology spread (<U> karpenter Topology / TopologyGroup).

CPU known-answer tests pin the oracle's restatement on hand-derived cases;
GPU tests require the HIP Solve to equal the oracle bit for bit on random
topology problems and on C3 (zone spread on 20 % of the pods).  Upstream
breaks ties between equally-loaded domains in Go map order (random); this
restatement takes the smallest domain name, so parity against the reference
itself is unpinned.
"""
import pytest

from gpusched import abi, lib, synth
from gpusched.problem import ProblemBuilder
from oracle import pyoracle

Z = "topology.kubernetes.io/zone"
H = "kubernetes.io/hostname"


def _base(zone_req=True, n_pods=6, spread=None, labels=None):
    b = ProblemBuilder()
    synth.build_catalog(b, synth.FAKE_PROFILES, synth.FAKE_ZONES, spot=False,
                        prices=synth.price_table(synth.FAKE_PROFILES))
    b.add_nodepool("default", requirements=[(Z, "In", synth.FAKE_ZONES)] if zone_req else [])
    for i in range(n_pods):
        b.add_pod(f"p{i}", 0, {"cpu": 1500, "memory": 1 << 30, "pods": 1000}, labels=labels or {"app": "web"},
                  spreads=[spread] if spread else [])
    return b


def _zones(res):
    out = []
    for c in res["claims"]:
        z = [ln.split("|")[2] for ln in c["requirements"].split("\n") if ln.startswith(Z + "|")]
        out.append((c["pods"], z[0] if z else None))
    return out


def test_zone_spread_balances_with_name_tie_break():
    sp = {"key": Z, "max_skew": 1, "selector": {"labels": {"app": "web"}}}
    st, res, _ = pyoracle.solve(_base(n_pods=7, spread=sp).build())
    assert st == abi.GS_OK and not res["errors"]
    assert _zones(res) == [([0, 3], "us-south-1"), ([1, 4], "us-south-2"), ([2, 5, 6], "us-south-3")]


def test_hostname_spread_caps_pods_per_nodeclaim():
    sp = {"key": H, "max_skew": 2, "selector": {"labels": {"app": "web"}}}
    b = _base(n_pods=5, spread=sp)
    st, res, _ = pyoracle.solve(b.build())
    assert st == abi.GS_OK
    assert [c["pods"] for c in res["claims"]] == [[0, 1], [2, 3], [4]]


def test_empty_zone_universe_do_not_schedule_fails_schedule_anyway_relaxes():
    # IBM instance types carry no zone requirement: without a NodePool zone
    # requirement (or labelled nodes) there is no zone domain to spread over
    sp = {"key": Z, "max_skew": 1, "selector": {"labels": {"app": "web"}}}
    st, res, _ = pyoracle.solve(_base(zone_req=False, n_pods=3, spread=sp).build())
    assert st == abi.GS_OK and res["errors"] == [0, 1, 2] and not res["claims"]
    sp["when"] = "ScheduleAnyway"
    st, res, _ = pyoracle.solve(_base(zone_req=False, n_pods=3, spread=sp).build())
    assert st == abi.GS_OK and not res["errors"] and len(res["claims"]) == 1


def test_nil_selector_counts_nothing():
    sp = {"key": Z, "max_skew": 1, "selector": None}
    st, res, _ = pyoracle.solve(_base(n_pods=4, spread=sp).build())
    assert st == abi.GS_OK
    assert _zones(res) == [([0, 1, 2, 3], "us-south-1")]


def test_existing_pods_count_toward_domains():
    b = _base(n_pods=2, spread={"key": Z, "max_skew": 1, "selector": {"labels": {"app": "web"}}})
    b.add_node("n0", {Z: "us-south-1", H: "n0"}, {"cpu": 0, "memory": 0, "pods": 0})
    for q in range(2):
        b.add_bound_pod(0, f"b{q}", 0, {"cpu": 1}, labels={"app": "web"})
    st, res, _ = pyoracle.solve(b.build())
    assert st == abi.GS_OK
    assert _zones(res) == [([0], "us-south-2"), ([1], "us-south-3")]


def test_match_label_keys_split_the_group():
    # two bound web pods of template hash h1 in us-south-1; pending pods of
    # hash h2 spread over zones: counted with the h1 pods they avoid
    # us-south-1, with matchLabelKeys [pod-template-hash] they start there
    def build(mlk):
        sp = {"key": Z, "max_skew": 1, "selector": {"labels": {"app": "web"}}}
        if mlk:
            sp["match_label_keys"] = ["pod-template-hash"]
        b = _base(n_pods=0)
        b.add_node("n0", {Z: "us-south-1", H: "n0"}, {"cpu": 0, "memory": 0, "pods": 0})
        for q in range(2):
            b.add_bound_pod(0, f"b{q}", 0, {"cpu": 1}, labels={"app": "web", "pod-template-hash": "h1"})
        for i in range(2):
            b.add_pod(f"p{i}", 0, {"cpu": 1500, "memory": 1 << 30, "pods": 1000},
                      labels={"app": "web", "pod-template-hash": "h2"}, spreads=[sp])
        return b
    st, res, _ = pyoracle.solve(build(False).build())
    assert _zones(res) == [([0], "us-south-2"), ([1], "us-south-3")]
    st, res, _ = pyoracle.solve(build(True).build())
    assert _zones(res) == [([0], "us-south-1"), ([1], "us-south-2")]


def test_refusals():
    b = _base(n_pods=1, spread={"key": "karpenter-ibm.sh/instance-family", "max_skew": 1, "selector": {}})
    assert pyoracle.solve(b.build())[0] == abi.GS_E_UNSUPPORTED
    assert lib.validate(b.build())[0] == abi.GS_E_UNSUPPORTED
    # zone and capacity-type spreads in one problem: the product has one
    # domain key beside the hostname (the oracle computes both)
    b = _base(n_pods=0)
    b.add_pod("p0", 0, {"cpu": 1500, "memory": 1 << 30, "pods": 1000}, labels={"app": "web"},
              spreads=[{"key": Z, "max_skew": 1, "selector": {"labels": {"app": "web"}}},
                       {"key": CT, "max_skew": 1, "selector": {"labels": {"app": "web"}}}])
    assert pyoracle.solve(b.build())[0] == abi.GS_OK
    assert lib.validate(b.build())[0] == abi.GS_E_UNSUPPORTED


CT = "karpenter.sh/capacity-type"


def _ct_case(np_cts, n_pods=6, skew=1, when="DoNotSchedule"):
    """pods spread over the capacity-type key; NodePools constrain it"""
    b = ProblemBuilder()
    synth.build_catalog(b, synth.FAKE_PROFILES, synth.FAKE_ZONES, spot=True,
                        prices=synth.price_table(synth.FAKE_PROFILES))
    for j, cts in enumerate(np_cts):
        b.add_nodepool(f"np{j}", requirements=[(CT, "In", cts)] if cts else [])
    sp = {"key": CT, "max_skew": skew, "when": when, "selector": {"labels": {"app": "web"}}}
    for i in range(n_pods):
        b.add_pod(f"p{i}", i, {"cpu": 1500, "memory": 1 << 30, "pods": 1000}, labels={"app": "web"}, spreads=[sp])
    return b.build()


def _cts(res):
    """the capacity types of each NodeClaim's requirement, pods sorted"""
    out = []
    for c in res["claims"]:
        vals = None
        for line in c["requirements"].split("\n"):
            f = line.split("|")
            if f[0] == CT and f[1] == "In":
                vals = f[2]
        out.append((sorted(c["pods"]), vals))
    return sorted(out)


def test_capacity_type_spread_balances_over_the_nodepool_domains():
    """<U> TopologyGroup on karpenter.sh/capacity-type: the domains are the
    NodePools' In values; maxSkew 1 alternates spot and on-demand claims"""
    st, res, _ = pyoracle.solve(_ct_case([["spot", "on-demand"]]))
    assert st == abi.GS_OK and not res["errors"]
    per = {}
    for pods, v in _cts(res):
        per[v] = per.get(v, 0) + len(pods)
    assert per == {"on-demand": 3, "spot": 3}, per
    assert lib.validate(_ct_case([["spot", "on-demand"]]))[0] == abi.GS_OK
    # one capacity type only in the universe: every pod lands there
    st, res, _ = pyoracle.solve(_ct_case([["on-demand"]]))
    assert st == abi.GS_OK and not res["errors"] and {v for _, v in _cts(res)} == {"on-demand"}


NP = "karpenter.sh/nodepool"


def _np_case(n_pools=2, n_pods=6, node_pool=None):
    """pods spread over the NodePool key (a NodeClaim's domain is its
    template's NodePool; the universe is the NodePools and labelled nodes)"""
    b = ProblemBuilder()
    synth.build_catalog(b, synth.FAKE_PROFILES, synth.FAKE_ZONES, spot=False,
                        prices=synth.price_table(synth.FAKE_PROFILES))
    for j in range(n_pools):
        b.add_nodepool(f"np{j}", weight=10 * (n_pools - j))
    if node_pool is not None:
        b.add_node("n0", {Z: "us-south-1", H: "n0", NP: node_pool}, {"cpu": 0, "memory": 0, "pods": 0})
        for q in range(2):
            b.add_bound_pod(0, f"b{q}", 0, {"cpu": 1}, labels={"app": "web"})
    sp = {"key": NP, "max_skew": 1, "selector": {"labels": {"app": "web"}}}
    for i in range(n_pods):
        b.add_pod(f"p{i}", i, {"cpu": 1500, "memory": 1 << 30, "pods": 1000}, labels={"app": "web"}, spreads=[sp])
    return b.build()


def test_nodepool_spread_balances_over_nodepools():
    """the heavier NodePool alone would take every pod; maxSkew 1 over the
    NodePool key alternates the two (and counts a labelled node's pods)"""
    st, res, _ = pyoracle.solve(_np_case())
    assert st == abi.GS_OK and not res["errors"]
    per = {}
    for c in res["claims"]:
        per[c["nodepool"]] = per.get(c["nodepool"], 0) + len(c["pods"])
    assert sorted(per.values()) == [3, 3], per
    assert lib.validate(_np_case())[0] == abi.GS_OK
    st, res, _ = pyoracle.solve(_np_case(node_pool="np0"))
    per = {}
    for c in res["claims"]:
        per[c["nodepool"]] = per.get(c["nodepool"], 0) + len(c["pods"])
    assert st == abi.GS_OK and sorted(per.values()) == [2, 4], per


def test_unlabeled_node_beside_multi_group_owner_refused():
    """two NodePool-key groups that pick different domains leave an empty
    requirement, which upstream lets a node lacking the label pass: the
    product refuses that input (one group per pod is exact)"""
    b = ProblemBuilder()
    synth.build_catalog(b, synth.FAKE_PROFILES, synth.FAKE_ZONES, spot=False,
                        prices=synth.price_table(synth.FAKE_PROFILES))
    b.add_nodepool("np0")
    b.add_nodepool("np1")
    b.add_node("n0", {Z: "us-south-1", H: "n0"}, {"cpu": 8000, "memory": 32 << 30, "pods": 20000})
    two = [{"key": NP, "max_skew": 1, "selector": {"labels": {"app": a}}} for a in ("web", "api")]
    b.add_pod("p0", 0, {"cpu": 500, "memory": 1 << 30, "pods": 1000}, labels={"app": "web"}, spreads=two)
    assert pyoracle.solve(b.build())[0] == abi.GS_OK
    assert lib.validate(b.build())[0] == abi.GS_E_UNSUPPORTED


@pytest.mark.parametrize("seed", range(60))
def test_nodepool_spread_random_accepted(seed):
    p = synth.random_topology(seed, domain_key=NP)
    assert pyoracle.solve(p)[0] == abi.GS_OK
    assert lib.validate(p)[0] == abi.GS_OK


@pytest.mark.parametrize("seed", range(60))
def test_capacity_type_spread_random_accepted(seed):
    p = synth.random_topology(seed, domain_key=CT)
    assert pyoracle.solve(p)[0] == abi.GS_OK
    assert lib.validate(p)[0] == abi.GS_OK


# ---------------------------------------------- <U> TopologyNodeFilter (oracle)
# The oracle applies the filter itself: a node / NodeClaim counts in a spread
# group (countDomains, Record) only when its requirements are Compatible with
# the owner's node selector AND one of its required terms (AffinityPolicy
# Honor) and the owner tolerates its taints (TaintPolicy Honor); under taint
# Honor a domain enters the minimum only if a NodePool / node providing it
# has taints the pod tolerates (TopologyDomainGroup.ForEachDomain).  Where the
# filter cannot change the answer (zone-only affinity, tolerated taints) both
# accept and the Honor run must equal the Ignore run.  Round 5: an affinity
# filter past the zone key is applied by the product too -- bound pods count
# only on matching nodes, and the pending pods a group counts must carry the
# owner's terms (every NodeClaim / node they land on then matches); other
# Honor inputs stay refused.
def _tainted_node_case(pol):
    sp = {"key": Z, "max_skew": 1, "selector": {"labels": {"app": "web"}}, "node_taints_policy": pol}
    b = _base(n_pods=0)
    b.add_node("n0", {Z: "us-south-1", H: "n0"}, {"cpu": 0, "memory": 0, "pods": 0},
               taints=[("dedicated", "x", "NoSchedule")])
    for q in range(2):
        b.add_bound_pod(0, f"b{q}", 0, {"cpu": 1}, labels={"app": "web"})
    for i in range(2):
        b.add_pod(f"p{i}", 0, {"cpu": 1500, "memory": 1 << 30, "pods": 1000}, labels={"app": "web"}, spreads=[sp])
    return b.build()


def test_filter_taint_honor_drops_intolerable_node():
    # Ignore: the tainted node's two web pods count -> the pods avoid us-south-1
    st, res, _ = pyoracle.solve(_tainted_node_case("Ignore"))
    assert st == abi.GS_OK and _zones(res) == [([0], "us-south-2"), ([1], "us-south-3")]
    # Honor: the owner does not tolerate the node's taint -> its pods do not count
    p = _tainted_node_case("Honor")
    st, res, _ = pyoracle.solve(p)
    assert st == abi.GS_OK and _zones(res) == [([0], "us-south-1"), ([1], "us-south-2")]
    assert lib.validate(p)[0] == abi.GS_OK  # applied by the product too (GPU: test_gpu_topology_kats)


def _family_node_case(pol):
    sp = {"key": Z, "max_skew": 1, "selector": {"labels": {"app": "web"}}, "node_affinity_policy": pol}
    b = _base(n_pods=0)
    b.add_node("n0", {Z: "us-south-1", H: "n0", "karpenter-ibm.sh/instance-family": "gx2"},
               {"cpu": 0, "memory": 0, "pods": 0})
    for q in range(2):
        b.add_bound_pod(0, f"b{q}", 0, {"cpu": 1}, labels={"app": "web"})
    for i in range(2):
        b.add_pod(f"p{i}", 0, {"cpu": 1500, "memory": 1 << 30, "pods": 1000}, labels={"app": "web"},
                  node_selector={"karpenter-ibm.sh/instance-family": "bx2"}, spreads=[sp])
    return b.build()


def test_filter_affinity_honor_drops_incompatible_node():
    st, res, _ = pyoracle.solve(_family_node_case("Ignore"))
    assert st == abi.GS_OK and _zones(res) == [([0], "us-south-2"), ([1], "us-south-3")]
    assert lib.validate(_family_node_case("Ignore"))[0] == abi.GS_OK
    # Honor: n0 (family gx2) is not Compatible with the owner's bx2 selector
    p = _family_node_case("Honor")
    st, res, _ = pyoracle.solve(p)
    assert st == abi.GS_OK and _zones(res) == [([0], "us-south-1"), ([1], "us-south-2")]
    assert lib.validate(p)[0] == abi.GS_OK  # the product drops n0's pods too (GPU: test_gpu_topology_kats)


def _family_counted_case(other_sel=None, other_pref=None):
    sp = {"key": Z, "max_skew": 1, "selector": {"labels": {"app": "web"}}, "node_affinity_policy": "Honor"}
    b = _base(n_pods=0)
    for i in range(2):
        b.add_pod(f"p{i}", 0, {"cpu": 1500, "memory": 1 << 30, "pods": 1000}, labels={"app": "web"},
                  node_selector={"karpenter-ibm.sh/instance-family": "bx2"}, spreads=[sp])
    b.add_pod("q", 1, {"cpu": 1500, "memory": 1 << 30, "pods": 1000}, labels={"app": "web"},
              node_selector=other_sel, preferred_terms=other_pref or ())
    return b.build()


def test_filter_affinity_honor_counted_pods_must_carry_the_filter():
    """a pod the group counts but whose node affinity differs from the
    owner's may land where the filter does not match (upstream then does not
    count it): the product refuses; the same affinity is accepted, and so is a
    preference on another key, but not one on a filter key"""
    F = "karpenter-ibm.sh/instance-family"
    assert pyoracle.solve(_family_counted_case())[0] == abi.GS_OK
    assert lib.validate(_family_counted_case())[0] == abi.GS_E_UNSUPPORTED
    assert lib.validate(_family_counted_case({F: "cx2"}))[0] == abi.GS_E_UNSUPPORTED
    assert lib.validate(_family_counted_case({F: "bx2"}))[0] == abi.GS_OK
    assert lib.validate(_family_counted_case({F: "bx2"}, [(10, [(Z, "In", ["us-south-2"])])]))[0] == abi.GS_OK
    assert lib.validate(_family_counted_case({F: "bx2"}, [(10, [(F, "In", ["bx2"])])]))[0] == abi.GS_E_UNSUPPORTED


def _tainted_pool_case(pol):
    # NodePool "a" offers us-south-1/2; NodePool "b" alone offers us-south-3
    # and carries a taint the pods do not tolerate
    sp = {"key": Z, "max_skew": 1, "selector": {"labels": {"app": "web"}}, "node_taints_policy": pol}
    b = ProblemBuilder()
    synth.build_catalog(b, synth.FAKE_PROFILES, synth.FAKE_ZONES, spot=False,
                        prices=synth.price_table(synth.FAKE_PROFILES))
    b.add_nodepool("a", requirements=[(Z, "In", synth.FAKE_ZONES[:2])])
    b.add_nodepool("b", requirements=[(Z, "In", synth.FAKE_ZONES[2:])], taints=[("dedicated", "x", "NoSchedule")])
    for i in range(4):
        b.add_pod(f"p{i}", 0, {"cpu": 1500, "memory": 1 << 30, "pods": 1000}, labels={"app": "web"}, spreads=[sp])
    return b.build()


def test_filter_taint_honor_drops_intolerable_domain_from_minimum():
    # Ignore: us-south-3 (count 0, unreachable) holds the minimum at 0 -> with
    # maxSkew 1 only one pod per reachable zone schedules
    st, res, _ = pyoracle.solve(_tainted_pool_case("Ignore"))
    assert st == abi.GS_OK and res["errors"] == [2, 3]
    # Honor: ForEachDomain skips us-south-3 (its only provider is intolerable)
    p = _tainted_pool_case("Honor")
    st, res, _ = pyoracle.solve(p)
    assert st == abi.GS_OK and not res["errors"]
    assert sorted(z for pods, z in _zones(res) for _ in pods) == ["us-south-1", "us-south-1", "us-south-2",
                                                                  "us-south-2"]
    assert lib.validate(p)[0] == abi.GS_OK  # applied by the product too (GPU: test_gpu_topology_kats)


def _unconstrained_pool_case(pol):
    """NodePool "a" has no requirement and no taint, NodePool "b"
    names us-south-3 only and carries a taint the pods do not tolerate, and
    an existing node in us-south-1 has room for every pod.  <U>
    buildDomainGroups combines each NodePool's requirements with each of its
    instance types'; the IBM instance types carry no zone requirement
    (pkg/providers/common/instancetype/instancetype.go:719-724), so "a"
    provides no zone domain and us-south-3's only provider is intolerable"""
    sp = {"key": Z, "max_skew": 1, "selector": {"labels": {"app": "web"}}, "node_taints_policy": pol}
    b = ProblemBuilder()
    synth.build_catalog(b, synth.FAKE_PROFILES, synth.FAKE_ZONES, spot=False,
                        prices=synth.price_table(synth.FAKE_PROFILES))
    b.add_nodepool("a")
    b.add_nodepool("b", requirements=[(Z, "In", synth.FAKE_ZONES[2:])], taints=[("dedicated", "x", "NoSchedule")])
    b.add_node("n0", {Z: "us-south-1", H: "n0"}, {"cpu": 64000, "memory": 64 << 40, "pods": 100_000})
    for i in range(4):
        b.add_pod(f"p{i}", i, {"cpu": 500, "memory": 1 << 30, "pods": 1000}, labels={"app": "web"}, spreads=[sp])
    return b.build()


def test_taint_honor_unconstrained_pool_provides_no_domain():
    """Honor: us-south-3 leaves domainMinCount, so the minimum is the node's
    zone's own count and every pod joins n0; Ignore keeps us-south-3 (count 0)
    in the minimum, so n0 and NodeClaims in us-south-3 (through the
    unconstrained NodePool "a") alternate"""
    st, res, _ = pyoracle.solve(_unconstrained_pool_case("Honor"))
    assert st == abi.GS_OK and not res["errors"] and not res["claims"]
    assert res["nodes"][0] == [0, 1, 2, 3]
    st, res, _ = pyoracle.solve(_unconstrained_pool_case("Ignore"))
    assert st == abi.GS_OK and res["nodes"][0] == [0, 2]
    assert sorted(p for pods, z in _zones(res) for p in pods if z == "us-south-3") == [1, 3]
    for pol in ("Honor", "Ignore"):
        assert lib.validate(_unconstrained_pool_case(pol)) == (abi.GS_OK, "")


def test_ambiguous_domain_universe_refused():
    """a NodePool NotIn on the spread key (buildDomainGroups would insert the
    excluded values) and instance types with a zone requirement (their values
    would enter the universe) are refused by oracle and product alike"""
    sp = {"key": Z, "max_skew": 1, "selector": {"labels": {"app": "web"}}}
    b = ProblemBuilder()
    synth.build_catalog(b, synth.FAKE_PROFILES, synth.FAKE_ZONES, spot=False,
                        prices=synth.price_table(synth.FAKE_PROFILES))
    b.add_nodepool("a", requirements=[(Z, "NotIn", synth.FAKE_ZONES[2:])])
    b.add_pod("p0", 0, {"cpu": 500, "memory": 1 << 30, "pods": 1000}, labels={"app": "web"}, spreads=[sp])
    assert pyoracle.solve(b.build())[0] == abi.GS_E_UNSUPPORTED
    st, msg = lib.validate(b.build())
    assert st == abi.GS_E_UNSUPPORTED and "NotIn" in msg


def test_taint_honor_counted_pod_tolerating_more_than_owner_refused():
    """a counted pod that tolerates a taint the owner does not may land where
    upstream does not count it: refused (the oracle computes it)"""
    sp = {"key": Z, "max_skew": 1, "selector": {"labels": {"app": "web"}}, "node_taints_policy": "Honor"}
    b = ProblemBuilder()
    synth.build_catalog(b, synth.FAKE_PROFILES, synth.FAKE_ZONES, spot=False,
                        prices=synth.price_table(synth.FAKE_PROFILES))
    b.add_nodepool("a", taints=[("dedicated", "x", "NoSchedule")])
    b.add_nodepool("b")
    b.add_pod("p0", 0, {"cpu": 1500, "memory": 1 << 30, "pods": 1000}, labels={"app": "web"}, spreads=[sp])
    b.add_pod("p1", 1, {"cpu": 1500, "memory": 1 << 30, "pods": 1000}, labels={"app": "web"},
              tolerations=[("dedicated", "Exists", "", "")])
    assert pyoracle.solve(b.build())[0] == abi.GS_OK
    assert lib.validate(b.build())[0] == abi.GS_E_UNSUPPORTED


@pytest.mark.parametrize("seed", range(60))
def test_taint_policy_honor_by_app_accepted_or_refused(seed):
    """apps tolerating the NodePools' taint or not: the oracle computes every
    problem; the product accepts it or refuses the counted-pod case"""
    p = synth.random_topology(seed, taint_policy="Honor", tol_by_app=True)
    assert pyoracle.solve(p)[0] == abi.GS_OK
    st, msg = lib.validate(p)
    assert st == abi.GS_OK or "tolerating a taint its owner does not" in msg


def _shared_group_case(zones_per_pod, pol="Honor"):
    sp = {"key": Z, "max_skew": 1, "selector": {"labels": {"app": "web"}}, "node_affinity_policy": pol}
    b = _base(n_pods=0)
    for i, zs in enumerate(zones_per_pod):
        b.add_pod(f"p{i}", i, {"cpu": 1500, "memory": 1 << 30, "pods": 1000}, labels={"app": "web"},
                  required_terms=[[(Z, "In", zs)]], spreads=[sp])
    return b.build()


def test_filter_group_keeps_first_owners_filter():
    """TopologyGroup.Hash covers the filter's requirement keys, not values
    (hashstructure skips unexported fields): owners with zone In [1] and
    zone In [2, 3] share one group whose filter is the first owner's, so the
    us-south-2/3 pods are never counted and the later owners always see 0"""
    zs = [["us-south-1"], ["us-south-2", "us-south-3"], ["us-south-2", "us-south-3"],
          ["us-south-2", "us-south-3"]]
    st, res, _ = pyoracle.solve(_shared_group_case(zs))
    assert st == abi.GS_OK
    honor = _zones(res)
    st, res, _ = pyoracle.solve(_shared_group_case(zs, "Ignore"))
    ignore = _zones(res)
    assert ignore == [([0], "us-south-1"), ([1, 3], "us-south-2"), ([2], "us-south-3")]
    assert honor == [([0], "us-south-1"), ([1, 2, 3], "us-south-2")]
    assert lib.validate(_shared_group_case(zs))[0] == abi.GS_E_UNSUPPORTED
    assert lib.validate(_shared_group_case(zs, "Ignore"))[0] == abi.GS_OK
    # the same filter on every owner: Honor == Ignore, accepted
    same = [["us-south-2", "us-south-3"]] * 4
    assert pyoracle.solve(_shared_group_case(same))[1] == pyoracle.solve(_shared_group_case(same, "Ignore"))[1]
    assert lib.validate(_shared_group_case(same))[0] == abi.GS_OK


def _merge_case(second_mind):
    """owners of one zone spread that differ only in tolerations: upstream
    keeps a group per toleration set (TopologyGroup.Hash), each with its first
    owner's minDomains; the product shares the groups whose minDomains agree"""
    b = _base(n_pods=0)
    b.add_node("n0", {Z: "us-south-1", H: "n0"}, {"cpu": 0, "memory": 0, "pods": 0})
    b.add_bound_pod(0, "b0", 0, {"cpu": 1}, labels={"app": "web"})
    for i in range(9):
        sp = {"key": Z, "max_skew": 1, "selector": {"labels": {"app": "web"}}}
        tols = [("spot", "Exists", "", "")] if i % 3 == 1 else []
        if i == 1 and second_mind is not None:
            sp["min_domains"] = second_mind
        b.add_pod(f"p{i}", i, {"cpu": 1500, "memory": 1 << 30, "pods": 1000}, labels={"app": "web"},
                  tolerations=tols, spreads=[sp])
    return b.build()


def test_groups_differing_in_tolerations_only():
    for mind in (None, 2, 5):
        assert pyoracle.solve(_merge_case(mind))[0] == abi.GS_OK
        assert lib.validate(_merge_case(mind))[0] == abi.GS_OK
    # minDomains 5 > 3 zones holds the first owner's group at a global minimum of 0
    assert pyoracle.solve(_merge_case(5))[1] != pyoracle.solve(_merge_case(None))[1]


def test_affinity_policy_honor_zone_only_equals_ignore():
    """nodeAffinityPolicy Honor with a zone-only node selector: the filter
    drops only nodes outside the owner's zones, so Honor == Ignore"""
    out = []
    for pol in ("Honor", "Ignore"):
        b = _base(n_pods=0)
        b.add_node("n0", {Z: "us-south-3", H: "n0"}, {"cpu": 0, "memory": 0, "pods": 0})
        b.add_bound_pod(0, "b0", 0, {"cpu": 1}, labels={"app": "web"})
        for i in range(4):
            b.add_pod(f"p{i}", i, {"cpu": 1500, "memory": 1 << 30, "pods": 1000}, labels={"app": "web"},
                      node_selector={Z: "us-south-1"} if i % 2 else {},
                      spreads=[{"key": Z, "max_skew": 1, "selector": {"labels": {"app": "web"}},
                                "node_affinity_policy": pol}])
        st, res, _ = pyoracle.solve(b.build())
        assert st == abi.GS_OK and lib.validate(b.build())[0] == abi.GS_OK
        out.append(_zones(res))
    assert out[0] == out[1]


@pytest.mark.parametrize("multi_term", [False, True])
@pytest.mark.parametrize("seed", range(60))
def test_affinity_policy_honor_random_equals_ignore(seed, multi_term):
    """the oracle's real filter on random problems whose spread owners carry
    zone-only node affinity (NotIn, or two In terms OR'd): Honor == Ignore"""
    ph = synth.random_topology(seed, affinity_policy="Honor", multi_term=multi_term)
    pi = synth.random_topology(seed, affinity_policy="Ignore", multi_term=multi_term)
    sh, rh, _ = pyoracle.solve(ph)
    si, ri, _ = pyoracle.solve(pi)
    assert sh == si == abi.GS_OK and rh == ri
    assert lib.validate(ph)[0] == abi.GS_OK


HONOR_REKEY_REFUSAL = "without its owner's node affinity"


@pytest.mark.parametrize("seed", range(60))
def test_affinity_policy_honor_family_filter_accepted(seed):
    """deployments with node affinity on instance family / type and Honor
    spreads, bound pods on nodes of every family: the oracle computes every
    problem; the encoder accepts it, or refuses a deployment with two OR'd
    terms, whose relaxation re-keys its spread to a filter of the remaining
    term (<U> Topology.Update) that its own unrelaxed pods do not carry
    (tests/test_relax_rekey.py).  The GPU parity runs are
    test_gpu_topology_honor_filter"""
    p = synth.random_honor_filter(seed)
    assert pyoracle.solve(p)[0] == abi.GS_OK
    st, msg = lib.validate(p)
    assert st == abi.GS_OK or HONOR_REKEY_REFUSAL in msg, msg


def test_affinity_policy_honor_family_filter_acceptance_floor():
    """a floor on the accepted seeds, so a tighter refusal rule
    cannot shrink the GPU coverage of the Honor filter to nothing"""
    accepted = sum(lib.validate(synth.random_honor_filter(seed))[0] == abi.GS_OK for seed in range(60))
    assert accepted >= 35, accepted


def test_taint_policy_honor_by_app_acceptance_floor():
    """at least a third of the tol_by_app problems run the
    intolerable-taint Honor path on the GPU (test_gpu_topology_taint_honor_by_app)"""
    accepted = sum(lib.validate(synth.random_topology(seed, taint_policy="Honor", tol_by_app=True))[0] == abi.GS_OK
                   for seed in range(60))
    assert accepted >= 30, accepted


def test_affinity_policy_honor_family_filter_changes_answers():
    """the filter matters on these problems: Honor differs from Ignore"""
    differ = 0
    for seed in range(30):
        rh = pyoracle.solve(synth.random_honor_filter(seed))[1]
        ri = pyoracle.solve(synth.random_honor_filter(seed, affinity_policy="Ignore"))[1]
        differ += rh != ri
    assert differ >= 5, differ


def test_taint_policy_honor_without_taints_equals_ignore():
    """TopologyNodeFilter.Matches: with no taint in the problem Honor filters
    nothing (the group is the Ignore group)"""
    out = []
    for pol in ("Honor", "Ignore"):
        b = _base(n_pods=4, spread={"key": Z, "max_skew": 1, "selector": {}, "node_taints_policy": pol})
        st, res, _ = pyoracle.solve(b.build())
        assert st == abi.GS_OK and lib.validate(b.build())[0] == abi.GS_OK
        out.append(_zones(res))
    assert out[0] == out[1] and len(out[0]) == 3


@pytest.mark.parametrize("seed", range(60))
def test_taint_policy_honor_tolerated_equals_ignore(seed):
    """owners that tolerate every NodePool / node taint: Honor == Ignore,
    accepted by the encoder and the oracle alike"""
    ph = synth.random_topology(seed, taint_policy="Honor")
    pi = synth.random_topology(seed, taint_policy="Ignore")
    sh, rh, _ = pyoracle.solve(ph)
    si, ri, _ = pyoracle.solve(pi)
    assert sh == si == abi.GS_OK and rh == ri
    assert lib.validate(ph)[0] == abi.GS_OK


@pytest.mark.parametrize("seed", range(40))
def test_oracle_and_encoder_accept_random_topology(seed):
    p = synth.random_topology(seed)
    assert pyoracle.solve(p)[0] == abi.GS_OK
    assert lib.validate(p)[0] == abi.GS_OK


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
@pytest.mark.parametrize("seed", range(150))
def test_gpu_topology_random(solver, seed):
    _check(solver, synth.random_topology(seed))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(20))
def test_gpu_topology_taint_policy_honor(solver, seed):
    _check(solver, synth.random_topology(seed, taint_policy="Honor"))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(20))
def test_gpu_topology_affinity_policy_honor(solver, seed):
    _check(solver, synth.random_topology(seed, affinity_policy="Honor"))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(40))
def test_gpu_topology_honor_filter(solver, seed):
    p = synth.random_honor_filter(seed)
    if lib.validate(p)[0] != abi.GS_OK:
        pytest.skip("refused: relaxation re-keys the spread (test_affinity_policy_honor_family_filter_acceptance_floor)")
    _check(solver, p)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(8))
def test_gpu_topology_honor_filter_many_pods(solver, seed):
    p = synth.random_honor_filter(700 + seed, n_pods=400)
    if lib.validate(p)[0] != abi.GS_OK:
        pytest.skip("refused: relaxation re-keys the spread")
    _check(solver, p)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(40))
def test_gpu_topology_capacity_type_spread(solver, seed):
    _check(solver, synth.random_topology(seed, domain_key=CT))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(60))
def test_gpu_topology_taint_honor_by_app(solver, seed):
    p = synth.random_topology(seed, taint_policy="Honor", tol_by_app=True)
    if lib.validate(p)[0] != abi.GS_OK:
        pytest.skip("refused (counted pod tolerating more than its owner)")
    _check(solver, p)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(40))
def test_gpu_topology_nodepool_spread(solver, seed):
    _check(solver, synth.random_topology(seed, domain_key=NP))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_gpu_topology_nodepool_spread_many_pods(solver, seed):
    _check(solver, synth.random_topology(900 + seed, n_pods=300, domain_key=NP))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_gpu_topology_capacity_type_spread_many_pods(solver, seed):
    _check(solver, synth.random_topology(900 + seed, n_pods=300, domain_key=CT))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(10))
def test_gpu_topology_random_many_pods(solver, seed):
    _check(solver, synth.random_topology(900 + seed, n_pods=300))


@pytest.mark.gpu
def test_gpu_topology_kats(solver):
    for mlk in (False, True):
        sp = {"key": Z, "max_skew": 1, "selector": {"labels": {"app": "web"}}}
        if mlk:
            sp["match_label_keys"] = ["pod-template-hash"]
        b = _base(n_pods=0)
        b.add_node("n0", {Z: "us-south-1", H: "n0"}, {"cpu": 0, "memory": 0, "pods": 0})
        for q in range(2):
            b.add_bound_pod(0, f"b{q}", 0, {"cpu": 1}, labels={"app": "web", "pod-template-hash": "h1"})
        for i in range(2):
            b.add_pod(f"p{i}", 0, {"cpu": 1500, "memory": 1 << 30, "pods": 1000},
                      labels={"app": "web", "pod-template-hash": "h2"}, spreads=[sp])
        _check(solver, b.build())
    _check(solver, _base(n_pods=7, spread={"key": Z, "max_skew": 1, "selector": {"labels": {"app": "web"}}}).build())
    _check(solver, _family_node_case("Honor"))
    for mind in (None, 2, 5):
        _check(solver, _merge_case(mind))
    for np_cts in ([["spot", "on-demand"]], [["on-demand"]], [["spot"], ["on-demand"]], [None]):
        _check(solver, _ct_case(np_cts))
        _check(solver, _ct_case(np_cts, n_pods=9, skew=2, when="ScheduleAnyway"))
    for npools, node_pool in ((2, None), (2, "np0"), (3, "np1"), (1, "other")):
        _check(solver, _np_case(npools, node_pool=node_pool))
    _check(solver, _tainted_node_case("Honor"))
    _check(solver, _tainted_pool_case("Honor"))
    for pol in ("Honor", "Ignore"):
        _check(solver, _unconstrained_pool_case(pol))
    _check(solver, _family_counted_case({"karpenter-ibm.sh/instance-family": "bx2"}))
    _check(solver, _base(n_pods=5, spread={"key": H, "max_skew": 2, "selector": {"labels": {"app": "web"}}}).build())


@pytest.mark.gpu
def test_gpu_topology_c3(solver):
    _check(solver, synth.make_c3(n_pods=5000))

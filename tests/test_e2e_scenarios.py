"""The reference e2e suite's expectations as Solve-level known-answer scenarios
(VERDICT r2 Missing 3 / next-round item 2): the only evidence the reference
itself holds about what a Solve must produce.

tests/golden/e2e_scenarios.json (written by tests/golden/make_e2e_scenarios.py)
restates each test's NodePool, workloads, arrival order and assertion with
its reference file:line:
  * scheduling_test.go:246-344  3 replicas, required hostname anti-affinity
                                -> 3 distinct NodeClaims
  * scheduling_test.go:359-475  instance-type node affinity -> only that type
  * multizone_test.go:188-289   zone spread maxSkew 1 -> skew <= 1, > 1 zone
  * multizone_test.go:83-174    preferred zone anti-affinity -> > 1 zone
  * scheduling_test.go:38-176   4 replicas, preferred hostname anti-affinity
                                -> several nodes; scaled down, consolidation
  * e2e_taints_test.go:458-611  tainted NodePool: the tolerating pod lands on
                                its NodeClaim, the intolerant one stays pending
  * basic_workflow_test.go:76-115  every NodeClaim's types within the
                                NodePool's allowed list, its requirements met
  * multizone_test.go:384-431   preferred zone anti-affinity, 4 -> 8 replicas:
                                still more than one zone
  * e2e_taints_test.go:43-258   NodePool startup taints: the pod gets a
                                NodeClaim of the pool; (derived) a pod without
                                the tolerations packs onto the initializing
                                node, not once it is initialized and tainted
  * e2e_taints_test.go:614-776  Equal tolerations of a NoSchedule and a
                                PreferNoSchedule taint with values; (derived)
                                Relax tolerates PreferNoSchedule, a wrong
                                value stays pending
Workloads marked "derived" extend a reference test with a step it implies.
The CPU tests run every scenario through the oracle and assert the reference
test's property; the GPU tests require both HIP Solve kernels (and the
consolidation simulation kernel) to equal the oracle at every step, so the
property holds for the product too.
"""
import json
import os

import pytest

from gpusched import abi, synth
from gpusched.consolidation import ConsolidationInput
from gpusched.problem import ProblemBuilder
from oracle import pyoracle

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "e2e_scenarios.json")) as f:
    GOLD = json.load(f)
ZONES = GOLD["zones"]
IT = "node.kubernetes.io/instance-type"
Z = "topology.kubernetes.io/zone"
H = "kubernetes.io/hostname"
NP = "e2e-nodepool"
GI = 1 << 30
MI = 1 << 20


def zones_of(claim):
    for line in claim["requirements"].split("\n"):
        f = line.split("|")
        if f[0] == Z and f[1] == "In":
            return sorted(v for v in f[2].split(",") if v)
    return list(ZONES)


class Cluster:
    """the e2e cluster between Solves: launched nodes with their bound pods"""

    def __init__(self, sc):
        self.sc = sc
        self.nodes = []  # dict(name, it, zone, pods)
        self.pods = []   # every pod spec created so far, in creation order
        b = ProblemBuilder()
        self.its = synth.build_catalog(b, synth.FAKE_PROFILES, ZONES, spot=False,
                                       prices=synth.price_table(synth.FAKE_PROFILES))
        self.first_type = None

    def make_pods(self, w, first=0, count=None):
        out = []
        count = w["replicas"] if count is None else count
        for r in range(first, first + count):
            anti = [dict(a, selector={"labels": {"app": w["app"]}}) for a in w.get("anti_affinity", [])]
            sp = w.get("spread")
            spreads = [dict(sp, selector={"labels": {"app": w["app"]}}, node_affinity_policy="Ignore")] if sp else []
            req_terms = []
            if w.get("node_affinity_first_node_type"):
                req_terms = [[(IT, "In", [self.first_type])]]
            sel = w.get("node_selector", {"karpenter.sh/nodepool": NP})
            tols = [tuple(t) for t in w.get("tolerations", [])]
            out.append(dict(uid=f"{w['app']}-{r:02d}", app=w["app"], cpu=w["cpu_m"], mem=w["memory_mi"] * MI * 1000,
                            anti=anti, spreads=spreads, req_terms=req_terms, ts=len(self.pods) + len(out),
                            sel=sel, tols=tols))
        return out

    def _add(self, b, p, node=None):
        kw = dict(node_selector=p["sel"], required_terms=p["req_terms"], tolerations=p["tols"],
                  labels={"app": p["app"], "test": "e2e"}, anti_affinity=p["anti"], spreads=p["spreads"])
        req = {"cpu": p["cpu"], "memory": p["mem"], "pods": 1000}
        ts = 1_700_000_000_000_000_000 + p["ts"] * 1_000_000_000
        if node is None:
            b.add_pod(p["uid"], ts, req, **kw)
        else:
            b.add_bound_pod(node, p["uid"], ts, req, **kw)

    def problem(self, pending):
        b = ProblemBuilder()
        synth.build_catalog(b, synth.FAKE_PROFILES, ZONES, spot=False, prices=synth.price_table(synth.FAKE_PROFILES))
        npd = self.sc["nodepool"]
        taints = [tuple(t) for t in npd.get("taints", [])]
        startup = [tuple(t) for t in npd.get("startup_taints", [])]
        b.add_nodepool(NP, requirements=[tuple(r) for r in npd["requirements"]], labels=npd.get("labels"),
                       taints=taints)
        for k, n in enumerate(self.nodes):
            it = self.its[n["it"]]
            # a launched node carries the template's labels and taints (NodeClaimTemplate.ToNodeClaim)
            labels = dict(npd.get("labels") or {})
            labels.update({r[0]: r[2][0] for r in it.requirements})
            labels.update({Z: n["zone"], "karpenter.sh/capacity-type": "on-demand", "karpenter.sh/nodepool": NP,
                           H: n["name"]})
            alloc = {r: it.capacity[r] - it.overhead.get(r, 0) for r in it.capacity}
            used = {"cpu": sum(p["cpu"] for p in n["pods"]), "memory": sum(p["mem"] for p in n["pods"]),
                    "pods": 1000 * len(n["pods"])}
            # karpenter launched it: its NodeClaim carries the template's taints and startup taints
            b.add_node(n["name"], labels, {r: alloc[r] - used.get(r, 0) for r in alloc},
                       taints=n.get("node_taints", taints), initialized=n.get("initialized", True), managed=True,
                       claim_taints=taints, startup_taints=startup)
        for k, n in enumerate(self.nodes):
            for p in n["pods"]:
                self._add(b, p, node=k)
        for p in pending:
            self._add(b, p)
        return b.build()

    def launch(self, res, pending, **node):
        """NodeClaims become nodes (Create: the first compatible type in
        catalog order, the first allowed zone); placed pods become bound.
        node: initialized / node_taints of the new nodes (default: ready,
        carrying the template's taints)"""
        for k, pods in enumerate(res["nodes"]):
            self.nodes[k]["pods"].extend(pending[i] for i in pods)
        for c in res["claims"]:
            it = min(c["its"])
            self.nodes.append(dict(name=f"launched-{len(self.nodes):02d}", it=it, zone=zones_of(c)[0],
                                   pods=[pending[i] for i in c["pods"]], **node))
            if self.first_type is None:
                self.first_type = self.its[it].name
        self.pods.extend(pending)
        return [pending[i] for i in res["errors"]]


def _solve_all(problem, solvers):
    st, want, _ = pyoracle.solve(problem)
    assert st == abi.GS_OK
    if solvers:
        from test_gpu_parity import _diff
        for s in solvers:
            got, _ = s.solve(problem)
            d = _diff(got, want)
            assert d is None, d
    return want


def run_scenario(sc, solvers=(), consolidator=None):
    """replays the scenario; returns (cluster, last result, last pending)"""
    cl = Cluster(sc)
    cl.steps = {}
    arrival = sc["arrival"]
    res, pending, errors = None, [], []
    if arrival == "startup":
        # the pod, its NodeClaim launched as a node that is still initializing
        # (Node.Spec.Taints: the startup taints and not-ready); then a second
        # workload while it initializes, and again once it is initialized
        # with one startup taint still on it
        w0, w1 = sc["workloads"]
        startup = [tuple(t) for t in sc["nodepool"]["startup_taints"]]
        pending = cl.make_pods(w0)
        res = _solve_all(cl.problem(pending), solvers)
        cl.steps["first"] = (res, pending)
        cl.launch(res, pending, initialized=False, node_taints=startup + [("node.kubernetes.io/not-ready", "", "NoSchedule")])
        pending = cl.make_pods(w1)
        res = _solve_all(cl.problem(pending), solvers)
        cl.steps["initializing"] = (res, pending)
        for n in cl.nodes:
            n.update(initialized=True, node_taints=[("example.com/initializing", "true", "NoSchedule")])
        res = _solve_all(cl.problem(pending), solvers)
        cl.steps["initialized"] = (res, pending)
    elif arrival == "together":
        pending = [p for w in sc["workloads"] for p in cl.make_pods(w)]
        res = _solve_all(cl.problem(pending), solvers)
    elif arrival == "one_by_one":
        for w in sc["workloads"]:
            for r in range(w["replicas"]):
                pending = errors + cl.make_pods(w, first=r, count=1)
                res = _solve_all(cl.problem(pending), solvers)
                errors = cl.launch(res, pending)
    elif arrival == "scale":  # the replicas together, launched; then the Deployment scales up
        for w in sc["workloads"]:
            pending = cl.make_pods(w)
            res = _solve_all(cl.problem(pending), solvers)
            errors = cl.launch(res, pending)
            pending = errors + cl.make_pods(w, first=w["replicas"], count=sc["scale_to"] - w["replicas"])
            res = _solve_all(cl.problem(pending), solvers)
            errors = cl.launch(res, pending)
    else:  # by_workload: each deployment after the previous one launched
        for w in sc["workloads"]:
            pending = cl.make_pods(w)
            res = _solve_all(cl.problem(pending), solvers)
            errors = cl.launch(res, pending)
    return cl, res, pending


def _app_claims(res, pending, app):
    return [c for c in res["claims"] if any(pending[i]["app"] == app for i in c["pods"])]


def check_expectation(sc, cl, res, pending, consolidator=None):
    e = sc["expect"]
    app = e["app"]
    if e["kind"] == "distinct_nodeclaims":
        assert not res["errors"]
        claims = _app_claims(res, pending, app)
        assert len(claims) == e["n"]
        assert all(sum(pending[i]["app"] == app for i in c["pods"]) == 1 for c in claims)
    elif e["kind"] == "instance_type_is_first_node_type":
        assert not res["errors"]
        names = {k: cl.its[k].name for k in range(len(cl.its))}
        for k, pods in enumerate(res["nodes"]):
            if any(pending[i]["app"] == app for i in pods):
                assert names[cl.nodes[k]["it"]] == cl.first_type
        for c in _app_claims(res, pending, app):
            assert [names[i] for i in c["its"]] == [cl.first_type]
        placed = sum(len(c["pods"]) for c in res["claims"]) + sum(len(p) for p in res["nodes"])
        assert placed == len(pending)
    elif e["kind"] == "zone_skew":
        assert not res["errors"]
        count = {z: 0 for z in ZONES}
        for c in _app_claims(res, pending, app):
            zs = zones_of(c)
            assert len(zs) == 1
            count[zs[0]] += sum(pending[i]["app"] == app for i in c["pods"])
        used = [v for v in count.values() if v]
        assert len(used) >= e["min_zones"]
        assert max(count.values()) - min(count.values()) <= e["max_skew"]
    elif e["kind"] == "min_zones":
        zones = {n["zone"] for n in cl.nodes if any(p["app"] == app for p in n["pods"])}
        assert len(zones) >= e["min_zones"]
        if "placed" in e:
            assert sum(p["app"] == app for n in cl.nodes for p in n["pods"]) == e["placed"]
    elif e["kind"] == "taint_split":
        # by_workload: the tolerant deployment launched a node of the tainted pool; the
        # intolerant pod was solved last (res/pending) and found no NodePool or node
        tol_nodes = [n for n in cl.nodes if any(p["app"] == app for p in n["pods"])]
        assert len(tol_nodes) == 1
        assert [pending[i]["app"] for i in res["errors"]] == [e["pending_app"]]
        assert not res["claims"] and not any(res["nodes"])
    elif e["kind"] == "types_within_allowed":
        assert not res["errors"]
        claims = _app_claims(res, pending, app)
        assert len(claims) == e["n"]
        names = [cl.its[k].name for k in range(len(cl.its))]
        allowed = set(e["allowed"])
        for c in claims:
            assert c["its"] and {names[i] for i in c["its"]} <= allowed
            lines = {ln.split("|")[0]: ln.split("|") for ln in c["requirements"].split("\n") if ln}
            for key, op, vals in sc["nodepool"]["requirements"]:
                if key == IT:
                    continue  # FinalizeScheduling rewrites it as the ordered options
                assert lines[key][1] == op and set(lines[key][2].split(",")) <= set(vals), (key, lines.get(key))
    elif e["kind"] == "multi_node_then_consolidate":
        assert not res["errors"]
        assert len(_app_claims(res, pending, app)) >= e["min_nodes"]
        cl.launch(res, pending)
        # the Deployment scales down: the newest replicas go
        keep = {p["uid"] for p in sorted(cl.pods, key=lambda p: p["ts"])[: e["scale_to"]]}
        for n in cl.nodes:
            n["pods"] = [p for p in n["pods"] if p["uid"] in keep]
        p = cl.problem([])
        cin = ConsolidationInput(p, list(range(len(cl.nodes))), mode=abi.CONSOLIDATE_SINGLE)
        st, cmds, chosen, _ = pyoracle.consolidate(cin)
        assert st == abi.GS_OK
        empty = [k for k, n in enumerate(cl.nodes) if not n["pods"]]
        assert empty and all(cmds[k]["decision"] == abi.DECISION_DELETE for k in empty)
        assert chosen >= 0 and cmds[chosen]["decision"] == abi.DECISION_DELETE
        if consolidator is not None:
            got, gchosen, _, _ = consolidator.consolidate(cin)
            assert (got, gchosen) == (cmds, chosen)
            mcin = ConsolidationInput(p, list(range(len(cl.nodes))), mode=abi.CONSOLIDATE_MULTI)
            st, mw, mc, mm = pyoracle.consolidate(mcin)
            assert st == abi.GS_OK
            g, gc, gm, _ = consolidator.consolidate(mcin)
            assert (g, gc, gm) == (mw, mc, mm)
    elif e["kind"] == "startup_taints":
        first, fp = cl.steps["first"]
        assert not first["errors"] and not any(first["nodes"])
        claims = _app_claims(first, fp, app)
        assert len(claims) == 1 and claims[0]["nodepool"] == 0
        res1, p1 = cl.steps["initializing"]
        assert not res1["errors"] and not res1["claims"]
        assert res1["nodes"] == [[0]] and p1[0]["app"] == e["followup_app"]
        res2, _ = cl.steps["initialized"]
        assert not res2["errors"] and res2["nodes"] == [[]] and len(res2["claims"]) == 1
    elif e["kind"] == "taint_values":
        assert [pending[i]["app"] for i in res["errors"]] == [e["pending_app"]]
        for a in (app, e["relaxed_app"]):
            cs = _app_claims(res, pending, a)
            assert len(cs) == 1 and cs[0]["nodepool"] == 0
    else:
        raise AssertionError(e["kind"])


IDS = [s["id"] for s in GOLD["scenarios"]]


@pytest.mark.parametrize("k", range(len(IDS)), ids=IDS)
def test_scenario_on_oracle(k):
    sc = GOLD["scenarios"][k]
    cl, res, pending = run_scenario(sc)
    check_expectation(sc, cl, res, pending)


def test_fixture_is_current():
    """the committed JSON is what make_e2e_scenarios.py writes"""
    import importlib.util
    spec = importlib.util.spec_from_file_location("mk", os.path.join(HERE, "golden", "make_e2e_scenarios.py"))
    mk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mk)
    assert json.loads(json.dumps({"zones": mk.ZONES, "scenarios": mk.SCENARIOS})) == GOLD


# ------------------------------------------------------------------- GPU
@pytest.fixture(scope="module")
def solvers():
    from gpusched.lib import Solver
    ss = [Solver(0), Solver(0, abi.GS_CFG_BLOCK_SOLVE)]
    yield ss
    for s in ss:
        s.close()


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(len(IDS)), ids=IDS)
def test_scenario_on_gpu(solvers, k):
    sc = GOLD["scenarios"][k]
    cl, res, pending = run_scenario(sc, solvers=solvers)
    check_expectation(sc, cl, res, pending, consolidator=solvers[0])

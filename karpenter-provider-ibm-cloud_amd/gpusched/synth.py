"""Deterministic synthetic Solve inputs for the BASELINE configs.

C1  500 pods, the 8 fake IBM profiles (reference pkg/fake/zz_generated_ibm_test_data.go:27-243),
    us-south-1..3, on-demand only, 1 NodePool like examples/nodepool.yaml
C2  10k pods x ~200 synthetic profiles x 3 zones x {on-demand, spot}
CM  100k pods x the C2 catalog (BASELINE metric workload)
C3  50k pods, 4 weighted NodePools, taints/tolerations, node affinity (In/NotIn),
    preferred affinity (topology spread is not supported yet and is omitted)
C5  200k pods x 2,000 synthetic ITs x 6 zones x 2 capacity types
random_problem(seed): small adversarial problems exercising the full
    requirement algebra (complements, Gt/Lt, custom keys), limits, relaxation,
    existing nodes.
"""
import uuid

import numpy as np

from . import catalog as cat
from .problem import ProblemBuilder

GI = 1 << 30
MI = 1 << 20

FAKE_PROFILES = [  # name, vcpu, memory GiB, gpu (pkg/fake/zz_generated_ibm_test_data.go:27-243)
    ("bx2-2x8", 2, 8, None), ("bx2-4x16", 4, 16, None), ("bx2-8x32", 8, 32, None),
    ("cx2-2x4", 2, 4, None), ("cx2-4x8", 4, 8, None),
    ("mx2-2x16", 2, 16, None), ("mx2-4x32", 4, 32, None),
    ("gx2-8x64x1v100", 8, 64, 1),
]
FAKE_ZONES = ["us-south-1", "us-south-2", "us-south-3"]  # zz_generated_ibm_test_data.go:286-314

FAMILIES = ["bx2", "bx3d", "cx2", "cx3d", "mx2", "mx3d", "ux2d", "vx2d", "ox2", "gx2", "gx3"]  # webhook :333
MEM_RATIO = {"b": 4, "c": 2, "m": 8, "o": 8, "v": 14, "u": 28, "g": 8}

CPU_CHOICES = np.array([100, 250, 500, 1000, 2000], dtype=np.int64)
CPU_W = np.array([30, 30, 20, 15, 5], dtype=np.float64)
MEM_CHOICES = np.array([128 * MI, 256 * MI, 512 * MI, 1 * GI, 2 * GI, 4 * GI], dtype=np.int64) * 1000


def price_table(profiles):
    """committed synthetic price table: 0.0475/vCPU + 0.006/GiB + 1.25/GPU (4 dp)"""
    out = {}
    for name, v, m, g in profiles:
        out[name] = round(0.0475 * v + 0.006 * m + 1.25 * (g or 0), 4)
    return out


def c2_profiles(n_target=200):
    sizes = [2, 4, 8, 16, 24, 32, 48, 64, 80, 96, 112, 128, 144, 160, 176, 192, 208, 224]
    out = []
    for fam in FAMILIES:
        ratio = MEM_RATIO[fam[0]]
        for v in sizes:
            m = v * ratio
            if fam.startswith("g"):
                g = max(1, v // 16)
                out.append((f"{fam}-{v}x{m}x{g}v100", v, m, g))
            else:
                out.append((f"{fam}-{v}x{m}", v, m, None))
            if len(out) >= n_target:
                return out
    return out


def c5_profiles(n_target=2000):
    fams = []
    for base in FAMILIES:
        for suf in ["", "a", "b", "c", "e", "f", "h", "i", "k", "l", "n", "p", "q", "r", "s", "t", "w", "y"]:
            fams.append(base + suf)
    sizes = [2, 4, 6, 8, 12, 16, 20, 24, 32, 40, 48, 56, 64, 72, 80, 96, 112, 128, 144, 160, 176]
    out = []
    for fam in fams:
        ratio = MEM_RATIO[fam[0]]
        for v in sizes:
            m = v * ratio
            if fam.startswith("g"):
                g = max(1, v // 16)
                out.append((f"{fam}-{v}x{m}x{g}v100", v, m, g))
            else:
                out.append((f"{fam}-{v}x{m}", v, m, None))
            if len(out) >= n_target:
                return out
    return out


def build_catalog(b: ProblemBuilder, profiles, zones, spot, prices, rng=None, unavailable_frac=0.0,
                  missing_price=()):
    unavailable = set()
    if rng is not None and unavailable_frac > 0:
        for name, *_ in profiles:
            for z in zones:
                for ct in (["on-demand", "spot"] if spot else ["on-demand"]):
                    if rng.random() < unavailable_frac:
                        unavailable.add(f"{name}:{z}:{ct}")
    ac = ("enum", ["standard", "spot"]) if spot else None
    profs = [cat.Profile(name, v, m, "amd64", g, ac) for name, v, m, g in profiles]

    def price_of(name, zone):
        if name in missing_price:
            return None
        return prices.get(name)

    its = cat.list_instance_types(profs, zones, price_of, unavailable=unavailable)
    for it in its:
        b.add_instance_type(it.name, it.requirements, it.capacity, it.overhead, it.offerings)
    return its


def _uid(rng):
    return str(uuid.UUID(bytes=rng.bytes(16), version=4))


def _pods_basic(b, rng, n, its, gpu_frac=0.0, selector_frac=0.0):
    cpu = rng.choice(CPU_CHOICES, size=n, p=CPU_W / CPU_W.sum())
    mem = rng.choice(MEM_CHOICES, size=n)
    ts = 1_700_000_000_000_000_000 + rng.integers(0, 8, size=n) * 1_000_000_000
    fams = sorted({cat.instance_family(it.name) for it in its})
    sizes = sorted({cat.instance_size(it.name) for it in its})
    for i in range(n):
        req = {"cpu": int(cpu[i]), "memory": int(mem[i]), "pods": 1000}
        if gpu_frac and rng.random() < gpu_frac:
            req["nvidia.com/gpu"] = 1000
        sel = {}
        if selector_frac and rng.random() < selector_frac:
            k = rng.integers(0, 3)
            if k == 0:
                sel["kubernetes.io/arch"] = "amd64"
            elif k == 1:
                sel["karpenter-ibm.sh/instance-family"] = fams[rng.integers(0, len(fams))]
            else:
                sel["karpenter-ibm.sh/instance-size"] = sizes[rng.integers(0, len(sizes))]
        b.add_pod(_uid(rng), int(ts[i]), req, node_selector=sel)


def make_c1(n_pods=500, seed=0x5EED0001):
    rng = np.random.default_rng(seed)
    b = ProblemBuilder()
    prices = price_table(FAKE_PROFILES)
    prices.pop("gx2-8x64x1v100")  # no price -> 0.0 (instancetype.go:753)
    its = build_catalog(b, FAKE_PROFILES, FAKE_ZONES, spot=False, prices=prices)
    b.add_nodepool("default", weight=100,
                   requirements=[("kubernetes.io/arch", "In", ["amd64"]), ("kubernetes.io/os", "In", ["linux"])])
    _pods_basic(b, rng, n_pods, its)
    return b.build()


def make_c2(n_pods=10_000, seed=0x5EED0002, n_its=200):
    rng = np.random.default_rng(seed)
    b = ProblemBuilder()
    profs = c2_profiles(n_its)
    its = build_catalog(b, profs, FAKE_ZONES, spot=True, prices=price_table(profs), rng=rng,
                        unavailable_frac=0.02)
    b.add_nodepool("default", weight=0,
                   requirements=[("kubernetes.io/arch", "In", ["amd64"]), ("kubernetes.io/os", "In", ["linux"])],
                   daemon={"cpu": 200, "memory": 256 * MI * 1000, "pods": 2000})
    _pods_basic(b, rng, n_pods, its, gpu_frac=0.01, selector_frac=0.10)
    return b.build()


def make_cm(n_pods=100_000, seed=0x5EED0006):
    return make_c2(n_pods=n_pods, seed=seed)


def make_c5(n_pods=200_000, seed=0x5EED0005, n_its=2000):
    rng = np.random.default_rng(seed)
    b = ProblemBuilder()
    profs = c5_profiles(n_its)
    zones = [f"us-south-{i}" for i in range(1, 7)]
    its = build_catalog(b, profs, zones, spot=True, prices=price_table(profs), rng=rng, unavailable_frac=0.02)
    b.add_nodepool("default", weight=0, requirements=[("kubernetes.io/arch", "In", ["amd64"])],
                   daemon={"cpu": 200, "memory": 256 * MI * 1000, "pods": 2000})
    _pods_basic(b, rng, n_pods, its, gpu_frac=0.01, selector_frac=0.10)
    return b.build()


APPS = ["web", "api", "batch", "cache"]


def make_c3(n_pods=50_000, seed=0x5EED0003, spread_frac=0.2):
    """C3: 4 weighted NodePools, taints/tolerations, required node affinity
    (In/NotIn), preferred affinity and a `spread_frac` share of pods with a
    zone topology spread (maxSkew 1 on their app label, ScheduleAnyway on half)"""
    rng = np.random.default_rng(seed)
    b = ProblemBuilder()
    profs = c2_profiles(200)
    its = build_catalog(b, profs, FAKE_ZONES, spot=True, prices=price_table(profs), rng=rng,
                        unavailable_frac=0.02)
    fams = sorted({cat.instance_family(it.name) for it in its})
    daemon = {"cpu": 200, "memory": 256 * MI * 1000, "pods": 2000}
    b.add_nodepool("gpu", weight=100, requirements=[("karpenter-ibm.sh/instance-family", "In", ["gx2", "gx3"])],
                   taints=[("nvidia.com/gpu", "true", "NoSchedule")], daemon=daemon)
    b.add_nodepool("spot", weight=50, requirements=[("karpenter.sh/capacity-type", "In", ["spot"]),
                                                    ("karpenter-ibm.sh/instance-family", "NotIn", ["gx2", "gx3"])],
                   taints=[("spot", "true", "NoSchedule")], daemon=daemon)
    b.add_nodepool("memory", weight=10, requirements=[("karpenter-ibm.sh/instance-family", "In",
                                                       ["mx2", "mx3d", "ux2d", "vx2d", "ox2"])],
                   labels={"tier": "memory"}, daemon=daemon, limits={"cpu": 4000 * 1000})
    b.add_nodepool("default", weight=0, requirements=[("karpenter.sh/capacity-type", "In", ["on-demand"]),
                                                      ("topology.kubernetes.io/zone", "In", FAKE_ZONES)],
                   daemon=daemon)
    cpu = rng.choice(CPU_CHOICES, size=n_pods, p=CPU_W / CPU_W.sum())
    mem = rng.choice(MEM_CHOICES, size=n_pods)
    ts = 1_700_000_000_000_000_000 + rng.integers(0, 8, size=n_pods) * 1_000_000_000
    for i in range(n_pods):
        req = {"cpu": int(cpu[i]), "memory": int(mem[i]), "pods": 1000}
        tols, required, preferred, sel = [], [], [], {}
        u = rng.random()
        if u < 0.02:
            req["nvidia.com/gpu"] = 1000
            tols.append(("nvidia.com/gpu", "Exists", "", "NoSchedule"))
        if rng.random() < 0.30:
            tols.append(("spot", "Equal", "true", "NoSchedule"))
        if rng.random() < 0.40:
            z = FAKE_ZONES[rng.integers(0, 3)]
            f = fams[rng.integers(0, len(fams))]
            kind = rng.integers(0, 3)
            if kind == 0:
                required.append([("topology.kubernetes.io/zone", "In", [z])])
            elif kind == 1:
                required.append([("karpenter-ibm.sh/instance-family", "NotIn", [f])])
            else:
                required.append([("topology.kubernetes.io/zone", "NotIn", [z]),
                                 ("karpenter-ibm.sh/instance-family", "In", [f, fams[rng.integers(0, len(fams))]])])
                required.append([("topology.kubernetes.io/zone", "In", [z])])
        if rng.random() < 0.10:
            preferred.append((int(rng.integers(1, 100)),
                              [("karpenter.sh/capacity-type", "In", ["spot"])]))
            if rng.random() < 0.5:
                preferred.append((int(rng.integers(1, 100)), [("tier", "In", ["memory"])]))
        if rng.random() < 0.03:
            sel["tier"] = "memory"
        app = APPS[rng.integers(0, len(APPS))]
        spreads = []
        if rng.random() < spread_frac and not required and not sel:
            spreads.append({"key": "topology.kubernetes.io/zone", "max_skew": 1,
                            "when": "ScheduleAnyway" if rng.random() < 0.5 else "DoNotSchedule",
                            "selector": {"labels": {"app": app}}})
        b.add_pod(_uid(rng), int(ts[i]), req, node_selector=sel, required_terms=required,
                  preferred_terms=preferred, tolerations=tols, labels={"app": app}, spreads=spreads)
    return b.build()


CONFIGS = {"C1": make_c1, "C2": make_c2, "CM": make_cm, "C3": make_c3, "C5": make_c5}


# ---------------------------------------------------------------- fuzzing
_KEYS_IT = ["node.kubernetes.io/instance-type", "kubernetes.io/arch", "karpenter-ibm.sh/instance-family",
            "karpenter-ibm.sh/instance-size"]
_KEYS_OFF = ["topology.kubernetes.io/zone", "karpenter.sh/capacity-type"]
_KEYS_FREE = ["kubernetes.io/os", "karpenter.sh/nodepool", "team", "karpenter-ibm.sh/instance-cpu",
              "kubernetes.io/hostname", "tier"]


def random_problem(seed, n_pods=None, with_nodes=True, with_limits=True, free_values=3, inflight=False,
                   partial_labels=False):
    """small adversarial problem over the whole supported feature set;
    free_values > 3 widens the custom (free) keys team / tier to that many
    values (tier's integers then reach free_values - 1 for Gt / Lt);
    inflight: the existing nodes are karpenter-launched ones, some still
    initializing, with startup / ephemeral taints (inflight_node);
    partial_labels: nodes may lack instance-type / zone / capacity-type labels
    (nodes karpenter did not launch, drop_node_labels)"""
    rng = np.random.default_rng(seed)
    b = ProblemBuilder()
    zones = ["z1", "z2", "z3"][: int(rng.integers(1, 4))]
    fams = ["bx2", "cx2", "mx2"]
    profs = []
    for i in range(int(rng.integers(2, 9))):
        f = fams[rng.integers(0, 3)]
        v = int(rng.choice([2, 4, 8, 16]))
        m = v * MEM_RATIO[f[0]] if rng.random() < 0.8 else 2
        g = 1 if rng.random() < 0.15 else None
        profs.append((f"{f}-{v}x{m}" + (f"x{i}" if rng.random() < 0.3 else ""), v, m, g))
    seen = set()
    profs = [p for p in profs if not (p[0] in seen or seen.add(p[0]))]
    prices = {p[0]: float(rng.choice([0.1, 0.2, 0.2, 0.4, 0.8])) for p in profs}
    spot = bool(rng.random() < 0.6)
    its = build_catalog(b, profs, zones, spot=spot, prices=prices, rng=rng, unavailable_frac=0.15,
                        missing_price={profs[0][0]} if rng.random() < 0.2 else ())
    names = [it.name for it in its]
    vocab = {
        "node.kubernetes.io/instance-type": names + ["nope"],
        "kubernetes.io/arch": ["amd64", "arm64"],
        "karpenter-ibm.sh/instance-family": fams + ["gx2"],
        "karpenter-ibm.sh/instance-size": sorted({cat.instance_size(n) for n in names}),
        "topology.kubernetes.io/zone": zones + ["z9"],
        "karpenter.sh/capacity-type": ["on-demand", "spot"],
        "kubernetes.io/os": ["linux", "windows"],
        "karpenter.sh/nodepool": ["np0", "np1", "np2"],
        "team": ["a", "b", "c"] if free_values <= 3 else [f"t{i:03d}" for i in range(free_values)],
        "karpenter-ibm.sh/instance-cpu": ["2", "4", "8", "x"],
        "kubernetes.io/hostname": ["host-a", "host-b"],
        "tier": ["1", "2", "3"] if free_values <= 3 else [str(i) for i in range(free_values)],
    }
    nteam = len(vocab["team"])
    bound_hi = 10 if free_values <= 3 else free_values
    all_keys = _KEYS_IT + _KEYS_OFF + _KEYS_FREE

    def rand_req(keys=all_keys):
        k = keys[rng.integers(0, len(keys))]
        vals = vocab[k]
        op = rng.choice(["In", "In", "In", "NotIn", "Exists", "DoesNotExist", "Gt", "Lt"],
                        p=[0.3, 0.1, 0.1, 0.2, 0.1, 0.05, 0.075, 0.075])
        if op in ("Gt", "Lt"):
            if rng.random() < 0.4:
                op = op + "e"  # Gte / Lte
            return (k, op, [str(int(rng.integers(0, bound_hi)))])
        if op in ("Exists", "DoesNotExist"):
            return (k, op, [])
        n = int(rng.integers(1, min(3, len(vals)) + 1))
        return (k, op, list(rng.choice(vals, size=n, replace=False)))

    effects = ["NoSchedule", "PreferNoSchedule", "NoExecute"]
    n_np = int(rng.integers(1, 4))
    np_taints = []
    for j in range(n_np):
        reqs = [rand_req(_KEYS_IT + _KEYS_OFF + ["kubernetes.io/os", "team"]) for _ in range(int(rng.integers(0, 3)))]
        labels = {"team": vocab["team"][rng.integers(0, nteam)]} if rng.random() < 0.4 else {}
        taints = [("dedicated", str(rng.choice(["x", "y"])), str(rng.choice(effects)))] if rng.random() < 0.4 else []
        np_taints.append(taints)
        limits = None
        if with_limits and rng.random() < 0.3:
            limits = {"cpu": int(rng.choice([8, 16, 32, 64])) * 1000}
        daemon = {"cpu": int(rng.choice([0, 100, 500])), "pods": int(rng.integers(0, 3)) * 1000}
        b.add_nodepool(f"np{j}", weight=int(rng.choice([0, 10, 10, 50])), requirements=reqs, labels=labels,
                       taints=taints, limits=limits, daemon=daemon)
    if with_nodes and rng.random() < 0.5:
        for k in range(int(rng.integers(1, 4))):
            it = its[rng.integers(0, len(its))]
            labels = {r[0]: r[2][0] for r in it.requirements}
            labels["topology.kubernetes.io/zone"] = zones[rng.integers(0, len(zones))]
            labels["karpenter.sh/capacity-type"] = "on-demand"
            labels["kubernetes.io/hostname"] = f"node-{k}"
            if rng.random() < 0.5:
                labels["team"] = vocab["team"][rng.integers(0, nteam)]
            avail = {"cpu": int(rng.choice([500, 1000, 4000])), "memory": int(rng.choice([1, 4, 16])) * GI * 1000,
                     "pods": 10_000}
            if partial_labels:
                drop_node_labels(rng, labels)
            if inflight:
                b.add_node(f"node-{k}", labels, avail, **inflight_node(rng, np_taints[rng.integers(0, n_np)]))
            else:
                taints = [("dedicated", "x", "NoSchedule")] if rng.random() < 0.3 else []
                b.add_node(f"node-{k}", labels, avail, taints=taints, initialized=bool(rng.random() < 0.8))
    n = int(n_pods if n_pods is not None else rng.integers(1, 40))
    for i in range(n):
        req = {"cpu": int(rng.choice([100, 500, 1000, 3000, 9000])),
               "memory": int(rng.choice([128 * MI, GI, 4 * GI, 30 * GI])) * 1000, "pods": 1000}
        if rng.random() < 0.1:
            req["nvidia.com/gpu"] = 1000
        if rng.random() < 0.05:
            req["example.com/widget"] = 1000
        sel = {}
        if rng.random() < 0.2:
            k = all_keys[rng.integers(0, len(all_keys))]
            sel[k] = str(rng.choice(vocab[k]))
        required = [[rand_req() for _ in range(int(rng.integers(1, 3)))] for _ in range(int(rng.integers(0, 3)))] \
            if rng.random() < 0.4 else []
        preferred = [(int(rng.integers(1, 4)), [rand_req()]) for _ in range(int(rng.integers(0, 3)))] \
            if rng.random() < 0.3 else []
        tols = []
        if rng.random() < 0.4:
            tols.append(("dedicated", str(rng.choice(["Equal", "Exists"])), str(rng.choice(["x", "y"])),
                         str(rng.choice(effects + [""]))))
        if rng.random() < 0.1:
            tols.append(("", "Exists", "", ""))
        if inflight and rng.random() < 0.3:
            tols.append(("example.com/initializing", str(rng.choice(["Equal", "Exists"])), "true", "NoSchedule"))
        b.add_pod(_uid(rng), 1_700_000_000_000_000_000 + int(rng.integers(0, 4)) * 1_000_000_000, req,
                  node_selector=sel, required_terms=required, preferred_terms=preferred, tolerations=tols)
    return b.build()


PARTIAL_LABEL_KEYS = ["karpenter-ibm.sh/instance-family", "karpenter-ibm.sh/instance-size", "kubernetes.io/arch",
                      "karpenter.sh/capacity-type", "node.kubernetes.io/instance-type", "topology.kubernetes.io/zone"]


def drop_node_labels(rng, labels, p=0.6):
    """a node karpenter did not launch (no karpenter-ibm.sh/* labels, labels.go:37-45) or
    without some well-known label: drops a random subset of those keys, in place"""
    if rng.random() < p:
        for k in PARTIAL_LABEL_KEYS:
            if k in labels and rng.random() < 0.4:
                del labels[k]
    return labels


# NodeClaim spec.startupTaints seen on in-flight nodes (e.g. NodePool
# startupTaints, reference test/e2e/e2e_taints_test.go:105-115) and the taints
# a registering node carries (<U> scheduling.KnownEphemeralTaints)
STARTUP_TAINTS = [("example.com/initializing", "true", "NoSchedule"), ("node.kubernetes.io/not-ready", "", "NoSchedule"),
                  ("cilium.io/agent-not-ready", "true", "NoExecute")]
EPHEMERAL_TAINTS = [("node.kubernetes.io/not-ready", "", "NoSchedule"), ("node.kubernetes.io/unreachable", "", "NoSchedule"),
                    ("node.cloudprovider.kubernetes.io/uninitialized", "true", "NoSchedule"),
                    ("karpenter.sh/unregistered", "", "NoExecute")]


def inflight_node(rng, claim_taints):
    """add_node keyword arguments of a state node as the cluster state holds
    it: karpenter-launched (managed) or not, initialized or not, its
    Node.Spec.Taints (the NodeClaim's taints, startup taints and ephemeral
    ones while it registers; a startup taint that came back after
    initialization) and its NodeClaim's taints / startup taints"""
    managed = bool(rng.random() < 0.8)
    initialized = bool(rng.random() < 0.5)
    startup = [t for t in STARTUP_TAINTS if rng.random() < 0.5] if managed else []
    node_taints = list(claim_taints) if managed else []
    if not initialized:
        node_taints += startup + [t for t in EPHEMERAL_TAINTS if rng.random() < 0.4]
    elif startup and rng.random() < 0.3:
        node_taints.append(startup[0])
    if rng.random() < 0.2:
        node_taints.append(EPHEMERAL_TAINTS[int(rng.integers(0, len(EPHEMERAL_TAINTS)))])
    if rng.random() < 0.2:
        node_taints.append(("dedicated", "x", "NoSchedule"))
    return dict(managed=managed, initialized=initialized, taints=node_taints,
                claim_taints=list(claim_taints) if managed else [], startup_taints=startup)


def make_c4_sim(n_nodes=500, n_pods=2000, seed=0x5EED0004):
    """one consolidation-style simulation (SURVEY §3.2 SimulateScheduling):
    existing nodes sampled from the C2 catalog at 60-90% cpu use, plus the
    pods of removed candidates to reschedule onto them or onto new NodeClaims"""
    rng = np.random.default_rng(seed)
    b = ProblemBuilder()
    profs = c2_profiles(200)
    its = build_catalog(b, profs, FAKE_ZONES, spot=True, prices=price_table(profs), rng=rng, unavailable_frac=0.02)
    daemon = {"cpu": 200, "memory": 256 * MI * 1000, "pods": 2000}
    b.add_nodepool("default", weight=0, requirements=[("kubernetes.io/arch", "In", ["amd64"]),
                                                      ("kubernetes.io/os", "In", ["linux"])], daemon=daemon)
    cand = [it for it in its if it.capacity["nvidia.com/gpu"] == 0 and it.capacity["cpu"] <= 32000]
    for k in range(n_nodes):
        it = cand[rng.integers(0, len(cand))]
        labels = {r[0]: r[2][0] for r in it.requirements}
        zone = FAKE_ZONES[rng.integers(0, 3)]
        ct = "spot" if rng.random() < 0.3 else "on-demand"
        labels.update({"topology.kubernetes.io/zone": zone, "karpenter.sh/capacity-type": ct,
                       "karpenter.sh/nodepool": "default", "kubernetes.io/os": "linux",
                       "kubernetes.io/hostname": f"node-{k:05d}"})
        alloc = {r: it.capacity[r] - it.overhead.get(r, 0) for r in it.capacity}
        used = float(rng.uniform(0.6, 0.9))
        avail = {"cpu": int(alloc["cpu"] * (1 - used)), "memory": int(alloc["memory"] * (1 - used)),
                 "pods": alloc["pods"] - int(rng.integers(10, 25)) * 1000, "nvidia.com/gpu": 0}
        b.add_node(f"node-{k:05d}", labels, avail, initialized=bool(rng.random() < 0.95))
    _pods_basic(b, rng, n_pods, its, gpu_frac=0.005, selector_frac=0.10)
    return b.build()


CONFIGS["C4sim"] = make_c4_sim


BIG_CPU = np.array([1000, 2000, 3000, 4000, 6000], dtype=np.int64)


def make_c4(n_nodes=5000, n_pending=0, seed=0x5EED0004, util=(0.6, 0.9), n_its=200, full_frac=0.15, big_frac=0.3,
            pack=False):
    """C4 consolidation cluster: state nodes sampled from the C2
    catalog in 2 NodePools, each carrying bound reschedulable pods that use
    `util` of its allocatable cpu (a `full_frac` share of nodes run at ~97 %;
    a `big_frac` share of nodes carry 1-6 vCPU pods),
    plus `n_pending` pending pods.  Node available = allocatable - daemon -
    bound pods (StateNode.Available).  pack=True keeps adding the node's
    smallest pod shape after the first misfit, so no node keeps room for
    another pod of its kind (consolidation then mixes Delete, Replace and
    NoOp)."""
    rng = np.random.default_rng(seed)
    b = ProblemBuilder()
    profs = c2_profiles(n_its)
    its = build_catalog(b, profs, FAKE_ZONES, spot=True, prices=price_table(profs), rng=rng, unavailable_frac=0.02)
    daemon = {"cpu": 200, "memory": 256 * MI * 1000, "pods": 2000}
    b.add_nodepool("general", weight=10, requirements=[("kubernetes.io/arch", "In", ["amd64"]),
                                                       ("kubernetes.io/os", "In", ["linux"])],
                   labels={"team": "general"}, daemon=daemon)
    b.add_nodepool("spot-batch", weight=0, requirements=[("karpenter.sh/capacity-type", "In", ["spot"])],
                   daemon=daemon)
    cand = [it for it in its if it.capacity["nvidia.com/gpu"] == 0 and it.capacity["cpu"] <= 32000]
    for k in range(n_nodes):
        it = cand[rng.integers(0, len(cand))]
        labels = {r[0]: r[2][0] for r in it.requirements}
        zone = FAKE_ZONES[rng.integers(0, 3)]
        pool = "spot-batch" if rng.random() < 0.25 else "general"
        ct = "spot" if pool == "spot-batch" or rng.random() < 0.2 else "on-demand"
        labels.update({"topology.kubernetes.io/zone": zone, "karpenter.sh/capacity-type": ct,
                       "karpenter.sh/nodepool": pool, "kubernetes.io/os": "linux",
                       "kubernetes.io/hostname": f"node-{k:05d}"})
        if pool == "general":
            labels["team"] = "general"
        alloc = {r: it.capacity[r] - it.overhead.get(r, 0) for r in it.capacity}
        target = float(rng.uniform(*util)) if rng.random() >= full_frac else 0.97
        used = {"cpu": daemon["cpu"], "memory": daemon["memory"], "pods": daemon["pods"]}
        ts = 1_700_000_000_000_000_000 + int(rng.integers(0, 8)) * 1_000_000_000
        big = rng.random() < big_frac
        while True:
            if big:
                cpu = int(rng.choice(BIG_CPU))
                mem = int(rng.choice(MEM_CHOICES[2:]))
            else:
                cpu = int(rng.choice(CPU_CHOICES, p=CPU_W / CPU_W.sum()))
                mem = int(rng.choice(MEM_CHOICES[:4]))
            if used["cpu"] + cpu > target * alloc["cpu"] or used["memory"] + mem > alloc["memory"] \
                    or used["pods"] + 1000 > alloc["pods"]:
                if not pack:
                    break
                cpu = int(min(BIG_CPU)) if big else int(min(CPU_CHOICES))
                mem = int(MEM_CHOICES[2]) if big else int(MEM_CHOICES[0])
                if used["cpu"] + cpu > target * alloc["cpu"] or used["memory"] + mem > alloc["memory"] \
                        or used["pods"] + 1000 > alloc["pods"]:
                    break
            used["cpu"] += cpu
            used["memory"] += mem
            used["pods"] += 1000
            b.add_bound_pod(k, _uid(rng), ts, {"cpu": cpu, "memory": mem, "pods": 1000})
        avail = {r: alloc[r] - used.get(r, 0) for r in alloc}
        b.add_node(f"node-{k:05d}", labels, avail, initialized=bool(rng.random() < 0.97))
    _pods_basic(b, rng, n_pending, its, gpu_frac=0.0, selector_frac=0.05)
    return b.build()


CONFIGS["C4"] = make_c4


def random_consolidation(seed, n_nodes=None, n_pending=None, inflight=False, partial_labels=False):
    """small adversarial consolidation cluster: nodes with taints, custom
    labels, spot/on-demand, uninitialized nodes and bound pods with
    selectors/tolerations; pending pods; 1-3 NodePools (taints, limits)"""
    rng = np.random.default_rng(seed)
    b = ProblemBuilder()
    zones = FAKE_ZONES[: int(rng.integers(1, 4))]
    profs = []
    for fam in ["bx2", "cx2", "mx2"]:
        for v in [2, 4, 8, 16]:
            if rng.random() < 0.6:
                profs.append((f"{fam}-{v}x{v * MEM_RATIO[fam[0]]}", v, v * MEM_RATIO[fam[0]], None))
    if len(profs) < 2:
        profs = [("bx2-2x8", 2, 8, None), ("bx2-8x32", 8, 32, None)]
    prices = {p[0]: round(float(rng.choice([0.05, 0.1, 0.1, 0.2, 0.4])) * p[1] / 2, 4) for p in profs}
    its = build_catalog(b, profs, zones, spot=True, prices=prices, rng=rng, unavailable_frac=0.1)
    effects = ["NoSchedule", "PreferNoSchedule"]
    n_np = int(rng.integers(1, 4))
    np_taints = []
    for j in range(n_np):
        reqs = []
        if rng.random() < 0.3:
            reqs.append(("karpenter.sh/capacity-type", "In", [str(rng.choice(["spot", "on-demand"]))]))
        if rng.random() < 0.2:
            reqs.append(("karpenter-ibm.sh/instance-family", "NotIn", ["mx2"]))
        taints = [("dedicated", "x", str(rng.choice(effects)))] if rng.random() < 0.3 else []
        np_taints.append(taints)
        limits = {"cpu": int(rng.choice([16, 64, 256])) * 1000} if rng.random() < 0.2 else None
        b.add_nodepool(f"np{j}", weight=int(rng.choice([0, 10, 50])), requirements=reqs,
                       labels={"team": str(rng.choice(["a", "b"]))} if rng.random() < 0.4 else {},
                       taints=taints, limits=limits, daemon={"cpu": 100, "pods": 1000})
    nn = int(n_nodes if n_nodes is not None else rng.integers(2, 16))
    for k in range(nn):
        it = its[rng.integers(0, len(its))]
        labels = {r[0]: r[2][0] for r in it.requirements}
        labels["topology.kubernetes.io/zone"] = zones[rng.integers(0, len(zones))]
        labels["karpenter.sh/capacity-type"] = str(rng.choice(["spot", "on-demand"]))
        labels["karpenter.sh/nodepool"] = f"np{rng.integers(0, n_np)}"
        labels["kubernetes.io/hostname"] = f"n-{k:03d}"
        if rng.random() < 0.4:
            labels["team"] = str(rng.choice(["a", "b"]))
        alloc = {r: it.capacity[r] - it.overhead.get(r, 0) for r in it.capacity}
        used = {"cpu": 100, "memory": 0, "pods": 1000}
        target = float(rng.uniform(0.3, 1.0))
        ts = 1_700_000_000_000_000_000 + int(rng.integers(0, 4)) * 1_000_000_000
        for _ in range(int(rng.integers(0, 12))):
            cpu = int(rng.choice([100, 250, 500, 1000, 2000, 4000]))
            mem = int(rng.choice([128 * MI, GI, 4 * GI])) * 1000
            if used["cpu"] + cpu > target * alloc["cpu"] or used["memory"] + mem > alloc["memory"]:
                break
            used["cpu"] += cpu
            used["memory"] += mem
            used["pods"] += 1000
            sel = {"team": labels["team"]} if "team" in labels and rng.random() < 0.3 else {}
            tols = [("dedicated", "Exists", "", "")] if rng.random() < 0.3 else []
            if inflight and rng.random() < 0.3:
                tols.append(("example.com/initializing", "Exists", "", ""))
            req_terms = []
            if partial_labels:
                r = rng.random()
                if r < 0.3:
                    req_terms = [[("karpenter-ibm.sh/instance-family", "NotIn", [str(rng.choice(["mx2", "gx2"]))])]]
                elif r < 0.4:
                    req_terms = [[("karpenter-ibm.sh/instance-size", "DoesNotExist", [])]]
                elif r < 0.5:
                    req_terms = [[("karpenter.sh/capacity-type", "NotIn", ["spot"])]]
                elif r < 0.6:
                    req_terms = [[("kubernetes.io/arch", "In", ["amd64"])]]
            b.add_bound_pod(k, _uid(rng), ts, {"cpu": cpu, "memory": mem, "pods": 1000}, node_selector=sel,
                            tolerations=tols, required_terms=req_terms)
        avail = {r: alloc[r] - used.get(r, 0) for r in alloc}
        if partial_labels:
            drop_node_labels(rng, labels)
        if inflight:
            b.add_node(f"n-{k:03d}", labels, avail, **inflight_node(rng, np_taints[int(labels["karpenter.sh/nodepool"][2:])]))
        else:
            taints = [("dedicated", "x", "NoSchedule")] if rng.random() < 0.15 else []
            b.add_node(f"n-{k:03d}", labels, avail, taints=taints, initialized=bool(rng.random() < 0.85))
    npend = int(n_pending if n_pending is not None else rng.choice([0, 0, 1, 3]))
    for i in range(npend):
        b.add_pod(_uid(rng), 1_700_000_000_000_000_000, {"cpu": int(rng.choice([100, 1000, 3000])),
                                                         "memory": int(GI) * 1000, "pods": 1000})
    return b.build()


def random_topology(seed, n_pods=None, taint_policy=None, affinity_policy="Ignore", multi_term=False,
                    domain_key="topology.kubernetes.io/zone", tol_by_app=False, pns_frac=0.3):
    """small adversarial topology-spread problems: zone / hostname spreads
    (DoNotSchedule and ScheduleAnyway, maxSkew 1-3, minDomains, matchLabels
    and matchExpressions selectors, nil selectors, nodeAffinityPolicy Ignore
    with node affinity), NodePools with and without zone requirements,
    existing nodes with labelled bound pods, taints and relaxation.
    taint_policy "Honor" / "Ignore": every pod with a spread tolerates the
    NodePools' taint and its spreads carry that nodeTaintsPolicy (the random
    stream is the same for both, so the two problems differ only in it).
    affinity_policy: the nodeAffinityPolicy of the spreads of pods with a
    (zone-only) required node-affinity term; multi_term: those spread owners
    carry two zone In terms instead (OR; relaxation drops the first).
    domain_key "karpenter.sh/capacity-type": the non-hostname spreads use
    that key, NodePools constrain it and nodes carry spot / on-demand (those
    draws come from their own stream).  tol_by_app (with taint_policy): each
    app's pods tolerate the NodePools' taint or not, as a whole, so Honor
    groups see intolerable NodePools and nodes; "karpenter.sh/nodepool": nodes carry
    NodePool labels (np0..np2, some of no NodePool of the problem; a node
    lacking the label beside multi-group owners is refused)"""
    rng = np.random.default_rng(seed)
    ctk = "karpenter.sh/capacity-type"
    cts = np.random.default_rng(seed + 0xC7) if domain_key == ctk else None
    nps = np.random.default_rng(seed + 0xD7) if domain_key == "karpenter.sh/nodepool" else None
    b = ProblemBuilder()
    zones = ["z1", "z2", "z3", "z4"][: int(rng.integers(2, 5))]
    profs = []
    for fam in ["bx2", "cx2", "mx2"]:
        for v in [2, 4, 8]:
            if rng.random() < 0.7:
                profs.append((f"{fam}-{v}x{v * MEM_RATIO[fam[0]]}", v, v * MEM_RATIO[fam[0]], None))
    if not profs:
        profs = [("bx2-4x16", 4, 16, None)]
    prices = {p_[0]: round(0.05 * p_[1] + 0.01 * float(rng.random()), 4) for p_ in profs}
    spot = bool(rng.random() < 0.5)
    its = build_catalog(b, profs, zones, spot=spot or cts is not None, prices=prices, rng=rng,
                        unavailable_frac=0.1)
    n_np = int(rng.integers(1, 3))
    for j in range(n_np):
        reqs = []
        if rng.random() < 0.7:
            zs = sorted(rng.choice(zones, size=int(rng.integers(1, len(zones) + 1)), replace=False).tolist())
            reqs.append(("topology.kubernetes.io/zone", "In", zs))
        if cts is not None and cts.random() < 0.8:
            reqs.append((ctk, "In", [["spot"], ["on-demand"], ["on-demand", "spot"]][int(cts.integers(0, 3))]))
        taints = [("dedicated", "x", "PreferNoSchedule")] if rng.random() < pns_frac else []
        limits = {"cpu": int(rng.choice([8, 32])) * 1000} if rng.random() < 0.2 else None
        b.add_nodepool(f"np{j}", weight=int(rng.choice([0, 10])), requirements=reqs, taints=taints, limits=limits,
                       daemon={"cpu": 100, "pods": 1000})
    nn = int(rng.integers(0, 5))
    for k in range(nn):
        it = its[rng.integers(0, len(its))]
        labels = {r[0]: r[2][0] for r in it.requirements}
        labels["topology.kubernetes.io/zone"] = str(rng.choice(zones + ["z9"]))
        labels["karpenter.sh/capacity-type"] = "on-demand" if cts is None or cts.random() < 0.5 else "spot"
        labels["kubernetes.io/hostname"] = f"n{k}"
        if nps is not None:
            labels["karpenter.sh/nodepool"] = f"np{int(nps.integers(0, 3))}"
        avail = {"cpu": int(rng.choice([1000, 3000, 6000])), "memory": 8 * GI * 1000, "pods": 20_000}
        b.add_node(f"n{k}", labels, avail, initialized=True)
        for q in range(int(rng.integers(0, 4))):
            b.add_bound_pod(k, _uid(rng), 0, {"cpu": 100, "pods": 1000},
                            labels={"app": str(rng.choice(APPS[:3]))},
                            namespace=str(rng.choice(["default", "default", "other"])))
    # a palette of constraints (deployments share them): at most 16 groups
    palette = []
    for _ in range(int(rng.integers(1, 9))):
        key = domain_key if rng.random() < 0.7 else "kubernetes.io/hostname"
        tgt = str(rng.choice(APPS[:3]))
        r = rng.random()
        if r < 0.6:
            selector = {"labels": {"app": tgt}}
        elif r < 0.8:
            selector = {"exprs": [("app", str(rng.choice(["In", "NotIn"])), [tgt, "cache"])]}
        elif r < 0.9:
            selector = {"exprs": [("app", "Exists", [])]}
        else:
            selector = None
        sp = {"key": key, "max_skew": int(rng.choice([1, 1, 2, 3])),
              "when": "ScheduleAnyway" if rng.random() < 0.4 else "DoNotSchedule", "selector": selector}
        if rng.random() < 0.15:
            sp["min_domains"] = int(rng.integers(2, 6))
        if selector is not None and rng.random() < 0.25:
            sp["match_label_keys"] = ["pod-template-hash"] + (["absent-key"] if rng.random() < 0.3 else [])
        palette.append(sp)
    side = np.random.default_rng(seed + 0x7A11)
    tol_apps = {str(a) for a in np.random.default_rng(seed + 0x70A).choice(APPS[:3], size=2, replace=False)}
    avoid = str(side.choice(zones))
    two = [str(z) for z in side.choice(zones, size=2, replace=False)]
    n = int(n_pods if n_pods is not None else rng.integers(1, 40))
    for i in range(n):
        app = str(rng.choice(APPS[:3]))
        req = {"cpu": int(rng.choice([250, 500, 1000, 2000])), "memory": int(rng.choice([1, 2, 4])) * GI * 1000,
               "pods": 1000}
        required, sel = [], {}
        spreads = [dict(palette[k]) for k in rng.choice(len(palette), size=int(rng.choice([0, 1, 1, 2])))]
        if rng.random() < 0.2:
            if spreads:
                for sp in spreads:
                    sp["node_affinity_policy"] = affinity_policy
            # one avoided zone per problem (a deployment's replicas share their
            # node affinity): a Honor group keeps its first owner's filter, so
            # owners with different filter values are refused by the product
            drawn = str(rng.choice(zones))
            if spreads and multi_term:
                required += [[("topology.kubernetes.io/zone", "In", [two[0]])],
                             [("topology.kubernetes.io/zone", "In", [two[1]])]]
            else:
                required.append([("topology.kubernetes.io/zone", "NotIn", [avoid if spreads else drawn])])
        if rng.random() < 0.1 and not spreads:
            sel["topology.kubernetes.io/zone"] = str(rng.choice(zones))
        tols = [("dedicated", "Exists", "", "")] if rng.random() < 0.3 else []
        if taint_policy and spreads:
            tols = [("dedicated", "Exists", "", "")]
            for sp in spreads:
                sp["node_taints_policy"] = taint_policy
        if taint_policy and tol_by_app:
            tols = [("dedicated", "Exists", "", "")] if app in tol_apps else []
        labels = {"app": app}
        if rng.random() < 0.6:
            labels["pod-template-hash"] = str(rng.choice(["h1", "h2"]))
        b.add_pod(_uid(rng), 1_700_000_000_000_000_000 + int(rng.integers(0, 3)) * 1_000_000_000, req,
                  node_selector=sel, required_terms=required, tolerations=tols, labels=labels,
                  namespace=str(rng.choice(["default", "default", "other"])), spreads=spreads)
    return b.build()


def random_relax(seed, n_pods=None):
    """relax-heavy topology problems (<U> Topology.Update re-keying): most
    NodePools carry a PreferNoSchedule taint, so pods without the toleration
    relax into it, and spread owners with node affinity carry two OR'd zone
    terms, so relaxation drops one; both change the spread groups' node filter
    and so their TopologyGroup.Hash.  nodeAffinityPolicy alternates by seed."""
    return random_topology(seed, n_pods=n_pods, multi_term=True, pns_frac=0.85,
                           affinity_policy="Honor" if seed % 2 else "Ignore")


def random_honor_filter(seed, n_pods=None, affinity_policy="Honor", consolidation=False):
    """small problems for nodeAffinityPolicy Honor past the zone key: each
    deployment (app) shares one node affinity on instance family / instance
    type (In, NotIn, two OR'd terms, with or without a zone term) and spreads
    over zone or hostname selecting its own app; existing nodes of every
    family hold bound pods of those apps, which count only where the node
    matches the deployment's filter (<U> TopologyNodeFilter).  The random
    stream does not depend on affinity_policy, so the Honor and Ignore
    problems of one seed differ only in it.  consolidation: the bound pods
    carry their deployment's node affinity and spreads too (consolidation
    reschedules them as pending pods), nodes belong to a NodePool (they are
    candidates) and few pods are pending."""
    F, IT = "karpenter-ibm.sh/instance-family", "node.kubernetes.io/instance-type"
    rng = np.random.default_rng(seed)
    b = ProblemBuilder()
    zones = ["z1", "z2", "z3", "z4"][: int(rng.integers(2, 5))]
    fams = ["bx2", "cx2", "mx2"]
    profs = [(f"{f}-{v}x{v * MEM_RATIO[f[0]]}", v, v * MEM_RATIO[f[0]], None) for f in fams for v in (2, 4, 8)]
    prices = {p_[0]: round(0.05 * p_[1] + 0.01 * float(rng.random()), 4) for p_ in profs}
    its = build_catalog(b, profs, zones, spot=bool(rng.random() < 0.5), prices=prices, rng=rng,
                        unavailable_frac=0.1)
    for j in range(int(rng.integers(1, 3))):
        reqs = []
        if rng.random() < 0.5:
            zs = sorted(rng.choice(zones, size=int(rng.integers(1, len(zones) + 1)), replace=False).tolist())
            reqs.append(("topology.kubernetes.io/zone", "In", zs))
        limits = {"cpu": int(rng.choice([16, 64])) * 1000} if rng.random() < 0.2 else None
        b.add_nodepool(f"np{j}", weight=int(rng.choice([0, 10])), requirements=reqs, limits=limits,
                       daemon={"cpu": 100, "pods": 1000})
    apps = APPS[:3]
    # one node affinity and one or two spreads per deployment
    deps = []
    for app in apps:
        f1, f2 = [str(x) for x in rng.choice(fams, size=2, replace=False)]
        r = rng.random()
        if r < 0.3:
            terms = [[(F, "In", [f1])]]
        elif r < 0.45:
            terms = [[(F, "In", sorted([f1, f2]))]]
        elif r < 0.6:
            terms = [[(F, "NotIn", [f1])]]
        elif r < 0.75:
            terms = [[(F, "In", [f1])], [(F, "In", [f2])]]
        elif r < 0.9:
            terms = [[(F, "In", [f1]), ("topology.kubernetes.io/zone", "NotIn", [str(rng.choice(zones))])]]
        else:
            names = sorted({str(its[int(x)].name) for x in rng.choice(len(its), size=3)})
            terms = [[(IT, "In", names)]]
        sps = []
        for _ in range(int(rng.integers(1, 3))):
            sps.append({"key": "topology.kubernetes.io/zone" if rng.random() < 0.7 else "kubernetes.io/hostname",
                        "max_skew": int(rng.choice([1, 1, 2])),
                        "when": "ScheduleAnyway" if rng.random() < 0.3 else "DoNotSchedule",
                        "selector": {"labels": {"app": app}}, "node_affinity_policy": affinity_policy})
        deps.append((app, terms, sps))
    for k in range(int(rng.integers(0, 7))):
        it = its[rng.integers(0, len(its))]
        labels = {r[0]: r[2][0] for r in it.requirements}
        labels["topology.kubernetes.io/zone"] = str(rng.choice(zones))
        labels["karpenter.sh/capacity-type"] = "on-demand"
        labels["kubernetes.io/hostname"] = f"n{k}"
        avail = {"cpu": int(rng.choice([1000, 3000, 6000])), "memory": 8 * GI * 1000, "pods": 20_000}
        if consolidation:
            labels["karpenter.sh/nodepool"] = "np0"
            avail = {r: it.capacity[r] - it.overhead.get(r, 0) for r in it.capacity}
        for q in range(int(rng.integers(0, 5))):
            app, terms, sps = deps[int(rng.integers(0, len(deps)))]
            extra = {"required_terms": terms, "spreads": [dict(sp) for sp in sps]} if consolidation else {}
            b.add_bound_pod(k, _uid(rng), 0, {"cpu": 100, "pods": 1000}, labels={"app": app}, **extra)
            if consolidation:
                avail["cpu"] -= 100
                avail["pods"] -= 1000
        b.add_node(f"n{k}", labels, avail, initialized=True)
    n = int(n_pods if n_pods is not None else (rng.choice([0, 0, 1, 2]) if consolidation else rng.integers(4, 40)))
    for i in range(n):
        req = {"cpu": int(rng.choice([250, 500, 1000, 2000])), "memory": int(rng.choice([1, 2, 4])) * GI * 1000,
               "pods": 1000}
        if rng.random() < 0.15:  # a pod no spread counts, with its own affinity
            b.add_pod(_uid(rng), 1_700_000_000_000_000_000 + i, req, labels={"app": "cache"},
                      required_terms=[[(F, "In", [str(rng.choice(fams))])]] if rng.random() < 0.5 else (),
                      preferred_terms=[(10, [(F, "In", [str(rng.choice(fams))])])] if rng.random() < 0.3 else ())
            continue
        app, terms, sps = deps[int(rng.integers(0, len(deps)))]
        b.add_pod(_uid(rng), 1_700_000_000_000_000_000 + i, req, labels={"app": app}, required_terms=terms,
                  spreads=[dict(sp) for sp in sps])
    return b.build()


def _selector(rng, tgt):
    r = rng.random()
    if r < 0.6:
        return {"labels": {"app": tgt}}
    if r < 0.8:
        return {"exprs": [("app", str(rng.choice(["In", "NotIn"])), [tgt, "cache"])]}
    if r < 0.9:
        return {"exprs": [("app", "Exists", [])]}
    return None


def random_affinity(seed, n_pods=None):
    """small adversarial problems for pod anti-affinity and host ports:
    required and preferred hostname anti-affinity (self- and other-selecting,
    namespace lists, nil selectors), inverse groups from pending and bound
    carriers, host ports over protocols and specific / unspecified host IPs,
    hostname pod affinity (required and preferred, bootstrap by self-selecting
    pods), mixed with topology spread, existing nodes, NodePool limits
    (relaxation) and taints"""
    rng = np.random.default_rng(seed)
    b = ProblemBuilder()
    zones = ["z1", "z2", "z3"][: int(rng.integers(1, 4))]
    profs = []
    for fam in ["bx2", "cx2", "mx2"]:
        for v in [2, 4, 8]:
            if rng.random() < 0.7:
                profs.append((f"{fam}-{v}x{v * MEM_RATIO[fam[0]]}", v, v * MEM_RATIO[fam[0]], None))
    if not profs:
        profs = [("bx2-4x16", 4, 16, None)]
    prices = {p_[0]: round(0.05 * p_[1] + 0.01 * float(rng.random()), 4) for p_ in profs}
    its = build_catalog(b, profs, zones, spot=bool(rng.random() < 0.5), prices=prices, rng=rng,
                        unavailable_frac=0.1)
    for j in range(int(rng.integers(1, 3))):
        reqs = [("topology.kubernetes.io/zone", "In", zones)] if rng.random() < 0.7 else []
        taints = [("dedicated", "x", "PreferNoSchedule")] if rng.random() < 0.2 else []
        limits = {"cpu": int(rng.choice([8, 16, 32])) * 1000} if rng.random() < 0.35 else None
        b.add_nodepool(f"np{j}", weight=int(rng.choice([0, 10])), requirements=reqs, taints=taints, limits=limits,
                       daemon={"cpu": 100, "pods": 1000})
    # palettes shared by pods (deployments share their terms)
    b.add_namespace("default", {"team": "a"})
    b.add_namespace("other", {"team": "b", "tier": "web"})
    b.add_namespace("kube", {})
    anti_pal = []
    for _ in range(int(rng.integers(1, 5))):
        t = {"required": bool(rng.random() < 0.35), "weight": int(rng.choice([1, 10, 50, 100])),
             "selector": _selector(rng, str(rng.choice(APPS[:3])))}
        if rng.random() < 0.15:
            t["namespaces"] = sorted(set(rng.choice(["default", "other", "kube"], size=2).tolist()))
        r = rng.random()
        if r < 0.1:
            t["namespace_selector"] = {}  # every namespace
        elif r < 0.25:
            t["namespace_selector"] = {"labels": {"team": str(rng.choice(["a", "b"]))}}
        elif r < 0.3:
            t["namespace_selector"] = {"exprs": [("tier", "Exists", [])]}
        anti_pal.append(t)
    aff_pal = []
    for _ in range(int(rng.integers(0, 3))):
        t = {"required": bool(rng.random() < 0.4), "weight": int(rng.choice([1, 20, 80])),
             "selector": _selector(rng, str(rng.choice(APPS[:3])))}
        if rng.random() < 0.15:
            t["namespaces"] = ["default", "other"]
        aff_pal.append(t)
    port_pal = [(int(rng.choice([80, 443, 8080])), str(rng.choice(["TCP", "TCP", "", "UDP"])),
                 str(rng.choice(["", "", "10.0.0.1", "10.0.0.2", "0.0.0.0"]))) for _ in range(int(rng.integers(1, 6)))]
    spread_pal = []
    for _ in range(int(rng.integers(0, 3))):
        spread_pal.append({"key": "topology.kubernetes.io/zone" if rng.random() < 0.5 else "kubernetes.io/hostname",
                           "max_skew": int(rng.choice([1, 2])), "node_affinity_policy": "Ignore",
                           "when": "ScheduleAnyway" if rng.random() < 0.5 else "DoNotSchedule",
                           "selector": {"labels": {"app": str(rng.choice(APPS[:3]))}}})

    def pick(pal, kmax):
        if not pal:
            return []
        k = int(rng.integers(0, kmax + 1))
        return [dict(pal[i]) if isinstance(pal[i], dict) else pal[i]
                for i in sorted(set(rng.choice(len(pal), size=k).tolist()))] if k else []

    for k in range(int(rng.integers(0, 5))):
        it = its[rng.integers(0, len(its))]
        labels = {r[0]: r[2][0] for r in it.requirements}
        labels["topology.kubernetes.io/zone"] = str(rng.choice(zones))
        labels["karpenter.sh/capacity-type"] = "on-demand"
        labels["kubernetes.io/hostname"] = f"n{k}"
        avail = {"cpu": int(rng.choice([1000, 3000, 6000])), "memory": 8 * GI * 1000, "pods": 20_000}
        b.add_node(f"n{k}", labels, avail, initialized=True)
        for q in range(int(rng.integers(0, 4))):
            anti = [t for t in pick(anti_pal, 1) if t["required"]] if rng.random() < 0.3 else []
            b.add_bound_pod(k, _uid(rng), 0, {"cpu": 100, "pods": 1000},
                            labels={"app": str(rng.choice(APPS[:3]))},
                            namespace=str(rng.choice(["default", "default", "other"])),
                            anti_affinity=anti, host_ports=pick(port_pal, 1) if rng.random() < 0.3 else [])
    n = int(n_pods if n_pods is not None else rng.integers(1, 40))
    for i in range(n):
        req = {"cpu": int(rng.choice([250, 500, 1000, 2000])), "memory": int(rng.choice([1, 2, 4])) * GI * 1000,
               "pods": 1000}
        tols = [("dedicated", "Exists", "", "")] if rng.random() < 0.3 else []
        b.add_pod(_uid(rng), 1_700_000_000_000_000_000 + int(rng.integers(0, 3)) * 1_000_000_000, req,
                  tolerations=tols, labels={"app": str(rng.choice(APPS[:3]))},
                  namespace=str(rng.choice(["default", "default", "other"])),
                  anti_affinity=pick(anti_pal, 2) if rng.random() < 0.6 else [],
                  host_ports=pick(port_pal, 2) if rng.random() < 0.3 else [],
                  spreads=pick(spread_pal, 1) if rng.random() < 0.3 else [],
                  affinity=pick(aff_pal, 1) if rng.random() < 0.3 else [])
    return b.build()


def e2e_deployments(n_deployments=8, replicas=20, with_nodes=False, seed=0x5EED00E2):
    """the reference e2e suite's deployments (test/e2e/config.go:455-490):
    labels app/test/purpose, requests 100m-1 CPU, and a preferred (weight 100)
    podAntiAffinity on kubernetes.io/hostname selecting its own app; over the
    C2-family catalog in 3 zones x {on-demand, spot}"""
    rng = np.random.default_rng(seed)
    b = ProblemBuilder()
    profs = []
    for fam in ["bx2", "cx2", "mx2"]:
        for v in [2, 4, 8, 16]:
            profs.append((f"{fam}-{v}x{v * MEM_RATIO[fam[0]]}", v, v * MEM_RATIO[fam[0]], None))
    its = build_catalog(b, profs, FAKE_ZONES, spot=True, prices=price_table(profs))
    b.add_nodepool("default", requirements=[("topology.kubernetes.io/zone", "In", FAKE_ZONES)],
                   daemon={"cpu": 100, "pods": 1000})
    if with_nodes:
        for k in range(6):
            it = its[k % len(its)]
            labels = {r[0]: r[2][0] for r in it.requirements}
            labels["topology.kubernetes.io/zone"] = FAKE_ZONES[k % 3]
            labels["kubernetes.io/hostname"] = f"node-{k}"
            b.add_node(f"node-{k}", labels, {"cpu": 4000, "memory": 16 * GI * 1000, "pods": 30_000})
            b.add_bound_pod(k, f"bound-{k}", 0, {"cpu": 100, "pods": 1000},
                            labels={"app": f"e2e-{k % max(1, n_deployments)}", "test": "e2e"})
    for d in range(n_deployments):
        name = f"e2e-{d}"
        cpu = int(rng.choice([100, 250, 500, 1000]))
        mem = int(rng.choice([128, 256, 512, 1024])) * MI * 1000
        for r in range(replicas):
            b.add_pod(f"{name}-{r:04d}", 1_700_000_000_000_000_000 + d * 1_000_000_000, {"cpu": cpu, "memory": mem,
                                                                                          "pods": 1000},
                      labels={"app": name, "test": "e2e", "purpose": "karpenter-test"},
                      anti_affinity=[{"required": False, "weight": 100, "selector": {"labels": {"app": name}}}])
    return b.build()


IT_KEY = "node.kubernetes.io/instance-type"
FAMILY_KEY = "karpenter-ibm.sh/instance-family"
SIZE_KEY = "karpenter-ibm.sh/instance-size"


def random_min_values(seed, n_pods=None):
    """small adversarial problems for NodePool minValues (Strict): minimums on
    the instance-type, family and size keys (and, rarely, on a key instance
    types do not carry), pods whose selectors and requests narrow the options
    below the minimum, NodePool limits, several NodePools, existing nodes"""
    rng = np.random.default_rng(seed)
    b = ProblemBuilder()
    zones = ["z1", "z2", "z3"][: int(rng.integers(1, 4))]
    profs = []
    for fam in ["bx2", "cx2", "mx2", "ox2"]:
        for v in [2, 4, 8, 16, 32]:
            if rng.random() < 0.75:
                profs.append((f"{fam}-{v}x{v * MEM_RATIO[fam[0]]}", v, v * MEM_RATIO[fam[0]], None))
    if len(profs) < 2:
        profs = [("bx2-4x16", 4, 16, None), ("cx2-4x8", 4, 8, None)]
    prices = {p_[0]: round(0.05 * p_[1] + 0.01 * float(rng.random()), 4) for p_ in profs}
    its = build_catalog(b, profs, zones, spot=bool(rng.random() < 0.5), prices=prices, rng=rng,
                        unavailable_frac=0.1)
    fams = sorted({it.name.split("-")[0] for it in its})
    for j in range(int(rng.integers(1, 3))):
        reqs = []
        r = rng.random()
        if r < 0.35:
            reqs.append((FAMILY_KEY, "In", fams, int(rng.integers(1, len(fams) + 2))))
        elif r < 0.6:
            reqs.append((IT_KEY, "Exists", [], int(rng.choice([1, 2, 3, 5, 8]))))
        elif r < 0.8:
            reqs.append((SIZE_KEY, "Exists", [], int(rng.integers(1, 5))))
            if rng.random() < 0.5:
                reqs.append((FAMILY_KEY, "Exists", [], int(rng.integers(1, 3))))
        elif r < 0.85:
            reqs.append(("topology.kubernetes.io/zone", "In", zones, 1))  # instance types carry no zone value
        limits = {"cpu": int(rng.choice([16, 64])) * 1000} if rng.random() < 0.25 else None
        b.add_nodepool(f"np{j}", weight=int(rng.choice([0, 10])), requirements=reqs, limits=limits,
                       daemon={"cpu": 100, "pods": 1000})
    for k in range(int(rng.integers(0, 3))):
        it = its[rng.integers(0, len(its))]
        labels = {r_[0]: r_[2][0] for r_ in it.requirements}
        labels["topology.kubernetes.io/zone"] = str(rng.choice(zones))
        labels["kubernetes.io/hostname"] = f"n{k}"
        b.add_node(f"n{k}", labels, {"cpu": int(rng.choice([1000, 4000])), "memory": 8 * GI * 1000, "pods": 20_000})
    n = int(n_pods if n_pods is not None else rng.integers(1, 50))
    for i in range(n):
        req = {"cpu": int(rng.choice([250, 500, 1000, 2000, 6000, 14000])),
               "memory": int(rng.choice([1, 2, 4, 16])) * GI * 1000, "pods": 1000}
        sel, required = {}, []
        r = rng.random()
        if r < 0.15:
            sel[FAMILY_KEY] = str(rng.choice(fams))
        elif r < 0.25:
            sel[IT_KEY] = its[rng.integers(0, len(its))].name
        elif r < 0.35:
            required.append([(FAMILY_KEY, "In", sorted(set(rng.choice(fams, size=2).tolist())))])
        b.add_pod(_uid(rng), 1_700_000_000_000_000_000 + int(rng.integers(0, 3)) * 1_000_000_000, req,
                  node_selector=sel, required_terms=required)
    return b.build()


def min_values_truncation(n_cheap=70):
    """a NodePool with minValues 2 on the family whose 60 cheapest options are
    all one family: the NodeClaim passes CanAdd but Truncate(60) drops it"""
    b = ProblemBuilder()
    profs = [(f"cx2-{v}x{2 * v}", v, 2 * v, None) for v in range(2, 2 + n_cheap)]
    profs += [("mx2-2x16", 2, 16, None), ("mx2-4x32", 4, 32, None)]
    prices = {p_[0]: round(0.01 * p_[1], 4) for p_ in profs}
    prices["mx2-2x16"] = 50.0
    prices["mx2-4x32"] = 60.0
    build_catalog(b, profs, FAKE_ZONES, spot=False, prices=prices)
    b.add_nodepool("default", requirements=[(FAMILY_KEY, "In", ["cx2", "mx2"], 2)])
    for i in range(3):
        b.add_pod(f"p{i}", 0, {"cpu": 500, "memory": GI * 1000, "pods": 1000})
    return b.build()


def random_volumes(seed, n_pods=None):
    """small adversarial problems for CSI attach limits on existing nodes
    (<U> VolumeUsage): 1-3 drivers, per-node limits (some nodes unlimited or
    already at / over their limit), bound pods holding volumes, pending pods
    with new and shared volumes, NodeClaims (no limits) as the overflow"""
    rng = np.random.default_rng(seed)
    b = ProblemBuilder()
    zones = ["z1", "z2"]
    profs = [("bx2-4x16", 4, 16, None), ("bx2-8x32", 8, 32, None), ("cx2-4x8", 4, 8, None)]
    its = build_catalog(b, profs, zones, spot=False, prices=price_table(profs))
    b.add_nodepool("np0", daemon={"cpu": 100, "pods": 1000})
    drivers = ["ebs.csi", "vpc.block.csi.ibm.io", "nfs.csi"][: int(rng.integers(1, 4))]
    vols = [(str(rng.choice(drivers)), f"pv-{k}") for k in range(int(rng.integers(2, 24)))]
    for k in range(int(rng.integers(1, 6))):
        it = its[rng.integers(0, len(its))]
        labels = {r_[0]: r_[2][0] for r_ in it.requirements}
        labels["topology.kubernetes.io/zone"] = str(rng.choice(zones))
        labels["kubernetes.io/hostname"] = f"n{k}"
        lim = {d: int(rng.integers(0, 5)) for d in drivers if rng.random() < 0.7}
        b.add_node(f"n{k}", labels, {"cpu": 16000, "memory": 64 * GI * 1000, "pods": 110_000}, volume_limits=lim)
        for q in range(int(rng.integers(0, 4))):
            mine = [vols[i] for i in sorted(set(rng.integers(0, len(vols), size=int(rng.integers(0, 3))).tolist()))]
            b.add_bound_pod(k, _uid(rng), 0, {"cpu": 100, "pods": 1000}, volumes=mine)
    n = int(n_pods if n_pods is not None else rng.integers(1, 30))
    for i in range(n):
        mine = [vols[j] for j in sorted(set(rng.integers(0, len(vols), size=int(rng.integers(0, 3))).tolist()))]
        b.add_pod(_uid(rng), 1_700_000_000_000_000_000 + int(rng.integers(0, 3)) * 1_000_000_000,
                  {"cpu": int(rng.choice([250, 500, 1000])), "memory": GI * 1000, "pods": 1000},
                  volumes=mine if rng.random() < 0.7 else [])
    return b.build()


def random_consolidation_general(seed, n_nodes=None, n_pending=None, min_values=None, ct_spreads=False,
                                 np_spreads=False, pns=False):
    """small adversarial consolidation clusters for the general simulation
    variant: bound and pending pods with zone / hostname topology spread,
    hostname and zone pod anti-affinity (required, preferred, inverse
    carriers), hostname pod affinity, host ports, CSI volumes (shared and
    per-pod, node attach limits) and NodePools with minValues.  ct_spreads:
    the spreads use the capacity-type key instead of the zone (anti-affinity
    then stays on the hostname key); np_spreads: the NodePool key; pns: most
    NodePools carry a PreferNoSchedule taint (rescheduled pods relax into its
    toleration, re-keying their spread groups; its own random stream)"""
    rng = np.random.default_rng(0xC0A50000 + seed)
    prng = np.random.default_rng(0x9A5 + seed)
    b = ProblemBuilder()
    zones = FAKE_ZONES[: int(rng.integers(2, 4))]
    profs = []
    for fam in ["bx2", "cx2", "mx2"]:
        for v in [2, 4, 8, 16]:
            if rng.random() < 0.7:
                profs.append((f"{fam}-{v}x{v * MEM_RATIO[fam[0]]}", v, v * MEM_RATIO[fam[0]], None))
    if len(profs) < 3:
        profs = [("bx2-2x8", 2, 8, None), ("bx2-8x32", 8, 32, None), ("cx2-4x8", 4, 8, None)]
    prices = {p[0]: round(float(rng.choice([0.05, 0.1, 0.1, 0.2, 0.4])) * p[1] / 2, 4) for p in profs}
    its = build_catalog(b, profs, zones, spot=True, prices=prices, rng=rng, unavailable_frac=0.1)
    mv = bool(rng.random() < 0.3) if min_values is None else min_values
    n_np = int(rng.integers(1, 3))
    for j in range(n_np):
        reqs = [("topology.kubernetes.io/zone", "In", list(zones))]
        if mv and j == 0:
            reqs.append(("karpenter-ibm.sh/instance-family", "Exists", [], int(rng.integers(1, 3))))
        limits = {"cpu": int(rng.choice([16, 64, 256])) * 1000} if rng.random() < 0.2 else None
        taints = [("dedicated", "x", "PreferNoSchedule")] if pns and prng.random() < 0.75 else []
        b.add_nodepool(f"np{j}", weight=int(rng.choice([0, 10])), requirements=reqs, limits=limits,
                       daemon={"cpu": 100, "pods": 1000}, taints=taints)
    apps = ["web", "db", "cache"]
    dkey = ("karpenter.sh/capacity-type" if ct_spreads else "karpenter.sh/nodepool" if np_spreads
            else "topology.kubernetes.io/zone")
    anti_keys = ["kubernetes.io/hostname"] * 2 if ct_spreads or np_spreads else ["kubernetes.io/hostname", "topology.kubernetes.io/zone"]
    anti_pal = [{"key": str(rng.choice(anti_keys)),
                 "required": bool(rng.random() < 0.3), "weight": int(rng.choice([1, 50, 100])),
                 "selector": {"labels": {"app": str(rng.choice(apps))}}} for _ in range(int(rng.integers(1, 4)))]
    aff_pal = [{"required": bool(rng.random() < 0.3), "weight": 10,
                "selector": {"labels": {"app": str(rng.choice(apps))}}} for _ in range(int(rng.integers(0, 2)))]
    spread_pal = [{"key": str(rng.choice([dkey, "kubernetes.io/hostname"])),
                   "max_skew": int(rng.choice([1, 2])), "node_affinity_policy": "Ignore",
                   "when": "ScheduleAnyway" if rng.random() < 0.5 else "DoNotSchedule",
                   "selector": {"labels": {"app": str(rng.choice(apps))}}} for _ in range(int(rng.integers(0, 3)))]
    port_pal = [(int(rng.choice([80, 443, 8080])), "TCP", "") for _ in range(int(rng.integers(1, 3)))]
    drivers = ["vpc.block.csi.ibm.io", "nfs.csi"]
    shared_vols = [(str(rng.choice(drivers)), f"shared-{k}") for k in range(4)]
    uid_n = [0]

    def feats():
        f = {}
        if rng.random() < 0.35 and anti_pal:
            f["anti_affinity"] = [anti_pal[int(rng.integers(0, len(anti_pal)))]]
        if rng.random() < 0.15 and aff_pal:
            f["affinity"] = [aff_pal[int(rng.integers(0, len(aff_pal)))]]
        if rng.random() < 0.25 and spread_pal:
            f["spreads"] = [spread_pal[int(rng.integers(0, len(spread_pal)))]]
        if rng.random() < 0.15:
            f["host_ports"] = [port_pal[int(rng.integers(0, len(port_pal)))]]
        if rng.random() < 0.3:
            uid_n[0] += 1
            v = [(str(rng.choice(drivers)), f"pv-{seed}-{uid_n[0]}")]
            if rng.random() < 0.3:
                v.append(shared_vols[int(rng.integers(0, len(shared_vols)))])
            f["volumes"] = v
        return f

    nn = int(n_nodes if n_nodes is not None else rng.integers(2, 14))
    for k in range(nn):
        it = its[rng.integers(0, len(its))]
        labels = {r[0]: r[2][0] for r in it.requirements}
        labels["topology.kubernetes.io/zone"] = zones[rng.integers(0, len(zones))]
        labels["karpenter.sh/capacity-type"] = str(rng.choice(["spot", "on-demand"]))
        labels["karpenter.sh/nodepool"] = f"np{rng.integers(0, n_np)}"
        labels["kubernetes.io/hostname"] = f"n-{k:03d}"
        alloc = {r: it.capacity[r] - it.overhead.get(r, 0) for r in it.capacity}
        used = {"cpu": 100, "memory": 0, "pods": 1000}
        target = float(rng.uniform(0.2, 0.9))
        for _ in range(int(rng.integers(0, 8))):
            cpu = int(rng.choice([100, 250, 500, 1000, 2000]))
            mem = int(rng.choice([128 * MI, GI, 2 * GI])) * 1000
            if used["cpu"] + cpu > target * alloc["cpu"] or used["memory"] + mem > alloc["memory"]:
                break
            used["cpu"] += cpu
            used["memory"] += mem
            used["pods"] += 1000
            b.add_bound_pod(k, _uid(rng), 1_700_000_000_000_000_000 + int(rng.integers(0, 3)) * 1_000_000_000,
                            {"cpu": cpu, "memory": mem, "pods": 1000}, labels={"app": str(rng.choice(apps))},
                            **feats())
        avail = {r: alloc[r] - used.get(r, 0) for r in alloc}
        lim = {d: int(rng.integers(1, 6)) for d in drivers if rng.random() < 0.5}
        b.add_node(f"n-{k:03d}", labels, avail, initialized=bool(rng.random() < 0.9), volume_limits=lim)
    npend = int(n_pending if n_pending is not None else rng.choice([0, 0, 1, 2]))
    for i in range(npend):
        b.add_pod(_uid(rng), 1_700_000_000_000_000_000, {"cpu": int(rng.choice([100, 500, 1000])),
                                                         "memory": int(GI) * 1000, "pods": 1000},
                  labels={"app": str(rng.choice(apps))}, **feats())
    return b.build()


def e2e_consolidation_cluster(n_nodes=5000, replicas=4, seed=0x5EED0C4E, util=(0.5, 0.95)):
    """C4-scale cluster of the reference e2e workload shape
    (test/e2e/scheduling_test.go:38-122 TestE2EConsolidationWithPDB and
    test/e2e/config.go:455-490): deployments of `replicas` pods, each pod
    1 vCPU / 1 GiB with a preferred (weight 100) hostname anti-affinity on its
    own app, spread over 2-8 vCPU nodes of the C2 catalog in 3 zones (a node
    holds pods of distinct deployments, as the anti-affinity placed them);
    one NodePool"""
    import collections
    rng = np.random.default_rng(seed)
    b = ProblemBuilder()
    profs = c2_profiles(200)
    its = build_catalog(b, profs, FAKE_ZONES, spot=True, prices=price_table(profs), rng=rng, unavailable_frac=0.02)
    daemon = {"cpu": 200, "memory": 256 * MI * 1000, "pods": 2000}
    b.add_nodepool("default", requirements=[("topology.kubernetes.io/zone", "In", FAKE_ZONES)], daemon=daemon)
    cand = [it for it in its if it.capacity["nvidia.com/gpu"] == 0 and 2000 <= it.capacity["cpu"] <= 8000]
    active = collections.deque()  # [deployment, replicas left]
    n_dep = 0
    for k in range(n_nodes):
        it = cand[rng.integers(0, len(cand))]
        labels = {r[0]: r[2][0] for r in it.requirements}
        labels.update({"topology.kubernetes.io/zone": FAKE_ZONES[k % 3], "karpenter.sh/capacity-type": "on-demand",
                       "karpenter.sh/nodepool": "default", "kubernetes.io/hostname": f"node-{k:05d}"})
        alloc = {r: it.capacity[r] - it.overhead.get(r, 0) for r in it.capacity}
        used = dict(daemon)
        target = float(rng.uniform(*util))
        here = []
        while used["cpu"] + 1000 <= target * alloc["cpu"] and used["memory"] + GI * 1000 <= alloc["memory"]:
            while len(active) < 8:
                active.append([n_dep, replicas])
                n_dep += 1
            d = active.popleft()
            if d[0] in here:  # every active deployment already runs here
                active.appendleft(d)
                break
            here.append(d[0])
            d[1] -= 1
            if d[1]:
                active.append(d)
            used["cpu"] += 1000
            used["memory"] += GI * 1000
            used["pods"] += 1000
            name = f"e2e-{d[0]:05d}"
            b.add_bound_pod(k, f"{name}-{replicas - d[1]:02d}", 1_700_000_000_000_000_000 + d[0] * 1_000_000_000,
                            {"cpu": 1000, "memory": GI * 1000, "pods": 1000},
                            labels={"app": name, "test": "e2e"},
                            anti_affinity=[{"required": False, "weight": 100, "selector": {"labels": {"app": name}}}])
        avail = {r: alloc[r] - used.get(r, 0) for r in alloc}
        b.add_node(f"node-{k:05d}", labels, avail, initialized=True)
    return b.build()

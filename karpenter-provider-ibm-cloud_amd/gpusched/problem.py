"""Builder for gs_problem: the Solve inputs a Go caller would marshal.

Objects mirror what karpenter-core hands to scheduling.NewScheduler/Solve:
instance types exactly as CloudProvider.GetInstanceTypes returns them
(reference pkg/cloudprovider/cloudprovider.go:553-583), NodePools, pending
pods (requests = resources.RequestsForPods) and existing state nodes.
"""
import ctypes as C

import numpy as np

from . import abi


def _op(op):
    return abi.OPS[op] if isinstance(op, str) else int(op)


class ProblemBuilder:
    def __init__(self):
        self.strings = [""]
        self._sid = {"": 0}
        self.value_ids = []
        self.reqs = []
        self.quantities = []
        self.labels = []
        self.taints = []
        self.tolerations = []
        self.terms = []
        self.it_refs = []
        self.offerings = []
        self.instance_types = []
        self.nodepools = []
        self.pods = []
        self.nodes = []
        self.bound_pods = []  # pods bound to state nodes (topology counts; consolidation moves them)
        self.bound_node = []
        self.spreads = []
        self.affinity_terms = []
        self.host_ports = []
        self.volumes = []
        self.volume_limits = []
        self.namespaces = []
        self.claim_queries = []  # gs_claim_query (launch-time re-filter)

    # ------------------------------------------------------------ primitives
    def s(self, x: str) -> int:
        i = self._sid.get(x)
        if i is None:
            i = len(self.strings)
            self.strings.append(x)
            self._sid[x] = i
        return i

    def _reqs(self, reqs):
        """reqs: iterable of (key, op, values[, minValues])"""
        b = len(self.reqs)
        for r in reqs:
            key, op, values = r[0], r[1], r[2]
            mv = r[3] if len(r) > 3 and r[3] is not None else -1
            vb = len(self.value_ids)
            self.value_ids.extend(self.s(v) for v in values)
            self.reqs.append((self.s(key), _op(op), (vb, len(values)), mv))
        return (b, len(self.reqs) - b)

    def _qty(self, res):
        b = len(self.quantities)
        for k, v in res.items():
            self.quantities.append((self.s(k), int(v)))
        return (b, len(self.quantities) - b)

    def _labels(self, labels):
        b = len(self.labels)
        for k, v in labels.items():
            self.labels.append((self.s(k), self.s(v)))
        return (b, len(self.labels) - b)

    def _taints(self, taints):
        b = len(self.taints)
        for t in taints:
            key, value, effect = t
            self.taints.append((self.s(key), self.s(value), self.s(effect)))
        return (b, len(self.taints) - b)

    def _tols(self, tols):
        b = len(self.tolerations)
        for t in tols:
            key, op, value, effect = t
            opi = abi.TOL_EXISTS if op == "Exists" else abi.TOL_EQUAL
            self.tolerations.append((self.s(key), opi, self.s(value), self.s(effect)))
        return (b, len(self.tolerations) - b)

    def _terms(self, terms):
        b = len(self.terms)
        for weight, reqs in terms:
            self.terms.append((self._reqs(reqs), int(weight)))
        return (b, len(self.terms) - b)

    # --------------------------------------------------------------- objects
    def add_instance_type(self, name, requirements, capacity, overhead, offerings):
        """offerings: list of (zone, capacity_type, price, available)"""
        ob = len(self.offerings)
        for zone, ct, price, avail in offerings:
            rq = self._reqs([("topology.kubernetes.io/zone", "In", [zone]),
                             ("karpenter.sh/capacity-type", "In", [ct])])
            self.offerings.append((rq, float(price), 1 if avail else 0))
        idx = len(self.instance_types)
        self.instance_types.append((self.s(name), self._reqs(requirements), self._qty(capacity),
                                    self._qty(overhead), (ob, len(offerings))))
        return idx

    def add_nodepool(self, name, weight=0, requirements=(), labels=None, taints=(), limits=None,
                     daemon=None, instance_types=None):
        if instance_types is None:
            instance_types = range(len(self.instance_types))
        rb = len(self.it_refs)
        self.it_refs.extend(int(i) for i in instance_types)
        self.nodepools.append((self.s(name), int(weight), self._reqs(requirements), self._labels(labels or {}),
                               self._taints(taints), self._qty(limits or {}), 1 if limits is not None else 0,
                               self._qty(daemon or {}), (rb, len(self.it_refs) - rb)))
        return len(self.nodepools) - 1

    def _spreads(self, spreads):
        """spreads: dicts with key, max_skew, when ("DoNotSchedule"|"ScheduleAnyway"),
        selector (None = nil, else {"labels": {...}, "exprs": [(key, op, values)]}),
        min_domains, node_affinity_policy ("Honor"|"Ignore"), node_taints_policy"""
        b = len(self.spreads)
        for sp in spreads:
            sel = sp.get("selector")
            ml = self._labels((sel or {}).get("labels", {}))
            me = self._reqs((sel or {}).get("exprs", []))
            mk = list(sp.get("match_label_keys", []))
            kb = len(self.value_ids)
            self.value_ids.extend(self.s(k) for k in mk)
            self.spreads.append((self.s(sp["key"]), int(sp.get("max_skew", 1)),
                                 abi.SPREAD_SCHEDULE_ANYWAY if sp.get("when") == "ScheduleAnyway"
                                 else abi.SPREAD_DO_NOT_SCHEDULE,
                                 int(sp.get("min_domains", 0)), 0 if sel is None else 1, ml, me,
                                 abi.POLICY_IGNORE if sp.get("node_affinity_policy") == "Ignore" else abi.POLICY_HONOR,
                                 abi.POLICY_HONOR if sp.get("node_taints_policy") == "Honor" else abi.POLICY_IGNORE,
                                 (kb, len(mk))))
        return (b, len(self.spreads) - b)

    def _anti(self, terms):
        """terms: dicts with key (default kubernetes.io/hostname), required
        (bool), weight, selector (None = nil, else {"labels": {...},
        "exprs": [(key, op, values)]}), namespaces (list; empty = the pod's)"""
        b = len(self.affinity_terms)
        for t in terms:
            sel = t.get("selector")
            ml = self._labels((sel or {}).get("labels", {}))
            me = self._reqs((sel or {}).get("exprs", []))
            nss = list(t.get("namespaces", []))
            vb = len(self.value_ids)
            self.value_ids.extend(self.s(x) for x in nss)
            nsel = t.get("namespace_selector")  # None = unset, else {"labels": {...}, "exprs": [...]}
            nml = self._labels((nsel or {}).get("labels", {}))
            nme = self._reqs((nsel or {}).get("exprs", []))
            self.affinity_terms.append((self.s(t.get("key", "kubernetes.io/hostname")), 1 if t.get("required") else 0,
                                        int(t.get("weight", 1)), 0 if sel is None else 1, ml, me, (vb, len(nss)),
                                        0 if nsel is None else 1, nml, nme))
        return (b, len(self.affinity_terms) - b)

    def _ports(self, ports):
        """ports: (port, protocol, ip) tuples (protocol "" = TCP, ip "" = unspecified)"""
        b = len(self.host_ports)
        for pt in ports:
            port, proto, ip = (tuple(pt) + ("", ""))[:3]
            self.host_ports.append((self.s(proto), self.s(ip), int(port)))
        return (b, len(self.host_ports) - b)

    def _pod(self, uid, creation_ns, requests, node_selector, required_terms, preferred_terms, tolerations, flags,
             namespace, labels, spreads, anti_affinity=(), host_ports=(), affinity=(), volumes=()):
        vb = len(self.volumes)
        self.volumes.extend((self.s(drv), self.s(vid)) for drv, vid in volumes)
        return (self.s(uid), int(creation_ns), self._qty(requests), self._labels(node_selector or {}),
                self._terms([(0, t) for t in required_terms]), self._terms(preferred_terms),
                self._tols(tolerations), int(flags), self.s(namespace), self._labels(labels or {}),
                self._spreads(spreads), self._anti(anti_affinity), self._ports(host_ports), self._anti(affinity),
                (vb, len(self.volumes) - vb))

    def add_pod(self, uid, creation_ns, requests, node_selector=None, required_terms=(), preferred_terms=(),
                tolerations=(), flags=0, namespace="default", labels=None, spreads=(), anti_affinity=(),
                host_ports=(), affinity=(), volumes=()):
        """required_terms: list of reqs lists; preferred_terms: list of (weight, reqs);
        anti_affinity / affinity: pod (anti-)affinity term dicts (see _anti);
        volumes: (csi driver, volume id) pairs"""
        self.pods.append(self._pod(uid, creation_ns, requests, node_selector, required_terms, preferred_terms,
                                   tolerations, flags, namespace, labels, spreads, anti_affinity, host_ports, affinity,
                                   volumes))
        return len(self.pods) - 1

    def add_bound_pod(self, node, uid, creation_ns, requests, node_selector=None, required_terms=(),
                      preferred_terms=(), tolerations=(), flags=0, namespace="default", labels=None, spreads=(),
                      anti_affinity=(), host_ports=(), affinity=(), volumes=()):
        """a pod bound to state node `node` (counted by topology selectors;
        consolidation reschedules the candidates' pods)"""
        self.bound_pods.append(self._pod(uid, creation_ns, requests, node_selector, required_terms, preferred_terms,
                                         tolerations, flags, namespace, labels, spreads, anti_affinity, host_ports,
                                         affinity, volumes))
        self.bound_node.append(int(node))
        return len(self.bound_pods) - 1

    def add_namespace(self, name, labels=None):
        """a namespace and its labels (namespaceSelector of pod affinity terms)"""
        self.namespaces.append((self.s(name), self._labels(labels or {})))
        return len(self.namespaces) - 1

    def add_claim_query(self, requirements=(), requests=None):
        """a NodeClaim for gs_create_filter: spec.requirements (key, op,
        values) and spec.resources.requests"""
        self.claim_queries.append((self._reqs(requirements), self._qty(requests or {})))
        return len(self.claim_queries) - 1

    def add_node(self, name, labels, available, requests=None, taints=(), initialized=True, volume_limits=None,
                 managed=False, claim_taints=(), startup_taints=()):
        """volume_limits: {csi driver: CSINode allocatable count}; taints:
        Node.Spec.Taints; managed nodes also carry their NodeClaim's
        spec.taints and spec.startupTaints (the library derives
        StateNode.Taints() from them, include/gpusched.h gs_node)"""
        lb = len(self.volume_limits)
        self.volume_limits.extend((self.s(k), int(v)) for k, v in (volume_limits or {}).items())
        self.nodes.append((self.s(name), 1 if initialized else 0, self._labels(labels), self._taints(taints),
                           self._qty(available), self._qty(requests or {}), (lb, len(self.volume_limits) - lb),
                           1 if managed else 0, self._taints(claim_taints), self._taints(startup_taints)))
        return len(self.nodes) - 1

    def build(self):
        return Problem(self)


def _np(rows, dtype):
    a = np.zeros(len(rows), dtype=dtype)
    if rows:
        a[:] = rows
    return a


class Problem:
    """Owns the numpy arrays backing a gs_problem struct."""

    def __init__(self, b: ProblemBuilder):
        self._builder = b
        self.strings = list(b.strings)
        self._bytes = [x.encode() for x in self.strings]
        self._cstrs = (C.c_char_p * len(self._bytes))(*self._bytes)
        self.value_ids = np.asarray(b.value_ids, dtype=np.uint32)
        self.reqs = _np(b.reqs, abi.DT_REQ)
        self.quantities = _np(b.quantities, abi.DT_QTY)
        self.labels = _np(b.labels, abi.DT_LABEL)
        self.taints = _np(b.taints, abi.DT_TAINT)
        self.tolerations = _np(b.tolerations, abi.DT_TOL)
        self.terms = _np(b.terms, abi.DT_TERM)
        self.it_refs = np.asarray(b.it_refs, dtype=np.uint32)
        self.offerings = _np(b.offerings, abi.DT_OFFERING)
        self.instance_types = _np(b.instance_types, abi.DT_IT)
        self.nodepools = _np(b.nodepools, abi.DT_NODEPOOL)
        self.pods = _np(b.pods, abi.DT_POD)
        self.nodes = _np(b.nodes, abi.DT_NODE)
        self.bound_pods = _np(b.bound_pods, abi.DT_POD)
        self.bound_node = np.asarray(b.bound_node, dtype=np.uint32)
        self.spreads = _np(b.spreads, abi.DT_SPREAD)
        self.affinity_terms = _np(b.affinity_terms, abi.DT_AFFINITY)
        self.host_ports = _np(b.host_ports, abi.DT_HOSTPORT)
        self.volumes = _np(b.volumes, abi.DT_VOLUME)
        self.volume_limits = _np(b.volume_limits, abi.DT_VOLUME_LIMIT)
        self.namespaces = _np(b.namespaces, abi.DT_NAMESPACE)
        self.claim_queries = (abi.GsClaimQuery * max(1, len(b.claim_queries)))()
        self.n_claim_queries = len(b.claim_queries)
        for i, (rq, qt) in enumerate(b.claim_queries):
            self.claim_queries[i].requirements.begin, self.claim_queries[i].requirements.count = rq
            self.claim_queries[i].requests.begin, self.claim_queries[i].requests.count = qt
        self.struct = abi.GsProblem()
        st = self.struct
        st.strings = self._cstrs
        st.n_strings = len(self._bytes)
        for name in ("value_ids", "reqs", "quantities", "labels", "taints", "tolerations", "terms", "it_refs",
                     "offerings", "instance_types", "nodepools", "pods", "nodes", "spreads", "bound_pods",
                     "affinity_terms", "host_ports", "volumes", "volume_limits", "namespaces"):
            arr = getattr(self, name)
            setattr(st, name, arr.ctypes.data if len(arr) else None)
            setattr(st, "n_" + name, len(arr))
        st.bound_pod_node = self.bound_node.ctypes.data if len(self.bound_node) else None

    _DUMP_ARRAYS = ("value_ids", "reqs", "quantities", "labels", "taints", "tolerations", "terms", "it_refs",
                    "offerings", "instance_types", "nodepools", "pods", "nodes", "spreads", "bound_pods", "bound_node",
                    "affinity_terms", "host_ports", "volumes", "volume_limits", "namespaces")

    def dump(self, path):
        """binary dump read by tools/encode_harness.cpp (host-only encoder
        runs: sanitizers, profiling)"""
        import struct
        with open(path, "wb") as f:
            f.write(b"GSPD" + struct.pack("<II", 4, len(self._bytes)))
            for s in self._bytes:
                f.write(struct.pack("<I", len(s)) + s)
            for name in self._DUMP_ARRAYS:
                a = np.ascontiguousarray(getattr(self, name))
                f.write(struct.pack("<QQ", len(a), a.dtype.itemsize))
                f.write(a.tobytes())

    def with_pods(self, idx):
        """a view with pending pods pods[idx] (same pools: requirement, label
        and quantity ranges stay valid) — e.g. an oracle check on a sample of
        a problem too large for the oracle"""
        import copy
        q = copy.copy(self)
        q.pods = self.pods[np.asarray(idx, dtype=np.int64)].copy()
        q.struct = abi.GsProblem()
        C.memmove(C.byref(q.struct), C.byref(self.struct), C.sizeof(abi.GsProblem))
        q.struct.pods = q.pods.ctypes.data if len(q.pods) else None
        q.struct.n_pods = len(q.pods)
        return q

    def extended(self, fn):
        """a new Problem: this one's builder after fn(builder) appends to it
        (string / value / requirement ids of this problem stay valid)"""
        fn(self._builder)
        return Problem(self._builder)

    @property
    def n_pods(self):
        return len(self.pods)

    @property
    def n_offerings_per_pool(self):
        """offerings reachable per NodePool (for checks accounting)"""
        out = []
        for np_ in self.nodepools:
            b, c = np_["instance_types"]
            its = self.it_refs[b:b + c]
            out.append(int(self.instance_types["offerings"]["count"][its].sum()))
        return out

    def checks(self):
        return self.n_pods * sum(self.n_offerings_per_pool)

"""ctypes binding of libgpusched.so (the C-ABI in include/gpusched.h).

This is the product path: it loads ONLY the in-tree HIP library and fails
loudly when it is missing or no gfx950 device is visible.  There is no CPU
fallback.
"""
import ctypes as C
import os

from . import abi

HERE = os.path.dirname(os.path.abspath(__file__))
# GPUSCHED_LIB selects an in-tree diagnostic build of the same library
# (csrc/Makefile targets tl / diag / phases write libgpusched_<variant>.so)
LIB_PATH = os.path.join(HERE, os.environ.get("GPUSCHED_LIB", "libgpusched.so"))

EXPORTS = ["gs_create", "gs_destroy", "gs_prepare", "gs_run", "gs_fetch", "gs_solve", "gs_feasibility",
           "gs_last_error", "gs_version", "gs_validate", "gs_abi_sizes", "gs_last_run_ms",
           "gs_consolidate", "gs_consolidate_rerun", "gs_consolidation_choose", "gs_feasibility_shard",
           "gs_feasibility_shard_device", "gs_rank_instance_types", "gs_create_filter", "gs_build_catalog", "gs_build_id"]


def source_digest():
    """The digest csrc/Makefile bakes into gs_build_id(): sha256 over the
    library's sources in make's $(sort) order, first 16 hex digits."""
    import hashlib
    csrc = os.path.join(HERE, "..", "csrc")
    names = [n for n in os.listdir(csrc) if n.endswith((".hip", ".cpp", ".hpp"))] + ["Makefile"]
    paths = {n: os.path.join(csrc, n) for n in names}
    paths["../../include/gpusched.h"] = os.path.join(csrc, "..", "..", "include", "gpusched.h")
    h = hashlib.sha256()
    for n in sorted(paths):
        with open(paths[n], "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def check_build_id():
    """Fail loudly when the loaded library was built from other sources."""
    got = load().gs_build_id().decode()
    want = source_digest()
    if got != want:
        raise GpuSchedError(abi.GS_E_INVALID, f"{LIB_PATH} was built from sources {got}, the tree holds {want}: rebuild")
    return got


class GpuSchedError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__(f"{abi.STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status


_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise GpuSchedError(abi.GS_E_NO_DEVICE, f"{LIB_PATH} is not built (run __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        vp = C.c_void_p
        L.gs_create.argtypes = [C.POINTER(abi.GsConfig), C.POINTER(vp)]
        L.gs_create.restype = C.c_int
        L.gs_destroy.argtypes = [vp]
        L.gs_destroy.restype = None
        L.gs_prepare.argtypes = [vp, C.POINTER(abi.GsProblem)]
        L.gs_prepare.restype = C.c_int
        L.gs_run.argtypes = [vp]
        L.gs_run.restype = C.c_int
        L.gs_fetch.argtypes = [vp, C.POINTER(abi.GsResult)]
        L.gs_fetch.restype = C.c_int
        L.gs_solve.argtypes = [vp, C.POINTER(abi.GsProblem), C.POINTER(abi.GsResult)]
        L.gs_solve.restype = C.c_int
        L.gs_feasibility.argtypes = [vp, C.POINTER(abi.GsFeasResult)]
        L.gs_feasibility.restype = C.c_int
        L.gs_feasibility_shard.argtypes = [vp, C.c_uint32, C.c_uint32, C.POINTER(abi.GsFeasResult)]
        L.gs_feasibility_shard.restype = C.c_int
        L.gs_feasibility_shard_device.argtypes = [vp, C.c_uint32, C.c_uint32, C.POINTER(abi.GsFeasDevice)]
        L.gs_feasibility_shard_device.restype = C.c_int
        L.gs_create_filter.argtypes = [vp, C.POINTER(abi.GsProblem), C.POINTER(abi.GsClaimQuery), C.c_uint32,
                                       C.POINTER(abi.GsClaimFilterResult)]
        L.gs_create_filter.restype = C.c_int
        L.gs_build_catalog.argtypes = [vp, C.POINTER(abi.GsVpcProfile), C.c_uint32, C.POINTER(abi.GsCatalogEnv),
                                       C.POINTER(abi.GsCatalog)]
        L.gs_build_catalog.restype = C.c_int
        L.gs_rank_instance_types.argtypes = abi.RANK_ARGTYPES
        L.gs_rank_instance_types.restype = C.c_int
        L.gs_last_error.argtypes = [vp, C.c_char_p, C.c_size_t]
        L.gs_last_error.restype = C.c_size_t
        L.gs_version.argtypes = []
        L.gs_version.restype = C.c_char_p
        L.gs_build_id.argtypes = []
        L.gs_build_id.restype = C.c_char_p
        L.gs_validate.argtypes = [C.POINTER(abi.GsProblem), C.c_char_p, C.c_size_t]
        L.gs_validate.restype = C.c_int
        L.gs_abi_sizes.argtypes = [C.POINTER(C.c_uint32), C.c_uint32]
        L.gs_abi_sizes.restype = C.c_uint32
        L.gs_last_run_ms.argtypes = [vp, C.POINTER(C.c_double)]
        L.gs_last_run_ms.restype = C.c_int
        L.gs_consolidate.argtypes = [vp, C.POINTER(abi.GsConsolidation), C.POINTER(abi.GsConsolidationResult)]
        L.gs_consolidate.restype = C.c_int
        L.gs_consolidate_rerun.argtypes = [vp, C.POINTER(abi.GsConsolidationResult)]
        L.gs_consolidate_rerun.restype = C.c_int
        L.gs_consolidation_choose.argtypes = [C.POINTER(abi.GsConsolidation), C.POINTER(abi.GsCommand), C.c_uint32,
                                              C.POINTER(C.c_uint32), C.POINTER(C.c_double), C.POINTER(C.c_int32),
                                              C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        L.gs_consolidation_choose.restype = C.c_int
        _lib = L
    return _lib


def rank_instance_types(cpu_milli, memory_bytes, price, arch, want_arch=abi.GS_ARCH_ANY, min_cpu=0,
                        min_memory_gb=0, max_price=0.0):
    """gs_rank_instance_types (FilterInstanceTypes + rankInstanceTypes,
    instancetype.go:259-379) -> (List indices ranked, scores)"""
    st, order, score = abi.call_rank(load().gs_rank_instance_types, cpu_milli, memory_bytes, price, arch,
                                     want_arch, min_cpu, min_memory_gb, max_price)
    if st != abi.GS_OK:
        raise GpuSchedError(st, "gs_rank_instance_types")
    return order, score


def _multi(res):
    return [int(res.multi_options[i]) for i in range(res.n_multi_options)]


def choose(cin, commands):
    """gs_consolidation_choose (host only): replay SINGLE/MULTI over a complete
    command table, e.g. gathered from sharded evaluations -> (chosen, multi_options)"""
    n = len(commands)
    cmds = (abi.GsCommand * max(n, 1))()
    opts, prices = [], []
    for i, c in enumerate(commands):
        x = cmds[i]
        x.decision, x.reason, x.n_new_claims = c["decision"], c["reason"], c["n_new_claims"]
        x.n_failed_pods, x.n_candidates = c["n_failed_pods"], c["n_candidates"]
        x.nodepool = c["nodepool"] if c["nodepool"] is not None else 0
        x.spot_only = c["spot_only"]
        x.options.begin, x.options.count = len(opts), len(c["options"])
        x.candidate_price = c["candidate_price"]
        opts += c["options"]
        prices += c["option_prices"]
    oa = (C.c_uint32 * max(len(opts), 1))(*opts)
    pa = (C.c_double * max(len(prices), 1))(*prices)
    chosen = C.c_int32(-1)
    mo = (C.c_uint32 * 60)()
    nmo = C.c_uint32(0)
    st = load().gs_consolidation_choose(C.byref(cin.struct), cmds, n, oa, pa, C.byref(chosen), mo, C.byref(nmo))
    if st != abi.GS_OK:
        raise GpuSchedError(st, "gs_consolidation_choose failed")
    return int(chosen.value), [int(mo[i]) for i in range(nmo.value)]


def validate(problem):
    """host-only encode check (no device): (status, message)"""
    buf = C.create_string_buffer(512)
    st = load().gs_validate(C.byref(problem.struct), buf, 512)
    return st, buf.value.decode()


class Solver:
    """One gs_ctx on one device (karpenter-core drives one provisioning
    Solve and one consolidation simulation at a time per context)."""

    def __init__(self, device=0, flags=0, shard_devices=None):
        self.L = load()
        self.ctx = C.c_void_p()
        self.flags = flags
        cfg = abi.GsConfig(device, 0, flags)
        if shard_devices:
            self._shards = (C.c_int32 * len(shard_devices))(*shard_devices)
            cfg.n_shards = len(shard_devices)
            cfg.shard_devices = self._shards
        st = self.L.gs_create(C.byref(cfg), C.byref(self.ctx))
        if st != abi.GS_OK:
            raise GpuSchedError(st, "gs_create failed (no gfx950 device?)")
        self.problem = None

    def close(self):
        if self.ctx:
            self.L.gs_destroy(self.ctx)
            self.ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _err(self):
        buf = C.create_string_buffer(1024)
        self.L.gs_last_error(self.ctx, buf, 1024)
        return buf.value.decode()

    def _check(self, st):
        if st != abi.GS_OK:
            raise GpuSchedError(st, self._err())

    def prepare(self, problem):
        self.problem = problem
        self._check(self.L.gs_prepare(self.ctx, C.byref(problem.struct)))

    def run(self):
        self._check(self.L.gs_run(self.ctx))

    def last_run_ms(self):
        """(feasibility, ffd, truncate) device ms of the last run"""
        out = (C.c_double * 3)()
        self._check(self.L.gs_last_run_ms(self.ctx, out))
        return tuple(out)

    def fetch(self):
        res = abi.GsResult()
        self._check(self.L.gs_fetch(self.ctx, C.byref(res)))
        return abi.result_to_dict(res, self.problem), res

    def solve_raw(self, problem):
        """one gs_solve call (encode + H2D + kernels + D2H + decode into the
        library's result memory) -> gs_result, no Python-side copy"""
        self.problem = problem
        res = abi.GsResult()
        self._check(self.L.gs_solve(self.ctx, C.byref(problem.struct), C.byref(res)))
        return res

    def solve(self, problem):
        self.prepare(problem)
        self.run()
        return self.fetch()

    def consolidate(self, cin):
        """gs_consolidate: (commands, chosen, multi_options, raw result)"""
        res = abi.GsConsolidationResult()
        self._check(self.L.gs_consolidate(self.ctx, C.byref(cin.struct), C.byref(res)))
        return abi.commands_to_list(res), int(res.chosen), _multi(res), res

    def consolidate_rerun(self, raw=False):
        """re-run the device simulations on the resident input; raw=True
        returns only the gs_consolidation_result (no Python-side copy)"""
        res = abi.GsConsolidationResult()
        self._check(self.L.gs_consolidate_rerun(self.ctx, C.byref(res)))
        if raw:
            return res
        return abi.commands_to_list(res), int(res.chosen), _multi(res), res

    def create_filter(self, problem, raw=False):
        """gs_create_filter over problem.claim_queries: per claim
        {compatible, requirements, n_compatible, selected, capacity_type}"""
        res = abi.GsClaimFilterResult()
        self._check(self.L.gs_create_filter(self.ctx, C.byref(problem.struct), problem.claim_queries,
                                            problem.n_claim_queries, C.byref(res)))
        if raw:
            return res
        return abi.claim_filter_to_list(res, len(problem.instance_types))

    def build_catalog(self, profiles, zones, price_rows=(), unavailable=(), now_ns=0, spot_discount_percent=0,
                      kubelet=None, raw=False, region=None):
        """gs_build_catalog.  profiles: dicts with name, vcpu, memory_gib, arch,
        gpu, availability_class (None | ("enum", [..]) | ("fixed", v)) and
        optional vcpu_kind / memory_kind / gpu_kind; price_rows: (name, zone
        or None, price); unavailable: (key, expiry_ns).  -> (types, skipped
        [(index, reason)], raw gs_catalog)"""
        keep = []
        arr = (abi.GsVpcProfile * max(1, len(profiles)))()
        enc = lambda x: None if x is None else x.encode()  # noqa: E731
        for i, p in enumerate(profiles):
            a = arr[i]
            a.name = enc(p.get("name"))
            a.vcpu_kind = p.get("vcpu_kind", abi.GS_VPC_NIL if p.get("vcpu") is None else abi.GS_VPC_VALUE)
            a.vcpu = p.get("vcpu") or 0
            a.memory_kind = p.get("memory_kind", abi.GS_VPC_NIL if p.get("memory_gib") is None else abi.GS_VPC_VALUE)
            a.memory_gib = p.get("memory_gib") or 0
            a.arch = enc(p.get("arch"))
            a.gpu_kind = p.get("gpu_kind", abi.GS_VPC_NIL if p.get("gpu") is None else abi.GS_VPC_VALUE)
            a.gpu = p.get("gpu") or 0
            ac = p.get("availability_class")
            if ac is None:
                a.avail_kind = abi.GS_AVAIL_NIL
            else:
                kind, val = ac
                vals = list(val) if kind == "enum" else ([] if val is None else [val])
                va = (C.c_char_p * max(1, len(vals)))(*[v.encode() for v in vals])
                keep.append(va)
                a.avail_kind = abi.GS_AVAIL_ENUM if kind == "enum" else abi.GS_AVAIL_FIXED
                a.avail_values, a.n_avail_values = va, len(vals)
        e = abi.GsCatalogEnv()
        za = (C.c_char_p * max(1, len(zones)))(*[z.encode() for z in zones])
        pr = (abi.GsPrice * max(1, len(price_rows)))(*[abi.GsPrice(enc(n), enc(z), float(v)) for n, z, v in price_rows])
        ua = (abi.GsUnavailable * max(1, len(unavailable)))(*[abi.GsUnavailable(enc(k), int(x)) for k, x in unavailable])
        keep += [za, pr, ua]
        e.zones, e.n_zones = za, len(zones)
        e.spot_discount_percent = spot_discount_percent
        e.prices, e.n_prices = pr, len(price_rows)
        e.unavailable, e.n_unavailable = ua, len(unavailable)
        e.now_unix_ns = now_ns
        e.region = enc(region)
        if kubelet is not None:
            e.has_kubelet = 1
            kr, sr, eh = kubelet.get("kubeReserved", {}), kubelet.get("systemReserved", {}), kubelet.get("evictionHard", {})
            e.kube_reserved_cpu = enc(kr.get("cpu"))
            e.kube_reserved_memory = enc(kr.get("memory"))
            e.system_reserved_cpu = enc(sr.get("cpu"))
            e.system_reserved_memory = enc(sr.get("memory"))
            e.eviction_memory_available = enc(eh.get("memory.available"))
        out = abi.GsCatalog()
        self._check(self.L.gs_build_catalog(self.ctx, arr, len(profiles), C.byref(e), C.byref(out)))
        skipped = [(int(out.skipped[i]), out.skip_reasons[i].decode()) for i in range(out.n_skipped)]
        return abi.catalog_to_list(out), skipped, out

    def feasibility(self):
        res = abi.GsFeasResult()
        self._check(self.L.gs_feasibility(self.ctx, C.byref(res)))
        return abi.feas_to_dict(res), res

    def feasibility_shard(self, word_begin, word_end):
        """gs_feasibility_shard: the static matrix over instance-type words [begin, end)"""
        res = abi.GsFeasResult()
        self._check(self.L.gs_feasibility_shard(self.ctx, word_begin, word_end, C.byref(res)))
        return abi.feas_to_dict(res), res

    def feasibility_shard_device(self, word_begin, word_end):
        """gs_feasibility_shard_device: the shard left in HBM (gs_feas_device, pointers valid until the next call)"""
        res = abi.GsFeasDevice()
        self._check(self.L.gs_feasibility_shard_device(self.ctx, word_begin, word_end, C.byref(res)))
        return res

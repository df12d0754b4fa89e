"""CPU-side checks of the C-ABI library: it loads, exports every symbol
include/gpusched.h declares, and its host-only encoder accepts/refuses the
right inputs (no compute call needs a GPU here)."""
import re
import os

import pytest

from gpusched import abi, lib, synth

HEADER = os.path.join(os.path.dirname(__file__), "..", "include", "gpusched.h")


def declared():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(gs_[a-z_]+)\s*\(", txt)))


def test_exports_every_declared_symbol():
    L = lib.load()
    names = declared()
    assert set(names) == set(lib.EXPORTS)
    for n in names:
        assert hasattr(L, n), n


def test_build_id_matches_sources():
    """The shipped libgpusched.so was built from this tree's sources."""
    assert lib.check_build_id() == lib.source_digest()


@pytest.mark.gpu
def test_gpu_box_build_id_matches_sources():
    """Same check in the GPU run: the library the -m gpu suite loads on the
    box is the one built from the sources it ships with."""
    assert lib.check_build_id() == lib.source_digest()


def test_version():
    assert b"gfx950" in lib.load().gs_version()


@pytest.mark.parametrize("name", ["C1", "C2", "C3"])
def test_validate_configs(name):
    f = {"C1": synth.make_c1, "C2": lambda: synth.make_c2(500), "C3": lambda: synth.make_c3(500)}[name]
    assert lib.validate(f()) == (abi.GS_OK, "")


def _one_pod_problem(**pod):
    b = synth.ProblemBuilder()
    synth.build_catalog(b, synth.FAKE_PROFILES, synth.FAKE_ZONES, spot=False, prices={})
    b.add_nodepool("default")
    b.add_pod("u1", 0, {"cpu": 100, "pods": 1000}, **pod)
    return b


def test_validate_refuses_topology():
    b = _one_pod_problem(flags=abi.POD_TOPOLOGY_SPREAD)
    st, msg = lib.validate(b.build())
    assert st == abi.GS_E_UNSUPPORTED and "topology" in msg


def test_validate_refuses_min_values():
    b = _one_pod_problem(required_terms=[[("kubernetes.io/arch", "In", ["amd64"], 2)]])
    assert lib.validate(b.build())[0] == abi.GS_E_UNSUPPORTED


def test_validate_accepts_gte_lte():
    for op in ("Gte", "Lte"):
        b = _one_pod_problem(required_terms=[[("karpenter-ibm.sh/instance-cpu", op, ["4"])]])
        assert lib.validate(b.build())[0] == abi.GS_OK


def test_validate_gte_lte_bounds():
    b = _one_pod_problem(required_terms=[[("karpenter-ibm.sh/instance-cpu", "Gte", ["-9223372036854775808"])]])
    assert lib.validate(b.build())[0] == abi.GS_E_INVALID
    b = _one_pod_problem(required_terms=[[("karpenter-ibm.sh/instance-cpu", "Lte", ["x"])]])
    assert lib.validate(b.build())[0] == abi.GS_E_INVALID


def test_validate_invalid_gt_value():
    b = _one_pod_problem(required_terms=[[("karpenter-ibm.sh/instance-cpu", "Gt", ["four"])]])
    assert lib.validate(b.build())[0] == abi.GS_E_INVALID


def test_validate_duplicate_uid():
    b = _one_pod_problem()
    b.add_pod("u1", 0, {"cpu": 100})
    assert lib.validate(b.build())[0] == abi.GS_E_INVALID


def test_validate_random_accepts():
    for s in range(100):
        st, msg = lib.validate(synth.random_problem(s, with_nodes=False))
        assert st == abi.GS_OK, (s, msg)


def test_struct_layouts_match_library():
    import ctypes as C
    out = (C.c_uint32 * 31)()
    assert lib.load().gs_abi_sizes(out, 31) == 31
    mine = [8, abi.DT_REQ.itemsize, abi.DT_QTY.itemsize, abi.DT_LABEL.itemsize, abi.DT_TAINT.itemsize,
            abi.DT_TOL.itemsize, abi.DT_TERM.itemsize, abi.DT_OFFERING.itemsize, abi.DT_IT.itemsize,
            abi.DT_NODEPOOL.itemsize, abi.DT_POD.itemsize, abi.DT_NODE.itemsize, C.sizeof(abi.GsProblem),
            C.sizeof(abi.GsResult), C.sizeof(abi.GsFeasResult), C.sizeof(abi.GsConfig),
            C.sizeof(abi.GsConsolidation), C.sizeof(abi.GsCommand), C.sizeof(abi.GsConsolidationResult),
            C.sizeof(abi.GsClaimQuery), C.sizeof(abi.GsClaimFilterResult), C.sizeof(abi.GsVpcProfile),
            C.sizeof(abi.GsPrice), C.sizeof(abi.GsUnavailable), C.sizeof(abi.GsCatalogEnv), C.sizeof(abi.GsCatalog),
            abi.DT_AFFINITY.itemsize, abi.DT_HOSTPORT.itemsize,
            abi.DT_VOLUME.itemsize, abi.DT_VOLUME_LIMIT.itemsize, abi.DT_NAMESPACE.itemsize]
    assert list(out) == mine

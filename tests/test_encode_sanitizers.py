"""The host encoder (csrc/encode.cpp) under AddressSanitizer + UBSan on the CPU.

encode.cpp parses caller-owned arrays (ranges, string ids, value ids) before
anything reaches the device, so it is built here with
g++ -fsanitize=address,undefined (host only, tools/encode_harness.cpp) and run
over the randomised generators the parity tests use — Solve problems, topology
problems, consolidation clusters with bound pods — plus deliberately corrupted
inputs (out-of-range ranges and ids), which must come back as GS_E_INVALID
instead of reading out of bounds.  Statuses must agree with the product
library's gs_validate (same encoder, compiled by hipcc).
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

from gpusched import abi, lib, synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "karpenter-provider-ibm-cloud_amd", "csrc")


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ absent")
    out = str(tmp_path_factory.mktemp("asan") / "encode_harness_asan")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", "-pthread", "-o", out, os.path.join(ROOT, "tools", "encode_harness.cpp"),
           os.path.join(CSRC, "encode.cpp")]
    subprocess.run(cmd, check=True, capture_output=True, timeout=600)
    return out


def _problems():
    out = []
    for s in range(24):
        out.append((f"solve{s}", synth.random_problem(s)))
    for s in range(12):
        out.append((f"topo{s}", synth.random_topology(s)))
    for s in range(8):
        out.append((f"cons{s}", synth.random_consolidation(s)))
    for s in range(10):
        out.append((f"anti{s}", synth.random_affinity(s)))
    for s in range(8):
        out.append((f"minv{s}", synth.random_min_values(s)))
    for s in range(8):
        out.append((f"vol{s}", synth.random_volumes(s)))
    out.append(("c1", synth.make_c1()))
    out.append(("c3_2k", synth.make_c3(n_pods=2000)))
    out.append(("c4_200", synth.make_c4(n_nodes=200, n_pending=5)))
    return out


def _corrupt(kind):
    p = synth.random_problem(3, with_nodes=True)
    if kind == "pod_requests_range":
        p.pods["requests"]["begin"][0] = len(p.quantities) + 5
    elif kind == "req_key_id":
        p.reqs["key"][0] = len(p.strings) + 100
    elif kind == "value_range":
        p.reqs["values"]["count"][len(p.reqs) - 1] = 1 << 30
    elif kind == "it_offerings_range":
        p.instance_types["offerings"]["begin"][0] = len(p.offerings)
        p.instance_types["offerings"]["count"][0] = 3
    elif kind == "node_labels_range":
        if len(p.nodes):
            p.nodes["labels"]["begin"][0] = len(p.labels) + 1
            p.nodes["labels"]["count"][0] = 1
    elif kind == "quantity_resource_id":
        p.quantities["resource"][0] = len(p.strings) + 7
    elif kind == "nodepool_it_refs":
        p.nodepools["instance_types"]["count"][0] = len(p.it_refs) + 1
    elif kind == "anti_affinity_range":
        p.pods["anti_affinity"]["begin"][0] = len(p.affinity_terms) + 2
        p.pods["anti_affinity"]["count"][0] = 1
    elif kind == "host_port_range":
        p.pods["host_ports"]["count"][len(p.pods) - 1] = 1 << 31
    return p


CORRUPT = ["pod_requests_range", "req_key_id", "value_range", "it_offerings_range", "node_labels_range",
           "quantity_resource_id", "nodepool_it_refs", "anti_affinity_range", "host_port_range"]


def _run(harness, dumps):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([harness] + dumps, capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    return [int(line.split()[0]) for line in r.stdout.strip().split("\n")]


def test_encoder_clean_under_asan_ubsan(harness, tmp_path):
    probs = _problems()
    dumps = []
    for name, p in probs:
        path = str(tmp_path / f"{name}.gspd")
        p.dump(path)
        dumps.append(path)
    got = _run(harness, dumps)
    for (name, p), st in zip(probs, got):
        want, msg = lib.validate(p)
        if want == abi.GS_E_CAPACITY:  # device capacity check runs after encode
            want = abi.GS_OK
        assert st == want, (name, st, want, msg)


def test_encoder_rejects_corrupt_inputs_under_asan(harness, tmp_path):
    dumps = []
    for kind in CORRUPT:
        path = str(tmp_path / f"{kind}.gspd")
        _corrupt(kind).dump(path)
        dumps.append(path)
    got = _run(harness, dumps)
    for kind, st in zip(CORRUPT, got):
        assert st == abi.GS_E_INVALID, (kind, st)


def test_dump_roundtrip_status_matches_validate(tmp_path):
    """the dump carries the whole problem: a plain (unsanitised) harness
    build gives the library's statuses too"""
    p = synth.random_problem(5)
    path = str(tmp_path / "p.gspd")
    p.dump(path)
    with open(path, "rb") as f:
        assert f.read(4) == b"GSPD"
    assert os.path.getsize(path) > np.asarray(p.pods).nbytes

"""bench.py's stdout contract (CPU): the last line is a compact headline the
driver can parse from its 8 KB stdout tail (a 24 KB line was not
parsed), carrying the contract keys, `roofline` and `cpu_baseline`."""
import copy
import io
import json
import os
import sys
from contextlib import redirect_stdout

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

R3_LINE = os.path.join(ROOT, "profiles", "r3", "bench_v3.json")


def _full_line():
    with open(R3_LINE) as f:
        line = json.load(f)
    # the round-4 bench adds the unique-byte view beside the §8(d) roofline
    line["roofline_unique_bytes"] = copy.deepcopy(line["roofline"])
    return line


def test_headline_fits_and_has_contract_keys():
    line = _full_line()
    assert len(json.dumps(line)) > 20000  # the round-3 record the driver could not parse
    h = bench.headline(line)
    s = json.dumps(h)
    assert len(s) <= bench.HEADLINE_MAX_BYTES
    for k in bench.HEADLINE_KEYS:
        assert k in h, k
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in h["roofline"], k
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in h["cpu_baseline"], k
    assert h["value"] > 0 and h["ms_per_step"] > 0
    assert "legs" in h and "C5_SOLVE" in h["legs"] and "c4_e2e" in h["legs"]


def test_headline_sheds_detail_never_contract_keys():
    line = _full_line()
    line["config"]["workload"] = "x" * 3000
    for i in range(200):  # a bench with many more legs
        line.setdefault("configs", {})[f"EXTRA{i}"] = line["configs"]["C3"]
    h = bench.headline(line)
    assert len(json.dumps(h)) <= bench.HEADLINE_MAX_BYTES
    for k in bench.HEADLINE_KEYS:
        assert k in h, k


def test_emit_last_stdout_line_is_the_headline(tmp_path):
    line = _full_line()
    buf = io.StringIO()
    with redirect_stdout(buf):
        bench.emit(line, str(tmp_path / "detail.json"), 0)
    out = buf.getvalue().splitlines()
    last = json.loads(out[-1])
    assert len(out[-1].encode()) <= bench.HEADLINE_MAX_BYTES
    assert last["metric"] == bench.METRIC and last["roofline"] and last["cpu_baseline"]
    assert all(x.startswith("# leg ") for x in out[:-1])
    with open(tmp_path / "detail.json") as f:
        detail = json.load(f)
    assert detail["configs"]["C3"] == line["configs"]["C3"]
    buf = io.StringIO()
    with redirect_stdout(buf):
        assert bench.emit(_full_line(), None, 1) is None
    assert buf.getvalue() == ""

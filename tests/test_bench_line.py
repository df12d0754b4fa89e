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


# ---------------------------------------------- N > 1: the strong-scaling legs
def _scaling_worker(rank, world, port, q):
    """one gloo rank: bench's max-over-ranks reduction and the section builder"""
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def max_over_ranks(x):
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    per_rank = {
        "c5_static_matrix_it_columns": {"ms_per_step": 0.2, "kernel_ms": 0.05 + 0.01 * rank,
                                        "combine_ms": 0.03 * (rank + 1), "words_per_rank": 32 // world,
                                        "checks_per_s": 1e12, "shards_equal_whole": True},
        "c4_candidates": {"ms_per_sweep": 1.0, "sim_kernel_ms": 0.3 - 0.1 * rank, "gather_choose_ms": 0.2 + rank,
                          "simulations": 5000, "simulations_per_s": 5e6},
    }
    sec = bench.strong_scaling_section(per_rank, dist.get_world_size(), dist.get_backend(), max_over_ranks)
    q.put((rank, sec))
    dist.destroy_process_group()


def test_strong_scaling_section_gloo_world2():
    import socket
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [ctx.Process(target=_scaling_worker, args=(r, world, port, q)) for r in range(world)]
    for p_ in procs:
        p_.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p_ in procs:
        p_.join(timeout=60)
        assert p_.exitcode == 0
    sec = res[0]
    assert res[1] == sec  # every rank holds the same reduced section
    assert sec["ranks"] == 2 and sec["backend"] == "gloo" and sec["scaling"] == "strong"
    c5 = sec["c5_static_matrix_it_columns"]
    assert c5["kernel_ms"] == 0.06 and c5["combine_ms"] == 0.06 and c5["words_per_rank"] == 16
    c4 = sec["c4_candidates"]
    assert c4["sim_kernel_ms"] == 0.3 and c4["gather_choose_ms"] == 1.2 and c4["simulations"] == 5000
    # the headline carries it, within the driver's size budget
    line = _full_line()
    line["n_gpus"] = 2
    line["strong_scaling"] = sec
    h = bench.headline(line)
    assert h["strong_scaling"] == sec and len(json.dumps(h)) <= bench.HEADLINE_MAX_BYTES

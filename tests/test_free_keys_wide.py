"""Custom (free) requirement keys with wide vocabularies:
a label key such as `team` named with up to 255 distinct values across the
problem's pods, NodePools and nodes.  The device keeps a free key's state as
four 64-bit words (layout.hpp FK, FKW); round 3 refused keys over 63 values.

CPU: the encoder accepts these problems and refuses a 256-value vocabulary.
GPU: the whole Solve (both kernels and the HBM claim mode) and the static
matrix equal the oracle, which has no vocabulary limit."""
import pytest

from gpusched import abi, synth
from gpusched.problem import ProblemBuilder
from oracle import pyoracle

SEEDS = range(24)


def _wide(seed):
    return synth.random_problem(9000 + seed, n_pods=160, free_values=int(90 + (seed * 37) % 160))


@pytest.mark.parametrize("seed", SEEDS[:8])
def test_encoder_accepts_wide_vocabularies(seed):
    from gpusched import lib
    st, msg = lib.validate(_wide(seed))
    assert st == abi.GS_OK, msg
    st, _, _ = pyoracle.solve(_wide(seed))
    assert st == abi.GS_OK


def _team_problem(n_values):
    b = ProblemBuilder()
    synth.build_catalog(b, synth.FAKE_PROFILES, synth.FAKE_ZONES, spot=False,
                        prices=synth.price_table(synth.FAKE_PROFILES))
    b.add_nodepool("np", requirements=[("team", "In", [f"t{i}" for i in range(n_values)])])
    b.add_pod("p0", 1, {"cpu": 100, "pods": 1000}, node_selector={"team": "t0"})
    return b.build()


def test_vocabulary_limit():
    from gpusched import lib
    st, _ = lib.validate(_team_problem(255))  # 255 values + the unmentioned value: four words
    assert st == abi.GS_OK
    st, msg = lib.validate(_team_problem(256))
    assert st == abi.GS_E_UNSUPPORTED and "255" in msg


@pytest.fixture(scope="module", params=["wave", "block", "hbm"])
def solver(request):
    from gpusched.lib import Solver
    s = Solver(0, {"wave": 0, "block": abi.GS_CFG_BLOCK_SOLVE, "hbm": abi.GS_CFG_CLAIMS_HBM}[request.param])
    yield s
    s.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS)
def test_gpu_solve_wide_free_keys(solver, seed):
    from test_gpu_parity import check_solve
    check_solve(solver, _wide(seed))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS[:8])
def test_gpu_feasibility_wide_free_keys(solver, seed):
    from test_gpu_parity import check_feas
    check_feas(solver, synth.random_problem(9500 + seed, n_pods=160, with_nodes=False, free_values=200))

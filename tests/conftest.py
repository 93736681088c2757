import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

MAXU64 = (1 << 64) - 1


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs under gpurun)")
    config.addinivalue_line("markers", "slow: long-running (large ranges)")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def ctx():
    """One GPU context for the whole gpu session (one process on the card)."""
    from distributed_bitcoinminer_amd import _lib
    c = _lib.Context([0])
    yield c
    c.close()


@pytest.fixture(params=["fused", "per_segment"])
def ctx_paths(request, ctx):
    """The session context once per small-request path.  Since round 5 a
    request of <= 2^27 nonces runs as ONE fused launch (HM_OPT_FUSED=1, the
    default); HM_OPT_FUSED=0 sends the same request through the per-segment
    kernels, which requests above 2^27 nonces always take.  Sweeps over small
    ranges use this fixture so both paths keep their layout coverage."""
    from distributed_bitcoinminer_amd import _lib
    ctx.set_option(_lib.HM_OPT_FUSED, 1 if request.param == "fused" else 0)
    try:
        yield ctx
    finally:
        ctx.set_option(_lib.HM_OPT_FUSED, 1)

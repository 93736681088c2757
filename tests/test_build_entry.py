"""__graft_entry__.build()'s build-identity gate (no GPU, no compiler runs):
make is replaced by a recorder and the library's embedded id by a stub, so
the test checks the decisions only -- an up-to-date library is left alone, a
library whose id differs from the tree's digest is rebuilt with `make -B`, and
one that still differs afterwards fails the build loudly."""
import pytest

import __graft_entry__ as entry
from distributed_bitcoinminer_amd import build_id as bid


class _Make:
    def __init__(self):
        self.calls = []

    def __call__(self, cmd, check=True, **kw):
        self.calls.append(cmd)

        class R:
            returncode = 0
        return R()


@pytest.fixture()
def make(monkeypatch):
    m = _Make()
    monkeypatch.setattr(entry.subprocess, "run", m)
    return m


def _forced(calls):
    return [c for c in calls if "-B" in c]


def test_current_library_is_not_rebuilt(make, monkeypatch):
    monkeypatch.setattr(bid, "embedded_id", lambda path: bid.tree_digest())
    entry.build()
    assert not _forced(make.calls)
    assert any(c[-1].endswith("csrc") for c in make.calls)     # the library's make
    assert any(c[-1].endswith("oracle") for c in make.calls)   # the checker's make


def test_stale_library_is_rebuilt_from_scratch(make, monkeypatch):
    ids = iter(["0" * 16, bid.tree_digest(), bid.tree_digest()])
    monkeypatch.setattr(bid, "embedded_id", lambda path: next(ids))
    entry.build()
    assert len(_forced(make.calls)) == 1


def test_library_that_stays_stale_fails_the_build(make, monkeypatch):
    monkeypatch.setattr(bid, "embedded_id", lambda path: "f" * 16)
    with pytest.raises(RuntimeError, match="build id"):
        entry.build()
    assert len(_forced(make.calls)) == 1

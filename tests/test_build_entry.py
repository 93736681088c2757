"""__graft_entry__.build()'s build-identity gate (no GPU, no compiler runs):
make is replaced by a recorder and the library's embedded id by a stub, so
the test checks the decisions only -- an up-to-date library is left alone, a
library whose id differs from the tree's digest is rebuilt with `make -B`, and
one that still differs afterwards fails the build loudly.  And its report:
which artifacts make wrote (a fresh tree) or reused (an up-to-date one)."""
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


def _tree(tmp_path, monkeypatch):
    pkg = tmp_path / "pkg"
    bd = tmp_path / "build" / "hipminer"
    pkg.mkdir()
    monkeypatch.setattr(entry, "PKG", str(pkg))
    monkeypatch.setattr(entry, "BUILD_DIR", str(bd))
    monkeypatch.setattr(entry, "ROOT", str(tmp_path))
    return pkg, bd


def test_report_fresh_tree(tmp_path, monkeypatch, capsys):
    """A tree with no artifacts: make writes every object, the code object,
    the library and the miner; the report lists them, mode "compiled"."""
    pkg, bd = _tree(tmp_path, monkeypatch)
    names = ["api.o", "kernels.o", "hipminer_scan.hsaco"]

    def fake_make(cmd, check=True, **kw):
        if cmd[-1].endswith("csrc"):
            bd.mkdir(parents=True, exist_ok=True)
            for n in names:
                (bd / n).write_bytes(b"x")
            (pkg / "libhipminer.so").write_bytes(b"hipminer-build-id:" + bid.tree_digest().encode())
            (pkg / "hm_miner").write_bytes(b"x")

        class R:
            returncode = 0
        return R()
    monkeypatch.setattr(entry.subprocess, "run", fake_make)
    entry.build()
    out = capsys.readouterr().out
    import json
    rep = json.loads((bd / "BUILD_REPORT").read_text())
    assert rep["mode"] == "compiled" and rep["build_id"] == bid.tree_digest()
    assert sorted(rep["compiled"]) == sorted(["pkg/libhipminer.so", "pkg/hm_miner"] +
                                             [f"build/hipminer/{n}" for n in names])
    assert rep["reused"] == []
    assert out.startswith("build: compiled (5 artifacts written") and bid.tree_digest() in out


def test_report_up_to_date_tree(tmp_path, monkeypatch, capsys):
    """Everything already built: make writes nothing, mode "reused"."""
    pkg, bd = _tree(tmp_path, monkeypatch)
    bd.mkdir(parents=True)
    (bd / "api.o").write_bytes(b"x")
    (pkg / "libhipminer.so").write_bytes(b"hipminer-build-id:" + bid.tree_digest().encode())
    monkeypatch.setattr(entry.subprocess, "run", _Make())
    entry.build()
    import json
    rep = json.loads((bd / "BUILD_REPORT").read_text())
    assert rep["mode"] == "reused" and rep["compiled"] == []
    assert rep["reused"] == ["build/hipminer/api.o", "pkg/libhipminer.so"]
    assert capsys.readouterr().out.startswith("build: reused (0 artifacts written")


def test_real_make_on_the_built_tree_reuses_everything():
    """The in-tree build is current (the suite runs after build()): a real
    make writes no artifact."""
    if bid.embedded_id(f"{entry.PKG}/libhipminer.so") != bid.tree_digest() or \
            not any(p.endswith(".o") for p in entry._artifacts()):
        pytest.skip("the in-tree build is not current (or its objects did not travel)")
    before = entry._artifacts()
    import subprocess
    subprocess.run(["make", "-s", "-C", f"{entry.PKG}/csrc"], check=True, capture_output=True)
    rep = entry.build_report(before, entry._artifacts(), None, 0.0)
    assert rep["mode"] == "reused", rep
    assert any(p.endswith("libhipminer.so") for p in rep["reused"])


def test_smoke_prints_the_build_record(tmp_path):
    """smoke() prints BUILD_REPORT's mode and compiled count next
    to the build id, so the driver's GPU-test tail shows whether the box
    compiled (stub reports; the real one is build()'s)."""
    import json
    rep = tmp_path / "BUILD_REPORT"
    rep.write_text(json.dumps({"mode": "compiled", "compiled": ["a.o", "b.o", "lib.so"],
                               "reused": ["x.hsaco"], "build_id": "0123456789abcdef",
                               "seconds": 12.5}))
    line = entry.build_record(str(rep))
    assert line == ("build_report mode=compiled compiled=3 reused=1 "
                    "build_id=0123456789abcdef seconds=12.5")
    rep.write_text(json.dumps({"mode": "reused", "compiled": [], "reused": ["a.o"],
                               "build_id": "f" * 16, "seconds": 0.4}))
    assert entry.build_record(str(rep)).startswith("build_report mode=reused compiled=0 reused=1")
    assert entry.build_record(str(tmp_path / "missing")).startswith("build_report none")
    rep.write_text("{not json")
    assert entry.build_record(str(rep)).startswith("build_report none")
    src = open(entry.__file__).read()
    assert "print(build_record()" in src.split("def smoke")[1]

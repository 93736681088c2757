"""The C-ABI library: loads, exports every symbol include/hipminer.h declares,
host-side semantics (hm_hash), error handling.  No GPU compute here."""
import ctypes
import os

import pytest

from distributed_bitcoinminer_amd import _lib


def test_exports_every_header_symbol():
    lib = _lib.load()
    syms = _lib.header_symbols()
    assert set(syms) >= {"hm_hash", "hm_open", "hm_scan", "hm_scan_stats", "hm_set_option",
                         "hm_strerror", "hm_close", "hm_version", "hm_scan_checked",
                         "hm_scan_many", "hm_partition", "hm_scan_stats_sized", "hm_build_id",
                         "hm_scan_cpu"}
    for s in syms:
        assert hasattr(lib, s), s


def test_library_is_gfx950_code_object():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_version_and_strerror():
    lib = _lib.load()
    assert lib.hm_version() >> 16 == 1
    assert lib.hm_version() & 0xFFFF >= 8  # 1.8: HM_OPT_DEADLINE_MS / HM_ERR_TIMEOUT
    for rc in range(0, -8, -1):
        assert _lib.strerror(rc) != "unknown error", rc
    assert _lib.strerror(-99) == "unknown error"
    assert "deadline" in _lib.strerror(_lib.HM_ERR_TIMEOUT)


def test_timeout_code_and_deadline_option_in_header():
    """ABI 1.8 (SURVEY §8(b) liveness): the header defines HM_ERR_TIMEOUT and
    HM_OPT_DEADLINE_MS with the values the bindings use (ctypes, cgo via the
    header itself), and hm_set_option checks the option's range."""
    import re
    text = open(_lib.HEADER_PATH).read()
    assert int(re.search(r"#define HM_ERR_TIMEOUT \((-?\d+)\)", text).group(1)) == \
        _lib.HM_ERR_TIMEOUT == -7
    assert int(re.search(r"#define HM_OPT_DEADLINE_MS (\d+)", text).group(1)) == \
        _lib.HM_OPT_DEADLINE_MS == 13
    assert _lib.load().hm_set_option(None, _lib.HM_OPT_DEADLINE_MS, 5) == _lib.HM_ERR_INVALID


def test_hm_hash_matches_golden(golden):
    for k in golden["hash_kats"]:
        m = bytes.fromhex(k["msg_hex"])
        assert _lib.host_hash(m, int(k["nonce"])) == int(k["hash"]), (k["name"], k["nonce"])


def test_null_args():
    lib = _lib.load()
    assert lib.hm_scan(None, b"x", 1, 0, 1, None) == _lib.HM_ERR_INVALID
    assert lib.hm_scan_checked(None, b"x", 1, 0, 1, None, None, None) == _lib.HM_ERR_INVALID
    assert lib.hm_open(None, -1, None) == _lib.HM_ERR_INVALID
    assert lib.hm_set_option(None, 1, 1) == _lib.HM_ERR_INVALID
    lib.hm_close(None)


def test_open_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(_lib.HipMinerError) as ei:
        _lib.Context([0])
    assert ei.value.rc == _lib.HM_ERR_NO_DEVICE


def test_struct_layouts_match_header(tmp_path):
    """The ctypes mirrors of hm_stats / hm_request / hm_result have the C
    layout (size and every field offset) that include/hipminer.h gives."""
    import subprocess
    fields = [f for f, _ in _lib.hm_stats._fields_]
    src = tmp_path / "layout.c"
    lines = ['#include <stddef.h>', '#include <stdio.h>', f'#include "{_lib.HEADER_PATH}"',
             "int main(void) {",
             '  printf("%zu %zu %zu\\n", sizeof(hm_stats), sizeof(hm_request), sizeof(hm_result));']
    lines += [f'  printf("%zu\\n", offsetof(hm_stats, {f}));' for f in fields]
    lines += ["  return 0;", "}"]
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-o", str(exe), str(src)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()
    sizes = [int(x) for x in out[:3]]
    assert sizes == [ctypes.sizeof(_lib.hm_stats), ctypes.sizeof(_lib.hm_request),
                     ctypes.sizeof(_lib.hm_result)]
    assert [int(x) for x in out[3:]] == [getattr(_lib.hm_stats, f).offset for f in fields]


def test_stats_size_is_pinned(tmp_path):
    """hm_stats only grows at its end: the 1.0-1.3 callers' 136-byte struct is
    the prefix before dom_compressions_eff, the 1.4/1.5 struct the 144 bytes
    before enqueue_ms, the 1.6/1.7 struct is 160 bytes, the 1.8 struct 168
    (+ deadline_ms), and hm_scan_stats_sized refuses a size below the oldest
    layout."""
    import subprocess
    src = tmp_path / "sz.c"
    src.write_text("\n".join([
        '#include <stddef.h>', '#include <stdio.h>', f'#include "{_lib.HEADER_PATH}"',
        "int main(void) {",
        '  printf("%zu %zu %zu %zu %d %d %d %d\\n", sizeof(hm_stats),',
        "         offsetof(hm_stats, dom_compressions_eff), offsetof(hm_stats, enqueue_ms),",
        "         offsetof(hm_stats, deadline_ms),",
        "         HM_STATS_SIZE_1_0, HM_STATS_SIZE_1_4, HM_STATS_SIZE_1_6, HM_STATS_SIZE_1_8);",
        "  return 0;", "}"]))
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-std=c11", "-o", str(exe), str(src)], check=True)
    out = [int(x) for x in subprocess.run([str(exe)], check=True, capture_output=True,
                                          text=True).stdout.split()]
    assert out == [168, 136, 144, 160, 136, 144, 160, 168]
    assert ctypes.sizeof(_lib.hm_stats) == 168
    lib = _lib.load()
    st = _lib.hm_stats()
    assert lib.hm_scan_stats_sized(None, ctypes.byref(st), 144) == _lib.HM_ERR_INVALID


def test_code_object_hash_is_the_embedded_blob():
    """bench.py matches PMC summaries to the code object inside the loaded
    library; that is the hsaco the Makefile embedded."""
    import hashlib
    import os
    sha = _lib.code_object_sha16()
    hsaco = os.path.join(os.path.dirname(os.path.dirname(_lib.LIB_PATH)), "build", "hipminer",
                         "hipminer_scan.hsaco")
    if os.path.exists(hsaco):
        assert sha == hashlib.sha256(open(hsaco, "rb").read()).hexdigest()[:16]
    assert len(sha) == 16


def test_build_id_is_this_trees_digest():
    """hm_build_id (ABI 1.6) is the digest of the sources the library was built
    from; the in-tree build matches this tree, the tag in the file's bytes
    (what build() reads) equals what the loaded library returns, and the
    digest covers every library source plus the header."""
    from distributed_bitcoinminer_amd import build_id as bid
    assert _lib.build_id() == bid.embedded_id(_lib.LIB_PATH)
    assert _lib.build_matches_tree(), (_lib.build_id(), bid.tree_digest())
    files = bid.source_files()
    for f in ("api.cpp", "scan_kernels.hip", "kernels.hip", "plan.cpp", "sha_device.hpp",
              "align_loops.py", "scan_blob.S", "Makefile"):
        assert f"distributed_bitcoinminer_amd/csrc/{f}" in files, f
    assert "include/hipminer.h" in files


def test_build_id_changes_with_any_source(tmp_path):
    """One changed byte in any covered source changes the digest."""
    import shutil
    from distributed_bitcoinminer_amd import build_id as bid
    root = tmp_path / "tree"
    for rel in bid.source_files():
        dst = root / rel
        dst.parent.mkdir(parents=True, exist_ok=True)
        shutil.copyfile(os.path.join(bid.ROOT, rel), dst)
    base = bid.tree_digest(str(root))
    assert base == bid.tree_digest()
    for rel in ("distributed_bitcoinminer_amd/csrc/scan_kernels.hip", "include/hipminer.h"):
        p = root / rel
        data = p.read_bytes()
        p.write_bytes(data + b" ")
        assert bid.tree_digest(str(root)) != base, rel
        p.write_bytes(data)
    assert bid.tree_digest(str(root)) == base


@pytest.mark.gpu
def test_scan_stats_writes_only_the_frozen_144_bytes(ctx):
    """ABI 1.7: hm_scan_stats writes HM_STATS_SIZE_1_4 bytes, never more, so a
    caller built against the 1.4/1.5 header (144-byte struct) is safe; the
    later fields come through hm_scan_stats_sized."""
    ctx.scan(b"bradfitz", 0, 99_999)
    lib = _lib.load()
    buf = (ctypes.c_uint8 * 256)(*([0xA5] * 256))
    assert lib.hm_scan_stats(ctx._h, ctypes.cast(buf, ctypes.POINTER(_lib.hm_stats))) == 0
    assert all(b == 0xA5 for b in buf[144:]), "hm_scan_stats wrote past 144 bytes"
    st = _lib.hm_stats.from_buffer_copy(bytes(buf[:ctypes.sizeof(_lib.hm_stats)]))
    full = ctx.stats()
    assert st.nonces == full["nonces"] == 100_000
    assert st.dom_compressions_eff == full["dom_compressions_eff"] > 0
    buf2 = (ctypes.c_uint8 * 256)(*([0xA5] * 256))
    assert lib.hm_scan_stats_sized(ctx._h, ctypes.cast(buf2, ctypes.POINTER(_lib.hm_stats)), 160) == 0
    assert all(b == 0xA5 for b in buf2[160:]) and bytes(buf2[:144]) == bytes(buf[:144])


def test_host_blocking_calls_only_in_counting_helpers():
    """hm_stats.mid_call_syncs counts host waits issued while a call is still
    enqueuing.  That holds by construction only if every host-blocking HIP
    call of the library (stream/device/event waits, hipFree, synchronous
    hipMemcpy) sits in the counting helpers host_wait / host_read, or in
    device_free (hm_close, outside any call).  Since ABI 1.8 no call frees
    device memory at all (hipFree waits for the whole device, other
    contexts' work included).  Scan every C++ source of the library for
    stray ones."""
    import re
    csrc = os.path.join(os.path.dirname(_lib.__file__), "csrc")
    blocking = re.compile(r"\b(hipStreamSynchronize|hipDeviceSynchronize|hipEventSynchronize|"
                          r"hipFree|hipMemcpy)\s*\(")
    allowed = {"host_wait", "host_read", "device_free"}
    func = re.compile(r"^[A-Za-z_][\w:<>*& ]*?\b(\w+)\s*\([^;]*\)\s*(const\s*)?\{\s*$")
    stray = []
    for name in sorted(os.listdir(csrc)):
        if not name.endswith((".cpp", ".hpp")):
            continue
        current = None
        for no, line in enumerate(open(os.path.join(csrc, name)), 1):
            m = func.match(line)
            if m:
                current = m.group(1)
            if blocking.search(line) and current not in allowed:
                stray.append(f"{name}:{no} in {current}: {line.strip()}")
    assert not stray, stray


def test_auto_deadline_model():
    """HM_OPT_DEADLINE_MS = -1 (ABI 1.8): 2 s + 8 x the modelled kernel time
    (seg_cost: measured SIMD cycles per 64 nonces per layout, over 4 SIMDs per
    CU at 2.4 GHz).  Host-only: the model a GPU miner's deadline comes from."""
    lib = _lib.load()

    def dl(msg, lo, hi, cus=256):
        return lib.hm_debug_auto_deadline_ms(msg, len(msg), lo, hi, cus)
    assert dl(b"bradfitz", 5, 4) == 2000.0                    # empty range
    assert 2000 < dl(b"bradfitz", 0, 10**7 + 1) < 2010        # config 1: ~0.3 ms of kernels
    cfg2 = dl(b"bradfitz", 0, 2**32 - 1)
    # 2^32 nonces at ~4150 SIMD cycles / 64 nonces on 1024 SIMDs: ~0.11 s
    assert 2800 < cfg2 < 3000, cfg2
    cfg4 = dl(b"bradfitz", 0, 2**40 - 1)
    assert 200_000 < cfg4 < 260_000, cfg4                    # ~29 s of kernels, x 8
    assert dl(b"bradfitz", 0, 2**32 - 1, cus=128) > cfg2      # fewer CUs: later deadline
    # the 120-B message runs C = 2 layouts partly: a later deadline than cfg2's
    import bench
    assert dl(bench.long120(), 0, 2**32 - 1) > 2000
    assert dl(b"", (1 << 64) - 10, (1 << 64) - 1) < 2001

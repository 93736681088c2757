"""The C-ABI library: loads, exports every symbol include/hipminer.h declares,
host-side semantics (hm_hash), error handling.  No GPU compute here."""
import ctypes

import pytest

from distributed_bitcoinminer_amd import _lib


def test_exports_every_header_symbol():
    lib = _lib.load()
    syms = _lib.header_symbols()
    assert set(syms) >= {"hm_hash", "hm_open", "hm_scan", "hm_scan_stats", "hm_set_option",
                         "hm_strerror", "hm_close", "hm_version", "hm_scan_checked",
                         "hm_scan_many", "hm_partition", "hm_scan_stats_sized"}
    for s in syms:
        assert hasattr(lib, s), s


def test_library_is_gfx950_code_object():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_version_and_strerror():
    lib = _lib.load()
    assert lib.hm_version() >> 16 == 1
    assert lib.hm_version() & 0xFFFF >= 5  # 1.5: hm_scan_stats_sized
    for rc in range(0, -7, -1):
        assert _lib.strerror(rc)
    assert _lib.strerror(-99) == "unknown error"


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
    the prefix before dom_compressions_eff, the 1.4+ struct is 144 bytes, and
    hm_scan_stats_sized refuses a size below the oldest layout."""
    import subprocess
    src = tmp_path / "sz.c"
    src.write_text("\n".join([
        '#include <stddef.h>', '#include <stdio.h>', f'#include "{_lib.HEADER_PATH}"',
        "int main(void) {",
        '  printf("%zu %zu %d %d\\n", sizeof(hm_stats), offsetof(hm_stats, dom_compressions_eff),',
        "         HM_STATS_SIZE_1_0, HM_STATS_SIZE_1_4);",
        "  return 0;", "}"]))
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-std=c11", "-o", str(exe), str(src)], check=True)
    out = [int(x) for x in subprocess.run([str(exe)], check=True, capture_output=True,
                                          text=True).stdout.split()]
    assert out == [144, 136, 136, 144]
    assert ctypes.sizeof(_lib.hm_stats) == 144
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

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
                         "hm_scan_many", "hm_partition"}
    for s in syms:
        assert hasattr(lib, s), s


def test_library_is_gfx950_code_object():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_version_and_strerror():
    lib = _lib.load()
    assert lib.hm_version() >> 16 == 1
    assert lib.hm_version() & 0xFFFF >= 4  # 1.4: hm_stats.merge / dom_compressions_eff
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

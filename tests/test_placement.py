"""The build-time instruction placement pass (distributed_bitcoinminer_amd/csrc/
align_loops.py, DESIGN.md §4 "Instruction placement"): its fix-up planner on
synthetic loops, and the invariant on the shipped scan-kernel assembly (every
8-byte VALU instruction of every hot loop starts at 4 mod 8).  CPU only."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "distributed_bitcoinminer_amd", "csrc")
sys.path.insert(0, CSRC)
import align_loops as al  # noqa: E402

ALIGNED = os.path.join(ROOT, "build", "hipminer", "scan_kernels.aligned.s")


def _insts(spec, base=0x100):
    """spec: list of (size, opcode) -> [(addr, size, op, None)]"""
    out, a = [], base
    for size, op in spec:
        out.append((a, size, op, None))
        a += size
    return out


def _layout(insts, order, promote, nops):
    """Addresses after applying a plan; returns [(addr, size, op)] in new order."""
    a, out = insts[order[0]][0], []
    for k in order:
        _, size, op, _ = insts[k]
        if k in nops:
            a += 4
        if k in promote:
            size, op = 8, al.PROMOTE[op]
        out.append((a, size, op))
        a += size
    return out


@pytest.mark.parametrize("all_e64", [True, False])
def test_plan_puts_every_8byte_valu_at_4_mod_8(all_e64, monkeypatch):
    monkeypatch.setattr(al, "ALL_E64", all_e64)
    spec = [(8, "v_alignbit_b32"), (8, "v_alignbit_b32"), (4, "v_lshrrev_b32_e32"),
            (8, "v_bitop3_b32"), (4, "s_add_i32"), (8, "v_add3_u32"), (4, "v_add_u32_e32"),
            (4, "v_add_u32_e32"), (8, "v_alignbit_b32"), (4, "s_lshl_b32"), (4, "s_nop"),
            (4, "s_add_i32"), (8, "v_bitop3_b32"), (4, "s_cbranch_scc1")]
    insts = _insts(spec)
    text = {k: f"\t{op} v{k}, v{k + 20}, v{k + 40}" for k, (_, op) in enumerate(spec)}
    order, promote, nops = al.plan_fixes(insts, 0, len(insts) - 1, text)
    assert sorted(order) == list(range(len(insts)))
    lay = _layout(insts, order, promote, nops)
    assert all(a % 8 == 4 for a, size, op in lay if size == 8 and op.startswith("v_"))
    if all_e64:
        assert not any(op.endswith("_e32") and op.startswith("v_") and op in al.PROMOTE
                       for _, _, op in lay)


def test_moves_respect_dependencies(monkeypatch):
    monkeypatch.setattr(al, "ALL_E64", False)
    # v_lshlrev (movable, not promotable) feeds the next 8-byte op: no move, s_nop instead
    spec = [(8, "v_alignbit_b32"), (4, "v_lshlrev_b32_e32"), (8, "v_bitop3_b32")]
    insts = _insts(spec, base=0x104)
    text = {0: "\tv_alignbit_b32 v1, v2, v2, 7", 1: "\tv_lshlrev_b32_e32 v3, 2, v1",
            2: "\tv_bitop3_b32 v4, v3, v5, v6 bitop3:0x96"}
    order, promote, nops = al.plan_fixes(insts, 0, 2, text)
    assert order == [0, 1, 2] and nops == {2}
    # independent: moved behind the 8-byte op, no padding
    text[1] = "\tv_lshlrev_b32_e32 v7, 2, v1"
    order, promote, nops = al.plan_fixes(insts, 0, 2, text)
    assert order == [0, 2, 1] and not nops and not promote


def test_moves_stay_in_their_block_and_clear_of_hazards(monkeypatch):
    """No swap across a label (another basic block) or in front of an
    instruction with wait-state rules (DPP / permlane / readlane): s_nop."""
    monkeypatch.setattr(al, "ALL_E64", False)
    spec = [(8, "v_alignbit_b32"), (4, "v_lshlrev_b32_e32"), (8, "v_bitop3_b32"),
            (8, "v_add3_u32")]
    insts = _insts(spec, base=0x104)
    text = {0: "\tv_alignbit_b32 v1, v2, v2, 7", 1: "\tv_lshlrev_b32_e32 v7, 2, v1",
            2: "\tv_bitop3_b32 v4, v3, v5, v6 bitop3:0x96", 3: "\tv_add3_u32 v8, v9, v9, v9"}
    between = {1: [], 2: [".LBB0_7:"], 3: []}
    order, promote, nops = al.plan_fixes(insts, 0, 3, text, between)
    assert order == [0, 1, 2, 3] and nops == {2}
    between[2] = ["\t; comment only"]
    order, promote, nops = al.plan_fixes(insts, 0, 3, text, between)
    assert order == [0, 2, 3, 1] and not nops  # moved behind both (independent)
    text[3] = "\tv_permlane32_swap_b32_e32 v7, v9"
    order, promote, nops = al.plan_fixes(insts, 0, 3, text, between)
    assert order == [0, 1, 2, 3] and nops == {2}


def test_block_structure_check():
    before = ["k:", "\tv_add_u32_e32 v1, v2, v3", "\ts_add_i32 s0, s1, 1",
              "\tv_xor_b32_e32 v4, v5, v6", ".LBB0_1:", "\tv_alignbit_b32 v1, v1, v1, 2",
              "\ts_cbranch_scc1 .LBB0_1"]
    ok = ["k:", "\tv_add_u32_e64 v1, v2, v3", "\ts_add_i32 s0, s1, 1",
          "\ts_nop 0", "\tv_xor_b32_e32 v4, v5, v6", ".LBB0_1:",
          "\tv_alignbit_b32 v1, v1, v1, 2", "\ts_cbranch_scc1 .LBB0_1"]
    al.check_blocks(before, ok)
    moved = ["k:", "\tv_add_u32_e32 v1, v2, v3", "\ts_add_i32 s0, s1, 1", ".LBB0_1:",
             "\tv_xor_b32_e32 v4, v5, v6", "\tv_alignbit_b32 v1, v1, v1, 2",
             "\ts_cbranch_scc1 .LBB0_1"]
    with pytest.raises(SystemExit):
        al.check_blocks(before, moved)
    scalar_moved = ["k:", "\ts_add_i32 s0, s1, 1", "\tv_add_u32_e32 v1, v2, v3",
                    "\tv_xor_b32_e32 v4, v5, v6", ".LBB0_1:", "\tv_alignbit_b32 v1, v1, v1, 2",
                    "\ts_cbranch_scc1 .LBB0_1"]
    with pytest.raises(SystemExit):
        al.check_blocks(before, scalar_moved)


@pytest.mark.skipif(not os.path.exists(ALIGNED), reason="library not built")
def test_shipped_scan_kernels_are_placed():
    with open(ALIGNED) as f:
        lines = f.read().split("\n")
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        obj = os.path.join(td, "a.o")
        al.assemble(ALIGNED, obj)
        funcs = al.disassemble(obj)
    where = al.source_insts(lines)
    production = [s for s in where if "hm_tiled_kernel" in s or "hm_chained_kernel" in s]
    assert len(production) == 33  # 32 tiled layouts + chained
    for sym in production:
        insts = funcs[sym]
        loop = al.hot_loop(insts, al.inner_headers(lines, where[sym]))
        assert loop is not None, sym
        good, n = al.stats(insts, *loop)
        assert good == n and n > 300, (sym, good, n)


FUSED = os.path.join(ROOT, "build", "hipminer", "fused_kernels.aligned.s")


@pytest.mark.skipif(not os.path.exists(FUSED), reason="library not built")
def test_shipped_fused_kernel_loops_are_placed():
    """The fused small-request kernel holds one hot loop per segment layout
    (32 tiled, chained, generic); the pass places every one of them."""
    with open(FUSED) as f:
        lines = f.read().split("\n")
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        obj = os.path.join(td, "a.o")
        al.assemble(FUSED, obj)
        funcs = al.disassemble(obj)
    where = al.source_insts(lines)
    sym = next(s for s in where if "hm_fused_kernel" in s)
    # placed code: e64 re-encoding can push a latch block up to twice as far
    # in front of its loop header
    loops = al.kernel_loops(sym, funcs[sym], al.inner_headers(lines, where[sym]),
                            latch_bytes=2 * al.LATCH_BYTES)
    assert len(loops) >= 34, len(loops)
    for lp in loops:
        good, n = al.stats(funcs[sym], *lp)
        assert good == n and n > 300, (lp, good, n)

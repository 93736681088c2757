#!/usr/bin/env python3
"""Instruction placement pass for the scan kernels' hot loops (build step).

gfx950 issues a long VALU stream measurably faster when its 8-byte (VOP3)
instructions start at addresses = 4 mod 8: the same hm_tiled_kernel inner
loop ran at 34.6 GH/s with 75 % of its 8-byte VALU instructions at 4 mod 8
and at 32.9 GH/s with 24 % (one 4-byte `s_nop` apart; same box, one process;
DESIGN.md §4 "Instruction placement").  hipcc leaves this to chance, so any
edit of the kernels could move a kernel by +-5 %.  MI355X_MICROARCH.md
("Code-placement sensitivity of hand-written streams") reports the same
effect for hand-written asm.

A second measured effect: beside half-rate ops, 4-byte (VOP2) full-rate ops
cost more than their 8-byte (VOP3, e64) encodings at 4 mod 8 -- a
half-rate + two full-rate pattern ran at 3.98 cycles per instruction with
v_add_u32_e32 and 3.32 with v_add_u32_e64 (tools/place_ubench.hip).

This pass makes the placement deliberate.  For every kernel whose innermost
loop holds >= MIN_LOOP instructions it first re-encodes every full-rate
4-byte VALU op of the loop that has an e64 form of the same rate (v_add_u32,
v_xor_b32, v_lshrrev_b32, ...: same operation, 8 bytes).  It then walks the
loop in address order and, whenever an 8-byte VALU instruction would start
at 0 mod 8 (behind an odd run of the remaining 4-byte instructions, which
are scalar ops), moves a 4-byte VALU op behind it when the two are
independent, or inserts `s_nop 0` in front of it.  Nothing else changes:
the same instructions, registers, order and waits.

usage: align_loops.py <in.s> <out.s> [--report] [--phase 4|0] [--no-nop] [--keep-e32]
(--phase 0, --no-nop and --keep-e32 are for placement experiments only.)
The input is `hipcc --cuda-device-only -S` output for gfx950; the output is
assembled into the code object that api.cpp loads (see the Makefile).  The
pass re-assembles its output and fails unless every 8-byte VALU instruction
of every hot loop starts at 4 mod 8.
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MIN_LOOP = 500
LATCH_BYTES = 64  # a latch block placed in front of the loop header
PROMOTE = {"v_add_u32_e32": "v_add_u32_e64", "v_xor_b32_e32": "v_xor_b32_e64",
           "v_or_b32_e32": "v_or_b32_e64", "v_and_b32_e32": "v_and_b32_e64",
           "v_sub_u32_e32": "v_sub_u32_e64", "v_mov_b32_e32": "v_mov_b32_e64",
           "v_lshrrev_b32_e32": "v_lshrrev_b32_e64"}
INST = re.compile(r"^\s+([a-z][a-z0-9_]*)(\s|$)")
FUNC = re.compile(r"^(_Z\w+):")
DIS = re.compile(r"^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-F]+):((?:\s[0-9A-F]{8})+)"
                 r"(?:\s*<(\S+)\+0x([0-9a-f]+)>)?")


def assemble(src_path, obj_path):
    subprocess.run([f"{LLVM}/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa",
                    "-mcpu=gfx950", "-c", src_path, "-o", obj_path], check=True)


def disassemble(obj_path):
    """symbol -> [(addr, size, opcode, branch_target_or_None)]"""
    out = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", obj_path],
                         capture_output=True, text=True, check=True).stdout
    funcs, base, cur = {}, {}, None
    for line in out.split("\n"):
        m = re.match(r"^([0-9a-f]+) <(\S+)>:", line)
        if m:
            cur = m.group(2)
            base[cur] = int(m.group(1), 16)
            funcs[cur] = []
            continue
        m = DIS.match(line)
        if m and cur:
            tgt = None
            if m.group(5) and m.group(5) in base:
                tgt = base[m.group(5)] + int(m.group(6), 16)
            funcs[cur].append((int(m.group(3), 16), 4 * len(m.group(4).split()), m.group(1), tgt))
    return funcs


def source_insts(lines):
    """symbol -> [line index of each instruction, in order]"""
    out, cur = {}, None
    for i, line in enumerate(lines):
        m = FUNC.match(line)
        if m:
            cur = m.group(1)
            out[cur] = []
            continue
        if line.startswith(".Lfunc_end"):
            cur = None
            continue
        if cur and INST.match(line):
            out[cur].append(i)
    return out


def inner_headers(lines, idx):
    """Instruction indices (into idx) that open an innermost loop, from the
    compiler's '; => This Inner Loop Header' annotations."""
    pos = {line_no: k for k, line_no in enumerate(idx)}
    heads = []
    for k, line_no in enumerate(idx):
        j = line_no - 1
        while j >= 0 and lines[j].lstrip().startswith(";"):
            if "Inner Loop Header" in lines[j]:
                heads.append(k)
                break
            j -= 1
    return heads


def hot_loop(insts, heads):
    """(first, last) instruction index of the innermost loop with the most
    instructions (>= MIN_LOOP), from its first block to its back-edge.  hipcc
    may place the loop's latch block just in front of the header; the back-edge
    then targets the latch.  Rare-path blocks placed after the back-edge are
    excluded."""
    best = None
    addr_index = {x[0]: i for i, x in enumerate(insts)}
    for k in heads:
        if k >= len(insts):
            continue
        head = insts[k][0]
        ends = [(i, x[3]) for i, x in enumerate(insts)
                if i > k and x[3] is not None and head - LATCH_BYTES <= x[3] <= head]
        if not ends:
            continue
        end, target = max(ends)
        first = addr_index[target]
        if end - first + 1 >= MIN_LOOP and (best is None or end - first > best[1] - best[0]):
            best = (first, end)
    return best


def all_loops(insts, heads, latch_bytes=None):
    """Every innermost loop with >= MIN_LOOP instructions, in address order
    (the fused kernel holds one hot loop per segment layout).  latch_bytes:
    how far before its header a loop's latch block may start (LATCH_BYTES;
    checks of already placed code pass more, since re-encoding grows it)."""
    latch = LATCH_BYTES if latch_bytes is None else latch_bytes
    out = []
    addr_index = {x[0]: i for i, x in enumerate(insts)}
    for k in heads:
        if k >= len(insts):
            continue
        head = insts[k][0]
        ends = [(i, x[3]) for i, x in enumerate(insts)
                if i > k and x[3] is not None and head - latch <= x[3] <= head]
        if not ends:
            continue
        end, target = max(ends)
        first = addr_index[target]
        if end - first + 1 >= MIN_LOOP:
            out.append((first, end))
    out = sorted(set(out))
    # innermost loops do not overlap; keep the first of any that would
    keep = []
    for lp in out:
        if not keep or lp[0] > keep[-1][1]:
            keep.append(lp)
    return keep


def kernel_loops(sym, insts, heads, latch_bytes=None):
    """The loops the pass places: every hot loop of the fused kernels, the
    single hottest loop of every other kernel."""
    if "fused" in sym:
        return all_loops(insts, heads, latch_bytes)
    lp = hot_loop(insts, heads)
    return [lp] if lp else []


PHASE = 4  # target start address mod 8 of 8-byte VALU instructions
NO_NOP = False
ALL_E64 = True  # re-encode every full-rate 4-byte VALU op of the loop


def stats(insts, lo, hi):
    big = [x for x in insts[lo:hi + 1] if x[1] == 8 and x[2].startswith("v_")]
    return sum(1 for x in big if x[0] % 8 == PHASE), len(big)


REG = re.compile(r"\b([vs])(\d+)\b|\b([vs])\[(\d+):(\d+)\]|\b(vcc|exec|scc|m0)\b")
# 4-byte VALU instructions that may trade places with the next 8-byte one:
# plain two-operand ALU ops without implicit operands
MOVABLE = set(PROMOTE) | {"v_lshrrev_b32_e32", "v_lshlrev_b32_e32", "v_ashrrev_i32_e32"}
# 8-byte VALU instructions they may be moved across: plain ALU, no lane
# crossing, no implicit VCC/EXEC
PLAIN8 = re.compile(r"^v_(alignbit|alignbyte|add3|bitop3|xad|lshl_add|lshl_or|and_or|or3|"
                    r"bfi|perm|add_u32_e64|xor_b32_e64|sub_u32_e64|lshl_add_u64)")


def regs(operands):
    out = set()
    for m in REG.finditer(operands):
        if m.group(1):
            out.add(m.group(1) + m.group(2))
        elif m.group(3):
            out.update(f"{m.group(3)}{r}" for r in range(int(m.group(4)), int(m.group(5)) + 1))
        else:
            out.add(m.group(6))
    return out


def rw(text):
    """(written, read) register sets of one VALU instruction line."""
    ops = text.split(None, 1)[1] if len(text.split(None, 1)) > 1 else ""
    ops = ops.split(";")[0].split("//")[0]
    parts = [p.strip() for p in ops.split(",")]
    return regs(parts[0]), regs(",".join(parts[1:]))


# instructions whose inputs are subject to gfx950 wait-state rules (lane
# crossing, VGPR -> SGPR reads) or that are such padding themselves: a swap
# must not bring a VALU write closer to them
HAZARD = re.compile(r"readlane|readfirstlane|writelane|permlane|_dpp|row_|quad_perm|"
                    r"bank_mask|s_nop|s_setreg|s_getreg|v_cmpx")


def same_block(between):
    """True when the source lines between two instructions hold no label or
    directive (only blank lines and comments), i.e. both sit in one block."""
    for line in between:
        t = line.strip()
        if t and not t.startswith(";") and not t.startswith("//"):
            return False
    return True


def plan_fixes(insts, lo, hi, text, between=None):
    """Make every 8-byte VALU instruction of insts[lo..hi] start at 4 mod 8.

    Returns (order, promote, nops): the new order of the loop's instruction
    indices, the indices re-encoded from 4 to 8 bytes, and the indices to be
    prefixed with `s_nop 0`.  Between two consecutive 8-byte VALU
    instructions an odd number of 4-byte instructions flips the parity; each
    such gap gets one fix, cheapest first: re-encode a full-rate 4-byte VALU
    op of the gap as e64; move the gap's last 4-byte VALU op behind the next
    8-byte instruction when the two are independent, in one basic block
    (`between[p]` = the source lines separating loop slots p-1 and p) and
    no hazard-sensitive instruction follows within three slots; else insert
    s_nop."""
    order = list(range(lo, hi + 1))
    promote, nops = set(), set()
    if ALL_E64:
        # every full-rate 4-byte VALU op becomes its 8-byte e64 form first
        promote = {k for k in order if insts[k][1] == 4 and insts[k][2] in PROMOTE}
        insts = list(insts)
        shift = 0
        for k in range(lo, len(insts)):
            a, size, op, tgt = insts[k]
            if k in promote:
                insts[k] = (a + shift, 8, PROMOTE[op], tgt)
                shift += 4
            else:
                insts[k] = (a + shift, size, op, tgt)
    addr = insts[lo][0]
    pos = 0
    gap = []  # positions (in order) of 4-byte instructions since the last 8-byte VALU
    while pos < len(order):
        k = order[pos]
        _, size, op, _ = insts[k]
        if size == 8 and op.startswith("v_"):
            if addr % 8 != PHASE:
                prom = [p for p in gap if insts[order[p]][2] in PROMOTE]
                last = gap[-1] if gap else None
                if prom:
                    promote.add(order[prom[-1]])
                    addr += 4
                elif (last == pos - 1 and insts[order[last]][2] in MOVABLE
                      and PLAIN8.match(op)
                      and (between is None or same_block(between[pos]))
                      and not any(HAZARD.search(text[order[q]])
                                  for q in range(pos + 1, min(pos + 4, len(order))))):
                    lw, lr = rw(text[order[last]])
                    ew, er = rw(text[k])
                    if not (lw & (ew | er)) and not (ew & lr):
                        # the 8-byte op now starts where the 4-byte one did
                        # (addr - 4, = 4 mod 8); the 4-byte op follows it and
                        # opens the next gap
                        order[last], order[pos] = order[pos], order[last]
                        addr += 4 + 4
                        gap = [pos]
                        pos += 1
                        continue
                    if not NO_NOP:
                        nops.add(k)
                        addr += 4
                elif not NO_NOP:
                    nops.add(k)
                    addr += 4
            gap = []
        elif size == 4:
            gap.append(pos)
        addr += size
        pos += 1
    return order, promote, nops


def blocks(lines, drop_nops):
    """Per basic block (split at labels): the non-VALU instructions with their
    index among the block's instructions, and the sorted VALU instructions,
    normalised (e64 re-encodings undone; with drop_nops, `s_nop 0` lines --
    the ones the pass inserts -- left out)."""
    undo = {v: k for k, v in PROMOTE.items()}
    out, cur = [], None
    for line in lines:
        t = line.split(";")[0].split("//")[0].strip()
        if not t:
            continue
        if re.match(r"^[\w.$]+:", t):
            cur = [t, [], []]
            out.append(cur)
            continue
        m = INST.match(line)
        if not m or cur is None:
            continue
        if drop_nops and t == "s_nop 0":
            continue
        op = m.group(1)
        t = t.replace(op, undo.get(op, op), 1)
        n = len(cur[1]) + len(cur[2])
        if op.startswith("v_"):
            cur[2].append(t)
        else:
            cur[1].append((n, t))
    return [(lab, scal, sorted(vec)) for lab, scal, vec in out]


def check_blocks(before, after):
    """The pass only re-encodes, swaps VALU ops inside a block and adds
    `s_nop 0`: every block must keep its label, its scalar/control
    instructions at the same positions and the same multiset of VALU ops
    (`s_nop 0` ignored on both sides; the count of the compiler's own is
    checked separately: the pass never removes one)."""
    a, b = blocks(before, True), blocks(after, True)
    if len(a) != len(b):
        raise SystemExit(f"block structure changed: {len(a)} -> {len(b)} blocks")
    nops = lambda ls: sum(1 for l in ls if l.split(";")[0].strip() == "s_nop 0")
    if nops(after) < nops(before):
        raise SystemExit("the placement pass lost an s_nop")
    for x, y in zip(a, b):
        if x != y:
            raise SystemExit(f"block {x[0]} changed by the placement pass")


def place(lines, report):
    """One placement pass over the assembly lines: returns the edited lines
    and {kernel: number of loops placed}."""
    with tempfile.TemporaryDirectory() as td:
        obj = os.path.join(td, "in.o")
        path = os.path.join(td, "in.s")
        with open(path, "w") as f:
            f.write("\n".join(lines))
        assemble(path, obj)
        funcs = disassemble(obj)
    where = source_insts(lines)
    edits = {}  # line index -> replacement text
    placed = {}
    for sym, insts in funcs.items():
        if sym not in where:
            continue
        idx = where[sym]
        # the disassembly may list the inter-function alignment padding too
        if len(idx) > len(insts):
            raise SystemExit(f"{sym}: {len(idx)} source vs {len(insts)} encoded instructions")
        loops = kernel_loops(sym, insts, inner_headers(lines, idx))
        if not loops:
            continue
        placed[sym] = len(loops)
        for k, (_, _, op, _) in enumerate(insts[:len(idx)]):
            if INST.match(lines[idx[k]]).group(1) != op:
                raise SystemExit(f"{sym}: instruction {k} is {op} in the object, "
                                 f"'{lines[idx[k]].strip()}' in the source")
        shift = 0  # bytes the edits of earlier loops of this kernel add
        for lo, hi in loops:
            shifted = [(a + shift, sz, op, t) for a, sz, op, t in insts] if shift else insts
            text = {k: lines[idx[k]] for k in range(lo, hi + 1)}
            between = {p: lines[idx[lo + p - 1] + 1: idx[lo + p]] for p in range(1, hi - lo + 1)}
            order, promote, nops = plan_fixes(shifted, lo, hi, text, between)
            shift += 4 * (len(promote) + len(nops))
            new = {}
            for k in range(lo, hi + 1):
                t = text[k]
                if k in promote:
                    t = t.replace(insts[k][2], PROMOTE[insts[k][2]], 1)
                if k in nops:
                    t = "\ts_nop 0\n" + t
                new[k] = t
            for slot, k in zip(range(lo, hi + 1), order):
                edits[idx[slot]] = new[k]
            if report:
                good, n = stats(shifted, lo, hi)
                moved = sum(1 for a, b in zip(range(lo, hi + 1), order) if a != b) // 2
                print(f"{sym[:64]:64s} loop {hi - lo + 1:5d} insts: {good:4d}/{n} 8-B VALU at "
                      f"4 mod 8 -> re-encode {len(promote)}, move {moved}, s_nop {len(nops)}")
    return [edits.get(i, l) for i, l in enumerate(lines)], placed


def misplaced(lines):
    """{kernel: 8-byte VALU instructions of its placed loops not at PHASE mod 8}."""
    with tempfile.TemporaryDirectory() as td:
        path, obj = os.path.join(td, "out.s"), os.path.join(td, "out.o")
        with open(path, "w") as f:
            f.write("\n".join(lines))
        assemble(path, obj)
        funcs = disassemble(obj)
    # the placed text may hold several instructions per line (s_nop + op)
    lines = "\n".join(lines).split("\n")
    where = source_insts(lines)
    bad = {}
    for sym, insts in funcs.items():
        if sym not in where:
            continue
        for lp in kernel_loops(sym, insts, inner_headers(lines, where[sym])):
            good, n = stats(insts, *lp)
            if good != n:
                bad[sym] = bad.get(sym, 0) + n - good
    return bad


def main():
    global PHASE, NO_NOP, ALL_E64
    src, dst = sys.argv[1], sys.argv[2]
    report = "--report" in sys.argv
    if "--phase" in sys.argv:
        PHASE = int(sys.argv[sys.argv.index("--phase") + 1])
    NO_NOP = "--no-nop" in sys.argv
    ALL_E64 = "--keep-e32" not in sys.argv
    with open(src) as f:
        lines = f.read().split("\n")
    out, placed = place(lines, report)
    # an alignment directive between two loops of one kernel can absorb the
    # bytes an earlier loop's edits add: place again until every loop holds
    for _ in range(4):
        bad = misplaced(out)
        if not bad or NO_NOP:
            break
        out, _ = place("\n".join(out).split("\n"), report)
    with open(dst, "w") as f:
        f.write("\n".join(out))
    with open(dst) as f:
        lines2 = f.read().split("\n")
    check_blocks(lines, lines2)
    bad = misplaced(lines2)
    if report:
        for sym, n in placed.items():
            print(f"  after: {sym[:60]:60s} {n} loop(s), {bad.get(sym, 0)} 8-byte VALU off {PHASE} mod 8")
    if bad and not NO_NOP:
        raise SystemExit(f"8-byte VALU instructions not at {PHASE} mod 8: {bad}")


if __name__ == "__main__":
    main()

"""Instruction alignment of a kernel's hot loop in a gfx950 code object (dev tool).

usage: python tools/loop_align.py <code-object.o> <symbol-substring>...
Reports, for the innermost loop holding >= 500 instructions: instruction
count, 8-byte (or longer) instructions, and how many of those start at an
address = 4 mod 8 (MI355X_MICROARCH.md "Code-placement sensitivity").
"""
import re
import subprocess
import sys

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
LINE = re.compile(r"^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-F]+):((?:\s[0-9A-F]{8})+)(?:\s*<(\S+)\+0x([0-9a-f]+)>)?")


def parse(path):
    out = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", path], capture_output=True,
                         text=True, check=True).stdout
    funcs, cur = {}, None
    for l in out.split("\n"):
        m = re.match(r"^([0-9a-f]+) <(\S+)>:", l)
        if m:
            cur = m.group(2)
            funcs[cur] = (int(m.group(1), 16), [])
            continue
        m = LINE.match(l)
        if m and cur:
            addr = int(m.group(3), 16)
            size = 4 * len(m.group(4).split())
            tgt = None
            if m.group(5):
                tgt = funcs[m.group(5)][0] + int(m.group(6), 16) if m.group(5) in funcs else None
            funcs[cur][1].append((addr, size, m.group(1), tgt))
    return funcs


def hot_loop(insts):
    best = None
    for i, (addr, size, op, tgt) in enumerate(insts):
        if tgt is not None and tgt <= addr and op.startswith("s_"):
            body = [x for x in insts if tgt <= x[0] <= addr]
            if len(body) >= 500 and (best is None or len(body) < len(best)):
                best = body
    return best


def main():
    funcs = parse(sys.argv[1])
    for pat in sys.argv[2:]:
        for name, (base, insts) in funcs.items():
            if pat not in name:
                continue
            body = hot_loop(insts)
            if not body:
                print(f"{name}: no hot loop")
                continue
            big = [x for x in body if x[1] >= 8]
            mis = [x for x in big if x[0] % 8 == 4]
            valu_big = [x for x in big if x[2].startswith("v_")]
            valu_mis = [x for x in valu_big if x[0] % 8 == 4]
            print(f"{name[:60]:60s} loop@{body[0][0] - base:#x} (mod 8 = {body[0][0] % 8}) "
                  f"insts={len(body)} bytes={sum(x[1] for x in body)} 8B+={len(big)} "
                  f"misaligned={len(mis)} ({100 * len(mis) / max(1, len(big)):.0f}%) "
                  f"valu8B misaligned={len(valu_mis)}/{len(valu_big)}")


if __name__ == "__main__":
    main()

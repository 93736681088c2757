"""ISA audit of the scan kernels (dev tool): per kernel the register use,
spills and scratch from the code-object metadata, and the VALU instruction
mix of the innermost loop body (one iteration = 64 nonces per wave for the
tiled and chained kernels).

usage: make -C distributed_bitcoinminer_amd/csrc asm
       python tools/isa_audit.py build/hipminer/scan_kernels.aligned.s > profiles/r03/isa_audit.txt
(the scan kernels as shipped, after the placement pass align_loops.py)

lane-spill-ops counts the v_writelane/v_readlane instructions SGPR spills
compile into, in the whole kernel and inside its hot loop.
model_cyc prices the loop with the measured gfx950 issue costs of DESIGN.md
§4 (half-rate 4.3, full-rate 2.4 cycles per wave64 instruction: the issue floor
of the placed hot loops, which the measured kernels reach within ≈1 %).
"""
import collections
import re
import sys

HALF = {"v_alignbit_b32", "v_add3_u32", "v_xad_u32", "v_bfi_b32", "v_lshl_or_b32",
        "v_lshl_add_u32", "v_or3_b32", "v_perm_b32", "v_and_or_b32", "v_alignbyte_b32",
        "v_mul_lo_u32", "v_lshlrev_b32_e64"}


def metadata(text):
    """kernel symbol -> dict of the metadata fields we report."""
    out = {}
    for block in re.split(r"\n  - ", text.split("amdhsa.kernels:")[-1]):
        m = re.search(r"\.name:\s+(\S+)", block)
        if not m:
            continue
        f = {}
        for key in ("vgpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
                    "private_segment_fixed_size"):
            k = re.search(r"\." + key + r":\s+(\d+)", block)
            f[key] = int(k.group(1)) if k else None
        out[m.group(1)] = f
    return out


def loop_mix(lines, start, end):
    body = lines[start:end]
    hdrs = [i for i, l in enumerate(body) if "Inner Loop Header" in l]
    if not hdrs:
        return None
    hdr = max(hdrs)
    stop = next((i for i in range(hdr, len(body)) if "s_cbranch_vccz" in body[i]), None)
    if stop is None:
        return None
    ops = [l.split()[0] for l in body[hdr:stop] if re.match(r"\s+v_", l)]
    return collections.Counter(ops)


def lane_spills(lines, start, end):
    """(in the hot loop, in the whole kernel) counts of the v_writelane /
    v_readlane pairs SGPR spills to VGPR lanes compile into."""
    body = lines[start:end]
    hdrs = [i for i, l in enumerate(body) if "Inner Loop Header" in l]
    lane = [i for i, l in enumerate(body) if re.match(r"\s+v_(read|write)lane_b32", l)]
    if not hdrs:
        return None, len(lane)
    hdr = max(hdrs)
    stop = next((i for i in range(hdr, len(body)) if "s_cbranch_vccz" in body[i]), hdr)
    return sum(1 for i in lane if hdr <= i < stop), len(lane)


def main(path):
    text = open(path).read()
    lines = text.split("\n")
    meta = metadata(text)
    starts = {}
    for i, l in enumerate(lines):
        m = re.match(r"^(_ZN2hm\w+):", l)
        if m:
            starts[m.group(1)] = i
    print("gfx950 ISA audit of distributed_bitcoinminer_amd/csrc/scan_kernels.hip "
          "(hipcc -O3, ROCm 7.2, after align_loops.py; tools/isa_audit.py)")
    print("inner loop = the per-nonce-iteration body (64 nonces per wave per iteration)\n")
    for sym in sorted(starts):
        if sym not in meta:
            continue
        i0 = starts[sym]
        i1 = next(i for i in range(i0, len(lines)) if lines[i].startswith(".Lfunc_end"))
        m = meta[sym]
        row = (f"{sym:60s} vgpr={m['vgpr_count']} sgpr={m['sgpr_count']} "
               f"spills={m['vgpr_spill_count']}/{m['sgpr_spill_count']} "
               f"scratch={m['private_segment_fixed_size']}")
        mix = loop_mix(lines, i0, i1) if ("tiled" in sym or "chained" in sym) else None
        in_loop, in_kernel = lane_spills(lines, i0, i1)
        if in_kernel:
            row += f" lane-spill-ops={in_kernel} (hot loop: {in_loop})"
        if mix:
            n = sum(mix.values())
            half = sum(v for k, v in mix.items() if k.split("_e32")[0] in HALF or k in HALF)
            cyc = half * 4.3 + (n - half) * 2.4
            top = " ".join(f"{k}:{v}" for k, v in mix.most_common(6))
            row += f"  loop VALU={n} half-rate={half} model_cyc={cyc:.0f} | {top}"
        print(row)


if __name__ == "__main__":
    main(sys.argv[1])

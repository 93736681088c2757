"""Hot-loop diff of each production scan kernel against its checked (CSUM)
twin (dev tool): what hm_scan_checked's kernels execute beyond the shipped
ones.  The production kernels are separate template instantiations
(CSUM = false); the checked ones add the key-sum / count accumulation and
skip the placement pass (align_loops.py re-encodes only production loops),
so the instruction multiset is compared with the _e32/_e64 encodings folded.

usage: make -C distributed_bitcoinminer_amd/csrc asm
       python tools/csum_isa_diff.py build/hipminer/scan_kernels.aligned.s > profiles/r04/csum_isa_diff.txt
"""
import collections
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from isa_audit import loop_mix  # noqa: E402


def fold(mix):
    out = collections.Counter()
    for k, v in mix.items():
        out[re.sub(r"_e(32|64)$", "", k)] += v
    return out


def main(path):
    lines = open(path).read().split("\n")
    spans = {}
    for i, l in enumerate(lines):
        m = re.match(r"^(_ZN2hm\w+):", l)
        if m:
            j = next(k for k in range(i, len(lines)) if lines[k].startswith(".Lfunc_end"))
            spans[m.group(1)] = (i, j)
    print("hot-loop VALU diff, checked (CSUM) minus production kernel, encodings folded "
          "(tools/csum_isa_diff.py)\n")
    worst = 0
    for sym in sorted(spans):
        if "_csum_" in sym or not ("tiled" in sym or "chained" in sym):
            continue
        twin = sym.replace("15hm_tiled_kernel", "20hm_tiled_csum_kernel") \
                  .replace("17hm_chained_kernel", "22hm_chained_csum_kernel")
        if twin not in spans:
            print(f"{sym}: no checked twin")
            continue
        a = fold(loop_mix(lines, *spans[sym]) or {})
        b = fold(loop_mix(lines, *spans[twin]) or {})
        extra = {k: b[k] - a[k] for k in sorted(set(a) | set(b)) if b[k] != a[k]}
        core_equal = all(b[k] >= a[k] for k in a)
        worst = max(worst, sum(b.values()) - sum(a.values()))
        print(f"{sym:58s} prod={sum(a.values()):5d} csum={sum(b.values()):5d} "
              f"+{sum(b.values()) - sum(a.values()):3d} production ops all present: "
              f"{core_equal} | {' '.join(f'{k}:{v:+d}' for k, v in extra.items())}")
    print(f"\nlargest addition: {worst} VALU instructions per 64-nonce iteration")


if __name__ == "__main__":
    main(sys.argv[1])

"""Count VALU instructions in a kernel's innermost loop body (dev tool).
usage: python tools/isa_count.py build/hipminer/kernels.s <symbol-substring>..."""
import re, sys
text = open(sys.argv[1]).read().split("\n")
for pat in sys.argv[2:]:
    start = next(i for i, l in enumerate(text) if l.startswith("_ZN") and pat in l and l.split(":")[0].endswith("E"))
    end = next(i for i in range(start, len(text)) if text[i].startswith(".Lfunc_end"))
    body = text[start:end]
    # innermost loop: the last "Inner Loop Header" label up to its back-edge region's first vccz branch
    hdr = max(i for i, l in enumerate(body) if "Inner Loop Header" in l)
    stop = next(i for i in range(hdr, len(body)) if "s_cbranch_vccz" in body[i])
    ops = [l.split()[0] for l in body[hdr:stop] if re.match(r"\s+v_", l)]
    from collections import Counter
    c = Counter(ops)
    half = sum(v for k, v in c.items() if k.split("_e")[0] in ("v_alignbit_b32", "v_add3_u32", "v_xad_u32", "v_bfi_b32", "v_lshl_or_b32", "v_lshl_add_u32", "v_or3_b32", "v_perm_b32"))
    print(f"{pat}: VALU={len(ops)} half-rate={half} model_cycles={half*4.28 + (len(ops)-half)*3.45:.0f}  {dict(c.most_common(6))}")

#!/bin/bash
# Placement experiment (dev tool): builds libhipminer variants whose scan
# kernels are shifted by 8*k bytes (k = the arguments), by inserting 2k
# `s_nop 0` at every kernel entry of the shipped assembly
# (build/hipminer/scan_kernels.aligned.s).  The 8-byte multiple keeps every
# hot-loop VALU op at 4 mod 8 (align_loops.py) and moves the loops' offset
# within the 64/128-B instruction-cache lines.  Output:
# ${PAD_OUT:-build/ab_pad}/<k>/libhipminer.so, for tools/ab_libs.py on the GPU box.
# usage: tools/build_pad_variants.sh 0 1 2 ...   (after a normal build)
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
B=$ROOT/build/hipminer
LLVM=/opt/rocm/lib/llvm/bin
for k in "$@"; do
    D=$ROOT/${PAD_OUT:-build/ab_pad}/$k
    mkdir -p $D
    python3 - "$B/scan_kernels.aligned.s" "$D/scan.s" "$k" <<'EOF'
import re, sys
src, dst, k = sys.argv[1], sys.argv[2], int(sys.argv[3])
out = []
for line in open(src):
    out.append(line)
    if re.match(r"^_ZN2hm\w+_kernel\w*:", line):
        out.extend(["\ts_nop 0\n"] * (2 * k))
open(dst, "w").writelines(out)
EOF
    $LLVM/clang -x assembler -target amdgcn-amd-amdhsa -mcpu=gfx950 -c $D/scan.s -o $D/scan.o
    $LLVM/ld.lld -shared $D/scan.o -o $D/hipminer_scan.hsaco
    g++ -c $ROOT/distributed_bitcoinminer_amd/csrc/scan_blob.S -Wa,-I,$D -o $D/scan_blob.o
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $D/libhipminer.so \
        $B/kernels.o $B/api.o $B/plan.o $D/scan_blob.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
    rm -f $D/scan.s $D/scan.o
done

#!/bin/bash
# Compiler-flag experiment (dev tool): builds libhipminer variants whose scan
# kernels are compiled with extra device flags (e.g. an LLVM scheduling
# strategy), through the same placement pass and link as the Makefile.
# usage: tools/build_flag_variants.sh name1 "flags1" name2 "flags2" ...
#   (after a normal build; output build/ab_flags/<name>/libhipminer.so)
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
B=$ROOT/build/hipminer
C=$ROOT/distributed_bitcoinminer_amd/csrc
LLVM=/opt/rocm/lib/llvm/bin
while [ $# -ge 2 ]; do
    name=$1; flags=$2; shift 2
    D=$ROOT/build/ab_flags/$name
    mkdir -p $D
    (cd $C && /opt/rocm/bin/hipcc -O3 -std=c++20 --offload-arch=gfx950 --cuda-device-only -S \
        $flags scan_kernels.hip -o $D/scan.s)
    python3 $C/align_loops.py $D/scan.s $D/scan.aligned.s --report > $D/align_report.txt
    $LLVM/clang -x assembler -target amdgcn-amd-amdhsa -mcpu=gfx950 -c $D/scan.aligned.s -o $D/scan.o
    $LLVM/ld.lld -shared $D/scan.o -o $D/hipminer_scan.hsaco
    g++ -c $C/scan_blob.S -Wa,-I,$D -o $D/scan_blob.o
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $D/libhipminer.so \
        $B/kernels.o $B/api.o $B/plan.o $D/scan_blob.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
    python3 $ROOT/tools/isa_audit.py $D/scan.aligned.s | grep -E "tiled_kernelILi4ELb0ELb0|chained_kernelENS" \
        | sed "s/^/$name: /" | cut -c1-200
    rm -f $D/scan.s $D/scan.o
done

#!/bin/bash
# Experiment builds (dev tool): libhipminer variants whose scan kernels are
# compiled with extra device flags (e.g. -DHM_LDS_DISPENSER), through the
# same placement pass and link as the Makefile.  Run after a normal build.
# usage: tools/build_variant.sh name1 "flags1" [name2 "flags2" ...]
#   -> build/ab_var/<name>/libhipminer.so
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
B=$ROOT/build/hipminer
C=$ROOT/distributed_bitcoinminer_amd/csrc
LLVM=/opt/rocm/lib/llvm/bin
while [ $# -ge 2 ]; do
    name=$1; flags=$2; shift 2
    D=$ROOT/build/ab_var/$name
    mkdir -p $D
    objs=""
    for k in scan_kernels fused_kernels; do
        (cd $C && /opt/rocm/bin/hipcc -O3 -std=c++20 --offload-arch=gfx950 --cuda-device-only -S \
            $flags $k.hip -o $D/$k.s)
        python3 $C/align_loops.py $D/$k.s $D/$k.aligned.s --report > $D/$k.align_report.txt
        $LLVM/clang -x assembler -target amdgcn-amd-amdhsa -mcpu=gfx950 -c $D/$k.aligned.s -o $D/$k.o
        objs="$objs $D/$k.o"
        rm -f $D/$k.s
    done
    $LLVM/ld.lld -shared $objs -o $D/hipminer_scan.hsaco
    g++ -c $C/scan_blob.S -Wa,-I,$D -o $D/scan_blob.o
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $D/libhipminer.so \
        $B/kernels.o $B/api.o $B/plan.o $B/host_scan.o $D/scan_blob.o -L/opt/rocm/lib -lrccl \
        -pthread -Wl,-rpath,/opt/rocm/lib
    rm -f $D/*.o
    echo "$name: $D/libhipminer.so"
done

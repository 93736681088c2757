set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02cq2; mkdir -p $O
M3=$(python -c "import random;r=random.Random(440);print(''.join(chr(r.choice(range(0x21,0x7f))) for _ in range(120)))")
timeout -k 10 300 python -u tools/ab_libs.py 15 build/ab/lib_l3.so build/ab/lib_cq5.so -- "$M3" 0 4294967295 > $O/ab_cfg3_a.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py 15 build/ab/lib_cq5.so build/ab/lib_l3.so -- "$M3" 0 4294967295 > $O/ab_cfg3_b.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab_libs.py 15 build/ab/lib_base.so build/ab/lib_cq5.so > $O/ab_cfg2.txt 2>&1
rc=$?; cat $O/*.txt; exit $rc

/* scan_blob.S -- embeds the scan kernels' code object (hipminer_scan.hsaco,
 * built from scan_kernels.hip by the Makefile: hipcc -S, align_loops.py,
 * clang -x assembler, ld.lld) into libhipminer.so; api.cpp loads it per
 * device with hipModuleLoadData. */
    .section .rodata.hm_scan_code_object, "a", @progbits
    .globl hm_scan_code_object
    .type hm_scan_code_object, @object
    .p2align 12
hm_scan_code_object:
    .incbin "hipminer_scan.hsaco"
    .size hm_scan_code_object, . - hm_scan_code_object
    .globl hm_scan_code_object_end
hm_scan_code_object_end:
    .section .note.GNU-stack, "", @progbits

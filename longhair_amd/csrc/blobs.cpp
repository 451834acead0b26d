// blobs.cpp -- embeds data files into the shared library at build time.
//
//  lh_cauchy_tables_blob : data/cauchy_tables_256.bin (the reference's generator
//                          constants, see tools/extract_tables.py)
//  lh_jit_source         : csrc/jit_codec.hip, the kernel template compiled at run time
//                          by hiprtc for each (k, m, bytes) configuration (jit.cpp)
//  lh_inv_jump_source    : csrc/inv_jump.inc, the computed-jump GF(256) multiply (asm
//                          text) that the fused large-m decode module includes
//
// LH_SRC_DIR is the absolute path of longhair_amd/ (set by the Makefile).
#ifndef LH_SRC_DIR
#error "LH_SRC_DIR must be defined"
#endif

#define LH_STR2(x) #x
#define LH_STR(x) LH_STR2(x)

__asm__(
    ".section .rodata\n"
    ".balign 16\n"
    ".global lh_cauchy_tables_blob\n"
    ".hidden lh_cauchy_tables_blob\n"
    "lh_cauchy_tables_blob:\n"
    ".incbin \"" LH_STR(LH_SRC_DIR) "/data/cauchy_tables_256.bin\"\n"
    ".global lh_cauchy_tables_blob_end\n"
    ".hidden lh_cauchy_tables_blob_end\n"
    "lh_cauchy_tables_blob_end:\n"
    ".byte 0\n"
    ".balign 16\n"
    ".global lh_jit_source\n"
    ".hidden lh_jit_source\n"
    "lh_jit_source:\n"
    ".incbin \"" LH_STR(LH_SRC_DIR) "/csrc/jit_codec.hip\"\n"
    ".byte 0\n"
    ".balign 16\n"
    ".global lh_inv_jump_source\n"
    ".hidden lh_inv_jump_source\n"
    "lh_inv_jump_source:\n"
    ".incbin \"" LH_STR(LH_SRC_DIR) "/csrc/inv_jump.inc\"\n"
    ".byte 0\n"
    ".previous\n");

#!/usr/bin/env python3
"""Generate longhair_amd/csrc/inv_jump.inc: the asm text of the large-m decode's phase-B
multiply (kernels.hip lh_inverse_gt_kernel and its fallback; jit.cpp's fused windowed
decode).  Body c (68 bytes: 8 VOP3 v_bitop3_b32 + the return) adds B(c) V to the 8
accumulator words of one output: output sub-row y is acc ^= tl[lo] ^ th[hi] with (lo, hi)
the nibbles of c * 2^y in GF(2^8)/0x187, tl / th the 16-entry XOR tables of V's sub-rows
0..3 / 4..7 (entry 0 = the inline constant 0).

Two renderings of the same 256 bodies:
  LH_INV_JUMPI8_*   the table inside the asm statement (one copy per call site), 8 outputs
  LH_INV_GTAB_TEXT  the table once per code object, entered by LH_INV_JUMPG<n>_ASM
Run `make -C longhair_amd/csrc regen-inv-jump` after editing; tests/test_abi.py checks that
the committed file equals this script's output."""
import os


def xt(v):
    return ((v << 1) ^ (0x87 if v & 0x80 else 0)) & 0xFF


# Indexed variant: one copy of the table serves all JO outputs of a wave.  The accumulators
# of output i are pinned to v[BASE + 8i .. BASE + 8i + 7]; the table is written for output 0
# and reached with GPR indexing on (SRC0 and DST relative, index 8i), each body returning
# through s[94:95].  Entry 0 of the nibble tables is the inline constant 0.
IDX_BASE = 40


def render_indexed(jo):
    """Asm text of LH_INV_JUMPI<jo>_ASM.  Operands: the JO x 8 pinned accumulators (not
    named in the text), [c0] / [c1] the coefficient bytes of outputs 0-3 / 4-7 (SGPRs),
    [t1]..[t15] / [h1]..[h15] the nibble tables (VGPRs)."""
    # Per output: the body address from the coefficient byte (4 SALU), the accumulator index
    # (GPR indexing stays on across the outputs: only SALU runs between the bodies, so the
    # index just moves on), and s_swappc_b64, which jumps and leaves the return address in
    # s[94:95] for the body's s_setpc_b64.
    body = ["s_mov_b32 s97, m0", "s_getpc_b64 s[88:89]", "1:",
            "s_add_u32 s90, s88, (3f-1b)", "s_addc_u32 s91, s89, 0"]
    for i in range(jo):
        body += [f"s_bfe_u32 s96, %[c{i // 4}], {0x80000 | (8 * (i % 4)):#x}",
                 "s_mul_i32 s96, s96, 68",
                 "s_add_u32 s92, s90, s96", "s_addc_u32 s93, s91, 0",
                 "s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)" if i == 0 else f"s_set_gpr_idx_idx {8 * i}",
                 "s_nop 0",
                 "s_swappc_b64 s[94:95], s[92:93]"]
    body += ["s_set_gpr_idx_off", "s_branch 4f", "3:"]
    for c in range(256):
        v = c
        for y in range(8):
            lo, hi = v & 15, v >> 4
            a = f"v{IDX_BASE + y}"
            s1 = f"%[t{lo}]" if lo else "0"
            s2 = f"%[h{hi}]" if hi else "0"
            body.append(f"v_bitop3_b32 {a}, {a}, {s1}, {s2} bitop3:0x96")
            v = xt(v)
        body.append("s_setpc_b64 s[94:95]")
    body += ["4:", "s_mov_b32 m0, s97"]
    lines = [f"#define LH_INV_JUMPI{jo}_ASM \\"]
    for i, b in enumerate(body):
        lines.append(f'    "{b}\\n"' + (" \\" if i + 1 < len(body) else ""))
    return lines


# Global-table variant (lh_inverse_gt_kernel): the 256 bodies live once per code object, in
# the never-launched kernel lh_inv_gtab_holder, under the hidden symbol lh_inv_gtab; every
# register they touch is fixed: tl[q] in v[GT_TL + q], th[q] in v[GT_TH + q] (q = 1..15),
# the accumulators of output i in v[IDX_BASE + 8i ..] reached by GPR indexing on VSRC2 and
# VDST (the accumulator is the bitop's third source, so v_readlane's VGPR source is not
# moved by the index).  The caller holds the absolute low address of each output's body in a
# VGPR (lane r: row r's coefficient), so per output only v_readlane + the index + s_swappc
# run: 3 SALU with the body's s_setpc_b64, against 7 for LH_INV_JUMPI.
GT_TL, GT_TH = 8, 24
GT_MAX = 8


def render_global_table():
    """Asm text of LH_INV_GTAB_TEXT: s_endpgm (the holder kernel's own code), then the table."""
    body = ["s_endpgm", ".p2align 8", ".hidden lh_inv_gtab", ".globl lh_inv_gtab", "lh_inv_gtab:"]
    for c in range(256):
        v = c
        for y in range(8):
            lo, hi = v & 15, v >> 4
            a = f"v{IDX_BASE + y}"
            s1 = f"v{GT_TL + lo}" if lo else "0"
            s2 = f"v{GT_TH + hi}" if hi else "0"
            body.append(f"v_bitop3_b32 {a}, {s1}, {s2}, {a} bitop3:0x96")
            v = xt(v)
        body.append("s_setpc_b64 s[94:95]")
    lines = ["#define LH_INV_GTAB_TEXT \\"]
    for i, b in enumerate(body):
        lines.append(f'    "{b}\\n"' + (" \\" if i + 1 < len(body) else ""))
    return lines


def render_global_call(n):
    """Asm text of LH_INV_JUMPG<n>_ASM: outputs 0 .. n-1 of one row.  Operands: [a0]..[a7]
    the outputs' body addresses (VGPRs, lane r = row r), [r] the row (SGPR), [hi] the high
    word of the table address (SGPR), the pinned tables and accumulators (not named)."""
    body = ["s_mov_b32 s97, m0", "s_mov_b32 s93, %[hi]"]
    for i in range(n):
        body.append(f"v_readlane_b32 s92, %[a{i}], %[r]")
        body.append("s_set_gpr_idx_on 0, gpr_idx(SRC2,DST)" if i == 0 else f"s_set_gpr_idx_idx {8 * i}")
        body.append("s_swappc_b64 s[94:95], s[92:93]")
    body += ["s_set_gpr_idx_off", "s_mov_b32 m0, s97"]
    lines = [f"#define LH_INV_JUMPG{n}_ASM \\"]
    for i, b in enumerate(body):
        lines.append(f'    "{b}\\n"' + (" \\" if i + 1 < len(body) else ""))
    outs = ", ".join(f'"+{{v{IDX_BASE + 8 * i + y}}}"(acc[{i}][{y}])' for i in range(n) for y in range(8))
    lines.append(f"#define LH_INV_JUMPG{n}_OUTS(acc) {outs}")
    return lines


# Two-dword table (round 5): a lane owns 8 bytes of every sub-block, so one jump adds B(c) V
# to 16 accumulator words -- half the jumps per byte of the one-dword table, whose cost is the
# jump (s_swappc / s_setpc round trip, ~100 cycles per jump per SIMD in phase B) more than its 8
# VALU.  Body c (132 bytes: 16 v_bitop3_b32 + the return) in lh_inv_gtab2; tl[q] in
# v[W2_TL + 2q .. + 1], th[q] in v[W2_TH + 2q .. + 1] (q = 1..15), the 16 accumulators of output
# i in v[W2_ACC + 16 i ..] (sub-row y, dword d at + 2y + d), reached by GPR indexing (16 i).
W2_TL, W2_TH, W2_ACC = 8, 40, 72
W2_MAX = 4


def render_global_table2():
    """Asm text of LH_INV_GTAB2_TEXT: s_endpgm, then the 256 two-dword bodies."""
    body = ["s_endpgm", ".p2align 8", ".hidden lh_inv_gtab2", ".globl lh_inv_gtab2", "lh_inv_gtab2:"]
    for c in range(256):
        v = c
        for y in range(8):
            lo, hi = v & 15, v >> 4
            for d in range(2):
                a = f"v{W2_ACC + 2 * y + d}"
                s1 = f"v{W2_TL + 2 * lo + d}" if lo else "0"
                s2 = f"v{W2_TH + 2 * hi + d}" if hi else "0"
                body.append(f"v_bitop3_b32 {a}, {s1}, {s2}, {a} bitop3:0x96")
            v = xt(v)
        body.append("s_setpc_b64 s[94:95]")
    lines = ["#define LH_INV_GTAB2_TEXT \\"]
    for i, b in enumerate(body):
        lines.append(f'    "{b}\\n"' + (" \\" if i + 1 < len(body) else ""))
    return lines


def render_global_call2(n):
    """Asm text of LH_INV_JUMPG2_<n>_ASM: outputs 0 .. n-1 of one row through lh_inv_gtab2
    (operands as LH_INV_JUMPG<n>_ASM; the index steps by 16)."""
    body = ["s_mov_b32 s97, m0", "s_mov_b32 s93, %[hi]"]
    for i in range(n):
        body.append(f"v_readlane_b32 s92, %[a{i}], %[r]")
        body.append("s_set_gpr_idx_on 0, gpr_idx(SRC2,DST)" if i == 0 else f"s_set_gpr_idx_idx {16 * i}")
        body.append("s_swappc_b64 s[94:95], s[92:93]")
    body += ["s_set_gpr_idx_off", "s_mov_b32 m0, s97"]
    lines = [f"#define LH_INV_JUMPG2_{n}_ASM \\"]
    for i, b in enumerate(body):
        lines.append(f'    "{b}\\n"' + (" \\" if i + 1 < len(body) else ""))
    outs = ", ".join(f'"+{{v{W2_ACC + 16 * i + j}}}"(acc[{i}][{j}])' for i in range(n) for j in range(16))
    lines.append(f"#define LH_INV_JUMPG2_{n}_OUTS(acc) {outs}")
    return lines


def render():
    """The text of inv_jump.inc."""
    lines = ["// generated by tools/gen_inv_jump.py -- do not edit",
             f"#define LH_INV_IDX_BASE {IDX_BASE}"]
    lines += render_indexed(8)
    outs = ", ".join(f'"+{{v{IDX_BASE + 8 * i + y}}}"(a[{i}][{y}])' for i in range(8) for y in range(8))
    lines.append(f"#define LH_INV_JUMPI8_OUTS(a) {outs}")
    ins = ", ".join([f'[t{q}] "v"(tl[{q}])' for q in range(1, 16)] + [f'[h{q}] "v"(th[{q}])' for q in range(1, 16)])
    lines.append(f"#define LH_INV_JUMPI_INS(tl, th) {ins}")
    lines += render_global_table()
    for n in range(1, GT_MAX + 1):
        lines += render_global_call(n)
    gins = ", ".join([f'"{{v{GT_TL + q}}}"(tl[{q}])' for q in range(1, 16)]
                     + [f'"{{v{GT_TH + q}}}"(th[{q}])' for q in range(1, 16)]
                     + [f'[a{i}] "v"(t[{i}])' for i in range(GT_MAX)])
    lines.append(f"#define LH_INV_JUMPG_INS(tl, th, t) {gins}")
    lines.append(f"#define LH_INV_W2_ACC {W2_ACC}")
    lines += render_global_table2()
    for n in range(1, W2_MAX + 1):
        lines += render_global_call2(n)
    gins2 = ", ".join([f'"{{v{W2_TL + 2 * q + d}}}"(tl[{q}][{d}])' for q in range(1, 16) for d in range(2)]
                      + [f'"{{v{W2_TH + 2 * q + d}}}"(th[{q}][{d}])' for q in range(1, 16) for d in range(2)]
                      + [f'[a{i}] "v"(t[{i}])' for i in range(W2_MAX)])
    lines.append(f"#define LH_INV_JUMPG2_INS(tl, th, t) {gins2}")
    return "\n".join(lines) + "\n"


OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "longhair_amd", "csrc",
                   "inv_jump.inc")


def main():
    """Writes inv_jump.inc (`make -C longhair_amd/csrc regen-inv-jump`)."""
    with open(OUT, "w") as f:
        f.write(render())


if __name__ == "__main__":
    main()

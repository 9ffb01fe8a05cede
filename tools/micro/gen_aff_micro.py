#!/usr/bin/env python3
"""Generates tools/micro/aff_micro.inc: candidate steady-state steps of the affine fill
as 32-step inline-asm blocks, for tools/micro/aff_micro.hip (cycles per step of one
wave alone, of one wave per SIMD, of two per SIMD).  Register numbers follow
tools/gen_block_asm.py's affine loop: TOP (G, F) pairs v64.., cells v128..
Variants:
  L_cur   the round-2 local step (G space, clamp by a per-step SGPR, best by G - Zb)
  L_x     X space (X = H + (r+2)|ge|): clamp folded into E (a per-lane constant),
          best = max X (no per-step offset), subject weight by cmp/cndmask
  L_xl    L_x with the weight from a per-lane byte LUT (v_perm_b32 on 4 subject codes)
  L_xl_np L_xl without the publishing shift register
  L_xl_ds L_xl publishing by ds_write_b128 of two steps' (G, F) from every lane
  G_cur   the round-2 plain step (global / semiglobal)
  G_l     G_cur with the LUT weight
"""
import os

AT0, AO0 = 64, 128
AW, AA, AH, AT = 192, 193, 194, 195
SW = 196   # 8 subject words v196..v203
WB = 204   # LUT weight bytes

v = lambda n: f"v{n}"
TG = lambda u: v(AT0 + 2 * u)
TF = lambda u: v(AT0 + 2 * u + 1)
OG = lambda u: v(AO0 + 2 * u)
OF = lambda u: v(AO0 + 2 * u + 1)


def step_cur(e, u, L, pub=True):
    tg = "%[tfg]" if u == 0 else TG(u - 1)
    tf = "%[tff]" if u == 0 else TF(u - 1)
    g = "%[cur]" if u == 0 else OG(u - 1)
    f = "%[fd]" if u == 0 else OF(u - 1)
    dg = "%[dg]" if u == 0 else ("%[tfg]" if u == 1 else TG(u - 2))
    e(f"v_cmp_eq_u32_sdwa vcc, %[q], {v(SW + u // 4)} src0_sel:DWORD src1_sel:BYTE_{u % 4}")
    e(f"v_cndmask_b32_e32 v{AW}, %[wx], %[wm], vcc")
    e(f"v_mov_b32_dpp {tf}, {f} wave_shr:1 row_mask:0xf bank_mask:0xf")
    e(f"v_mov_b32_dpp {tg}, {g} wave_shr:1 row_mask:0xf bank_mask:0xf")
    e("v_max_i32_e32 %[e], %[e], %[hg]")
    e(f"v_add_u32_e32 v{AA}, {dg}, v{AW}")
    e(f"v_max3_i32 {OG(u)}, v{AA}, %[e], {tf}")
    if L:
        e(f"v_max_i32_e32 {OG(u)}, %[z], {OG(u)}")
    e(f"v_add_u32_e32 %[hg], %[go], {OG(u)}")
    e(f"v_max_i32_e32 {OF(u)}, {tf}, %[hg]")
    if L:
        if u % 2 == 0:
            e(f"v_subrev_u32_e32 v{AH}, %[zb], {OG(u)}")
        else:
            e(f"v_subrev_u32_e32 v{AT}, %[zb], {OG(u)}")
            e(f"v_max3_i32 %[best], %[best], v{AH}, v{AT}")
        e("s_add_u32 %[z], %[z], %[nge]")
        e("s_add_u32 %[zb], %[zb], %[nge]")
    if pub and u >= 2:
        e(f"v_mov_b32_dpp {OG(u - 1)}, {OG(u - 2)} wave_shl:1 row_mask:0xf bank_mask:0xf")
        e(f"v_mov_b32_dpp {OF(u - 1)}, {OF(u - 2)} wave_shl:1 row_mask:0xf bank_mask:0xf")


def step_x(e, u, L, lut, pub="shift"):
    tg = "%[tfg]" if u == 0 else TG(u - 1)
    tf = "%[tff]" if u == 0 else TF(u - 1)
    g = "%[cur]" if u == 0 else OG(u - 1)
    f = "%[fd]" if u == 0 else OF(u - 1)
    dg = "%[dg]" if u == 0 else ("%[tfg]" if u == 1 else TG(u - 2))
    e(f"v_mov_b32_dpp {tf}, {f} wave_shr:1 row_mask:0xf bank_mask:0xf")
    e(f"v_mov_b32_dpp {tg}, {g} wave_shr:1 row_mask:0xf bank_mask:0xf")
    if lut:
        if u % 4 == 0:
            e(f"v_perm_b32 v{WB}, %[lh], %[ll], {v(SW + u // 4)}")
        e(f"v_add_u32_sdwa v{AA}, {dg}, sext(v{WB}) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD "
          f"src1_sel:BYTE_{u % 4}")
    else:
        e(f"v_cmp_eq_u32_sdwa vcc, %[q], {v(SW + u // 4)} src0_sel:DWORD src1_sel:BYTE_{u % 4}")
        e(f"v_cndmask_b32_e32 v{AW}, %[wx], %[wm], vcc")
        e(f"v_add_u32_e32 v{AA}, {dg}, v{AW}")
    if L:
        e("v_max3_i32 %[e], %[e], %[hg], %[zl]")
        e("v_add_u32_e32 %[e], %[ge], %[e]")
    else:
        e("v_max_i32_e32 %[e], %[e], %[hg]")
    e(f"v_max3_i32 {OG(u)}, v{AA}, %[e], {tf}")
    e(f"v_add_u32_e32 %[hg], %[go], {OG(u)}")
    e(f"v_max_i32_e32 {OF(u)}, {tf}, %[hg]")
    if L and u % 2 == 1:
        e(f"v_max3_i32 %[best], %[best], {OG(u - 1)}, {OG(u)}")
    if pub == "shift" and u >= 2:
        e(f"v_mov_b32_dpp {OG(u - 1)}, {OG(u - 2)} wave_shl:1 row_mask:0xf bank_mask:0xf")
        e(f"v_mov_b32_dpp {OF(u - 1)}, {OF(u - 2)} wave_shl:1 row_mask:0xf bank_mask:0xf")
    if pub == "ds" and u % 2 == 1:
        e(f"ds_write_b128 %[pa], v[{AO0 + 2 * (u - 1)}:{AO0 + 2 * u + 1}] offset:{16 * (u // 2)}")


def step_es(e, u, pub="none"):
    """X-space local step with the E update split (round 4 experiment): E + ge from the
    previous E alone, hge = X + go + ge beside hg = X + go, E' = max3(E + ge, hge, zl + ge):
    one more instruction, but the E recurrence is X -> hge -> E -> X (3 links, was 4)."""
    tg = "%[tfg]" if u == 0 else TG(u - 1)
    tf = "%[tff]" if u == 0 else TF(u - 1)
    g = "%[cur]" if u == 0 else OG(u - 1)
    f = "%[fd]" if u == 0 else OF(u - 1)
    dg = "%[dg]" if u == 0 else ("%[tfg]" if u == 1 else TG(u - 2))
    if u % 4 == 0:
        e(f"v_perm_b32 v{WB}, %[lh], %[ll], {v(SW + u // 4)}")
    e(f"v_add_u32_e32 %[e], %[ge], %[e]")
    e(f"v_add_u32_sdwa v{AA}, {dg}, sext(v{WB}) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD "
      f"src1_sel:BYTE_{u % 4}")
    e("v_max3_i32 %[e], %[e], %[hg], %[zl]")       # hg holds X + go + ge here
    e(f"v_mov_b32_dpp {tf}, {f} wave_shr:1 row_mask:0xf bank_mask:0xf")
    e(f"v_mov_b32_dpp {tg}, {g} wave_shr:1 row_mask:0xf bank_mask:0xf")
    e(f"v_max3_i32 {OG(u)}, v{AA}, %[e], {tf}")
    e(f"v_add_u32_e32 %[hg], %[go], {OG(u)}")
    e(f"v_max_i32_e32 {OF(u)}, {tf}, %[hg]")
    e(f"v_add_u32_e32 %[hg], %[ge], %[hg]")       # + ge for the next E
    if u % 2 == 1:
        e(f"v_max3_i32 %[best], %[best], {OG(u - 1)}, {OG(u)}")


def step_ro(e, u, L, pub=True):
    """X-space (L) / G-space LUT step with the instructions reordered so that no VALU
    reads the result of the instruction right before it (round 4 experiment):
    e1 = max3(e, hg, zl) first, the DPP moves between the E pair, the shift-register
    moves between OG -> hg -> OF, and the best after hg."""
    tg = "%[tfg]" if u == 0 else TG(u - 1)
    tf = "%[tff]" if u == 0 else TF(u - 1)
    g = "%[cur]" if u == 0 else OG(u - 1)
    f = "%[fd]" if u == 0 else OF(u - 1)
    dg = "%[dg]" if u == 0 else ("%[tfg]" if u == 1 else TG(u - 2))
    if L:
        e("v_max3_i32 %[e], %[e], %[hg], %[zl]")
    else:
        e("v_max_i32_e32 %[e], %[e], %[hg]")
    if u % 4 == 0:
        e(f"v_perm_b32 v{WB}, %[lh], %[ll], {v(SW + u // 4)}")
    e(f"v_add_u32_sdwa v{AA}, {dg}, sext(v{WB}) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD "
      f"src1_sel:BYTE_{u % 4}")
    e(f"v_mov_b32_dpp {tf}, {f} wave_shr:1 row_mask:0xf bank_mask:0xf")
    if L:
        e("v_add_u32_e32 %[e], %[ge], %[e]")
    e(f"v_mov_b32_dpp {tg}, {g} wave_shr:1 row_mask:0xf bank_mask:0xf")
    e(f"v_max3_i32 {OG(u)}, v{AA}, %[e], {tf}")
    if pub and u >= 2:
        e(f"v_mov_b32_dpp {OF(u - 1)}, {OF(u - 2)} wave_shl:1 row_mask:0xf bank_mask:0xf")
    e(f"v_add_u32_e32 %[hg], %[go], {OG(u)}")
    if L and u % 2 == 1:
        e(f"v_max3_i32 %[best], %[best], {OG(u - 1)}, {OG(u)}")
    if pub and u >= 2:
        e(f"v_mov_b32_dpp {OG(u - 1)}, {OG(u - 2)} wave_shl:1 row_mask:0xf bank_mask:0xf")
    e(f"v_max_i32_e32 {OF(u)}, {tf}, %[hg]")


def block(variant):
    out = []
    e = out.append
    for i in range(8):   # the block's subject words (as the real loop's double-buffered reads)
        e(f"ds_read_b32 {v(SW + i)}, %[sa] offset:{4 * i}")
    e("s_waitcnt lgkmcnt(0)")
    for u in range(32):
        if variant == "L_cur":
            step_cur(e, u, True)
        elif variant == "G_cur":
            step_cur(e, u, False)
        elif variant == "L_x":
            step_x(e, u, True, False)
        elif variant == "L_xl":
            step_x(e, u, True, True)
        elif variant == "L_xl_np":
            step_x(e, u, True, True, pub="none")
        elif variant == "L_xl_ds":
            step_x(e, u, True, True, pub="ds")
        elif variant == "G_l":
            step_x(e, u, False, True)
        elif variant == "L_es_np":
            step_es(e, u)
        elif variant == "L_ro":
            step_ro(e, u, True)
        elif variant == "L_ro_np":
            step_ro(e, u, True, pub=False)
        elif variant == "G_ro":
            step_ro(e, u, False)
        else:
            raise ValueError(variant)
    e(f"v_mov_b32_e32 %[cur], {OG(31)}")
    e(f"v_mov_b32_e32 %[fd], {OF(31)}")
    e(f"v_mov_b32_e32 %[dg], {TG(30)}")
    e(f"v_mov_b32_e32 %[tfg], {TG(31)}")
    e(f"v_mov_b32_e32 %[tff], {TF(31)}")
    if variant == "L_xl_ds":
        e("s_waitcnt lgkmcnt(0)")
    return out


VARIANTS = ["L_cur", "L_x", "L_xl", "L_xl_np", "L_xl_ds", "G_cur", "G_l", "L_es_np", "L_ro", "L_ro_np", "G_ro"]


def main():
    here = os.path.dirname(os.path.abspath(__file__))
    lines = ["// GENERATED by tools/micro/gen_aff_micro.py", ""]
    for name in VARIANTS:
        lines.append(f"#define AFFM_{name} \\")
        for ln in block(name):
            lines.append(f'    "{ln}\\n" \\')
        lines.append("")
    clob = ", ".join(f'"v{n}"' for n in range(AT0, WB + 1))
    lines.append(f"#define AFFM_CLOBBERS {clob}, \"vcc\"")
    lines.append("")
    open(os.path.join(here, "aff_micro.inc"), "w").write("\n".join(lines))


if __name__ == "__main__":
    main()

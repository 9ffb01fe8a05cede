#!/usr/bin/env python3
"""Variants of the production affine steady-state loop for the two-waves-per-SIMD question
(verdict round 4, item 4).  Takes one loop macro of anyseq_amd/csrc/anyseq_block_asm.inc
(two unrolled blocks, every hand-off counter treated as satisfied: the poll sub-loops and
the loop branches are cut out) and writes one macro per instruction subset:

  FULL        everything that remains (VALU, SALU, LDS, code loads, waits)
  VALU        the VALU instructions only (no v_readfirstlane)
  VALU_LDS    + LDS instructions and lgkmcnt waits
  VALU_SALU   + scalar ALU instructions (no waits, no branches)
  VALU_WAIT   + every s_waitcnt (nothing outstanding but the block's own)
  VALU_GLOB   + the code-row loads and vmcnt waits
  NODPP       VALU with every DPP move a plain v_mov (timing only: wrong values)
  NOSDWA      VALU with the byte-select adds plain v_add
  NOMAX3      VALU with v_max3 as v_max of its first two sources
  PLAIN       all three substitutions
  PLAIN64     PLAIN in 64-bit encodings (v_*_e64)
  R2FULL / R2VALU, R3FULL / R3VALU   two / three rows per lane (rn_transform: the projection
              that preceded the product's gen_aff2 nrows; its whole loop / its VALU)

tools/micro/mix_micro.hip times each at one and two compute waves per SIMD.
Diagnostic tool, not part of the product.
usage: gen_mix_micro.py MACRO_NAME OUT.inc
"""
import re
import sys


def macro_lines(text, name):
    start = text.index(f"#define {name} \\")
    out = []
    for line in text[start:].splitlines()[1:]:
        m = re.match(r'\s*"(.*)\\n"\s*\\?$', line)
        if not m:
            break
        out.append(m.group(1))
    return out


def loop_body(lines):
    i0 = lines.index("L_top_%=:") + 1
    i1 = max(i for i, l in enumerate(lines) if l.startswith("s_cbranch_scc1 L_top_%="))
    body, skip = [], None
    for l in lines[i0:i1]:
        if skip:
            if l == skip:
                skip = None
            continue
        m = re.match(r"s_cbranch_scc1 (L_\w+_ok)_%=", l)
        if m:
            skip = m.group(1) + "_%=:"
            continue
        m = re.match(r"s_cbranch_scc1 (L_\w+)_%=", l)
        if m and m.group(1).startswith(("L_cw", "L_no")):
            # short forward branches of the generator (code wait, ts, ...): keep the
            # taken-never path by dropping the branch, the label stays harmless
            continue
        if l.startswith(("s_cbranch", "s_branch")) or l.endswith(":"):
            continue
        body.append(l)
    return body


def kind(l):
    op = l.split()[0]
    if op == "v_readfirstlane_b32":
        return "rfl"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("global_"):
        return "glob"
    if op == "s_waitcnt":
        return "vmwait" if "vmcnt" in l else "lgkwait"
    if op in ("s_sleep", "s_memrealtime", "s_memtime", "s_setprio"):
        return "misc"
    if op.startswith("s_"):
        return "salu"
    return "other"


SUBSETS = {
    "FULL": {"valu", "rfl", "lds", "glob", "vmwait", "lgkwait", "salu", "misc"},
    "VALU": {"valu"},
    "VALU_LDS": {"valu", "lds", "lgkwait"},
    "VALU_SALU": {"valu", "salu"},
    "VALU_WAIT": {"valu", "vmwait", "lgkwait"},
    "VALU_GLOB": {"valu", "glob", "vmwait"},
}


def nodpp(l):
    if l.startswith("v_mov_b32_dpp"):
        a = l.split()
        return f"v_mov_b32_e32 {a[1]} {a[2]}"
    return l


def nosdwa(l):
    m = re.match(r"v_add_u32_sdwa (\S+), (\S+), sext\((\S+)\)", l)
    return f"v_add_u32_e32 {m.group(1)}, {m.group(2)}, {m.group(3)}" if m else l


def nomax3(l):
    m = re.match(r"v_max3_i32 (\S+), (\S+), (\S+), (\S+)", l)
    return f"v_max_i32_e32 {m.group(1)}, {m.group(2)}, {m.group(3)}" if m else l


SUBST = {
    "NODPP": nodpp,
    "NOSDWA": nosdwa,
    "NOMAX3": nomax3,
    "PLAIN": lambda l: nomax3(nosdwa(nodpp(l))),
    # the same plain operations in the 64-bit VOP3 encoding: instruction bytes, not kind
    "PLAIN64": lambda l: nomax3(nosdwa(nodpp(l))).replace("_e32 ", "_e64 "),
}


def rn_transform(body, nrows=2):
    """nrows rows per lane (round 5 projection, G space): after each step's cell A (row
    nrows*l) the lane computes the cells below it (rows nrows*l+1 ..) from the cell above
    without a lane shift -- each its own E chain, its LUT (another query code, the same
    subject byte), its diagonal from the row above's previous cell, F and H from the row
    above's new cell -- and the lane shifts, the shift register and the publish carry the
    last row's cells (the band's bottom row).  A's rotation v128..v135 is mirrored by row
    k's v(128 + 40 + 10 (k-1)) ..; the two registers after each rotation are its diagonal
    sum and weight bytes.  Named operands of row k: eb/hgb/llb/lhb (k = 1), ec/hgc/llc/lhc."""
    def base(k):
        return 40 + 10 * (k - 1)

    def kmap(r, k):
        n = int(r[1:])
        return f"v{n + base(k)}" if k and 128 <= n <= 135 else r

    last = nrows - 1
    tag = {1: "b", 2: "c", 3: "d"}
    # each row's cell of the previous step (row k's diagonal: row k-1's; step 0: the last rotation slot)
    out, prev = [], ["v134"] + [f"v{134 + base(k)}" for k in range(1, nrows - 1)]
    perm_src, byte, cur_oga = None, 0, None
    for l in body:
        m = re.match(r"v_mov_b32_dpp (v\d+), (\S+) (wave_shr|wave_shl)(.*)", l)
        if m:
            dst, src = m.group(1), m.group(2)
            if m.group(3) == "wave_shl":
                dst = kmap(dst, last)
            src = kmap(src, last) if src.startswith("v") else src
            out.append(f"v_mov_b32_dpp {dst}, {src} {m.group(3)}{m.group(4)}")
            continue
        m = re.match(r"ds_write_b64 (v\d+), v\[(\d+):(\d+)\](.*)", l)
        if m:
            a0, a1 = int(m.group(2)), int(m.group(3))
            if 128 <= a0 <= 135:
                a0, a1 = a0 + base(last), a1 + base(last)
            out.append(f"ds_write_b64 {m.group(1)}, v[{a0}:{a1}]{m.group(4)}")
            continue
        m = re.match(r"v_mov_b32_e32 (%\[(?:cur|fd)\]), (v\d+)$", l)
        if m:
            out.append(f"v_mov_b32_e32 {m.group(1)}, {kmap(m.group(2), last)}")
            continue
        m = re.match(r"v_perm_b32 v160, %\[lh\], %\[ll\], (v\d+)", l)
        if m:
            perm_src = m.group(1)
        m = re.search(r"src1_sel:BYTE_(\d)", l)
        if m and l.startswith("v_add_u32_sdwa v137"):
            byte = int(m.group(1))
        m = re.match(r"v_max3_i32 (v\d+), v137, %\[e\], (v\d+)", l)
        if m:
            cur_oga = m.group(1)
        out.append(l)
        m = re.match(r"v_max_i32_e32 (v\d+), (v\d+), %\[hg\]$", l)
        if m and cur_oga:
            above_g, above_f = cur_oga, m.group(1)
            for k in range(1, nrows):
                t, bk = tag[k], base(k)
                og, of = kmap(cur_oga, k), kmap(m.group(1), k)
                aa, wb = f"v{136 + bk}", f"v{137 + bk}"
                out.append(f"v_max_i32_e32 %[e{t}], %[e{t}], %[hg{t}]")
                if perm_src:
                    out.append(f"v_perm_b32 {wb}, %[lh{t}], %[ll{t}], {perm_src}")
                out.append(f"v_add_u32_sdwa {aa}, {prev[k - 1]}, sext({wb}) dst_sel:DWORD dst_unused:UNUSED_PAD "
                           f"src0_sel:DWORD src1_sel:BYTE_{byte}")
                out.append(f"v_max3_i32 {og}, {aa}, %[e{t}], {above_f}")
                out.append(f"v_add_u32_e32 %[hg{t}], %[go], {og}")
                out.append(f"v_max_i32_e32 {of}, {above_f}, %[hg{t}]")
                prev[k - 1] = above_g
                above_g, above_f = og, of
            perm_src = None
            cur_oga = None
    return out


def r2_transform(body):
    return rn_transform(body, 2)



def steady_path(lines):
    """The loop's executed path in the steady state (every counter satisfied, the cached
    hand-off counter sufficient): from L_top, conditional branches to the cached-counter
    read paths (L_sar / L_sbd) and to the poll exits (*_ok) taken, every other conditional
    branch not taken; ends at the loop's back branch."""
    labels = {l[:-1]: i for i, l in enumerate(lines) if l.endswith(":")}
    i, out = labels["L_top_%="] + 1, []
    while True:
        l = lines[i]
        if l.startswith("s_cbranch_scc1 L_top_%="):
            return out
        m = re.match(r"s_cbranch_scc[01] (L_\w+_%=)", l)
        if m:
            lab = m.group(1)
            if re.match(r"L_(sar|sbd)\d|L_\w+_ok_", lab):
                i = labels[lab] + 1
            else:
                i += 1
            continue
        m = re.match(r"s_branch (L_\w+_%=)", l)
        if m:
            i = labels[m.group(1)] + 1
            continue
        if not l.endswith(":"):
            out.append(l)
        i += 1


def lgkm_ops(l):
    op = l.split()[0]
    return 1 if op.startswith("ds_") else 0


def remap_waits(orig, new):
    """`new` is `orig` with LDS operations inserted (a leading '+') or removed (a leading
    '-': still counted in the original numbering, not issued): every s_waitcnt
    lgkmcnt(N) of `orig` keeps waiting for the same original operations.  Two copies of
    the body stand for the loop's steady state; the second is returned."""
    n2 = new + new
    res, k_orig, ops = [], 0, []   # ops issued: (is_orig, orig_index)
    for l in n2:
        tag = l[0] if l[:1] in "+-" else ""
        body = l[1:] if tag else l
        m = re.match(r"s_waitcnt lgkmcnt\((\d+)\)", body)
        if m and not tag:
            need = k_orig - int(m.group(1))          # original ops [0, need) complete
            cand = [j for j, (io, oi) in enumerate(ops) if io and oi < need]
            n2v = len(ops) - (max(cand) + 1) if cand else len(ops)
            body = f"s_waitcnt lgkmcnt({min(15, n2v)})"
        elif lgkm_ops(body):
            if tag == "-":
                k_orig += 1
                continue
            ops.append((tag != "+", k_orig if tag != "+" else -1))
            if tag != "+":
                k_orig += 1
        elif tag == "-":
            continue
        res.append(body)
    return res[len(res) // 2:]


def dspub_transform(body, width=2):
    """Publishing without the DPP shift register: every step's cell pair leaves by one
    ds_write_b64 from every lane (lane 63 into the next band's ring chunk, the others into
    a dummy area: per-lane address %[pds] + the chunk slot masked by %[pm63]), so the two
    wave_shl moves per step go and the half publish keeps only its counter write.
    width 1: only G (ds_write_b32; timing only)."""
    out = [
        "s_sub_u32 %[x3], %[b], 2",
        "s_lshl_b32 %[x3], %[x3], 8",
        "s_and_b32 %[x3], %[x3], 4095",
        "s_add_u32 %[x3], %[x3], %[nb]",
        "v_and_or_b32 v156, %[x3], %[pm63], %[pds]",
    ]
    out = ["+" + l if l.startswith("ds_") else l for l in out]
    u, hold = 0, False
    for l in body:
        if "wave_shl" in l:
            continue
        if l.startswith("ds_write_b64") and "v156" in l:
            out.append("-" + l)          # the half's data (the counter write stays)
            continue
        if l.startswith("v_and_or_b32 v156") :
            continue
        out.append(l)
        m = re.match(r"v_max_i32_e32 (v\d+), v\d+, %\[hg\]$", l)
        if m:
            of = int(m.group(1)[1:])
            og = of - 1
            if width == 2:
                out.append(f"+ds_write_b64 v156, v[{og}:{of}] offset:{8 * (u % 32)}")
            else:
                out.append(f"+ds_write_b32 v156, v{og} offset:{8 * (u % 32)}")
            u += 1
    # the block-start address for the second block of the body
    res, blk = [], 0
    for l in out:
        res.append(l)
    # second block: recompute the address after the first block's end (s_mov b, x1)
    final = []
    for l in res:
        final.append(l)
        if l.startswith("s_mov_b32 %[b], %[x1]") and blk == 0:
            blk = 1
            final += ["s_sub_u32 %[x3], %[b], 2", "s_lshl_b32 %[x3], %[x3], 8", "s_and_b32 %[x3], %[x3], 4095",
                      "s_add_u32 %[x3], %[x3], %[nb]", "v_and_or_b32 v156, %[x3], %[pm63], %[pds]"]
    return final


def packed_body(nrows):
    """Projection of a packed 16-bit G-space step, VALU + lane moves only:
    two lane-aligned problems in the low / high halves of every register, nrows rows per
    lane, 64 steps.  Per row and step: E v_pk_max_i16; the weight pair from the two
    problems' LUT bytes (one v_perm per problem every 4 steps, one v_perm per step packing
    the step's two bytes zero-extended); diagonal v_pk_add_u16; the cell two v_pk_max_i16
    (no packed max3); H+go v_pk_add_u16; F v_pk_max_i16.  Per step two DPP moves in (row 0's
    top G and F-in) and two shift-register moves out (the last row's pair).  Registers
    v64..v127 (the product loop's clobber range); values are not meaningful (timing only)."""
    CA, CB = 64, 72                      # 32 steps of codes per problem
    RB = lambda k: 80 + 12 * k           # per row: E, hg, G0, G1, F, lutAlo, lutAhi, lutBlo, lutBhi, wA, wB, aa
    TF, TG0, TG1, WP, SRG, SRF, GO = 116, 117, 118, 119, 120, 121, 122
    SEL = [123, 124, 125, 126]
    assert nrows <= 3
    out = []
    e = out.append
    for step in range(64):
        u = step % 32
        cur, prv = step % 2, 1 - step % 2
        tg, dg = (TG0, TG1) if cur == 0 else (TG1, TG0)
        last = nrows - 1
        for k in range(nrows):
            b = RB(k)
            if u % 4 == 0:
                e(f"v_perm_b32 v{b + 9}, v{b + 6}, v{b + 5}, v{CA + u // 4}")
                e(f"v_perm_b32 v{b + 10}, v{b + 8}, v{b + 7}, v{CB + u // 4}")
            e(f"v_pk_max_i16 v{b}, v{b}, v{b + 1}")
            if k == 0:
                # the lane above's last row (previous step's cell and F-down)
                e(f"v_mov_b32_dpp v{TF}, v{RB(last) + 4} wave_shr:1 row_mask:0xf bank_mask:0xf")
                e(f"v_mov_b32_dpp v{tg}, v{RB(last) + 2 + prv} wave_shr:1 row_mask:0xf bank_mask:0xf")
            e(f"v_perm_b32 v{WP}, v{b + 10}, v{b + 9}, v{SEL[u % 4]}")
            diag = dg if k == 0 else RB(k - 1) + 2 + prv
            e(f"v_pk_add_u16 v{b + 11}, v{diag}, v{WP}")
            fin = TF if k == 0 else RB(k - 1) + 4
            e(f"v_pk_max_i16 v{b + 2 + cur}, v{b + 11}, v{b}")
            e(f"v_pk_max_i16 v{b + 2 + cur}, v{b + 2 + cur}, v{fin}")
            e(f"v_pk_add_u16 v{b + 1}, v{b + 2 + cur}, v{GO}")
            e(f"v_pk_max_i16 v{b + 4}, v{fin}, v{b + 1}")
        e(f"v_mov_b32_dpp v{SRG}, v{RB(last) + 2 + cur} wave_shl:1 row_mask:0xf bank_mask:0xf")
        e(f"v_mov_b32_dpp v{SRF}, v{RB(last) + 4} wave_shl:1 row_mask:0xf bank_mask:0xf")
    return out


def main():
    name, out = sys.argv[1], sys.argv[2]
    text = open("anyseq_amd/csrc/anyseq_block_asm.inc").read()
    body = loop_body(macro_lines(text, name))
    with open(out, "w") as f:
        f.write(f"// generated by tools/micro/gen_mix_micro.py from {name}\n")
        counts = {}
        for l in body:
            counts[kind(l)] = counts.get(kind(l), 0) + 1
        f.write("// instructions per two blocks: " + ", ".join(f"{k} {v}" for k, v in sorted(counts.items())) + "\n")
        for sub, keep in SUBSETS.items():
            sel = [l for l in body if kind(l) in keep]
            f.write(f"#define MIX_{sub}_N {len(sel)}\n")
            f.write(f"#define MIX_{sub} \\\n")
            for l in sel:
                f.write(f'    "{l}\\n" \\\n')
            f.write('    ""\n')
        for nr in (2, 3):
            rn = rn_transform(body, nr)
            for sub, keep in ((f"R{nr}FULL", SUBSETS["FULL"]), (f"R{nr}VALU", SUBSETS["VALU"])):
                sel = [l for l in rn if kind(l) in keep]
                f.write(f"#define MIX_{sub}_N {len(sel)}\n")
                f.write(f"#define MIX_{sub} \\\n")
                for l in sel:
                    f.write(f'    "{l}\\n" \\\n')
                f.write('    ""\n')
        sp = steady_path(macro_lines(text, name))
        sp2 = sp + sp[:0]
        for sub, lines in (("SPFULL", sp), ("DSFULL", remap_waits(sp, dspub_transform(sp))),
                           ("DS1FULL", remap_waits(sp, dspub_transform(sp, 1)))):
            f.write(f"#define MIX_{sub}_N {len(lines)}\n")
            f.write(f"#define MIX_{sub} \\\n")
            for l in lines:
                f.write(f'    "{l}\\n" \\\n')
            f.write('    ""\n')
        for nr in (2, 3):
            lines = packed_body(nr)
            f.write(f"#define MIX_PK{nr}_N {len(lines)}\n")
            f.write(f"#define MIX_PK{nr} \\\n")
            for l in lines:
                f.write(f'    "{l}\\n" \\\n')
            f.write('    ""\n')
        f.write("#define MIX_R2_CLOBBERS " + ", ".join(f'"v{n}"' for n in range(168, 178)) + "\n")
        f.write("#define MIX_R3_CLOBBERS " + ", ".join(f'"v{n}"' for n in range(168, 188)) + "\n")
        valu = [l for l in body if kind(l) == "valu"]
        for sub, fn in SUBST.items():
            f.write(f"#define MIX_{sub}_N {len(valu)}\n")
            f.write(f"#define MIX_{sub} \\\n")
            for l in valu:
                f.write(f'    "{fn(l)}\\n" \\\n')
            f.write('    ""\n')


if __name__ == "__main__":
    main()

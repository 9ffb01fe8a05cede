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

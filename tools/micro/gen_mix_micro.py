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


def r2_transform(body):
    """Two rows per lane (round 5 projection, G space): after each step's cell A (row 2l)
    the lane computes cell B (row 2l+1) from A without a lane shift -- B's own E chain,
    its LUT (the other query code, the same subject byte), its diagonal from A's previous
    step, F and H from A's new cell -- and the lane shifts, the shift register and the
    publish carry B's cells (the band's bottom row).  A's rotation v128..v135 is mirrored
    by B's v168..v175; v176 / v177 are B's diagonal sum and weight bytes."""
    def bmap(r):
        n = int(r[1:])
        return f"v{n + 40}" if 128 <= n <= 135 else r
    out, prev_oga, perm_src, byte, cur_oga = [], "v134", None, 0, None
    for l in body:
        m = re.match(r"v_mov_b32_dpp (v\d+), (\S+) (wave_shr|wave_shl)(.*)", l)
        if m:
            dst, src = m.group(1), m.group(2)
            if m.group(3) == "wave_shl":
                dst = bmap(dst)
            src = bmap(src) if src.startswith("v") else src
            out.append(f"v_mov_b32_dpp {dst}, {src} {m.group(3)}{m.group(4)}")
            continue
        m = re.match(r"ds_write_b64 (v\d+), v\[(\d+):(\d+)\](.*)", l)
        if m:
            a0, a1 = int(m.group(2)), int(m.group(3))
            if 128 <= a0 <= 135:
                a0, a1 = a0 + 40, a1 + 40
            out.append(f"ds_write_b64 {m.group(1)}, v[{a0}:{a1}]{m.group(4)}")
            continue
        m = re.match(r"v_mov_b32_e32 (%\[(?:cur|fd)\]), (v\d+)$", l)
        if m:
            out.append(f"v_mov_b32_e32 {m.group(1)}, {bmap(m.group(2))}")
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
            ofa = m.group(1)
            out.append("v_max_i32_e32 %[eb], %[eb], %[hgb]")
            if perm_src:
                out.append(f"v_perm_b32 v177, %[lhb], %[llb], {perm_src}")
                perm_src = None
            out.append(f"v_add_u32_sdwa v176, {prev_oga}, sext(v177) dst_sel:DWORD dst_unused:UNUSED_PAD "
                       f"src0_sel:DWORD src1_sel:BYTE_{byte}")
            out.append(f"v_max3_i32 {bmap(cur_oga)}, v176, %[eb], {ofa}")
            out.append(f"v_add_u32_e32 %[hgb], %[go], {bmap(cur_oga)}")
            out.append(f"v_max_i32_e32 {bmap(ofa)}, {ofa}, %[hgb]")
            prev_oga, cur_oga = cur_oga, None
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
        r2 = r2_transform(body)
        for sub, keep in (("R2FULL", SUBSETS["FULL"]), ("R2VALU", SUBSETS["VALU"])):
            sel = [l for l in r2 if kind(l) in keep]
            f.write(f"#define MIX_{sub}_N {len(sel)}\n")
            f.write(f"#define MIX_{sub} \\\n")
            for l in sel:
                f.write(f'    "{l}\\n" \\\n')
            f.write('    ""\n')
        f.write("#define MIX_R2_CLOBBERS " + ", ".join(f'"v{n}"' for n in range(168, 178)) + "\n")
        valu = [l for l in body if kind(l) == "valu"]
        for sub, fn in SUBST.items():
            f.write(f"#define MIX_{sub}_N {len(valu)}\n")
            f.write(f"#define MIX_{sub} \\\n")
            for l in valu:
                f.write(f'    "{fn(l)}\\n" \\\n')
            f.write('    ""\n')


if __name__ == "__main__":
    main()

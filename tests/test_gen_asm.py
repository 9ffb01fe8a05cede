"""CPU checks of the generated steady-state loops (tools/gen_block_asm.py ->
anyseq_amd/csrc/anyseq_block_asm.inc): every affine / linear-on-affine macro, one to three
rows per lane, keeps the CDNA hazard rule the generator schedules for -- a DPP move never
reads a VGPR that a VALU instruction wrote fewer than two wait states (VALU or s_nop slots)
before it -- and every label of a macro is defined once.  Generated into a temporary file,
so the in-tree include is not touched."""
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def macros(tmp_path_factory):
    out = tmp_path_factory.mktemp("gen") / "asm.inc"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_block_asm.py"), str(out)], check=True,
                   capture_output=True)
    text = out.read_text()
    found = {}
    for m in re.finditer(r'#define (ANYSEQ_AF2\w*) \\\n((?:    ".*\\n" \\\n)*)', text):
        found[m.group(1)] = [re.match(r'\s*"(.*)\\n"', l).group(1) for l in m.group(2).split("\n") if '"' in l]
    return found


def test_variant_families_present(macros):
    for fam in ("AF2_G", "AF2_L", "AF2E_L", "AF2F_G", "AF2R_G", "AF2RE_L", "AF2R3F_G", "AF2R3_L", "AF2_N", "AF2E_M"):
        assert any(n.startswith("ANYSEQ_" + fam + "_") for n in macros), fam
    assert len(macros) >= 360


def test_dpp_reads_wait_two_states(macros):
    bad = []
    for name, lines in macros.items():
        last_write, ws = {}, 0
        for l in lines:
            parts = l.split()
            op = parts[0] if parts else ""
            if op.startswith("v_") or op == "s_nop":
                if op == "v_mov_b32_dpp":
                    src = parts[2]
                    if src in last_write and ws - last_write[src] < 2:
                        bad.append((name, l))
                if op == "s_nop":
                    ws += int(parts[1]) + 1
                    continue
                ws += 1
                last_write[parts[1].rstrip(",")] = ws
            elif l.endswith(":") or op.startswith(("s_cbranch", "s_branch")):
                last_write = {}   # (control flow: branch targets are loop heads behind the block's waits)
    assert not bad, bad[:5]


def test_labels_defined_once(macros):
    for name, lines in macros.items():
        labels = [l for l in lines if l.endswith(":")]
        assert len(labels) == len(set(labels)), name

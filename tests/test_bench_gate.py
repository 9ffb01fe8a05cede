"""CPU tests of bench.py's result gate (verdict round 5, item 1): every bench line --
above all the N > 1 lines, whose RCCL paths have never run on hardware -- is checked
against a committed fixture (configs[2]: the oracle's score and strings; configs[4]: the
single-GPU score of the synthetic genome pair) or the single-GPU result, and a mismatch
exits non-zero with no JSON value.  Driven through a stubbed result: --gate-only SCORE runs
the same gate with SCORE as the bench's result, without a GPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def run(*args):
    return subprocess.run([sys.executable, BENCH, *args], cwd=ROOT, capture_output=True, text=True, timeout=300)


@pytest.mark.parametrize("config,good", [(4, 7821754), (2, 26231)])
def test_gate_passes_the_fixture_score(config, good):
    r = run("--config", str(config), "--gate-only", str(good))
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["gate"] == "ok" and d["checked"] and d["score"] == good


@pytest.mark.parametrize("config,bad", [(4, 7821753), (2, 26232)])
def test_gate_refuses_a_wrong_score(config, bad):
    r = run("--config", str(config), "--gate-only", str(bad))
    assert r.returncode == 3, (r.returncode, r.stdout, r.stderr)
    assert "RESULT GATE FAILED" in r.stderr and '"value"' not in r.stdout


def test_construct_gate_checks_both_strings():
    """configs[2]'s fixture: the right score with strings of the wrong hash fails."""
    sys.path.insert(0, ROOT)
    import bench
    import anyseq_amd as A
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "config2_65536.json")))
    q, s = A.main_random_pair(65536, 65536)
    fx = bench.find_fixture("local", q, s, dict(bench.AFFINE))
    assert fx is not None and fx["sha_alq"] == g["sha_alq"] and fx["sha_als"] == g["sha_als"]
    with pytest.raises(SystemExit) as e:
        bench.check_construct("local", q, s, dict(bench.AFFINE), g["score"], b"A" * 10, b"C" * 10)
    assert e.value.code == bench.GATE_EXIT


def test_construct_gate_reference_fallback():
    """Inputs without a fixture: the single-GPU reference decides (stubbed here)."""
    sys.path.insert(0, ROOT)
    import bench
    q, s = b"ACGT" * 50, b"ACGA" * 60
    sc = dict(bench.AFFINE)
    ref = (17, b"x" * 440, b"y" * 440)
    info = bench.check_construct("local", q, s, sc, 17, ref[1], ref[2], reference=lambda: ref)
    assert info["checked"] and info["against"].startswith("single-GPU")
    with pytest.raises(SystemExit) as e:
        bench.check_construct("local", q, s, sc, 17, ref[1], b"z" * 440, reference=lambda: ref)
    assert e.value.code == bench.GATE_EXIT
    with pytest.raises(SystemExit):
        bench.check_score("semiglobal", q, s, sc, 5, reference=lambda: 6)
    assert bench.check_score("semiglobal", q, s, sc, 6, reference=lambda: 6)["checked"]

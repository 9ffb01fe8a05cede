"""The CPU oracle under AddressSanitizer + UBSan (verdict round 5, item 7).

oracle/anyseq_oracle.c is hand-indexed C with pthreads and an unset-split sentinel, and every
parity claim rests on it.  `make -C oracle asan` builds the same source with
-fsanitize=address,undefined and every finding fatal; a child process (libasan preloaded,
ORACLE_LIB pointing at the sanitizer build) runs its score, construct, affine and fulltb
paths on the golden shapes -- empty sequences, m <= 64 (the reference's degenerate split),
one-block and multi-block Hirschberg levels, main.cpp's 1024 x 1024 pair, several threads --
and must exit cleanly with results equal to the regular build's."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")
ASAN_LIB = os.path.join(ORACLE, "_asan", "liboracle_asan.so")

# (n, m): empty, tiny, m <= 64, m around the 128-column blocks, the stride classes of
# hb_sum (m > 1024), tall and wide
SHAPES = [(0, 0), (0, 7), (7, 0), (1, 1), (3, 64), (64, 64), (200, 63), (65, 129), (128, 128), (300, 257),
          (257, 1100), (1100, 300), (700, 2100)]

CHILD = r"""
import json, random, sys
sys.path.insert(0, sys.argv[1])
from oracle import oracle as O
shapes = json.loads(sys.argv[2])
rng = random.Random(77)
out = []
for threads in (1, 4):
    O.set_threads(threads)
    for n, m in shapes:
        q = bytes(rng.choice(b"ACGT") for _ in range(n))
        s = bytes(rng.choice(b"ACGT") for _ in range(m))
        r = {"n": n, "m": m, "t": threads}
        for kind in ("global", "semiglobal", "local"):
            r[kind + "_score"] = O.score(kind, q, s, with_pos=True)
            r[kind + "_construct"] = [x if isinstance(x, int) else x.hex() for x in O.construct(kind, q, s)]
            r[kind + "_aff_score"] = O.affine_score(kind, q, s, 2, -1, -2, -1, with_pos=True)
            r[kind + "_aff_construct"] = [x if isinstance(x, int) else x.hex()
                                          for x in O.affine_construct(kind, q, s, 2, -1, -2, -1)]
        if n > 0 and m > 0:
            r["fulltb"] = [x if isinstance(x, int) else x.hex() for x in O.construct_fulltb(q, s)]
        out.append(r)
import os
maps = open("/proc/self/maps").read()
assert os.path.basename(O._LIB) in maps, "the requested oracle build is not the one loaded"
print(json.dumps(out))
"""


def run_child(lib, env_extra):
    env = dict(os.environ, ORACLE_LIB=lib, **env_extra)
    return subprocess.run([sys.executable, "-c", CHILD, ROOT, json.dumps(SHAPES)], env=env,
                          capture_output=True, text=True, timeout=900)


def asan_runtime():
    try:
        p = subprocess.check_output(["gcc", "-print-file-name=libasan.so"], text=True).strip()
    except (OSError, subprocess.CalledProcessError):
        return None
    return p if os.path.isabs(p) and os.path.exists(p) else None


def test_oracle_clean_under_asan_ubsan():
    rt = asan_runtime()
    if rt is None:
        pytest.skip("gcc's libasan is not installed")
    subprocess.check_call(["make", "-s", "-C", ORACLE, "asan"])
    san = run_child(ASAN_LIB, {"LD_PRELOAD": rt, "ASAN_OPTIONS": "detect_leaks=0:abort_on_error=1",
                               "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"})
    assert san.returncode == 0, san.stderr[-4000:]
    assert "AddressSanitizer" not in san.stderr and "runtime error" not in san.stderr, san.stderr[-4000:]
    subprocess.check_call(["make", "-s", "-C", ORACLE])
    plain = run_child(os.path.join(ORACLE, "liboracle.so"), {})
    assert plain.returncode == 0, plain.stderr[-2000:]
    assert json.loads(san.stdout) == json.loads(plain.stdout)


def test_oracle_main_1024_under_asan():
    """main.cpp's `-r 1024 1024` pair (configs[0]) through the sanitizer build: the six
    reference results of the committed fixture."""
    rt = asan_runtime()
    if rt is None:
        pytest.skip("gcc's libasan is not installed")
    subprocess.check_call(["make", "-s", "-C", ORACLE, "asan"])
    code = r"""
import hashlib, json, sys
sys.path.insert(0, sys.argv[1])
from oracle import oracle as O
import anyseq_amd as A
q, s = A.main_random_pair(1024, 1024)
O.set_threads(4)
out = {k: O.score(k, q, s) for k in ("global", "semiglobal", "local")}
for k in ("global", "semiglobal", "local"):
    r, aq, as_ = O.construct(k, q, s)
    out["c_" + k] = [r, hashlib.sha256(aq).hexdigest(), hashlib.sha256(as_).hexdigest()]
print(json.dumps(out))
"""
    env = dict(os.environ, ORACLE_LIB=ASAN_LIB, LD_PRELOAD=rt, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([sys.executable, "-c", code, ROOT], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "runtime error" not in r.stderr, r.stderr[-4000:]
    got = json.loads(r.stdout)
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "main_1024.json")))
    import hashlib
    for k in ("global", "semiglobal", "local"):
        assert got[k] == g["score"][k]
        c = g["construct"][k]
        assert got["c_" + k] == [c["ret"], hashlib.sha256(c["alq"].encode("latin-1")).hexdigest(),
                                 hashlib.sha256(c["als"].encode("latin-1")).hexdigest()], k

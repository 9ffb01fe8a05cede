#!/usr/bin/env python3
"""Generates the full-size affine construct fixtures (run from the repo root; CPU only,
a few minutes single-threaded):

  config2_65536.json   BASELINE.json configs[2]: local (SW) affine (+2/-1, open -2,
                       extend -1) score + traceback of main.cpp's `-r 65536 65536` pair;
  config3_prefix.json  configs[3] workload at a prefix size the oracle finishes: the
                       first 262,144 bytes of both sequences of the synthetic 4.64 Mbp
                       related pair (anyseq_amd/genome.py), semiglobal affine;
  config2_nonpow2.json configs[2]'s local scheme on main.cpp's 65536 pair with the subject
                       cut to 60,001 bytes (469 blocks of 128 columns: not a power of two,
                       so every level's parts split at their middle block, round 4);
  config3_nonpow2.json the configs[3] semiglobal workload on prefixes of 150,001 x 140,001
                       bytes (1,094 blocks).

Each holds the optimal score, the SHA-256 of both sparse i+j+1 strings, the aligned
rectangle and the dense extended CIGAR.  The expected values come from the oracle
restatement (oracle_affine_construct): affine gaps have no reference semantics
(align.impala:153-166 is dead), so these pin the build-defined semantics at full size.
The inputs are not stored: main.cpp's generator (anyseq_main_random_pair, host code)
and genome.synthetic_related_pair rebuild them; their SHA-256 are stored to check that.
"""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
HERE = os.path.dirname(os.path.abspath(__file__))

import anyseq_amd as A  # noqa: E402  (host-side helpers only: the generator and the CIGAR adapter)
from anyseq_amd import genome  # noqa: E402
from oracle import oracle as O  # noqa: E402

SCHEME = (2, -1, -2, -1)
PREFIX = 262144


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def fixture(kind, q, s, source):
    t = time.time()
    score, aq, as_ = O.affine_construct(kind, q, s, *SCHEME)
    rect = O.affine_last_rect()
    return {"source": source, "kind": kind, "scoring": dict(zip(("match", "mismatch", "gap_open", "gap_extend"), SCHEME)),
            "lq": len(q), "ls": len(s), "sha_q": sha(q), "sha_s": sha(s), "score": score,
            "sha_alq": sha(aq), "sha_als": sha(as_), "rect": list(rect), "cigar": A.cigar(aq, as_),
            "oracle_seconds": round(time.time() - t, 1)}


def main():
    O.build()
    which = sys.argv[1:] or ["config2", "config3", "config2_nonpow2", "config3_nonpow2"]
    O.set_threads(os.cpu_count() or 1)
    if "config2" in which:
        q, s = A.main_random_pair(65536, 65536)
        d = fixture("local", q, s, "oracle_affine_construct on main.cpp `-r 65536 65536` inputs (configs[2])")
        json.dump(d, open(os.path.join(HERE, "config2_65536.json"), "w"), indent=1)
        print("config2", d["score"], d["oracle_seconds"], "s", flush=True)
    if "config3" in which:
        q, s = genome.synthetic_related_pair(4_641_652, 0.9)
        q, s = q[:PREFIX], s[:PREFIX]
        d = fixture("semiglobal", q, s, f"oracle_affine_construct on the first {PREFIX} bytes of the synthetic "
                                        "4,641,652-bp related pair (genome.synthetic_related_pair(4641652, 0.9))")
        json.dump(d, open(os.path.join(HERE, "config3_prefix.json"), "w"), indent=1)
        print("config3", d["score"], d["oracle_seconds"], "s", flush=True)
    if "config2_nonpow2" in which:
        q, s = A.main_random_pair(65536, 65536)
        s = s[:60001]
        d = fixture("local", q, s, "oracle_affine_construct on main.cpp `-r 65536 65536` inputs, subject cut to "
                                   "60001 bytes (non-power-of-two block count)")
        json.dump(d, open(os.path.join(HERE, "config2_nonpow2.json"), "w"), indent=1)
        print("config2_nonpow2", d["score"], d["oracle_seconds"], "s", flush=True)
    if "config3_nonpow2" in which:
        q, s = genome.synthetic_related_pair(4_641_652, 0.9)
        q, s = q[:150001], s[:140001]
        d = fixture("semiglobal", q, s, "oracle_affine_construct on the first 150001 / 140001 bytes of the "
                                        "synthetic 4,641,652-bp related pair (non-power-of-two block count)")
        json.dump(d, open(os.path.join(HERE, "config3_nonpow2.json"), "w"), indent=1)
        print("config3_nonpow2", d["score"], d["oracle_seconds"], "s", flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Generates the committed golden fixtures under tests/golden/ (run from the repo root).

Sources of truth, in order of independence from this build:
  kat.json          SURVEY.md Appendix C known answers, derived by hand from the
                    reference code (align.impala / traceback.impala) — NOT from the oracle;
  main_inputs.json  SURVEY.md Appendix B fingerprints of main.cpp's `-r` inputs
                    (FNV-1a 64 over the raw bytes; produced by linking the unmodified
                    reference main.cpp against a hashing stub);
  oracle_*.json     outputs of the oracle restatement (oracle/anyseq_oracle.c) on seeded
                    inputs — a regression pin for the oracle and the GPU parity target.
"""
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
HERE = os.path.dirname(os.path.abspath(__file__))

from oracle import oracle as O  # noqa: E402

KINDS = ("global", "semiglobal", "local")


def kat():
    # SURVEY.md Appendix C (hand-derived; +2/-1, linear -1)
    cases = [
        {"q": "A", "s": "A", "score": {"global": 2, "local": 2, "semiglobal": 2}},
        {"q": "A", "s": "C", "score": {"global": -1, "local": 0, "semiglobal": 0}},
        {"q": "AC", "s": "C", "score": {"global": 1}},
        {"q": "ACGT", "s": "GT", "score": {"global": 2, "semiglobal": 4}},
        {"q": "ACGT", "s": "ACGT", "score": {"global": 8, "semiglobal": 8, "local": 8}},
        {"q": "TTACGTT", "s": "GGACGGG", "score": {"local": 6}},
    ]
    constructs = [
        {"kind": "global", "q": "AC", "s": "C", "ret": -2, "alq": "_  ", "als": "C  "},
        {"kind": "local", "q": "A", "s": "A", "ret": -2147483647, "alq": "  ", "als": "  "},
        {"kind": "global", "q": "A" * 65, "s": "A" * 65, "ret": -65, "alq": " A" * 65, "als": " A" * 65},
        {"kind": "semiglobal", "q": "A" * 65, "s": "A" * 65, "ret": 0, "alq": " A" * 65, "als": " A" * 65},
        {"kind": "local", "q": "A" * 65, "s": "A" * 65, "ret": -2147483647, "alq": " A" * 65, "als": " A" * 65},
    ]
    return {"source": "SURVEY.md Appendix C (hand-derived from align.impala:46-90, traceback.impala:47-80)",
            "scores": cases, "constructs": constructs}


def main_inputs():
    return {"source": "SURVEY.md Appendix B (main.cpp -r generator, FNV-1a 64)",
            "cases": [
                {"args": [1024, 1024], "lq": 1024, "ls": 1024, "q32": "CGTACCAGCCGAGGTCCGAACTAAAGTTACCT",
                 "s32": "AAGTGGTAAGTCAACCGTTATGAATAGCAGAG", "fnv_q": "a73a37f7a8d64c9f", "fnv_s": "f9224f342874a59f"},
                {"args": [65536, 65536], "lq": 65536, "ls": 65536, "q32": "CGTACCAGCCGAGGTCCGAACTAAAGTTACCT",
                 "s32": "ATAGGAAGGGGCAGACAGCCAATCTGTACGCC", "fnv_q": "533518aa82d8b636", "fnv_s": "a2707193d7e314a6"},
                {"args": [256, 1024], "lq": 861, "ls": 914, "q32": "CGTACCAGCCGAGGTCCGAACTAAAGTTACCT",
                 "s32": "CCACAGCTTATCAATCGCGTCTTGACATGTAG", "fnv_q": "4de67cd69011a8a7", "fnv_s": "08f2452b0e6358ff"},
            ]}


def oracle_cases():
    rng = random.Random(20261015)
    out = []
    shapes = [(1, 1), (3, 5), (64, 64), (65, 65), (127, 129), (200, 300), (513, 257), (1000, 700), (700, 1000),
              (0, 10), (10, 0), (0, 0), (1500, 130), (130, 1500)]
    for n, m in shapes:
        q = "".join(rng.choice("ACGT") for _ in range(n))
        s = "".join(rng.choice("ACGT") for _ in range(m))
        ent = {"q": q, "s": s, "score": {}, "construct": {}}
        for k in KINDS:
            ent["score"][k] = O.score(k, q, s)
            r, aq, as_ = O.construct(k, q, s)
            ent["construct"][k] = {"ret": r, "alq": aq.decode(), "als": as_.decode()}
        out.append(ent)
    return {"source": "oracle/anyseq_oracle.c on seeded inputs (random.Random(20261015))", "cases": out}


def main_1024(A):
    q, s = A.main_random_pair(1024, 1024)
    ent = {"args": [1024, 1024], "score": {}, "construct": {}}
    for k in KINDS:
        ent["score"][k] = O.score(k, q, s)
        r, aq, as_ = O.construct(k, q, s)
        ent["construct"][k] = {"ret": r, "alq": aq.decode(), "als": as_.decode()}
    return ent


def main_65536(A):
    """configs[1] pair: the three scores, and the reference-semantics construct_*
    (export.impala:19-34,75-90,131-147: 9 Hirschberg levels with hb_sum's stride-class
    candidate order) as return value + SHA-256 of both sparse strings (~5 s each)."""
    import hashlib
    q, s = A.main_random_pair(65536, 65536)
    O.set_threads(8)
    ent = {"args": [65536, 65536], "score": {k: O.score(k, q, s) for k in KINDS}, "construct": {}}
    for k in KINDS:
        r, aq, as_ = O.construct(k, q, s)
        ent["construct"][k] = {"ret": r, "sha256_alq": hashlib.sha256(aq).hexdigest(),
                               "sha256_als": hashlib.sha256(as_).hexdigest(), "n_blank": aq.count(b" "),
                               "n_gap_q": aq.count(b"_"), "n_gap_s": as_.count(b"_")}
    O.set_threads(4)
    return ent


if __name__ == "__main__":
    import anyseq_amd as A
    O.build()
    json.dump(kat(), open(os.path.join(HERE, "kat.json"), "w"), indent=1)
    json.dump(main_inputs(), open(os.path.join(HERE, "main_inputs.json"), "w"), indent=1)
    json.dump(oracle_cases(), open(os.path.join(HERE, "oracle_cases.json"), "w"))
    json.dump({"source": "oracle on main.cpp `-r 1024 1024` inputs (configs[0])", **main_1024(A)},
              open(os.path.join(HERE, "main_1024.json"), "w"))
    json.dump({"source": "oracle on main.cpp `-r 65536 65536` inputs (configs[1]); scores, and the reference-"
                         "semantics construct_* (export.impala:19-34,75-90,131-147; hb_sum stride classes, "
                         "traceback_lintime.impala:44-135) as return value + SHA-256 of both sparse strings",
               **main_65536(A)},
              open(os.path.join(HERE, "main_65536.json"), "w"))
    print("golden fixtures written")

"""Writes tests/golden/config4_synthetic.json: the correctness anchor of the configs[3] /
configs[4] bench lines at N > 1 (verdict round 5, item 1).

The pair is anyseq_amd.genome.synthetic_related_pair(4_641_652, 0.9) (E. coli K-12 length,
90 % identity; the reference's FASTAs are absent).  The oracle cannot reach 4.64 Mbp^2, so the
score is the single-GPU result, agreed on by three independent GPU paths of round 5: the
score-only fill, the 2-shard column-blocked fill and the Hirschberg construct, whose strings
re-score to it (tests/test_gpu_golden_affine.py::test_config3_genome_length_construct,
BENCH_r05 scaling_anchor).  `construct_sha_*` (configs[3]'s strings, single GPU) are added by
`--construct` on a GPU box.

Usage:  python tests/golden/make_config4_fixture.py [--construct]
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
SCORE = 7821754   # semiglobal affine (+2/-1, open -2, extend -1), single GPU, round 5


def main():
    from anyseq_amd import genome
    q, s = genome.synthetic_related_pair(4_641_652, 0.9)
    path = os.path.join(HERE, "config4_synthetic.json")
    g = json.load(open(path)) if os.path.exists(path) else {}
    g.update({"source": "single-GPU semiglobal affine score of the synthetic related genome pair, agreed on by "
                        "the score fill, the 2-shard column-blocked fill and the construct (round 5)",
              "pair": "anyseq_amd.genome.synthetic_related_pair(4_641_652, 0.9)", "kind": "semiglobal",
              "scoring": {"match": 2, "mismatch": -1, "gap_open": -2, "gap_extend": -1},
              "lq": len(q), "ls": len(s), "sha_q": hashlib.sha256(q).hexdigest(),
              "sha_s": hashlib.sha256(s).hexdigest(), "score": SCORE})
    if "--construct" in sys.argv:
        import anyseq_amd as A
        v, aq, as_ = A.construct("semiglobal", q, s, gap_open=-2, gap_extend=-1)
        assert v == SCORE and genome.affine_rescore(aq, as_) == v, v
        g.update({"construct_score": v, "construct_sha_alq": hashlib.sha256(aq).hexdigest(),
                  "construct_sha_als": hashlib.sha256(as_).hexdigest(),
                  "construct_source": "single-GPU construct (configs[3] N=1), strings re-scored to the score"})
    with open(path, "w") as f:
        json.dump(g, f, indent=1)
        f.write("\n")
    print(path)


if __name__ == "__main__":
    main()

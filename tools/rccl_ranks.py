"""Worker: the RCCL sharded path, one process per GPU, checked against the single-GPU path.

Launch (repo root, a node with >= WORLD GPUs):
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29533 tools/rccl_ranks.py

Rank r runs on device r.  Each rank first computes the single-GPU scores and
constructs (anyseq_score / anyseq_construct), then the same through
anyseq_shard_score / anyseq_shard_construct, whose boundary columns and level
columns travel over RCCL; rank 0 prints one JSON line per case and
ALL_MATCH / MISMATCH; the exit status is 0 only if every case matches.

Construct cases (CONSTRUCT_CASES): subjects longer than the query and square or wide
pairs; level 1 (and, at world >= 4, level 2) is column-blocked over the ranks whenever
the query gives every rank a column (shard_plan.level1_blocked, the engine's own test:
blocked_rccl, the boundary columns over RCCL send/recv); every case asserts through
anyseq_last_shard_plan which plan ran.  RCCL_FIXTURE=1 adds the configs[2] fixture
(tests/golden/config2_65536.json, SW affine 65536^2: score and SHA-256 of both strings).

RCCL refuses two ranks on one device ("Duplicate GPU detected", ncclInvalidUsage,
measured on the 1-GPU box), so this needs a multi-GPU node;
tests/test_gpu_rccl_ranks.py runs it there and skips on fewer GPUs.
"""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCORE_CASES = [("global", 0), ("semiglobal", 0), ("local", 0), ("global", -2), ("semiglobal", -2), ("local", -2)]
# (kind, n, m): level 1 column-blocked iff shard_plan.level1_blocked(n, m, world)
CONSTRUCT_CASES = [("semiglobal", 8000, 16384), ("local", 8000, 16500), ("local", 16384, 16384),
                   ("semiglobal", 16384, 16384), ("global", 12000, 9000), ("local", 100, 120)]


def expected_blocked_levels(world: int, nb: int) -> int:
    """Leading column-blocked levels of a construct with nb 128-column blocks: P = 1, 2, 4 ..
    parts while 2P <= world and P < nb (shard_plan.blocked_level; rows to spare)."""
    k, P = 0, 1
    while 2 * P <= world and P < nb:
        k, P = k + 1, 2 * P
    return k


def main():
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    import anyseq_amd as A
    from anyseq_amd import sharded
    from anyseq_amd.shard_plan import level1_blocked

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local_rank = int(os.environ.get("LOCAL_RANK", rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    if torch.cuda.device_count() < world:
        raise SystemExit(f"rccl_ranks: {world} ranks need {world} GPUs (RCCL refuses two ranks on one device)")
    A.set_device(local_rank)
    n, m = int(os.environ.get("PROBE_N", "8192")), int(os.environ.get("PROBE_M", "16384"))
    L = max(n, m, max(c[1] for c in CONSTRUCT_CASES), max(c[2] for c in CONSTRUCT_CASES))
    Q, S = A.main_random_pair(L, L)
    q, s = Q[:n], S[:m]
    ref = {c: A.score(c[0], q, s, gap_open=c[1]) for c in SCORE_CASES}
    ref_c = {c: A.construct(c[0], Q[:c[1]], S[:c[2]], gap_open=-2) for c in CONSTRUCT_CASES}
    dist.barrier()
    sharded.init(dist, rank, world)
    sharded.load(q, s, rank, world)
    ok = True
    for c in SCORE_CASES:
        t = time.time()
        got = sharded.score(c[0], gap_open=c[1])
        dt = time.time() - t
        good = got == ref[c]
        ok &= good
        if rank == 0:
            print(json.dumps({"op": "score", "kind": c[0], "gap_open": c[1], "n": n, "m": m, "world": world,
                              "single": ref[c], "rccl": got, "match": good, "s": round(dt, 4)}), flush=True)
    for c in CONSTRUCT_CASES:
        k, cn, cm = c
        t = time.time()
        A.last_shard_plan()
        got = sharded.construct(k, Q[:cn], S[:cm], gap_open=-2)
        plan = A.last_shard_plan()
        dt = time.time() - t
        exp = ref_c[c]
        good = got[0] == exp[0] and got[1] == exp[1] and got[2] == exp[2]
        plan_ok = (plan >= 1) == level1_blocked(cn, cm, world)
        if level1_blocked(cn, cm, world) and min(cn, cm) >= 8 * world:
            # (levels 2 / 3 too at world >= 4 / 8, when their parts keep a column per rank)
            plan_ok &= plan >= min(expected_blocked_levels(world, (cm + 127) // 128), 2 if world >= 4 else 1)
        ok &= good and plan_ok
        if rank == 0:
            print(json.dumps({"op": "construct", "kind": k, "n": cn, "m": cm, "gap_open": -2, "world": world,
                              "single": exp[0], "rccl": got[0], "strings_equal": good, "blocked_levels": plan,
                              "plan_ok": plan_ok, "s": round(dt, 4)}), flush=True)
    if os.environ.get("RCCL_FIXTURE") == "1":
        with open(os.path.join(ROOT, "tests", "golden", "config2_65536.json")) as f:
            fx = json.load(f)
        Qf, Sf = A.main_random_pair(65536, 65536)
        sc = fx["scoring"]
        t = time.time()
        A.last_shard_plan()
        got = sharded.construct(fx["kind"], Qf, Sf, sc["match"], sc["mismatch"], sc["gap_open"], sc["gap_extend"])
        plan = A.last_shard_plan()
        dt = time.time() - t
        h = [hashlib.sha256(x).hexdigest() for x in got[1:]]
        # every level with 2P <= world is column-blocked at 65536^2 (512 blocks): 1 at two
        # ranks, 2 at four, 3 at eight (verdict round 5, item 1)
        want = expected_blocked_levels(world, (len(Sf) + 127) // 128)
        good = got[0] == fx["score"] and h[0] == fx["sha_alq"] and h[1] == fx["sha_als"] and plan == want
        ok &= good
        if rank == 0:
            print(json.dumps({"op": "fixture", "name": "config2_65536", "world": world, "score": got[0],
                              "match": good, "blocked_levels": plan, "want_blocked": want, "s": round(dt, 4)}),
                  flush=True)
    dist.barrier()
    sharded.finalize()
    dist.destroy_process_group()
    if rank == 0:
        print("ALL_MATCH" if ok else "MISMATCH", flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()

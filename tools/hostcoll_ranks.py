"""Worker: the one-rank-per-process sharded construct (rank >= 0 branch) with host reductions.

Launch (repo root; every rank may share device 0):
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 \
      --master-addr 127.0.0.1 --master-port 29541 tools/hostcoll_ranks.py

Each rank runs anyseq_shard_construct_hostcoll: the device plan deals the Hirschberg
halves and the final blocks round-robin and this process fills only its own (rank >= 0:
the other ranks' halves get no groups, the rowpool and level columns are zeroed per level,
the columns / bottom rows SUM-reduced and the best cells MAX-reduced, per-rank final blocks
merged by a byte-wise MAX) -- the code the RCCL path runs, with gloo all-reduces on host
copies instead of ncclAllReduce.  Every case must equal the single-GPU construct bit for
bit, with the device-planned levels (ANYSEQ_SHARD_DEVPLAN=1, the default) and the
host-built ones (0).  HOSTCOLL_FIXTURE=1 adds the configs[2] fixture
(tests/golden/config2_65536.json).  Rank 0 prints one JSON line per case, then ALL_MATCH or
MISMATCH; the exit status is 0 only if every case matches on every rank.
"""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [("local", 2000, 3000), ("semiglobal", 1500, 2600), ("global", 1200, 900), ("local", 100, 120),
         ("semiglobal", 3000, 700), ("local", 700, 5000), ("global", 64, 129), ("local", 4000, 4000)]


def main():
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    import anyseq_amd as A
    from anyseq_amd import sharded

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local_rank = int(os.environ.get("LOCAL_RANK", rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ndev = max(1, torch.cuda.device_count())
    A.set_device(local_rank % ndev)
    L = max(max(c[1], c[2]) for c in CASES)
    Q, S = A.main_random_pair(L, L)
    ok = True
    for devplan in ("1", "0"):
        os.environ["ANYSEQ_SHARD_DEVPLAN"] = devplan
        for kind, n, m in CASES:
            q, s = Q[:n], S[:m]
            exp = A.construct(kind, q, s, gap_open=-2)
            dist.barrier()
            t = time.time()
            got = sharded.construct_hostcoll(dist, rank, world, kind, q, s, gap_open=-2)
            dt = time.time() - t
            good = got == exp
            flags = torch.tensor([0 if good else 1], dtype=torch.int32)
            dist.all_reduce(flags, op=dist.ReduceOp.MAX)
            good = good and int(flags.item()) == 0
            ok &= good
            if rank == 0:
                print(json.dumps({"op": "construct", "kind": kind, "n": n, "m": m, "world": world, "devplan": devplan,
                                  "single": exp[0], "hostcoll": got[0], "match": good, "s": round(dt, 3)}),
                      flush=True)
    os.environ["ANYSEQ_SHARD_DEVPLAN"] = "1"
    if os.environ.get("HOSTCOLL_FIXTURE") == "1":
        with open(os.path.join(ROOT, "tests", "golden", "config2_65536.json")) as f:
            fx = json.load(f)
        Qf, Sf = A.main_random_pair(65536, 65536)
        sc = fx["scoring"]
        dist.barrier()
        t = time.time()
        got = sharded.construct_hostcoll(dist, rank, world, fx["kind"], Qf, Sf, sc["match"], sc["mismatch"],
                                         sc["gap_open"], sc["gap_extend"])
        dt = time.time() - t
        h = [hashlib.sha256(x).hexdigest() for x in got[1:]]
        good = got[0] == fx["score"] and h[0] == fx["sha_alq"] and h[1] == fx["sha_als"]
        flags = torch.tensor([0 if good else 1], dtype=torch.int32)
        dist.all_reduce(flags, op=dist.ReduceOp.MAX)
        good = good and int(flags.item()) == 0
        ok &= good
        if rank == 0:
            print(json.dumps({"op": "fixture", "name": "config2_65536", "world": world, "score": got[0],
                              "match": good, "s": round(dt, 3)}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0:
        print("ALL_MATCH" if ok else "MISMATCH", flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()

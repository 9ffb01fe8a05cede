"""Worker: the RCCL sharded path, one process per GPU, checked against the single-GPU path.

Launch (repo root, a node with >= WORLD GPUs):
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29533 tools/rccl_ranks.py

Rank r runs on device r.  Each rank first computes the single-GPU scores and
constructs (anyseq_score / anyseq_construct), then the same through
anyseq_shard_score / anyseq_shard_construct, whose boundary columns and level
columns travel over RCCL; rank 0 prints one JSON line per case and
ALL_MATCH / MISMATCH; the exit status is 0 only if every case matches.

RCCL refuses two ranks on one device ("Duplicate GPU detected", ncclInvalidUsage,
measured on the 1-GPU box), so this needs a multi-GPU node;
tests/test_gpu_rccl_ranks.py runs it there and skips on fewer GPUs.
"""
import json
import os
import sys
import time

os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch.distributed as dist  # noqa: E402

import anyseq_amd as A  # noqa: E402
from anyseq_amd import sharded  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local_rank = int(os.environ.get("LOCAL_RANK", rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    A.set_device(local_rank)
    n, m = int(os.environ.get("PROBE_N", "8192")), int(os.environ.get("PROBE_M", "16384"))
    q, s = A.main_random_pair(max(n, m), max(n, m))
    q, s = q[:n], s[:m]
    cases = [("global", 0), ("semiglobal", 0), ("local", 0), ("global", -2), ("semiglobal", -2), ("local", -2)]
    ref = {c: A.score(c[0], q, s, gap_open=c[1]) for c in cases}
    ref_c = {k: A.construct(k, q, s, gap_open=-2) for k in ("semiglobal", "local")}
    dist.barrier()
    sharded.init(dist, rank, world)
    sharded.load(q, s, rank, world)
    ok = True
    for c in cases:
        t = time.time()
        got = sharded.score(c[0], gap_open=c[1])
        dt = time.time() - t
        good = got == ref[c]
        ok &= good
        if rank == 0:
            print(json.dumps({"op": "score", "kind": c[0], "gap_open": c[1], "n": n, "m": m, "world": world,
                              "single": ref[c], "rccl": got, "match": good, "s": round(dt, 4)}), flush=True)
    for k in ("semiglobal", "local"):
        t = time.time()
        got = sharded.construct(k, q, s, gap_open=-2)
        dt = time.time() - t
        exp = ref_c[k]
        good = got[0] == exp[0] and got[1] == exp[1] and got[2] == exp[2]
        ok &= good
        if rank == 0:
            print(json.dumps({"op": "construct", "kind": k, "gap_open": -2, "world": world, "single": exp[0],
                              "rccl": got[0], "strings_equal": good, "s": round(dt, 4)}), flush=True)
    dist.barrier()
    sharded.finalize()
    dist.destroy_process_group()
    if rank == 0:
        print("ALL_MATCH" if ok else "MISMATCH", flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()

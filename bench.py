#!/usr/bin/env python3
"""bench.py — GCUPS of the AnySeq hot path on MI355X (driver contract).

Workload at N=1 (BASELINE.json configs[1]): global (NW) alignment score, linear
gap (+2/-1/-1, the reference ABI's scheme), 65536 x 65536, on the exact inputs
the reference driver generates for ``align -r 65536 65536`` (main.cpp:200-210,
reproduced by anyseq_main_random_pair; fingerprints in SURVEY.md App. B).
One step = one global_alignment_score-equivalent fill of the whole matrix with
both sequences already resident in HBM (anyseq_score_device), score copied back.

N>1 (one process per GPU, torch.distributed.run): weak scaling over ONE
column-blocked matrix of 65536 rows x 65536*N columns; rank g owns columns
[65536 g, 65536 (g+1)); the two fronts' boundary columns travel between
neighbouring ranks in 1024-row chunks with RCCL send/recv over xGMI while the
fills run (libanyseq.so, anyseq_shard.cpp).  torch.distributed
(gloo) is the control plane only: barrier, max-over-ranks time, RCCL ids.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: 8.0 TB/s spec
BYTES_PER_CELL = 4           # one int32 H store per cell


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--m", type=int, default=65536)
    ap.add_argument("--kind", default="global", choices=["global", "semiglobal", "local"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sharded", action="store_true",
                    help="run the RCCL column-block path even at N=1 (plumbing check; the N=1 line is single GPU)")
    ap.add_argument("--cpu-threads", type=int, default=4,
                    help="oracle threads (reference get_thread_count() = 4, backend_cpu.impala:13)")
    return ap.parse_args()


def load_traffic(kernel_tag: str):
    """HBM bytes per launch from the newest committed PMC summary (profiles/*pmc*.json)."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")))
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        ent = d.get("kernels", {}).get(kernel_tag)
        if ent and ent.get("hbm_bytes_per_launch"):
            return ent["hbm_bytes_per_launch"], os.path.basename(f)
    return None, None


def cpu_baseline(q: bytes, s: bytes, kind: str, threads: int, expect: int):
    from oracle import oracle as O   # bench.py's cpu_baseline leg is allowed to use the oracle
    O.build()
    O.set_threads(threads)
    t = time.perf_counter()
    v = O.score(kind, q, s)
    dt = time.perf_counter() - t
    if v != expect:
        raise SystemExit(f"cpu baseline disagrees with GPU: {v} != {expect}")
    return {"value": round(len(q) * len(s) / dt / 1e9, 4), "unit": "GCUPS", "cores": threads, "kind": "port",
            "sample": f"full {len(q)}x{len(s)} {kind} linear score (oracle restatement of iteration_cpu/"
                      f"scoring_cpu, 1024^2 tiles, {threads} threads), {dt:.2f} s"}


def main():
    args = parse()
    # the sharded path's fill + transport streams each need a hardware queue of their own
    # (anyseq_shard.cpp check_hw_queues); HIP reads this at its first call
    if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 16:
        os.environ["GPU_MAX_HW_QUEUES"] = "16"
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import anyseq_amd as A

    dist = None
    if world > 1 or args.sharded:
        # control plane only (barrier, timing max, RCCL id broadcast): gloo on the host.
        # The data path is libanyseq.so's own RCCL communicators (anyseq_shard.cpp).
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    A.set_device(local_rank if world > 1 else 0)
    torch.cuda.set_device(local_rank if world > 1 else 0)
    dev = torch.device("cuda", torch.cuda.current_device())

    kind = args.kind
    parallelism = "single GPU"
    if dist:
        from anyseq_amd import sharded
        step, n, m, parallelism = sharded.make_weak_step(dist, rank, world, kind, rows=args.n, cols_per_rank=args.m)
        q = s = None
    else:
        q, s = A.main_random_pair(args.n, args.m)
        n, m = len(q), len(s)
        stream = torch.cuda.current_stream()
        sh = stream.cuda_stream
        dq = torch.frombuffer(bytearray(q), dtype=torch.uint8).to(dev)
        ds = torch.frombuffer(bytearray(s), dtype=torch.uint8).to(dev)

        def step():
            return A.score_device(kind, dq.data_ptr(), n, ds.data_ptr(), m, stream=sh)

    for _ in range(args.warmup):
        score = step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    A.last_fill_timing()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        score = step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    fill_ms, launches = A.last_fill_timing()
    elapsed = t1 - t0
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    cells_per_step = n * m * world          # weak scaling: each rank owns n x m cells
    ms_per_step = elapsed * 1e3 / args.steps
    gcups = cells_per_step * args.steps / elapsed / 1e9
    kernel_ms = fill_ms / max(launches, 1)
    cells_per_launch = n * m
    achieved = cells_per_launch * BYTES_PER_CELL / (kernel_ms * 1e-3) / 1e9 if kernel_ms > 0 else None
    tag = f"fill_kernel<{kind}> {n}x{m}"
    traffic, traffic_src = load_traffic(tag)

    if rank == 0:
        out = {
            "metric": "GCUPS (DP cell updates/s) at 1/2/4/8 GPUs; % of HBM roofline",
            "value": round(gcups, 2),
            "unit": "GCUPS",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic: main.cpp `-r 65536 65536` generator (mt19937_64 default seed, uniform ACGT)",
            "config": {"workload": f"{kind} alignment score, linear gap (+2/-1/-1), {n}x{m} cells per GPU",
                       "query_len": n, "subject_len": m,
                       "parallelism": parallelism,
                       "score": int(score)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2) if achieved else None,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                         "traffic": traffic,
                         "kernel_ms": round(kernel_ms, 4),
                         "bytes_model": f"{BYTES_PER_CELL} B/cell x {cells_per_launch} cells per launch "
                                        "(SURVEY.md 8(d))",
                         "traffic_source": traffic_src},
        }
        if world == 1 and not dist and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(q, s, kind, args.cpu_threads, int(score))
        print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        sharded.finalize()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

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

--config 2 (BASELINE.json configs[2], the north-star target): local (SW) affine
alignment (+2/-1, open -2, extend -1) of the same 65536^2 pair, score + Hirschberg
traceback: one step = anyseq_construct_device into device strings.
--config 3 (configs[3]): semi-global affine linear-memory traceback of a 4.64 Mbp
synthetic related-genome pair (the E. coli / S. boydii FASTAs are absent from the
reference snapshot; anyseq_amd/genome.py), or of --fasta Q S (first records).

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
    ap.add_argument("--config", type=int, default=1, choices=[1, 2, 3, 4],
                    help="BASELINE.json configs index: 1 NW linear score, 2 SW affine score+traceback, "
                         "3 genome semi-global affine traceback, 4 genome semi-global affine score "
                         "column-blocked over the ranks (strong scaling)")
    ap.add_argument("--gap-open", type=int, default=0,
                    help="config 1 only: affine gap open (extend -1); 0 = the reference's linear scheme")
    ap.add_argument("--fasta", nargs=2, metavar=("QUERY", "SUBJECT"), help="config 3: real genome files")
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


def cpu_baseline(q: bytes, s: bytes, kind: str, threads: int, expect: int, gap_open: int = 0):
    from oracle import oracle as O   # bench.py's cpu_baseline leg is allowed to use the oracle
    O.build()
    O.set_threads(threads)
    t = time.perf_counter()
    if gap_open:
        v = O.affine_score(kind, q, s, 2, -1, gap_open, -1)   # single-threaded restatement
        threads = 1
    else:
        v = O.score(kind, q, s)
    dt = time.perf_counter() - t
    if v != expect:
        raise SystemExit(f"cpu baseline disagrees with GPU: {v} != {expect}")
    what = (f"affine (open {gap_open}) score (oracle_affine_score, 1 thread)" if gap_open else
            f"linear score (oracle restatement of iteration_cpu/scoring_cpu, 1024^2 tiles, {threads} threads)")
    return {"value": round(len(q) * len(s) / dt / 1e9, 4), "unit": "GCUPS", "cores": threads, "kind": "port",
            "sample": f"full {len(q)}x{len(s)} {kind} {what}, {dt:.2f} s"}


AFFINE = dict(match=2, mismatch=-1, gap_open=-2, gap_extend=-1)


def cpu_baseline_construct(q: bytes, s: bytes, kind: str, side: int):
    """Oracle affine construct (single-threaded restatement) on a side x side prefix sample."""
    from oracle import oracle as O   # bench.py's cpu_baseline leg is allowed to use the oracle
    O.build()
    qs, ss = q[:side], s[:side]
    t = time.perf_counter()
    O.affine_construct(kind, qs, ss, **AFFINE)
    dt = time.perf_counter() - t
    return {"value": round(len(qs) * len(ss) / dt / 1e9, 4), "unit": "GCUPS", "cores": 1, "kind": "port",
            "sample": f"{len(qs)}x{len(ss)} prefix of the same pair, {kind} affine score + linear-memory "
                      f"traceback (oracle_affine_construct, 1 thread), {dt:.2f} s"}


def construct_bench(args):
    """configs[2] / configs[3]: affine construct (score + Hirschberg traceback) on one GPU."""
    import torch
    import anyseq_amd as A
    from anyseq_amd import genome
    A.set_device(0)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    if args.config == 2:
        kind = "local"
        q, s = A.main_random_pair(args.n, args.m)
        data = "synthetic: main.cpp `-r 65536 65536` generator (mt19937_64 default seed, uniform ACGT)"
        workload = f"local (SW) affine alignment, score + Hirschberg traceback, {len(q)}x{len(s)}"
    else:
        kind = "semiglobal"
        if args.fasta:
            (_, q), (_, s) = genome.first_record(args.fasta[0]), genome.first_record(args.fasta[1])
            data = f"FASTA first records: {os.path.basename(args.fasta[0])}, {os.path.basename(args.fasta[1])}"
        else:
            q, s = genome.synthetic_related_pair(4_641_652, 0.9)
            data = ("synthetic related-genome pair (E. coli K-12 length, 90% identity; the reference's "
                    "ecoli/sboydii FASTAs are absent)")
        workload = f"semi-global affine alignment, linear-memory traceback, {len(q)}x{len(s)}"
    n, m = len(q), len(s)
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    dq = torch.frombuffer(bytearray(q), dtype=torch.uint8).to(dev)
    ds = torch.frombuffer(bytearray(s), dtype=torch.uint8).to(dev)
    alq = torch.empty(n + m, dtype=torch.uint8, device=dev)
    als = torch.empty(n + m, dtype=torch.uint8, device=dev)

    def step():
        return A.construct_device(kind, dq.data_ptr(), n, ds.data_ptr(), m, alq.data_ptr(), als.data_ptr(),
                                  stream=sh, **AFFINE)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    A.last_fill_stats()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        score = step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    fill_ms, launches, fill_cells = A.last_fill_stats()
    # the alignment re-scored on the host equals the fill's optimum (size-independent check)
    rs = genome.affine_rescore(alq.cpu().numpy().tobytes(), als.cpu().numpy().tobytes(), **AFFINE)
    if rs != score:
        raise SystemExit(f"construct strings score {rs} != optimum {score}")
    cells = n * m
    gcups = cells * args.steps / elapsed / 1e9
    achieved = fill_cells * BYTES_PER_CELL / (fill_ms * 1e-3) / 1e9 if fill_ms > 0 else None
    traffic, traffic_src = load_traffic(f"fill_affine_kernel<{kind}> construct {n}x{m}")
    out = {
        "metric": "GCUPS (DP cell updates/s) at 1/2/4/8 GPUs; % of HBM roofline",
        "value": round(gcups, 2), "unit": "GCUPS", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "int32", "data": data,
        "config": {"workload": workload, "baseline_config": args.config, "query_len": n, "subject_len": m,
                   "scoring": "match +2, mismatch -1, gap open -2, extend -1", "parallelism": "single GPU",
                   "score": int(score), "fill_cells_per_step": fill_cells // max(args.steps, 1),
                   "fill_launches_per_step": launches // max(args.steps, 1)},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2) if achieved else None, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                     "traffic": traffic, "kernel_ms": round(fill_ms / max(launches, 1), 4),
                     "bytes_model": f"{BYTES_PER_CELL} B/cell x cells computed by the fill launches "
                                    "(Hirschberg halves included) / their summed duration (SURVEY.md 8(d))",
                     "traffic_source": traffic_src},
    }
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_construct(q, s, kind, 16384)
    print(json.dumps(out), flush=True)


def main():
    args = parse()
    if args.config in (2, 3):
        if int(os.environ.get("WORLD_SIZE", "1")) > 1:
            raise SystemExit("--config 2/3 run on one GPU (the column-block sharded path is config 1 / 4)")
        return construct_bench(args)
    genome = args.config == 4
    if genome:   # configs[4]: semi-global affine, one genome-length matrix split over the ranks
        args.kind, args.sharded = "semiglobal", True
        args.gap_open = args.gap_open or -2
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
    if dist and genome:
        from anyseq_amd import sharded, genome as G
        if args.fasta:
            (_, q), (_, s) = G.first_record(args.fasta[0]), G.first_record(args.fasta[1])
        else:
            q, s = G.synthetic_related_pair(4_641_652, 0.9)
        step, n, m, parallelism = sharded.make_strong_step(dist, rank, world, q, s, kind, gap_open=args.gap_open)
    elif dist:
        from anyseq_amd import sharded
        step, n, m, parallelism = sharded.make_weak_step(dist, rank, world, kind, rows=args.n, cols_per_rank=args.m,
                                                         gap_open=args.gap_open)
        q = s = None
    else:
        q, s = A.main_random_pair(args.n, args.m)
        n, m = len(q), len(s)
        stream = torch.cuda.current_stream()
        sh = stream.cuda_stream
        dq = torch.frombuffer(bytearray(q), dtype=torch.uint8).to(dev)
        ds = torch.frombuffer(bytearray(s), dtype=torch.uint8).to(dev)

        def step():
            return A.score_device(kind, dq.data_ptr(), n, ds.data_ptr(), m, stream=sh, gap_open=args.gap_open,
                                  gap_extend=-1)

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

    if genome:   # strong scaling: one n x m matrix, rank 0's launch covers its column block
        from anyseq_amd import shard_plan
        cells_per_step = n * m
        cells_per_launch = n * shard_plan.block(0, world, m)[1]
    else:        # weak scaling: each rank owns n x m cells
        cells_per_step = n * m * world
        cells_per_launch = n * m
    ms_per_step = elapsed * 1e3 / args.steps
    gcups = cells_per_step * args.steps / elapsed / 1e9
    kernel_ms = fill_ms / max(launches, 1)
    achieved = cells_per_launch * BYTES_PER_CELL / (kernel_ms * 1e-3) / 1e9 if kernel_ms > 0 else None
    tag = f"fill_kernel<{kind}> {n}x{m}" if not args.gap_open else f"fill_affine_kernel<{kind}> {n}x{m}"
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
            "scaling": "strong" if genome else "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": ("synthetic related-genome pair (E. coli K-12 length, 90% identity; the reference's "
                     "ecoli/sboydii FASTAs are absent)" if genome and not args.fasta else
                     "FASTA first records" if genome else
                     "synthetic: main.cpp `-r 65536 65536` generator (mt19937_64 default seed, uniform ACGT)"),
            "config": {"workload": f"{kind} alignment score, "
                                   + (f"affine gap (+2/-1, open {args.gap_open}, extend -1)" if args.gap_open
                                      else "linear gap (+2/-1/-1)")
                                   + (f", one {n}x{m} matrix column-blocked over {world} GPU(s)" if genome
                                      else f", {n}x{m} cells per GPU"),
                       "baseline_config": args.config,
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
            out["cpu_baseline"] = cpu_baseline(q, s, kind, args.cpu_threads, int(score), args.gap_open)
        elif world == 1 and genome and not args.no_cpu_baseline:
            qs, ss = q[:16384], s[:16384]
            v = A.score(kind, qs, ss, gap_open=args.gap_open, gap_extend=-1)
            out["cpu_baseline"] = cpu_baseline(qs, ss, kind, 1, v, args.gap_open)
            out["cpu_baseline"]["sample"] = "16384x16384 prefix of the pair: " + out["cpu_baseline"]["sample"]
        print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        sharded.finalize()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

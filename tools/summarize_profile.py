#!/usr/bin/env python3
"""Summarise a tools/profile.sh run into profiles/<tag>_*.{csv,json} (committed evidence).

HBM traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE
(KiB) from separate --pmc passes; gfx950 tallies wide streaming reads at half
their bytes, so the read side is reported raw and x2-corrected; the corrected
sum is the `traffic` figure (an upper estimate for our 4- and 8-byte sc1 loads).
SQ counters (one --pmc pass, 8 SQ + GRBM_GUI_ACTIVE) give the VALU issue rate and
the effective clock (GRBM_GUI_ACTIVE / 8 XCDs / kernel time).
usage: summarize_profile.py <tag>   (reads gpurun_out/prof_<tag>/)
"""
import csv
import hashlib
import json
import os
import shutil
import sys
from collections import defaultdict

FILL_AFF = "void anyseq::fill_affine_kernel<"
FILL_LIN = "void anyseq::fill_kernel<"
KIND = {"0": "global", "1": "semiglobal", "2": "local"}


def last_json(path):
    return json.loads(open(path).read().strip().splitlines()[-1])


def kernel_tag(name: str, bench: dict) -> str:
    cfg = bench.get("config", {})
    dims = f"{cfg.get('query_len')}x{cfg.get('subject_len')}"
    wl = cfg.get("workload", "")
    kind = wl.split()[0] if wl else "?"
    if name.startswith(FILL_AFF):
        return f"fill_affine_kernel<{kind}>" + (" construct " if "traceback" in wl else " ") + dims
    if name.startswith(FILL_LIN):
        k = name.split("<", 1)[1].split(",")[0].strip()
        return f"fill_kernel<{KIND.get(k, k)}> {dims}"
    return name.split("(")[0]


def pmc(path, counters):
    vals = defaultdict(lambda: defaultdict(list))
    if not os.path.exists(path):
        return vals
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] in counters:
                vals[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return vals


def mean(x):
    return sum(x) / max(len(x), 1)


def summarize(src, suffix, bench):
    stats = {}
    p = f"{src}/trace{suffix}/run_kernel_stats.csv"
    with open(p) as f:
        for row in csv.DictReader(f):
            stats[row["Name"]] = {"calls": int(row["Calls"]), "avg_ns": float(row["AverageNs"]),
                                  "pct": float(row["Percentage"])}
    fetch = pmc(f"{src}/pmc_fetch{suffix}/run_counter_collection.csv", {"FETCH_SIZE"})
    write = pmc(f"{src}/pmc_write{suffix}/run_counter_collection.csv", {"WRITE_SIZE"})
    sq = pmc(f"{src}/pmc_sq{suffix}/run_counter_collection.csv",
             {"SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_WAIT_ANY",
              "SQ_WAIT_INST_ANY", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "GRBM_GUI_ACTIVE"})
    kernels = {}
    for name in set(stats) | set(fetch) | set(write):
        if not (name.startswith(FILL_AFF) or name.startswith(FILL_LIN)) and name not in stats:
            continue
        f_kib = mean(fetch.get(name, {}).get("FETCH_SIZE", []))
        w_kib = mean(write.get(name, {}).get("WRITE_SIZE", []))
        ent = {"name": name, "fetch_kib_raw": f_kib, "write_kib": w_kib,
               "hbm_bytes_per_launch": int((2 * f_kib + w_kib) * 1024),
               "hbm_bytes_per_launch_uncorrected": int((f_kib + w_kib) * 1024)}
        ent.update(stats.get(name, {}))
        c = {k: mean(v) for k, v in sq.get(name, {}).items()}
        if c and ent.get("avg_ns"):
            ent["sq"] = c
            ent["clock_ghz"] = c.get("GRBM_GUI_ACTIVE", 0) / 8 / ent["avg_ns"]
        kernels[kernel_tag(name, bench)] = ent
    return kernels


def main():
    tag = sys.argv[1]
    src = f"gpurun_out/prof_{tag}"
    dst = "profiles"
    os.makedirs(dst, exist_ok=True)
    lib = os.path.join("anyseq_amd", "libanyseq.so")
    out = {"tag": tag, "lib_sha16": hashlib.sha256(open(lib, "rb").read()).hexdigest()[:16],
           "method": "rocprofv3 --kernel-trace --stats; separate --pmc passes FETCH_SIZE / WRITE_SIZE / 8 SQ "
                     "counters + GRBM_GUI_ACTIVE; traffic = (2*FETCH_SIZE + WRITE_SIZE) KiB per launch (gfx950 "
                     "read correction); clock = GRBM_GUI_ACTIVE / 8 XCDs / average kernel time",
           "benches": {}, "kernels": {}}
    for name, suffix in (("bench", ""), ("bench_c1", "_c1"), ("bench_aff_local", "_aff_local"), ("bench_c4", "_c4")):
        p = f"{src}/{name}.json"
        if not os.path.exists(p):
            continue
        bench = last_json(p)
        out["benches"][name] = bench
        if os.path.exists(f"{src}/trace{suffix}/run_kernel_stats.csv"):
            shutil.copy(f"{src}/trace{suffix}/run_kernel_stats.csv", f"{dst}/{tag}{suffix or '_c2'}_kernel_stats.csv")
            out["kernels"].update(summarize(src, suffix, bench))
    json.dump(out, open(f"{dst}/{tag}_pmc.json", "w"), indent=1)
    for k, v in out["kernels"].items():
        if "fill" in k:
            print(k, round(v.get("avg_ns", 0) / 1e6, 4), "ms", v["hbm_bytes_per_launch"], "B",
                  round(v.get("clock_ghz", 0), 3), "GHz")


if __name__ == "__main__":
    main()

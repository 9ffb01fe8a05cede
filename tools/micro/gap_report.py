#!/usr/bin/env python3
"""Gaps before / after each big_kernel launch of tools/micro/gap_micro.hip in a rocprofv3
kernel trace, by variant (template arguments).  Diagnostic tool, not part of the product.
usage: gap_report.py <run_kernel_trace.csv>"""
import csv
import statistics
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    before, after, dur = defaultdict(list), defaultdict(list), defaultdict(list)
    for i, r in enumerate(rows):
        k = r["Kernel_Name"]
        if "big_kernel" not in k or i == 0 or i + 1 >= len(rows):
            continue
        tag = k[k.index("<"):k.index(">") + 1] + f" grid {r['Grid_Size_X']} wg {r['Workgroup_Size_X']} #{(i // 60)}"
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        before[tag].append((s - int(rows[i - 1]["End_Timestamp"])) / 1000)
        after[tag].append((int(rows[i + 1]["Start_Timestamp"]) - e) / 1000)
        dur[tag].append((e - s) / 1000)
    for tag in before:
        print(f"{tag:45s} gap before {statistics.median(before[tag]):6.2f} us, after {statistics.median(after[tag]):6.2f} us,"
              f" duration {statistics.median(dur[tag]):8.2f} us")
    small = [(int(rows[i + 1]["Start_Timestamp"]) - int(r["End_Timestamp"])) / 1000
             for i, r in enumerate(rows[:-1]) if "small_kernel" in r["Kernel_Name"] and "small_kernel" in rows[i + 1]["Kernel_Name"]]
    if small:
        print(f"small -> small gap {statistics.median(small):.2f} us")


if __name__ == "__main__":
    main()

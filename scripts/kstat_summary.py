#!/usr/bin/env python3
"""Summarize a rocprofv3 --stats kernel_stats.csv: per kernel (short name) calls, mean us,
share.  usage: kstat_summary.py FILE [top]"""
import csv
import re
import sys


def short(name: str) -> str:
    n = re.sub(r"^void ", "", name)
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"\((?!\().*$", "", n) if "(" in n else n
    return n[:70]


rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    print(f"{short(r['Name']):70s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:8.2f} us {float(r['Percentage']):6.2f}%")

#!/usr/bin/env python3
"""Per-kernel average FETCH_SIZE / WRITE_SIZE per dispatch from two rocprofv3 --pmc
passes (counter_collection.csv), with the gfx950 correction of
/opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE reports half the bytes of a
wide streaming read -> doubled.  Prints JSON {kernel: {...}}."""
import csv
import os
import re
import glob
import json
import sys
from collections import defaultdict


def load(d, counter):
    files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    acc = defaultdict(list)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                name = row.get("Kernel_Name", "").replace("(anonymous namespace)::", "")
                m = re.search(r"(k_[a-z_0-9]+)", name)
                short = m.group(1) if m else name.split("(")[0].strip()
                acc[short].append(float(row["Counter_Value"]))
    return acc


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        fa = sum(f) / len(f) if f else None
        wa = sum(w) / len(w) if w else None
        out[k] = {
            "dispatches": max(len(f), len(w)),
            "fetch_size_raw_avg": fa,
            "write_size_raw_avg": wa,
            # rocprofv3 FETCH_SIZE / WRITE_SIZE are in KiB; FETCH doubled on gfx950
            "hbm_bytes_per_launch": (2 * fa * 1024 if fa is not None else 0) + (wa * 1024 if wa is not None else 0),
        }
    # per training step: every kernel's bytes x its launches, over the step count (one
    # tail per step -- the bench's tail probe must be off; copies included)
    steps = 0
    for k in ("k_step_tail", "k_dp_tail", "k_shard_update", "k_step_begin", "k_counters"):
        if k in out:
            steps = out[k]["dispatches"]
            break
    if steps:
        # HIP kernels of the library (k_*, incl. the rocprim sort's) + the blob copy;
        # torch fill kernels belong to setup, not to the step
        tot = sum(v["hbm_bytes_per_launch"] * v["dispatches"] for k, v in out.items()
                  if k.startswith("k_") or k.startswith("__amd_rocclr_copyBuffer"))
        out["_per_step"] = {"steps": steps, "hbm_bytes_per_step": tot / steps}
    # the kernels these counters belong to: bench.py ignores a profile whose sources differ
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "gat-recommendation_amd"))
    from etpgt.backend._lib import source_hash

    out["_source_hash"] = source_hash()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

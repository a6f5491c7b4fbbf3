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


def _short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    m = re.search(r"(k_[a-z_0-9]+)", name)
    return m.group(1) if m else name.split("(")[0].strip()


def load(d, counter):
    """{kernel: [value per dispatch]} and the run's dispatches in order [(kernel, value)]."""
    files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    acc = defaultdict(list)
    seq = []
    for f in files:
        with open(f) as fh:
            for i, row in enumerate(csv.DictReader(fh)):
                if row.get("Counter_Name") != counter:
                    continue
                short = _short(row.get("Kernel_Name", ""))
                v = float(row["Counter_Value"])
                acc[short].append(v)
                key = row.get("Dispatch_Id") or row.get("Correlation_Id") or i
                seq.append((int(key), short, v))
    seq.sort(key=lambda t: t[0])
    return acc, [(k, v) for _, k, v in seq]


STEP_END = ("k_step_tail", "k_step_tail_wgrad", "k_dp_tail", "k_shard_update")


def per_step(seq):
    """Bytes of one training step, over the steady-state steps only.

    The run is cut into intervals that end at a step's last kernel (the optimizer tail).
    The intervals whose kernel sequence is the most common one are the timed / warm-up
    steps of the bench; the rest (autograd-path steps, the first eager steps, one-time
    work such as k_lazy_flush or setup fills) are reported apart, not folded in."""
    steps, cur = [], []
    for k, v in seq:
        cur.append((k, v))
        if k in STEP_END:
            steps.append(cur)
            cur = []
    tail = cur  # dispatches after the last step (one-time flushes, checks)
    if not steps:
        return None
    sig = defaultdict(list)
    for st in steps:
        sig[tuple(k for k, _ in st if k.startswith("k_") or k.startswith("__amd_rocclr_copyBuffer"))].append(st)
    modal = max(sig.values(), key=len)
    byte_steps = [sum(v for k, v in st if k.startswith("k_") or k.startswith("__amd_rocclr_copyBuffer"))
                  for st in modal]
    other = defaultdict(float)
    for st in [s for v in sig.values() if v is not modal for s in v] + [tail]:
        for k, v in st:
            other[k] += v
    return {"steps": len(modal), "value_per_step": sum(byte_steps) / len(modal),
            "other_intervals": sum(len(v) for v in sig.values()) - len(modal), "outside_steps": dict(other)}


def main():
    fetch, fseq = load(sys.argv[1], "FETCH_SIZE")
    write, wseq = load(sys.argv[2], "WRITE_SIZE")
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
    # per training step: the steady-state steps of each pass (per_step), HIP kernels of the
    # library (k_*, incl. the sort's) + the blob copy; one-time work reported separately
    pf, pw = per_step(fseq), per_step(wseq)
    if pf and pw:
        once = {k: 2 * pf["outside_steps"].get(k, 0.0) * 1024 + pw["outside_steps"].get(k, 0.0) * 1024
                for k in set(pf["outside_steps"]) | set(pw["outside_steps"])}
        out["_per_step"] = {"steps": min(pf["steps"], pw["steps"]),
                            "hbm_bytes_per_step": 2 * pf["value_per_step"] * 1024 + pw["value_per_step"] * 1024,
                            "method": "steady-state steps only: intervals ending at the optimizer tail whose kernel "
                                      "sequence is the run's most common one",
                            "other_step_intervals": pf["other_intervals"],
                            "outside_steady_steps_bytes": {k: v for k, v in sorted(once.items()) if v > 0}}
    # the kernels these counters belong to: bench.py ignores a profile whose sources differ
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "gat-recommendation_amd"))
    from etpgt.backend._lib import source_hash

    out["_source_hash"] = source_hash()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Overflow rate of the row-sharded table's fitted exchange blocks (CPU, no GPU).

The bench sizes the all-to-all blocks to the most distinct rows any rank asks one owner
for over its pre-staged batches (FusedTrainStep.fit_shard_blocks; etpgt.train.sharded.
block_rows).  A later batch that needs more rows overflows: the step is applied as a
zero-gradient step and the host raises.  This script draws the same synthetic C4 data the
bench uses (seed 42), computes per rank-batch the (class 0, class 1) rows per owner, fits
the blocks on the first `--fit` batches per rank exactly as the bench does, and reports how
often the following batches (several epochs) exceed the fitted blocks, with and without a
headroom factor.  usage: block_overflow.py [--world 8] [--batch 1024] [--fit 64]
[--eval 2000] [--out FILE]
"""
import argparse
import json
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gat-recommendation_amd"))

from etpgt.data.synthetic import make_batches, make_sessions_and_graph  # noqa: E402
from etpgt.train.sharded import block_rows, shard_capacity  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--batch", type=int, default=1024, help="sessions per rank")
    ap.add_argument("--n-neg", type=int, default=100)
    ap.add_argument("--fit", type=int, default=64, help="staged batches per rank the bench fits on")
    ap.add_argument("--eval", type=int, default=2000, help="rank-batches drawn after the fitted ones")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    data = make_sessions_and_graph(seed=42)
    T, P, B = data.table_rows, a.world, a.batch
    # the bench's rank r stages batches from session position r * B * fit (build_workload)
    fit = []
    for r in range(P):
        for b in make_batches(data, B, a.fit, a.n_neg, seed=42, start=r * B * a.fit):
            fit.append(block_rows([b], P, True))
    fit = np.array(fit)
    cap0, cap1 = int(fit[:, 0].max()), int(fit[:, 1].max())
    start = P * B * a.fit  # batches no rank staged (the epoch continues past them)
    ev = []
    chunk = 64
    for k in range(0, a.eval, chunk):
        for b in make_batches(data, B, min(chunk, a.eval - k), a.n_neg, seed=43 + k, start=start + k * B):
            ev.append(block_rows([b], P, True))
    ev = np.array(ev)
    m_cap_nodes = int(B * 50)  # not binding: the static bound is the rows per owner
    static0 = shard_capacity(m_cap_nodes, T, P) - 1
    static1 = shard_capacity(B * (50 + 1 + a.n_neg), T, P) - 1

    def rate(c0, c1):
        over = (ev[:, 0] > c0) | (ev[:, 1] > c1)
        per_rank_batch = float(over.mean())
        # a global step overflows if ANY of its P rank-batches does
        per_step = 1.0 - (1.0 - per_rank_batch) ** P
        return per_rank_batch, per_step

    out = {"world": P, "per_rank_batch": B, "n_neg": a.n_neg, "fit_batches": int(len(fit)),
           "eval_rank_batches": int(len(ev)), "sessions_per_epoch": int(data.session_ptr.shape[0] - 1),
           "fitted_blocks": [cap0, cap1], "static_blocks": [static0, static1],
           "rows_mean": [float(ev[:, 0].mean()), float(ev[:, 1].mean())],
           "rows_std": [float(ev[:, 0].std()), float(ev[:, 1].std())],
           "rows_max_eval": [int(ev[:, 0].max()), int(ev[:, 1].max())]}
    rows = []
    for h in (1.0, 1.05, 1.1, 1.15, 1.2, 1.3):
        c0, c1 = min(static0, math.ceil(cap0 * h)), min(static1, math.ceil(cap1 * h))
        pr, ps = rate(c0, c1)
        rows.append({"headroom": h, "blocks": [c0, c1], "overflow_per_rank_batch": pr, "overflow_per_step": ps})
    out["by_headroom"] = rows
    s = json.dumps(out, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()

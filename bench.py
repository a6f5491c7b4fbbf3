#!/usr/bin/env python3
"""Benchmark: training sessions/sec of the fused GraphTransformer step on MI355X.

One "step" = one training step of trainer.py:80-133 (forward over the session
subgraphs, BPR/listwise sampled loss, backward, AdamW over every parameter incl.
the full item table) on one pre-staged synthetic batch already resident in HBM.
On one GPU each step launches straight on its pre-staged batch image (one captured
hipGraph per image, no copy); with N > 1 ranks or the row-sharded table the image is
copied D2D into the step's input buffer inside the timed step (the analogue of the
reference's ``batch.to(device)``).

Workloads (BASELINE.json configs):
  c2   (default) configs[1]: RetailRocket shape -- 82,173 items (T = 82,174 rows),
       737,716 co-occurrence edges, d=64, 2 layers, 1 head, BPR with 5 negatives,
       dropout 0.1, AdamW(1e-3, 1e-5), B = 32 sessions per GPU (params.yaml:6).  N > 1:
       data parallel, B per GPU fixed ("weak"), gradients averaged by one RCCL
       all-gather per step (etpgt.train.distributed).
  c3   configs[2]: d=128, 4 heads, LapPE k=16, listwise with 100 negatives.
  c4   configs[3]: the C3 model on the RetailRocket table, row-sharded across the ranks
       (etpgt.train.sharded: rows / row gradients by RCCL all-to-all), SyncBN, global
       batch 8192 fixed ("strong": per-rank batch 8192 / N).
  c5   configs[4] at N = 1: Yoochoose-scale 1M-node / 9M-edge graph, the C3 model,
       B = 8192, lazy table.
  c5s  configs[4] as the strong-scaling curve: the C5 table row-sharded, SyncBN, global
       batch 8192 fixed.

Multi-GPU: one process per GPU.  Under a launcher (torchrun / torch.distributed.run:
RANK / WORLD_SIZE in the environment) every rank runs this file; ``--gpus N`` WITHOUT a
launcher starts one itself (``python -m torch.distributed.run --nproc-per-node N`` as a
child process, before anything touches the GPU) and passes its output through.
GTR_SHARE_DEVICE=1 puts every rank on cuda:0 over gloo (a rehearsal on a one-GPU box).

Prints ONE JSON line (rank 0).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gat-recommendation_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "training sessions/sec + Recall@10 parity, 82k-node graph, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)

CONFIGS = {
    "c2": dict(D=64, H=1, K=0, loss="bpr", n_neg=5,
               name="C2 RetailRocket 82k-node/738k-edge, d=64, 2 layers, 1 head, BPR (5 neg)"),
    "c3": dict(D=128, H=4, K=16, loss="listwise", n_neg=100,
               name="C3 RetailRocket 82k-node/738k-edge, d=128, 2 layers, 4 heads, LapPE k=16, listwise (100 neg)"),
    # configs[3]: the C3 model node-sharded across the GPUs of one node -- the item table
    # row-sharded (rows fetched / gradients returned by RCCL all-to-all: the layer-0 halo),
    # SyncBN, the global batch fixed (strong scaling)
    "c4": dict(D=128, H=4, K=16, loss="listwise", n_neg=100, global_batch=8192, shard=True,
               name="C4 RetailRocket 82k-node/738k-edge node-sharded, d=128, 2 layers, 4 heads, LapPE k=16, "
                    "listwise (100 neg), row-sharded table + RCCL all-to-all, SyncBN"),
    # configs[4] on one GPU (the strong-scaling curve's N=1 point): C3 model on the
    # Yoochoose-scale graph, global batch 8192
    "c5": dict(D=128, H=4, K=16, loss="listwise", n_neg=100, scale="yoochoose", batch=8192, lazy=True,
               name="C5 Yoochoose-scale synthetic 1M-node/9M-edge, d=128, 2 layers, 4 heads, LapPE k=16, "
                    "listwise (100 neg)"),
    # configs[4] as the 1/2/4/8 strong-scaling curve: the 1M-row table row-sharded, SyncBN,
    # global batch 8192 fixed
    "c5s": dict(D=128, H=4, K=16, loss="listwise", n_neg=100, scale="yoochoose", global_batch=8192, shard=True,
                name="C5 Yoochoose-scale synthetic 1M-node/9M-edge strong scaling, d=128, 2 layers, 4 heads, "
                     "LapPE k=16, listwise (100 neg), row-sharded table + RCCL all-to-all, SyncBN"),
}


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def _claim_stdout():
    """The bench line must be the only thing on stdout, but libraries write there at the
    file-descriptor level (RCCL prints its version banner on every rank's communicator
    init): fd 1 is pointed at stderr for the whole run and the JSON line goes to a saved
    duplicate of the original stdout."""
    sys.stdout.flush()
    fd = os.dup(1)
    os.dup2(2, 1)
    return fd


def _spawn_ranks(n: int) -> int:
    """``bench.py --gpus N`` without a launcher: run this file under
    ``torch.distributed.run`` (one process per GPU, rendezvous on 127.0.0.1) as a child
    process and return its exit code.  Called before anything touches the GPU (no exec
    from a GPU-initialised process); the ranks write straight to the inherited stdout /
    stderr, so rank 0's JSON line is this command's only stdout line."""
    import socket
    import subprocess

    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    log(f"--gpus {n}: launching {n} ranks ({' '.join(cmd[1:6])} ...)")
    return subprocess.run(cmd, env={**os.environ, "GTR_BENCH_SPAWNED": "1"}).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--batch-size", type=int, default=None, help="sessions per GPU (default 32; c5: 8192)")
    ap.add_argument("--num-batches", type=int, default=None,
                    help="distinct pre-staged batches per GPU (default 64, fewer at large batches: about 32k "
                         "sessions, at least 4)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="bounded CPU-baseline sample (0 = skip)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--resident", type=int, default=None,
                    help="1: launch on the pre-staged batch images (one graph per image); 0: copy each image "
                         "into the step's blob per step (default: 1 on one GPU without the sharded table, "
                         "else 0)")
    ap.add_argument("--step-graph", type=int, default=1,
                    help="one GPU on resident images: the K timed steps launched as hipGraphs of up to 256 "
                         "consecutive steps (FusedTrainStep.capture_steps; every step the full step) instead of "
                         "one graph launch per step (0)")
    ap.add_argument("--dp", action="store_true", help="force the data-parallel step (exchange) even at N=1")
    ap.add_argument("--global-batch", type=int, default=None,
                    help="strong scaling: fixed global batch split over the ranks, SyncBN (1 GPU semantics)")
    ap.add_argument("--sync-bn", action="store_true", help="BatchNorm statistics over every rank's batch")
    ap.add_argument("--shard-table", action="store_true",
                    help="row-sharded item table + AdamW state (rank p owns rows r %% P == p), rows and row "
                         "gradients by all-to-all (etpgt.train.sharded)")
    ap.add_argument("--fit-blocks", type=int, default=1,
                    help="row-sharded table: exchange blocks sized to the staged batches' distinct rows per "
                         "owner (FusedTrainStep.fit_shard_blocks; the ranks agree on the maximum) instead of the "
                         "static bound (1/0)")
    ap.add_argument("--lazy", type=int, default=None,
                    help="deferred zero-gradient AdamW of untouched table rows (1/0; default: per config)")
    ap.add_argument("--lagged", type=int, default=None,
                    help="lazy-table stamps with the previous step's untouched rows swept inside the chain "
                         "(1/0; default: on for the data-parallel step)")
    ap.add_argument("--recall-steps", type=int, default=100,
                    help="Recall@10 parity leg: training steps of the HIP and oracle trainers (0 = skip)")
    ap.add_argument("--recall-sessions", type=int, default=2048, help="held-out sessions of the Recall@10 leg")
    ap.add_argument("--e2e-steps", type=int, default=200,
                    help="end-to-end leg: steps with the batch built on the device inside the step (0 = skip)")
    ap.add_argument("--trainer-epochs", type=int, default=1,
                    help="drop-in leg: timed Trainer.train_epoch epochs over a DeviceSessionLoader (0 = skip)")
    ap.add_argument("--tail-probe", type=int, default=1,
                    help="re-launch the step tail alone to time it (0 = skip; PMC passes skip it so that the "
                         "per-step kernel counts stay exact)")
    ap.add_argument("--gather-batch", type=int, default=8192,
                    help="embedding-gather roofline legs: C5 (512 MB table, HBM) and C3 (42 MB, Infinity Cache) "
                         "shapes (d=128, 100 negatives) at this batch (0 = skip)")
    ap.add_argument("--strong-batches", default="8192,65536",
                    help="strong-scaling legs (comma-separated global batches; '0' = skip): the C4 mode -- C3 model, "
                         "82k table row-sharded, SyncBN, global batch split over the same N GPUs -- run after the "
                         "main line as a child launch (its own process group) and reported under strong_scaling")
    ap.add_argument("--strong-steps", type=int, default=0, help="timed steps per strong leg (0: 40 up to B=16384, "
                                                                 "else 10)")
    ap.add_argument("--c1-reps", type=int, default=5,
                    help="config C1 quick-validation leg (run_full_pipeline.py: model + 3 Adam steps), HIP and CPU "
                         "oracle, median of this many runs (0 = skip)")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        raise SystemExit(_spawn_ranks(args.gpus))
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != args.gpus and args.gpus != 1:
        raise SystemExit(f"--gpus {args.gpus} but the launcher started WORLD_SIZE={os.environ['WORLD_SIZE']} ranks")
    json_fd = _claim_stdout()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal on a one-GPU box (GTR_SHARE_DEVICE=1): every rank on cuda:0, gloo transport
    share = os.environ.get("GTR_SHARE_DEVICE") == "1"
    backend = "gloo" if share else "nccl"
    dev_index = 0 if share else local
    # GTR_FORCE_PG=1: a process group even at world 1 (rehearses the RCCL exchange path
    # on a one-GPU box: `--dp` then all-gathers over RCCL with one rank)
    if world > 1 or os.environ.get("GTR_FORCE_PG") == "1":
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        torch.cuda.set_device(dev_index)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:
            dist.init_process_group("gloo")
    pg_world = None
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        pg_world = torch.distributed.get_world_size()
        if pg_world != world:
            raise SystemExit(f"process group spans {pg_world} ranks, WORLD_SIZE says {world}")
    dev = torch.device("cuda", dev_index)
    torch.cuda.set_device(dev)
    coll_dev = dev if backend == "nccl" else torch.device("cpu")
    cfg = CONFIGS[args.config]
    if args.global_batch is None and args.batch_size is None and cfg.get("global_batch"):
        args.global_batch = cfg["global_batch"]
    if cfg.get("shard"):
        args.shard_table = True
    strong = args.global_batch is not None
    if strong:
        if args.global_batch % world:
            raise SystemExit("--global-batch must divide by the number of GPUs")
        args.batch_size = args.global_batch // world
        args.sync_bn = True
    if args.batch_size is None:
        args.batch_size = cfg.get("batch", 32)
    if args.num_batches is None:
        args.num_batches = 64 if args.batch_size <= 512 else max(4, 32768 // args.batch_size)

    t0 = time.time()
    lazy = bool(args.lazy) if args.lazy is not None else bool(cfg.get("lazy", False))
    dp_on = bool(args.dp or args.sync_bn or world > 1)
    shard = bool(args.shard_table)
    if shard:
        lazy = False  # the shards keep their own lazy stamps
    lagged = (bool(args.lagged) if args.lagged is not None else dp_on) and not lazy and not shard
    w = build_workload(args.config, args.batch_size, args.num_batches, dev, rank, use_graph=not args.no_graph,
                       data_parallel=True if (args.dp or args.sync_bn) else None, lazy=lazy,
                       sync_bn=args.sync_bn and world > 1, lagged=lagged, shard_table=shard,
                       fit_blocks=bool(args.fit_blocks))
    step, staged, batches, data, T, B, touched, st = (w[k] for k in ("step", "staged", "batches", "data", "T", "B",
                                                                   "touched", "stats"))
    log(f"data: T={T} sessions={data.num_sessions} edges={data.edge_keys.size} setup {time.time()-t0:.1f}s {st}")

    # one GPU: each step launches straight on its pre-staged batch image, already in HBM
    # (FusedTrainStep.bind_resident: one captured graph per image; C2 0.0808 -> 0.0796 ms).
    # The data-parallel step trains bitwise the same on resident images
    # (test_dp_resident_images_equal_copied_blob; --resident 1), but measured equal at
    # world 1 over RCCL (0.1108 vs 0.1110 ms), so N > 1 keeps one captured graph and one
    # D2D copy of the image per step inside the timed step, as does the sharded table.
    resident = bool(args.resident) if args.resident is not None else (world == 1 and not shard and not args.dp
                                                                          and not args.sync_bn and not args.no_graph)
    if resident:
        step.bind_resident(staged)

    def one(i):
        if resident:
            return step.run_resident(i % len(staged))
        step.load_blob(staged[i % len(staged)])
        return step.run()

    for i in range(args.warmup):
        one(i)
    if resident and not args.no_graph:
        if args.warmup == 0:
            one(0)  # the images' graphs are captured after one eager step (FusedTrainStep)
        step.prepare_resident()  # no capture inside the timed region
    # K timed steps as multi-step graphs (captured here, outside the timed region): the
    # steps follow each other inside one graph instead of one graph launch per step.
    # Chunks of S <= 256 steps; above 256, S is a multiple of the image count, so every
    # chunk starts on the same image and one graph serves them all.
    seq = None
    if resident and not args.no_graph and args.step_graph and args.steps > 0 and pg_world is None:
        S, full, rem = step_graph_plan(args.steps, len(staged))
        seq = (step.capture_steps(args.warmup, S) if full else None, full,
               step.capture_steps(args.warmup, rem) if rem else None, S)
    elif not resident and not args.no_graph and args.step_graph and args.steps > 0 and (pg_world is not None
                                                                                      or shard):
        # data parallel with the RCCL collectives inside the step's graph, or the one-rank
        # sharded step (aliased exchange, no collective): the timed steps (image copy +
        # step) as multi-step graphs too; None on every rank if any rank's capture was
        # refused (then one graph launch per step, as before)
        S, full, rem = step_graph_plan(args.steps, len(staged))
        g_full = step.capture_steps_copied(staged, args.warmup, S, reserve=args.steps) if full else None
        g_rem = step.capture_steps_copied(staged, args.warmup, rem, reserve=args.steps) if rem else None
        if (g_full is not None or not full) and (g_rem is not None or not rem):
            seq = (g_full, full, g_rem, S)
    torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    t_start = time.perf_counter()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    if seq is not None:
        for _ in range(seq[1]):
            loss = step.run_steps(seq[0])
        if seq[2] is not None:
            loss = step.run_steps(seq[2])
    else:
        for i in range(args.steps):
            loss = one(args.warmup + i)
    ev1.record()
    torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t_start
    gpu_ms = ev0.elapsed_time(ev1)
    if world > 1:
        t = torch.tensor([elapsed], device=coll_dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    final_loss = float(loss)
    step.sync_table()  # lazy table: rows brought to the last step; sharded: gathered from the shards
    replicas_identical = None
    if world > 1:  # data parallel: every rank must hold the same parameters
        chk = torch.stack([step.model.item_embedding.weight.double().sum(), step.eng.flat.flat.double().sum()])
        chk = chk.to(coll_dev)
        allc = [torch.zeros_like(chk) for _ in range(world)]
        torch.distributed.all_gather(allc, chk)
        replicas_identical = all(torch.equal(allc[0], c) for c in allc)
    ms_per_step = elapsed * 1e3 / args.steps
    value = world * B * args.steps / elapsed

    # ---- roofline: the fused step (one hipGraph launch) against HBM; the table AdamW
    # sweep rides in the layer kernels, so the step is the unit that streams the table
    D = cfg["D"]
    step_ms = gpu_ms / args.steps
    alg_bytes = step_bytes(step, cfg, T, st["nodes_per_session"] * B, B, touched, lazy or shard)
    if shard:  # fetched rows written by the owner, gradient rows written + read by the owner
        alg_bytes += 3 * 4.0 * touched * D
    achieved = alg_bytes / (step_ms * 1e-3) / 1e9
    traffic, traffic_src = (load_traffic(args.config if B == cfg.get("batch", 32) else f"{args.config}_b{B}",
                                         lazy) if step.dp is None and not shard else (None, None))
    tail_ms = measure_tail(step, args.steps) if args.tail_probe and not shard else None

    log(f"timed: {value:.1f} sessions/s, {ms_per_step:.4f} ms/step")
    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(cfg, batches, T, args.cpu_seconds)
        log(f"cpu baseline: {cpu['value']} sessions/s")
    e2e = None
    if rank == 0 and world == 1 and args.e2e_steps > 0:
        e2e = e2e_probe(cfg, data, dev, B, args.e2e_steps)
        log(f"end to end: {e2e['device_batch_build_sessions_per_s']} sessions/s")
    trainer_leg = None
    if rank == 0 and world == 1 and args.trainer_epochs > 0 and not shard:
        trainer_leg = trainer_epoch_probe(cfg, data, dev, B, args.trainer_epochs)
        trainer_leg["vs_headline_ms_per_step"] = round(trainer_leg["ms_per_step"] / ms_per_step, 4)
        log(f"trainer epoch: {trainer_leg['sessions_per_s']} sessions/s, {trainer_leg['ms_per_step']} ms/step")
    gather = gather_c = None
    if rank == 0 and world == 1 and args.gather_batch > 0:
        gather = gather_probe(dev, args.gather_batch, "c5")
        log(f"gather roofline (C5 table): frac {gather['frac']}")
        gather_c = gather_probe(dev, args.gather_batch, "c3")
        log(f"gather roofline (C3 table): frac {gather_c['frac']}")
    c1 = None
    if rank == 0 and world == 1 and args.c1_reps > 0:
        c1 = c1_quick(dev, args.c1_reps)
        log(f"C1 quick validation: HIP {c1['hip_ms_per_3_steps']} ms, CPU oracle {c1['cpu_oracle_ms_per_3_steps']} ms "
            "per 3 steps")
    recall = None
    if rank == 0 and world == 1 and args.recall_steps > 0:
        recall = recall_parity(cfg, data, T, dev, args.recall_steps, args.recall_sessions)
        log(f"recall parity: {recall['gpu']} vs {recall['oracle']}")

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "sessions/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "gemm_precision": gemm_mode(D),
            "build": build_provenance(),
            "data": ("synthetic Yoochoose-scale" if cfg.get("scale") else "synthetic RetailRocket-shaped")
                    + " sessions/graph (seed 42), random-init weights",
            "config": {
                "workload": cfg["name"],
                "global_batch": B * world,
                "per_gpu_batch": B,
                "num_items": T,
                "graph_edges": int(data.edge_keys.size),
                "nodes_per_session": round(st["nodes_per_session"], 3),
                "edges_per_session": round(st["edges_per_session"], 3),
                "parallelism": f"dp{world}" + ("+rowshard" if shard else ""),
                "transport": "rccl" if backend == "nccl" else "gloo (shared-device rehearsal)",
                "process_group_world": pg_world,
                "visible_gpus": torch.cuda.device_count(),
                "launcher": ("bench.py --gpus (torch.distributed.run child)" if os.environ.get("GTR_BENCH_SPAWNED")
                             else "external (torchrun / torch.distributed.run)" if "WORLD_SIZE" in os.environ
                             else "none (one process)"),
                "dp_exchange": ("row-sharded table: all-to-all of row ids, rows and row gradients "
                                f"({step.shard.volume()}; blocks "
                                + ("fitted to the staged batches, +10 % headroom" if args.fit_blocks else "static bound") + ")")
                               if shard else step.dp is not None,
                "hip_graph": not args.no_graph,
                "batch_images": "resident, one graph per image" if resident else "copied per step (D2D)",
                "step_graph": (f"{seq[3]} consecutive steps per hipGraph launch ({seq[1]} x {seq[3]}"
                               + (f" + {args.steps % seq[3]}" if seq[2] is not None else "") + ")"
                               if seq is not None else "one graph launch per step"),
                "lazy_table": lazy,
                "lagged_sweep": lagged,
                "gemm": gemm_mode(D),
                "graph_collectives": bool((step.dp is not None or shard) and step._graph_collectives()),
                "sync_bn": bool(args.sync_bn and world > 1),
                "gpu_ms_per_step_events": round(gpu_ms / args.steps, 4),
                "final_loss": round(final_loss, 6),
                "replicas_identical": replicas_identical,
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "fused training step = one hipGraph launch (begin, conv_fwd x2, readout, conv_bwd x2, "
                          "wgrad, tail; the untouched-row AdamW sweep runs as extra workgroups of the layer "
                          "kernels)" + (" + RCCL all-gather + dp tail" if step.dp is not None else ""),
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": None if traffic is None else round(traffic),
                "traffic_unit": "HBM bytes per step (PMC FETCH_SIZE x2 + WRITE_SIZE, summed over the step's kernels)",
                "traffic_source": traffic_src,
                "alg_bytes_per_launch": int(alg_bytes),
                "alg_bytes_terms": ("(24*D + 4) per touched row (lazy table: no untouched-row sweep)" if lazy
                                    else "24*T*D table p/m/v + 4*T stamps")
                                   + " + gathered rows/ids + 36*4*N*D per layer + small params (24 + 4*P slab partials "
                                     "per element)",
                "touched_rows_per_step": round(touched, 1),
                "avg_launch_ms": round(step_ms, 5),
                "tail_kernel": {"name": ("k_dp_tail" if step.dp is not None else
                                         "k_step_tail_wgrad" if getattr(step, "tail_wgrad", False) else "k_step_tail"),
                                "avg_launch_ms": None if tail_ms is None else round(tail_ms, 5)},
            },
            "cpu_baseline": cpu,
            "end_to_end": e2e,
            "trainer_epoch": trainer_leg,
            "gather_roofline": gather,
            "gather_roofline_infinity_cache": gather_c,
            "recall_parity": recall,
            "c1_quick_validation": c1,
        }
    if world > 1:
        # every collective of the run is done (the MAX all-reduce and the replica check
        # above).  The captured graphs hold RCCL collectives, and a communicator whose
        # collectives are still captured in a live graph does not come back from
        # destroy_process_group (scripts/dbg/teardown_probe.py): release them first
        seq = None
        step.close()
        torch.distributed.barrier()
        torn_down = _bounded(torch.distributed.destroy_process_group, 120.0)
        if not torn_down:  # guard only: the released-graph teardown returns in < 1 s (profiles/r06)
            print("bench: destroy_process_group did not return within 120 s; the line is printed and the "
                  "process exits without it", file=sys.stderr, flush=True)
    else:
        torn_down = True
    if rank == 0:
        legs = [int(x) for x in args.strong_batches.split(",") if x.strip() and int(x) > 0]
        if legs and not cfg.get("shard") and os.environ.get("GTR_STRONG_CHILD") != "1":
            del w, step, staged
            torch.cuda.empty_cache()
            out["strong_scaling"] = strong_scaling_legs(world, legs, args.strong_steps)
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    if not torn_down:
        sys.stderr.flush()
        os._exit(0)


def _bounded(fn, seconds: float) -> bool:
    """Run ``fn`` in a daemon thread; True when it returned within ``seconds``."""
    import threading

    t = threading.Thread(target=fn, daemon=True)
    t.start()
    t.join(seconds)
    return not t.is_alive()


def _child_line(cmd: list, env: dict, timeout: float) -> dict:
    """Run one bench child (its stdout: ONE JSON line) with a time limit; errors are
    returned, not raised, so the main line is always printed."""
    import subprocess

    try:
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    except subprocess.TimeoutExpired:
        return {"error": f"timed out after {timeout:.0f} s"}
    lines = [ln for ln in r.stdout.splitlines() if ln.strip().startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": f"exit {r.returncode}: {r.stderr.strip()[-600:]}"}
    return json.loads(lines[-1])


def strong_scaling_legs(world: int, global_batches: list, steps: int = 0) -> dict:
    """North star: ">= 6x strong scaling at 8 GPUs".  The C4 mode (configs[3]: the C3 model
    on the RetailRocket table, the table row-sharded across the ranks, rows / row
    gradients by RCCL all-to-all, SyncBN) at each fixed global batch, split over the SAME
    N GPUs as this run: one child launch per batch (``torch.distributed.run`` with N
    ranks, or one process at N = 1) after this run's process group is gone, so a failure
    there cannot take the main line with it.  At N = 1 the unsharded single-GPU step at
    the same batch (C3 at B = G) is reported beside it.  The driver's N = 1 / 2 / 4 / 8
    lines together give the curve: value(N) / value(1) per global batch."""
    import socket

    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                        "ROLE_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID", "GTR_BENCH_SPAWNED")
           and not k.startswith("TORCHELASTIC")
           # a launcher may pin each rank to one device: the N-rank child must see all N
           and k not in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES")}
    env["GTR_STRONG_CHILD"] = "1"
    lean = ["--cpu-seconds", "0", "--gather-batch", "0", "--recall-steps", "0", "--e2e-steps", "0", "--c1-reps", "0",
            "--trainer-epochs", "0",
            "--tail-probe", "0", "--strong-batches", "0"]
    res = {"config": "c4", "workload": CONFIGS["c4"]["name"], "n_gpus": world, "legs": []}
    for G in global_batches:
        st = steps or (40 if G <= 16384 else 10)
        wu = 5 if G <= 16384 else 3
        nb = 4 if G // world <= 16384 else 2
        args = [os.path.abspath(__file__), "--config", "c4", "--gpus", str(world), "--global-batch", str(G),
                "--steps", str(st), "--warmup", str(wu), "--num-batches", str(nb), *lean]
        if G % world:
            res["legs"].append({"global_batch": G, "error": "global batch does not divide by the GPUs"})
            continue
        if world > 1:
            sock = socket.socket()
            sock.bind(("127.0.0.1", 0))
            port = sock.getsockname()[1]
            sock.close()
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
                   "--master-addr", "127.0.0.1", "--master-port", str(port), *args]
        else:
            cmd = [sys.executable, *args]
        log(f"strong scaling leg: C4 global batch {G} over {world} GPU(s)")
        t0 = time.time()
        line = _child_line(cmd, env, 600.0)
        leg = {"global_batch": G, "per_gpu_batch": G // world, "wall_s": round(time.time() - t0, 1)}
        if "error" in line:
            leg["error"] = line["error"]
        else:
            c = line["config"]
            seen = c.get("visible_gpus")
            if c.get("process_group_world", 1) not in (None, world) or (
                    seen is not None and seen < world and not str(c.get("transport", "")).startswith("gloo")):
                leg["error"] = (f"the child ran {c.get('process_group_world')} ranks on {seen} visible GPU(s), "
                                f"not {world}")
            leg.update({"value": line["value"], "unit": line["unit"], "ms_per_step": line["ms_per_step"],
                        "gpu_ms_per_step_events": c["gpu_ms_per_step_events"], "steps": line["steps"],
                        "parallelism": c["parallelism"], "process_group_world": c["process_group_world"],
                        "transport": c["transport"], "graph_collectives": c["graph_collectives"],
                        "sync_bn": c["sync_bn"], "replicas_identical": c["replicas_identical"],
                        "exchange": c["dp_exchange"], "final_loss": c["final_loss"]})
        if world == 1 and "error" not in leg:  # the plain single-GPU step at the same batch, beside it
            one = _child_line([sys.executable, os.path.abspath(__file__), "--config", "c3", "--batch-size", str(G),
                               "--steps", str(st), "--warmup", str(wu), "--num-batches", str(nb), *lean], env, 600.0)
            leg["unsharded_single_gpu"] = ({"error": one["error"]} if "error" in one else
                                           {"value": one["value"], "ms_per_step": one["ms_per_step"],
                                            "config": "c3 (same model and table, no row sharding)"})
        log(f"  -> {leg}")
        res["legs"].append(leg)
    return res


def build_workload(config: str, B: int, num_batches: int, dev, rank: int = 0, use_graph: bool = True,
                   data_parallel: bool | None = None, lazy: bool = False, sync_bn: bool = False,
                   lagged: bool = False, shard_table: bool = False, fit_blocks: bool = False) -> dict:
    """Synthetic RetailRocket-shaped data, the model of `config`, a bound fused step
    and `num_batches` packed batches pre-staged in HBM."""
    from etpgt.data.batch import Caps
    from etpgt.data.synthetic import batch_stats, make_batches, make_sessions_and_graph, random_pe_table
    from etpgt.model import create_graph_transformer_optimized
    from etpgt.train.fused import FusedTrainStep

    cfg = CONFIGS[config]
    if cfg.get("scale") == "yoochoose":
        from etpgt.data.synthetic import YOOCHOOSE_SCALE

        data = make_sessions_and_graph(seed=42, **YOOCHOOSE_SCALE)
    else:
        data = make_sessions_and_graph(seed=42)
    T = data.table_rows
    batches = make_batches(data, B, num_batches, cfg["n_neg"], seed=42, start=rank * B * num_batches)
    st = batch_stats(batches)
    torch.manual_seed(42)
    model = create_graph_transformer_optimized(T, embedding_dim=cfg["D"], hidden_dim=cfg["D"], num_layers=2,
                                               num_heads=cfg["H"], dropout=0.1, use_laplacian_pe=cfg["K"] > 0,
                                               laplacian_k=max(cfg["K"], 1))
    if cfg["K"] > 0:
        model.laplacian_pe._cached_pe = random_pe_table(T, cfg["K"])
    model = model.to(dev).train()
    step = FusedTrainStep(model, lr=1e-3, weight_decay=1e-5, loss=cfg["loss"], use_graph=use_graph,
                          data_parallel=data_parallel, lazy=lazy, sync_bn=sync_bn, lagged=lagged,
                          shard_table=shard_table)
    caps = Caps(max(b.num_nodes for b in batches), B, max(b.num_edges for b in batches), cfg["n_neg"])
    step._bind(caps)  # data parallel: the ranks agree on the largest capacities
    caps = step.caps
    if shard_table and fit_blocks:  # exchange blocks sized to these batches (collective)
        step.fit_shard_blocks(batches)
    staged = [torch.from_numpy(b.packed(caps)[1]).to(dev) for b in batches]
    touched = float(np.mean([len(set(b.x.tolist()) | set(b.target_item.tolist()) | set(b.negative_items.tolist()))
                             for b in batches]))
    return dict(step=step, staged=staged, batches=batches, data=data, T=T, B=B, touched=touched, stats=st,
                caps=caps, model=model)


def load_traffic(config: str, lazy: bool = False):
    """HBM bytes per training step from the newest committed PMC summary
    (profiles/rNN/<config>_pmc.json, scripts/gpu/profile.sh: two rocprofv3 --pmc passes,
    FETCH_SIZE doubled per the gfx950 note + WRITE_SIZE, summed over the step's kernels
    by scripts/pmc_parse.py).  Only a profile of THESE kernel sources counts (its
    ``_source_hash`` must equal the tree's); otherwise traffic is null."""
    import glob

    from etpgt.backend._lib import source_hash

    name = f"{config}_lazy" if lazy and not config.startswith("c5") else config
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", f"{name}_pmc.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    rec = d.get("_per_step")
    if not rec or d.get("_source_hash") != source_hash():
        return None, None
    return float(rec["hbm_bytes_per_step"]), os.path.relpath(files[-1], ROOT)


def measure_tail(step, iters) -> float:
    """Average duration (ms) of the step-tail kernel (AdamW over every item-table row
    + small parameters), bracketed by HIP events on the stream it is launched on.
    Re-launches the last step's tail: a valid optimizer update on that step's gradients."""
    main = torch.cuda.current_stream()
    durs = []
    n = max(10, min(iters, 200))
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(main)
        step._launch_b(False)  # the step's own tail: dp tail, tail with weight gradients, or plain
        e1.record(main)
        durs.append((e0, e1))
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in durs]))


def step_graph_plan(steps: int, nimg: int, cap: int = 256) -> tuple[int, int, int]:
    """Chunking of K timed steps into multi-step graphs: (S, full, rem) with K = full * S +
    rem.  K <= cap: one graph of K steps.  Above, S is a multiple of the image count (so
    every chunk, and the remainder, starts on the same resident image and one graph serves
    all full chunks)."""
    if steps <= cap:
        return steps, 1, 0
    S = max(nimg, (cap // nimg) * nimg)
    full, rem = divmod(steps, S)
    return S, full, rem


def gemm_mode(D: int) -> str:
    """The layer GEMMs' arithmetic (gemm_split in csrc/gtr_common.cuh)."""
    e = os.environ.get("GTR_GEMM", "").lower()
    split = e.startswith("s")  # opt-in only (csrc/gtr_common.cuh gemm_split)
    return ("split-bf16 MFMA (hi/lo operands, 3 bf16 MFMAs, fp32 accumulate)" if split
            else "f32-input MFMA (exact f32)")


def step_bytes(step, cfg, T, N, B, touched: float, lazy: bool) -> float:
    """Algorithmic HBM bytes of one training step (each distinct tensor
    read or written once): the table AdamW (p, m, v read + write = 24 B per element; no
    dense gradient) + the stamps; the gathered node / PE / scoring rows and their ids;
    layer activations (12 forward + 24 backward D-vectors per node and layer, §8d); the
    small parameters (p, m, v + one read of each split-K partial).  The lazy table
    (gtr_lazy) does not sweep the untouched rows: its table term is the touched rows
    only (catch-up and update of a row = one read + write of p, m, v, 24 B per element)
    plus their stamps."""
    D, K, n = cfg["D"], cfg["K"], cfg["n_neg"]
    table = (24.0 * D + 4.0) * (touched if lazy else T)
    gather = 4.0 * N * D + 4.0 * N * K + 4.0 * B * (1 + n) * D + 4.0 * (N + B * (1 + n))
    acts = step.eng.L * 36 * 4.0 * N * D
    small = step.eng.flat.layout.total * (24.0 + 4.0 * step.ws.P)
    return table + gather + acts + small


def e2e_probe(cfg, data, dev, B, steps):
    """End to end from resident session data: the batch is built
    on the device (etpgt.data.gpu_batch: SessionDataset.__getitem__ + collate_fn as
    kernels) inside the captured step, walking a shuffled epoch order.  Beside it, the
    host pipeline: per-session example + collate + pack on the host, one H2D copy, the
    same fused step."""
    from etpgt.data.batch import collate_sessions
    from etpgt.data.gpu_batch import GpuBatchBuilder, GpuSessionStore
    from etpgt.data.synthetic import random_pe_table, session_example
    from etpgt.model import create_graph_transformer_optimized
    from etpgt.train.fused import FusedTrainStep

    T = data.table_rows
    kw = dict(embedding_dim=cfg["D"], hidden_dim=cfg["D"], num_layers=2, num_heads=cfg["H"], dropout=0.1,
              use_laplacian_pe=cfg["K"] > 0, laplacian_k=max(cfg["K"], 1))
    torch.manual_seed(42)
    model = create_graph_transformer_optimized(T, **kw)
    if cfg["K"] > 0:
        model.laplacian_pe._cached_pe = random_pe_table(T, cfg["K"])
    model = model.to(dev).train()
    t0 = time.perf_counter()
    store = GpuSessionStore.from_synthetic(data, dev)
    torch.cuda.synchronize(dev)
    store_s = time.perf_counter() - t0
    bld = GpuBatchBuilder(store, B, cfg["n_neg"], seed=9)
    order = np.random.default_rng(9).permutation(data.num_sessions)
    bld.set_epoch_order(order)
    step = FusedTrainStep(model, lr=1e-3, weight_decay=1e-5, loss=cfg["loss"])
    step.attach_builder(bld)  # capacities for the whole epoch order
    for _ in range(20):
        step.run()
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    for _ in range(steps):
        step.run()
    torch.cuda.synchronize(dev)
    dev_s = (time.perf_counter() - t) / steps
    # host pipeline on the same model / step object (builder detached)
    step.detach_builder()
    rng = np.random.default_rng(10)
    hs = max(10, steps // 10)
    pos = 0
    for i in range(3 + hs):
        if i == 3:
            torch.cuda.synchronize(dev)
            t = time.perf_counter()
        ids = order[(pos + np.arange(B)) % order.size]
        pos += B
        sb = collate_sessions([session_example(data, int(s), cfg["n_neg"], rng) for s in ids])
        step(sb)
    torch.cuda.synchronize(dev)
    host_s = (time.perf_counter() - t) / hs
    return {
        "device_batch_build_sessions_per_s": round(B / dev_s, 1),
        "device_ms_per_step": round(dev_s * 1e3, 4),
        "host_batch_build_sessions_per_s": round(B / host_s, 1),
        "host_ms_per_step": round(host_s * 1e3, 3),
        "batch": B,
        "store_setup_s": round(store_s, 3),
        "note": "device: k_bb_scan + k_bb_write in the captured step, epoch order walked by a device cursor; "
                "host: per-session example + collate + pack + H2D per step",
    }


def trainer_epoch_probe(cfg, data, dev, B, epochs: int = 1, steps_per_graph: int | None = None):
    """The drop-in path at the headline shape: ``Trainer.train_epoch`` (trainer.py:80-133)
    over a ``DeviceSessionLoader`` on the synthetic sessions, i.e. what
    ``scripts/train/train_baseline.py`` runs -- every batch built on the device inside the
    step, the epoch's full batches as multi-step hipGraphs (``steps_per_graph``), the
    partial last batch eager, the epoch loss read once.  One untimed epoch (captures),
    then ``epochs`` timed epochs, wall clock around ``train_epoch`` (host work included:
    the epoch order draw, its upload, capacity planning)."""
    from etpgt.data.gpu_batch import GpuSessionStore
    from etpgt.data.synthetic import random_pe_table
    from etpgt.model import create_graph_transformer_optimized
    from etpgt.train.dataloader import DeviceSessionLoader
    from etpgt.train.losses import create_loss_function
    from etpgt.train.trainer import Trainer

    T = data.table_rows
    torch.manual_seed(42)
    model = create_graph_transformer_optimized(T, embedding_dim=cfg["D"], hidden_dim=cfg["D"], num_layers=2,
                                               num_heads=cfg["H"], dropout=0.1, use_laplacian_pe=cfg["K"] > 0,
                                               laplacian_k=max(cfg["K"], 1))
    if cfg["K"] > 0:
        model.laplacian_pe._cached_pe = random_pe_table(T, cfg["K"])
    store = GpuSessionStore.from_synthetic(data, dev)
    loader = DeviceSessionLoader.from_store(store, B, cfg["n_neg"], shuffle=True, seed=42)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3, weight_decay=1e-5)
    lf = None if cfg["loss"] == "bpr" else create_loss_function(cfg["loss"])
    import tempfile

    with tempfile.TemporaryDirectory() as tmp:
        tr = Trainer(model, loader, None, opt, device=str(dev), output_dir=tmp, loss_fn=lf)
        if steps_per_graph is not None:
            tr.steps_per_graph = steps_per_graph
        tr.train_epoch()  # untimed: captures the step and chunk graphs
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        losses = [tr.train_epoch() for _ in range(epochs)]
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t
    n_steps = len(loader.batch_sizes()) * epochs
    sessions = loader.num_sessions * epochs
    out = {
        "sessions_per_s": round(sessions / el, 1),
        "ms_per_step": round(el * 1e3 / n_steps, 4),
        "steps": n_steps,
        "epochs": epochs,
        "batch": B,
        "steps_per_graph": tr.steps_per_graph,
        "chunk_graphs": tr._chunk_graph is not None,
        "epoch_loss": round(losses[-1], 6),
        "note": "Trainer.train_epoch over DeviceSessionLoader (train_baseline.py's path): batch build inside the "
                "step, full batches as multi-step hipGraphs, partial last batch eager; wall clock per epoch",
    }
    del tr, model
    torch.cuda.empty_cache()
    return out


def gather_probe(dev, B, config="c5", nbatch=4, steps=20):
    """North-star embedding-gather target: the sampled-scoring gather at
    d=128, n=100 negatives, large batch.  The dominant gather kernel is the readout /
    scoring kernel (wave per session at this size): per launch it reads B*(1+n) table
    rows + ids, the last layer's out/xin node rows, writes se, dy and the score
    coefficients.  Its average launch time is measured with HIP events around re-launches
    of that kernel (FWD|LOSS|BWD, the same work as inside the step) on the step's stream;
    the full-step rate at this batch is reported beside it.

    ``config="c5"`` gathers from the 1M x 128 table (512 MB: larger than the 256 MB
    Infinity Cache, so the rows come from HBM -- the honest number for the target);
    ``"c3"`` from the 82k x 128 table (42 MB, Infinity-Cache resident).

    The re-launches rotate over ``nbatch`` (>= 4) distinct pre-staged batches (the batch
    image is copied in before each timed launch, outside its events), so no batch's rows
    are still resident in the 256 MB Infinity Cache when the batch comes round again
    (4 x ~290 MB of distinct rows at B = 8192, C5); the same-batch re-launch rate of
    round 2 is reported beside it (``same_batch``)."""
    from etpgt.backend import _lib as L

    cfg = CONFIGS[config]
    w = build_workload(config, B, nbatch, dev, 0, use_graph=True, lazy=bool(cfg.get("lazy", False)))
    step, staged, batches, T = w["step"], w["staged"], w["batches"], w["T"]
    for i in range(3):
        step.load_blob(staged[i % nbatch])
        step.run()
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    for i in range(steps):
        step.load_blob(staged[i % nbatch])
        step.run()
    torch.cuda.synchronize(dev)
    step_s = (time.perf_counter() - t) / steps
    last = batches[(steps - 1) % nbatch]
    eng, ws = step.eng, step.ws
    flags = L.RO_FWD | L.RO_LOSS | L.RO_BWD
    main = torch.cuda.current_stream(dev)
    D, n = cfg["D"], cfg["n_neg"]

    def alg_bytes(b):
        N, Bl = b.num_nodes, b.num_graphs
        rows = 4.0 * Bl * (1 + n) * D
        return rows + 4.0 * Bl * (1 + n) + 4.0 * (Bl + 1) + 3 * 4.0 * N * D + 4.0 * Bl * D + 4.0 * Bl * (1 + n)

    def relaunch(rotate):
        durs = []
        for i in range(8 * nbatch if rotate else 30):
            j = i % nbatch if rotate else (steps - 1) % nbatch
            if rotate:
                step.load_blob(staged[j])  # outside the events: the copy is not timed
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(main)
            eng.run_head(ws, step.cfg, step.bs, flags, step.loss_kind, step.temperature, step.alpha)
            e1.record(main)
            durs.append((alg_bytes(batches[j]), e0, e1))
        torch.cuda.synchronize(dev)
        durs = durs[nbatch if rotate else 5:]
        ms = float(np.median([a.elapsed_time(b) for _, a, b in durs]))
        gbs = float(np.median([by / (a.elapsed_time(b) * 1e-3) / 1e9 for by, a, b in durs]))
        return ms, gbs

    step.load_blob(staged[(steps - 1) % nbatch])
    ms_same, ach_same = relaunch(False)
    ms, ach = relaunch(True)
    N, Bl = last.num_nodes, last.num_graphs
    rows = 4.0 * Bl * (1 + n) * D
    alg = alg_bytes(last)
    traffic, src = load_kernel_traffic(f"{config}_b{B}" if B != cfg.get("batch", 32) else config, "k_readout_wave")
    table_mb = T * D * 4 / 1e6
    step.flush()
    del w, step
    torch.cuda.empty_cache()
    return {
        "bound": "hbm",
        "kernel": "k_readout_wave (mean readout + sampled scoring gather + listwise loss fwd/bwd)",
        "workload": f"{config.upper()} model (d=128, 4 heads, LapPE), listwise with {n} negatives, B={Bl}, N={N} nodes, "
                    f"table {T} x {D} fp32 ({table_mb:.0f} MB)",
        "achieved": round(ach, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(ach / HBM_PEAK_GBS, 4),
        "traffic": traffic,
        "traffic_unit": "bytes/launch (PMC FETCH_SIZE x2 + WRITE_SIZE)",
        "traffic_source": src,
        "alg_bytes_per_launch": int(alg),
        "scoring_row_bytes_per_launch": int(rows),
        "avg_launch_ms": round(ms, 5),
        "rotating_batches": nbatch,
        "same_batch": {"achieved": round(ach_same, 1), "frac": round(ach_same / HBM_PEAK_GBS, 4),
                       "avg_launch_ms": round(ms_same, 5),
                       "note": "30 re-launches on ONE batch (round 2's method): part of its rows may be "
                               "Infinity-Cache hits"},
        "step_sessions_per_s": round(Bl / step_s, 1),
        "note": ("table larger than the 256 MB Infinity Cache: scoring rows are served from HBM; re-launches "
                 f"rotate over {nbatch} distinct batches (median of per-launch rates)" if table_mb > 256
                 else "table sits in the 256 MB Infinity Cache: rows are algorithmic bytes, not HBM bytes"),
    }


def load_kernel_traffic(name: str, kernel: str):
    """Per-launch HBM bytes of one kernel from profiles/rNN/<name>_pmc.json, if that
    profile was taken on these kernel sources."""
    import glob

    from etpgt.backend._lib import source_hash

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", f"{name}_pmc.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    rec = d.get(kernel)
    if not rec or d.get("_source_hash") != source_hash():
        return None, None
    return round(float(rec["hbm_bytes_per_launch"])), os.path.relpath(files[-1], ROOT)


def recall_parity(cfg, data, T, dev, steps, n_val, B=32):
    """Recall@10 parity (the metric's second half, trainer.py:138-173): the HIP fused
    trainer and the oracle trainer start from the same weights and take the same `steps`
    AdamW steps on the same batches (dropout 0: the HIP dropout stream cannot reproduce
    the CPU generator), then both evaluate Recall@10 / NDCG@10 over the same held-out
    sessions — HIP forward + gtr_score_topk vs oracle forward + torch matmul/topk.  Also
    times the HIP evaluation (forward + full-catalog top-k) in sessions/s."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import etpgt_ref as R

    from etpgt.data.synthetic import make_batches, random_pe_table
    from etpgt.model import create_graph_transformer_optimized
    from etpgt.train.fused import FusedTrainStep
    from etpgt.utils.metrics import compute_ndcg_at_k, compute_recall_at_k

    t0 = time.time()
    kw = dict(embedding_dim=cfg["D"], hidden_dim=cfg["D"], num_layers=2, num_heads=cfg["H"], dropout=0.0,
              use_laplacian_pe=cfg["K"] > 0, laplacian_k=max(cfg["K"], 1))
    torch.manual_seed(7)
    m = create_graph_transformer_optimized(T, **kw)
    ref = R.ref_create_graph_transformer_optimized(T, **kw)
    if cfg["K"] > 0:
        pe = random_pe_table(T, cfg["K"])
        m.laplacian_pe._cached_pe = pe.clone()
        ref.laplacian_pe._cached_pe = pe.clone()
    ref.load_state_dict({k: v.detach().clone() for k, v in m.state_dict().items()})
    m = m.to(dev).train()
    ref.train()
    fused = FusedTrainStep(m, lr=1e-3, weight_decay=1e-5, loss=cfg["loss"])
    ropt = torch.optim.AdamW(ref.parameters(), lr=1e-3, weight_decay=1e-5)
    train = make_batches(data, B, steps, cfg["n_neg"], seed=7, start=96_000)
    for sb in train:
        fused(sb.to(dev))
        R.ref_train_step(ref, R.ref_batch_from(sb), ropt, cfg["loss"])
    vb = make_batches(data, 256, max(1, n_val // 256), cfg["n_neg"], seed=7, start=112_000)
    m.eval()
    ref.eval()
    staged = [sb.to(dev) for sb in vb]
    with torch.no_grad():
        for sb in staged[:2]:  # warm-up (workspaces, top-k scratch)
            m.predict(m(sb), k=10)
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        preds = [m.predict(m(sb), k=10) for sb in staged]
        torch.cuda.synchronize(dev)
        eval_s = time.perf_counter() - t
        rpreds = [ref.predict(ref(R.ref_batch_from(sb)), k=10) for sb in vb]
    tg = torch.cat([sb.target_item for sb in vb])
    p = torch.cat(preds).cpu()
    rp = torch.cat(rpreds)
    n = int(tg.numel())
    out = {
        "train_steps": steps, "train_batch": B, "val_sessions": n, "dropout": 0.0, "loss": cfg["loss"],
        "gpu": {"recall@10": round(compute_recall_at_k(p, tg, 10), 5), "ndcg@10": round(compute_ndcg_at_k(p, tg, 10), 5)},
        "oracle": {"recall@10": round(compute_recall_at_k(rp, tg, 10), 5),
                   "ndcg@10": round(compute_ndcg_at_k(rp, tg, 10), 5)},
        "top10_overlap": round(sum(len(set(a) & set(b)) for a, b in zip(p.tolist(), rp.tolist())) / (10.0 * n), 5),
        "hip_eval_sessions_per_s": round(n / eval_s, 1),
        "wall_s": round(time.time() - t0, 1),
    }
    out["abs_diff_recall@10"] = round(abs(out["gpu"]["recall@10"] - out["oracle"]["recall@10"]), 5)
    return out


def build_provenance() -> dict:
    """Which binary ran: the source hash compiled into the loaded libgtr_hip.so, this
    tree's source hash, and the library's path and modification time."""
    from etpgt.backend import _lib

    lib_hash, tree_hash = _lib.library_source_hash(), _lib.source_hash()
    return {"lib": os.path.relpath(_lib.LIB_PATH, os.path.dirname(os.path.abspath(__file__))),
            "lib_source_hash": lib_hash, "tree_source_hash": tree_hash, "built_from_tree": lib_hash == tree_hash,
            "lib_mtime_utc": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(os.path.getmtime(_lib.LIB_PATH)))}


C1_PUBLISHED_T = 188  # 45,952 parameters of the optimized model, d=64, H=2, L=2, no PE


def c1_quick(dev, reps: int) -> dict:
    """Config C1 (BASELINE.json configs[0]): run_full_pipeline.py's quick
    validation -- the reference's own 100-session synthetic data (scripts/data 00 -> 02 ->
    04 restated by etpgt.pipeline), the 16-session bidirectional batch, model creation +
    3 Adam steps with the listwise loss, timed like the reference (``duration`` spans model
    creation and the three steps, run_full_pipeline.py:200-236) -- on the HIP model
    (etpgt.pipeline.test_model_with_real_data) and on the CPU oracle restatement, beside
    the published 7 ms on an M1 (docs/EXPERIMENTS.md:88).  Median of ``reps`` runs after
    one warm-up run each."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import etpgt_ref as R

    from etpgt import pipeline as P
    from etpgt.model import create_graph_transformer_optimized

    ev = P.generate_synthetic_events(num_sessions=100, num_items=1000, seed=42)
    sd = P.sessionize_events(ev)
    g = P.build_co_event_graph(sd)
    sub, gs = P.create_test_subset(sd, g, num_sessions=100)
    batch, T_data = P.create_batch_from_sessions(sub, gs, batch_size=16, num_negatives=5)
    # the published run's catalog: T = 188 items (45,952 parameters, docs/EXPERIMENTS.md:88),
    # from the reference's processed data, which the synthetic generator does not reproduce
    # (its first 100 sessions hold T_data distinct items); the batch's ids all lie below it
    T = max(T_data, C1_PUBLISHED_T)
    cfg = dict(num_items=T, embedding_dim=64, hidden_dim=64, num_layers=2, num_heads=2, use_laplacian_pe=False,
               dropout=0.1)
    hip, hip_loss, params = [], None, None
    for i in range(reps + 1):
        torch.manual_seed(i)
        res = P.test_model_with_real_data("GraphTransformer (optimized, no FFN)", create_graph_transformer_optimized,
                                          cfg, batch, num_epochs=3, device=str(dev))
        if res["status"] != "PASS":
            raise RuntimeError(f"C1 quick validation failed: {res}")
        torch.cuda.synchronize(dev)
        if i > 0:
            hip.append(res["duration"])
            hip_loss, params = res["final_loss"], res["param_count"]
    rb = R.ref_batch_from(batch)
    cpu, cpu_loss = [], None
    for i in range(reps + 1):
        torch.manual_seed(i)
        t = time.time()
        ref = R.ref_create_graph_transformer_optimized(**cfg)
        opt = torch.optim.Adam(ref.parameters(), lr=0.001)
        for _ in range(3):
            ref.train()
            opt.zero_grad()
            se = ref(rb)
            loss = R.ref_loss("listwise", se, rb.target_item, rb.negative_items.view(se.shape[0], -1),
                              ref.item_embedding)
            loss.backward()
            opt.step()
            cpu_loss = float(loss.item())
        if i > 0:
            cpu.append(time.time() - t)
    return {
        "workload": f"run_full_pipeline.py quick validation: 100 synthetic sessions (reference generator, seed 42; "
                    f"{T_data} distinct items), 16-session batch, catalog T={T} as in the published run, d=64, "
                    f"2 heads, 2 layers, no LapPE, listwise, Adam(1e-3), 3 steps",
        "hip_ms_per_3_steps": round(1e3 * float(np.median(hip)), 3),
        "cpu_oracle_ms_per_3_steps": round(1e3 * float(np.median(cpu)), 3),
        "cpu_threads": torch.get_num_threads(),
        "published_ms_per_3_steps": 7.0,
        "published_hardware": "MacBook Pro M1 (docs/EXPERIMENTS.md:26,88)",
        "final_loss_hip": round(hip_loss, 4),
        "final_loss_cpu_oracle": round(cpu_loss, 4),
        "published_final_loss": 1.21,
        "param_count": params,
        "note": "duration = model creation + 3 steps (run_full_pipeline.py:200-236); dropout 0.1 as in the "
                "reference, so HIP and CPU losses differ by their dropout streams",
    }


def _cpu_share() -> tuple[int, str]:
    """Threads for the CPU baseline: the CPU share this process may actually use.  On the
    GPU box ``os.cpu_count()`` reports the whole machine while a cgroup quota grants this
    job a slice of it (16 CPUs per GPU); oversubscribing the quota with one thread per
    machine core stalls torch's OpenMP pool, so the quota (or the affinity set, whichever
    is smaller) is the honest core count."""
    share, why = os.cpu_count() or 1, "os.cpu_count()"
    try:
        aff = len(os.sched_getaffinity(0))
        if aff < share:
            share, why = aff, "sched_getaffinity"
    except (AttributeError, OSError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
            if quota < share:
                share, why = quota, "cgroup cpu.max quota"
    except (OSError, ValueError):
        pass
    return share, why


def cpu_baseline(cfg, batches, T, seconds):
    """The reference CPU path (oracle restatement: PyG TransformerConv semantics,
    Python-loop mean readout, loss, torch AdamW) on the host cores, bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import etpgt_ref as R

    from etpgt.data.synthetic import random_pe_table

    torch.manual_seed(42)
    ref = R.ref_create_graph_transformer_optimized(T, embedding_dim=cfg["D"], hidden_dim=cfg["D"], num_layers=2,
                                                   num_heads=cfg["H"], dropout=0.1, use_laplacian_pe=cfg["K"] > 0,
                                                   laplacian_k=max(cfg["K"], 1))
    if cfg["K"] > 0:
        ref.laplacian_pe._cached_pe = random_pe_table(T, cfg["K"])
    ref.train()
    opt = torch.optim.AdamW(ref.parameters(), lr=1e-3, weight_decay=1e-5)
    rbs = [R.ref_batch_from(b) for b in batches]
    threads, why = _cpu_share()
    torch.set_num_threads(threads)
    log(f"cpu baseline: {threads} threads ({why}; host reports {os.cpu_count()} CPUs)")
    for i in range(3):
        R.ref_train_step(ref, rbs[i % len(rbs)], opt, cfg["loss"])
    times = []
    t_end = time.perf_counter() + seconds
    i = 0
    while time.perf_counter() < t_end or len(times) < 5:
        t = time.perf_counter()
        R.ref_train_step(ref, rbs[i % len(rbs)], opt, cfg["loss"])
        times.append(time.perf_counter() - t)
        i += 1
    B = batches[0].num_graphs
    med = float(np.median(times))
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {
        "value": round(B / med, 1),
        "unit": "sessions/s",
        "cores": threads,
        "cores_source": why,
        "host_cpus": os.cpu_count(),
        "kind": "port",
        "sample": f"{len(times)} training steps of B={B} ({len(times)*B} sessions, median step {med*1e3:.2f} ms) "
                  f"on the same pre-staged batches; oracle/etpgt_ref.py restatement, torch CPU, {cpu_model}",
    }


if __name__ == "__main__":
    main()

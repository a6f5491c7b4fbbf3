#!/usr/bin/env python3
"""Counterpart of the reference's scripts/train/train_baseline.py on the MI355X path.

Same command line (reference train_baseline.py:27-85) and the same steps
(:123-290): seed, split info, train / val loaders, model factory, LapPE precompute on
the full graph (graph_transformer models), AdamW(lr, weight_decay), Trainer.train().
Differences, each deliberate:

* No Google Cloud Storage: the reference imports ``google.cloud.storage``
  unconditionally (:10).  ``--gcs-bucket`` is accepted and
  refused (cloud I/O is outside the hot-path scope).
* ``num_items``: the reference reads ``split_info["num_items"]`` (:145-149), a key the
  split script never writes.  It is used when present;
  otherwise the loaders' own table size (max item id + 1 over sessions and graph,
  dataloader.py:51-58) is used.
* ``--device-batches`` (added): batches built on the GPU inside the captured training
  step (``create_dataloader(device_builder=True)``), default on for CUDA runs of the
  graph-transformer models; ``off`` keeps the host DataLoader + collate_fn.
* GAT / GraphSAGE are outside the hot-path scope: ``--model gat|graphsage`` raises.
* Data parallel (added; the reference trains on one GPU): under ``torchrun`` /
  ``torch.distributed.run`` (WORLD_SIZE > 1) every process joins the default process
  group (RCCL; gloo with every rank on cuda:0 when GTR_SHARE_DEVICE=1), binds
  cuda:LOCAL_RANK, and trains on its share of each global batch of
  ``world * --batch-size`` sessions (``DeviceSessionLoader(rank, world)``) with gradients
  averaged and BatchNorm statistics synchronised across the ranks (SyncBN), i.e. like one
  GPU on the global batch.  Every rank evaluates the full validation set (the replicas
  are identical); rank 0 writes the outputs.  ``--shard-table on`` (added) keeps the item
  table and its AdamW moments row-sharded across the ranks instead of replicated
  (etpgt.train.sharded; bitwise the replicated step).  At the end the captured step graphs
  are released and the process group destroyed.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
from pathlib import Path

_PKG = Path(__file__).resolve().parents[2] / "gat-recommendation_amd"
if _PKG.is_dir() and str(_PKG) not in sys.path:
    sys.path.insert(0, str(_PKG))

import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402
import torch  # noqa: E402

from etpgt.data import Data  # noqa: E402
from etpgt.model import (  # noqa: E402
    create_gat,
    create_graph_transformer,
    create_graph_transformer_optimized,
    create_graphsage,
)
from etpgt.train.dataloader import create_dataloader  # noqa: E402
from etpgt.train.trainer import Trainer  # noqa: E402
from etpgt.utils.logging import get_logger  # noqa: E402
from etpgt.utils.seed import set_seed  # noqa: E402

logger = get_logger(__name__)


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="Train baseline models")
    p.add_argument("--model", type=str, required=True,
                   choices=["graphsage", "gat", "graph_transformer", "graph_transformer_optimized"], help="Model type")
    p.add_argument("--embedding-dim", type=int, default=256, help="Embedding dimension")
    p.add_argument("--hidden-dim", type=int, default=256, help="Hidden dimension")
    p.add_argument("--num-layers", type=int, default=3, help="Number of layers")
    p.add_argument("--num-heads", type=int, default=4, help="Number of attention heads")
    p.add_argument("--dropout", type=float, default=0.1, help="Dropout rate")
    p.add_argument("--readout-type", type=str, default="mean", choices=["mean", "max", "last", "attention"],
                   help="Session readout type")
    p.add_argument("--train-sessions", type=str, default="data/processed/train.csv", help="Training sessions")
    p.add_argument("--val-sessions", type=str, default="data/processed/val.csv", help="Validation sessions")
    p.add_argument("--graph-edges", type=str, default="data/processed/graph_edges.csv", help="Graph edges")
    p.add_argument("--batch-size", type=int, default=32, help="Batch size")
    p.add_argument("--num-negatives", type=int, default=5, help="Number of negative samples")
    p.add_argument("--max-session-length", type=int, default=50, help="Maximum session length")
    p.add_argument("--num-workers", type=int, default=4, help="Number of data workers")
    p.add_argument("--max-epochs", type=int, default=100, help="Maximum epochs")
    p.add_argument("--lr", type=float, default=0.001, help="Learning rate")
    p.add_argument("--weight-decay", type=float, default=1e-5, help="Weight decay")
    p.add_argument("--patience", type=int, default=10, help="Early stopping patience")
    p.add_argument("--eval-every", type=int, default=1, help="Evaluate every N epochs")
    p.add_argument("--output-dir", type=str, default="outputs", help="Output directory")
    p.add_argument("--gcs-bucket", type=str, default=None, help="GCS bucket for outputs (not supported)")
    p.add_argument("--seed", type=int, default=42, help="Random seed")
    p.add_argument("--device", type=str, default="cuda", help="Device (cuda/cpu)")
    p.add_argument("--device-batches", type=str, default="auto", choices=["auto", "on", "off"],
                   help="build batches on the GPU inside the training step (auto: on for CUDA graph transformers)")
    p.add_argument("--shard-table", type=str, default="auto", choices=["auto", "on", "off"],
                   help="data parallel: row-shard the item table and its AdamW moments across the ranks "
                        "(auto: GTR_SHARD_TABLE=1)")
    return p.parse_args(argv)


def init_distributed(args) -> tuple[int, int]:
    """Join the launcher's process group (one process per GPU); returns (rank, world)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return 0, 1
    import torch.distributed as dist

    if torch.device(args.device).type != "cuda":
        raise NotImplementedError("data-parallel training runs on the GPUs (one process per GPU)")
    share = os.environ.get("GTR_SHARE_DEVICE") == "1"  # rehearsal: every rank on cuda:0, gloo
    dev_index = 0 if share else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(dev_index)
    args.device = f"cuda:{dev_index}"
    if not dist.is_initialized():
        if share:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
    return dist.get_rank(), dist.get_world_size()


def main(argv=None):
    args = parse_args(argv)
    if args.gcs_bucket:
        raise NotImplementedError("GCS I/O (--gcs-bucket) is outside the MI355X hot-path scope; stage files locally")
    rank, world = init_distributed(args)
    set_seed(args.seed)
    logger.info("Training arguments:")
    logger.info(json.dumps(vars(args), indent=2))

    split_info_path = Path(args.train_sessions).parent / "split_info.json"
    split_info = {}
    if split_info_path.exists():
        with open(split_info_path) as f:
            split_info = json.load(f)

    gt = args.model in ("graph_transformer", "graph_transformer_optimized")
    on_gpu = torch.device(args.device).type == "cuda"
    dev_batches = args.device_batches == "on" or (args.device_batches == "auto" and gt and on_gpu)
    logger.info("Creating data loaders%s...", " (batches built on the GPU)" if dev_batches else "")
    kw = dict(graph_edges_path=args.graph_edges, batch_size=args.batch_size, num_negatives=args.num_negatives,
              max_session_length=args.max_session_length, num_workers=args.num_workers)
    if world > 1 and not dev_batches:
        raise NotImplementedError("data-parallel training builds its batches on the GPU (--device-batches on)")
    if dev_batches:
        kw.update(device_builder=True, device=args.device, seed=args.seed)
    train_loader = create_dataloader(sessions_path=args.train_sessions, shuffle=True, rank=rank, world=world, **kw)
    val_loader = create_dataloader(sessions_path=args.val_sessions, shuffle=False, **kw)  # full set on every rank
    if world > 1:
        logger.info(f"Data parallel: rank {rank} of {world}, global batch {world * args.batch_size} sessions")
    data_items = max(train_loader.dataset.num_items, val_loader.dataset.num_items)
    num_items = int(split_info.get("num_items", data_items))
    if num_items < data_items:
        raise ValueError(f"split_info num_items {num_items} < largest item id + 1 in the data ({data_items})")
    logger.info(f"Number of items: {num_items}")
    logger.info(f"Train batches: {len(train_loader)}")
    logger.info(f"Val batches: {len(val_loader)}")

    logger.info(f"Creating {args.model} model...")
    if args.model == "graphsage":
        model = create_graphsage(num_items=num_items, embedding_dim=args.embedding_dim, hidden_dim=args.hidden_dim,
                                 num_layers=args.num_layers, dropout=args.dropout, readout_type=args.readout_type)
    elif args.model == "gat":
        model = create_gat(num_items=num_items, embedding_dim=args.embedding_dim, hidden_dim=args.hidden_dim,
                           num_layers=args.num_layers, num_heads=args.num_heads, dropout=args.dropout,
                           readout_type=args.readout_type)
    else:
        factory = create_graph_transformer if args.model == "graph_transformer" else create_graph_transformer_optimized
        extra = {} if args.model == "graph_transformer" else dict(use_ffn=False, ffn_expansion=2)
        model = factory(num_items=num_items, embedding_dim=args.embedding_dim, hidden_dim=args.hidden_dim,
                        num_layers=args.num_layers, num_heads=args.num_heads, dropout=args.dropout,
                        readout_type=args.readout_type, use_laplacian_pe=True, **extra)
        logger.info("Precomputing Laplacian PE for the full graph...")
        graph_df = pd.read_csv(args.graph_edges)
        edge_index = torch.from_numpy(
            np.stack([graph_df["item_i"].to_numpy(), graph_df["item_j"].to_numpy()]).astype(np.int64))
        model.laplacian_pe.precompute(Data(edge_index=edge_index, num_nodes=num_items))
        logger.info("Laplacian PE precomputed successfully")

    num_params = sum(p.numel() for p in model.parameters() if p.requires_grad)
    logger.info(f"Model parameters: {num_params:,}")
    optimizer = torch.optim.AdamW(model.parameters(), lr=args.lr, weight_decay=args.weight_decay)
    output_dir = Path(args.output_dir) / args.model
    shard = None if args.shard_table == "auto" else args.shard_table == "on"
    trainer = Trainer(model=model, train_loader=train_loader, val_loader=val_loader, optimizer=optimizer,
                      device=args.device, output_dir=output_dir, max_epochs=args.max_epochs, patience=args.patience,
                      eval_every=args.eval_every, shard_table=shard)
    if world > 1 and trainer.shard_table:
        logger.info("Item table row-sharded across the ranks")
    logger.info("Starting training...")
    try:
        trainer.train()
    finally:
        # captured graphs hold RCCL collectives: released before the communicator goes
        trainer.close()
        if world > 1:
            import torch.distributed as dist

            if dist.is_initialized():
                dist.destroy_process_group()
    logger.info("Training complete!")
    logger.info(f"Best validation recall@10: {trainer.best_val_metric:.4f}")
    return trainer


if __name__ == "__main__":
    os.environ.setdefault("PYTHONUNBUFFERED", "1")
    main()

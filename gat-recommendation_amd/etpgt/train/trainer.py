"""Trainer — API of etpgt/train/trainer.py (reference, :23-252).

``train_epoch`` keeps the reference step semantics (trainer.py:80-133): forward,
reshape negatives to [B, n], loss (model.compute_loss = BPR by default, or the
custom ``loss_fn``), zero_grad, backward, optimizer.step.  When the model is a
GraphTransformer on the GPU and the optimizer is a single-group
``torch.optim.AdamW``/``Adam``, the whole step runs as the fused HIP step
(etpgt.train.fused, captured once into a hipGraph); otherwise the generic
autograd loop runs (HIP forward/backward kernels, torch optimizer).  The per-step
``loss.item()`` host sync of the reference (trainer.py:130) is replaced by a
device-side running sum read once per epoch; the returned average is the same.
"""

from __future__ import annotations

import json
import logging
import os
from pathlib import Path

import torch
import torch.nn as nn

from etpgt.utils.metrics import compute_ndcg_at_k, compute_recall_at_k

logger = logging.getLogger(__name__)


def _fused_loss_spec(loss_fn):
    if loss_fn is None:
        return ("bpr", 1.0, 0.7)
    kind = getattr(loss_fn, "kind", None)
    if kind == "bpr":
        return ("bpr", 1.0, 0.7)
    if kind in ("listwise", "sampled_softmax"):
        return ("listwise", float(loss_fn.temperature), 0.7)
    if kind == "dual":
        return ("dual", float(loss_fn.temperature), float(loss_fn.alpha))
    return None


class Trainer:
    def __init__(self, model: nn.Module, train_loader, val_loader, optimizer: torch.optim.Optimizer,
                 device: str = "cuda", output_dir: Path | str = "outputs", max_epochs: int = 100,
                 patience: int = 10, eval_every: int = 1, k_values: list[int] | None = None,
                 loss_fn: nn.Module | None = None, fused: bool | None = None, sync_bn: bool | None = None,
                 shard_table: bool | None = None):
        """Reference signature (trainer.py:23-67) plus three optional keywords: ``fused``
        (force / forbid the fused HIP step), ``sync_bn`` (data parallel: BatchNorm
        statistics over every rank's batch; default on when the default process group spans
        more than one rank, so P ranks train exactly like one GPU on the global batch) and
        ``shard_table`` (data parallel: the item table and its AdamW moments row-sharded
        across the ranks -- rank p owns rows r % P == p, rows and row gradients travel by
        all-to-all, etpgt.train.sharded -- instead of replicated on every rank; default
        off, ``GTR_SHARD_TABLE=1`` turns it on).  Results equal the replicated step bit for
        bit.  Under a process group only rank 0 writes checkpoints and history.json."""
        from etpgt.train.distributed import world_info

        self.rank, self.world = world_info()
        if sync_bn is None:
            # SyncBN covers the FFN variant at dim 64 / 128 with expansion 4 (gtr_ffn_fwd folds
            # the gathered rows); elsewhere its data-parallel step keeps per-rank statistics
            ffn_sync = (not getattr(model, "use_ffn", False)
                        or (getattr(model, "embedding_dim", 0) in (64, 128) and getattr(model, "ffn_expansion", 4) == 4))
            sync_bn = self.world > 1 and ffn_sync
        self.sync_bn = bool(sync_bn)
        if shard_table is None:
            shard_table = os.environ.get("GTR_SHARD_TABLE") == "1"
        self.shard_table = bool(shard_table) and self.world > 1
        self.model = model.to(device)
        self.train_loader = train_loader
        self.val_loader = val_loader
        self.optimizer = optimizer
        self.device = device
        self.output_dir = Path(output_dir)
        self.max_epochs = max_epochs
        self.patience = patience
        self.eval_every = eval_every
        self.k_values = k_values if k_values is not None else [10, 20]
        self.loss_fn = loss_fn
        self.output_dir.mkdir(parents=True, exist_ok=True)
        self.current_epoch = 0
        self.best_val_metric = 0.0
        self.patience_counter = 0
        self.history = {"train_loss": [], "val_metrics": []}
        self._fused_flag = fused
        self._fused = None
        # device-built epochs: full batches per multi-step hipGraph (1: one graph per batch)
        self.steps_per_graph = max(1, int(os.environ.get("GTR_TRAINER_STEPS_PER_GRAPH", "32")))
        self._chunk_graph = None

    # ------------------------------------------------------------------ fused path
    def _fused_step(self):
        if self._fused is not None:
            return self._fused
        if self._fused_flag is False:
            return None
        from etpgt.model.graph_transformer import GraphTransformer

        spec = _fused_loss_spec(self.loss_fn)
        opt = self.optimizer
        ok = (isinstance(self.model, GraphTransformer) and torch.device(self.device).type == "cuda"
              and spec is not None and type(opt) in (torch.optim.AdamW, torch.optim.Adam)
              and len(opt.param_groups) == 1 and not opt.state
              and not opt.param_groups[0].get("amsgrad", False)
              and not opt.param_groups[0].get("maximize", False))
        if ok:
            names = {id(p) for p in opt.param_groups[0]["params"]}
            ok = all(id(p) in names for p in self.model.parameters() if p.requires_grad)
        if not ok:
            if self._fused_flag:
                raise RuntimeError("fused training step requested but the model/optimizer/loss is unsupported")
            return None
        from etpgt.train.fused import FusedTrainStep

        g = opt.param_groups[0]
        self._fused = FusedTrainStep(self.model, lr=g["lr"], betas=g["betas"], eps=g["eps"],
                                     weight_decay=g["weight_decay"], decoupled=type(opt) is torch.optim.AdamW,
                                     loss=spec[0], temperature=spec[1], alpha=spec[2],
                                     sync_bn=self.sync_bn and self.world > 1, shard_table=self.shard_table)
        return self._fused

    def _sync_table(self):
        """Row-sharded table: bring the ranks' shards into the model's item table before
        anything reads the model (evaluation, checkpoints).  Collective: every rank calls it
        at the same point of ``train``."""
        if self._fused is not None and self._fused.shard_state is not None:
            self._fused.sync_table()

    def close(self):
        """Release the captured step graphs (they hold RCCL collectives under a process
        group): call before ``dist.destroy_process_group()``, whose communicator teardown
        waits for every graph that captured one of its collectives to be destroyed."""
        self._chunk_graph = None
        if self._fused is not None:
            self._fused.close()

    def _sync_optimizer_state(self):
        if self._fused is not None:
            self._fused.export_optimizer_state(self.optimizer)

    # ------------------------------------------------------------------ loops
    def _train_epoch_device_batches(self, fused) -> float:
        """One epoch of a ``DeviceSessionLoader`` through the fused step: the batch build
        runs inside the captured step (no host work per batch).  The full batches run in
        chunks of ``steps_per_graph`` consecutive steps captured as ONE hipGraph
        (``FusedTrainStep.capture_steps_built``: each step's build advances the device
        cursor), so the queue runs batch after batch without a host round trip between
        them; the batches that do not fill a chunk launch one step graph each, and the
        partial last batch is launched eagerly.  The epoch's loss is the tail's device-side
        running sum (``gtr_tail.loss_acc``), read once: the mean over batches of the
        per-batch losses, as trainer.py:130-133 computes it."""
        loader = self.train_loader
        loader.start_epoch()
        sizes = loader.batch_sizes()
        bld = loader.builder
        # the last, partial batch of rank r starts at i*P*B + r*b, off the stride grid the
        # full batches follow: plan its window explicitly, before the ranks agree on caps
        full = sum(1 for b in sizes if b == loader.batch_size)
        extra = [(loader.batch_start(i), b) for i, b in enumerate(sizes) if b != loader.batch_size]
        if fused.builder is not bld:
            fused.attach_builder(bld, num_batches=max(full, 1), extra=extra)
        else:  # capacities for this epoch's order (rebinds only if they grew; agreed over ranks)
            fused.refresh_builder_caps(max(full, 1), extra=extra)
        fused.loss_acc.zero_()
        K = self.steps_per_graph
        i = 0
        if full > 0:
            fused.run()  # first full batch: eager warm-up + per-step capture on a fresh binding
            i = 1
        while K > 1 and full - i >= K:
            h = self._chunk_graph
            if h is None or h["n"] != K or h.get("step") is not fused or fused.stale_reason(h) is not None:
                # captured once per binding (and again when the lazy / sharded per-step
                # constants must grow); every rank counts the same steps, so every rank
                # reaches this point together
                self._chunk_graph = h = None  # a stale graph is released before the next capture
                h = fused.capture_steps_built(K, reserve=full)
                if h is None:
                    break  # not capturable whole (gloo): one step graph per batch
                h["step"] = fused
                self._chunk_graph = h
            fused.run_steps(h)
            i += K
        for _ in range(i, full):
            fused.run()  # the captured build advances the cursor by the global batch
        for j, b in enumerate(sizes):
            if b != loader.batch_size:  # last, partial batch: this rank's even share
                bld.seek(loader.batch_start(j))
                fused.run_partial(b)
        bld.check_status(fused.group)  # collective under a process group: every rank raises together
        return float(fused.loss_acc.item()) / max(len(sizes), 1)

    def train_epoch(self) -> float:
        self.model.train()
        fused = self._fused_step()
        if fused is None and self.world > 1:
            # the generic autograd loop averages nothing across ranks: each rank would train
            # its own replica on its own shard of the data and the replicas would drift apart
            raise RuntimeError(f"data-parallel training ({self.world} ranks) needs the fused HIP step; this "
                               "model / optimizer / loss takes the single-process autograd loop (the FFN "
                               "variant, fused=False, or an unsupported optimizer or loss)")
        from etpgt.train.dataloader import DeviceSessionLoader

        if fused is not None and isinstance(self.train_loader, DeviceSessionLoader):
            return self._train_epoch_device_batches(fused)
        total = torch.zeros((), dtype=torch.float64, device=self.device)
        num_batches = 0
        for batch in self.train_loader:
            batch = batch.to(self.device)
            if fused is not None:
                total += fused(batch).double()
                num_batches += 1
                continue
            session_embeddings = self.model(batch)
            batch_size = batch.target_item.shape[0]
            num_negatives = batch.negative_items.shape[0] // batch_size if batch.negative_items.dim() == 1 \
                else batch.negative_items.shape[1]
            negative_items = batch.negative_items.reshape(batch_size, num_negatives)
            if self.loss_fn is not None:
                out = self.loss_fn(session_embeddings, batch.target_item, negative_items, self.model.item_embedding)
                loss = out[0] if isinstance(out, tuple) else out
            else:
                loss = self.model.compute_loss(session_embeddings, batch.target_item, negative_items)
            self.optimizer.zero_grad()
            loss.backward()
            self.optimizer.step()
            total += loss.detach().double()
            num_batches += 1
        return float(total.item()) / max(num_batches, 1)

    @torch.no_grad()
    def evaluate(self) -> dict:
        self._sync_table()
        self.model.eval()
        preds, targets = [], []
        for batch in self.val_loader:
            batch = batch.to(self.device)
            se = self.model(batch)
            preds.append(self.model.predict(se, k=max(self.k_values)).cpu())
            targets.append(batch.target_item.cpu())
        preds = torch.cat(preds, dim=0)
        targets = torch.cat(targets, dim=0)
        metrics = {}
        for k in self.k_values:
            metrics[f"recall@{k}"] = compute_recall_at_k(preds[:, :k], targets, k=k)
            metrics[f"ndcg@{k}"] = compute_ndcg_at_k(preds[:, :k], targets, k=k)
        return metrics

    def save_checkpoint(self, is_best: bool = False) -> None:
        self._sync_optimizer_state()
        if self.rank != 0:  # replicas are identical: one writer
            return
        ckpt = {
            "epoch": self.current_epoch,
            "model_state_dict": self.model.state_dict(),
            "optimizer_state_dict": self.optimizer.state_dict(),
            "best_val_metric": self.best_val_metric,
            "history": self.history,
        }
        torch.save(ckpt, self.output_dir / "checkpoint_latest.pt")
        if is_best:
            torch.save(ckpt, self.output_dir / "checkpoint_best.pt")

    def train(self) -> dict:
        for epoch in range(self.max_epochs):
            self.current_epoch = epoch
            train_loss = self.train_epoch()
            self.history["train_loss"].append(train_loss)
            logger.info(f"Epoch {epoch}: train_loss={train_loss:.4f}")
            if (epoch + 1) % self.eval_every == 0:
                val = self.evaluate()
                self.history["val_metrics"].append(val)
                metric = val[f"recall@{self.k_values[0]}"]
                is_best = metric > self.best_val_metric
                if is_best:
                    self.best_val_metric = metric
                    self.patience_counter = 0
                else:
                    self.patience_counter += 1
                self.save_checkpoint(is_best=is_best)
                if self.patience_counter >= self.patience:
                    logger.info(f"Early stopping at epoch {epoch}")
                    break
        self._sync_optimizer_state()
        if self.rank == 0:
            with open(self.output_dir / "history.json", "w") as f:
                json.dump(self.history, f, indent=2)
        return self.history

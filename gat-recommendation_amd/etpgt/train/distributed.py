"""Data-parallel training over one process per GPU (torch.distributed, RCCL over xGMI).

Semantics (DistributedDataParallel with BatchNorm statistics local to each rank):
every rank trains on its own batch of sessions (trainer.py:80-133 per rank), the
gradients are averaged over the ranks, and every rank applies the same AdamW update,
so the replicas stay identical without ever exchanging parameters.

Exchange, once per step — one RCCL all-gather of a fixed-size pack per rank
(``gtr_dp_layout`` in include/gtr.h):

    [0, F)                  summed small-parameter gradient (engine.ParamLayout order)
    [F]                     local loss
    [keys_off, +m_cap)      sorted item-table contribution keys (int32 bits, sentinel T)
    [rows_off, +m_cap*D)    summed table-gradient row at each key's first slot

The item table is never reduced densely: only the rows a rank touched travel
(m_cap*D floats, ~88 KB per rank at the C2 shape against 21 MB for the table).
``gtr_dp_tail`` then stamps the union of touched rows, averages each touched row
over the ranks that hold it (lowest rank owns the row, rank-order sum:
deterministic) and runs the untouched-row / small-parameter AdamW like the
single-GPU step tail.  Fixed sizes keep both halves of the step graph-capturable.

The pure-Python ``pack_reference`` / ``combine_reference`` restate the same
protocol on CPU tensors; the gloo tests (tests/test_distributed.py) drive them
with the oracle's autograd gradients.
"""

from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist

from etpgt.backend import _lib as L


def _al4(n: int) -> int:
    return (int(n) + 3) & ~3


@dataclass(frozen=True)
class DpLayout:
    flat_total: int
    m_cap: int
    dim: int
    world: int

    @property
    def loss_off(self) -> int:
        return self.flat_total

    @property
    def keys_off(self) -> int:
        return self.flat_total + 1

    @property
    def rows_off(self) -> int:
        return _al4(self.keys_off + self.m_cap)

    @property
    def words(self) -> int:
        return _al4(self.rows_off + self.m_cap * self.dim)

    def struct(self) -> L.GtrDpLayout:
        s = L.GtrDpLayout()
        s.flat_total, s.loss_off, s.keys_off = self.flat_total, self.loss_off, self.keys_off
        s.rows_off, s.words, s.m_cap, s.world = self.rows_off, self.words, self.m_cap, self.world
        return s


def world_info(group=None) -> tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def all_gather_packs(recv: torch.Tensor, pack: torch.Tensor, group=None) -> None:
    """recv[world, words] <- every rank's pack (one collective).  RCCL on device
    tensors; a gloo group (CPU transport: the tests, incl. several ranks sharing one
    GPU) round-trips device tensors through host memory.  Without an initialised
    process group the single rank's pack is copied."""
    if not (dist.is_available() and dist.is_initialized()):
        if recv.shape[0] != 1:
            raise RuntimeError("data-parallel exchange without a process group needs world size 1")
        recv[0].copy_(pack)
        return
    backend = dist.get_backend(group)
    if backend == "gloo":
        host = torch.empty(recv.numel(), dtype=pack.dtype)
        dist.all_gather_into_tensor(host, pack.detach().cpu().reshape(-1), group=group)
        recv.copy_(host.view_as(recv))
    else:
        dist.all_gather_into_tensor(recv.view(-1), pack.reshape(-1), group=group)


def all_to_all(recv: torch.Tensor, send: torch.Tensor, group=None) -> None:
    """recv[p] <- rank p's send[my rank] for equal blocks along dim 0 (one collective).
    RCCL on device tensors; a gloo group round-trips through host memory; without an
    initialised process group (one rank) the block is copied."""
    if not (dist.is_available() and dist.is_initialized()):
        recv.copy_(send)
        return
    if dist.get_backend(group) == "gloo":
        host = torch.empty(send.shape, dtype=send.dtype)
        dist.all_to_all_single(host, send.detach().cpu(), group=group)
        recv.copy_(host)
    else:
        dist.all_to_all_single(recv, send, group=group)


class _Done:
    def wait(self):
        return None


def start_all_gather(out: torch.Tensor, inp: torch.Tensor, group=None):
    """Asynchronous all-gather (out[world, n] <- every rank's inp[n]) on the collective
    stream; ``.wait()`` makes the current stream wait for it (RCCL).  gloo (CPU
    transport) completes it before returning."""
    if not (dist.is_available() and dist.is_initialized()):
        out[0].copy_(inp)
        return _Done()
    if dist.get_backend(group) == "gloo":
        host = torch.empty(out.numel(), dtype=inp.dtype)
        dist.all_gather_into_tensor(host, inp.detach().cpu().reshape(-1), group=group)
        out.copy_(host.view_as(out))
        return _Done()
    return dist.all_gather_into_tensor(out.view(-1), inp.reshape(-1), group=group, async_op=True)


# ---------------------------------------------------------------------------------
# CPU restatement of the protocol (tests; mirrors gtr_dp_pack / gtr_dp_tail)
# ---------------------------------------------------------------------------------
def pack_reference(lay: DpLayout, flat_grad: torch.Tensor, loss: float, table_grad: torch.Tensor,
                   touched_keys: torch.Tensor, num_items: int) -> torch.Tensor:
    """One rank's pack from dense CPU gradients.  touched_keys: the rank's contribution
    keys (any order, duplicates allowed); table_grad: dense [T, D] gradient."""
    pack = torch.zeros(lay.words, dtype=torch.float32)
    pack[: lay.flat_total] = flat_grad
    pack[lay.loss_off] = float(loss)
    keys = torch.full((lay.m_cap,), num_items, dtype=torch.int32)
    k = torch.sort(touched_keys.to(torch.int32)).values
    keys[: k.numel()] = k
    pack[lay.keys_off: lay.keys_off + lay.m_cap] = keys.view(torch.float32)
    rows = pack[lay.rows_off: lay.rows_off + lay.m_cap * lay.dim].view(lay.m_cap, lay.dim)
    for i in range(lay.m_cap):
        key = int(keys[i])
        if 0 < key < num_items and (i == 0 or int(keys[i - 1]) != key):
            rows[i] = table_grad[key]
    return pack


def combine_reference(lay: DpLayout, recv: torch.Tensor, num_items: int):
    """Rank-averaged gradients from the gathered packs: (flat_grad, {row: grad}, loss)."""
    W = lay.world
    flat = recv[:, : lay.flat_total].sum(0) / W
    loss = float(recv[:, lay.loss_off].sum()) / W
    rows: dict[int, torch.Tensor] = {}
    for r in range(W):
        keys = recv[r, lay.keys_off: lay.keys_off + lay.m_cap].contiguous().view(torch.int32)
        data = recv[r, lay.rows_off: lay.rows_off + lay.m_cap * lay.dim].view(lay.m_cap, lay.dim)
        for i in range(lay.m_cap):
            key = int(keys[i])
            if 0 < key < num_items and (i == 0 or int(keys[i - 1]) != key):
                rows[key] = rows.get(key, torch.zeros(lay.dim)) + data[i]
    return flat, {k: v / W for k, v in rows.items()}, loss


# ---------------------------------------------------------------------------------
# device path
# ---------------------------------------------------------------------------------
class DpExchange:
    """Device buffers and launches of the data-parallel half of a fused step."""

    def __init__(self, step, group=None):
        self.step = step
        self.group = group
        self.rank, self.world = world_info(group)
        eng = step.eng
        caps = step.caps
        m_cap = caps.n_cap + caps.b_cap * (1 + caps.n_neg)
        self.lay = DpLayout(eng.flat.layout.total, m_cap, eng.D, self.world)
        self.lay_s = self.lay.struct()
        dev = step.dev
        # one rank: the gathered packs ARE the rank's pack (no copy, no collective, and the
        # step is one graph); GTR_DP_NOALIAS=1 keeps the RCCL all-gather (a one-rank rehearsal)
        self.alias = self.world == 1 and os.environ.get("GTR_DP_NOALIAS") != "1"
        self.recv = torch.zeros(self.world, self.lay.words, dtype=torch.float32, device=dev)
        self.pack = self.recv[0] if self.alias else torch.zeros(self.lay.words, dtype=torch.float32, device=dev)
        self.slot = torch.full((eng.T, self.world, 2), -1, dtype=torch.int32, device=dev)

    def launch_pack(self, bs, stream_handle):
        st = self.step
        L.check(L.lib().gtr_dp_pack(C.byref(bs), st.eng.T, st.eng.D, C.byref(st.tail), st.segs, st.nseg,
                                    C.byref(self.lay_s), self.pack.data_ptr(), stream_handle), "dp_pack")

    def exchange(self):
        if not self.alias:
            all_gather_packs(self.recv, self.pack, self.group)

    def launch_tail(self, bs, stream_handle):
        st = self.step
        L.check(L.lib().gtr_dp_tail(C.byref(bs), st.eng.T, st.eng.D, C.byref(st.tail), C.byref(self.lay_s),
                                    self.recv.data_ptr(), self.slot.data_ptr(), C.byref(st.adam), stream_handle),
                "dp_tail")

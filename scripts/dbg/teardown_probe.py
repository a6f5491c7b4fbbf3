"""RCCL teardown after graph-captured collectives (debug probe, one rank).

usage: python teardown_probe.py <keep|del|reset|nocapture>
  keep      the captured graph is still alive at destroy_process_group()
  del       the graph is dropped (del + gc) and the device synchronized first
  reset     CUDAGraph.reset() first, the object kept
  nocapture the collective runs eagerly only (control)
Prints 'teardown ok' once destroy_process_group() has returned.
"""
import gc
import os
import sys
import time

import torch
import torch.distributed as dist

mode = sys.argv[1]
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29541")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
torch.cuda.set_device(0)
a = torch.arange(1024, device="cuda", dtype=torch.float32)
b = torch.empty_like(a)
dist.all_to_all_single(b, a)
torch.cuda.synchronize()
gr = None
if mode != "nocapture":
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        dist.all_to_all_single(b, a)
    a.add_(1)
    gr.replay()
    torch.cuda.synchronize()
    print(mode, "replay ok", bool(torch.equal(a, b)), flush=True)
if mode == "del":
    del gr
    gc.collect()
    torch.cuda.synchronize()
elif mode == "reset":
    gr.reset()
    torch.cuda.synchronize()
t0 = time.time()
dist.destroy_process_group()
print(mode, f"teardown ok in {time.time() - t0:.2f} s", flush=True)

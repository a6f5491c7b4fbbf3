"""Which RCCL all-to-all forms survive hipGraph capture at world 1 (debug probe)."""
import os, sys
import torch, torch.distributed as dist

mode = sys.argv[1]
os.environ.setdefault("MASTER_ADDR", "127.0.0.1"); os.environ.setdefault("MASTER_PORT", "29533")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
torch.cuda.set_device(0)
g = dist.new_group([0]) if "side" in mode else None
comm = None
if "raw" in mode:
    import ctypes
    lib = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so"))
    uid = ctypes.create_string_buffer(128)
    assert lib.ncclGetUniqueId(uid) == 0
    comm = ctypes.c_void_p()
    class U(ctypes.Structure):
        _fields_ = [("b", ctypes.c_char * 128)]
    u = U(); ctypes.memmove(ctypes.addressof(u), uid, 128)
    assert lib.ncclCommInitRank(ctypes.byref(comm), 1, u, 0) == 0
    lib.ncclAllToAll.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    def raw(b, a):
        st = torch.cuda.current_stream().cuda_stream
        r = lib.ncclAllToAll(a.data_ptr(), b.data_ptr(), a.numel(), 7, comm, st)
        assert r == 0, r
a = torch.arange(1024, device="cuda", dtype=torch.float32); b = torch.empty_like(a)
SIDE = torch.cuda.Stream()
def body():
    if mode == "raw":
        raw(b, a)
    elif mode == "raw_fork":
        s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            raw(b, a)
        c = a * 2
        torch.cuda.current_stream().wait_stream(s)
    elif mode == "fork_only":
        s = SIDE; s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            b.copy_(a)
        c = a * 2
        torch.cuda.current_stream().wait_stream(s)
    elif mode == "raw_fork2":
        s = SIDE; s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            raw(b, a)
        c = a * 2
        torch.cuda.current_stream().wait_stream(s)
    elif mode == "inv":
        s = SIDE; s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            c = a * 2
        dist.all_to_all_single(b, a, group=g)
        torch.cuda.current_stream().wait_stream(s)
    elif "async" in mode:
        w = dist.all_to_all_single(b, a, group=g, async_op=True)
        c = a * 2
        w.wait()
    elif "stream" in mode:
        s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            dist.all_to_all_single(b, a, group=g)
        torch.cuda.current_stream().wait_stream(s)
    else:
        dist.all_to_all_single(b, a, group=g)
body(); torch.cuda.synchronize()
gr = torch.cuda.CUDAGraph()
with torch.cuda.graph(gr):
    body()
a.add_(1); gr.replay(); torch.cuda.synchronize()
print(mode, "ok", bool(torch.equal(a, b)), flush=True)
dist.destroy_process_group()

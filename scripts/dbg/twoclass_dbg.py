"""Debug: the two-class row-sharded step over RCCL at world 1 (side stream + side
communicator), step by step with prints."""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gat-recommendation_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29611", GTR_GRAPH_COLL=os.environ.get("GTR_GRAPH_COLL", "1"))
from gpu_helpers import batches, make_pair, small_data  # noqa: E402

from etpgt.data.batch import Caps  # noqa: E402
from etpgt.train.fused import FusedTrainStep  # noqa: E402

torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
print("pg ok", flush=True)
data = small_data()
T = data.table_rows
m1, _ = make_pair(T, 64, 2, K=0, seed=35)
m2 = copy.deepcopy(m1)
m1.train(); m2.train()
bl = batches(data, 16, 5, 3, seed=36)
caps = Caps(max(b.num_nodes for b in bl), 16, max(b.num_edges for b in bl), 5)
kw = dict(lr=1e-2, weight_decay=1e-2, loss="bpr", shard_table=True, sync_bn=True, caps=caps)
f1 = FusedTrainStep(m1, **kw)
print("f1 ok", flush=True)
os.environ.update(GTR_SHARD_SPLIT="1", GTR_SHARD_NOALIAS=os.environ.get("NOALIAS", "1"))
f2 = FusedTrainStep(m2, **kw)
print("f2 ok", f2.shard.cap, f2.shard.cap_s, f2.shard.can_overlap, f2.shard.alias, flush=True)
st1 = [torch.from_numpy(b.packed(f1.caps)[1]).cuda() for b in bl]
st2 = [torch.from_numpy(b.packed(f2.caps)[1]).cuda() for b in bl]
for i in range(3):
    f1.load_blob(st1[i]); l1 = float(f1.run())
    print("f1 step", i, l1, flush=True)
    f2.load_blob(st2[i]); l2 = float(f2.run())
    print("f2 step", i, l2, flush=True)
f1.sync_table(); f2.sync_table()
print("same", all(torch.equal(a, b) for a, b in zip(m1.parameters(), m2.parameters())), flush=True)
dist.destroy_process_group()

import copy, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (os.path.join(ROOT, "gat-recommendation_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)
import torch
from gpu_helpers import batches, make_pair, small_data
from etpgt.train.fused import FusedTrainStep
data = small_data(); T = data.table_rows
m1, _ = make_pair(T, 64, 2, K=0, seed=21); m2 = copy.deepcopy(m1); m1.train(); m2.train()
f1 = FusedTrainStep(m1, lr=1e-2, weight_decay=1e-2, loss="bpr")
f2 = FusedTrainStep(m2, lr=1e-2, weight_decay=1e-2, loss="bpr", data_parallel=True, use_graph=len(sys.argv) > 1)
for s, sb in enumerate(batches(data, 16, 5, 3, seed=22)):
    l1 = float(f1(sb.to("cuda"))); l2 = float(f2(sb.to("cuda")))
    d = (m1.item_embedding.weight - m2.item_embedding.weight).abs()
    rows = torch.nonzero(d.max(1).values > 0).flatten().tolist()
    touched = set(sb.x.tolist()) | set(sb.target_item.tolist()) | set(sb.negative_items.tolist())
    print("step", s, l1, l2, "maxdiff", float(d.max()), "rows", rows[:10], len(rows), "touched?", [r in touched for r in rows[:10]])
    for n, p in m1.named_parameters():
        q = dict(m2.named_parameters())[n]
        md = float((p - q).abs().max())
        if md > 0: print("  ", n, md)

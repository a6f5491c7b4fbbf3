"""Config C1 (BASELINE.json configs[0]): the reference's run_full_pipeline.py quick path
— 100 synthetic sessions over a 1k-item catalogue (the reference generator's own output,
pinned by tests/golden/c1_data.npz), the 16-session bidirectional batch,
graph_transformer_optimized (d=64, 2 heads, 2 layers, no LapPE), listwise loss,
Adam(1e-3), 3 epochs — on the HIP model against the same plumbing on the oracle.

Value-level parity runs with dropout 0 (the HIP dropout stream cannot reproduce the
CPU generator); the reference's dropout 0.1 run is checked for PASS / finite losses."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - collected only on the GPU box
    pytest.skip("no GPU", allow_module_level=True)

import etpgt_ref as R  # noqa: E402
from gpu_helpers import OracleTrio  # noqa: E402

from etpgt.model import create_graph_transformer_optimized  # noqa: E402
from etpgt import pipeline as P  # noqa: E402

CFG = {"embedding_dim": 64, "hidden_dim": 64, "num_layers": 2, "num_heads": 2, "use_laplacian_pe": False}


def _c1_batch():
    """The reference's own C1 data (scripts/data 00 -> 02 -> 04, pinned by
    tests/golden/c1_data.npz) -> run_full_pipeline.py's 16-session batch."""
    from dropin_helpers import c1_inputs

    _, _, _, (sub, g) = c1_inputs()
    return P.create_batch_from_sessions(sub, g, batch_size=16, num_negatives=5)


def test_c1_pipeline_matches_oracle():
    batch, T = _c1_batch()
    cfg = {**CFG, "num_items": T, "dropout": 0.0}
    torch.manual_seed(0)
    res = P.test_model_with_real_data("GraphTransformer (optimized, no FFN)", create_graph_transformer_optimized,
                                      cfg, batch, num_epochs=3, device="cuda")
    assert res["status"] == "PASS", res
    # oracle: same init (same seed), same batch, same loop
    torch.manual_seed(0)
    init = create_graph_transformer_optimized(**cfg)
    ref = R.ref_create_graph_transformer_optimized(**cfg)
    ref.load_state_dict(init.state_dict())
    assert sum(p.numel() for p in ref.parameters()) == res["param_count"]
    rb = R.ref_batch_from(batch)
    trio = OracleTrio(ref, lambda ps: torch.optim.Adam(ps, lr=0.001))

    def epoch(mod, opt):
        mod.train()
        opt.zero_grad()
        se = mod(rb)
        loss = R.ref_loss("listwise", se, rb.target_item, rb.negative_items.view(se.shape[0], -1), mod.item_embedding)
        loss.backward()
        opt.step()
        return float(loss)

    rl = [trio.step(epoch) for _ in range(3)]
    np.testing.assert_allclose(res["losses"], rl, rtol=1e-3)
    # every trained parameter ELEMENTWISE (gpu_helpers.close_trained)
    m = res["model_obj"]
    trio.compare({n: p.detach().cpu() for n, p in m.named_parameters()}, lr=1e-3)


def test_c1_pipeline_reference_config_runs():
    """The reference's own settings (dropout 0.1): PASS, finite, decreasing loss."""
    batch, T = _c1_batch()
    res = P.test_model_with_real_data("GraphTransformer (optimized, no FFN)", create_graph_transformer_optimized,
                                    {**CFG, "num_items": T, "dropout": 0.1}, batch, num_epochs=3, device="cuda")
    assert res["status"] == "PASS", res
    assert all(np.isfinite(res["losses"]))
    assert res["losses"][-1] < res["losses"][0]

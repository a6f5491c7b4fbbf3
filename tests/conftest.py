"""Test configuration: package path, the `gpu` marker, shared fixtures."""

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gat-recommendation_amd")
for p in (PKG, ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and libgtr_hip.so")
    if "GTR_PARITY_AUDIT" not in os.environ:  # one audit file per run; rank processes inherit it
        import tempfile

        fd, path = tempfile.mkstemp(prefix="gtr_parity_audit_", suffix=".jsonl")
        os.close(fd)
        os.environ["GTR_PARITY_AUDIT"] = path


def pytest_terminal_summary(terminalreporter):
    """The elementwise bar's audit (gpu_helpers.close_trained): trained tensors checked,
    elements, and how many passed only through the tensor-wide fp32-noise fallback."""
    import json

    path = os.environ.get("GTR_PARITY_AUDIT")
    if not path or not os.path.exists(path):
        return
    with open(path) as f:
        recs = [json.loads(ln) for ln in f if ln.strip()]
    if not recs:
        return
    tr = terminalreporter
    tr.section("elementwise parity audit (close_trained)")
    tr.write_line(f"{len(recs)} trained tensors, {sum(r['elements'] for r in recs)} elements checked, "
                  f"{sum(r['fallback'] for r in recs)} accepted only through the fp32-noise fallback, "
                  f"{sum(r['bad'] for r in recs)} mismatches, "
                  f"{sum(r['noise_floor_elements'] for r in recs)} noise-floor elements (bounded by 2 lr/step)")
    for r in recs:
        if r["fallback"] or r["bad"]:
            tr.write_line(f"  {r['name']}: {r['fallback']} fallback, {r['bad']} bad of {r['elements']}")


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")

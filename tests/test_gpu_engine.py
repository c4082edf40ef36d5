"""End-to-end rounds on the GPU for every model family: the engine picks the native trainer
(fused kernel for TransformerModel, graph-replayed layer programs for CNN/RNN/HAR) and the native
eval forward; fedavg and hyper modes."""
import os

import pytest

from attackfl_amd.config import from_dict
from attackfl_amd.fl.engine import FLEngine

pytestmark = pytest.mark.gpu


def _run(tmp_path, model, data, mode, clients=4, rounds=2):
    d = {
        "server": {"num-round": rounds, "clients": clients, "mode": mode, "model": model, "data-name": data,
                   "data-distribution": {"num-data-range": [300, 500] if data == "ICU" else [40, 60]}},
        "learning": {"epoch": 2, "batch-size": 128 if data == "ICU" else 16},
        "data": {"synthetic": True, "train-size": 4000, "test-size": 1000, "har-train-size": 256,
                 "har-test-size": 64},
        "engine": {"checkpoint-dir": str(tmp_path), "trainer": "auto"},
        "log_path": str(tmp_path),
    }
    eng = FLEngine(from_dict(d), device="cuda", verbose=False)
    hist = eng.run()
    kind = eng.trainer.kind
    eng.close()
    return hist, kind


@pytest.mark.parametrize("model,data,kind", [("CNNModel", "ICU", "graph"), ("RNNModel", "ICU", "fused"),
                                             ("TransformerModel", "ICU", "fused"),
                                             ("TransformerClassifier", "HAR", "graph")])
@pytest.mark.parametrize("mode", ["fedavg", "hyper"])
def test_engine_rounds_native(gpu, tmp_path, model, data, kind, mode):
    if data == "HAR" and mode == "hyper":
        pytest.skip("hyper validation is ICU-only in the reference (test_hyper)")
    hist, got_kind = _run(tmp_path, model, data, mode)
    assert got_kind == kind
    assert sum(r["ok"] for r in hist) == 2
    assert all(0.0 <= r["metric"] <= 1.0 for r in hist)
    assert os.path.exists(os.path.join(tmp_path, "app.log"))

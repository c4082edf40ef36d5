import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
os.environ.setdefault("ATTACKFL_QUIET", "1")

if os.environ.get("PYTEST_XDIST_WORKER"):  # pytest -n: split the cores instead of oversubscribing them
    import torch

    _n = int(os.environ.get("PYTEST_XDIST_WORKER_COUNT", "1"))
    torch.set_num_threads(max(1, (os.cpu_count() or 1) // max(1, _n)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built native extension")


@pytest.fixture
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from attackfl_amd import ops

    ops.native()  # fail loudly if the extension is missing on a GPU box
    return torch.device("cuda", 0)

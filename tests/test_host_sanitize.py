"""Host-side sanitizer coverage (the reference has none).

``csrc/host/host_check.hip`` runs the integer math that the GPU kernels share with their Python
oracles (the Feistel visit plans of ``csrc/kernels/plan.hip`` and the dropout hash of
``csrc/common.h``) on the CPU, built with AddressSanitizer + UndefinedBehaviorSanitizer on the host
half.  These tests build it with hipcc (a CPU-only cross compile), run its self-test, and compare
its output bit-for-bit with ``attackfl_amd/fl/trainers.py`` / ``attackfl_amd/ops/masks.py``.  GPU
ASan / XNACK runs are not available on this pool, so device code is covered by the GPU numerics
tests instead.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

from attackfl_amd.fl import trainers
from attackfl_amd.ops import masks

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0", UBSAN_OPTIONS="print_stacktrace=1")

pytestmark = pytest.mark.skipif(not os.path.exists(HIPCC) or shutil.which("nm") is None,
                                reason="hipcc / nm not available")


@pytest.fixture(scope="module")
def host_check(tmp_path_factory):
    out = tmp_path_factory.mktemp("host")
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "host_sanitize.sh"), str(out)], env=ENV,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "selftest ok" in r.stdout
    exe = str(out / "host_check")
    syms = subprocess.run(["nm", exe], capture_output=True, text=True).stdout
    assert "__asan_init" in syms and "__ubsan_handle" in syms, "sanitizer runtime not linked"
    return exe


def _run(exe, *args):
    r = subprocess.run([exe, *map(str, args)], env=ENV, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr
    return r.stdout


def test_plan_matches_python_mirror(host_check):
    n_train, epochs = 20011, 3
    clients = [(12345, 1), (2**64 - 1, 4096), (987654321987, 12000), (7, 20011)]
    out = _run(host_check, "plan", n_train, epochs, *[f"{s}:{n}" for s, n in clients]).splitlines()
    assert len(out) == len(clients) * epochs
    ref = trainers._feistel_plan(n_train, [n for _, n in clients], epochs, [s for s, _ in clients], "cpu")
    for c, (_, nd) in enumerate(clients):
        for e in range(epochs):
            got = np.array(out[c * epochs + e].split(), dtype=np.int64)
            np.testing.assert_array_equal(got, ref.order[c, e, :nd].numpy())


@pytest.mark.parametrize("p", [0.1, 0.2, 0.5])
def test_dropout_mask_matches_python_mirror(host_check, p):
    key = masks.step_key(0xDEADBEEF, 17)
    rows, cols = 37, 67
    out = _run(host_check, "mask", key, 5, rows, cols, p).splitlines()
    got = np.array([[ch == "1" for ch in line] for line in out])
    np.testing.assert_array_equal(got, masks.keep_grid(key, 5, rows, cols, p).numpy())


def test_step_key_hash(host_check):
    for a, b in [(0, 0), (1, 2), (2**32 - 1, 2**32 - 1), (0xDEADBEEF, 17)]:
        assert int(_run(host_check, "hash", a, b)) == masks.hash32(a, b)


def test_bad_input_is_rejected_not_crashing(host_check):
    r = subprocess.run([host_check, "plan", "100", "2", "5:101"], env=ENV, capture_output=True, text=True)
    assert r.returncode == 1 and "nd out of range" in r.stderr

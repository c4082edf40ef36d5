"""In-tree build of the native extension ``attackfl_amd/_C.so`` for gfx950.

Device code lives in ``csrc/kernels/*.hip`` (pure HIP, no torch headers, so each file compiles
in seconds); ``csrc/bindings.cpp`` and ``csrc/comm/*.cpp`` hold the host side (torch op
bindings, the IPC all-gather runtime).  Objects are cached under ``build/`` by content hash,
so rebuilding after a one-kernel edit only recompiles that file.

Usage: ``python -m attackfl_amd._build`` (or ``python setup.py build_ext --inplace``).
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import hashlib
import os
import re
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "attackfl_amd")
BUILD = os.path.join(ROOT, "build", "obj")
OUT = os.environ.get("AFL_BUILD_OUT") or os.path.join(PKG, "_C.so")  # AFL_BUILD_OUT: A/B variant builds
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _torch_paths():
    import torch
    import torch.utils.cpp_extension as ce

    inc = ce.include_paths()
    lib = ce.library_paths()[0]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _hash(path: str, flags) -> str:
    h = hashlib.sha1()
    with open(path, "rb") as fh:
        src = fh.read()
    h.update(src)
    # sources included by path (e.g. tf2_stamps.hip includes tf2.hip) participate too
    for inc in re.findall(rb'#include\s+"([^"]+\.(?:hip|cpp|inc))"', src):
        p = os.path.join(os.path.dirname(path), inc.decode())
        if os.path.exists(p):
            with open(p, "rb") as fh:
                h.update(fh.read())
    # headers under csrc/ participate in every hash (cheap, conservative)
    for hdr in sorted(glob.glob(os.path.join(ROOT, "csrc", "**", "*.h"), recursive=True)):
        with open(hdr, "rb") as fh:
            h.update(fh.read())
    h.update(" ".join(flags).encode())
    return h.hexdigest()[:16]


def _compile(src: str, flags, verbose: bool) -> str:
    os.makedirs(BUILD, exist_ok=True)
    obj = os.path.join(BUILD, os.path.basename(src) + "." + _hash(src, flags) + ".o")
    if os.path.exists(obj):
        return obj
    cmd = [os.path.join(ROCM, "bin", "hipcc")] + flags + ["-c", src, "-o", obj + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"compile failed: {src}")
    os.replace(obj + ".tmp", obj)
    return obj


def build(verbose: bool = False, jobs: int = 0) -> str:
    inc, lib, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    common = ["-O3", "-fPIC", "-std=c++17", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-D__HIP_PLATFORM_AMD__",
              "-I" + os.path.join(ROOT, "csrc")]
    dev_flags = common + [f"--offload-arch={ARCH}", "-ffast-math", "-fno-gpu-rdc", "-munsafe-fp-atomics"]
    dev_flags = [f for f in dev_flags if f != "-ffast-math"]  # keep IEEE semantics (NaN checks in kernels)
    host_flags = common + ["-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H", "-DUSE_ROCM",
                           "-I" + py_inc, "-I" + os.path.join(ROCM, "include")] + ["-I" + p for p in inc] + ["-x", "c++"]
    kernels = sorted(glob.glob(os.path.join(ROOT, "csrc", "kernels", "*.hip")))
    # per-file device flags: the on-chip trainers (tf2 / rnn2) keep their optimizer state in AGPRs, so its MFMAs must accumulate
    # in VGPRs (otherwise their accumulators compete with that state for the AGPR half of the budget)
    extra = {f: ["-mllvm", "-amdgpu-mfma-vgpr-form"] for f in ("tf2.hip", "tf2_stamps.hip", "rnn2.hip", "rnn2_stamps.hip")}
    if os.environ.get("AFL_DEV_DEFINES"):  # A/B variant builds (tools/ab_native.sh): extra -D flags on every kernel
        dev_flags = dev_flags + os.environ["AFL_DEV_DEFINES"].split()
    if os.environ.get("AFL_TF2_ABL"):  # diagnostic ablation build of the timed kernel (tools/phase_profile.py)
        extra["tf2_stamps.hip"] = extra["tf2_stamps.hip"] + ["-DTF2_ABL=" + str(int(os.environ["AFL_TF2_ABL"]))]
    if os.environ.get("AFL_RNN2_ABL"):  # diagnostic ablation build of the stamped RNN trainer
        extra["rnn2_stamps.hip"] = extra["rnn2_stamps.hip"] + ["-DRNN2_ABL=" + str(int(os.environ["AFL_RNN2_ABL"]))]
    if os.environ.get("AFL_RNN2_DEBUG"):  # diagnostic printf build of the on-chip RNN trainer
        extra["rnn2.hip"] = extra["rnn2.hip"] + ["-DRNN2_" + os.environ["AFL_RNN2_DEBUG"]]
    hosts = sorted(glob.glob(os.path.join(ROOT, "csrc", "*.cpp")) + glob.glob(os.path.join(ROOT, "csrc", "comm", "*.cpp")))
    jobs = jobs or min(8, int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = [ex.submit(_compile, s, dev_flags + extra.get(os.path.basename(s), []), verbose) for s in kernels]
        futs += [ex.submit(_compile, s, host_flags, verbose) for s in hosts]
        objs = [f.result() for f in futs]
    cmd = [os.path.join(ROCM, "bin", "hipcc"), "-shared", "-fPIC", f"--offload-arch={ARCH}"] + objs + [
        "-o", OUT + ".tmp", "-L" + lib, "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-lc10", "-lc10_hip",
        "-ltorch_python", "-Wl,-rpath," + lib]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("link failed")
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    p = build(verbose="-v" in sys.argv)
    print(p)

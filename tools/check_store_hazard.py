"""Audit of the gfx950 "wide store data" hazard in our kernels' ISA: a vector-memory store of more than
8 bytes (dwordx3 / dwordx4) reads its data VGPRs after issue, so the very next instruction may not write
them (observed on MI355X: rnn2.hip's moment stores picked up the next v_mov's value in element 0 of some
lanes; the backend inserted no wait state).  Compiles every csrc/kernels/*.hip to gfx950 assembly with the
build's flags and lists each store whose data registers the following instruction overwrites.

Second audit (round 4): an inline-asm instruction that READS the result of a recent `v_mfma`.  The compiler
pads its own VALU reads of an MFMA result with the required wait states, but not an asm block's (har.hip's
first dQ keep select, an asm `v_cndmask`, read the dP accumulator two instructions after its MFMA and
returned garbage).  Flagged: an asm source VGPR that an MFMA wrote fewer than MFMA_WAIT wait states earlier.

    python tools/check_store_hazard.py [file.hip ...]
"""
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STORE = re.compile(r"^\s+(global|buffer|flat|scratch)_store_(dwordx3|dwordx4|b96|b128)\s+(.*)$")
INSN = re.compile(r"^\s+([a-z_0-9]+)(\s+(.*))?$")


def regs(spec):
    """'v[4:7]' / 'v5' / 'a[0:3]' -> set of register names"""
    m = re.match(r"([va])\[(\d+):(\d+)\]", spec)
    if m:
        return {f"{m.group(1)}{i}" for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.match(r"([va])(\d+)$", spec)
    return {spec} if m else set()


def data_regs(kind, ops):
    parts = [p.strip() for p in ops.split(",")]
    # global_store vaddr, vdata, saddr ; buffer_store vdata, vaddr, srsrc, soffset ; flat_store vaddr, vdata
    idx = 0 if kind in ("buffer", "scratch") else 1
    if kind == "scratch":
        idx = 1 if parts[0].startswith("v") and len(parts) > 2 else 0
    return regs(parts[idx]) if idx < len(parts) else set()


def written(line):
    m = INSN.match(line)
    if not m or m.group(1).startswith(("s_", "buffer_store", "global_store", "flat_store", "scratch_store", "ds_write")):
        return set()
    ops = (m.group(3) or "").split(",")
    return regs(ops[0].strip()) if ops and ops[0].strip() else set()


def scan(asm_path):
    lines = [l for l in open(asm_path) if l.strip() and not l.lstrip().startswith((";", ".", "//")) and not l.rstrip().endswith(":")]
    hits = []
    for i, l in enumerate(lines):
        m = STORE.match(l)
        if not m or i + 1 >= len(lines):
            continue
        nxt = lines[i + 1]
        if nxt.strip().startswith("s_nop"):
            continue
        dr = data_regs(m.group(1), m.group(3))
        w = written(nxt)
        if dr & w:
            hits.append((l.strip(), nxt.strip()))
    return hits


MFMA_WAIT = 19  # the longest MFMA result latency (32x32, 16 passes) plus margin, in wait states


def src_regs(line):
    """source VGPR / AGPR names of an instruction line (every operand after the destination)"""
    m = INSN.match(line)
    if not m:
        return set()
    out = set()
    for op in (m.group(3) or "").split(",")[1:]:
        out |= regs(op.strip().split()[0]) if op.strip() else set()
    return out


def scan_asm_mfma(asm_path):
    """(asm line, mfma line, wait states) for every inline-asm read of a too-recent MFMA result"""
    recent = []  # [(dest regs, mfma line, wait states since)]
    hits = []
    in_asm = False
    for raw in open(asm_path):
        l = raw.rstrip()
        st = l.strip()
        if st.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if st.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not st or st.startswith((";", ".", "//")) or st.endswith(":"):
            if st.endswith(":"):
                recent = []  # a label: control flow merges, stay conservative only within a block
            continue
        m = INSN.match(l)
        if not m:
            continue
        if in_asm:
            srcs = src_regs(l)
            for dr, ml, w in recent:
                if dr & srcs:
                    hits.append((st, ml, w))
        ws = 1
        if m.group(1) == "s_nop":
            try:
                ws = int((m.group(3) or "0").split()[0], 0) + 1
            except ValueError:
                ws = 1
        recent = [(dr, ml, w + ws) for dr, ml, w in recent if w + ws < MFMA_WAIT]
        if m.group(1).startswith("v_mfma"):
            ops = (m.group(3) or "").split(",")
            recent.append((regs(ops[0].strip()), st, 0))
    return hits


def check_file(f):
    extra = ["-mllvm", "-amdgpu-mfma-vgpr-form"] if os.path.basename(f).startswith(("tf2", "rnn2")) else []
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "k.s")
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I" + os.path.join(ROOT, "csrc"),
               "--offload-arch=gfx950", "-fno-gpu-rdc", "-munsafe-fp-atomics", "--cuda-device-only", "-S", f,
               "-o", out] + extra
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            return None
        return scan(out) + [(a, f"{m}  ({w} wait states)") for a, m, w in scan_asm_mfma(out)]


def main(files=None, jobs=8):
    import concurrent.futures as cf

    files = files or sorted(glob.glob(os.path.join(ROOT, "csrc", "kernels", "*.hip")))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        results = list(ex.map(check_file, files))
    total = 0
    for f, hits in zip(files, results):
        if hits is None:
            print(f"{os.path.basename(f)}: compile failed")
            total += 1
            continue
        total += len(hits)
        print(f"{os.path.basename(f)}: {len(hits)} hazard(s)")
        for st, nx in hits[:6]:
            print(f"    {st}\n      -> {nx}")
    return total


if __name__ == "__main__":
    sys.exit(1 if main(sys.argv[1:]) else 0)

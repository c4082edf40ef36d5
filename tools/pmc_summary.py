"""Per-kernel totals of rocprofv3 --pmc passes (tools/pmc_har.sh, tools/pmc_bench.sh): markdown table.

    python tools/pmc_summary.py gpurun_out/pmc_har [--kernels post_bwd,attn] [--title "..."]

Reads every *counter_collection.csv under the directory, sums Counter_Value per (kernel, counter) over all
dispatches, and prints the raw sums plus derived ratios (VALU : MFMA instructions, busy fractions, LDS bank
conflict cycles per LDS instruction, wave-cycles waiting).
"""
import argparse
import collections
import csv
import glob
import os


def load(root):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                k = row.get("Kernel_Name", "?").replace("(anonymous namespace)::", "")
                tot[k][row["Counter_Name"]] += float(row["Counter_Value"])
                disp[k].add(row.get("Dispatch_Id", ""))
    return tot, disp


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--kernels", default="", help="comma-separated substrings (default: all)")
    ap.add_argument("--title", default="PMC counters per kernel")
    a = ap.parse_args()
    tot, disp = load(a.root)
    want = [w for w in a.kernels.split(",") if w]
    names = sorted((k for k in tot if not want or any(w in k for w in want)),
                   key=lambda k: -tot[k].get("SQ_WAVE_CYCLES", 0.0))
    print(f"# {a.title}\n")
    print("VALU / wave-cycles = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (share of a wave's cycles spent issuing VALU); "
          "MFMA busy / busy = SQ_VALU_MFMA_BUSY_CYCLES / SQ_BUSY_CYCLES (raw counter ratio: the two count in different "
          "units, compare it between kernels only).\n")
    print("| kernel | dispatches | VALU:MFMA | VALU / wave-cycles | MFMA busy / busy | wait / wave-cycles | LDS conflicts / LDS inst |")
    print("|---|---|---|---|---|---|---|")
    for k in names:
        c = tot[k]
        g = lambda n: c.get(n, 0.0)
        ratio = g("SQ_INSTS_VALU") / g("SQ_INSTS_MFMA") if g("SQ_INSTS_MFMA") else float("nan")
        busy = g("SQ_BUSY_CYCLES") or float("nan")
        vb = g("SQ_ACTIVE_INST_VALU") / g("SQ_WAVE_CYCLES") if g("SQ_WAVE_CYCLES") else float("nan")
        mb = g("SQ_VALU_MFMA_BUSY_CYCLES") / busy
        wt = g("SQ_WAIT_ANY") / g("SQ_WAVE_CYCLES") if g("SQ_WAVE_CYCLES") else float("nan")
        lc = g("SQ_LDS_BANK_CONFLICT") / g("SQ_INSTS_LDS") if g("SQ_INSTS_LDS") else float("nan")
        short = k.split("(")[0][:60]
        print(f"| `{short}` | {len(disp[k])} | {ratio:.1f} | {vb:.2f} | {mb:.2f} | {wt:.2f} | {lc:.2f} |")
    print("\nRaw sums:\n")
    for k in names:
        print(f"* `{k.split('(')[0][:60]}`: " + ", ".join(f"{n} {v:.4g}" for n, v in sorted(tot[k].items())))


if __name__ == "__main__":
    main()

"""GPU idle time between consecutive training kernels of a rocprofv3 ``--kernel-trace`` run.

  python tools/round_gaps.py gpurun_out/prof_tf/run_kernel_trace.csv [kernel_substring] > profiles/x.md

Prints, per round, the training kernel's duration and the gap to the next round's training kernel (the
round's aggregate / validation / checkpoint / next-round preparation as the GPU sees it), then the
kernels inside the last gap with their offsets from the end of the training kernel.
"""
import csv
import sys


def main():
    path = sys.argv[1]
    name = sys.argv[2] if len(sys.argv) > 2 else "k_tf2_train"
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if name in r["Kernel_Name"]]
    print(f"# Gaps between `{name}` launches ({path.split('/')[-1]})\n")
    print("| round | train ms | gap to next train ms |")
    print("|---|---|---|")
    gaps = []
    for n, (a, b) in enumerate(zip(idx[:-1], idx[1:])):
        s0, e0 = int(rows[a]["Start_Timestamp"]), int(rows[a]["End_Timestamp"])
        gap = (int(rows[b]["Start_Timestamp"]) - e0) / 1e6
        gaps.append(gap)
        print(f"| {n} | {(e0 - s0) / 1e6:.3f} | {gap:.3f} |")
    if len(gaps) > 2:
        steady = sorted(gaps[2:])
        print(f"\nsteady-state median gap (rounds >= 2): {steady[len(steady) // 2]:.3f} ms\n")
    if len(idx) >= 2:
        a, b = idx[-2], idx[-1]
        e0 = int(rows[a]["End_Timestamp"])
        print("Kernels between the last two training launches (offset from the end of the first, duration):\n")
        print("| +ms | dur ms | kernel |")
        print("|---|---|---|")
        for r in rows[a + 1:b + 1]:
            st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            print(f"| {(st - e0) / 1e6:+.3f} | {(en - st) / 1e6:.3f} | `{r['Kernel_Name'][:80]}` |")


if __name__ == "__main__":
    main()

"""Markdown summary of a rocprofv3 ``--kernel-trace --stats --output-format csv`` run.

  python tools/rocprof_summary.py gpurun_out/prof_x/run_kernel_stats.csv "title" [top_n] > profiles/x.md
"""
import csv
import sys


def main():
    path, title = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    rows = list(csv.DictReader(open(path)))
    total = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# {title}\n")
    print("| kernel | calls | total ms | avg us | % |")
    print("|---|---|---|---|---|")
    for r in rows[:top]:
        name = r["Name"].replace("(anonymous namespace)::", "").replace("|", "/")[:96]
        print(f"| `{name}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.3f} | "
              f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} |")
    print(f"\nTotal GPU kernel time {total / 1e6:.1f} ms ({len(rows)} distinct kernels).")


if __name__ == "__main__":
    main()

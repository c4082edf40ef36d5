"""Markdown kernel summary (and optional timeline helpers) from a rocprofv3 SQLite database (``rocpd``).

  python tools/rocpd_summary.py gpurun_out/prof_x/run_results.db "title" [top_n] > profiles/x.md
"""
import sqlite3
import sys


def dispatches(db_path):
    """[(kernel name, start ns, end ns, stream/queue id)] in start order."""
    db = sqlite3.connect(db_path)
    rows = db.execute(
        "select s.kernel_name, d.start, d.end, d.queue_id from rocpd_kernel_dispatch d "
        "join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start").fetchall()
    return rows


def main():
    path, title = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 18
    agg = {}
    for name, a, b, _ in dispatches(path):
        n, t = agg.get(name, (0, 0))
        agg[name] = (n + 1, t + (b - a))
    total = sum(t for _, t in agg.values())
    print(f"# {title}\n")
    print("| kernel | calls | total ms | avg us | % |")
    print("|---|---|---|---|---|")
    for name, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        nm = name.replace("(anonymous namespace)::", "").replace("|", "/")[:96]
        print(f"| `{nm}` | {n} | {t / 1e6:.3f} | {t / n / 1e3:.1f} | {100.0 * t / total:.2f} |")
    print(f"\nTotal GPU kernel time {total / 1e6:.1f} ms ({len(agg)} distinct kernels).")


if __name__ == "__main__":
    main()

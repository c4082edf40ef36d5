"""Markdown tables from tools/attack_study.py JSONL output.

    python tools/study_table.py A.jsonl [B.jsonl ...]            # final AUC per (mode, attack), one column per file
    python tools/study_table.py --seeds S.jsonl                   # mean / min / max over seeds per cell

A column header is the file's stem.  A cell shows the final test AUC after the study's rounds; "F" marks a run with
failed rounds and "S" one that stalled (no accepted update for the rest of the run).
"""
import argparse
import json
import os
import statistics


def load(path):
    with open(path) as f:
        return [json.loads(l) for l in f if l.strip()]


def cell(r):
    s = f"{r['final_auc']:.3f}"
    if r.get("failed_rounds"):
        s += " F"
    if r.get("stalled"):
        s += " S"
    return s


def grid(paths):
    cols = [os.path.splitext(os.path.basename(p))[0] for p in paths]
    rows, order = {}, []
    for c, p in zip(cols, paths):
        for r in load(p):
            k = (r["mode"], r["attack"])
            if k not in rows:
                rows[k] = {}
                order.append(k)
            rows[k][c] = cell(r)
    out = ["| mode | attack | " + " | ".join(cols) + " |", "|---|---|" + "---|" * len(cols)]
    for k in order:
        out.append(f"| {k[0]} | {k[1]} | " + " | ".join(rows[k].get(c, "—") for c in cols) + " |")
    return "\n".join(out)


def seeds(path):
    cells, order = {}, []
    for r in load(path):
        k = (r["device"], r["mode"], r["attack"])
        if k not in cells:
            cells[k] = []
            order.append(k)
        cells[k].append((r.get("seed"), r["final_auc"]))
    out = ["| device | mode | attack | seeds | mean AUC | stdev | min | max |", "|---|---|---|---|---|---|---|---|"]
    for k in order:
        v = [a for _, a in sorted(cells[k], key=lambda t: (t[0] is None, t[0]))]
        sd = statistics.stdev(v) if len(v) > 1 else 0.0
        out.append(f"| {k[0]} | {k[1]} | {k[2]} | {len(v)} | {statistics.mean(v):.3f} | {sd:.3f} | "
                   f"{min(v):.3f} | {max(v):.3f} |")
    return "\n".join(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--seeds", action="store_true")
    a = ap.parse_args()
    print("\n\n".join(seeds(p) for p in a.files) if a.seeds else grid(a.files))


if __name__ == "__main__":
    main()

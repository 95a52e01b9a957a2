"""Per-step kernel breakdown from a rocprofv3 kernel_trace.csv: the last complete step
between two launches of a marker kernel (the first kernel of every step), grouped by
kernel name, plus the step's span and GPU-busy time.  Markdown for profiles/*/README.md.

    python scripts/step_breakdown.py gpurun_out/prof_resnet/rn_kernel_trace.csv --marker xent_kernel
"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", required=True, help="substring of the step's first kernel")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if len(idx) < 2:
        raise SystemExit("need two marker launches")
    i0, i1 = idx[-2], idx[-1]
    step = rows[i0:i1]
    t0, t1 = int(step[0]["Start_Timestamp"]), int(rows[i1]["Start_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step) / 1e3
    tot, cnt = defaultdict(float), defaultdict(int)
    for r in step:
        n = r["Kernel_Name"].split("(")[0].replace("void ", "")
        tot[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        cnt[n] += 1
    print(f"one step: {len(step)} kernels, span {(t1 - t0) / 1e3:.1f} us, GPU busy {busy:.1f} us\n")
    print("| kernel | launches | total us | % of busy |")
    print("|---|---|---|---|")
    for n, v in sorted(tot.items(), key=lambda kv: -kv[1])[:a.top]:
        print(f"| `{n[:100]}` | {cnt[n]} | {v:.1f} | {100 * v / busy:.1f} |")


if __name__ == "__main__":
    main()

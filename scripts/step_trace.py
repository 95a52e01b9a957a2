"""Per-step device timeline of the LAST n steps of a rocprofv3 kernel trace (csv).

    python scripts/step_trace.py <rocprof out dir> [n_steps=20] [marker=conv3x3_fwd]

A step starts at a launch of the marker kernel (the SimpleCNN forward) and ends where the
next one starts (the last step: at the end of the last kernel).  Prints, per step, its
span and the sum of kernel durations in it, then the idle gap in front of the first of
the n steps, and the steady-state comparison (median of the last half) - VERDICT r3 #2's
"per-step device time for steps 1..20 against steady state".
"""
import csv
import glob
import os
import statistics
import sys


def load(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def main(d, n=20, marker="conv3x3_fwd"):
    n = int(n)
    rows = load(d)
    starts = [i for i, r in enumerate(rows) if marker in r[2]]
    if len(starts) < n:
        raise SystemExit(f"only {len(starts)} {marker} launches in {d}")
    first = starts[-n:]
    out = []
    # the last step: as many kernels as the other steps have (what follows belongs to the
    # run's tail - isolated all-reduce timings, synchronisation)
    kps = statistics.median(first[j + 1] - first[j] for j in range(n - 1)) if n > 1 else len(rows) - first[0]
    for j, i0 in enumerate(first):
        i1 = first[j + 1] if j + 1 < n else min(len(rows), i0 + int(kps))
        seg = rows[i0:i1]
        t0 = seg[0][0]
        t1 = rows[i1][0] if (i1 < len(rows) and j + 1 < n) else max(r[1] for r in seg)
        busy = sum(r[1] - r[0] for r in seg)
        out.append(((t1 - t0) / 1000.0, busy / 1000.0, len(seg), [(r[1] - r[0]) / 1000.0 for r in seg]))
    gap = (rows[first[0]][0] - rows[first[0] - 1][1]) / 1000.0 if first[0] > 0 else float("nan")
    steady = statistics.median(s for s, _, _, _ in out[n // 2:])
    print(f"idle gap before the first of the last {n} steps: {gap:.1f} us")
    print("| step | span us | busy us | kernels | per-kernel us | vs steady |")
    print("|---|---|---|---|---|---|")
    for j, (s, b, k, ks) in enumerate(out):
        print(f"| {j + 1} | {s:.2f} | {b:.2f} | {k} | {' '.join(f'{x:.2f}' for x in ks)} | {s - steady:+.2f} |")
    tot = sum(s for s, _, _, _ in out)
    print(f"\ntotal span {tot:.1f} us = {tot / n:.2f} us/step; steady median {steady:.2f} us; "
          f"excess over steady {tot - n * steady:.1f} us")


if __name__ == "__main__":
    main(*sys.argv[1:])

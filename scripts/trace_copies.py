"""Runtime copy / fill kernels per training step, from a rocprofv3 kernel trace (csv).

    python scripts/trace_copies.py <rocprof out dir> [marker=sgd_kernel] [n_steps=10]

Segments the trace at each launch of the marker kernel (the step's last kernel: one per
step), takes the last n steps (steady state: graph replays) and lists, per step, every
HIP runtime blit kernel (``__amd_rocclr_copyBuffer*`` / ``__amd_rocclr_fillBuffer*``) with
its grid size (threads; the runtime's blit kernels move 16 B per thread in the aligned
path, so grid x 16 ~ bytes) and duration, plus their share of the step's kernel time.
VERDICT r5 #4: attribute the ResNet-18 step's copies and fills.  Then the per-step kernel
time by kernel family over the same steps, and the BatchNorm share (kernels named bn_*).
"""
import collections
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
                grid = r.get("Grid_Size") or r.get("Grid_Size_X") or "0"
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(grid)))
    rows.sort()
    return rows


def main(d, marker="sgd_kernel", n=10):
    n = int(n)
    rows = load(d)
    ends = [i for i, r in enumerate(rows) if marker in r[2]]
    if len(ends) < n + 1:
        raise SystemExit(f"only {len(ends)} {marker} launches in {d}")
    print(f"| step | kernels | kernel us | blit kernels (name: grid, us) | blit us | blit % |")
    print("|---|---|---|---|---|---|")
    shares = []
    for j in range(len(ends) - n, len(ends)):
        seg = rows[ends[j - 1] + 1:ends[j] + 1]
        tot = sum(r[1] - r[0] for r in seg) / 1000.0
        blit = [r for r in seg if r[2].startswith("__amd_rocclr")]
        bt = sum(r[1] - r[0] for r in blit) / 1000.0
        desc = "; ".join(f"{r[2].replace('__amd_rocclr_', '')}: {r[3]}, {(r[1] - r[0]) / 1000.0:.1f}" for r in blit)
        shares.append(bt / tot if tot else 0.0)
        print(f"| {j} | {len(seg)} | {tot:.1f} | {desc or '-'} | {bt:.1f} | {100 * bt / tot:.2f} |")
    print(f"\nmedian blit share of the step's kernel time: {100 * statistics.median(shares):.2f} %")
    allb = [r for r in rows if r[2].startswith("__amd_rocclr")]
    inside = sum(1 for j in range(len(ends) - n, len(ends)) for r in rows[ends[j - 1] + 1:ends[j] + 1]
                 if r[2].startswith("__amd_rocclr"))
    print(f"blit kernels in the whole trace: {len(allb)}; in the last {n} steps: {inside} "
          f"(the rest: set-up, data generation, warm-up / capture)")
    fam, cnt, tot = collections.Counter(), collections.Counter(), 0
    for j in range(len(ends) - n, len(ends)):
        for r in rows[ends[j - 1] + 1:ends[j] + 1]:
            k = r[2].split("(")[0].split("<")[0].replace("void ", "").replace("ddp_amd::", "")
            fam[k] += r[1] - r[0]
            cnt[k] += 1
            tot += r[1] - r[0]
    bn = sum(v for k, v in fam.items() if k.startswith("bn_"))
    print(f"\n| kernel | launches/step | us/step | share |\n|---|---|---|---|")
    for k, v in fam.most_common():
        print(f"| {k} | {cnt[k] / n:.1f} | {v / n / 1000.0:.1f} | {100.0 * v / tot:.1f} % |")
    print(f"\nkernel time per step {tot / n / 1000.0:.1f} us; BatchNorm (bn_*) {100.0 * bn / tot:.1f} %")


if __name__ == "__main__":
    main(*sys.argv[1:])

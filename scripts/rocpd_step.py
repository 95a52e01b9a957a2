"""Per-step kernel table from a rocprofv3 rocpd database (one step = the span between two
consecutive launches of a marker kernel, default the ResNet maxpool forward)."""
import sqlite3
import sys


def main(db, marker="maxpool_fwd", out=None):
    c = sqlite3.connect(db)
    st = [r[0] for r in c.execute("select start from kernels where name like ? order by start", (f"%{marker}%",))]
    a, b = st[-3], st[-2]
    rows = c.execute("select name, count(*), sum(end-start)/1000.0 from kernels where start>=? and start<? "
                     "group by name order by 3 desc", (a, b)).fetchall()
    busy = sum(r[2] for r in rows)
    lines = [f"One step: {sum(r[1] for r in rows)} kernels, span {(b - a) / 1000:.1f} us, GPU busy {busy:.1f} us", "",
             "| kernel | launches | total us | % of busy |", "|---|---|---|---|"]
    for n, k, t in rows:
        lines.append(f"| `{n.split('(')[0][:100]}` | {k} | {t:.1f} | {100 * t / busy:.1f} |")
    text = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(text)
    print(text)


if __name__ == "__main__":
    main(*sys.argv[1:])

"""Markdown table from a rocprofv3 --stats kernel_stats.csv (for profiles/*/README.md)."""
import csv
import sys


def main(path, steps):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print("| kernel | calls | avg us | % |")
    print("|---|---|---|---|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        name = r["Name"].replace("|", "\\|")[:90]
        print(f"| `{name}` | {r['Calls']} | {float(r['AverageNs']) / 1000:.2f} | "
              f"{100 * float(r['TotalDurationNs']) / tot:.1f} |")
    print(f"\nkernel time per step (sum over kernels / {steps} steps): {tot / steps / 1000:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 220)

"""Per-kernel hardware-counter table from rocprofv3 --pmc counter_collection.csv files
(one or more passes of the same workload), averaged per dispatch.  Derived columns:

* MFMA TFLOP/s = SQ_INSTS_MFMA x 16384 FLOP (every MFMA here is a 16x16x32 bf16 one,
  issued per wave) / kernel duration;
* LDS conflict/instr = SQ_LDS_BANK_CONFLICT (cycles) / SQ_INSTS_LDS;
* fetch / write GB/s = FETCH_SIZE / WRITE_SIZE (KB, L2 <-> memory) / duration.

    python scripts/pmc_summary.py gpurun_out/pmc_r/s1/s_counter_collection.csv ... [--top 12]
"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--match", default="ddp_amd", help="substring of the kernels to list")
    a = ap.parse_args()
    val = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(lambda: defaultdict(set))
    dur = defaultdict(list)
    for f in a.files:
        seen = set()
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if a.match not in name:
                continue
            c = r["Counter_Name"]
            val[name][c] += float(r["Counter_Value"])
            disp[name][c].add((f, r["Dispatch_Id"]))
            key = (f, r["Dispatch_Id"])
            if key not in seen:
                seen.add(key)
                dur[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    rows = []
    for name, cs in val.items():
        avg = {c: v / max(1, len(disp[name][c])) for c, v in cs.items()}
        d = sum(dur[name]) / len(dur[name])
        rows.append((d, name, avg))
    rows.sort(key=lambda t: -t[0] * len(dur[t[1]]))
    print("| kernel | us/dispatch | MFMA TFLOP/s | LDS instr | LDS conflict cycles / instr | fetch GB/s | write GB/s "
          "| VALU instr | MFMA instr | LDS-wait / wave cycles |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for d, name, c in rows[:a.top]:
        mf = c.get("SQ_INSTS_MFMA")
        tf = f"{mf * 16384 / (d * 1e-6) / 1e12:.0f}" if mf else "-"
        li = c.get("SQ_INSTS_LDS")
        lc = f"{c['SQ_LDS_BANK_CONFLICT'] / li:.2f}" if li and "SQ_LDS_BANK_CONFLICT" in c else "-"
        fs = f"{c['FETCH_SIZE'] * 1024 / (d * 1e-6) / 1e9:.0f}" if "FETCH_SIZE" in c else "-"
        ws = f"{c['WRITE_SIZE'] * 1024 / (d * 1e-6) / 1e9:.0f}" if "WRITE_SIZE" in c else "-"
        va = f"{c['SQ_INSTS_VALU']:.0f}" if "SQ_INSTS_VALU" in c else "-"
        mi = f"{mf:.0f}" if mf else "-"
        lw = (f"{c['SQ_WAIT_INST_LDS'] / c['SQ_WAVE_CYCLES']:.2f}"
              if c.get("SQ_WAVE_CYCLES") and "SQ_WAIT_INST_LDS" in c else "-")
        lis = f"{li:.0f}" if li is not None else "-"
        print(f"| `{name[:80]}` | {d:.1f} | {tf} | {lis} | {lc} | {fs} | {ws} | {va} | {mi} | {lw} |")


if __name__ == "__main__":
    main()

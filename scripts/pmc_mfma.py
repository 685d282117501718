"""MFMA utilisation per kernel from one rocprofv3 PMC pass
(SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_VALU_MFMA_MOPS_BF16, GRBM_GUI_ACTIVE) plus
its kernel trace (durations).  Per MI355X_MICROARCH.md: GRBM_GUI_ACTIVE is
summed over the 8 XCDs (cycles = value / 8); SQ_VALU_MFMA_BUSY_CYCLES is the
sum over SIMDs of matrix-pipe busy cycles (1024 SIMDs); MOPS_BF16 x 512 =
bf16 MFMA flops.  MfmaUtil = busy / (1024 * cycles) (counter_defs.yaml's
definition); counter TFLOP/s = MOPS x 512 / kernel duration.

usage: python scripts/pmc_mfma.py <pmc_dir> [out.json]"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict

SIMDS = 1024


def tag_of(name):
    m = re.search(r"unet::(\w+<[^>]*>|\w+)\(", name)
    return m.group(1) if m else re.sub(r"\(.*", "", name).replace("void ", "")[:80]


def main():
    d = sys.argv[1]
    out_path = sys.argv[2] if len(sys.argv) > 2 else None
    vals = defaultdict(lambda: defaultdict(float))
    names = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            key = (f.rsplit("/", 1)[0], r["Dispatch_Id"])
            vals[key][r["Counter_Name"]] += float(r["Counter_Value"])
            names[key] = r["Kernel_Name"]
    durs = {}
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            durs[(f.rsplit("/", 1)[0], r["Dispatch_Id"])] = (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) * 1e-9
    per = defaultdict(lambda: [0, 0.0, 0.0, 0.0, 0.0])  # n, dur, busy, mops, cycles
    for k, v in vals.items():
        t = per[tag_of(names[k])]
        t[0] += 1
        t[1] += durs.get(k, 0.0)
        t[2] += v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        t[3] += v.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0)
        t[4] += v.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
    table = {}
    for tag, (n, dur, busy, mops, cyc) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        if mops <= 0:
            continue
        util = busy / (SIMDS * cyc) if cyc > 0 else 0.0
        tf = mops * 512 / dur / 1e12 if dur > 0 else 0.0
        clk = cyc / dur / 1e9 if dur > 0 else 0.0
        table[tag] = {"launches": n, "avg_us": round(dur / n * 1e6, 2), "mfma_util": round(util, 4),
                      "counter_tflops": round(tf, 1), "clock_ghz": round(clk, 3)}
        print(f"{tag:58s} n={n:4d} avg {dur / n * 1e6:8.1f} us  MfmaUtil {100 * util:5.1f}%  "
              f"{tf:7.1f} TFLOP/s (counters)  clk {clk:.2f} GHz")
    if out_path:
        json.dump(table, open(out_path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()

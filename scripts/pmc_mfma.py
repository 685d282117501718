"""MFMA utilisation per kernel from one rocprofv3 PMC pass
(SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_VALU_MFMA_MOPS_BF16, GRBM_GUI_ACTIVE) plus
its kernel trace (durations).  Per MI355X_MICROARCH.md: GRBM_GUI_ACTIVE is
summed over the 8 XCDs (cycles = value / 8); SQ_VALU_MFMA_BUSY_CYCLES is the
sum over SIMDs of matrix-pipe busy cycles (1024 SIMDs); MOPS_BF16 x 512 =
bf16 MFMA flops; counter TFLOP/s = MOPS x 512 / kernel duration.

MfmaUtil = busy / (1024 SIMDs x kernel duration x shader clock).  The clock is
the in-kernel one (s_memtime / s_memrealtime stamps of the conv kernels,
scripts/conv_timing.py: 1.9-2.4 GHz by kernel, median 2.1 GHz in
profiles/r04/s1), passed as --clk (default 2.1).  GRBM_GUI_ACTIVE / 8 is NOT
used as the cycle count: on dispatches shorter than ~0.3 ms it implies clocks
of 2.4-3.3 GHz, above the 2.4 GHz maximum (MI355X_MICROARCH.md 'DVFS
give-back'), and biased the utilisation low; it is still printed ("grbm clk")
for reference.  "util@2.4" is the floor (the clock never exceeds 2.4 GHz).

usage: python scripts/pmc_mfma.py <pmc_dir> [out.json] [--clk GHz]"""
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
    args = [x for x in sys.argv[1:] if not x.startswith("--")]
    clk_ghz = 2.1
    if "--clk" in sys.argv:
        clk_ghz = float(sys.argv[sys.argv.index("--clk") + 1])
        args = [x for x in args if x != sys.argv[sys.argv.index("--clk") + 1]]
    d = args[0]
    out_path = args[1] if len(args) > 1 else None
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
        util = busy / (SIMDS * dur * clk_ghz * 1e9) if dur > 0 else 0.0
        floor = busy / (SIMDS * dur * 2.4e9) if dur > 0 else 0.0
        tf = mops * 512 / dur / 1e12 if dur > 0 else 0.0
        grbm_clk = cyc / dur / 1e9 if dur > 0 else 0.0
        table[tag] = {"launches": n, "avg_us": round(dur / n * 1e6, 2), "mfma_util": round(util, 4),
                      "mfma_util_floor_2p4ghz": round(floor, 4), "clock_ghz_assumed": clk_ghz,
                      "counter_tflops": round(tf, 1), "grbm_clock_ghz": round(grbm_clk, 3)}
        print(f"{tag:58s} n={n:4d} avg {dur / n * 1e6:8.1f} us  MfmaUtil {100 * util:5.1f}% (@{clk_ghz} GHz; "
              f"floor {100 * floor:5.1f}% @2.4)  {tf:7.1f} TFLOP/s (counters)  grbm clk {grbm_clk:.2f} GHz")
    if out_path:
        json.dump(table, open(out_path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()

"""Summarise rocprofv3 --pmc databases: per kernel (name filter), the mean of
each counter summed over instances per dispatch.  usage:
python scripts/pmc_summary.py <filter> gpurun_out/pmc_c1 gpurun_out/pmc_c2 ..."""
import glob
import sqlite3
import sys
from collections import defaultdict

flt = sys.argv[1]
for d in sys.argv[2:]:
    for db in glob.glob(f"{d}/**/*.db", recursive=True):
        c = sqlite3.connect(db)
        per = defaultdict(lambda: defaultdict(float))
        names, dur = {}, {}
        for disp, name, cn, v, du in c.execute(
                "select dispatch_id, name, counter_name, counter_value, duration from pmc_events"):
            if flt not in name:
                continue
            per[disp][cn] += v
            names[disp] = name.split("(")[0][-60:] + " " + name[name.find("<"):name.find(">") + 1][:40]
            dur[disp] = du
        agg = defaultdict(lambda: defaultdict(list))
        for disp, cs in per.items():
            for cn, v in cs.items():
                agg[names[disp]][cn].append(v)
            agg[names[disp]]["dur_ns"].append(dur[disp])
        for k, cs in agg.items():
            print(d, k, " ".join(f"{cn}={sum(v) / len(v):.4g}" for cn, v in sorted(cs.items())))

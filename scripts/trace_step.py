"""Per-dispatch view of one graph-replayed step from a rocprofv3 kernel trace:
kernel durations, idle gaps between dispatches, grouped by kind.
usage: python scripts/trace_step.py <kernel_trace.csv> [--step K] [--list]"""
import csv, sys, collections, re
path = sys.argv[1]
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# a step starts at the first pack_kernel (weights packed at the start of forward)
starts = [i for i, r in enumerate(rows) if "pack_kernel" in r["Kernel_Name"] and "unpack" not in r["Kernel_Name"]
          and (i == 0 or "pack_kernel" not in rows[i - 1]["Kernel_Name"])]
k = int(sys.argv[sys.argv.index("--step") + 1]) if "--step" in sys.argv else len(starts) // 2
seg = rows[starts[k]:starts[k + 1]]
t0 = int(seg[0]["Start_Timestamp"]); t1 = int(seg[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
print(f"step {k}: {len(seg)} dispatches, wall {(t1 - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us, "
      f"gaps {(t1 - t0 - busy) / 1e3:.1f} us")
def kind(n):
    n = n.split("(")[0]
    n = re.sub(r"^void ", "", n)
    n = re.sub(r"at::native::.*", "torch", n)
    return n.replace("unet::", "")
agg = collections.defaultdict(lambda: [0, 0.0])
prev_end = None
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    a = agg[kind(r["Kernel_Name"])]
    a[0] += 1; a[1] += (e - s) / 1e3
    if "--list" in sys.argv:
        gap = (s - prev_end) / 1e3 if prev_end else 0
        print(f"{(e - s) / 1e3:8.1f} us  gap {gap:6.1f}  grid {r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']} "
              f"wg {r['Workgroup_Size_X']}  {kind(r['Kernel_Name'])[:70]}")
    prev_end = e
for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{t:9.1f} us  n={c:3d}  {n[:90]}")

"""HBM traffic per launch of every conv kernel instance from two rocprofv3 PMC
passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950), corrected as
MI355X_MICROARCH.md's HBM section prescribes: FETCH_SIZE counts 64 B per 128-B
request, so it is doubled; WRITE_SIZE is taken as is.  Both are in KiB.

usage: python scripts/pmc_traffic.py <fetch_dir> <write_dir> [out.json] [--config KEY]
(scripts/profile_round.sh runs the passes and this script).  KEY names the
workload the passes profiled (bench.config_key: backbone/width/decoder/dtype/
batch x size); bench.py quotes bytes only from a file of its own config."""
import csv
import glob
import json
import re
import sys
from collections import defaultdict


def load(d, counter):
    per = defaultdict(float)
    names = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] != counter:
                    continue
                key = (f, r["Dispatch_Id"])
                per[key] += float(r["Counter_Value"])
                names[key] = r["Kernel_Name"]
    out = defaultdict(list)
    for k, v in per.items():
        m = re.search(r"unet::(\w+<[^>]*>)", names[k])
        tag = m.group(1) if m else re.sub(r"\(.*", "", names[k]).replace("void ", "")[:80]
        out[tag].append(v)
    return out


def main():
    argv = list(sys.argv[1:])
    config = "resnet34/w1/plain/bf16/16x512"  # layer_profile.py's default workload
    if "--config" in argv:
        i = argv.index("--config")
        config = argv[i + 1]
        del argv[i:i + 2]
    fetch, write = load(argv[0], "FETCH_SIZE"), load(argv[1], "WRITE_SIZE")
    out_path = argv[2] if len(argv) > 2 else "profiles/pmc_traffic.json"
    table = {}
    for tag in sorted(set(fetch) & set(write)):
        f = sum(fetch[tag]) / len(fetch[tag]) * 1024 * 2
        w = sum(write[tag]) / len(write[tag]) * 1024
        table[tag] = {"bytes_per_launch": round(f + w), "fetch_bytes": round(f), "write_bytes": round(w),
                      "launches": len(fetch[tag])}
        print(f"{tag:60s} n={len(fetch[tag]):4d} fetch {f / 1e6:9.2f} MB  write {w / 1e6:9.2f} MB")
    with open(out_path, "w") as fh:
        json.dump({"config": config, "kernels": table}, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Averages rocprofv3 PMC counters and kernel-trace durations per kernel
name over a tools/counters.sh output directory; prints JSON."""
import collections
import csv
import glob
import json
import os
import sys


def short(name: str) -> str:
    n = name.split("(")[0]
    return n.replace("void ", "").replace("dpfk::", "")


def main(d: str) -> None:
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "p*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in acc.items():
        out[k] = {c: sum(v) / len(v) for c, v in cs.items()}
    for f in glob.glob(os.path.join(d, "kt", "*kernel_stats.csv")):
        for r in csv.DictReader(open(f)):
            out.setdefault(short(r["Name"]), {})["avg_ns"] = float(r["AverageNs"])
            out[short(r["Name"])]["calls"] = int(r["Calls"])
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1])

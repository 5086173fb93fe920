"""Mean PMC counter values per kernel from rocprofv3 --pmc output dirs.
Usage: python tools/pmc_mean.py <dir> [<dir> ...] > summary.json
(each <dir> holds p_counter_collection.csv from one --pmc pass)."""
import collections
import csv
import glob
import json
import sys


def main(dirs):
    out = {}
    for d in dirs:
        for f in glob.glob(d + "/*counter_collection.csv"):
            agg = collections.defaultdict(lambda: collections.defaultdict(list))
            for r in csv.DictReader(open(f)):
                agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
            for k, v in agg.items():
                o = out.setdefault(d.rstrip("/").split("/")[-1], {}).setdefault(k, {})
                for c, x in v.items():
                    o[c] = sum(x) / len(x)
                    o["dispatches"] = len(x)
    json.dump(out, sys.stdout, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1:])

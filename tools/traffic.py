#!/usr/bin/env python3
"""Per-launch HBM traffic of each kernel from rocprofv3 PMC passes.

Reads a tools/counters.sh summary.json (FETCH_SIZE and WRITE_SIZE from
separate passes, KiB per dispatch) and applies MI355X_MICROARCH.md's gfx950
correction: FETCH_SIZE reports half the bytes of wide coalesced streaming
reads, so reads are doubled (an upper bound for narrower accesses); WRITE_SIZE
is exact for 16-byte-per-lane stores, which is what the tree kernel issues.
Writes {kernel: {"fetch_bytes", "write_bytes", "traffic_bytes"}} as JSON."""
import json
import sys


def main(src: str, dst: str) -> None:
    s = json.load(open(src))
    out = {}
    for k, v in s.items():
        if "FETCH_SIZE" not in v or "WRITE_SIZE" not in v:
            continue
        f = v["FETCH_SIZE"] * 1024 * 2
        w = v["WRITE_SIZE"] * 1024
        out[k] = {"fetch_bytes": f, "write_bytes": w, "traffic_bytes": f + w,
                  "avg_ns": v.get("avg_ns")}
    json.dump(out, open(dst, "w"), indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])

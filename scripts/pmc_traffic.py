#!/usr/bin/env python3
"""Turn two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; one counter per
pass, as MI355X_MICROARCH.md's HBM section prescribes) into HBM bytes per
launch of one kernel, with the gfx950 correction: FETCH_SIZE (KiB) reports
exactly half of a 16-B/lane coalesced streaming read, so it is doubled;
WRITE_SIZE (KiB) is taken as is.

usage: pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> <kernel-substring> <out.json>
"""
import csv
import json
import sys


def per_dispatch(path, kernel, counter):
    vals = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                vals[row["Dispatch_Id"]] = vals.get(row["Dispatch_Id"], 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    fpath, wpath, kernel, out = sys.argv[1:5]
    fetch = per_dispatch(fpath, kernel, "FETCH_SIZE")
    write = per_dispatch(wpath, kernel, "WRITE_SIZE")
    if not fetch or not write:
        raise SystemExit(f"no samples for {kernel!r}")
    f_kib = sum(fetch) / len(fetch)
    w_kib = sum(write) / len(write)
    res = {"kernel": kernel, "dispatches": [len(fetch), len(write)],
           "fetch_size_kib_raw": f_kib, "write_size_kib_raw": w_kib,
           "read_bytes_per_launch": 2 * f_kib * 1024, "write_bytes_per_launch": w_kib * 1024,
           "hbm_bytes_per_launch": int(2 * f_kib * 1024 + w_kib * 1024),
           "correction": "FETCH_SIZE x2 (gfx950, 16-B/lane streaming reads), KiB -> bytes"}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()

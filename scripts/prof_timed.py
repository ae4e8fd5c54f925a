#!/usr/bin/env python3
"""Per-kernel durations from a rocprofv3 --kernel-trace CSV, split into the
whole run (what --stats averages, warmup and clock ramp included) and the
bench's timed region: the LAST <steps> dispatches of each kernel that ran at
least that often (bench.py times exactly its last K steps of the exact
arithmetic; with --no-fma-variant nothing runs after them).  This is the
profile figure to compare with the bench line's ms_per_step.

usage: prof_timed.py <kernel_trace.csv> <steps> <out.json> [bench_line.json]
"""
import csv
import json
import statistics
import sys


def main():
    path, steps, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    bench = None
    if len(sys.argv) > 4:
        with open(sys.argv[4]) as f:
            txt = f.read().strip().splitlines()
        bench = json.loads(txt[-1]) if txt else None
    durs = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            d = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3  # us
            durs.setdefault(row["Kernel_Name"], []).append((int(row["Start_Timestamp"]), d))
    res = {"source": path, "timed_steps": steps, "kernels": []}
    for name, v in sorted(durs.items(), key=lambda kv: -sum(d for _, d in kv[1])):
        v.sort()
        all_d = [d for _, d in v]
        ent = {"kernel": name[:160], "calls": len(all_d), "avg_us_all": round(statistics.mean(all_d), 3),
               "min_us": round(min(all_d), 3), "max_us": round(max(all_d), 3)}
        if len(all_d) >= steps:
            last = all_d[-steps:]
            ent["avg_us_timed"] = round(statistics.mean(last), 3)
            ent["median_us_timed"] = round(statistics.median(last), 3)
            # span of the timed region: first start .. last end (includes gaps between launches)
            t0 = v[-steps][0]
            t1 = v[-1][0] + v[-1][1] * 1e3
            ent["span_us_timed"] = round((t1 - t0) / 1e3, 3)
        res["kernels"].append(ent)
    if bench:
        res["bench_ms_per_step"] = bench.get("ms_per_step")
        res["bench_value"] = bench.get("value")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    top = res["kernels"][0]
    print(json.dumps({k: top.get(k) for k in ("kernel", "calls", "avg_us_all", "avg_us_timed", "median_us_timed")}))


if __name__ == "__main__":
    main()

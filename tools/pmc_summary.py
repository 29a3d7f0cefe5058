#!/usr/bin/env python3
"""Summarise one workload's rocprofv3 passes (tools/gpu/full_round1.sh) into
profiles/:

  <prof>/trace/run_kernel_stats.csv   --kernel-trace --stats pass
  <prof>/fetch/run_counter_collection.csv   --pmc FETCH_SIZE pass
  <prof>/write/run_counter_collection.csv   --pmc WRITE_SIZE pass
  <prof>/bench.json                  bench.py line of the traced command

writes profiles/<round>_kernel_stats_<workload>.csv (the rocprof summary as
is), profiles/pmc_<workload>.json (HBM bytes per expand launch, read by
bench.py as roofline.traffic) and prints the cross-check of the rocprof
average expand duration against bench.py's live in-kernel measurement.

Correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are
in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced read,
so the read side is doubled.  The expand kernel's reads are mostly 8-32 B
gathers (node-table probes, pair-table cells) for which the counter is not
calibrated, so `hbm_bytes_per_launch` prices every read as if it were the
wide-read case (an upper bound for the read side); the raw figure is kept
beside it.
"""
import argparse
import csv
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(path, counter):
    vals = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            name = row["Kernel_Name"]
            vals.setdefault(name, []).append(float(row["Counter_Value"]))
    return vals


def is_expand(name):
    """The dominant search kernel: the batched engine's expand kernel, or the
    LDS-resident search (one launch per search)."""
    return ("expand_kernel" in name and "expand_api" not in name) or "solo_kernel" in name


def is_search_start(name):
    return "pairalign" in name or "solo_kernel" in name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof")
    ap.add_argument("workload")
    ap.add_argument("--round", default="r2")
    ap.add_argument("--commit", default="", help="commit the traced command ran at")
    ap.add_argument("--cmd", default="", help="the traced bench command")
    args = ap.parse_args()

    stats_src = os.path.join(args.prof, "trace", "run_kernel_stats.csv")
    stats_dst = os.path.join(ROOT, "profiles", "%s_kernel_stats_%s.csv" % (args.round, args.workload))
    shutil.copyfile(stats_src, stats_dst)
    calls = dur = 0
    with open(stats_src) as f:
        for row in csv.DictReader(f):
            if is_expand(row["Name"]):
                calls += int(row["Calls"])
                dur += float(row["TotalDurationNs"])
    rocprof_avg_us = dur / calls / 1e3 if calls else None
    # the same average over the timed searches only: bench.py's steps start
    # with the PairAlign launch, so the first `warmup` of them are untimed
    bench_pre = None
    bpath0 = os.path.join(args.prof, "bench.json")
    if os.path.exists(bpath0):
        with open(bpath0) as f:
            lines0 = [l for l in f if l.startswith("{")]
        bench_pre = json.loads(lines0[-1]) if lines0 else None
    timed_avg_us = timed_calls = per_search_us = None
    trace_path = os.path.join(args.prof, "trace", "run_kernel_trace.csv")
    if bench_pre and os.path.exists(trace_path):
        with open(trace_path) as f:
            rows = sorted(csv.DictReader(f), key=lambda r: int(r["Start_Timestamp"]))
        starts = [i for i, r in enumerate(rows) if is_search_start(r["Kernel_Name"])]
        warm = bench_pre.get("warmup", 0)
        if len(starts) > warm:
            tail = rows[starts[warm]:]
            d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tail if is_expand(r["Kernel_Name"])]
            if d:
                timed_avg_us = sum(d) / len(d) / 1e3
                timed_calls = len(d)
                per_search_us = sum(d) / bench_pre["steps"] / 1e3

    fetch = per_kernel(os.path.join(args.prof, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(args.prof, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    fk = [v for k, vs in fetch.items() if is_expand(k) for v in vs]
    wk = [v for k, vs in write.items() if is_expand(k) for v in vs]
    fetch_kib = sum(fk) / len(fk) if fk else 0.0
    write_kib = sum(wk) / len(wk) if wk else 0.0

    bench = None
    bpath = os.path.join(args.prof, "bench.json")
    if os.path.exists(bpath):
        with open(bpath) as f:
            lines = [l for l in f if l.startswith("{")]
        bench = json.loads(lines[-1]) if lines else None
    out = {
        "workload": args.workload,
        "kernel": "solo_kernel" if any("solo_kernel" in k for k in fetch) else "expand_kernel",
        "launches_fetch_pass": len(fk),
        "launches_write_pass": len(wk),
        "fetch_kib_per_launch_raw": fetch_kib,
        "write_kib_per_launch_raw": write_kib,
        "hbm_bytes_per_launch_raw": (fetch_kib + write_kib) * 1024,
        "hbm_bytes_per_launch": (2 * fetch_kib + write_kib) * 1024,
        "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), KiB -> bytes; reads are mostly "
                      "8-32 B gathers, uncalibrated: read side is an upper bound",
        "rocprof_avg_expand_us": rocprof_avg_us,
        "rocprof_expand_calls": calls,
        "rocprof_avg_expand_us_timed_searches": timed_avg_us,
        "rocprof_expand_calls_timed_searches": timed_calls,
        "rocprof_expand_us_per_search_timed": per_search_us,
        "commit": args.commit,
        "cmd": args.cmd,
        "kernel_stats": os.path.relpath(stats_dst, ROOT),
    }
    if bench:
        rl = bench["roofline"]
        out["bench_avg_launch_us"] = rl["avg_launch_us"]
        out["bench_algorithmic_bytes_per_launch"] = rl["achieved"] * 1e9 * rl["avg_launch_us"] * 1e-6
        out["bench_launches"] = rl["launches"]
    with open(os.path.join(ROOT, "profiles", "pmc_%s.json" % args.workload), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

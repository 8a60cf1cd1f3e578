#!/usr/bin/env python3
"""Per-kernel mean duration over the bench's TIMED launches, from a rocprofv3 kernel trace.

bench.py runs W warmup steps, K timed steps and (with --overlap on) 8 unmeasured + 9 measured solo steps, so
rocprof's --stats average mixes overlapped and solo launches of the same kernel.  This splits a
kernel's launches in order: per_step launches per step, the first W*per_step are warmup, the
next K*per_step timed, the rest solo.
usage: trace_timed_avg.py kernel_trace.csv --warmup W --steps K [--kernel SUBSTR --per-step P]
"""
import argparse
import csv
import json

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--warmup", type=int, default=3)
ap.add_argument("--steps", type=int, default=10)
ap.add_argument("--kernel", action="append",
                default=None, help="kernel-name substring (repeatable)")
ap.add_argument("--per-step", type=int, default=1)
ap.add_argument("--solo-skip", type=int, default=8,
                help="unmeasured solo pairs before the measured ones (bench.py SOLO_WARM)")
a = ap.parse_args()
kernels = a.kernel or ["rs2_decode_kernel", "leaf_hash_kernel", "merkle_trees_kernel"]
rows = list(csv.DictReader(open(a.trace)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
out = {}
for k in kernels:
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
         for r in rows if k in r["Kernel_Name"]]
    ps = 2 if k == "leaf_hash_kernel" and a.per_step == 1 else a.per_step  # runs A and C
    w, t = a.warmup * ps, a.steps * ps
    timed, solo = d[w:w + t], d[w + t + a.solo_skip * ps:]
    out[k] = {"launches": len(d),
              "all_mean_ms": round(sum(d) / len(d), 4) if d else None,
              "timed_mean_ms": round(sum(timed) / len(timed), 4) if timed else None,
              "solo_mean_ms": round(sum(solo) / len(solo), 4) if solo else None,
              "solo_median_ms": round(sorted(solo)[len(solo) // 2], 4) if solo else None}
print(json.dumps(out, indent=1))

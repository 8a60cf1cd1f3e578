#!/usr/bin/env python3
"""How busy the GPU is over a bench run's timed region, from a rocprofv3 kernel trace.

    python3 tools/trace_busy.py KERNEL_TRACE.csv [--warmup 5] [--steps 30]

The timed region is taken from the decode launches (one per step): from 2 ms before the
(warmup+1)-th decode starts to the end of the (warmup+steps)-th.  Over that span it reports the
time with no kernel running at all, with only small launches (< 256 workgroups, fewer than one per CU) running, and with
exactly one large launch running.  Idle time near zero means the step is bounded by the kernels'
CU-time, not by launch gaps or host issue.
"""
import argparse
import csv
import json


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=30)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    dec = [r for r in rows if "decode_kernel" in r["Kernel_Name"]]
    t0 = int(dec[a.warmup]["Start_Timestamp"]) - 2_000_000
    t1 = int(dec[a.warmup + a.steps - 1]["End_Timestamp"])
    ev = []
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if e < t0 or s > t1:
            continue
        wgs = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        big = wgs >= 256
        ev += [(max(s, t0), 1, big), (min(e, t1), -1, big)]
    ev.sort()
    n_big = n_small = 0
    last = t0
    idle = small_only = one_big = 0
    for t, d, big in ev:
        dt = t - last
        if n_big == 0 and n_small == 0:
            idle += dt
        elif n_big == 0:
            small_only += dt
        elif n_big == 1:
            one_big += dt
        last = t
        if big:
            n_big += d
        else:
            n_small += d
    span = t1 - t0
    print(json.dumps({
        "span_ms": round(span / 1e6, 3),
        "idle_ms": round(idle / 1e6, 3),
        "idle_frac": round(idle / span, 5),
        "small_launches_only_ms": round(small_only / 1e6, 3),
        "one_large_launch_ms": round(one_big / 1e6, 3),
        "one_large_launch_frac": round(one_big / span, 4),
    }, indent=1))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Summarise an RS2_HOST_TRACE file (rs2_engine.cpp host_trace) and the bench line beside it:
per section the call count, mean, max and the calls above a threshold (index, ms)."""
import collections
import json
import sys


def main(trace, bench=None, thr=0.3):
    if bench:
        d = json.loads(open(bench).read().strip().splitlines()[-1])
        print(bench, d["value"], d["ms_per_step"], d.get("host_issue_ms_per_step"))
        print({k: v for k, v in d["stages_ms_per_step"].items() if "host" in k or "dec" in k})
    by = collections.defaultdict(list)
    for line in open(trace):
        name, v = line.split()
        by[name].append(float(v))
    for name, v in by.items():
        big = [(i, round(x, 3)) for i, x in enumerate(v) if x > thr]
        print(f"  {name:22s} n={len(v):5d} mean={sum(v) / len(v):.4f} max={max(v):.3f} "
              f"big={big[:8]}")


if __name__ == "__main__":
    main(*sys.argv[1:3])

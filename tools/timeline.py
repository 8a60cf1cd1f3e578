"""Per-step kernel timeline from a rocprofv3 --kernel-trace CSV (bench.py's step loop).

usage: python tools/timeline.py KERNEL_TRACE_CSV [first_kernel_substring] [steps_to_show]

Splits the trace into steps at each dispatch of the first kernel (default: the column codec of
the step), then prints for a few late steps every kernel's start / end relative to the step
start (us) and the step's idle time (no kernel running), and the mean over all steps."""
import csv
import sys


def main(path, first="rs2_encode_shared_pipe", show=3):
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                 for r in rows), key=lambda x: x[0])
    starts = [i for i, k in enumerate(ks) if first in k[2]]
    steps = []
    for a, b in zip(starts, starts[1:]):
        steps.append(ks[a:b])
    if not steps:
        print("no steps found")
        return
    idle_all, span_all = [], []
    for si, st in enumerate(steps):
        t0 = st[0][0]
        t_end = max(k[1] for k in st)
        iv = sorted((k[0], k[1]) for k in st)
        busy, cur_s, cur_e = 0, iv[0][0], iv[0][1]
        for s, e in iv[1:]:
            if s > cur_e:
                busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        idle_all.append((t_end - t0) - busy)
        span_all.append(t_end - t0)
        if si >= len(steps) - show:
            print(f"== step {si}: span {(t_end - t0) / 1e3:.1f} us, idle {((t_end - t0) - busy) / 1e3:.1f} us")
            for s, e, name in st:
                print(f"   {(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:8.1f}  {name[:90]}")
    n = len(span_all)
    print(f"steps {n}: mean span {sum(span_all) / n / 1e3:.1f} us, mean idle {sum(idle_all) / n / 1e3:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3]), *([int(sys.argv[3])] if len(sys.argv) > 3 else []))

#!/usr/bin/env python3
"""The bench's decode alone, repeated (profiling target: kernel traces, PMC passes, phase stamps).

One 256 MiB blob at n = 1000 is encoded once; then the primary decode from a seeded random K_p
subset runs `--reps` times on one stream (--fresh: a new subset each call).  Prints one JSON line
with the mean decode time.  usage: python3 tools/dec_only.py [--reps 50] [--fresh]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--fresh", action="store_true")
    ap.add_argument("--blob-mib", type=float, default=256.0)
    args = ap.parse_args()
    import numpy as np
    import torch
    import walrus_amd as W
    n = 1000
    blob_len = int(args.blob_mib * (1 << 20))
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(42)
    blob = torch.randint(0, 256, (blob_len,), dtype=torch.uint8, device=dev, generator=g)
    plan = W.DevicePlan(n, blob_len)
    info = plan.info
    pl, kp = info.primary_sliver_len, info.n_primary
    prim = torch.empty(n * pl + 256, dtype=torch.uint8, device=dev)
    sec = torch.empty(n * info.secondary_sliver_len + 256, dtype=torch.uint8, device=dev)
    hashes = torch.empty(n * 64, dtype=torch.uint8, device=dev)
    bid = torch.empty(32, dtype=torch.uint8, device=dev)
    out = torch.empty_like(blob)
    st = torch.cuda.current_stream(dev).cuda_stream
    plan.encode_async(blob.data_ptr(), prim.data_ptr(), sec.data_ptr(), hashes.data_ptr(),
                      bid.data_ptr(), st)
    rng = np.random.default_rng(42)
    subs = [[int(i) for i in rng.permutation(n)[:kp]]
            for _ in range(args.reps + 1 if args.fresh else 1)]
    k = [0]

    def dec():
        sel = subs[k[0] % len(subs)]
        k[0] += 1
        plan.decode_async("primary", sel, prim.data_ptr(), [i * pl for i in sel],
                          out.data_ptr(), st)
    dec()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        dec()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.reps
    print(json.dumps({"decode_ms": round(dt * 1e3, 4), "reps": args.reps, "fresh": args.fresh,
                      "ok": bool(torch.equal(out, blob))}))


if __name__ == "__main__":
    main()

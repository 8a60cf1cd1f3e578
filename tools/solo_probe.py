#!/usr/bin/env python3
"""Why does the bench's solo decode (roofline.solo) read slower than its C2 leg?  (VERDICT r05
weak #4.)  The decode kernel's own duration (the plan's dec_codec stage events) and the wall
time per call, for the same 256 MiB blob at n = 1000, in the situations the two bench figures
come from and a few that separate their differences:

  c2_cached      back-to-back decodes of one subset (bench c1_c2_leg c2_decode_random)
  c2_fresh       back-to-back decodes, a fresh subset per call (c2_decode_random_fresh)
  after_encode   encode, then decode from a fresh subset, repeated (the bench's solo pass)
  after_flush    a 2 GiB device write, then decode of one subset (cold L2 / MALL)
  after_flush_f  the same with fresh subsets
  after_sync     back-to-back decodes of one subset with a host synchronize between calls

usage: python3 tools/solo_probe.py [--reps 12]   -> one JSON line
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
    ap.add_argument("--reps", type=int, default=12)
    args = ap.parse_args()
    import numpy as np
    import torch
    import walrus_amd as W
    n, blob_len = 1000, 256 << 20
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
    flush = torch.empty(2 << 30, dtype=torch.uint8, device=dev)
    ts = torch.cuda.Stream(dev)
    st = ts.cuda_stream
    rng = np.random.default_rng(7)
    fixed = [int(i) for i in rng.permutation(n)[:kp]]

    def fresh():
        return [int(i) for i in rng.permutation(n)[:kp]]

    def enc():
        plan.encode_async(blob.data_ptr(), prim.data_ptr(), sec.data_ptr(), hashes.data_ptr(),
                          bid.data_ptr(), st)

    def dec(sel):
        plan.decode_async("primary", sel, prim.data_ptr(), [i * pl for i in sel],
                          out.data_ptr(), st)

    def do_flush():
        with torch.cuda.stream(ts):
            flush.fill_(1)

    enc()
    torch.cuda.synchronize()
    res = {}

    def run(name, body, sync_each=False):
        dec(fixed)  # warm the plan
        torch.cuda.synchronize()
        plan.profile(True)
        t0 = time.perf_counter()
        for _ in range(args.reps):
            body()
            if sync_each:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / args.reps
        st_ = plan.profile_read()
        plan.profile(False)
        ms, k = st_.get("dec_codec", (0.0, 1))
        res[name] = {"dec_codec_ms": round(ms / max(k, 1), 4), "wall_ms_per_call": round(wall * 1e3, 4),
                     "launches": k}
        if "enc_cols_sys_codec" in st_:
            res[name]["enc_stages_ms"] = {kk: round(v[0] / max(v[1], 1), 4)
                                          for kk, v in st_.items() if kk.startswith("enc_")}

    run("c2_cached", lambda: dec(fixed))
    run("c2_fresh", lambda: dec(fresh()))
    run("after_encode", lambda: (enc(), dec(fresh())))
    run("after_encode_cached", lambda: (enc(), dec(fixed)))
    run("after_flush", lambda: (do_flush(), dec(fixed)))
    run("after_flush_f", lambda: (do_flush(), dec(fresh())))
    run("after_sync", lambda: dec(fixed), sync_each=True)
    run("c2_cached_again", lambda: dec(fixed))
    ok = bool(torch.equal(out, blob))
    print(json.dumps({"probe": "solo decode", "reps": args.reps, "ok": ok, **res}), flush=True)


if __name__ == "__main__":
    main()

"""C2 decode_and_verify (Default check) on device slivers, a few calls, for a rocprofv3 kernel
trace: where the Default check's time goes.  usage: python tools/prof_c2_default.py [check]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import walrus_amd as W  # noqa: E402


def main(check="default", stream_mode="torch"):
    n, blob_len = 1000, 256 << 20
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(42)
    blob = torch.randint(0, 256, (blob_len,), dtype=torch.uint8, device=dev, generator=g)
    plan = W.DevicePlan(n, blob_len)
    info = plan.info
    pl = info.primary_sliver_len
    prim = torch.empty(n * pl + 256, dtype=torch.uint8, device=dev)
    sec = torch.empty(n * info.secondary_sliver_len + 256, dtype=torch.uint8, device=dev)
    hashes = torch.empty(n * 64, dtype=torch.uint8, device=dev)
    bid = torch.empty(32, dtype=torch.uint8, device=dev)
    out = torch.empty_like(blob)
    ts = torch.cuda.Stream(dev)
    st = ts.cuda_stream if stream_mode == "torch" else 0  # 0: the plan's own stream
    plan.encode_async(blob.data_ptr(), prim.data_ptr(), sec.data_ptr(), hashes.data_ptr(),
                      bid.data_ptr(), st)
    torch.cuda.synchronize()
    idx = [int(i) for i in np.random.default_rng(42).permutation(n)[:info.n_primary]]
    offs = [i * pl for i in idx]
    h_meta, h_id = bytes(hashes.cpu().numpy()), bytes(bid.cpu().numpy())
    plan.decode_async("primary", idx, prim.data_ptr(), offs, out.data_ptr(), st)
    torch.cuda.synchronize()
    print("plain decode ok", bool(torch.equal(out, blob)), flush=True)
    for k in range(6):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        try:
            plan.decode_and_verify("primary", idx, prim.data_ptr(), offs, h_meta, h_id, check,
                                   out.data_ptr(), st)
        except Exception as e:  # noqa: BLE001
            print("verify failed:", e, flush=True)
        torch.cuda.synchronize()
        print(f"call {k}: {(time.perf_counter() - t0) * 1e3:.3f} ms", flush=True)
    print("ok", bool(torch.equal(out, blob)))


if __name__ == "__main__":
    main(*sys.argv[1:3])

#!/usr/bin/env python3
"""C3 diagnosis: per-stage times of one 4 MiB blob encode (n=1000, s=20), and batch time of 16
blobs over S streams."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import walrus_amd as W  # noqa: E402

dev = torch.device("cuda", 0)
n, blob_len, blobs = 1000, 4 << 20, 16
plans = [W.DevicePlan(n, blob_len) for _ in range(blobs)]
info = plans[0].info
g = torch.Generator(device=dev)
g.manual_seed(3)
bufs = [dict(blob=torch.randint(0, 256, (blob_len,), dtype=torch.uint8, device=dev, generator=g),
             prim=torch.empty(n * info.primary_sliver_len + 256, dtype=torch.uint8, device=dev),
             sec=torch.empty(n * info.secondary_sliver_len + 256, dtype=torch.uint8, device=dev),
             hashes=torch.empty(n * 64 + 32, dtype=torch.uint8, device=dev)) for _ in range(blobs)]
st = torch.cuda.current_stream(dev).cuda_stream


def enc(P, b, s):
    P.encode_async(b["blob"].data_ptr(), b["prim"].data_ptr(), b["sec"].data_ptr(),
                   b["hashes"].data_ptr(), b["hashes"][n * 64:].data_ptr(), s)


P = plans[0]
for _ in range(3):
    enc(P, bufs[0], st)
torch.cuda.synchronize()
P.profile(True)
for _ in range(5):
    enc(P, bufs[0], st)
torch.cuda.synchronize()
stages = P.profile_read()
P.profile(False)
print("stages ms/launch:", {k: round(v[0] / max(v[1], 1), 4) for k, v in stages.items()})
for S in (1, 2, 4, 8, 16):
    streams = [torch.cuda.Stream(dev) for _ in range(S)]
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(blobs):
            enc(plans[i], bufs[i], streams[i % S].cuda_stream)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    print(f"streams={S}: {dt*1e3:.3f} ms/batch, {blobs*blob_len/(1<<30)/dt:.2f} GiB/s", flush=True)

"""One 256 MiB n=1000 encode + primary decode (random K_p subset) through the stamp-instrumented
library (walrus_amd/libwalrus_rs2_stamps.so, `make -C walrus_amd/csrc stamps`), writing the
phase stamps of every codec launch to $RS2_STAMP_FILE.  Diagnostic only.

usage: RS2_STAMP_FILE=gpurun_out/stamps.bin python tools/stamps_run.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("WALRUS_RS2_LIB", os.path.join(ROOT, "walrus_amd", "libwalrus_rs2_stamps.so"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import walrus_amd as W  # noqa: E402


def main():
    n, blob_len = 1000, 256 << 20
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    blob = torch.randint(0, 256, (blob_len,), dtype=torch.uint8, device=dev, generator=g)
    plan = W.DevicePlan(n, blob_len)
    info = plan.info
    pl = info.primary_sliver_len
    prim = torch.empty(n * pl + 256, dtype=torch.uint8, device=dev)
    sec = torch.empty(n * info.secondary_sliver_len + 256, dtype=torch.uint8, device=dev)
    meta = torch.empty(n * 64 + 32, dtype=torch.uint8, device=dev)
    out = torch.empty_like(blob)
    idx = [int(i) for i in np.random.default_rng(42).permutation(n)[:info.n_primary]]
    st = torch.cuda.current_stream(dev).cuda_stream
    plan.encode_async(blob.data_ptr(), prim.data_ptr(), sec.data_ptr(), meta.data_ptr(),
                      meta[n * 64:].data_ptr(), st)
    plan.decode_async("primary", idx, prim.data_ptr(), [i * pl for i in idx], out.data_ptr(), st)
    torch.cuda.synchronize()
    print("decode ok:", bool(torch.equal(out, blob)))


if __name__ == "__main__":
    main()

"""C3's 128 x 4 MiB blobs through one batched encode, 5 times (for rocprofv3 --stats)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import walrus_amd as W  # noqa: E402


def main():
    n, blob_len, nb = 1000, 4 << 20, 128
    dev = torch.device("cuda", 0)
    plan = W.DevicePlan(n, blob_len)
    info = plan.info
    pl, sl = info.primary_sliver_len, info.secondary_sliver_len
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    blobs = torch.randint(0, 256, (nb, blob_len), dtype=torch.uint8, device=dev, generator=g)
    prim = torch.empty((nb, n * pl), dtype=torch.uint8, device=dev)
    sec = torch.empty((nb, n * sl), dtype=torch.uint8, device=dev)
    hashes = torch.empty((nb, n * 64), dtype=torch.uint8, device=dev)
    ids = torch.empty((nb, 32), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(5):
        plan.encode_batch_async(nb, blobs.data_ptr(), blob_len, None, prim.data_ptr(), n * pl,
                                sec.data_ptr(), n * sl, hashes.data_ptr(), ids.data_ptr(), st)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()

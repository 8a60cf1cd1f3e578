"""Diagnose large-blob decode mismatches: encode a blob of each given size on the device,
decode it from a random and from the worst-case K_p primary subset, and print where the
decoded bytes differ (row / column / byte in symbol)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import walrus_amd as W  # noqa: E402


def run(length, n=1000):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    blob = torch.randint(0, 256, (length,), dtype=torch.uint8, device=dev, generator=g)
    plan = W.DevicePlan(n, length)
    info = plan.info
    kp, ks, s, pl = info.n_primary, info.n_secondary, info.symbol_size, info.primary_sliver_len
    prim = torch.empty(n * pl + 256, dtype=torch.uint8, device=dev)
    sec = torch.empty(n * info.secondary_sliver_len + 256, dtype=torch.uint8, device=dev)
    meta = torch.empty(n * 64 + 32, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    plan.encode_async(blob.data_ptr(), prim.data_ptr(), sec.data_ptr(), meta.data_ptr(),
                      meta[n * 64:].data_ptr(), st)
    out = torch.empty_like(blob)
    for name, idx in (("random", [int(i) for i in np.random.default_rng(42).permutation(n)[:kp]]),
                      ("worst", list(range(kp, 2 * kp))),
                      ("systematic", list(range(kp)))):
        out.fill_(0xEE)
        plan.decode_async("primary", idx, prim.data_ptr(), [i * pl for i in idx], out.data_ptr(), st)
        torch.cuda.synchronize()
        diff = out != blob
        row = ks * s
        parts = []
        for r in range((length + row - 1) // row):
            seg = diff[r * row:(r + 1) * row]
            if bool(seg.any()):
                parts.append(seg.nonzero().flatten().cpu().numpy() + r * row)
        b = np.concatenate(parts) if parts else np.zeros(0, dtype=np.int64)
        msg = f"len={length} s={s} {name}: {b.size} bad bytes"
        if b.size:
            rows = b // (ks * s)
            cols = (b % (ks * s)) // s
            pos = b % s
            msg += (f"; rows {rows.min()}..{rows.max()} ({len(np.unique(rows))}), cols "
                    f"{cols.min()}..{cols.max()} ({len(np.unique(cols))}), in-symbol bytes "
                    f"{pos.min()}..{pos.max()}; first {b[:4]}; got "
                    f"{out[int(b[0]):int(b[0]) + 8].tolist()} want {blob[int(b[0]):int(b[0]) + 8].tolist()}")
            torch.cuda.synchronize()
            import time
            time.sleep(0.5)
            msg += f"; after 0.5 s: {int((out != blob).sum())} bad"
            # rerun the same decode and check again
            out.fill_(0xEE)
            plan.decode_async("primary", idx, prim.data_ptr(), [i * pl for i in idx], out.data_ptr(), st)
            plan.sync(st)
            torch.cuda.synchronize()
            msg += f"; rerun: {int((out != blob).sum())} bad"
            cnt = torch.zeros(1, dtype=torch.int64, device=dev)
            msg += f"; bad==0xEE: {int(((out != blob) & (out == 0xEE)).sum())}"
        print(msg, flush=True)
    del prim, sec, out, blob
    torch.cuda.empty_cache()


if __name__ == "__main__":
    for arg in sys.argv[1:]:
        run(int(eval(arg)))

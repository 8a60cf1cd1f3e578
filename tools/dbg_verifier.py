import sys, os
sys.path[:0] = ["/root/repo", "/root/repo/oracle", os.environ.get("GRAFT_REPO_ROOT", "") + "/oracle"]
import numpy as np, torch
import walrus_amd as W
import rs2_oracle as O
dev = torch.device("cuda", 0)
for n, s, count in [(13, 112, 1), (13, 112, 3), (13, 200, 2), (40, 64, 4), (100, 1206, 3)]:
    kp, ks = O.source_symbols_for_n_shards(n)
    K = ks  # primary slivers: K_s symbols
    rng = np.random.default_rng(n * 1000 + s)
    data = rng.integers(0, 256, (count, K * s), dtype=np.uint8)
    want = []
    for r in range(count):
        syms = data[r].reshape(K, s)
        allsym = O.rs_encode_all(syms, n)
        want.append(O.merkle_root([bytes(x) for x in allsym]))
    v = W.SliverVerifier(n, s, "primary")
    d = torch.from_numpy(data.reshape(-1).copy()).to(dev)
    out = torch.zeros(count * 32, dtype=torch.uint8, device=dev)
    v.roots_async(count, d.data_ptr(), out.data_ptr())
    torch.cuda.synchronize()
    got = [bytes(out[32 * i:32 * i + 32].cpu().numpy()) for i in range(count)]
    print(n, s, count, [g == w for g, w in zip(got, want)], flush=True)

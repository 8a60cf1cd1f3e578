"""Stage-by-stage comparison of the HIP engine with the oracle (debug aid)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'oracle'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
import numpy as np
import rs2_oracle as O
import walrus_amd as W

def check(n, blob):
    ref = O.encode_with_metadata(blob, n)
    cfg = W.ReedSolomonEncodingConfig(n)
    pairs, meta = cfg.encode_with_metadata(blob)
    p = ref.params
    print(f"n={n} B={len(blob)} kp={p.n_primary} ks={p.n_secondary} s={p.symbol_size}")
    bad_p = [i for i in range(n) if pairs[i].primary.symbols.data != ref.primary[i].tobytes()]
    bad_s = [j for j in range(n) if pairs[n-1-j].secondary.symbols.data != ref.secondary[j].tobytes()]
    print("  bad primary slivers:", bad_p[:20], len(bad_p))
    print("  bad secondary slivers:", bad_s[:20], len(bad_s))
    if bad_p:
        i = bad_p[0]
        print("   prim", i, "gpu", pairs[i].primary.symbols.data[:16].hex(), "ref", ref.primary[i].tobytes()[:16].hex())
    if bad_s:
        j = bad_s[0]
        print("   sec", j, "gpu", pairs[n-1-j].secondary.symbols.data[:16].hex(), "ref", ref.secondary[j].tobytes()[:16].hex())
    hb = [h for h in meta.metadata.hashes]
    badh = [i for i in range(n) if hb[i] != ref.pair_hashes[i]]
    print("  bad pair hashes:", badh[:10], len(badh))
    if badh:
        i = badh[0]
        print("   gpu", hb[i][0].hex()[:16], hb[i][1].hex()[:16], "ref", ref.pair_hashes[i][0].hex()[:16], ref.pair_hashes[i][1].hex()[:16])
    print("  blob id gpu", str(meta.blob_id), "ref", O.blob_id_to_str(ref.blob_id))
    # host utility check of the root from the GPU's own hashes
    print("  root(host utility over gpu hashes) == gpu id:", meta.metadata.compute_blob_id() == meta.blob_id)
    print("  oracle blob_id over gpu hashes == gpu id:", O.blob_id(hb, len(blob)) == bytes(meta.blob_id))

def check_1d(k, n, s):
    rng = np.random.default_rng(k*100+n)
    data = rng.integers(0, 256, k*s, dtype=np.uint8)
    ref = O.rs_encode_all(data.reshape(k, s), n).reshape(-1)
    enc = W.ReedSolomonEncoder(s, k, n)
    got = np.frombuffer(enc.encode_all(data.tobytes()).data, dtype=np.uint8)
    bad = [i for i in range(n) if not (got[i*s:(i+1)*s] == ref[i*s:(i+1)*s]).all()]
    print(f"1d k={k} n={n} s={s} high={O.use_high_rate(k, n-k)} bad symbols: {bad[:10]} ({len(bad)})")

for k, n, s in [(4, 10, 2), (7, 10, 2), (3, 4, 2), (2, 4, 2), (4, 10, 64), (7, 10, 128), (4, 10, 130), (69, 102, 8), (36, 102, 8), (334, 1000, 4), (667, 1000, 4)]:
    check_1d(k, n, s)
check(10, b"walrus blob id v1 regression test")
check(10, bytes(range(256)) * 4)

"""Generate tests/golden/rs2_fullsize.json: digests of full-size encodes by the C restatement.

The C/AVX2 restatement (oracle/rs2_cpu.c) reproduces every case of rs2_fixtures.json bit for bit
(tests/test_cpu_port.py), and those fixtures are pinned by the reference's only codeword-level
golden vector (test_v1_blob_id_stability, crates/walrus-core/src/encoding/blob_encoding.rs:
1227-1244).  This script runs it on the BASELINE.json configurations at their full sizes --
shapes the reference's own criterion harness encodes (crates/walrus-core/benches/
blob_encoding.rs:35-122, 1 B ... 1 GiB at n=1000) but never pins -- and records, per case:

  blob_id, all n pair hashes (metadata.rs:611-643), and a SHA-256 (first 16 bytes) of every
  primary and secondary sliver (by sliver index).

Blobs are `blob_bytes(seed, length)`: PCG64 raw words, so the GPU tests regenerate the same
bytes without storing them.  Test infrastructure only (the product never imports oracle/).
Run (about 2 minutes, 25 GB RAM for the 4 GiB case):  python tests/golden/make_fullsize.py [names]
"""
import ctypes
import hashlib
import json
import os
import subprocess
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))

# (name, n_shards, blob bytes, seed, what it exercises)
CASES = [
    ("c0_n10_1MiB", 10, 1 << 20, 100,
     "BASELINE config C0: s=37450 = 585 chunks + 10-byte tail"),
    ("smax_n10", 10, 28 * 65534 - 7, 105,
     "largest symbol size (65534 = 1023 chunks + 62-byte tail), n=10"),
    ("smax_n100", 100, 34 * 67 * 65534 - 1001, 106,
     "largest symbol size at n=100 (64/128-point transforms)"),
    ("c3_n1000_4MiB", 1000, 4 << 20, 103,
     "BASELINE config C3's blob: s=20 (tail only)"),
    ("c1_n1000_256MiB", 1000, 256 << 20, 101,
     "BASELINE configs C1/C2 (the bench metric's shape): s=1206 = 18 chunks + 54-byte tail"),
    ("c4_n1000_4GiB", 1000, 4 << 30, 104,
     "BASELINE config C4: s=19280 = 301 chunks + 16-byte tail"),
    # n_shards above 2048 (the reference takes any NonZeroU16, config.rs:446-460); compact
    # records (SHA-256 over all pair hashes / all primary / all secondary slivers)
    ("large_n2049", 2049, 3 << 20, 107,
     "n=2049 (K_p=685, K_s=1367): 4096-point low-rate columns, 4096-leaf trees"),
    ("large_n3001", 3001, 40 << 20, 108,
     "n=3001 (K_p=1001, K_s=2001), s=22"),
    ("large_n4096", 4096, 16 << 20, 109,
     "n=4096 (K_p=1366, K_s=2731): 8192-point transforms (16 blocks of 512), s=6"),
    # above the one-workgroup tree bound (the trees' first level in a kernel of its own)
    ("large_n4500", 4500, 4 << 20, 111,
     "n=4500 (K_p=1502, K_s=3001): 4,500-leaf trees, s=2"),
    ("large_n6000", 6000, 24 << 20, 112,
     "n=6000 (K_p=2002, K_s=4001): 6,000-leaf trees, 8192-point decodes on both axes, "
     "high-rate columns (the rate tie 4096 = 4096), s=4"),
    # above two levels of the one-workgroup tree bound, 16384-point transforms (32 blocks)
    ("large_n10000", 10000, 40 << 20, 113,
     "n=10000 (K_p=3334, K_s=6667): 10,000-leaf trees (two levels in their own kernels), "
     "16384-point decodes on both axes, s=2"),
    # the largest n this build takes: 32768-point decodes on both axes (64 blocks of 512)
    ("large_n16384", 16384, 64 << 20, 114,
     "n=16384 (K_p=5462, K_s=10923): 16,384-leaf trees, 32768-point decodes on both axes, s=2"),
    # config C4's shape (n=1000, one blob row/column-partitioned over ranks) at a size two
    # processes sharing one GPU encode in seconds (tests/test_gpu_dist.py)
    ("c4s_n1000_24MiB", 1000, 24 << 20, 110,
     "C4's partitioned encode/decode over 2 processes on one GPU: s=114 = 1 chunk + 50-byte tail"),
]
COMPACT_ABOVE = 1000  # n_shards above this: compact digests
COMPACT = {"c4s_n1000_24MiB"}  # compact digests at any n


def blob_bytes(seed: int, length: int) -> np.ndarray:
    """Deterministic synthetic blob (numpy PCG64 raw 64-bit words, little endian)."""
    words = np.random.PCG64(seed).random_raw((length + 7) // 8)
    return words.view(np.uint8)[:length]


def sliver_digest(data) -> str:
    return hashlib.sha256(data).hexdigest()[:32]


def load_cpu():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "librs2cpu.so"))
    P = ctypes.c_void_p
    lib.rs2cpu_encode.argtypes = [ctypes.c_uint32, P, ctypes.c_uint64, P, P, P, P]
    lib.rs2cpu_params.argtypes = [ctypes.c_uint32, ctypes.c_uint64] + [P] * 3
    return lib


def encode_case(lib, n, length, seed, compact=False):
    kp, ks, s = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    lib.rs2cpu_params(n, length, ctypes.byref(kp), ctypes.byref(ks), ctypes.byref(s))
    kp, ks, s = kp.value, ks.value, s.value
    blob = blob_bytes(seed, length)
    prim = np.empty((n, ks * s), dtype=np.uint8)
    sec = np.empty((n, kp * s), dtype=np.uint8)
    hashes = np.empty(n * 64, dtype=np.uint8)
    bid = np.empty(32, dtype=np.uint8)
    t0 = time.time()
    lib.rs2cpu_encode(n, blob.ctypes.data, length, prim.ctypes.data, sec.ctypes.data,
                      hashes.ctypes.data, bid.ctypes.data)
    dt = time.time() - t0
    import base64
    h = hashes.tobytes()
    case = {
        "n_shards": n, "blob_len": length, "seed": seed,
        "n_primary": kp, "n_secondary": ks, "symbol_size": s,
        "blob_id": base64.urlsafe_b64encode(bid.tobytes()).decode().rstrip("="),
    }
    if n > COMPACT_ABOVE or compact:
        case.update({"pair_hashes_sha256": hashlib.sha256(h).hexdigest(),
                     "primary_all_sha256": hashlib.sha256(prim.tobytes()).hexdigest(),
                     "secondary_all_sha256": hashlib.sha256(sec.tobytes()).hexdigest()})
    else:
        case.update({"pair_hashes": [h[64 * i:64 * i + 64].hex() for i in range(n)],
                     "primary_sha256_16": [sliver_digest(prim[i]) for i in range(n)],
                     "secondary_sha256_16": [sliver_digest(sec[j]) for j in range(n)]})
    return case, dt


def main(names=None):
    lib = load_cpu()
    out_path = os.path.join(HERE, "rs2_fullsize.json")
    old = {}
    if os.path.exists(out_path):
        with open(out_path) as f:
            old = {c["name"]: c for c in json.load(f)["cases"]}
    cases = []
    for name, n, length, seed, what in CASES:
        if names and name not in names and name in old:
            cases.append(old[name])
            continue
        case, dt = encode_case(lib, n, length, seed, name in COMPACT)
        case = {"name": name, "what": what, **case}
        cases.append(case)
        print(f"{name}: s={case['symbol_size']} blob_id={case['blob_id']} ({dt:.1f} s)",
              flush=True)
    with open(out_path, "w") as f:
        json.dump({"generator": "tests/golden/make_fullsize.py (oracle/rs2_cpu.c, C restatement "
                                "pinned by tests/test_cpu_port.py)",
                   "blob": "numpy PCG64(seed).random_raw(ceil(len/8)) as little-endian bytes",
                   "cases": cases}, f, indent=0)


if __name__ == "__main__":
    main(set(sys.argv[1:]) or None)

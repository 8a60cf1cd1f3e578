"""Generate tests/golden/rs2_fixtures.json with the CPU oracle (oracle/rs2_oracle.py).

The oracle is pinned by the reference's only codeword-level golden vector
(test_v1_blob_id_stability, blob_encoding.rs:1227-1244), which is included as case 0.  The
other cases extend coverage to shapes the reference tests do not pin (full 64-byte chunks,
odd tails, rate ties, n=1000): they are fixtures of the restatement, re-checked against the
HIP engine by tests/test_gpu_parity.py.  Run: python tests/golden/make_fixtures.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import rs2_oracle as O  # noqa: E402

CASES = [
    # (name, n_shards, blob spec)
    ("golden_v1", 10, "walrus blob id v1 regression test"),
    ("n10_s2_1000", 10, ("rand", 1000, 1)),
    ("n10_s64", 10, ("rand", 4 * 7 * 64, 2)),         # exactly one full chunk per symbol
    ("n10_s66", 10, ("rand", 4 * 7 * 66 - 5, 3)),     # one chunk + 2-byte tail
    ("n10_s130", 10, ("rand", 4 * 7 * 130, 4)),       # two chunks + 2-byte tail, odd elements
    ("n10_s1206", 10, ("rand", 4 * 7 * 1206 - 11, 5)),  # the n=1000 symbol-size layout
    ("n11_tie", 11, ("rand", 3000, 6)),               # column code rate tie (K=5, R=6)
    ("n13", 13, ("rand", 777, 7)),
    ("n102", 102, ("rand", 31415, 8)),
    ("n1000_tiny", 1000, ("rand", 1000, 9)),
    ("empty", 10, ("rand", 0, 10)),
    # the reference's second codeword-level vector, at mainnet's n = 1000 (s = 2): the publisher
    # example of docs/content/http-api/storing-blobs.mdx:114-127 (also
    # walrus-client/verifying-availability.mdx:111-115): `-d "some other string"` (17 B) ->
    # blobId M4hsZGQ1oCktdzegB6HnI6Mi28S2nqOPHxK-W7_4BUk, encodedLength 66,034,000.  It pins the
    # chunked n = 1000 transforms (512 + 155 row inputs, 512 + 154 column outputs).
    ("ref_some_other_string_n1000", 1000, "some other string"),
]

# BlobIds the reference itself publishes for a case (the generator refuses to drift from them)
REFERENCE_IDS = {
    "golden_v1": "RcU82Mwf-CFkv1LaI_2qcpANwpGUuG3TMwnVzZxD2kY",  # blob_encoding.rs:1227-1244
    "ref_some_other_string_n1000": "M4hsZGQ1oCktdzegB6HnI6Mi28S2nqOPHxK-W7_4BUk",
}


def blob_for(spec):
    if isinstance(spec, str):
        return spec.encode()
    _, length, seed = spec
    return np.random.default_rng(seed).integers(0, 256, length, dtype=np.uint8).tobytes()


def main():
    out = []
    for name, n, spec in CASES:
        blob = blob_for(spec)
        enc = O.encode_with_metadata(blob, n)
        p = enc.params
        case = {
            "name": name, "n_shards": n, "blob_len": len(blob),
            "blob": blob.hex() if isinstance(spec, str) else None,
            "blob_seed": None if isinstance(spec, str) else spec[2],
            "n_primary": p.n_primary, "n_secondary": p.n_secondary, "symbol_size": p.symbol_size,
            "blob_id": O.blob_id_to_str(enc.blob_id),
            "pair_hashes": [[a.hex(), b.hex()] for a, b in enc.pair_hashes],
            "primary_sha256": [hashlib.sha256(x.tobytes()).hexdigest() for x in enc.primary],
            "secondary_sha256": [hashlib.sha256(x.tobytes()).hexdigest() for x in enc.secondary],
        }
        if name in REFERENCE_IDS:
            assert case["blob_id"] == REFERENCE_IDS[name], (name, case["blob_id"])
        if n <= 13 and len(blob) <= 4000:
            case["primary"] = [x.tobytes().hex() for x in enc.primary]
            case["secondary"] = [x.tobytes().hex() for x in enc.secondary]
        out.append(case)
        print(name, case["blob_id"])
    with open(os.path.join(HERE, "rs2_fixtures.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_fixtures.py (oracle/rs2_oracle.py)",
                   "cases": out}, f, indent=0)


if __name__ == "__main__":
    main()

"""First GPU parity checks: the HIP engine against the CPU oracle (oracle/rs2_oracle.py)."""
import numpy as np
import pytest

import rs2_oracle as O

pytestmark = pytest.mark.gpu

GOLDEN_BLOB = b"walrus blob id v1 regression test"
GOLDEN_ID = "RcU82Mwf-CFkv1LaI_2qcpANwpGUuG3TMwnVzZxD2kY"  # blob_encoding.rs:1227-1244


def test_golden_blob_id(gpu):
    cfg = gpu.ReedSolomonEncodingConfig(10)
    pairs, meta = cfg.encode_with_metadata(GOLDEN_BLOB)
    assert str(meta.blob_id) == GOLDEN_ID


@pytest.mark.parametrize("n,blob_len", [(10, 33), (10, 1000), (10, 5000), (13, 777), (7, 100),
                                        (102, 31415), (102, 27182), (4, 10), (40, 100000),
                                        (300, 500000)])
def test_encode_matches_oracle(gpu, n, blob_len):
    rng = np.random.default_rng(n * 7 + blob_len)
    blob = rng.integers(0, 256, blob_len, dtype=np.uint8).tobytes()
    ref = O.encode_with_metadata(blob, n)
    cfg = gpu.ReedSolomonEncodingConfig(n)
    pairs, meta = cfg.encode_with_metadata(blob)
    for i, pair in enumerate(pairs):
        rp, rs = ref.sliver_pair(i)
        assert pair.primary.symbols.data == rp.tobytes(), f"primary {i}"
        assert pair.secondary.symbols.data == rs.tobytes(), f"secondary {n-1-i}"
    assert meta.metadata.hashes == ref.pair_hashes
    assert bytes(meta.blob_id) == ref.blob_id


@pytest.mark.parametrize("n,blob_len", [(10, 1000), (102, 31415), (13, 777), (300, 500000),
                                        (600, 2000000), (1000, 3000000), (11, 999), (21, 4096)])
def test_decode_both_axes(gpu, n, blob_len):
    rng = np.random.default_rng(blob_len)
    blob = rng.integers(0, 256, blob_len, dtype=np.uint8).tobytes()
    cfg = gpu.ReedSolomonEncodingConfig(n)
    pairs, meta = cfg.encode_with_metadata(blob)
    kp, ks = cfg.n_primary_source_symbols, cfg.n_secondary_source_symbols
    order = rng.permutation(n)
    prim = [pairs[i].primary for i in order]
    assert cfg.decode(blob_len, prim) == blob
    worst = [pairs[i].primary for i in range(n - 1, -1, -1)][:kp]
    assert cfg.decode(blob_len, worst) == blob
    sec = [pairs[n - 1 - i].secondary for i in order]
    assert cfg.decode(blob_len, sec) == blob

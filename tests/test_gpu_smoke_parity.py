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


REF_N1000_BLOB = b"some other string"
REF_N1000_ID = "M4hsZGQ1oCktdzegB6HnI6Mi28S2nqOPHxK-W7_4BUk"  # storing-blobs.mdx:114-127


def test_reference_publisher_example_n1000(gpu):
    """The reference's n = 1000 vector (docs/content/http-api/storing-blobs.mdx:114-139) through
    the host ABI (encode_with_metadata, compute_metadata, encoded_blob_length), the device plan
    (rs2_encode_device_async on torch buffers) and a decode from the worst-case subset."""
    import torch
    cfg = gpu.ReedSolomonEncodingConfig(1000)
    assert cfg.encoded_blob_length(len(REF_N1000_BLOB)) == 66_034_000
    pairs, meta = cfg.encode_with_metadata(REF_N1000_BLOB)
    assert str(meta.blob_id) == REF_N1000_ID
    assert str(cfg.compute_metadata(REF_N1000_BLOB).blob_id) == REF_N1000_ID
    assert meta.verify()

    plan = gpu.DevicePlan(1000, len(REF_N1000_BLOB))
    info = plan.info
    dev = torch.device("cuda:0")
    blob_t = torch.frombuffer(bytearray(REF_N1000_BLOB), dtype=torch.uint8).to(dev)
    prim = torch.empty(1000 * info.primary_sliver_len + 256, dtype=torch.uint8, device=dev)
    sec = torch.empty(1000 * info.secondary_sliver_len + 256, dtype=torch.uint8, device=dev)
    hashes = torch.empty(1000 * 64, dtype=torch.uint8, device=dev)
    bid = torch.empty(32, dtype=torch.uint8, device=dev)
    plan.encode_async(blob_t.data_ptr(), prim.data_ptr(), sec.data_ptr(), hashes.data_ptr(),
                      bid.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    assert str(gpu.BlobId(bytes(bid.cpu().numpy()))) == REF_N1000_ID
    assert bytes(hashes.cpu().numpy()) == meta.metadata.hashes_bytes()
    plen = info.primary_sliver_len
    host_prim = prim.cpu().numpy()
    for i in (0, 333, 334, 999):
        assert host_prim[i * plen:(i + 1) * plen].tobytes() == pairs[i].primary.symbols.data
    kp = cfg.n_primary_source_symbols
    assert cfg.decode(len(REF_N1000_BLOB),
                      [pairs[i].primary for i in range(999, 999 - kp, -1)]) == REF_N1000_BLOB


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

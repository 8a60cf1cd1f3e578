"""BlobEncoder::compute_metadata (blob_encoding.rs:406-486) on the device.

With the blob read in place (the fused systematic-column codec), compute_metadata writes no
systematic sliver at all: the primary slivers' leaves are hashed from the blob's whole rows,
the zero-padded tail rows and the repair rows (rs2_engine.cpp encode_device, meta_only).  The
pair hashes and BlobId must equal the full encode's (itself oracle-pinned) and, for small
shapes, the C restatement's, through the host ABI (rs2_compute_metadata) and the device entry
point (rs2_compute_metadata_device_async); Strict decode_and_verify re-derives metadata the
same way.
"""
import ctypes
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
from make_fullsize import load_cpu  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cpu():
    return load_cpu()


def _c_meta(cpu, n, blob):
    kp, ks, s = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    cpu.rs2cpu_params(n, len(blob), ctypes.byref(kp), ctypes.byref(ks), ctypes.byref(s))
    src = np.frombuffer(blob, dtype=np.uint8) if blob else np.zeros(1, dtype=np.uint8)
    prim = np.empty((n, ks.value * s.value), dtype=np.uint8)
    sec = np.empty((n, kp.value * s.value), dtype=np.uint8)
    hashes = np.empty(n * 64, dtype=np.uint8)
    bid = np.empty(32, dtype=np.uint8)
    cpu.rs2cpu_encode(n, src.ctypes.data, len(blob), prim.ctypes.data, sec.ctypes.data,
                      hashes.ctypes.data, bid.ctypes.data)
    return hashes.tobytes(), bid.tobytes()


# blobs that fill every row (r_full = K_p), end inside a row, leave whole zero rows, are tiny
# (s = 2, the unfused 2-byte path) and large enough for the split leaf launches (>= 64 MiB)
CASES = [(10, 28 * 50), (10, 28 * 50 - 7), (10, 1000), (10, 3), (13, 5000), (100, 70_000),
         (100, 1 << 20), (1000, 40_000), (1000, 3 << 20), (1000, 222_778 * 40),
         (1000, (64 << 20) + 12345)]


@pytest.mark.parametrize("n,length", CASES)
def test_compute_metadata_matches_encode(gpu, cpu, n, length):
    import torch
    blob = np.random.default_rng(n + length).integers(0, 256, length, dtype=np.uint8).tobytes()
    cfg = gpu.ReedSolomonEncodingConfig(n)
    meta = cfg.compute_metadata(blob)
    _, full = cfg.encode_with_metadata(blob)
    assert meta.blob_id == full.blob_id and meta.metadata == full.metadata
    if length <= 10 << 20:
        h, bid = _c_meta(cpu, n, blob)
        assert meta.metadata.hashes_bytes() == h and bytes(meta.blob_id) == bid
    # device entry point, twice (the plan's scratch reused), beside a plain device encode
    dev = torch.device("cuda", 0)
    d_blob = torch.from_numpy(np.frombuffer(blob, dtype=np.uint8).copy()).to(dev) if length \
        else torch.zeros(1, dtype=torch.uint8, device=dev)
    plan = gpu.DevicePlan(n, length)
    d_h = torch.zeros(n * 64, dtype=torch.uint8, device=dev)
    d_id = torch.zeros(32, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(2):
        plan.compute_metadata_async(d_blob.data_ptr(), d_h.data_ptr(), d_id.data_ptr(), st)
        torch.cuda.synchronize()
        assert bytes(d_h.cpu().numpy()) == full.metadata.hashes_bytes()
        assert bytes(d_id.cpu().numpy()) == bytes(full.blob_id)


def test_strict_check_uses_metadata_path(gpu):
    """Strict decode_and_verify (config.rs:613-658) re-derives the metadata of the decoded blob
    through the same metadata-only encode: a good decode passes, a corrupt received systematic
    sliver fails Strict."""
    n, length = 1000, 5_000_000
    blob = np.random.default_rng(3).integers(0, 256, length, dtype=np.uint8).tobytes()
    cfg = gpu.ReedSolomonEncodingConfig(n)
    pairs, meta = cfg.encode_with_metadata(blob)
    kp = cfg.n_primary_source_symbols
    good = [pairs[i].primary for i in range(kp)]
    assert cfg.decode_and_verify(meta, good, "strict") == blob
    bad = bytearray(good[5].symbols.data)
    bad[17] ^= 0x40
    good[5] = gpu.SliverData(gpu.Symbols(bytes(bad), good[5].symbol_size), 5, gpu.PRIMARY)
    with pytest.raises(gpu.VerificationError):
        cfg.decode_and_verify(meta, good, "strict")

"""Blob batches (rs2_encode_batch_device_async / rs2_encode_batch_with_metadata): many blobs of
one symbol size in one launch per stage -- the upload relay's server-side encode
(walrus-upload-relay/src/controller.rs:177) and the client's per-blob encode loop
(walrus-sdk/src/node_client.rs:3156-3221), each blob a BlobEncoder::encode_with_metadata
(blob_encoding.rs:277-368).  Every blob's slivers, pair hashes and BlobId must equal the
single-blob encode (itself oracle-checked) and, for small shapes, the oracle directly.
"""
import numpy as np
import pytest

import rs2_oracle as O

pytestmark = pytest.mark.gpu


def _blobs(lengths, seed):
    rng = np.random.default_rng(seed)
    return [rng.integers(0, 256, L, dtype=np.uint8).tobytes() for L in lengths]


def _same_symbol_lengths(n, s, count, seed, cap=None):
    """`count` blob lengths that all give symbol size s at n shards (at most `cap` bytes)."""
    kp, ks = O.Rs2Params.for_blob(n, 1).n_primary, O.Rs2Params.for_blob(n, 1).n_secondary
    lo, hi = (s - 2) * kp * ks + 1, s * kp * ks
    if cap:
        hi = max(lo, min(hi, cap))
    rng = np.random.default_rng(seed)
    return [int(x) for x in rng.integers(lo, hi + 1, count)]


@pytest.mark.parametrize("n,s,count", [(10, 6, 5), (13, 40, 7), (100, 14, 4)])
def test_batch_host_matches_oracle(gpu, n, s, count):
    lengths = _same_symbol_lengths(n, s, count, seed=n)
    blobs = _blobs(lengths, seed=n + 1)
    cfg = gpu.ReedSolomonEncodingConfig(n)
    got = cfg.encode_batch_with_metadata(blobs)
    for blob, (pairs, meta) in zip(blobs, got):
        want = O.encode_with_metadata(blob, n)
        assert want.params.symbol_size == s
        assert bytes(meta.blob_id) == want.blob_id
        assert meta.metadata.hashes == [tuple(h) for h in want.pair_hashes]
        for i in range(n):
            assert pairs[i].primary.symbols.data == want.primary[i].tobytes()
            assert pairs[i].secondary.symbols.data == want.secondary[n - 1 - i].tobytes()


def test_batch_host_mixed_symbol_sizes(gpu):
    """Blobs of different symbol sizes (and an empty blob) are grouped per symbol size; the
    results come back in input order and equal the single-blob encodes."""
    n = 16
    lengths = [0, 1, 700, 5000, 5001, 123, 40000, 2, 7000, 39999]
    blobs = _blobs(lengths, seed=5)
    cfg = gpu.ReedSolomonEncodingConfig(n)
    got = cfg.encode_batch_with_metadata(blobs)
    for blob, (pairs, meta) in zip(blobs, got):
        wp, wm = cfg.encode_with_metadata(blob)
        assert meta.blob_id == wm.blob_id
        assert meta.metadata == wm.metadata
        assert [(p.primary.symbols.data, p.secondary.symbols.data) for p in pairs] == \
            [(p.primary.symbols.data, p.secondary.symbols.data) for p in wp]


def test_batch_host_wide_trees(gpu):
    """Host batch at n = 4,500 (above one wave's tree slab): equals the single-blob encodes."""
    n = 4500
    blobs = _blobs([3_000_000, 2_500_000, 1], seed=9)
    cfg = gpu.ReedSolomonEncodingConfig(n)
    got = cfg.encode_batch_with_metadata(blobs)
    for blob, (pairs, meta) in zip(blobs, got):
        wp, wm = cfg.encode_with_metadata(blob)
        assert meta.blob_id == wm.blob_id and meta.metadata == wm.metadata
        assert all(a.primary.symbols.data == b.primary.symbols.data and
                   a.secondary.symbols.data == b.secondary.symbols.data for a, b in zip(pairs, wp))


@pytest.mark.parametrize("n,blob_len,count", [(1000, 4 << 20, 12), (100, 300000, 33),
                                               (5000, 1 << 20, 3), (24600, 20 << 20, 2)])
def test_batch_device_matches_single(gpu, n, blob_len, count):
    """Device form at the C3 shape (n = 1000, 4 MiB, s = 20): strided blobs and sliver
    buffers, per-blob lengths, against one single-blob device encode per blob.  n = 5000 and
    24,600: trees wider than one wave's slab, folded a blob at a time; 128-block codec jobs."""
    import torch
    dev = torch.device("cuda", 0)
    plan = gpu.DevicePlan(n, blob_len)
    info = plan.info
    s = info.symbol_size
    pl, sl = info.primary_sliver_len, info.secondary_sliver_len
    lengths = [blob_len] + _same_symbol_lengths(n, s, count - 1, seed=count, cap=2 * blob_len)
    assert all(gpu.ReedSolomonEncodingConfig(n).symbol_size_for_blob(L) == s for L in lengths)
    g = torch.Generator(device=dev)
    g.manual_seed(11)
    bstride = (max(lengths) + 511) // 512 * 512
    blobs = torch.randint(0, 256, (count, bstride), dtype=torch.uint8, device=dev, generator=g)
    pstride, sstride = n * pl + 256, n * sl + 512
    prim = torch.full((count, pstride), 7, dtype=torch.uint8, device=dev)
    sec = torch.full((count, sstride), 7, dtype=torch.uint8, device=dev)
    hashes = torch.zeros((count, n * 64), dtype=torch.uint8, device=dev)
    ids = torch.zeros((count, 32), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    plan.encode_batch_async(count, blobs.data_ptr(), bstride, lengths, prim.data_ptr(), pstride,
                            sec.data_ptr(), sstride, hashes.data_ptr(), ids.data_ptr(), st)
    torch.cuda.synchronize()
    for b in range(count):
        one = gpu.DevicePlan(n, lengths[b])
        assert one.info.symbol_size == s
        p1 = torch.zeros(n * pl + 256, dtype=torch.uint8, device=dev)
        s1 = torch.zeros(n * sl + 256, dtype=torch.uint8, device=dev)
        h1 = torch.zeros(n * 64, dtype=torch.uint8, device=dev)
        i1 = torch.zeros(32, dtype=torch.uint8, device=dev)
        blob1 = blobs[b, :lengths[b]].clone()
        one.encode_async(blob1.data_ptr(), p1.data_ptr(), s1.data_ptr(), h1.data_ptr(),
                         i1.data_ptr(), st)
        torch.cuda.synchronize()
        assert torch.equal(ids[b], i1), f"blob {b}"
        assert torch.equal(hashes[b], h1)
        assert torch.equal(prim[b, :n * pl], p1[:n * pl])
        assert torch.equal(sec[b, :n * sl], s1[:n * sl])
        # the stride padding past each blob's slivers is untouched
        assert bool((prim[b, n * pl:] == 7).all()) and bool((sec[b, n * sl:] == 7).all())


def test_batch_rejects_other_symbol_size(gpu):
    import ctypes
    from walrus_amd import _lib
    n = 10
    cfg = gpu.ReedSolomonEncodingConfig(n)
    plan = cfg._plan(5000)
    a = np.zeros(5000, dtype=np.uint8)
    b = np.zeros(50000, dtype=np.uint8)
    bp = (ctypes.c_void_p * 2)(a.ctypes.data, b.ctypes.data)
    lens = (ctypes.c_uint64 * 2)(5000, 50000)
    rc = _lib.lib().rs2_encode_batch_with_metadata(plan.handle, 2, bp, lens, None, None, None, None)
    assert rc == _lib.RS2_E_INVALID_ARGUMENT

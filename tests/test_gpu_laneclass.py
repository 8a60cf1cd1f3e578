"""Every lane class of the codec kernels' symbol I/O against the C restatement.

The codec kernels (rs2_codec.hip) move a symbol as 64-byte lo/hi chunks, one packed element
pair per lane; a symbol of s bytes ends in a tail chunk of t = s mod 64 bytes, whose lanes take
their own load / store / copy-out regions, and symbols below 4 bytes take the 2-byte path.
Those regions read per-position offsets across lanes (readlane) inside lane-divergent code,
which is correct only while the offsets stay live in every lane (the keep_live rule; a
violation faulted in round 4, gpurun_out/r04g/1.tests.log).  This sweep drives the loads,
stores and fused copy-outs through every tail class t in {2, 4, ..., 62}, through s < 4,
through whole-chunk symbols (s a multiple of 64) and past one chunk, at n = 10 and n = 1000,
on the single-blob and the batched encode paths and on both decode axes, and compares every
byte with the C restatement (oracle/rs2_cpu.c, fixture-exact against the reference's goldens
in test_cpu_port.py), so a compiler change that breaks the rule fails here, not on a node.

  blob_encoding.rs:277-368  encode_with_metadata      blob_encoding.rs:888-993  decode
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


def _params(cpu, n, length):
    kp, ks, s = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    cpu.rs2cpu_params(n, length, ctypes.byref(kp), ctypes.byref(ks), ctypes.byref(s))
    return kp.value, ks.value, s.value


def _length_for(n, s, cpu, frac=0.6):
    """A blob length whose symbol size is exactly s (s even, >= 2)."""
    kp, ks, _ = _params(cpu, n, 1)
    lo, hi = max((s - 2) * kp * ks + 1, 1), s * kp * ks
    length = int(lo + frac * (hi - lo))
    assert _params(cpu, n, length)[2] == s
    return length


def _c_encode(cpu, n, blob):
    kp, ks, s = _params(cpu, n, len(blob))
    src = np.frombuffer(blob, dtype=np.uint8) if blob else np.zeros(1, dtype=np.uint8)
    prim = np.empty((n, ks * s), dtype=np.uint8)
    sec = np.empty((n, kp * s), dtype=np.uint8)
    hashes = np.empty(n * 64, dtype=np.uint8)
    bid = np.empty(32, dtype=np.uint8)
    cpu.rs2cpu_encode(n, src.ctypes.data, len(blob), prim.ctypes.data, sec.ctypes.data,
                      hashes.ctypes.data, bid.ctypes.data)
    return prim, sec, hashes, bid


def _check(n, pairs, meta, want):
    prim, sec, hashes, bid = want
    assert bytes(meta.blob_id) == bid.tobytes()
    assert meta.metadata.hashes_bytes() == hashes.tobytes()
    for i, p in enumerate(pairs):
        assert p.primary.symbols.data == prim[i].tobytes(), ("primary", i)
        assert p.secondary.symbols.data == sec[n - 1 - i].tobytes(), ("secondary", n - 1 - i)


# every tail class below one chunk (s < 64: t = s), whole chunks, and tails past one chunk
SIZES_N10 = list(range(2, 132, 2)) + [192, 254, 256]
SIZES_N1000 = [2, 4, 6, 30, 62, 64, 66, 94, 126, 128]


@pytest.mark.parametrize("n,s", [(10, s) for s in SIZES_N10] + [(1000, s) for s in SIZES_N1000])
def test_lane_classes_single_and_decode(gpu, cpu, n, s):
    length = _length_for(n, s, cpu)
    blob = np.random.default_rng(n * 1000 + s).integers(0, 256, length, dtype=np.uint8).tobytes()
    cfg = gpu.ReedSolomonEncodingConfig(n)
    pairs, meta = cfg.encode_with_metadata(blob)
    _check(n, pairs, meta, _c_encode(cpu, n, blob))
    kp, ks = cfg.n_primary_source_symbols, cfg.n_secondary_source_symbols
    rng = np.random.default_rng(s)
    order = rng.permutation(n)
    # random subsets (present originals copied out by the decode, erased ones stored) and the
    # worst case (no systematic sliver: every original is a decode store)
    assert cfg.decode(length, [pairs[i].primary for i in order[:kp]]) == blob
    assert cfg.decode(length, [pairs[i].primary for i in range(n - kp, n)]) == blob
    assert cfg.decode(length, [pairs[i].secondary for i in order[:ks]]) == blob


@pytest.mark.parametrize("n,s", [(10, s) for s in (2, 4, 6, 34, 62, 64, 66, 128)] +
                         [(1000, s) for s in (2, 6, 62, 64, 66)])
def test_lane_classes_batch(gpu, cpu, n, s):
    """The batched encode (one launch per stage over every blob of one symbol size) through the
    same lane classes: blobs of different lengths with symbol size s, each byte-equal to the C
    restatement."""
    kp, ks, _ = _params(cpu, n, 1)
    fracs = (0.05, 0.5, 1.0)
    lengths = [_length_for(n, s, cpu, f) for f in fracs]
    rng = np.random.default_rng(n + s)
    blobs = [rng.integers(0, 256, L, dtype=np.uint8).tobytes() for L in lengths]
    cfg = gpu.ReedSolomonEncodingConfig(n)
    for blob, (pairs, meta) in zip(blobs, cfg.encode_batch_with_metadata(blobs)):
        _check(n, pairs, meta, _c_encode(cpu, n, blob))

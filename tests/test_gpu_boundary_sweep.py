"""Shard counts at the codes' power-of-two edges, against the C restatement.

reed-solomon-simd sizes a code's transforms by powers of two of K and R = n - K
(basic_encoding.rs:335-337; the engine's chunk and block plan, rs2_engine.cpp plan_encode /
plan_decode), so the shard counts at which K_p = n - 2f or K_s = n - f crosses 2^k change the
number of input / output chunks, the last chunk's fill and which rate path a code takes.  This
sweep runs the n on both sides of K_p in {256, 512, 1024, 2048} and K_s in {512, 1024, 2048,
4096}, the smallest n with a recovery code (n = 4 .. 9; n <= 3 has f = 0 repair symbols, which
reed-solomon-simd refuses and basic_encoding.rs:128-133 reports as IncompatibleParameters) and a
seeded random draw of n, each at a seeded random blob length: the full encode (every sliver, the pair hashes, the
BlobId), compute_metadata, and decodes from a random subset on both axes and from the worst
case (no systematic sliver), byte-equal to oracle/rs2_cpu.c (pinned to the reference's goldens
in test_cpu_port.py).

  config.rs:446-460, bft.rs:12-25   K_p / K_s of n       blob_encoding.rs:277-368  encode
  blob_encoding.rs:406-486          compute_metadata     blob_encoding.rs:888-993  decode
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


def _kp_ks(n):
    f = (n - 1) // 3
    return n - 2 * f, n - f


# (n, K_p, K_s) at the edges: K_p 255 / 256 / 257, K_s 511 / 512 / 513, K_p 511 / 512 / 513,
# K_s 1023 / 1024 / 1025
EDGE_N = [763, 764, 766, 767, 769, 1531, 1532, 1534, 1535, 1537]
# K_p 1024 / 1025, K_s 2047 / 2048 / 2049, K_p 2048 / 2049, K_s 4095 / 4097 (small symbols)
LARGE_EDGE_N = [3070, 3071, 3073, 6142, 6145]
SMALL_N = [4, 5, 6, 7, 8, 9]
RANDOM_N = sorted(int(x) for x in np.random.default_rng(2026).integers(10, 1300, 6))


@pytest.fixture(scope="module")
def cpu():
    return load_cpu()


def _c_encode(cpu, n, blob, threads=1):
    kp, ks, s = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    cpu.rs2cpu_params(n, len(blob), ctypes.byref(kp), ctypes.byref(ks), ctypes.byref(s))
    kp, ks, s = kp.value, ks.value, s.value
    src = np.frombuffer(blob, dtype=np.uint8) if blob else np.zeros(1, dtype=np.uint8)
    prim = np.empty((n, ks * s), dtype=np.uint8)
    sec = np.empty((n, kp * s), dtype=np.uint8)
    hashes = np.empty(n * 64, dtype=np.uint8)
    bid = np.empty(32, dtype=np.uint8)
    if threads > 1:  # the threaded restatement, pinned to the single-thread one (test_cpu_port.py)
        assert cpu.rs2cpu_encode_mt(n, src.ctypes.data, len(blob), prim.ctypes.data,
                                    sec.ctypes.data, hashes.ctypes.data, bid.ctypes.data,
                                    threads) == 0
    else:
        cpu.rs2cpu_encode(n, src.ctypes.data, len(blob), prim.ctypes.data, sec.ctypes.data,
                          hashes.ctypes.data, bid.ctypes.data)
    return prim, sec, hashes, bid


def test_edge_n_are_edges():
    ks = [_kp_ks(n) for n in EDGE_N + LARGE_EDGE_N]
    assert {kp for kp, _ in ks} >= {255, 256, 257, 511, 512, 513, 1024, 1025, 2048, 2049}
    assert {k for _, k in ks} >= {511, 512, 513, 1023, 1024, 1025, 2047, 2048, 2049, 4095, 4097}


@pytest.mark.parametrize("n", [1, 2, 3])
def test_no_recovery_code_is_incompatible(gpu, n):
    cfg = gpu.ReedSolomonEncodingConfig(n)
    with pytest.raises(gpu.IncompatibleParameters):
        cfg.encode_with_metadata(b"abc")


def _threads():
    # the box's CPU share (OMP_NUM_THREADS = 16 there; os.cpu_count() shows the whole machine)
    return max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", 0)) or (os.cpu_count() or 1)))


@pytest.mark.parametrize("n", SMALL_N + EDGE_N + RANDOM_N + LARGE_EDGE_N)
def test_boundary_n_encode_decode(gpu, cpu, n):
    rng = np.random.default_rng(n)
    kp, ks = _kp_ks(n)
    # symbol sizes 2 .. 40 bytes (2 .. 4 above n = 3000) (s = roundup_even(ceil(B / (K_p K_s))),
    # utils.rs:10-25), and an odd length so the last row is padded
    length = int(rng.integers(1, (4 if n > 3000 else 40) * kp * ks)) | 1
    blob = rng.integers(0, 256, length, dtype=np.uint8).tobytes()
    cfg = gpu.ReedSolomonEncodingConfig(n)
    assert (cfg.n_primary_source_symbols, cfg.n_secondary_source_symbols) == (kp, ks)
    pairs, meta = cfg.encode_with_metadata(blob)
    prim, sec, hashes, bid = _c_encode(cpu, n, blob, _threads() if n > 3000 else 1)
    assert bytes(meta.blob_id) == bid.tobytes()
    assert meta.metadata.hashes_bytes() == hashes.tobytes()
    for i, p in enumerate(pairs):
        assert p.primary.symbols.data == prim[i].tobytes(), ("primary", i)
        assert p.secondary.symbols.data == sec[n - 1 - i].tobytes(), ("secondary", n - 1 - i)
    cm = cfg.compute_metadata(blob)
    assert bytes(cm.blob_id) == bid.tobytes()
    assert cm.metadata.hashes_bytes() == hashes.tobytes()
    order = rng.permutation(n)
    assert cfg.decode(length, [pairs[i].primary for i in order[:kp]]) == blob
    assert cfg.decode(length, [pairs[i].secondary for i in order[:ks]]) == blob
    # as few systematic primary slivers as n allows (primary slivers 0 .. K_p-1 are the blob's
    # rows): decode from the last K_p pairs
    assert cfg.decode(length, [pairs[i].primary for i in range(n - kp, n)]) == blob

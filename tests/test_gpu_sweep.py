"""Seeded random sweep of shapes: n_shards in 4 .. 1100 and blob lengths from 0 to 2 MiB (every
rate, chunk / tail mix and block split the planner can produce in that range), each encoded by
the HIP engine and by the C restatement (oracle/rs2_cpu.c, fixture-exact against the
reference's golden vector via tests/test_cpu_port.py), compared byte for byte: BlobId, every
pair hash, every primary and secondary sliver.  Each case then decodes on the GPU from a random
K_p primary subset, from a random K_s secondary subset and through Default.

  blob_encoding.rs:277-368  encode_with_metadata      blob_encoding.rs:888-993  decode
  config.rs:613-658         decode_and_verify
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


def _cases(count=60, seed=2026):
    rng = np.random.default_rng(seed)
    out = []
    for k in range(count):
        n = int(rng.integers(4, 1101))
        kind = k % 4
        if kind == 0:
            length = int(rng.integers(0, 64))                  # empty / tiny: s = 2
        elif kind == 1:
            length = int(rng.integers(64, 1 << 16))
        else:
            length = int(rng.integers(1 << 16, 2 << 20))
        out.append((n, length, 100 + k))
    return out


@pytest.fixture(scope="module")
def cpu():
    return load_cpu()


@pytest.mark.parametrize("n,length,seed", _cases())
def test_random_shape_matches_c_restatement(gpu, cpu, n, length, seed):
    rng = np.random.default_rng(seed)
    blob = rng.integers(0, 256, length, dtype=np.uint8).tobytes()
    cfg = gpu.ReedSolomonEncodingConfig(n)
    pairs, meta = cfg.encode_with_metadata(blob)

    kp, ks, s = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    cpu.rs2cpu_params(n, length, ctypes.byref(kp), ctypes.byref(ks), ctypes.byref(s))
    kp, ks, s = kp.value, ks.value, s.value
    assert cfg.symbol_size_for_blob(length) == s
    src = np.frombuffer(blob, dtype=np.uint8) if length else np.zeros(1, dtype=np.uint8)
    prim = np.empty((n, ks * s), dtype=np.uint8)
    sec = np.empty((n, kp * s), dtype=np.uint8)
    hashes = np.empty(n * 64, dtype=np.uint8)
    bid = np.empty(32, dtype=np.uint8)
    cpu.rs2cpu_encode(n, src.ctypes.data, length, prim.ctypes.data, sec.ctypes.data,
                      hashes.ctypes.data, bid.ctypes.data)
    assert bytes(meta.blob_id) == bid.tobytes()
    assert meta.metadata.hashes_bytes() == hashes.tobytes()
    for i, p in enumerate(pairs):
        assert p.primary.symbols.data == prim[i].tobytes(), ("primary", i)
        assert p.secondary.symbols.data == sec[n - 1 - i].tobytes(), ("secondary", n - 1 - i)

    order = rng.permutation(n)
    assert cfg.decode(length, [pairs[i].primary for i in order[:kp]]) == blob
    assert cfg.decode(length, [pairs[i].secondary for i in order[:ks]]) == blob
    assert cfg.decode_and_verify(meta, [pairs[i].primary for i in order[-kp:]], "default") == blob

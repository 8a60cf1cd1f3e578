"""Block decomposition parity: transforms split into smaller on-chip blocks (block-level mixing
of the top butterfly layers, rs2_engine.cpp sym_ifft_top / sym_fft_top / mixing_matrices) must
give byte-identical slivers, metadata and decodes for every block limit."""
import numpy as np
import pytest

import rs2_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture
def block_limit(gpu):
    from walrus_amd import _lib

    def set_limit(b):
        assert _lib.lib().rs2_set_block_limit(b) == 0

    yield set_limit
    set_limit(512)


@pytest.mark.parametrize("n,blob_len,block", [
    (1000, 3_000_000, 256), (1000, 3_000_000, 128), (300, 500_000, 32), (300, 500_000, 64),
    (102, 31_415, 16), (102, 31_415, 32), (40, 100_000, 8), (13, 777, 2), (10, 5000, 1),
])
def test_blocks_encode_decode(gpu, block_limit, n, blob_len, block):
    block_limit(block)
    rng = np.random.default_rng(n + block)
    blob = rng.integers(0, 256, blob_len, dtype=np.uint8).tobytes()
    ref = O.encode_with_metadata(blob, n)
    cfg = gpu.ReedSolomonEncodingConfig(n)
    pairs, meta = cfg.encode_with_metadata(blob)
    assert bytes(meta.blob_id) == ref.blob_id
    assert meta.metadata.hashes == ref.pair_hashes
    for i in (0, n // 3, n - 1):
        rp, rs = ref.sliver_pair(i)
        assert pairs[i].primary.symbols.data == rp.tobytes()
        assert pairs[i].secondary.symbols.data == rs.tobytes()
    order = rng.permutation(n)
    assert cfg.decode(blob_len, [pairs[i].primary for i in order]) == blob
    kp = cfg.n_primary_source_symbols
    assert cfg.decode(blob_len, [pairs[i].primary for i in range(n - 1, -1, -1)][:kp]) == blob
    assert cfg.decode(blob_len, [pairs[n - 1 - i].secondary for i in order]) == blob

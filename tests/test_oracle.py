"""CPU tests of the oracle (oracle/rs2_oracle.py): the reference's golden vector, the
reference's own parameter tables, layout tests and algebraic properties.  No GPU."""
import hashlib
import json
import os

import numpy as np
import pytest

import rs2_oracle as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "rs2_fixtures.json")


def test_v1_blob_id_stability():
    """blob_encoding.rs:1227-1244 -- the only codeword-level golden vector of the reference."""
    enc = O.encode_with_metadata(b"walrus blob id v1 regression test", 10)
    assert O.blob_id_to_str(enc.blob_id) == "RcU82Mwf-CFkv1LaI_2qcpANwpGUuG3TMwnVzZxD2kY"


def test_reference_publisher_example_n1000():
    """docs/content/http-api/storing-blobs.mdx:114-127: `-d "some other string"` stored on
    mainnet (n = 1000, s = 2) -> blobId M4hsZGQ1oCktdzegB6HnI6Mi28S2nqOPHxK-W7_4BUk.  The only
    reference-held vector that runs the chunked 512-point codes of the metric's n = 1000 shape
    (row code 512 + 155 inputs, column code 512 + 154 outputs)."""
    enc = O.encode_with_metadata(b"some other string", 1000)
    p = enc.params
    assert (p.n_primary, p.n_secondary, p.symbol_size) == (334, 667, 2)
    assert O.blob_id_to_str(enc.blob_id) == "M4hsZGQ1oCktdzegB6HnI6Mi28S2nqOPHxK-W7_4BUk"
    # encodedLength / storageSize 66,034,000 (storing-blobs.mdx:133,139; config.rs:791-826)
    assert 1000 * (p.n_primary + p.n_secondary) * p.symbol_size + 1000 * (1000 * 64 + 32) \
        == 66_034_000


@pytest.mark.parametrize("length,n_symbols,align,expected", [
    (0, 1, 1, 1), (0, 42, 1, 1), (15, 5, 1, 3), (13, 13, 1, 1), (16, 5, 1, 4), (19, 5, 1, 4),
    (0, 1, 2, 2), (0, 42, 2, 2), (15, 5, 2, 4), (13, 13, 2, 2), (21, 5, 2, 6), (24, 5, 2, 6)])
def test_compute_symbol_size(length, n_symbols, align, expected):
    """utils.rs:58-89."""
    assert O.compute_symbol_size(length, n_symbols, align) == expected


@pytest.mark.parametrize("n,primary,secondary", [
    (1, 1, 1), (3, 3, 3), (7, 3, 5), (10, 4, 7), (31, 11, 21), (100, 34, 67), (301, 101, 201),
    (1000, 334, 667), (4, 2, 3), (9, 5, 7), (51, 19, 35), (101, 35, 68)])
def test_source_symbols_for_n_shards(n, primary, secondary):
    """config.rs:884-923."""
    assert O.source_symbols_for_n_shards(n) == (primary, secondary)


def test_data_too_large():
    """max blob = K_p*K_s*65534 at n=1000 (config.rs:770-773)."""
    assert O.compute_symbol_size(334 * 667 * 65534, 334 * 667) == 65534
    with pytest.raises(O.DataTooLargeError):
        O.compute_symbol_size(334 * 667 * 65535 + 1, 334 * 667)


@pytest.mark.parametrize("kp,ks,blob,rows,cols", [
    (2, 2, [1, 2, 3, 4, 5, 6, 7, 8], [[1, 2, 3, 4], [5, 6, 7, 8]], [[1, 2, 5, 6], [3, 4, 7, 8]]),
    (2, 3, list(range(1, 13)), [[1, 2, 3, 4, 5, 6], [7, 8, 9, 10, 11, 12]],
     [[1, 2, 7, 8], [3, 4, 9, 10], [5, 6, 11, 12]]),
    (2, 2, [1, 2, 3, 4, 5], [[1, 2, 3, 4], [5, 0, 0, 0]], [[1, 2, 5, 0], [3, 4, 0, 0]]),
    (2, 3, [1, 2, 3, 4, 5, 6, 7, 8], [[1, 2, 3, 4, 5, 6], [7, 8, 0, 0, 0, 0]],
     [[1, 2, 7, 8], [3, 4, 0, 0], [5, 6, 0, 0]]),
])
def test_matrix_construction(kp, ks, blob, rows, cols):
    """blob_encoding.rs:1011-1073 (new_for_test with n = 3 (kp + ks))."""
    p = O.Rs2Params.for_test(kp, ks, 3 * (kp + ks), len(blob))
    enc = O.encode_with_metadata(bytes(blob), p.n_shards, p)
    assert [list(enc.primary[i]) for i in range(kp)] == rows
    assert [list(enc.secondary[j]) for j in range(ks)] == cols


def test_merkle_edge_cases():
    """merkle.rs:378-400: empty tree -> zeros; single (even empty) element -> its leaf hash."""
    assert O.merkle_root([]) == bytes(32)
    assert O.merkle_root([b"Test"]) == O.leaf_hash(b"Test")
    assert O.merkle_root([b""]) == O.leaf_hash(b"")
    leaves = [b"foo", b"bar", b"fizz"]
    l = [O.leaf_hash(x) for x in leaves]
    assert O.merkle_root(leaves) == O.inner_hash(O.inner_hash(l[0], l[1]),
                                                 O.inner_hash(l[2], bytes(32)))


@pytest.mark.parametrize("data,k,rng_,ok", [
    ([1, 2, 3, 4], 2, (0, 2), True), ([1, 2], 1, (1, 2), True),
    ([1, 2, 3, 4, 5, 6, 7, 8], 2, (2, 4), True), ([1, 2, 3, 4, 5, 6], 3, (3, 6), True),
    ([1, 2, 3, 4], 2, (2, 3), False), ([1, 2, 3, 4, 5, 6], 3, (1, 3), False)])
def test_encode_decode_1d(data, k, rng_, ok):
    """basic_encoding.rs:487-533."""
    start, end = rng_
    n = max(end, k + 1)
    s = O.compute_symbol_size(len(data), k)
    allsym = O.rs_encode_all(np.array(data, dtype=np.uint8).reshape(k, s), n)
    syms = [(i, allsym[i]) for i in range(start, end)]
    if ok:
        assert O.rs_decode_symbols(k, n, s, syms).reshape(-1).tolist() == data
    else:
        with pytest.raises(ValueError):
            O.rs_decode_symbols(k, n, s, syms)


@pytest.mark.parametrize("k,r", [(2, 1), (3, 3), (5, 6), (4, 6), (7, 3), (9, 12), (12, 9),
                                 (5, 5), (1, 4), (4, 1), (33, 17), (17, 33)])
def test_fft_decoder_matches_gaussian(k, r):
    """The FFT decoder and an independent Gaussian-elimination decoder agree."""
    rng = np.random.default_rng(k * 31 + r)
    orig = rng.integers(0, 65536, (k, 4)).astype(np.uint16)
    allsh = np.concatenate([orig, O.rs_encode_elems(orig, r)])
    for _ in range(3):
        idx = rng.permutation(k + r)[:k]
        rec = {int(i): allsh[i] for i in idx}
        assert (O.rs_decode_elems(k, r, rec) == orig).all()
        if k <= 12:
            assert (O.rs_decode_gauss(k, r, rec) == orig).all()


def test_blob_round_trip_and_hashes():
    """blob_encoding.rs:1092-1188 and slivers.rs recovery tests at n=102 / n=13."""
    rng = np.random.default_rng(3)
    for n, size in [(102, 31415), (13, 777)]:
        blob = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
        enc = O.encode_with_metadata(blob, n)
        p = enc.params
        idx = rng.permutation(n)
        assert O.decode_blob(n, size, "primary", [(int(i), enc.primary[i]) for i in idx]) == blob
        assert O.decode_blob(n, size, "secondary",
                             [(int(i), enc.secondary[i]) for i in idx]) == blob
        for i in range(n):
            prim, sec = enc.sliver_pair(i)
            assert O.sliver_merkle_root(prim, "primary", p) == enc.pair_hashes[i][0]
            assert O.sliver_merkle_root(sec, "secondary", p) == enc.pair_hashes[i][1]


def test_golden_fixtures_reproduce():
    """The committed fixtures are reproduced by the current oracle (guards oracle edits)."""
    fx = json.load(open(GOLDEN))
    assert fx["cases"][0]["blob_id"] == "RcU82Mwf-CFkv1LaI_2qcpANwpGUuG3TMwnVzZxD2kY"
    for case in fx["cases"]:
        if case["n_shards"] > 102:
            continue
        if case["blob"] is not None:
            blob = bytes.fromhex(case["blob"])
        else:
            blob = np.random.default_rng(case["blob_seed"]).integers(
                0, 256, case["blob_len"], dtype=np.uint8).tobytes()
        enc = O.encode_with_metadata(blob, case["n_shards"])
        assert O.blob_id_to_str(enc.blob_id) == case["blob_id"], case["name"]
        assert [hashlib.sha256(x.tobytes()).hexdigest() for x in enc.primary] == \
            case["primary_sha256"]

"""The C/AVX2 CPU restatement (oracle/rs2_cpu.c, the bench's cpu_baseline) against the golden
fixtures and the numpy oracle.  CPU only.

The restatement is what bench.py times as the reference's CPU path, so it has to be the same
algorithm producing the same bytes: BlobId / pair hashes / sliver digests of every fixture case
(case 0 is the reference's test_v1_blob_id_stability vector, blob_encoding.rs:1227-1244), and
BlobDecoder::decode round trips from random and no-systematic primary subsets.
"""
import ctypes
import hashlib
import json
import os
import shutil
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import rs2_oracle as O  # noqa: E402

FIXTURES = os.path.join(ROOT, "tests", "golden", "rs2_fixtures.json")

pytestmark = pytest.mark.skipif(shutil.which("gcc") is None and shutil.which("cc") is None,
                                reason="no C compiler")


@pytest.fixture(scope="module")
def cpu():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "librs2cpu.so"))
    P = ctypes.c_void_p
    lib.rs2cpu_encode.argtypes = [ctypes.c_uint32, P, ctypes.c_uint64, P, P, P, P]
    lib.rs2cpu_decode_primary.argtypes = [ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32, P,
                                          P, P]
    lib.rs2cpu_encode_1d.argtypes = [ctypes.c_uint32] * 4 + [P, P]
    return lib


def _params(n, blob_len):
    p = O.Rs2Params.for_blob(n, blob_len)
    return p.n_primary, p.n_secondary, p.symbol_size


def _encode(lib, n, blob):
    kp, ks, s = _params(n, len(blob))
    src = np.frombuffer(blob, dtype=np.uint8).copy() if blob else np.zeros(1, np.uint8)
    prim = np.zeros((n, ks * s), np.uint8)
    sec = np.zeros((n, kp * s), np.uint8)
    hashes = np.zeros((n, 64), np.uint8)
    bid = np.zeros(32, np.uint8)
    rc = lib.rs2cpu_encode(n, src.ctypes.data, len(blob), prim.ctypes.data, sec.ctypes.data,
                           hashes.ctypes.data, bid.ctypes.data)
    assert rc == 0
    return prim, sec, hashes, bid


def _decode(lib, n, blob_len, prim, idx):
    rows = [np.ascontiguousarray(prim[i]) for i in idx]
    ptrs = (ctypes.c_void_p * len(rows))(*[r.ctypes.data for r in rows])
    ids = np.array(idx, dtype=np.uint16)
    out = np.zeros(max(blob_len, 1), np.uint8)
    rc = lib.rs2cpu_decode_primary(n, blob_len, len(idx), ids.ctypes.data, ptrs, out.ctypes.data)
    return rc, out[:blob_len].tobytes()


def _blob(case):
    if case["blob"] is not None:
        return bytes.fromhex(case["blob"])
    return np.random.default_rng(case["blob_seed"]).integers(
        0, 256, case["blob_len"], dtype=np.uint8).tobytes()


CASES = json.load(open(FIXTURES))["cases"]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_fixture_encode(cpu, case):
    n = case["n_shards"]
    blob = _blob(case)
    prim, sec, hashes, bid = _encode(cpu, n, blob)
    assert O.blob_id_to_str(bid.tobytes()) == case["blob_id"]
    assert [[h[:32].tobytes().hex(), h[32:].tobytes().hex()] for h in hashes] == case["pair_hashes"]
    assert [hashlib.sha256(x.tobytes()).hexdigest() for x in prim] == case["primary_sha256"]
    assert [hashlib.sha256(x.tobytes()).hexdigest() for x in sec] == case["secondary_sha256"]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_fixture_decode(cpu, case):
    n, kp = case["n_shards"], case["n_primary"]
    blob = _blob(case)
    prim, _, _, _ = _encode(cpu, n, blob)
    rng = np.random.default_rng(7)
    subsets = [list(rng.permutation(n)[:kp]), list(range(kp, 2 * kp)),
               list(range(n - kp, n))[::-1]]
    for idx in subsets:
        rc, out = _decode(cpu, n, len(blob), prim, [int(i) for i in idx])
        assert rc == 0 and out == blob
    rc, _ = _decode(cpu, n, len(blob), prim, list(range(kp - 1)))
    assert rc != 0


@pytest.mark.parametrize("k,n,s", [(1, 2, 2), (3, 7, 64), (5, 11, 130), (8, 9, 6), (16, 17, 100),
                                   (33, 100, 2), (100, 130, 66), (334, 1000, 4), (667, 1000, 2)])
def test_encode_1d_matches_numpy_oracle(cpu, k, n, s):
    rng = np.random.default_rng(k * 1000 + n)
    batch = 2
    data = rng.integers(0, 256, (batch, k, s), dtype=np.uint8)
    out = np.zeros((batch, n, s), np.uint8)
    assert cpu.rs2cpu_encode_1d(k, n, s, batch, data.ctypes.data, out.ctypes.data) == 0
    for b in range(batch):
        want = O.rs_encode_all(data[b], n)
        assert np.array_equal(out[b], want)


def test_bench_binary_round_trip(cpu):
    exe = os.path.join(ROOT, "oracle", "build", "rs2_cpu_bench")
    res = subprocess.run([exe, "100", str(3 << 20)], capture_output=True, text=True, timeout=120)
    assert res.returncode == 0, res.stderr
    d = json.loads(res.stdout.strip().splitlines()[-1])
    assert d["ok"] is True and d["gibs"] > 0 and d["cores"] == 1


# ---- storage-node side: the C port's twins of bench.node_leg ------------------------------------
@pytest.mark.parametrize("n,blob_len", [(10, 5000), (100, 30000), (1000, 40000)])
def test_node_side_matches_numpy_oracle(cpu, n, blob_len):
    """rs2cpu_sliver_root / rs2cpu_recovery_symbol / rs2cpu_recover_sliver (the CPU twins the
    bench times beside the device verifier) against the numpy oracle's sliver_merkle_root,
    merkle_proof (MerkleTree::get_proof, merkle.rs:281-309) and recover_sliver, and the pair
    hashes of the encode."""
    P = ctypes.c_void_p
    cpu.rs2cpu_sliver_root.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, P, P]
    cpu.rs2cpu_recovery_symbol.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, P,
                                           ctypes.c_uint32, P, P]
    cpu.rs2cpu_recover_sliver.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                          ctypes.c_uint32, P, P, P, P]
    blob = np.random.default_rng(n).integers(0, 256, blob_len, dtype=np.uint8).tobytes()
    prim, sec, hashes, _ = _encode(cpu, n, blob)
    p = O.Rs2Params.for_blob(n, blob_len)
    s = p.symbol_size
    root = np.zeros(32, np.uint8)
    for i in (0, n // 3, n - 1):
        for axis, sliver, want in ((0, prim[i], hashes[i, :32]), (1, sec[i], hashes[n - 1 - i, 32:])):
            sliver = np.ascontiguousarray(sliver)
            assert cpu.rs2cpu_sliver_root(n, s, axis, sliver.ctypes.data, root.ctypes.data) == 0
            assert root.tobytes() == want.tobytes()
    L = len(O.merkle_proof([b"\0\0"] * n, 0))
    sym = np.zeros(s, np.uint8)
    proof = np.zeros(L * 32, np.uint8)
    for i, t in ((1, n - 1), (n - 1, 0), (n // 2, n // 3)):
        sliver = np.ascontiguousarray(prim[i])
        assert cpu.rs2cpu_recovery_symbol(n, s, 0, sliver.ctypes.data, t, sym.ctypes.data,
                                          proof.ctypes.data) == L
        exp = O.recovery_symbols(sliver, "primary", p)
        assert sym.tobytes() == exp[t].tobytes()
        want = O.merkle_proof([x.tobytes() for x in exp], t)
        assert proof.tobytes() == b"".join(want)
        assert O.merkle_proof_root(want, sym.tobytes(), t) == hashes[i, :32].tobytes()
    # recover primary sliver t from K_s symbols of secondary slivers n-1, n-2, ... (expanded)
    t = n // 2
    srcs = list(range(n - 1, n - 1 - p.n_secondary, -1))
    symbols = np.ascontiguousarray(O.expanded_matrix(blob, p)[t, srcs])  # symbol (t, c)
    ids = np.array(srcs, np.uint16)
    out = np.zeros(p.n_secondary * s, np.uint8)
    assert cpu.rs2cpu_recover_sliver(n, s, 0, len(srcs), ids.ctypes.data, symbols.ctypes.data,
                                     out.ctypes.data, root.ctypes.data) == 0
    assert out.tobytes() == prim[t].tobytes() and root.tobytes() == hashes[t, :32].tobytes()
    assert cpu.rs2cpu_recover_sliver(n, s, 0, len(srcs) - 1, ids.ctypes.data,
                                     symbols.ctypes.data, out.ctypes.data, root.ctypes.data) != 0


def test_bench_binary_node_mode(cpu):
    exe = os.path.join(ROOT, "oracle", "build", "rs2_cpu_bench")
    res = subprocess.run([exe, "node", "100", str(1 << 20), "2", "4"], capture_output=True,
                         text=True, timeout=120)
    assert res.returncode == 0, res.stderr
    d = json.loads(res.stdout.strip().splitlines()[-1])
    assert d["ok"] is True and d["verify_gibs"] > 0 and d["recovery_symbols_per_s"] > 0
    assert d["recover_sliver_ms"] > 0 and d["cores"] == 2


@pytest.mark.parametrize("n,blob_len,threads", [(10, 5000, 2), (13, 777, 3), (100, 30000, 4),
                                                (1000, 40000, 8), (1000, 3 << 20, 5),
                                                (4097, 100, 8)])
def test_encode_mt_matches_single_thread(cpu, n, blob_len, threads):
    """rs2cpu_encode_mt (the golden generator for large n_shards: no n x n leaf array, rows'
    trees streamed per column chunk and finished over the chunks' level-k nodes) gives the
    same slivers, pair hashes and BlobId as the single-thread restatement."""
    P = ctypes.c_void_p
    cpu.rs2cpu_encode_mt.argtypes = [ctypes.c_uint32, P, ctypes.c_uint64, P, P, P, P, ctypes.c_int]
    blob = np.random.default_rng(n + blob_len).integers(0, 256, blob_len, dtype=np.uint8).tobytes()
    prim, sec, hashes, bid = _encode(cpu, n, blob)
    kp, ks, s = _params(n, blob_len)
    src = np.frombuffer(blob, dtype=np.uint8).copy()
    p2 = np.zeros((n, ks * s), np.uint8)
    s2 = np.zeros((n, kp * s), np.uint8)
    h2 = np.zeros((n, 64), np.uint8)
    b2 = np.zeros(32, np.uint8)
    assert cpu.rs2cpu_encode_mt(n, src.ctypes.data, blob_len, p2.ctypes.data, s2.ctypes.data,
                                h2.ctypes.data, b2.ctypes.data, threads) == 0
    assert np.array_equal(h2, hashes) and np.array_equal(b2, bid)
    assert np.array_equal(p2, prim) and np.array_equal(s2, sec)

"""CPU oracle for the Red Stuff (RS2) hot path -- TEST INFRASTRUCTURE ONLY.

This module is a plain numpy restatement of the reference algorithm.  It exists to
check the HIP engine (``walrus_amd``); it is never the thing measured or shipped.
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import it.

What it restates (all paths relative to the reference checkout):

* Walrus layer (``crates/walrus-core``):
  - ``bft.rs:12-25`` / ``encoding/config.rs:717-725``  -> ``source_symbols_for_n_shards``
  - ``encoding/utils.rs:10-25``                         -> ``compute_symbol_size``
  - ``encoding/blob_encoding.rs:277-368``               -> ``encode_with_metadata``
  - ``encoding/blob_encoding.rs:161-196``               -> ``compute_metadata_from_symbol_hashes``
  - ``encoding/blob_encoding.rs:406-486``               -> ``compute_metadata``
  - ``encoding/blob_encoding.rs:836-993``               -> ``decode_blob``
  - ``encoding/basic_encoding.rs:107-429``              -> ``rs_encode`` / ``rs_decode`` wrappers
  - ``encoding/slivers.rs:100-392``                     -> ``recovery_symbols`` / ``recover_sliver``
  - ``merkle.rs:18-20,216-332``                         -> ``merkle_root_from_leaf_hashes``
  - ``metadata.rs:571-578,638-643``, ``lib.rs:159-189`` -> ``blob_id``
* Arithmetic: the third-party crate ``reed-solomon-simd`` 3.1.0 (``Cargo.lock:8813-8821``,
  called from ``basic_encoding.rs:128-133,305-329,375-427``).  Its source is not in the
  reference checkout; this file restates its published Leopard-style algorithm: GF(2^16)
  with polynomial 0x1002D in the Cantor basis, log/exp/skew tables, the additive (LCH)
  FFT/IFFT, the high/low rate encoders and the 64-byte lo/hi shard layout.
* Hashing: ``fastcrypto::hash::Blake2b256`` == RustCrypto ``blake2`` 0.10.6 ``Blake2b<U32>``
  == ``hashlib.blake2b(digest_size=32)``.

Parity pin: ``test_v1_blob_id_stability`` (``blob_encoding.rs:1227-1244``) -- the 33-byte
blob at n_shards=10 must give BlobId ``RcU82Mwf-CFkv1LaI_2qcpANwpGUuG3TMwnVzZxD2kY``.  It is
the only codeword-level golden vector the reference holds; ``tests/test_oracle.py`` checks
it, and the decoders are checked by encode -> erase -> decode round trips and against an
independent Gaussian-elimination decoder.
"""

from __future__ import annotations

import base64
import hashlib
from dataclasses import dataclass

import numpy as np

# ---------------------------------------------------------------------------------------------
# GF(2^16) -- reed-solomon-simd 3.1.0 engine/tables.rs (restated)
# ---------------------------------------------------------------------------------------------

GF_BITS = 16
GF_ORDER = 1 << GF_BITS
GF_MODULUS = GF_ORDER - 1
GF_POLYNOMIAL = 0x1002D
CANTOR_BASIS = (
    0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
    0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E,
)


def _init_exp_log():
    exp = [0] * GF_ORDER
    log = [0] * GF_ORDER
    state = 1
    for i in range(GF_MODULUS):
        exp[state] = i
        state <<= 1
        if state >= GF_ORDER:
            state ^= GF_POLYNOMIAL
    exp[0] = GF_MODULUS
    # Convert to the Cantor basis.
    log[0] = 0
    for i in range(GF_BITS):
        width = 1 << i
        b = CANTOR_BASIS[i]
        for j in range(width):
            log[j + width] = log[j] ^ b
    for i in range(GF_ORDER):
        log[i] = exp[log[i]]
    for i in range(GF_ORDER):
        exp[log[i]] = i
    exp[GF_MODULUS] = exp[0]
    return np.array(exp, dtype=np.uint32), np.array(log, dtype=np.uint32)


EXP, LOG = _init_exp_log()


def add_mod(a, b):
    s = np.asarray(a, dtype=np.uint32) + np.asarray(b, dtype=np.uint32)
    return (s + (s >> GF_BITS)) & 0xFFFF


def sub_mod(a, b):
    d = (np.asarray(a, dtype=np.int64) - np.asarray(b, dtype=np.int64)) & 0xFFFFFFFF
    return (d + (d >> GF_BITS)) & 0xFFFF


def _mul_scalar(x: int, log_m: int) -> int:
    if x == 0:
        return 0
    s = int(LOG[x]) + log_m
    return int(EXP[(s + (s >> 16)) & 0xFFFF])


def gf_mul(x: np.ndarray, log_m) -> np.ndarray:
    """``mul(x, log_m) = exp[add_mod(log[x], log_m)]``, 0 for x == 0 (vectorised)."""
    x = np.asarray(x)
    r = EXP[add_mod(LOG[x], log_m)]
    return np.where(x == 0, 0, r).astype(np.uint16)


def _init_skew():
    skew = [0] * GF_MODULUS
    temp = [0] * (GF_BITS - 1)
    for i in range(1, GF_BITS):
        temp[i - 1] = 1 << i
    for m in range(GF_BITS - 1):
        step = 1 << (m + 1)
        skew[(1 << m) - 1] = 0
        for i in range(m, GF_BITS - 1):
            s = 1 << (i + 1)
            j = (1 << m) - 1
            while j < s:
                skew[j + s] = skew[j] ^ temp[i]
                j += step
        temp[m] = GF_MODULUS - int(LOG[_mul_scalar(temp[m], int(LOG[temp[m] ^ 1]))])
        for i in range(m + 1, GF_BITS - 1):
            t = int(add_mod(int(LOG[temp[i] ^ 1]), temp[m]))
            temp[i] = _mul_scalar(temp[i], t)
    return np.array([int(LOG[v]) for v in skew], dtype=np.uint32)


SKEW = _init_skew()

# ---------------------------------------------------------------------------------------------
# Additive FFT / IFFT over GF(2^16) in the LCH basis.
#
# `work` is a uint16 array of shape (positions, elements).  Every column is an independent
# codeword (one GF element position of the shards); every butterfly uses one constant for the
# whole row, which is what makes the GPU mapping "lanes = codewords" possible.
#
# The reference engine uses radix-4 passes ("two layers at a time") plus one odd radix-2 layer;
# the constants are skew[r + d + skew_delta - 1] for a group starting at r with half distance d,
# so the radix-2 statement below evaluates the identical linear map.
# ---------------------------------------------------------------------------------------------


def fft(work: np.ndarray, pos: int, size: int, trunc: int, skew_delta: int) -> None:
    """FFT butterfly: ``x ^= mul(y, m); y ^= x`` (m == GF_MODULUS means multiply by zero)."""
    d = size >> 1
    while d >= 1:
        for r in range(0, trunc, 2 * d):
            log_m = int(SKEW[r + d + skew_delta - 1])
            x = work[pos + r: pos + r + d]
            y = work[pos + r + d: pos + r + 2 * d]
            if log_m != GF_MODULUS:
                x ^= gf_mul(y, log_m)
            y ^= x
        d >>= 1


def ifft(work: np.ndarray, pos: int, size: int, trunc: int, skew_delta: int) -> None:
    """IFFT butterfly: ``y ^= x; x ^= mul(y, m)``.  Inputs at positions >= trunc are zero."""
    d = 1
    while d < size:
        for r in range(0, trunc, 2 * d):
            log_m = int(SKEW[r + d + skew_delta - 1])
            x = work[pos + r: pos + r + d]
            y = work[pos + r + d: pos + r + 2 * d]
            y ^= x
            if log_m != GF_MODULUS:
                x ^= gf_mul(y, log_m)
        d <<= 1


def formal_derivative(work: np.ndarray, size: int) -> None:
    for i in range(1, size):
        w = i & (-i)
        work[i - w: i] ^= work[i: i + w]


def next_pow2(x: int) -> int:
    return 1 << (x - 1).bit_length() if x > 1 else 1


def use_high_rate(original_count: int, recovery_count: int) -> bool:
    """reed-solomon-simd DefaultRate: HighRate iff pow2(recovery) <= pow2(original).

    Ties go to the high rate.  Walrus never hits a tie on the row (secondary) code; it can on
    the column code for some n (e.g. n=11); the tie rule is not pinned by a reference vector.
    """
    if original_count == 0 or recovery_count == 0:
        raise ValueError("unsupported shard count")
    op, rp = next_pow2(original_count), next_pow2(recovery_count)
    if min(op, rp) + max(original_count, recovery_count) > GF_ORDER:
        raise ValueError("unsupported shard count")
    return rp <= op


def rs_encode_elems(orig: np.ndarray, recovery_count: int) -> np.ndarray:
    """Encode K original codeword rows (shape (K, E), uint16) to R recovery rows."""
    k, e = orig.shape
    r_cnt = recovery_count
    if use_high_rate(k, r_cnt):
        cs = next_pow2(r_cnt)
        acc = np.zeros((cs, e), dtype=np.uint16)
        for start in range(0, k, cs):
            cnt = min(cs, k - start)
            buf = np.zeros((cs, e), dtype=np.uint16)
            buf[:cnt] = orig[start: start + cnt]
            ifft(buf, 0, cs, cnt, start + cs)
            acc ^= buf
        fft(acc, 0, cs, r_cnt, 0)
        return acc[:r_cnt].copy()
    cs = next_pow2(k)
    buf = np.zeros((cs, e), dtype=np.uint16)
    buf[:k] = orig
    ifft(buf, 0, cs, k, 0)
    out = np.zeros((r_cnt, e), dtype=np.uint16)
    for start in range(0, r_cnt, cs):
        cnt = min(cs, r_cnt - start)
        tmp = buf.copy()
        fft(tmp, 0, cs, cnt, start + cs)
        out[start: start + cnt] = tmp[:cnt]
    return out


def codeword_layout(k: int, r_cnt: int):
    """Positions of originals / recovery shards in the decoder's codeword and its size W."""
    if use_high_rate(k, r_cnt):
        cs = next_pow2(r_cnt)
        orig_pos = cs + np.arange(k)
        rec_pos = np.arange(r_cnt)
        end = cs + k
        return True, cs, orig_pos, rec_pos, end, next_pow2(end)
    cs = next_pow2(k)
    orig_pos = np.arange(k)
    rec_pos = cs + np.arange(r_cnt)
    end = cs + r_cnt
    return False, cs, orig_pos, rec_pos, end, next_pow2(end)


def erasure_logs(k: int, r_cnt: int, present_orig: np.ndarray, present_rec: np.ndarray):
    """log of the erasure-locator values over the decoder's subspace of size W.

    For a known position p:  L[p] = log prod_{e erased} (w_p + w_e)          (= log l(w_p))
    For an erased position p: L[p] = log prod_{e erased, e != p} (w_p + w_e) (= log l'(w_p))
    Points are the Cantor-basis elements w_p = p, so w_p + w_e has bits p ^ e.  The erased set
    is: missing shards; in the high rate the never-sent recovery slots [R, cs); in the low rate
    the positions [end, W) (whose codeword values are not zero).  Zero padding of the originals
    is known (value 0).  The sum uses LOG[0] = 65535 == 0 (mod 65535), which drops e == p.
    """
    high, cs, orig_pos, rec_pos, end, w = codeword_layout(k, r_cnt)
    erased = np.zeros(w, dtype=bool)
    erased[orig_pos[~present_orig]] = True
    erased[rec_pos[~present_rec]] = True
    if high:
        erased[r_cnt:cs] = True
    else:
        erased[end:w] = True
    acc = np.zeros(w, dtype=np.int64)
    idx = np.arange(w)
    for e in np.nonzero(erased)[0]:
        acc += LOG[idx ^ e]
    return (acc % GF_MODULUS).astype(np.uint32), erased


def rs_decode_elems(k: int, r_cnt: int, received: dict) -> np.ndarray:
    """Decode the K originals from {shard index: (E,) uint16 row} (index < K original)."""
    high, cs, orig_pos, rec_pos, end, w = codeword_layout(k, r_cnt)
    present_orig = np.zeros(k, dtype=bool)
    present_rec = np.zeros(r_cnt, dtype=bool)
    e = None
    for idx, row in received.items():
        e = row.shape[0]
        if idx < k:
            present_orig[idx] = True
        else:
            present_rec[idx - k] = True
    if present_orig.sum() + present_rec.sum() < k:
        raise ValueError("not enough shards")
    out = np.zeros((k, e), dtype=np.uint16)
    for idx, row in received.items():
        if idx < k:
            out[idx] = row
    if present_orig.all():
        return out
    logs, erased = erasure_logs(k, r_cnt, present_orig, present_rec)
    work = np.zeros((w, e), dtype=np.uint16)
    for idx, row in received.items():
        p = orig_pos[idx] if idx < k else rec_pos[idx - k]
        work[p] = gf_mul(row, int(logs[p]))
    ifft(work, 0, w, end, 0)
    formal_derivative(work, w)
    fft(work, 0, w, end if high else k, 0)
    for i in np.nonzero(~present_orig)[0]:
        p = orig_pos[i]
        out[i] = gf_mul(work[p], GF_MODULUS - int(logs[p]))
    return out


# --- independent decoder (Gaussian elimination on the encoder's linear map), small K only -----


def _gf_inv(x: int) -> int:
    return int(EXP[(GF_MODULUS - int(LOG[x])) % GF_MODULUS])


def _gf_mul_s(a: int, b: int) -> int:
    if a == 0 or b == 0:
        return 0
    return int(EXP[(int(LOG[a]) + int(LOG[b])) % GF_MODULUS])


def rs_decode_gauss(k: int, r_cnt: int, received: dict) -> np.ndarray:
    """Decode by solving the systematic generator's K x K subsystem over GF(2^16)."""
    gen = rs_encode_elems(np.eye(k, dtype=np.uint16), r_cnt)  # (R, K): rec_j = sum_i G[j,i] o_i
    idxs = sorted(received)[:k]
    rows = []
    for idx in idxs:
        if idx < k:
            row = [0] * k
            row[idx] = 1
        else:
            row = [int(v) for v in gen[idx - k]]
        rows.append(row)
    rhs = [received[i].astype(np.uint16).copy() for i in idxs]
    a = rows
    for col in range(k):
        piv = next(r for r in range(col, k) if a[r][col] != 0)
        a[col], a[piv] = a[piv], a[col]
        rhs[col], rhs[piv] = rhs[piv], rhs[col]
        inv = _gf_inv(a[col][col])
        a[col] = [_gf_mul_s(v, inv) for v in a[col]]
        rhs[col] = gf_mul(rhs[col], int(LOG[inv]))
        for r in range(k):
            if r != col and a[r][col] != 0:
                f = a[r][col]
                a[r] = [a[r][c] ^ _gf_mul_s(f, a[col][c]) for c in range(k)]
                rhs[r] = rhs[r] ^ gf_mul(rhs[col], int(LOG[f]))
    return np.stack(rhs)


# ---------------------------------------------------------------------------------------------
# Shard byte <-> GF element layout (reed-solomon-simd `Shards::insert` / `undo_last_chunk`)
#   full 64-byte chunk q:  element 32q+j = b[64q+j] | b[64q+32+j] << 8      (j < 32)
#   tail of t = s % 64:    element 32Q+j = b[64Q+j] | b[64Q+t/2+j] << 8     (j < t/2)
# ---------------------------------------------------------------------------------------------


def bytes_to_elems(arr: np.ndarray) -> np.ndarray:
    arr = np.asarray(arr, dtype=np.uint8)
    s = arr.shape[-1]
    assert s % 2 == 0
    q, t = divmod(s, 64)
    h = t // 2
    lead = arr.shape[:-1]
    full = arr[..., : 64 * q].reshape(lead + (q, 64)).astype(np.uint16)
    parts = [(full[..., :32] | (full[..., 32:] << 8)).reshape(lead + (32 * q,))]
    if t:
        tail = arr[..., 64 * q:].astype(np.uint16)
        parts.append(tail[..., :h] | (tail[..., h:] << 8))
    return np.concatenate(parts, axis=-1)


def elems_to_bytes(el: np.ndarray) -> np.ndarray:
    el = np.asarray(el, dtype=np.uint16)
    n = el.shape[-1]
    s = 2 * n
    q, t = divmod(s, 64)
    h = t // 2
    lead = el.shape[:-1]
    out = np.zeros(lead + (s,), dtype=np.uint8)
    full = el[..., : 32 * q].reshape(lead + (q, 32))
    fb = out[..., : 64 * q].reshape(lead + (q, 64))
    fb[..., :32] = full & 0xFF
    fb[..., 32:] = full >> 8
    out[..., : 64 * q] = fb.reshape(lead + (64 * q,))
    if t:
        tail = el[..., 32 * q:]
        out[..., 64 * q: 64 * q + h] = tail & 0xFF
        out[..., 64 * q + h:] = tail >> 8
    return out


def rs_encode_symbols(data: np.ndarray, recovery_count: int) -> np.ndarray:
    """`ReedSolomonEncoder::encode(..).recovery_iter()` on (K, s) bytes -> (R, s) bytes."""
    return elems_to_bytes(rs_encode_elems(bytes_to_elems(data), recovery_count))


def rs_encode_all(data: np.ndarray, n_shards: int) -> np.ndarray:
    """`ReedSolomonEncoder::encode_all` (basic_encoding.rs:195-211): source || repair."""
    k = data.shape[0]
    return np.concatenate([data, rs_encode_symbols(data, n_shards - k)], axis=0)


def rs_decode_symbols(k: int, n_shards: int, symbol_size: int, symbols) -> np.ndarray:
    """`ReedSolomonDecoder::decode` (basic_encoding.rs:387-429) on (index, bytes) pairs.

    Wrong-size symbols are dropped; duplicate indices keep the first copy (the crate
    ignores duplicates).  Raises ValueError when fewer than k distinct shards arrive.
    """
    received = {}
    for idx, data in symbols:
        data = np.asarray(data, dtype=np.uint8)
        if data.shape[-1] != symbol_size or idx >= n_shards:
            continue
        if idx not in received:
            received[idx] = bytes_to_elems(data)
    return elems_to_bytes(rs_decode_elems(k, n_shards - k, received))


# ---------------------------------------------------------------------------------------------
# Walrus layer
# ---------------------------------------------------------------------------------------------


class DataTooLargeError(ValueError):
    pass


def max_n_faulty(n_shards: int) -> int:
    return (n_shards - 1) // 3


def source_symbols_for_n_shards(n_shards: int):
    """(primary = n - 2f, secondary = n - f) -- config.rs:717-725, bft.rs:12-25."""
    f = max_n_faulty(n_shards)
    return n_shards - 2 * f, n_shards - f


def compute_symbol_size(data_length: int, n_symbols: int, required_alignment: int = 2) -> int:
    """utils.rs:10-25; DataTooLarge if the size does not fit a u16."""
    data_length = max(data_length, 1)
    size = -(-data_length // n_symbols)
    size = -(-size // required_alignment) * required_alignment
    if size > 0xFFFF:
        raise DataTooLargeError("symbol size too large")
    return size


def leaf_hash(data: bytes) -> bytes:
    return hashlib.blake2b(b"\x00" + bytes(data), digest_size=32).digest()


def inner_hash(left: bytes, right: bytes) -> bytes:
    return hashlib.blake2b(b"\x01" + left + right, digest_size=32).digest()


EMPTY_NODE = bytes(32)


def merkle_root_from_leaf_hashes(leaves) -> bytes:
    """merkle.rs:226-266: odd levels padded with an all-zero node; no leaves -> zeros."""
    nodes = list(leaves)
    if not nodes:
        return EMPTY_NODE
    while len(nodes) > 1:
        if len(nodes) % 2:
            nodes.append(EMPTY_NODE)
        nodes = [inner_hash(nodes[i], nodes[i + 1]) for i in range(0, len(nodes), 2)]
    return nodes[0]


def merkle_root(leaf_data) -> bytes:
    return merkle_root_from_leaf_hashes([leaf_hash(x) for x in leaf_data])


def merkle_nodes(leaf_data) -> list:
    """MerkleTree::build's `nodes` (merkle.rs:216-266): levels from the leaf hashes up, every
    level of more than one node padded to even with the zero node, the root last."""
    level = [leaf_hash(x) for x in leaf_data]
    nodes = []
    while len(level) > 1:
        if len(level) % 2:
            level.append(EMPTY_NODE)
        nodes += level
        level = [inner_hash(level[i], level[i + 1]) for i in range(0, len(level), 2)]
    return nodes + level


def merkle_proof(leaf_data, leaf_index: int) -> list:
    """MerkleTree::get_proof (merkle.rs:281-309): sibling path leaf -> root."""
    n = len(leaf_data)
    if leaf_index >= n:
        raise IndexError("LeafIndexOutOfBounds")
    nodes = merkle_nodes(leaf_data)
    path, idx, cnt, base = [], leaf_index, n, 0
    while cnt > 1:
        cnt += cnt % 2
        path.append(nodes[base + (idx ^ 1)])
        idx //= 2
        base += cnt
        cnt //= 2
    return path


def merkle_proof_root(path, leaf: bytes, leaf_index: int) -> bytes:
    """MerkleProof::compute_root (merkle.rs:150-169)."""
    if leaf_index >> len(path):
        raise IndexError("LeafIndexOutOfBounds")
    cur, idx = leaf_hash(leaf), leaf_index
    for sib in path:
        cur = inner_hash(cur, sib) if idx % 2 == 0 else inner_hash(sib, cur)
        idx //= 2
    return cur


def blob_id(pair_hashes, unencoded_length: int, encoding_type: int = 1) -> bytes:
    """metadata.rs:571-578 + lib.rs:159-176."""
    root = merkle_root([p + s for p, s in pair_hashes])
    h = hashlib.blake2b(digest_size=32)
    h.update(bytes([encoding_type]))
    h.update(int(unencoded_length).to_bytes(8, "little"))
    h.update(root)
    return h.digest()


def blob_id_to_str(bid: bytes) -> str:
    return base64.urlsafe_b64encode(bid).decode().rstrip("=")


@dataclass
class Rs2Params:
    n_shards: int
    n_primary: int      # K_p: rows of the message matrix = symbols per secondary sliver
    n_secondary: int    # K_s: columns of the message matrix = symbols per primary sliver
    symbol_size: int
    blob_len: int

    @classmethod
    def for_blob(cls, n_shards: int, blob_len: int) -> "Rs2Params":
        kp, ks = source_symbols_for_n_shards(n_shards)
        return cls(n_shards, kp, ks, compute_symbol_size(blob_len, kp * ks), blob_len)

    @classmethod
    def for_test(cls, kp: int, ks: int, n_shards: int, blob_len: int) -> "Rs2Params":
        """ReedSolomonEncodingConfig::new_for_test (config.rs:506-523)."""
        return cls(n_shards, kp, ks, compute_symbol_size(blob_len, kp * ks), blob_len)


def message_matrix(blob: bytes, p: Rs2Params) -> np.ndarray:
    """(K_p, K_s, s) symbols; symbol (r, c) = blob[(r*K_s + c)*s ..], zero padded."""
    total = p.n_primary * p.n_secondary * p.symbol_size
    buf = np.zeros(total, dtype=np.uint8)
    b = np.frombuffer(bytes(blob), dtype=np.uint8)
    buf[: len(b)] = b
    return buf.reshape(p.n_primary, p.n_secondary, p.symbol_size)


def expanded_matrix(blob: bytes, p: Rs2Params) -> np.ndarray:
    """The full n x n symbol matrix (ExpandedMessageMatrix, blob_encoding.rs:620-714)."""
    n, kp, ks = p.n_shards, p.n_primary, p.n_secondary
    m = bytes_to_elems(message_matrix(blob, p))           # (kp, ks, E)
    e = m.shape[-1]
    x = np.zeros((n, n, e), dtype=np.uint16)
    x[:kp, :ks] = m
    # rows: secondary encoding (K = K_s) -> columns K_s..n
    rows_in = np.ascontiguousarray(m.transpose(1, 0, 2)).reshape(ks, kp * e)
    rec = rs_encode_elems(rows_in, n - ks).reshape(n - ks, kp, e)
    x[:kp, ks:] = rec.transpose(1, 0, 2)
    # columns: primary encoding (K = K_p) -> rows K_p..n, for all n columns
    cols_in = x[:kp].reshape(kp, n * e)
    x[kp:] = rs_encode_elems(cols_in, n - kp).reshape(n - kp, n, e)
    return elems_to_bytes(x)                               # (n, n, s)


def compute_metadata_from_symbol_hashes(hashes, p: Rs2Params):
    """blob_encoding.rs:161-196: primary i = tree over row i, secondary i = column n-1-i."""
    n = p.n_shards
    pairs = []
    for i in range(n):
        prim = merkle_root_from_leaf_hashes([hashes[i][c] for c in range(n)])
        sec = merkle_root_from_leaf_hashes([hashes[r][n - 1 - i] for r in range(n)])
        pairs.append((prim, sec))
    return pairs, blob_id(pairs, p.blob_len)


@dataclass
class EncodedBlob:
    params: Rs2Params
    primary: np.ndarray      # (n, K_s*s) primary sliver i (by sliver index)
    secondary: np.ndarray    # (n, K_p*s) secondary sliver j (by sliver index)
    pair_hashes: list        # [(primary_hash, secondary_hash)] by sliver-pair index
    blob_id: bytes

    def sliver_pair(self, i: int):
        """SliverPair i = (primary i, secondary n-1-i) (blob_encoding.rs:357-361)."""
        return self.primary[i], self.secondary[self.params.n_shards - 1 - i]


def encode_with_metadata(blob: bytes, n_shards: int, params: Rs2Params = None) -> EncodedBlob:
    p = params or Rs2Params.for_blob(n_shards, len(blob))
    x = expanded_matrix(blob, p)
    n, kp, ks, s = p.n_shards, p.n_primary, p.n_secondary, p.symbol_size
    hashes = [[leaf_hash(x[r, c].tobytes()) for c in range(n)] for r in range(n)]
    pairs, bid = compute_metadata_from_symbol_hashes(hashes, p)
    primary = x[:, :ks].reshape(n, ks * s).copy()
    secondary = np.ascontiguousarray(x[:kp].transpose(1, 0, 2)).reshape(n, kp * s)
    return EncodedBlob(p, primary, secondary, pairs, bid)


def compute_metadata(blob: bytes, n_shards: int):
    enc = encode_with_metadata(blob, n_shards)
    return enc.pair_hashes, enc.blob_id


def decode_blob(n_shards: int, blob_len: int, axis: str, slivers) -> bytes:
    """BlobDecoder::decode (blob_encoding.rs:888-993).

    `slivers` is an iterable of (sliver_index, bytes).  Surplus slivers beyond the required
    count are dropped, duplicate indices are skipped and wrong-length slivers are dropped; too
    few distinct slivers -> ValueError (DecodeError::DecodingUnsuccessful).
    """
    p = Rs2Params.for_blob(n_shards, blob_len)
    n, kp, ks, s = p.n_shards, p.n_primary, p.n_secondary, p.symbol_size
    primary = axis == "primary"
    k, sliver_len = (kp, ks) if primary else (ks, kp)
    chosen, seen = [], set()
    for idx, data in slivers:
        if len(chosen) == k:
            break
        if idx in seen:
            continue
        data = np.frombuffer(bytes(data), dtype=np.uint8)
        if data.size != sliver_len * s:
            continue
        chosen.append((idx, data.reshape(sliver_len, s)))
        seen.add(idx)
    if len(chosen) != k:
        raise ValueError("DecodingUnsuccessful")
    # one 1D decode per codeword position of the sliver; all share the erasure pattern
    stacked = {idx: bytes_to_elems(d).reshape(-1) for idx, d in chosen}   # sliver_len*E
    dec = rs_decode_elems(k, n - k, stacked)                                # (k, sliver_len*E)
    e = s // 2
    dec = dec.reshape(k, sliver_len, e)
    if primary:
        m = dec                                  # rows
    else:
        m = dec.transpose(1, 0, 2)               # secondary sliver j = column j
    return elems_to_bytes(m).reshape(-1)[:blob_len].tobytes()


def recovery_symbols(sliver: np.ndarray, axis: str, p: Rs2Params) -> np.ndarray:
    """SliverData::recovery_symbols (slivers.rs:169-178): expand on the orthogonal axis."""
    s = p.symbol_size
    data = np.asarray(sliver, dtype=np.uint8).reshape(-1, s)
    return rs_encode_all(data, p.n_shards)


def sliver_merkle_root(sliver: np.ndarray, axis: str, p: Rs2Params) -> bytes:
    """SliverData::get_merkle_root (slivers.rs:387-392)."""
    return merkle_root([sym.tobytes() for sym in recovery_symbols(sliver, axis, p)])


def recover_sliver(axis: str, symbols, p: Rs2Params) -> np.ndarray:
    """SliverData::recover_sliver_without_verification (slivers.rs:246-289).

    Recovering a primary sliver decodes the row code (K = K_s) from symbols indexed by the
    secondary sliver they came from; a secondary sliver decodes the column code (K = K_p).
    """
    k = p.n_secondary if axis == "primary" else p.n_primary
    return rs_decode_symbols(k, p.n_shards, p.symbol_size, symbols).reshape(-1)

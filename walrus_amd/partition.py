"""One large blob across G GPUs: row/column-partitioned Red Stuff encode and decode.

SURVEY.md 8(e) / config C4.  The reference encodes one blob on one thread
(BlobEncoder::encode_with_metadata, blob_encoding.rs:277-368: rows, then columns, then the
n^2 leaf hashes and 2n Merkle trees, then the primary slivers and the pair zip, :345-361); here
rank g of G (one process per GPU) owns

  rows R_g      a contiguous slice of the K_p message rows (so the host-to-device copy of the
                blob needs no gather),
  sliver pairs  P_g = [g*nt, (g+1)*nt) (nt = ceil(n/G)), and with them
  columns C_g   = { n-1-i : i in P_g }, the columns whose secondary slivers pair with P_g's
                primary slivers (SliverPairIndex::to_sliver_index, lib.rs:485-491) -- a
                contiguous column range, so a pair's secondary sliver never leaves its rank,

and runs

  rows phase    row code on R_g -> the rows' n - K_s repair symbols
  exchange 1    one all-to-all (RCCL over xGMI) of the K_p x n row-expanded symbols into column
                ownership; it lands directly in X [n][nt][s], the rank's columns row-major
                (blob_encoding.rs:309-324)
  columns phase column code on C_g -> all n symbols of those columns, n leaf hashes per column,
                the column Merkle trees = secondary hashes (blob_encoding.rs:161-196, 337-354)
  exchange 2    all-to-all of leaf digests into row (pair) ownership -- X's leaf rows are already
                grouped by destination, so there is no packing
  trees phase   row Merkle trees of rows P_g = primary hashes
  exchange 3    all-to-all of the systematic-column symbols of every row into pair ownership:
                rank g assembles its primary slivers P_g [nt][K_s*s] (blob_encoding.rs:345-353),
                and gathers its secondary slivers C_g [nt][K_p*s] from X locally
  exchange 4    all-gather of the 2n roots -> metadata and BlobId on every rank
                (metadata.rs:571-578, lib.rs:159-176)

so each rank ends with its sliver pairs P_g (primary i, secondary n-1-i: blob_encoding.rs:357-361)
and the metadata -- what a store operation uploads from that GPU.

The primary-axis decode (BlobDecoder::decode, blob_encoding.rs:888-993) is column-partitioned
by systematic columns (rank g decodes columns [g*ns, (g+1)*ns), ns = ceil(K_s/G)): column c of
the blob needs only symbol c of each received primary sliver, so after one ingest exchange (a
scatter from the rank the slivers arrived on, or an all-to-all from the ranks that hold them)
each rank decodes its columns and the decoded columns are gathered (RCCL) to the root, which
lays them into the blob.

Compute runs through an `ops` object: `DeviceOps` (the HIP engine's C ABI: rs2_codec_*,
rs2_copy_segments_device_async, rs2_leaf_hashes_device_async, rs2_merkle_roots_device_async,
rs2_blob_id_device_async) in the product; tests substitute a CPU checker to exercise the
partitioning and the exchanges on gloo without a GPU.  Exchanges run through an `exchange`
object: `DistExchange` (torch.distributed: nccl = RCCL on ROCm, or gloo), `LocalExchange` (one
rank), or `simulate_*` below, which runs all G ranks' phases in one process and shuffles the
exchanged tensors itself (multi-rank parity on a single GPU).
"""
from __future__ import annotations

import ctypes
import math
from collections import OrderedDict
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

from . import _lib


def _cdiv(a: int, b: int) -> int:
    return -(-a // b)


@dataclass(frozen=True)
class Partition:
    """Row / column / sliver-pair ownership of one blob's 2D code across `world` ranks."""
    n: int
    kp: int
    ks: int
    s: int
    blob_len: int
    world: int

    @classmethod
    def for_blob(cls, n_shards: int, blob_len: int, world: int) -> "Partition":
        from .encoding import source_symbols_for_n_shards, compute_symbol_size
        kp, ks = source_symbols_for_n_shards(n_shards)
        s = compute_symbol_size(blob_len, kp * ks)
        if world < 1:
            raise ValueError("world must be >= 1")
        return cls(n_shards, kp, ks, s, blob_len, world)

    @property
    def geo(self) -> Tuple[int, int, int, int, int]:
        """Everything the layouts depend on (not the blob length): offset-table cache key."""
        return (self.n, self.kp, self.ks, self.s, self.world)

    # message rows (row code, K = K_s) -----------------------------------------------------
    @property
    def nr(self) -> int:           # rows per rank (padded)
        return _cdiv(self.kp, self.world)

    def rows(self, g: int) -> range:
        return range(min(g * self.nr, self.kp), min((g + 1) * self.nr, self.kp))

    def row_bytes(self, g: int) -> range:
        """Blob bytes of rank g's rows (the rest of the rows' symbols is zero padding)."""
        r = self.rows(g)
        row = self.ks * self.s
        return range(min(r.start * row, self.blob_len), min(r.stop * row, self.blob_len))

    # sliver pairs and the columns that pair with them -------------------------------------
    @property
    def nt(self) -> int:           # sliver pairs (and column slots) per rank (padded)
        return _cdiv(self.n, self.world)

    def pairs(self, g: int) -> range:
        """Rank g's sliver pairs = its primary slivers = the rows of its primary trees."""
        return range(min(g * self.nt, self.n), min((g + 1) * self.nt, self.n))

    tree_rows = pairs

    def nv(self, g: int) -> int:   # valid column slots (= pairs) of rank g
        return len(self.pairs(g))

    def cstart(self, g: int) -> int:
        """First column of rank g; its slot j holds column cstart + j (j < nv)."""
        return self.n - self.pairs(g).stop

    def cols(self, g: int) -> range:
        return range(self.cstart(g), self.cstart(g) + self.nv(g))

    def col(self, g: int, j: int) -> int:
        """Global column of rank g's column slot j, or -1 for a padding slot."""
        return self.cstart(g) + j if j < self.nv(g) else -1

    def col_owner(self, c: int) -> Tuple[int, int]:
        """(rank, slot) holding column c: the owner of pair n-1-c."""
        g = (self.n - 1 - c) // self.nt
        return g, c - self.cstart(g)

    def msys(self, g: int) -> int:
        """Rank g's systematic columns (c < K_s): slots [0, msys), its share of the primary
        slivers' bytes."""
        return max(0, min(self.ks - self.cstart(g), self.nv(g)))

    @property
    def x_rows(self) -> int:       # rows of X (exchange 1 lands world*nr padded rows in it)
        return max(self.n, self.world * self.nr)

    # the primary-axis decode's column partition -----------------------------------------
    @property
    def ns(self) -> int:           # systematic columns per rank in the decode (padded)
        return _cdiv(self.ks, self.world)

    def sys_cols(self, g: int) -> range:
        """Rank g's systematic columns in the decode."""
        return range(min(g * self.ns, self.ks), min((g + 1) * self.ns, self.ks))


def _unit(*vals) -> int:
    """Widest copy width (16, 8, 4, 2 or 1 bytes) dividing every value."""
    g = 0
    for v in vals:
        g = math.gcd(g, int(v))
    for u in (16, 8, 4, 2):
        if g % u == 0:
            return u
    return 1


def _groups(items: Sequence[Tuple[int, int, int]]) -> Dict[int, Tuple[List[int], List[int]]]:
    """(length, src offset, dst offset) segments grouped by length (one copy launch each)."""
    out: Dict[int, Tuple[List[int], List[int]]] = {}
    for ln, so, do in items:
        if ln > 0:
            a, b = out.setdefault(ln, ([], []))
            a.append(so)
            b.append(do)
    return out


# ---------------------------------------------------------------------------------------------
# compute backends
# ---------------------------------------------------------------------------------------------
class DeviceOps:
    """The HIP engine (C ABI) on torch device tensors; work goes on torch's current stream."""

    MAX_TABLES = 512  # offset tables kept on the device (LRU)

    def __init__(self):
        self._codecs = {}
        self._offs: "OrderedDict" = OrderedDict()

    def _codec(self, k: int, n: int, s: int):
        key = (k, n, s)
        h = self._codecs.get(key)
        if h is None:
            from .encoding import _ok
            h = ctypes.c_void_p()
            _ok(_lib.lib().rs2_codec_create(k, n, s, ctypes.byref(h)))
            self._codecs[key] = h
        return h

    def __del__(self):
        if _lib._LIB is not None:
            for h in getattr(self, "_codecs", {}).values():
                _lib.lib().rs2_codec_destroy(h)

    @staticmethod
    def _stream(t):
        import torch
        return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)

    def encode_lines(self, k, n, s, lines, src, src_off, src_ss, src_ls, dst, dst_off,
                     dst_ss, dst_ls):
        from .encoding import _ok
        if lines == 0:
            return
        _ok(_lib.lib().rs2_codec_encode_device_async(
            self._codec(k, n, s), lines, src.data_ptr() + src_off, src_ss, src_ls,
            dst.data_ptr() + dst_off, dst_ss, dst_ls, self._stream(src)))

    def decode_lines(self, k, n, s, lines, idx, base, sym_off, line_stride, out, out_ss,
                     out_ls, out_limit):
        from .encoding import _ok
        if lines == 0:
            return
        m = len(idx)
        ia = (ctypes.c_uint16 * m)(*idx)
        oa = (ctypes.c_uint64 * m)(*sym_off)
        _ok(_lib.lib().rs2_codec_decode_device_async(
            self._codec(k, n, s), lines, m, ia, base.data_ptr(), oa, line_stride,
            out.data_ptr(), out_ss, out_ls, out_limit, self._stream(base)), decode=True)

    def offsets(self, key, build, device):
        """Device copy of the int64 offset table build() and the gcd of its entries (the
        copy-width bound).  Cached under `key` (layout parameters only, never a blob length;
        None = not cached), at most MAX_TABLES tables, least recently used out first."""
        import numpy as np
        import torch
        k = None if key is None else (key, str(device))
        t = self._offs.get(k) if k is not None else None
        if t is None:
            a = np.ascontiguousarray(build(), dtype=np.int64)
            t = (torch.from_numpy(a).to(device), int(np.gcd.reduce(a)) if a.size else 0)
            if k is not None:
                self._offs[k] = t
                while len(self._offs) > self.MAX_TABLES:
                    self._offs.popitem(last=False)
        elif k is not None:
            self._offs.move_to_end(k)
        return t

    def copy_segments(self, src, dst, src_a, dst_a, count_b, ssb, dsb, seg_len):
        """rs2_copy_segments_device_async: segment (a, b) = seg_len bytes from
        src + src_a[a] + b*ssb to dst + dst_a[a] + b*dsb (offset tables from offsets())."""
        from .encoding import _ok
        (sa, gs), (da, gd) = src_a, dst_a
        if sa.numel() == 0 or count_b == 0 or seg_len == 0:
            return
        unit = _unit(gs, gd, ssb, dsb, seg_len, src.data_ptr(), dst.data_ptr())
        _ok(_lib.lib().rs2_copy_segments_device_async(
            src.data_ptr(), dst.data_ptr(), sa.numel(), sa.data_ptr(), da.data_ptr(), count_b, ssb,
            dsb, seg_len, unit, self._stream(src)))

    def leaf_hashes(self, symbols, count, s, out):
        from .encoding import _ok
        _ok(_lib.lib().rs2_leaf_hashes_device_async(symbols.data_ptr(), count, s, out.data_ptr(),
                                                    self._stream(symbols)))

    def merkle_roots(self, leaves, n_trees, n_leaves, tree_stride, leaf_stride, out,
                     root_stride):
        from .encoding import _ok
        if n_trees == 0:
            return
        _ok(_lib.lib().rs2_merkle_roots_device_async(
            leaves.data_ptr(), n_trees, n_leaves, tree_stride, leaf_stride, out.data_ptr(),
            root_stride, self._stream(leaves)))

    def blob_id(self, hashes, n, blob_len, out):
        from .encoding import _ok
        _ok(_lib.lib().rs2_blob_id_device_async(hashes.data_ptr(), n, blob_len, out.data_ptr(),
                                                self._stream(hashes)))


def _copy_grouped(ops, src, dst, segs, count_b, ssb, dsb, key, device):
    """copy_segments over segments of several lengths: segs = [(len, src_off, dst_off)], one
    launch per distinct length (a handful: full, last-rank and partial ranges)."""
    for ln, (so, do) in sorted(_groups(segs).items()):
        sa = ops.offsets(None if key is None else key + ("s", ln), lambda: so, device)
        da = ops.offsets(None if key is None else key + ("d", ln), lambda: do, device)
        ops.copy_segments(src, dst, sa, da, count_b, ssb, dsb, ln)


# ---------------------------------------------------------------------------------------------
# exchanges
# ---------------------------------------------------------------------------------------------
class DistExchange:
    """Collectives over torch.distributed (backend nccl = RCCL over xGMI, or gloo on CPU)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)

    def all_to_all(self, send, in_splits=None, out_splits=None, out=None):
        """all_to_all_single: send's chunk h (equal chunks, or in_splits[h] bytes) to rank h;
        the chunks received from ranks 0..G-1 back to back (equal, or out_splits[g] bytes),
        into `out` when given."""
        import torch
        if out is None:
            total = send.numel() if out_splits is None else sum(out_splits)
            out = torch.empty(total, dtype=send.dtype, device=send.device)
        self.dist.all_to_all_single(out, send, output_split_sizes=out_splits,
                                    input_split_sizes=in_splits, group=self.group)
        return out

    def all_gather(self, t):
        import torch
        parts = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(parts, t, group=self.group)
        return torch.cat(parts)

    def gather(self, t, dst: int = 0):
        import torch
        parts = [torch.empty_like(t) for _ in range(self.world)] if self.rank == dst else None
        self.dist.gather(t, parts, dst=dst, group=self.group)
        return torch.cat(parts) if parts is not None else None

    def scatter(self, parts, like, src: int = 0):
        """parts: `world` equal tensors on `src` (None elsewhere) -> this rank's part."""
        import torch
        out = torch.empty_like(like)
        self.dist.scatter(out, list(parts) if self.rank == src else None, src=src,
                          group=self.group)
        return out


class HostStagedExchange(DistExchange):
    """DistExchange for device tensors over a host backend (gloo): every collective stages its
    tensors through host memory.  Several ranks that share one GPU (RCCL refuses two ranks on
    one device) then run the real multi-process exchanges beside the device engine
    (tests/test_gpu_dist.py); a multi-GPU run uses DistExchange over nccl (RCCL) instead."""

    def all_to_all(self, send, in_splits=None, out_splits=None, out=None):
        got = super().all_to_all(send.cpu(), in_splits, out_splits)
        if out is None:
            return got.to(send.device)
        out.copy_(got)
        return out

    def all_gather(self, t):
        return super().all_gather(t.cpu()).to(t.device)

    def gather(self, t, dst: int = 0):
        out = super().gather(t.cpu(), dst)
        return out.to(t.device) if out is not None else None

    def scatter(self, parts, like, src: int = 0):
        host = [p.cpu() for p in parts] if parts is not None else None
        return super().scatter(host, like.cpu(), src).to(like.device)


class LocalExchange:
    """The exchanges of a one-rank world (no process group): every collective is the identity."""
    world, rank = 1, 0

    def all_to_all(self, send, in_splits=None, out_splits=None, out=None):
        if out is None or out.data_ptr() == send.data_ptr():
            return send if out is None else out
        out.copy_(send)
        return out

    def all_gather(self, t):
        return t

    def gather(self, t, dst: int = 0):
        return t

    def scatter(self, parts, like, src: int = 0):
        return parts[0]


# ---------------------------------------------------------------------------------------------
# the partitioned encoder (one instance per rank)
# ---------------------------------------------------------------------------------------------
class RankEncoder:
    """Rank g's share of encode_with_metadata for one blob (phases; see module docstring)."""

    def __init__(self, part: Partition, rank: int, ops, device):
        self.p, self.g, self.ops, self.device = part, rank, ops, device

    def _t(self, nbytes):
        import torch
        return torch.empty(max(nbytes, 1), dtype=torch.uint8, device=self.device)

    def _offs(self, name, build):
        return self.ops.offsets((name, self.p.geo), build, self.device)

    def alloc_x(self):
        """X [x_rows][nt][s]: this rank's columns, row-major (slot j = column cstart + j)."""
        p = self.p
        return self._t(p.x_rows * p.nt * p.s)

    def rows_phase(self, rows, send=None):
        """rows: this rank's message rows, len(rows(g)) * K_s * s bytes (zero-padded blob
        slice).  Fills the exchange-1 send buffer [G][nr][nt][s] (chunk h = this rank's rows of
        rank h's columns; allocated unless given) and returns it."""
        p, g = self.p, self.g
        G, nt, nr, s, ks, n = p.world, p.nt, p.nr, p.s, p.ks, p.n
        nrg = len(p.rows(g))
        if send is None:
            send = self._t(G * nr * nt * s)
        if nrg == 0:
            return send
        rep = self._t(nrg * (n - ks) * s)
        # row code: line = row, source symbol c at row*ks*s + c*s -> repair j at row*(n-ks)*s + j*s
        self.ops.encode_lines(ks, n, s, nrg, rows, 0, s, ks * s, rep, 0, s, (n - ks) * s)

        def dst_of(c):
            h, j = p.col_owner(c)
            return (h * nr * nt + j) * s
        # pack: column c of local row b -> chunk of c's owner, its slot, row b
        src = self._offs("r1_sys_src", lambda: [c * s for c in range(ks)])
        dst = self._offs("r1_sys_dst", lambda: [dst_of(c) for c in range(ks)])
        self.ops.copy_segments(rows, send, src, dst, nrg, ks * s, nt * s, s)
        src = self._offs("r1_rep_src", lambda: [q * s for q in range(n - ks)])
        dst = self._offs("r1_rep_dst", lambda: [dst_of(ks + q) for q in range(n - ks)])
        self.ops.copy_segments(rep, send, src, dst, nrg, (n - ks) * s, nt * s, s)
        return send

    def columns_phase(self, X):
        """X [x_rows][nt][s] with rows 0..K_p received.  Column code (rows K_p..n), leaf hashes
        and column trees.  Returns (leaves [G*nt][nt][32] = the exchange-2 send buffer,
        secondary roots [nt][32] by slot)."""
        p = self.p
        G, nt, s, kp, n = p.world, p.nt, p.s, p.kp, p.n
        nv = p.nv(self.g)
        # column code: line = slot, source row r at r*nt*s -> repair row kp + j at (kp+j)*nt*s
        self.ops.encode_lines(kp, n, s, nv, X, 0, nt * s, s, X, kp * nt * s, nt * s, s)
        leaves = self._t(G * nt * nt * 32)      # rows >= n: padding of the last chunk
        self.ops.leaf_hashes(X, n * nt, s, leaves)
        sec = self._t(nt * 32)
        self.ops.merkle_roots(leaves, nv, n, 32, nt * 32, sec, 32)
        return leaves[:G * nt * nt * 32], sec[:nt * 32]

    def trees_phase(self, recv2):
        """recv2 [G][nt][nt][32]: from rank h, the leaf digests of my rows in h's column
        slots.  Returns primary roots [nt][32] of my rows (pairs(g))."""
        p = self.p
        G, nt, n = p.world, p.nt, p.n
        nvm = p.nv(self.g)
        prim = self._t(nt * 32)
        if nvm:
            # row t's leaves in column order: rank h's slots go to columns cstart(h)..
            row_leaves = self._t(nvm * n * 32)
            segs = [(p.nv(h) * 32, h * nt * nt * 32, p.cstart(h) * 32) for h in range(G)]
            _copy_grouped(self.ops, recv2, row_leaves, segs, nvm, nt * 32, n * 32,
                          ("trees", p.geo), self.device)
            self.ops.merkle_roots(row_leaves, nvm, n, n * 32, 32, prim, 32)
        return prim[:nt * 32]

    def primary_send(self, X):
        """Exchange-3 send buffer [G*nt][msys][s]: every row's symbols in my systematic slots
        (chunk h = the rows of h's pairs).  For one rank this is the primary slivers already."""
        p = self.p
        m = p.msys(self.g)
        send = self._t(p.world * p.nt * m * p.s)[:p.world * p.nt * m * p.s]
        if m:
            zero = self._offs("zero", lambda: [0])
            self.ops.copy_segments(X, send, zero, zero, p.n, p.nt * p.s, m * p.s, m * p.s)
        return send

    def primary_splits(self):
        p = self.p
        return ([p.nt * p.msys(self.g) * p.s] * p.world,
                [p.nt * p.msys(h) * p.s for h in range(p.world)])

    def assemble_primary(self, recv3):
        """recv3: from every rank h its [nt][msys(h)][s] systematic symbols of my rows ->
        my primary slivers [nv][K_s*s] (pair order)."""
        p = self.p
        if p.world == 1:
            return recv3[:p.n * p.ks * p.s]
        nvm = p.nv(self.g)
        prim = self._t(nvm * p.ks * p.s)
        segs, off = [], 0
        for h in range(p.world):
            m = p.msys(h)
            segs.append((m * p.s, off, p.cstart(h) * p.s))
            off += p.nt * m * p.s
        # segment (h, t): ms bytes of h's row t to my sliver t at column cstart(h); grouped by
        # msys (the row stride of h's chunk), which the length also fixes
        for ln, (so, do) in sorted(_groups(segs).items()):
            sa = self.ops.offsets(("asm_s", p.geo, self.g, ln), lambda: so, self.device)
            da = self.ops.offsets(("asm_d", p.geo, self.g, ln), lambda: do, self.device)
            self.ops.copy_segments(recv3, prim, sa, da, nvm, ln, p.ks * p.s, ln)
        return prim[:nvm * p.ks * p.s]

    def secondary_slivers(self, X):
        """My columns' secondary slivers [nv][K_p*s], slot order (sliver index cstart + j):
        rows 0..K_p of each slot of X."""
        p = self.p
        nv, kp, s, nt = p.nv(self.g), p.kp, p.s, p.nt
        sec = self._t(nv * kp * s)
        if nv:
            src = self._offs("sec_src", lambda: [r * nt * s for r in range(kp)])
            dst = self._offs("sec_dst", lambda: [r * s for r in range(kp)])
            self.ops.copy_segments(X, sec, src, dst, nv, s, kp * s, s)
        return sec[:nv * kp * s]

    def finish(self, all_prim, all_sec):
        """all_prim [G*nt][32] (row order), all_sec [G*nt][32] (rank, slot order) -> (hashes
        [n][64] by sliver-pair index, blob_id [32])."""
        p = self.p
        n, nt, ops, dev = p.n, p.nt, self.ops, self.device
        hashes = self._t(n * 64)
        zero = self._offs("zero", lambda: [0])
        ops.copy_segments(all_prim, hashes, zero, zero, n, 32, 64, 32)   # pair i <- row root i

        def sec_slot(i):  # column n-1-i sits on rank i // nt, slot pairs(g).stop - 1 - i
            g = i // nt
            return g * nt + p.pairs(g).stop - 1 - i
        src = self._offs("fin_sec_src", lambda: [sec_slot(i) * 32 for i in range(n)])
        dst = self._offs("fin_sec_dst", lambda: [i * 64 + 32 for i in range(n)])
        ops.copy_segments(all_sec, hashes, src, dst, 1, 0, 0, 32)
        bid = self._t(32)
        self.ops.blob_id(hashes, n, p.blob_len, bid)
        return hashes[:n * 64], bid[:32]


@dataclass
class RankEncoded:
    """What one rank holds after a partitioned encode: its sliver pairs and the metadata."""
    pairs: range         # sliver-pair indices P_g
    primary: object      # [len(pairs)][K_s*s]: primary sliver i at row i - pairs.start
    secondary: object    # [len(pairs)][K_p*s]: secondary sliver cstart + q at row q, i.e. pair
    #                      i's secondary (index n-1-i) at row pairs.stop - 1 - i
    hashes: object       # [n][64] pair hashes (every rank)
    blob_id: object      # [32] (every rank)

    def sliver_pair(self, i: int, part: Partition):
        """(primary i, secondary n-1-i) of pair i (views)."""
        a, b = part.ks * part.s, part.kp * part.s
        q, r = i - self.pairs.start, self.pairs.stop - 1 - i
        return self.primary[q * a:(q + 1) * a], self.secondary[r * b:(r + 1) * b]


def encode_distributed(part: Partition, rows, ops, exchange, device) -> RankEncoded:
    """Partitioned encode_with_metadata on this rank: rank g's message rows in, its sliver
    pairs and the blob's metadata out (exchange = DistExchange, or LocalExchange)."""
    p = part
    enc = RankEncoder(p, exchange.rank, ops, device)
    X = enc.alloc_x()
    head = X[:p.world * p.nr * p.nt * p.s]
    if p.world == 1:   # the exchange is the identity: pack straight into X
        enc.rows_phase(rows, send=head)
    else:
        exchange.all_to_all(enc.rows_phase(rows), out=head)
    send2, sec_roots = enc.columns_phase(X)
    prim_roots = enc.trees_phase(exchange.all_to_all(send2))
    send3 = enc.primary_send(X)
    ins, outs = enc.primary_splits()
    primary = enc.assemble_primary(exchange.all_to_all(send3, ins, outs))
    secondary = enc.secondary_slivers(X)
    del X, head, send2, send3
    hashes, bid = enc.finish(exchange.all_gather(prim_roots), exchange.all_gather(sec_roots))
    return RankEncoded(p.pairs(exchange.rank), primary, secondary, hashes, bid)


# ---------------------------------------------------------------------------------------------
# the partitioned decoder
# ---------------------------------------------------------------------------------------------
def _decode_my_columns(p: Partition, rank: int, ops, idx: Sequence[int], base, sym_off,
                       line_stride: int, device):
    """Primary-axis decode of rank g's systematic columns sys_cols(g): symbol (column j of
    the range) of sliver idx[i] at base + sym_off[i] + j*line_stride.  Returns [K_p][ns][s]
    (rows of the decoded message columns; padding columns unwritten)."""
    import torch
    cols = p.sys_cols(rank)
    out = torch.empty(max(p.kp * p.ns * p.s, 1), dtype=torch.uint8, device=device)
    ops.decode_lines(p.kp, p.n, p.s, len(cols), list(idx), base, list(sym_off), line_stride,
                     out, p.ns * p.s, p.s, p.kp * p.ns * p.s)
    return out[:p.kp * p.ns * p.s]


def assemble_blob(part: Partition, gathered, ops):
    """Root side of the decode: gathered [G][K_p][ns][s] decoded columns -> blob bytes (column c
    of row r from rank c // ns, its slot c % ns)."""
    import torch
    p = part
    kp, ks, ns, s = p.kp, p.ks, p.ns, p.s
    if p.world == 1:  # one rank's columns are the whole rows: the layout is the blob's
        return gathered.reshape(-1)[:p.blob_len]
    out = torch.empty(max(kp * ks * s, 1), dtype=torch.uint8, device=gathered.device)
    segs = [(len(p.sys_cols(g)) * s, g * kp * ns * s, g * ns * s) for g in range(p.world)]
    _copy_grouped(ops, gathered, out, segs, kp, ns * s, ks * s, ("asm_blob", p.geo),
                  gathered.device)
    return out[:p.blob_len]


def decode_distributed(part: Partition, enc: RankEncoded, idx: Sequence[int], ops, exchange,
                       device, root: int = 0):
    """BlobDecoder::decode (blob_encoding.rs:888-993) from the K_p primary slivers `idx` where
    the partitioned encode left them (each on the rank that owns its pair): one all-to-all
    sends every rank its decode columns of the chosen slivers this rank holds, each rank
    decodes its columns, one gather (RCCL) brings them to `root`.  Returns the blob on the
    root, None elsewhere."""
    import torch
    p = part
    G, me, ns, s, ks = p.world, exchange.rank, p.ns, p.s, p.ks
    held = [[int(i) for i in idx if int(i) in p.pairs(h)] for h in range(G)]
    lo = p.pairs(me).start
    if G == 1:
        cols = _decode_my_columns(p, me, ops, held[0], enc.primary,
                                  [(i - lo) * ks * s for i in held[0]], s, device)
    else:
        mine = held[me]
        cnt = len(mine)
        send = torch.empty(max(G * cnt * ns * s, 1), dtype=torch.uint8, device=device)
        segs = [(len(p.sys_cols(h)) * s, (i - lo) * ks * s + h * ns * s, (h * cnt + k) * ns * s)
                for h in range(G) for k, i in enumerate(mine)]
        _copy_grouped(ops, enc.primary, send, segs, 1, 0, 0, None, device)
        recv = exchange.all_to_all(send[:G * cnt * ns * s], [cnt * ns * s] * G,
                                   [len(held[h]) * ns * s for h in range(G)])
        order = [i for h in range(G) for i in held[h]]
        cols = _decode_my_columns(p, me, ops, order, recv, [k * ns * s for k in range(len(order))],
                                  s, device)
    gathered = exchange.gather(cols, dst=root)
    return assemble_blob(p, gathered, ops) if gathered is not None else None


def scatter_sliver_columns(part: Partition, slivers, world: int, ops):
    """Root side of the decode ingest: K_p received primary slivers [K_p][K_s*s] (in the order
    of `idx`) -> per-rank column slices [G][K_p][ns][s] (rank g gets columns sys_cols(g) of every
    sliver; padding columns zero)."""
    import torch
    p = part
    kp, ks, ns, s = p.kp, p.ks, p.ns, p.s
    if world == 1:  # one rank takes every column: the slivers as they are
        return slivers[:kp * ks * s].view(1, kp, ks, s)
    send = torch.zeros((world, kp, ns, s), dtype=torch.uint8, device=slivers.device)
    segs = [(len(p.sys_cols(g)) * s, g * ns * s, g * kp * ns * s) for g in range(world)]
    _copy_grouped(ops, slivers, send, segs, kp, ks * s, ns * s, ("scatter", p.geo),
                  slivers.device)
    return send


def decode_from_slivers(part: Partition, slivers, idx: Sequence[int], ops, exchange, device,
                        root: int = 0):
    """BlobDecoder::decode (blob_encoding.rs:888-993) of one large blob from K_p full primary
    slivers that arrived on `root` (slivers [K_p][K_s*s] in the order of `idx`, None on the
    other ranks): scatter each rank its column range (one RCCL scatter: column c of the blob
    needs only symbol c of every sliver), decode the columns on every rank, gather the decoded
    columns back to the root (one RCCL gather).  Returns the blob on the root, None
    elsewhere."""
    import torch
    p = part
    like = torch.empty((p.kp, p.ns, p.s), dtype=torch.uint8, device=device)
    parts = None
    if exchange.rank == root:
        parts = list(scatter_sliver_columns(p, slivers, exchange.world, ops).unbind(0))
    mine = exchange.scatter(parts, like, src=root)
    # symbol j of received sliver i at i*ns*s + j*s
    cols = _decode_my_columns(p, exchange.rank, ops, idx, mine.reshape(-1),
                              [i * p.ns * p.s for i in range(len(idx))], p.s, device)
    gathered = exchange.gather(cols, dst=root)
    return assemble_blob(p, gathered, ops) if gathered is not None else None


def collect_primary(part: Partition, enc: RankEncoded, idx: Sequence[int], exchange,
                    root: int = 0):
    """The primary slivers `idx` ([K_p][K_s*s] in idx order) on `root`, gathered from the ranks
    that hold them (None elsewhere): stands for slivers a client downloaded."""
    import torch
    p = part
    G, L = p.world, p.ks * p.s
    held = [[int(i) for i in idx if int(i) in p.pairs(h)] for h in range(G)]
    lo = p.pairs(exchange.rank).start
    pv = enc.primary.view(-1, L) if L else enc.primary.view(0, 0)
    if G == 1:
        return pv[torch.tensor([i - lo for i in idx], device=pv.device)].reshape(-1)
    cmax = max(len(h) for h in held)
    mine = held[exchange.rank]
    buf = torch.zeros((cmax, L), dtype=torch.uint8, device=enc.primary.device)
    if mine:
        buf[:len(mine)] = pv[torch.tensor([i - lo for i in mine], device=pv.device)]
    got = exchange.gather(buf.reshape(-1), dst=root)
    if got is None:
        return None
    got = got.view(G, cmax, L)
    where = {i: (h, k) for h in range(G) for k, i in enumerate(held[h])}
    return torch.stack([got[where[int(i)][0], where[int(i)][1]] for i in idx]).reshape(-1)


# ---------------------------------------------------------------------------------------------
# single-process simulation of G ranks (multi-rank parity on one device)
# ---------------------------------------------------------------------------------------------
def _a2a(sends: List, in_splits=None) -> List:
    """All-to-all among the simulated ranks: sends[g] split into G chunks (equal, or
    in_splits[g]); rank h receives every g's chunk h, in rank order."""
    import torch
    G = len(sends)
    if in_splits is None:
        chunks = [list(s.view(G, -1).unbind(0)) for s in sends]
    else:
        chunks = [list(torch.split(s, list(sp))) for s, sp in zip(sends, in_splits)]
    return [torch.cat([chunks[g][h] for g in range(G)]) for h in range(G)]


def simulate_encode(part: Partition, blob_rows: List, ops, device) -> List[RankEncoded]:
    """All ranks' phases in one process; blob_rows[g] = rank g's rows (see rows_phase)."""
    import torch
    p = part
    G = p.world
    encs = [RankEncoder(p, g, ops, device) for g in range(G)]
    recv1 = _a2a([e.rows_phase(r) for e, r in zip(encs, blob_rows)])
    Xs = []
    for e, r in zip(encs, recv1):
        X = e.alloc_x()
        X[:r.numel()].copy_(r)
        Xs.append(X)
    del recv1
    outs = [e.columns_phase(X) for e, X in zip(encs, Xs)]
    recv2 = _a2a([o[0] for o in outs])
    prims = [e.trees_phase(r) for e, r in zip(encs, recv2)]
    del recv2
    sends3 = [e.primary_send(X) for e, X in zip(encs, Xs)]
    recv3 = _a2a(sends3, [e.primary_splits()[0] for e in encs])
    del sends3
    primary = [e.assemble_primary(r) for e, r in zip(encs, recv3)]
    del recv3
    secondary = [e.secondary_slivers(X) for e, X in zip(encs, Xs)]
    del Xs
    all_p, all_s = torch.cat(prims), torch.cat([o[1] for o in outs])
    res = []
    for g, e in enumerate(encs):
        h, b = e.finish(all_p, all_s)
        res.append(RankEncoded(p.pairs(g), primary[g], secondary[g], h, b))
    return res


def simulate_decode(part: Partition, encs: List[RankEncoded], idx: Sequence[int], ops, device):
    """decode_distributed with all G ranks in this process (the ingest all-to-all simulated)."""
    import torch
    p = part
    G, ns, s, ks = p.world, p.ns, p.s, p.ks
    held = [[int(i) for i in idx if int(i) in p.pairs(h)] for h in range(G)]
    order = [i for h in range(G) for i in held[h]]
    cols = []
    for g in range(G):
        # rank g's columns of every chosen sliver, straight from the holders' primary slivers
        recv = torch.empty(max(len(order) * ns * s, 1), dtype=torch.uint8, device=device)
        for k, i in enumerate(order):
            h = i // p.nt
            e = encs[h]
            a = (i - e.pairs.start) * ks * s + g * ns * s
            w = len(p.sys_cols(g)) * s
            recv[k * ns * s:k * ns * s + w].copy_(e.primary[a:a + w])
        cols.append(_decode_my_columns(p, g, ops, order, recv,
                                       [k * ns * s for k in range(len(order))], s, device))
    return assemble_blob(p, torch.cat(cols), ops)


def simulate_decode_from_slivers(part: Partition, slivers, idx: Sequence[int], ops, device):
    """decode_from_slivers with all G ranks in this process (scatter / gather simulated)."""
    import torch
    p = part
    send = scatter_sliver_columns(p, slivers, p.world, ops)
    cols = [_decode_my_columns(p, g, ops, idx, send[g].reshape(-1),
                               [i * p.ns * p.s for i in range(len(idx))], p.s, device)
            for g in range(p.world)]
    return assemble_blob(p, torch.cat(cols), ops)


def rows_of_blob(part: Partition, blob, g: int, device=None):
    """Rank g's message rows from the whole blob (tensor), zero-padded."""
    import torch
    r = part.rows(g)
    out = torch.zeros(max(len(r) * part.ks * part.s, 1), dtype=torch.uint8,
                      device=device if device is not None else blob.device)
    b = part.row_bytes(g)
    if len(b):
        out[:len(b)].copy_(blob[b.start:b.stop])
    return out


def gather_slivers(part: Partition, encs: List[RankEncoded]):
    """Every rank's assembled sliver pairs back in sliver-index order (tests): primary
    [n][K_s*s], secondary [n][K_p*s]."""
    import torch
    p = part
    prim = torch.cat([e.primary.reshape(-1) for e in encs]).view(p.n, p.ks * p.s)
    sec = torch.cat([encs[g].secondary.reshape(-1) for g in reversed(range(p.world))])
    return prim, sec.view(p.n, p.kp * p.s)

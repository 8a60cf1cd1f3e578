"""One large blob across G GPUs: row/column-partitioned Red Stuff encode and decode.

SURVEY.md 8(e) / config C4.  The reference encodes one blob on one thread
(BlobEncoder::encode_with_metadata, blob_encoding.rs:277-368: rows, then columns, then the
n^2 leaf hashes and 2n Merkle trees); here rank g of G (one process per GPU) does:

  rows phase    rows R_g of the K_p message rows (a contiguous slice of the blob, so the
                host-to-device copy needs no gather) -> their n - K_s row-code repair symbols
  exchange 1    one all-to-all (RCCL over xGMI) of the K_p x n row-encoded symbols into column
                ownership: rank g receives the K_p source symbols of its columns C_g, i.e. the
                secondary slivers C_g (blob_encoding.rs:309-324)
  columns phase column code on C_g -> all n symbols of those columns (secondary slivers C_g
                complete, primary slivers K_p..n column-sliced), n leaf hashes per column and
                the column Merkle trees = secondary hashes (blob_encoding.rs:161-196, 337-354)
  exchange 2    all-to-all of leaf digests (32 B per symbol) into row ownership P_g
  trees phase   row Merkle trees of rows P_g = primary hashes
  exchange 3    all-gather of the 2n roots -> metadata + BlobId on every rank
                (metadata.rs:571-578, lib.rs:159-176)

Columns are dealt so every rank gets the same number of systematic columns (c < K_s) and of
repair columns (c >= K_s): C_g = [g*ns, (g+1)*ns) u [K_s + g*nrp, K_s + (g+1)*nrp).  The
primary-axis decode (BlobDecoder::decode, blob_encoding.rs:888-993) is column-partitioned the
same way -- column c of the blob needs only symbol c of each received primary sliver, so there
is no exchange until the decoded columns are gathered (RCCL gather) to the root, which lays
them into the blob.  That is the only collective on the decode path.

Compute runs through an `ops` object: `DeviceOps` (the HIP engine's C ABI: rs2_codec_*,
rs2_leaf_hashes_device_async, rs2_merkle_roots_device_async, rs2_blob_id_device_async) in
the product; tests substitute a CPU checker to exercise the partitioning and the exchanges on
gloo without a GPU.  Exchanges run through an `exchange` object: `DistExchange`
(torch.distributed: nccl = RCCL on ROCm, or gloo), or `simulate_*` below, which runs all G
ranks' phases in one process and shuffles the exchanged tensors itself (multi-rank parity on a
single GPU).
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass
from typing import List, Optional, Sequence

from . import _lib


def _cdiv(a: int, b: int) -> int:
    return -(-a // b)


@dataclass(frozen=True)
class Partition:
    """Row / column ownership of one blob's 2D code across `world` ranks."""
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

    # columns (column code, K = K_p) ------------------------------------------------------
    @property
    def ns(self) -> int:           # systematic columns per rank (padded)
        return _cdiv(self.ks, self.world)

    @property
    def nrp(self) -> int:          # repair columns per rank (padded)
        return _cdiv(self.n - self.ks, self.world)

    @property
    def nc(self) -> int:           # column slots per rank
        return self.ns + self.nrp

    def col(self, g: int, j: int) -> int:
        """Global column of rank g's column slot j, or -1 for a padding slot."""
        if j < self.ns:
            c = g * self.ns + j
            return c if c < self.ks else -1
        c = self.ks + g * self.nrp + (j - self.ns)
        return c if c < self.n else -1

    def sys_cols(self, g: int) -> range:
        """Rank g's systematic columns (its share of the primary-axis decode)."""
        return range(min(g * self.ns, self.ks), min((g + 1) * self.ns, self.ks))

    def col_slots(self) -> List[int]:
        """slot index (g*nc + j) of every global column c, in column order."""
        pos = [0] * self.n
        for g in range(self.world):
            for j in range(self.nc):
                c = self.col(g, j)
                if c >= 0:
                    pos[c] = g * self.nc + j
        return pos

    # rows of the primary Merkle trees ----------------------------------------------------
    @property
    def nt(self) -> int:
        return _cdiv(self.n, self.world)

    def tree_rows(self, g: int) -> range:
        return range(min(g * self.nt, self.n), min((g + 1) * self.nt, self.n))


def _unit(*vals) -> int:
    """Widest copy width (16, 8, 4, 2 or 1 bytes) dividing every value."""
    g = 0
    for v in vals:
        g = math.gcd(g, int(v))
    for u in (16, 8, 4, 2):
        if g % u == 0:
            return u
    return 1


# ---------------------------------------------------------------------------------------------
# compute backends
# ---------------------------------------------------------------------------------------------
class DeviceOps:
    """The HIP engine (C ABI) on torch device tensors; work goes on torch's current stream."""

    def __init__(self):
        self._codecs = {}
        self._offs = {}

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
        m = len(idx)
        ia = (ctypes.c_uint16 * m)(*idx)
        oa = (ctypes.c_uint64 * m)(*sym_off)
        _ok(_lib.lib().rs2_codec_decode_device_async(
            self._codec(k, n, s), lines, m, ia, base.data_ptr(), oa, line_stride,
            out.data_ptr(), out_ss, out_ls, out_limit, self._stream(base)), decode=True)

    def offsets(self, key, build, device):
        """Device copy of the int64 offset table build() (cached under `key`) and the gcd of
        its entries (the copy-width bound)."""
        import numpy as np
        import torch
        k = (key, str(device))
        t = self._offs.get(k)
        if t is None:
            a = np.ascontiguousarray(build(), dtype=np.int64)
            t = (torch.from_numpy(a).to(device), int(np.gcd.reduce(a)) if a.size else 0)
            self._offs[k] = t
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

    def all_to_all(self, send):
        import torch
        recv = torch.empty_like(send)
        self.dist.all_to_all_single(recv, send, group=self.group)
        return recv

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

    def all_to_all(self, send):
        return super().all_to_all(send.cpu()).to(send.device)

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

    def all_to_all(self, send):
        return send

    def all_gather(self, t):
        return t

    def gather(self, t, dst: int = 0):
        return t

    def scatter(self, parts, like, src: int = 0):
        return parts[0]


# ---------------------------------------------------------------------------------------------
# the partitioned encoder / decoder (one instance per rank)
# ---------------------------------------------------------------------------------------------
class RankEncoder:
    """Rank g's share of encode_with_metadata for one blob (phases; see module docstring)."""

    def __init__(self, part: Partition, rank: int, ops, device):
        self.p, self.g, self.ops, self.device = part, rank, ops, device

    def _t(self, nbytes):
        import torch
        return torch.empty(max(nbytes, 1), dtype=torch.uint8, device=self.device)

    def rows_phase(self, rows):
        """rows: this rank's message rows, len(rows(g)) * K_s * s bytes (zero-padded blob
        slice).  Returns the exchange-1 send buffer [G][nc][nr][s]: for every destination
        rank h and its column slot j, the symbols of column col(h, j) in this rank's rows."""
        import torch
        p, g = self.p, self.g
        G, nc, nr, s, ks, n = p.world, p.nc, p.nr, p.s, p.ks, p.n
        nrg = len(p.rows(g))
        send = self._t(G * nc * nr * s)
        if nrg == 0:
            return send
        rep = self._t(nrg * (n - ks) * s)
        # row code: line = row, source symbol c at row*ks*s + c*s -> repair j at row*(n-ks)*s + j*s
        self.ops.encode_lines(ks, n, s, nrg, rows, 0, s, ks * s, rep, 0, s, (n - ks) * s)
        # pack (segment copies, one launch per source): systematic column c < K_s goes to rank
        # c // ns, slot c % ns; repair column K_s + q to rank q // nrp, slot ns + q % nrp; row r
        # of this rank at symbol r of the slot
        ns, nrp, ops, dev = p.ns, p.nrp, self.ops, self.device
        src = ops.offsets(("rows_sys_src", p), lambda: [c * s for c in range(ks)], dev)
        dst = ops.offsets(("rows_sys_dst", p),
                          lambda: [((c // ns) * nc + c % ns) * nr * s for c in range(ks)], dev)
        ops.copy_segments(rows, send, src, dst, nrg, ks * s, s, s)
        src = ops.offsets(("rows_rep_src", p), lambda: [q * s for q in range(n - ks)], dev)
        dst = ops.offsets(("rows_rep_dst", p),
                          lambda: [((q // nrp) * nc + ns + q % nrp) * nr * s for q in range(n - ks)],
                          dev)
        ops.copy_segments(rep, send, src, dst, nrg, (n - ks) * s, s, s)
        return send

    def columns_phase(self, recv1):
        """recv1 [G][nc][nr][s] (rank h's rows of my columns).  Builds X [nc][n][s] (all n
        symbols of each column slot), hashes it, and returns (X, exchange-2 send buffer
        [G][nc][nt][32] of leaf digests by destination row owner, secondary roots [nc][32])."""
        p = self.p
        G, nc, nr, s, kp, n, nt = p.world, p.nc, p.nr, p.s, p.kp, p.n, p.nt
        X = self._t(nc * n * s)
        ops, dev = self.ops, self.device
        # unpack: message row r (from rank r // nr, its row r % nr) of every slot j
        src = ops.offsets(("cols_x_src", p), lambda: [((r // nr) * nc * nr + r % nr) * s
                                                       for r in range(kp)], dev)
        dst = ops.offsets(("cols_x_dst", p), lambda: [r * s for r in range(kp)], dev)
        ops.copy_segments(recv1, X, src, dst, nc, nr * s, n * s, s)
        # column code: line = column slot, source r at r*s -> repair j at (kp + j)*s
        self.ops.encode_lines(kp, n, s, nc, X, 0, s, n * s, X, kp * s, s, n * s)
        leaves = self._t(nc * n * 32)
        self.ops.leaf_hashes(X, nc * n, s, leaves)
        sec = self._t(nc * 32)
        self.ops.merkle_roots(leaves, nc, n, n * 32, 32, sec, 32)
        send2 = self._t(G * nc * nt * 32)
        # leaf of row t, slot j -> row owner t // nt, slot j, its row t % nt
        src = ops.offsets(("cols_leaf_src", p), lambda: [t * 32 for t in range(n)], dev)
        dst = ops.offsets(("cols_leaf_dst", p), lambda: [((t // nt) * nc * nt + t % nt) * 32
                                                         for t in range(n)], dev)
        ops.copy_segments(leaves, send2, src, dst, nc, n * 32, nt * 32, 32)
        return X, send2, sec[:nc * 32]

    def trees_phase(self, recv2):
        """recv2 [G][nc][nt][32]: leaf digests of my tree rows from every column slot.
        Returns primary roots [nt][32] of rows tree_rows(g)."""
        p = self.p
        nt, n = p.nt, p.n
        rows_t = p.tree_rows(self.g)
        prim = self._t(nt * 32)
        if len(rows_t):
            # row_leaves [rows][n][32]: column c's digest of row r from slot col_slots[c]
            row_leaves = self._t(len(rows_t) * n * 32)
            src = self.ops.offsets(("trees_src", p), lambda: [q * nt * 32 for q in p.col_slots()],
                                   self.device)
            dst = self.ops.offsets(("trees_dst", p), lambda: [c * 32 for c in range(n)],
                                   self.device)
            self.ops.copy_segments(recv2, row_leaves, src, dst, len(rows_t), 32, n * 32, 32)
            self.ops.merkle_roots(row_leaves, len(rows_t), n, n * 32, 32, prim, 32)
        return prim[:nt * 32]

    def finish(self, all_prim, all_sec):
        """all_prim [G*nt][32] (row order), all_sec [G*nc][32] (slot order) -> (hashes [n][64]
        by sliver-pair index, blob_id [32])."""
        p = self.p
        n, ops, dev = p.n, self.ops, self.device
        hashes = self._t(n * 64)
        zero = ops.offsets(("zero",), lambda: [0], dev)
        ops.copy_segments(all_prim, hashes, zero, zero, n, 32, 64, 32)   # pair i <- row root i
        # pair i <- the root of column n-1-i, which sits in slot col_slots[n-1-i]
        slots = p.col_slots()
        src = ops.offsets(("finish_sec_src", p), lambda: [slots[n - 1 - i] * 32 for i in range(n)],
                          dev)
        dst = ops.offsets(("finish_sec_dst", p), lambda: [i * 64 + 32 for i in range(n)], dev)
        ops.copy_segments(all_sec, hashes, src, dst, 1, 0, 0, 32)
        bid = self._t(32)
        self.ops.blob_id(hashes, n, p.blob_len, bid)
        return hashes[:n * 64], bid[:32]


@dataclass
class RankEncoded:
    """What one rank holds after a partitioned encode."""
    columns: object      # X [nc][n][s]: slot j = all n symbols of column col(g, j)
    hashes: object       # [n][64] pair hashes (every rank)
    blob_id: object      # [32] (every rank)


def encode_distributed(part: Partition, rows, ops, exchange, device) -> RankEncoded:
    """Partitioned encode_with_metadata on this rank (exchange = DistExchange)."""
    enc = RankEncoder(part, exchange.rank, ops, device)
    send1 = enc.rows_phase(rows)
    recv1 = exchange.all_to_all(send1)
    X, send2, sec = enc.columns_phase(recv1)
    recv2 = exchange.all_to_all(send2)
    prim = enc.trees_phase(recv2)
    hashes, bid = enc.finish(exchange.all_gather(prim), exchange.all_gather(sec))
    return RankEncoded(X, hashes, bid)


def decode_columns(part: Partition, rank: int, ops, idx: Sequence[int], base, sym_off,
                   line_stride: int, device):
    """Primary-axis decode of rank g's systematic columns sys_cols(g) from K_p primary slivers:
    symbol (column slot j) of sliver idx[i] at base + sym_off[i] + j*line_stride.  Returns
    [K_p][ns][s] (rows of the decoded message columns; padding columns unwritten)."""
    import torch
    p = part
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
    src = ops.offsets(("asm_src", p), lambda: [((c // ns) * kp * ns + c % ns) * s
                                               for c in range(ks)], gathered.device)
    dst = ops.offsets(("asm_dst", p), lambda: [c * s for c in range(ks)], gathered.device)
    ops.copy_segments(gathered, out, src, dst, kp, ns * s, ks * s, s)
    return out[:p.blob_len]


def decode_distributed(part: Partition, enc: RankEncoded, idx: Sequence[int], ops, exchange,
                       device, root: int = 0):
    """Decode from the primary slivers idx (K_p distinct indices) using the column slices this
    rank already holds after encode_distributed (its systematic columns), then RCCL-gather the
    decoded columns to `root`.  Returns the blob on the root, None elsewhere."""
    p = part
    offs = [int(i) * p.s for i in idx]
    cols = decode_columns(p, exchange.rank, ops, idx, enc.columns, offs, p.n * p.s, device)
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
    src = ops.offsets(("scatter_src", p), lambda: [c * s for c in range(ks)], slivers.device)
    dst = ops.offsets(("scatter_dst", p), lambda: [((c // ns) * kp * ns + c % ns) * s
                                                   for c in range(ks)], slivers.device)
    ops.copy_segments(slivers, send, src, dst, kp, ks * s, ns * s, s)
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
    cols = p.sys_cols(exchange.rank)
    out = torch.empty(max(p.kp * p.ns * p.s, 1), dtype=torch.uint8, device=device)
    # symbol j of received sliver i at i*ns*s + j*s; decoded row r, column slot j at r*ns*s + j*s
    ops.decode_lines(p.kp, p.n, p.s, len(cols), list(idx), mine.reshape(-1),
                     [i * p.ns * p.s for i in range(len(idx))], p.s, out, p.ns * p.s, p.s,
                     p.kp * p.ns * p.s)
    gathered = exchange.gather(out[:p.kp * p.ns * p.s], dst=root)
    return assemble_blob(p, gathered, ops) if gathered is not None else None


# ---------------------------------------------------------------------------------------------
# single-process simulation of G ranks (multi-rank parity on one device)
# ---------------------------------------------------------------------------------------------
def _a2a(sends: List) -> List:
    import torch
    G = len(sends)
    chunks = [s.view(G, -1) for s in sends]
    return [torch.cat([chunks[h][g] for h in range(G)]) for g in range(G)]


def simulate_encode(part: Partition, blob_rows: List, ops, device) -> List[RankEncoded]:
    """All ranks' phases in one process; blob_rows[g] = rank g's rows (see rows_phase)."""
    import torch
    G = part.world
    encs = [RankEncoder(part, g, ops, device) for g in range(G)]
    recv1 = _a2a([e.rows_phase(r) for e, r in zip(encs, blob_rows)])
    outs = [e.columns_phase(r) for e, r in zip(encs, recv1)]
    recv2 = _a2a([o[1] for o in outs])
    prims = [e.trees_phase(r) for e, r in zip(encs, recv2)]
    all_p, all_s = torch.cat(prims), torch.cat([o[2] for o in outs])
    res = []
    for e, o in zip(encs, outs):
        h, b = e.finish(all_p, all_s)
        res.append(RankEncoded(o[0], h, b))
    return res


def simulate_decode(part: Partition, encs: List[RankEncoded], idx: Sequence[int], ops, device):
    import torch
    offs = [int(i) * part.s for i in idx]
    cols = [decode_columns(part, g, ops, idx, encs[g].columns, offs, part.n * part.s, device)
            for g in range(part.world)]
    return assemble_blob(part, torch.cat(cols), ops)


def simulate_decode_from_slivers(part: Partition, slivers, idx: Sequence[int], ops, device):
    """decode_from_slivers with all G ranks in this process (scatter / gather simulated)."""
    import torch
    p = part
    send = scatter_sliver_columns(p, slivers, p.world, ops)
    cols = []
    for g in range(p.world):
        out = torch.empty(max(p.kp * p.ns * p.s, 1), dtype=torch.uint8, device=device)
        ops.decode_lines(p.kp, p.n, p.s, len(p.sys_cols(g)), list(idx), send[g].reshape(-1),
                         [i * p.ns * p.s for i in range(len(idx))], p.s, out, p.ns * p.s, p.s,
                         p.kp * p.ns * p.s)
        cols.append(out[:p.kp * p.ns * p.s])
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


def gather_slivers(part: Partition, encs: List[RankEncoded], blob):
    """Reassemble full primary / secondary slivers from the ranks' column slots (tests and the
    host-side D2H of a real deployment): primary [n][K_s*s], secondary [n][K_p*s]."""
    import torch
    p = part
    n, kp, ks, s = p.n, p.kp, p.ks, p.s
    full = torch.empty((n, n, s), dtype=torch.uint8, device=encs[0].columns.device)
    for g, e in enumerate(encs):
        xv = e.columns[:p.nc * n * s].view(p.nc, n, s)
        for j in range(p.nc):
            c = p.col(g, j)
            if c >= 0:
                full[:, c] = xv[j]
    primary = full[:, :ks].reshape(n, ks * s)
    secondary = full[:kp].transpose(0, 1).reshape(n, kp * s)
    return primary, secondary

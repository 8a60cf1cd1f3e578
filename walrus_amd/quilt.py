"""Quilt V1: many small blobs packed column-aligned into one Red Stuff blob.

Mirrors crates/walrus-core/src/encoding/quilt_encoding.rs (QuiltVersionV1) and the quilt types
of crates/walrus-core/src/metadata.rs:63-310.  The only new work beside the 2D encode is the
column-aligned layout: every blob (header + identifier + optional tags + data) occupies whole,
consecutive columns of the K_p x K_s symbol matrix, the quilt index occupies the first columns.
The layout is a strided byte scatter: on the host with numpy (construct_quilt), or on the GPU
from a column table over the serialized payload stream (layout() + quilt_layout_device_async ->
rs2_quilt_layout_device_async, HBM-bound).  The quilt is then encoded by the device engine
exactly as any blob, and a patch is read back from the secondary slivers that hold its columns
(QuiltDecoderV1).

Wire formats (BCS, as the reference's serde derives produce them):
  QuiltIndexV1   = ULEB128(#patches) ++ patch*      (metadata.rs:241-244)
  QuiltPatchV1   = u16le end_index ++ String identifier ++ Map<String,String> tags
                   (start_index is #[serde(skip)], metadata.rs:66-78)
  String         = ULEB128(len) ++ utf-8;  Map = ULEB128(#entries) ++ (key, value)*, entries
                   in the canonical order of their serialized keys (bcs sorts map entries)
  blob header    = u8 version(0x01) ++ u32le length ++ u8 mask   (quilt_encoding.rs:906-990)
  meta blob      = u8 version ++ u32le index_size ++ BCS(QuiltIndexV1)
  patch id       = u8 version ++ u16le start ++ u16le end          (metadata.rs:166-222)
"""

from __future__ import annotations

import unicodedata
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from .encoding import BlobId, BlobMetadata, ReedSolomonEncodingConfig, SliverData, SliverPair

QUILT_VERSION_BYTE = 0x01  # quilt_encoding.rs:651
BLOB_HEADER_SIZE = 6  # quilt_encoding.rs:652
QUILT_INDEX_SIZE_BYTES_LENGTH = 4  # quilt_encoding.rs:50-51
QUILT_VERSION_BYTES_LENGTH = 1
BLOB_IDENTIFIER_SIZE_BYTES_LENGTH = 2
TAGS_SIZE_BYTES_LENGTH = 2
MAX_BLOB_IDENTIFIER_BYTES_LENGTH = (1 << 16) - 1
QUILT_INDEX_PREFIX_SIZE = QUILT_INDEX_SIZE_BYTES_LENGTH + QUILT_VERSION_BYTES_LENGTH
MAX_NUM_SLIVERS_FOR_QUILT_INDEX = 10  # quilt_encoding.rs:69-70
MAX_SERIALIZED_BLOB_SIZE = 0xFFFFFFFF  # BlobHeaderV1::MAX_SERIALIZED_BLOB_SIZE
TAGS_ENABLED = 1
RS2_REQUIRED_ALIGNMENT = 2  # lib.rs:843-856
RS2_MAX_SYMBOL_SIZE = 65534


class QuiltError(Exception):
    """encoding/errors.rs:174-240; `kind` is the reference variant name, `args` its fields."""

    def __init__(self, kind: str, *args):
        super().__init__(kind, *args)
        self.kind = kind

    def __eq__(self, other):
        return isinstance(other, QuiltError) and self.args == other.args

    def __hash__(self):
        return hash(self.args)


# ---- BCS helpers -----------------------------------------------------------------------------
def _uleb(n: int) -> bytes:
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        out.append(b | (0x80 if n else 0))
        if not n:
            return bytes(out)


def _bcs_str(s: str) -> bytes:
    raw = s.encode("utf-8")
    return _uleb(len(raw)) + raw


def _bcs_map(m: Dict[str, str]) -> bytes:
    entries = sorted((_bcs_str(k), _bcs_str(v)) for k, v in m.items())
    return _uleb(len(entries)) + b"".join(k + v for k, v in entries)


class _Reader:
    """Strict BCS reader (canonical ULEB128, valid utf-8, canonical map order, no trailing)."""

    def __init__(self, raw: bytes):
        self.raw, self.pos = bytes(raw), 0

    def take(self, n: int) -> bytes:
        if self.pos + n > len(self.raw):
            raise QuiltError("QuiltIndexSerDerError", "unexpected end of input")
        out = self.raw[self.pos:self.pos + n]
        self.pos += n
        return out

    def uleb(self) -> int:
        n, shift = 0, 0
        while True:
            b = self.take(1)[0]
            n |= (b & 0x7F) << shift
            shift += 7
            if not b & 0x80:
                if b == 0 and shift > 7:
                    raise QuiltError("QuiltIndexSerDerError", "non-canonical ULEB128")
                break
            if shift > 28:
                raise QuiltError("QuiltIndexSerDerError", "ULEB128 overflow")
        if n > 0xFFFFFFFF:
            raise QuiltError("QuiltIndexSerDerError", "length overflow")
        return n

    def u16(self) -> int:
        return int.from_bytes(self.take(2), "little")

    def string(self) -> str:
        raw = self.take(self.uleb())
        try:
            return raw.decode("utf-8")
        except UnicodeDecodeError as e:
            raise QuiltError("QuiltIndexSerDerError", "invalid utf-8") from e

    def str_map(self) -> Dict[str, str]:
        out: Dict[str, str] = {}
        prev = None
        for _ in range(self.uleb()):
            k = self.string()
            kb = _bcs_str(k)
            if prev is not None and kb <= prev:
                raise QuiltError("QuiltIndexSerDerError", "non-canonical map")
            prev = kb
            out[k] = self.string()
        return out

    def end(self):
        if self.pos != len(self.raw):
            raise QuiltError("QuiltIndexSerDerError", "remaining input")


# ---- identifiers, headers, patches -----------------------------------------------------------
def validate_quilt_identifier(identifier: str) -> None:
    """quilt_encoding.rs:132-158."""
    if len(identifier.encode("utf-8")) > MAX_BLOB_IDENTIFIER_BYTES_LENGTH:
        raise QuiltError("InvalidIdentifier", f"identifier too long: {len(identifier)}")
    if not identifier:
        raise QuiltError("InvalidIdentifier", "identifier is empty")
    if identifier.rstrip() != identifier:
        raise QuiltError("InvalidIdentifier", f"identifier contains trailing whitespace: {identifier}")
    if any(unicodedata.category(c) == "Cc" for c in identifier):
        raise QuiltError("InvalidIdentifier", f"identifier contains control characters: {identifier}")


@dataclass
class BlobHeaderV1:
    """quilt_encoding.rs:906-990: version byte, u32le length (extensions + data), mask."""
    length: int = 0
    mask: int = 0

    def as_bytes(self) -> bytes:
        return bytes([QUILT_VERSION_BYTE]) + int(self.length).to_bytes(4, "little") + \
            bytes([self.mask])

    @classmethod
    def from_bytes(cls, raw: bytes) -> "BlobHeaderV1":
        raw = bytes(raw)
        if len(raw) != BLOB_HEADER_SIZE:
            raise QuiltError("InvalidQuiltData", "blob header has wrong length")
        if raw[0] != QUILT_VERSION_BYTE:
            raise QuiltError("InvalidQuiltData",
                             f"invalid blob header version byte: {raw[0]}, expected: 1")
        return cls(int.from_bytes(raw[1:5], "little"), raw[5])

    def has_tags(self) -> bool:
        return bool(self.mask & TAGS_ENABLED)

    def set_has_tags(self, on: bool) -> None:
        self.mask = (self.mask | TAGS_ENABLED) if on else (self.mask & ~TAGS_ENABLED & 0xFF)


@dataclass
class QuiltStoreBlob:
    """quilt_encoding.rs:563-640: a blob with its identifier and tags."""
    blob: bytes
    identifier: str
    tags: Dict[str, str] = field(default_factory=dict)

    def __post_init__(self):
        self.blob = bytes(self.blob)
        validate_quilt_identifier(self.identifier)
        self.tags = dict(self.tags)

    def data(self) -> bytes:
        return self.blob


@dataclass
class QuiltPatchInternalIdV1:
    """metadata.rs:157-232."""
    start_index: int
    end_index: int

    def to_bytes(self) -> bytes:
        return bytes([QUILT_VERSION_BYTE]) + self.start_index.to_bytes(2, "little") + \
            self.end_index.to_bytes(2, "little")

    @classmethod
    def from_bytes(cls, raw: bytes) -> "QuiltPatchInternalIdV1":
        raw = bytes(raw)
        if len(raw) != 5:
            raise QuiltError("Other", "QuiltPatchInternalIdV1 requires 5 bytes")
        if raw[0] != QUILT_VERSION_BYTE:
            raise QuiltError("QuiltVersionMismatch", raw[0], QUILT_VERSION_BYTE)
        return cls(int.from_bytes(raw[1:3], "little"), int.from_bytes(raw[3:5], "little"))

    def sliver_indices(self) -> List[int]:
        return list(range(self.start_index, self.end_index))


@dataclass
class QuiltPatchV1:
    """metadata.rs:63-134 (start_index is not on the wire)."""
    identifier: str
    tags: Dict[str, str] = field(default_factory=dict)
    start_index: int = 0
    end_index: int = 0

    def quilt_patch_internal_id(self) -> QuiltPatchInternalIdV1:
        return QuiltPatchInternalIdV1(self.start_index, self.end_index)

    def has_matched_tag(self, tag: str, value: str) -> bool:
        return self.tags.get(tag) == value

    def sliver_indices(self) -> List[int]:
        return list(range(self.start_index, self.end_index))

    def to_bcs(self) -> bytes:
        return self.end_index.to_bytes(2, "little") + _bcs_str(self.identifier) + \
            _bcs_map(self.tags)


@dataclass
class QuiltIndexV1:
    """metadata.rs:234-282; quilt_encoding.rs:228-300 (QuiltIndexApi lookups)."""
    quilt_patches: List[QuiltPatchV1] = field(default_factory=list)

    def to_bcs(self) -> bytes:
        return _uleb(len(self.quilt_patches)) + b"".join(p.to_bcs() for p in self.quilt_patches)

    @classmethod
    def from_bcs(cls, raw: bytes) -> "QuiltIndexV1":
        r = _Reader(raw)
        patches = []
        for _ in range(r.uleb()):
            end = r.u16()
            ident = r.string()
            patches.append(QuiltPatchV1(ident, r.str_map(), 0, end))
        r.end()
        return cls(patches)

    def populate_start_indices(self, first_start: int) -> None:
        prev = first_start
        for p in self.quilt_patches:
            p.start_index = prev
            prev = p.end_index

    def identifiers(self) -> List[str]:
        return [p.identifier for p in self.quilt_patches]

    def __len__(self):
        return len(self.quilt_patches)

    def get_quilt_patches_by_identifiers(self, identifiers: Sequence[str]) -> List[QuiltPatchV1]:
        want = set(identifiers)
        out = []
        for p in self.quilt_patches:
            if p.identifier in want:
                want.discard(p.identifier)
                out.append(p)
        if want:
            raise QuiltError("BlobsNotFoundInQuilt", sorted(want))
        return out

    def get_quilt_patches_by_tag(self, tag: str, value: str) -> List[QuiltPatchV1]:
        return [p for p in self.quilt_patches if p.has_matched_tag(tag, value)]

    def get_sliver_indices_for_tag(self, tag: str, value: str) -> List[int]:
        return [i for p in self.get_quilt_patches_by_tag(tag, value) for i in p.sliver_indices()]

    def get_sliver_indices_for_identifiers(self, identifiers: Sequence[str]) -> List[int]:
        return [i for p in self.get_quilt_patches_by_identifiers(identifiers)
                for i in p.sliver_indices()]


@dataclass
class QuiltMetadataV1:
    """metadata.rs:298-330: the quilt's BlobId, its blob metadata and the index."""
    quilt_id: BlobId
    metadata: BlobMetadata
    index: QuiltIndexV1


# ---- sizes -----------------------------------------------------------------------------------
def _header_and_extension_bytes(blob: QuiltStoreBlob) -> bytes:
    """QuiltEncoderV1::get_header_and_extension_bytes (quilt_encoding.rs:1364-1418)."""
    ident = _bcs_str(blob.identifier)
    ext = len(ident).to_bytes(2, "little") + ident
    header = BlobHeaderV1()
    if blob.tags:
        header.set_has_tags(True)
        tags = _bcs_map(blob.tags)
        if len(tags) > 0xFFFF:
            raise QuiltError("Other", "Failed to convert tags size to u16")
        ext += len(tags).to_bytes(2, "little") + tags
    total = len(ext) + len(blob.blob)
    if total > MAX_SERIALIZED_BLOB_SIZE:
        raise QuiltError("QuiltOversize", f"blob size ({total} bytes) exceeds the maximum size")
    header.length = total
    return header.as_bytes() + ext


def serialized_blob_size(blob: QuiltStoreBlob) -> int:
    """QuiltVersionV1::serialized_blob_size (quilt_encoding.rs:724-756)."""
    ident = len(_bcs_str(blob.identifier))
    if ident >= MAX_BLOB_IDENTIFIER_BYTES_LENGTH:
        raise QuiltError("InvalidIdentifier", "identifier size exceeds maximum allowed value")
    prefix = ident + BLOB_IDENTIFIER_SIZE_BYTES_LENGTH
    if blob.tags:
        prefix += len(_bcs_map(blob.tags)) + TAGS_SIZE_BYTES_LENGTH
    content = prefix + len(blob.blob)
    if content > MAX_SERIALIZED_BLOB_SIZE:
        raise QuiltError("QuiltOversize", f"blob size ({content} bytes) exceeds the maximum size")
    return content + BLOB_HEADER_SIZE


def _fits(sizes: Sequence[int], n_columns: int, column_size: int) -> bool:
    """utils::can_blobs_fit_into_matrix (quilt_encoding.rs:2043-2053)."""
    return n_columns >= sum(-(-b // column_size) for b in sizes)


def compute_symbol_size(blobs_sizes: Sequence[int], n_columns: int, n_rows: int,
                        max_num_columns_for_quilt_index: int,
                        required_alignment: int = RS2_REQUIRED_ALIGNMENT,
                        max_symbol_size: int = RS2_MAX_SYMBOL_SIZE) -> int:
    """utils::compute_symbol_size (quilt_encoding.rs:1971-2041): the smallest even symbol size
    at which every blob (the index first) fits in whole, consecutive columns."""
    if len(blobs_sizes) > n_columns:
        raise QuiltError("TooManyBlobs", len(blobs_sizes) - 1, n_columns - 1)
    if not blobs_sizes:
        raise QuiltError("EmptyInput", "blobs")
    lo = max(-(-sum(blobs_sizes) // (n_columns * n_rows)),
             -(-blobs_sizes[0] // (n_rows * max_num_columns_for_quilt_index)))
    lo = max(lo, -(-QUILT_INDEX_PREFIX_SIZE // n_rows))
    hi = -(-max(blobs_sizes) // (n_columns // len(blobs_sizes) * n_rows))
    while lo < hi:
        mid = (lo + hi) // 2
        if _fits(blobs_sizes, n_columns, mid * n_rows):
            hi = mid
        else:
            lo = mid + 1
    symbol_size = -(-lo // required_alignment) * required_alignment
    if symbol_size > max_symbol_size:
        raise QuiltError("QuiltOversize", f"the resulting symbol size {symbol_size} is larger "
                         f"than the maximum symbol size {max_symbol_size}; remove some blobs")
    return symbol_size


# ---- column readers (quilt_encoding.rs:640-888, QuiltColumnRangeReader) -----------------------
class _ColumnSource:
    def range_read_from_columns(self, start_col: int, skip: int, count: int) -> bytes:
        raise NotImplementedError

    def total_data_size(self) -> int:
        raise NotImplementedError


def decode_quilt_index(src: _ColumnSource, column_size: int) -> QuiltIndexV1:
    """QuiltVersionV1::decode_quilt_index (quilt_encoding.rs:665-722)."""
    ver = src.range_read_from_columns(0, 0, QUILT_VERSION_BYTES_LENGTH)
    if ver[0] != QUILT_VERSION_BYTE:
        raise QuiltError("QuiltVersionMismatch", ver[0], QUILT_VERSION_BYTE)
    size = int.from_bytes(src.range_read_from_columns(0, QUILT_VERSION_BYTES_LENGTH,
                                                      QUILT_INDEX_SIZE_BYTES_LENGTH), "little")
    max_size = max(column_size * MAX_NUM_SLIVERS_FOR_QUILT_INDEX - QUILT_INDEX_PREFIX_SIZE, 0)
    if size > max_size:
        raise QuiltError("InvalidQuiltData",
                         f"quilt index size ({size}) exceeds maximum ({max_size})")
    index = QuiltIndexV1.from_bcs(src.range_read_from_columns(0, QUILT_INDEX_PREFIX_SIZE, size))
    cols = -(-(size + QUILT_INDEX_PREFIX_SIZE) // column_size)
    if cols > 0xFFFF:
        raise QuiltError("InvalidQuiltData", f"quilt index spans too many columns: {cols}")
    index.populate_start_indices(cols)
    return index


def decode_blob(src: _ColumnSource, start_col: int) -> QuiltStoreBlob:
    """QuiltVersionV1::decode_blob (quilt_encoding.rs:758-888)."""
    header = BlobHeaderV1.from_bytes(src.range_read_from_columns(start_col, 0, BLOB_HEADER_SIZE))
    off = BLOB_HEADER_SIZE
    remaining = header.length
    total = src.total_data_size()
    if remaining > total:
        raise QuiltError("InvalidQuiltData",
                         f"blob claims {remaining} bytes but data source only has {total}")
    id_size = int.from_bytes(src.range_read_from_columns(
        start_col, off, BLOB_IDENTIFIER_SIZE_BYTES_LENGTH), "little")
    r = _Reader(src.range_read_from_columns(start_col, off + BLOB_IDENTIFIER_SIZE_BYTES_LENGTH,
                                            id_size))
    try:
        identifier = r.string()
        r.end()
    except QuiltError as e:
        raise QuiltError("InvalidIdentifier", "Failed to deserialize identifier") from e
    used = BLOB_IDENTIFIER_SIZE_BYTES_LENGTH + id_size
    off += used
    if remaining < used:
        raise QuiltError("InvalidQuiltData", "blob header length is smaller than identifier overhead")
    remaining -= used
    tags: Dict[str, str] = {}
    if header.has_tags():
        tsize = int.from_bytes(src.range_read_from_columns(start_col, off, TAGS_SIZE_BYTES_LENGTH),
                               "little")
        r = _Reader(src.range_read_from_columns(start_col, off + TAGS_SIZE_BYTES_LENGTH, tsize))
        try:
            tags = r.str_map()
            r.end()
        except QuiltError as e:
            raise QuiltError("FailedToDecodeExtension", "tags", str(e)) from e
        used = TAGS_SIZE_BYTES_LENGTH + tsize
        off += used
        if remaining < used:
            raise QuiltError("InvalidQuiltData",
                             "blob header length is smaller than identifier + tags overhead")
        remaining -= used
    data = src.range_read_from_columns(start_col, off, remaining)
    return QuiltStoreBlob(data, identifier, tags)


class QuiltV1(_ColumnSource):
    """quilt_encoding.rs:992-1200: the unencoded quilt (K_p rows x K_s columns of symbols)."""

    def __init__(self, data: bytes, row_size: int, symbol_size: int,
                 quilt_index: Optional[QuiltIndexV1] = None):
        self.data, self.row_size, self.symbol_size = bytes(data), row_size, symbol_size
        self.quilt_index = quilt_index

    @classmethod
    def new_from_quilt_blob(cls, quilt_blob: bytes, config: ReedSolomonEncodingConfig) -> "QuiltV1":
        if not quilt_blob:
            raise QuiltError("EmptyInput", "quilt_blob")
        kp, ks = config.n_primary_source_symbols, config.n_secondary_source_symbols
        if len(quilt_blob) % (kp * ks):
            raise QuiltError("InvalidFormatNotAligned",
                             f"quilt_blob length {len(quilt_blob)} is not a multiple of "
                             f"n_source_symbols {kp * ks}")
        s = len(quilt_blob) // (kp * ks)
        q = cls(quilt_blob, s * ks, s)
        q.get_or_decode_quilt_index()
        return q

    def total_data_size(self) -> int:
        return len(self.data)

    def range_read_from_columns(self, start_col: int, skip: int, count: int) -> bytes:
        if self.symbol_size == 0 or self.row_size == 0 or not self.data:
            raise QuiltError("Other", "empty quilt data")
        s, n_rows = self.symbol_size, len(self.data) // self.row_size
        sym_skip = skip // s
        col, row = start_col + sym_skip // n_rows, sym_skip % n_rows
        skip -= sym_skip * s
        out = bytearray()
        while count > 0:
            base = row * self.row_size + col * s
            start = base + skip
            end = min(base + s, start + count, len(self.data))
            if start >= len(self.data):
                raise QuiltError("IndexOutOfBounds", start, len(self.data))
            out += self.data[start:end]
            count -= end - start
            row = (row + 1) % n_rows
            col += row == 0
            skip = 0
        return bytes(out)

    def get_or_decode_quilt_index(self) -> QuiltIndexV1:
        if self.quilt_index is None:
            self.quilt_index = decode_quilt_index(self, self.symbol_size *
                                                  (len(self.data) // self.row_size))
        return self.quilt_index

    def get_blobs_by_identifiers(self, identifiers: Sequence[str]) -> List[QuiltStoreBlob]:
        return [decode_blob(self, p.start_index)
                for p in self.get_or_decode_quilt_index().get_quilt_patches_by_identifiers(identifiers)]

    def get_blob_by_patch_internal_id(self, patch_id: bytes) -> QuiltStoreBlob:
        return decode_blob(self, QuiltPatchInternalIdV1.from_bytes(patch_id).start_index)

    def get_blobs_by_tag(self, tag: str, value: str) -> List[QuiltStoreBlob]:
        return [decode_blob(self, p.start_index)
                for p in self.get_or_decode_quilt_index().get_quilt_patches_by_tag(tag, value)]

    def get_all_blobs(self) -> List[QuiltStoreBlob]:
        return [decode_blob(self, p.start_index) for p in self.get_or_decode_quilt_index().quilt_patches]


def _write_columns(mat: np.ndarray, payload: bytes, start_col: int) -> int:
    """add_blob_to_quilt + write_bytes_to_columns (quilt_encoding.rs:1447-1528) as one strided
    scatter: the payload fills column start_col top to bottom (symbol by symbol), then the next
    column.  mat is the (K_p, K_s, s) view of the quilt; returns the columns used."""
    n_rows, _, s = mat.shape
    col_bytes = n_rows * s
    k = -(-len(payload) // col_bytes)
    buf = np.zeros(k * col_bytes, dtype=np.uint8)
    buf[:len(payload)] = np.frombuffer(payload, dtype=np.uint8)
    mat[:, start_col:start_col + k, :] = buf.reshape(k, n_rows, s).transpose(1, 0, 2)
    return k


@dataclass
class QuiltLayout:
    """Where every column of a quilt comes from: the serialized runs (the meta blob, then each
    blob's header + identifier + tags + data, in identifier order) packed in one payload stream,
    each run at a 16-byte aligned offset; column c holds col_len[c] bytes of the stream from
    col_off[c] (0 bytes: an unused, all-zero column).  Input of the device column fill."""
    n_rows: int
    n_cols: int
    symbol_size: int
    payload: bytes
    col_off: np.ndarray  # int64[n_cols]
    col_len: np.ndarray  # uint32[n_cols]
    index: QuiltIndexV1

    @property
    def quilt_len(self) -> int:
        return self.n_rows * self.n_cols * self.symbol_size


def quilt_layout_device_async(layout: QuiltLayout, d_payload: int, d_col_off: int,
                              d_col_len: int, d_quilt: int, stream: int = 0) -> None:
    """rs2_quilt_layout_device_async: the column fill on the GPU (payload and column tables
    already in device memory, e.g. copied from layout.payload / col_off / col_len)."""
    from . import _lib
    from .encoding import _ok
    _ok(_lib.lib().rs2_quilt_layout_device_async(layout.n_rows, layout.n_cols, layout.symbol_size,
                                                 d_payload, d_col_off, d_col_len, d_quilt,
                                                 stream or None))


class QuiltEncoderV1:
    """quilt_encoding.rs:1344-1684."""

    def __init__(self, config: ReedSolomonEncodingConfig, blobs: Sequence[QuiltStoreBlob]):
        self.config, self.blobs = config, list(blobs)

    def layout(self) -> QuiltLayout:
        """The same placement as construct_quilt, as a column table over a payload stream."""
        n_rows = self.config.n_primary_source_symbols
        n_cols = self.config.n_secondary_source_symbols
        blobs = sorted(self.blobs, key=lambda b: b.identifier.encode("utf-8"))
        for a, b in zip(blobs, blobs[1:]):
            if a.identifier == b.identifier:
                raise QuiltError("DuplicateIdentifier", a.identifier)
        index = QuiltIndexV1([QuiltPatchV1(b.identifier, dict(b.tags)) for b in blobs])
        index_size = len(index.to_bcs())
        index_total = QUILT_INDEX_PREFIX_SIZE + index_size
        sizes = [index_total] + [serialized_blob_size(b) for b in blobs]
        s = compute_symbol_size(sizes, n_cols, n_rows, MAX_NUM_SLIVERS_FOR_QUILT_INDEX)
        col_bytes = s * n_rows
        col = -(-index_total // col_bytes)
        runs = []
        for patch, b in zip(index.quilt_patches, blobs):
            run = _header_and_extension_bytes(b) + b.blob
            used = -(-len(run) // col_bytes)
            patch.start_index, patch.end_index = col, col + used
            runs.append((col, run))
            col += used
        meta = bytes([QUILT_VERSION_BYTE]) + index_size.to_bytes(4, "little") + index.to_bcs()
        runs.insert(0, (0, meta))
        col_off = np.zeros(n_cols, dtype=np.int64)
        col_len = np.zeros(n_cols, dtype=np.uint32)
        stream = bytearray()
        for c0, run in runs:
            pos = -(-len(stream) // 16) * 16
            stream += bytes(pos - len(stream)) + run
            for j in range(-(-len(run) // col_bytes)):
                col_off[c0 + j] = pos + j * col_bytes
                col_len[c0 + j] = min(col_bytes, len(run) - j * col_bytes)
        return QuiltLayout(n_rows, n_cols, s, bytes(stream), col_off, col_len, index)

    def construct_quilt(self) -> QuiltV1:
        n_rows = self.config.n_primary_source_symbols
        n_cols = self.config.n_secondary_source_symbols
        blobs = sorted(self.blobs, key=lambda b: b.identifier.encode("utf-8"))
        for a, b in zip(blobs, blobs[1:]):
            if a.identifier == b.identifier:
                raise QuiltError("DuplicateIdentifier", a.identifier)
        index = QuiltIndexV1([QuiltPatchV1(b.identifier, dict(b.tags)) for b in blobs])
        index_size = len(index.to_bcs())  # end indices are fixed-width u16: size is final now
        index_total = QUILT_INDEX_PREFIX_SIZE + index_size
        sizes = [index_total] + [serialized_blob_size(b) for b in blobs]
        s = compute_symbol_size(sizes, n_cols, n_rows, MAX_NUM_SLIVERS_FOR_QUILT_INDEX)
        mat = np.zeros((n_rows, n_cols, s), dtype=np.uint8)
        column_size = s * n_rows
        col = -(-index_total // column_size)
        assert col <= MAX_NUM_SLIVERS_FOR_QUILT_INDEX
        first = col
        for patch, b in zip(index.quilt_patches, blobs):
            used = _write_columns(mat, _header_and_extension_bytes(b) + b.blob, col)
            patch.start_index, patch.end_index = col, col + used
            col += used
        meta = bytes([QUILT_VERSION_BYTE]) + index_size.to_bytes(4, "little") + index.to_bcs()
        assert len(meta) == index_total
        assert _write_columns(mat, meta, 0) == first
        return QuiltV1(mat.tobytes(), s * n_cols, s, index)

    def encode_with_metadata(self) -> Tuple[List[SliverPair], QuiltMetadataV1]:
        """Layout on the host, then the 2D encode + metadata on the device engine."""
        quilt = self.construct_quilt()
        pairs, meta = self.config.encode_with_metadata(quilt.data)
        assert self.config.symbol_size_for_blob(len(quilt.data)) == quilt.symbol_size
        index = QuiltIndexV1([QuiltPatchV1(p.identifier, dict(p.tags), p.start_index, p.end_index)
                              for p in quilt.quilt_index.quilt_patches])
        return pairs, QuiltMetadataV1(meta.blob_id, meta.metadata, index)


class QuiltDecoderV1(_ColumnSource):
    """quilt_encoding.rs:1688-1960: reads patches from the secondary slivers (= columns)."""

    def __init__(self, slivers: Iterable[SliverData] = (),
                 quilt_index: Optional[QuiltIndexV1] = None):
        self.slivers: Dict[int, SliverData] = {}
        self.quilt_index = quilt_index
        self.column_size: Optional[int] = None
        self.add_slivers(slivers)

    def add_slivers(self, slivers: Iterable[SliverData]) -> None:
        for sl in slivers:
            size = len(sl.symbols.data)
            if self.column_size is None:
                self.column_size = size
            elif size != self.column_size:
                raise QuiltError("ColumnSizeMismatch", self.column_size, size)
            self.slivers[sl.index] = sl

    def _check_missing(self, start: int, end: int) -> None:
        missing = [i for i in range(start, end) if i not in self.slivers]
        if missing:
            raise QuiltError("MissingSlivers", missing)

    def total_data_size(self) -> int:
        return len(self.slivers) * (self.column_size or 0)

    def range_read_from_columns(self, start_col: int, skip: int, count: int) -> bytes:
        want = count
        self._check_missing(start_col, start_col + 1)
        cs = self.column_size
        end_col = start_col + -(-(skip + count) // cs)
        self._check_missing(start_col, end_col)
        out = bytearray()
        for c in range(start_col, end_col):
            if count == 0:
                break
            data = self.slivers[c].symbols.data
            if skip >= len(data):
                skip -= len(data)
                continue
            take = min(len(data) - skip, count)
            out += data[skip:skip + take]
            count -= take
            skip = 0
        if len(out) != want:
            raise QuiltError("InsufficientQuiltData", want, len(out))
        return bytes(out)

    def get_or_decode_quilt_index(self) -> QuiltIndexV1:
        if self.quilt_index is None:
            self._check_missing(0, 1)
            self.quilt_index = decode_quilt_index(self, self.column_size)
        return self.quilt_index

    def _patch(self, p: QuiltPatchV1) -> QuiltStoreBlob:
        self._check_missing(p.start_index, p.end_index)
        return decode_blob(self, p.start_index)

    def get_blobs_by_identifiers(self, identifiers: Sequence[str]) -> List[QuiltStoreBlob]:
        if self.quilt_index is None:
            raise QuiltError("MissingQuiltIndex")
        return [self._patch(p) for p in self.quilt_index.get_quilt_patches_by_identifiers(identifiers)]

    def get_blob_by_patch_internal_id(self, patch_id: bytes) -> QuiltStoreBlob:
        pid = QuiltPatchInternalIdV1.from_bytes(patch_id)
        self._check_missing(pid.start_index, pid.end_index)
        return decode_blob(self, pid.start_index)

    def get_blobs_by_tag(self, tag: str, value: str) -> List[QuiltStoreBlob]:
        if self.quilt_index is None:
            raise QuiltError("MissingQuiltIndex")
        return [self._patch(p) for p in self.quilt_index.get_quilt_patches_by_tag(tag, value)]


def get_quilt_version_byte(data: bytes) -> int:
    """quilt_encoding.rs:73-90 / utils::get_quilt_version_byte."""
    if not data:
        raise QuiltError("EmptyInput", "data")
    if data[0] != QUILT_VERSION_BYTE:
        raise QuiltError("QuiltVersionMismatch", data[0], QUILT_VERSION_BYTE)
    return data[0]

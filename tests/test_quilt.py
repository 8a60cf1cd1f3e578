"""Quilt V1 layout, index and patch reads (walrus_amd/quilt.py) on the CPU, and the quilt's
2D encode through the device engine on the GPU.

Mirrors crates/walrus-core/src/encoding/quilt_encoding.rs tests:
  :2100-2150 test_quilt_find_min_length      -> test_symbol_size_golden (the reference's cases)
  :2590-2634 test_quilt_blob_header          -> test_blob_header_round_trip
  :2274-2335 test_quilt_construct_quilt      -> test_construct_quilt_reads_back
  :2360-2590 test_quilt_encoder_and_decoder  -> test_quilt_encode_decode_device (GPU)
  :120-131   validate_quilt_identifier doc   -> test_identifier_validation
  :2944-3100 malformed quilt data            -> test_malformed_*
"""
import numpy as np
import pytest

from walrus_amd import ReedSolomonEncodingConfig, SliverData, Symbols, SECONDARY
from walrus_amd import quilt as Q

TOO_MANY = Q.QuiltError("TooManyBlobs", 3, 2)
EMPTY = Q.QuiltError("EmptyInput", "blobs")
CASE_11 = [416, 253, 258, 384, 492, 303, 276, 464, 143, 251, 388, 263, 515, 433, 505, 385, 346,
           69, 48, 495, 329, 450, 494, 104, 539, 245, 109, 317, 60]


@pytest.mark.parametrize("blobs,n_cols,n_rows,max_idx,expected", [
    ([2, 1, 2, 1], 3, 3, 1, TOO_MANY),
    ([1000, 1, 1], 4, 7, 2, 72),
    ([], 3, 1, 1, EMPTY),
    ([1], 3, 2, 1, 4),
    ([115, 80, 4], 17, 9, 3, 6),
    ([20, 20, 20], 3, 5, 2, 4),
    ([5, 5, 5], 5, 1, 1, 6),
    ([25, 35, 45], 200, 1, 3, 10),
    ([10, 0, 0, 0], 17, 9, 2, 2),
    (CASE_11, 34, 16, 3, 32),
])
def test_symbol_size_golden(blobs, n_cols, n_rows, max_idx, expected):
    if isinstance(expected, Q.QuiltError):
        with pytest.raises(Q.QuiltError) as e:
            Q.compute_symbol_size(blobs, n_cols, n_rows, max_idx)
        assert e.value == expected
        return
    s = Q.compute_symbol_size(blobs, n_cols, n_rows, max_idx)
    assert s == expected
    assert sum(-(-b // (s * n_rows)) for b in blobs) <= n_cols


@pytest.mark.parametrize("length,mask", [(10233, 5), (10, 3), (125, 10), (1, 1), (0, 0),
                                         (0xFFFFFFFF, 0), (0, 255), (0xFFFFFFFF, 255), (1, 255),
                                         (0xFFFFFFFF, 1)])
def test_blob_header_round_trip(length, mask):
    h = Q.BlobHeaderV1(length, mask)
    raw = h.as_bytes()
    assert len(raw) == Q.BLOB_HEADER_SIZE and raw[0] == 1
    assert raw[1:5] == length.to_bytes(4, "little") and raw[5] == mask
    assert Q.BlobHeaderV1.from_bytes(raw) == h
    with pytest.raises(Q.QuiltError):
        Q.BlobHeaderV1.from_bytes(b"\x02" + raw[1:])


@pytest.mark.parametrize("ident", ["te\x08st", "\x1btest", "test\x00", "test\x01", "test\x1f",
                                   "test\x7f", "test\u0080", "test\u0081", "test\u009f", "",
                                   "trailing ", "x" * 65536])
def test_identifier_validation(ident):
    with pytest.raises(Q.QuiltError) as e:
        Q.validate_quilt_identifier(ident)
    assert e.value.kind == "InvalidIdentifier"


def test_identifier_accepts_unicode_and_inner_spaces():
    for ident in ["a", "test-blob-0", "with inner space", "日本語.txt", " leading"]:
        Q.validate_quilt_identifier(ident)


def test_index_bcs_bytes_and_round_trip():
    """QuiltIndexV1 BCS: ULEB128 count, then end_index u16le, identifier string, tag map with
    entries in the order of their serialized keys (a shorter key sorts first)."""
    idx = Q.QuiltIndexV1([Q.QuiltPatchV1("a", {"bb": "1", "c": "22"}, 1, 3),
                          Q.QuiltPatchV1("b", {}, 3, 0x0104)])
    raw = idx.to_bcs()
    assert raw == (b"\x02" + b"\x03\x00" + b"\x01a" + b"\x02" + b"\x01c\x0222" + b"\x02bb\x011"
                   + b"\x04\x01" + b"\x01b" + b"\x00")
    back = Q.QuiltIndexV1.from_bcs(raw)
    back.populate_start_indices(1)
    assert back == idx
    for bad in (raw + b"\x00", raw[:-1], b"\x81\x00"):
        with pytest.raises(Q.QuiltError):
            Q.QuiltIndexV1.from_bcs(bad)
    pid = idx.quilt_patches[1].quilt_patch_internal_id()
    assert pid.to_bytes() == b"\x01\x03\x00\x04\x01"
    assert Q.QuiltPatchInternalIdV1.from_bytes(pid.to_bytes()) == pid
    with pytest.raises(Q.QuiltError):
        Q.QuiltPatchInternalIdV1.from_bytes(b"\x02\x03\x00\x04\x01")


def _blobs(num, lo, hi, seed, tags=True):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(num):
        data = rng.integers(0, 256, int(rng.integers(lo, hi + 1)), dtype=np.uint8).tobytes()
        t = {"tag1": "value1", f"k{i % 3}": f"v{i}"} if tags and i % 2 == 0 else {}
        out.append(Q.QuiltStoreBlob(data, f"blob-{(num - i) * 7919 % 1000:03d}-{i}", t))
    return out


def _columns(quilt, config):
    """The quilt's columns as secondary slivers (sliver j = column j of the K_p x K_s matrix)."""
    kp, ks, s = config.n_primary_source_symbols, config.n_secondary_source_symbols, \
        quilt.symbol_size
    mat = np.frombuffer(quilt.data, dtype=np.uint8).reshape(kp, ks, s)
    return [SliverData(Symbols(mat[:, j, :].tobytes(), s), j, SECONDARY) for j in range(ks)]


def _check_reads(src, blobs):
    by_id = {b.identifier: b for b in blobs}
    for got in src.get_blobs_by_identifiers(list(by_id)):
        assert got == by_id[got.identifier]
    for got in src.get_blobs_by_tag("tag1", "value1"):
        assert got.tags.get("tag1") == "value1" and got == by_id[got.identifier]
    assert len(src.get_blobs_by_tag("tag1", "value1")) == sum(
        1 for b in blobs if b.tags.get("tag1") == "value1")


@pytest.mark.parametrize("num,lo,hi,n", [(3, 5, 16, 7), (3, 3, 800, 7), (3, 1024, 10240, 7),
                                         (1, 10, 1000, 7), (60, 1, 1000, 100), (2, 1, 5, 100),
                                         (10, 0, 2, 100)])
def test_construct_quilt_reads_back(num, lo, hi, n):
    cfg = ReedSolomonEncodingConfig(n)
    blobs = _blobs(num, lo, hi, seed=num * 1000 + n)
    quilt = Q.QuiltEncoderV1(cfg, blobs).construct_quilt()
    kp, ks = cfg.n_primary_source_symbols, cfg.n_secondary_source_symbols
    assert len(quilt.data) == kp * ks * quilt.symbol_size and quilt.symbol_size % 2 == 0
    index = quilt.quilt_index
    # patches sorted by identifier, contiguous, starting after the index columns
    assert index.identifiers() == sorted(b.identifier for b in blobs)
    for a, b in zip(index.quilt_patches, index.quilt_patches[1:]):
        assert a.end_index == b.start_index
    assert index.quilt_patches[-1].end_index <= ks
    # the unencoded quilt re-parses to the same index and every blob
    again = Q.QuiltV1.new_from_quilt_blob(quilt.data, cfg)
    assert again.get_or_decode_quilt_index() == index
    _check_reads(again, blobs)
    for p in index.quilt_patches:
        got = again.get_blob_by_patch_internal_id(p.quilt_patch_internal_id().to_bytes())
        assert got.identifier == p.identifier
    # the column reader over secondary slivers: index from the first column(s), patches from
    # exactly their columns
    cols = _columns(quilt, cfg)
    dec = Q.QuiltDecoderV1()
    with pytest.raises(Q.QuiltError) as e:
        dec.get_or_decode_quilt_index()
    assert e.value.kind == "MissingSlivers"
    first = index.quilt_patches[0].start_index
    dec.add_slivers(cols[:first])
    assert dec.get_or_decode_quilt_index() == index
    target = index.quilt_patches[len(index) // 2]
    with pytest.raises(Q.QuiltError) as e:
        dec.get_blobs_by_identifiers([target.identifier])
    assert e.value.kind == "MissingSlivers"
    dec.add_slivers(cols[target.start_index:target.end_index])
    (got,) = dec.get_blobs_by_identifiers([target.identifier])
    assert got == next(b for b in blobs if b.identifier == target.identifier)
    dec.add_slivers(cols)
    _check_reads(dec, blobs)
    with pytest.raises(Q.QuiltError) as e:
        dec.get_blobs_by_identifiers(["not-there"])
    assert e.value.kind == "BlobsNotFoundInQuilt"


def test_construct_quilt_errors():
    cfg = ReedSolomonEncodingConfig(7)
    a = Q.QuiltStoreBlob(b"x", "same")
    with pytest.raises(Q.QuiltError) as e:
        Q.QuiltEncoderV1(cfg, [a, Q.QuiltStoreBlob(b"y", "same")]).construct_quilt()
    assert e.value.kind == "DuplicateIdentifier"
    ks = cfg.n_secondary_source_symbols
    many = [Q.QuiltStoreBlob(b"z", f"b{i}") for i in range(ks)]
    with pytest.raises(Q.QuiltError) as e:
        Q.QuiltEncoderV1(cfg, many).construct_quilt()
    assert e.value.kind == "TooManyBlobs"
    with pytest.raises(Q.QuiltError) as e:
        Q.QuiltV1.new_from_quilt_blob(b"", cfg)
    assert e.value.kind == "EmptyInput"
    with pytest.raises(Q.QuiltError) as e:
        Q.QuiltV1.new_from_quilt_blob(b"\x01" * 7, cfg)
    assert e.value.kind == "InvalidFormatNotAligned"
    dec = Q.QuiltDecoderV1([SliverData(Symbols(b"\x00" * 8, 2), 0, SECONDARY)])
    with pytest.raises(Q.QuiltError) as e:
        dec.add_slivers([SliverData(Symbols(b"\x00" * 6, 2), 1, SECONDARY)])
    assert e.value.kind == "ColumnSizeMismatch"


def test_malformed_quilt_data():
    """Forged headers and index sizes are rejected, never read out of bounds."""
    cfg = ReedSolomonEncodingConfig(7)
    blobs = _blobs(3, 20, 60, seed=3)
    quilt = Q.QuiltEncoderV1(cfg, blobs).construct_quilt()
    mat_cols = _columns(quilt, cfg)
    col_size = len(mat_cols[0].symbols.data)
    # index size beyond 10 columns
    c0 = bytearray(mat_cols[0].symbols.data)
    c0[1:5] = (col_size * 10).to_bytes(4, "little")
    dec = Q.QuiltDecoderV1([SliverData(Symbols(bytes(c0), quilt.symbol_size), 0, SECONDARY)]
                           + mat_cols[1:])
    with pytest.raises(Q.QuiltError) as e:
        dec.get_or_decode_quilt_index()
    assert e.value.kind == "InvalidQuiltData"
    # wrong version byte
    c0 = bytearray(mat_cols[0].symbols.data)
    c0[0] = 2
    dec = Q.QuiltDecoderV1([SliverData(Symbols(bytes(c0), quilt.symbol_size), 0, SECONDARY)])
    with pytest.raises(Q.QuiltError) as e:
        dec.get_or_decode_quilt_index()
    assert e.value.kind == "QuiltVersionMismatch"
    # a blob header claiming more bytes than the quilt holds
    p = quilt.quilt_index.quilt_patches[0]
    cp = bytearray(mat_cols[p.start_index].symbols.data)
    cp[1:5] = (0xFFFFFFF0).to_bytes(4, "little")
    cols = list(mat_cols)
    cols[p.start_index] = SliverData(Symbols(bytes(cp), quilt.symbol_size), p.start_index,
                                     SECONDARY)
    dec = Q.QuiltDecoderV1(cols, quilt.quilt_index)
    with pytest.raises(Q.QuiltError) as e:
        dec.get_blobs_by_identifiers([p.identifier])
    assert e.value.kind == "InvalidQuiltData"


@pytest.mark.gpu
@pytest.mark.parametrize("num,lo,hi,n", [(3, 5, 16, 7), (3, 1024, 10240, 7), (60, 1, 1000, 100),
                                         (10, 0, 2, 100), (200, 1000, 40000, 1000)])
def test_quilt_encode_decode_device(gpu, num, lo, hi, n):
    """encode_with_metadata of a quilt on the device: the quilt id and slivers equal the
    oracle's encode of the constructed quilt blob, the metadata verifies, and every patch reads
    back from the secondary slivers (quilt_encoding.rs:2393-2590)."""
    import rs2_oracle as O
    cfg = ReedSolomonEncodingConfig(n)
    blobs = _blobs(num, lo, hi, seed=num + n)
    enc = Q.QuiltEncoderV1(cfg, blobs)
    pairs, meta = enc.encode_with_metadata()
    quilt = enc.construct_quilt()
    assert meta.index == quilt.quilt_index
    if n <= 100:
        ref = O.encode_with_metadata(quilt.data, n)
        assert bytes(meta.quilt_id) == ref.blob_id
        for i, pr in enumerate(pairs):
            assert pr.primary.symbols.data == ref.primary[i].tobytes()
    else:
        assert meta.quilt_id == cfg.compute_blob_id(quilt.data)
    secondary = [pr.secondary for pr in pairs]
    first = next(sl for sl in secondary if sl.index == 0)
    assert Q.get_quilt_version_byte(first.symbols.data) == 1
    dec = Q.QuiltDecoderV1([first])
    try:
        dec.get_or_decode_quilt_index()
    except Q.QuiltError as e:
        assert e.kind == "MissingSlivers"
        dec.add_slivers([sl for sl in secondary if sl.index in set(e.args[1])])
    assert dec.get_or_decode_quilt_index() == meta.index
    dec.add_slivers(secondary)
    _check_reads(dec, blobs)


def test_layout_plan_matches_construct_quilt():
    """The column table (input of the device column fill) reproduces construct_quilt's bytes
    when applied on the host."""
    for num, lo, hi, n in [(3, 5, 16, 7), (60, 1, 1000, 100), (10, 0, 2, 100)]:
        cfg = ReedSolomonEncodingConfig(n)
        enc = Q.QuiltEncoderV1(cfg, _blobs(num, lo, hi, seed=7 * num + n))
        quilt, lay = enc.construct_quilt(), enc.layout()
        assert lay.index == quilt.quilt_index and lay.symbol_size == quilt.symbol_size
        s, kp, ks = lay.symbol_size, lay.n_rows, lay.n_cols
        mat = np.zeros((kp, ks, s), dtype=np.uint8)
        pay = np.frombuffer(lay.payload, dtype=np.uint8)
        for c in range(ks):
            col = np.zeros(kp * s, dtype=np.uint8)
            col[:lay.col_len[c]] = pay[lay.col_off[c]:lay.col_off[c] + lay.col_len[c]]
            mat[:, c, :] = col.reshape(kp, s)
        assert mat.tobytes() == quilt.data
        assert all(o % 2 == 0 for o in lay.col_off)


@pytest.mark.gpu
@pytest.mark.parametrize("num,lo,hi,n", [(3, 5, 16, 7), (60, 1, 1000, 100), (10, 0, 2, 100),
                                         (300, 1000, 60000, 1000)])
def test_quilt_layout_device(gpu, num, lo, hi, n):
    """rs2_quilt_layout_device_async writes exactly construct_quilt's bytes, and the device
    encode of the device-built quilt gives the same quilt id as the host API."""
    import torch
    dev = torch.device("cuda", 0)
    cfg = ReedSolomonEncodingConfig(n)
    enc = Q.QuiltEncoderV1(cfg, _blobs(num, lo, hi, seed=num * 31 + n))
    quilt, lay = enc.construct_quilt(), enc.layout()
    d_pay = torch.from_numpy(np.frombuffer(lay.payload, dtype=np.uint8).copy()).to(dev)
    d_off = torch.from_numpy(lay.col_off).to(dev)
    d_len = torch.from_numpy(lay.col_len.astype(np.int32)).to(dev)
    d_q = torch.full((lay.quilt_len,), 0xAB, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    Q.quilt_layout_device_async(lay, d_pay.data_ptr(), d_off.data_ptr(), d_len.data_ptr(),
                                d_q.data_ptr(), st)
    torch.cuda.synchronize()
    assert bytes(d_q.cpu().numpy()) == quilt.data
    plan = gpu.DevicePlan(n, lay.quilt_len)
    info = plan.info
    prim = torch.empty(n * info.primary_sliver_len + 256, dtype=torch.uint8, device=dev)
    sec = torch.empty(n * info.secondary_sliver_len + 256, dtype=torch.uint8, device=dev)
    meta = torch.empty(n * 64 + 32, dtype=torch.uint8, device=dev)
    plan.encode_async(d_q.data_ptr(), prim.data_ptr(), sec.data_ptr(), meta.data_ptr(),
                      meta[n * 64:].data_ptr(), st)
    torch.cuda.synchronize()
    assert bytes(meta[n * 64:].cpu().numpy()) == bytes(cfg.compute_blob_id(quilt.data))

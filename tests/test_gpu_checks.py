"""decode_and_verify consistency checks, decode error kinds, stream ordering and the threading
contract of the C ABI, on the GPU.

  config.rs:613-658, blob_encoding.rs:579-612   Default skips the systematic primary slivers
                                                that were among the input (already verified)
  blob_encoding.rs:904-951                      dropped slivers: wrong length / symbol size
  basic_encoding.rs:387-429                     an out-of-range index ends in NotEnoughShards
  include/walrus_rs2.h threading rule           many OS threads, one plan each (C program)
"""
import os
import subprocess

import numpy as np
import pytest

import rs2_oracle as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _setup(gpu, n=13, length=5000, seed=3):
    blob = np.random.default_rng(seed).integers(0, 256, length, dtype=np.uint8).tobytes()
    cfg = gpu.ReedSolomonEncodingConfig(n)
    pairs, meta = cfg.encode_with_metadata(blob)
    return cfg, pairs, meta, blob


def _corrupt(gpu, sliver, byte=0):
    d = bytearray(sliver.symbols.data)
    d[byte] ^= 0x5A
    return gpu.SliverData(gpu.Symbols(bytes(d), sliver.symbol_size), sliver.index, sliver.axis)


def test_default_check_skips_received_systematic_slivers(gpu):
    """A corrupt systematic primary sliver that the decoder received is 'already verified'
    (config.rs:621-640): its row goes into the blob unchecked, so Default returns the altered
    blob -- the reference's outcome -- while Strict rejects it."""
    cfg, pairs, meta, blob = _setup(gpu)
    kp = cfg.n_primary_source_symbols
    prim = [pairs[i].primary for i in range(kp)]           # all systematic
    prim[2] = _corrupt(gpu, prim[2])
    got = cfg.decode_and_verify(meta, prim, "default")
    row = cfg.n_secondary_source_symbols * cfg.symbol_size_for_blob(len(blob))
    want = bytearray(blob)
    want[2 * row] ^= 0x5A
    assert got == bytes(want)
    with pytest.raises(gpu.VerificationError):
        cfg.decode_and_verify(meta, prim, "strict")
    assert cfg.decode_and_verify(meta, prim, "skip") == bytes(want)


def test_default_check_catches_unreceived_rows(gpu):
    """A corrupt repair sliver changes the decoded systematic rows that were NOT received, and
    those are re-encoded and Merkle-checked: VerificationError.  With secondary slivers every
    systematic primary sliver is checked."""
    cfg, pairs, meta, blob = _setup(gpu)
    n, kp = cfg.n_shards, cfg.n_primary_source_symbols
    prim = [pairs[i].primary for i in range(1, kp)] + [_corrupt(gpu, pairs[n - 1].primary)]
    with pytest.raises(gpu.VerificationError):
        cfg.decode_and_verify(meta, prim, "default")
    good = [pairs[i].primary for i in range(1, kp + 1)]
    assert cfg.decode_and_verify(meta, good, "default") == blob
    sec = [pairs[i].secondary for i in range(n)]
    assert cfg.decode_and_verify(meta, sec, "default") == blob
    ks = cfg.n_secondary_source_symbols
    bad = sec[:ks - 1] + [_corrupt(gpu, sec[ks - 1], 1)]
    with pytest.raises(gpu.VerificationError):
        cfg.decode_and_verify(meta, bad, "default")


def test_default_check_marks_the_pulled_surplus(gpu):
    """The sliver that finds the workspace full is pulled from the iterator and marked as
    verified although it is dropped (the reference's inspect runs before the surplus check):
    a wrong metadata hash for exactly that systematic row then goes unnoticed, while the same
    hash is caught when that sliver is not in the input."""
    cfg, pairs, meta, blob = _setup(gpu)
    n, kp = cfg.n_shards, cfg.n_primary_source_symbols
    md = meta.metadata
    hashes = list(md.hashes)
    hashes[0] = (b"\1" * 32, hashes[0][1])
    bad = gpu.VerifiedBlobMetadataWithId(meta.blob_id, gpu.BlobMetadata(hashes, md.unencoded_length))
    rep = [pairs[i].primary for i in range(kp, 2 * kp)]
    assert cfg.decode_and_verify(bad, rep + [pairs[0].primary], "default") == blob
    with pytest.raises(gpu.VerificationError):
        cfg.decode_and_verify(bad, rep, "default")


@pytest.mark.parametrize("n,length", [(13, 5000), (40, 123_457), (100, 1_000_003)])
def test_device_decode_and_verify(gpu, n, length):
    """rs2_decode_and_verify_device: the same verdicts as the host mirror on device slivers
    (blob_len-sized output, so the Default check rebuilds the zero-padded last row itself)."""
    import torch
    dev = torch.device("cuda", 0)
    blob = np.random.default_rng(n).integers(0, 256, length, dtype=np.uint8)
    ref = O.encode_with_metadata(blob.tobytes(), n)
    plan = gpu.DevicePlan(n, length)
    info = plan.info
    pl, kp = info.primary_sliver_len, info.n_primary
    b = torch.from_numpy(blob).to(dev)
    prim = torch.zeros(n * pl + 256, dtype=torch.uint8, device=dev)
    sec = torch.zeros(n * info.secondary_sliver_len + 256, dtype=torch.uint8, device=dev)
    meta = torch.zeros(n * 64 + 32, dtype=torch.uint8, device=dev)
    plan.encode_async(b.data_ptr(), prim.data_ptr(), sec.data_ptr(), meta.data_ptr(),
                      meta[n * 64:].data_ptr())
    plan.sync()
    hashes, bid = bytes(meta[:n * 64].cpu().numpy()), bytes(meta[n * 64:].cpu().numpy())
    assert bid == ref.blob_id
    out = torch.zeros(length, dtype=torch.uint8, device=dev)
    rng = np.random.default_rng(length)
    for sel in (list(rng.permutation(n)[:kp]), list(range(kp, 2 * kp)), list(range(kp))):
        for check in ("skip", "default", "strict"):
            out.zero_()
            plan.decode_and_verify("primary", sel, prim.data_ptr(), [i * pl for i in sel],
                                   hashes, bid, check, out.data_ptr())
            assert torch.equal(out, b), (sel[:4], check)
    # a corrupt repair sliver: Default and Strict reject it, Skip returns the altered blob
    sel = list(range(1, kp)) + [n - 1]
    row = prim[(n - 1) * pl:(n - 1) * pl + 1]
    row ^= 0x5A
    for check in ("default", "strict"):
        with pytest.raises(gpu.VerificationError):
            plan.decode_and_verify("primary", sel, prim.data_ptr(), [i * pl for i in sel],
                                   hashes, bid, check, out.data_ptr())
    plan.decode_and_verify("primary", sel, prim.data_ptr(), [i * pl for i in sel], hashes, bid,
                           "skip", out.data_ptr())
    plan.sync()
    assert not torch.equal(out, b)


@pytest.mark.parametrize("stream_kind", ["legacy", "torch"])
def test_device_decode_and_verify_streams(gpu, stream_kind):
    """Default and Strict on the caller's stream: the HIP null stream (handle 0, passed as
    RS2_STREAM_LEGACY) and a torch stream.  The Default check's verifier must run on that stream
    behind the decode (the C2 blob, 256 MiB at n = 1000: before the fix the null-stream case
    failed the first two of six calls this way)."""
    import torch
    dev = torch.device("cuda", 0)
    n, length = 1000, 256 << 20
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    b = torch.randint(0, 256, (length,), dtype=torch.uint8, device=dev, generator=g)
    plan = gpu.DevicePlan(n, length)
    info = plan.info
    pl, kp = info.primary_sliver_len, info.n_primary
    prim = torch.zeros(n * pl + 256, dtype=torch.uint8, device=dev)
    sec = torch.zeros(n * info.secondary_sliver_len + 256, dtype=torch.uint8, device=dev)
    meta = torch.zeros(n * 64 + 32, dtype=torch.uint8, device=dev)
    ts = torch.cuda.Stream(dev)
    st = 0 if stream_kind == "legacy" else ts.cuda_stream
    plan.encode_async(b.data_ptr(), prim.data_ptr(), sec.data_ptr(), meta.data_ptr(),
                      meta[n * 64:].data_ptr(), st)
    torch.cuda.synchronize()
    hashes, bid = bytes(meta[:n * 64].cpu().numpy()), bytes(meta[n * 64:].cpu().numpy())
    out = torch.zeros(length, dtype=torch.uint8, device=dev)
    sel = [int(i) for i in np.random.default_rng(42).permutation(n)[:kp]]
    for check in ("default", "default", "strict", "default"):
        out.zero_()
        torch.cuda.synchronize()
        plan.decode_and_verify("primary", sel, prim.data_ptr(), [i * pl for i in sel], hashes,
                               bid, check, out.data_ptr(), st)
        torch.cuda.synchronize()
        assert torch.equal(out, b), check


def test_decode_error_kinds(gpu):
    """blob_encoding.rs:904-951 + basic_encoding.rs:387-429."""
    cfg, pairs, meta, blob = _setup(gpu)
    n, kp = cfg.n_shards, cfg.n_primary_source_symbols
    s = cfg.symbol_size_for_blob(len(blob))
    prim = [pairs[i].primary for i in range(kp + 2)]
    # an out-of-range index is taken, then the column decodes fail: DecoderError
    oob = gpu.SliverData(prim[0].symbols, n + 7, gpu.PRIMARY)
    with pytest.raises(gpu.DecoderError):
        cfg.decode(len(blob), [oob] + prim[1:kp])
    # ... but not when it comes after the K_p-th sliver (surplus, dropped)
    assert cfg.decode(len(blob), prim[:kp] + [oob]) == blob
    # right length, wrong symbol size: dropped like a wrong-length sliver
    half = gpu.SliverData(gpu.Symbols(prim[0].symbols.data, s // 2), 0, gpu.PRIMARY)
    with pytest.raises(gpu.DecodingUnsuccessful):
        cfg.decode(len(blob), [half] + prim[1:kp])
    assert cfg.decode(len(blob), [half] + prim[1:kp + 1]) == blob
    with pytest.raises(gpu.DecodingUnsuccessful):
        cfg.decode(len(blob), prim[:kp - 1])
    # decode_and_verify maps a blob size too large for n_shards to DecodeDataTooLarge
    too_big = cfg.max_blob_size() + 1
    big = gpu.VerifiedBlobMetadataWithId(meta.blob_id,
                                         gpu.BlobMetadata(meta.metadata.hashes, too_big))
    with pytest.raises(gpu.encoding.DecodeDataTooLarge):
        cfg.decode_and_verify(big, prim[:kp], "skip")


def test_first_encode_on_side_stream(gpu):
    """a fresh plan's first encode, issued on a torch side stream, must see its
    offset tables (bound on that same stream) -- compared with the oracle."""
    import torch
    n, length = 40, 100_000
    blob = np.random.default_rng(11).integers(0, 256, length, dtype=np.uint8)
    ref = O.encode_with_metadata(blob.tobytes(), n)
    dev = torch.device("cuda", 0)
    side = torch.cuda.Stream(dev)
    with torch.cuda.stream(side):
        b = torch.from_numpy(blob).to(dev, non_blocking=False)
        plan = gpu.DevicePlan(n, length)
        info = plan.info
        prim = torch.zeros(n * info.primary_sliver_len + 256, dtype=torch.uint8, device=dev)
        sec = torch.zeros(n * info.secondary_sliver_len + 256, dtype=torch.uint8, device=dev)
        meta = torch.zeros(n * 64 + 32, dtype=torch.uint8, device=dev)
        plan.encode_async(b.data_ptr(), prim.data_ptr(), sec.data_ptr(), meta.data_ptr(),
                          meta[n * 64:].data_ptr(), side.cuda_stream)
    side.synchronize()
    assert bytes(meta[n * 64:].cpu().numpy()) == ref.blob_id
    pl = info.primary_sliver_len
    got = prim[:n * pl].cpu().numpy().reshape(n, pl)
    for i in range(n):
        assert got[i].tobytes() == ref.primary[i].tobytes()


def test_plan_cache_threads(gpu):
    """encoding.py's plan cache and per-plan locks: many Python threads sharing one config
    (and so its plans) encode and decode concurrently."""
    from concurrent.futures import ThreadPoolExecutor
    cfg = gpu.ReedSolomonEncodingConfig(100)
    blobs = [np.random.default_rng(i).integers(0, 256, 50_000 + (i % 3) * 999,
                                               dtype=np.uint8).tobytes() for i in range(12)]

    def job(b):
        pairs, meta = cfg.encode_with_metadata(b)
        kp = cfg.n_primary_source_symbols
        return cfg.decode_and_verify(meta, [p.primary for p in pairs[-kp:]], "default") == b, \
            meta.blob_id

    with ThreadPoolExecutor(6) as ex:
        res = list(ex.map(job, blobs))
    assert all(ok for ok, _ in res)
    serial = [gpu.ReedSolomonEncodingConfig(100).compute_blob_id(b) for b in blobs]
    assert [bid for _, bid in res] == serial


def test_c_abi_threads(gpu):
    """tests/capi/threads.c: 6 OS threads, one plan each, encode / decode / decode_and_verify /
    sliver roots concurrently through the C ABI with the system ROCm runtime (no torch in the
    process), then a serial re-encode of every blob id."""
    exe = os.path.join(ROOT, "tests", "capi", "build", "threads")
    assert os.path.exists(exe), "build it first: make -C tests/capi (done by build())"
    env = dict(os.environ)
    res = subprocess.run([exe, "6", "3", "1000", str(4 << 20)], capture_output=True, text=True,
                         timeout=240, env=env)
    assert res.returncode == 0, res.stdout + res.stderr
    assert "threads ok" in res.stdout


def test_plan_rebind(gpu):
    """rs2_plan_rebind: one plan per (n_shards, symbol size) serves every length of that size
    class -- encode and decode after a rebind equal the oracle's; a length of another symbol
    size is IncompatibleParameters and leaves the plan as it was."""
    import ctypes
    from walrus_amd import _lib
    n = 40
    cfg = gpu.ReedSolomonEncodingConfig(n)
    k = cfg.source_symbols_per_blob()
    lens = [k * 10 - 3, k * 9 + 1, k * 10, k * 9 + 2]           # all symbol size 10
    assert {cfg.symbol_size_for_blob(x) for x in lens} == {10}
    plans = set()
    for length in lens:
        blob = np.random.default_rng(length).integers(0, 256, length, dtype=np.uint8).tobytes()
        pairs, meta = cfg.encode_with_metadata(blob)
        plans.add(id(cfg._plan(length)))
        ref = O.encode_with_metadata(blob, n)
        assert bytes(meta.blob_id) == ref.blob_id
        kp = cfg.n_primary_source_symbols
        assert cfg.decode_and_verify(meta, [p.primary for p in pairs[n - kp:]], "strict") == blob
        assert cfg.decode(length, [p.primary for p in pairs[:kp]]) == blob
    assert len(plans) == 1
    p = cfg._plan(lens[0])
    with p.lock:
        rc = _lib.lib().rs2_plan_rebind(p.handle, k * 20)
        assert rc == _lib.RS2_E_INCOMPATIBLE_PARAMETERS
        info = _lib.PlanInfo()
        _lib.lib().rs2_plan_info_get(p.handle, ctypes.byref(info))
        assert info.blob_len == p.blob_len and info.symbol_size == 10


def test_c_abi_arena(gpu):
    """tests/capi/arena.c: 8 OS threads share a plan cache keyed by symbol size over 200
    distinct blob lengths (n = 1000, 1 KiB .. 256 MiB), encode + decode_and_verify each, pass
    after pass until one whole pass calls hipMalloc zero times and pins no host memory (at most
    6 warm-up passes), every pass reproducing the blob ids.  Prints the arena's peak live bytes."""
    exe = os.path.join(ROOT, "tests", "capi", "build", "arena")
    assert os.path.exists(exe), "build it first: make -C tests/capi (done by build())"
    res = subprocess.run([exe, "8", "200", "1000", str(256 << 20), "8", "6"], capture_output=True,
                         text=True, timeout=400)
    print(res.stdout)
    assert res.returncode == 0, res.stdout + res.stderr
    assert "arena ok" in res.stdout
    # a fixed budget (12 GiB of device arena, 8 pinned rings reserved up front): the first pass
    # already runs on the reserve and the second allocates nothing at all
    env = dict(os.environ, RS2_ARENA_RESERVE_MIB="12288", RS2_STAGING_RINGS="8")
    res = subprocess.run([exe, "8", "200", "1000", str(256 << 20), "8", "1"], capture_output=True,
                         text=True, timeout=400, env=env)
    print(res.stdout)
    assert res.returncode == 0, res.stdout + res.stderr
    assert "pass 1: " in res.stdout and "1 hipMalloc in all" in res.stdout


def test_host_register_direct_dma(gpu):
    """rs2_host_register: host-buffer calls whose buffers are registered move them by DMA
    straight to / from the device (no staging ring); the slivers, hashes, BlobId and the decoded
    blob are identical to the staged path's, with only some buffers registered (direct and
    staged segments in one call) and with all of them.  Overlapping ranges and unknown pointers
    are refused."""
    import ctypes
    from walrus_amd import _lib
    L = _lib.lib()
    n, length = 100, (5 << 20) + 777  # every buffer above the 4 MiB direct-DMA threshold
    cfg = gpu.ReedSolomonEncodingConfig(n)
    plan = cfg._plan(length)
    info = plan.info
    pl, sl, kp = info.primary_sliver_len, info.secondary_sliver_len, info.n_primary
    blob = np.random.default_rng(5).integers(0, 256, length, dtype=np.uint8)

    def run(register):
        prim = np.zeros((n, pl), dtype=np.uint8)
        sec = np.zeros((n, sl), dtype=np.uint8)
        hashes = np.zeros(n * 64, dtype=np.uint8)
        bid = np.zeros(32, dtype=np.uint8)
        out = np.zeros(length, dtype=np.uint8)
        regs = [b for b, name in ((blob, "blob"), (prim, "prim"), (sec, "sec"), (out, "out"))
                if name in register]
        for b in regs:
            assert L.rs2_host_register(b.ctypes.data, b.nbytes) == 0, _lib.last_error()
        try:
            pp = (ctypes.c_void_p * n)(*[prim[i].ctypes.data for i in range(n)])
            sp = (ctypes.c_void_p * n)(*[sec[i].ctypes.data for i in range(n)])
            assert L.rs2_encode_with_metadata(plan.handle, blob.ctypes.data, pp, sp,
                                              hashes.ctypes.data, bid.ctypes.data) == 0
            idx = [int(i) for i in np.random.default_rng(1).permutation(n)[:kp]]
            ia = (ctypes.c_uint16 * kp)(*idx)
            sa = (ctypes.c_void_p * kp)(*[prim[i].ctypes.data for i in idx])
            la = (ctypes.c_uint64 * kp)(*([pl] * kp))
            assert L.rs2_decode_blob(plan.handle, 0, kp, ia, sa, la, None, out.ctypes.data) == 0
        finally:
            for b in regs:
                assert L.rs2_host_unregister(b.ctypes.data) == 0
        return prim, sec, hashes, bid, out

    want = run(())
    assert np.array_equal(want[4], blob)
    for register in (("prim",), ("blob", "sec"), ("blob", "prim", "sec", "out")):
        got = run(register)
        for a, b in zip(got, want):
            assert np.array_equal(a, b), register
    buf = np.zeros(1 << 20, dtype=np.uint8)
    assert L.rs2_host_register(buf.ctypes.data, buf.nbytes) == 0
    try:
        assert L.rs2_host_register(buf.ctypes.data + 4096, 4096) != 0  # overlap
        assert L.rs2_host_unregister(buf.ctypes.data + 4096) != 0      # not a registered start
    finally:
        assert L.rs2_host_unregister(buf.ctypes.data) == 0
    assert L.rs2_host_unregister(buf.ctypes.data) != 0


def test_device_memory_trim(gpu):
    """rs2_device_memory_trim: after a transient large plan is gone, its arena
    segments go back to hipFree on request and the reserve shrinks by what was released."""
    import gc
    from walrus_amd.encoding import device_memory_stats, device_memory_trim
    plan = gpu.DevicePlan(1000, 1 << 30)  # ~7 GB of plan buffers
    assert device_memory_stats()["reserved"] >= 1 << 30
    del plan
    gc.collect()
    before = device_memory_stats()
    released = device_memory_trim()
    after = device_memory_stats()
    # (the plan's ranges may share a segment with live buffers of earlier tests, so how much
    # comes back depends on the arena's history; what was released left the reserve)
    assert after["reserved"] == before["reserved"] - released
    assert after["reserved"] >= after["live"]
    assert (after["frees"] > before["frees"]) == (released > 0)
    assert device_memory_trim() == 0  # nothing wholly free is left
    # the engine still works on a fresh segment afterwards
    cfg = gpu.ReedSolomonEncodingConfig(10)
    _, meta = cfg.encode_with_metadata(b"walrus blob id v1 regression test")
    assert str(meta.blob_id) == "RcU82Mwf-CFkv1LaI_2qcpANwpGUuG3TMwnVzZxD2kY"


def test_arena_churn_past_cache_cap(gpu):
    """plan churn with more device memory live than the arena's 8 GiB cache
    (tests/capi/arena.c churn mode: 8 OS threads, blobs up to 1 GiB, two cached plans, so
    plans are destroyed and rebuilt all the time and the live peak passes the cap).  Segments
    falling wholly free past the cap must go back to hipFree (outside the arena lock, while the
    other threads keep allocating), the reserve must end below the live peak, and every blob id
    and decode must still match."""
    exe = os.path.join(ROOT, "tests", "capi", "build", "arena")
    assert os.path.exists(exe), "build it first: make -C tests/capi (done by build())"
    res = subprocess.run([exe, "8", "24", "1000", str(1 << 30), "2", "1", "churn"],
                         capture_output=True, text=True, timeout=400)
    print(res.stdout)
    assert res.returncode == 0, res.stdout + res.stderr
    assert "arena churn ok" in res.stdout


def test_fresh_erasure_patterns_device(gpu):
    """A new erasure pattern on every call (a client read: a new sliver subset per blob), as the
    bench's headline step decodes: every decode re-plans (locator FWHT, block mixing, table
    uploads, multiplier-table kernel) on the plan's two alternating slots while the previous
    decode may still run, and must return the blob each time (basic_encoding.rs:387-429)."""
    import torch
    n, blob_len = 1000, 40_000_000
    dev = torch.device("cuda", 0)
    blob = torch.from_numpy(np.random.default_rng(21).integers(0, 256, blob_len,
                                                                 dtype=np.uint8)).to(dev)
    plan = gpu.DevicePlan(n, blob_len)
    info = plan.info
    pl, kp = info.primary_sliver_len, info.n_primary
    prim = torch.empty(n * pl + 256, dtype=torch.uint8, device=dev)
    sec = torch.empty(n * info.secondary_sliver_len + 256, dtype=torch.uint8, device=dev)
    meta = torch.empty(n * 64 + 32, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    plan.encode_async(blob.data_ptr(), prim.data_ptr(), sec.data_ptr(), meta.data_ptr(),
                      meta[n * 64:].data_ptr(), st)
    outs = [torch.empty_like(blob) for _ in range(3)]
    rng = np.random.default_rng(22)
    subsets = [[int(i) for i in rng.permutation(n)[:kp]] for _ in range(24)]
    subsets += [list(range(n - kp, n)), list(range(kp)), list(range(0, 2 * kp, 2))]
    for k, sel in enumerate(subsets):
        out = outs[k % 3]
        out.zero_()
        plan.decode_async("primary", sel, prim.data_ptr(), [i * pl for i in sel], out.data_ptr(),
                          st)
        if k % 3 == 2:  # three decodes in flight between checks
            torch.cuda.synchronize(dev)
            for o in outs:
                assert torch.equal(o, blob), k
    torch.cuda.synchronize(dev)

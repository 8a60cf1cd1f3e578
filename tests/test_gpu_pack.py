"""rs2_copy_segments_device_async (the partitioned encode's exchange packing, partition.py):
every copy width against a numpy restatement of the same segment map, and the rows-phase
transposition of a C4-shaped partition against torch's own transpose."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _copy(gpu, src, dst, sa, da, count_b, ssb, dsb, seg_len, unit):
    import torch
    from walrus_amd import _lib
    dev = src.device
    tsa = torch.from_numpy(np.asarray(sa, dtype=np.int64)).to(dev)
    tda = torch.from_numpy(np.asarray(da, dtype=np.int64)).to(dev)
    rc = _lib.lib().rs2_copy_segments_device_async(
        src.data_ptr(), dst.data_ptr(), len(sa), tsa.data_ptr(), tda.data_ptr(), count_b, ssb, dsb,
        seg_len, unit, ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
    torch.cuda.synchronize(dev)
    return rc


@pytest.mark.parametrize("unit,seg_len,count_b", [(16, 48, 3), (8, 40, 5), (4, 1204, 2),
                                                   (2, 1206, 7), (1, 33, 4), (16, 19280, 2)])
def test_copy_segments_widths(gpu, unit, seg_len, count_b):
    import torch
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(unit * 1000 + seg_len)
    count_a = 37
    ssb, dsb = seg_len * count_a + unit * 3, seg_len
    n_src = count_b * ssb + count_a * seg_len + 64
    src_h = rng.integers(0, 256, n_src, dtype=np.uint8)
    sa = [a * seg_len for a in rng.permutation(count_a)]
    da = [a * count_b * seg_len for a in range(count_a)]
    dst_h = np.zeros(count_a * count_b * seg_len + 64, dtype=np.uint8)
    want = dst_h.copy()
    for a in range(count_a):
        for b in range(count_b):
            want[da[a] + b * dsb:da[a] + b * dsb + seg_len] = \
                src_h[sa[a] + b * ssb:sa[a] + b * ssb + seg_len]
    src = torch.from_numpy(src_h).to(dev)
    dst = torch.from_numpy(dst_h).to(dev)
    assert _copy(gpu, src, dst, sa, da, count_b, ssb, dsb, seg_len, unit) == 0
    assert np.array_equal(dst.cpu().numpy(), want)


def test_copy_segments_rejects_misaligned(gpu):
    import torch
    from walrus_amd import _lib
    dev = torch.device("cuda", 0)
    src = torch.zeros(4096, dtype=torch.uint8, device=dev)
    dst = torch.zeros(4096, dtype=torch.uint8, device=dev)
    assert _copy(gpu, src, dst, [0], [0], 1, 0, 0, 40, 16) == _lib.RS2_E_INVALID_ARGUMENT
    assert _copy(gpu, src[2:], dst, [0], [0], 1, 0, 0, 32, 4) == _lib.RS2_E_INVALID_ARGUMENT


@pytest.mark.parametrize("n,blob_len,world", [(40, 300_001, 3), (100, 1_000_003, 8)])
def test_rows_phase_pack_matches_transpose(gpu, n, blob_len, world):
    """rows_phase's send buffer equals the transposed copies it replaced (torch reference)."""
    import torch
    from walrus_amd import partition as P
    dev = torch.device("cuda", 0)
    p = P.Partition.for_blob(n, blob_len, world)
    ops = P.DeviceOps()
    blob = torch.from_numpy(np.random.default_rng(n).integers(0, 256, blob_len, dtype=np.uint8))
    for g in range(world):
        rows = P.rows_of_blob(p, blob.to(dev), g)
        enc = P.RankEncoder(p, g, ops, dev)
        send = enc.rows_phase(rows)
        torch.cuda.synchronize()
        nrg = len(p.rows(g))
        if nrg == 0:
            continue
        # send layout [G][nr][nt][s]: column c of local row b -> its owner's chunk and slot
        G, nt, nr, s, ks = p.world, p.nt, p.nr, p.s, p.ks
        sv = send[:G * nr * nt * s].view(G, nr, nt, s)
        rv = rows[:nrg * ks * s].view(nrg, ks, s)
        for c in range(ks):
            h, j = p.col_owner(c)
            assert torch.equal(sv[h, :nrg, j], rv[:, c])

"""Row/column-partitioned encode + decode of one blob across G ranks (walrus_amd/partition.py,
SURVEY.md 8(e), config C4).

CPU tests run the partitioning and the exchanges with the numpy oracle as the compute backend
(tests/cpu_ops.py, test-only): in one process (`simulate_*`, the exchanges done by hand) and
across 2 gloo processes (`encode_distributed` / `decode_distributed`, the same collectives the
RCCL path issues).  The GPU tests run the same phases through the HIP engine's C ABI
(DeviceOps: rs2_codec_*, rs2_leaf_hashes / merkle_roots / blob_id device calls) and compare
with the engine's single-GPU plan encode (itself oracle-pinned) and with the blob.
Expected values: oracle.encode_with_metadata (blob_encoding.rs:277-368) and the blob itself.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import rs2_oracle as O  # noqa: E402
from walrus_amd import partition as P  # noqa: E402


def _blob(n_bytes, seed):
    return np.random.default_rng(seed).integers(0, 256, n_bytes, dtype=np.uint8)


def _oracle_pairs(enc):
    return np.frombuffer(b"".join(p + s for p, s in enc.pair_hashes), dtype=np.uint8)


# ---- partition geometry -----------------------------------------------------------------------
@pytest.mark.parametrize("n", [4, 7, 10, 13, 31, 100, 1000])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_partition_covers_everything_once(n, world):
    p = P.Partition.for_blob(n, 12345, world)
    rows = [r for g in range(world) for r in p.rows(g)]
    assert rows == list(range(p.kp))
    cols = sorted(p.col(g, j) for g in range(world) for j in range(p.nt) if p.col(g, j) >= 0)
    assert cols == list(range(n))
    assert [i for g in range(world) for i in p.pairs(g)] == list(range(n))
    for g in range(world):
        # a rank's columns are exactly the secondary slivers of its pairs (lib.rs:485-491)
        assert sorted(p.cols(g)) == sorted(n - 1 - i for i in p.pairs(g))
        # its systematic columns (< K_s) are its first msys slots
        for j in range(p.nv(g)):
            assert (p.col(g, j) < p.ks) == (j < p.msys(g))
            assert p.col_owner(p.col(g, j)) == (g, j)
    assert sum(p.msys(g) for g in range(world)) == p.ks
    assert [c for g in range(world) for c in p.sys_cols(g)] == list(range(p.ks))
    spans = [p.row_bytes(g) for g in range(world)]
    assert spans[0].start == 0 and spans[-1].stop == min(p.blob_len, p.kp * p.ks * p.s)
    assert all(a.stop == b.start for a, b in zip(spans, spans[1:]))
    assert p.x_rows >= world * p.nr and p.x_rows >= n


# ---- single-process simulation on CPU ---------------------------------------------------------
def _check_encoded(part, encs, blob, n):
    enc = O.encode_with_metadata(blob.tobytes(), n)
    for e in encs:
        assert bytes(e.blob_id.numpy()) == enc.blob_id
        assert np.array_equal(e.hashes.numpy(), _oracle_pairs(enc))
    prim, sec = P.gather_slivers(part, encs)
    assert np.array_equal(prim.numpy(), enc.primary)
    assert np.array_equal(sec.numpy(), enc.secondary)
    # every rank holds the sliver pairs P_g it owns: primary i with secondary n-1-i
    for g, e in enumerate(encs):
        assert e.pairs == part.pairs(g)
        for i in e.pairs:
            pr, se = e.sliver_pair(i, part)
            assert np.array_equal(pr.numpy(), enc.primary[i])
            assert np.array_equal(se.numpy(), enc.secondary[n - 1 - i])


@pytest.mark.parametrize("n,blob_len,world", [(10, 333, 1), (10, 333, 2), (10, 1000, 3),
                                              (13, 2222, 4), (7, 50, 8), (31, 4000, 4),
                                              (100, 20000, 3)])
def test_simulated_encode_decode_matches_oracle(n, blob_len, world):
    from cpu_ops import CpuOps
    blob = _blob(blob_len, seed=n * 1000 + world)
    part = P.Partition.for_blob(n, blob_len, world)
    t = torch.from_numpy(blob.copy())
    rows = [P.rows_of_blob(part, t, g) for g in range(world)]
    ops = CpuOps()
    cpu = torch.device("cpu")
    encs = P.simulate_encode(part, rows, ops, cpu)
    _check_encoded(part, encs, blob, n)
    rng = np.random.default_rng(7)
    # a random K_p subset, and the worst case with no systematic sliver at all
    for idx in (rng.permutation(n)[:part.kp], np.arange(part.kp, 2 * part.kp) % n):
        out = P.simulate_decode(part, encs, [int(i) for i in idx], ops, cpu)
        assert bytes(out.numpy()) == blob.tobytes()


# ---- two gloo processes -----------------------------------------------------------------------
N_D, LEN_D = 10, 777


def _worker(rank, world, port, q, N_D=N_D, LEN_D=LEN_D):
    import torch.distributed as dist
    from cpu_ops import CpuOps
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        blob = torch.from_numpy(_blob(LEN_D, seed=5))
        part = P.Partition.for_blob(N_D, LEN_D, world)
        ex = P.DistExchange()
        ops = CpuOps()
        cpu = torch.device("cpu")
        enc = P.encode_distributed(part, P.rows_of_blob(part, blob, rank), ops, ex, cpu)
        idx = [int(i) for i in np.random.default_rng(3).permutation(N_D)[:part.kp]]
        out = P.decode_distributed(part, enc, idx, ops, ex, cpu)
        # decode ingest: K_p full primary slivers arrive on rank 0 (as from storage nodes) and
        # are scattered by column range; they come from the oracle's encode of the blob
        sl = None
        if rank == 0:
            ref = O.encode_with_metadata(blob.numpy().tobytes(), N_D)
            sl = torch.from_numpy(np.concatenate([ref.primary[i] for i in idx]).copy())
        out2 = P.decode_from_slivers(part, sl, idx, ops, ex, cpu)
        sl0 = P.collect_primary(part, enc, idx, ex)
        q.put((rank, enc.primary.numpy().copy(), enc.secondary.numpy().copy(),
               enc.hashes.numpy().copy(), enc.blob_id.numpy().copy(),
               None if out is None else out.numpy().copy(),
               None if out2 is None else out2.numpy().copy(),
               None if sl0 is None else sl0.numpy().copy()))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,N_D,LEN_D", [(2, N_D, LEN_D), (4, 100, 5000), (8, 1000, 4000)])
def test_distributed_encode_decode_gloo(world, N_D, LEN_D):
    """world 4 at n = 100: rank 0's columns are all repair columns, so its primary-sliver
    exchange sends nothing (zero split sizes).  world 8 at n = 1000 is the call sequence the
    8-GPU C4 run issues (nt = 125 pairs per rank, K_p = 334 rows over 8 ranks: uneven row
    slices; ranks 0 and 1 own only repair columns, so zero split sizes in exchange 3)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, N_D, LEN_D))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r = q.get(timeout=240)
        res[r[0]] = r[1:]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    blob = _blob(LEN_D, seed=5)
    part = P.Partition.for_blob(N_D, LEN_D, world)
    encs = [P.RankEncoded(part.pairs(g), *[torch.from_numpy(res[g][k]) for k in range(4)])
            for g in range(world)]
    _check_encoded(part, encs, blob, N_D)
    assert res[0][4] is not None and bytes(res[0][4]) == blob.tobytes()
    assert all(res[g][4] is None for g in range(1, world))
    assert res[0][5] is not None and bytes(res[0][5]) == blob.tobytes()
    assert all(res[g][5] is None for g in range(1, world))
    ref = O.encode_with_metadata(blob.tobytes(), N_D)
    idx = [int(i) for i in np.random.default_rng(3).permutation(N_D)[:part.kp]]
    assert res[world - 1][6] is None and bytes(res[0][6]) == b"".join(ref.primary[i].tobytes() for i in idx)


# ---- GPU: the same phases through the HIP engine ------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("n,blob_len,world", [(10, 3333, 2), (100, 1 << 20, 3),
                                              (1000, 4 << 20, 2), (1000, 4 << 20, 8)])
def test_gpu_partitioned_encode_decode(gpu, n, blob_len, world):
    dev = torch.device("cuda", 0)
    blob = torch.from_numpy(_blob(blob_len, seed=11)).to(dev)
    part = P.Partition.for_blob(n, blob_len, world)
    ops = P.DeviceOps()
    rows = [P.rows_of_blob(part, blob, g) for g in range(world)]
    encs = P.simulate_encode(part, rows, ops, dev)
    torch.cuda.synchronize()
    # the single-GPU plan encode of the same blob (oracle-pinned by the other gpu tests)
    plan = gpu.DevicePlan(n, blob_len)
    info = plan.info
    pl, sl = info.primary_sliver_len, info.secondary_sliver_len
    prim = torch.empty(n * pl + 256, dtype=torch.uint8, device=dev)
    sec = torch.empty(n * sl + 256, dtype=torch.uint8, device=dev)
    hashes = torch.empty(n * 64, dtype=torch.uint8, device=dev)
    bid = torch.empty(32, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    plan.encode_async(blob.data_ptr(), prim.data_ptr(), sec.data_ptr(), hashes.data_ptr(),
                      bid.data_ptr(), st)
    torch.cuda.synchronize()
    for e in encs:
        assert torch.equal(e.blob_id, bid)
        assert torch.equal(e.hashes, hashes)
    gp, gs = P.gather_slivers(part, encs)
    assert torch.equal(gp.reshape(-1), prim[:n * pl])
    assert torch.equal(gs.reshape(-1), sec[:n * sl])
    if blob_len < 1 << 16:
        enc = O.encode_with_metadata(blob.cpu().numpy().tobytes(), n)
        assert bytes(bid.cpu().numpy()) == enc.blob_id
    idx = [int(i) for i in np.random.default_rng(9).permutation(n)[:part.kp]]
    out = P.simulate_decode(part, encs, idx, ops, dev)
    torch.cuda.synchronize()
    assert torch.equal(out, blob)
    received = torch.cat([prim[i * pl:(i + 1) * pl] for i in idx])
    out = P.simulate_decode_from_slivers(part, received, idx, ops, dev)
    torch.cuda.synchronize()
    assert torch.equal(out, blob)

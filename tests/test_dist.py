"""Multi-rank placement of independent blobs (walrus_amd/dist.py) on CPU with gloo, world 2.

The data path has no collective (each rank encodes its own blobs); these tests check the
sharding is a partition and that the per-blob BlobIds come back in blob order on every rank.
The per-blob encode is the CPU oracle here (test-only checker); on a GPU box the same code
runs the HIP engine (bench.py / dist.encode_blobs default).
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from walrus_amd import dist as D  # noqa: E402


def test_shard_blobs_is_partition():
    for n in (0, 1, 7, 128):
        for w in (1, 2, 3, 8):
            seen = sorted(i for r in range(w) for i in D.shard_blobs(n, r, w))
            assert seen == list(range(n))
            sizes = [len(D.shard_blobs(n, r, w)) for r in range(w)]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        D.shard_blobs(4, 2, 2)


def _blobs():
    return [np.random.default_rng(100 + i).integers(0, 256, 200 + 37 * i, dtype=np.uint8).tobytes()
            for i in range(5)]


def _oracle_blob_id(blob: bytes, n: int) -> bytes:
    import rs2_oracle as O
    return bytes(O.encode_with_metadata(blob, n).blob_id)


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ids = D.encode_blobs(_blobs(), 10, rank, world, encode_fn=_oracle_blob_id)
        q.put((rank, [i.hex() for i in ids]))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_encode_blobs_world2_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [_oracle_blob_id(b, 10).hex() for b in _blobs()]
    assert res[0] == want and res[1] == want

"""Multi-GPU placement for the RS2 engine: one process per GPU, independent blobs.

Red Stuff blobs are independent units of work, so the data path shards with no collective:
every rank encodes (or decodes) its own blobs on its own GPU (the
reference spreads blobs over rayon workers, walrus-sdk/src/node_client.rs:3182).  The only
exchange is the small per-blob result records (BlobId / metadata digests, 32 bytes each),
gathered once at the end so every rank sees the same ordered list, as the client does when
it registers a batch of blobs.
"""
from __future__ import annotations

import os
from typing import Callable, List, Optional, Sequence


def world() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torchrun environment (1 process = 1 GPU)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_blobs(n_blobs: int, rank: int, world_size: int) -> List[int]:
    """Blob indices owned by `rank`: round-robin, so ranks differ by at most one blob."""
    if world_size < 1 or not 0 <= rank < world_size:
        raise ValueError("invalid rank / world size")
    return list(range(rank, n_blobs, world_size))


def gather_digests(local: Sequence[bytes], n_blobs: int, rank: int, world_size: int,
                   group=None) -> List[bytes]:
    """All-gather 32-byte per-blob digests into blob order (rank r owns shard_blobs(r))."""
    import torch
    import torch.distributed as dist

    per_rank = (n_blobs + world_size - 1) // world_size
    buf = torch.zeros(per_rank * 32, dtype=torch.uint8)
    for j, d in enumerate(local):
        if len(d) != 32:
            raise ValueError("digest must be 32 bytes")
        buf[j * 32:(j + 1) * 32] = torch.frombuffer(bytearray(d), dtype=torch.uint8)
    backend = dist.get_backend(group) if dist.is_initialized() else "gloo"
    if backend == "nccl":
        buf = buf.cuda()
    out = [torch.zeros_like(buf) for _ in range(world_size)]
    dist.all_gather(out, buf, group=group)
    result: List[Optional[bytes]] = [None] * n_blobs
    for r in range(world_size):
        rows = out[r].cpu().numpy().tobytes()
        for j, b in enumerate(shard_blobs(n_blobs, r, world_size)):
            result[b] = rows[j * 32:(j + 1) * 32]
    return result  # type: ignore[return-value]


def encode_blobs(blobs: Sequence[bytes], n_shards: int, rank: int, world_size: int,
                 encode_fn: Optional[Callable[[bytes, int], bytes]] = None,
                 group=None) -> List[bytes]:
    """Encode this rank's share of `blobs` and return every blob's BlobId (all ranks).

    `encode_fn(blob, n_shards) -> blob_id` defaults to the HIP engine
    (ReedSolomonEncodingConfig.compute_blob_id); tests pass a CPU checker to exercise the
    placement and gather logic without a GPU."""
    if encode_fn is None:
        from .encoding import ReedSolomonEncodingConfig

        cfg = ReedSolomonEncodingConfig(n_shards)

        def encode_fn(b: bytes, n: int) -> bytes:  # noqa: ARG001
            return bytes(cfg.compute_blob_id(b))

    mine = shard_blobs(len(blobs), rank, world_size)
    local = [encode_fn(blobs[i], n_shards) for i in mine]
    if world_size == 1:
        return local
    return gather_digests(local, len(blobs), rank, world_size, group)

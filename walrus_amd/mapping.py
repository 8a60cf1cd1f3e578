"""Sliver pair <-> shard assignment (crates/walrus-core/src/encoding/mapping.rs:24-135).

The encoder's pair i goes to shard (i + rotation) mod n, where the rotation is the BlobId read as
a big-endian integer mod n (the storage-side format around the path).
"""

from __future__ import annotations

from typing import List, MutableSequence


class SliverAssignmentError(Exception):
    """mapping.rs:14-22: `kind` is InconsistentRotation or InvalidInputOrder."""

    def __init__(self, kind: str):
        super().__init__(kind)
        self.kind = kind


def bytes_mod(data: bytes, modulus: int) -> int:
    """mapping.rs:128-135: big-endian integer mod `modulus` (Horner)."""
    acc = 0
    for b in bytes(data):
        acc = (acc * 256 + b) % modulus
    return acc


def rotation_offset(n_shards: int, blob_id: bytes) -> int:
    return bytes_mod(blob_id, n_shards)


def pair_to_shard_index(pair_index: int, n_shards: int, blob_id: bytes) -> int:
    """SliverPairIndex::to_shard_index (mapping.rs:90-99)."""
    return (pair_index + rotation_offset(n_shards, blob_id)) % n_shards


def shard_to_pair_index(shard_index: int, n_shards: int, blob_id: bytes) -> int:
    """ShardIndex::to_pair_index (mapping.rs:101-112)."""
    return (n_shards + shard_index - rotation_offset(n_shards, blob_id)) % n_shards


def _is_rotation(pairs) -> bool:
    """mapping.rs:79-86 (checks only the pair indices)."""
    first = pairs[0].index
    return all(p.index == (i + first) % len(pairs) for i, p in enumerate(pairs))


def _rotate_right(pairs: MutableSequence, k: int) -> None:
    if k:
        pairs[:] = list(pairs[-k:]) + list(pairs[:-k])


def rotate_pairs_unchecked(pairs: MutableSequence, blob_id: bytes) -> None:
    """mapping.rs:69-77: the last `blob_id % len` pairs move to the front."""
    if pairs:
        _rotate_right(pairs, bytes_mod(blob_id, len(pairs)))


def rotate_pairs(pairs: MutableSequence, blob_id: bytes) -> None:
    """mapping.rs:43-67: rotate in place; no-op if already rotated for this blob id."""
    n = len(pairs)
    if n == 0:
        return
    if n > 0xFFFF:
        raise ValueError("there must not be more than u16::MAX sliver pairs")
    if not _is_rotation(pairs):
        raise SliverAssignmentError("InvalidInputOrder")
    if pairs[0].index == 0:
        rotate_pairs_unchecked(pairs, blob_id)
    elif pairs[0].index != shard_to_pair_index(0, n, blob_id):
        raise SliverAssignmentError("InconsistentRotation")


def pairs_for_shards(n_shards: int, blob_id: bytes) -> List[int]:
    """Pair index stored on each shard 0..n-1 (the rotated order as plain indices)."""
    off = rotation_offset(n_shards, blob_id)
    return [(n_shards + s - off) % n_shards for s in range(n_shards)]

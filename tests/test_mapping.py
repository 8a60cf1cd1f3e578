"""Pair <-> shard rotation (walrus_amd/mapping.py) against the reference's own cases
(crates/walrus-core/src/encoding/mapping.rs:145-310)."""
from dataclasses import dataclass

import pytest

from walrus_amd import mapping as M


def blob_id_from_u64(v: int) -> bytes:
    """test_utils.rs:272-283: u64 big-endian in the last 8 bytes."""
    return bytes(24) + v.to_bytes(8, "big")


@dataclass
class Pair:
    index: int


def pairs(n):
    return [Pair(i) for i in range(n)]


@pytest.mark.parametrize("index,bid", [(0, 0), (1, 0), (0, 1), (11, 27)])
def test_shard_pair_conversion_round_trips(index, bid):
    b = blob_id_from_u64(bid)
    assert M.pair_to_shard_index(M.shard_to_pair_index(index, 13, b), 13, b) == index
    assert M.shard_to_pair_index(M.pair_to_shard_index(index, 13, b), 13, b) == index


@pytest.mark.parametrize("n,bid,pair,shard", [(7, 15, 0, 1), (7, 15, 5, 6), (7, 15, 6, 0)])
def test_shard_index_for_pair(n, bid, pair, shard):
    assert M.pair_to_shard_index(pair, n, blob_id_from_u64(bid)) == shard


@pytest.mark.parametrize("n,bid,shard,pair", [(7, 16, 0, 5), (7, 16, 1, 6), (7, 16, 6, 4)])
def test_pair_index_for_shard(n, bid, shard, pair):
    assert M.shard_to_pair_index(shard, n, blob_id_from_u64(bid)) == pair


def test_rotate_pairs_and_unchecked_composition():
    b17 = blob_id_from_u64(17)
    p = pairs(7)
    M.rotate_pairs(p, b17)
    assert [q.index for q in p] == [M.shard_to_pair_index(i, 7, b17) for i in range(7)]
    assert [q.index for q in p] == M.pairs_for_shards(7, b17)
    q = pairs(7)
    M.rotate_pairs_unchecked(q, b17)
    M.rotate_pairs_unchecked(q, blob_id_from_u64(15))
    b18 = blob_id_from_u64(18)  # 17 % 7 + 15 % 7 = 18 % 7
    assert [x.index for x in q] == [M.shard_to_pair_index(i, 7, b18) for i in range(7)]


def test_rotation_checks():
    b17 = blob_id_from_u64(17)
    p = pairs(7)
    M.rotate_pairs(p, b17)
    before = [x.index for x in p]
    M.rotate_pairs(p, b17)  # idempotent
    assert [x.index for x in p] == before
    with pytest.raises(M.SliverAssignmentError) as e:
        M.rotate_pairs(p, blob_id_from_u64(18))
    assert e.value.kind == "InconsistentRotation"
    p[2], p[5] = p[5], p[2]
    with pytest.raises(M.SliverAssignmentError) as e:
        M.rotate_pairs(p, b17)
    assert e.value.kind == "InvalidInputOrder"
    M.rotate_pairs([], b17)


def test_bytes_mod():
    """mapping.rs test_bytes_mod: agrees with integer arithmetic."""
    for x in range(0, 10_000, 37):
        for y in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29):
            raw = x.to_bytes(8, "big")
            assert M.bytes_mod(raw, y) == x % y
    big = bytes(range(1, 33))
    assert M.bytes_mod(big, 1000) == int.from_bytes(big, "big") % 1000

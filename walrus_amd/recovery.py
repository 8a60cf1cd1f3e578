"""Recovery symbols with Merkle proofs, sliver recovery and inconsistency proofs.

Host-side mirror of the walrus-core types over the device engine (include/walrus_rs2.h):

  MerkleProof                  merkle.rs:100-185 (compute_root :150-169, verify_proof :78-99)
  RecoverySymbol               encoding/symbols.rs:587-651
  GeneralRecoverySymbol        encoding/symbols.rs:407-531
  InconsistencyProof           inconsistency.rs:107-190
  recovery_symbol_for_sliver   encoding/slivers.rs:180-213
  recover_sliver_or_generate_inconsistency_proof     encoding/slivers.rs:341-379
  try_recover_sliver_from_decoding_symbols           encoding/slivers.rs:303-327
  recovery_symbols_for_requests  the storage node's recovery-symbol service, batched
                                 (walrus-service/src/node/recovery_symbol_service.rs:161-235)

Every expansion, tree and proof root runs on the GPU (rs2_recovery_symbols,
rs2_merkle_proof_roots); only index bookkeeping is done here.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Iterable, List, Optional, Sequence

import numpy as np

from . import _lib
from .encoding import (PRIMARY, SECONDARY, _AXIS, _ORTHOGONAL, BlobMetadata, DecodingSymbol,
                       DecodingUnsuccessful, SliverData, Symbols, VerificationError, _ok)


# --------------------------------------------------------------------------------------------
# errors (merkle.rs MerkleProofError, symbols.rs SymbolVerificationError,
# inconsistency.rs InconsistencyVerificationError, slivers.rs SliverRecoveryError)
# --------------------------------------------------------------------------------------------
class MerkleProofError(Exception):
    """kind: 'LeafIndexOutOfBounds' | 'PathLengthTooLarge' | 'RootMismatch'"""

    def __init__(self, kind: str):
        super().__init__(kind)
        self.kind = kind


class SymbolVerificationError(Exception):
    """kind: 'IndexTooLarge' | 'SymbolSizeMismatch' | 'SymbolNotUsable' | 'InvalidMetadata'
    | 'InvalidProof'"""

    def __init__(self, kind: str):
        super().__init__(kind)
        self.kind = kind


class InconsistencyVerificationError(Exception):
    """kind: 'IncorrectSymbolCount' | 'InvalidRecoverySymbols' | 'RecoveryFailure'
    | 'SliverNotInconsistent' | 'SliverVerification'"""

    def __init__(self, kind: str, detail=None):
        super().__init__(kind if detail is None else f"{kind}{detail}")
        self.kind = kind
        self.detail = detail


class SliverRecoveryError(Exception):
    """slivers.rs SliverRecoveryError::DecodingFailure"""


class RecoverySymbolError(Exception):
    """slivers.rs RecoverySymbolError::IndexTooLarge (and encode errors)"""


def path_length(n_leaves: int) -> int:
    """merkle.rs path_length."""
    pl = ctypes.c_uint32()
    _ok(_lib.lib().rs2_merkle_tree_shape(n_leaves, ctypes.byref(pl), None))
    return pl.value


# --------------------------------------------------------------------------------------------
# Merkle proofs
# --------------------------------------------------------------------------------------------
@dataclass
class MerkleProof:
    """merkle.rs:100-185: the sibling hashes on the path from a leaf to the root."""
    path: List[bytes]

    def check_path_length(self, max_path_length: int) -> None:
        if len(self.path) > max_path_length:
            raise MerkleProofError("PathLengthTooLarge")

    def compute_root(self, leaf: bytes, leaf_index: int) -> bytes:
        return compute_roots([self], [leaf], [leaf_index])[0]

    def verify_proof(self, root: bytes, leaf_count: int, leaf: bytes, leaf_index: int) -> None:
        """MerkleAuth::verify_proof (merkle.rs:78-99)."""
        self.check_path_length(path_length(leaf_count))
        if self.compute_root(leaf, leaf_index) != bytes(root):
            raise MerkleProofError("RootMismatch")


def compute_roots(proofs: Sequence[MerkleProof], leaves: Sequence[bytes],
                  leaf_indices: Sequence[int]) -> List[bytes]:
    """MerkleProof::compute_root for many (proof, leaf, index) in one device call; proofs of one
    path length and leaves of one (even) length per call are batched together."""
    out: List[Optional[bytes]] = [None] * len(proofs)
    groups = {}
    for i, (p, leaf, li) in enumerate(zip(proofs, leaves, leaf_indices)):
        if li < 0 or li >> len(p.path):
            raise MerkleProofError("LeafIndexOutOfBounds")
        groups.setdefault((len(p.path), len(leaf)), []).append(i)
    for (plen, llen), members in groups.items():
        if llen % 2:
            raise ValueError("leaf length must be even")
        m = len(members)
        lv = np.frombuffer(b"".join(bytes(leaves[i]) for i in members) or b"\0\0", dtype=np.uint8)
        paths = np.frombuffer(b"".join(b"".join(proofs[i].path) for i in members) or b"\0" * 32,
                              dtype=np.uint8)
        idx = (ctypes.c_uint32 * m)(*[leaf_indices[i] for i in members])
        roots = np.zeros(32 * m, dtype=np.uint8)
        _ok(_lib.lib().rs2_merkle_proof_roots(m, lv.ctypes.data, llen, idx, paths.ctypes.data,
                                              plen, roots.ctypes.data))
        raw = roots.tobytes()
        for k, i in enumerate(members):
            out[i] = raw[32 * k:32 * k + 32]
    return out  # type: ignore[return-value]


# --------------------------------------------------------------------------------------------
# recovery symbols
# --------------------------------------------------------------------------------------------
def _sliver_hash(metadata: BlobMetadata, n_shards: int, index: int, axis: str) -> bytes:
    """BlobMetadata::get_sliver_hash of sliver `index` of `axis` (pair index via
    SliverIndex::to_pair_index, lib.rs:485-503)."""
    pair = index if axis == PRIMARY else n_shards - 1 - index
    h = metadata.hashes[pair]
    return h[0] if axis == PRIMARY else h[1]


@dataclass
class RecoverySymbol:
    """symbols.rs:587-651: a DecodingSymbol that recovers a sliver of `axis`, with the proof
    that it is symbol `target` of the expansion of source sliver `index` (orthogonal axis)."""
    axis: str
    index: int            # source sliver index (orthogonal axis)
    data: bytes
    proof: MerkleProof

    def __len__(self):
        return len(self.data)

    def verify_proof(self, root: bytes, total_leaf_count: int, target_index: int) -> None:
        self.proof.verify_proof(root, total_leaf_count, self.data, target_index)

    def verify(self, n_shards: int, expected_symbol_size: int, metadata: BlobMetadata,
               target_index: int) -> None:
        """RecoverySymbol::verify (symbols.rs:617-642)."""
        if self.index >= n_shards:
            raise SymbolVerificationError("IndexTooLarge")
        if len(self.data) != expected_symbol_size:
            raise SymbolVerificationError("SymbolSizeMismatch")
        root = _sliver_hash(metadata, n_shards, self.index, _ORTHOGONAL[self.axis])
        try:
            self.verify_proof(root, n_shards, target_index)
        except MerkleProofError as e:
            raise SymbolVerificationError("InvalidProof") from e

    def into_decoding_symbol(self) -> DecodingSymbol:
        return DecodingSymbol(self.index, self.data)


@dataclass
class GeneralRecoverySymbol:
    """symbols.rs:407-531: a recovery symbol usable for either sliver it lies on."""
    symbol: RecoverySymbol
    target_index: int

    def proof_axis(self) -> str:
        return _ORTHOGONAL[self.symbol.axis]

    def verify(self, metadata: BlobMetadata, config, target_index: int,
               target_type: str) -> None:
        n = config.n_shards
        sym = self.symbol
        if sym.index >= n or self.target_index >= n:
            raise SymbolVerificationError("IndexTooLarge")
        s = config.symbol_size_for_blob(metadata.unencoded_length)
        if len(sym.data) != s:
            raise SymbolVerificationError("SymbolSizeMismatch")
        source_type = _ORTHOGONAL[sym.axis]
        if not ((source_type != target_type and self.target_index == target_index)
                or sym.index == target_index):
            raise SymbolVerificationError("SymbolNotUsable")
        root = _sliver_hash(metadata, n, sym.index, source_type)
        try:
            sym.proof.verify_proof(root, n, sym.data, self.target_index)
        except MerkleProofError as e:
            raise SymbolVerificationError("InvalidProof") from e


def recovery_symbols_for_requests(config, slivers: Sequence[SliverData],
                                  target_pair_indices: Sequence[int]) -> List[RecoverySymbol]:
    """recovery_symbol_for_sliver (slivers.rs:180-213) for many (source sliver, target pair)
    requests: one device call per (axis, symbol size) group expands every source sliver,
    builds its Merkle tree and gathers the target symbol and its sibling path
    (rs2_recovery_symbols) -- what the node's recovery-symbol service computes per request on a
    CPU thread pool (recovery_symbol_service.rs:161-235)."""
    n = config.n_shards
    L = path_length(n)
    out: List[Optional[RecoverySymbol]] = [None] * len(slivers)
    groups = {}
    for i, (sl, tp) in enumerate(zip(slivers, target_pair_indices)):
        if tp >= n:
            raise RecoverySymbolError("IndexTooLarge")
        groups.setdefault((sl.axis, sl.symbol_size), []).append(i)
    for (axis, s), members in groups.items():
        orth = _ORTHOGONAL[axis]
        m = len(members)
        keep = [np.frombuffer(slivers[i].symbols.data, dtype=np.uint8) for i in members]
        ptrs = (ctypes.c_void_p * m)(*[a.ctypes.data for a in keep])
        lens = (ctypes.c_uint64 * m)(*[len(a) for a in keep])
        tgt = [target_pair_indices[i] if orth == PRIMARY else n - 1 - target_pair_indices[i]
               for i in members]
        ta = (ctypes.c_uint16 * m)(*tgt)
        syms = np.zeros(m * s, dtype=np.uint8)
        proofs = np.zeros(max(m * L * 32, 1), dtype=np.uint8)
        _ok(_lib.lib().rs2_recovery_symbols(n, s, _AXIS[axis], m, ptrs, lens, ta,
                                            syms.ctypes.data, proofs.ctypes.data),
            expected=len(keep[0]))
        sb, pb = syms.tobytes(), proofs.tobytes()
        for k, i in enumerate(members):
            path = [pb[(k * L + l) * 32:(k * L + l + 1) * 32] for l in range(L)]
            out[i] = RecoverySymbol(orth, slivers[i].index, sb[k * s:(k + 1) * s],
                                    MerkleProof(path))
    return out  # type: ignore[return-value]


def recovery_symbol_for_sliver(sliver: SliverData, target_pair_index: int,
                               config) -> RecoverySymbol:
    """SliverData::recovery_symbol_for_sliver (slivers.rs:180-213)."""
    return recovery_symbols_for_requests(config, [sliver], [target_pair_index])[0]


# --------------------------------------------------------------------------------------------
# recovery and inconsistency proofs
# --------------------------------------------------------------------------------------------
def _recover_without_verification(symbols: Sequence[DecodingSymbol], target_index: int,
                                  symbol_size: int, config, axis: str) -> SliverData:
    """slivers.rs:246-289: a too-short list fails before decoding (DecodingUnsuccessful)."""
    if len(symbols) < config.n_symbols_for_recovery(axis):
        raise DecodingUnsuccessful("not enough recovery symbols")
    data = config.decode_from_decoding_symbols(axis, symbol_size, symbols)
    return SliverData(Symbols(data, symbol_size), target_index, axis)


@dataclass
class InconsistencyProof:
    """inconsistency.rs:107-190: recovery symbols whose decoded sliver contradicts the
    metadata."""
    axis: str
    target_sliver_index: int
    recovery_symbols: List[RecoverySymbol] = field(default_factory=list)

    def verify(self, metadata: BlobMetadata, config) -> None:
        try:
            s = config.symbol_size_for_blob(metadata.unencoded_length)
        except Exception as e:
            raise InconsistencyVerificationError("RecoveryFailure") from e
        need = config.n_symbols_for_recovery(self.axis)
        if len(self.recovery_symbols) != need:
            raise InconsistencyVerificationError("IncorrectSymbolCount",
                                                 (need, len(self.recovery_symbols)))
        n = config.n_shards
        # every symbol's proof against the metadata, in one batched device call
        roots = compute_roots([r.proof for r in self.recovery_symbols],
                              [r.data for r in self.recovery_symbols],
                              [self.target_sliver_index] * need) \
            if all(len(r.data) == s and len(r.proof.path) <= path_length(n)
                   and r.index < n and self.target_sliver_index >> len(r.proof.path) == 0
                   for r in self.recovery_symbols) else None
        if roots is None or any(
                root != _sliver_hash(metadata, n, r.index, _ORTHOGONAL[self.axis])
                for root, r in zip(roots, self.recovery_symbols)):
            raise InconsistencyVerificationError("InvalidRecoverySymbols")
        try:
            sliver = _recover_without_verification(
                [r.into_decoding_symbol() for r in self.recovery_symbols],
                self.target_sliver_index, s, config, self.axis)
        except Exception as e:
            raise InconsistencyVerificationError("RecoveryFailure") from e
        try:
            sliver.verify(config, metadata)
        except VerificationError:
            return  # MerkleRootMismatch: the proof holds
        except ValueError as e:
            raise InconsistencyVerificationError("SliverVerification", str(e)) from e
        raise InconsistencyVerificationError("SliverNotInconsistent")


def recover_sliver_or_generate_inconsistency_proof(
        verified_recovery_symbols: Iterable[RecoverySymbol], target_index: int,
        metadata: BlobMetadata, config, axis: str = PRIMARY):
    """slivers.rs:341-379: the first n_symbols_for_recovery symbols are decoded into the target
    sliver; a sliver that verifies is returned, a Merkle-root mismatch yields an
    InconsistencyProof, any other failure raises."""
    s = config.symbol_size_for_blob(metadata.unencoded_length)
    need = config.n_symbols_for_recovery(axis)
    syms = []
    for r in verified_recovery_symbols:
        if len(syms) == need:
            break
        syms.append(r)
    try:
        sliver = _recover_without_verification([r.into_decoding_symbol() for r in syms],
                                               target_index, s, config, axis)
    except Exception as e:
        raise SliverRecoveryError("DecodingFailure") from e
    try:
        sliver.verify(config, metadata)
    except VerificationError:
        return InconsistencyProof(axis, target_index, syms)
    return sliver


def try_recover_sliver_from_decoding_symbols(decoding_symbols: Sequence[DecodingSymbol],
                                             target_index: int, metadata: BlobMetadata, config,
                                             axis: str = PRIMARY) -> SliverData:
    """slivers.rs:303-327: recover, then verify against the metadata (raises on either)."""
    s = config.symbol_size_for_blob(metadata.unencoded_length)
    try:
        sliver = _recover_without_verification(list(decoding_symbols), target_index, s, config,
                                               axis)
    except Exception as e:
        raise SliverRecoveryError("DecodingFailure") from e
    sliver.verify(config, metadata)
    return sliver

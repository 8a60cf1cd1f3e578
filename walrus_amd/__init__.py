"""walrus_amd: MI355X-native Red Stuff (RS2) erasure-coding engine for Walrus.

The hot path (2D sliver encode, Blake2b Merkle metadata, blob decode / sliver recovery) runs
as HIP kernels for gfx950 in libwalrus_rs2.so behind the C ABI of include/walrus_rs2.h.
`walrus_amd.encoding` mirrors the crates/walrus-core encoding API on top of it.
"""

from . import _lib
from . import mapping  # noqa: F401  (sliver pair <-> shard rotation)
from . import quilt  # noqa: F401  (QuiltV1 layout, index, encoder/decoder)
from . import recovery  # noqa: F401  (recovery symbols, Merkle proofs, inconsistency proofs)
from .encoding import (  # noqa: F401
    PRIMARY,
    SECONDARY,
    BlobId,
    BlobMetadata,
    DataTooLargeError,
    DecodeError,
    DecoderError,
    DecodingSymbol,
    DecodingUnsuccessful,
    DevicePlan,
    EncodeError,
    IncompatibleParameters,
    IncorrectDataLength,
    ReedSolomonDecoder,
    ReedSolomonEncoder,
    ReedSolomonEncodingConfig,
    SliverData,
    SliverPair,
    SliverVerifier,
    Symbols,
    VerificationError,
    VerifiedBlobMetadataWithId,
    compute_symbol_size,
    sliver_merkle_roots,
    source_symbols_for_n_shards,
    verify_slivers,
)

from .recovery import (  # noqa: F401
    GeneralRecoverySymbol,
    InconsistencyProof,
    MerkleProof,
    RecoverySymbol,
    recover_sliver_or_generate_inconsistency_proof,
    recovery_symbol_for_sliver,
    recovery_symbols_for_requests,
    try_recover_sliver_from_decoding_symbols,
)

build_library = _lib.build_library
device_available = _lib.device_available

__all__ = [n for n in dir() if not n.startswith("_")]

/*
 * walrus_rs2.h -- C ABI of the MI355X-native Red Stuff (RS2) engine.
 *
 * This is the drop-in boundary for the Red Stuff hot path of MystenLabs/walrus
 * (crates/walrus-core/src/encoding).  Every entry point below names the reference
 * interface it replaces (paths relative to the reference checkout).  The Rust side
 * would bind these through a thin `extern "C"` block; see INTEGRATION.md.
 *
 * Conventions
 *  - Plain pointers and sizes only.  No torch / HIP types in signatures; device
 *    streams are passed as an opaque `void*` (a hipStream_t).  For plans and verifiers
 *    NULL selects the object's own stream and RS2_STREAM_LEGACY the HIP null stream.  The
 *    codec / hashing primitives take the stream as given (NULL = null stream).
 *  - Caller-allocated outputs.  The engine never frees caller memory.
 *  - Every call is synchronous (blocks until the results are in the caller's buffers)
 *    unless its name ends in `_async`.  Calls are re-entrant: one plan per thread, or
 *    serialise use of a plan (the reference call sites are rayon / tokio blocking
 *    threads, walrus-sdk/src/node_client.rs:3182, walrus-service/src/node.rs:2615).
 *  - Return value: RS2_OK or a negative error code mapping 1:1 onto the reference
 *    error enums (encoding/errors.rs:34-66, encoding/basic_encoding.rs:148-150).
 *  - Byte layouts are exactly the reference's: a symbol is `symbol_size` bytes, a
 *    sliver is its symbols concatenated, slivers are indexed by sliver index (primary
 *    sliver i = row i of the expanded matrix, secondary sliver j = column j); sliver
 *    pair i = (primary i, secondary n-1-i) (lib.rs:485-491).
 *  - Metadata layout: `hashes` is n_shards x {primary_hash[32], secondary_hash[32]}
 *    ordered by sliver-pair index (metadata.rs:611-643); `blob_id` is 32 bytes
 *    (lib.rs:159-176).
 */
#ifndef WALRUS_RS2_H
#define WALRUS_RS2_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- error codes (encoding/errors.rs) --------------------------------------------------- */
#define RS2_OK 0
#define RS2_E_DATA_TOO_LARGE (-1)          /* DataTooLargeError / DecodeError::DataTooLarge     */
#define RS2_E_EMPTY_DATA (-2)              /* InvalidDataSizeError::EmptyData                    */
#define RS2_E_INCORRECT_DATA_LENGTH (-3)   /* EncodeError::IncorrectDataLength(expected)         */
#define RS2_E_INCOMPATIBLE_PARAMETERS (-4) /* EncodeError/DecodeError::IncompatibleParameters    */
#define RS2_E_NOT_ENOUGH_SHARDS (-5)       /* DecodeError::DecoderError(NotEnoughShards)         */
#define RS2_E_DECODING_UNSUCCESSFUL (-6)   /* DecodeError::DecodingUnsuccessful                  */
#define RS2_E_VERIFICATION (-7)            /* DecodeError::VerificationError                     */
#define RS2_E_INVALID_ARGUMENT (-8)        /* null pointer, index out of range (a panic in Rust) */
#define RS2_E_UNSUPPORTED (-9)             /* shape outside this build's kernels                 */
#define RS2_E_DEVICE (-10)                 /* HIP runtime failure / no GPU                       */
#define RS2_E_INTERNAL (-11)               /* an `expect` in the reference                        */

#define RS2_AXIS_PRIMARY 0   /* common.rs:11-25 Primary   */
#define RS2_AXIS_SECONDARY 1 /* common.rs:11-25 Secondary */

#define RS2_CHECK_SKIP 0    /* ConsistencyCheckType::Skip    (common.rs:47-56) */
#define RS2_CHECK_DEFAULT 1 /* ConsistencyCheckType::Default */
#define RS2_CHECK_STRICT 2  /* ConsistencyCheckType::Strict  */

/* Stream argument of the plan / verifier calls: NULL selects the object's own stream; this
 * value selects the HIP null stream (the legacy default stream, e.g. torch's default). */
#define RS2_STREAM_LEGACY ((void*)1)

#define RS2_DIGEST_LEN 32
#define RS2_ENCODING_TYPE_RS2 1

/* ---- parameters (pure functions, no device needed) -------------------------------------- */

/* ReedSolomonEncodingConfig::new -> (source_symbols_primary, source_symbols_secondary);
 * encoding/config.rs:446-460,717-725 and bft.rs:12-25. */
int rs2_source_symbols_for_n_shards(uint16_t n_shards, uint16_t* n_primary, uint16_t* n_secondary);

/* utils::compute_symbol_size (encoding/utils.rs:10-25) for the blob of `blob_len` bytes. */
int rs2_symbol_size_for_blob(uint16_t n_shards, uint64_t blob_len, uint16_t* symbol_size);

/* EncodingFactory::encoded_blob_length (config.rs:791-826): slivers + metadata bytes. */
int rs2_encoded_blob_length(uint16_t n_shards, uint64_t blob_len, uint64_t* encoded_len);

/* ---- device context ---------------------------------------------------------------------- */

/* Select the HIP device used by plans created afterwards on this thread (default 0). */
int rs2_set_device(int device);
/* Human-readable message for the last error on this thread (never NULL). */
const char* rs2_last_error(void);
/* 1 when the HIP engine is usable (a GPU is visible and the kernels load), else 0. */
int rs2_device_available(void);

/* Engine tuning (no reference counterpart): largest transform block a codec workgroup holds
 * on chip (a power of two <= 512, default 512 or $RS2_BLOCK_MAX).  Larger transforms are split
 * into blocks with block-level mixing; outputs are identical for every setting.  Applies to
 * plans created afterwards. */
int rs2_set_block_limit(uint32_t max_block);

/* ---- blob plans ---------------------------------------------------------------------------
 * A plan binds (n_shards, blob_len): it derives K_p, K_s and the symbol size
 * (BlobEncoder::new, blob_encoding.rs:239-264) and owns device scratch, constant
 * tables and a HIP stream.  Creating it returns RS2_E_DATA_TOO_LARGE like
 * BlobEncoder::new does.                                                                     */
typedef struct rs2_plan rs2_plan;

typedef struct rs2_plan_info {
  uint16_t n_shards;
  uint16_t n_primary;   /* K_p: rows of the message matrix, symbols per secondary sliver */
  uint16_t n_secondary; /* K_s: columns, symbols per primary sliver                      */
  uint16_t symbol_size;
  uint64_t blob_len;
  uint64_t primary_sliver_len;   /* K_s * symbol_size */
  uint64_t secondary_sliver_len; /* K_p * symbol_size */
} rs2_plan_info;

int rs2_plan_create(uint16_t n_shards, uint64_t blob_len, rs2_plan** out);
int rs2_plan_info_get(const rs2_plan* plan, rs2_plan_info* info);
/* Drains the plan's streams and returns its device buffers to the device's arena (below). */
void rs2_plan_destroy(rs2_plan* plan);

/* Re-points a plan at another blob length of the same symbol size (K_p, K_s, s unchanged):
 * its tables and buffers are kept, so one plan per (n_shards, symbol size) serves every blob
 * of that size class.  The reference builds a BlobEncoder / BlobDecoder per call
 * (config.rs:545-567, 591-603); a cache keyed by (n_shards, symbol_size) plus this call is
 * the bounded equivalent.  RS2_E_INCOMPATIBLE_PARAMETERS if the length needs another symbol
 * size, RS2_E_DATA_TOO_LARGE if it fits none.  Not concurrent with other calls on the plan.  */
int rs2_plan_rebind(rs2_plan* plan, uint64_t blob_len);

/* Device memory accounting.  Every device buffer of plans, codecs, verifiers and contexts is a
 * range of a per-device arena: a few large hipMalloc'd segments, best fit over coalesced free
 * ranges.  A segment is added only when nothing fits (max(request, reserve / 2, 256 MiB)), so
 * plan churn stops calling hipMalloc once the reserve covers its peak; RS2_ARENA_RESERVE_MIB
 * reserves a first segment up front (a fixed device-memory budget), RS2_ARENA_CACHE_MIB
 * (default 8192) caps the reserve kept when segments fall wholly free.  stats_out[7]:
 *   0 hipMalloc calls (segments)   1 hipFree calls   2 live bytes   3 reserved bytes
 *   4 peak live bytes   5 device synchronizes for quarantined ranges
 *   6 pinned host allocations (the host-buffer ABI's staging rings, pooled per device)      */
int rs2_device_memory_stats(int device, uint64_t* stats_out);

/* Counters of the small per-call uploads (a decode's position offsets and multiplier logs,
 * verifier targets, large codec jobs), which travel through a ring of pinned, device-mapped
 * slots and a copy kernel.  stats_out[3]:
 *   0 uploads through the slot ring   1 codec jobs through the job ring
 *   2 slot reuses that had to wait for the slot's previous copy (a completion word the copy
 *     kernel stores; no event and no device-wide synchronize is ever taken for a slot)
 * Device-wide synchronizes the engine takes are rs2_device_memory_stats slot 5.
 * No reference counterpart (the reference computes on the host).                            */
int rs2_upload_stats(uint64_t* stats_out);

/* Hand every wholly free arena segment of `device` back to hipFree (after a device synchronize
 * when ranges wait in quarantine), e.g. after a transient large blob, so the memory is the
 * process's other allocators' again (torch's caching allocator).  *released_bytes (may be
 * NULL) = the bytes returned.  No reference counterpart (the reference's buffers are Vec<u8>). */
int rs2_device_memory_trim(int device, uint64_t* released_bytes);

/* ---- 2D Red Stuff: host buffers ------------------------------------------------------------ */

/* Caller-owned host buffers registered with the engine (page-locked in place, hipHostRegister):
 * a host-buffer call's transfer whose host range lies wholly inside a registered range skips the
 * pinned staging ring and its host copies and moves by DMA straight between the caller's memory
 * and the device.  For callers that reuse long-lived buffers (a node's or publisher's sliver
 * and blob buffers); page-locking costs about as much as one staged transfer of the range, so
 * it does not pay for one-shot buffers.  The range must stay allocated, and no host-buffer call
 * may be using it, until rs2_host_unregister(ptr) with the same start.  Process-wide (every
 * device).  RS2_E_INVALID_ARGUMENT on an empty range, an overlap with a registered range or an
 * unregistered pointer.  Extension: the reference has no counterpart (its CPU path has no
 * staging). */
int rs2_host_register(void* ptr, uint64_t len);
int rs2_host_unregister(void* ptr);

/* BlobEncoder::encode_with_metadata (blob_encoding.rs:277-368) /
 * EncodingFactory::encode_with_metadata (config.rs:591-596).
 * primary_out[i]   : n_shards pointers, primary sliver i (K_s*s bytes) by sliver index
 * secondary_out[j] : n_shards pointers, secondary sliver j (K_p*s bytes) by sliver index
 * hashes_out       : n_shards*64 bytes (may be NULL), blob_id_out: 32 bytes (may be NULL).
 * primary_out / secondary_out (or single entries) may be NULL to skip those slivers.
 * Host buffers move through a per-plan pinned staging ring (host copies on worker threads
 * under the DMA); the primary slivers leave while the secondary codecs and hashing run. */
int rs2_encode_with_metadata(rs2_plan* plan, const uint8_t* blob, uint8_t* const* primary_out,
                             uint8_t* const* secondary_out, uint8_t* hashes_out,
                             uint8_t* blob_id_out);

/* BlobEncoder::compute_metadata (blob_encoding.rs:406-486) / config.rs:598-603. */
int rs2_compute_metadata(rs2_plan* plan, const uint8_t* blob, uint8_t* hashes_out,
                         uint8_t* blob_id_out);

/* ---- blob batches ---------------------------------------------------------------------------
 * Many blobs of the plan's symbol size encoded together (the upload relay's server-side encode,
 * walrus-upload-relay/src/controller.rs:177, and the client's per-blob encode loop
 * encode_blobs_as, walrus-sdk/src/node_client.rs:3156-3221, each blob a
 * BlobEncoder::encode_with_metadata, blob_encoding.rs:277-368): every stage is one launch over
 * the whole batch.  Blob b has blob_lens[b] bytes (blob_lens NULL = the plan's blob_len for
 * every blob); each length must give the plan's symbol size (rs2_symbol_size_for_blob), else
 * RS2_E_INVALID_ARGUMENT.  At most 65535 blobs.
 *
 * Device form: blob b at d_blobs + b*blob_stride; its slivers in the single-blob layouts at
 * d_primary + b*primary_stride (>= n*primary_sliver_len) and d_secondary + b*secondary_stride;
 * its n pair hashes at d_hashes + b*64*n, its BlobId at d_blob_ids + b*32.  Same stream rules
 * as rs2_encode_device_async. */
int rs2_encode_batch_device_async(rs2_plan* plan, uint32_t n_blobs, const void* d_blobs,
                                  uint64_t blob_stride, const uint64_t* blob_lens, void* d_primary,
                                  uint64_t primary_stride, void* d_secondary,
                                  uint64_t secondary_stride, void* d_hashes, void* d_blob_ids,
                                  void* stream);
/* Host form: blobs[b] (blob_lens[b] bytes); primary_out / secondary_out hold n_blobs*n sliver
 * pointers, blob-major (either array, or any entry, may be NULL: not returned); hashes_out
 * n_blobs*n*64 bytes and blob_ids_out n_blobs*32 bytes (either may be NULL).  Blocking. */
int rs2_encode_batch_with_metadata(rs2_plan* plan, uint32_t n_blobs, const uint8_t* const* blobs,
                                   const uint64_t* blob_lens, uint8_t* const* primary_out,
                                   uint8_t* const* secondary_out, uint8_t* hashes_out,
                                   uint8_t* blob_ids_out);

/* BlobDecoder::decode (blob_encoding.rs:888-993) / EncodingFactory::decode (config.rs:605-611).
 * `count` slivers of axis `axis`, sliver i at slivers[i] with index sliver_idx[i], length
 * sliver_len[i] bytes and symbol size sliver_symbol_size[i] (NULL: all equal to the plan's).
 * As check_and_write_slivers_to_workspace (blob_encoding.rs:904-951): a repeated index is
 * skipped, a sliver of the wrong length or symbol size dropped, the surplus beyond K
 * dropped; too few -> RS2_E_DECODING_UNSUCCESSFUL.  An index >= n_shards is taken like the
 * reference takes it and then fails the column decodes -> RS2_E_NOT_ENOUGH_SHARDS
 * (DecodeError::DecoderError).  blob_out: blob_len bytes. */
int rs2_decode_blob(rs2_plan* plan, int axis, uint32_t count, const uint16_t* sliver_idx,
                    const uint8_t* const* slivers, const uint64_t* sliver_len,
                    const uint16_t* sliver_symbol_size, uint8_t* blob_out);

/* EncodingFactory::decode_and_verify (config.rs:613-658).  `hashes` / `blob_id` are the
 * metadata being verified against (n_shards*64 and 32 bytes).
 *   RS2_CHECK_DEFAULT: BlobEncoder::default_consistency_check (blob_encoding.rs:579-612) --
 *     with primary slivers, every systematic index (< K_p) the decoder pulled from the input
 *     counts as already verified (config.rs:621-640) and only the other systematic primary
 *     slivers are re-encoded and Merkle-checked (on the device); with secondary slivers all
 *     K_p are checked.
 *   RS2_CHECK_STRICT: the decoded blob's metadata is re-derived and its blob id compared
 *     (config.rs:164-172).
 * A failed check -> RS2_E_VERIFICATION (blob_out then unspecified). */
int rs2_decode_and_verify(rs2_plan* plan, int axis, uint32_t count, const uint16_t* sliver_idx,
                          const uint8_t* const* slivers, const uint64_t* sliver_len,
                          const uint16_t* sliver_symbol_size, const uint8_t* hashes,
                          const uint8_t* blob_id, int consistency_check, uint8_t* blob_out);

/* ---- 2D Red Stuff: device-resident (the measured path) ----------------------------------------
 * Same semantics with device buffers: d_blob (blob_len bytes); d_primary n*K_s*s bytes
 * (primary sliver i at i*K_s*s); d_secondary n*K_p*s bytes (secondary sliver j at j*K_p*s);
 * d_hashes n*64; d_blob_id 32.  Work is enqueued on `stream` (hipStream_t, NULL = the
 * plan's stream); the call returns after enqueueing.                                          */
int rs2_encode_device_async(rs2_plan* plan, const void* d_blob, void* d_primary, void* d_secondary,
                            void* d_hashes, void* d_blob_id, void* stream);

/* BlobEncoder::compute_metadata (blob_encoding.rs:406-486) on a device-resident blob: every
 * symbol is expanded and hashed, only d_hashes (n*64) and d_blob_id (32) are written (the
 * slivers go to the plan's own scratch).  The upload relay's call (walrus-upload-relay/src/
 * controller.rs:177) when the blob is already in HBM. */
int rs2_compute_metadata_device_async(rs2_plan* plan, const void* d_blob, void* d_hashes,
                                      void* d_blob_id, void* stream);

/* rs2_encode_device_async with an early hand-off of the primary slivers: `primary_stream`
 * (non-NULL, not `stream`) is made to wait only until every primary sliver is written, so
 * work queued on it next (a decode from primary slivers, their D2H to the storage backend)
 * runs beside the secondary codecs and the hashing still in flight on `stream`.  Outputs are
 * identical to rs2_encode_device_async.  The caller must order `stream` after its
 * primary_stream work before the next encode rewrites those buffers.  No reference
 * counterpart: the reference returns all slivers at once (blob_encoding.rs:277-368). */
int rs2_encode_device_split_async(rs2_plan* plan, const void* d_blob, void* d_primary,
                                  void* d_secondary, void* d_hashes, void* d_blob_id, void* stream,
                                  void* primary_stream);

/* Decode from `count` device slivers of `axis`: sliver i lives at d_slivers_base +
 * sliver_off[i] (bytes) and has index sliver_idx[i].  Host-side validation as in
 * rs2_decode_blob (all given slivers must have the correct length).  d_blob_out:
 * blob_len bytes. */
int rs2_decode_device_async(rs2_plan* plan, int axis, uint32_t count, const uint16_t* sliver_idx,
                            const void* d_slivers_base, const uint64_t* sliver_off,
                            void* d_blob_out, void* stream);

/* EncodingFactory::decode_and_verify (config.rs:613-658) on device-resident slivers (as
 * rs2_decode_device_async) into the device buffer d_blob_out (blob_len bytes); `hashes` /
 * `blob_id` are host copies of the metadata.  The checks are those of rs2_decode_and_verify and
 * run on the device; the call returns once the verdict is known (RS2_E_VERIFICATION on a
 * failed check). */
int rs2_decode_and_verify_device(rs2_plan* plan, int axis, uint32_t count,
                                 const uint16_t* sliver_idx, const void* d_slivers_base,
                                 const uint64_t* sliver_off, const uint8_t* hashes,
                                 const uint8_t* blob_id, int consistency_check, void* d_blob_out,
                                 void* stream);

/* Wait for the plan's outstanding work on `stream` (NULL = plan stream). */
int rs2_sync(rs2_plan* plan, void* stream);

/* Stage profiler (no reference counterpart; the reference uses tracing spans,
 * blob_encoding.rs:261).  When enabled, the plan records a HIP event between consecutive
 * kernel launches on the stream; rs2_profile_read synchronises, returns per-stage totals
 * (names: 32-byte NUL-padded slots) and resets the totals. */
int rs2_profile_enable(rs2_plan* plan, int enable);
int rs2_profile_read(rs2_plan* plan, uint32_t max_stages, char* names, double* total_ms,
                     uint32_t* launches, uint32_t* n_stages);

/* ---- 1D codec (basic_encoding.rs) and sliver helpers ------------------------------------------ */

/* ReedSolomonEncoder::encode_all (basic_encoding.rs:195-211): `k*symbol_size` bytes of data ->
 * all n_shards symbols (source || repair), n_shards*symbol_size bytes.  `batch` independent
 * codewords laid out back to back (data stride k*s, output stride n*s). */
int rs2_encode_1d(uint16_t k, uint16_t n_shards, uint16_t symbol_size, uint32_t batch,
                  const uint8_t* data, uint8_t* out_all);

/* ReedSolomonDecoder::decode (basic_encoding.rs:387-429): `count` symbols with indices idx[]
 * (index < k: source symbol, else repair symbol index-k) -> the k source symbols.
 * Wrong-size symbols cannot occur at this ABI (fixed symbol_size); duplicates are ignored;
 * fewer than k distinct -> RS2_E_NOT_ENOUGH_SHARDS. */
int rs2_decode_1d(uint16_t k, uint16_t n_shards, uint16_t symbol_size, uint32_t count,
                  const uint16_t* idx, const uint8_t* const* symbols, uint8_t* out_source);

/* SliverData::get_merkle_root (slivers.rs:387-392): expand a sliver of `axis` on the
 * orthogonal axis and return the Merkle root over the n_shards symbols (the value
 * SliverData::verify / check_hash compares with the metadata, slivers.rs:100-135). */
int rs2_sliver_merkle_root(uint16_t n_shards, uint16_t symbol_size, int axis,
                           const uint8_t* sliver, uint64_t sliver_len, uint8_t root_out[32]);

/* Batched form of the above for `count` slivers of one axis and symbol size (the storage
 * node's verify_sliver_against_metadata, walrus-service/src/node.rs:2615-2633, and the
 * recovery-symbol service's per-sliver Merkle trees, node/recovery_symbol_service.rs:132-159).
 * A sliver of the wrong length -> RS2_E_INCORRECT_DATA_LENGTH.  roots_out: count*32 bytes. */
int rs2_sliver_merkle_roots(uint16_t n_shards, uint16_t symbol_size, int axis, uint32_t count,
                            const uint8_t* const* slivers, const uint64_t* sliver_len,
                            uint8_t* roots_out);

/* Device-resident batched sliver verification: a verifier binds (n_shards, symbol_size,
 * axis) and owns scratch + a stream; d_slivers holds `count` slivers back to back
 * (K*symbol_size bytes each, K = source symbols of the orthogonal axis' code), d_roots
 * receives count*32 bytes.  Same stream conventions as the plan API. */
typedef struct rs2_verifier rs2_verifier;
int rs2_verifier_create(uint16_t n_shards, uint16_t symbol_size, int axis, rs2_verifier** out);
int rs2_verifier_roots_device_async(rs2_verifier* v, uint32_t count, const void* d_slivers,
                                    void* d_roots, void* stream);
void rs2_verifier_destroy(rs2_verifier* v);

/* ---- recovery symbols with Merkle proofs ------------------------------------------------------
 * SliverData::recovery_symbol_for_sliver (slivers.rs:180-213), batched as the storage node's
 * recovery-symbol service runs it (walrus-service/src/node/recovery_symbol_service.rs:161-235):
 * request i expands source sliver i (of `axis`) on the orthogonal axis to n_shards symbols,
 * builds the MerkleTree over them (merkle.rs:216-266) and returns
 *   symbols_out + i*symbol_size : expanded symbol target_sliver_index[i] (the recovery symbol's
 *                                 data; its DecodingSymbol index is the source sliver's index)
 *   proofs_out + i*path_len*32  : MerkleTree::get_proof(target) (merkle.rs:281-309), the sibling
 *                                 path leaf -> root, path_len = rs2_merkle_tree_shape(n_shards).
 * target_sliver_index[i] is the index on the orthogonal axis (SliverPairIndex::to_sliver_index,
 * lib.rs:485-491); >= n_shards -> RS2_E_INVALID_ARGUMENT (RecoverySymbolError::IndexTooLarge).
 * A sliver of the wrong length -> RS2_E_INCORRECT_DATA_LENGTH. */
int rs2_recovery_symbols(uint16_t n_shards, uint16_t symbol_size, int axis, uint32_t count,
                         const uint8_t* const* slivers, const uint64_t* sliver_len,
                         const uint16_t* target_sliver_index, uint8_t* symbols_out,
                         uint8_t* proofs_out);

/* Device form on a verifier (slivers back to back as for rs2_verifier_roots_device_async;
 * target_sliver_index is a HOST array of `count` entries).  d_nodes (may be NULL) receives each
 * tree's full node array (count * n_nodes * 32 bytes, MerkleTree::nodes order: levels from the
 * leaves, each padded to even with the zero node, root last) -- what the service caches per
 * (blob, source sliver) (recovery_symbol_service.rs:132-159). */
int rs2_verifier_recovery_symbols_device_async(rs2_verifier* v, uint32_t count,
                                               const void* d_slivers,
                                               const uint16_t* target_sliver_index,
                                               void* d_symbols, void* d_proofs, void* d_nodes,
                                               void* stream);

/* Path length (merkle.rs path_length) and node count (n_nodes) of a tree over n_leaves. */
int rs2_merkle_tree_shape(uint32_t n_leaves, uint32_t* path_len, uint64_t* n_nodes);

/* MerkleProof::compute_root (merkle.rs:150-169) for `count` proofs, on the device: leaf r is
 * leaf_len bytes (even) at leaves + r*leaf_len (leaf_hash'ed, merkle.rs:313-321), its index
 * leaf_index[r], its path path_len nodes at paths + r*path_len*32.  roots_out: count*32.  The
 * checks of MerkleAuth::verify_proof (path length, index bound, merkle.rs:78-99,150-156) are the
 * caller's (they need no data). */
int rs2_merkle_proof_roots(uint32_t count, const uint8_t* leaves, uint32_t leaf_len,
                           const uint32_t* leaf_index, const uint8_t* paths, uint32_t path_len,
                           uint8_t* roots_out);

/* ---- device 1D codec over strided lines (partitioned 2D code, batched recovery) --------------
 * A codec binds one 1D Reed-Solomon code (k source symbols -> n_shards, symbol_size bytes):
 * the device form of ReedSolomonEncoder / ReedSolomonDecoder (basic_encoding.rs:107-429)
 * applied to `lines` independent codewords per call.  Codeword `l`'s source symbol i lives at
 * d_src + l*src_line_stride + i*src_sym_stride; repair symbol j (shard index k+j) is written
 * to d_repair + l*repair_line_stride + j*repair_sym_stride.  This is what the reference runs
 * once per row / column inside BlobEncoder (blob_encoding.rs:309-354) and once per sliver in
 * SliverData::recovery_symbols (slivers.rs:100-118); the multi-GPU partitioned encode calls it
 * on a rank's row / column range.  Same stream conventions as the plan API (NULL = default
 * stream); one codec per thread, or serialise its use. */
typedef struct rs2_codec rs2_codec;
int rs2_codec_create(uint16_t k, uint16_t n_shards, uint16_t symbol_size, rs2_codec** out);
void rs2_codec_destroy(rs2_codec* codec);
int rs2_codec_encode_device_async(rs2_codec* codec, uint32_t lines, const void* d_src,
                                  uint64_t src_sym_stride, uint64_t src_line_stride,
                                  void* d_repair, uint64_t repair_sym_stride,
                                  uint64_t repair_line_stride, void* stream);

/* ReedSolomonDecoder::decode (basic_encoding.rs:387-429) for `lines` codewords sharing one
 * erasure pattern: `count` shard indices idx[] (index < k: source symbol, else repair index-k;
 * duplicates and indices >= n_shards ignored, the first k distinct used), shard idx[i] of line
 * l at d_base + sym_off[i] + l*line_stride.  All k source symbols of line l are written to
 * d_out + l*out_line_stride + i*out_sym_stride (present ones copied, missing ones decoded);
 * bytes at offsets >= out_limit (relative to d_out) are not written (the BlobDecoder's
 * truncation to the blob length, blob_encoding.rs:970-993).  Fewer than k distinct shards ->
 * RS2_E_NOT_ENOUGH_SHARDS.  Column-partitioned multi-GPU decode runs it on a rank's columns. */
int rs2_codec_decode_device_async(rs2_codec* codec, uint32_t lines, uint32_t count,
                                  const uint16_t* idx, const void* d_base, const uint64_t* sym_off,
                                  uint64_t line_stride, void* d_out, uint64_t out_sym_stride,
                                  uint64_t out_line_stride, uint64_t out_limit, void* stream);

/* Segment copies: the exchange packing of the partitioned encode / decode (walrus_amd/
 * partition.py), i.e. the row -> column transposition of blob_encoding.rs:309-324 split by
 * rank.  Segment (a, b), a < count_a, b < count_b, is seg_len bytes from
 * d_src + d_src_a[a] + b*src_b_stride to d_dst + d_dst_a[a] + b*dst_b_stride; d_src_a / d_dst_a
 * are device arrays of count_a int64 byte offsets.  `unit` (1, 2, 4, 8 or 16) is the copy
 * width: seg_len, the strides and the bases must be multiples of it, else
 * RS2_E_INVALID_ARGUMENT.  Every offset in d_src_a / d_dst_a must be a multiple of it too:
 * those live in device memory and are NOT checked (an unaligned one makes misaligned wide
 * accesses -- a fault or wrong bytes); walrus_amd/partition.py passes the gcd of each table.
 * Segments must not overlap their sources. */
int rs2_copy_segments_device_async(const void* d_src, void* d_dst, uint32_t count_a,
                                   const int64_t* d_src_a, const int64_t* d_dst_a, uint32_t count_b,
                                   int64_t src_b_stride, int64_t dst_b_stride, uint32_t seg_len,
                                   uint32_t unit, void* stream);

/* leaf_hash (merkle.rs:313-321) of `count` contiguous symbols of symbol_size bytes ->
 * count*32 bytes of digests (blob_encoding.rs:161-196 hashes every expanded symbol). */
int rs2_leaf_hashes_device_async(const void* d_symbols, uint64_t count, uint16_t symbol_size,
                                 void* d_leaves, void* stream);

/* MerkleTree::build_from_leaf_hashes(..).root() (merkle.rs:216-266, inner_hash :323-332) of
 * `n_trees` trees of `n_leaves` (1..65535; above 4,096 through a device scratch buffer) leaf
 * digests: leaf i of tree t at d_leaves + t*tree_stride + i*leaf_stride (strides multiples of
 * 16), root t written to d_roots + t*root_stride. */
int rs2_merkle_roots_device_async(const void* d_leaves, uint32_t n_trees, uint32_t n_leaves,
                                  uint64_t tree_stride, uint64_t leaf_stride, void* d_roots,
                                  uint64_t root_stride, void* stream);

/* Device form of rs2_blob_id_from_hashes (metadata.rs:571-578, lib.rs:159-176). */
int rs2_blob_id_device_async(const void* d_hashes, uint16_t n_shards, uint64_t blob_len,
                             void* d_blob_id, void* stream);

/* MerkleTree::build(..).root() over `n_leaves` leaves of `leaf_len` bytes each
 * (merkle.rs:216-266, leaf_hash :313-321, inner_hash :323-332).  Hashed on the device. */
int rs2_merkle_root(const uint8_t* leaves, uint32_t n_leaves, uint32_t leaf_len,
                    uint8_t root_out[32]);

/* BlobId::from_sliver_pair_metadata (lib.rs:147-157 via metadata.rs:571-578).  Hashed on the
 * device. */
int rs2_blob_id_from_hashes(const uint8_t* hashes, uint16_t n_shards, uint64_t blob_len,
                            uint8_t blob_id_out[32]);

/* QuiltEncoderV1::construct_quilt's column fill (quilt_encoding.rs:1447-1528, 1530-1646) on the
 * device: the quilt is n_rows x n_cols symbols of symbol_size bytes, row-major, and column c
 * holds bytes [0, d_col_len[c]) of the payload starting at d_payload + d_col_off[c], laid
 * down symbol by symbol from row 0 (the rest of the column is zero).  Each blob's serialized
 * bytes (header, identifier, tags, data) fill whole consecutive columns: column j of a blob
 * starting at payload offset P is d_col_off = P + j*n_rows*symbol_size.  Offsets even,
 * d_col_len[c] <= n_rows*symbol_size; d_quilt: n_rows*n_cols*symbol_size bytes, 16-byte
 * aligned.  The column
 * tables (int64 / uint32, n_cols entries) are device arrays built by the host layout plan. */
int rs2_quilt_layout_device_async(uint16_t n_rows, uint16_t n_cols, uint16_t symbol_size,
                                  const void* d_payload, const int64_t* d_col_off,
                                  const uint32_t* d_col_len, void* d_quilt, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* WALRUS_RS2_H */

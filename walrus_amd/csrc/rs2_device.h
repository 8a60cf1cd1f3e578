// Device-side job descriptors shared by the HIP kernels (rs2_kernels.hip) and the host
// planner (rs2_engine.cpp).  Plain structs, no HIP types, so both sides agree on layout.
#pragma once
#include <stdint.h>

namespace rs2 {

constexpr int kMaxBlocks = 64;  // input / output blocks of a job passed by value (W <= 32768)
// Jobs with more blocks (n_shards above about 24,580: W = 65536 = 128 blocks of 512) live in
// device memory and reach the kernel by pointer (CodecJobBig, C = 512 only); their block arrays
// and mixing kinds would not fit the kernel argument.
constexpr int kMaxBlocksBig = 128;
constexpr int kMaxC = 512;      // largest transform block held on chip (positions)
constexpr int kTabU16 = 128;    // one multiplier table: u16 sub-tables of 64 + 32 + 32 entries
                                // for operand bits 0-5, 6-10, 11-15 (rs2_engine.cpp nib_table)
// Codeword positions one wave holds in VGPRs; a size-C transform uses C / PPW waves.  The
// kernel's table consumption order and the host's sd_stream order both derive from it.
constexpr int kPpwTarget = 32;

// One input block of a codec job: up to C codeword positions, loaded from symbols in HBM,
// optionally pre-multiplied per position, then inverse-transformed (IFFT) with skew offset
// `sd` (the tables in `sd_tab` are that transform's constants in consumption order).
struct InBlock {
  const uint8_t* base;       // symbol (pos, line) lives at base + pos_off[pos] + line*line_stride
  const int64_t* pos_off;    // [C]; -1 = position absent (zero)
  const uint16_t* pre_tab;   // [C][64] per-position multiplier tables, or null
  const uint16_t* sd_tab;    // [C-1][64] IFFT constant tables
  int64_t line_stride;
  // fused copy-out of the loaded symbols (systematic secondary slivers on encode, present
  // originals on decode): symbol (pos, line) -> copy_base + copy_off[pos] + line*copy_stride,
  // bytes at offset >= copy_limit not written.  copy_off null = no copy.
  uint8_t* copy_base;
  const int64_t* copy_off;   // [C]; -1 = not copied
  int64_t copy_line_stride;
  int64_t copy_limit;
  int32_t count;             // positions >= count are zero
  int32_t zero_first;        // 1: group 0 of every cross-wave layer multiplies by zero (sd = 0)
  // split input: positions >= alt_from read from alt_base instead of base (same offsets); the
  // encode reads the blob's whole rows in place and its zero-padded last row from a small
  // buffer.  alt_base null = unused.
  const uint8_t* alt_base;
  int32_t alt_from;
  // second fused copy-out at the input's own layout: symbol (pos, line) is also written to
  // copy2_base + pos_off[pos] + line*line_stride (the encode's systematic primary slivers, so
  // no separate blob copy).  Null = none.
  uint8_t* copy2_base;
};

// codec kernel variants (one __global__ each, so profiles attribute time per stage)
// kModeColsPipe / kModeRowsPipe: the shared-input / mixing encode as a persistent,
// tile-pipelined kernel (launch_codec_c picks them when the last output block's active waves fit
// below the head input block's); kModeDecodePersist: the decode with one persistent workgroup
// per CU walking an XCD-interleaved tile range (CodecJob::n_tiles tiles)
enum CodecMode : int {
  kModeRows = 0, kModeCols = 1, kModeDecode = 2, kModeColsPipe = 3, kModeRowsPipe = 4,
  kModeDecodePersist = 5
};

// One output block: FFT with skew offset `sd`, optional per-position post-multiply,
// store of positions < trunc whose pos_off >= 0; bytes at offset >= limit are not stored.
struct OutBlock {
  uint8_t* base;
  const int64_t* pos_off;
  const uint16_t* post_tab;
  const uint16_t* sd_tab;
  int64_t line_stride;
  int64_t limit;
  int32_t trunc;
  int32_t zero_first;        // as InBlock::zero_first
};

// The scalar fields of a codec job (CodecJobT below derives from it, so they are read as
// job.n_in etc.).  Kept in a base of their own so that narrowing a planned CodecJobBig to the
// by-value CodecJob (rs2_engine.cpp narrow_job) copies them all at once: a field added here can
// not be left at its default in the kernel argument.
struct CodecScalars {
  const uint16_t* mix_tab;
  int32_t n_in;
  int32_t n_out;
  int32_t symbol_size;
  int32_t n_pairs;           // element pairs per symbol = ceil(symbol_size / 4)
  int32_t shared_in;         // 1: single input, every output = FFT_o(X_0) (low-rate encode)
  int32_t line_base;         // line of blockIdx.y == 0 (launches are split at 65535 lines)
  // decode: the pre-multiplier tables of output block z start at in[b].pre_tab + z * pre_z_stride
  // (u16 elements), because each output folds its own mixing coefficient into them
  int64_t pre_z_stride;
  // lanes walk a flattened (line, pair) space: pairs_span (even, >= n_pairs) pairs per line,
  // n_lines lines from line_base (set per launch)
  int32_t pairs_span;
  int32_t n_lines;
  // diagnostics (RS2_STAMP_FILE): wave 0 of every workgroup records s_memtime at its phase
  // boundaries into stamps[blockIdx.x * kStamps + k]; null = off
  uint64_t* stamps;
  // blob batches (rs2_encode_batch_*): tile t (after the XCD order) belongs to blob
  // t / tiles_per_blob, whose symbols lie in_blob_stride / out_blob_stride / copy_blob_stride
  // bytes past blob 0's for every input / output / copy base; tiles_per_blob 0 = one blob
  int32_t tiles_per_blob;
  int64_t in_blob_stride, out_blob_stride, copy_blob_stride;
  // pipelined kernels: tiles of the whole launch (gridDim.x workgroups each walk a contiguous
  // range); kModeRowsPipe: the input block loaded beside the previous tile's tail
  int32_t n_tiles;
  int32_t pipe_head;
  // pipelined kernels, dynamic tile order (null = static XCD-interleaved ranges): kTileCtrWords
  // zeroed words of device memory; word x < 8 counts the tiles taken from XCD x's contiguous
  // range, word 8 the workgroups that have finished (the last one zeroes them all again, so the
  // next launch on the same words starts from zero).  A workgroup takes its XCD's next tile,
  // then the other XCDs' leftovers, so a workgroup that got its CU late (another kernel held
  // it) takes fewer tiles instead of finishing its fixed range late.
  uint32_t* tile_ctr;
};

// out_o = FFT_o( sum_b  M1[o][b] * Dw(X_b)  +  M2[o][b] * X_b ),  X_b = IFFT_b(in_b)
// where Dw is the in-block formal derivative.  Coefficient kinds: 0 zero, 1 one, 2 table
// (mix_tab + ((o*MB + b)*2 + {0:M1, 1:M2}) * 64).  MB = kMaxBlocks (CodecJob, the kernel
// argument) or kMaxBlocksBig (CodecJobBig, by pointer); the host plans in CodecJobBig and
// narrows jobs of <= kMaxBlocks blocks to CodecJob at launch.  Every per-block array is listed
// in kArrayBytes, so a new array field that narrow_job does not copy breaks the build.
template <int MB>
struct CodecJobT : CodecScalars {
  static constexpr int kBlocks = MB;
  InBlock in[MB];
  OutBlock out[MB];
  uint8_t m1_kind[MB][MB];
  uint8_t m2_kind[MB][MB];
  // decode, output block z: two input blocks whose active waves fit one workgroup together are
  // loaded and run their in-wave IFFT layers side by side (rs2_codec.hip load_ifft): block
  // pair_p[z] on waves [0, pair_nw[z]), block pair_q[z] (no formal derivative) on the rest.
  // pair_q is always the last input block; pair_nw 0 = no pair.
  int8_t pair_p[MB], pair_q[MB], pair_nw[MB];
  static constexpr size_t kArrayBytes =
      MB * (sizeof(InBlock) + sizeof(OutBlock)) + 2 * MB * MB + 3 * MB;
};
using CodecJob = CodecJobT<kMaxBlocks>;
using CodecJobBig = CodecJobT<kMaxBlocksBig>;
static_assert(sizeof(CodecJob) ==
                  (sizeof(CodecScalars) + CodecJob::kArrayBytes + 7) / 8 * 8 &&
              sizeof(CodecJobBig) ==
                  (sizeof(CodecScalars) + CodecJobBig::kArrayBytes + 7) / 8 * 8,
              "a CodecJobT field outside CodecScalars and kArrayBytes: narrow_job would drop it");
constexpr int kTileCtrWords = 16;
constexpr int kStamps = 64;
// CodecJob travels by value as the codec kernels' argument.  tools/micro/kernarg20.hip probed a
// 20 KiB by-value argument on the box (gfx950, ROCm 7.2); keep the job (plus the few hidden
// arguments) below that instead of relying on an untested larger limit.
static_assert(sizeof(CodecJob) <= 19 * 1024 + 512, "CodecJob outgrows the probed kernel-argument size");

// Where the n x n expanded-matrix symbol (r, c) lives after an encode (leaf hashing).
struct SymbolMap {
  const uint8_t* primary;    // [n][K_s][s]  rows, columns < K_s
  const uint8_t* secondary;  // [n][K_p][s]  columns >= K_s hold rows < K_p
  const uint8_t* both;       // [n-K_p][n-K_s][s]  rows >= K_p, columns >= K_s
  int32_t n, kp, ks, s;
  // blob batches: blob y (grid.y) at these byte offsets from blob 0 (leaves: out + y*leaf_stride)
  int64_t primary_stride, secondary_stride, both_stride, leaf_stride;
};

}  // namespace rs2

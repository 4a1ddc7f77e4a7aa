// kernels.h — device-kernel interface shared by the kernels (conv_kernels.hip)
// and the host orchestration (hifigan_capi.cpp).  No torch types anywhere.
#pragma once

#include <hip/hip_runtime.h>

#include <mutex>
#include <stdint.h>

namespace hfg {

// One-time launch setup of a kernel entry, safe across threads and devices:
// the dynamic-LDS limit is a per-device function attribute, so it is set once per
// (kernel, device) under a lock; entry names are formatted under the same lock.
hipError_t ensure_max_lds(const void* fn);
std::mutex& setup_mutex();

constexpr float kLReluSlope = 0.1f;  // F.leaky_relu(x, 0.1), models/hifigan.py:81,83,244,254

// split formats of the split-precision kernels (bf16x3_common.h): bf16 halves (bf16x3) or
// power-of-two-scaled f16 halves (f16x3; scale exponents clamped to +-kX3ExpMax)
constexpr int kFmtBf16 = 0;
constexpr int kFmtF16 = 1;
constexpr int kX3ExpMax = 60;
// (producer launch, batch item) scale slot: waves fold their max into one of kAmaxSpread
// words, each on its own 128-B line (kAmaxLineWords apart); consumers take the max of all.
// Device-scope atomics on one line serialise at ~4.7 ns each on MI355X whatever the word
// (tests/tools/atomic_probe.hip: 8192 waves into one line 40 us, into 64 lines 3 us), so the
// round-5 layout (64 words on 2 lines) put a whole single-round grid's commits in a queue.
constexpr int kAmaxSpread = 16;
constexpr int kAmaxLineWords = 32;
constexpr int kAmaxSlotWords = kAmaxSpread * kAmaxLineWords;

// One implicit-GEMM convolution launch:
//   out[b][m][n] = bias[m] + sum_{ci, j} Wt[m][ci][j] * act_in(x[b][ci][n + off + j*dil])
// with x zero outside [0, L_in).  Regular Conv1d: m = output channel.
// Polyphase ConvTranspose1d (UPS): m = co*s + r and the result lands at
// y[b][co][n*s + r - p].
struct ConvParams {
  const float* x;    // [B][C_in][L_in] (or [B][L_in][C_in] for a BTC mel: see x_cs/x_ts)
  int64_t x_bs;      // batch stride of x (elements)
  int64_t x_cs, x_ts;  // channel / time strides of x (L_in, 1 for [B][C][L])
  int C_in, L_in;
  const int32_t* len_in;   // per-item valid input length (device, [B]) or null = L_in
  const int32_t* len_out;  // per-item valid output length (device, [B]) or null = N / L_out
  const float* w;    // packed weights (see pack layout in hifigan_capi.cpp)
  const float* bias; // per GEMM row m, length >= m_tiles * MT
  float* y;          // output [B][M][N] (regular) or [B][C_out][L_out] (UPS)
  int64_t y_bs;
  int M, N;          // GEMM rows (valid), output columns per batch item
  int off, dil;      // input index = n + off + j*dil
  int kt;            // taps (used when the kernel's KT template arg is 0)
  int act_in;        // leaky_relu on the staged input
  int act_out;       // leaky_relu on the output
  const float* res;  // residual added to the output (same layout as y) or null
  float* mrf;        // MRF accumulator; when set the result goes here, not to y
  int mrf_mode;      // bit0: add existing mrf value, bit1: divide by mrf_div
  float mrf_div;
  int ups_s, ups_p, L_out;  // UPS store mapping
  int ups_swz;              // UPS: XCD swizzle of the block order (bf16x3 kernel)
  int n_chunks;      // ceil(C_in / CK)
  int n_base;        // first GEMM column of this launch (bf16x3 kernel; 0 elsewhere)
  int epi_lds;       // bf16x3 layer kernel: LDS-staged float4 epilogue (epilogue.h)
  // f16x3 scaling (bf16x3_common.h): amax_in[b] = max |x| of item b (producer slot, null:
  // unscaled input), ew = the weights' packing exponent; amax_out[b] <- max |stored y|
  // (null: not committed)
  const uint32_t* amax_in;
  uint32_t* amax_out;
  int ew;
  int dbg;           // ablation flags (HFG_DEBUG_FLAGS, builds with -DHFG_ABLATE=1 only; wrong
                     // results when set), bf16x3 kernel: bit0 skip input restaging after the
                     // first chunk, bit2 no per-chunk barrier, bit3 no epilogue, bit7 every
                     // group's input loads re-read group 0 (L2-warm)
};

// kernel ablation switches (timing experiments) exist only in -DHFG_ABLATE=1 builds
#ifndef HFG_ABLATE
#define HFG_ABLATE 0
#endif
constexpr bool kAblate = HFG_ABLATE != 0;

// Tile configurations of conv1d_mfma_f32 (fp32 MFMA 32x32x2).
//   MT = 32*WM*WAVES_M rows, NTILE = 32*WN*WAVES_N columns,
//   64*WAVES_M*WAVES_N threads.  The C_in chunk CK depends on the tap count.
struct TileCfg {
  int WM, WN, WAVES_M, WAVES_N;
  constexpr int MT() const { return 32 * WM * WAVES_M; }
  constexpr int NTILE() const { return 32 * WN * WAVES_N; }
  constexpr int threads() const { return 64 * WAVES_M * WAVES_N; }
};

enum TileId { TILE_M128 = 0, TILE_M64 = 1, TILE_M32 = 2, TILE_COUNT = 3 };

constexpr TileCfg kTiles[TILE_COUNT] = {
    {2, 2, 2, 2},  // M128: 128 x 128 tile, 4 waves of 64x64
    {2, 2, 1, 4},  // M64 :  64 x 256 tile, 4 waves of 64x64
    {1, 4, 1, 4},  // M32 :  32 x 512 tile, 4 waves of 32x128
};

// the fp32 kernel of `tile` handles kt taps at dilation dil (staging registers, LDS)
bool fp32_conv_supported(int tile, int kt, int dil);

inline TileId tile_for_rows(int M) {
  if (M >= 128) return TILE_M128;
  if (M >= 64) return TILE_M64;
  return TILE_M32;
}

// Tap counts with a dedicated (fully unrolled) instantiation; others use the
// runtime-KT instantiation (template KT = 0).
constexpr bool kt_specialised(int kt) {
  return kt == 2 || kt == 3 || kt == 5 || kt == 7 || kt == 11;
}
constexpr int dispatch_kt(int kt) { return kt_specialised(kt) ? kt : 0; }

// Input channels per LDS chunk for an instantiation: one weight slab of
// ~12-24 KB so that two pipeline stages leave room for 3 blocks per CU; the
// 512-column M32 tile stages wide input rows, so its chunk is capped at 8.
constexpr int ck_for(int dkt, int tile) {
  return (dkt == 0 || dkt >= 7) ? 4 : (dkt >= 3 || tile == TILE_M32) ? 8 : 16;
}

// Largest (KT-1)*dilation halo an instantiation stages (sizes the per-thread
// input-staging registers).  Checked by the host before launch.
constexpr int kMaxDil = 16;
constexpr int halo_max(int dkt) { return dkt == 0 ? 192 : (dkt - 1) * kMaxDil; }

// ---- split-precision bf16x3 conv (conv_bf16x3.hip) ----
// WD = depth of the weight-slab ring (chunks in flight: WD - 1).
struct Bf16x3Cfg {
  int WAVES_M, WAVES_N, WM, WN, TPC, WD;
  int AREG;  // 1: A fragments loaded from global straight into registers (no LDS ring)
  constexpr int MT() const { return 32 * WM * WAVES_M; }
  constexpr int NTILE() const { return 32 * WN * WAVES_N; }
  constexpr int threads() const { return 64 * WAVES_M * WAVES_N; }
};
constexpr int kBf16x3Tiles_n = 7;
// 0: (removed in round 4: 128x256, 2x4 waves of 64x64, 3-deep weight ring, 1 block/CU —
//    slower than tile 3 / 5; the slot keeps the other tiles' indices)
// 1: 64x256, 1x4 waves of 64x64, 2 taps/chunk (2 blocks/CU)
// 2: 32x256, 1x4 waves of 32x64, 4 taps/chunk (2 blocks/CU)
// 3: 128x256, 2x2 waves of 64x128, 2 taps/chunk (2 blocks/CU: one block's epilogue
//    overlaps the other's main loop)
// 4: 64x64, 2x1 waves of 32x64, 4 taps/chunk: the small-grid tile.  A launch whose
//    tile-3 grid would leave most CUs idle (small batches, short utterances) runs on it
//    instead; every output element sees the same MFMA sequence (channel groups x taps in
//    order, lo*hi, hi*lo, hi*hi) on either tile, so the choice is bitwise invisible.
// 5: tile 3's geometry and packing with the A fragments read by each wave from global
//    (L2) into registers two taps ahead instead of through an LDS slab ring: LDS holds
//    only the input windows, and the block synchronises once per channel group instead
//    of once per 2-tap chunk (layer convs with compile-time taps; HFG_AREG)
// 6: tile 5's schedule on a 256x128 block, 4x1 waves of 64x128 (round 6; layers with 256
//    output rows: one m-tile, so each input window is staged once per 128 output columns
//    instead of twice per 256 — half the staging loads and conversions per output; every
//    wave reads its own A rows: twice tile 5's A traffic from L2)
constexpr Bf16x3Cfg kBf16x3Tiles[kBf16x3Tiles_n] = {
    {2, 4, 2, 2, 4, 3, 0}, {1, 4, 2, 2, 2, 2, 0}, {1, 4, 1, 2, 4, 2, 0}, {2, 2, 2, 4, 2, 2, 0},
    {2, 1, 1, 2, 4, 2, 0}, {2, 2, 2, 4, 2, 2, 1}, {4, 1, 2, 4, 2, 2, 1}};
constexpr int kAregTile = 5;
constexpr int kAregTallTile = 6;
constexpr int kBf16x3SmallTile = 4;
// a layer launch runs on the small tile when its tile-3 grid has fewer blocks than this
// (tile 3 fits 2 blocks per CU: 512 slots on 256 CUs)
constexpr int kSmallGridBlocks = 256;
constexpr int kBf16x3Ck = 16;  // channels per chunk (one MFMA k-step per tap)
// largest (KT-1)*dil window halo of the bf16x3 layer kernel (sizes its staging
// registers: 3 tasks per thread for the 256-column tiles); wider layers run on the fp32 path
constexpr int kBf16x3MaxHalo = 128;
// rows of one staged input plane on the AREG tile: one per staging task (XQ * NT / 2),
// as conv1d_bf16x3 computes XQ from the largest window of the instantiation
constexpr int bf16x3_areg_rows(int kt, const Bf16x3Cfg& t) {
  const int halo = (kt - 1) * kMaxDil < kBf16x3MaxHalo ? (kt - 1) * kMaxDil : kBf16x3MaxHalo;
  const int xw_max = t.NTILE() + halo;
  const int nt = t.threads();
  return (2 * xw_max + nt - 1) / nt * nt / 2;
}
// AREG tile: byte offset of the m-tile's bias copy in LDS (read by the LDS-staged epilogue:
// no global load between its stores) = past both the input planes and the epilogue staging
constexpr int bf16x3_areg_bias_off(int kt, const Bf16x3Cfg& t) {
  const int xbytes = 2 * 4 * (bf16x3_areg_rows(kt, t) * 16 + 64);
  const int stage = t.threads() / 64 * 32 * (32 * t.WN + 8) * 4;
  return ((xbytes > stage ? xbytes : stage) + 15) & ~15;
}
inline int bf16x3_tile_for_rows(int M) { return M >= 128 ? 3 : (M >= 64 ? 1 : (M >= 32 ? 2 : -1)); }
size_t bf16x3_lds_bytes(int tile, int kt, int dil);
// the bf16x3 layer kernel handles kt taps at dilation dil (else the fp32 kernel runs)
inline bool bf16x3_supported(int kt, int dil) {
  return dil >= 1 && dil <= kMaxDil && kt >= 1 && kt <= 16 && (kt - 1) * dil <= kBf16x3MaxHalo;
}
// np: MFMA products per multiply-add, 3 (bf16x3) or 2 (bf16-valued weights, tiles 1-4)
// fmt: kFmtBf16 (bf16x3) or kFmtF16 (f16x3), bf16x3_common.h
hipError_t launch_conv_bf16x3(int tile, int kt, bool ups, int fmt, int np, const ConvParams& p,
                              int n_tiles, int m_tiles, int batch, hipStream_t stream,
                              const char** name);

// ---- upsampler over output frames (ups_bf16x3.hip) ----
// lrelu -> ConvTranspose1d(k = 2u, stride u, padding u/2) as a GEMM whose columns are the T
// input frames: rows of class L (samples s < u/2 of a frame: taps x[m-1], x[m]) and class R
// (s >= u/2: x[m], x[m+1]), both computed by every wave.  Bitwise the polyphase
// conv1d_bf16x3 upsampler.
struct UpsCfg {
  int WAVES_M, WAVES_N, WM, WN;
  constexpr int MT() const { return 32 * WM * WAVES_M; }  // rows per class and m-tile
  constexpr int NTILE() const { return 32 * WN * WAVES_N; }
  constexpr int threads() const { return 64 * WAVES_M * WAVES_N; }
};
// 0: 64 rows x 256 frames, 2x2 waves of 32 rows x 128 frames (x 2 classes)
// 1: 32 rows x 256 frames, 1x4 waves of 32 x 64 (C_out * u / 2 = 32: V1 ups.3)
// (128-frame tiles of both, 3 blocks per CU, measured 30 % slower on ups.2 / 8 % on ups.3
// and 2x on ups.0 + ups.1: profiles/r03/ups/nt_ab.txt)
constexpr int kUpsCfgs_n = 2;
constexpr UpsCfg kUpsCfgs[kUpsCfgs_n] = {{2, 2, 1, 4}, {1, 4, 1, 2}};
// rates whose two classes store whole runs: u = 2 (8 B), u = 4 (16 B), u/2 % 4 == 0 (16 B)
inline constexpr bool ups_rate_ok(int u) { return u == 2 || u == 4 || (u % 8 == 0 && u > 0); }
struct UpsParams {
  const float* x;        // stage input [B][C_in][L]
  int64_t x_bs;          // batch stride of x (C_in * L)
  int C_in, L;           // channels, row length (L % 4 == 0)
  int T;                 // frames (GEMM columns) per item, <= L
  const int32_t* len_in; // per-item valid frames (device, [B]) or null = T
  const __bf16* w;       // packed [m_tile][g][class][tap][plane][wave_m][wm][lane][8]
  const float* bias;     // [C_out]
  float* y;              // [B][C_out][L_out]
  int64_t y_bs;
  int C_out, L_out, u;
  int m_tiles, n_tiles, batch;
  const uint32_t* amax_in;  // f16x3: per-item max |x| (producer slot) or null
  uint32_t* amax_out;       // f16x3: per-item max |y| slot or null
  int ew;                   // weight packing exponent (f16x3)
  int dbg;               // ablations (HFG_DEBUG_FLAGS, timing only, wrong results): bit9 no
                         // input conversion after group 0, bit10 no input loads after group 0
};
size_t ups_lds_bytes(int cfg);
hipError_t launch_ups_bf16x3(int cfg, int fmt, int np, const UpsParams& p, hipStream_t stream,
                             const char** name);

// ---- whole ResBlock per launch (resblock_bf16x3.hip) ----
// All 2*n_dil convs of one ResBlock of a C in {32, 64, 128} stage on a window of nwin
// columns (256 or 512); x in registers, the conv operand in LDS.  Each wave owns wm row
// tiles (32 or 64 rows) x 4/wm column tiles.
constexpr int kRbMaxConv = 16;
// spare operand rows per side (every conv's (k-1)/2*dil must fit): 48 for the 512-column
// windows, 28 for C = 128 (its 256-column window then just fits the 160 KB LDS), 16 for the
// narrow C = 64 window (256 columns: 74 KB, two blocks per CU, used for k = 3)
constexpr int rb_marg(int C, int nwin) {
  return C >= 128 ? 28 : (C == 64 && nwin == 256) ? 16 : 48;
}
struct RbParams {
  const float* x;        // stage input [B][C][L]
  int64_t bs;            // batch stride of x and mrf (C * L)
  int L;                 // row length
  const int32_t* len;    // per-item valid length (device, [B]) or null = L
  const __bf16* w;       // packed A stream [wave_m][conv][group][tap][plane][lane][8]
  int w_bytes;           // its size (buffer descriptor range)
  const float* bias;     // [conv][C]
  int n_conv;            // convs of this launch (even), order conv1_0, conv2_0, conv1_1, ...
  int conv0;             // index of its first conv in the packed stream
  int n_conv_stream;     // convs in the packed stream (the whole ResBlock)
  int dil[kRbMaxConv];   // dilation of each conv
  int halo, W;           // receptive-field radius, output columns per block
  float* mrf;            // MRF accumulator [B][C][L]
  int mrf_mode;          // bit0: add the existing value, bit1: divide by mrf_div
  float mrf_div;
  float mrf_rcp;         // fp32(1 / mrf_div) when fast_div_ok(mrf_div) (exact fma quotient), else 0
  int ew[kRbMaxConv];    // f16x3: packing exponent of each conv's weights (stream order)
  uint32_t* amax_out;    // f16x3: per-item max |stored mrf| slot (final MRF write) or null
  // fused conv_post + tanh (C = 32, the last MRF write; L % 4 == 0): wav [B][L] written on the
  // centre [halo, halo + W) of each window, mrf not stored; halo includes the conv's radius 3.
  // Windows past an item's length write nothing (the host zeroes wav first).  Null: off
  const float* post_w;   // conv_post weight [C][7] fp32
  const float* post_b;   // conv_post bias [1]
  float* wav;
  int batch;             // items (set by launch_resblock_bf16x3)
  // persistent grid (one-block-per-CU instances; not with the fused conv_post): 0 = one window
  // per block, else the launch runs min(windows, persist) blocks that walk the windows and
  // overlap each window's MRF read-modify-write with the next window's x loads
  int persist;
  int dbg;               // ablations (HFG_DEBUG_FLAGS, wrong results when set): bit4 no MRF
                         // epilogue, bit5 no x loads, bit6 no operand writes
};
// divisors whose fma-refined reciprocal quotient equals the IEEE quotient for every fp32
// input (div_exact, bf16x3_common.h; verified exhaustively, tests/tools/verify_fast_div.c)
inline bool fast_div_ok(float d) {
  return d == 1.f || d == 2.f || d == 3.f || d == 4.f || d == 5.f || d == 7.f || d == 8.f;
}
bool rb_supported(int C, int kt, int nwin, int wm);
size_t rb_lds_bytes(int C, int nwin, int n_conv);
hipError_t launch_resblock_bf16x3(int C, int nwin, int wm, int kt, int fmt, int np,
                                  const RbParams& p, int batch, hipStream_t stream,
                                  const char** name);

// ---- whole MRF per launch for thin stages, C <= 16 (mrf_thin.hip) ----
// All ResBlocks of one MRF on a time window in LDS, packed-fp32 VALU dot products (exact
// fp32 products).  Weights packed per conv [tap][ci][co] (fp32), biases [conv][C].
constexpr int kThinMarg = 64;      // spare operand columns per side: every (k-1)/2*d must fit
constexpr int kThinMaxRes = 8;
constexpr int kThinMaxConv = 64;
struct ThinParams {
  const float* x;            // stage input [B][C][L]
  int64_t bs;                // batch stride of x and y (C * L)
  int L;
  const int32_t* len;        // per-item valid length (device, [B]) or null = L
  const float* w;            // packed weights (floats)
  const float* bias;         // [conv][C]
  int n_res;                 // ResBlocks in this launch
  int rb_conv0[kThinMaxRes + 1];  // ResBlock r runs convs [rb_conv0[r], rb_conv0[r+1])
  int kt[kThinMaxConv], dil[kThinMaxConv], w_off[kThinMaxConv];  // per conv (conv1, conv2, ...)
  int halo, W;               // largest ResBlock radius, output columns per block
  float* y;                  // [B][C][L] <- (sum of the ResBlocks' outputs) / div
  float div;
  // bf16x3 MFMA variant (mrf_thin_mfma.hip): A stream [conv][step][plane][lane][8] bf16
  const __bf16* wm;          // this launch's stream
  int wm_bytes;              // its size (buffer descriptor range)
  int wm_off[kThinMaxConv];  // byte offset of each conv's first k-step
  int ew[kThinMaxConv];      // f16x3: packing exponent of each conv's weights
  uint32_t* amax_out;        // per-item max |y| slot (f16x3 consumers) or null
};
int thin_window(int C);      // window columns of the C-channel instance (0: unsupported C)
size_t thin_lds_bytes(int C);
hipError_t launch_mrf_thin(int C, const ThinParams& p, int batch, hipStream_t stream,
                           const char** name);
// the same MRF on the 16x16x32 matrix cores in split precision (bf16x3 / f16x3 products):
// 4 waves x kThinMfmaTiles 16-column tiles (a 512-column window), C = 16
constexpr int kThinMfmaTiles = 8;
// operand buffers of mrf_thin_mfma: 2 = one barrier per conv (conv1 / conv2 alternate),
// 1 = rewritten in place (two barriers per conv; round 2)
#ifndef HFG_THIN_BUFS
#define HFG_THIN_BUFS 2
#endif
constexpr int kThinMfmaBufs = HFG_THIN_BUFS;
constexpr int kThinMfmaMaxSteps = 4;  // k-steps per conv (k <= 7 at C = 16)
int thin_mfma_window(int C);  // 0: unsupported C
size_t thin_mfma_lds_bytes(int C);
hipError_t launch_mrf_thin_mfma(int C, int fmt, int np, const ThinParams& p, int batch,
                                hipStream_t stream, const char** name);

// Launch the conv kernel for (tile, taps, ups).  Returns a hipError_t and,
// via *name, the kernel's template-instance name (as rocprofv3 prints it).
hipError_t launch_conv(TileId tile, int kt, bool ups, const ConvParams& p, int n_tiles,
                       int m_tiles, int batch, hipStream_t stream, const char** name);

// conv_post + tanh: input rows staged in LDS kConvPostCB channels at a time
constexpr int kConvPostCB = 32;
inline size_t conv_post_lds_bytes(int C) {
  return sizeof(float) * ((size_t)((C * 7 + 3) & ~3) + (size_t)(C < kConvPostCB ? C : kConvPostCB) * (256 + 6));
}
// conv_post + tanh: wav[b][t] = tanh(bias + sum_{c,j} w[c][j] * lrelu(x[b][c][t+j-3]))
// for t < lens[b] (lens null = L); 0 beyond.  quad: the 4-samples-per-thread kernel
// (conv_post4_tanh) where L % 4 == 0 — bitwise the LDS-staged one.
inline bool conv_post4_ok(int L) { return L % 4 == 0; }
hipError_t launch_conv_post(const float* x, int64_t x_bs, int C, int L, const float* w,
                            const float* bias, float* wav, const int32_t* lens, int batch,
                            hipStream_t stream, const char** name, bool quad = true);

// Content hash of up to kChecksumMax fp32 tensors per launch: out[base + i] +=
// sum_w mix(word_w, w) over tensor i's n[i] 32-bit words (out zeroed by the caller).
constexpr int kChecksumMax = 64;
struct ChecksumArgs {
  const uint32_t* p[kChecksumMax];
  int64_t n[kChecksumMax];
  int count, base;
};
hipError_t launch_checksum(const ChecksumArgs& a, uint32_t* out, hipStream_t stream);

// y = (o_0 + o_1 + ... (in order)) / div over [B][C][L], columns < len[b] (len null = L)
constexpr int kMrfCombineMax = 8;
struct MrfCombineArgs {
  const float* o[kMrfCombineMax];
  int n, C, L;
  const int32_t* len;
  float* y;
  float div;
  uint32_t* amax_out;  // per-item max |y| slot (f16x3 consumers) or null
};
hipError_t launch_mrf_combine(const MrfCombineArgs& a, int batch, hipStream_t stream);

// Per-stage valid lengths of a ragged batch: out[s*B + b] = length after s
// upsample stages of an utterance with lens[b] frames (clamped to [0, T]).
struct StageLenParams {
  int n_up, T;
  int up_rates[8], up_kernels[8];
};
// out[b] <- max(out[b], max |x[b][c][t]|) over c < C, t < len[b] (len null = L): the f16x3
// scale slot of a tensor no producing kernel reported (the mel, a caller's MRF input)
hipError_t launch_absmax(const float* x, int64_t x_bs, int64_t x_cs, int64_t x_ts, int C, int L,
                         const int32_t* len, int batch, uint32_t* out, hipStream_t stream);

hipError_t launch_stage_lengths(const int32_t* lens, int B, const StageLenParams& sp,
                                int32_t* out, hipStream_t stream);

}  // namespace hfg

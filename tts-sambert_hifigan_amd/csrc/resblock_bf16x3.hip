// resblock_bf16x3.hip — one whole ResBlock per launch (bf16x3 MFMA), for the
// narrow stages (C in {32, 64}) where a layer-per-launch schedule is bound by HBM
// round trips, not by the matrix cores:
//
//   for m in dilations:  x = x + conv2_m(lrelu(conv1_m(lrelu(x))))   models/hifigan.py:79-85
//   mrf = (mrf + x) [/ n_res]                                         models/hifigan.py:125-131
//
// A block owns a window of NWIN time columns [ws, ws + NWIN) of one utterance and
// writes the centre [ws + halo, ws + halo + W), W = NWIN - 2*halo, where halo is the
// receptive-field radius of the launch's convs after the first (sum of (k-1)/2 * dilation).
// All convs run on the whole window.  The first conv's operand also covers its radius on
// either side (the LDS margin rows, staged from x), so its output is exact on the whole
// window; from the second conv on, the columns within a conv's radius of the window edge
// become garbage and the garbage front moves inwards by exactly that radius, so the
// centre is exact.  Columns outside [0, len) are re-zeroed after every conv — the
// reference's zero padding of each conv input.
//
// State: the residual stream x lives in registers (fp32, MFMA accumulator layout:
// every wave owns 32 rows x 128 columns of the window for the whole block), the
// current conv's B operand lives in LDS as bf16 hi/lo planes [group][plane][col][16]
// (one buffer, rewritten in place after a barrier).  The A operand (weights) is
// streamed from global memory (L2/L1-resident: every block reads the same stream)
// straight into registers two k-steps ahead; it is packed per wave row-block as
// [wave_m][conv][group][tap][plane][lane][8] so each k-step is 2 x 1 KB coalesced.
//
// Channel order inside a 16-channel group is permuted (slot 8h+e <-> channel
// 4h + (e&3) + 8(e>>2)) so that the rows one lane holds in the accumulator layout are
// exactly the 8 slots it reads as a B fragment: the epilogue writes the next conv's
// operand with one ds_write_b128 per plane and group.  The weight packer applies the
// same permutation to the K index.
//
// HBM traffic per ResBlock: x once (+ halo), MRF read-modify-write once, vs 5 tensor
// passes per dilation for the layer-per-launch schedule.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <mutex>

#include <cstdio>

#include "bf16x3_common.h"
#include "kernels.h"

// diagnostic build only (-DHFG_RB_TIMING=1, profiles/r04): wave 0 of every block stamps the
// shader clock at the phase boundaries into g_rb_ts (one region per instance and launch half),
// read back by hfg_debug_rb_ts (tests/tools/rb_phases.py)
#ifndef HFG_RB_TIMING
#define HFG_RB_TIMING 0
#endif

namespace hfg {

#if HFG_RB_TIMING
constexpr int kRbTsSlots = 24, kRbTsBlocks = 8192, kRbTsRegions = 20;
__device__ uint64_t g_rb_ts[kRbTsRegions * kRbTsBlocks * kRbTsSlots];
#endif

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

// conv_post + tanh (models/hifigan.py:254-256) fused into the network's last MRF write (C = 32,
// one 32-row wave per window slice): the exact final x on the window columns [halo - 3,
// halo + W + 3) is staged as lrelu(x) in LDS ([channel][column + sh] fp32, 0 outside those
// columns and outside [0, len)), then one thread per 2 consecutive samples (each quad split over
// the two halves of the block) sums over (channel, tap) in conv_post4_tanh's order (channel-
// major, fma from 0, bias last): bitwise the separate kernel's wav, without the stage output's
// HBM write and read.
template <int NT, int NWIN, int WN>
__device__ __forceinline__ void conv_post_tail(const RbParams& p, const floatx16 (&xcur)[1][WN],
                                               const bool (&ok)[WN], char* lds, int b, int len_b,
                                               int t0, int tid, int cbase, int half, int col) {
  constexpr int C = 32, KP = 7;
  constexpr int S = NWIN + 8;  // row stride (floats): the two lane halves' rows, 4 apart, 32 banks apart
  typedef float f4 __attribute__((ext_vector_type(4)));
  float* const s = reinterpret_cast<float*>(lds);
  const int sh = (4 - (p.halo & 3)) & 3;  // staged column = window column + sh: 16-B aligned quads
  lds_barrier();                          // every wave is done reading the last conv's operand
#pragma unroll
  for (int k = 0; k < WN; ++k)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float v = xcur[0][k][r];
      s[((r & 3) + 8 * (r >> 2) + 4 * half) * S + cbase + 32 * k + col + sh] =
          ok[k] ? (v > 0.f ? v : v * kLReluSlope) : 0.f;
    }
  lds_barrier();
  const float bias = p.post_b[0];
  float* const wav = p.wav + (int64_t)b * p.L;
  // the first half of the threads computes samples 0, 1 of each quad, the second half samples
  // 2, 3 (wave-uniform: two specialised code paths), so every wave works on the tail
  static_assert(NT % 128 == 0, "whole waves per half");
  const int hq = __builtin_amdgcn_readfirstlane(tid / (NT / 2));
  auto run = [&](auto h_tag) {
    constexpr int H = decltype(h_tag)::value;
    for (int q = tid - H * (NT / 2); q < p.W / 4; q += NT / 2) {
      const int t = t0 + 4 * q;  // p.L % 4 == 0 (host): a quad is wholly inside or past the row
      if (t >= p.L) break;
      // element k of v = column t - 4 + k (conv_post4_tanh's layout)
      const float* xs = s + p.halo + sh + 4 * q - 4;
      float acc[2] = {0.f, 0.f};
#pragma unroll 4
      for (int c = 0; c < C; ++c) {
        const f4 q0 = *reinterpret_cast<const f4*>(xs + c * S);
        const f4 q1 = *reinterpret_cast<const f4*>(xs + c * S + 4);
        const f4 q2 = *reinterpret_cast<const f4*>(xs + c * S + 8);
        const float v[12] = {q0[0], q0[1], q0[2], q0[3], q1[0], q1[1],
                             q1[2], q1[3], q2[0], q2[1], q2[2], q2[3]};
        const float* w = p.post_w + c * KP;
#pragma unroll
        for (int o = 0; o < 2; ++o)
#pragma unroll
          for (int j = 0; j < KP; ++j) acc[o] = fmaf(w[j], v[2 * H + o + j + 1], acc[o]);
      }
      floatx2 r;
#pragma unroll
      for (int o = 0; o < 2; ++o) r[o] = t + 2 * H + o >= len_b ? 0.f : tanhf(acc[o] + bias);
      *reinterpret_cast<floatx2*>(wav + t + 2 * H) = r;
    }
  };
  if (hq == 0)
    run(std::integral_constant<int, 0>{});
  else
    run(std::integral_constant<int, 1>{});
}

template <int KT, int WAVES_M, int WAVES_N, int WM, int NP, int FMT, bool PERSIST>
__global__ void __launch_bounds__(64 * WAVES_M * WAVES_N, 2)  // 2 waves/SIMD: <= 256 VGPRs
resblock_bf16x3(const RbParams p) {
  constexpr int NW = WAVES_M * WAVES_N;
  constexpr int NT = 64 * NW;
  static_assert(WM == 1 || WM == 2, "32 or 64 rows per wave");
  constexpr int C = 32 * WM * WAVES_M;
  constexpr int NG = C / 16;               // 16-channel groups
  constexpr int WN = 4 / WM;               // 32-column MFMA tiles per wave (WM row tiles)
  constexpr int NWIN = 32 * WN * WAVES_N;  // window columns
  constexpr int STEPS = NG * KT;           // MFMA k-steps per conv
  static_assert(STEPS % 2 == 0, "two-deep A register ring needs an even step count");
  // operand rows: the window plus MARG spare rows on each side, read by the taps of edge
  // columns: the first conv's operand fills its radius of them from x (write_margins), later
  // operands leave them stale (their contents only reach garbage columns)
  constexpr int MARG = rb_marg(C, NWIN);
  constexpr int ROWS = NWIN + 2 * MARG;
  constexpr int PS = ROWS * 16;            // bytes per plane: [row][8 bf16]
  constexpr int HPS = 2 * PS;              // half-group (slots 0-7 | 8-15): hi, lo planes
  constexpr int GS = 2 * HPS;              // 16-channel group
  constexpr int ASTEP = 2 * 64 * 16;       // bytes per k-step of one wave row-block (hi, lo)
  static_assert(C != 32 || (WM == 1 && 32 * (NWIN + 8) * 4 <= NG * GS),
                "conv_post staging fits the operand planes");

  extern __shared__ __attribute__((aligned(16))) char lds[];
  float* const bias_s = reinterpret_cast<float*>(lds + NG * GS);
  // f16x3: per-wave max |next operand| (NW floats after the biases)
  float* const amax_s = bias_s + p.n_conv * C;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wave_m = wave % WAVES_M;
  const int wave_n = wave / WAVES_M;
  const int half = lane >> 5;
  const int col = lane & 31;
  // ---- windows: w = tile + n_tiles * item.  One window per block (grid n_tiles x B), or
  // with p.persist a grid of G blocks that walks the windows w, w + G, w + 2G, ... and issues
  // the next window's x and margin loads beside the current window's MRF read-modify-write
  // (one-block-per-CU instances: nothing else on the CU hides those round trips).  Windows past
  // an item's length are skipped (block-uniform). ----
  const int n_tiles = (p.L + p.W - 1) / p.W;
  const int n_win = n_tiles * p.batch;
  const int wstride = PERSIST ? (int)gridDim.x : n_win;
  auto item_of = [&](int wi) { return __builtin_amdgcn_readfirstlane(wi / n_tiles); };
  auto len_of = [&](int bi) { return p.len ? min(p.len[bi], p.L) : p.L; };
  auto valid = [&](int wi) {
    const int bi = item_of(wi);
    return (wi - bi * n_tiles) * p.W < len_of(bi);
  };
  int w = PERSIST ? (int)blockIdx.x : (int)(blockIdx.x + n_tiles * blockIdx.y);
  while (w < n_win && !valid(w)) {
    if (!PERSIST) return;  // whole block past this utterance's end (block-uniform)
    w += wstride;
  }
  if (w >= n_win) return;
  int b = item_of(w);
  int len_b = len_of(b);
  int t0 = (w - b * n_tiles) * p.W;
#if HFG_RB_TIMING
  const int ts_region = NWIN == 256 && C == 64 ? 18 + (p.conv0 > 0 ? 1 : 0)
                        : ((KT == 3 ? 0 : KT == 7 ? 1 : 2) * 3 + (C == 32 ? 0 : C == 64 ? 1 : 2)) * 2 +
                              (p.conv0 > 0 ? 1 : 0);
  const int ts_blk = blockIdx.y * gridDim.x + blockIdx.x;
  uint64_t* const ts = g_rb_ts + ((size_t)ts_region * kRbTsBlocks + (ts_blk < kRbTsBlocks ? ts_blk : 0)) * kRbTsSlots;
  // stamps kept in LDS (past the f16x3 maxima) and stored once at the end: a global (or
  // scratch) store mid-kernel would make every later vmcnt wait also wait for its write (one
  // in-order queue for vector loads and stores).  A persistent block keeps its last window's.
  uint64_t* const tsv = reinterpret_cast<uint64_t*>(amax_s + 16);
  auto stamp = [&](int i) {
    const uint64_t t = __builtin_amdgcn_s_memtime();
    if (tid == 0) tsv[i] = t;
  };
  if (tid < kRbTsSlots) tsv[tid] = 0;
  __syncthreads();
  if (tid == 0) tsv[0] = __builtin_amdgcn_s_memrealtime();
  stamp(1);
#else
  auto stamp = [](int) {};
#endif
  int ws = t0 - p.halo;
  const int cbase = wave_n * 32 * WN;      // first window column of this wave
  const int row0 = wave_m * 32 * WM;     // first row of this wave (WM row tiles of 32)
  const int n_conv = p.n_conv;
  // A stream: the whole ResBlock's convs (p.n_conv_stream per wave row-block); this launch
  // runs convs p.conv0 .. p.conv0 + n_conv - 1 of it (a ResBlock split into two launches)
  const int QT = p.n_conv_stream * STEPS;
  const int Q0 = p.conv0 * STEPS;
  const int dbg = p.dbg;
  auto rrow = [&](int r) { return (r & 3) + 8 * (r >> 2) + 4 * half; };

  for (int i = tid; i < n_conv * C; i += NT) bias_s[i] = p.bias[i];

  bool vk[WN];
  auto set_vk = [&]() {
#pragma unroll
    for (int k = 0; k < WN; ++k) vk[k] = (unsigned)(ws + cbase + 32 * k + col) < (unsigned)len_b;
  };
  set_vk();

  // ---- A stream (buffer loads: SGPR descriptor + scalar step offset, no address VALU) ----
  const __amdgpu_buffer_rsrc_t wrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.w, 0, p.w_bytes, 0x00020000);
  const int a_base = wave_m * WM * QT * ASTEP;  // row tile i: + i * QT * ASTEP
  const int a_lane = lane * 16;
  bf16x8 ra_h[2][WM], ra_l[2][WM];
  auto load_a = [&](int slot, int q) {
    const int so = a_base + min(q, QT - 1) * ASTEP;
#pragma unroll
    for (int i = 0; i < WM; ++i) {
      ra_h[slot][i] = __builtin_bit_cast(
          bf16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, a_lane, so + i * QT * ASTEP, 0));
      ra_l[slot][i] = __builtin_bit_cast(
          bf16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, a_lane + 1024, so + i * QT * ASTEP, 0));
    }
  };
  load_a(0, Q0);
  load_a(1, Q0 + 1);
  stamp(20);

  // ---- x and the MRF accumulator of utterance b through buffer descriptors ----
  // Element (row, column) sits at soffset = (row0 + row part of accumulator element r) * L * 4
  // (wave-uniform: SALU) + voffset = (4 * half * L + column) * 4 (one VGPR per column tile):
  // no per-element address VALU and no branches.  An item is fewer than 2^30 floats (the C
  // ABI's bound: a dword is dropped when voffset + soffset + 4 passes num_records, so a
  // 4-GiB item would lose its last float), so every offset and its dword end fit 32 bits;
  // the range is never relied on otherwise (masked lanes read offset 0).
  unsigned Lb = (unsigned)p.L * 4u;
  auto srow = [&](int i, int r) { return (unsigned)(row0 + 32 * i + (r & 3) + 8 * (r >> 2)) * Lb; };
  const unsigned lrow = 4u * (unsigned)half * (unsigned)p.L;
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.x + (int64_t)b * p.bs), 0, (int)0xFFFFFFFFu, 0x00020000);

  // ---- residual stream x: window -> registers (zero outside [0, len): masked after the wait) ----
  floatx16 xcur[WM][WN];
  auto issue_x = [&](floatx16 (&dst)[WM][WN], const __amdgpu_buffer_rsrc_t& rs, int wsx, int lenx) {
#pragma unroll
    for (int k = 0; k < WN; ++k) {
      const int gc = wsx + cbase + 32 * k + col;
      const unsigned vo = (unsigned)gc < (unsigned)lenx ? (lrow + (unsigned)gc) * 4u : 0u;
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          dst[i][k][r] = __builtin_bit_cast(
              float, __builtin_amdgcn_raw_buffer_load_b32(rs, (int)vo, (int)srow(i, r), 0));
    }
  };
  auto mask_x = [&]() {
    // ablation bit 5 zeroes x after the loads (a select on a uniform flag inside the load
    // expression made the compiler branch per element)
    const bool xz = kAblate && (dbg & 32);
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int k = 0; k < WN; ++k)
#pragma unroll
        for (int r = 0; r < 16; ++r) xcur[i][k][r] = (vk[k] && !xz) ? xcur[i][k][r] : 0.f;
  };
  // ---- persistent grid: a window's x [C][ROWS] (columns ws - MARG ..) goes to the operand
  // planes' LDS by buffer-load-to-LDS (no VGPRs), issued beside the previous window's MRF
  // read-modify-write; the window then reads its x and margins from LDS.  The item's buffer
  // range (C * L floats) turns the columns outside it into zeros; columns outside [0, len)
  // are masked as in the register path. ----
  constexpr int XD_N = C * ROWS / 64;  // 64-dword pieces (ROWS % 4 == 0: C * ROWS % 64 == 0)
  static_assert(C * ROWS % 64 == 0 && C * ROWS * 4 == NG * GS, "x copy fills the operand planes");
  constexpr int XD_T = (XD_N + NW - 1) / NW;
  auto dma_x = [&](int wsx, int bi) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.x + (int64_t)bi * p.bs), 0, (int)(C * Lb), 0x00020000);
    int c = (wave * 64 + lane) / ROWS;
    int cl = wave * 64 + lane - c * ROWS;
#pragma unroll 4
    for (int q = 0; q < XD_T; ++q) {
      const int j = wave + NW * q;
      if (j < XD_N) {
        const unsigned vo = ((unsigned)c * (unsigned)p.L + (unsigned)(wsx - MARG + cl)) * 4u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t3)(lds + j * 256), 4, (int)vo, 0, 0,
                                                 0);
      }
      static_assert(64 * NW < 3 * ROWS, "two wraps at most");
      cl += 64 * NW;
      c += cl >= ROWS ? 1 : 0;
      cl -= cl >= ROWS ? ROWS : 0;
      c += cl >= ROWS ? 1 : 0;
      cl -= cl >= ROWS ? ROWS : 0;
    }
  };
  if constexpr (PERSIST) {
    dma_x(ws, b);
    wait_vm<0>();
    lds_barrier();
  } else {
    issue_x(xcur, xrs, ws, len_b);
  }
  // ---- the first conv's margins: operand columns [-R0, 0) and [NWIN, NWIN + R0) of the
  // window read from x (R0 = that conv's receptive-field radius <= MARG, host-checked), so the
  // first conv is exact on the whole window and the launch's halo leaves out its radius.  One
  // task = one column of one half-group: its 8 slot channels (write_operand's permutation) ----
  constexpr int MG_T = (4 * MARG * NG + NT - 1) / NT;  // margin tasks per thread
  const int R0 = (KT - 1) / 2 * p.dil[0];
  const int n_mg = 4 * R0 * NG;
  float mg[MG_T][8];
  auto mg_col = [&](int q, int wsx) {  // global column of margin task q (window origin wsx)
    const int t = tid + q * NT;
    const int m = (t >> 1) / NG;
    return wsx + (m < R0 ? m - R0 : NWIN + m - R0);
  };
  auto issue_mg = [&](float (&dst)[MG_T][8], const __amdgpu_buffer_rsrc_t& rs, int wsx, int lenx) {
#pragma unroll
    for (int q = 0; q < MG_T; ++q) {
      const int t = tid + q * NT;
      const int hh = t & 1, gq = (t >> 1) % NG;
      const int gc = mg_col(q, wsx);
      const bool ok = t < n_mg && (unsigned)gc < (unsigned)lenx;
      const unsigned vo = ok ? ((unsigned)(16 * gq + 4 * hh) * (unsigned)p.L + (unsigned)gc) * 4u : 0u;
#pragma unroll
      for (int e = 0; e < 8; ++e)
        dst[q][e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                  rs, (int)vo, (int)(((e & 3) + 8 * (e >> 2)) * Lb), 0));
    }
  };
  auto mask_mg = [&]() {
#pragma unroll
    for (int q = 0; q < MG_T; ++q) {
      const int gc = mg_col(q, ws);
      const bool ok = tid + q * NT < n_mg && (unsigned)gc < (unsigned)len_b;
#pragma unroll
      for (int e = 0; e < 8; ++e) mg[q][e] = ok ? mg[q][e] : 0.f;
    }
  };
  if constexpr (!PERSIST) issue_mg(mg, xrs, ws, len_b);
  // persistent grid: x and the margins from the LDS copy
  auto read_x_lds = [&]() {
    const float* xl = reinterpret_cast<const float*>(lds);
    // the lane's base index, opaque per window: the loop-invariant addresses of the 16 x WM x WN
    // elements would otherwise be hoisted out of the window loop and held in VGPRs across it
    int xb = (row0 + 4 * half) * ROWS + MARG + cbase + col;
    asm volatile("" : "+v"(xb));
#pragma unroll
    for (int k = 0; k < WN; ++k)
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          xcur[i][k][r] = xl[xb + (32 * i + (r & 3) + 8 * (r >> 2)) * ROWS + 32 * k];
#pragma unroll
    for (int q = 0; q < MG_T; ++q) {
      const int t = min(tid + q * NT, n_mg > 0 ? n_mg - 1 : 0);
      const int hh = t & 1, gq = (t >> 1) % NG, m = (t >> 1) / NG;
      const int cw = MARG + (m < R0 ? m - R0 : NWIN + m - R0);
#pragma unroll
      for (int e = 0; e < 8; ++e)
        mg[q][e] = xl[(16 * gq + 4 * hh + (e & 3) + 8 * (e >> 2)) * ROWS + cw];
    }
  };
  auto write_margins = [&](float sc) {
#pragma unroll
    for (int q = 0; q < MG_T; ++q) {
      const int t = tid + q * NT;
      if (t < n_mg) {
        const int hh = t & 1, gq = (t >> 1) % NG, m = (t >> 1) / NG;
        const int c = m < R0 ? m - R0 : NWIN + m - R0;  // window column
        const int off = gq * GS + hh * HPS + (c + MARG) * 16;
        bf16x8 h, l;
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          floatx2 a;
          a[0] = fmaxf(mg[q][e] * sc, mg[q][e] * (kLReluSlope * sc));
          a[1] = fmaxf(mg[q][e + 1] * sc, mg[q][e + 1] * (kLReluSlope * sc));
          bf16x2 hh2, ll;
          split2<FMT>(a, hh2, ll);
          h[e] = hh2[0];
          h[e + 1] = hh2[1];
          l[e] = ll[0];
          l[e + 1] = ll[1];
        }
        *reinterpret_cast<bf16x8*>(lds + off) = h;
        *reinterpret_cast<bf16x8*>(lds + off + PS) = l;
      }
    }
  };

  // lane's byte address of window column (cbase + col) in its half-group's hi plane
  const int vb = half * HPS + (cbase + col + MARG) * 16;

  // leaky_relu and the zero padding as one max(v * f1, v * f2) per value: (1, 0.1) inside
  // [0, len) = bitwise max(v, 0.1 v), (0, 0) outside = 0 (3 VALU ops, no select; both
  // operands are products, so no canonicalising max of the raw value is needed)
  // (the factors are formed per write from vk: kept live across the kernel they cost the
  // C = 128 instance 16 VGPRs and spills)
  // B operand of the next conv: lrelu(v), zero outside [0, len), split hi/lo -> LDS.
  // The 8 accumulator rows a lane holds per 16-channel group are exactly the 8 slots
  // (one 16-B row of its half-group) it reads as a B fragment.
  // f16x3: the operand is scaled by sc = 2^e (block_exp) inside the same two factors
  // Two scalar v_mul_f32 per value, not one v_pk_mul_f32 per value pair (rounds 3-5): packed f32
  // VALU costs ~22 cycles more per instruction than its two scalar halves beside MFMAs
  // (MI355X_MICROARCH.md; same-box -0.9 % ResBlock time, profiles/r06/ab_rewrite.txt).
  auto write_operand = [&](const floatx16 (&v)[WM][WN], float sc) {
    if (kAblate && (dbg & 64)) return;
#pragma unroll
    for (int k = 0; k < WN; ++k) {
      const float f1 = vk[k] ? sc : 0.0f, f2 = vk[k] ? kLReluSlope * sc : 0.0f;
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int gg = 0; gg < 2; ++gg) {
          bf16x8 h, l;
#pragma unroll
          for (int e = 0; e < 8; e += 2) {
            floatx2 a;
            const float v0 = v[i][k][gg * 8 + e], v1 = v[i][k][gg * 8 + e + 1];
            a[0] = fmaxf(v0 * f1, v0 * f2);
            a[1] = fmaxf(v1 * f1, v1 * f2);
            bf16x2 hh, ll;
            split2<FMT>(a, hh, ll);
            h[e] = hh[0];
            h[e + 1] = hh[1];
            l[e] = ll[0];
            l[e + 1] = ll[1];
          }
          char* dst = lds + (row0 / 16 + 2 * i + gg) * GS + vb + k * 512;
          *reinterpret_cast<bf16x8*>(dst) = h;
          *reinterpret_cast<bf16x8*>(dst + PS) = l;
        }
    }
  };
  // f16x3: the block's largest |value| over the window's exact columns sets the power-of-two
  // scale of each operand it writes (per block: the window of an item, and so the result, is
  // the same whatever else is in the batch).  Exact = inside [0, len) and at least `radius`
  // (the receptive-field radius of the convs run so far) from the window edges: the garbage
  // columns outside read the never-written margin rows (stale LDS), so counting them would
  // make the scale depend on earlier launches; garbage that overflows f16 stays in garbage
  // columns.  Each wave posts its max before the barrier that ends every read of the previous
  // operand, and all read the NW maxima after it.
  auto wave_amax = [&](const floatx16 (&v)[WM][WN], int radius, float m = 0.f) {
#pragma unroll
    for (int k = 0; k < WN; ++k) {
      const int c = cbase + 32 * k + col;
      float mk = 0.f;  // v_max3 over the column's 16 x WM rows, one select per column
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) mk = fmaxf(mk, fabsf(v[i][k][r]));
      m = (vk[k] && c >= radius && c < NWIN - radius) ? fmaxf(m, mk) : m;
    }
    m = wave_max(m);
    if (lane == 0) amax_s[wave] = m;
  };
  auto block_exp = [&]() {
    float m = amax_s[0];
#pragma unroll
    for (int w_ = 1; w_ < NW; ++w_) m = fmaxf(m, amax_s[w_]);
    return x3_exp(m);
  };

  // conv cv over the whole window: acc = bias + W_cv * operand (one LDS barrier at the
  // end: every wave has read the operand, which the caller then overwrites in place)
  floatx16 acc[WM][WN];
  auto run_conv = [&](int cv) {
    const int d = p.dil[cv];
    const int pad = (KT - 1) / 2 * d;
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        // f16x3: the bias joins after the unscale (finalize)
        const float bv = FMT == kFmtF16 ? 0.f : bias_s[cv * C + row0 + 32 * i + rrow(r)];
#pragma unroll
        for (int k = 0; k < WN; ++k) acc[i][k][r] = bv;
      }
    bf16x8 bh[2][WN], bl[2][WN];
    // step s = (group g, tap j): rows shifted by j*d - pad, one VALU add per step,
    // tiles / planes by immediate offsets
    auto load_b = [&](int buf, int s_) {
      const int g = s_ / KT, j = s_ - (s_ / KT) * KT;
      const char* src = lds + vb + (g * GS + (j * d - pad) * 16);
#pragma unroll
      for (int k = 0; k < WN; ++k) {
        bh[buf][k] = *reinterpret_cast<const bf16x8*>(src + k * 512);
        // ablation bit 11: no lo-plane reads (the hi fragment stands in; half the LDS reads)
        bl[buf][k] = (kAblate && (dbg & 2048)) ? bh[buf][k]
                                               : *reinterpret_cast<const bf16x8*>(src + k * 512 + PS);
      }
    };
    const int qb = Q0 + cv * STEPS;
    prio_mfma();
    load_b(0, 0);
    // software pipeline: B fragments one step ahead (interleaved with this step's
    // MFMAs), A fragments two steps ahead
#pragma unroll
    for (int s_ = 0; s_ < STEPS; ++s_) {
      const int cur = s_ & 1;
      if (s_ + 1 < STEPS) load_b(cur ^ 1, s_ + 1);
#pragma unroll
      for (int k = 0; k < WN; ++k)
#pragma unroll
        for (int i = 0; i < WM; ++i) {
          if constexpr (NP == 3)  // the weights' lo plane (zero for bf16-valued weights: NP 2)
            acc[i][k] = mfma32<FMT>(ra_l[cur][i], bh[cur][k], acc[i][k]);
          acc[i][k] = mfma32<FMT>(ra_h[cur][i], bl[cur][k], acc[i][k]);
          acc[i][k] = mfma32<FMT>(ra_h[cur][i], bh[cur][k], acc[i][k]);
        }
      load_a(cur, qb + s_ + 2);
      if (s_ + 1 < STEPS) {
#pragma unroll
        for (int i = 0; i < 2 * WN; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read
        }
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);    // 2 MFMA
      __builtin_amdgcn_sched_group_barrier(0x020, 2 * WM, 0);  // A loads
      __builtin_amdgcn_sched_group_barrier(0x008, NP * WM * WN, 0);  // rest of the MFMAs
      __builtin_amdgcn_sched_barrier(0);
    }
    prio_other();
  };
  // f16x3: acc = acc * 2^-(e_x + e_w) + bias (exact unscale, one rounding for the bias)
  int ex = 0;
  auto finalize = [&](int cv) {
    const float inv = exp2i(-(ex + p.ew[cv]));
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float bv = bias_s[cv * C + row0 + 32 * i + rrow(r)];
#pragma unroll
        for (int k = 0; k < WN; ++k) acc[i][k][r] = __builtin_fmaf(acc[i][k][r], inv, bv);
      }
  };

  const bool add = p.mrf_mode & 1;
  const bool div = p.mrf_mode & 2;
  // fused conv_post (C = 32, the network's last MRF write): the stage output is not stored;
  // it is computed on the centre plus the conv's radius 3 on either side and consumed from LDS
  const bool post = C == 32 && p.wav != nullptr;
  const int c_lo = post ? p.halo - 3 : p.halo, c_hi = post ? p.halo + p.W + 3 : p.halo + p.W;
  for (;;) {
    // persistent grid: the row offsets (16 x WM scalars) stay per-window values instead of
    // being hoisted out of the window loop and held (spilled) across it
    if constexpr (PERSIST) asm volatile("" : "+s"(Lb));
    // ---- this window's x (in flight, or in LDS) -> operand ----
    if constexpr (PERSIST) read_x_lds();
    mask_x();
    mask_mg();
    int radius = 0;  // f16x3: receptive-field radius of the convs run so far
    if constexpr (FMT == kFmtF16) {
#if HFG_RB_TIMING
      wait_vm<0>();
      stamp(21);
#endif
      float mm = 0.f;  // the margin columns are part of the first operand
#pragma unroll
      for (int q = 0; q < MG_T; ++q)
#pragma unroll
        for (int e = 0; e < 8; ++e) mm = fmaxf(mm, fabsf(mg[q][e]));
      wave_amax(xcur, 0, mm);
      lds_barrier();
      ex = block_exp();
      stamp(22);
    } else if (PERSIST) {
      lds_barrier();  // every wave has read x from LDS (the copy the operand overwrites)
    }
    write_operand(xcur, exp2i(ex));
    write_margins(exp2i(ex));
    lds_barrier();
    stamp(2);

    // dilation pairs: xt = lrelu(conv1(lrelu(x)) + b1); x = x + (conv2(xt) + b2)
    if constexpr (FMT == kFmtBf16) {
      for (int cv = 0; cv < n_conv; cv += 2) {
        run_conv(cv);
        lds_barrier();
        write_operand(acc, 1.0f);
        lds_barrier();
        run_conv(cv + 1);
        lds_barrier();
#pragma unroll
        for (int i = 0; i < WM; ++i)
#pragma unroll
          for (int k = 0; k < WN; ++k)
#pragma unroll
            for (int r = 0; r < 16; ++r) xcur[i][k][r] = xcur[i][k][r] + acc[i][k][r];
        if (cv + 2 < n_conv) {
          write_operand(xcur, 1.0f);
          lds_barrier();
        }
      }
    } else {
      for (int cv = 0; cv < n_conv; cv += 2) {
        run_conv(cv);
        stamp(3 + 2 * cv);
        finalize(cv);
        if (cv > 0) radius += (KT - 1) / 2 * p.dil[cv];  // conv 0: exact (margins from x)
        wave_amax(acc, radius);
        lds_barrier();  // every wave is done reading the operand; the maxima are posted
        ex = block_exp();
        write_operand(acc, exp2i(ex));
        lds_barrier();
        stamp(4 + 2 * cv);
        run_conv(cv + 1);
        stamp(5 + 2 * cv);
        finalize(cv + 1);
        radius += (KT - 1) / 2;  // conv2: dilation 1
#pragma unroll
        for (int i = 0; i < WM; ++i)
#pragma unroll
          for (int k = 0; k < WN; ++k)
#pragma unroll
            for (int r = 0; r < 16; ++r) xcur[i][k][r] = xcur[i][k][r] + acc[i][k][r];
        if (cv + 2 < n_conv) {
          wave_amax(xcur, radius);
          lds_barrier();
          ex = block_exp();
          write_operand(xcur, exp2i(ex));
          lds_barrier();
        }
        stamp(6 + 2 * cv);
      }
    }

    // ---- the next window of a persistent block (block-uniform) ----
    int wn = w + wstride;
    if constexpr (PERSIST)
      while (wn < n_win && !valid(wn)) wn += wstride;
    const bool more = PERSIST && wn < n_win;

    // ---- MRF: (mrf + x) [/ n_res] on the window centre ----
    const __amdgpu_buffer_rsrc_t mrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.mrf + (int64_t)b * p.bs), 0, (int)0xFFFFFFFFu, 0x00020000);
    bool ok[WN];
    unsigned vo[WN];
#pragma unroll
    for (int k = 0; k < WN; ++k) {
      const int c = cbase + 32 * k + col;
      ok[k] = vk[k] && c >= c_lo && c < c_hi;
      vo[k] = ok[k] ? (lrow + (unsigned)(ws + c)) * 4u : 0u;
    }
    const bool skip_mrf = kAblate && (dbg & 16);  // ablation: no MRF epilogue
    // persistent grid: the next window's x copy is issued first, then the MRF loads, so the
    // two round trips overlap (one wait for both)
    int bn = b, len_n = len_b, wsn = ws;
    if (more) {
      bn = item_of(wn);
      len_n = len_of(bn);
      wsn = (wn - bn * n_tiles) * p.W - p.halo;
      lds_barrier();  // every wave is done reading the last conv's operand
      dma_x(wsn, bn);
    }
    // every MRF load is issued before any use (one wait for all 16 x WN), then the adds /
    // divisions for every tile; the empty asm keeps the compiler from sinking a tile's loads
    // into its store branch (which serialised one HBM round trip per element)
    // (the MRF values land in the accumulator registers, dead after the last conv: the
    // persistent variant has no VGPRs to spare for a separate set)
    floatx16 (&mv)[WM][WN] = acc;
    if (add && !skip_mrf) {
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int k = 0; k < WN; ++k)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            mv[i][k][r] = __builtin_bit_cast(
                float, __builtin_amdgcn_raw_buffer_load_b32(mrs, (int)vo[k], (int)srow(i, r), 0));
    }
    if (more) wait_vm<0>();  // the x copy (and the MRF values) have landed
    if (add && !skip_mrf) {
#if HFG_RB_TIMING
      wait_vm<0>();
      stamp(23);
#endif
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int k = 0; k < WN; ++k)
#pragma unroll
          for (int r = 0; r < 16; ++r) xcur[i][k][r] = mv[i][k][r] + xcur[i][k][r];
    }
    if (!skip_mrf) {
      if (div && p.mrf_rcp != 0.f) {
#pragma unroll
        for (int i = 0; i < WM; ++i)
#pragma unroll
          for (int k = 0; k < WN; ++k)
#pragma unroll
            for (int r = 0; r < 16; ++r) xcur[i][k][r] = div_fast(xcur[i][k][r], p.mrf_div, p.mrf_rcp);
      } else if (div) {
#pragma unroll
        for (int i = 0; i < WM; ++i)
#pragma unroll
          for (int k = 0; k < WN; ++k)
#pragma unroll
            for (int r = 0; r < 16; ++r) xcur[i][k][r] = xcur[i][k][r] / p.mrf_div;
      }
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int k = 0; k < WN; ++k)
#pragma unroll
          for (int r = 0; r < 16; ++r) asm volatile("" ::"v"(xcur[i][k][r]));
      if constexpr (C == 32) {
        if (post) conv_post_tail<NT, NWIN, WN>(p, xcur, ok, lds, b, len_b, t0, tid, cbase, half, col);
      }
#pragma unroll
      for (int k = 0; k < WN; ++k) {
        if (ok[k] && !post) {
#pragma unroll
          for (int i = 0; i < WM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              // through a scalar: __builtin_bit_cast of an ext_vector element lvalue compiled to
              // element 0 of the vector (every row stored the same value)
              const float v = xcur[i][k][r];
              __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), mrs, (int)vo[k], (int)srow(i, r), 0);
            }
        }
      }
      stamp(3 + 2 * n_conv);
      if (p.amax_out) {  // f16x3 consumers of the stage output (block-uniform branch)
        float m = 0.f;
#pragma unroll
        for (int k = 0; k < WN; ++k) {
          float mk = 0.f;
#pragma unroll
          for (int i = 0; i < WM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) mk = fmaxf(mk, fabsf(xcur[i][k][r]));
          m = ok[k] ? fmaxf(m, mk) : m;
        }
        amax_commit(m, p.amax_out, b);
      }
    } else if (xcur[0][0][0] == 1.2345e-30f) {
      p.mrf[0] = xcur[WM - 1][WN - 1][15];
    }
    if (!more) break;
    // ---- advance: the next window's x becomes the residual stream ----
    w = wn;
    b = bn;
    len_b = len_n;
    ws = wsn;
    t0 = ws + p.halo;
    set_vk();
    load_a(0, Q0);
    load_a(1, Q0 + 1);
    lds_barrier();  // every wave's x pieces are in LDS (each waited for its own above)
  }
#if HFG_RB_TIMING
  if (tid == 0) {
    tsv[4 + 2 * n_conv] = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < kRbTsSlots; ++i) ts[i] = tsv[i];
  }
#endif
}

namespace {

typedef void (*RbFn)(const RbParams);

struct EntryRb {
  int kt, waves_m, waves_n, wm, np, fmt;
  bool persist;
  RbFn fn;
  char name[64];
  int C() const { return 32 * wm * waves_m; }
  int nwin() const { return 32 * (4 / wm) * waves_n; }
};

#define HFGRB_ENTRY(KT, WMS, WNS, WM, NP, FMT, PS) \
  { KT, WMS, WNS, WM, NP, FMT, PS, resblock_bf16x3<KT, WMS, WNS, WM, NP, FMT, PS>, {0} }
#define HFGRB_KTS(WMS, WNS, WM, NP, FMT, PS)                                                 \
  HFGRB_ENTRY(3, WMS, WNS, WM, NP, FMT, PS), HFGRB_ENTRY(5, WMS, WNS, WM, NP, FMT, PS),      \
      HFGRB_ENTRY(7, WMS, WNS, WM, NP, FMT, PS), HFGRB_ENTRY(11, WMS, WNS, WM, NP, FMT, PS)
// 32-row waves (WM 1): C = 64 (2 x 4 waves), C = 32 (1 x 4), C = 128 (4 x 2, k = 3),
// C = 64 narrow (2 x 2, k = 3).  64-row waves (WM 2: half the LDS operand reads per MFMA,
// twice the weight-fragment loads) measured the same in a same-box A/B (round 4) and are not
// instantiated.
// Persistent variants (PERSIST: a grid of resident blocks walks the windows, each window's
// x copied to LDS beside the previous window's MRF round trip) for C = 64 with the
// 512-column window (one block per CU).  Measured and not built: C = 128 (+0.9 %) and
// C = 32 (two blocks per CU: +2 to +5 %), profiles/r05/ab.
#define HFGRB_SET(NP, FMT)                                                                   \
  HFGRB_KTS(2, 4, 1, NP, FMT, false), HFGRB_KTS(1, 4, 1, NP, FMT, false),                     \
      HFGRB_ENTRY(3, 4, 2, 1, NP, FMT, false), HFGRB_ENTRY(3, 2, 2, 1, NP, FMT, false),        \
      HFGRB_KTS(2, 4, 1, NP, FMT, true)

// bf16x3 (NP 3, bf16), f16x3 (NP 3, f16), bf16w (NP 2 on the f16 kernels)
EntryRb g_entriesRb[] = {HFGRB_SET(3, 0), HFGRB_SET(3, 1), HFGRB_SET(2, 1)};

EntryRb* find_rb(int C, int nwin, int wm, int kt, int np, int fmt, bool persist = false) {
  for (auto& e : g_entriesRb)
    if (e.kt == kt && e.C() == C && e.nwin() == nwin && e.wm == wm && e.np == np && e.fmt == fmt &&
        e.persist == persist)
      return &e;
  return nullptr;
}

}  // namespace

bool rb_supported(int C, int kt, int nwin, int wm) {
  return find_rb(C, nwin, wm, kt, 3, 0) != nullptr;
}

size_t rb_lds_bytes(int C, int nwin, int n_conv) {
  const size_t rows = (size_t)nwin + 2 * rb_marg(C, nwin);
  // operand planes, biases, the per-wave maxima of f16x3 (<= 16 waves)
  return (size_t)C * rows * 4 + sizeof(float) * ((size_t)n_conv * C + 16);
}

hipError_t launch_resblock_bf16x3(int C, int nwin, int wm, int kt, int fmt, int np,
                                  const RbParams& p_in, int batch, hipStream_t stream,
                                  const char** name) {
  RbParams p = p_in;
  p.batch = batch;
  // a persistent variant where one is built (one-block-per-CU shapes), else one window per block
  EntryRb* e = p.persist ? find_rb(C, nwin, wm, kt, np, fmt, true) : nullptr;
  if (!e) {
    p.persist = 0;
    e = find_rb(C, nwin, wm, kt, np, fmt);
  }
  if (!e) return hipErrorInvalidValue;
  if (p.n_conv < 2 || p.n_conv > kRbMaxConv || (p.n_conv & 1)) return hipErrorInvalidValue;
  if (p.conv0 < 0 || p.conv0 + p.n_conv > p.n_conv_stream) return hipErrorInvalidValue;
  if (p.W <= 0 || p.halo < 0 || p.W + 2 * p.halo > nwin) return hipErrorInvalidValue;
  if (p.wav && (C != 32 || wm != 1 || p.L % 4 || p.W % 4 || p.halo < 4 || !p.post_w || !p.post_b ||
                p.amax_out || p.persist))
    return hipErrorInvalidValue;
  if (p.persist < 0 || batch < 1) return hipErrorInvalidValue;
  for (int i = 0; i < p.n_conv; ++i)
    if (p.dil[i] < 1 || (kt - 1) / 2 * p.dil[i] > rb_marg(C, nwin)) return hipErrorInvalidValue;
  {
    std::lock_guard<std::mutex> lk(setup_mutex());
    if (!e->name[0])
      snprintf(e->name, sizeof(e->name), "resblock_bf16x3<%d, %d, %d, %d, %d, %d%s>", e->kt,
               e->waves_m, e->waves_n, e->wm, e->np, e->fmt, e->persist ? ", persist" : "");
  }
#if HFG_RB_TIMING
  const size_t lds = rb_lds_bytes(C, nwin, p.n_conv) + kRbTsSlots * 8;  // + the stamps
#else
  const size_t lds = rb_lds_bytes(C, nwin, p.n_conv);
#endif
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (hipError_t err = ensure_max_lds(reinterpret_cast<const void*>(e->fn)))
    return err;
  if (name) *name = e->name;
  const int n_tiles = (p.L + p.W - 1) / p.W;
  if (p.persist) {
    const int64_t n_win = (int64_t)n_tiles * batch;
    if (n_win >= (1ll << 31)) return hipErrorInvalidValue;
    const int g = (int)std::min<int64_t>(n_win, p.persist);
    e->fn<<<dim3(g, 1), dim3(64 * e->waves_m * e->waves_n), lds, stream>>>(p);
  } else {
    e->fn<<<dim3(n_tiles, batch), dim3(64 * e->waves_m * e->waves_n), lds, stream>>>(p);
  }
  return hipGetLastError();
}

}  // namespace hfg

#if HFG_RB_TIMING
extern "C" int hfg_debug_rb_ts(void* dst, size_t bytes) {
  if (bytes > sizeof(hfg::g_rb_ts)) bytes = sizeof(hfg::g_rb_ts);
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(hfg::g_rb_ts), bytes, 0, hipMemcpyDeviceToHost);
}
extern "C" int hfg_debug_rb_ts_clear() {
  static uint64_t* z = nullptr;
  if (!z) z = (uint64_t*)calloc(1, sizeof(hfg::g_rb_ts));
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(hfg::g_rb_ts), z, sizeof(hfg::g_rb_ts), 0, hipMemcpyHostToDevice);
}
#endif

// conv_kernels.hip — gfx950 (CDNA4) kernels of the HiFi-GAN Generator hot path.
//
// conv1d_mfma_f32: every Conv1d / ConvTranspose1d of the Generator as an
// implicit GEMM on the fp32 matrix cores (v_mfma_f32_32x32x2_f32, exact f32,
// 64 FLOP/clk/SIMD).  GEMM rows = output channels (or channel x phase for the
// polyphase ConvTranspose1d), GEMM columns = time, K = C_in x taps.
//
//   * A block owns an MT x NTILE output tile and walks C_in in chunks of CK.
//     Per chunk it stages into LDS
//       - the weight slab, already in MFMA A-fragment order (packed on the
//         host), by a straight coalesced float4 copy, and
//       - the input rows x[ci0:ci0+CK][n0+off : n0+off+NTILE+(KT-1)*dil]
//         with zero padding and the pre-activation leaky_relu applied once
//         per element (models/hifigan.py:81, :244, :254).
//   * Dilation only moves the B-fragment read offset (j*dil) inside the
//     staged rows: one x tile serves all KT taps.
//   * Each wave owns WM x WN 32x32 accumulators (16 AGPR/VGPR each);
//     A fragments come from LDS as one ds_read_b64 (WM=2), B fragments as
//     ds_read_b32 of 32 consecutive floats per half-wave (conflict-free).
//   * Epilogue fuses bias, the ResBlock residual add (models/hifigan.py:85),
//     the post-activation leaky_relu (:83), the MRF running sum and the final
//     division by len(resblocks) (:125-131), or the polyphase scatter of the
//     ConvTranspose1d (:245).
//
// conv_post_tanh: the 32->1, k=7 output conv + tanh (models/hifigan.py:254-256),
// an HBM-bound reduction over C*7 inputs per sample, LDS-staged.
#include <hip/hip_runtime.h>

#include <mutex>

#include <algorithm>

#include <cstdio>

#include "epilogue.h"
#include "kernels.h"

namespace hfg {

typedef floatx16e floatx16;
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gptr_t;

__device__ __forceinline__ float lrelu(float v) { return v > 0.f ? v : v * kLReluSlope; }

template <int KT_, int WM, int WN, int WAVES_M, int WAVES_N, int CK, bool UPS>
__global__ void __launch_bounds__(64 * WAVES_M * WAVES_N, 3)
conv1d_mfma_f32(const ConvParams p) {
  constexpr int NW = WAVES_M * WAVES_N;
  constexpr int NT = 64 * NW;
  constexpr int MT = 32 * WM * WAVES_M;
  constexpr int NTILE = 32 * WN * WAVES_N;
  constexpr int KK = CK / 2;
  static_assert(CK % 2 == 0, "CK must be even (K=2 per MFMA)");
  // input-staging slots per thread (upper bound over the halos this instance accepts)
  constexpr int XQ = (CK * (NTILE + halo_max(KT_)) + NT - 1) / NT;
  const int KT = KT_ > 0 ? KT_ : p.kt;
  const int XW = NTILE + (KT - 1) * p.dil;
  const int nx = CK * XW;
  const float inv_xw = 1.0f / (float)XW;
  const int wchunk = MT * CK * KT;            // floats per weight slab
  const int stage_sz = wchunk + ((nx + 3) & ~3);

  extern __shared__ __attribute__((aligned(16))) float lds[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wave_m = wave % WAVES_M;
  const int wave_n = wave / WAVES_M;
  const int n0 = blockIdx.x * NTILE;
  const int mt = blockIdx.y;
  const int b = blockIdx.z;
  const float* __restrict__ xb = p.x + (int64_t)b * p.x_bs;
  const float* __restrict__ wsrc = p.w + (int64_t)mt * p.n_chunks * wchunk;
  const int gbase = n0 + p.off;
  const int half = lane >> 5;  // K index inside the MFMA (0/1)
  const int col = lane & 31;   // GEMM column inside a 32-wide tile
  // ragged batches: this item's valid input / output extent
  const int L_in_b = p.len_in ? p.len_in[b] : p.L_in;
  int N_b = p.N;
  if (p.len_out) {
    const int lo = p.len_out[b];
    N_b = UPS ? (lo > 0 ? (lo - 1 + p.ups_p) / p.ups_s + 1 : 0) : lo;
  }
  if (n0 >= N_b) return;  // whole tile past this utterance's end (block-uniform)
  const int L_out_b = (UPS && p.len_out) ? p.len_out[b] : p.L_out;

  // ---- weight slab: async global -> LDS copy (global_load_lds_dwordx4) ----
  auto issue_w = [&](int c, float* Ws) {
    const float* src = wsrc + (int64_t)c * wchunk;
    const int n16 = wchunk >> 2;
    for (int i = wave; i * 64 < n16; i += NW) {
      const int piece = i * 64 + lane;
      if (piece < n16)
        __builtin_amdgcn_global_load_lds((gptr_t)(src + piece * 4), (lds_ptr_t)(Ws + i * 256), 16,
                                         0, 0);
    }
  };
  // ---- input rows: registers (zero padding, branch-free loads) ----
  float xv[XQ];
  auto load_x = [&](int c) {
    const int ci0 = c * CK;
#pragma unroll
    for (int q = 0; q < XQ; ++q) {
      const int i = tid + q * NT;
      const int ci = (int)(((float)i + 0.5f) * inv_xw);
      const int t = i - ci * XW;
      const int gi = gbase + t;
      const int cg = ci0 + ci;
      const bool ok = (i < nx) && (cg < p.C_in) && ((unsigned)gi < (unsigned)L_in_b);
      // byte offset from the block-uniform base (SGPR base + 32-bit VGPR offset load)
      const unsigned boff = ok ? (unsigned)(cg * (int)p.x_cs + gi * (int)p.x_ts) * 4u : 0u;
      const float v = *reinterpret_cast<const float*>(reinterpret_cast<const char*>(xb) + boff);
      xv[q] = ok ? v : 0.f;
    }
  };
  auto store_x = [&](float* Xs) {
#pragma unroll
    for (int q = 0; q < XQ; ++q) {
      const int i = tid + q * NT;
      float v = xv[q];
      if (p.act_in) v = lrelu(v);
      if (i < nx) Xs[i] = v;
    }
  };

  floatx16 acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int k = 0; k < WN; ++k)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][k][r] = 0.f;

  // fragment loads for MFMA step s = j*KK + kk of one stage
  auto load_frag = [&](const float* Ws, const float* Xs, int j, int kk, float (&a)[WM],
                       float (&bv)[WN]) {
    const float* wa = Ws + ((j * KK + kk) * WAVES_M + wave_m) * 64 * WM + lane * WM;
    if constexpr (WM == 2) {
      const float2 a2 = *reinterpret_cast<const float2*>(wa);
      a[0] = a2.x;
      a[1] = a2.y;
    } else {
#pragma unroll
      for (int i = 0; i < WM; ++i) a[i] = wa[i];
    }
    const float* xr = Xs + (2 * kk + half) * XW + wave_n * 32 * WN + col + j * p.dil;
#pragma unroll
    for (int k = 0; k < WN; ++k) bv[k] = xr[k * 32];
  };
  auto mma = [&](const float (&a)[WM], const float (&bv)[WN]) {
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int k = 0; k < WN; ++k)
        acc[i][k] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], bv[k], acc[i][k], 0, 0, 0);
  };

  // ---- prologue: stage chunk 0 ----
  issue_w(0, lds);
  load_x(0);
  store_x(lds + wchunk);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- main loop: compute chunk c from stage c&1 while chunk c+1 lands in the other ----
  for (int c = 0; c < p.n_chunks; ++c) {
    float* Ws = lds + (c & 1) * stage_sz;
    float* Xs = Ws + wchunk;
    float* Wn = lds + ((c + 1) & 1) * stage_sz;
    const bool has_next = c + 1 < p.n_chunks;
    if (has_next) {
      issue_w(c + 1, Wn);
      load_x(c + 1);
    }
    if constexpr (KT_ > 0) {
      constexpr int S = KT_ * KK;
      float a0[WM], b0[WN], a1[WM], b1[WN];
      load_frag(Ws, Xs, 0, 0, a0, b0);
#pragma unroll
      for (int s = 0; s < S; s += 2) {
        if (s + 1 < S) load_frag(Ws, Xs, (s + 1) / KK, (s + 1) % KK, a1, b1);
        mma(a0, b0);
        if (s + 2 < S) load_frag(Ws, Xs, (s + 2) / KK, (s + 2) % KK, a0, b0);
        if (s + 1 < S) mma(a1, b1);
      }
    } else {
      for (int j = 0; j < KT; ++j) {
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) {
          float a[WM], bv[WN];
          load_frag(Ws, Xs, j, kk, a, bv);
          mma(a, bv);
        }
      }
    }
    if (has_next) store_x(Wn + wchunk);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue ----
  if constexpr (UPS) {
    float vmax = 0.f;  // max |stored value| (f16x3 consumers: p.amax_out)
#pragma unroll
    for (int i = 0; i < WM; ++i) {
      float bv[16];  // batch the bias loads ahead of the scattered stores
#pragma unroll
      for (int r = 0; r < 16; ++r)
        bv[r] = p.bias[mt * MT + wave_m * 32 * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half];
#pragma unroll
      for (int k = 0; k < WN; ++k) {
        const int n = n0 + wave_n * 32 * WN + k * 32 + col;
        if (n >= N_b) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = mt * MT + wave_m * 32 * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
          if (row >= p.M) continue;
          const float v = acc[i][k][r] + bv[r];
          const int co = row / p.ups_s;
          const int ph = row - co * p.ups_s;
          const int t = n * p.ups_s + ph - p.ups_p;
          if (t >= 0 && t < L_out_b) {
            p.y[(int64_t)b * p.y_bs + (int64_t)co * p.L_out + t] = v;
            vmax = fmaxf(vmax, fabsf(v));
          }
        }
      }
    }
    if (p.amax_out) amax_commit(vmax, p.amax_out, b);
  } else if (p.epi_lds && (p.N & 3) == 0) {
    // LDS-staged float4 epilogue (epilogue.h; the host sized the LDS for it)
    // every wave is done with the main loop's LDS and no weight LDS-DMA is in flight
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    conv_epilogue_lds<WM, WN>(p, acc, b, mt * MT + wave_m * 32 * WM, n0 + wave_n * 32 * WN, N_b,
                              half, col, lds + (threadIdx.x >> 6) * 32 * (32 * WN + 8),
                              threadIdx.x & 63);
  } else {
    conv_epilogue<WM, WN>(p, acc, b, mt * MT + wave_m * 32 * WM, n0 + wave_n * 32 * WN, N_b,
                          half, col);
  }
}

// conv_post (C -> 1, k=7, pad=3) + tanh over lrelu(x).  One thread per sample; the
// 256-sample tile's input rows are staged in LDS kConvPostCB channels at a time (the
// halo columns are shared between neighbouring threads), so any channel count fits.
__global__ void __launch_bounds__(256)
conv_post_tanh(const float* __restrict__ x, int64_t x_bs, int C, int L, const float* __restrict__ w,
               const float* __restrict__ bias, float* __restrict__ wav,
               const int32_t* __restrict__ lens) {
  constexpr int TT = 256, KP = 7, HALO = 3;
  constexpr int XW = TT + KP - 1;
  constexpr int CBLK = kConvPostCB;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* Ws = lds;              // C*7
  float* Xs = lds + ((C * KP + 3) & ~3);  // CBLK*XW
  const int t0 = blockIdx.x * TT;
  const int b = blockIdx.y;
  const float* xb = x + (int64_t)b * x_bs;
  const int Lb = lens ? lens[b] : L;
  if (t0 >= Lb) {  // past this utterance's end: zeros
    const int t = t0 + threadIdx.x;
    if (t < L) wav[(int64_t)b * L + t] = 0.f;
    return;
  }
  for (int i = threadIdx.x; i < C * KP; i += TT) Ws[i] = w[i];
  // staging: each thread loads its column (and the first KP-1 threads one halo column)
  // of CB channels at a time, all loads in flight before any use (one memory round trip
  // per CB channels instead of one per channel)
  constexpr int CB = 8;
  const int tt = threadIdx.x;
  const int gm = t0 - HALO + tt;       // main column
  const int gh = t0 - HALO + TT + tt;  // halo column (tt < KP - 1), always >= 0
  const bool okm = gm >= 0 && gm < Lb;
  const bool okh = tt < KP - 1 && gh < Lb;
  float acc = 0.f;
  for (int cb = 0; cb < C; cb += CBLK) {
    const int nc = min(CBLK, C - cb);
    if (cb > 0) __syncthreads();  // the previous block's rows are consumed
    for (int c0 = 0; c0 < nc; c0 += CB) {
      float vm[CB], vh[CB];
#pragma unroll
      for (int e = 0; e < CB; ++e) {
        const int64_t row = (int64_t)(cb + min(c0 + e, nc - 1)) * L;
        vm[e] = xb[okm ? row + gm : 0];
        vh[e] = xb[okh ? row + gh : 0];
      }
#pragma unroll
      for (int e = 0; e < CB; ++e) {
        if (c0 + e >= nc) break;
        Xs[(c0 + e) * XW + tt] = okm ? lrelu(vm[e]) : 0.f;
        if (tt < KP - 1) Xs[(c0 + e) * XW + TT + tt] = okh ? lrelu(vh[e]) : 0.f;
      }
    }
    __syncthreads();
    for (int c = 0; c < nc; ++c) {
      const float* xs = Xs + c * XW + threadIdx.x;
      const float* ws = Ws + (cb + c) * KP;
#pragma unroll
      for (int j = 0; j < KP; ++j) acc = fmaf(ws[j], xs[j], acc);
    }
  }
  const int t = t0 + threadIdx.x;
  if (t >= L) return;
  wav[(int64_t)b * L + t] = t >= Lb ? 0.f : tanhf(acc + bias[0]);
}

// conv_post + tanh for L % 4 == 0 (every V1 / V2* wav): four consecutive samples per
// thread, no LDS and no barrier.  Per channel a thread reads the 16-B quads at t - 4, t and
// t + 4 (its neighbours' quads: the same cache lines, so HBM bytes stay one pass over x),
// eight channels' loads in flight at a time; quads outside the row read offset 0 (masked).  Per output the sum runs over (channel, tap) in the order conv_post_tanh
// uses (channel-major, fma from 0, bias last): bitwise its result.
__global__ void __launch_bounds__(256)
conv_post4_tanh(const float* __restrict__ x, int64_t x_bs, int C, int L, const float* __restrict__ w,
                const float* __restrict__ bias, float* __restrict__ wav,
                const int32_t* __restrict__ lens) {
  constexpr int KP = 7, CB = 8;
  typedef float f4 __attribute__((ext_vector_type(4)));
  const int b = blockIdx.y;
  const int t = (blockIdx.x * 256 + threadIdx.x) * 4;  // first of this thread's 4 samples
  if (t >= L) return;
  const int Lb = lens ? min(lens[b], L) : L;
  float* out = wav + (int64_t)b * L + t;
  if (t >= Lb) {  // past this utterance's end: zeros
    *reinterpret_cast<f4*>(out) = f4{0.f, 0.f, 0.f, 0.f};
    return;
  }
  // an item holds fewer than 2^30 floats: byte offsets from the item base fit 32 bits (a
  // buffer descriptor cannot: a 4-GiB item's range does not fit its 32-bit record count)
  const char* xb = reinterpret_cast<const char*>(x + (int64_t)b * x_bs);
  // the three quads [t-4, t), [t, t+4), [t+4, t+8); element k of v = x[t - 4 + k]
  const bool okq[3] = {t - 4 >= 0, true, t + 4 < L};
  bool okv[12];
#pragma unroll
  for (int k = 0; k < 12; ++k) okv[k] = (unsigned)(t - 4 + k) < (unsigned)Lb;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int c0 = 0; c0 < C; c0 += CB) {
    f4 q[CB][3];
#pragma unroll
    for (int e = 0; e < CB; ++e) {
      const int c = min(c0 + e, C - 1);
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        const unsigned off = okq[s] ? (unsigned)(c * L + t - 4 + 4 * s) * 4u : 0u;
        q[e][s] = *reinterpret_cast<const f4*>(xb + off);
      }
    }
    // every load of the batch issued before the first use: left alone, the compiler sank
    // each channel's loads past the loop-exit test below to their uses (28 VGPRs, one memory
    // round trip per channel); an empty asm that takes every value pins them here (same-box
    // C1 / streaming-chunk A/B: -0.5 to -2 %, profiles/r06/c1/c1_ab_post.txt)
#pragma unroll
    for (int e = 0; e < CB; ++e)
#pragma unroll
      for (int s = 0; s < 3; ++s) asm volatile("" : "+v"(q[e][s]));
#pragma unroll
    for (int e = 0; e < CB; ++e) {
      if (c0 + e >= C) break;
      float v[12];
#pragma unroll
      for (int k = 0; k < 12; ++k) {
        const float r = q[e][k >> 2][k & 3];
        v[k] = okv[k] ? lrelu(r) : 0.f;
      }
      const float* ws = w + (c0 + e) * KP;
#pragma unroll
      for (int o = 0; o < 4; ++o)
#pragma unroll
        for (int j = 0; j < KP; ++j) acc[o] = fmaf(ws[j], v[o + j + 1], acc[o]);
    }
  }
  f4 r;
#pragma unroll
  for (int o = 0; o < 4; ++o) r[o] = t + o >= Lb ? 0.f : tanhf(acc[o] + bias[0]);
  *reinterpret_cast<f4*>(out) = r;
}

// ------------------------------------------------------------------------
// dispatch
// ------------------------------------------------------------------------
namespace {

typedef void (*ConvFn)(const ConvParams);

template <int KT, int TILE, bool UPS>
struct Inst {
  static constexpr TileCfg t = kTiles[TILE];
  static ConvFn fn() {
    return conv1d_mfma_f32<KT, t.WM, t.WN, t.WAVES_M, t.WAVES_N, ck_for(KT, TILE), UPS>;
  }
};

struct Entry {
  int kt;
  int tile;
  bool ups;
  ConvFn fn;
  char name[96];  // template-instance name as rocprofv3 prints it
};

#define HFG_ENTRY(KT, TILE, UPS) \
  { KT, TILE, UPS, Inst<KT, TILE, UPS>::fn(), {0} }

#define HFG_ENTRIES_KT(KT, UPS) \
  HFG_ENTRY(KT, 0, UPS), HFG_ENTRY(KT, 1, UPS), HFG_ENTRY(KT, 2, UPS)

Entry g_entries[] = {
    HFG_ENTRIES_KT(3, false), HFG_ENTRIES_KT(5, false), HFG_ENTRIES_KT(7, false),
    HFG_ENTRIES_KT(11, false), HFG_ENTRIES_KT(2, false), HFG_ENTRIES_KT(0, false),
    HFG_ENTRIES_KT(2, true),   HFG_ENTRIES_KT(3, true),  HFG_ENTRIES_KT(0, true),
};

}  // namespace

hipError_t launch_conv(TileId tile, int kt, bool ups, const ConvParams& p, int n_tiles,
                       int m_tiles, int batch, hipStream_t stream, const char** name) {
  Entry* e = nullptr;
  Entry* generic = nullptr;
  for (auto& cand : g_entries) {
    if (cand.tile != tile || cand.ups != ups) continue;
    if (cand.kt == kt) e = &cand;
    if (cand.kt == 0) generic = &cand;
  }
  if (!e) e = generic;
  if (!e) return hipErrorInvalidValue;
  const TileCfg& t = kTiles[tile];
  const int ck = ck_for(e->kt, tile);
  {
    std::lock_guard<std::mutex> lk(setup_mutex());
    if (!e->name[0])
      snprintf(e->name, sizeof(e->name), "conv1d_mfma_f32<%d, %d, %d, %d, %d, %d, %s>", e->kt, t.WM,
               t.WN, t.WAVES_M, t.WAVES_N, ck, e->ups ? "true" : "false");
  }
  if ((kt - 1) * p.dil > halo_max(e->kt)) return hipErrorInvalidValue;
  const int xw = t.NTILE() + (kt - 1) * p.dil;
  const size_t stage = (size_t)t.MT() * ck * kt + (((size_t)ck * xw + 3) & ~(size_t)3);
  size_t lds = sizeof(float) * 2 * stage;
  // the LDS-staged epilogue only where its staging fits the main loop's footprint
  ConvParams pe = p;
  const size_t epi = sizeof(float) * (size_t)t.threads() / 64 * 32 * (32 * t.WN + 8);
  if (ups || epi > lds) pe.epi_lds = 0;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (hipError_t err = ensure_max_lds(reinterpret_cast<const void*>(e->fn)))
    return err;
  if (name) *name = e->name;
  dim3 grid(n_tiles, m_tiles, batch);
  e->fn<<<grid, dim3(t.threads()), lds, stream>>>(pe);
  return hipGetLastError();
}

hipError_t launch_conv_post(const float* x, int64_t x_bs, int C, int L, const float* w,
                            const float* bias, float* wav, const int32_t* lens, int batch,
                            hipStream_t stream, const char** name, bool quad) {
  if (quad && conv_post4_ok(L) && (int64_t)C * L <= ((int64_t)1 << 30)) {
    if (name) *name = "conv_post4_tanh";
    dim3 grid((L / 4 + 255) / 256, batch);
    conv_post4_tanh<<<grid, dim3(256), 0, stream>>>(x, x_bs, C, L, w, bias, wav, lens);
    return hipGetLastError();
  }
  const size_t lds = conv_post_lds_bytes(C);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (hipError_t err = ensure_max_lds(reinterpret_cast<const void*>(conv_post_tanh)))
    return err;
  if (name) *name = "conv_post_tanh";
  dim3 grid((L + 255) / 256, batch);
  conv_post_tanh<<<grid, dim3(256), lds, stream>>>(x, x_bs, C, L, w, bias, wav, lens);
  return hipGetLastError();
}

__global__ void stage_lengths_kernel(const int32_t* __restrict__ lens, int B, StageLenParams sp,
                                     int32_t* __restrict__ out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  int L = lens ? lens[b] : sp.T;
  L = L < 0 ? 0 : (L > sp.T ? sp.T : L);
  out[b] = L;
  for (int s = 0; s < sp.n_up; ++s) {
    const int u = sp.up_rates[s], k = sp.up_kernels[s];
    const int d = k - u;
    const int pad = d >= 0 ? d / 2 : -((-d + 1) / 2);  // Python floor division
    L = L > 0 ? (L - 1) * u - 2 * pad + k : 0;
    out[(s + 1) * B + b] = L;
  }
}

hipError_t launch_stage_lengths(const int32_t* lens, int B, const StageLenParams& sp,
                                int32_t* out, hipStream_t stream) {
  stage_lengths_kernel<<<dim3((B + 255) / 256), dim3(256), 0, stream>>>(lens, B, sp, out);
  return hipGetLastError();
}

// MRF mean of ResBlock outputs computed on concurrent streams (models/hifigan.py:125-131):
// y = (((o_0 + o_1) + o_2) + ...) / n, the same additions in the same order as the
// sequential schedule's epilogue running sum, so the result is bitwise the same.
// float4 over [B][C][L] rows (L % 4 == 0) with a scalar tail; columns past len[b] skipped.
// An item holds < 2^30 elements (the C ABI's limit), so offsets within it are 32-bit.  The
// grid is capped near two blocks per CU and each block folds its max into one atomic: a grid
// that finishes all at once queues its scale atomics on the item's slot lines (kernels.h;
// round 6: 48 us for 8192 waves on the 2-line slots at C1).
#ifndef HFG_COMBINE_BLOCKS
#define HFG_COMBINE_BLOCKS 512
#endif
template <int NMAX>
__device__ __forceinline__ void mrf_combine_body(const MrfCombineArgs& a, int b, float& vmax) {
  const int len_b = a.len ? min(a.len[b], a.L) : a.L;
  const int64_t base = (int64_t)b * a.C * a.L;
  const int n = a.C * a.L;
  const float* o[NMAX];
#pragma unroll
  for (int j = 0; j < NMAX; ++j) o[j] = a.o[j < a.n ? j : 0] + base;
  float* y = a.y + base;
  const int stride = gridDim.x * 256 * 4;
  for (int i = (blockIdx.x * 256 + threadIdx.x) * 4; i < n; i += stride) {
    const int t = i % a.L;
    if ((a.L & 3) == 0) {
      // 4 samples of one channel row (L % 4 == 0): one test for the group
      if (t >= len_b) continue;
      // every operand's load issued before the first addition
      float4 v[NMAX];
#pragma unroll
      for (int j = 0; j < NMAX; ++j)
        if (j < a.n) v[j] = *reinterpret_cast<const float4*>(o[j] + i);
      float4 acc = v[0];
#pragma unroll
      for (int j = 1; j < NMAX; ++j)
        if (j < a.n) {
          acc.x = acc.x + v[j].x;
          acc.y = acc.y + v[j].y;
          acc.z = acc.z + v[j].z;
          acc.w = acc.w + v[j].w;
        }
      acc.x = acc.x / a.div;
      acc.y = acc.y / a.div;
      acc.z = acc.z / a.div;
      acc.w = acc.w / a.div;
      *reinterpret_cast<float4*>(y + i) = acc;
      vmax = fmaxf(vmax, fmaxf(fmaxf(fabsf(acc.x), fabsf(acc.y)), fmaxf(fabsf(acc.z), fabsf(acc.w))));
    } else {
      // a group of 4 can straddle two channel rows: each sample tests its own column
      // (skipping the group on its first sample's column lost the next row's first
      // samples of a ragged item)
      for (int e = 0; e < 4 && i + e < n; ++e) {
        if ((t + e) % a.L >= len_b) continue;
        float acc = o[0][i + e];
        for (int j = 1; j < NMAX; ++j)
          if (j < a.n) acc = acc + o[j][i + e];
        y[i + e] = acc / a.div;
        vmax = fmaxf(vmax, fabsf(acc / a.div));
      }
    }
  }
}

__global__ void __launch_bounds__(256) mrf_combine_kernel(MrfCombineArgs a) {
  const int b = blockIdx.y;
  float vmax = 0.f;  // max |stored value| (f16x3 consumers: a.amax_out)
  if (a.n <= 3)
    mrf_combine_body<3>(a, b, vmax);
  else
    mrf_combine_body<kMrfCombineMax>(a, b, vmax);
  if (!a.amax_out) return;
  __shared__ float wmax[4];
  vmax = wave_max(vmax);
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = vmax;
  __syncthreads();
  if (threadIdx.x < 64) amax_commit(threadIdx.x < 4 ? wmax[threadIdx.x] : 0.f, a.amax_out, b);
}

hipError_t launch_mrf_combine(const MrfCombineArgs& a, int batch, hipStream_t stream) {
  if (a.n < 1 || a.n > kMrfCombineMax || batch < 1) return hipErrorInvalidValue;
  if ((int64_t)a.C * a.L >= (int64_t{1} << 30)) return hipErrorInvalidValue;
  const int64_t n4 = ((int64_t)a.C * a.L + 3) / 4;
  // about two blocks per CU over the whole batch (the launch is HBM-bound: 256 CUs x 2 x 256
  // threads keep enough float4 loads in flight), at least one block per item
  const int64_t cap = std::max<int64_t>(1, HFG_COMBINE_BLOCKS / batch);
  const int gx = (int)std::min<int64_t>((n4 + 255) / 256, cap);
  mrf_combine_kernel<<<dim3(gx, batch), dim3(256), 0, stream>>>(a);
  return hipGetLastError();
}

// max |x| per item over its valid columns, folded into out[b] (one atomic per wave).  The
// item is walked as rows of its contiguous dimension: channels x [0, len) for [C][T]
// (x_ts == 1), frames [0, len) x channels for [T][C] (x_cs == 1) — no per-element division.
__global__ void __launch_bounds__(256)
absmax_kernel(const float* __restrict__ x, int64_t x_bs, int64_t x_cs, int64_t x_ts, int C, int L,
              const int32_t* __restrict__ len, uint32_t* __restrict__ out) {
  const int b = blockIdx.y;
  const int len_b = len ? min(max(len[b], 0), L) : L;
  const float* xb = x + (int64_t)b * x_bs;
  const bool tc = x_ts == 1;  // [C][T]: rows = channels
  const int rows = tc ? C : len_b, row_len = tc ? len_b : C;
  const int64_t rs = tc ? x_cs : x_ts;
  float m = 0.f;
  for (int r = blockIdx.x; r < rows; r += gridDim.x)
    for (int i = threadIdx.x; i < row_len; i += 256) m = fmaxf(m, fabsf(xb[r * rs + i]));
  amax_commit(m, out, b);
}

hipError_t launch_absmax(const float* x, int64_t x_bs, int64_t x_cs, int64_t x_ts, int C, int L,
                         const int32_t* len, int batch, uint32_t* out, hipStream_t stream) {
  const int rows = x_ts == 1 ? C : L;
  const int gx = rows < 256 ? (rows > 0 ? rows : 1) : 256;
  absmax_kernel<<<dim3(gx, batch), dim3(256), 0, stream>>>(x, x_bs, x_cs, x_ts, C, L, len, out);
  return hipGetLastError();
}

bool fp32_conv_supported(int tile, int kt, int dil) {
  const int dkt = dispatch_kt(kt);
  if (kt < 1 || dil < 1 || (kt - 1) * dil > halo_max(dkt)) return false;
  const TileCfg& t = kTiles[tile];
  const int ck = ck_for(dkt, tile);
  const int xw = t.NTILE() + (kt - 1) * dil;
  const size_t stage = (size_t)t.MT() * ck * kt + (((size_t)ck * xw + 3) & ~(size_t)3);
  return sizeof(float) * 2 * stage <= 160 * 1024;
}

// Order-independent 32-bit content hash of fp32 tensors (the drop-in module's check that
// its parameters did not change behind its back, e.g. through ``param.data``): every
// word is mixed with its index and the mixes are summed mod 2^32 (vector atomics).
__device__ __forceinline__ uint32_t ck_mix(uint32_t w, uint32_t i) {
  uint32_t h = w * 0x9E3779B1u ^ (i * 0x85EBCA77u + 0x165667B1u);
  h ^= h >> 15;
  h *= 0xC2B2AE3Du;
  h ^= h >> 13;
  return h;
}

__global__ void __launch_bounds__(256) checksum_kernel(ChecksumArgs a, uint32_t* __restrict__ out) {
  const int t = blockIdx.y;
  const uint32_t* p = a.p[t];
  const int64_t n = a.n[t];
  uint32_t acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    acc += ck_mix(p[i], (uint32_t)i);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(out + a.base + t, acc);
}

hipError_t launch_checksum(const ChecksumArgs& a, uint32_t* out, hipStream_t stream) {
  int64_t mx = 1;
  for (int i = 0; i < a.count; ++i) mx = a.n[i] > mx ? a.n[i] : mx;
  const int64_t want = (mx + 256 * 8 - 1) / (256 * 8);
  const int gx = (int)(want < 512 ? want : 512);
  checksum_kernel<<<dim3(gx, a.count), dim3(256), 0, stream>>>(a, out);
  return hipGetLastError();
}

}  // namespace hfg

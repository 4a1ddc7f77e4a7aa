// conv_bf16x3.hip — split-precision ("bf16x3") implicit-GEMM Conv1d on the
// gfx950 bf16 matrix cores (v_mfma_f32_32x32x16_bf16, 16x the f32 MFMA rate).
//
// Every fp32 operand v is split as hi = bf16(v), lo = bf16(v - hi) and the
// product is accumulated in fp32 as hi*hi + hi*lo + lo*hi (the lo*lo term,
// 2^-16 relative, is dropped).  Three bf16 MFMAs per product = 5.3x the fp32
// MFMA throughput at ~16-bit-mantissa product accuracy; measured output error on
// the Generator is ~1e-6 against the 1e-4 bar (plain bf16 fails it: 2.8e-4).
//
// GEMM mapping: M = output channels, N = time, K = (tap, channel).  One MFMA
// k-step covers 16 input channels of ONE tap (lane half h holds channels 8h..8h+7).
//   * A (weights): split and packed on the host in fragment order
//     [m_tile][ch_group][tap_group][tap][plane hi/lo][wave_m][wm][lane][8],
//     so a chunk's slab is one contiguous run copied to LDS by
//     global_load_lds_dwordx4 (no VGPRs, no conversion on the device).
//   * B (activations): staged transposed as [t][16 ch] bf16 planes (hi, lo),
//     row stride 48 B (conflict-free ds_read_b128); pre-activation leaky_relu
//     and the split happen once per element at staging.
// A chunk = 16 channels x TPC taps; two LDS stages (chunk c+1 lands while chunk c
// is multiplied), one barrier per chunk.  Epilogue identical to conv1d_mfma_f32.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "kernels.h"

namespace hfg {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void* lds_ptr_t3;
typedef __attribute__((address_space(1))) void* gptr_t1;

__device__ __forceinline__ float lrelu3(float v) { return v > 0.f ? v : v * kLReluSlope; }

template <int KT_, int TPC, int WAVES_M, int WAVES_N, int WM, int WN>
__global__ void __launch_bounds__(64 * WAVES_M * WAVES_N, 2)
conv1d_bf16x3(const ConvParams p) {
  constexpr int NW = WAVES_M * WAVES_N;
  constexpr int NT = 64 * NW;
  constexpr int MT = 32 * WM * WAVES_M;
  constexpr int NTILE = 32 * WN * WAVES_N;
  constexpr int XROW = 24;                        // bf16 per staged row: 16 ch + 8 pad (48 B)
  constexpr int TAP_ELEMS = 2 * WAVES_M * WM * 64 * 8;  // bf16 per tap of a slab (hi+lo)
  constexpr int SLAB = TPC * TAP_ELEMS;           // bf16 per chunk slab
  constexpr int XW_MAX = NTILE + (TPC - 1) * kMaxDil;
  constexpr int XQ = (2 * XW_MAX + NT - 1) / NT;  // staging tasks per thread
  const int KT = KT_ > 0 ? KT_ : p.kt;
  const int n_tg = (KT + TPC - 1) / TPC;          // tap groups per channel group
  const int XW = NTILE + (TPC - 1) * p.dil;       // staged rows per chunk
  const int xplane = XW * XROW;                   // bf16 per X plane
  const int stage_elems = SLAB + 2 * ((xplane + 7) & ~7);

  extern __shared__ __attribute__((aligned(16))) __bf16 lds16[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wave_m = wave % WAVES_M;
  const int wave_n = wave / WAVES_M;
  const int n0 = blockIdx.x * NTILE;
  const int mt = blockIdx.y;
  const int b = blockIdx.z;
  const int half = lane >> 5;
  const int col = lane & 31;
  const float* __restrict__ xb = p.x + (int64_t)b * p.x_bs;
  const __bf16* __restrict__ wsrc =
      reinterpret_cast<const __bf16*>(p.w) + (int64_t)mt * p.n_chunks * SLAB;
  const int L_in_b = p.len_in ? p.len_in[b] : p.L_in;
  const int N_b = p.len_out ? p.len_out[b] : p.N;
  if (n0 >= N_b) return;  // whole tile past this utterance's end (block-uniform)

  auto taps_in = [&](int c) {
    const int tg = c % n_tg;
    const int rem = KT - tg * TPC;
    return rem < TPC ? rem : TPC;
  };
  // ---- weight slab: global -> LDS by LDS-DMA, only the taps that exist ----
  auto issue_w = [&](int c, __bf16* Ws) {
    const __bf16* src = wsrc + (int64_t)c * SLAB;
    const int n16 = taps_in(c) * TAP_ELEMS / 8;  // 16-B pieces
    for (int i = wave; i * 64 < n16; i += NW) {
      const int piece = i * 64 + lane;
      if (piece < n16)
        __builtin_amdgcn_global_load_lds((gptr_t1)(src + piece * 8), (lds_ptr_t3)(Ws + i * 512),
                                         16, 0, 0);
    }
  };
  // ---- activations: 8 channels of one time step per task, in registers ----
  float xv[XQ][8];
  auto load_x = [&](int c) {
    const int g = c / n_tg, tg = c % n_tg;
    const int ws = n0 + p.off + tg * TPC * p.dil;
#pragma unroll
    for (int q = 0; q < XQ; ++q) {
      const int i = tid + q * NT;
      const int t = i >> 1;
      const int cb = g * 16 + (i & 1) * 8;
      const int gi = ws + t;
      const bool tok = (i < 2 * XW) && ((unsigned)gi < (unsigned)L_in_b);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const bool ok = tok && (cb + e < p.C_in);
        const int64_t idx = ok ? (int64_t)(cb + e) * p.x_cs + (int64_t)gi * p.x_ts : 0;
        const float v = xb[idx];
        xv[q][e] = ok ? v : 0.f;
      }
    }
  };
  auto store_x = [&](__bf16* Xh) {
    __bf16* Xl = Xh + ((xplane + 7) & ~7);
#pragma unroll
    for (int q = 0; q < XQ; ++q) {
      const int i = tid + q * NT;
      if (i < 2 * XW) {
        bf16x8 h, l;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float v = xv[q][e];
          if (p.act_in) v = lrelu3(v);
          const __bf16 hh = (__bf16)v;
          h[e] = hh;
          l[e] = (__bf16)(v - (float)hh);
        }
        const int off = (i >> 1) * XROW + (i & 1) * 8;
        *reinterpret_cast<bf16x8*>(Xh + off) = h;
        *reinterpret_cast<bf16x8*>(Xl + off) = l;
      }
    }
  };

  floatx16 acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int k = 0; k < WN; ++k)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][k][r] = 0.f;

  struct Frag {
    bf16x8 ah[WM], al[WM], bh[WN], bl[WN];
  };
  auto load_frag = [&](const __bf16* Ws, const __bf16* Xh, int jj, Frag& f) {
    const __bf16* Xl = Xh + ((xplane + 7) & ~7);
#pragma unroll
    for (int i = 0; i < WM; ++i) {
      const __bf16* a = Ws + jj * TAP_ELEMS + ((0 * WAVES_M + wave_m) * WM + i) * 512 + lane * 8;
      f.ah[i] = *reinterpret_cast<const bf16x8*>(a);
      f.al[i] = *reinterpret_cast<const bf16x8*>(a + WAVES_M * WM * 512);
    }
#pragma unroll
    for (int k = 0; k < WN; ++k) {
      const int t = wave_n * 32 * WN + k * 32 + col + jj * p.dil;
      const int off = t * XROW + half * 8;
      f.bh[k] = *reinterpret_cast<const bf16x8*>(Xh + off);
      f.bl[k] = *reinterpret_cast<const bf16x8*>(Xl + off);
    }
  };
  auto mma = [&](const Frag& f) {
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int k = 0; k < WN; ++k) {
        acc[i][k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.al[i], f.bh[k], acc[i][k], 0, 0, 0);
        acc[i][k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.ah[i], f.bl[k], acc[i][k], 0, 0, 0);
        acc[i][k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.ah[i], f.bh[k], acc[i][k], 0, 0, 0);
      }
  };

  // ---- prologue ----
  issue_w(0, lds16);
  load_x(0);
  store_x(lds16 + SLAB);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int c = 0; c < p.n_chunks; ++c) {
    __bf16* Ws = lds16 + (c & 1) * stage_elems;
    __bf16* Xh = Ws + SLAB;
    __bf16* Wn = lds16 + ((c + 1) & 1) * stage_elems;
    const bool has_next = c + 1 < p.n_chunks;
    if (has_next) {
      issue_w(c + 1, Wn);
      load_x(c + 1);
    }
    const int nt = taps_in(c);
    Frag f0, f1;
    load_frag(Ws, Xh, 0, f0);
#pragma unroll
    for (int jj = 0; jj < TPC; jj += 2) {
      if (jj < nt) {
        if (jj + 1 < nt) load_frag(Ws, Xh, jj + 1, f1);
        mma(f0);
        if (jj + 2 < nt) load_frag(Ws, Xh, jj + 2, f0);
        if (jj + 1 < nt) mma(f1);
      }
    }
    if (has_next) store_x(Wn + SLAB);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue (same contract as conv1d_mfma_f32) ----
#pragma unroll
  for (int i = 0; i < WM; ++i) {
#pragma unroll
    for (int k = 0; k < WN; ++k) {
      const int n = n0 + wave_n * 32 * WN + k * 32 + col;
      if (n >= N_b) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = mt * MT + wave_m * 32 * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
        if (row >= p.M) continue;
        float v = acc[i][k][r] + p.bias[row];
        const int64_t o = (int64_t)b * p.y_bs + (int64_t)row * p.N + n;
        if (p.res) v = p.res[o] + v;
        if (p.act_out) v = lrelu3(v);
        if (p.mrf) {
          float m = (p.mrf_mode & 1) ? p.mrf[o] + v : v;
          if (p.mrf_mode & 2) m = m / p.mrf_div;
          p.mrf[o] = m;
        } else {
          p.y[o] = v;
        }
      }
    }
  }
}

namespace {

typedef void (*ConvFn3)(const ConvParams);

template <int KT, int TILE>
struct Inst3 {
  static constexpr Bf16x3Cfg t = kBf16x3Tiles[TILE];
  static ConvFn3 fn() {
    return conv1d_bf16x3<KT, kBf16x3Tpc, t.WAVES_M, t.WAVES_N, t.WM, t.WN>;
  }
};

struct Entry3 {
  int kt;
  int tile;
  ConvFn3 fn;
  bool attr;
  char name[96];
};

#define HFG3_ENTRY(KT, TILE) \
  { KT, TILE, Inst3<KT, TILE>::fn(), false, {0} }

Entry3 g_entries3[] = {
    HFG3_ENTRY(3, 0), HFG3_ENTRY(5, 0), HFG3_ENTRY(7, 0), HFG3_ENTRY(11, 0), HFG3_ENTRY(0, 0),
    HFG3_ENTRY(3, 1), HFG3_ENTRY(5, 1), HFG3_ENTRY(7, 1), HFG3_ENTRY(11, 1), HFG3_ENTRY(0, 1),
};

}  // namespace

size_t bf16x3_lds_bytes(int tile, int dil) {
  const Bf16x3Cfg& t = kBf16x3Tiles[tile];
  const size_t slab = (size_t)kBf16x3Tpc * 2 * t.MT() * 16;  // bf16: taps x planes x rows x 16 ch
  const int xw = t.NTILE() + (kBf16x3Tpc - 1) * dil;
  const size_t xplane = ((size_t)xw * 24 + 7) & ~(size_t)7;
  return 2 * sizeof(__bf16) * (slab + 2 * xplane);
}

hipError_t launch_conv_bf16x3(int tile, int kt, const ConvParams& p, int n_tiles, int m_tiles,
                              int batch, hipStream_t stream, const char** name) {
  Entry3* e = nullptr;
  Entry3* generic = nullptr;
  for (auto& cand : g_entries3) {
    if (cand.tile != tile) continue;
    if (cand.kt == kt) e = &cand;
    if (cand.kt == 0) generic = &cand;
  }
  if (!e) e = generic;
  if (!e) return hipErrorInvalidValue;
  if (p.dil > kMaxDil) return hipErrorInvalidValue;
  const Bf16x3Cfg& t = kBf16x3Tiles[tile];
  if (!e->name[0])
    snprintf(e->name, sizeof(e->name), "conv1d_bf16x3<%d, %d, %d, %d, %d, %d>", e->kt, kBf16x3Tpc,
             t.WAVES_M, t.WAVES_N, t.WM, t.WN);
  const size_t lds = bf16x3_lds_bytes(tile, p.dil);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (!e->attr) {
    hipError_t err = hipFuncSetAttribute(reinterpret_cast<const void*>(e->fn),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (err != hipSuccess) return err;
    e->attr = true;
  }
  if (name) *name = e->name;
  dim3 grid(n_tiles, m_tiles, batch);
  e->fn<<<grid, dim3(t.threads()), lds, stream>>>(p);
  return hipGetLastError();
}

}  // namespace hfg

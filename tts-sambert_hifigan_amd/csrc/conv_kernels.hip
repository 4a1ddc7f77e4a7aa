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

#include <cstdio>

#include "kernels.h"

namespace hfg {

typedef float floatx16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float lrelu(float v) { return v > 0.f ? v : v * kLReluSlope; }

template <int KT_, int WM, int WN, int WAVES_M, int WAVES_N, int CK, bool UPS>
__global__ void __launch_bounds__(64 * WAVES_M * WAVES_N)
conv1d_mfma_f32(const ConvParams p) {
  constexpr int NT = 64 * WAVES_M * WAVES_N;
  constexpr int MT = 32 * WM * WAVES_M;
  constexpr int NTILE = 32 * WN * WAVES_N;
  constexpr int KK = CK / 2;
  static_assert(CK % 2 == 0, "CK must be even (K=2 per MFMA)");
  const int KT = KT_ > 0 ? KT_ : p.kt;

  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int wchunk = MT * CK * KT;
  float* Ws = lds;
  float* Xs = lds + wchunk;
  const int XW = NTILE + (KT - 1) * p.dil;

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

  floatx16 acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int k = 0; k < WN; ++k)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][k][r] = 0.f;

  const int half = lane >> 5;     // K index inside the MFMA (0/1)
  const int col = lane & 31;      // GEMM column inside a 32-wide tile

  for (int c = 0; c < p.n_chunks; ++c) {
    // ---- stage the weight slab (fragment-ordered, contiguous) ----
    {
      const float4* __restrict__ s4 = reinterpret_cast<const float4*>(wsrc + (int64_t)c * wchunk);
      float4* d4 = reinterpret_cast<float4*>(Ws);
      const int n4 = wchunk >> 2;
      for (int i = tid; i < n4; i += NT) d4[i] = s4[i];
    }
    // ---- stage input rows with zero padding + pre-activation ----
    {
      const int ci0 = c * CK;
      const int gbase = n0 + p.off;
#pragma unroll
      for (int ci = 0; ci < CK; ++ci) {
        const int cg = ci0 + ci;
        const bool row_ok = cg < p.C_in;
        const float* __restrict__ xrow = xb + (int64_t)cg * p.L_in;
        for (int t = tid; t < XW; t += NT) {
          const int gi = gbase + t;
          float v = 0.f;
          if (row_ok && gi >= 0 && gi < p.L_in) {
            v = xrow[gi];
            if (p.act_in) v = lrelu(v);
          }
          Xs[ci * XW + t] = v;
        }
      }
    }
    __syncthreads();

    const float* wa_base = Ws + wave_m * 64 * WM + lane * WM;
    const float* xr_base = Xs + half * XW + wave_n * 32 * WN + col;
    constexpr int KT_UNROLL = KT_ > 0 ? KT_ : 1;
#pragma unroll KT_UNROLL
    for (int j = 0; j < KT; ++j) {
      const float* xr_j = xr_base + j * p.dil;
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        const float* wa = wa_base + (j * KK + kk) * WAVES_M * 64 * WM;
        float a[WM];
        if constexpr (WM == 2) {
          const float2 a2 = *reinterpret_cast<const float2*>(wa);
          a[0] = a2.x;
          a[1] = a2.y;
        } else {
#pragma unroll
          for (int i = 0; i < WM; ++i) a[i] = wa[i];
        }
        const float* xr = xr_j + 2 * kk * XW;
        float bv[WN];
#pragma unroll
        for (int k = 0; k < WN; ++k) bv[k] = xr[k * 32];
#pragma unroll
        for (int i = 0; i < WM; ++i)
#pragma unroll
          for (int k = 0; k < WN; ++k)
            acc[i][k] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], bv[k], acc[i][k], 0, 0, 0);
      }
    }
    __syncthreads();
  }

  // ---- epilogue ----
#pragma unroll
  for (int i = 0; i < WM; ++i) {
#pragma unroll
    for (int k = 0; k < WN; ++k) {
      const int n = n0 + wave_n * 32 * WN + k * 32 + col;
      if (n >= p.N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = mt * MT + wave_m * 32 * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
        if (row >= p.M) continue;
        float v = acc[i][k][r] + p.bias[row];
        if constexpr (UPS) {
          const int co = row / p.ups_s;
          const int ph = row - co * p.ups_s;
          const int t = n * p.ups_s + ph - p.ups_p;
          if (t >= 0 && t < p.L_out) p.y[(int64_t)b * p.y_bs + (int64_t)co * p.L_out + t] = v;
        } else {
          const int64_t o = (int64_t)b * p.y_bs + (int64_t)row * p.N + n;
          if (p.res) v = p.res[o] + v;  // x + conv2(...)   models/hifigan.py:85
          if (p.act_out) v = lrelu(v);
          if (p.mrf) {
            float m = (p.mrf_mode & 1) ? p.mrf[o] + v : v;   // output + resblock(x)  :129
            if (p.mrf_mode & 2) m = m / p.mrf_div;            // output / len(...)     :131
            p.mrf[o] = m;
          } else {
            p.y[o] = v;
          }
        }
      }
    }
  }
}

// conv_post (C -> 1, k=7, pad=3) + tanh over lrelu(x).  One thread per sample,
// a 256-sample tile of all C input rows staged in LDS.
__global__ void __launch_bounds__(256)
conv_post_tanh(const float* __restrict__ x, int64_t x_bs, int C, int L, const float* __restrict__ w,
               const float* __restrict__ bias, float* __restrict__ wav) {
  constexpr int TT = 256, KP = 7, HALO = 3;
  constexpr int XW = TT + KP - 1;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* Ws = lds;              // C*7
  float* Xs = lds + ((C * KP + 3) & ~3);  // C*XW
  const int t0 = blockIdx.x * TT;
  const int b = blockIdx.y;
  const float* xb = x + (int64_t)b * x_bs;
  for (int i = threadIdx.x; i < C * KP; i += TT) Ws[i] = w[i];
  for (int c = 0; c < C; ++c) {
    for (int t = threadIdx.x; t < XW; t += TT) {
      const int gi = t0 - HALO + t;
      float v = 0.f;
      if (gi >= 0 && gi < L) v = lrelu(xb[(int64_t)c * L + gi]);
      Xs[c * XW + t] = v;
    }
  }
  __syncthreads();
  const int t = t0 + threadIdx.x;
  if (t >= L) return;
  float acc = 0.f;
  for (int c = 0; c < C; ++c) {
    const float* xs = Xs + c * XW + threadIdx.x;
    const float* ws = Ws + c * KP;
#pragma unroll
    for (int j = 0; j < KP; ++j) acc = fmaf(ws[j], xs[j], acc);
  }
  wav[(int64_t)b * L + t] = tanhf(acc + bias[0]);
}

// ------------------------------------------------------------------------
// dispatch
// ------------------------------------------------------------------------
namespace {

typedef void (*ConvFn)(const ConvParams);

template <int KT, int TILE, bool UPS>
struct Inst {
  static constexpr TileCfg t = kTiles[TILE];
  static ConvFn fn() { return conv1d_mfma_f32<KT, t.WM, t.WN, t.WAVES_M, t.WAVES_N, t.CK, UPS>; }
};

struct Entry {
  int kt;
  int tile;
  bool ups;
  ConvFn fn;
  bool lds_attr_set;
  char name[96];  // template-instance name as rocprofv3 prints it
};

#define HFG_ENTRY(KT, TILE, UPS) \
  { KT, TILE, UPS, Inst<KT, TILE, UPS>::fn(), false, {0} }

Entry g_entries[] = {
    HFG_ENTRY(3, 0, false),  HFG_ENTRY(3, 1, false),  HFG_ENTRY(3, 2, false),
    HFG_ENTRY(5, 0, false),  HFG_ENTRY(5, 1, false),  HFG_ENTRY(5, 2, false),
    HFG_ENTRY(7, 0, false),  HFG_ENTRY(7, 1, false),  HFG_ENTRY(7, 2, false),
    HFG_ENTRY(11, 0, false), HFG_ENTRY(11, 1, false), HFG_ENTRY(11, 2, false),
    HFG_ENTRY(0, 0, false),  HFG_ENTRY(0, 1, false),  HFG_ENTRY(0, 2, false),
    HFG_ENTRY(2, 0, true),   HFG_ENTRY(2, 1, true),   HFG_ENTRY(2, 2, true),
    HFG_ENTRY(0, 0, true),   HFG_ENTRY(0, 1, true),   HFG_ENTRY(0, 2, true),
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
  if (!e->name[0])
    snprintf(e->name, sizeof(e->name), "conv1d_mfma_f32<%d, %d, %d, %d, %d, %d, %s>", e->kt, t.WM,
             t.WN, t.WAVES_M, t.WAVES_N, t.CK, e->ups ? "true" : "false");
  const int xw = t.NTILE() + (kt - 1) * p.dil;
  const size_t lds = sizeof(float) * ((size_t)t.MT() * t.CK * kt + (size_t)t.CK * xw);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (lds > 64 * 1024 && !e->lds_attr_set) {
    hipError_t err = hipFuncSetAttribute(reinterpret_cast<const void*>(e->fn),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (err != hipSuccess) return err;
    e->lds_attr_set = true;
  }
  if (name) *name = e->name;
  dim3 grid(n_tiles, m_tiles, batch);
  e->fn<<<grid, dim3(t.threads()), lds, stream>>>(p);
  return hipGetLastError();
}

hipError_t launch_conv_post(const float* x, int64_t x_bs, int C, int L, const float* w,
                            const float* bias, float* wav, int batch, hipStream_t stream,
                            const char** name) {
  const size_t lds = sizeof(float) * ((size_t)((C * 7 + 3) & ~3) + (size_t)C * (256 + 6));
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  static bool attr = false;
  if (lds > 64 * 1024 && !attr) {
    hipError_t err = hipFuncSetAttribute(reinterpret_cast<const void*>(conv_post_tanh),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (err != hipSuccess) return err;
    attr = true;
  }
  if (name) *name = "conv_post_tanh";
  dim3 grid((L + 255) / 256, batch);
  conv_post_tanh<<<grid, dim3(256), lds, stream>>>(x, x_bs, C, L, w, bias, wav);
  return hipGetLastError();
}

}  // namespace hfg

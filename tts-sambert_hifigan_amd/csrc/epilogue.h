// epilogue.h — fused output stage shared by conv1d_mfma_f32 and conv1d_bf16x3
// (regular Conv1d, not the polyphase upsampler):
//   v = acc + bias[row]; v = res + v (ResBlock residual, models/hifigan.py:85);
//   v = lrelu(v) (post-activation, :83); MRF running sum / final division (:125-131)
// Per 32x32 accumulator tile the 16 bias, 16 residual and 16 MRF loads are issued
// as independent batches (unconditional, clamped offsets) before any store, so a
// tile costs one memory round trip instead of one per element (the residual may
// alias the output: every element is still read before its own write).
// Addresses are 32-bit byte offsets from block-uniform batch bases.
#pragma once

#include <hip/hip_runtime.h>

#include "kernels.h"

namespace hfg {

typedef float floatx16e __attribute__((ext_vector_type(16)));

template <int WM, int WN>
__device__ __forceinline__ void conv_epilogue(const ConvParams& p, const float* __restrict__ bias,
                                              floatx16e (&acc)[WM][WN], int b, int row_base,
                                              int n_base, int N_b, int half, int col) {
  const int64_t bo = (int64_t)b * p.y_bs;
  const char* resb = p.res ? reinterpret_cast<const char*>(p.res + bo) : nullptr;
  char* outb = reinterpret_cast<char*>((p.mrf ? p.mrf : p.y) + bo);
  const bool add_mrf = p.mrf && (p.mrf_mode & 1);
  const bool div_mrf = p.mrf && (p.mrf_mode & 2);
  const bool act = p.act_out != 0;
  // the tile origin is wave-uniform: a tile wholly inside [0, M) x [0, N_b) stores
  // without per-element exec-mask branches
  const int row_u = __builtin_amdgcn_readfirstlane(row_base);
  const int n_u = __builtin_amdgcn_readfirstlane(n_base);
  // bias: padded to the m-tile, every row index is readable
#pragma unroll
  for (int i = 0; i < WM; ++i) {
    float bv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r)
      bv[r] = bias[row_base + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half];
#pragma unroll
    for (int k = 0; k < WN; ++k) {
      const int n = n_base + k * 32 + col;
      const bool nok = n < N_b;
      unsigned off[16];
      bool ok[16];
      float v[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = row_base + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
        ok[r] = nok && row < p.M;
        off[r] = ok[r] ? (unsigned)(row * p.N + n) * 4u : 0u;
        v[r] = acc[i][k][r] + bv[r];
      }
      if (resb) {
        float rv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) rv[r] = *reinterpret_cast<const float*>(resb + off[r]);
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = rv[r] + v[r];
      }
      if (act) {
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * kLReluSlope;
      }
      if (add_mrf) {
        float mv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) mv[r] = *reinterpret_cast<const float*>(outb + off[r]);
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = mv[r] + v[r];
      }
      if (div_mrf) {
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = v[r] / p.mrf_div;
      }
      if (n_u + k * 32 + 31 < N_b && row_u + i * 32 + 31 < p.M) {
#pragma unroll
        for (int r = 0; r < 16; ++r) *reinterpret_cast<float*>(outb + off[r]) = v[r];
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (ok[r]) *reinterpret_cast<float*>(outb + off[r]) = v[r];
      }
    }
  }
}

template <int WM, int WN>
__device__ __forceinline__ void conv_epilogue(const ConvParams& p, floatx16e (&acc)[WM][WN],
                                              int b, int row_base, int n_base, int N_b,
                                              int half, int col) {
  conv_epilogue<WM, WN>(p, p.bias, acc, b, row_base, n_base, N_b, half, col);
}

}  // namespace hfg

// epilogue.h — fused output stage shared by conv1d_mfma_f32 and conv1d_bf16x3
// (regular Conv1d, not the polyphase upsampler):
//   v = acc + bias[row]; v = res + v (ResBlock residual, models/hifigan.py:85);
//   v = lrelu(v) (post-activation, :83); MRF running sum / final division (:125-131)
// Addresses are 32-bit byte offsets from block-uniform batch bases so every
// load/store is an SGPR-base + VGPR-offset access (no per-element 64-bit math).
#pragma once

#include <hip/hip_runtime.h>

#include "kernels.h"

namespace hfg {

typedef float floatx16e __attribute__((ext_vector_type(16)));

template <int WM, int WN>
__device__ __forceinline__ void conv_epilogue(const ConvParams& p, floatx16e (&acc)[WM][WN],
                                              int b, int row_base, int n_base, int N_b,
                                              int half, int col) {
  const int64_t bo = (int64_t)b * p.y_bs;
  const char* __restrict__ resb = p.res ? reinterpret_cast<const char*>(p.res + bo) : nullptr;
  char* __restrict__ outb = reinterpret_cast<char*>((p.mrf ? p.mrf : p.y) + bo);
  const bool add_mrf = p.mrf && (p.mrf_mode & 1);
  const bool div_mrf = p.mrf && (p.mrf_mode & 2);
  const bool act = p.act_out != 0;
#pragma unroll
  for (int i = 0; i < WM; ++i) {
#pragma unroll
    for (int k = 0; k < WN; ++k) {
      const int n = n_base + k * 32 + col;
      if (n >= N_b) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = row_base + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
        if (row >= p.M) continue;
        const unsigned off = (unsigned)(row * p.N + n) * 4u;
        float v = acc[i][k][r] + p.bias[row];
        if (resb) v = *reinterpret_cast<const float*>(resb + off) + v;
        if (act) v = v > 0.f ? v : v * kLReluSlope;
        if (add_mrf) v = *reinterpret_cast<const float*>(outb + off) + v;
        if (div_mrf) v = v / p.mrf_div;
        *reinterpret_cast<float*>(outb + off) = v;
      }
    }
  }
}

}  // namespace hfg

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

#include <type_traits>
#include <utility>

#include "kernels.h"

namespace hfg {

typedef float floatx16e __attribute__((ext_vector_type(16)));

// f(integral_constant<int, 0>) ... f(integral_constant<int, N - 1>): a compile-time loop (a
// `#pragma unroll` loop around a large body can stay a loop, and an accumulator array it
// indexes then lives in scratch)
template <typename F, int... Is>
__device__ __forceinline__ void static_for_impl(F& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// largest value over a wave (every lane active): DPP max within each 16-lane row (quad swaps,
// then row rotations by 4 and 8), then the 4 row maxima by readlane — a few cycles per step,
// where ds_bpermute shuffles put ~6 LDS round trips on the critical path
__device__ __forceinline__ float wave_max(float m) {
  auto step = [&](auto ctrl_tag) {
    constexpr int CTRL = decltype(ctrl_tag)::value;
    const float o = __builtin_bit_cast(
        float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, m), CTRL, 0xF, 0xF, false));
    m = fmaxf(m, o);
  };
  step(std::integral_constant<int, 0xB1>{});   // quad_perm [1,0,3,2]
  step(std::integral_constant<int, 0x4E>{});   // quad_perm [2,3,0,1]
  step(std::integral_constant<int, 0x124>{});  // row_ror:4
  step(std::integral_constant<int, 0x128>{});  // row_ror:8
  const int mi = __builtin_bit_cast(int, m);
  const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(mi, 0));
  const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(mi, 16));
  const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(mi, 32));
  const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(mi, 48));
  return fmaxf(fmaxf(r0, r1), fmaxf(r2, r3));
}
// fold a lane's max |value| into item b's producer slot: one vector atomic per wave (the
// slots are zeroed by the host before the forward; non-negative floats order like their bit
// patterns).  An item's slot is kAmaxSpread words on separate 128-B lines and each wave
// updates the one its block and wave index select, so same-line atomics do not serialise a
// whole grid (kernels.h); the consumer takes the max of the kAmaxSpread words (x3_exp_slot).
__device__ __forceinline__ void amax_commit(float m, uint32_t* slots, int b) {
  m = wave_max(m);
  const unsigned blk = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  const unsigned w = blk * (blockDim.x >> 6) + (threadIdx.x >> 6);
  uint32_t* slot = slots + (size_t)b * kAmaxSlotWords + (w & (kAmaxSpread - 1)) * kAmaxLineWords;
  if ((threadIdx.x & 63) == 0) atomicMax(slot, __builtin_bit_cast(uint32_t, m));
}

// sc: the accumulator's scale (f16x3: 2^-(e_x + e_w); 1 otherwise): v = fma(acc, sc, bias),
// bitwise acc + bias for sc = 1
template <int WM, int WN>
__device__ __forceinline__ void conv_epilogue(const ConvParams& p, const float* __restrict__ bias,
                                              floatx16e (&acc)[WM][WN], int b, int row_base,
                                              int n_base, int N_b, int half, int col,
                                              float sc = 1.0f) {
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
  float vmax = 0.f;  // max |stored value| (f16x3 consumers: p.amax_out)
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
        v[r] = __builtin_fmaf(acc[i][k][r], sc, bv[r]);
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
      if (p.amax_out) {
#pragma unroll
        for (int r = 0; r < 16; ++r) vmax = ok[r] ? fmaxf(vmax, fabsf(v[r])) : vmax;
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
  if (p.amax_out) amax_commit(vmax, p.amax_out, b);
}

template <int WM, int WN>
__device__ __forceinline__ void conv_epilogue(const ConvParams& p, floatx16e (&acc)[WM][WN],
                                              int b, int row_base, int n_base, int N_b,
                                              int half, int col, float sc = 1.0f) {
  conv_epilogue<WM, WN>(p, p.bias, acc, b, row_base, n_base, N_b, half, col, sc);
}

// The same contract with the tile staged through LDS: each wave writes 32 accumulator
// rows x 32*WN columns at a time into its own LDS region (row stride 32*WN + 8 floats:
// the two row quads a ds_write_b32 touches land 32 banks apart) and reads them back as
// row-contiguous float4, so the residual / MRF loads and the stores are 16-B per lane
// and fully coalesced (4x fewer memory instructions than the accumulator layout's
// one-dword-per-row stores).  Needs N % 4 == 0 (16-B aligned rows) and
// 32 * (32*WN + 8) * 4 bytes of LDS per wave at `stage`; the caller has barriered the
// block (every wave is done with the main loop's LDS).
template <int WM, int WN>
__device__ __forceinline__ void conv_epilogue_lds(const ConvParams& p, floatx16e (&acc)[WM][WN],
                                                  int b, int row_base, int n_base, int N_b,
                                                  int half, int col, float* stage, int lane,
                                                  float sc = 1.0f) {
  constexpr int SROW = 32 * WN + 8;
  constexpr int C4 = 8 * WN;                 // float4 per staged row
  const int64_t bo = (int64_t)b * p.y_bs;
  const float* resb = p.res ? p.res + bo : nullptr;
  float* outb = (p.mrf ? p.mrf : p.y) + bo;
  const bool add_mrf = p.mrf && (p.mrf_mode & 1);
  const bool div_mrf = p.mrf && (p.mrf_mode & 2);
  const bool act = p.act_out != 0;
  float vmax = 0.f;  // max |stored value| (f16x3 consumers: p.amax_out)
#pragma unroll
  for (int i = 0; i < WM; ++i) {
#pragma unroll
    for (int k = 0; k < WN; ++k)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        stage[((r & 3) + 8 * (r >> 2) + 4 * half) * SROW + k * 32 + col] = acc[i][k][r];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's writes are in LDS
    __builtin_amdgcn_wave_barrier();
    constexpr int IT = 32 * C4 / 64;          // float4 per lane
    // the residual / MRF loads of group it0 + 4 are issued before group it0's stores: the
    // stores may alias later loads as far as the compiler knows, so loads placed after them
    // cost one HBM round trip per group (same values, same additions in the same order)
    float4 rvb[2][4], mvb[2][4];
    auto geom = [&](int it, int& row, int& n, bool& ok) {
      const int e = it * 64 + lane;
      const int rr = e / C4, c4 = e - rr * C4;
      row = row_base + i * 32 + rr;
      n = n_base + 4 * c4;
      ok = row < p.M && n < N_b;
    };
    auto load_group = [&](int it0, float4 (&rv)[4], float4 (&mv)[4]) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        int row, n;
        bool ok;
        geom(it0 + u, row, n, ok);
        const int64_t o = (int64_t)row * p.N + n;
        rv[u] = resb && ok ? *reinterpret_cast<const float4*>(resb + o) : float4{0.f, 0.f, 0.f, 0.f};
        mv[u] = add_mrf && ok ? *reinterpret_cast<const float4*>(outb + o)
                              : float4{0.f, 0.f, 0.f, 0.f};
      }
    };
    load_group(0, rvb[0], mvb[0]);
#pragma unroll
    for (int it0 = 0; it0 < IT; it0 += 4) {
      const int cur = (it0 / 4) & 1;
      if (it0 + 4 < IT) load_group(it0 + 4, rvb[cur ^ 1], mvb[cur ^ 1]);
      float4 v[4];
      int row[4], n[4];
      bool ok[4], full[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = (it0 + u) * 64 + lane;
        const int rr = e / C4, c4 = e - rr * C4;
        geom(it0 + u, row[u], n[u], ok[u]);
        full[u] = ok[u] && n[u] + 3 < N_b;
        v[u] = *reinterpret_cast<const float4*>(stage + rr * SROW + 4 * c4);
        const float bv = p.bias[row[u]];
        v[u].x = __builtin_fmaf(v[u].x, sc, bv);
        v[u].y = __builtin_fmaf(v[u].y, sc, bv);
        v[u].z = __builtin_fmaf(v[u].z, sc, bv);
        v[u].w = __builtin_fmaf(v[u].w, sc, bv);
      }
      if (resb) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float4 rv = rvb[cur][u];
          v[u].x = rv.x + v[u].x;
          v[u].y = rv.y + v[u].y;
          v[u].z = rv.z + v[u].z;
          v[u].w = rv.w + v[u].w;
        }
      }
      if (act) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          v[u].x = v[u].x > 0.f ? v[u].x : v[u].x * kLReluSlope;
          v[u].y = v[u].y > 0.f ? v[u].y : v[u].y * kLReluSlope;
          v[u].z = v[u].z > 0.f ? v[u].z : v[u].z * kLReluSlope;
          v[u].w = v[u].w > 0.f ? v[u].w : v[u].w * kLReluSlope;
        }
      }
      if (add_mrf) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float4 mv = mvb[cur][u];
          v[u].x = mv.x + v[u].x;
          v[u].y = mv.y + v[u].y;
          v[u].z = mv.z + v[u].z;
          v[u].w = mv.w + v[u].w;
        }
      }
      if (div_mrf) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          v[u].x = v[u].x / p.mrf_div;
          v[u].y = v[u].y / p.mrf_div;
          v[u].z = v[u].z / p.mrf_div;
          v[u].w = v[u].w / p.mrf_div;
        }
      }
      if (p.amax_out) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          // the stored elements only: a partial quad's tail past N_b is not written
          if (full[u]) {
            vmax = fmaxf(vmax, fmaxf(fmaxf(fabsf(v[u].x), fabsf(v[u].y)),
                                     fmaxf(fabsf(v[u].z), fabsf(v[u].w))));
          } else if (ok[u]) {
            const int nv = N_b - n[u];
            vmax = fmaxf(vmax, fabsf(v[u].x));
            if (nv > 1) vmax = fmaxf(vmax, fabsf(v[u].y));
            if (nv > 2) vmax = fmaxf(vmax, fabsf(v[u].z));
          }
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float* dst = outb + (int64_t)row[u] * p.N + n[u];
        if (full[u]) {
          // streamed once (the next launch reads it from HBM / MALL): non-temporal
          typedef float f4v __attribute__((ext_vector_type(4)));
          const f4v nv = {v[u].x, v[u].y, v[u].z, v[u].w};
          __builtin_nontemporal_store(nv, reinterpret_cast<f4v*>(dst));
        } else if (ok[u]) {
          dst[0] = v[u].x;
          if (n[u] + 1 < N_b) dst[1] = v[u].y;
          if (n[u] + 2 < N_b) dst[2] = v[u].z;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  if (p.amax_out) amax_commit(vmax, p.amax_out, b);
}

// conv_epilogue_lds with the m-tile's bias in LDS (bias_lds[row - m-tile origin], copied at
// kernel start): vmcnt counts loads and stores in one in-order queue, so a global load issued
// after a store cannot complete for the wave before that store has; the per-float4 bias loads
// of conv_epilogue_lds each waited for the stores before them.  Here the only global loads are
// the residual / MRF batches, every one issued before the batch's stores (the whole row tile
// with one of them, half of it with both: register budget).
template <int WM, int WN>
__device__ __forceinline__ void conv_epilogue_lds2(const ConvParams& p, floatx16e (&acc)[WM][WN],
                                                   int b, int row_base, int row_tile0, int n_base,
                                                   int N_b, int half, int col, float* stage,
                                                   const float* bias_lds, int lane, float sc,
                                                   uint64_t* tsv = nullptr) {
  // tsv (clock-stamp diagnostic builds): row tile i's staging done -> tsv[8 + 2i], its stores
  // issued -> tsv[9 + 2i] (registers: the caller stores them at the end)
  auto ts = [&](int s_) {
    if (tsv) tsv[s_] = __builtin_amdgcn_s_memtime();
  };
  constexpr int SROW = 32 * WN + 8;
  constexpr int C4 = 8 * WN;                 // float4 per staged row
  constexpr int IT = 32 * C4 / 64;           // float4 per lane and row tile
  const int64_t bo = (int64_t)b * p.y_bs;
  const float* resb = p.res ? p.res + bo : nullptr;
  float* outb = (p.mrf ? p.mrf : p.y) + bo;
  const bool add_mrf = p.mrf && (p.mrf_mode & 1);
  const bool div_mrf = p.mrf && (p.mrf_mode & 2);
  const bool act = p.act_out != 0;
  float vmax = 0.f;  // max |stored value| (f16x3 consumers: p.amax_out)
  static_for<WM>([&](auto i_tag) {
    constexpr int i = decltype(i_tag)::value;
#pragma unroll
    for (int k = 0; k < WN; ++k)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        stage[((r & 3) + 8 * (r >> 2) + 4 * half) * SROW + k * 32 + col] = acc[i][k][r];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's writes are in LDS
    __builtin_amdgcn_wave_barrier();
    ts(8 + 2 * i);
    // wave-uniform: the whole 32 x 32*WN tile of this row tile lies inside [0, M) x [0, N_b)
    // -> unmasked float4 stores (the masked path branches per element)
    const bool interior = __builtin_amdgcn_readfirstlane(row_base) + i * 32 + 31 < p.M &&
                          __builtin_amdgcn_readfirstlane(n_base) + 32 * WN - 1 < N_b;
    auto batch = [&](auto bs_tag, auto r_tag, auto m_tag, auto u0_tag) {
      constexpr int BS = decltype(bs_tag)::value, U0 = decltype(u0_tag)::value;
      constexpr bool R = decltype(r_tag)::value, M = decltype(m_tag)::value;
      float4 rv[BS], mv[BS], sv[BS];
      float bv[BS];
      // global loads first, then every LDS read of the batch (one latency each, not one per
      // float4), then the arithmetic and the stores
      static_for<BS>([&](auto j_tag) {
        constexpr int j = decltype(j_tag)::value;
        const int e = (U0 + j) * 64 + lane;
        const int rr = e / C4, c4 = e - rr * C4;
        const int row = row_base + i * 32 + rr, n = n_base + 4 * c4;
        const bool ok = row < p.M && n < N_b;
        const int64_t o = (int64_t)row * p.N + n;
        // ablation bits 15 / 16 (timing only): the residual read from the tile's columns of row
        // 0 (L2-warm after the first wave) / not read at all
        const int64_t orr = (kAblate && (p.dbg & 32768)) ? (int64_t)n : o;
        if constexpr (R)
          rv[j] = ok && !(kAblate && (p.dbg & 65536)) ? *reinterpret_cast<const float4*>(resb + orr)
                                                      : float4{0.f, 0.f, 0.f, 0.f};
        if constexpr (M)
          mv[j] = ok ? *reinterpret_cast<const float4*>(outb + o) : float4{0.f, 0.f, 0.f, 0.f};
      });
      static_for<BS>([&](auto j_tag) {
        constexpr int j = decltype(j_tag)::value;
        const int e = (U0 + j) * 64 + lane;
        const int rr = e / C4, c4 = e - rr * C4;
        sv[j] = *reinterpret_cast<const float4*>(stage + rr * SROW + 4 * c4);
        bv[j] = bias_lds[row_base + i * 32 + rr - row_tile0];
      });
      static_for<BS>([&](auto j_tag) {
        constexpr int j = decltype(j_tag)::value;
        const int e = (U0 + j) * 64 + lane;
        const int rr = e / C4, c4 = e - rr * C4;
        const int row = row_base + i * 32 + rr, n = n_base + 4 * c4;
        float4 v = sv[j];
        v.x = __builtin_fmaf(v.x, sc, bv[j]);
        v.y = __builtin_fmaf(v.y, sc, bv[j]);
        v.z = __builtin_fmaf(v.z, sc, bv[j]);
        v.w = __builtin_fmaf(v.w, sc, bv[j]);
        if constexpr (R) {
          v.x = rv[j].x + v.x;
          v.y = rv[j].y + v.y;
          v.z = rv[j].z + v.z;
          v.w = rv[j].w + v.w;
        }
        if (act) {
          v.x = v.x > 0.f ? v.x : v.x * kLReluSlope;
          v.y = v.y > 0.f ? v.y : v.y * kLReluSlope;
          v.z = v.z > 0.f ? v.z : v.z * kLReluSlope;
          v.w = v.w > 0.f ? v.w : v.w * kLReluSlope;
        }
        if constexpr (M) {
          v.x = mv[j].x + v.x;
          v.y = mv[j].y + v.y;
          v.z = mv[j].z + v.z;
          v.w = mv[j].w + v.w;
        }
        if (div_mrf) {
          v.x = v.x / p.mrf_div;
          v.y = v.y / p.mrf_div;
          v.z = v.z / p.mrf_div;
          v.w = v.w / p.mrf_div;
        }
        float* dst = outb + (int64_t)row * p.N + n;
        typedef float f4v __attribute__((ext_vector_type(4)));
        if (interior) {
          vmax = fmaxf(vmax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
          if (kAblate && (p.dbg & 16384)) {
            // ablation bit 14: no stores (timing only)
            if (v.x == 1.2345e-30f) dst[0] = v.y;
          } else {
            // streamed once (the next launch reads it from HBM / MALL): non-temporal
            const f4v nv = {v.x, v.y, v.z, v.w};
            __builtin_nontemporal_store(nv, reinterpret_cast<f4v*>(dst));
          }
          return;
        }
        const bool ok = row < p.M && n < N_b;
        const bool full = ok && n + 3 < N_b;
        // the stored elements only: a partial quad's tail past N_b is not written
        if (full) {
          vmax = fmaxf(vmax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
          const f4v nv = {v.x, v.y, v.z, v.w};
          __builtin_nontemporal_store(nv, reinterpret_cast<f4v*>(dst));
        } else if (ok) {
          const int nv = N_b - n;
          vmax = fmaxf(vmax, fabsf(v.x));
          dst[0] = v.x;
          if (nv > 1) vmax = fmaxf(vmax, fabsf(v.y)), dst[1] = v.y;
          if (nv > 2) vmax = fmaxf(vmax, fabsf(v.z)), dst[2] = v.z;
        }
      });
    };
    using T_ = std::true_type;
    using F_ = std::false_type;
    using IFull = std::integral_constant<int, IT>;
    using IHalf = std::integral_constant<int, IT / 2>;
    using Z = std::integral_constant<int, 0>;
    if (resb && add_mrf) {  // block-uniform branches
      batch(IHalf{}, T_{}, T_{}, Z{});
      batch(IHalf{}, T_{}, T_{}, IHalf{});
    } else if (resb) {
      batch(IHalf{}, T_{}, F_{}, Z{});
      batch(IHalf{}, T_{}, F_{}, IHalf{});
    } else if (add_mrf) {
      batch(IHalf{}, F_{}, T_{}, Z{});
      batch(IHalf{}, F_{}, T_{}, IHalf{});
    } else {
      batch(IFull{}, F_{}, F_{}, Z{});
    }
    ts(9 + 2 * i);
    __builtin_amdgcn_wave_barrier();
  });
  if (p.amax_out) amax_commit(vmax, p.amax_out, b);
}

}  // namespace hfg

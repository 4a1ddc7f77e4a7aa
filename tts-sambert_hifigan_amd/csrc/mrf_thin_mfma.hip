// mrf_thin_mfma.hip — the whole MRF of a thin stage (C = 16 channels: V2*'s third stage) in
// one launch on the 16x16x32 matrix cores in split precision (bf16x3 or f16x3 products,
// bf16x3_common.h; fp32 accumulation).  Same algorithm, windowing and HBM traffic as
// mrf_thin.hip (the packed-fp32 VALU kernel, which the exact-fp32 mode and the C = 8 stage
// keep: its 2-4 MFMAs per conv left the per-conv barriers exposed, round 2):
//
//   for j in resblocks:  xr = x
//                        for m in dilations: xr = xr + conv2_jm(lrelu(conv1_jm(lrelu(xr))))
//                                                            models/hifigan.py:79-85
//                        mrf = xr (j = 0) | mrf + xr          models/hifigan.py:125-130
//   y = mrf / n_res                                           models/hifigan.py:131
//
// MFMA shape 16x16x32: rows = the 16 output channels; one k-step = 16 input channels x 2
// taps; per k-step and column tile: lo*hi, hi*lo, hi*hi (3 MFMAs).  Taps past k carry zero
// weights.
//
// Mapping.  4 waves, each 8 column tiles of 16: a 512-column window.  Accumulator layout
// (16x16): lane l holds column (l & 15) and rows 4*(l >> 4) + r.  The ResBlock state xr,
// the MRF sum and the conv accumulator stay in registers in that layout.  The conv
// operand (lrelu, zero outside [0, len), split into hi / lo planes) lives in LDS as
// [row = column][16 channels] per plane; rows are 32 B whose two 16-B halves are swapped
// when bit 3 of the row is set, so the 16 lanes of a B-fragment read (16 B each,
// consecutive rows) hit distinct banks.  Weights (A fragments) are host-packed per
// (conv, k-step) as [plane][lane][8] = 2 KB and loaded from L2 by buffer loads (uniform
// across the block) into registers one conv ahead.
// f16x3: every operand the block writes is scaled by the power of two of the block's largest
// |value| (posted per wave before one extra barrier per conv); the conv result is unscaled
// by 2^-(e_x + e_w) before its bias.
#include <hip/hip_runtime.h>

#include <mutex>

#include <cstdio>

#include "bf16x3_common.h"
#include "kernels.h"

namespace hfg {

namespace {
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
}  // namespace

template <int C, int NP, int FMT>
__global__ void __launch_bounds__(256, 2)
mrf_thin_mfma(const ThinParams p) {
  static_assert(C == 16, "thin MFMA kernel: C = 16");
  constexpr int NW = 4;
  constexpr int NCT = kThinMfmaTiles;       // 16-column tiles per wave
  constexpr int NWIN = NW * NCT * 16;
  constexpr int MARG = kThinMarg;
  constexpr int ROWS = NWIN + 2 * MARG;
  constexpr int RB = 2 * C;                 // bytes per operand row (one plane)
  constexpr int PS = ROWS * RB;             // bytes per plane
  constexpr int TPS = 32 / C;               // taps per k-step
  extern __shared__ __attribute__((aligned(16))) char lds[];
  // f16x3: per-wave max |next operand|, after the operand buffers
  float* const amax_s = reinterpret_cast<float*>(lds + kThinMfmaBufs * 2 * PS);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4;                  // accumulator row quad / B-fragment K block
  const int c = lane & 15;                  // column inside a tile
  const int b = blockIdx.y;
  const int len_b = p.len ? min(p.len[b], p.L) : p.L;
  const int t0 = blockIdx.x * p.W;
  if (t0 >= len_b) return;  // whole block past this utterance's end (block-uniform)
  const int ws = t0 - p.halo;
  const int cbase = wave * NCT * 16 + c;    // window column of tile 0 for this lane

  bool vk[NCT];
#pragma unroll
  for (int t = 0; t < NCT; ++t) vk[t] = (unsigned)(ws + cbase + 16 * t) < (unsigned)len_b;

  // zero the margin rows of every plane once (operand writes cover the window only)
  for (int i = tid; i < 2 * MARG * RB / 4; i += NW * 64) {
    const int row = i / (RB / 4), w4 = i - row * (RB / 4);
    const int r = row < MARG ? row : NWIN + row;
#pragma unroll
    for (int pl = 0; pl < 2 * kThinMfmaBufs; ++pl)
      *reinterpret_cast<float*>(lds + pl * PS + r * RB + w4 * 4) = 0.f;
  }

  // channel of accumulator element i
  auto chan = [&](int i) { return 4 * q + i; };
  // byte offset of (row, channel group of 4 at ch) inside a plane; the 16-B halves are
  // swizzled by bit 3 of the row
  auto opnd_off = [&](int row, int ch) {
    return row * RB + ((((ch >> 3) ^ (row >> 3)) & 1) << 4) + (ch & 7) * 2;
  };

  // ---- A stream: buffer loads of [conv][step][plane][lane][8] ----
  const __amdgpu_buffer_rsrc_t wrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.wm, 0, p.wm_bytes, 0x00020000);
  const int a_lane = lane * 16;

  // operand <- lrelu(v) * sc, zero outside [0, len), hi/lo split
  auto write_operand = [&](const floatx4 (&v)[NCT], char* buf, float sc) {
    const float sc1 = kLReluSlope * sc;
#pragma unroll
    for (int t = 0; t < NCT; ++t) {
      bf16x4 h, l;
#pragma unroll
      for (int i = 0; i < 4; i += 2) {
        floatx2 a;
        a[0] = vk[t] ? fmaxf(v[t][i] * sc, v[t][i] * sc1) : 0.f;
        a[1] = vk[t] ? fmaxf(v[t][i + 1] * sc, v[t][i + 1] * sc1) : 0.f;
        bf16x2 hh, ll;
        split2<FMT>(a, hh, ll);
        h[i] = hh[0];
        h[i + 1] = hh[1];
        l[i] = ll[0];
        l[i + 1] = ll[1];
      }
      const int off = opnd_off(cbase + 16 * t + MARG, chan(0));
      *reinterpret_cast<bf16x4*>(buf + off) = h;
      *reinterpret_cast<bf16x4*>(buf + PS + off) = l;
    }
  };
  // f16x3: block-wide max |v| over the window's exact columns (inside [0, len), at least the
  // current ResBlock's receptive-field radius so far from the window edges: garbage columns
  // do not set the scale) -> scale exponent (the barrier inside also ends every read of the
  // previous operand)
  auto block_exp = [&](const floatx4 (&v)[NCT], int radius) {
    float m = 0.f;
#pragma unroll
    for (int t = 0; t < NCT; ++t) {
      const int cw = cbase + 16 * t;
      const bool ex_t = vk[t] && cw >= radius && cw < NWIN - radius;
#pragma unroll
      for (int i = 0; i < 4; ++i) m = ex_t ? fmaxf(m, fabsf(v[t][i])) : m;
    }
    m = wave_max(m);
    if (lane == 0) amax_s[wave] = m;
    __syncthreads();
    m = fmaxf(fmaxf(amax_s[0], amax_s[1]), fmaxf(amax_s[2], amax_s[3]));
    return x3_exp(m);
  };

  floatx4 acc[NCT];
  constexpr int MS = kThinMfmaMaxSteps;
  const int cv_end = p.rb_conv0[p.n_res];
  // A fragments of one conv (every k-step, both planes); two sets, so the next conv's
  // loads are in flight for the whole of the current conv (one L2 latency per launch
  // instead of one per conv)
  bf16x8 sa0[MS], sa1[MS], sb0[MS], sb1[MS];
  auto load_a = [&](bf16x8 (&a0)[MS], bf16x8 (&a1)[MS], int cv) {
    cv = min(cv, cv_end - 1);
    const int steps = (p.kt[cv] + TPS - 1) / TPS;
    const int wo = p.wm_off[cv];
#pragma unroll
    for (int s = 0; s < MS; ++s) {
      const int so = wo + min(s, steps - 1) * 2048;
      a0[s] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, a_lane, so, 0));
      a1[s] =
          __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, a_lane + 1024, so, 0));
    }
  };
  // acc = bias + W_cv * operand (f16x3: unscaled by inv first), with (a0, a1) = conv cv's A
  // fragments; the next conv's are loaded into (n0, n1)
  auto run_conv = [&](int cv, const char* buf, const bf16x8 (&a0)[MS], const bf16x8 (&a1)[MS],
                      bf16x8 (&n0)[MS], bf16x8 (&n1)[MS], float inv) {
    load_a(n0, n1, cv + 1);
    const int kt = p.kt[cv], d = p.dil[cv];
    const int steps = (kt + TPS - 1) / TPS;
#pragma unroll
    for (int t = 0; t < NCT; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
    // B-fragment tap and channel offset of this lane: tap 2s + (q >> 1), channels 8 (q & 1)
    const int tap_q = q >> 1;
    const int ch_q = 8 * (q & 1);
    const int row_q = cbase + MARG + (tap_q - (kt - 1) / 2) * d;
    // B fragments streamed one (step, tile) unit ahead of the MFMAs that use them
    bf16x8 bh[2], bl[2];
    auto load_b = [&](int slot, int s, int t) {
      const int off = opnd_off(row_q + s * TPS * d + 16 * t, ch_q);
      bh[slot] = *reinterpret_cast<const bf16x8*>(buf + off);
      bl[slot] = *reinterpret_cast<const bf16x8*>(buf + PS + off);
    };
    load_b(0, 0, 0);
#pragma unroll
    for (int s = 0; s < MS; ++s) {
      if (s >= steps) break;
#pragma unroll
      for (int t = 0; t < NCT; ++t) {
        const int u = s * NCT + t;
        if (t + 1 < NCT) load_b((u + 1) & 1, s, t + 1);
        else if (s + 1 < steps) load_b((u + 1) & 1, s + 1, 0);
        if constexpr (NP == 3)  // the weights' lo plane (zero for bf16-valued weights)
          acc[t] = mfma16<FMT>(a1[s], bh[u & 1], acc[t]);
        acc[t] = mfma16<FMT>(a0[s], bl[u & 1], acc[t]);
        acc[t] = mfma16<FMT>(a0[s], bh[u & 1], acc[t]);
      }
    }
    float bv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) bv[i] = p.bias[cv * C + chan(i)];
#pragma unroll
    for (int t = 0; t < NCT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        acc[t][i] = FMT == kFmtF16 ? __builtin_fmaf(acc[t][i], inv, bv[i]) : acc[t][i] + bv[i];
  };

  const float* __restrict__ xb = p.x + (int64_t)b * p.bs;
  load_a(sa0, sa1, p.rb_conv0[0]);
  floatx4 mrf[NCT];
  for (int r = 0; r < p.n_res; ++r) {
    floatx4 xr[NCT];
#pragma unroll
    for (int t = 0; t < NCT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        // the 32-bit offset is formed here, not hoisted out of the ResBlock loop
        unsigned off = vk[t] ? (unsigned)(chan(i) * p.L + ws + cbase + 16 * t) : 0u;
        asm volatile("" : "+v"(off));
        const float v = xb[off];
        xr[t][i] = vk[t] ? v : 0.f;
      }
    const int cv0 = p.rb_conv0[r], cv1 = p.rb_conv0[r + 1];
    int radius = 0;  // f16x3: receptive-field radius of this ResBlock's convs run so far
    for (int cv = cv0; cv < cv1; cv += 2) {
      // two operand buffers (kThinMfmaBufs = 2): conv1 reads buffer 0, conv2 buffer 1, so a
      // buffer is rewritten only after the barrier that follows every read of it (one
      // barrier per conv; f16x3 adds the one of block_exp); one buffer: rewritten in place
      // between two barriers
      char* const b0 = lds;
      char* const b1 = lds + (kThinMfmaBufs - 1) * 2 * PS;
      int ex = 0;
      if (kThinMfmaBufs == 1 && FMT != kFmtF16) __syncthreads();
      if constexpr (FMT == kFmtF16) ex = block_exp(xr, radius);
      write_operand(xr, b0, exp2i(ex));
      __syncthreads();
      run_conv(cv, b0, sa0, sa1, sb0, sb1, exp2i(-(ex + p.ew[cv])));
      if (kThinMfmaBufs == 1 && FMT != kFmtF16) __syncthreads();
      radius += (p.kt[cv] - 1) / 2 * p.dil[cv];
      if constexpr (FMT == kFmtF16) ex = block_exp(acc, radius);
      write_operand(acc, b1, exp2i(ex));
      __syncthreads();
      run_conv(cv + 1, b1, sb0, sb1, sa0, sa1, exp2i(-(ex + p.ew[cv + 1])));
      radius += (p.kt[cv + 1] - 1) / 2 * p.dil[cv + 1];
#pragma unroll
      for (int t = 0; t < NCT; ++t) xr[t] = acc[t] + xr[t];  // xt + x, :85
    }
    if (r == 0) {
#pragma unroll
      for (int t = 0; t < NCT; ++t) mrf[t] = xr[t];
    } else {
#pragma unroll
      for (int t = 0; t < NCT; ++t) mrf[t] = mrf[t] + xr[t];
    }
  }

  // y = mrf / n_res on the window centre
  float* __restrict__ yb = p.y + (int64_t)b * p.bs;
  float vmax = 0.f;  // max |stored value| (f16x3 consumers: p.amax_out)
#pragma unroll
  for (int t = 0; t < NCT; ++t) {
    const int col = cbase + 16 * t;
    if (!(vk[t] && col >= p.halo && col < p.halo + p.W)) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float v = mrf[t][i] / p.div;
      yb[(unsigned)(chan(i) * p.L + ws + col)] = v;
      vmax = fmaxf(vmax, fabsf(v));
    }
  }
  if (p.amax_out) amax_commit(vmax, p.amax_out, b);
}

namespace {

typedef void (*ThinMfmaFn)(const ThinParams);

struct EntryThinMfma {
  int C, np, fmt;
  ThinMfmaFn fn;
  char name[48];
};

// bf16x3 (NP 3, bf16), f16x3 (NP 3, f16), bf16w (NP 2 on the f16 kernel)
EntryThinMfma g_entriesThinMfma[] = {{16, 3, 0, mrf_thin_mfma<16, 3, 0>, {0}},
                                     {16, 3, 1, mrf_thin_mfma<16, 3, 1>, {0}},
                                     {16, 2, 1, mrf_thin_mfma<16, 2, 1>, {0}}};

EntryThinMfma* find_thin_mfma(int C, int fmt = 0, int np = 3) {
  for (auto& e : g_entriesThinMfma)
    if (e.C == C && e.np == np && e.fmt == fmt) return &e;
  return nullptr;
}

}  // namespace

int thin_mfma_window(int C) { return find_thin_mfma(C) ? 4 * kThinMfmaTiles * 16 : 0; }

size_t thin_mfma_lds_bytes(int C) {
  // operand planes + the f16x3 per-wave maxima
  return (size_t)kThinMfmaBufs * 2 * (4 * kThinMfmaTiles * 16 + 2 * kThinMarg) * 2 * C + 16;
}

hipError_t launch_mrf_thin_mfma(int C, int fmt, int np, const ThinParams& p, int batch,
                                hipStream_t stream, const char** name) {
  EntryThinMfma* e = find_thin_mfma(C, fmt, np);
  if (!e) return hipErrorInvalidValue;
  const int nwin = thin_mfma_window(C);
  if (p.n_res < 1 || p.n_res > kThinMaxRes || !p.wm) return hipErrorInvalidValue;
  if (p.W <= 0 || p.halo < 0 || p.W + 2 * p.halo > nwin) return hipErrorInvalidValue;
  if (p.rb_conv0[0] < 0 || p.rb_conv0[p.n_res] > kThinMaxConv) return hipErrorInvalidValue;
  for (int r = 0; r < p.n_res; ++r) {
    const int a = p.rb_conv0[r], z = p.rb_conv0[r + 1];
    if (z <= a || ((z - a) & 1)) return hipErrorInvalidValue;
    for (int cv = a; cv < z; ++cv)
      if (p.kt[cv] < 1 || p.dil[cv] < 1 || (p.kt[cv] - 1) / 2 * p.dil[cv] > kThinMarg ||
          (p.kt[cv] + 32 / C - 1) / (32 / C) > kThinMfmaMaxSteps ||
          // the last k-step's zero taps read (32/C - 1) * d rows past the conv's reach
          ((p.kt[cv] + 32 / C - 1) / (32 / C) * (32 / C) - 1 - (p.kt[cv] - 1) / 2) * p.dil[cv] >
              kThinMarg)
        return hipErrorInvalidValue;
  }
  const size_t lds = thin_mfma_lds_bytes(C);
  if (hipError_t err = ensure_max_lds(reinterpret_cast<const void*>(e->fn)))
    return err;
  {
    std::lock_guard<std::mutex> lk(setup_mutex());
    if (!e->name[0])
      snprintf(e->name, sizeof(e->name), "mrf_thin_mfma<%d, %d, %d>", e->C, e->np, e->fmt);
  }
  if (name) *name = e->name;
  const int n_tiles = (p.L + p.W - 1) / p.W;
  e->fn<<<dim3(n_tiles, batch), dim3(256), lds, stream>>>(p);
  return hipGetLastError();
}

}  // namespace hfg

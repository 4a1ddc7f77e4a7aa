// conv_ws_bf16x3.hip — warp-specialized split-precision implicit-GEMM Conv1d /
// polyphase ConvTranspose1d for the wide stages (GEMM rows M a multiple of 128).
//
// Same arithmetic as conv1d_bf16x3 (bf16 hi/lo operands, hi*hi + hi*lo + lo*hi in fp32
// on v_mfma_f32_32x32x16_bf16) and the same fused epilogues, organised so that the
// matrix cores never wait on HBM:
//
//   * 4 consumer waves (2 x 2, each 64 rows x 128 columns of the 128 x 256 block tile,
//     one per SIMD) run the MFMAs.  B (activations) comes from LDS, double-buffered per
//     k-step; A (weights) is streamed from global memory (L2-resident: every block of
//     the launch reads the same stream) by buffer loads two k-steps ahead, packed per
//     wave row-block as [m_tile][wave_m][group][tap][wm][plane][lane][8] — 4 x 1 KB
//     coalesced per k-step.
//   * 4 producer waves stage the input window of the NEXT 16-channel group (global
//     loads, pre-activation leaky_relu, hi/lo split) into the other half of a double
//     buffer.  vmcnt is per wave, so their HBM latency never stalls a consumer's wait
//     for its weight fragments.
//   * one block barrier per channel group (KT k-steps), none inside it.
//
// LDS operand layout per buffer: [half-group hp][plane hi/lo][row t][8 bf16], hp = the
// 8-channel half a lane reads (lane >> 5); 16-B rows, so the 16 lanes of a
// ds_read_b128 phase hit 16 distinct rows: conflict-free without a swizzle, and every
// tile / plane / tap offset is an immediate or one scalar add.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "bf16x3_common.h"
#include "epilogue.h"
#include "kernels.h"

namespace hfg {

namespace {
typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
}  // namespace

template <int KT, bool UPS>
__global__ void __launch_bounds__(64 * kWsWaves, 2)
conv_ws_bf16x3(const ConvParams p) {
  constexpr int WAVES_M = 2, WAVES_N = 2, WM = 2, WN = 4;
  constexpr int NCW = WAVES_M * WAVES_N;   // consumer waves (one per SIMD)
  constexpr int NPT = 64 * (kWsWaves - NCW);  // producer threads
  constexpr int MT = 32 * WM * WAVES_M;    // 128
  constexpr int NTILE = 32 * WN * WAVES_N; // 256
  constexpr int ASTEP = WM * 2 * 64 * 16;  // bytes per k-step of one wave row-block
  constexpr int XT = 4;                    // max staging tasks per producer thread
  static_assert(MT == kWsMT && NTILE == kWsNT, "tile constants");

  const int XW = NTILE + (KT - 1) * p.dil;  // staged window rows
  const int PS = XW * 16;                   // bytes per plane
  const int HPS = 2 * PS;                   // bytes per half-group (hi, lo)
  const int BUF = 2 * HPS;                  // bytes per buffer
  extern __shared__ __attribute__((aligned(16))) char lds[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n0 = blockIdx.x * NTILE;
  const int mt = blockIdx.y;
  const int b = blockIdx.z;
  const int half = lane >> 5;
  const int col = lane & 31;
  const int L_in_b = p.len_in ? p.len_in[b] : p.L_in;
  int N_b = p.N;
  if (p.len_out) {
    const int lo = p.len_out[b];
    N_b = UPS ? (lo > 0 ? (lo - 1 + p.ups_p) / p.ups_s + 1 : 0) : lo;
  }
  if (n0 >= N_b) return;  // whole tile past this utterance's end (block-uniform)
  const int L_out_b = (UPS && p.len_out) ? p.len_out[b] : p.L_out;
  const int NG = p.n_chunks;  // 16-channel groups

  if (wave >= NCW) {
    // ================= producer waves: stage input windows =================
    const int pt = tid - 64 * NCW;
    const float* __restrict__ xb = p.x + (int64_t)b * p.x_bs;
    const int xcs = (int)p.x_cs, xts = (int)p.x_ts;
    const int wbase = n0 + p.off;
    float xv[XT][8];
    auto load = [&](int g) {
      const bool full = g * 16 + 16 <= p.C_in;
#pragma unroll
      for (int q = 0; q < XT; ++q) {
        const int i = pt + q * NPT;
        const int t = i >> 1;
        const int cb = g * 16 + (i & 1) * 8;
        const int gi = wbase + t;
        const bool tok = (i < 2 * XW) && ((unsigned)gi < (unsigned)L_in_b);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const bool ok = tok && (full || cb + e < p.C_in);
          const unsigned off = ok ? (unsigned)((cb + e) * xcs + gi * xts) : 0u;
          const float v = xb[off];
          xv[q][e] = ok ? v : 0.f;
        }
      }
    };
    auto store = [&](int buf) {
#pragma unroll
      for (int q = 0; q < XT; ++q) {
        const int i = pt + q * NPT;
        if (i < 2 * XW) {
          bf16x8 h, l;
#pragma unroll
          for (int e = 0; e < 8; e += 2) {
            floatx2 a;
            a[0] = xv[q][e];
            a[1] = xv[q][e + 1];
            if (p.act_in) {
              a[0] = lrelu3(a[0]);
              a[1] = lrelu3(a[1]);
            }
            const bf16x2 hh = __builtin_convertvector(a, bf16x2);
            const floatx2 hf = __builtin_convertvector(hh, floatx2);
            const bf16x2 ll = __builtin_convertvector(a - hf, bf16x2);
            h[e] = hh[0];
            h[e + 1] = hh[1];
            l[e] = ll[0];
            l[e + 1] = ll[1];
          }
          char* dst = lds + buf * BUF + (i & 1) * HPS + (i >> 1) * 16;
          *reinterpret_cast<bf16x8*>(dst) = h;
          *reinterpret_cast<bf16x8*>(dst + PS) = l;
        }
      }
    };
    load(0);
    store(0);
    __syncthreads();
    for (int g = 0; g < NG; ++g) {
      if (g + 1 < NG) {
        load(g + 1);
        store((g + 1) & 1);
      }
      __syncthreads();
    }
    return;
  }

  // ================= consumer waves: MFMAs =================
  const int wave_m = wave % WAVES_M;
  const int wave_n = wave / WAVES_M;
  const int cbase = wave_n * 32 * WN;
  const int QT = NG * KT;
  const __amdgpu_buffer_rsrc_t wrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.w, 0, 0x7fffffff, 0x00020000);
  const int a_base = (mt * WAVES_M + wave_m) * QT * ASTEP;
  const int a_lane = lane * 16;
  bf16x8 ra_h[2][WM], ra_l[2][WM];
  auto load_a = [&](int slot, int q) {
    const int so = a_base + min(q, QT - 1) * ASTEP;
#pragma unroll
    for (int i = 0; i < WM; ++i) {
      ra_h[slot][i] = __builtin_bit_cast(
          bf16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, a_lane + i * 2048, so, 0));
      ra_l[slot][i] = __builtin_bit_cast(
          bf16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, a_lane + i * 2048 + 1024, so, 0));
    }
  };
  load_a(0, 0);
  load_a(1, 1);

  floatx16 acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int k = 0; k < WN; ++k)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][k][r] = 0.f;

  const int vb = half * HPS + (cbase + col) * 16;
  const int d = p.dil;
  bf16x8 bh[2][WN], bl[2][WN];
  // one channel group: KT k-steps from buffer `buf`; A ring slot of step j is (j + par) & 1,
  // B fragments double-buffered (step j+1's issued while step j's MFMAs run)
  auto group = [&](int g, int buf, int par) {
    const char* src0 = lds + buf * BUF + vb;
    auto load_b = [&](int bb, int j) {
      const char* src = src0 + j * d * 16;
#pragma unroll
      for (int k = 0; k < WN; ++k) {
        bh[bb][k] = *reinterpret_cast<const bf16x8*>(src + k * 512);
        bl[bb][k] = *reinterpret_cast<const bf16x8*>(src + k * 512 + PS);
      }
    };
    load_b(0, 0);
#pragma unroll
    for (int j = 0; j < KT; ++j) {
      const int sl = (j + par) & 1;
      const int cur = j & 1;
      if (j + 1 < KT) load_b(cur ^ 1, j + 1);
#pragma unroll
      for (int k = 0; k < WN; ++k)
#pragma unroll
        for (int i = 0; i < WM; ++i) {
          acc[i][k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ra_l[sl][i], bh[cur][k], acc[i][k], 0, 0, 0);
          acc[i][k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ra_h[sl][i], bl[cur][k], acc[i][k], 0, 0, 0);
          acc[i][k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ra_h[sl][i], bh[cur][k], acc[i][k], 0, 0, 0);
        }
      load_a(sl, g * KT + j + 2);
      if (j + 1 < KT) {
#pragma unroll
        for (int q = 0; q < 2 * WN; ++q) {
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // 2 MFMA
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read (next step's B)
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      } else {
        __builtin_amdgcn_sched_group_barrier(0x008, 18, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x020, 2 * WM, 0);  // A loads
      __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  __syncthreads();  // group 0 staged
  // groups in pairs so the A ring slot stays a compile-time index for odd KT
  for (int g = 0; g < NG; g += 2) {
    group(g, 0, 0);
    lds_barrier();  // paired with the producers' __syncthreads
    if (g + 1 < NG) {
      group(g + 1, 1, KT & 1);
      lds_barrier();
    }
  }

  // ---- epilogue ----
  const int row_base = mt * MT + wave_m * 32 * WM;
  const int n_base = n0 + cbase;
  if constexpr (UPS) {
    const int s_ = p.ups_s, p_ = p.ups_p;
    const bool vec4 = (s_ & 3) == 0 && (p_ & 3) == 0 && (p.L_out & 3) == 0;
    float* __restrict__ yb = p.y + (int64_t)b * p.y_bs;
#pragma unroll
    for (int i = 0; i < WM; ++i) {
    const int rb = row_base + i * 32 + 4 * half;
    float bv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) bv[r] = p.bias[rb + (r & 3) + 8 * (r >> 2)];
#pragma unroll
    for (int k = 0; k < WN; ++k) {
      const int n = n_base + k * 32 + col;
      if (n >= N_b) continue;
      if (vec4) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int row = rb + 8 * q;
          if (row >= p.M) continue;
          const int co = row / s_;
          const int t = n * s_ + (row - co * s_) - p_;
          float4 v;
          v.x = acc[i][k][4 * q + 0] + bv[4 * q + 0];
          v.y = acc[i][k][4 * q + 1] + bv[4 * q + 1];
          v.z = acc[i][k][4 * q + 2] + bv[4 * q + 2];
          v.w = acc[i][k][4 * q + 3] + bv[4 * q + 3];
          float* dst = yb + (int64_t)co * p.L_out + t;
          if (t >= 0 && t + 3 < L_out_b) {
            *reinterpret_cast<float4*>(dst) = v;
          } else {
            if (t + 0 >= 0 && t + 0 < L_out_b) dst[0] = v.x;
            if (t + 1 >= 0 && t + 1 < L_out_b) dst[1] = v.y;
            if (t + 2 >= 0 && t + 2 < L_out_b) dst[2] = v.z;
            if (t + 3 >= 0 && t + 3 < L_out_b) dst[3] = v.w;
          }
        }
        continue;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rb + (r & 3) + 8 * (r >> 2);
        if (row >= p.M) continue;
        const int co = row / s_;
        const int t = n * s_ + (row - co * s_) - p_;
        if (t >= 0 && t < L_out_b) yb[(int64_t)co * p.L_out + t] = acc[i][k][r] + bv[r];
      }
    }
    }
  } else {
    conv_epilogue<WM, WN>(p, acc, b, row_base, n_base, N_b, half, col);
  }
}

namespace {

typedef void (*WsFn)(const ConvParams);

struct EntryWs {
  int kt;
  bool ups;
  WsFn fn;
  bool attr;
  char name[64];
};

#define HFGWS_ENTRY(KT, UPS) \
  { KT, UPS, conv_ws_bf16x3<KT, UPS>, false, {0} }

EntryWs g_entriesWs[] = {HFGWS_ENTRY(3, false), HFGWS_ENTRY(5, false), HFGWS_ENTRY(7, false),
                         HFGWS_ENTRY(11, false), HFGWS_ENTRY(2, true)};

}  // namespace

bool ws_supported(int kt, bool ups, int M, int dil) {
  if (M % kWsMT != 0 || dil < 1 || dil > kMaxDil) return false;
  for (auto& e : g_entriesWs)
    if (e.kt == kt && e.ups == ups) return 2 * (kWsNT + (kt - 1) * dil) <= 4 * 64 * (kWsWaves - 4);
  return false;
}

size_t ws_lds_bytes(int kt, int dil) {
  return (size_t)2 * 4 * (kWsNT + (size_t)(kt - 1) * dil) * 16;
}

hipError_t launch_conv_ws_bf16x3(int kt, bool ups, const ConvParams& p, int n_tiles, int m_tiles,
                                 int batch, hipStream_t stream, const char** name) {
  EntryWs* e = nullptr;
  for (auto& cand : g_entriesWs)
    if (cand.kt == kt && cand.ups == ups) e = &cand;
  if (!e || !ws_supported(kt, ups, p.M, p.dil)) return hipErrorInvalidValue;
  if (!e->name[0])
    snprintf(e->name, sizeof(e->name), "conv_ws_bf16x3<%d, %s>", e->kt, e->ups ? "true" : "false");
  const size_t lds = ws_lds_bytes(kt, p.dil);
  if (!e->attr) {
    hipError_t err = hipFuncSetAttribute(reinterpret_cast<const void*>(e->fn),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (err != hipSuccess) return err;
    e->attr = true;
  }
  if (name) *name = e->name;
  e->fn<<<dim3(n_tiles, m_tiles, batch), dim3(64 * kWsWaves), lds, stream>>>(p);
  return hipGetLastError();
}

}  // namespace hfg

// resblock16_bf16x3.hip — the whole-ResBlock kernel of resblock_bf16x3.hip on the
// 16x16x32 bf16 MFMA shape (v_mfma_f32_16x16x32_bf16).
//
// Same algorithm, windowing and HBM traffic as resblock_bf16x3 (see that file):
//
//   for m in dilations:  x = x + conv2_m(lrelu(conv1_m(lrelu(x))))   models/hifigan.py:79-85
//   mrf = (mrf + x) [/ n_res]                                         models/hifigan.py:125-131
//
// Why a second shape: on random data the chip holds a higher clock under the 16x16x32
// instruction than under 32x32x16 at equal cycles per FLOP (MI355X_MICROARCH.md, MFMA
// shape note: 1.12-1.15x FLOP/s), and this kernel is matrix-core bound.
//
// Mapping.  Every wave owns 32 rows (2 row tiles of 16) x 128 columns (8 column tiles of
// 16) of the window; x (residual stream) and the conv accumulators live in registers in
// the 16x16 accumulator layout: lane l holds column (l & 15) and rows 4*(l >> 4) + r of a
// tile.  One k-step = 32 input channels (one wave row-block) x one tap: lane l reads the
// 8 slots 8q .. 8q+7 (q = l >> 4) of its column.  The operand slots of a 32-channel group
// are permuted, slot 8q + e <-> channel 16*(e >> 2) + 4q + (e & 3), so the 8 accumulator
// rows a lane holds for one column (2 row tiles x 4) are exactly the 8 slots it reads:
// writing the next conv's operand is one ds_write_b128 per plane and column tile.
//
// LDS operand layout per 32-channel group: [quarter q][plane hi/lo][row][8 bf16], 16-B
// rows: the 16 lanes of a quarter read 16 consecutive rows (conflict-free).
// A stream (host-packed, pack_resblock in hifigan_capi.cpp):
//   [wave_m][conv][group][tap][row tile][plane][lane][8], 4 KB per k-step and wave_m.
#include <hip/hip_runtime.h>

#include <mutex>

#include <cstdio>
#include <type_traits>

#include "bf16x3_common.h"
#include "kernels.h"

namespace hfg {

namespace {
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
}  // namespace

template <int KT, int WAVES_M, int WAVES_N, int NP>
__global__ void __launch_bounds__(64 * WAVES_M * WAVES_N, 2)  // 2 waves/SIMD: <= 256 VGPRs
resblock16_bf16x3(const RbParams p) {
  constexpr int NW = WAVES_M * WAVES_N;
  constexpr int NT = 64 * NW;
  constexpr int C = 32 * WAVES_M;
  constexpr int NG = C / 32;               // 32-channel groups (= wave row-blocks)
  constexpr int WI = 2;                    // 16-row MFMA tiles per wave
  constexpr int WN = 8;                    // 16-column MFMA tiles per wave
  constexpr int NWIN = 16 * WN * WAVES_N;  // window columns
  constexpr int STEPS = NG * KT;           // MFMA k-steps per conv
  constexpr int U = STEPS * WN;            // (step, column tile) units per conv
  constexpr int PF = 3;                    // B fragments prefetched this many units ahead
  constexpr int NB = 4;                    // B ring (WN % NB == 0: slot = column tile % NB)
  static_assert(WN % NB == 0 && PF < NB, "B ring");
  constexpr int MARG = rb_marg(C, WAVES_N);
  constexpr int ROWS = NWIN + 2 * MARG;
  constexpr int PS = ROWS * 16;            // bytes per plane: [row][8 bf16]
  constexpr int QS = 2 * PS;               // per quarter: hi, lo planes
  constexpr int GS = 4 * QS;               // per 32-channel group
  constexpr int ASTEP = WI * 2 * 64 * 16;  // bytes per k-step of one wave row-block
  static_assert(kRbColsPerWave == 16 * WN, "window columns per wave");

  extern __shared__ __attribute__((aligned(16))) char lds[];
  float* const bias_s = reinterpret_cast<float*>(lds + NG * GS);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wave_m = wave % WAVES_M;
  const int wave_n = wave / WAVES_M;
  const int quarter = lane >> 4;
  const int col = lane & 15;
  const int b = blockIdx.y;
  const int len_b = p.len ? min(p.len[b], p.L) : p.L;
  const int t0 = blockIdx.x * p.W;
  if (t0 >= len_b) return;  // whole block past this utterance's end (block-uniform)
  const int ws = t0 - p.halo;
  const int cbase = wave_n * 16 * WN;      // first window column of this wave
  const int row0 = wave_m * 32;
  const int n_conv = p.n_conv;
  // A stream: the whole ResBlock's convs (p.n_conv_stream per wave row-block); this launch
  // runs convs p.conv0 .. p.conv0 + n_conv - 1 of it (a ResBlock split into two launches)
  const int QT = p.n_conv_stream * STEPS;
  const int Q0 = p.conv0 * STEPS;
  const int dbg = p.dbg;
  // channel row of accumulator element r of row tile i
  auto rrow = [&](int i, int r) { return row0 + 16 * i + 4 * quarter + r; };

  for (int i = tid; i < n_conv * C; i += NT) bias_s[i] = p.bias[i];

  bool vk[WN];
#pragma unroll
  for (int k = 0; k < WN; ++k) vk[k] = (unsigned)(ws + cbase + 16 * k + col) < (unsigned)len_b;
  // every column of this wave inside [0, len)
  const bool wave_valid = (unsigned)(ws + cbase) < (unsigned)len_b &&
                          (unsigned)(ws + cbase + 16 * WN - 1) < (unsigned)len_b;

  // ---- A stream (buffer loads: SGPR descriptor + scalar step offset) ----
  const __amdgpu_buffer_rsrc_t wrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.w, 0, p.w_bytes, 0x00020000);
  const int a_base = wave_m * QT * ASTEP;
  const int a_lane = lane * 16;
  bf16x8 ra_h[2][WI], ra_l[2][WI];
  auto load_a = [&](int slot, int q) {
    asm volatile("" : "+s"(q));  // formed here, not hoisted (see load_b)
    const int so = a_base + min(q, QT - 1) * ASTEP;
#pragma unroll
    for (int i = 0; i < WI; ++i) {
      ra_h[slot][i] = __builtin_bit_cast(
          bf16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, a_lane + i * 2048, so, 0));
      ra_l[slot][i] = __builtin_bit_cast(
          bf16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, a_lane + i * 2048 + 1024, so, 0));
    }
  };
  load_a(0, Q0);
  load_a(1, Q0 + 1);

  // ---- residual stream x: window -> registers (zero outside [0, len)) ----
  floatx4 xcur[WI][WN];
  {
    const float* __restrict__ xb = p.x + (int64_t)b * p.bs;
#pragma unroll
    for (int k = 0; k < WN; ++k) {
      const int ta = ws + cbase + 16 * k + col;
#pragma unroll
      for (int i = 0; i < WI; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const unsigned off = vk[k] ? (unsigned)(rrow(i, r) * p.L + ta) : 0u;
          xcur[i][k][r] = (dbg & 32) ? 0.f : xb[off];
        }
    }
#pragma unroll
    for (int k = 0; k < WN; ++k)
#pragma unroll
      for (int i = 0; i < WI; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) xcur[i][k][r] = vk[k] ? xcur[i][k][r] : 0.f;
  }

  // lane's byte address of window column (cbase + col) in its quarter's hi plane
  const int vb = quarter * QS + (cbase + col + MARG) * 16;

  // B operand of the next conv: lrelu(v), zero outside [0, len), split hi/lo -> LDS
  auto write_operand = [&](const floatx4 (&v)[WI][WN]) {
    if (dbg & 64) return;
#pragma unroll
    for (int k = 0; k < WN; ++k) {
      bf16x8 h, l;
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        floatx2 a;
        a[0] = lrelu3(v[e >> 2][k][e & 3]);
        a[1] = lrelu3(v[e >> 2][k][(e & 3) + 1]);
        if (!wave_valid) {
          a[0] = vk[k] ? a[0] : 0.f;
          a[1] = vk[k] ? a[1] : 0.f;
        }
        const bf16x2 hh = __builtin_convertvector(a, bf16x2);
        const floatx2 hf = __builtin_convertvector(hh, floatx2);
        const bf16x2 ll = __builtin_convertvector(a - hf, bf16x2);
        h[e] = hh[0];
        h[e + 1] = hh[1];
        l[e] = ll[0];
        l[e + 1] = ll[1];
      }
      char* dst = lds + wave_m * GS + vb + k * 256;
      *reinterpret_cast<bf16x8*>(dst) = h;
      *reinterpret_cast<bf16x8*>(dst + PS) = l;
    }
  };
  write_operand(xcur);
  lds_barrier();

  // conv cv over the whole window: acc = bias + W_cv * operand.  PAR: A ring slot of the
  // conv's first step (its global step index cv*STEPS is odd for odd cv and odd STEPS).
  floatx4 acc[WI][WN];
  auto run_conv = [&](int cv, auto par_tag) {
    constexpr int PAR = decltype(par_tag)::value;
    const int d = p.dil[cv];
    const int pad = (KT - 1) / 2 * d;
#pragma unroll
    for (int i = 0; i < WI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float bv = bias_s[cv * C + rrow(i, r)];
#pragma unroll
        for (int k = 0; k < WN; ++k) acc[i][k][r] = bv;
      }
    bf16x8 bh[NB], bl[NB];
    // B fragment of (step s = (group g, tap j), column tile k): rows shifted by j*d - pad.
    // The address is formed here, not hoisted: with the conv unrolled the compiler would
    // otherwise keep every step's address live (VGPR / SGPR spills).
    auto load_b = [&](int s, int k) {
      const int g = s / KT, j = s - (s / KT) * KT;
      int va = vb, d16 = d * 16;
      asm volatile("" : "+v"(va), "+s"(d16));
      const char* src = lds + va + (g * GS + (j - (KT - 1) / 2) * d16) + k * 256;
      bh[k % NB] = *reinterpret_cast<const bf16x8*>(src);
      bl[k % NB] = *reinterpret_cast<const bf16x8*>(src + PS);
    };
    const int qb = Q0 + cv * STEPS;
    // one (step, column tile) unit: 6 MFMAs, the B fragment PF units ahead (the next
    // step's first ones clamped to the last step: a harmless re-read), and after the
    // step's last unit the A loads of step s + 2 into the step's ring slot SL
    auto unit = [&](int s, int k, auto sl_tag, bool pf) {
      constexpr int SL = decltype(sl_tag)::value;
      if (pf) {
        if (k + PF < WN) load_b(s, k + PF);
        else load_b(min(s + 1, STEPS - 1), k + PF - WN);
      }
#pragma unroll
      for (int i = 0; i < WI; ++i) {
        if constexpr (NP == 3)  // the weights' lo plane (zero for bf16-valued weights: NP 2)
          acc[i][k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ra_l[SL][i], bh[k % NB], acc[i][k], 0, 0, 0);
        acc[i][k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ra_h[SL][i], bl[k % NB], acc[i][k], 0, 0, 0);
        acc[i][k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ra_h[SL][i], bh[k % NB], acc[i][k], 0, 0, 0);
      }
      if (pf) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, NP * WI - 2, 0);  // rest of the unit's MFMAs
      } else {
        __builtin_amdgcn_sched_group_barrier(0x008, NP * WI, 0);
      }
      if (k == WN - 1) {
        load_a(SL, qb + s + 2);  // this step's A fragments are dead
        __builtin_amdgcn_sched_group_barrier(0x020, 2 * WI, 0);  // A loads
      }
      __builtin_amdgcn_sched_barrier(0);
    };
    using S0 = std::integral_constant<int, PAR>;
    using S1 = std::integral_constant<int, PAR ^ 1>;
#pragma unroll
    for (int k = 0; k < PF; ++k) load_b(0, k);
    if constexpr (STEPS <= 12) {
      // short convs: fully unrolled
#pragma unroll
      for (int s = 0; s < STEPS; ++s)
#pragma unroll
        for (int k = 0; k < WN; ++k) {
          const bool pf = s * WN + k + PF < U;
          if ((s & 1) == 0) unit(s, k, S0{}, pf);
          else unit(s, k, S1{}, pf);
        }
    } else {
      // long convs: two steps per iteration (keeps the A ring slot compile-time)
      static_assert(STEPS % 2 == 0, "runtime step loop needs an even step count");
      for (int s = 0; s < STEPS; s += 2) {
#pragma unroll
        for (int k = 0; k < WN; ++k) unit(s, k, S0{}, true);
#pragma unroll
        for (int k = 0; k < WN; ++k) unit(s + 1, k, S1{}, true);
      }
    }
    lds_barrier();
  };

  using P0 = std::integral_constant<int, 0>;
  using P1 = std::integral_constant<int, (STEPS & 1)>;
  // dilation pairs: xt = lrelu(conv1(lrelu(x)) + b1); x = x + (conv2(xt) + b2)
  for (int cv = 0; cv < n_conv; cv += 2) {
    run_conv(cv, P0{});
    write_operand(acc);
    lds_barrier();
    run_conv(cv + 1, P1{});
#pragma unroll
    for (int i = 0; i < WI; ++i)
#pragma unroll
      for (int k = 0; k < WN; ++k) xcur[i][k] = xcur[i][k] + acc[i][k];
    if (cv + 2 < n_conv) {
      write_operand(xcur);
      lds_barrier();
    }
  }

  // ---- MRF: (mrf + x) [/ n_res] on the window centre ----
  if (dbg & 16) {  // ablation: no MRF epilogue
    if (xcur[0][0][0] == 1.2345e-30f) p.mrf[0] = xcur[WI - 1][WN - 1][3];
    return;
  }
  float* __restrict__ mb = p.mrf + (int64_t)b * p.bs;
  const bool add = p.mrf_mode & 1;
  const bool div = p.mrf_mode & 2;
  // every column tile's MRF loads are issued before any store (see resblock_bf16x3.hip)
  unsigned rowoff[WI][4];
#pragma unroll
  for (int i = 0; i < WI; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) rowoff[i][r] = (unsigned)(rrow(i, r) * p.L);
  bool ok[WN];
  unsigned ta[WN];
#pragma unroll
  for (int k = 0; k < WN; ++k) {
    const int c = cbase + 16 * k + col;
    ok[k] = vk[k] && c >= p.halo && c < p.halo + p.W;
    ta[k] = ok[k] ? (unsigned)(ws + c) : 0u;
  }
  auto off = [&](int k, int i, int r) { return ok[k] ? rowoff[i][r] + ta[k] : 0u; };
  if (add) {
    float mv[WN][WI][4];
#pragma unroll
    for (int k = 0; k < WN; ++k)
#pragma unroll
      for (int i = 0; i < WI; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) mv[k][i][r] = mb[off(k, i, r)];
#pragma unroll
    for (int k = 0; k < WN; ++k)
#pragma unroll
      for (int i = 0; i < WI; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) xcur[i][k][r] = mv[k][i][r] + xcur[i][k][r];
  }
#pragma unroll
  for (int k = 0; k < WN; ++k) {
    if (div) {
#pragma unroll
      for (int i = 0; i < WI; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) xcur[i][k][r] = xcur[i][k][r] / p.mrf_div;
    }
    if (ok[k]) {
#pragma unroll
      for (int i = 0; i < WI; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) mb[off(k, i, r)] = xcur[i][k][r];
    }
  }
}

namespace {

typedef void (*Rb16Fn)(const RbParams);

struct EntryRb16 {
  int kt, waves_m, waves_n, np;
  Rb16Fn fn;
  char name[64];
};

#define HFGRB16_ENTRY(KT, WMS, WNS, NP) \
  { KT, WMS, WNS, NP, resblock16_bf16x3<KT, WMS, WNS, NP>, {0} }
#define HFGRB16_KTS(WMS, WNS, NP)                                                           \
  HFGRB16_ENTRY(3, WMS, WNS, NP), HFGRB16_ENTRY(5, WMS, WNS, NP),                         \
      HFGRB16_ENTRY(7, WMS, WNS, NP), HFGRB16_ENTRY(11, WMS, WNS, NP)

// NP 3: bf16x3 products; NP 2: bf16-valued weights (HFG_DTYPE_BF16W)
EntryRb16 g_entriesRb16[] = {HFGRB16_KTS(2, 4, 3), HFGRB16_KTS(1, 8, 3), HFGRB16_KTS(1, 4, 3),
                             HFGRB16_ENTRY(3, 4, 2, 3), HFGRB16_KTS(2, 4, 2),
                             HFGRB16_KTS(1, 8, 2), HFGRB16_KTS(1, 4, 2), HFGRB16_ENTRY(3, 4, 2, 2)};

}  // namespace

bool rb16_supported(int C, int kt, int waves_n) {
  if (C % 32 != 0) return false;
  for (auto& e : g_entriesRb16)
    if (e.kt == kt && e.waves_m == C / 32 && e.waves_n == waves_n && e.np == 3) return true;
  return false;
}

hipError_t launch_resblock16_bf16x3(int C, int waves_n, int kt, int np, const RbParams& p,
                                    int batch, hipStream_t stream, const char** name) {
  const int wm = C / 32;
  EntryRb16* e = nullptr;
  for (auto& cand : g_entriesRb16)
    if (cand.kt == kt && cand.waves_m == wm && cand.waves_n == waves_n && cand.np == np) e = &cand;
  if (!e || C % 32 != 0) return hipErrorInvalidValue;
  const int nwin = kRbColsPerWave * waves_n;
  if (p.n_conv < 2 || p.n_conv > kRbMaxConv || (p.n_conv & 1)) return hipErrorInvalidValue;
  if (p.conv0 < 0 || p.conv0 + p.n_conv > p.n_conv_stream) return hipErrorInvalidValue;
  if (p.W <= 0 || p.halo < 0 || p.W + 2 * p.halo > nwin) return hipErrorInvalidValue;
  for (int i = 0; i < p.n_conv; ++i)
    if (p.dil[i] < 1 || (kt - 1) / 2 * p.dil[i] > rb_marg(C, waves_n)) return hipErrorInvalidValue;
  {
    std::lock_guard<std::mutex> lk(setup_mutex());
    if (!e->name[0])
      snprintf(e->name, sizeof(e->name), "resblock16_bf16x3<%d, %d, %d, %d>", e->kt, e->waves_m,
               e->waves_n, e->np);
  }
  const size_t lds = rb_lds_bytes(C, waves_n, p.n_conv);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (hipError_t err = ensure_max_lds(reinterpret_cast<const void*>(e->fn)))
    return err;
  if (name) *name = e->name;
  const int n_tiles = (p.L + p.W - 1) / p.W;
  e->fn<<<dim3(n_tiles, batch), dim3(64 * wm * waves_n), lds, stream>>>(p);
  return hipGetLastError();
}

}  // namespace hfg

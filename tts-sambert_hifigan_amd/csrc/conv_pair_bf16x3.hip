// conv_pair_bf16x3.hip — one ResBlock dilation step in one launch (bf16x3 MFMA):
//
//   out = x + conv2(lrelu(conv1(lrelu(x))))        models/hifigan.py:79-85
//
// (plus the MRF running sum / final division when the step ends a ResBlock,
// :125-131) for C in {32, 64} channels, where a layer-per-launch schedule is bound by
// HBM round trips and launch tails rather than by the matrix cores: conv1's output
// (the reference's `xt`) stays in LDS.
//
// A block owns T = 128 - (k-1) output columns [n0, n0+T) of one utterance.
//   phase 1: conv1 over the 128 columns t1 = n0 - p2 + j (p2 = (k-1)/2, conv2's
//            padding), K = (channel group of 16, tap), input window staged per channel
//            group exactly as in conv1d_bf16x3; the epilogue adds the bias, applies
//            leaky_relu, zeroes t1 outside [0, len) (conv2's zero padding), splits
//            hi/lo and writes all C channels to LDS as [group][plane][row][16 ch].
//   phase 2: conv2 (dilation 1) reading those rows as its B operand; epilogue =
//            bias + residual x (+ MRF), columns >= T discarded.
// The weight-slab ring runs across both phases (conv2's first slabs land while
// conv1 finishes).  Weights use the layer-wise packing of conv1d_bf16x3 tile 1
// (C = 64: one 64-row m-tile, 2 taps per chunk) or tile 2 (C = 32, 4 taps per chunk).
#include <hip/hip_runtime.h>

#include <cstdio>

#include "bf16x3_common.h"
#include "epilogue.h"
#include "kernels.h"

namespace hfg {

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

template <int KT_, int TPC, int WM, int WD>
__global__ void __launch_bounds__(256, 2)
conv_pair_bf16x3(const ConvParams p) {
  constexpr int NW = 4;                   // 1 x 4 waves, each 32*WM rows x 32 columns
  constexpr int NT = 64 * NW;
  constexpr int MT = 32 * WM;             // = C (C_in = C_out)
  constexpr int NTILE = kPairCols;        // GEMM columns per phase
  static_assert(NTILE == 32 * NW, "one 32-column block per wave");
  constexpr int NG = MT / 16;             // channel groups
  constexpr int XROW = 16;
  constexpr int TAP_ELEMS = 2 * WM * 64 * 8;
  constexpr int SLAB = TPC * TAP_ELEMS;
  constexpr int KT_MAX = KT_ > 0 ? KT_ : 16;
  constexpr int XW_MAX = NTILE + (KT_MAX - 1) * kMaxDil;
  constexpr int XQ = (2 * XW_MAX + NT - 1) / NT;
  static_assert(XQ * 8 <= 32, "ok mask");
  constexpr int NX = XQ * 8;
  constexpr int PW = SLAB / 8 / 64 / NW;
  static_assert(PW * 8 * 64 * NW == SLAB, "slab must split evenly over the waves");
  static_assert(NX + PW < 64, "vmcnt range");
  const int KT = KT_ > 0 ? KT_ : p.kt;
  const int n_tg = (KT + TPC - 1) / TPC;
  const int n1 = NG * n_tg;               // chunks per conv
  const int n_all = 2 * n1;
  const int dil = p.dil;
  const int p1 = (KT - 1) * dil / 2, p2 = (KT - 1) / 2;
  const int T_out = NTILE - (KT - 1);
  const int XW = NTILE + (KT - 1) * dil;
  const int xplane = (XW * XROW + 7) & ~7;
  const int xbuf = 2 * xplane;
  const int trows = (NTILE + KT - 1 + 7) & ~7;  // conv1 rows kept per group (+ k-1 spare)
  const int tplane = trows * XROW;

  extern __shared__ __attribute__((aligned(16))) __bf16 lds16[];
  __bf16* const Wbuf0 = lds16;
  __bf16* const Xbuf0 = lds16 + WD * SLAB;
  __bf16* const Tbuf0 = Xbuf0 + 2 * xbuf;  // [group][plane hi/lo][trows][16]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int half = lane >> 5;
  const int col = lane & 31;
  const int n0 = blockIdx.x * T_out;
  const int b = blockIdx.z;
  const int N_b = p.len_out ? p.len_out[b] : p.N;
  if (n0 >= N_b) return;
  const int L_b = p.len_in ? p.len_in[b] : p.L_in;
  const float* __restrict__ xb = p.x + (int64_t)b * p.x_bs;
  const __bf16* __restrict__ w1 = reinterpret_cast<const __bf16*>(p.w);
  const __bf16* __restrict__ w2 = reinterpret_cast<const __bf16*>(p.w2);
  const int xcs = (int)p.x_cs;
  const int wbase = n0 - p2 - p1;         // input index of window row 0

  auto taps_in = [&](int c) {
    const int rem = KT - (c % n_tg) * TPC;
    return rem < TPC ? rem : TPC;
  };
  auto issue_w = [&](int c, __bf16* Ws) {
    const __bf16* src = c < n1 ? w1 + (int64_t)c * SLAB : w2 + (int64_t)(c - n1) * SLAB;
#pragma unroll
    for (int q = 0; q < PW; ++q) {
      const int i = wave + q * NW;
      __builtin_amdgcn_global_load_lds((gptr_t1)(src + (i * 64 + lane) * 8),
                                       (lds_ptr_t3)(Ws + i * 512), 16, 0, 0);
    }
  };
  // input window of channel group g: raw loads now, leaky_relu + split at store
  float xv[XQ][8];
  uint32_t xok = 0;
  auto load_x = [&](int g) {
    xok = 0;
#pragma unroll
    for (int q = 0; q < XQ; ++q) {
      const int i = tid + q * NT;
      const int t = i >> 1;
      const int cb = g * 16 + (i & 1) * 8;
      const int gi = wbase + t;
      const bool tok = (i < 2 * XW) && ((unsigned)gi < (unsigned)L_b);
      const unsigned o0 = tok ? (unsigned)(cb * xcs + gi) * 4u : 0u;
      const unsigned step = tok ? (unsigned)xcs * 4u : 0u;
      xok |= (tok ? 0xffu : 0u) << (q * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e)
        xv[q][e] = *reinterpret_cast<const float*>(reinterpret_cast<const char*>(xb) + o0 + e * step);
    }
  };
  auto store_x = [&](__bf16* Xh) {
    __bf16* Xl = Xh + xplane;
#pragma unroll
    for (int q = 0; q < XQ; ++q) {
      const int i = tid + q * NT;
      if (i < 2 * XW) {
        bf16x8 h, l;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = lrelu3((xok >> (q * 8 + e)) & 1u ? xv[q][e] : 0.f);
          const __bf16 hh = (__bf16)v;
          h[e] = hh;
          l[e] = (__bf16)(v - (float)hh);
        }
        const int t = i >> 1;
        const int off = t * XROW + 8 * ((i & 1) ^ ((t >> 3) & 1));
        *reinterpret_cast<bf16x8*>(Xh + off) = h;
        *reinterpret_cast<bf16x8*>(Xl + off) = l;
      }
    }
  };

  floatx16 acc[WM];
  auto zero_acc = [&]() {
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
  };
  struct Frag {
    bf16x8 ah[WM], al[WM], bh, bl;
  };
  // B rows: column (wave*32 + col) + tap*dl of the staged [row][16] planes at Xh / Xh+pl
  auto load_frag = [&](const __bf16* Ws, const __bf16* Xh, int pl, int jj, int tap, int dl,
                       Frag& f) {
#pragma unroll
    for (int i = 0; i < WM; ++i) {
      const __bf16* a = Ws + jj * TAP_ELEMS + i * 512 + lane * 8;
      f.ah[i] = *reinterpret_cast<const bf16x8*>(a);
      f.al[i] = *reinterpret_cast<const bf16x8*>(a + WM * 512);
    }
    const int t = wave * 32 + col + tap * dl;
    const int off = t * XROW + 8 * (half ^ ((t >> 3) & 1));
    f.bh = *reinterpret_cast<const bf16x8*>(Xh + off);
    f.bl = *reinterpret_cast<const bf16x8*>(Xh + pl + off);
  };
  auto mma = [&](const Frag& f) {
#pragma unroll
    for (int i = 0; i < WM; ++i) {
      acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.al[i], f.bh, acc[i], 0, 0, 0);
      acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.ah[i], f.bl, acc[i], 0, 0, 0);
      acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.ah[i], f.bh, acc[i], 0, 0, 0);
    }
  };
  // taps of chunk c from the B planes at Xh (plane stride pl), dilation dl
  auto chunk_mma = [&](int c, const __bf16* Ws, const __bf16* Xh, int pl, int dl) {
    const int nt = taps_in(c);
    const int tap0 = (c % n_tg) * TPC;
    Frag f0, f1;
    load_frag(Ws, Xh, pl, 0, tap0, dl, f0);
#pragma unroll
    for (int jj = 0; jj < TPC; jj += 2) {
      if (jj < nt) {
        if (jj + 1 < nt) load_frag(Ws, Xh, pl, jj + 1, tap0 + jj + 1, dl, f1);
        mma(f0);
        if (jj + 2 < nt) load_frag(Ws, Xh, pl, jj + 2, tap0 + jj + 2, dl, f0);
        if (jj + 1 < nt) mma(f1);
      }
    }
  };

  // ---- prologue: zero conv1's spare rows, first slabs, input window of group 0 ----
  for (int i = tid; i < NG * 2 * (trows - NTILE); i += NT) {
    const int gp = i / (trows - NTILE), r = NTILE + i % (trows - NTILE);
    *reinterpret_cast<bf16x8*>(Tbuf0 + gp * tplane + r * XROW) = bf16x8{};
    *reinterpret_cast<bf16x8*>(Tbuf0 + gp * tplane + r * XROW + 8) = bf16x8{};
  }
  load_x(0);
#pragma unroll
  for (int c = 0; c < WD - 1; ++c) issue_w(c, Wbuf0 + c * SLAB);
  store_x(Xbuf0);
  wait_vm<0>();
  lds_barrier();
  zero_acc();

  int wslot = 0;
  const int xg = n_tg >= 2 ? n_tg - 2 : 0;
  for (int c = 0; c < n_all; ++c) {
    const bool ph1 = c < n1;
    const int cc = ph1 ? c : c - n1;
    const int g = cc / n_tg, tg = cc - (cc / n_tg) * n_tg;
    const __bf16* Ws = Wbuf0 + wslot * SLAB;
    const bool more_groups = ph1 && (g + 1) * n_tg < n1;
    const bool issue_x = more_groups && tg == xg;
    const bool store_now = more_groups && tg == n_tg - 1;
    auto issue_next_w = [&]() {
      int s2 = wslot + WD - 1;
      if (s2 >= WD) s2 -= WD;
      issue_w(min(c + WD - 1, n_all - 1), Wbuf0 + s2 * SLAB);
    };
    const bool w_late = WD > 2 && store_now;
    if (!w_late) issue_next_w();
    if (issue_x) load_x(g + 1);
    if (ph1)
      chunk_mma(c, Ws, Xbuf0 + (g & 1) * xbuf, xplane, dil);
    else
      chunk_mma(c, Ws, Tbuf0 + g * 2 * tplane, tplane, 1);
    if (store_now) store_x(Xbuf0 + ((g + 1) & 1) * xbuf);
    if (w_late) issue_next_w();
    if (issue_x && !store_now) wait_vm<NX + PW * (WD - 2)>();
    else wait_vm<PW * (WD - 2)>();
    lds_barrier();
    if (++wslot == WD) wslot = 0;

    if (c == n1 - 1) {
      // ---- phase-1 epilogue: xt = lrelu(conv1 + bias) -> LDS (hi/lo split) ----
      const int j = wave * 32 + col;
      const int t1 = n0 - p2 + j;
      const bool tok = (unsigned)t1 < (unsigned)L_b;
      const int swz = (j >> 3) & 1;
#pragma unroll
      for (int i = 0; i < WM; ++i) {
#pragma unroll
        for (int grp = 0; grp < 2; ++grp) {
          __bf16* Th = Tbuf0 + (2 * i + grp) * 2 * tplane + j * XROW + 4 * half;
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            bf16x4 vh, vl;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int r = grp * 8 + hh * 4 + e;
              float v = acc[i][r] + p.bias[i * 32 + 16 * grp + 8 * hh + 4 * half + e];
              v = tok ? lrelu3(v) : 0.f;
              const __bf16 vhi = (__bf16)v;
              vh[e] = vhi;
              vl[e] = (__bf16)(v - (float)vhi);
            }
            *reinterpret_cast<bf16x4*>(Th + 8 * (hh ^ swz)) = vh;
            *reinterpret_cast<bf16x4*>(Th + tplane + 8 * (hh ^ swz)) = vl;
          }
        }
      }
      lds_barrier();
      zero_acc();
    }
  }

  // ---- phase-2 epilogue: bias + residual (+ MRF), columns [n0, n0 + T_out) ----
  floatx16 acc2[WM][1];
#pragma unroll
  for (int i = 0; i < WM; ++i) acc2[i][0] = acc[i];
  conv_epilogue<WM, 1>(p, p.bias2, acc2, b, 0, n0 + wave * 32, min(N_b, n0 + T_out), half, col);
}

namespace {

typedef void (*PairFn)(const ConvParams);

struct PairCfg {
  int TPC, WM, WD;
};
// tile 1 (C = 64) and tile 2 (C = 32) of the layer-wise kernel: same weight packing
constexpr PairCfg kPairCfg[3] = {{0, 0, 0}, {2, 2, 2}, {4, 1, 2}};

template <int KT, int TILE>
struct InstP {
  static constexpr PairCfg c = kPairCfg[TILE];
  static PairFn fn() { return conv_pair_bf16x3<KT, c.TPC, c.WM, c.WD>; }
};

struct EntryP {
  int kt;
  int tile;
  PairFn fn;
  bool attr;
  char name[80];
};

#define HFGP_ENTRY(KT, TILE) \
  { KT, TILE, InstP<KT, TILE>::fn(), false, {0} }
#define HFGP_TILES(KT) HFGP_ENTRY(KT, 1), HFGP_ENTRY(KT, 2)

EntryP g_entriesP[] = {HFGP_TILES(3), HFGP_TILES(5), HFGP_TILES(7), HFGP_TILES(11),
                       HFGP_TILES(0)};

}  // namespace

size_t pair_lds_bytes(int tile, int kt, int dil) {
  const PairCfg& c = kPairCfg[tile];
  const size_t slab = (size_t)c.TPC * 2 * 32 * c.WM * 16;  // bf16
  const size_t xw = kPairCols + (size_t)(kt - 1) * dil;
  const size_t xplane = (xw * 16 + 7) & ~(size_t)7;
  const size_t trows = (kPairCols + kt - 1 + 7) & ~(size_t)7;
  const size_t ng = 2 * c.WM;  // 16-channel groups of C = 32*WM
  return sizeof(__bf16) * (c.WD * slab + 2 * 2 * xplane + ng * 2 * trows * 16);
}

hipError_t launch_pair_bf16x3(int tile, int kt, const ConvParams& p, int n_tiles, int batch,
                              hipStream_t stream, const char** name) {
  if (tile != 1 && tile != 2) return hipErrorInvalidValue;
  if (kt < 1 || kt > 16 || p.dil < 1 || p.dil > kMaxDil) return hipErrorInvalidValue;
  if (p.C_in != 32 * kPairCfg[tile].WM || p.M != p.C_in || p.x_ts != 1) return hipErrorInvalidValue;
  EntryP* e = nullptr;
  EntryP* generic = nullptr;
  for (auto& cand : g_entriesP) {
    if (cand.tile != tile) continue;
    if (cand.kt == kt) e = &cand;
    if (cand.kt == 0) generic = &cand;
  }
  if (!e) e = generic;
  if (!e) return hipErrorInvalidValue;
  const PairCfg& c = kPairCfg[tile];
  if (!e->name[0])
    snprintf(e->name, sizeof(e->name), "conv_pair_bf16x3<%d, %d, %d, %d>", e->kt, c.TPC, c.WM,
             c.WD);
  const size_t lds = pair_lds_bytes(tile, kt, p.dil);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (!e->attr) {
    hipError_t err = hipFuncSetAttribute(reinterpret_cast<const void*>(e->fn),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (err != hipSuccess) return err;
    e->attr = true;
  }
  if (name) *name = e->name;
  e->fn<<<dim3(n_tiles, 1, batch), dim3(256), lds, stream>>>(p);
  return hipGetLastError();
}

}  // namespace hfg

// conv16_bf16x3.hip — the wide-layer split-precision implicit-GEMM Conv1d / polyphase
// ConvTranspose1d of conv_bf16x3.hip (tile 3) on the 16x16x32 bf16 MFMA shape
// (v_mfma_f32_16x16x32_bf16).  Same arithmetic (hi*hi + hi*lo + lo*hi in fp32), same
// epilogue contracts.  Why: on random data the chip holds a higher clock under the
// 16x16x32 instruction at equal cycles per FLOP (MI355X_MICROARCH.md, MFMA shape note),
// and this kernel is bound by the matrix pipe.
//
// Block tile 128 x 256: 2 x 2 waves of 64 x 128 = 4 x 8 tiles of 16 x 16 (128 fp32
// accumulators per lane), 256 threads, 2 blocks per CU.
//
// K order.  K is walked as the flattened list f = g*KT + j of (16-channel group g, tap j)
// entries; one k-step (K = 32) takes the two entries f = 2s (lanes 0-31) and f = 2s + 1
// (lanes 32-63), lane l holding channels 8*((l >> 4) & 1) .. +7 of its entry.  With an
// odd tap count a step straddles two channel groups, so no tap is padded.  The channel
// group count is even (host-checked): a unit of two groups is KT k-steps whose entries
// are compile-time, and the input windows of the two groups live in the two buffers.
//   * A: host-packed per k-step [m_tile][step][plane][wave_m][row tile][lane][8]
//     (16 KB), streamed to LDS by global_load_lds_dwordx4 through a 2-slot ring;
//   * B: a group's input window [t][16 ch] bf16 hi/lo planes, 16-B halves XOR-swizzled
//     by (t >> 3) & 1 (conflict-free ds_read_b128 of 16 consecutive rows per quarter);
//     the next groups' windows are loaded one step before they are stored, and both the
//     loads and the conversion + store are interleaved into that step's MFMA stream.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <type_traits>

#include "bf16x3_common.h"
#include "kernels.h"

namespace hfg {

namespace {
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

// staging schedule of one unit (two groups G0, G1 = KT k-steps): G1's window is stored
// at the end of step st1 (it is first read at step KT/2), the next unit's G0 at the last
// step; each is loaded one step earlier when the previous store leaves room
struct C16Sched {
  int st1, ld1, st2, ld2;
};
constexpr C16Sched c16_sched(int KT) {
  const int st1 = KT / 2 - 1;
  const int ld1 = st1 - 1 > -1 ? st1 - 1 : st1;
  const int st2 = KT - 1;
  const int ld2 = st2 - 1 > st1 ? st2 - 1 : st2;
  return {st1, ld1, st2, ld2};
}
}  // namespace

template <int KT, bool UPS>
__global__ void __launch_bounds__(256, 2)
conv16_bf16x3(const ConvParams p) {
  static_assert(KT >= 2, "two entries per k-step");
  constexpr int WAVES_M = 2, WI = 4, WN = 8;
  constexpr int NW = 4, NT = 256;
  constexpr int MT = kC16MT, NTILE = kC16NT;
  constexpr int XROW = 16;                         // bf16 per staged row (16 channels)
  constexpr int SLAB = 2 * MT * 32;                // bf16 per k-step slab (hi, lo)
  constexpr int PSTR = WAVES_M * WI * 512;         // bf16 between the hi and lo planes
  constexpr int PW = SLAB / 8 / 64 / NW;           // LDS-DMA pieces per thread per slab
  static_assert(PW * 8 * 64 * NW == SLAB, "slab split");
  constexpr int XW_MAX = NTILE + kC16MaxHalo;
  constexpr int XQ = (2 * XW_MAX + NT - 1) / NT;   // staging tasks per thread
  static_assert(XQ * 8 <= 32, "ok mask");
  constexpr int NX = XQ * 8;
  static_assert(NX + PW < 64, "vmcnt range");
  constexpr C16Sched SCH = c16_sched(KT);

  const int XW = NTILE + (KT - 1) * p.dil;
  const int xplane = XW * XROW;
  const int xbuf = 2 * xplane;
  extern __shared__ __attribute__((aligned(16))) __bf16 lds16[];
  __bf16* const Wbuf0 = lds16;
  __bf16* const Xbuf0 = lds16 + 2 * SLAB;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const int wave_m = wave % WAVES_M;
  const int wave_n = wave / WAVES_M;
  const int quarter = lane >> 4;
  const int col = lane & 15;
  const bool ent = lane >= 32;       // entry f = 2s + 1 of the k-step
  const int hh = quarter & 1;        // 8-channel half of the entry's group
  const int n0 = blockIdx.x * NTILE;
  const int mt = blockIdx.y;
  const int b = blockIdx.z;
  const float* __restrict__ xb = p.x + (int64_t)b * p.x_bs;
  const int P = p.n_chunks;          // k-steps
  const __bf16* __restrict__ wsrc = reinterpret_cast<const __bf16*>(p.w) + (int64_t)mt * P * SLAB;
  const int L_in_b = p.len_in ? p.len_in[b] : p.L_in;
  int N_b = p.N;
  if (p.len_out) {
    const int lo = p.len_out[b];
    N_b = UPS ? (lo > 0 ? (lo - 1 + p.ups_p) / p.ups_s + 1 : 0) : lo;
  }
  if (n0 >= N_b) return;  // whole tile past this utterance's end (block-uniform)
  const int L_out_b = (UPS && p.len_out) ? p.len_out[b] : p.L_out;
  const int xcs = (int)p.x_cs, xts = (int)p.x_ts;
  const int wbase = n0 + p.off;
  const int NG = (p.C_in + 15) / 16;  // even (host-checked)
  const int NU = NG / 2;

  // ---- weight slab of k-step s -> LDS slot (PW pieces per thread, always) ----
  auto issue_w = [&](int s, int slot) {
    const __bf16* src = wsrc + (int64_t)s * SLAB;
    __bf16* dst = Wbuf0 + slot * SLAB;
    int lo = lane * 8;  // opaque: per-step addresses are formed here, not hoisted
    asm volatile("" : "+v"(lo));
#pragma unroll
    for (int q = 0; q < PW; ++q) {
      const int i = wave_u + q * NW;
      __builtin_amdgcn_global_load_lds((gptr_t1)(src + i * 512 + lo),
                                       (lds_ptr_t3)(dst + i * 512), 16, 0, 0);
    }
  };
  // ---- input window of channel group g: raw loads (clamped offsets), zero padding
  // applied at the LDS store from a bit mask ----
  float xv[XQ][8];
  uint32_t xok = 0;
  // a wave with no task in the last staging row skips its loads: 8 fewer in flight, which
  // the vmcnt wait after the loading step must count (else it passes before the slab DMA)
  const bool x_short = XQ > 1 && (XQ - 1) * NT + wave_u * 64 >= 2 * XW;
  auto load_x = [&](int g) {
    const bool full = g * 16 + 16 <= p.C_in;  // block-uniform
    xok = 0;
#pragma unroll
    for (int q = 0; q < XQ; ++q) {
      if (q == XQ - 1 && q > 0 && x_short) continue;
      const int i = tid + q * NT;
      const int t = i >> 1;
      const int cb = g * 16 + (i & 1) * 8;
      const int gi = wbase + t;
      const bool tok = (i < 2 * XW) && ((unsigned)gi < (unsigned)L_in_b);
      const unsigned o0 = tok ? (unsigned)(cb * xcs + gi * xts) * 4u : 0u;
      const unsigned step = tok ? (unsigned)xcs * 4u : 0u;
      const int ecap = full ? 7 : min(p.C_in - 1 - cb, 7);
      const uint32_t m8 = tok ? (ecap >= 7 ? 0xffu : (ecap < 0 ? 0u : (1u << (ecap + 1)) - 1u)) : 0u;
      xok |= m8 << (q * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const unsigned oe = o0 + (unsigned)(full ? e : max(min(e, ecap), 0)) * step;
        xv[q][e] = *reinterpret_cast<const float*>(reinterpret_cast<const char*>(xb) + oe);
      }
    }
  };
  auto store_x = [&](int buf) {
    __bf16* Xh = Xbuf0 + buf * xbuf;
    __bf16* Xl = Xh + xplane;
#pragma unroll
    for (int q = 0; q < XQ; ++q) {
      const int i = tid + q * NT;
      if (i < 2 * XW) {
        bf16x8 h, l;
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          floatx2 a;
          a[0] = (xok >> (q * 8 + e)) & 1u ? xv[q][e] : 0.f;
          a[1] = (xok >> (q * 8 + e + 1)) & 1u ? xv[q][e + 1] : 0.f;
          if (p.act_in) {
            a[0] = lrelu3(a[0]);
            a[1] = lrelu3(a[1]);
          }
          const bf16x2 hb = __builtin_convertvector(a, bf16x2);
          const floatx2 hf = __builtin_convertvector(hb, floatx2);
          const bf16x2 lb = __builtin_convertvector(a - hf, bf16x2);
          h[e] = hb[0];
          h[e + 1] = hb[1];
          l[e] = lb[0];
          l[e + 1] = lb[1];
        }
        const int t = i >> 1;
        const int off = t * XROW + 8 * ((i & 1) ^ ((t >> 3) & 1));
        *reinterpret_cast<bf16x8*>(Xh + off) = h;
        *reinterpret_cast<bf16x8*>(Xl + off) = l;
      }
    }
  };

  floatx4 acc[WI][WN];
#pragma unroll
  for (int i = 0; i < WI; ++i)
#pragma unroll
    for (int k = 0; k < WN; ++k) acc[i][k] = floatx4{0.f, 0.f, 0.f, 0.f};

  // one k-step: A fragments of the 4 row tiles, B fragments streamed per column tile
  // (two in flight).  gg0/j0, gg1/j1: (group in unit, tap) of the step's two entries.
  // The B address is formed inside the step from opaque copies of its inputs: with the
  // unit unrolled the compiler would otherwise hoist every step's address out of the
  // unit loop and keep them all live (VGPR spills).
  auto kstep = [&](int slot, int gg0, int j0, int gg1, int j1) {
    const __bf16* Ws = Wbuf0 + slot * SLAB;
    bf16x8 ah[WI], al[WI], bh[2], bl[2];
#pragma unroll
    for (int i = 0; i < WI; ++i) {
      const __bf16* a = Ws + (wave_m * WI + i) * 512 + lane * 8;
      ah[i] = *reinterpret_cast<const bf16x8*>(a);
      al[i] = *reinterpret_cast<const bf16x8*>(a + PSTR);
    }
    int tr = wave_n * 128 + col, dd = p.dil;
    asm volatile("" : "+v"(tr), "+s"(dd));
    tr += (ent ? j1 : j0) * dd;
    const __bf16* Xb = Xbuf0 + (ent ? gg1 : gg0) * xbuf + tr * XROW + 8 * (hh ^ ((tr >> 3) & 1));
    auto ldb = [&](int k) {
      bh[k & 1] = *reinterpret_cast<const bf16x8*>(Xb + k * 256);
      bl[k & 1] = *reinterpret_cast<const bf16x8*>(Xb + xplane + k * 256);
    };
    ldb(0);
#pragma unroll
    for (int k = 0; k < WN; ++k) {
      if (k + 1 < WN) ldb(k + 1);
#pragma unroll
      for (int i = 0; i < WI; ++i) {
        acc[i][k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[k & 1], acc[i][k], 0, 0, 0);
        acc[i][k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[k & 1], acc[i][k], 0, 0, 0);
        acc[i][k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[k & 1], acc[i][k], 0, 0, 0);
      }
    }
  };
  // pinned interleave of staging work into a k-step's 96 MFMAs: the A reads and the
  // first B pair, then per MFMA up to NV VALU (+ one VMEM load every 3rd MFMA: LD; a DS
  // write every 8th: ST), the next B pair after each column tile's first MFMA
  auto pin = [&](auto nv_tag, auto ld_tag, auto st_tag) {
    constexpr int NV = decltype(nv_tag)::value;
    constexpr bool LD = decltype(ld_tag)::value, ST = decltype(st_tag)::value;
    __builtin_amdgcn_sched_group_barrier(0x100, 2 * WI + 2, 0);
#pragma unroll
    for (int s = 0; s < 3 * WI * WN; ++s) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      if (NV) __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);
      if (LD && s % 3 == 0) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      if (ST && s % 8 == 7) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
      if (s % (3 * WI) == 0 && s / (3 * WI) + 1 < WN)
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  using I0 = std::integral_constant<int, 0>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  using T_ = std::true_type;
  using F_ = std::false_type;

  // ---- prologue: window of group 0, slab of step 0 ----
  load_x(0);
  issue_w(0, 0);
  store_x(0);
  wait_vm<0>();
  lds_barrier();

  for (int u = 0; u < NU; ++u) {
    const int s0 = u * KT;
    const int g1 = min(2 * u + 1, NG - 1), g2 = min(2 * u + 2, NG - 1);
#pragma unroll
    for (int sp = 0; sp < KT; ++sp) {
      const int s = s0 + sp;
      const int slot = s & 1;
      const int f0 = 2 * sp, f1 = 2 * sp + 1;
      const int gg0 = f0 / KT, j0 = f0 - gg0 * KT, gg1 = f1 / KT, j1 = f1 - gg1 * KT;
      const bool ld_1 = sp == SCH.ld1, st_1 = sp == SCH.st1;
      const bool ld_2 = sp == SCH.ld2, st_2 = sp == SCH.st2;
      const bool ldx = ld_1 || ld_2, stx = st_1 || st_2;
      const int gl = ld_1 ? g1 : g2;       // group whose loads this step issues
      const int bs = st_1 ? 1 : 0;         // buffer this step stores into
      auto next_w = [&]() { issue_w(min(s + 1, P - 1), slot ^ 1); };
      if (stx && !ldx) {
        // conversion + store interleaved; the slab DMA after it, so the input
        // registers' wait does not also wait for the new slab
        store_x(bs);
        kstep(slot, gg0, j0, gg1, j1);
        pin(I2{}, F_{}, T_{});
        next_w();
      } else if (ldx && !stx) {
        next_w();
        __builtin_amdgcn_sched_barrier(0);  // the slab DMA stays older than the input loads
        load_x(gl);
        kstep(slot, gg0, j0, gg1, j1);
        pin(I0{}, T_{}, F_{});
      } else {
        next_w();
        if (ldx) load_x(gl);
        kstep(slot, gg0, j0, gg1, j1);
        if (stx) store_x(bs);
      }
      (void)I3{};
      // the slab of step s+1 must have landed; younger: input loads not yet stored
      const bool pending = (sp >= SCH.ld1 && sp < SCH.st1) || (sp >= SCH.ld2 && sp < SCH.st2);
      if (pending && x_short) wait_vm<(NX >= 8 ? NX - 8 : 0)>();
      else if (pending) wait_vm<NX>();
      else wait_vm<0>();
      lds_barrier();
    }
  }
  if (p.dbg & 8) {  // ablation: no epilogue
    if (acc[0][0][0] == 1.2345e-30f) p.y[0] = acc[WI - 1][WN - 1][3];
    return;
  }

  // ---- epilogue: lane holds column n of tile k and rows 4*quarter + r of tile i ----
  const int row_base = mt * MT + wave_m * 64 + 4 * quarter;
  const int n_base = n0 + wave_n * 128 + col;
  if constexpr (UPS) {
    // polyphase scatter (GEMM row m = co*s + r -> t = n*s + r - p): the 4 consecutive
    // rows of a lane are 4 consecutive phases when s % 4 == 0: one float4 store
    const int s_ = p.ups_s, p_ = p.ups_p;
    const bool vec4 = (s_ & 3) == 0 && (p_ & 3) == 0 && (p.L_out & 3) == 0;
    const bool pow2 = (s_ & (s_ - 1)) == 0;
    const int sh = __builtin_ctz((unsigned)s_);
    auto co_of = [&](int row) { return pow2 ? row >> sh : row / s_; };
    float* __restrict__ yb = p.y + (int64_t)b * p.y_bs;
#pragma unroll
    for (int i = 0; i < WI; ++i) {
      const int rb = row_base + 16 * i;
      floatx4 bv;
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[r] = p.bias[rb + r];
#pragma unroll
      for (int k = 0; k < WN; ++k) {
        const int n = n_base + 16 * k;
        if (n >= N_b) continue;
        const floatx4 v = acc[i][k] + bv;
        if (vec4) {
          if (rb >= p.M) continue;
          const int co = co_of(rb);
          const int t = n * s_ + (rb - co * s_) - p_;
          float* dst = yb + (int64_t)co * p.L_out + t;
          if (t >= 0 && t + 3 < L_out_b) {
            *reinterpret_cast<floatx4*>(dst) = v;
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (t + r >= 0 && t + r < L_out_b) dst[r] = v[r];
          }
          continue;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rb + r;
          if (row >= p.M) continue;
          const int co = co_of(row);
          const int t = n * s_ + (row - co * s_) - p_;
          if (t >= 0 && t < L_out_b) yb[(int64_t)co * p.L_out + t] = v[r];
        }
      }
    }
  } else {
    // bias, residual (x + conv2(..), models/hifigan.py:85), post-lrelu (:83), MRF running
    // sum / mean (:125-131); loads of 4 column tiles issued as one batch before any store
    const int64_t bo = (int64_t)b * p.y_bs;
    const char* resb = p.res ? reinterpret_cast<const char*>(p.res + bo) : nullptr;
    char* outb = reinterpret_cast<char*>((p.mrf ? p.mrf : p.y) + bo);
    const bool add_mrf = p.mrf && (p.mrf_mode & 1);
    const bool div_mrf = p.mrf && (p.mrf_mode & 2);
    const bool act = p.act_out != 0;
#pragma unroll
    for (int i = 0; i < WI; ++i) {
      const int rb = row_base + 16 * i;
      float bv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[r] = p.bias[rb + r];  // padded to the m-tile
#pragma unroll
      for (int k0 = 0; k0 < WN; k0 += 4) {
        unsigned off[4][4];
        bool ok[4][4];
        float v[4][4];
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const int n = n_base + 16 * (k0 + kk);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            ok[kk][r] = n < N_b && rb + r < p.M;
            off[kk][r] = ok[kk][r] ? (unsigned)((rb + r) * p.N + n) * 4u : 0u;
            v[kk][r] = acc[i][k0 + kk][r] + bv[r];
          }
        }
        if (resb) {
          float rv[4][4];
#pragma unroll
          for (int kk = 0; kk < 4; ++kk)
#pragma unroll
            for (int r = 0; r < 4; ++r) rv[kk][r] = *reinterpret_cast<const float*>(resb + off[kk][r]);
#pragma unroll
          for (int kk = 0; kk < 4; ++kk)
#pragma unroll
            for (int r = 0; r < 4; ++r) v[kk][r] = rv[kk][r] + v[kk][r];
        }
        if (act) {
#pragma unroll
          for (int kk = 0; kk < 4; ++kk)
#pragma unroll
            for (int r = 0; r < 4; ++r) v[kk][r] = v[kk][r] > 0.f ? v[kk][r] : v[kk][r] * kLReluSlope;
        }
        if (add_mrf) {
          float mv[4][4];
#pragma unroll
          for (int kk = 0; kk < 4; ++kk)
#pragma unroll
            for (int r = 0; r < 4; ++r) mv[kk][r] = *reinterpret_cast<const float*>(outb + off[kk][r]);
#pragma unroll
          for (int kk = 0; kk < 4; ++kk)
#pragma unroll
            for (int r = 0; r < 4; ++r) v[kk][r] = mv[kk][r] + v[kk][r];
        }
        if (div_mrf) {
#pragma unroll
          for (int kk = 0; kk < 4; ++kk)
#pragma unroll
            for (int r = 0; r < 4; ++r) v[kk][r] = v[kk][r] / p.mrf_div;
        }
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (ok[kk][r]) *reinterpret_cast<float*>(outb + off[kk][r]) = v[kk][r];
      }
    }
  }
}

namespace {

typedef void (*C16Fn)(const ConvParams);

struct EntryC16 {
  int kt;
  bool ups;
  C16Fn fn;
  bool attr;
  char name[64];
};

#define HFGC16_ENTRY(KT, UPS) \
  { KT, UPS, conv16_bf16x3<KT, UPS>, false, {0} }

EntryC16 g_entriesC16[] = {HFGC16_ENTRY(3, false), HFGC16_ENTRY(5, false), HFGC16_ENTRY(7, false),
                           HFGC16_ENTRY(11, false), HFGC16_ENTRY(2, true)};

}  // namespace

bool c16_supported(int kt, bool ups, int M, int C_in, int dil) {
  if (M < kC16MT || dil < 1 || (kt - 1) * dil > kC16MaxHalo) return false;
  if (((C_in + 15) / 16) % 2 != 0) return false;  // whole units of two channel groups
  for (auto& e : g_entriesC16)
    if (e.kt == kt && e.ups == ups) return true;
  return false;
}

size_t c16_lds_bytes(int kt, int dil) {
  const size_t xw = kC16NT + (size_t)(kt - 1) * dil;
  return sizeof(__bf16) * (2 * (size_t)2 * kC16MT * 32 + 2 * 2 * xw * 16);
}

hipError_t launch_conv16_bf16x3(int kt, bool ups, const ConvParams& p, int n_tiles, int m_tiles,
                                int batch, hipStream_t stream, const char** name) {
  EntryC16* e = nullptr;
  for (auto& cand : g_entriesC16)
    if (cand.kt == kt && cand.ups == ups) e = &cand;
  if (!e || !c16_supported(kt, ups, p.M, p.C_in, p.dil)) return hipErrorInvalidValue;
  const int ng = (p.C_in + 15) / 16;
  if (p.n_chunks * 2 != ng * kt) return hipErrorInvalidValue;
  if (!e->name[0])
    snprintf(e->name, sizeof(e->name), "conv16_bf16x3<%d, %s>", e->kt, e->ups ? "true" : "false");
  const size_t lds = c16_lds_bytes(kt, p.dil);
  if (lds > 80 * 1024) return hipErrorInvalidValue;
  if (!e->attr) {
    hipError_t err = hipFuncSetAttribute(reinterpret_cast<const void*>(e->fn),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (err != hipSuccess) return err;
    e->attr = true;
  }
  if (name) *name = e->name;
  e->fn<<<dim3(n_tiles, m_tiles, batch), dim3(256), lds, stream>>>(p);
  return hipGetLastError();
}

}  // namespace hfg

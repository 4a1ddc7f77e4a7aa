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

#include <mutex>

#include <algorithm>

#include <cstdio>
#include <type_traits>

#include "bf16x3_common.h"
#include "epilogue.h"
#include "kernels.h"

#ifndef HFG_AREG_AD
#define HFG_AREG_AD 2
#endif
// tile-5 tap schedule: the next group's input loads issue at tap KT - HFG_AREG_XT; VALU
// fillers per MFMA on the plain taps (HFG_AREG_NV) and on the last (store) tap
// (HFG_AREG_NVST)
#ifndef HFG_AREG_XT
#define HFG_AREG_XT 4
#endif
#ifndef HFG_AREG_NV
#define HFG_AREG_NV 2
#endif
#ifndef HFG_AREG_NVST
#define HFG_AREG_NVST 6
#endif

// diagnostic build only (-DHFG_CONV_TIMING=1, profiles/r04): wave 0 of every tile-5 block
// stamps the shader clock (start, prologue end, loop end, epilogue end) and sums its
// barrier waits into g_cv_ts (one region per KT), read back by hfg_debug_cv_ts
#ifndef HFG_CONV_TIMING
#define HFG_CONV_TIMING 0
#endif

namespace hfg {

#if HFG_CONV_TIMING
constexpr int kCvTsSlots = 16, kCvTsBlocks = 8192, kCvTsRegions = 12;
__device__ uint64_t g_cv_ts[kCvTsRegions * kCvTsBlocks * kCvTsSlots];
#endif

namespace {
typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
}  // namespace

template <int KT_, int TPC, int WAVES_M, int WAVES_N, int WM, int WN, int WD, bool UPS, int NP,
          bool AREG, int FMT>
__global__ void __launch_bounds__(64 * WAVES_M * WAVES_N, 2)
conv1d_bf16x3(const ConvParams p) {
  static_assert(!AREG || (KT_ > 0 && !UPS && WM * WN >= 8), "AREG: compile-time taps, layer convs");
  constexpr int NW = WAVES_M * WAVES_N;
  constexpr int NT = 64 * NW;
  constexpr int MT = 32 * WM * WAVES_M;
  constexpr int NTILE = 32 * WN * WAVES_N;
  constexpr int XROW = 16;  // bf16 per staged row: 16 channels (32 B), 16-B halves XOR-swizzled
  constexpr int TAP_ELEMS = 2 * WAVES_M * WM * 64 * 8;  // bf16 per tap of a slab (hi+lo)
  constexpr int SLAB = TPC * TAP_ELEMS;           // bf16 per chunk slab
  constexpr int KT_MAX = KT_ > 0 ? KT_ : 16;
  constexpr int XW_MAX = NTILE + ((KT_MAX - 1) * kMaxDil < kBf16x3MaxHalo
                                       ? (KT_MAX - 1) * kMaxDil : kBf16x3MaxHalo);
  constexpr int XQ = (2 * XW_MAX + NT - 1) / NT;  // staging tasks per thread
  static_assert(XQ * 8 <= 32, "ok mask");
  constexpr int NX = XQ * 8;                      // input loads per thread per channel group
  constexpr int PW = SLAB / 8 / 64 / NW;          // LDS-DMA pieces per thread per slab
  static_assert(PW * 8 * 64 * NW == SLAB, "slab must split evenly over the waves");
  static_assert(NX + PW < 64, "vmcnt range");
  const int KT = KT_ > 0 ? KT_ : p.kt;
  const int n_tg = (KT + TPC - 1) / TPC;          // tap groups per channel group
  // one staged input window per 16-channel group serves all KT taps
  const int XW = NTILE + (KT - 1) * p.dil;
  // AREG: the planes hold a row for every staging task (XQ*NT/2 >= XW_MAX rows), so
  // store_x writes all its tasks unconditionally (rows >= XW are never read) and stays
  // straight-line code the tap schedule interleaves into the MFMA stream
  constexpr int XROWS_AREG = XQ * NT / 2;
  static_assert(XROWS_AREG >= XW_MAX, "AREG planes");
  // AREG half planes (8 channels, 16-B rows) padded by 64 B: a ds_write_b128 lane group
  // (8 lanes: 4 rows of each half) then covers the 32 write banks once
  constexpr int HPS_AREG = XROWS_AREG * 8 + 32;
  const int xplane = AREG ? 2 * HPS_AREG : (XW * XROW + 7) & ~7;  // bf16 per X plane
  const int xbuf = 2 * xplane;                    // hi + lo planes

  extern __shared__ __attribute__((aligned(16))) __bf16 lds16[];
  __bf16* const Wbuf0 = lds16;
  __bf16* const Xbuf0 = lds16 + (AREG ? 0 : WD * SLAB);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wave_m = wave % WAVES_M;
  const int wave_n = wave / WAVES_M;
  // block -> (column tile, m-tile, item).  Upsamplers: the m-tiles of one input window
  // (16 for ups.0) read the same x rows, so they are swizzled onto one XCD's L2 (blocks b
  // and b + 8 share an XCD under the round-robin placement; speed only, any placement is
  // correct): linear id -> (id % 8) * (total / 8) + id / 8, then m-tile fastest.
  int tx = blockIdx.x, mt = blockIdx.y, b = blockIdx.z;
  if (UPS && p.ups_swz) {
    const int nx = gridDim.x, ny = gridDim.y;
    const int total = nx * ny * gridDim.z;
    int id = blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z);
    const int q = total >> 3;
    if (id < (q << 3)) id = (id & 7) * q + (id >> 3);
    mt = id % ny;
    id /= ny;
    tx = id % nx;
    b = id / nx;
    // the divisions expand to VALU code: without this the compiler treats the results as
    // per-lane values, and every buffer load whose descriptor derives from b (the input
    // staging) became a readfirstlane waterfall loop
    mt = __builtin_amdgcn_readfirstlane(mt);
    tx = __builtin_amdgcn_readfirstlane(tx);
    b = __builtin_amdgcn_readfirstlane(b);
  }
  const int n0 = p.n_base + tx * NTILE;
  const int half = lane >> 5;
  const int col = lane & 31;
  const float* __restrict__ xb = p.x + (int64_t)b * p.x_bs;
  const __bf16* __restrict__ wsrc =
      reinterpret_cast<const __bf16*>(p.w) + (int64_t)mt * p.n_chunks * SLAB;
  const int L_in_b = p.len_in ? p.len_in[b] : p.L_in;
  int N_b = p.N;
  if (p.len_out) {
    const int lo = p.len_out[b];
    N_b = UPS ? (lo > 0 ? (lo - 1 + p.ups_p) / p.ups_s + 1 : 0) : lo;
  }
  if (n0 >= N_b) return;  // whole tile past this utterance's end (block-uniform)
  const int L_out_b = (UPS && p.len_out) ? p.len_out[b] : p.L_out;
  const int xcs = (int)p.x_cs, xts = (int)p.x_ts;
  // f16x3 (bf16x3_common.h): the input's power-of-two scale from its producer's per-item max
  // (folded into the staging factors below) and the accumulator's unscale after the loop
  const int ex = FMT == kFmtF16 ? x3_exp_slot(p.amax_in, b) : 0;
  const float sx = FMT == kFmtF16 ? exp2i(ex) : 1.0f;
  const int wbase = n0 + p.off;                   // input index of window row 0

  auto taps_in = [&](int c) {
    const int tg = c % n_tg;
    const int rem = KT - tg * TPC;
    return rem < TPC ? rem : TPC;
  };
  // ---- weight slab: global -> LDS by LDS-DMA, PW pieces per thread (whole slab:
  // the packer zero-fills the taps past KT, so every thread issues the same count) ----
  auto issue_w = [&](int c, __bf16* Ws) {
    const __bf16* src = wsrc + (int64_t)c * SLAB;
#pragma unroll
    for (int q = 0; q < PW; ++q) {
      const int i = wave + q * NW;
      __builtin_amdgcn_global_load_lds((gptr_t1)(src + (i * 64 + lane) * 8),
                                       (lds_ptr_t3)(Ws + i * 512), 16, 0, 0);
    }
  };
  // raw loads (clamped offsets) into registers; the zero padding is applied at store
  // time from a bit mask, so the loads' latency hides behind the chunk's MFMAs
  float xv[XQ][8];
  uint32_t xok = 0;
  // AREG (whole groups: one in-window flag per task row): the zero padding and the
  // pre-activation as max(v*s1, v*s2) with per-row factors (s1, s2) = (1, slope) inside
  // the window (slope 1 without act_in: v) and (0, 0) outside (+-0): bitwise lrelu3(v) or
  // v or 0, in 3 VALU ops and no canonicalising max on the loaded value
  float xs1[XQ], xs2[XQ];
  const float slope = p.act_in ? kLReluSlope : 1.0f;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  // a wave with no task in the (mostly idle) last staging row skips that row's loads, so
  // it has 8 fewer input loads in flight than NX: every vmcnt wait that lets the input
  // loads stay outstanding counts them per wave (wait_x), or it would pass before the
  // older weight-slab DMA has landed
  // (AREG: no skip, and whole channel groups only (host-checked): the staging is
  // straight-line code the tap schedule can interleave; the compiler counts its vmcnt)
  const bool x_short = !AREG && XQ > 1 && (XQ - 1) * NT + wave_u * 64 >= 2 * XW;
  auto wait_x = [&](auto n_tag) {
    constexpr int N = decltype(n_tag)::value;
    static_assert(XQ == 1 || N >= 8, "vmcnt");
    if (x_short) wait_vm<(N >= 8 ? N - 8 : 0)>();
    else wait_vm<N>();
  };
  // whole 32-bit range: an item holds fewer than 2^30 floats (the C ABI refuses 2^30:
  // the hardware drops a dword whose end passes num_records 0xFFFFFFFF, which would be
  // a 4-GiB item's last float), and every offset the staging forms stays below that
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)xb, 0, -1, 0x00020000);
  // whole 16-channel groups (every group of the V1 / V2* layers): the window mask and the
  // pre-activation as max(v*s1, v*s2) like the AREG path (3 VALU per value instead of a
  // per-element mask select + leaky_relu); partial groups keep the per-element mask
  bool xfull = true;
  auto load_x = [&](int g) {
    const bool full = AREG || g * 16 + 16 <= p.C_in;  // block-uniform
    xfull = full;
    xok = 0;
#pragma unroll
    for (int q = 0; q < XQ; ++q) {
      // the last task row is mostly idle: a wave with no task in the window skips its loads
      if (q == XQ - 1 && q > 0 && x_short) continue;
      const int i = tid + q * NT;
      const int t = i >> 1;
      // (ablation bit7: always re-read channel group 0, i.e. L2-warm loads)
      const int cb = ((kAblate && (p.dbg & 128)) ? 0 : g) * 16 + (i & 1) * 8;
      const int gi = wbase + t;
      const bool tok = (i < 2 * XW) && ((unsigned)gi < (unsigned)L_in_b);
      // byte offsets from the block-uniform base: SGPR base + 32-bit VGPR offset loads
      const unsigned o0 = tok ? (unsigned)(cb * xcs + gi * xts) * 4u : 0u;
      const unsigned step = tok ? (unsigned)xcs * 4u : 0u;
      // channels past C_in (a partial last group) re-read the last valid channel
      const int ecap = full ? 7 : min(p.C_in - 1 - cb, 7);
      const uint32_t m8 = tok ? (ecap >= 7 ? 0xffu : (ecap < 0 ? 0u : (1u << (ecap + 1)) - 1u)) : 0u;
      xok |= m8 << (q * 8);
      xs1[q] = tok ? sx : 0.0f;
      xs2[q] = tok ? slope * sx : 0.0f;
      if (full) {
        // whole group: buffer loads with the channel step in the scalar offset (one offset
        // VGPR per row instead of eight); a lane outside the window reads channel e at
        // t = 0 of its item (valid memory, masked by xok)
#pragma unroll
        for (int e = 0; e < 8; ++e)
          xv[q][e] = __builtin_bit_cast(
              float, __builtin_amdgcn_raw_buffer_load_b32(xrs, (int)o0, e * xcs * 4, 0));
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const unsigned oe = o0 + (unsigned)max(min(e, ecap), 0) * step;
          xv[q][e] = *reinterpret_cast<const float*>(reinterpret_cast<const char*>(xb) + oe);
        }
      }
    }
  };
  auto store_x = [&](__bf16* Xh) {
    __bf16* Xl = Xh + xplane;
#pragma unroll
    for (int q = 0; q < XQ; ++q) {
      const int i = tid + q * NT;
      if (AREG || i < 2 * XW) {
        bf16x8 h, l;
        if (kAblate && UPS && (p.dbg & 256)) {
          // ablation (upsamplers, timing only): the raw fp32 halves, no pre-activation or split
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const unsigned u = __float_as_uint(xv[q][e]);
            h[e] = __builtin_bit_cast(__bf16, (unsigned short)(u >> 16));
            l[e] = __builtin_bit_cast(__bf16, (unsigned short)(u & 0xffffu));
          }
        } else
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          floatx2 a;
          if (AREG || xfull) {
            a[0] = fmaxf(xv[q][e] * xs1[q], xv[q][e] * xs2[q]);
            a[1] = fmaxf(xv[q][e + 1] * xs1[q], xv[q][e + 1] * xs2[q]);
          } else {
            a[0] = (xok >> (q * 8 + e)) & 1u ? xv[q][e] : 0.f;
            a[1] = (xok >> (q * 8 + e + 1)) & 1u ? xv[q][e + 1] : 0.f;
            if (p.act_in) {
              a[0] = lrelu3(a[0]);
              a[1] = lrelu3(a[1]);
            }
            if constexpr (FMT == kFmtF16) a = a * sx;
          }
          bf16x2 hh, ll;
          split2<FMT>(a, hh, ll);
          h[e] = hh[0];
          h[e + 1] = hh[1];
          l[e] = ll[0];
          l[e + 1] = ll[1];
        }
        const int t = i >> 1;
        // AREG: the two 8-channel halves in planes of their own (16-B rows: a half-wave's
        // 32 consecutive rows are one conflict-free 512-B run for any tap shift, so a tap
        // is one address add and the reads take immediate offsets); else one 32-B row per
        // t with the 16-B halves XOR-swizzled
        const int off = AREG ? (i & 1) * HPS_AREG + t * 8
                             : t * XROW + 8 * ((i & 1) ^ ((t >> 3) & 1));
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
  // jj: tap inside the chunk's slab; tap: tap index inside the window
  auto load_frag = [&](const __bf16* Ws, const __bf16* Xh, int jj, int tap, Frag& f) {
    const __bf16* Xl = Xh + xplane;
#pragma unroll
    for (int i = 0; i < WM; ++i) {
      const __bf16* a = Ws + jj * TAP_ELEMS + (wave_m * WM + i) * 512 + lane * 8;
      f.ah[i] = *reinterpret_cast<const bf16x8*>(a);
      f.al[i] = *reinterpret_cast<const bf16x8*>(a + WAVES_M * WM * 512);
    }
#pragma unroll
    for (int k = 0; k < WN; ++k) {
      const int t = wave_n * 32 * WN + k * 32 + col + tap * p.dil;
      // rows t..t+31 of one half-wave: (t mod 16) distinct -> conflict-free ds_read_b128
      const int off = t * XROW + 8 * (half ^ ((t >> 3) & 1));
      f.bh[k] = *reinterpret_cast<const bf16x8*>(Xh + off);
      f.bl[k] = *reinterpret_cast<const bf16x8*>(Xl + off);
    }
  };
  auto mma = [&](const Frag& f) {
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int k = 0; k < WN; ++k) {
        if constexpr (NP == 3)  // the weights' lo plane (zero for bf16-valued weights: NP 2)
          acc[i][k] = mfma32<FMT>(f.al[i], f.bh[k], acc[i][k]);
        acc[i][k] = mfma32<FMT>(f.ah[i], f.bl[k], acc[i][k]);
        acc[i][k] = mfma32<FMT>(f.ah[i], f.bh[k], acc[i][k]);
      }
  };

  // One tap of the 64x128-per-wave tile with the B fragments streamed per column tile
  // (two in flight): only the A fragments stay live across the tap, which leaves room
  // for the input staging interleaved into the same MFMA stream.
  auto tap_stream = [&](const __bf16* Ws, const __bf16* Xh, int jj, int tap) {
    const __bf16* Xl = Xh + xplane;
    bf16x8 ah[WM], al[WM], bh[2], bl[2];
#pragma unroll
    for (int i = 0; i < WM; ++i) {
      const __bf16* a = Ws + jj * TAP_ELEMS + (wave_m * WM + i) * 512 + lane * 8;
      ah[i] = *reinterpret_cast<const bf16x8*>(a);
      al[i] = *reinterpret_cast<const bf16x8*>(a + WAVES_M * WM * 512);
    }
    auto ldb = [&](int k) {
      const int t = wave_n * 32 * WN + k * 32 + col + tap * p.dil;
      const int off = t * XROW + 8 * (half ^ ((t >> 3) & 1));
      bh[k & 1] = *reinterpret_cast<const bf16x8*>(Xh + off);
      bl[k & 1] = *reinterpret_cast<const bf16x8*>(Xl + off);
    };
    ldb(0);
#pragma unroll
    for (int k = 0; k < WN; ++k) {
      if (k + 1 < WN) ldb(k + 1);
#pragma unroll
      for (int i = 0; i < WM; ++i) {
        if constexpr (NP == 3)
          acc[i][k] = mfma32<FMT>(al[i], bh[k & 1], acc[i][k]);
        acc[i][k] = mfma32<FMT>(ah[i], bl[k & 1], acc[i][k]);
        acc[i][k] = mfma32<FMT>(ah[i], bh[k & 1], acc[i][k]);
      }
    }
  };
  // sched_group_barrier pattern for tap_stream + staging work in one basic block: the A
  // reads and the first B pair, then per MFMA up to NV VALU (+ one VMEM load when LD),
  // the next B pair after each column tile's first MFMA, a DS write every 4th MFMA (ST)
  auto pin_stream = [&](auto nv_tag, auto ld_tag, auto st_tag) {
    constexpr int NV = decltype(nv_tag)::value;
    constexpr bool LD = decltype(ld_tag)::value, ST = decltype(st_tag)::value;
    __builtin_amdgcn_sched_group_barrier(0x100, 2 * WM + 2, 0);
#pragma unroll
    for (int s = 0; s < NP * WM * WN; ++s) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);
      if (LD) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      if (ST && s % 4 == 3) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
      if (s % (NP * WM) == 0 && s / (NP * WM) + 1 < WN)
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  };

#if HFG_CONV_TIMING
  uint64_t* const cts = g_cv_ts + ((size_t)((KT_ == 3 ? 0 : KT_ == 7 ? 1 : KT_ == 11 ? 2 : 3) * 3 +
                                           (p.res ? ((p.mrf && (p.mrf_mode & 1)) ? 2 : 1) : 0)) * kCvTsBlocks +
                                   ((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) % kCvTsBlocks) *
                                      kCvTsSlots;
  // stamps kept in SGPRs and stored once at the end: a stamp store mid-kernel would make
  // every later vmcnt wait also wait for its write (one in-order queue for loads and stores)
  uint64_t tsv[16] = {};
  auto cstamp = [&](int i) { tsv[i] = __builtin_amdgcn_s_memtime(); };
  uint64_t bar_wait = 0;
  tsv[0] = __builtin_amdgcn_s_memrealtime();
  // placement: HW_ID (CU, SE, SIMD, wave) and XCC of wave 0
  tsv[12] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
            ((uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32);
  cstamp(1);
#else
  auto cstamp = [](int) {};
#endif
  // AREG: the m-tile's bias in LDS for the epilogue (conv_epilogue_lds2), visible after the
  // prologue barrier
  // the AREG tiles (5, 6): the host sizes the LDS from the same configuration
  constexpr Bf16x3Cfg TCFG{WAVES_M, WAVES_N, WM, WN, TPC, WD, AREG ? 1 : 0};
  constexpr int BIAS_OFF = AREG ? bf16x3_areg_bias_off(KT_MAX, TCFG) : 0;
  float* const bias_lds = reinterpret_cast<float*>(reinterpret_cast<char*>(lds16) + BIAS_OFF);
  if constexpr (AREG)
    for (int i = tid; i < MT; i += NT) bias_lds[i] = p.bias[mt * MT + i];
  // ---- prologue: weight slabs of chunks 0..WD-2, input window of channel group 0 ----
  load_x(0);
  if constexpr (!AREG) {
#pragma unroll
    for (int c = 0; c < WD - 1; ++c)
      if (c < p.n_chunks) issue_w(c, Wbuf0 + c * SLAB);
  }
  store_x(Xbuf0);
  wait_vm<0>();
  lds_barrier();
  cstamp(2);

  if constexpr (AREG) {
    // ---- A fragments from global into registers, AD taps ahead; one barrier per
    // channel group.  Every wave reads its own (wave_m) rows of the packed slab stream
    // (L2-resident; tile 3's packing) -- the two wave_n waves read the same rows -- so
    // the weights need no LDS and no cross-wave handoff.  The input window is
    // double-buffered per channel group as in the LDS-slab path: group g+1's loads issue
    // at tap XT, land in the idle buffer at the group's last tap, and the barrier ending
    // group g makes them visible (and frees the buffer group g read).  Per output element
    // the MFMA sequence is the LDS-slab path's (channel groups x taps in order; lo*hi,
    // hi*lo, hi*hi), so the result is bitwise the same.
    constexpr int KT = KT_;
    constexpr int NTG = (KT + TPC - 1) / TPC;
    constexpr int AD = HFG_AREG_AD;           // A prefetch distance in taps (1 or 2)
    constexpr int XT = KT >= HFG_AREG_XT ? KT - HFG_AREG_XT : 0;  // tap issuing the next
                                                                  // group's input loads
    static_assert(AD <= KT && XT < KT - 1, "AREG schedule");
    using I0 = std::integral_constant<int, 0>;
    using I2 = std::integral_constant<int, HFG_AREG_NV>;
    using I6 = std::integral_constant<int, HFG_AREG_NVST>;
    using T_ = std::true_type;
    using F_ = std::false_type;
    const int NG = p.n_chunks / NTG;
    const int wm_u = wave_u % WAVES_M;
    // buffer loads: SGPR descriptor over this m-tile's stream + scalar tap offset + the
    // lane's 16 B (no 64-bit address VGPRs per tap)
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)wsrc, 0, (int)((int64_t)p.n_chunks * SLAB * 2), 0x00020000);
    const int a_lane = lane * 16;
    typedef bf16x8 ASet[2][WM];
    ASet a0, a1, a2;
    (void)a2;
    auto load_a = [&](ASet& d, int g, int t) {
      const int so = ((g * NTG + t / TPC) * SLAB + (t % TPC) * TAP_ELEMS + wm_u * WM * 512) * 2;
#pragma unroll
      for (int pl = 0; pl < 2; ++pl)
#pragma unroll
        for (int i = 0; i < WM; ++i)
          d[pl][i] = __builtin_bit_cast(
              bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                          wrs, a_lane + (pl * WAVES_M * WM + i) * 1024, so, 0));
    };
    // B fragments: a two-deep ring over the column tiles that carries across the taps of
    // a channel group (the last tile of tap t reads tap t+1's first pair), so a tap's first
    // MFMAs do not wait on an LDS round trip; only the first tap after the group barrier
    // reads its first pair on the spot
    bf16x8 bh[2], bl[2];
    auto ldb = [&](const __bf16* Xh, int tap, int k) {
      const int off = half * HPS_AREG + (wave_n * 32 * WN + col) * 8 + (k % WN) * 32 * 8 +
                      (tap + k / WN) * p.dil * 8;
      bh[k & 1] = *reinterpret_cast<const bf16x8*>(Xh + off);
      // ablation bit 12: no lo-plane reads (the hi fragment stands in; half the LDS reads)
      bl[k & 1] = (kAblate && (p.dbg & 4096)) ? bh[k & 1]
                                              : *reinterpret_cast<const bf16x8*>(Xh + xplane + off);
    };
    static_assert(WN % 2 == 0, "B ring parity across taps");
    auto tap_regs = [&](const ASet& a, const __bf16* Xh, int tap, bool pre_in, bool pre_out) {
      if (!pre_in) ldb(Xh, tap, 0);
#pragma unroll
      for (int k = 0; k < WN; ++k) {
        if (k + 1 < WN || pre_out) ldb(Xh, tap, k + 1);  // k + 1 == WN: tap + 1, tile 0
#pragma unroll
        for (int i = 0; i < WM; ++i) {
          if constexpr (NP == 3)
            acc[i][k] = mfma32<FMT>(a[1][i], bh[k & 1], acc[i][k]);
          acc[i][k] = mfma32<FMT>(a[0][i], bl[k & 1], acc[i][k]);
          acc[i][k] = mfma32<FMT>(a[0][i], bh[k & 1], acc[i][k]);
        }
      }
    };
    // one tap's interleave: B(0) first (unless the previous tap read it), then per MFMA up to
    // NV VALU and (LD) one global load, the next B pair after each column tile's first MFMA
    // (after the last tile's: the next tap's first pair when pre_out), a DS write every 4th
    // MFMA (ST)
    auto pin_regs = [&](auto nv_tag, auto ld_tag, auto st_tag, bool pre_in, bool pre_out) {
      constexpr int NV = decltype(nv_tag)::value;
      constexpr bool LD = decltype(ld_tag)::value, ST = decltype(st_tag)::value;
      if (!pre_in) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
      for (int s = 0; s < NP * WM * WN; ++s) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);
        if (LD) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        if (ST && s % 4 == 3) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
        if (s % (NP * WM) == 0 && (s / (NP * WM) + 1 < WN || pre_out))
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    };
    load_a(a0, 0, 0);
    if constexpr (AD == 2) load_a(a1, 0, 1);
    prio_mfma();
    for (int g = 0; g < NG; ++g) {
      const __bf16* Xh = Xbuf0 + (g & 1) * xbuf;
      __bf16* const Xn = Xbuf0 + ((g + 1) & 1) * xbuf;
      const int gn = min(g + 1, NG - 1);
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        // A of tap t + AD: the next group's first taps near the end (past the last group
        // a harmless re-read of its own)
        ASet& an = AD == 2 ? a2 : a1;
        if (t + AD < KT) load_a(an, g, t + AD);
        else load_a(an, gn, t + AD - KT);
        const bool pre_in = t > 0, pre_out = t + 1 < KT;
        if (t == XT) {
          load_x(gn);
          tap_regs(a0, Xh, t, pre_in, pre_out);
          pin_regs(I0{}, T_{}, F_{}, pre_in, pre_out);
        } else if (t == KT - 1) {
          store_x(Xn);
          tap_regs(a0, Xh, t, pre_in, pre_out);
          pin_regs(I6{}, T_{}, T_{}, pre_in, pre_out);
        } else {
          tap_regs(a0, Xh, t, pre_in, pre_out);
          pin_regs(I2{}, T_{}, F_{}, pre_in, pre_out);
        }
#pragma unroll
        for (int pl = 0; pl < 2; ++pl)
#pragma unroll
          for (int i = 0; i < WM; ++i) {
            a0[pl][i] = a1[pl][i];
            if constexpr (AD == 2) a1[pl][i] = a2[pl][i];
          }
      }
#if HFG_CONV_TIMING
      const uint64_t tb0 = __builtin_amdgcn_s_memtime();
#endif
      if (!(kAblate && (p.dbg & 4))) lds_barrier();
#if HFG_CONV_TIMING
      bar_wait += __builtin_amdgcn_s_memtime() - tb0;
#endif
    }
#if HFG_CONV_TIMING
    tsv[5] = bar_wait;
#endif
    prio_other();
    cstamp(3);
  } else if constexpr (KT_ > 0 && WM * WN >= 8) {
    // ---- 64x128-per-wave tile, compile-time taps: the chunk loop unrolled over one
    // channel group, so the chunks that stage the next input window are their own
    // straight-line code.  That staging (the loads, or the conversion and LDS store)
    // shares a basic block with the first tap's MFMAs and is interleaved into them: its
    // VALU / memory issue hides under the matrix pipe instead of running as a serial
    // phase in which both waves of a SIMD leave the pipe idle.  The last group re-stages
    // itself into the idle buffer (no branch; one group of extra loads per block).
    // Ablation bit0 (no restaging) is not available on this path.
    static_assert(WD == 2, "fast path: two-slab weight ring");
    constexpr int NTG = (KT_ + TPC - 1) / TPC;
    constexpr int XG = NTG >= 2 ? NTG - 2 : 0;
    using I6 = std::integral_constant<int, 6>;
    using I3 = std::integral_constant<int, 3>;
    using I0 = std::integral_constant<int, 0>;
    // every other tap stream pinned too: the next column tile's B reads issue after the
    // current tile's first MFMA, not after its last (the default schedule waits on them
    // right before use: one exposed LDS round trip per column tile)
    constexpr bool p_pin = true;
    using T_ = std::true_type;
    using F_ = std::false_type;
    const int NG = p.n_chunks / NTG;
    int wslot = 0;
    for (int g = 0; g < NG; ++g) {
      const __bf16* Xh = Xbuf0 + (g & 1) * xbuf;
      __bf16* const Xn = Xbuf0 + ((g + 1) & 1) * xbuf;
      const int gn = min(g + 1, NG - 1);
#pragma unroll
      for (int tg = 0; tg < NTG; ++tg) {
        const int c = g * NTG + tg;
        const __bf16* Ws = Wbuf0 + wslot * SLAB;
        const bool ISX = tg == XG, STX = tg == NTG - 1;
        const int nt = KT_ - tg * TPC < TPC ? KT_ - tg * TPC : TPC;
        const int tap0 = tg * TPC;
        auto issue_next_w = [&]() {
          issue_w(min(c + 1, p.n_chunks - 1), Wbuf0 + (wslot ^ 1) * SLAB);
        };
        if (STX && !ISX) {
          // the slab DMA after the store: the input registers' vmcnt wait then does not
          // also wait for the new slab
          store_x(Xn);
          tap_stream(Ws, Xh, 0, tap0);
          pin_stream(I6{}, F_{}, T_{});
          issue_next_w();
        } else if (ISX && !STX) {
          issue_next_w();
          __builtin_amdgcn_sched_barrier(0);  // the slab DMA stays older than the input loads
          load_x(gn);
          tap_stream(Ws, Xh, 0, tap0);
          pin_stream(I3{}, T_{}, F_{});
        } else {
          issue_next_w();
          if (ISX) load_x(gn);
          tap_stream(Ws, Xh, 0, tap0);
          if constexpr (p_pin) pin_stream(I0{}, F_{}, F_{});
          if (STX) store_x(Xn);
        }
#pragma unroll
        for (int jj = 1; jj < TPC; ++jj)
          if (jj < nt) {
            tap_stream(Ws, Xh, jj, tap0 + jj);
            if constexpr (p_pin) pin_stream(I0{}, F_{}, F_{});
          }
        // the slab of chunk c+1 must have landed; younger: this chunk's input loads
        if (ISX && !STX) wait_x(std::integral_constant<int, NX>{});
        else wait_vm<0>();
        if (!(kAblate && (p.dbg & 4))) lds_barrier();
        wslot ^= 1;
      }
    }
  } else {
  // chunk c = (channel group g, tap group tg).  Weights: a ring of WD slabs, chunk c+WD-1
  // issued while chunk c is multiplied.  Input window: double-buffered per channel
  // group; group g+1's loads are issued at tap group xg = max(n_tg-2, 0) of group g
  // and land in LDS at the group's last tap group.
  const int xg = n_tg >= 2 ? n_tg - 2 : 0;
  int wslot = 0;                                  // ring slot of chunk c
  for (int c = 0; c < p.n_chunks; ++c) {
    const int g = c / n_tg, tg = c - (c / n_tg) * n_tg;
    const __bf16* Ws = Wbuf0 + wslot * SLAB;
    const __bf16* Xh = Xbuf0 + (g & 1) * xbuf;
    const bool more_groups = (g + 1) * n_tg < p.n_chunks;
    const bool issue_x = more_groups && tg == xg && !(kAblate && (p.dbg & 1));
    const bool store_now = more_groups && tg == n_tg - 1 && !(kAblate && (p.dbg & 1));
    // always PW pieces per thread, so every vmcnt below is a constant: past the last
    // chunk the last slab is re-read into the free slot (that of chunk c-1)
    auto issue_next_w = [&]() {
      int s2 = wslot + WD - 1;
      if (s2 >= WD) s2 -= WD;
      issue_w(min(c + WD - 1, p.n_chunks - 1), Wbuf0 + s2 * SLAB);
    };
    // with a deeper ring, the chunk that stores the next input window issues its slab
    // after that store: the compiler's vmcnt(0) for the input registers then does not
    // also wait for the new slab
    const bool w_late = WD > 2 && store_now;
    if (!w_late) issue_next_w();
    // after the slab DMA (kept older by the sched barrier): a vmcnt can wait for it, not
    // for these
    __builtin_amdgcn_sched_barrier(0);
    if (issue_x) load_x(g + 1);
    const int nt = taps_in(c);
    const int tap0 = tg * TPC;
    Frag f0, f1;
    (void)f1;
    if constexpr (WM * WN >= 8) {
      // 64x128 per wave: one fragment set in flight (the accumulators hold 128 VGPRs)
#pragma unroll
      for (int jj = 0; jj < TPC; ++jj)
        if (jj < nt) tap_stream(Ws, Xh, jj, tap0 + jj);
    } else {
      load_frag(Ws, Xh, 0, tap0, f0);
#pragma unroll
      for (int jj = 0; jj < TPC; jj += 2) {
        if (jj < nt) {
          if (jj + 1 < nt) load_frag(Ws, Xh, jj + 1, tap0 + jj + 1, f1);
          mma(f0);
          if (jj + 2 < nt) load_frag(Ws, Xh, jj + 2, tap0 + jj + 2, f0);
          if (jj + 1 < nt) mma(f1);
        }
      }
    }
    if (store_now) store_x(Xbuf0 + ((g + 1) & 1) * xbuf);
    if (w_late) issue_next_w();
    // the slab of chunk c+1 must have landed.  Younger than it: the slabs of chunks
    // c+2..c+WD-1 (PW pieces each) and this chunk's input loads when a later chunk
    // consumes them.
    if (issue_x && !store_now) wait_x(std::integral_constant<int, NX + PW * (WD - 2)>{});
    else wait_vm<PW * (WD - 2)>();
    if (!(kAblate && (p.dbg & 4))) lds_barrier();
    if (++wslot == WD) wslot = 0;
  }
  }
  if (kAblate && (p.dbg & 8)) {  // ablation: no epilogue
    if (acc[0][0][0] == 1.2345e-30f) p.y[0] = acc[WM - 1][WN - 1][15];
    return;
  }
  // products of 2^ex-scaled inputs and 2^ew-scaled weights: the exact power-of-two unscale
  // joins the bias add (fma(acc, sc, bias); bitwise acc + bias for sc = 1)
  const float sc = FMT == kFmtF16 ? exp2i(-(ex + p.ew)) : 1.0f;

  // ---- epilogue (same contract as conv1d_mfma_f32) ----
  if constexpr (UPS) {
    // polyphase scatter: GEMM row m = co*s + r lands at t = n*s + r - p.  A lane holds
    // rows 4q..4q+3 (q = r>>2 block of its half): with s % 4 == 0 and p % 4 == 0 those
    // are 4 consecutive phases of one co, i.e. 4 consecutive output samples at a 16-B
    // aligned t: one float4 store instead of four scattered dword stores.
    const int s_ = p.ups_s, p_ = p.ups_p;
    const bool vec4 = (s_ & 3) == 0 && (p_ & 3) == 0 && (p.L_out & 3) == 0;
    float* __restrict__ yb = p.y + (int64_t)b * p.y_bs;
    // row -> (co, phase): a shift for the power-of-two rates (V1/V2: 8, 8, 2, 2) instead
    // of an integer division per accumulator row
    const bool pow2 = (s_ & (s_ - 1)) == 0;
    const int sh = __builtin_ctz((unsigned)s_);
    auto co_of = [&](int row) { return pow2 ? row >> sh : row / s_; };
    float vmax = 0.f;  // max |stored value| (f16x3 consumers: p.amax_out)
    auto track4 = [&](const float4& v) {
      vmax = fmaxf(vmax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    };
#pragma unroll
    for (int i = 0; i < WM; ++i) {
      const int rb = mt * MT + wave_m * 32 * WM + i * 32 + 4 * half;  // row of r = 0
      float bv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) bv[r] = p.bias[rb + (r & 3) + 8 * (r >> 2)];
#pragma unroll
      for (int k = 0; k < WN; ++k) {
        const int n = n0 + wave_n * 32 * WN + k * 32 + col;
        // wave-uniform interior test (the whole 32-column x 32-row tile lands inside
        // [0, L_out)): unmasked float4 stores, one instruction each (the masked path
        // below compiles to a tail-merged dwordx3 + dword pair)
        const int nt_u = n0 + (wave_u / WAVES_M) * 32 * WN + k * 32;
        const int rt_u = mt * MT + (wave_u % WAVES_M) * 32 * WM + i * 32;
        if (vec4 && rt_u + 31 < p.M && nt_u + 31 < N_b && nt_u * s_ - p_ >= 0 &&
            (nt_u + 32) * s_ - 1 - p_ < L_out_b) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int row = rb + 8 * q;
            const int co = co_of(row);
            const int t = n * s_ + (row - co * s_) - p_;
            float4 v;
            v.x = __builtin_fmaf(acc[i][k][4 * q + 0], sc, bv[4 * q + 0]);
            v.y = __builtin_fmaf(acc[i][k][4 * q + 1], sc, bv[4 * q + 1]);
            v.z = __builtin_fmaf(acc[i][k][4 * q + 2], sc, bv[4 * q + 2]);
            v.w = __builtin_fmaf(acc[i][k][4 * q + 3], sc, bv[4 * q + 3]);
            *reinterpret_cast<float4*>(yb + (int64_t)co * p.L_out + t) = v;
            track4(v);
          }
          continue;
        }
        if (n >= N_b) continue;
        if (vec4) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int row = rb + 8 * q;
            if (row >= p.M) continue;
            const int co = co_of(row);
            const int t = n * s_ + (row - co * s_) - p_;
            float4 v;
            v.x = __builtin_fmaf(acc[i][k][4 * q + 0], sc, bv[4 * q + 0]);
            v.y = __builtin_fmaf(acc[i][k][4 * q + 1], sc, bv[4 * q + 1]);
            v.z = __builtin_fmaf(acc[i][k][4 * q + 2], sc, bv[4 * q + 2]);
            v.w = __builtin_fmaf(acc[i][k][4 * q + 3], sc, bv[4 * q + 3]);
            float* dst = yb + (int64_t)co * p.L_out + t;
            if (t >= 0 && t + 3 < L_out_b) {
              *reinterpret_cast<float4*>(dst) = v;
              track4(v);
            } else {
              if (t + 0 >= 0 && t + 0 < L_out_b) dst[0] = v.x, vmax = fmaxf(vmax, fabsf(v.x));
              if (t + 1 >= 0 && t + 1 < L_out_b) dst[1] = v.y, vmax = fmaxf(vmax, fabsf(v.y));
              if (t + 2 >= 0 && t + 2 < L_out_b) dst[2] = v.z, vmax = fmaxf(vmax, fabsf(v.z));
              if (t + 3 >= 0 && t + 3 < L_out_b) dst[3] = v.w, vmax = fmaxf(vmax, fabsf(v.w));
            }
          }
          continue;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = rb + (r & 3) + 8 * (r >> 2);
          if (row >= p.M) continue;
          const int co = co_of(row);
          const int t = n * s_ + (row - co * s_) - p_;
          if (t >= 0 && t < L_out_b) {
            const float v = __builtin_fmaf(acc[i][k][r], sc, bv[r]);
            yb[(int64_t)co * p.L_out + t] = v;
            vmax = fmaxf(vmax, fabsf(v));
          }
        }
      }
    }
    if (p.amax_out) amax_commit(vmax, p.amax_out, b);
  } else {
    // LDS-staged float4 epilogue (epilogue.h) when the rows are 16-B aligned and the host
    // sized the LDS for it (p.epi_lds); the accumulator-layout epilogue otherwise
    if (p.epi_lds && (p.N & 3) == 0) {
      // every wave is done with the weight slabs and input windows, and no weight-slab
      // LDS-DMA is still in flight (a deeper ring leaves the re-read past-the-end slabs
      // outstanding; they count in vmcnt, not lgkmcnt)
      wait_vm<0>();
      lds_barrier();
      cstamp(7);
      float* stage = reinterpret_cast<float*>(lds16) + wave * 32 * (32 * WN + 8);
      if constexpr (AREG)
        conv_epilogue_lds2<WM, WN>(p, acc, b, mt * MT + wave_m * 32 * WM, mt * MT,
                                   n0 + wave_n * 32 * WN, N_b, half, col, stage, bias_lds, lane,
#if HFG_CONV_TIMING
                                   sc, tsv);
#else
                                   sc);
#endif
      else
        conv_epilogue_lds<WM, WN>(p, acc, b, mt * MT + wave_m * 32 * WM, n0 + wave_n * 32 * WN,
                                  N_b, half, col, stage, lane, sc);
    } else {
      conv_epilogue<WM, WN>(p, acc, b, mt * MT + wave_m * 32 * WM, n0 + wave_n * 32 * WN, N_b,
                            half, col, sc);
    }
  }
  cstamp(4);
#if HFG_CONV_TIMING
  tsv[6] = __builtin_amdgcn_s_memrealtime();
  if (AREG && tid == 0)
#pragma unroll
    for (int i = 0; i < 16; ++i) cts[i] = tsv[i];
#endif
}

namespace {

typedef void (*ConvFn3)(const ConvParams);

template <int KT, int TILE, bool UPS, int NP, int FMT>
struct Inst3 {
  static constexpr Bf16x3Cfg t = kBf16x3Tiles[TILE];
  static ConvFn3 fn() {
    return conv1d_bf16x3<KT, t.TPC, t.WAVES_M, t.WAVES_N, t.WM, t.WN, t.WD, UPS, NP, t.AREG != 0,
                         FMT>;
  }
};

struct Entry3 {
  int kt;
  int tile;
  bool ups;
  int np, fmt;
  ConvFn3 fn;
  char name[112];
};

#define HFG3_ENTRY(KT, TILE, UPS, NP, FMT) \
  { KT, TILE, UPS, NP, FMT, Inst3<KT, TILE, UPS, NP, FMT>::fn(), {0} }
// per tile: bf16x3 (NP 3, bf16), f16x3 (NP 3, f16) and bf16w (NP 2 on the f16 kernels: the
// bf16-rounded weights are exact f16 halves after their power-of-two scale, lo(w) = 0)
#define HFG3_VARIANTS(KT, TILE, UPS) \
  HFG3_ENTRY(KT, TILE, UPS, 3, 0), HFG3_ENTRY(KT, TILE, UPS, 3, 1), HFG3_ENTRY(KT, TILE, UPS, 2, 1)
// tiles 1-4 (tile 0, the 8-wave 128x256 tile with a 3-deep slab ring, was removed in round 4:
// slower than tile 3 / 5 everywhere it applied)
#define HFG3_TILES(KT, UPS)                                                            \
  HFG3_VARIANTS(KT, 1, UPS), HFG3_VARIANTS(KT, 2, UPS), HFG3_VARIANTS(KT, 3, UPS),     \
      HFG3_VARIANTS(KT, 4, UPS)

// tiles 5 and 6 (AREG): compile-time taps, layer convs only
#define HFG3_AREG(KT) HFG3_VARIANTS(KT, 5, false), HFG3_VARIANTS(KT, 6, false)
Entry3 g_entries3[] = {
    HFG3_TILES(3, false), HFG3_TILES(5, false), HFG3_TILES(7, false), HFG3_TILES(11, false),
    HFG3_TILES(0, false), HFG3_TILES(2, true),  HFG3_TILES(0, true),
    HFG3_AREG(3),         HFG3_AREG(5),         HFG3_AREG(7),         HFG3_AREG(11),
};

}  // namespace

size_t bf16x3_lds_bytes(int tile, int kt, int dil) {
  const Bf16x3Cfg& t = kBf16x3Tiles[tile];
  // bf16: taps x planes x rows x 16 ch (no slab ring on the AREG tile)
  const size_t slab = t.AREG ? 0 : (size_t)t.TPC * 2 * t.MT() * 16;
  // AREG: a plane row per staging task (the kernel's XROWS_AREG)
  const int xw = t.AREG ? bf16x3_areg_rows(kt, t) : t.NTILE() + (kt - 1) * dil;
  // AREG: two padded half planes (the kernel's HPS_AREG)
  const size_t xplane = t.AREG ? (size_t)xw * 16 + 64 : ((size_t)xw * 16 + 7) & ~(size_t)7;
  return sizeof(__bf16) * (t.WD * slab + 2 * 2 * xplane);  // weight ring + 2 (hi,lo) windows
}

hipError_t launch_conv_bf16x3(int tile, int kt, bool ups, int fmt, int np, const ConvParams& p,
                              int n_tiles, int m_tiles, int batch, hipStream_t stream,
                              const char** name) {
  Entry3* e = nullptr;
  Entry3* generic = nullptr;
  for (auto& cand : g_entries3) {
    if (cand.tile != tile || cand.ups != ups || cand.np != np || cand.fmt != fmt) continue;
    if (cand.kt == kt) e = &cand;
    if (cand.kt == 0) generic = &cand;
  }
  if (!e) e = generic;
  if (!e) return hipErrorInvalidValue;
  if (p.dil > kMaxDil || (e->kt == 0 && kt > 16) || (kt - 1) * p.dil > kBf16x3MaxHalo)
    return hipErrorInvalidValue;
  const Bf16x3Cfg& t = kBf16x3Tiles[tile];
  {
    std::lock_guard<std::mutex> lk(setup_mutex());
    if (!e->name[0])
      snprintf(e->name, sizeof(e->name), "conv1d_bf16x3<%d, %d, %d, %d, %d, %d, %d, %s, %d, %s, %d>",
               e->kt, t.TPC, t.WAVES_M, t.WAVES_N, t.WM, t.WN, t.WD, e->ups ? "true" : "false",
               e->np, t.AREG ? "true" : "false", e->fmt);
  }
  size_t lds = bf16x3_lds_bytes(tile, kt, p.dil);
  if (p.epi_lds && !ups)
    lds = std::max(lds, (size_t)t.threads() / 64 * 32 * (32 * t.WN + 8) * sizeof(float));
  // AREG: + the m-tile's bias copy (its kernel instance is compiled for its KT)
  if (t.AREG) lds = (size_t)bf16x3_areg_bias_off(e->kt, t) + (size_t)t.MT() * sizeof(float);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (hipError_t err = ensure_max_lds(reinterpret_cast<const void*>(e->fn)))
    return err;
  if (name) *name = e->name;
  dim3 grid(n_tiles, m_tiles, batch);
  e->fn<<<grid, dim3(t.threads()), lds, stream>>>(p);
  return hipGetLastError();
}

}  // namespace hfg

#if HFG_CONV_TIMING
extern "C" int hfg_debug_cv_ts(void* dst, size_t bytes) {
  if (bytes > sizeof(hfg::g_cv_ts)) bytes = sizeof(hfg::g_cv_ts);
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(hfg::g_cv_ts), bytes, 0, hipMemcpyDeviceToHost);
}
extern "C" int hfg_debug_cv_ts_clear() {
  static uint64_t* z = nullptr;
  if (!z) z = (uint64_t*)calloc(1, sizeof(hfg::g_cv_ts));
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(hfg::g_cv_ts), z, sizeof(hfg::g_cv_ts), 0, hipMemcpyHostToDevice);
}
#endif

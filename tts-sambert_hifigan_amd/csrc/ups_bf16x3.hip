// ups_bf16x3.hip — the HiFi-GAN upsampler, lrelu -> ConvTranspose1d(C_in, C_out, k = 2u,
// stride u, padding u/2) (models/hifigan.py:195-203, 244-245), as a split-precision
// ("bf16x3") GEMM over OUTPUT FRAMES on the gfx950 bf16 matrix cores.
//
// Output sample t = m*u + s of frame m (s in [0, u), h = u/2) receives exactly two taps:
//   class L (s <  h):  W[ci][co][s+h+u] * x[m-1]  +  W[ci][co][s+h] * x[m]
//   class R (s >= h):  W[ci][co][s+h]   * x[m]    +  W[ci][co][s-h] * x[m+1]
// so the GEMM columns are the T input frames themselves (no T+1 polyphase column and no
// tail tile of one column), and every class has one block-uniform input offset per tap.
// GEMM rows of a class: rr = co*h + s' (s' = s - class*h); a wave computes BOTH classes of
// its rows and columns, so a lane ends up holding whole runs of consecutive samples:
//   u = 2 (h = 1): (L, R) = samples 2m, 2m+1 of one channel; a DPP swap with the lane of
//                  frame m^1 makes it 4 samples -> one 16-B store per channel pair
//   u = 4 (h = 2): rows (co,0),(co,1) x (L, R) = samples 4m..4m+3 -> one 16-B store
//   h % 4 == 0:    4 consecutive rows = 4 consecutive samples      -> 16-B stores per class
// (the polyphase kernel in conv_bf16x3.hip stores u = 2 stages one dword per value).
//
// Per output element the MFMA sequence is the polyphase kernel's (channel groups in order;
// the x[m-1|m] tap before the x[m|m+1] tap; lo*hi, hi*lo, hi*hi), the split of lrelu(x) and
// the zero padding are the same, the bias is added last: the result is bitwise equal to
// conv1d_bf16x3<..., UPS> (tests/test_gpu_parity.py::test_ups_frames_kernel_bitwise).
//
// Data flow per 16-channel group g (one barrier per group):
//   * A (weights): the host packs [m_tile][g][class][tap][plane][wave_m][wm][lane][8] bf16;
//     the group's slab (128 * MT_c bf16) is copied to a 2-slot LDS ring by LDS-DMA one group
//     ahead (no VGPRs).
//   * B (lrelu'd, split input): the window of frames [m0-4, m0+NTILE+4) (quad-aligned, so
//     every load is one 16-B dwordx4: 4 frames of one channel) is loaded one group ahead into
//     registers, converted after the group's MFMAs and written as [frame][16 ch] bf16 hi / lo
//     planes (16-B slots XOR-swizzled per 256-B block, xrow_off: conflict-free ds_read_b128
//     for the three tap offsets -1, 0, +1, and staging writes within their transfer cycles).
#include <hip/hip_runtime.h>

#include <mutex>

#include <cstdio>

#include "bf16x3_common.h"
#include "kernels.h"

// u = 2 epilogue: 16-B stores through a DPP pair swap (1) or 8-B stores (0)
#ifndef HFG_UPS_PAIR
#define HFG_UPS_PAIR 1
#endif

#ifndef HFG_UPS_SMALL_OCC
#define HFG_UPS_SMALL_OCC 3
#endif

namespace hfg {

namespace {
typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
}  // namespace

// occupancy: the small tile (2 x 32 x 32 accumulators per class) fits 168 VGPRs, 3 waves per
// SIMD; its launches (the thin last upsampler) are bound by HBM latency, not the matrix pipe
template <int WAVES_M, int WAVES_N, int WM, int WN>
constexpr int ups_min_blocks() { return WAVES_M * WM * WN <= 2 ? HFG_UPS_SMALL_OCC : 2; }

template <int WAVES_M, int WAVES_N, int WM, int WN, int NP, int FMT>
__global__ void __launch_bounds__(64 * WAVES_M * WAVES_N, (ups_min_blocks<WAVES_M, WAVES_N, WM, WN>()))
ups_bf16x3(const UpsParams p) {
  constexpr int NW = WAVES_M * WAVES_N;
  constexpr int MT = 32 * WM * WAVES_M;      // rows per class and m-tile
  constexpr int NTILE = 32 * WN * WAVES_N;   // frames per block
  constexpr int XR = NTILE + 8;              // staged frames: [m0 - 4, m0 + NTILE + 4)
  constexpr int NQ = XR / 4;                 // frame quads
  constexpr int NTASK = 2 * NQ;              // (quad, 8-channel half) staging tasks
  constexpr int TPW = (NTASK + NW - 1) / NW; // tasks per wave (one per lane)
  static_assert(TPW <= 64, "one staging task per lane");
  constexpr int XPLANE = XR * 32;            // bytes per bf16 plane [frame][16 ch]
  constexpr int XBUF = 2 * XPLANE;           // hi + lo
  constexpr int SLAB = 2 * 2 * 2 * WAVES_M * WM * 1024;  // bytes: class x tap x plane x rows
  constexpr int PW = SLAB / 1024 / NW;       // LDS-DMA pieces per thread per slab
  static_assert(PW * 1024 * NW == SLAB, "slab must split evenly over the waves");

  // byte offset of (frame row r, 8-channel half h) in a staged plane: the 16-B slot 2r + h
  // XOR-swizzled inside its 256-B block by bits 2-3 of r.  The B reads (16 consecutive rows of
  // one half per 16-lane group) stay conflict-free, and so do the staging writes (8 lanes =
  // 4 quads x 2 halves, task order below), which the unswizzled layout put on 2 of the 8 16-B
  // slots of a bank window (1.2 conflict cycles per LDS-active cycle; bank model
  // tests/tools/ups_lds_banks.py)
  auto xrow_off = [](int r, int h) {
    return 16 * ((2 * r + h) ^ (((r >> 3) & 1) * 5 + ((r >> 2) & 1) * 2));
  };
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* const Abuf = lds;                    // 2 slabs
  char* const Xbuf = lds + 2 * SLAB;         // 2 x (hi, lo) planes

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wave_m = wave % WAVES_M;
  const int wave_n = wave / WAVES_M;
  const int half = lane >> 5;
  const int col = lane & 31;

  // block -> (m-tile fastest, frame tile, item), through an XCD swizzle: the m-tiles of one
  // window run on one XCD (blocks b and b + 8 share an XCD under round-robin placement)
  int mt, tx, b;
  {
    const int total = p.m_tiles * p.n_tiles * p.batch;
    int id = blockIdx.x;
    const int q = total >> 3;
    if (id < (q << 3)) id = (id & 7) * q + (id >> 3);
    mt = id % p.m_tiles;
    id /= p.m_tiles;
    tx = id % p.n_tiles;
    b = id / p.n_tiles;
    mt = __builtin_amdgcn_readfirstlane(mt);
    tx = __builtin_amdgcn_readfirstlane(tx);
    b = __builtin_amdgcn_readfirstlane(b);
  }
  const int T_b = p.len_in ? min(p.len_in[b], p.T) : p.T;
  // f16x3 (bf16x3_common.h): input scale from the producer's per-item max, unscale after
  const int ex = FMT == kFmtF16 ? x3_exp_slot(p.amax_in, b) : 0;
  const float sx = FMT == kFmtF16 ? exp2i(ex) : 1.0f;
  const int m0 = tx * NTILE;
  if (m0 >= T_b) return;  // whole tile past this utterance's end (block-uniform)
  const int NG = p.C_in / 16;

  // ---- A slab ring: LDS-DMA, PW pieces per thread ----
  const char* wsrc = reinterpret_cast<const char*>(p.w) + (int64_t)mt * NG * SLAB;
  auto issue_a = [&](int g, int slot) {
    const char* src = wsrc + (int64_t)g * SLAB;
    char* dst = Abuf + slot * SLAB;
#pragma unroll
    for (int q = 0; q < PW; ++q) {
      const int i = wave + q * NW;
      __builtin_amdgcn_global_load_lds((gptr_t1)(src + i * 1024 + lane * 16),
                                       (lds_ptr_t3)(dst + i * 1024), 16, 0, 0);
    }
  };

  // ---- input staging: one (quad, half) task per lane of the first TPW lanes ----
  // one buffer descriptor per 16-channel group (SGPR base + record count: a whole 4-GiB
  // item would not fit the 32-bit count); a quad outside its row reads offset 0 (masked)
  const char* xb = reinterpret_cast<const char*>(p.x + (int64_t)b * p.x_bs);
  const int64_t grp_bytes = (int64_t)16 * p.L * 4;
  const int grp_rec = (int)(unsigned)(grp_bytes < 0xFFFFFFFFll ? grp_bytes : 0xFFFFFFFFll);
  const int task = wave * TPW + lane;
  const bool has_task = lane < TPW && task < NTASK;
  // (quad, half) interleaved: the 8 lanes of a ds_write_b128 group write 4 quads x both
  // halves, which xrow_off's swizzle puts on the 8 distinct 16-B slots of a bank window
  const int hf = task & 1;                   // channel half of the task
  const int xq = task >> 1;                  // quad of the task
  const int t0 = m0 - 4 + 4 * xq;            // first frame of the quad
  // leaky_relu as max(v * sx, v * 0.1 sx) (f16x3 scale sx; bitwise max(v, 0.1 v) for bf16x3)
  // and the zero padding as a select: frames in [T_b, L) of a ragged item were never written
  // (0 * NaN would be NaN), and the polyphase kernel reads no such frame
  const float sx1 = kLReluSlope * sx;
  bool okt[4];
#pragma unroll
  for (int tt = 0; tt < 4; ++tt) okt[tt] = has_task && (unsigned)(t0 + tt) < (unsigned)T_b;
  // whole quads only (L % 4 == 0, host-checked): a quad is inside the row or wholly outside
  const bool q_in = has_task && t0 >= 0 && t0 < p.L;
  const unsigned xoff_lane = q_in ? (unsigned)(8 * hf * p.L + t0) * 4u : 0u;
  const int xcs4 = p.L * 4;
  typedef float f4 __attribute__((ext_vector_type(4)));
  f4 xv[8];
  auto load_x = [&](int g) {
    const __amdgpu_buffer_rsrc_t xrs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(xb + g * grp_bytes), 0, grp_rec, 0x00020000);
#pragma unroll
    for (int e = 0; e < 8; ++e)
      xv[e] = __builtin_bit_cast(
          f4, __builtin_amdgcn_raw_buffer_load_b128(xrs, (int)xoff_lane, e * xcs4, 0));
  };
  auto store_x = [&](int buf) {
    if (!has_task) return;
    char* xh = Xbuf + buf * XBUF;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bf16x8 hv, lv;
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        floatx2 a;
        a[0] = okt[j] ? fmaxf(xv[e][j] * sx, xv[e][j] * sx1) : 0.f;
        a[1] = okt[j] ? fmaxf(xv[e + 1][j] * sx, xv[e + 1][j] * sx1) : 0.f;
        bf16x2 hh, ll;
        split2<FMT>(a, hh, ll);
        hv[e] = hh[0];
        hv[e + 1] = hh[1];
        lv[e] = ll[0];
        lv[e + 1] = ll[1];
      }
      const int off = xrow_off(4 * xq + j, hf);
      *reinterpret_cast<bf16x8*>(xh + off) = hv;
      *reinterpret_cast<bf16x8*>(xh + XPLANE + off) = lv;
    }
  };

  floatx16 acc[2][WM][WN];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int k = 0; k < WN; ++k)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[c][i][k][r] = 0.f;

  // ---- prologue: group 0 ----
  issue_a(0, 0);
  load_x(0);
  store_x(0);
  wait_vm<0>();
  lds_barrier();

  // B fragment rows: window row of frame m0 + colw is colw + 4
  const int colw = wave_n * 32 * WN + col + 4;
  for (int g = 0; g < NG; ++g) {
    const bool more = g + 1 < NG;  // block-uniform
    // ablation bit 17 (timing only): no weight slab after group 0's (every group re-reads it)
    const bool slab0 = kAblate && (p.dbg & 131072);
    if (more) {
      if (!slab0) issue_a(g + 1, (g + 1) & 1);
      if (!(kAblate && (p.dbg & 1024))) load_x(g + 1);
    }
    // A fragments of both classes and taps: [class][tap][plane][wm]
    const char* as = Abuf + (slab0 ? 0 : (g & 1)) * SLAB;
    bf16x8 a[2][2][2][WM];
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int tp = 0; tp < 2; ++tp)
#pragma unroll
        for (int pl = 0; pl < 2; ++pl)
#pragma unroll
          for (int i = 0; i < WM; ++i)
            a[c][tp][pl][i] = *reinterpret_cast<const bf16x8*>(
                as + ((((c * 2 + tp) * 2 + pl) * WAVES_M + wave_m) * WM + i) * 1024 + lane * 16);
    const char* xh = Xbuf + (g & 1) * XBUF;
    prio_mfma();
#pragma unroll
    for (int k = 0; k < WN; ++k) {
      // B at tap offsets -1, 0, +1 (hi, lo)
      bf16x8 bh[3], bl[3];
#pragma unroll
      for (int o = 0; o < 3; ++o) {
        const int off = xrow_off(colw + 32 * k + o - 1, half);
        bh[o] = *reinterpret_cast<const bf16x8*>(xh + off);
        bl[o] = *reinterpret_cast<const bf16x8*>(xh + XPLANE + off);
      }
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int tp = 0; tp < 2; ++tp) {
            const int o = c + tp;  // class L: offsets -1, 0 (o = 0, 1); class R: 0, +1 (1, 2)
            if constexpr (NP == 3)
              acc[c][i][k] = mfma32<FMT>(a[c][tp][1][i], bh[o],
                                                                    acc[c][i][k]);
            acc[c][i][k] = mfma32<FMT>(a[c][tp][0][i], bl[o],
                                                                  acc[c][i][k]);
            acc[c][i][k] = mfma32<FMT>(a[c][tp][0][i], bh[o],
                                                                  acc[c][i][k]);
          }
    }
    prio_other();
    if (more && !(kAblate && (p.dbg & 512))) store_x((g + 1) & 1);
    wait_vm<0>();
    lds_barrier();
  }

  // f16x3: the exact power-of-two unscale joins the bias add (fma; bitwise acc + bias at 1)
  const float sc = FMT == kFmtF16 ? exp2i(-(ex + p.ew)) : 1.0f;

  // ---- epilogue: bias, stores of whole sample runs ----
  float* yb = p.y + (int64_t)b * p.y_bs;
  float vmax = 0.f;  // max |stored value| (f16x3 consumers: p.amax_out)
  auto t2 = [&](float a, float c) { vmax = fmaxf(vmax, fmaxf(fabsf(a), fabsf(c))); };
  const int h = p.u >> 1;
#pragma unroll
  for (int i = 0; i < WM; ++i) {
    const int rb = mt * MT + wave_m * 32 * WM + i * 32 + 4 * half;  // row of r = 0
#pragma unroll
    for (int k = 0; k < WN; ++k) {
      const int m = m0 + wave_n * 32 * WN + k * 32 + col;
      if (m >= T_b) continue;
      if (h == 1 && HFG_UPS_PAIR) {
        // rows = channels: (L, R) = samples 2m, 2m + 1.  Adjacent lanes (frames m, m + 1,
        // m even) swap one channel's pair (DPP quad_perm [1,0,3,2]): the even lane then
        // holds samples 2m .. 2m + 3 of channel r, the odd lane those of channel r + 1 ->
        // one 16-B store per lane and channel pair instead of two 8-B stores
        const bool odd = col & 1;
        const int me = m - (odd ? 1 : 0);  // even frame of the pair
        const bool quad_ok = me + 1 < T_b;
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          const int co0 = rb + (r & 3) + 8 * (r >> 2);
          const float b0 = p.bias[co0], b1 = p.bias[co0 + 1];
          const float l0 = __builtin_fmaf(acc[0][i][k][r], sc, b0);
          const float r0 = __builtin_fmaf(acc[1][i][k][r], sc, b0);
          const float l1 = __builtin_fmaf(acc[0][i][k][r + 1], sc, b1);
          const float r1 = __builtin_fmaf(acc[1][i][k][r + 1], sc, b1);
          const float s0 = odd ? l0 : l1, s1 = odd ? r0 : r1;
          const float v0 = __builtin_bit_cast(
              float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, s0), 0xB1, 0xF, 0xF, false));
          const float v1 = __builtin_bit_cast(
              float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, s1), 0xB1, 0xF, 0xF, false));
          if (quad_ok) {
            float4 v;
            v.x = odd ? v0 : l0;
            v.y = odd ? v1 : r0;
            v.z = odd ? l1 : v0;
            v.w = odd ? r1 : v1;
            if (!(kAblate && (p.dbg & 262144))) *reinterpret_cast<float4*>(yb + (int64_t)(odd ? co0 + 1 : co0) * p.L_out + 2 * me) = v;
            t2(v.x, v.y);
            t2(v.z, v.w);
          } else {
            // last frame of an odd-length utterance (even lane, its odd partner past T_b):
            // both channels' pairs as 8-B stores
            floatx2 a, c;
            a[0] = l0;
            a[1] = r0;
            c[0] = l1;
            c[1] = r1;
            if (!(kAblate && (p.dbg & 262144))) *reinterpret_cast<floatx2*>(yb + (int64_t)co0 * p.L_out + 2 * m) = a;
            if (!(kAblate && (p.dbg & 262144))) *reinterpret_cast<floatx2*>(yb + (int64_t)(co0 + 1) * p.L_out + 2 * m) = c;
            t2(l0, r0);
            t2(l1, r1);
          }
        }
      } else if (h == 1) {
        // rows = channels: (L, R) = samples 2m, 2m + 1
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int co = rb + (r & 3) + 8 * (r >> 2);
          const float bv = p.bias[co];
          floatx2 v;
          v[0] = __builtin_fmaf(acc[0][i][k][r], sc, bv);
          v[1] = __builtin_fmaf(acc[1][i][k][r], sc, bv);
          if (!(kAblate && (p.dbg & 262144))) *reinterpret_cast<floatx2*>(yb + (int64_t)co * p.L_out + 2 * m) = v;
          t2(v[0], v[1]);
        }
      } else if (h == 2) {
        // rows (co, 0), (co, 1), (co + 1, 0), (co + 1, 1): samples 4m .. 4m + 3 of co, co + 1
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int pr = 0; pr < 2; ++pr) {
            const int r0 = 4 * q + 2 * pr;
            const int co = (rb + 8 * q + 2 * pr) >> 1;
            const float bv = p.bias[co];
            float4 v;
            v.x = __builtin_fmaf(acc[0][i][k][r0], sc, bv);
            v.y = __builtin_fmaf(acc[0][i][k][r0 + 1], sc, bv);
            v.z = __builtin_fmaf(acc[1][i][k][r0], sc, bv);
            v.w = __builtin_fmaf(acc[1][i][k][r0 + 1], sc, bv);
            if (!(kAblate && (p.dbg & 262144))) *reinterpret_cast<float4*>(yb + (int64_t)co * p.L_out + 4 * m) = v;
            t2(v.x, v.y);
            t2(v.z, v.w);
          }
      } else {
        // h % 4 == 0: 4 consecutive rows = s' .. s' + 3 of one channel, per class
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int row = rb + 8 * q;
          const int co = row / h, sp = row - co * h;
          const float bv = p.bias[co];
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            float4 v;
            v.x = __builtin_fmaf(acc[c][i][k][4 * q + 0], sc, bv);
            v.y = __builtin_fmaf(acc[c][i][k][4 * q + 1], sc, bv);
            v.z = __builtin_fmaf(acc[c][i][k][4 * q + 2], sc, bv);
            v.w = __builtin_fmaf(acc[c][i][k][4 * q + 3], sc, bv);
            if (!(kAblate && (p.dbg & 262144))) *reinterpret_cast<float4*>(yb + (int64_t)co * p.L_out + m * p.u + c * h + sp) = v;
            t2(v.x, v.y);
            t2(v.z, v.w);
          }
        }
      }
    }
  }
  if (p.amax_out) amax_commit(vmax, p.amax_out, b);
}

namespace {

typedef void (*UpsFn)(const UpsParams);

struct EntryUps {
  int cfg, np, fmt;
  UpsFn fn;
  char name[64];
};

#define HFGUPS_ENTRY(CFG, NP, FMT)                                                           \
  {                                                                                          \
    CFG, NP, FMT,                                                                            \
        ups_bf16x3<kUpsCfgs[CFG].WAVES_M, kUpsCfgs[CFG].WAVES_N, kUpsCfgs[CFG].WM,          \
                   kUpsCfgs[CFG].WN, NP, FMT>,                                               \
    {                                                                                        \
      0                                                                                      \
    }                                                                                        \
  }

// bf16x3 (NP 3, bf16), f16x3 (NP 3, f16), bf16w (NP 2 on the f16 kernel)
EntryUps g_entriesUps[] = {HFGUPS_ENTRY(0, 3, 0), HFGUPS_ENTRY(1, 3, 0), HFGUPS_ENTRY(0, 3, 1),
                           HFGUPS_ENTRY(1, 3, 1), HFGUPS_ENTRY(0, 2, 1), HFGUPS_ENTRY(1, 2, 1)};

}  // namespace

size_t ups_lds_bytes(int cfg) {
  const UpsCfg& t = kUpsCfgs[cfg];
  const size_t slab = (size_t)2 * 2 * 2 * t.WAVES_M * t.WM * 1024;
  const size_t xr = (size_t)t.NTILE() + 8;
  return 2 * slab + 2 * 2 * xr * 32;
}

hipError_t launch_ups_bf16x3(int cfg, int fmt, int np, const UpsParams& p, hipStream_t stream,
                             const char** name) {
  EntryUps* e = nullptr;
  for (auto& cand : g_entriesUps)
    if (cand.cfg == cfg && cand.np == np && cand.fmt == fmt) e = &cand;
  if (!e) return hipErrorInvalidValue;
  const UpsCfg& t = kUpsCfgs[cfg];
  // shapes the kernel's indexing assumes
  if (p.C_in % 16 != 0 || p.L % 4 != 0 || p.T > p.L || p.u < 2 || (p.u & 1) ||
      !ups_rate_ok(p.u) || p.L_out < p.L * p.u || p.m_tiles * t.MT() * 2 != p.C_out * p.u ||
      p.n_tiles * t.NTILE() < p.T || (int64_t)p.C_in * p.L > ((int64_t)1 << 30))
    return hipErrorInvalidValue;
  {
    std::lock_guard<std::mutex> lk(setup_mutex());
    if (!e->name[0])
      snprintf(e->name, sizeof(e->name), "ups_bf16x3<%d, %d, %d, %d, %d, %d>", t.WAVES_M,
               t.WAVES_N, t.WM, t.WN, np, fmt);
  }
  const size_t lds = ups_lds_bytes(cfg);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (hipError_t err = ensure_max_lds(reinterpret_cast<const void*>(e->fn))) return err;
  if (name) *name = e->name;
  const int blocks = p.m_tiles * p.n_tiles * p.batch;
  e->fn<<<dim3(blocks), dim3(t.threads()), lds, stream>>>(p);
  return hipGetLastError();
}

}  // namespace hfg

// mrf_thin.hip — a whole MRF stage of a thin-channel stage (C <= 16) in one launch:
//
//   for j in resblocks:  xr = x
//                        for m in dilations: xr = xr + conv2_jm(lrelu(conv1_jm(lrelu(xr))))
//                                                            models/hifigan.py:79-85
//                        mrf = xr (j = 0) | mrf + xr          models/hifigan.py:125-130
//   y = mrf / n_res                                           models/hifigan.py:131
//
// Why a VALU kernel.  With C = 8 or 16 channels a conv's contraction (C x k per output) is
// too thin for the matrix cores' 16/32-row tiles (the layer kernels padded it to 32 rows and
// streamed five tensor passes per dilation through HBM: ~8 of V2*'s 10 ms at [16,80,2048]).
// Here the whole MRF runs on a time window held in LDS — x is read from HBM (L2 after the
// first ResBlock) and y written once — and every conv is an LDS dot product on the packed
// fp32 VALU (v_pk_fma_f32, 2 columns per lane per instruction): exact fp32 products with
// fp32 accumulation, in both precision modes.
//
// Mapping.  A block of NT threads owns a window of NWIN = NT * NCOL columns; lane l of wave
// w owns columns w*64*NCOL + l + 64*i (i < NCOL), so a wave's LDS reads of one channel row
// are 64 consecutive floats (conflict-free, ds_read2_b32 pairs).  Each thread keeps, for its
// columns, every channel of the ResBlock state xr, the MRF sum and the conv accumulator in
// registers.  The conv operand (lrelu of the previous conv's output, zero outside [0, len))
// is one LDS buffer [C][MARG + NWIN + MARG], rewritten after every conv.  Weights are
// uniform across the block: packed per conv as [tap][ci][co] and read with scalar loads
// (s_load_dwordx16 of the C output channels of one (tap, ci)).
//
// Receptive field: edge columns turn to garbage one conv radius at a time; the block
// stores only the centre [halo, halo + W) where halo = the largest ResBlock radius
// (sum over its convs of (k - 1) / 2 * d).  Columns outside [0, len) are re-zeroed in
// every operand write — the zero padding of each reference conv input.
#include <hip/hip_runtime.h>

#include <mutex>

#include <cstdio>

#include "bf16x3_common.h"
#include "kernels.h"

namespace hfg {

namespace {
typedef float floatx2 __attribute__((ext_vector_type(2)));
// constant address space: block-uniform weight / bias reads become scalar loads (SGPRs)
typedef __attribute__((address_space(4))) const float cfloat;
}  // namespace

template <int C, int NCOL, int NT, int WPE>
__global__ void __launch_bounds__(NT, WPE)  // waves/SIMD: they hide each other's
mrf_thin(const ThinParams p) {             // lgkmcnt(0) waits on the scalar weight loads
  static_assert(NCOL % 2 == 0, "columns go in pairs (packed fp32)");
  constexpr int NP = NCOL / 2;            // column pairs per thread
  constexpr int NWIN = NT * NCOL;
  constexpr int MARG = kThinMarg;
  constexpr int RS = NWIN + 2 * MARG;     // LDS row stride (floats)
  constexpr int CG = C < 2 ? C : 2;       // input channels per scalar-load group
  extern __shared__ __attribute__((aligned(16))) float op[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int b = blockIdx.y;
  const int len_b = p.len ? min(p.len[b], p.L) : p.L;
  const int t0 = blockIdx.x * p.W;
  if (t0 >= len_b) return;  // whole block past this utterance's end (block-uniform)
  const int ws = t0 - p.halo;
  const int cbase = wave * 64 * NCOL + lane;  // column of pair element (q, e): cbase + 64*(2q+e)

  bool vk[NCOL];
#pragma unroll
  for (int i = 0; i < NCOL; ++i) vk[i] = (unsigned)(ws + cbase + 64 * i) < (unsigned)len_b;
  // zero margins (never rewritten: operand writes cover the window only)
  for (int idx = tid; idx < C * 2 * MARG; idx += NT) {
    const int c = idx / (2 * MARG), m = idx - c * (2 * MARG);
    op[c * RS + (m < MARG ? m : NWIN + m)] = 0.f;
  }

  const float* __restrict__ xb = p.x + (int64_t)b * p.bs;
  // operand <- lrelu(v), zero outside [0, len)
  auto write_operand = [&](const floatx2 (&v)[C][NP]) {
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int q = 0; q < NP; ++q)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const float a = lrelu3(v[c][q][e]);
          op[c * RS + MARG + cbase + 64 * (2 * q + e)] = vk[2 * q + e] ? a : 0.f;
        }
  };

  floatx2 acc[C][NP];
  // acc = bias + W_cv * operand
  auto run_conv = [&](int cv) {
    const int kt = p.kt[cv], d = p.dil[cv];
    cfloat* wc = (cfloat*)(p.w + p.w_off[cv]);
    cfloat* bc = (cfloat*)(p.bias + cv * C);
#pragma unroll
    for (int co = 0; co < C; ++co) {
      const float bv = bc[co];
#pragma unroll
      for (int q = 0; q < NP; ++q) acc[co][q] = floatx2{bv, bv};
    }
    const float* src = op + MARG + cbase - (kt - 1) / 2 * d;
    for (int j = 0; j < kt; ++j, src += d) {
      // channel groups of CG: bounds the scalar weight loads the compiler hoists (SGPRs)
#pragma nounroll
      for (int cg = 0; cg < C; cg += CG) {
        cfloat* wj = wc + (j * C + cg) * C;
        const float* sg = src + cg * RS;
        // the group's operand reads and scalar weight loads first, one wait, then its
        // CG*C*NP packed FMAs (SMEM returns out of order: any use waits lgkmcnt(0))
        floatx2 xv[CG][NP];
        float wv[CG][C];
#pragma unroll
        for (int cc = 0; cc < CG; ++cc) {
#pragma unroll
          for (int q = 0; q < NP; ++q) {
            xv[cc][q][0] = sg[cc * RS + 128 * q];
            xv[cc][q][1] = sg[cc * RS + 128 * q + 64];
          }
#pragma unroll
          for (int co = 0; co < C; ++co) wv[cc][co] = wj[cc * C + co];
        }
#pragma unroll
        for (int cc = 0; cc < CG; ++cc)
#pragma unroll
          for (int co = 0; co < C; ++co) {
            const floatx2 w2{wv[cc][co], wv[cc][co]};
#pragma unroll
            for (int q = 0; q < NP; ++q)
              acc[co][q] = __builtin_elementwise_fma(xv[cc][q], w2, acc[co][q]);
          }
      }
    }
  };

  floatx2 mrf[C][NP];
  for (int r = 0; r < p.n_res; ++r) {
    floatx2 xr[C][NP];
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int q = 0; q < NP; ++q)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int i = 2 * q + e;
          // the 32-bit offset is formed here, not hoisted out of the ResBlock loop (64-bit
          // addresses of every element would stay live: 2 VGPRs each)
          unsigned off = vk[i] ? (unsigned)(c * p.L + ws + cbase + 64 * i) : 0u;
          asm volatile("" : "+v"(off));
          const float v = xb[off];
          xr[c][q][e] = vk[i] ? v : 0.f;
        }
    const int cv0 = p.rb_conv0[r], cv1 = p.rb_conv0[r + 1];
    for (int cv = cv0; cv < cv1; cv += 2) {
      __syncthreads();  // the previous conv's operand reads are done
      write_operand(xr);
      __syncthreads();
      run_conv(cv);
      __syncthreads();
      write_operand(acc);
      __syncthreads();
      run_conv(cv + 1);
#pragma unroll
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int q = 0; q < NP; ++q) xr[c][q] = acc[c][q] + xr[c][q];  // xt + x, :85
    }
    if (r == 0) {
#pragma unroll
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int q = 0; q < NP; ++q) mrf[c][q] = xr[c][q];
    } else {
#pragma unroll
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int q = 0; q < NP; ++q) mrf[c][q] = mrf[c][q] + xr[c][q];
    }
  }

  // y = mrf / n_res on the window centre
  float* __restrict__ yb = p.y + (int64_t)b * p.bs;
  float vmax = 0.f;  // max |stored value| (f16x3 consumers: p.amax_out)
#pragma unroll
  for (int q = 0; q < NP; ++q)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int i = 2 * q + e;
      const int c = cbase + 64 * i;
      if (!(vk[i] && c >= p.halo && c < p.halo + p.W)) continue;
#pragma unroll
      for (int ch = 0; ch < C; ++ch) {
        const float v = mrf[ch][q][e] / p.div;
        yb[(unsigned)(ch * p.L + ws + c)] = v;
        vmax = fmaxf(vmax, fabsf(v));
      }
    }
  if (p.amax_out) amax_commit(vmax, p.amax_out, b);
}

namespace {

typedef void (*ThinFn)(const ThinParams);

struct EntryThin {
  int C, ncol, nt, wpe;
  ThinFn fn;
  char name[48];
};

#define HFGTHIN_ENTRY(C_, NCOL_, NT_, WPE_) \
  { C_, NCOL_, NT_, WPE_, mrf_thin<C_, NCOL_, NT_, WPE_>, {0} }

EntryThin g_entriesThin[] = {HFGTHIN_ENTRY(16, 2, 256, 3), HFGTHIN_ENTRY(8, 4, 256, 3),
                             HFGTHIN_ENTRY(4, 8, 256, 3)};

EntryThin* find_thin(int C) {
  for (auto& e : g_entriesThin)
    if (e.C == C) return &e;
  return nullptr;
}

}  // namespace

int thin_window(int C) {
  EntryThin* e = find_thin(C);
  return e ? e->nt * e->ncol : 0;
}

size_t thin_lds_bytes(int C) {
  EntryThin* e = find_thin(C);
  return e ? sizeof(float) * (size_t)C * (e->nt * e->ncol + 2 * kThinMarg) : 0;
}

hipError_t launch_mrf_thin(int C, const ThinParams& p, int batch, hipStream_t stream,
                           const char** name) {
  EntryThin* e = find_thin(C);
  if (!e) return hipErrorInvalidValue;
  const int nwin = e->nt * e->ncol;
  if (p.n_res < 1 || p.n_res > kThinMaxRes) return hipErrorInvalidValue;
  if (p.W <= 0 || p.halo < 0 || p.W + 2 * p.halo > nwin) return hipErrorInvalidValue;
  if (p.rb_conv0[0] < 0 || p.rb_conv0[p.n_res] > kThinMaxConv) return hipErrorInvalidValue;
  for (int r = 0; r < p.n_res; ++r) {
    const int a = p.rb_conv0[r], z = p.rb_conv0[r + 1];
    if (z <= a || ((z - a) & 1)) return hipErrorInvalidValue;
    for (int cv = a; cv < z; ++cv)
      if (p.kt[cv] < 1 || p.dil[cv] < 1 || (p.kt[cv] - 1) / 2 * p.dil[cv] > kThinMarg)
        return hipErrorInvalidValue;
  }
  const size_t lds = thin_lds_bytes(C);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (hipError_t err = ensure_max_lds(reinterpret_cast<const void*>(e->fn)))
    return err;
  {
    std::lock_guard<std::mutex> lk(setup_mutex());
    if (!e->name[0]) snprintf(e->name, sizeof(e->name), "mrf_thin<%d, %d, %d, %d>", e->C, e->ncol, e->nt,
                               e->wpe);
  }
  if (name) *name = e->name;
  const int n_tiles = (p.L + p.W - 1) / p.W;
  e->fn<<<dim3(n_tiles, batch), dim3(e->nt), lds, stream>>>(p);
  return hipGetLastError();
}

}  // namespace hfg

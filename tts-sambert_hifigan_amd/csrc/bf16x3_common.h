// bf16x3_common.h — pieces shared by the split-precision conv kernels
// (conv_bf16x3.hip: one Conv1d / polyphase ConvTranspose1d per launch;
//  resblock_bf16x3.hip: a whole ResBlock, all dilations, per launch;
//  ups_bf16x3.hip, mrf_thin_mfma.hip).
//
// Split formats (template parameter FMT of every split kernel):
//   kFmtBf16 (bf16x3): hi = bf16(v), lo = bf16(v - hi); hi*hi + hi*lo + lo*hi in fp32 on the
//     bf16 matrix cores: ~16-bit-mantissa products.
//   kFmtF16 (f16x3): the same three products of f16 halves of a power-of-two SCALED operand:
//     hi = f16(v * 2^e), lo = f16(v * 2^e - hi) carry 22 significant bits, so a product misses
//     the exact one by <= ~3 * 2^-22 relative — fp32-class (an fp32 product rounds at 2^-24,
//     and the fp32 accumulation both modes share adds more than the split does).  f16 has 5
//     exponent bits, so every operand is scaled by a power of two into [2^14, 2^15) of its
//     tensor's (activations) or layer's (weights) largest magnitude; the scales are exact, the
//     accumulator is multiplied by 2^-(e_x + e_w) after the main loop, and a value the scaling
//     leaves below the f16 normal range (< 2^-17 of that largest magnitude) keeps an absolute
//     error <= 2^-39 of it.  The f16 MFMAs run at the bf16 rate (MI355X_MICROARCH.md).
//   Activation scales come from the producing launch: its epilogue folds max|stored value| of
//   each batch item into a per-(launch, item) slot (amax_commit); the consuming launch reads
//   the slot of its input (per item: a batch item's result does not depend on the others).  A
//   whole-ResBlock / whole-MRF kernel scales the operands it forms internally per block
//   (block_amax).
#pragma once

#include <hip/hip_runtime.h>

#include "epilogue.h"
#include "kernels.h"

namespace hfg {

typedef floatx16e floatx16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void* lds_ptr_t3;
typedef __attribute__((address_space(1))) void* gptr_t1;


typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));
typedef _Float16 halfx4_ __attribute__((ext_vector_type(4)));
typedef _Float16 halfx2_ __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_ __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x4_ __attribute__((ext_vector_type(4)));
typedef float floatx2_ __attribute__((ext_vector_type(2)));
typedef float floatx4_ __attribute__((ext_vector_type(4)));

// Fragments are carried as bf16x8 bit patterns in both formats (16 bytes); the MFMA
// wrappers reinterpret them for the f16 instructions.
template <int FMT>
__device__ __forceinline__ floatx16 mfma32(const bf16x8& a, const bf16x8& b, const floatx16& c) {
  if constexpr (FMT == kFmtBf16)
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(halfx8, a),
                                                  __builtin_bit_cast(halfx8, b), c, 0, 0, 0);
}
template <int FMT>
__device__ __forceinline__ floatx4_ mfma16(const bf16x8& a, const bf16x8& b, const floatx4_& c) {
  if constexpr (FMT == kFmtBf16)
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(halfx8, a),
                                                  __builtin_bit_cast(halfx8, b), c, 0, 0, 0);
}

// hi = fmt(a), lo = fmt(a - hi) of two values (a - hi is exact in fp32), as bit patterns.
// HFG_SPLIT_SCALAR: the residuals as two scalar subtractions (no v_pk_add_f32, which costs
// ~20 extra cycles per instruction beside MFMAs, MI355X_MICROARCH.md)
#ifndef HFG_SPLIT_SCALAR
#define HFG_SPLIT_SCALAR 1
#endif
// HFG_SPLIT_MIX (f16): the residual a - f32(hi) as one v_fma_mix_f32 per value (hi read as
// f16 straight from the packed pair) instead of a conversion back plus a subtraction
#ifndef HFG_SPLIT_MIX
#define HFG_SPLIT_MIX 1
#endif
template <int FMT>
__device__ __forceinline__ void split2(const floatx2_& a, bf16x2_& hi, bf16x2_& lo) {
  if constexpr (HFG_SPLIT_MIX && FMT == kFmtF16) {
    const halfx2_ h = __builtin_convertvector(a, halfx2_);
    const unsigned hb = __builtin_bit_cast(unsigned, h);
    float l0, l1;
    asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(l0) : "v"(hb), "v"(a[0]));
    asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
        : "=v"(l1) : "v"(hb), "v"(a[1]));
    floatx2_ l;
    l[0] = l0;
    l[1] = l1;
    hi = __builtin_bit_cast(bf16x2_, h);
    lo = __builtin_bit_cast(bf16x2_, __builtin_convertvector(l, halfx2_));
  } else if constexpr (HFG_SPLIT_SCALAR && FMT == kFmtF16) {
    const halfx2_ h = __builtin_convertvector(a, halfx2_);
    floatx2_ l;
    l[0] = a[0] - (float)h[0];
    l[1] = a[1] - (float)h[1];
    hi = __builtin_bit_cast(bf16x2_, h);
    lo = __builtin_bit_cast(bf16x2_, __builtin_convertvector(l, halfx2_));
  } else if constexpr (HFG_SPLIT_SCALAR) {
    hi = __builtin_convertvector(a, bf16x2_);
    floatx2_ l;
    l[0] = a[0] - (float)hi[0];
    l[1] = a[1] - (float)hi[1];
    lo = __builtin_convertvector(l, bf16x2_);
  } else if constexpr (FMT == kFmtBf16) {
    hi = __builtin_convertvector(a, bf16x2_);
    const floatx2_ hf = __builtin_convertvector(hi, floatx2_);
    lo = __builtin_convertvector(a - hf, bf16x2_);
  } else {
    const halfx2_ h = __builtin_convertvector(a, halfx2_);
    const floatx2_ hf = __builtin_convertvector(h, floatx2_);
    const halfx2_ l = __builtin_convertvector(a - hf, halfx2_);
    hi = __builtin_bit_cast(bf16x2_, h);
    lo = __builtin_bit_cast(bf16x2_, l);
  }
}

// f16x3 scale exponent e for values with |v| <= m: m * 2^e in [2^14, 2^15) (max f16 65504),
// clamped to +-kX3ExpMax so 2^-(e_x + e_w) stays a normal float; 0 for m = 0 / inf / NaN
__device__ __forceinline__ int x3_exp(float m) {
  if (!(m > 0.f) || !(m <= 3.0e38f)) return 0;
  const int e = 15 - __builtin_amdgcn_frexp_expf(m);  // m = f 2^x, f in [0.5, 1)
  return e < -kX3ExpMax ? -kX3ExpMax : (e > kX3ExpMax ? kX3ExpMax : e);
}
// 2^e as a float, |e| <= 126
__device__ __forceinline__ float exp2i(int e) { return __builtin_bit_cast(float, (unsigned)(127 + e) << 23); }
// scale exponent of item b's producer slot (slots null: no scaling): the max of its
// kAmaxSpread words (amax_commit), all uniform loads
__device__ __forceinline__ int x3_exp_slot(const uint32_t* slots, int b) {
  if (!slots) return 0;
  const uint32_t* s = slots + (size_t)b * kAmaxSlotWords;
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < kAmaxSpread; ++i) m = max(m, s[i * kAmaxLineWords]);
  return x3_exp(__builtin_bit_cast(float, m));
}


// leaky_relu(v, 0.1) as max(v, 0.1 v): bitwise the reference's select (slope < 1), two
// VALU ops (v_mul + v_max) instead of compare + multiply + select
__device__ __forceinline__ float lrelu3(float v) { return fmaxf(v, v * kLReluSlope); }

// x / d, bitwise the IEEE quotient, in 5 VALU ops instead of the ~10 of a full division:
// q0 = x r, e = fma(-q0, d, x), q = fma(e, r, q0) with r = fp32(1/d) is correctly rounded for
// every finite x except -0 when d is one of the divisors fast_div_ok() accepts (checked over
// all 2^32 inputs: tests/tools/verify_fast_div.c); q0 is kept where it is +-0 or +-inf.
// Callers branch on rcp != 0 (uniform) outside their loops and divide plainly otherwise.
__device__ __forceinline__ float div_fast(float x, float d, float rcp) {
  const float q0 = x * rcp;
  const float e = __builtin_fmaf(-q0, d, x);
  const float q = __builtin_fmaf(e, rcp, q0);
  // v_cmp_class_f32: +-0 (0x60) | +-inf (0x204)
  return __builtin_amdgcn_classf(q0, 0x264) ? q0 : q;
}

// HFG_PRIO (round 6): a wave raises its issue priority for its matrix phase (s_setprio 1) and
// drops it for staging / epilogue work, so a co-resident wave of ANOTHER block (2 blocks per CU)
// that is in its MFMA loop wins the SIMD's issue arbitration over this wave's VALU burst
// (MI355X_MICROARCH.md "Two waves per SIMD", items 2 and 4)
#ifndef HFG_PRIO
#define HFG_PRIO 1
#endif
__device__ __forceinline__ void prio_mfma() {
  if constexpr (HFG_PRIO) __builtin_amdgcn_s_setprio(1);
}
__device__ __forceinline__ void prio_other() {
  if constexpr (HFG_PRIO) __builtin_amdgcn_s_setprio(0);
}

// s_waitcnt vmcnt(N) with a compile-time N
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// workgroup barrier over LDS writes made by ds_write (lgkmcnt): the caller has already
// waited (vmcnt) for the LDS-DMA pieces the next chunk reads.  Written as one asm block
// so no fence makes the compiler wait for every outstanding global load / LDS-DMA
// piece, and the "memory" clobber keeps LDS accesses on their side of the barrier.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

}  // namespace hfg

// bf16x3_common.h — pieces shared by the split-precision conv kernels
// (conv_bf16x3.hip: one Conv1d / polyphase ConvTranspose1d per launch;
//  resblock_bf16x3.hip: a whole ResBlock, all dilations, per launch).
#pragma once

#include <hip/hip_runtime.h>

#include "epilogue.h"
#include "kernels.h"

namespace hfg {

typedef floatx16e floatx16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void* lds_ptr_t3;
typedef __attribute__((address_space(1))) void* gptr_t1;

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

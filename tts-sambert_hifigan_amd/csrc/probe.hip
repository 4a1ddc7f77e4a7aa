// probe.hip — sustained matrix-core rate of this GPU under load (hfg_probe_mfma_rate).
//
// The roofline "peak" of the bench line is the datasheet dense rate (2.5 PFLOP/s bf16,
// 157.3 TFLOP/s fp32 at 2.4 GHz).  Under a full-chip MFMA load the clock drops with
// power (DVFS), and how far depends on how much the operand bits toggle: a matrix
// kernel cannot exceed what a pure MFMA stream sustains on the same box at the same
// moment.  This kernel is that stream: every wave of 2 blocks x 4 waves per CU issues
// independent MFMAs back to back (4 accumulator chains, no memory traffic in the loop)
// on random operands that change every instruction, and wave 0 of block 0 reads the
// shader clock (s_memtime) against the 100 MHz real-time counter so the effective
// clock comes back too.  Measurement only; no product path calls it.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <new>

#include "../../include/hifigan_hip_inspect.h"

namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));

constexpr int kOps = 8;  // distinct operand registers cycled through

// kind 0: v_mfma_f32_32x32x16_bf16 (32768 flop); kind 1: v_mfma_f32_32x32x2_f32 (4096 flop);
// kind 2 (KIND 2 here): v_mfma_f32_32x32x16_f16 on operands with random 10-bit mantissas (the
// f16x3 kernels' instruction: its multiplier switches more bits per product than bf16's).
// CHAINS independent accumulators per wave (1: every MFMA accumulates onto the previous
// one's result, the order of the split-product triples in the conv kernels)
template <int KIND, int CHAINS>
__global__ void __launch_bounds__(256, 2) mfma_stream(const uint32_t* __restrict__ rnd, int iters,
                                                      float* __restrict__ sink,
                                                      uint64_t* __restrict__ clk) {
  const int lane = threadIdx.x & 63;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t t0 = 0, r0 = 0;
  const bool timer = blockIdx.x == 0 && threadIdx.x < 64;
  if (timer) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  floatx16 acc[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; ++c)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
  if constexpr (KIND == 0 || KIND == 2) {
    bf16x8 a[kOps], b[kOps];
#pragma unroll
    for (int i = 0; i < kOps; ++i) {
      uint32_t w[4], v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        // bf16 pairs with exponents kept in [2^-8, 2^8) so the chains never overflow
        // (f16: the same bits are sign + 10 random mantissa bits, exponent 2^0)
        w[e] = (rnd[(gid * 64 + i * 8 + e) & 0xFFFFF] & 0x83FF83FFu) | 0x3C003C00u;
        v[e] = (rnd[(gid * 64 + i * 8 + 4 + e) & 0xFFFFF] & 0x83FF83FFu) | 0x3C003C00u;
      }
      a[i] = *reinterpret_cast<bf16x8*>(w);
      b[i] = *reinterpret_cast<bf16x8*>(v);
    }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < kOps; ++i)
#pragma unroll
        for (int c = 0; c < CHAINS; ++c)
          if constexpr (KIND == 0)
            acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[(i + c + 1) % kOps], acc[c], 0, 0, 0);
          else
            acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(
                __builtin_bit_cast(halfx8, a[i]), __builtin_bit_cast(halfx8, b[(i + c + 1) % kOps]),
                acc[c], 0, 0, 0);
    }
  } else {
    float a[kOps], b[kOps];
#pragma unroll
    for (int i = 0; i < kOps; ++i) {
      a[i] = __uint_as_float((rnd[(gid * 16 + i) & 0xFFFFF] & 0x807FFFFFu) | 0x3F000000u);
      b[i] = __uint_as_float((rnd[(gid * 16 + 8 + i) & 0xFFFFF] & 0x807FFFFFu) | 0x3F000000u);
    }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < kOps; ++i)
#pragma unroll
        for (int c = 0; c < CHAINS; ++c)
          acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[(i + c + 1) % kOps], acc[c], 0, 0, 0);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c)
#pragma unroll
    for (int r = 0; r < 16; ++r) s += acc[c][r];
  if (s == 1.2345e-30f) sink[gid] = s;  // keeps the chains live; never true in practice
  if (timer && lane == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - t0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

}  // namespace

extern "C" int hfg_probe_mfma_rate(int device, int kind, int iters, double* tflops, double* mhz) {
  // kind 0 bf16, 1 fp32, 2 bf16 one chain, 3 fp32 one chain, 4 f16, 5 f16 one chain
  if (kind < 0 || kind > 5 || iters <= 0 || !tflops || !mhz) return HFG_EINVAL;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return HFG_ENODEV;
  int prev = 0;
  (void)hipGetDevice(&prev);
  if (hipSetDevice(device) != hipSuccess) return HFG_ENODEV;
  int rc = HFG_OK;
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
  const int blocks = 2 * (cus > 0 ? cus : 256);  // 2 blocks x 4 waves per CU = 2 waves per SIMD
  const size_t n_rnd = 1u << 20;
  uint32_t* rnd = nullptr;
  float* sink = nullptr;
  uint64_t* clk = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  hipStream_t st = nullptr;
  float ms = 0.f;
  uint64_t clk_h[2] = {0, 0};
  if (hipMalloc(&rnd, n_rnd * 4) != hipSuccess || hipMalloc(&sink, (size_t)blocks * 256 * 4) != hipSuccess ||
      hipMalloc(&clk, 16) != hipSuccess || hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) {
    rc = HFG_ENOMEM;
    goto done;
  }
  {
    // host LCG fill: the same operands on every call
    uint32_t* h = new (std::nothrow) uint32_t[n_rnd];
    if (!h) {
      rc = HFG_ENOMEM;
      goto done;
    }
    uint32_t x = 0x12345678u;
    for (size_t i = 0; i < n_rnd; ++i) h[i] = (x = x * 1664525u + 1013904223u);
    hipError_t e = hipMemcpy(rnd, h, n_rnd * 4, hipMemcpyHostToDevice);
    delete[] h;
    if (e != hipSuccess) {
      rc = HFG_EIO;
      goto done;
    }
  }
  {
    auto launch = [&](int it) {
      if (kind == 0) mfma_stream<0, 4><<<blocks, 256, 0, st>>>(rnd, it, sink, clk);
      else if (kind == 1) mfma_stream<1, 4><<<blocks, 256, 0, st>>>(rnd, it, sink, clk);
      else if (kind == 2) mfma_stream<0, 1><<<blocks, 256, 0, st>>>(rnd, it, sink, clk);
      else if (kind == 3) mfma_stream<1, 1><<<blocks, 256, 0, st>>>(rnd, it, sink, clk);
      else if (kind == 4) mfma_stream<2, 4><<<blocks, 256, 0, st>>>(rnd, it, sink, clk);
      else mfma_stream<2, 1><<<blocks, 256, 0, st>>>(rnd, it, sink, clk);
    };
    launch(iters / 4 > 0 ? iters / 4 : 1);  // warm the clocks up
    (void)hipEventRecord(e0, st);
    launch(iters);
    (void)hipEventRecord(e1, st);
    if (hipStreamSynchronize(st) != hipSuccess || hipGetLastError() != hipSuccess) {
      rc = HFG_EIO;
      goto done;
    }
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (hipMemcpy(clk_h, clk, 16, hipMemcpyDeviceToHost) != hipSuccess) {
      rc = HFG_EIO;
      goto done;
    }
    const bool f32 = kind == 1 || kind == 3;
    const double flop_per = f32 ? 4096.0 : 32768.0;
    const int chains = (kind == 0 || kind == 1 || kind == 4) ? 4 : 1;
    const double flop = flop_per * kOps * chains * (double)iters * blocks * 4;
    *tflops = ms > 0.f ? flop / (ms * 1e-3) / 1e12 : 0.0;
    *mhz = clk_h[1] ? (double)clk_h[0] / ((double)clk_h[1] / 100.0) : 0.0;  // realtime: 100 MHz
  }
done:
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (st) (void)hipStreamDestroy(st);
  if (rnd) (void)hipFree(rnd);
  if (sink) (void)hipFree(sink);
  if (clk) (void)hipFree(clk);
  (void)hipSetDevice(prev);
  return rc;
}

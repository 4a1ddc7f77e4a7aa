// FETCH_SIZE / WRITE_SIZE calibration for the access widths the HiFi-GAN kernels use
// (MI355X_MICROARCH.md §HBM: "other access widths are uncalibrated: calibrate on a known
// byte count in your own access pattern").  Each kernel streams a known number of bytes
// once, coalesced, through a 1 GiB buffer (4x the 256 MiB Infinity Cache, so nothing is
// served on-die):
//   rd4   4 B per lane  (global_load_dword:   the bf16x3 input-window staging, conv_post)
//   rd16 16 B per lane  (global_load_dwordx4: the bf16x3 epilogue residual / MRF reads)
//   wr4   4 B per lane  (global_store_dword:  the conv epilogue stores)
//   wr16 16 B per lane  (global_store_dwordx4: the upsampler float4 stores)
// profiles/pmc_calib.sh runs it under two rocprofv3 --pmc passes and prints
// counter KiB / known bytes per kernel.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void rd4(const float* __restrict__ x, size_t n, float* __restrict__ sink) {
  float acc = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    acc += x[i];
  if (acc == 12345.678f) sink[threadIdx.x] = acc;  // keeps the loads, never stores
}

__global__ void rd16(const float4* __restrict__ x, size_t n4, float* __restrict__ sink) {
  float acc = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4;
       i += (size_t)gridDim.x * blockDim.x) {
    float4 v = x[i];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 12345.678f) sink[threadIdx.x] = acc;
}

__global__ void wr4(float* __restrict__ y, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    y[i] = (float)(i & 7);
}

__global__ void wr16(float4* __restrict__ y, size_t n4) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4;
       i += (size_t)gridDim.x * blockDim.x)
    y[i] = make_float4(1.f, 2.f, 3.f, (float)(i & 7));
}

#define CK(e) do { hipError_t r_ = (e); if (r_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(r_)); return 1; } } while (0)

int main() {
  const size_t bytes = (size_t)1 << 30;
  const size_t n = bytes / 4;
  float *x = nullptr, *y = nullptr, *sink = nullptr;
  CK(hipMalloc(&x, bytes));
  CK(hipMalloc(&y, bytes));
  CK(hipMalloc(&sink, 4096));
  CK(hipMemset(x, 0, bytes));
  CK(hipDeviceSynchronize());
  const int grid = 256 * 8, block = 256;
  for (int rep = 0; rep < 2; ++rep) {
    rd4<<<grid, block>>>(x, n, sink);
    rd16<<<grid, block>>>(reinterpret_cast<const float4*>(x), n / 4, sink);
    wr4<<<grid, block>>>(y, n);
    wr16<<<grid, block>>>(reinterpret_cast<float4*>(y), n / 4);
  }
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  printf("known bytes per launch: %zu\n", bytes);
  CK(hipFree(x));
  CK(hipFree(y));
  CK(hipFree(sink));
  return 0;
}

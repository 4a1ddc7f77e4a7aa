// Cost of the f16x3 scale-slot atomics (epilogue.h amax_commit) when a whole grid commits at
// once: G blocks x 256 threads each fold one value into an item's 64-word slot, one atomicMax
// per wave (as the kernels do) or one per block (LDS max first).  Round-6 measurement tool.
// build: hipcc --offload-arch=gfx950 -O3 -I tts-sambert_hifigan_amd/csrc tests/tools/atomic_probe.hip -o /tmp/atomic_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include "epilogue.h"

__global__ void __launch_bounds__(256) per_wave(uint32_t* slots, float seed) {
  const float m = seed * (float)(blockIdx.x * 256 + threadIdx.x);
  hfg::amax_commit(m, slots, 0);
}
__global__ void __launch_bounds__(256) per_block(uint32_t* slots, float seed) {
  float m = seed * (float)(blockIdx.x * 256 + threadIdx.x);
  __shared__ float wm[4];
  m = hfg::wave_max(m);
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x < 64) hfg::amax_commit(threadIdx.x < 4 ? wm[threadIdx.x] : 0.f, slots, 0);
}
// the 64 words of the slot STRIDE words apart (distinct lines / channels), one atomic per wave
__global__ void __launch_bounds__(256) per_wave_spread(uint32_t* slots, float seed, int stride) {
  float m = seed * (float)(blockIdx.x * 256 + threadIdx.x);
  m = hfg::wave_max(m);
  const unsigned w = blockIdx.x * 4 + (threadIdx.x >> 6);
  if ((threadIdx.x & 63) == 0) atomicMax(slots + (size_t)(w & 63) * stride, __builtin_bit_cast(uint32_t, m));
}
__global__ void __launch_bounds__(256) none(uint32_t* slots, float seed) {
  const float m = seed * (float)(blockIdx.x * 256 + threadIdx.x);
  if (m == 1.2345e-30f) slots[0] = 1;
}

int main() {
  uint32_t* slots;
  hipMalloc(&slots, 64 * 4096 * 4);
  hipMemset(slots, 0, 64 * 4096 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int grids[] = {128, 512, 1024, 2048, 4096};
  for (int g : grids) {
    float t[3];
    for (int v = 0; v < 3; ++v) {
      auto run = [&]() {
        if (v == 0) none<<<g, 256>>>(slots, 1e-3f);
        if (v == 1) per_wave<<<g, 256>>>(slots, 1e-3f);
        if (v == 2) per_block<<<g, 256>>>(slots, 1e-3f);
      };
      for (int i = 0; i < 5; ++i) run();
      hipEventRecord(a);
      for (int i = 0; i < 50; ++i) run();
      hipEventRecord(b);
      hipEventSynchronize(b);
      hipEventElapsedTime(&t[v], a, b);
      t[v] *= 1000.f / 50;
    }
    printf("blocks %5d (%6d waves): no atomics %6.2f us, per wave %6.2f us, per block %6.2f us", g,
           g * 4, t[0], t[1], t[2]);
    for (int stride : {32, 64, 1024, 4096}) {
      for (int i = 0; i < 5; ++i) per_wave_spread<<<g, 256>>>(slots, 1e-3f, stride);
      hipEventRecord(a);
      for (int i = 0; i < 50; ++i) per_wave_spread<<<g, 256>>>(slots, 1e-3f, stride);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ts;
      hipEventElapsedTime(&ts, a, b);
      printf(", stride %d: %6.2f", stride, ts * 1000.f / 50);
    }
    printf("\n");
  }
  hipFree(slots);
  return 0;
}

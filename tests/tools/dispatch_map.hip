// Which CU runs which block (diagnostic, round 5): a grid of NB blocks x 256 threads with
// LDS_KB of dynamic LDS each records (HW_ID, XCC_ID, start / end real-time) per block, so the
// block -> (XCC, SE, CU) placement and the co-residency of the first round can be read.
// build: hipcc --offload-arch=gfx950 -O2 tests/tools/dispatch_map.hip -o tests/tools/dispatch_map
// run:   ./dispatch_map NB LDS_KB SPIN_US > map.csv
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void probe(unsigned* out, int spin_us) {
  extern __shared__ char lds[];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    lds[0] = 1;
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
    while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)spin_us * 100ull)
      __builtin_amdgcn_s_sleep(2);
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    unsigned* o = out + 6 * blockIdx.x;
    o[0] = hw;
    o[1] = xcc;
    o[2] = (unsigned)t0;
    o[3] = (unsigned)(t0 >> 32);
    o[4] = (unsigned)t1;
    o[5] = (unsigned)(t1 >> 32);
  }
}

int main(int argc, char** argv) {
  const int nb = argc > 1 ? atoi(argv[1]) : 2048;
  const int lds_kb = argc > 2 ? atoi(argv[2]) : 64;
  const int spin = argc > 3 ? atoi(argv[3]) : 50;
  unsigned* d;
  if (hipMalloc(&d, sizeof(unsigned) * 6 * nb) != hipSuccess) return 1;
  hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  for (int it = 0; it < 2; ++it) probe<<<nb, 256, lds_kb * 1024>>>(d, spin);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  std::vector<unsigned> h(6 * nb);
  hipMemcpy(h.data(), d, sizeof(unsigned) * 6 * nb, hipMemcpyDeviceToHost);
  printf("block,hw_id,xcc_id,t0,t1\n");
  for (int b = 0; b < nb; ++b) {
    const unsigned long long t0 = h[6 * b + 2] | ((unsigned long long)h[6 * b + 3] << 32);
    const unsigned long long t1 = h[6 * b + 4] | ((unsigned long long)h[6 * b + 5] << 32);
    printf("%d,%u,%u,%llu,%llu\n", b, h[6 * b], h[6 * b + 1], t0, t1);
  }
  hipFree(d);
  return 0;
}

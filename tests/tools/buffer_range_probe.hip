// Diagnostic (GPU box): which raw-buffer loads does the gfx950 range check drop?  A buffer of
// 64 floats (value i+1 at index i) read through a descriptor of num_records = 64*4 - 4 bytes
// (the last dword past the range) with the offset split between voffset and soffset.
// Prints the value each probe returns (0 = dropped).  Build: hipcc --offload-arch=gfx950 -O2
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void probe(const float* buf, float* out) {
  if (threadIdx.x != 0) return;
  const int nrec = 64 * 4 - 4;
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)buf, 0, nrec, 0x00020000);
  // dword at byte 248 (last in range) and 252 (first out): all in voffset / all in soffset
  out[0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, 248, 0, 0));
  out[1] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, 252, 0, 0));
  out[2] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, 0, 248, 0));
  out[3] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, 0, 252, 0));
  out[4] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, 4, 248, 0));
  // dwordx4 ending at 256 (last dword out) / ending at 252 (all in)
  f4 a = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, 240, 0, 0));
  f4 b = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, 236, 0, 0));
  f4 c = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, 0, 240, 0));
  for (int i = 0; i < 4; ++i) { out[5 + i] = a[i]; out[9 + i] = b[i]; out[13 + i] = c[i]; }
}
int main() {
  float h[64], o[17];
  for (int i = 0; i < 64; ++i) h[i] = (float)(i + 1);
  float *d, *dout;
  hipMalloc(&d, 4096); hipMalloc(&dout, 17 * 4);
  hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
  probe<<<1, 64>>>(d, dout);
  hipMemcpy(o, dout, sizeof(o), hipMemcpyDeviceToHost);
  printf("b32 voff 248 -> %g (exp 63)\nb32 voff 252 -> %g (exp 64 or 0)\n", o[0], o[1]);
  printf("b32 soff 248 -> %g\nb32 soff 252 -> %g\nb32 voff 4 + soff 248 -> %g\n", o[2], o[3], o[4]);
  printf("b128 voff 240 -> %g %g %g %g\n", o[5], o[6], o[7], o[8]);
  printf("b128 voff 236 -> %g %g %g %g\n", o[9], o[10], o[11], o[12]);
  printf("b128 soff 240 -> %g %g %g %g\n", o[13], o[14], o[15], o[16]);
  return 0;
}

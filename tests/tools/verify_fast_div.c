/* Exhaustive check of the division used by the MRF-mean epilogues (div_fast,
 * tts-sambert_hifigan_amd/csrc/bf16x3_common.h): for a divisor d,
 *   q0 = x * r, e = fma(-q0, d, x), q = fma(e, r, q0), r = fp32(1/d),
 * with q0 kept where it is +-0 or +-inf, must equal the IEEE quotient x / d for every fp32 x
 * (NaN inputs excepted: both give a NaN).  usage: verify_fast_div d [step]; step > 1 samples
 * every step-th bit pattern (the CPU test does that; the full run is in the header of
 * kernels.h fast_div_ok).  Prints the mismatch count; exit code 1 if any.
 * Test infrastructure only. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int main(int argc, char** argv) {
  const float d = (float)atof(argv[1]);
  const uint64_t step = argc > 2 ? strtoull(argv[2], 0, 10) : 1;
  const float r = 1.0f / d;
  uint64_t bad = 0, n = 0;
  for (uint64_t u = 0; u < (1ull << 32); u += step) {
    uint32_t b = (uint32_t)u;
    float x;
    memcpy(&x, &b, 4);
    if (isnan(x)) continue;
    const float ref = x / d;
    const float q0 = x * r;
    const float e = fmaf(-q0, d, x);
    float q = fmaf(e, r, q0);
    if (q0 == 0.0f || isinf(q0)) q = q0;
    uint32_t a, c;
    memcpy(&a, &ref, 4);
    memcpy(&c, &q, 4);
    bad += a != c;
    ++n;
  }
  printf("d=%g checked=%llu mismatches=%llu\n", d, (unsigned long long)n, (unsigned long long)bad);
  return bad != 0;
}

// mel_kernels.hip — on-device log-mel framing feeding the vocoder
// (data/audio_processing.py:98-133: torchaudio MelSpectrogram(power=2,
// center=True, reflect pad, periodic Hann) -> log10(mel + 1e-10)).
//
// stft_power_mfma: the windowed DFT of every frame as a GEMM on the fp32 matrix
//   cores: rows = 32 frames of one utterance (staged from a reflect-padded
//   signal tile in LDS), columns = frequency bins, K = n_fft samples.  The
//   twiddle tables (window folded in: w[n]cos(2 pi k n/N), w[n]sin(...)) are
//   precomputed on the host and stay L2-resident; each lane ends with Re and Im
//   of the same (frame, bin) in two accumulators and writes |X|^2.
// mel_log: mel[m][f] = log10(sum_k fb[k][m] * P[f][k] + eps), written as
//   [B][n_mels][frames], the vocoder's input layout.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "mel_kernels.h"

namespace hfg {

typedef float floatx16m __attribute__((ext_vector_type(16)));

// one block: 32 frames x all bins of one utterance; 4 waves split the bin tiles
__global__ void __launch_bounds__(256)
stft_power_mfma(const float* __restrict__ wav, int64_t N, int n_fft, int hop, int n_bins,
                int n_frames, const float* __restrict__ tcos, const float* __restrict__ tsin,
                int bins_pad, float* __restrict__ power) {
  extern __shared__ __attribute__((aligned(16))) float sig[];
  constexpr int FT = 32;
  const int b = blockIdx.y;
  const int f0 = blockIdx.x * FT;
  const int half_fft = n_fft / 2;
  const float* x = wav + (int64_t)b * N;
  // reflect-padded samples [f0*hop - n_fft/2, (f0+FT-1)*hop + n_fft/2)
  // stored skewed: sample s at s + s/hop, so the 32 frames a half-wave reads at
  // one k (addresses frame*hop + k) fall in 32 different LDS banks
  const int span = (FT - 1) * hop + n_fft;
  for (int i = threadIdx.x; i < span; i += blockDim.x) {
    int64_t g = (int64_t)f0 * hop - half_fft + i;
    if (g < 0) g = -g;                       // torch reflect: x[-i] = x[i]
    if (g >= N) g = 2 * (N - 1) - g;         // x[N-1+i] = x[N-1-i]
    float v = 0.f;
    if (g >= 0 && g < N) v = x[g];
    sig[i + i / hop] = v;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int half = lane >> 5, col = lane & 31;
  const int n_btiles = bins_pad / 32;
  for (int bt = wave; bt < n_btiles; bt += 4) {
    floatx16m re, im;
    for (int r = 0; r < 16; ++r) {
      re[r] = 0.f;
      im[r] = 0.f;
    }
    const int bin = bt * 32 + col;
    // A[i = frame][k = n] = sig[frame*hop + n]; B[k = n][j = bin] = table[n][bin]
    const int abase = col * hop + half;  // lane's frame = col (A layout: i = lane & 31)
    const float* cb = tcos + (int64_t)half * bins_pad + bin;
    const float* sb = tsin + (int64_t)half * bins_pad + bin;
#pragma unroll 4
    for (int k = 0; k < n_fft; k += 2) {
      const int s_ = abase + k;
      const float a = sig[s_ + s_ / hop];
      const float bc = cb[(int64_t)k * bins_pad];
      const float bs = sb[(int64_t)k * bins_pad];
      re = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bc, re, 0, 0, 0);
      im = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bs, im, 0, 0, 0);
    }
    if (bin < n_bins) {
      for (int r = 0; r < 16; ++r) {
        const int fr = f0 + (r & 3) + 8 * (r >> 2) + 4 * half;
        if (fr < n_frames)
          power[((int64_t)b * n_frames + fr) * n_bins + bin] = re[r] * re[r] + im[r] * im[r];
      }
    }
  }
}

// block: 16 frames of one utterance; power rows staged in LDS; thread = (frame, mel)
__global__ void __launch_bounds__(256)
mel_log(const float* __restrict__ power, int n_frames, int n_bins, const float* __restrict__ fb,
        int n_mels, float eps, int log_mode, float ln_base, float* __restrict__ mel) {
  extern __shared__ __attribute__((aligned(16))) float pw[];
  constexpr int FT = 16;
  const int b = blockIdx.y;
  const int f0 = blockIdx.x * FT;
  const int nf = min(FT, n_frames - f0);
  const float* src = power + ((int64_t)b * n_frames + f0) * n_bins;
  for (int i = threadIdx.x; i < nf * n_bins; i += blockDim.x) pw[i] = src[i];
  __syncthreads();
  for (int o = threadIdx.x; o < nf * n_mels; o += blockDim.x) {
    const int f = o / n_mels, m = o - f * n_mels;
    const float* p = pw + f * n_bins;
    float acc = 0.f;
    for (int k = 0; k < n_bins; ++k) acc = fmaf(fb[(int64_t)k * n_mels + m], p[k], acc);
    const float v = acc + eps;
    mel[((int64_t)b * n_mels + m) * n_frames + f0 + f] =
        log_mode == 1 ? log10f(v) : (log_mode == 0 ? logf(v) : logf(v) / ln_base);
  }
}

hipError_t launch_stft_power(const float* wav, int64_t B, int64_t N, int n_fft, int hop,
                             int n_bins, int n_frames, const float* tcos, const float* tsin,
                             int bins_pad, float* power, hipStream_t stream) {
  const size_t span = (size_t)31 * hop + n_fft;
  const size_t lds = sizeof(float) * (span + span / hop + 1);
  if (lds > 64 * 1024) return hipErrorInvalidValue;
  dim3 grid((n_frames + 31) / 32, (unsigned)B);
  stft_power_mfma<<<grid, dim3(256), lds, stream>>>(wav, N, n_fft, hop, n_bins, n_frames, tcos,
                                                    tsin, bins_pad, power);
  return hipGetLastError();
}

hipError_t launch_mel_log(const float* power, int64_t B, int n_frames, int n_bins,
                          const float* fb, int n_mels, float eps, int log_mode, float ln_base,
                          float* mel, hipStream_t stream) {
  const size_t lds = sizeof(float) * (size_t)16 * n_bins;
  if (lds > 64 * 1024) return hipErrorInvalidValue;
  dim3 grid((n_frames + 15) / 16, (unsigned)B);
  mel_log<<<grid, dim3(256), lds, stream>>>(power, n_frames, n_bins, fb, n_mels, eps, log_mode,
                                            ln_base, mel);
  return hipGetLastError();
}

// Polyphase sinc resampling (torchaudio _apply_sinc_resample_kernel: conv1d of the padded
// signal with the [n_phases][klen] kernel at stride `stride`, phases interleaved).  A block
// owns 256 consecutive outputs; the input span they read (<= 256/n_phases*stride + klen
// samples) is staged in LDS once, zero outside [0, n), and every output is one dot product
// of klen taps: an HBM-bound stream (reads ~stride/n_phases inputs per output).
__global__ void __launch_bounds__(256)
resample_sinc(const float* __restrict__ x, int64_t n, int64_t n_out,
              const float* __restrict__ kern, int n_phases, int stride, int klen, int width,
              float* __restrict__ y) {
  extern __shared__ float xs[];
  const int b = blockIdx.y;
  const int64_t m0 = (int64_t)blockIdx.x * 256;
  const int64_t q0 = m0 / n_phases;                     // first output frame of the block
  const int64_t q1 = (min(m0 + 256, n_out) - 1) / n_phases;
  const int64_t s0 = q0 * stride - width;               // first input sample read
  const int span = (int)((q1 - q0) * stride + klen);
  const float* xb = x + (int64_t)b * n;
  for (int i = threadIdx.x; i < span; i += 256) {
    const int64_t g = s0 + i;
    xs[i] = (g >= 0 && g < n) ? xb[g] : 0.f;
  }
  __syncthreads();
  const int64_t m = m0 + threadIdx.x;
  if (m >= n_out) return;
  const int64_t q = m / n_phases;
  const int j = (int)(m - q * n_phases);
  const float* kr = kern + (int64_t)j * klen;
  const float* xr = xs + (q - q0) * stride;
  float acc = 0.f;
  for (int k = 0; k < klen; ++k) acc = fmaf(xr[k], kr[k], acc);
  y[(int64_t)b * n_out + m] = acc;
}

hipError_t launch_resample(const float* x, int64_t B, int64_t n, int64_t n_out,
                           const float* kern, int n_phases, int stride, int klen, int width,
                           float* y, hipStream_t stream) {
  const int64_t span = (int64_t)(255 / n_phases + 1) * stride + klen;
  const size_t lds = sizeof(float) * (size_t)span;
  if (lds > 64 * 1024) return hipErrorInvalidValue;
  dim3 grid((unsigned)((n_out + 255) / 256), (unsigned)B);
  resample_sinc<<<grid, dim3(256), lds, stream>>>(x, n, n_out, kern, n_phases, stride, klen,
                                                  width, y);
  return hipGetLastError();
}

}  // namespace hfg

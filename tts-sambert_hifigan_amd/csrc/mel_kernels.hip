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

#include "kernels.h"
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

// ---------------------------------------------------------------------------------------
// logmel_fft: the whole log-mel of a tile of frames in one launch, FFT-based.
//
// Per frame (one wave): z[n] = w[2n] x[2n] + i w[2n+1] x[2n+1] (the window product in fp32,
// as torch.stft forms it), an N/2-point complex FFT in float64 by mixed-radix Stockham passes
// (radix 8, then 4 or 2) ping-ponging between two LDS buffers, the real-FFT split
// X[k] = (Z[k] + Z*[N/2-k]) / 2 - i e^{-2 pi i k / N} (Z[k] - Z*[N/2-k]) / 2 for
// k = 0..N/2, |X|^2, the slaney / htk mel projection over each band's nonzero bins, + eps,
// log.  float64 arithmetic makes the spectrum exact to ~1e-15 of the frame energy, so quiet
// bins (silence beside loud frames) keep their precision; the O(N log N) FFT replaces the
// O(N^2) DFT GEMM (stft_power_mfma, kept for n_fft that are not a power of two).
// Block: 4 waves x fpw frames; the block's reflect-padded sample span is staged once in
// LDS (fp32) and the [n_mels][frames] tile leaves through LDS as frame-contiguous rows.
struct cd {
  double x, y;
};
__device__ __forceinline__ cd cmul(cd a, cd b) {
  return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x};
}
__device__ __forceinline__ cd cadd(cd a, cd b) { return {a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ cd csub(cd a, cd b) { return {a.x - b.x, a.y - b.y}; }
__device__ __forceinline__ cd cmul_mi(cd a) { return {a.y, -a.x}; }  // (-i) a

// in-register DFT of R points: out[q] = sum_r v[r] e^{-2 pi i r q / R}
template <int R>
__device__ __forceinline__ void dft_r(cd (&v)[R]);
template <>
__device__ __forceinline__ void dft_r<2>(cd (&v)[2]) {
  const cd a = cadd(v[0], v[1]), b = csub(v[0], v[1]);
  v[0] = a;
  v[1] = b;
}
template <>
__device__ __forceinline__ void dft_r<4>(cd (&v)[4]) {
  const cd t0 = cadd(v[0], v[2]), t1 = csub(v[0], v[2]);
  const cd t2 = cadd(v[1], v[3]), t3 = cmul_mi(csub(v[1], v[3]));
  v[0] = cadd(t0, t2);
  v[2] = csub(t0, t2);
  v[1] = cadd(t1, t3);
  v[3] = csub(t1, t3);
}
template <>
__device__ __forceinline__ void dft_r<8>(cd (&v)[8]) {
  cd e[4] = {v[0], v[2], v[4], v[6]}, o[4] = {v[1], v[3], v[5], v[7]};
  dft_r<4>(e);
  dft_r<4>(o);
  constexpr double s = 0.70710678118654752440;
  o[1] = {s * (o[1].x + o[1].y), s * (o[1].y - o[1].x)};   // e^{-i pi/4}
  o[2] = cmul_mi(o[2]);                                      // e^{-i pi/2}
  o[3] = {s * (o[3].y - o[3].x), -s * (o[3].x + o[3].y)};  // e^{-3i pi/4}
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    v[q] = cadd(e[q], o[q]);
    v[q + 4] = csub(e[q], o[q]);
  }
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// one Stockham pass of radix R over an N2-point sequence: sub-transforms of Ns -> Ns * R
// points (twiddle e^{-2 pi i r k / (Ns R)} = tw[2 r k N2 / (Ns R) mod N], tw[t] =
// e^{-2 pi i t / N}, N = 2 N2)
template <int R>
__device__ __forceinline__ void stockham_pass(const cd* __restrict__ src, cd* __restrict__ dst,
                                              int N2, int Ns, const cd* __restrict__ tw,
                                              int lane) {
  const int nb = N2 / R;
  const int tstep = 2 * (N2 / (Ns * R));
  for (int j = lane; j < nb; j += 64) {
    const int k = j & (Ns - 1);
    cd v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = src[j + r * nb];
    if (Ns > 1) {
#pragma unroll
      for (int r = 1; r < R; ++r) v[r] = cmul(v[r], tw[(r * k * tstep) & (2 * N2 - 1)]);
    }
    dft_r<R>(v);
    const int base = (j - k) * R + k;
#pragma unroll
    for (int q = 0; q < R; ++q) dst[base + q * Ns] = v[q];
  }
}

__global__ void __launch_bounds__(256)
logmel_fft(const float* __restrict__ wav, int64_t n_samp, int n_fft, int hop, int n_frames,
           int fpw, const float* __restrict__ window, const cd* __restrict__ tw,
           const int* __restrict__ band, const float* __restrict__ bw, int n_mels, float eps,
           int log_mode, float ln_base, float* __restrict__ mel) {
  extern __shared__ __attribute__((aligned(16))) char lds_m[];
  const int N2 = n_fft / 2;
  const int fpb = 4 * fpw;
  const int span = (fpb - 1) * hop + n_fft;
  cd* const bufs = reinterpret_cast<cd*>(lds_m);                        // [4 waves][2][N2]
  float* const sig = reinterpret_cast<float*>(lds_m + sizeof(cd) * 8 * N2);  // [span]
  float* const mel_s = sig + ((span + 3) & ~3);                         // [n_mels][fpb]
  const int b = blockIdx.y;
  const int f0 = blockIdx.x * fpb;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const float* x = wav + (int64_t)b * n_samp;
  // reflect-padded samples [f0 hop - N/2, f0 hop - N/2 + span)  (torch reflect: x[-i] = x[i],
  // x[L-1+i] = x[L-1-i]; the host checks L > N/2)
  for (int i = threadIdx.x; i < span; i += 256) {
    int64_t g = (int64_t)f0 * hop - N2 + i;
    if (g < 0) g = -g;
    if (g >= n_samp) g = 2 * (n_samp - 1) - g;
    sig[i] = (g >= 0 && g < n_samp) ? x[g] : 0.f;
  }
  __syncthreads();
  cd* A = bufs + (size_t)wave * 2 * N2;
  cd* Bf = A + N2;
  for (int fi = 0; fi < fpw; ++fi) {
    const int fl = wave * fpw + fi;  // frame within the block
    if (f0 + fl >= n_frames) break;  // wave-uniform
    const float* fr = sig + fl * hop;
    for (int n = lane; n < N2; n += 64) {
      const float x0 = fr[2 * n] * window[2 * n], x1 = fr[2 * n + 1] * window[2 * n + 1];
      A[n] = {(double)x0, (double)x1};
    }
    wave_sync();
    cd* src = A;
    cd* dst = Bf;
    int Ns = 1, rem = __builtin_ctz(N2);
    while (rem > 0) {
      if (rem >= 3) {
        stockham_pass<8>(src, dst, N2, Ns, tw, lane);
        Ns *= 8;
        rem -= 3;
      } else if (rem == 2) {
        stockham_pass<4>(src, dst, N2, Ns, tw, lane);
        Ns *= 4;
        rem -= 2;
      } else {
        stockham_pass<2>(src, dst, N2, Ns, tw, lane);
        Ns *= 2;
        rem -= 1;
      }
      wave_sync();
      cd* t = src;
      src = dst;
      dst = t;
    }
    // real-FFT split and power, k = 0..N2, into the free buffer as doubles
    double* P = reinterpret_cast<double*>(dst);
    for (int k = lane; k <= N2; k += 64) {
      const cd zk = src[k & (N2 - 1)];
      const cd zm = src[(N2 - k) & (N2 - 1)];
      const cd zc = {zm.x, -zm.y};
      const cd s_ = cadd(zk, zc), d_ = csub(zk, zc);
      const cd wd = cmul(tw[k], d_);                 // e^{-2 pi i k/N} (Z[k] - Z*[N2-k])
      const double re = 0.5 * (s_.x + wd.y), im = 0.5 * (s_.y - wd.x);  // (s - i wd) / 2
      P[k] = re * re + im * im;
    }
    wave_sync();
    for (int m = lane; m < n_mels; m += 64) {
      const int lo = band[3 * m], hi = band[3 * m + 1], off = band[3 * m + 2];
      double acc = 0.0;
      for (int k = lo; k < hi; ++k) acc += (double)bw[off + k - lo] * P[k];
      const double v = acc + (double)eps;
      const double lv = log_mode == 1 ? log10(v) : (log_mode == 0 ? log(v) : log(v) / (double)ln_base);
      mel_s[m * fpb + fl] = (float)lv;
    }
    wave_sync();
  }
  __syncthreads();
  const int nf = min(fpb, n_frames - f0);
  for (int i = threadIdx.x; i < n_mels * fpb; i += 256) {
    const int m = i / fpb, fl = i - m * fpb;
    if (fl < nf) mel[((int64_t)b * n_mels + m) * n_frames + f0 + fl] = mel_s[m * fpb + fl];
  }
}

size_t logmel_fft_lds_bytes(int n_fft, int hop, int fpw, int n_mels) {
  const int fpb = 4 * fpw;
  const size_t span = (size_t)(fpb - 1) * hop + n_fft;
  return sizeof(cd) * 8 * (size_t)(n_fft / 2) + sizeof(float) * ((span + 3) & ~(size_t)3) +
         sizeof(float) * (size_t)n_mels * fpb;
}

hipError_t launch_logmel_fft(const float* wav, int64_t B, int64_t n_samp, int n_fft, int hop,
                             int n_frames, int fpw, const float* window, const void* tw,
                             const int* band, const float* bw, int n_mels, float eps,
                             int log_mode, float ln_base, float* mel, hipStream_t stream) {
  if (n_fft < 16 || (n_fft & (n_fft - 1)) || fpw < 1) return hipErrorInvalidValue;
  const size_t lds = logmel_fft_lds_bytes(n_fft, hop, fpw, n_mels);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (hipError_t err = ensure_max_lds(reinterpret_cast<const void*>(logmel_fft))) return err;
  dim3 grid((n_frames + 4 * fpw - 1) / (4 * fpw), (unsigned)B);
  logmel_fft<<<grid, dim3(256), lds, stream>>>(wav, n_samp, n_fft, hop, n_frames, fpw, window,
                                               reinterpret_cast<const cd*>(tw), band, bw, n_mels,
                                               eps, log_mode, ln_base, mel);
  return hipGetLastError();
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

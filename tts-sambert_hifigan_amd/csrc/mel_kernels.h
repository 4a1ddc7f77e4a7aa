// mel_kernels.h — on-device log-mel framing kernels (mel_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hfg {

// power[b][f][k] = |sum_n w[n] x_pad[f*hop + n] e^{-2 pi i k n / n_fft}|^2
// (tcos/tsin: [n_fft][bins_pad] tables with the window folded in).
hipError_t launch_stft_power(const float* wav, int64_t B, int64_t N, int n_fft, int hop,
                             int n_bins, int n_frames, const float* tcos, const float* tsin,
                             int bins_pad, float* power, hipStream_t stream);

// mel[b][m][f] = log(sum_k fb[k][m] * power[b][f][k] + eps): log_mode 1 log10, 0 ln,
// 2 ln(v) / ln_base (a custom base, audio_processing.py:131-133)
hipError_t launch_mel_log(const float* power, int64_t B, int n_frames, int n_bins,
                          const float* fb, int n_mels, float eps, int log_mode, float ln_base,
                          float* mel, hipStream_t stream);

// Whole log-mel, FFT-based (float64 spectrum): mel[b][m][f] = log(sum_{k in band m}
// bw[k] |X_f[k]|^2 + eps) with X_f the rfft of frame f (reflect-padded, window[n] x[n] in fp32).
// n_fft a power of two >= 16; tw: n_fft complex doubles e^{-2 pi i t / n_fft}; band: per mel
// (first bin, end bin, offset into bw); fpw frames per wave (4 waves per block).
size_t logmel_fft_lds_bytes(int n_fft, int hop, int fpw, int n_mels);
hipError_t launch_logmel_fft(const float* wav, int64_t B, int64_t n_samp, int n_fft, int hop,
                             int n_frames, int fpw, const float* window, const void* tw,
                             const int* band, const float* bw, int n_mels, float eps,
                             int log_mode, float ln_base, float* mel, hipStream_t stream);

// y[b][m] = sum_k x_pad[b][(m / n_phases) * stride + k] * kern[m % n_phases][k], m < n_out,
// x_pad = x zero-padded by `width` on the left (torchaudio _apply_sinc_resample_kernel)
hipError_t launch_resample(const float* x, int64_t B, int64_t n, int64_t n_out,
                           const float* kern, int n_phases, int stride, int klen, int width,
                           float* y, hipStream_t stream);

}  // namespace hfg

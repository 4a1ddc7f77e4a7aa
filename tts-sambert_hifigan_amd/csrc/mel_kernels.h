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

// mel[b][m][f] = log(sum_k fb[k][m] * power[b][f][k] + eps)  (log10 or ln)
hipError_t launch_mel_log(const float* power, int64_t B, int n_frames, int n_bins,
                          const float* fb, int n_mels, float eps, int log10_out, float* mel,
                          hipStream_t stream);

}  // namespace hfg

// mel_capi.cpp — C ABI of the on-device log-mel framing (include/hifigan_hip.h,
// "mel" section): the host builds the windowed DFT tables and the mel filterbank
// once per handle, forward is two async launches on the caller's stream.
//
// Restates torchaudio.transforms.MelSpectrogram as configured at
// data/audio_processing.py:99-110 (n_fft 1024, hop 256, win 1024, 80 mels,
// 0-8000 Hz, slaney scale + slaney norm, power 2, center=True, reflect pad,
// periodic Hann) and the log at :123-133.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/hifigan_hip.h"
#include "mel_kernels.h"

namespace {

thread_local std::string g_mel_err;

int mfail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_mel_err = buf;
  return code;
}

// torchaudio.functional._hz_to_mel / _mel_to_hz
double hz_to_mel(double f, int slaney) {
  if (!slaney) return 2595.0 * std::log10(1.0 + f / 700.0);
  const double f_sp = 200.0 / 3.0, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp;
  const double logstep = std::log(6.4) / 27.0;
  return f >= min_log_hz ? min_log_mel + std::log(f / min_log_hz) / logstep : f / f_sp;
}
double mel_to_hz(double m, int slaney) {
  if (!slaney) return 700.0 * (std::pow(10.0, m / 2595.0) - 1.0);
  const double f_sp = 200.0 / 3.0, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp;
  const double logstep = std::log(6.4) / 27.0;
  return m >= min_log_mel ? min_log_hz * std::exp(logstep * (m - min_log_mel)) : f_sp * m;
}

}  // namespace

struct hfg_mel_handle {
  hfg_mel_config cfg;
  int device;
  int n_bins, bins_pad;
  float* tcos = nullptr;  // [n_fft][bins_pad]
  float* tsin = nullptr;
  float* fb = nullptr;    // [n_bins][n_mels]
  std::vector<float> fb_host;
};

extern "C" {

const char* hfg_mel_last_error(void) { return g_mel_err.c_str(); }

int hfg_mel_filterbank(const hfg_mel_config* c, float* out) {
  // torchaudio.functional.melscale_fbanks(n_freqs, f_min, f_max, n_mels, sr, norm, mel_scale)
  const int n_freqs = c->n_fft / 2 + 1, n_mels = c->n_mels;
  const int slaney = c->mel_scale == 0;
  std::vector<double> all_freqs(n_freqs), f_pts(n_mels + 2);
  for (int i = 0; i < n_freqs; ++i)
    all_freqs[i] = (double)(c->sample_rate / 2) * i / (double)(n_freqs - 1);
  const double m_min = hz_to_mel(c->f_min, slaney), m_max = hz_to_mel(c->f_max, slaney);
  for (int i = 0; i < n_mels + 2; ++i)
    f_pts[i] = mel_to_hz(m_min + (m_max - m_min) * i / (double)(n_mels + 1), slaney);
  for (int k = 0; k < n_freqs; ++k)
    for (int m = 0; m < n_mels; ++m) {
      const double down = -(f_pts[m] - all_freqs[k]) / (f_pts[m + 1] - f_pts[m]);
      const double up = (f_pts[m + 2] - all_freqs[k]) / (f_pts[m + 2] - f_pts[m + 1]);
      double v = std::fmax(0.0, std::fmin(down, up));
      if (c->norm == 1) v *= 2.0 / (f_pts[m + 2] - f_pts[m]);
      out[(size_t)k * n_mels + m] = (float)v;
    }
  return HFG_OK;
}

int hfg_mel_create(const hfg_mel_config* c, int device, hfg_mel_handle** out) {
  if (!c || !out) return mfail(HFG_EINVAL, "NULL argument");
  *out = nullptr;
  if (c->n_fft <= 0 || (c->n_fft & 1) || c->hop_length <= 0 || c->win_length <= 0 ||
      c->win_length > c->n_fft || c->n_mels <= 0 || c->sample_rate <= 0 ||
      !(c->f_max > c->f_min) || c->f_min < 0)
    return mfail(HFG_EINVAL, "invalid mel configuration");
  if (c->mel_scale != 0 && c->mel_scale != 1) return mfail(HFG_EINVAL, "mel_scale 0|1");
  if (c->norm != 0 && c->norm != 1) return mfail(HFG_EINVAL, "norm 0|1");
  if (c->log_base != 10 && c->log_base != 0 && c->log_base != 1)
    return mfail(HFG_EINVAL, "log_base: 10 (log10), 0 (ln) or 1 (custom base)");
  if (c->log_base == 1 && !(c->log_base_value > 0.f && c->log_base_value != 1.f))
    return mfail(HFG_EINVAL, "custom log base must be > 0 and != 1");
  if ((size_t)(31 * c->hop_length + c->n_fft) * 4 * 33 / 32 > 64 * 1024)
    return mfail(HFG_EINVAL, "n_fft / hop too large for the LDS frame tile");
  auto* h = new (std::nothrow) hfg_mel_handle();
  if (!h) return mfail(HFG_ENOMEM, "host alloc");
  h->cfg = *c;
  h->device = device;
  h->n_bins = c->n_fft / 2 + 1;
  h->bins_pad = (h->n_bins + 31) / 32 * 32;
  if ((size_t)16 * h->n_bins * 4 > 64 * 1024) {
    delete h;
    return mfail(HFG_EINVAL, "n_fft too large for the mel tile");
  }
  // windowed DFT tables: periodic Hann of win_length centred in n_fft (torch.stft)
  const int N = c->n_fft, W = c->win_length, left = (N - W) / 2;
  std::vector<float> tc((size_t)N * h->bins_pad, 0.f), ts((size_t)N * h->bins_pad, 0.f);
  const double two_pi = 6.283185307179586476925286766559;
  for (int n = 0; n < N; ++n) {
    const int wi = n - left;
    const double w = (wi >= 0 && wi < W) ? 0.5 - 0.5 * std::cos(two_pi * wi / W) : 0.0;
    for (int k = 0; k < h->n_bins; ++k) {
      const double ang = two_pi * (double)(((long long)k * n) % N) / N;
      tc[(size_t)n * h->bins_pad + k] = (float)(w * std::cos(ang));
      ts[(size_t)n * h->bins_pad + k] = (float)(-w * std::sin(ang));
    }
  }
  h->fb_host.resize((size_t)h->n_bins * c->n_mels);
  hfg_mel_filterbank(c, h->fb_host.data());
  if (device >= 0) {
    int prev = -1;
    (void)hipGetDevice(&prev);
    if (hipSetDevice(device) != hipSuccess) {
      delete h;
      return mfail(HFG_ENODEV, "hipSetDevice(%d)", device);
    }
    const size_t tb = tc.size() * sizeof(float), fbb = h->fb_host.size() * sizeof(float);
    if (hipMalloc(&h->tcos, tb) != hipSuccess || hipMalloc(&h->tsin, tb) != hipSuccess ||
        hipMalloc(&h->fb, fbb) != hipSuccess) {
      hfg_mel_destroy(h);
      return mfail(HFG_ENOMEM, "hipMalloc(mel tables)");
    }
    if (hipMemcpy(h->tcos, tc.data(), tb, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(h->tsin, ts.data(), tb, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(h->fb, h->fb_host.data(), fbb, hipMemcpyHostToDevice) != hipSuccess) {
      hfg_mel_destroy(h);
      return mfail(HFG_EIO, "hipMemcpy(mel tables)");
    }
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  *out = h;
  return HFG_OK;
}

void hfg_mel_destroy(hfg_mel_handle* h) {
  if (!h) return;
  if (h->tcos) (void)hipFree(h->tcos);
  if (h->tsin) (void)hipFree(h->tsin);
  if (h->fb) (void)hipFree(h->fb);
  delete h;
}

int64_t hfg_mel_frames(const hfg_mel_handle* h, int64_t n_samples) {
  if (!h || n_samples <= 0) return -1;
  return n_samples / h->cfg.hop_length + 1;  // center=True
}

size_t hfg_mel_workspace_bytes(const hfg_mel_handle* h, int64_t B, int64_t n_samples) {
  if (!h || B <= 0 || n_samples <= 0) return 0;
  return sizeof(float) * (size_t)B * (size_t)hfg_mel_frames(h, n_samples) * (size_t)h->n_bins;
}

int hfg_mel_forward(hfg_mel_handle* h, const float* wav, int64_t B, int64_t n_samples, float* mel,
                    void* workspace, size_t workspace_bytes, void* stream) {
  if (!h || !wav || !mel || !workspace) return mfail(HFG_EINVAL, "NULL argument");
  if (h->device < 0) return mfail(HFG_EINVAL, "host-only mel handle");
  if (B <= 0) return mfail(HFG_EINVAL, "B must be > 0");
  if (n_samples <= h->cfg.n_fft / 2)
    return mfail(HFG_EINVAL, "reflect padding needs more than n_fft/2 = %d samples",
                 h->cfg.n_fft / 2);
  if (workspace_bytes < hfg_mel_workspace_bytes(h, B, n_samples))
    return mfail(HFG_EINVAL, "workspace too small");
  const int n_frames = (int)hfg_mel_frames(h, n_samples);
  int prev = -1;
  (void)hipGetDevice(&prev);
  if (prev != h->device && hipSetDevice(h->device) != hipSuccess)
    return mfail(HFG_ENODEV, "hipSetDevice(%d)", h->device);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  float* power = reinterpret_cast<float*>(workspace);
  hipError_t e = hfg::launch_stft_power(wav, B, n_samples, h->cfg.n_fft, h->cfg.hop_length,
                                        h->n_bins, n_frames, h->tcos, h->tsin, h->bins_pad, power,
                                        s);
  if (e == hipSuccess)
    e = hfg::launch_mel_log(power, B, n_frames, h->n_bins, h->fb, h->cfg.n_mels, h->cfg.log_eps,
                            h->cfg.log_base == 10 ? 1 : (h->cfg.log_base == 0 ? 0 : 2),
                            // torch.log(torch.tensor(log_base)): a float32 log of the base
                            std::log(h->cfg.log_base_value), mel, s);
  if (prev >= 0 && prev != h->device) (void)hipSetDevice(prev);
  if (e != hipSuccess) return mfail(HFG_EIO, "mel launch: %s", hipGetErrorString(e));
  return HFG_OK;
}

}  // extern "C"

// ---- resampling (torchaudio.transforms.Resample, audio_processing.py:81-88) ----------
struct hfg_resample_handle {
  int orig, new_, g;          // reduced rates orig / g, new / g
  int width, klen;
  int device;
  float* kern = nullptr;      // [new][klen] on the device
};

namespace {
long long gcd_ll(long long a, long long b) {
  while (b) {
    const long long t = a % b;
    a = b;
    b = t;
  }
  return a;
}
}  // namespace

extern "C" {

// torchaudio.functional._get_sinc_resample_kernel(orig, new, gcd, lowpass_filter_width,
// rolloff, "sinc_interp_hann", dtype=None): float64 arithmetic (the phase offsets j/new
// are a float32 division of an integer tensor, as there), stored float32.
int hfg_resample_kernel(int32_t orig_freq, int32_t new_freq, int32_t lpw, float rolloff,
                        float* kernel, int32_t* width_out, int32_t* n_phases, int32_t* klen_out) {
  if (orig_freq <= 0 || new_freq <= 0 || lpw <= 0 || !(rolloff > 0.f && rolloff <= 1.f))
    return mfail(HFG_EINVAL, "resample: rates and lowpass_filter_width must be > 0, "
                 "0 < rolloff <= 1");
  const long long g = gcd_ll(orig_freq, new_freq);
  const long long orig = orig_freq / g, nw = new_freq / g;
  const double base = (double)std::min(orig, nw) * (double)rolloff;
  const int width = (int)std::ceil((double)lpw * (double)orig / base);
  const int klen = 2 * width + (int)orig;
  if (width_out) *width_out = width;
  if (n_phases) *n_phases = (int32_t)nw;
  if (klen_out) *klen_out = klen;
  if (!kernel) return HFG_OK;
  const double pi = 3.14159265358979323846;
  for (long long j = 0; j < nw; ++j) {
    const double off = (double)((float)(-j) / (float)nw);
    for (int k = 0; k < klen; ++k) {
      double t = (off + (double)(k - width) / (double)orig) * base;
      t = std::min((double)lpw, std::max(-(double)lpw, t));
      const double c = std::cos(t * pi / lpw / 2);
      const double window = c * c;
      t *= pi;
      const double v = (t == 0.0 ? 1.0 : std::sin(t) / t) * (window * (base / (double)orig));
      kernel[j * klen + k] = (float)v;
    }
  }
  return HFG_OK;
}

int hfg_resample_create(int32_t orig_freq, int32_t new_freq, int32_t lpw, float rolloff,
                        int device, hfg_resample_handle** out) {
  if (!out) return mfail(HFG_EINVAL, "out is NULL");
  *out = nullptr;
  int32_t width = 0, np = 0, klen = 0;
  int rc = hfg_resample_kernel(orig_freq, new_freq, lpw, rolloff, nullptr, &width, &np, &klen);
  if (rc) return rc;
  const long long g = gcd_ll(orig_freq, new_freq);
  if ((long long)np * klen > (1LL << 24))
    return mfail(HFG_EINVAL, "resample kernel [%d][%d] too large (rates %d -> %d)", np, klen,
                 orig_freq, new_freq);
  if ((size_t)((255 / np + 1) * (orig_freq / g) + klen) * sizeof(float) > 64 * 1024)
    return mfail(HFG_EINVAL, "resample ratio %d -> %d too large for the LDS input span",
                 orig_freq, new_freq);
  auto* h = new (std::nothrow) hfg_resample_handle();
  if (!h) return mfail(HFG_ENOMEM, "host alloc");
  h->orig = (int)(orig_freq / g);
  h->new_ = np;
  h->g = (int)g;
  h->width = width;
  h->klen = klen;
  h->device = device;
  if (device >= 0) {
    std::vector<float> k((size_t)np * klen);
    hfg_resample_kernel(orig_freq, new_freq, lpw, rolloff, k.data(), nullptr, nullptr, nullptr);
    int prev = -1;
    (void)hipGetDevice(&prev);
    if (hipSetDevice(device) != hipSuccess) {
      delete h;
      return mfail(HFG_ENODEV, "hipSetDevice(%d)", device);
    }
    if (hipMalloc(&h->kern, k.size() * sizeof(float)) != hipSuccess ||
        hipMemcpy(h->kern, k.data(), k.size() * sizeof(float), hipMemcpyHostToDevice) !=
            hipSuccess) {
      hfg_resample_destroy(h);
      return mfail(HFG_ENOMEM, "resample kernel upload");
    }
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  *out = h;
  return HFG_OK;
}

void hfg_resample_destroy(hfg_resample_handle* h) {
  if (!h) return;
  if (h->kern) (void)hipFree(h->kern);
  delete h;
}

int64_t hfg_resample_out_len(const hfg_resample_handle* h, int64_t n) {
  if (!h || n < 0) return -1;
  // torch.ceil(torch.as_tensor(new * length / orig)) on the reduced rates (a float64 quotient)
  return (int64_t)std::ceil((double)h->new_ * (double)n / (double)h->orig);
}

int hfg_resample_forward(hfg_resample_handle* h, const float* x, int64_t B, int64_t n, float* y,
                         void* stream) {
  if (!h || !x || !y) return mfail(HFG_EINVAL, "NULL argument");
  if (h->device < 0) return mfail(HFG_EINVAL, "host-only resample handle");
  if (B <= 0 || n <= 0) return mfail(HFG_EINVAL, "B and n_samples must be > 0");
  const int64_t n_out = hfg_resample_out_len(h, n);
  int prev = -1;
  (void)hipGetDevice(&prev);
  if (prev != h->device && hipSetDevice(h->device) != hipSuccess)
    return mfail(HFG_ENODEV, "hipSetDevice(%d)", h->device);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipError_t e;
  if (h->orig == h->new_)
    e = hipMemcpyAsync(y, x, sizeof(float) * (size_t)(B * n), hipMemcpyDeviceToDevice, s);
  else
    e = hfg::launch_resample(x, B, n, n_out, h->kern, h->new_, h->orig, h->klen, h->width, y, s);
  if (prev >= 0 && prev != h->device) (void)hipSetDevice(prev);
  if (e != hipSuccess) return mfail(HFG_EIO, "resample launch: %s", hipGetErrorString(e));
  return HFG_OK;
}

}  // extern "C"

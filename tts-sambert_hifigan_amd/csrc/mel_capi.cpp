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
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/hifigan_hip.h"
#include "../../include/hifigan_hip_inspect.h"
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
  // FFT path (logmel_fft, n_fft a power of two): window [n_fft] fp32, twiddles [n_fft]
  // complex double, per-band (first bin, end bin, offset) and the bands' nonzero weights
  bool fft = false;
  int fpw = 2;
  float* win = nullptr;
  void* tw = nullptr;
  int* band = nullptr;
  float* bw = nullptr;
  // tables replaced by hfg_mel_set_tables: a forward still in flight on any stream may read
  // them, so they are freed at destroy (or, past kMaxRetired, after one device sync) instead of
  // syncing the device on every replacement
  std::vector<void*> retired;
};

namespace {

// Build and upload every device table from a window [n_fft] and a filterbank
// [n_bins][n_mels] (host, fp32): the DFT-GEMM path's windowed twiddles, the FFT path's
// window, e^{-2 pi i t / N} (float64) and each band's nonzero bins.
int upload_tables(hfg_mel_handle* h, const float* win, const float* fb) {
  const hfg_mel_config* c = &h->cfg;
  const int N = c->n_fft, n_mels = c->n_mels;
  const double two_pi = 6.283185307179586476925286766559;
  if (fb != h->fb_host.data()) h->fb_host.assign(fb, fb + (size_t)h->n_bins * n_mels);
  std::vector<float> tc, ts;
  if (!h->fft) {
    tc.assign((size_t)N * h->bins_pad, 0.f);
    ts.assign((size_t)N * h->bins_pad, 0.f);
    for (int n = 0; n < N; ++n)
      for (int k = 0; k < h->n_bins; ++k) {
        const double ang = two_pi * (double)(((long long)k * n) % N) / N;
        tc[(size_t)n * h->bins_pad + k] = (float)((double)win[n] * std::cos(ang));
        ts[(size_t)n * h->bins_pad + k] = (float)(-(double)win[n] * std::sin(ang));
      }
  }
  std::vector<double> tw_h(2 * (size_t)N);
  for (int t = 0; t < N; ++t) {
    tw_h[2 * t] = std::cos(two_pi * t / N);
    tw_h[2 * t + 1] = -std::sin(two_pi * t / N);
  }
  std::vector<int> band_h(3 * (size_t)n_mels);
  std::vector<float> bw_h;
  for (int m = 0; m < n_mels; ++m) {
    int lo = h->n_bins, hi = 0;
    for (int k = 0; k < h->n_bins; ++k)
      if (fb[(size_t)k * n_mels + m] != 0.f) {
        lo = std::min(lo, k);
        hi = k + 1;
      }
    if (hi <= lo) lo = hi = 0;
    band_h[3 * m] = lo;
    band_h[3 * m + 1] = hi;
    band_h[3 * m + 2] = (int)bw_h.size();
    for (int k = lo; k < hi; ++k) bw_h.push_back(fb[(size_t)k * n_mels + m]);
  }
  if (bw_h.empty()) bw_h.push_back(0.f);
  if (h->device < 0) return HFG_OK;
  int prev = -1;
  (void)hipGetDevice(&prev);
  if (hipSetDevice(h->device) != hipSuccess) return mfail(HFG_ENODEV, "hipSetDevice(%d)", h->device);
  // every new table is allocated and filled before any old one is released: a failure leaves
  // the handle's previous (complete) tables in place
  struct Tbl {
    void** dst;
    const void* src;
    size_t bytes;
    void* fresh;
  };
  std::vector<Tbl> tbls;
  if (!h->fft) {
    tbls.push_back({reinterpret_cast<void**>(&h->tcos), tc.data(), tc.size() * 4, nullptr});
    tbls.push_back({reinterpret_cast<void**>(&h->tsin), ts.data(), ts.size() * 4, nullptr});
    tbls.push_back({reinterpret_cast<void**>(&h->fb), fb, h->fb_host.size() * 4, nullptr});
  }
  tbls.push_back({reinterpret_cast<void**>(&h->win), win, (size_t)N * 4, nullptr});
  tbls.push_back({&h->tw, tw_h.data(), tw_h.size() * 8, nullptr});
  tbls.push_back({reinterpret_cast<void**>(&h->band), band_h.data(), band_h.size() * 4, nullptr});
  tbls.push_back({reinterpret_cast<void**>(&h->bw), bw_h.data(), bw_h.size() * 4, nullptr});
  bool ok = true;
  for (auto& t : tbls) {
    ok = hipMalloc(&t.fresh, t.bytes) == hipSuccess &&
         hipMemcpy(t.fresh, t.src, t.bytes, hipMemcpyHostToDevice) == hipSuccess;
    if (!ok) break;
  }
  constexpr size_t kMaxRetired = 256;
  if (ok && h->retired.size() + tbls.size() > kMaxRetired) {
    // rare (hundreds of replacements): one sync retires every old table at once
    ok = hipDeviceSynchronize() == hipSuccess;
    if (ok) {
      for (void* p : h->retired) (void)hipFree(p);
      h->retired.clear();
    }
  }
  for (auto& t : tbls) {
    if (ok) {
      // a forward in flight may still read the old table: retired, freed at destroy
      if (*t.dst) h->retired.push_back(*t.dst);
      *t.dst = t.fresh;
    } else if (t.fresh) {
      (void)hipFree(t.fresh);
    }
  }
  if (prev >= 0) (void)hipSetDevice(prev);
  return ok ? HFG_OK : mfail(HFG_ENOMEM, "mel tables: device allocation / copy failed");
}

}  // namespace

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
  // the DFT-GEMM path's LDS tiles (the fallback for n_fft that are not a power of two)
  const bool dft_fits = (size_t)(31 * c->hop_length + c->n_fft) * 4 * 33 / 32 <= 64 * 1024 &&
                        (size_t)16 * (c->n_fft / 2 + 1) * 4 <= 64 * 1024;
  auto* h = new (std::nothrow) hfg_mel_handle();
  if (!h) return mfail(HFG_ENOMEM, "host alloc");
  h->cfg = *c;
  h->device = device;
  h->n_bins = c->n_fft / 2 + 1;
  h->bins_pad = (h->n_bins + 31) / 32 * 32;
  // default tables: the periodic Hann window of win_length centred in n_fft (torch.stft)
  // and torchaudio's filterbank, both evaluated in double and rounded to fp32 (the Python
  // layer replaces them by the float32-evaluated torch tables, hfg_mel_set_tables)
  const int N = c->n_fft, W = c->win_length, left = (N - W) / 2;
  const double two_pi = 6.283185307179586476925286766559;
  std::vector<float> win_h(N, 0.f);
  for (int n = 0; n < N; ++n) {
    const int wi = n - left;
    win_h[n] = (wi >= 0 && wi < W) ? (float)(0.5 - 0.5 * std::cos(two_pi * wi / W)) : 0.f;
  }
  h->fb_host.resize((size_t)h->n_bins * c->n_mels);
  hfg_mel_filterbank(c, h->fb_host.data());
  h->fpw = N <= 1024 ? 2 : 1;
  int md = 0;  // 1: the DFT-GEMM path (A/B and fallback tests: hfg_debug_schedule_set)
  hfg_debug_schedule_get("MEL_DFT", &md);
  h->fft = (N & (N - 1)) == 0 && N >= 16 && md == 0 &&
           hfg::logmel_fft_lds_bytes(N, c->hop_length, h->fpw, c->n_mels) <= 160 * 1024;
  if (!h->fft && !dft_fits) {
    delete h;
    return mfail(HFG_EINVAL, "n_fft / hop too large for the LDS frame tiles");
  }
  int rc = upload_tables(h, win_h.data(), h->fb_host.data());
  if (rc) {
    hfg_mel_destroy(h);
    return rc;
  }
  *out = h;
  return HFG_OK;
}

void hfg_mel_destroy(hfg_mel_handle* h) {
  if (!h) return;
  if (h->tcos) (void)hipFree(h->tcos);
  if (h->tsin) (void)hipFree(h->tsin);
  if (h->fb) (void)hipFree(h->fb);
  if (h->win) (void)hipFree(h->win);
  if (h->tw) (void)hipFree(h->tw);
  if (h->band) (void)hipFree(h->band);
  if (h->bw) (void)hipFree(h->bw);
  for (void* p : h->retired) (void)hipFree(p);
  delete h;
}

int hfg_mel_set_tables(hfg_mel_handle* h, const float* window, const float* fb) {
  if (!h || !window || !fb) return mfail(HFG_EINVAL, "NULL argument");
  return upload_tables(h, window, fb);
}

int64_t hfg_mel_frames(const hfg_mel_handle* h, int64_t n_samples) {
  if (!h || n_samples <= 0) return -1;
  return n_samples / h->cfg.hop_length + 1;  // center=True
}

size_t hfg_mel_workspace_bytes(const hfg_mel_handle* h, int64_t B, int64_t n_samples) {
  if (!h || B <= 0 || n_samples <= 0) return 0;
  // the one-launch FFT path keeps its spectra in LDS: no workspace (a token 256 B, so callers
  // that allocate what this returns hold a valid pointer)
  if (h->fft) return 256;
  return sizeof(float) * (size_t)B * (size_t)hfg_mel_frames(h, n_samples) * (size_t)h->n_bins;
}

int hfg_mel_forward(hfg_mel_handle* h, const float* wav, int64_t B, int64_t n_samples, float* mel,
                    void* workspace, size_t workspace_bytes, void* stream) {
  if (!h || !wav || !mel || (!workspace && !h->fft)) return mfail(HFG_EINVAL, "NULL argument");
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
  const int log_mode = h->cfg.log_base == 10 ? 1 : (h->cfg.log_base == 0 ? 0 : 2);
  // torch.log(torch.tensor(log_base)): a float32 log of the base
  const float ln_base = std::log(h->cfg.log_base_value);
  if (h->fft) {
    hipError_t e = hfg::launch_logmel_fft(wav, B, n_samples, h->cfg.n_fft, h->cfg.hop_length,
                                          n_frames, h->fpw, h->win, h->tw, h->band, h->bw,
                                          h->cfg.n_mels, h->cfg.log_eps, log_mode, ln_base, mel, s);
    if (prev >= 0 && prev != h->device) (void)hipSetDevice(prev);
    if (e != hipSuccess) return mfail(HFG_EIO, "mel launch: %s", hipGetErrorString(e));
    return HFG_OK;
  }
  float* power = reinterpret_cast<float*>(workspace);
  hipError_t e = hfg::launch_stft_power(wav, B, n_samples, h->cfg.n_fft, h->cfg.hop_length,
                                        h->n_bins, n_frames, h->tcos, h->tsin, h->bins_pad, power,
                                        s);
  if (e == hipSuccess)
    e = hfg::launch_mel_log(power, B, n_frames, h->n_bins, h->fb, h->cfg.n_mels, h->cfg.log_eps,
                            log_mode, ln_base, mel, s);
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

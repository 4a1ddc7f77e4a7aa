/*
 * hifigan_hip.h — C ABI of libhifigan_hip.so, the MI355X (gfx950) HiFi-GAN
 * Generator inference path.
 *
 * The reference has no FFI layer: its boundary is the PyTorch module
 * HiFiGANGenerator (models/hifigan.py:134-283).  Each entry point below
 * replaces one piece of that module's interface:
 *
 *   hfg_create          ← HiFiGANGenerator.__init__        models/hifigan.py:149-222
 *                         (hyper-parameters only; no weights are created)
 *   hfg_set_weight      ← load_state_dict of one key       (keys: SURVEY.md §8(b))
 *                         incl. weight_g / weight_v from
 *                         apply_weight_norm                models/hifigan.py:274-283
 *   hfg_commit_weights  ← remove_weight_norm / fold        models/hifigan.py:263-272
 *   hfg_forward[_ws]    ← HiFiGANGenerator.forward         models/hifigan.py:224-261
 *   hfg_out_len         ← output-length contract           models/hifigan.py:195-203
 *                         ((L-1)u - 2((k-u)//2) + k per stage)
 *   hfg_forward_ex      ← acoustic→vocoder glue (spec-only in the reference,
 *                         .kiro/specs/.../design.md:905-906): [B,T,80] input
 *                         and per-utterance lengths of a padded batch
 *   hfg_mrf_create      ← MRF.__init__ / ResBlock.__init__  models/hifigan.py:96-114, 34-70
 *   hfg_mrf_forward     ← MRF.forward                       models/hifigan.py:116-131
 *   hfg_resblock_forward← ResBlock.forward                  models/hifigan.py:72-86
 *   hfg_checksum32      ← (no reference counterpart) content hash the Python
 *                         module uses to notice in-place parameter edits
 *
 * Conventions
 *   - Every int-returning call returns 0 on success or a negative errno-style
 *     code (HFG_E*), and sets a thread-local message read by hfg_last_error().
 *     Nothing throws across the ABI.
 *   - Tensors are fp32, contiguous, row-major: mel [B][n_mels][T],
 *     wav [B][1][L] with L = hfg_out_len(h, T).  Both live in device memory
 *     owned by the caller.  The input is never modified.
 *   - hfg_forward* is asynchronous on the caller's HIP stream (hipStream_t
 *     passed as void*; NULL = default stream): no host synchronisation and no
 *     allocation when weights are committed and the workspace is large enough,
 *     so it may be captured into a hipGraph.
 *   - Size limit: the kernels address one utterance with 32-bit byte offsets, so
 *     its largest stage activation (C x L) must hold fewer than 2^30 floats
 *     (V1: T <= 131071 frames, ~25 min of 22.05 kHz audio); a longer T is
 *     refused with HFG_EINVAL before any launch.
 *   - One handle per device.  Calls on one handle are serialised by a
 *     per-handle lock (a forward enqueues its launches, then releases it);
 *     hfg_forward with the internal workspace must not be used from two
 *     streams at once — use hfg_forward_ws with a per-stream workspace.
 */
#ifndef HIFIGAN_HIP_H
#define HIFIGAN_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HFG_MAX_STAGES 8
#define HFG_MAX_RES 8
#define HFG_MAX_DIL 8

#define HFG_OK 0
#define HFG_EINVAL (-22)   /* bad argument / shape / unknown key          */
#define HFG_ENOMEM (-12)   /* device allocation failed                    */
#define HFG_ENODEV (-19)   /* no HIP device / bad device index            */
#define HFG_EAGAIN (-11)   /* weights incomplete (a key was never set)    */
#define HFG_EIO (-5)       /* HIP runtime error (launch, memcpy, ...)     */

/* Arithmetic of the Generator's convolutions.  In every mode conv_post + tanh and the MRF
 * of a C = 8 stage (V2*'s last: one mrf_thin launch on the packed-fp32 vector ALUs) compute
 * exact fp32 products.
 *   FP32   : fp32 operands on the fp32 matrix cores (v_mfma_f32_32x32x2_f32), exact fp32
 *            products, every other conv.  157 TFLOP/s peak.
 *   F16X3  : (the default of the Python module) every fp32 operand scaled by a power of two
 *            and split into f16 halves hi = f16(v 2^e), lo = f16(v 2^e - hi) (22 significant
 *            bits); hi*hi + hi*lo + lo*hi accumulated in fp32 on the f16 matrix cores
 *            (v_mfma_f32_32x32x16_f16 / 16x16x32, 5.3x the fp32 MFMA rate).  Activation
 *            scales are per (tensor, batch item), from the producing kernel's max |value|,
 *            or per block inside a whole-ResBlock / whole-MRF kernel; weight scales per
 *            layer.  Products within ~2^-21 relative of exact: fp32-class output (within
 *            the reference's own fp32 rounding on every golden fixture, x4 weights included).
 *            Used by conv_pre, the upsamplers, the whole-ResBlock kernels of the C = 32 / 64
 *            / 128 stages, the C = 16 thin MRF and the layer convs of C >= 32; convs whose
 *            (k-1)*dilation exceeds the split kernels' window fall back to the fp32 kernels.
 *   BF16X3 : the same kernels with bf16 halves, unscaled: ~16-bit-mantissa products (within
 *            ~1e-5 of the reference at default weight scale; DESIGN.md §4 gives its x4 limit).
 *   BF16W  : bf16 weight storage — every conv weight rounded to bf16 (nearest-even) when
 *            the weights are committed; on the F16X3 kernels with the activations still split:
 *            hi(w)*hi(x) + hi(w)*lo(x) (2 MFMAs per multiply-add instead of 3), exact products
 *            of the bf16-rounded weights elsewhere.  Output is that of the reference
 *            Generator whose weights were cast to bf16 (1e-4 bar against that model), not of
 *            the fp32-weight model.  Biases stay fp32. */
#define HFG_DTYPE_FP32 0
#define HFG_DTYPE_BF16X3 1
#define HFG_DTYPE_BF16W 2
#define HFG_DTYPE_F16X3 3

typedef struct hfg_handle hfg_handle;

/* Hyper-parameters: models/hifigan.py:149-158 constructor arguments. */
typedef struct hfg_config {
    int32_t n_mels;                              /* 80                        */
    int32_t n_up;                                /* len(upsample_rates)       */
    int32_t up_rates[HFG_MAX_STAGES];            /* [8, 8, 2, 2]              */
    int32_t up_kernels[HFG_MAX_STAGES];          /* [16, 16, 4, 4]            */
    int32_t c0;                                  /* upsample_initial_channel  */
    int32_t n_res;                               /* len(resblock_kernel_sizes) */
    int32_t res_kernels[HFG_MAX_RES];            /* [3, 7, 11]                */
    int32_t n_dil[HFG_MAX_RES];                  /* len(dilations[j])         */
    int32_t dil[HFG_MAX_RES][HFG_MAX_DIL];       /* [[1,3,5],[1,3,5],[1,3,5]] */
    int32_t dtype;                               /* HFG_DTYPE_*               */
} hfg_config;

/* Library version string, e.g. "hifigan_hip 0.1.0 gfx950". */
const char* hfg_version(void);

/* Message of the last failing call on this thread ("" if none). */
const char* hfg_last_error(void);

/* Validate cfg, select `device` (hipSetDevice) and create a handle. */
int hfg_create(const hfg_config* cfg, int device, hfg_handle** out);

void hfg_destroy(hfg_handle* h);

/* Number of parameter tensors (state_dict keys without weight norm). */
int hfg_num_params(const hfg_handle* h);

/* Load one state_dict tensor by its reference key, e.g.
 * "mrfs.1.resblocks.2.convs1.0.weight".  `data` is fp32 contiguous, host
 * memory (is_device = 0) or device memory (is_device = 1, copied D2H with
 * a synchronous hipMemcpy).  Keys ending in weight_g / weight_v are folded
 * as w = g * v / ||v|| (norm over all dims but 0) once both are present.
 * Shapes are checked against the configuration. */
int hfg_set_weight(hfg_handle* h, const char* name, const void* data,
                   const int64_t* shape, int ndim, int is_device);

/* Pack every layer into the kernels' fragment-ordered layout and upload it
 * (synchronous).  Returns HFG_EAGAIN if a key was never set.  hfg_forward
 * commits implicitly when weights changed since the last commit. */
int hfg_commit_weights(hfg_handle* h);

/* Output length for T mel frames (T * prod(up_rates) for exact configs). */
int64_t hfg_out_len(const hfg_handle* h, int64_t T);

/* Bytes of device workspace hfg_forward_ws needs for a [B, n_mels, T] input. */
size_t hfg_workspace_bytes(const hfg_handle* h, int64_t B, int64_t T);

/* Grow the internal workspace to fit [B, n_mels, T] (synchronous alloc). */
int hfg_reserve(hfg_handle* h, int64_t B, int64_t T);

/* wav[B][1][out_len] = Generator(mel[B][n_mels][T]); internal workspace. */
int hfg_forward(hfg_handle* h, const float* mel, int64_t B, int64_t T,
                float* wav, int64_t out_len, void* stream);

/* Same with a caller-provided device workspace of >= hfg_workspace_bytes. */
int hfg_forward_ws(hfg_handle* h, const float* mel, int64_t B, int64_t T,
                   float* wav, int64_t out_len, void* workspace,
                   size_t workspace_bytes, void* stream);

/* Acoustic-model glue (design.md:905-906 of the
 * reference spec: mel_pred.transpose(1,2) -> HiFiGAN(mel)).
 *   mel_layout HFG_MEL_BTC reads mel as [B][T][n_mels] — the layout
 *   SAMBERTAcousticModel.inference emits (models/acoustic_model.py:267-297) —
 *   with the transpose fused into conv_pre's input staging.
 *   lengths (device int32[B], or NULL): valid frames per utterance of a
 *   zero-padded batch.  Every layer zero-pads at the utterance's own length,
 *   so wav[b][0][0 : hfg_out_len(len_b)] equals the Generator run on
 *   mel[b, :, :len_b] alone; samples past it are 0.  Tiles past an
 *   utterance's end are skipped. */
#define HFG_MEL_BCT 0
#define HFG_MEL_BTC 1
typedef struct hfg_forward_opts {
    int32_t mel_layout;      /* HFG_MEL_BCT (default) or HFG_MEL_BTC          */
    const int32_t* lengths;  /* device int32[B] valid frames, or NULL (all T)  */
} hfg_forward_opts;

int hfg_forward_ex(hfg_handle* h, const float* mel, int64_t B, int64_t T,
                   const hfg_forward_opts* opts, float* wav, int64_t out_len,
                   void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * One MRF (models/hifigan.py:89-131) as its own handle: the parameters are the
 * MRF module's state_dict keys "resblocks.{j}.convs{1,2}.{m}.{weight,bias}"
 * (hfg_set_weight / hfg_commit_weights / hfg_destroy as for a Generator).
 *   hfg_mrf_forward:      y = MRF.forward(x)      = mean_j ResBlock_j(x)
 *   hfg_resblock_forward: y = ResBlock_j.forward(x) (all its dilation pairs)
 * x, y: device fp32 [B][channels][L] (y must not alias x); workspace of
 * >= hfg_mrf_workspace_bytes(h, B, L) device bytes; async on `stream`.
 * ------------------------------------------------------------------------- */
typedef struct hfg_mrf_config {
    int32_t channels;
    int32_t n_res;
    int32_t res_kernels[HFG_MAX_RES];
    int32_t n_dil[HFG_MAX_RES];
    int32_t dil[HFG_MAX_RES][HFG_MAX_DIL];
    int32_t dtype;                               /* HFG_DTYPE_*               */
} hfg_mrf_config;

int hfg_mrf_create(const hfg_mrf_config* cfg, int device, hfg_handle** out);
size_t hfg_mrf_workspace_bytes(const hfg_handle* h, int64_t B, int64_t L);
int hfg_mrf_forward(hfg_handle* h, const float* x, int64_t B, int64_t L, float* y,
                    void* workspace, size_t workspace_bytes, void* stream);
int hfg_resblock_forward(hfg_handle* h, int j, const float* x, int64_t B, int64_t L,
                         float* y, void* workspace, size_t workspace_bytes,
                         void* stream);

/* Content hash of n device tensors: out[i] (device uint32) = an order-independent
 * 32-bit hash of the nbytes[i] bytes at ptrs[i] (a multiple of 4).  Async on
 * `stream`.  The drop-in module compares it with the hash at its last weight
 * commit to notice edits that bypass autograd's version counter (param.data). */
int hfg_checksum32(const void* const* ptrs, const int64_t* nbytes, int n,
                   uint32_t* out, void* stream);

/* Per-launch profiling with HIP events recorded on the launch stream.
 * While enabled, every kernel launch of hfg_forward* is bracketed by an
 * event pair.  hfg_profile_summary synchronises on the recorded events and
 * writes a JSON object {kernel_label: {"launches", "ms", "flop", "bytes"}}
 * (algorithmic FLOP and bytes) into buf. */
int hfg_set_profiling(hfg_handle* h, int enable);
int hfg_profile_reset(hfg_handle* h);

/* Streams a forward spreads its batch over: 2 (default) runs a batch of B >= 2 as two
 * halves, one on the caller's stream and one on an internal stream joined back by
 * events (each utterance's wav is bitwise unchanged); 1 keeps every launch on the
 * caller's stream.  Forwards under 4096 frames (B x T) stay on one stream.
 * hfg_workspace_bytes depends on this setting.  With 2 streams the
 * profile summary counts a layer's two half-batch dispatches as one launch whose time
 * is the union of their intervals (the halves overlap other layers: per-kernel
 * efficiency is measured with 1). */
int hfg_set_streams(hfg_handle* h, int n);
int hfg_profile_summary(hfg_handle* h, char* buf, size_t buflen);

/* ---------------------------------------------------------------------------
 * On-device log-mel framing feeding the vocoder:
 * replaces extract_mel's MelSpectrogram + log (data/audio_processing.py:98-133;
 * the same framing as VocoderLoss.mel_transform, models/losses.py:414-426).
 * wav [B][n_samples] fp32 -> mel [B][n_mels][n_samples/hop + 1] (center=True,
 * reflect pad, periodic Hann, power 2, mel filterbank, log).
 * ------------------------------------------------------------------------- */
typedef struct hfg_mel_handle hfg_mel_handle;
typedef struct hfg_mel_config {
    int32_t sample_rate;   /* 22050 (config.yaml:5)          */
    int32_t n_fft;         /* 1024                           */
    int32_t hop_length;    /* 256                            */
    int32_t win_length;    /* 1024                           */
    int32_t n_mels;        /* 80                             */
    float f_min, f_max;    /* 0, 8000                        */
    int32_t mel_scale;     /* 0 = slaney, 1 = htk            */
    int32_t norm;          /* 0 = none, 1 = slaney           */
    float log_eps;         /* 1e-10 (audio_processing.py:123) */
    int32_t log_base;      /* 10 = log10, 0 = natural log,   */
                           /* 1 = log(x) / log(log_base_value)*/
                           /* (audio_processing.py:125-133)   */
    float log_base_value;  /* the custom base (log_base == 1) */
} hfg_mel_config;

const char* hfg_mel_last_error(void);
int hfg_mel_create(const hfg_mel_config* cfg, int device, hfg_mel_handle** out);
void hfg_mel_destroy(hfg_mel_handle* h);
/* the [n_fft/2+1][n_mels] filterbank (torchaudio melscale_fbanks), host side */
int hfg_mel_filterbank(const hfg_mel_config* cfg, float* out);
/* Replace the handle's window [n_fft] (torch.stft's window, centred) and filterbank
 * [n_fft/2+1][n_mels] (host pointers, fp32).  The handle's own tables are evaluated in
 * double and rounded; a caller that has torchaudio's float32 tables (torch.hann_window,
 * melscale_fbanks -- audio_processing.py:99-110) passes them here so the spectrum is
 * taken with bitwise the reference's window (the Python layer, mel.py, does). */
int hfg_mel_set_tables(hfg_mel_handle* h, const float* window, const float* fb);
int64_t hfg_mel_frames(const hfg_mel_handle* h, int64_t n_samples);
size_t hfg_mel_workspace_bytes(const hfg_mel_handle* h, int64_t B, int64_t n_samples);
int hfg_mel_forward(hfg_mel_handle* h, const float* wav, int64_t B, int64_t n_samples,
                    float* mel, void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * On-device resampling ← extract_mel's torchaudio.transforms.Resample(orig, new)
 * (data/audio_processing.py:81-88; torchaudio defaults: sinc_interp_hann,
 * lowpass_filter_width 6, rolloff 0.99).  The polyphase sinc kernel
 * [new/g][2*width + orig/g] (g = gcd) is built on the host in float64 and
 * stored fp32; y[b][n*new/g + j] = sum_k x_pad[b][n*orig/g + k] * kernel[j][k]
 * with x zero-padded by width on the left, width + orig/g on the right;
 * out_len = ceil(n * new / orig).  orig == new copies.
 * ------------------------------------------------------------------------- */
typedef struct hfg_resample_handle hfg_resample_handle;
/* host side: the kernel table (NULL kernel = sizes only) */
int hfg_resample_kernel(int32_t orig_freq, int32_t new_freq, int32_t lowpass_filter_width,
                        float rolloff, float* kernel, int32_t* width, int32_t* n_phases,
                        int32_t* kernel_len);
int hfg_resample_create(int32_t orig_freq, int32_t new_freq, int32_t lowpass_filter_width,
                        float rolloff, int device, hfg_resample_handle** out);
void hfg_resample_destroy(hfg_resample_handle* h);
int64_t hfg_resample_out_len(const hfg_resample_handle* h, int64_t n_samples);
/* y[B][out_len] = Resample(x[B][n_samples]), async on stream */
int hfg_resample_forward(hfg_resample_handle* h, const float* x, int64_t B, int64_t n_samples,
                         float* y, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* HIFIGAN_HIP_H */

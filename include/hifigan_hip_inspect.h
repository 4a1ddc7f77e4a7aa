/*
 * hifigan_hip_inspect.h — host-only inspection entry points of
 * libhifigan_hip.so, used by the CPU test-suite to check weight packing
 * without a GPU.  Not part of the reference-facing boundary
 * (include/hifigan_hip.h); a handle created with device = -1 is host-only:
 * it validates the configuration, accepts hfg_set_weight with host data and
 * packs weights, but cannot run hfg_forward*.
 */
#ifndef HIFIGAN_HIP_INSPECT_H
#define HIFIGAN_HIP_INSPECT_H

#include <stddef.h>
#include <stdint.h>

#include "hifigan_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Copy the packed image of one layer (module prefix, e.g. "ups.0") into out:
 * w_len packed GEMM weights followed by b_len per-row biases.  info[10]
 * receives {kind (0 conv, 1 ups, 2 post), M, KT, tile, m_tiles, n_chunks,
 * w_len, b_len, CK, MT}.  With out == NULL only info is filled (no commit). */
int hfg_debug_packed_layer(hfg_handle* h, const char* mod, float* out, size_t cap,
                           int64_t* info);

/* *ew <- the f16x3 packing exponent of layer `mod` (its split planes hold f16 halves of
 * w * 2^ew; 0 in the other modes).  Commits pending weights first and returns that
 * commit's error (HFG_EINVAL while a weight is missing). */
int hfg_debug_layer_exponent(hfg_handle* h, const char* mod, int* ew);

/* Packed image of the whole-ResBlock launch of stage `stage`, ResBlock `j`
 * (resblock_bf16x3.hip; split-precision handles, stages with 32, 64 or 128 channels):
 * w_len floats of A stream (hi/lo pairs of each conv's split format and exponent, as
 * hfg_debug_packed_layer of that conv reports) followed by b_len biases.
 * info[8] receives {fused (0/1), C, KT, n_conv, halo, W, w_len, b_len}.
 * Returns HFG_OK with info[0] = 0 when the stage runs layer by layer. */
int hfg_debug_packed_resblock(hfg_handle* h, int stage, int j, float* out, size_t cap,
                              int64_t* info);

/* A Generator forward (one stream) that also copies the stage outputs the
 * reference's forward passes through (models/hifigan.py:238-251) into
 * caller-owned device buffers: taps[0] <- conv_pre [B][C0][T], taps[1 + 2i] <-
 * ups[i] [B][C_i+1][L_i+1], taps[2 + 2i] <- mrfs[i] [B][C_i+1][L_i+1].
 * n_taps must be 1 + 2 * n_up; NULL entries are skipped. */
int hfg_forward_taps(hfg_handle* h, const float* mel, int64_t B, int64_t T, float* wav,
                     int64_t out_len, void* workspace, size_t workspace_bytes,
                     float* const* taps, int n_taps, void* stream);

/* Schedule overrides for A/B runs and the parity suites (process-wide; read by every
 * later hfg_create / hfg_mrf_create / hfg_mel_create).  The library reads no environment
 * variable for its schedule (the HFG_* knobs of rounds 1-5 are only warned about), so a
 * production handle runs the default schedule whatever its process inherits.  Knobs:
 * FUSED_RB 0|1, FUSE_POST 0|1, RB_SPLIT 0|1, SMALL_TILE -1|0|1, RB_CONC -1|0|1,
 * UPS_FRAMES 1|2, SPLIT 1|2, RB_PERSIST 0..2, DEBUG_FLAGS (ablation builds), MEL_DFT 0|1,
 * AREG_TALL 0|1.
 * set: HFG_EINVAL for an unknown knob or a value out of range.  clear: one knob, or all
 * with knob == NULL.  get: 1 and *value if the knob is overridden, 0 if not. */
int hfg_debug_schedule_set(const char* knob, int value);
int hfg_debug_schedule_clear(const char* knob);
int hfg_debug_schedule_get(const char* knob, int* value);

/* Sustained matrix-core rate of GPU `device` under a full-chip load (csrc/probe.hip):
 * 2 blocks x 4 waves per CU issue independent MFMAs back to back on random operands
 * that change every instruction, `iters` rounds of 32 MFMAs per wave (after a warm-up
 * launch of iters / 4).  kind 0: v_mfma_f32_32x32x16_bf16, kind 1:
 * v_mfma_f32_32x32x2_f32, 4 independent accumulator chains per wave; kinds 2 / 3: the
 * same with one chain (each MFMA accumulates onto the previous one's result; 8 MFMAs
 * per round instead of 32); kinds 4 / 5: v_mfma_f32_32x32x16_f16 (the f16x3 kernels'
 * instruction) on operands with random 10-bit mantissas, 4 chains / 1 chain.
 * *tflops <- dense TFLOP/s over the timed launch (HIP events),
 * *mhz <- shader clock over it (s_memtime against the 100 MHz real-time counter).
 * Measurement only (bench.py's roofline "peak_sustained"); synchronous. */
int hfg_probe_mfma_rate(int device, int kind, int iters, double* tflops, double* mhz);

#ifdef __cplusplus
}
#endif
#endif /* HIFIGAN_HIP_INSPECT_H */

/*
 * distilcodec_amd.h -- C ABI of the MI355X-native DistilCodec encode -> quantize -> decode path.
 *
 * The reference (nabeelscicom/DistilCodec_nabeel, pure Python/PyTorch) has no native interface;
 * this ABI replaces the PyTorch library kernels under the reference's own Python surface
 * (`distilcodec.DistilCodec`, distilcodec/distil_codec.py).  Each entry point below names the
 * reference code it replaces (paths relative to the reference checkout).
 *
 * Conventions
 *  - One handle = one device (the HIP device current when dcx_create is called).
 *  - Feature tensors are channels-last fp32: [B][T][C] (T = frames, 93.75 frames/s at 24 kHz).
 *    The Python shim exposes the reference's channels-first (B, C, T) views on top.
 *  - Every stage call is stream-ordered on the given hipStream_t (passed as void*), allocates
 *    nothing, never synchronises the host, and is therefore hipGraph-capturable.  Device
 *    buffers (inputs, outputs, workspace) are owned by the caller.
 *  - Return value: DCX_OK (0) or a negative DCX_ERR_* status; dcx_last_error() has the text.
 *    No C++ exception crosses the ABI.  A handle is not re-entrant: callers serialise per handle.
 */
#ifndef DISTILCODEC_AMD_H
#define DISTILCODEC_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DCX_ABI_VERSION 4

enum {
  DCX_OK = 0,
  DCX_ERR_INVALID_ARG = -1,    /* bad shape / null pointer / unsupported config value */
  DCX_ERR_MISSING_WEIGHT = -2, /* dcx_finalize: a required checkpoint tensor was never set */
  DCX_ERR_STATE = -3,          /* call order violated (e.g. stage call before dcx_finalize) */
  DCX_ERR_HIP = -4,            /* a HIP runtime call failed */
  DCX_ERR_OOM = -5,            /* device allocation failed (dcx_finalize only) */
  DCX_ERR_WORKSPACE = -6,      /* workspace smaller than dcx_workspace_size() */
  DCX_ERR_UNSUPPORTED = -7     /* input in a format this build does not decode (dcx_mp3_*) */
};

typedef struct dcx_codec dcx_codec;

/* Geometry of the model; mirrors configs/model_config.json (DistilCodec.__init__,
 * distilcodec/distil_codec.py:30-70).  Only the published geometry family is supported
 * (G=1, R=1, downsample factor 1, no template branch); others return DCX_ERR_INVALID_ARG. */
typedef struct dcx_config {
  int32_t sample_rate;          /* 24000 */
  int32_t n_fft, hop, win;      /* 1024, 256, 1024 (mel_spec.py) */
  int32_t n_mels;               /* 128 */
  float f_min, f_max;           /* 0, 12000 */
  int32_t enc_depths[4];        /* 3,3,9,3 (encoders.py:21-60) */
  int32_t enc_dims[4];          /* 256,512,768,1024 */
  int32_t vq_dim;               /* 1024 (grfvq.py input_dim) */
  int32_t codebook_dim;         /* 3584 */
  int32_t codebook_size;        /* 32768 */
  int32_t gen_channels;         /* 1024 (upsample_initial_channel) */
  int32_t gen_pre_k, gen_post_k;/* 13, 13 */
  int32_t n_ups;                /* 5 */
  int32_t up_rates[8];          /* 8,4,2,2,2 */
  int32_t up_kernels[8];        /* 16,12,4,4,4 */
  int32_t n_res;                /* 3 */
  int32_t res_kernels[4];       /* 3,7,11 */
  int32_t res_dilations[4][4];  /* {1,3,5} x3 */
} dcx_config;

/* Fills the published DistilCodec 24 kHz geometry. */
void dcx_default_config(dcx_config* cfg);

/* Create a handle on the current HIP device.  Replaces DistilCodec.__init__ (:30-70). */
int dcx_create(const dcx_config* cfg, dcx_codec** out);
void dcx_destroy(dcx_codec* h);
const char* dcx_last_error(const dcx_codec* h);
const char* dcx_status_string(int status);
int dcx_abi_version(void);
/* First 16 hex digits of the SHA-256 of the library's sources (the .cpp/.hip/.h files under csrc,
 * sorted, then this header), fixed at build time.  The Python loader recomputes it and refuses a stale library. */
const char* dcx_build_id(void);

/* Checkpoint ingestion (replaces load_state_dict in DistilCodec.from_pretrained, :77-97).
 * `name` is "<part>.<state-dict key>" with part in {encoder, quantizer, generator}, e.g.
 * "generator.ups.0.parametrizations.weight.original1".  Weight-norm pairs (original0/1 or
 * weight_g/weight_v) are folded at finalize.  The host data is copied; the caller may free it. */
int dcx_set_tensor(dcx_codec* h, const char* name, const float* host_data, int32_t ndim, const int64_t* shape);
/* Fold, pack and upload every weight; precompute codebook norms and the decode table
 * E * W_out^T + b_out.  Blocking.  `with_generator` = 0 builds encode-side stages only. */
int dcx_finalize(dcx_codec* h, int32_t with_generator);

/* Frames for a padded clip of n_samples (= raw length + 1, distil_codec.py:133-136):
 * T = floor((n_samples + 2*384 - 1024)/256) + 1. */
int64_t dcx_num_frames(const dcx_codec* h, int64_t n_samples);
/* Bytes of device workspace any stage call needs for batch B and T frames.  After dcx_finalize
 * without the generator, the generator's share (13 buffers of B*T*8192 values) is left out. */
size_t dcx_workspace_size(const dcx_codec* h, int32_t batch, int64_t frames);

/* log-mel front end.  Replaces LogMelSpectrogram.forward (mel_spec.py:109-122) incl. the
 * reflect pad and the CPU-forced STFT (:26-57).  audio: [B][n_samples] (already carrying the
 * reference's 1-sample left pad); mel: [B][T][n_mels]. */
int dcx_mel(dcx_codec* h, const float* audio, int32_t batch, int64_t n_samples, float* mel,
            void* workspace, size_t ws_bytes, void* stream);
/* dcx_mel plus the linear spectrogram of LogMelSpectrogram.forward(return_linear=True)
 * (mel_spec.py:119-120): log_linear [B][T][n_fft/2 + 1] = log(clamp(|STFT|, 1e-5)). */
int dcx_mel_linear(dcx_codec* h, const float* audio, int32_t batch, int64_t n_samples, float* mel, float* log_linear,
                   void* workspace, size_t ws_bytes, void* stream);

/* ConvNeXt encoder.  Replaces ConvNeXtEncoder.forward (encoders.py:68-76).
 * mel: [B][T][n_mels] -> feat: [B][T][enc_dims[3]]. */
int dcx_encode(dcx_codec* h, const float* mel, int32_t batch, int64_t frames, float* feat,
               void* workspace, size_t ws_bytes, void* stream);

/* DownsampleGRVQ.forward (grfvq.py:105-132) in eval mode: down conv + ConvNeXt block,
 * project_in (residual_vq.py:152), nearest-code search (vector_quantize_pytorch.py:41-45,
 * 496-506; first index on ties), gather, project_out (residual_vq.py:241), up ConvT1x1 +
 * ConvNeXt block.  codes: [B][T] int32 (required).  x_pjt_in / quantized_fup ([B][T][3584])
 * and quantized ([B][T][vq_dim]) may be NULL to skip them (codes-only fast path). */
int dcx_vq_encode(dcx_codec* h, const float* feat, int32_t batch, int64_t frames, int32_t* codes,
                  float* x_pjt_in, float* quantized_fup, float* quantized,
                  void* workspace, size_t ws_bytes, void* stream);

/* DownsampleGRVQ.decode (grfvq.py:141-146): codes [B][T] int32 -> z [B][T][vq_dim].
 * Code -1 is the reference's masked code (residual_vq.py:120-127: fetched as code 0, then zeroed
 * before project_out), so its frame decodes project_out(0) = the project_out bias.  Other negative
 * codes in [-codebook_size, -1) wrap to code + codebook_size, like the torch indexing of the
 * reference's gather (distil_codec.py:584-586, residual_vq.py:123).  Codes still outside
 * [0, codebook_size) read row 0 and are counted into *n_invalid (device int, may be NULL); the
 * Python surface raises IndexError for them before calling, as torch indexing would. */
int dcx_vq_decode(dcx_codec* h, const int32_t* codes, int32_t batch, int64_t frames, float* z,
                  int32_t* n_invalid, void* workspace, size_t ws_bytes, void* stream);

/* HiFiGANGenerator.forward (generators.py:118-147): z [B][T][gen in] -> wav [B][256*T]. */
int dcx_generate(dcx_codec* h, const float* z, int32_t batch, int64_t frames, float* wav,
                 void* workspace, size_t ws_bytes, void* stream);

/* Whole path: audio -> mel -> encoder -> VQ -> decode(codes) -> generator (encode() followed
 * by decode_from_codes(), distil_codec.py:545-594).  codes [B][T] and wav [B][256*T] required. */
int dcx_encode_decode(dcx_codec* h, const float* audio, int32_t batch, int64_t n_samples,
                      int32_t* codes, float* wav, void* workspace, size_t ws_bytes, void* stream);

/* Sample-rate conversion by up/down for input audio at another rate (replaces librosa.resample,
 * distil_codec.py:108-110 and :676, and librosa.load(sr=...) in meldataset.py:18-20).  Polyphase FIR
 * in scipy.signal.resample_poly's form: y[b][i] = sum_m h[(i + pre)*down - up*m] * x[b][m] over the
 * taps inside h, fp64 taps and accumulation.  The caller designs h (distilcodec_nabeel_amd/resample.py:
 * Kaiser-windowed sinc, resample_poly's defaults) and passes it in device memory.  Rows of x and y
 * start x_stride / y_stride floats apart; batch <= 65535. */
int dcx_resample_poly(const float* x, int32_t batch, int64_t n_in, int64_t x_stride, const double* h, int32_t h_len,
                      int32_t up, int32_t down, int64_t pre, float* y, int64_t n_out, int64_t y_stride, void* stream);

/* MP3 input (host code, no device involved): an MPEG-1 Layer III decoder replacing librosa.load's MP3
 * path (meldataset.py:18-20, distil_codec.py:667; C1's test.mp3, README.md:116), with Xing/LAME
 * gapless trimming (encoder delay + 529 decoder-delay samples skipped, encoder padding dropped).
 * dcx_mp3_info: samples per channel, sample rate, channels.  dcx_mp3_decode: channel-major float
 * samples out[ch][samples] (capacity = samples per channel available).  MPEG-2/2.5, Layer I/II,
 * free format and intensity stereo return DCX_ERR_UNSUPPORTED; data with no decodable frame returns
 * DCX_ERR_INVALID_ARG; dcx_mp3_last_error() has the text (per thread).  Junk between frames is
 * skipped by resyncing on the next header confirmed by its successor, as mpg123 / ffmpeg do.
 * dcx_mp3_stats: granules of the last decode, and how many of them ended their Huffman data exactly
 * at part2_3_length (a check on the code books).  dcx_mp3_junk_bytes: bytes the last decode skipped
 * to resync (0 for a clean stream).  dcx_mp3_bad_frames: frames of the last decode whose data was
 * damaged (e.g. cut by junk); they decode as silence, as mpg123 / ffmpeg conceal decode errors. */
int dcx_mp3_info(const uint8_t* data, size_t nbytes, int64_t* samples, int32_t* sample_rate, int32_t* channels);
int dcx_mp3_decode(const uint8_t* data, size_t nbytes, float* out, int64_t capacity);
const char* dcx_mp3_last_error(void);
int dcx_mp3_stats(int64_t* granules, int64_t* exact);
int64_t dcx_mp3_junk_bytes(void);
int64_t dcx_mp3_bad_frames(void);

/* Batched 2-D transpose [B][R][C] -> [B][C][R] (channels-first <-> channels-last bridge). */
int dcx_transpose(const float* in, float* out, int32_t batch, int64_t rows, int64_t cols, void* stream);

/* Arithmetic of every contraction (convs, linears, STFT, mel, VQ distances):
 *  DCX_GEMM_X6  (default) fp32-tolerance emulation on the matrix cores, two forms:
 *               "x6": fp32 operands split into three bf16 planes (24 significant bits, the full fp32
 *               exponent range), six exact bf16 products per fp32 product, fp32 accumulation on
 *               v_mfma_f32_16x16x32_bf16 / 32x32x16_bf16 (the mel front end, the stem, the ConvTs
 *               and the VQ distance prefilter);
 *               "h3" (round 5; DCX_H3 / DCX_H3_1X1 / DCX_H3_PAIRS below): operands as two fp16
 *               values (22 significant bits), three exact fp16 products per fp32 product, fp32
 *               accumulation on v_mfma_f32_16x16x32_f16 (the generator's ResBlock convs, conv_pre,
 *               the wide ConvTs, the ConvNeXt 1x1 convs).  Each h3 operand tensor is scaled per clip
 *               (per row for the 1x1 convs' operands) by a power of two chosen from a rigorous bound of its values (round 6), so the fp16
 *               range covers it whatever the input scale; a violated bound (only with inf / NaN
 *               inputs) saturates and sets a flag (dcx_range_flags).
 *               Both forms are held to the fp32 tolerance of the product contract (tests/test_gpu_h3.py,
 *               tests/test_gpu_range.py: module outputs within 2e-4 relative of fp64 at input scales
 *               2^-12 .. 2^12); neither is IEEE fp32 arithmetic (that is DCX_GEMM_F32);
 *  DCX_GEMM_F32 v_mfma_f32_32x32x2_f32 (IEEE fp32 fma chain);
 *  DCX_GEMM_BF16 the reference's enable_bfloat16 (torch.autocast bf16, distil_codec.py:550): conv /
 *               linear operands rounded to bf16, one bf16 product, fp32 accumulation, results
 *               rounded to bf16 (after bias, and after GELU); LayerNorm, residual adds and the mel
 *               front end (computed before autocast in the reference) stay fp32-accurate, and the
 *               VQ search stays exact (prefilter + fp64 rescore) on the bf16-valued x_pjt_in.
 * May be changed at any time; the VQ decode table is always built in fp32 at dcx_finalize. */
#define DCX_GEMM_F32 0
#define DCX_GEMM_X6 1
#define DCX_GEMM_BF16 2
int dcx_set_gemm_mode(dcx_codec* h, int32_t mode);
int32_t dcx_get_gemm_mode(const dcx_codec* h);

/* Split-K latency mode for small batches (streaming hops, short clips; BASELINE configs[4]): x6
 * convs whose output tiles would leave most CUs idle run as up to max_splits (<= 16) K-slices
 * over input channels plus one reduce kernel that sums the partials in order and applies the
 * epilogue.  0 or 1 = off (default).  While on, dcx_workspace_size includes 128 MiB of partial
 * sums, and results depend on the tile count (a clip alone is no longer bit-equal to the same
 * clip inside a batch; fp32-level differences).  Takes effect for later calls; size workspaces after. */
int dcx_set_split_k(dcx_codec* h, int32_t max_splits);

/* A/B and test switches of the kernel selection (no reference counterpart).  dcx_create reads them
 * ONCE from the environment variables of the same names (DCX_RP_R, DCX_RP_OLD, DCX_RP_G64,
 * DCX_RP_SYNC, DCX_RP_W4, DCX_GELU_LUT, DCX_BF16_PERSIST, DCX_BF16_REG_EPI, DCX_DWCONV_TILED,
 * DCX_SPLIT_MIN_STEPS, DCX_SPLIT_GROUP_OFF; the h3 arithmetic of DCX_GEMM_X6 mode: DCX_H3,
 * DCX_H3_1X1, DCX_H3_PAIRS (0 = the x6 kernels for the wide generator convs, the ConvNeXt 1x1
 * convs, the small-C ResBlock pairs), DCX_H3_BN, DCX_H3_SPLIT, DCX_RP_RING (0 = per-wave weight loads in the h3
 * ResBlock pair kernel instead of its LDS ring); DCX_ENC_STREAMS (half-batches on the caller's stream
 * and a second stream, same bits: 0 none, 1 the encoder, 2 (default) dcx_encode_decode up to the
 * generator (mel, encoder, VQ encode / decode per half; the generator on the whole batch), 3 the
 * generator per half too)); no launch reads the environment.  This call changes
 * one for later calls on this handle (a hipGraph captured earlier keeps the kernels it captured).
 * Unset, every switch selects the shipped path.  DCX_ERR_INVALID_ARG for an unknown name,
 * DCX_ERR_STATE during a stage call. */
int dcx_set_knob(dcx_codec* h, const char* name, int32_t value);
/* The current value of a switch (DCX_ERR_INVALID_ARG for an unknown name). */
int dcx_get_knob(const dcx_codec* h, const char* name, int32_t* value);

/* h3 range flags (round 6; see DCX_GEMM_X6): bit 0 = an h3 operand's bound was not finite (an inf /
 * NaN upstream: that operand then carries inf / NaN, as the reference's fp32 would), bit 1 = a value
 * exceeded its bound (checked where the producer takes its maxima anyway; never for finite inputs:
 * the bounds are rigorous, from measured maxima).  Cumulative over the handle's calls; synchronises
 * the device; reset != 0 clears them. */
int dcx_range_flags(dcx_codec* h, int32_t* flags, int32_t reset);

/* Standalone 1-D convolution primitive (the kernel family behind every stage), for tests and
 * benchmarks.  weight: host fp32, Conv1d layout [Cout][Cin][k] (transposed=0) or
 * ConvTranspose1d layout [Cin][Cout][k] (transposed=1, padding (k-stride)/2); bias may be NULL.
 * dcx_conv_forward: x [B][Lin][Cin] -> y [B][Lout][Cout] (channels-last, Lout = Lin for a conv
 * with "same" padding, stride*Lin for the transposed form) with epilogue `epi`
 * (0 bias, 1 gelu, 3 residual add: y = res + v), optional second output y_silu = silu(v).
 * In x6 mode the input is split into planes in a buffer owned by the conv object (allocated on
 * first use and grown on demand), so unlike the stage calls this test primitive may allocate. */
typedef struct dcx_conv dcx_conv;
int dcx_conv_create(const float* weight, const float* bias, int32_t cin, int32_t cout, int32_t k, int32_t dilation,
                    int32_t transposed, int32_t stride, dcx_conv** out);
int dcx_conv_forward(dcx_conv* c, int32_t gemm_mode, const float* x, int32_t batch, int64_t lin, float* y,
                     float* y_silu, const float* res, int32_t epi, void* stream);
void dcx_conv_destroy(dcx_conv* c);

/* Single reference modules, for per-module parity tests (tests/test_gpu_modules.py against the
 * reference's own module outputs, tests/golden/modules.npz and bf16.npz).  `module` is the module's
 * state-dict prefix in the reference; the call runs it on the handle's packed weights through the same
 * kernels and launch code the stages use, in the handle's arithmetic mode (DCX_GEMM_BF16: the dtypes of
 * the reference's CUDA autocast).  x / y are channels-last fp32 [B][rows][C] unless noted:
 *   "encoder.downsample_layers.0": stem Conv1d k7 + channels-first LayerNorm; "encoder.downsample_layers.<i>"
 *       (i >= 1): channels-first LayerNorm + 1x1 Conv1d (encoders.py:22-39);
 *   "encoder.stages.<i>.<j>", "quantizer.downsample.0.1", "quantizer.upsample.0.1": ConvNeXtBlock
 *       (convnext_utils.py:263-282);
 *   "encoder.downsample_layers.0.1", "encoder.downsample_layers.<i>.0", "encoder.norm": channels-first
 *       LayerNorm (convnext_utils.py:186-213);
 *   "quantizer.downsample.0" / "quantizer.upsample.0": Conv1d / ConvTranspose1d + ConvNeXtBlock
 *       (grfvq.py:68-96); "quantizer.grvq.rvqs.0.project_in": Linear (residual_vq.py:152);
 *   "generator.conv_pre": Conv1d (generators.py:121);
 *   "generator.ups.<i>": ConvTranspose1d, y [B][rows * rate][Cout] (generators.py:29-116);
 *   "generator.resblocks.<i>.blocks.<j>": ResBlock1 (convnext_utils.py:106-113), per-conv launches;
 *   "generator.resblocks.<i>": the stage's ParralelBlock (convnext_utils.py:137-138) as the generator
 *       runs it, with the SiLU that follows it fused: y = silu(mean of the ResBlock1s) (fused pair
 *       kernels at C = 32 / 64);
 *   "generator.conv_post": the generator's tail, SiLU -> conv_post -> tanh (generators.py:141-145),
 *       y [B][rows][1];
 *   "quantizer.search": nearest code (vector_quantize_pytorch.py:41-45, 496-506) of x_pjt_in rows
 *       x [B][rows][codebook_dim]; y = int32 codes [B][rows] (every mode: the exact nearest code of x
 *       as given; in bf16 mode through the pipeline's compact-operand prefilter).
 * dcx_module_io reports a module's input channels, output channels (0: int32 codes) and output rows
 * per input row; unknown names return DCX_ERR_INVALID_ARG (and dcx_module_workspace_size 0).
 * dcx_module_forward takes the input's channel count and returns DCX_ERR_INVALID_ARG unless it is the
 * module's (the kernels read that many channels per row). */
int dcx_module_io(const dcx_codec* h, const char* module, int32_t* in_channels, int32_t* out_channels,
                  int32_t* out_rate);
size_t dcx_module_workspace_size(const dcx_codec* h, const char* module, int32_t batch, int64_t rows);
int dcx_module_forward(dcx_codec* h, const char* module, const float* x, int32_t batch, int64_t rows,
                       int32_t channels, void* y, void* workspace, size_t ws_bytes, void* stream);

/* VQ search diagnostics (x6 / bf16 mode): the search is a bf16 prefilter whose winner is certified
 * by a rigorous error bound; rows with more than one code inside the bound are rescored in fp64.
 * Returns the cumulative number of such rows and of codes rescored (synchronises the device);
 * reset != 0 zeroes the counters.  Counting is off until the first call (it costs two atomics per
 * rescored row) and stays on from then.  Replaces nothing in the reference (its search is one cdist). */
int dcx_vq_rescore_stats(dcx_codec* h, int64_t* rows_rescored, int64_t* codes_rescored, int32_t reset);

/* Optional per-kernel timing: when enabled, every launch is bracketed by HIP events on its
 * stream.  dcx_profile_read synchronises the device and returns, per kernel symbol, the
 * launch count, summed device milliseconds and summed algorithmic FLOPs / bytes. */
int dcx_profile_enable(dcx_codec* h, int32_t on);
int dcx_profile_reset(dcx_codec* h);
int32_t dcx_profile_count(const dcx_codec* h);
int dcx_profile_read(dcx_codec* h, int32_t i, const char** name, int64_t* launches, double* ms,
                     double* flops, double* bytes);

#ifdef __cplusplus
}
#endif
#endif /* DISTILCODEC_AMD_H */

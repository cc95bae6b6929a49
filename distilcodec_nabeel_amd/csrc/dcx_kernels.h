// Internal interface between the host orchestration (dcx_api.cpp) and the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dcx {

// Epilogue of the implicit-GEMM convolution (applied per output element v = acc + bias).
enum Epi : int {
  EPI_BIAS = 0,       // v
  EPI_GELU = 1,       // gelu_erf(v)                     ConvNeXt pwconv1 + nn.GELU()
  EPI_GAMMA_RES = 2,  // res + gamma * v                 ConvNeXt pwconv2, layer scale, residual
  EPI_RES = 3,        // res + v                         ResBlock1 `x = xt + x`
  EPI_LOGCLAMP = 4,   // log(max(v, 1e-5))               LogMelSpectrogram.compress
};

// ParallelBlock mean of the 3 ResBlock1 outputs (convnext_utils.py:137-138), folded into the
// epilogue of each ResBlock's last conv: first writes, mid adds, last adds and divides by 3.
enum Mean : int { MEAN_NONE = 0, MEAN_FIRST = 1, MEAN_MID = 2, MEAN_LAST = 3 };

constexpr int kMaxPhases = 8;

// ---- h3 activation range (round 6) ------------------------------------------------------------
// An h2 pair (h = fp16(y), l = fp16(y - h)) carries 22 significant bits only while |y| lies in
// [2^-3, 2^16): below, l goes subnormal (an absolute floor of 2^-25), above, fp16 saturates.  Every
// h2 tensor is therefore stored as y = x * 2^a, with a = h2_shift(bound) chosen per clip from an
// upper bound of |x| known BEFORE the tensor is produced (scaled bound in [2^14, 2^15): a 2x margin
// under 65504), and its consumer multiplies its accumulators by 2^-(a + w3_shift) (exact).  Two
// granularities:
//  * per ROW for the one-tap (1x1) consumers, whose output row depends on one input row: a kernel
//    that sees a whole row before splitting it (LayerNorm, launch_h2_rows) takes the row's exact max;
//    the ConvNeXt MLP hidden takes G max|LayerNorm row| + max|bias| (RangeProg::rowwise);
//  * per CLIP for the tap convs (the generator): G max|input| + max|bias| (+ max|residual|) with
//    max|input| MEASURED per clip by the input's producer (ConvParams::y_amax), so the looseness of
//    one layer never compounds; a caller's tensor by its exact clip max (launch_h2_ranged).
// G is the largest absolute row sum of the weights (host).  All bounds are rigorous; with the bound
// B the per-element error is at most 2^-22 |x| + 2^-39 B.
constexpr int kH2Top = 15;
constexpr int kH2ShiftMax = 64;
__host__ __device__ inline int h2_shift(float bound) {
  if (!(bound <= 3.0e38f)) return 0;  // NaN / inf bound: unscaled (the producer raises the range flag)
  if (bound < 1e-30f) return kH2ShiftMax;
  int e = 0;
  (void)frexpf(bound, &e);  // bound = f 2^e, f in [0.5, 1): bound * 2^(15 - e) < 2^15
  const int a = kH2Top - e;
  return a < -kH2ShiftMax ? -kH2ShiftMax : a > kH2ShiftMax ? kH2ShiftMax : a;
}
// Range flag bits (dcx_range_flags): an h2 output's bound was not finite / a value exceeded it.
enum RangeFlag : int { RANGE_NONFINITE = 1, RANGE_OVER = 2 };
// Bound program of an h2 output, evaluated on the device before the tensor is written, per clip b
// (or per row, rowwise: b = the launch's global row b * Lq + q):
// c + sum_{i < n} g[i] * max(m[i] ? m[i][b] : 0, f[i]).  m: measured maxima; f: floors.
constexpr int kRangeTerms = 6;
struct RangeProg {
  const float* m[kRangeTerms];
  float g[kRangeTerms], f[kRangeTerms];
  float c;
  int n;
  int rowwise;  // m indexed by row; the shift written per row (y_ash[row])
};
// (device) the program's bound for clip b; unrolled so the kernel-argument arrays are indexed
// statically (a dynamic index would copy them to scratch)
__device__ __forceinline__ float range_bound(const RangeProg& r, long long b) {
  float v = r.c;
#pragma unroll
  for (int i = 0; i < kRangeTerms; ++i)
    if (i < r.n) v += r.g[i] * fmaxf(r.m[i] ? r.m[i][b] : 0.f, r.f[i]);
  return v;
}
// (device) the current value of a running maximum slot (agent-scope atomic load: never a value newer
// than the slot's, possibly an older one, which only costs an atomic that was not needed)
__device__ __forceinline__ float range_cur(const float* amax, long long b) {
  return amax ? __hip_atomic_load(amax + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.f;
}
// (device) range_report for a whole workgroup of nt threads (all of them call it): the waves' maxima
// meet in LDS (barriers that leave the wave's global stores in flight) (red: nt / 64 floats the caller may overwrite, after its last LDS use) and one thread
// reports, so a launch's first round of tiles makes one atomic per workgroup, not one per wave (the
// atomics of all clips hit one L2 line)
__device__ __forceinline__ void range_report_wg(float vmax, float* amax, int b, float lim, int* rflag, float cur,
                                                float* red, int nt) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) vmax = fmaxf(vmax, __shfl_xor(vmax, off, 64));
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = vmax;
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  float m = 0.f;
  if (threadIdx.x == 0) {
    m = red[0];
    for (int w = 1; w < nt / 64; ++w) m = fmaxf(m, red[w]);
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // red read before any wave goes on to overwrite the LDS (persistent kernels)
  if (threadIdx.x == 0) {
    if (amax && m > cur) atomicMax(reinterpret_cast<unsigned*>(amax + b), __float_as_uint(m));
    if (rflag && m > lim) atomicOr(rflag, RANGE_OVER);
  }
}
// (device) a wave's largest |value| (vmax >= 0 per lane) into amax[b] (atomicMax on the fp32 bits,
// which order like the values for non-negative floats), and RANGE_OVER when it exceeds lim (the
// largest |value| the h2 output's scale admits; +inf when there is none).  At most one atomic per
// wave, and none when vmax does not exceed cur (range_cur of the slot, read earlier): the slots of
// all clips share one cache line, so every wave's atomic serialised in one L2 channel, and each
// later vmcnt wait of the wave (they count in issue order) waited behind it (round 6: C2 171 -> 181 ms
// before this test).
__device__ __forceinline__ void range_report(float vmax, float* amax, int b, float lim, int* rflag, float cur = -1.f) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) vmax = fmaxf(vmax, __shfl_xor(vmax, off, 64));
  if ((threadIdx.x & 63) == 0) {
    if (amax && vmax > cur) atomicMax(reinterpret_cast<unsigned*>(amax + b), __float_as_uint(vmax));
    if (rflag && vmax > lim) atomicOr(rflag, RANGE_OVER);
  }
}

// A/B and test switches.  dcx_create reads them from the environment ONCE into its handle
// (knobs_from_env, dcx_api.cpp) and dcx_set_knob changes them per handle; no launcher reads the
// environment, so a captured hipGraph and the eager calls after it run the same kernels.  Every
// default below is the shipped path.
struct Knobs {
  int rp_rows = 0;          // DCX_RP_R: pair-kernel tile height (an instantiated size; 0 = the launcher's choice)
  int rp_old = 0;           // DCX_RP_OLD=1: the step-schedule pair kernel (conv_res_pair) at C = 32 too
  int rp_g64 = 0;           // DCX_RP_G64=1: the barrier-free 8-wave pair kernel at C = 64
  int rp_sync = 0;          // DCX_RP_SYNC=n: a barrier after every n-th tap of conv_res_pair_g
  int rp_w4 = 0;            // DCX_RP_W4=1: conv_res_pair_w4 (4-wave workgroups, two per CU; A/B)
  int gelu_lut = -1;        // DCX_GELU_LUT: conv_gemm_bf16dp's table limit (-1 = the whole table, 0 = evaluated)
  int bf16_persist = 1;     // DCX_BF16_PERSIST=0: the staged bf16dm for pwconv1 instead of bf16dp
  int bf16_reg_epi = 1;     // DCX_BF16_REG_EPI=0: the LDS-staged epilogue for pwconv1 too
  int dwconv_tiled = 0;     // DCX_DWCONV_TILED=1: the round-2 tiled dwconv_ln (same bits)
  int split_min_steps = 0;  // DCX_SPLIT_MIN_STEPS: split-K only convs with at least this many K steps
  int split_group_off = 0;  // DCX_SPLIT_GROUP_OFF=1: per-conv split launches instead of grouped ones
  int h3 = 1;               // DCX_H3=0: the wide generator stages' ResBlock convs in x6 arithmetic (A/B, tests)
  int h3_bn = 0;            // DCX_H3_BN=128 / 256: the 256 x 128 / 128 x 256 h3 tiles instead of 256 x 256 (A/B)
  int h3_split = 1;         // DCX_H3_SPLIT=0: conv_gemm_x3dw's DMA issued by group 0 alone (A/B)
  int h3_pairs = 1;         // DCX_H3_PAIRS=0: the C = 32 / 64 ResBlock pairs in x6 arithmetic (A/B, tests)
  int h3_1x1 = 1;           // DCX_H3_1X1=0: the ConvNeXt blocks' 1x1 convs in x6 arithmetic (A/B, tests)
  int rp_ring = 1;          // DCX_RP_RING=0: conv_res_pair_h3's weights loaded per wave instead of the LDS ring (A/B)
  int enc_streams = 2;      // DCX_ENC_STREAMS: half-batches on two streams, 0 off, 1 the encoder, 2 up to the generator, 3 the whole path (same bits)
};

// out[b][q*out_mul + phase][co] = epi( sum_{m<taps} sum_{ci<Cin} x[b][q + in_base[phase] + m*in_step][ci]
//                                       * w[phase][co][m*Cin + ci] + bias[co] )
// Rows of x outside [0, Lin) read as zero (zero padding).  Channels-last everywhere.
// x6 activations ("planes"): an fp32 tensor [rows][C] held as three bf16 planes interleaved per
// 8 channels, [rows][C/8][plane 3][8] (6 bytes/element); hi + mid + lo reproduces x to 2^-27.
struct ConvParams {
  const float* x;
  const unsigned short* x6;     // x6 mode input planes (row stride 3*ldx elements)
  const float* w;               // fp32 weights [phase][Cout][taps*Cin]
  const unsigned short* w6;     // if set: x6 mode, bf16 split weights [phase][tap][Cin/16][Cout][2][3][8]
  const float* bias;   // may be null
  const float* gamma;  // EPI_GAMMA_RES
  const float* res;    // EPI_GAMMA_RES / EPI_RES, layout of y
  float* y;            // v (may be null)
  float* y2;           // silu(v) (may be null)
  float* macc;         // mean accumulator, layout of y (MEAN_* != NONE)
  unsigned short* y6;  // planes of v (may be null; needs ldy == Cout)
  unsigned short* y6s; // planes of silu(v) (may be null)
  long long x_bstride;      // elements between clips in x
  long long y_bstride;      // elements between clips in y / y2 / res / macc
  long long w_phase_stride; // elements between phases in w
  int Lin, Lq, Cin, Cout, ldx, ldy;
  int taps, in_step, out_mul;
  int in_base[kMaxPhases];
  int epi, mean_mode;
  // argmin epilogue (VQ search)
  const float* x2;      // [rows] squared norms of x rows
  const float* e2;      // [Cout] squared norms of the codebook rows
  float* part_val;      // [rows][ntiles]
  int* part_idx;        // [rows][ntiles]
  float* part_val2;     // [rows][ntiles] second-smallest value (VQ prefilter)
  // planes-mode arithmetic: 6 = x6 (fp32-accurate), 1 = bf16 (hi plane only, one product);
  // round_bf16: round the GEMM result (after bias, and after GELU) to bf16 like torch.autocast
  int nprod, round_bf16;
  // persistent x6 kernels: tiles are enumerated over (phase, clip, row tile, column tile)
  int batch, phases;
  // fp32-input (AF32) kernels: apply silu to the input while staging (the producer then writes
  // only the fp32 tensor, not its silu as well)
  int silu_in;
  // Layouts other than planes for x6 / y6 (dcx_planes.h), 0 = planes:
  //   1 = compact bf16 ([rows][C], hi plane only; bf16 mode; read by conv_gemm_bf16dm and
  //       vq_prefilter_bk; written with round_bf16, ldy == Cout);
  //   2 = "hm" ([rows][C/32][8][8], hi and mid planes per 32 channels; x6-mode x_pjt_in, read by
  //       vq_prefilter_dm only);
  //   3 = "h2" (x only: [rows][C/32][8][8] fp16 h and l per 32 channels; read by conv_gemm_x3dq).
  int x_compact, y_compact;
  // bf16-mode 1x1 weights as [phase][Cin/32][Cout][32] bf16 (hi only; conv_gemm_bf16dm), or null;
  // for the VQ prefilter: the codebook as launch_repack_codebook_bk writes it.
  const unsigned short* wc;
  // split-K (conv_gemm_x6pp / x6lm only): ksplit > 1 slices over input-channel chunks, each a
  // whole number of kunit chunks; batch = clips * ksplit, and slice s of clip c is output clip
  // s * clips + c (partial sums, plain fp32: launch_splitk_epilogue finishes them)
  int ksplit, kunit;
  // diagnostic builds (-DDCX_DIAG_DUP) only: 1 = compute the epilogue but store nothing, 2 = no
  // epilogue at all (a timing copy launched before the real launch, on the real inputs)
  int diag_skip;
  // conv_gemm_bf16dp with GELU: > 0 = GELU from its LDS table of the bf16 GELU (same bits), a wave
  // with a table offset >= gelu_lut storing the evaluated epilogue instead; 0 = evaluated (set by
  // launch_conv from kn)
  int gelu_lut;
  // the handle's switches (host only; null = the defaults)
  const Knobs* kn;
  // h3 arithmetic (conv_gemm_x3dq, x_compact == 3: the input in the fp16 "h2" layout of
  // dcx_planes.h): weights [phase][tap][Cin/32][Cout][4 groups][h 8 | l 8] fp16 of w * 2^w3_shift
  const unsigned short* w3;
  int w3_shift;
  // y6s in the h2 layout instead of planes (the input of a following h3 conv)
  int y6s_h2;
  // h3 activation range (round 6, see h2_shift): the h2 input holds x * 2^x_ash[clip] (x_ash null:
  // x_ash_c for every clip); an h2 output (y6 with y_compact == 3, or y6s with y6s_h2) is written as
  // v * 2^h2_shift(yb(clip)) and that shift stored to y_ash[clip] (may be null); y_amax (may be null)
  // receives the per-clip max |v| of the epilogue's final value v (atomicMax on the fp32 bits);
  // rflag (may be null) the RangeFlag bits
  const int* x_ash;
  int x_ash_c;
  const int* x_ash_row;  // one-tap convs: a per-row shift of the input row b * Lin + q (epilogue_lds)
  int* y_ash;
  float* y_amax;
  RangeProg yb;
  int* rflag;
};

// Independent convs issued as one launch (launch_conv_group); problem k owns logical tiles
// [start[k], start[k + 1]), tiles_per_clip[k] per clip.
constexpr int kMaxGroup = 3;
struct ConvGroup {
  ConvParams p[kMaxGroup];
  int start[kMaxGroup + 1];
  int tiles_per_clip[kMaxGroup];
};

// The reduces of a grouped split-K launch (launch_splitk_epilogue_group): member k's partials
// part[k] (splits[k] slices, stride[k] floats apart) finished with p[k]'s epilogue by the blocks
// [start[k], start[k + 1]), total4[k] 4-channel groups.
struct SplitEpiGroup {
  ConvParams p[kMaxGroup];
  const float* part[kMaxGroup];
  int splits[kMaxGroup];
  long long stride[kMaxGroup], total4[kMaxGroup];
  int start[kMaxGroup + 1];
  // chain (> 0: the member count): the members are a ParallelBlock's last convs with the mean folded
  // into their epilogues (MEAN_FIRST, MID.., LAST on one accumulator); one thread finishes an element
  // of every member in member order, so the mean is accumulated in ResBlock order as the per-conv
  // reduces do
  int chain;
};

// One pair (c1 dilated, c2 undilated) of each ResBlock1 of a small-channel ParallelBlock (C = 32 / 64,
// x6 arithmetic), fused: silu(c1) stays in LDS (dcx_resblock.hip).  Member m reads state src[m]
// ([clip][L][C] fp32) and writes src[m] + c2(silu(c1(silu(src[m])))) to dst[m] (dst != src: the
// tap halo makes in-place updates race), or, with mean_out set, silu of the mean over the members
// (ParralelBlock, ResBlock order) to mean_out.  Weights: the x6 planes packing of ConvParams::w6.
struct ResPairParams {
  const float* src[kMaxGroup];
  float* dst[kMaxGroup];
  const unsigned short* w1[kMaxGroup];
  const unsigned short* w2[kMaxGroup];
  const float* b1[kMaxGroup];
  const float* b2[kMaxGroup];
  int taps[kMaxGroup], dil[kMaxGroup];  // c1 taps (odd, (taps - 1) / 2 <= 8) and dilation (reach <= 32)
  int nmem;
  float* mean_out;
  long long bstride;  // elements between clips
  int L, batch, C;
  // conv_res_pair_g: a workgroup barrier after every tap_sync-th tap of a conv (0: none), which
  // bounds how far the two waves of a SIMD drift apart before the image hand-offs (set by
  // launch_res_pair from kn)
  int tap_sync;
  // h3 (conv_res_pair_h3): w1 / w2 are the ConvParams::w3 weights, scaled by 2^w3_shift{1,2}[m]
  int h3;
  int w3_shift1[kMaxGroup], w3_shift2[kMaxGroup];
  // h3 activation range (round 6): member m's S image is silu(src) * 2^h2_shift(src_amax[m][clip]),
  // its T image silu(c1 + b1) * 2^h2_shift(g1[m] src_amax[m][clip] + bm1[m]) (g1: the c1 weights'
  // largest absolute row sum, bm1: max |b1|); dst_amax[m] (may be null) receives the per-clip max
  // |dst| (atomicMax) for the next pair's S image.  src_amax null: 0 (x6 kernels ignore all of it).
  const float* src_amax[kMaxGroup];
  float* dst_amax[kMaxGroup];
  float g1[kMaxGroup], bm1[kMaxGroup];
  int* rflag;
  const Knobs* kn;  // host only; null = the defaults
};

// Launchers (all stream-ordered, no allocation).  Return hipError_t of the launch.
hipError_t launch_conv(const ConvParams& p, int batch, int phases, hipStream_t s, const char** kname);
// n <= kMaxGroup independent single-phase convs with one column tiling as one launch of the
// LDS-DMA 16x16x32 kernel; hipErrorNotSupported when they do not all qualify (the caller then
// launches them one by one, which gives the same bits).
hipError_t launch_conv_group(const ConvParams* ps, int n, int batch, hipStream_t s, const char** kname);
hipError_t launch_res_pair(const ResPairParams& p, hipStream_t s, const char** kname);
// Split-K latency mode: the reduce kernel that sums `splits` fp32 partial outputs of a
// ConvParams::ksplit launch (laid out like p.y, `stride` floats apart, in order) and applies p's
// whole epilogue (bias, epi, mean, every output and layout).
hipError_t launch_splitk_epilogue(const ConvParams& p, const float* partials, int splits, long long stride, int batch,
                                  int phases, hipStream_t s);
// Split-K latency mode, grouped (round 4): n <= kMaxGroup single-phase halo convs (ResBlock convs:
// Cout % 128, taps >= 3), member k with its own ps[k].ksplit (1 = unsplit: the member's epilogue runs
// in the conv) and virtual clips batch * ksplit, as one conv_gemm_x6pp launch; then one launch of
// the reduces of the split members.  hipErrorNotSupported when the members do not qualify.
hipError_t launch_conv_split_group(const ConvParams* ps, int n, int batch, hipStream_t s, const char** kname);
hipError_t launch_splitk_epilogue_group(const ConvParams* ps, const float* const* partials, const int* splits,
                                        const long long* strides, int n, int batch, bool chain, hipStream_t s);
hipError_t launch_vq_argmin(const ConvParams& p, int rows, hipStream_t s, const char** kname);
int vq_argmin_ntiles(int ncodes);
// per-row partial count of the x6 / bf16-mode prefilter launch_vq_prefilter runs for `rows` rows with
// x_pjt_in in layout x_layout (ConvParams::x_compact)
int vq_prefilter_ntiles(int ncodes, int dim, long long rows, int x_layout);
// VQ search, x6 mode: bf16x3 prefilter (approximate squared distances, per-tile top 2) ...
// x_bf16: the rows of x are bf16 values (mid and lo planes zero), which drops the mid*hi product.
// p.x_compact == 1 (bf16 mode) / 2 (x6 mode, "hm" layout) with p.wc the launch_repack_codebook_bk
// codebook: vq_prefilter_bk / vq_prefilter_dm reading contiguous runs.
// p.x_compact == 1 with p.wc the [CD/32][NC][32] bf16 hi codebook: vq_prefilter_b1 (one product,
// both modes; vq_b1_takes).  Built with -DDCX_VQ_OLD (A/B): p.x_compact == 1 (bf16 mode) / 2 (x6
// mode, "hm" layout) with p.wc the launch_repack_codebook_bk codebook: vq_prefilter_bq / _dm.
hipError_t launch_vq_prefilter(const ConvParams& p, int rows, bool x_bf16, hipStream_t s, const char** kname);
bool vq_b1_takes(int ncodes, int dim);
// ... then per row: certify the prefilter's winner with a rigorous error bound, or rescore every
// candidate inside the bound in fp64.  stats (optional): [0] rows rescored, [1] codes rescored.
constexpr float kVqPrefilterBound = 2.5e-4f;
// Coefficient cx of |x| in the half-width of the prefilter's error for x_pjt_in in layout x_layout
// (vq_rescore: bound = 2 (cx |x| + max|e| |x_r|) + 8 2^-24 (|x|^2 + max|e|^2)); dmax = max |e - bf16(e)|.
double vq_prefilter_cx(int x_layout, int ncodes, int dim, float emax, float dmax);
// vq_rescore arguments.  part_*: the prefilter's [rows][ntiles] partials; x: x_pjt_in fp32
// [rows][dim]; x2 / x2d: |x|^2 per row (row_sqnorm, fp32 / fp64); xr2 (optional): |x - bf16(x)|^2,
// required for vq_prefilter_b1's bound; e2d: |e|^2 per code in fp64; cx / emax / e2max: the bound
// (vq_prefilter_cx).  Workspace: pairs [cap] candidate list (cap a multiple of 8), cdist / ccode
// [cap / 8] per-chunk results, row_list [rows], npairs (zeroed by row_sqnorm before the prefilter).  stats (optional): [0] rows rescored, [1] codes rescored.
struct VqRescoreArgs {
  const float *part_val, *part_val2;
  const int* part_idx;
  long long rows;
  int ntiles, tile_codes, dim;
  const float *x, *x2, *xr2;
  const double* x2d;
  const float* codebook;
  const double* e2d;
  double cx;
  float emax, e2max;
  int32_t* codes;
  int* stats;
  int2* pairs;
  double* cdist;
  int* ccode;
  long long cap;
  int2* row_list;
  unsigned long long* npairs;
};
// the rescore's three launches, in this order (vq_certify lists, vq_pair_eval evaluates, vq_pair_reduce picks)
hipError_t launch_vq_certify(const VqRescoreArgs& a, hipStream_t s);
hipError_t launch_vq_pair_eval(const VqRescoreArgs& a, hipStream_t s);
hipError_t launch_vq_pair_reduce(const VqRescoreArgs& a, hipStream_t s);
hipError_t launch_vq_reduce(const float* part_val, const int* part_idx, int rows, int ntiles, int32_t* codes,
                            hipStream_t s);
// x2 (fp32) and optionally x2d (fp64) |x|^2, xr2 |x - bf16(x)|^2 per row; zero_me (optional) set to 0
hipError_t launch_row_sqnorm(const float* x, long long rows, int C, float* out, double* x2d, float* xr2,
                             unsigned long long* zero_me, hipStream_t s);
// y6c: y6 in the compact bf16 layout instead of planes; channels_first_form: 0 F.layer_norm, 1 the
// reference's channels_first LayerNorm, 2 the latter on a bf16 input under CUDA autocast.
// An h2 output (y6c == 3) is scaled per row by 2^h2_shift(the row's max |output|), that shift stored
// to ash_row[row] (required) and the max to amax_row[row] (may be null)
hipError_t launch_ln_rows(const float* x, float* y, unsigned short* y6, int y6c, const float* w, const float* b,
                          long long rows, int C, float eps, int channels_first_form, hipStream_t s,
                          int* ash_row = nullptr, float* amax_row = nullptr);
// bf16: the reference's CUDA autocast (DCX_GEMM_BF16): input, taps and bias rounded to bf16, the
// depthwise conv's result rounded to bf16, then the fp32 F.layer_norm
hipError_t launch_dwconv_ln(const float* x, float* y, unsigned short* y6, int y6c, const float* dww, const float* dwb,
                            const float* lnw, const float* lnb, int batch, int L, int C, int bf16, const Knobs* kn,
                            hipStream_t s, int* ash_row = nullptr, float* amax_row = nullptr);
// fp32 [rows][C] -> h2, each row scaled by 2^h2_shift(its max |x|), the shift to ash_row[row] (the
// input of a one-tap h3 conv handed in by the caller or written in fp32 by its producer)
hipError_t launch_h2_rows(const float* x, unsigned short* y6, long long rows, int C, int* ash_row, hipStream_t s);
// h3 activation range of a tensor handed in by the caller (round 6): amax[b] = max |x| over clip b's
// rows (batch clips of L rows, C channels; amax zeroed here first), then y6 = h2 of f(x) * 2^a with
// a = h2_shift(max(amax[b], floor)) stored to ash[b]; f = silu when silu != 0 (its |f(x)| <= |x|).
// yf (may be null) receives f(x) in fp32.
hipError_t launch_h2_ranged(const float* x, float* yf, unsigned short* y6, int batch, long long L, int C, int silu,
                            float floor, float* amax, int* ash, int* rflag, hipStream_t s);
// n 32-bit words zeroed by a kernel (capture-safe ordering; hipMemsetAsync is not used on the path)
hipError_t launch_zero_words(void* p, long long n, hipStream_t s);
// amax[b] = max |x| over clip b (batch clips of L rows, C channels), amax zeroed here first
hipError_t launch_clip_amax(const float* x, int batch, long long L, int C, float* amax, hipStream_t s);
// the CU count of the current device (cached per device, thread-safe)
int device_cus();
// x6 codebook planes -> the per-K32 hi/mid layout of vq_prefilter_bk ((dim / 32) * ncodes * 64 bf16)
hipError_t launch_repack_codebook_bk(const unsigned short* cb6, int ncodes, int dim, unsigned short* out,
                                     hipStream_t s);
// whether conv_gemm_bf16dm takes a one-tap conv of this shape (then its input may be compact)
bool bf16dm_takes(int cin, int cout, int lq, int ldx, int phases);
// whether vq_prefilter_bk takes the bf16-mode search (then x_pjt_in may be compact)
bool vq_bk_takes(int ncodes, int dim);
// whether vq_prefilter_dm takes the x6-mode search of `rows` rows with x_pjt_in in the "hm" layout
bool vq_hm_takes(int ncodes, int dim, long long rows);
hipError_t launch_frame_pad(const float* audio, float* frames, unsigned short* frames6, int batch, long long n, int rows,
                            int hop, int pad_left, hipStream_t s);
// h2: y6 in the h2 layout (dcx_planes.h) instead of planes
hipError_t launch_silu_act(const float* x, float* yf, unsigned short* y6, long long rows, int C, hipStream_t s,
                           int h2 = 0);
hipError_t launch_spec_mag(const float* spec, float* mag, unsigned short* mag6, float* loglin, long long rows, int nbins,
                           int ld_out, hipStream_t s);
hipError_t launch_split_planes(const float* x, unsigned short* y6, long long rows, int C, int compact, hipStream_t s);
hipError_t launch_gather_rows(const float* table, int ntable, const int32_t* idx, long long rows, int width,
                              float* out, int32_t* n_invalid, int masked_row, hipStream_t s);
hipError_t launch_conv_post_tanh(const float* x, const float* w, float bias, float* out, int batch, int L, int C,
                                 int k, int bf16, hipStream_t s);
hipError_t launch_transpose(const float* in, float* out, int batch, long long rows, long long cols, hipStream_t s);
hipError_t launch_resample_poly(const float* x, int batch, long long n_in, long long xs, const double* h, int hlen,
                                int up, int down, long long pre, float* y, long long n_out, long long ys,
                                hipStream_t s);

}  // namespace dcx

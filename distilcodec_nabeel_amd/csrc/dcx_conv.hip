// Implicit-GEMM 1-D convolution on gfx950 matrix cores.
//
// One kernel family serves every contraction on the DistilCodec path:
//   Conv1d k>1 / dilated (stem k7, conv_pre k13, ResBlock1 k3/7/11 x dil 1/3/5),
//   1x1 convs and nn.Linear (taps = 1), ConvTranspose1d as `stride` polyphase convs
//   (one tile range per phase, flat_tile), the STFT as a 4-tap conv over 256-sample rows, the mel matmul,
//   and the VQ distance GEMM (argmin epilogue, never materialising rows x 32768).
//
// GEMM view: rows = output time positions q (M), cols = output channels (N),
// K = taps x Cin.  Channels-last activations make every A-tile row a contiguous Cin slice and
// every store a contiguous Cout slice (coalesced).
//
// Two arithmetic modes, identical epilogues:
//  * conv_gemm_f32: v_mfma_f32_32x32x2_f32 (exact fp32 fmaf chain, 157 TF peak).
//  * conv_gemm_x6:  fp32-accurate 3-plane bf16 split.  Every fp32 operand x is held as
//    x = hi + mid + lo (three bf16, RNE; residual <= 2^-27|x|) and a product uses the six terms
//    hi*hi + hi*mid + mid*hi + hi*lo + mid*mid + lo*hi, each exact in fp32 (8x8-bit
//    significands), accumulated in fp32 by v_mfma_f32_32x32x16_bf16.  The dropped terms are
//    <= 2^-24 relative, i.e. fp32 rounding level; the MFMA ceiling is 16/6 = 2.67x the fp32 one.
//    Weights are split once at load; activations arrive already split (every producer writes
//    the planes, dcx_planes.h), so staging is a plain copy, and each staged input tile (with its
//    tap halo) serves every tap of the conv.
//
// MFMA fragment maps (cdna_hip_programming.md §3): 32x32x2 f32: lane l supplies A[l&31][k=l>>5]
// and B[k=l>>5][l&31]; 32x32x16 bf16: A[l&31][k=8(l>>5)+j], B[k=8(l>>5)+j][l&31], j<8;
// C/D for both: col=l&31, row=(r&3)+8*(r>>2)+4*(l>>5).
#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <type_traits>

#include "dcx_kernels.h"
#include "dcx_planes.h"

namespace dcx {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int BK = 16;    // K chunk per pipeline stage (both modes)
constexpr int LDSK = 20;  // f32 mode: padded LDS row (floats); 20*i mod 64 distinct per b128 group
// x6 mode LDS rows hold [half 2][plane 3][8] bf16 = 96 B of one row / column.  Two layouts, both
// conflict-free for ds_read_b128 of one piece by 16 lanes on 16 consecutive rows (any tap offset):
//  * padded (8-wave kernels): 112-byte rows, 28 r mod 64 distinct;
//  * swizzled (4-wave kernels, which must stay under 80 KB for two workgroups per CU): 96-byte
//    rows, and rows with bit 3 set store their two K halves swapped, so rows r and r+8 differ in
//    the parity of their 16-byte bank group (6 r + piece mod 16).  Measured 1-2 % slower than the
//    padded rows on the 8-wave kernels (the per-row XOR), hence only where LDS requires it.
template <bool SWZ>
struct XRow {
  static constexpr int kStride = SWZ ? 48 : 56;  // ushort
  __device__ static __forceinline__ int half(int row, int h) { return SWZ ? h ^ ((row >> 3) & 1) : h; }
  __device__ static __forceinline__ int off(int row, int piece) {  // piece = half * 3 + plane
    const int h = piece >= 3;
    return row * kStride + (half(row, h) * 3 + piece - 3 * h) * 8;
  }
};

// v * sigmoid(v) from v_exp_f32 and v_rcp_f32 (each ~1 ulp): 5 instructions instead of the
// library expf and an IEEE divide; silu(-inf side) -> -0, silu(+large) -> v.
__device__ __forceinline__ float silu_f(float v) { return v * __builtin_amdgcn_rcpf(1.0f + __expf(-v)); }
__device__ __forceinline__ float gelu_f(float v) { return 0.5f * v * (1.0f + erff(v * 0.70710678118654752440f)); }
// GELU of the bf16 mode, whose result is rounded to bf16 (2^-8 relative) right after: erf from
// the Chebyshev-fitted erfc of Numerical Recipes (erfcc, relative error < 1.2e-7 everywhere), one
// v_rcp_f32, one v_exp_f32 and 9 FMAs, branch-free.  ocml's erff branches on |x| (both paths run in
// mixed waves) and cost 9 of the 64 ms the bf16 1x1 convs take per C3 step (timing probe).  The x6
// mode uses it too (epilogue_lds and splitk_epi4 pick it for every planes-mode conv, p.w6): its
// absolute error against the fp64 GELU is 4.5e-7, below torch's fp32 erff GELU's 1.2e-6, so the
// fp32-level tolerances hold (tests/test_gpu_conv.py, 109 dB end to end).  Only the IEEE fp32-MFMA
// mode keeps the library erff.
__device__ __forceinline__ float gelu_bf16_f(float v) {
#ifdef DCX_GELU_ERF  // A/B builds: the library erff in the bf16 mode too
  return gelu_f(v);
#endif
  const float z = fabsf(v) * 0.70710678118654752440f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.5f, z, 1.0f));
  float q = 0.17087277f;
  q = fmaf(q, t, -0.82215223f);
  q = fmaf(q, t, 1.48851587f);
  q = fmaf(q, t, -1.13520398f);
  q = fmaf(q, t, 0.27886807f);
  q = fmaf(q, t, -0.18628806f);
  q = fmaf(q, t, 0.09678418f);
  q = fmaf(q, t, 0.37409196f);
  q = fmaf(q, t, 1.00002368f);
  const float c = t * __expf(fmaf(t, q, fmaf(-z, z, -1.26551223f)));  // erfc(|v| / sqrt 2)
  // erf(v / sqrt 2) rounded to fp32, then the reference's 0.5 v (1 + erf) with its cancellation
  // for large negative v (torch's GELU formula)
  const float e = v >= 0.0f ? 1.0f - c : c - 1.0f;
  return 0.5f * v * (1.0f + e);
}

// gelu_bf16_f on two values at once: the same operations in the same order (so the same bits), with
// the multiplies and FMAs as packed fp32 (v_pk_mul_f32 / v_pk_fma_f32, two lanes' worth per
// instruction); only v_rcp_f32 / v_exp_f32 and the sign select stay per value.  The bf16 1x1 convs'
// pwconv1 epilogue is bound by this VALU work (65 k GELUs per 256 x 256 tile).
__device__ __forceinline__ f32x2 gelu_bf16_f2(f32x2 v) {
#ifdef DCX_GELU_SCALAR  // A/B builds
  return f32x2{gelu_bf16_f(v[0]), gelu_bf16_f(v[1])};
#endif
  const f32x2 z = __builtin_elementwise_abs(v) * 0.70710678118654752440f;
  const f32x2 d = __builtin_elementwise_fma(f32x2{0.5f, 0.5f}, z, f32x2{1.0f, 1.0f});
  const f32x2 t = {__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
  auto fm = [&](f32x2 q, float c) { return __builtin_elementwise_fma(q, t, f32x2{c, c}); };
  f32x2 q = {0.17087277f, 0.17087277f};
  q = fm(q, -0.82215223f);
  q = fm(q, 1.48851587f);
  q = fm(q, -1.13520398f);
  q = fm(q, 0.27886807f);
  q = fm(q, -0.18628806f);
  q = fm(q, 0.09678418f);
  q = fm(q, 0.37409196f);
  q = fm(q, 1.00002368f);
  const f32x2 arg = __builtin_elementwise_fma(t, q, __builtin_elementwise_fma(-z, z, f32x2{-1.26551223f, -1.26551223f}));
  const f32x2 c = t * f32x2{__expf(arg[0]), __expf(arg[1])};
  const f32x2 e = {v[0] >= 0.0f ? 1.0f - c[0] : c[0] - 1.0f, v[1] >= 0.0f ? 1.0f - c[1] : c[1] - 1.0f};
  return 0.5f * v * (1.0f + e);
}

// The bf16 mode's GELU as a table (round 4).  Its input is a bf16 value (the GEMM result rounded
// after the bias) and its output is rounded to bf16 by the store, so GELU + rounding is a function
// of 16 bits.  conv_gemm_bf16dp tabulates it once per workgroup in LDS with gelu_bf16_f2 itself (so
// an entry is the evaluated result's bits) over the magnitudes [2^-31, 2^16): entry
// 2 (m - kGeluLo) + s = GELU of the bf16 (s << 15) | m, entry 2 kGeluN a sentinel that inputs
// outside the table read.  An element then costs half a packed convert, five packed 16-bit ops shared
// by two elements and a ds_read_u16, against ~18 VALU instructions evaluated (the pwconv1 epilogues
// were bound by that VALU work: 11.6 of their 28.7 ms per C3 step, DCX_DIAG_DUP).  A wave with an
// input outside the table (zeros, |x| < 2^-31 or >= 2^16, inf, NaN) stores the evaluated epilogue.
constexpr int kBf16dpBiasMax = 4096;  // conv_gemm_bf16dp: Cout bound (its bias lives in LDS)
constexpr int kGeluLo = 96 << 7, kGeluN = 47 << 7;  // bf16 magnitude bits [0x3000, 0x4780)
constexpr int kGeluLutUs = (2 * kGeluN + 1 + 7) / 8 * 8;  // ushorts, 16-byte multiple
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void gelu_lut_fill(unsigned short* lut, int tid, int nthreads) {
  for (int i = 2 * tid; i < 2 * kGeluN; i += 2 * nthreads) {  // (s = 0, s = 1) pairs of one m
    const int m = kGeluLo + (i >> 1);
    const f32x2 g = gelu_bf16_f2(f32x2{bf16_val((unsigned short)m), bf16_val((unsigned short)(0x8000 | m))});
    lut[i] = bf16_bits(g[0]);
    lut[i + 1] = bf16_bits(g[1]);
  }
  if (tid == 0) lut[2 * kGeluN] = 0xffff;
}
// GELU bits of two values rounded to bf16 here (the RNE of round_bf16x4) from the table at LDS byte
// address 0; `hi` keeps the largest table offset seen (>= 2 kGeluN: outside the table)
__device__ __forceinline__ unsigned gelu_lut2(const unsigned short* lut, f32x2 x, u16x2& hi) {
  const u16x2 r = __builtin_bit_cast(u16x2, __builtin_convertvector(x, bf16x2));
  const u16x2 key = (r << (unsigned short)1) | (r >> (unsigned short)15);  // 2 m + s
  const u16x2 t = key - (unsigned short)(2 * kGeluLo);                     // wraps below the table
  hi = __builtin_elementwise_max(hi, t);
  const u16x2 tc = __builtin_elementwise_min(t, u16x2{(unsigned short)(2 * kGeluN), (unsigned short)(2 * kGeluN)});
  const unsigned a = __builtin_bit_cast(unsigned, (u16x2)(tc << (unsigned short)1));  // byte offsets
#ifdef DCX_LUT_DIAG  // timing build: the table lookups left out (wrong results)
  return a ^ __builtin_bit_cast(unsigned, r);
#endif
  const char* const lb = reinterpret_cast<const char*>(lut);
  const unsigned lo16 = *reinterpret_cast<const unsigned short*>(lb + (a & 0xffff));
  const unsigned hi16 = *reinterpret_cast<const unsigned short*>(lb + (a >> 16));
  return lo16 | (hi16 << 16);
}

// XCD-aware bijective block remap (cdna_hip_programming.md §5 "XCD swizzle must be bijective"):
// blocks b and b+8 share an XCD, so consecutive logical tiles (same row panel, all column
// tiles) are dealt to the same XCD and share its L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// 1-D conv grids: tiles of (phase, clip, row tile, column tile), column tile fastest, XCD-remapped as
// one range, so the blocks of an XCD share input panels and weights across clips too.  (With a
// (tiles, batch, phases) grid, blockIdx.x & 7 is not the block's XCD unless tiles % 8 == 0.)
__device__ __forceinline__ void flat_tile(int tpc, int batch, int& wg, int& b, int& ph) {
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int per_ph = tpc * batch;
  ph = t / per_ph;
  const int r = t - ph * per_ph;
  b = r / tpc;
  wg = r - b * tpc;
}

// Split-K (ConvParams::ksplit > 1): the launch's clips are virtual, b = slice * clips + clip; slice
// `sl` owns the input-channel chunks [c0, c0 + nchunks) (whole units of kunit chunks, as even as
// the units allow) and writes its partial sums as clip b of the output (the caller's partial buffer).
__device__ __forceinline__ void ksplit_slice(const ConvParams& p, int b, int& clip, int& c0, int& nchunks) {
  clip = b;
  c0 = 0;
  nchunks = p.Cin / BK;
  if (p.ksplit > 1) {
    const int clips = p.batch / p.ksplit, sl = b / clips;
    clip = b - sl * clips;
    const int nunits = nchunks / p.kunit, base = nunits / p.ksplit, extra = nunits % p.ksplit;
    c0 = (sl * base + min(sl, extra)) * p.kunit;
    nchunks = (base + (sl < extra ? 1 : 0)) * p.kunit;
  }
}

// Zero page read in place of out-of-range input rows (conv zero padding): selecting the address
// instead of the loaded value keeps every staging load unconditional, so hipcc neither branches
// around it nor waits vmcnt(0) after it (cdna_hip_programming.md §5, trap 4(c)).
__device__ __attribute__((aligned(16))) float g_zero_row[32] = {0.f};

#ifdef DCX_CLOCK_DIAG
// Diagnostic build only: per-workgroup shader-clock and 100 MHz real-time ticks over the main
// loop, summed (in-kernel clock = sum(memtime) / sum(realtime) * 100 MHz).
__device__ unsigned long long g_clock_diag[3];
extern "C" int dcx_diag_clock(unsigned long long* out3, int reset) {
  if (hipMemcpyFromSymbol(out3, HIP_SYMBOL(g_clock_diag), sizeof(unsigned long long) * 3) != hipSuccess) return -1;
  if (reset) {
    const unsigned long long z[3] = {0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_clock_diag), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}
#endif
#ifdef DCX_SEG_DIAG
// Diagnostic build only: per-segment shader-clock sums of conv_gemm_x6pp's main loop, for wave 0
// (group 0, [0..5]) and wave 4 (group 1, [6..11]): MFMA issue, barrier wait, fragment-read issue,
// stores (with their vmcnt wait), loads + loop control, barrier wait; [12] steps.
__device__ unsigned long long g_seg_diag[13];
extern "C" int dcx_diag_seg(unsigned long long* out13, int reset) {
  if (hipMemcpyFromSymbol(out13, HIP_SYMBOL(g_seg_diag), sizeof(unsigned long long) * 13) != hipSuccess) return -1;
  if (reset) {
    const unsigned long long z[13] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_seg_diag), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}
// conv_gemm_x3dw: the same six sums for every wave of the workgroup, [wave * 6 + i], [48] steps
__device__ unsigned long long g_seg_diag8[49];
extern "C" int dcx_diag_seg8(unsigned long long* out49, int reset) {
  if (hipMemcpyFromSymbol(out49, HIP_SYMBOL(g_seg_diag8), sizeof(unsigned long long) * 49) != hipSuccess) return -1;
  if (reset) {
    const unsigned long long z[49] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_seg_diag8), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}
#define DCX_SEGT(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#else
#define DCX_SEGT(v)
#endif
#ifdef DCX_TILE_DIAG
// Diagnostic build only: per-workgroup 100 MHz real-time stamps of x6dq tiles (entry, main loop
// start, main loop end, exit) and the hardware ids of its CU (HW_ID, XCC_ID), in completion order.
constexpr int kTileDiagMax = 16384;
__device__ unsigned long long g_tile_diag[kTileDiagMax * 6];
__device__ unsigned int g_tile_cnt;
extern "C" int dcx_diag_tiles(unsigned long long* out, int max_tiles, int reset) {
  unsigned int n = 0;
  if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_tile_cnt), sizeof n) != hipSuccess) return -1;
  n = n < (unsigned)max_tiles ? n : (unsigned)max_tiles;
  n = n < (unsigned)kTileDiagMax ? n : (unsigned)kTileDiagMax;
  if (n && hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tile_diag), sizeof(unsigned long long) * 6 * n) != hipSuccess) return -1;
  if (reset) {
    const unsigned int z = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_tile_cnt), &z, sizeof z) != hipSuccess) return -1;
  }
  return (int)n;
}
#define DCX_TILET(v) const unsigned long long v = __builtin_amdgcn_s_memrealtime()
#else
#define DCX_TILET(v)
#endif

// ---------------------------------------------------------------------------------------------
// Conv epilogue through LDS: the accumulator tile is written to LDS (in row passes that fit the
// kernel's LDS), then each thread finishes 4 consecutive output channels of a row with 16-byte
// loads of bias / gamma / residual / mean accumulator and 16-byte fp32 stores (8-byte plane
// stores).  This keeps the per-element code out of the 64-way unrolled accumulator loop.
// ---------------------------------------------------------------------------------------------
// acc: f32x16[WR/32][WC/32] (32x32 MFMA blocks) or f32x4[WR/16][WC/16] (16x16 blocks).
// The epilogue's per-clip range values, read before a tile's main loop so that their memory round
// trips overlap its prologue instead of stalling the epilogue (round 6): the h2 output's shift from its
// bound program (stored to y_ash, non-finite bounds flagged) and the clip's running max |v| (acur).
struct EpiPre {
  int osh;
  float acur;
  bool track;
};
template <int RROW>
__device__ __forceinline__ EpiPre epi_range_pre(const ConvParams& p, const ConvParams& pr, int b) {
  EpiPre e{0, 0.f, false};
  const bool h2o = (p.y6 && p.y_compact == 3) || (p.y6s && p.y6s_h2);
  const bool h2row = (RROW & 2) && h2o && pr.yb.rowwise;
  if (h2o && !h2row) {
    const float bnd = range_bound(pr.yb, b);
    e.osh = __builtin_amdgcn_readfirstlane(h2_shift(bnd));
    if (threadIdx.x == 0) {
      if (pr.y_ash) pr.y_ash[b] = e.osh;
      if (pr.rflag && !(bnd <= 3.0e38f)) atomicOr(pr.rflag, RANGE_NONFINITE);
    }
  }
  const bool track = pr.y_amax != nullptr;
  e.track = track;
  e.acur = track && !h2row ? __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(
                                                           __builtin_bit_cast(int, range_cur(pr.y_amax, b))))
                           : 0.f;
  return e;
}

// RROW: which per-row range forms a kernel may meet (round 6).  Bit 0: an h2 input scaled per row
// (x_ash_row: the h3 one-tap kernels), loaded with the batch's rows; bit 1: a rowwise bound of an h2
// output (yb.rowwise: one-tap kernels).  Tap convs pass 0, which keeps these registers out of their
// epilogues (with them, round 6's first form spilled ~290 SGPRs into VGPR lanes in
// conv_gemm_x3dw_group: +5 % on the dominant kernel).  pr: where the range fields are read (the
// kernel argument itself in grouped launches, whose private copy then leaves them out).
template <int BM, int BN, int WM, int WN, int LDS_FLOATS, int NT, int RROW = 2, typename AccT>
__device__ __forceinline__ void epilogue_lds(const ConvParams& p, const ConvParams& pr, AccT& acc, int q0, int co0,
                                             int b, int ph, float* smem, const EpiPre* pre = nullptr) {
  constexpr int WR = BM / WM, WC = BN / WN;
  constexpr int TM = WR / 32, TN = WC / 32;
  constexpr bool M16 = sizeof(acc[0][0]) == 16;
  static_assert(sizeof(acc) == WR * WC * 4 / 64, "accumulator tile");
  constexpr int LDSW = BN + 4;
  constexpr int RPP = (BM * LDSW <= LDS_FLOATS) ? BM
                      : (BM / 2 * LDSW <= LDS_FLOATS) ? BM / 2
                      : (BM / 4 * LDSW <= LDS_FLOATS) ? BM / 4 : WR;
  static_assert(RPP % WR == 0 && RPP * LDSW <= LDS_FLOATS, "epilogue pass does not fit LDS");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int lrow = lane & 31, rhalf = 4 * (lane >> 5);
  const long long ob = (long long)b * p.y_bstride;
  unsigned short* y6 = p.y6 ? p.y6 + ob * (p.y_compact == 1 ? 1 : p.y_compact >= 2 ? 2 : 3) : nullptr;
  unsigned short* y6s = p.y6s ? p.y6s + ob * (p.y6s_h2 ? 2 : 3) : nullptr;
  // h2 output range (dcx_kernels.h h2_shift): the clip's scale from its bound program, the same in
  // every workgroup of the clip, or (pr.yb.rowwise, one-tap convs) each row's from its own bound
  // (wave-uniform values moved to scalar registers: the accumulators still occupy most VGPRs here)
  const bool h2o = (y6 && p.y_compact == 3) || (y6s && p.y6s_h2);
  constexpr bool RIN = RROW & 1, ROUT = RROW & 2;
  const bool h2row = ROUT && h2o && pr.yb.rowwise;
  int osh = 0;
  if (pre) {
    osh = pre->osh;
  } else if (h2o && !h2row) {
    const float bnd = range_bound(pr.yb, b);
    osh = __builtin_amdgcn_readfirstlane(h2_shift(bnd));
    if (tid == 0) {
      if (pr.y_ash) pr.y_ash[b] = osh;
      if (pr.rflag && !(bnd <= 3.0e38f)) atomicOr(pr.rflag, RANGE_NONFINITE);
    }
  }
  const float osc =
      __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, __builtin_ldexpf(1.0f, osh))));
#ifdef DCX_DIAG_NORANGE  // timing build: no range tracking in the epilogues (no maxima, no flags)
  const bool track = false;
#else
  // the clip's max |v| where a consumer's bound needs it; an h2 output checks its values against its
  // scale's limit only there (free: the max is taken anyway).  Elsewhere a finite value cannot pass
  // its bound (rigorous, from measured maxima), and a non-finite bound is flagged by the bound's own
  // evaluation (round 6: the per-element check cost ~1 VALU per element in every h2 epilogue)
  const bool track = pre ? pre->track : pr.y_amax != nullptr;
#endif
  const float acur = pre ? pre->acur : track && !h2row ? range_cur(pr.y_amax, b) : 0.f;  // the clip's running max (range_report)
  float vmax = 0.f;  // largest |v| this thread finishes (range_report)
  // Each thread finishes G consecutive output channels of a row (G = 8: 16-byte plane / compact
  // stores; the epilogue's store issue, not its bytes, sets its pace), the same channels for every
  // row, so bias and gamma are loaded once per tile.
#ifdef DCX_EPI4
  constexpr int G = 4;  // A/B builds: the round-2 form (8-byte plane stores)
#else
  constexpr int G = 8;
#endif
  constexpr int NH = G / 4;  // f32x4 halves per thread and row
  static_assert(NT % (BN / G) == 0, "each thread keeps one channel group");
  const int cg = (tid % (BN / G)) * G, trow = tid / (BN / G), co = co0 + cg;
  // LDS read order of the two halves: lanes with bit 3 set read the upper half first, which makes
  // both ds_read_b128 of a row conflict-free in every 16-lane group (MI355X_MICROARCH.md §LDS)
  const int hsw = G == 8 ? (lane >> 3) & 1 : 0;
  f32x4 bias4[NH], gamma4[NH];
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    bias4[h] = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + co + 4 * h) : f32x4{0.f, 0.f, 0.f, 0.f};
    gamma4[h] = p.epi == EPI_GAMMA_RES ? *reinterpret_cast<const f32x4*>(p.gamma + co + 4 * h) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
#ifdef DCX_DIAG_NOEPI
  if (q0 >= 0) return;  // timing-only build: main loop without the epilogue
#endif
#ifdef DCX_DIAG_DUP
  if (p.diag_skip == 2) return;  // the timing copy of a launch: main loop only
#endif
  // acc rows [r0, r0 + RPP) of the tile -> LDS
  auto stage_acc = [&](int r0) {
    __syncthreads();
    if (wm * WR >= r0 && wm * WR < r0 + RPP) {
      if constexpr (M16) {  // 16x16 block: lane holds column l & 15, rows 4 (l >> 4) + e
#pragma unroll
        for (int i = 0; i < WR / 16; ++i)
#pragma unroll
          for (int j = 0; j < WC / 16; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int row = wm * WR + i * 16 + 4 * (lane >> 4) + e - r0;
              smem[row * LDSW + wn * WC + j * 16 + (lane & 15)] = acc[i][j][e];
            }
      } else {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int row = wm * WR + i * 32 + (r & 3) + 8 * (r >> 2) + rhalf - r0;
              smem[row * LDSW + wn * WC + j * 32 + lrow] = acc[i][j][r];
            }
      }
    }
    __syncthreads();
  };
  // The residual / mean-accumulator rows of a batch are all loaded (unconditionally, past-the-end
  // rows clamped) before any of its stores, and the first batch of a pass before the pass's LDS
  // staging: with stores in flight hipcc can only wait with vmcnt(0), and conditional loads in a
  // rolled loop made it wait before every single load (one memory round trip per row).  The stores
  // may alias the loads (the in-place ResBlock state); each thread stores only elements it has
  // already loaded.
  constexpr int RSTEP = NT / (BN / G), ROWS_T = RPP / RSTEP;
  static_assert(RPP % RSTEP == 0, "epilogue rows per thread");
  const bool need_r = p.epi == EPI_GAMMA_RES || p.epi == EPI_RES;
  const bool need_m = p.mean_mode == MEAN_MID || p.mean_mode == MEAN_LAST;
  auto batch = [&](int r0, int rb, bool stage, auto ibt) {
    constexpr int IB = decltype(ibt)::value;
    f32x4 r[IB][NH], m[IB][NH];
    auto lofs = [&](int k) {
      const int q = min(q0 + r0 + trow + (rb + k) * RSTEP, p.Lq - 1);
      return ob + ((long long)q * p.out_mul + ph) * p.ldy + co;
    };
    if (need_r) {
#pragma unroll
      for (int k = 0; k < IB; ++k)
#pragma unroll
        for (int h = 0; h < NH; ++h) r[k][h] = *reinterpret_cast<const f32x4*>(p.res + lofs(k) + 4 * h);
    }
    if (need_m) {
#pragma unroll
      for (int k = 0; k < IB; ++k)
#pragma unroll
        for (int h = 0; h < NH; ++h) m[k][h] = *reinterpret_cast<const f32x4*>(p.macc + lofs(k) + 4 * h);
    }
    // per-row range data of a one-tap h3 conv (the input row's shift, the output row's bound), loaded
    // with the batch's other rows: inside the row loop each was a memory round trip
    // (a rowwise program has one term: prog_conv_rows)
    auto row_bound = [&](int q) { return fmaf(pr.yb.g[0], fmaxf(pr.yb.m[0][(long long)b * p.Lq + q], pr.yb.f[0]), pr.yb.c); };
    float rin[RIN ? IB : 1], rbnd[RIN ? IB : 1];
    if constexpr (RIN) {
#pragma unroll
      for (int k = 0; k < IB; ++k) {
        const int q = min(q0 + r0 + trow + (rb + k) * RSTEP, p.Lq - 1);
        rin[k] = pr.x_ash_row ? __builtin_ldexpf(1.0f, -pr.x_ash_row[(long long)b * p.Lin + q]) : 1.0f;
        rbnd[k] = h2row ? row_bound(q) : 0.f;
      }
    }
    if (stage) stage_acc(r0);
#pragma unroll
    for (int k = 0; k < IB; ++k) {
      const int rl = trow + (rb + k) * RSTEP;
      const int q = q0 + r0 + rl;
      if (q >= p.Lq) continue;
      const long long orow = (long long)q * p.out_mul + ph;
      const long long o = ob + orow * p.ldy + co;
      f32x4 x[NH];
      // a one-tap h3 conv's input scaled per row: undo the row's power of two (exact) before the bias
      const float rin_ = RIN ? rin[RIN ? k : 0] : 1.0f;
      if constexpr (NH == 2) {
        const f32x4 u = *reinterpret_cast<const f32x4*>(smem + rl * LDSW + cg + 4 * hsw);
        const f32x4 v = *reinterpret_cast<const f32x4*>(smem + rl * LDSW + cg + 4 * (1 - hsw));
        x[0] = (hsw ? v : u) * rin_ + bias4[0];
        x[1] = (hsw ? u : v) * rin_ + bias4[1];
      } else {
        x[0] = *reinterpret_cast<const f32x4*>(smem + rl * LDSW + cg) * rin_ + bias4[0];
      }
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        if (p.round_bf16) x[h] = round_bf16x4(x[h]);
        switch (p.epi) {
          case EPI_GELU:
            // planes modes (x6, bf16): the branch-free GELU (abs error 4.5e-7 against fp64, below
            // torch's fp32 erff GELU's 1.2e-6); the IEEE fp32 mode keeps erff
            if (p.w6) {
#ifndef DCX_EPI_NOGELU  // timing build: the bf16 GELU left out
#pragma unroll
              for (int e = 0; e < 4; e += 2) {
                const f32x2 g = gelu_bf16_f2(f32x2{x[h][e], x[h][e + 1]});
                x[h][e] = g[0];
                x[h][e + 1] = g[1];
              }
#endif
              // a compact-only output rounds to bf16 in its store (the same RNE bits)
              if (p.round_bf16 && (p.y || y6s || p.y2 || p.y_compact != 1)) x[h] = round_bf16x4(x[h]);
            } else {
#pragma unroll
              for (int e = 0; e < 4; ++e) x[h][e] = gelu_f(x[h][e]);
            }
            break;
          case EPI_GAMMA_RES: x[h] = r[k][h] + gamma4[h] * x[h]; break;
          case EPI_RES:  // bf16 mode: ResBlock1's `xt + x` of two bf16 tensors is bf16
            x[h] = r[k][h] + x[h];
            if (p.round_bf16) x[h] = round_bf16x4(x[h]);
            break;
          case EPI_LOGCLAMP:
#pragma unroll
            for (int e = 0; e < 4; ++e) x[h][e] = logf(fmaxf(x[h][e], 1e-5f));
            break;
          default: break;
        }
      }
#ifdef DCX_EPI_NOSTORE  // timing build: every output computed, (practically) none stored
      if (x[0][0] != -0x1.234p-100f) continue;
#endif
#ifdef DCX_DIAG_DUP  // the timing copy of a launch: every output computed, (practically) none stored
      if (p.diag_skip == 1 && x[0][0] != -0x1.234p-100f) continue;
#endif
      if (p.mean_mode == MEAN_FIRST) {
#pragma unroll
        for (int h = 0; h < NH; ++h) *reinterpret_cast<f32x4*>(p.macc + o + 4 * h) = x[h];
        continue;
      } else if (p.mean_mode == MEAN_MID) {
#pragma unroll
        for (int h = 0; h < NH; ++h) *reinterpret_cast<f32x4*>(p.macc + o + 4 * h) = m[k][h] + x[h];
        continue;
      } else if (p.mean_mode == MEAN_LAST) {
#pragma unroll
        for (int h = 0; h < NH; ++h) {  // bf16 mode: stack(...).mean(0) of bf16 tensors is bf16
          x[h] = (m[k][h] + x[h]) / 3.0f;
          if (p.round_bf16) x[h] = round_bf16x4(x[h]);
        }
      }
      float rsc = osc;  // the h2 output's scale for this row
      if (h2row) {
        const long long grow = (long long)b * p.Lq + q;
        const float bnd = RIN ? rbnd[RIN ? k : 0] : row_bound(q);
        const int sh = h2_shift(bnd);
        rsc = __builtin_ldexpf(1.0f, sh);
        if (cg == 0 && pr.y_ash) pr.y_ash[grow] = sh;
        if (pr.rflag && !(bnd <= 3.0e38f)) atomicOr(pr.rflag, RANGE_NONFINITE);
      }
      if (track) {  // per-row scales: the scaled values against 65504 (range_report)
        const float ts = h2row ? rsc : 1.0f;
#pragma unroll
        for (int h = 0; h < NH; ++h)
#pragma unroll
          for (int e = 0; e < 4; ++e) vmax = fmaxf(vmax, fabsf(x[h][e]) * ts);
      }
      if (p.y) {
#pragma unroll
        for (int h = 0; h < NH; ++h) *reinterpret_cast<f32x4*>(p.y + o + 4 * h) = x[h];
      }
      if constexpr (G == 8) {
        float xv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) xv[e] = x[e >> 2][e & 3];
        if (y6) {
          if (p.y_compact == 1) store_bf16x8(y6, orow, p.Cout, co, xv);
          else if (p.y_compact == 2) store_hm8(y6, orow, p.Cout, co, xv);
          else if (p.y_compact == 3) store_h2_8<false>(y6, orow, p.Cout, co, xv, rsc);
          else store_planes8(y6, orow, p.Cout, co, xv);
        }
        if (p.y2 || y6s) {
          float sv[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) sv[e] = p.round_bf16 ? bf16_val(bf16_bits(silu_f(xv[e]))) : silu_f(xv[e]);
          if (p.y2) {
            *reinterpret_cast<f32x4*>(p.y2 + o) = f32x4{sv[0], sv[1], sv[2], sv[3]};
            *reinterpret_cast<f32x4*>(p.y2 + o + 4) = f32x4{sv[4], sv[5], sv[6], sv[7]};
          }
          if (y6s) {
            if (p.y6s_h2) store_h2_8<false>(y6s, orow, p.Cout, co, sv, rsc);
            else store_planes8(y6s, orow, p.Cout, co, sv);
          }
        }
      } else {
        if (y6) {
          if (p.y_compact == 1) store_bf16x4(y6, orow, p.Cout, co, x[0][0], x[0][1], x[0][2], x[0][3]);
          else if (p.y_compact == 2) store_hm4(y6, orow, p.Cout, co, x[0][0], x[0][1], x[0][2], x[0][3]);
          else if (p.y_compact == 3) store_h2_4<false>(y6, orow, p.Cout, co, x[0][0], x[0][1], x[0][2], x[0][3], rsc);
          else store_planes4(y6, orow, p.Cout, co, x[0][0], x[0][1], x[0][2], x[0][3]);
        }
        if (p.y2 || y6s) {
          f32x4 sv;
#pragma unroll
          for (int e = 0; e < 4; ++e) sv[e] = p.round_bf16 ? bf16_val(bf16_bits(silu_f(x[0][e]))) : silu_f(x[0][e]);
          if (p.y2) *reinterpret_cast<f32x4*>(p.y2 + o) = sv;
          if (y6s) {
            if (p.y6s_h2) store_h2_4<false>(y6s, orow, p.Cout, co, sv[0], sv[1], sv[2], sv[3], rsc);
            else store_planes4(y6s, orow, p.Cout, co, sv[0], sv[1], sv[2], sv[3]);
          }
        }
      }
    }
  };
  // batches of 8 rows (4 when both the residual and the mean accumulator are loaded), halved for
  // 8-channel groups (the same registers)
  // (the largest batch within the cap that divides the rows per thread: 6 rows -> 3 + 3)
  constexpr int IBF0 = 8 / NH, IBM0 = 4 / NH;
  constexpr auto div_cap = [](int n, int cap) {
    int d = n < cap ? n : cap;
    while (n % d) --d;
    return d;
  };
  constexpr int IBF = div_cap(ROWS_T, IBF0), IBM = div_cap(ROWS_T, IBM0);
  static_assert(ROWS_T % IBF == 0 && ROWS_T % IBM == 0, "epilogue batches");
#pragma unroll 1
  for (int r0 = 0; r0 < BM; r0 += RPP) {
    if (need_m) {
#pragma unroll
      for (int rb = 0; rb < ROWS_T; rb += IBM) batch(r0, rb, rb == 0, std::integral_constant<int, IBM>{});
    } else {
#pragma unroll
      for (int rb = 0; rb < ROWS_T; rb += IBF) batch(r0, rb, rb == 0, std::integral_constant<int, IBF>{});
    }
  }
  // (rowwise: vmax holds scaled values, and pr.y_amax is not recorded)
  if (track)  // workgroup-uniform; the staging area is free after the last pass
    range_report_wg(vmax, h2row ? nullptr : pr.y_amax, b, h2row ? 65504.0f : h2o ? 65504.0f / osc : __builtin_inff(),
                    pr.rflag, acur, smem, NT);
}

// ---------------------------------------------------------------------------------------------
// Split-K reduce: v = bias + sum of the K-slices' partial sums (in slice order), then the epilogue
// of epilogue_lds element by element (one thread per 4 output channels of a row).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void splitk_epi4(const ConvParams& p, const float* __restrict__ part, int splits,
                                            long long stride, long long i4) {
  const int c4n = p.Cout / 4;
  const long long rowi = i4 / c4n;  // (phase, clip, q)
  const int co = (int)(i4 - rowi * c4n) * 4;
  const long long per_ph = (long long)p.batch * p.Lq;
  const int ph = (int)(rowi / per_ph);
  const long long r2 = rowi - ph * per_ph;
  const int b = (int)(r2 / p.Lq), q = (int)(r2 - (long long)b * p.Lq);
  const long long ob = (long long)b * p.y_bstride;
  const long long orow = (long long)q * p.out_mul + ph;
  const long long o = ob + orow * p.ldy + co;
  f32x4 x = *reinterpret_cast<const f32x4*>(part + o);
  for (int s = 1; s < splits; ++s) x += *reinterpret_cast<const f32x4*>(part + s * stride + o);
  if (p.bias) x += *reinterpret_cast<const f32x4*>(p.bias + co);
  if (p.round_bf16) x = round_bf16x4(x);
  switch (p.epi) {
    case EPI_GELU:
#pragma unroll
      for (int e = 0; e < 4; ++e) x[e] = p.w6 ? gelu_bf16_f(x[e]) : gelu_f(x[e]);
      if (p.round_bf16) x = round_bf16x4(x);
      break;
    case EPI_GAMMA_RES:
      x = *reinterpret_cast<const f32x4*>(p.res + o) + *reinterpret_cast<const f32x4*>(p.gamma + co) * x;
      break;
    case EPI_RES: x = *reinterpret_cast<const f32x4*>(p.res + o) + x; break;
    case EPI_LOGCLAMP:
#pragma unroll
      for (int e = 0; e < 4; ++e) x[e] = logf(fmaxf(x[e], 1e-5f));
      break;
    default: break;
  }
  if (p.mean_mode == MEAN_FIRST) {
    *reinterpret_cast<f32x4*>(p.macc + o) = x;
    return;
  } else if (p.mean_mode == MEAN_MID) {
    *reinterpret_cast<f32x4*>(p.macc + o) = *reinterpret_cast<const f32x4*>(p.macc + o) + x;
    return;
  } else if (p.mean_mode == MEAN_LAST) {
    x = (*reinterpret_cast<const f32x4*>(p.macc + o) + x) / 3.0f;
  }
  if (p.y) *reinterpret_cast<f32x4*>(p.y + o) = x;
  // h2 outputs (not produced in the split-K mode, which runs no h3 conv; kept consistent): the clip's
  // range scale (epilogue_lds); no maxima are recorded here
  const float osc = (p.y6 && p.y_compact == 3) || (p.y6s && p.y6s_h2)
                        ? __builtin_ldexpf(1.0f, h2_shift(range_bound(p.yb, b))) : 1.0f;
  if (p.y6) {
    unsigned short* y6 = p.y6 + ob * (p.y_compact == 1 ? 1 : p.y_compact >= 2 ? 2 : 3);
    if (p.y_compact == 1) store_bf16x4(y6, orow, p.Cout, co, x[0], x[1], x[2], x[3]);
    else if (p.y_compact == 2) store_hm4(y6, orow, p.Cout, co, x[0], x[1], x[2], x[3]);
    else if (p.y_compact == 3) store_h2_4(y6, orow, p.Cout, co, x[0], x[1], x[2], x[3], osc);
    else store_planes4(y6, orow, p.Cout, co, x[0], x[1], x[2], x[3]);
  }
  if (p.y2 || p.y6s) {
    f32x4 sv;
#pragma unroll
    for (int e = 0; e < 4; ++e) sv[e] = silu_f(x[e]);
    if (p.y2) *reinterpret_cast<f32x4*>(p.y2 + o) = sv;
    if (p.y6s && p.y6s_h2) store_h2_4(p.y6s + ob * 2, orow, p.Cout, co, sv[0], sv[1], sv[2], sv[3], osc);
    else if (p.y6s) store_planes4(p.y6s + ob * 3, orow, p.Cout, co, sv[0], sv[1], sv[2], sv[3]);
  }
}

__global__ void __launch_bounds__(256) splitk_epilogue_kernel(const ConvParams p, const float* __restrict__ part,
                                                              int splits, long long stride, long long total4) {
  const long long i4 = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i4 < total4) splitk_epi4(p, part, splits, stride, i4);
}

// the reduces of a grouped split-K launch in one grid (member k: blocks [start[k], start[k + 1]))
__global__ void __launch_bounds__(256) splitk_epilogue_group_kernel(const SplitEpiGroup g) {
  const int t = blockIdx.x;
  const int k = t >= g.start[1] ? (t >= g.start[2] ? 2 : 1) : 0;
  const long long i4 = (long long)(t - g.start[k]) * 256 + threadIdx.x;
  if (i4 >= g.total4[k]) return;
  if (g.chain) {  // g.chain members, one range of blocks (member 0's), every member in order
    splitk_epi4(g.p[0], g.part[0], g.splits[0], g.stride[0], i4);
    if (g.chain > 1) splitk_epi4(g.p[1], g.part[1], g.splits[1], g.stride[1], i4);
    if (g.chain > 2) splitk_epi4(g.p[2], g.part[2], g.splits[2], g.stride[2], i4);
    return;
  }
  if (k == 0) splitk_epi4(g.p[0], g.part[0], g.splits[0], g.stride[0], i4);
  else if (k == 1) splitk_epi4(g.p[1], g.part[1], g.splits[1], g.stride[1], i4);
  else splitk_epi4(g.p[2], g.part[2], g.splits[2], g.stride[2], i4);
}

// ---------------------------------------------------------------------------------------------
// VQ search epilogue (registers): per-row argmin of the distance tile.
// ---------------------------------------------------------------------------------------------
template <int BM, int BN, int WM, int WN, bool ARGMIN>
__device__ __forceinline__ void epilogue(const ConvParams& p, f32x16 (&acc)[BM / WM / 32][BN / WN / 32], int q0,
                                         int co0, int nt, int ntiles, int b, int ph, float* smem) {
  constexpr int WR = BM / WM, WC = BN / WN;
  constexpr int TM = WR / 32, TN = WC / 32;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int lrow = lane & 31;
  const int rhalf = 4 * (lane >> 5);
  static_assert(ARGMIN, "register epilogue is the VQ search's; convs use epilogue_lds");
  {
    // VQ search: dist = sqrt(clamp((|x|^2 + |e|^2) + (-2 x.e), 0)) exactly in the reference's
    // operation order (vector_quantize_pytorch.py:41-45); per row keep the smallest distance,
    // lowest code index on ties (torch argmax of -dist returns the first).
    __syncthreads();
    float* rv = smem;                                  // [WN][BM]
    int* ri = reinterpret_cast<int*>(smem + WN * BM);  // [WN][BM]
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rloc = wm * WR + i * 32 + (r & 3) + 8 * (r >> 2) + rhalf;
        const int q = q0 + rloc;
        const float xx = (q < p.Lq) ? p.x2[(long long)b * p.Lq + q] : 0.f;
        float bv = __builtin_inff();
        int bi = 0x7fffffff;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int co = co0 + wn * WC + j * 32 + lrow;
          const float d2 = (xx + p.e2[co]) + (-2.0f * acc[i][j][r]);
          const float d = sqrtf(fmaxf(d2, 0.0f));
          if (d < bv || (d == bv && co < bi)) { bv = d; bi = co; }
        }
#pragma unroll
        for (int off = 16; off >= 1; off >>= 1) {
          const float ov = __shfl_xor(bv, off, 64);
          const int oi = __shfl_xor(bi, off, 64);
          if (ov < bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
        }
        if (lrow == 0) { rv[wn * BM + rloc] = bv; ri[wn * BM + rloc] = bi; }
      }
    }
    __syncthreads();
    for (int rloc = tid; rloc < BM; rloc += 256) {
      const int q = q0 + rloc;
      if (q >= p.Lq) continue;
      float bv = rv[rloc];
      int bi = ri[rloc];
#pragma unroll
      for (int w = 1; w < WN; ++w) {
        const float ov = rv[w * BM + rloc];
        const int oi = ri[w * BM + rloc];
        if (ov < bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
      }
      const long long o = ((long long)b * p.Lq + q) * ntiles + nt;
      p.part_val[o] = bv;
      p.part_idx[o] = bi;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// VQ prefilter epilogue: per row of the tile, the smallest and second-smallest approximate
// squared distance (x2 + e2) - 2 x.e and the code of the smallest (lowest index on ties).
// vq_rescore_kernel (dcx_misc.hip) certifies the winner or rescores the candidates from these.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void top2_merge(float& v1, int& i1, float& v2, float ov1, int oi1, float ov2) {
  if (ov1 < v1 || (ov1 == v1 && oi1 < i1)) {
    v2 = fminf(v1, ov2);
    v1 = ov1;
    i1 = oi1;
  } else {
    v2 = fminf(v2, ov1);
  }
}

// top2_merge as selects (no divergent branch: the epilogues run it on every lane), same results
__device__ __forceinline__ void top2_merge_sel(float& v1, int& i1, float& v2, float ov1, int oi1, float ov2) {
  const bool take = (ov1 < v1) | ((ov1 == v1) & (oi1 < i1));  // (bitwise: no short-circuit branch)
  const float nv2 = take ? fminf(v1, ov2) : fminf(v2, ov1);
  v1 = take ? ov1 : v1;
  i1 = take ? oi1 : i1;
  v2 = nv2;
}
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) { return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, false); }
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, dpp_i<CTRL>(__builtin_bit_cast(int, v)));
}
template <int CTRL>
__device__ __forceinline__ void top2_dpp_step(float& v1, int& i1, float& v2) {
  top2_merge_sel(v1, i1, v2, dpp_f<CTRL>(v1), dpp_i<CTRL>(i1), dpp_f<CTRL>(v2));
}
// the top 2 over the 16 lanes of a DPP row (lanes 16 k .. 16 k + 15), left in every lane of it: quad
// xor 1, quad xor 2 (quad_perm), then the half-row mirror (quad 0 <-> 1, 2 <-> 3) and the row mirror
// (the two halves); VALU moves instead of four ds_bpermute round trips per value
__device__ __forceinline__ void top2_row16(float& v1, int& i1, float& v2) {
  top2_dpp_step<0xB1>(v1, i1, v2);   // quad_perm [1, 0, 3, 2]
  top2_dpp_step<0x4E>(v1, i1, v2);   // quad_perm [2, 3, 0, 1]
  top2_dpp_step<0x141>(v1, i1, v2);  // row_half_mirror
  top2_dpp_step<0x140>(v1, i1, v2);  // row_mirror
}

template <int BM, int BN, int WM, int WN>
__device__ __forceinline__ void epilogue_top2(const ConvParams& p, f32x16 (&acc)[BM / WM / 32][BN / WN / 32], int q0,
                                              int co0, int nt, int ntiles, float* smem) {
  constexpr int WR = BM / WM, WC = BN / WN;
  constexpr int TM = WR / 32, TN = WC / 32;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int lrow = lane & 31;
  const int rhalf = 4 * (lane >> 5);
  // every |x|^2 and |e|^2 this lane needs, loaded up front (unconditional, row index clamped: rows
  // past Lq are never stored), so their latency is paid once rather than once per row
  float xxv[TM][16], e2v[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r)
      xxv[i][r] = p.x2[min(q0 + wm * WR + i * 32 + (r & 3) + 8 * (r >> 2) + rhalf, p.Lq - 1)];
#pragma unroll
  for (int j = 0; j < TN; ++j) e2v[j] = p.e2[co0 + wn * WC + j * 32 + lrow];
  __syncthreads();
  float* rv = smem;                                      // [WN][BM]
  float* rv2 = smem + WN * BM;                           // [WN][BM]
  int* ri = reinterpret_cast<int*>(smem + 2 * WN * BM);  // [WN][BM]
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rloc = wm * WR + i * 32 + (r & 3) + 8 * (r >> 2) + rhalf;
      const float xx = xxv[i][r];
      float v1 = __builtin_inff(), v2 = __builtin_inff();
      int i1 = 0x7fffffff;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int co = co0 + wn * WC + j * 32 + lrow;
        const float d2 = (xx + e2v[j]) + (-2.0f * acc[i][j][r]);
        top2_merge(v1, i1, v2, d2, co, __builtin_inff());
      }
#pragma unroll
      for (int off = 16; off >= 1; off >>= 1)
        top2_merge(v1, i1, v2, __shfl_xor(v1, off, 64), __shfl_xor(i1, off, 64), __shfl_xor(v2, off, 64));
      if (lrow == 0) {
        rv[wn * BM + rloc] = v1;
        rv2[wn * BM + rloc] = v2;
        ri[wn * BM + rloc] = i1;
      }
    }
  }
  __syncthreads();
  for (int rloc = tid; rloc < BM; rloc += blockDim.x) {
    const int q = q0 + rloc;
    if (q >= p.Lq) continue;
    float v1 = rv[rloc], v2 = rv2[rloc];
    int i1 = ri[rloc];
#pragma unroll
    for (int w = 1; w < WN; ++w) top2_merge(v1, i1, v2, rv[w * BM + rloc], ri[w * BM + rloc], rv2[w * BM + rloc]);
    const long long o = (long long)q * ntiles + nt;
    p.part_val[o] = v1;
    p.part_val2[o] = v2;
    p.part_idx[o] = i1;
  }
}

// ---------------------------------------------------------------------------------------------
// fp32 MFMA kernel.  Register-staged double buffer, one barrier per 16-deep K chunk.
// ---------------------------------------------------------------------------------------------
template <int BM, int BN, int WM, int WN, bool ARGMIN>
__global__ void __launch_bounds__(256) conv_gemm_f32(const ConvParams p) {
  static_assert(WM * WN == 4, "4 waves per workgroup");
  constexpr int WR = BM / WM, WC = BN / WN;
  constexpr int TM = WR / 32, TN = WC / 32;
  static_assert(TM >= 1 && TN >= 1 && WR % 32 == 0 && WC % 32 == 0, "wave tile");
  constexpr int A_F4 = BM * (BK / 4), B_F4 = BN * (BK / 4);
  constexpr int A_PT = (A_F4 + 255) / 256, B_PT = (B_F4 + 255) / 256;

  __shared__ __attribute__((aligned(16))) float smem[2 * (BM + BN) * LDSK];
  float(*As)[BM][LDSK] = reinterpret_cast<float(*)[BM][LDSK]>(smem);
  float(*Bs)[BN][LDSK] = reinterpret_cast<float(*)[BN][LDSK]>(smem + 2 * BM * LDSK);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int ntiles = p.Cout / BN;
  int wg, b, ph;
  flat_tile(((p.Lq + BM - 1) / BM) * ntiles, p.batch, wg, b, ph);
  const int mt = wg / ntiles, nt = wg - mt * ntiles;
  const int q0 = mt * BM, co0 = nt * BN;
  const float* __restrict__ xb = p.x + (long long)b * p.x_bstride;
  const float* __restrict__ wp = p.w + (long long)ph * p.w_phase_stride + (long long)co0 * p.taps * p.Cin;
  const int inb = p.in_base[ph];
  const int kchunks = p.Cin / BK;
  const int nk = p.taps * kchunks;
  const long long wrow = (long long)p.taps * p.Cin;

  f32x4 ra[A_PT], rb[B_PT];

  auto gload = [&](int kt) {
    const int m = kt / kchunks;
    const int ci0 = (kt - m * kchunks) * BK;
    const int shift = inb + m * p.in_step;
#pragma unroll
    for (int i = 0; i < A_PT; ++i) {
      const int idx = tid + 256 * i;
      ra[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (A_F4 % 256 == 0 || idx < A_F4) {
        const int row = idx >> 2, c4 = idx & 3;
        const int q = q0 + row, ir = q + shift;
        if (q < p.Lq && ir >= 0 && ir < p.Lin)
          ra[i] = *reinterpret_cast<const f32x4*>(xb + (long long)ir * p.ldx + ci0 + c4 * 4);
      }
    }
#pragma unroll
    for (int i = 0; i < B_PT; ++i) {
      const int idx = tid + 256 * i;
      if (B_F4 % 256 == 0 || idx < B_F4) {
        const int row = idx >> 2, c4 = idx & 3;
        rb[i] = *reinterpret_cast<const f32x4*>(wp + (long long)row * wrow + m * p.Cin + ci0 + c4 * 4);
      }
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_PT; ++i) {
      const int idx = tid + 256 * i;
      if (A_F4 % 256 == 0 || idx < A_F4) *reinterpret_cast<f32x4*>(&As[buf][idx >> 2][(idx & 3) * 4]) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_PT; ++i) {
      const int idx = tid + 256 * i;
      if (B_F4 % 256 == 0 || idx < B_F4) *reinterpret_cast<f32x4*>(&Bs[buf][idx >> 2][(idx & 3) * 4]) = rb[i];
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  gload(0);
  sstore(0);
  __syncthreads();

  const int kof = (lane >> 5) * 8;
  const int lrow = lane & 31;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
    f32x4 a0[TM], a1[TM], b0[TN], b1[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const float* ap = &As[buf][wm * WR + i * 32 + lrow][kof];
      a0[i] = *reinterpret_cast<const f32x4*>(ap);
      a1[i] = *reinterpret_cast<const f32x4*>(ap + 4);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const float* bp = &Bs[buf][wn * WC + j * 32 + lrow][kof];
      b0[j] = *reinterpret_cast<const f32x4*>(bp);
      b1[j] = *reinterpret_cast<const f32x4*>(bp + 4);
    }
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[i][s], b0[j][s], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[i][s], b1[j][s], acc[i][j], 0, 0, 0);
    if (kt + 1 < nk) sstore(buf ^ 1);
    __syncthreads();
  }
  if constexpr (ARGMIN)
    epilogue<BM, BN, WM, WN, true>(p, acc, q0, co0, nt, ntiles, b, ph, smem);
  else
    epilogue_lds<BM, BN, WM, WN, 2 * (BM + BN) * LDSK, 256>(p, p, acc, q0, co0, b, ph, smem);
}

// ---------------------------------------------------------------------------------------------
// x6 kernel, WM x WN = 8 waves (512 threads) or 4 waves (256 threads, two workgroups per CU for
// the small-Cout tiles); 2 waves per SIMD either way.  Block tile 256 x 128 has wave tile 64 x 64.
// Same arithmetic and LDS images as conv_gemm_x6; the loads run two K16 steps ahead of their use
// (two register sets, loop unrolled by two), so a step's MFMAs (2 waves x 24 per SIMD = 1536
// cycles) cover the L2 / Infinity-Cache latency of the tiles two steps out.
// ---------------------------------------------------------------------------------------------
// AF32: the input is fp32 (p.x6 == nullptr) and is split into planes while staging (4 channels
// per 16-byte load, three 8-byte LDS stores).  Used for the small-Cout convs (Cout <= 64, Cin <= 128),
// which are bound by HBM traffic (planes cost 6 B per element against 4) and whose planes-input
// variant would need more than 256 VGPRs.
template <int BM, int BN, int WM, int WN, int HALO, bool ARGMIN, int PROD = 6, bool AF32 = false>
__global__ void __launch_bounds__(64 * WM * WN, 2) conv_gemm_x6w8(const ConvParams p) {
  static_assert(WM * WN == 8 || WM * WN == 4, "4 or 8 waves per workgroup");
  static_assert(PROD == 6 || PROD == 1, "x6 or bf16 products");
  constexpr int NT = 64 * WM * WN;
  using XR = XRow<WM * WN == 4>;
  constexpr int XROW = XR::kStride;
  // staged 16-byte pieces per row per K chunk: all (half, plane) pairs, or the two hi pieces
  constexpr int NPC = PROD == 6 ? 6 : 2;
  constexpr int NPL = PROD == 6 ? 3 : 1;  // planes read into fragments
  constexpr int APC = AF32 ? 4 : NPC;     // staged 16-byte pieces per input row per K chunk
  constexpr int WR = BM / WM, WC = BN / WN;
  constexpr int TM = WR / 32, TN = WC / 32;
  constexpr int AROWS = BM + HALO;
  constexpr int A_P = AROWS * APC;  // 16-byte pieces of a staged input tile
  constexpr int B_P = BN * NPC;
  constexpr int A_PT = (A_P + NT - 1) / NT, B_PT = (B_P + NT - 1) / NT;
  constexpr int ABUF = AROWS * XROW, BBUF = BN * XROW;

  // LDS: input tiles (2, by chunk parity) + weight-tile ring (3, by step mod 3).
  __shared__ __attribute__((aligned(16))) unsigned short lds[2 * ABUF + 3 * BBUF];

  static_assert(!ARGMIN, "x6 VQ search uses vq_prefilter_x3");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const long long ldx6 = (long long)p.ldx * 3;
  const int nchunks = p.Cin / BK;
  const int wchunks = nchunks;
  const int taps = p.taps;
  const int nsteps = nchunks * taps;
  const int lo_rel = p.in_step < 0 ? (taps - 1) * p.in_step : 0;
  const long long wslab = (long long)p.Cout * 48;
  const int lin = p.Lin;

  // Persistent tiles.  Iteration `it` of block w takes logical tile
  //   it * G + (w & 7) * (G / 8) + (w >> 3)      (G = gridDim.x, a multiple of 8)
  // so the blocks of one XCD (w & 7 equal) work on G/8 consecutive tiles, column tiles fastest,
  // i.e. they share input row panels in their L2.  Logical tiles run over
  // (phase, clip, row tile, column tile).
  const int ntn = p.Cout / BN, mtiles = (p.Lq + BM - 1) / BM;
  const int per_img = mtiles * ntn, total = per_img * p.batch * p.phases;
  const int G = gridDim.x;
  const int tile_base = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  int q0 = 0, co0 = 0, b = 0, ph = 0, row0 = 0;
  const unsigned short* __restrict__ xb6 = nullptr;
  const float* __restrict__ xbf = nullptr;
  const unsigned short* __restrict__ wbase = nullptr;
  auto setup = [&](int L) {
    ph = L / (per_img * p.batch);
    const int rem = L - ph * per_img * p.batch;
    b = rem / per_img;
    const int wg = rem - b * per_img;
    const int mt = wg / ntn, nt = wg - mt * ntn;
    q0 = mt * BM;
    co0 = nt * BN;
    row0 = q0 + p.in_base[ph] + lo_rel;
    if constexpr (AF32) xbf = p.x + (long long)b * p.x_bstride;
    else xb6 = p.x6 + (long long)b * p.x_bstride * 3;
    wbase = p.w6 + ((long long)ph * taps * wchunks) * p.Cout * 48 + (long long)co0 * 48;
  };
  int L = tile_base;
  if (L >= total) return;  // whole workgroup, before any barrier
  setup(L);

  // Branch-free staging slots (surplus slots duplicate the last element).
  int a_row[A_PT], a_k[A_PT], a_lds[A_PT];
#pragma unroll
  for (int i = 0; i < A_PT; ++i) {
    const int idx = min(tid + NT * i, A_P - 1);
    a_row[i] = idx / APC;
    a_k[i] = idx - a_row[i] * APC;
    if constexpr (AF32) {  // a_k = 4-channel group; LDS: its half's hi plane + (a_k & 1) * 4
      a_lds[i] = XR::off(a_row[i], (a_k[i] >> 1) * 3) + (a_k[i] & 1) * 4;
    } else {
      if (PROD == 1) a_k[i] *= 3;  // piece = half * 3 + plane
      a_lds[i] = XR::off(a_row[i], a_k[i]);
    }
  }
  int b_off[B_PT], b_lds[B_PT];
#pragma unroll
  for (int i = 0; i < B_PT; ++i) {
    const int idx = min(tid + NT * i, B_P - 1);
    const int col = idx / NPC, piece = (idx - col * NPC) * (PROD == 1 ? 3 : 1);
    b_off[i] = (col * 6 + piece) * 8;
    b_lds[i] = XR::off(col, piece);
  }

  // With a tap halo (taps >= 2) at most one input-chunk load is in flight, so one register set
  // suffices; 1-tap convs load a chunk every step and alternate two sets.
  constexpr int RA_SETS = HALO > 0 ? 1 : 2;
  f32x4 ra[RA_SETS][A_PT];
  f32x4 rb[2][B_PT];

  auto loadA = [&](int c, f32x4(&r)[A_PT]) {
#pragma unroll
    for (int i = 0; i < A_PT; ++i) {
      const int ir = row0 + a_row[i];
      const bool ok = ir >= 0 && ir < lin;
      if constexpr (AF32) {
        const float* src = ok ? xbf + (long long)ir * p.ldx + c * 16 + a_k[i] * 4 : g_zero_row;
        r[i] = *reinterpret_cast<const f32x4*>(src);
      } else {
        const unsigned short* src =
            ok ? xb6 + (long long)ir * ldx6 + c * 48 + a_k[i] * 8 : reinterpret_cast<const unsigned short*>(g_zero_row);
        r[i] = *reinterpret_cast<const f32x4*>(src);
      }
    }
  };
  auto storeA = [&](int buf, const f32x4(&r)[A_PT]) {
    unsigned short* A = lds + buf * ABUF;
#pragma unroll
    for (int i = 0; i < A_PT; ++i) {
      if constexpr (AF32) {
        s16x4 hv, mv, lv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          unsigned short hb, mb, lb;
          split3(p.silu_in ? silu_f(r[i][e]) : r[i][e], hb, mb, lb);  // silu(0) = 0: padding stays 0
          hv[e] = (short)hb;
          mv[e] = (short)mb;
          lv[e] = (short)lb;
        }
        *reinterpret_cast<s16x4*>(A + a_lds[i]) = hv;
        if constexpr (PROD == 6) {
          *reinterpret_cast<s16x4*>(A + a_lds[i] + 8) = mv;
          *reinterpret_cast<s16x4*>(A + a_lds[i] + 16) = lv;
        }
      } else {
        *reinterpret_cast<f32x4*>(A + a_lds[i]) = r[i];
      }
    }
  };
  auto loadB = [&](int c, int m, f32x4(&r)[B_PT]) {
    const unsigned short* src = wbase + ((long long)m * wchunks + c) * wslab;
#pragma unroll
    for (int i = 0; i < B_PT; ++i) r[i] = *reinterpret_cast<const f32x4*>(src + b_off[i]);
  };
  auto storeB = [&](int slot, const f32x4(&r)[B_PT]) {
    unsigned short* Bsm = lds + 2 * ABUF + slot * BBUF;
#pragma unroll
    for (int i = 0; i < B_PT; ++i) *reinterpret_cast<f32x4*>(Bsm + b_lds[i]) = r[i];
  };

  const int lrow = lane & 31;
  const int khalf = lane >> 5;
  int b_frag[TN];  // LDS offsets of this lane's weight-fragment rows (bit 3 is fixed per lane)
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int cc = wn * WC + j * 32 + lrow;
    b_frag[j] = cc * XROW + XR::half(cc, khalf) * 24;
  }
  s16x8 af[2][TM][3], bfr[2][TN][3];
  // fragments of step (c, m) in ring slot `slot` -> register set F
  auto readF = [&](int c, int m, int slot, s16x8(&a)[TM][3], s16x8(&bb)[TN][3]) {
    const int off = m * p.in_step - lo_rel;
    const unsigned short* A = lds + (c & 1) * ABUF;
    const unsigned short* Bsm = lds + 2 * ABUF + slot * BBUF;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int rr = wm * WR + i * 32 + lrow + off;
      const unsigned short* ap = A + rr * XROW + XR::half(rr, khalf) * 24;
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl) a[i][pl] = *reinterpret_cast<const s16x8*>(ap + pl * 8);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const unsigned short* bp = Bsm + b_frag[j];
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl) bb[j][pl] = *reinterpret_cast<const s16x8*>(bp + pl * 8);
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto adv = [&](int& c_, int& m_) {
    if (++m_ == taps) { m_ = 0; ++c_; }
  };
  // step positions (chunk, tap) of s+1, s+2, s+3 and the ring slot of step s
  int c1, m1, c2, m2, c3, m3, slot;
  // ---- prologue, part 1 (issued before the previous tile's epilogue): A(0), B(0), B(1), and
  //      for 1-tap convs A(1), into the staging registers
  const int s1c = taps > 1 ? 0 : 1, s1m = taps > 1 ? 1 : 0;  // position of step 1 (nsteps >= 2)
  auto prologue_loads = [&]() {
    loadA(0, ra[0]);
    if constexpr (HALO == 0) loadA(1 < nchunks ? 1 : 0, ra[1 % RA_SETS]);
    loadB(0, 0, rb[0]);
    loadB(s1c, s1m, rb[1]);
  };
  // ---- part 2: to LDS, then the loads in flight for the first loop step: the input chunk
  //      staged next (1-tap: the one first used at step 2; with a halo: chunk 1, held in
  //      registers until step taps - 2 stores it) and B(2)
  auto prologue_stores = [&]() {
    storeA(0, ra[0]);
    if constexpr (HALO == 0) storeA(1, ra[1 % RA_SETS]);
    storeB(0, rb[0]);
    storeB(1, rb[1]);
    c1 = s1c;
    m1 = s1m;
    c2 = c1;
    m2 = m1;
    adv(c2, m2);
    c3 = c2;
    m3 = m2;
    adv(c3, m3);
    slot = 0;
    if constexpr (HALO > 0) {
      if (nchunks > 1) loadA(1, ra[0]);
    } else {
      if (m2 == 0 && c2 < nchunks) loadA(c2, ra[1 % RA_SETS]);
    }
    loadB(min(c2, nchunks - 1), c2 < nchunks ? m2 : taps - 1, rb[1]);
    __syncthreads();
    readF(0, 0, 0, af[0], bfr[0]);
  };
  prologue_loads();

  auto step = [&](int s, auto qtag) {
    constexpr int Q = decltype(qtag)::value;
    const int slot1 = slot == 2 ? 0 : slot + 1, slot2 = slot1 == 2 ? 0 : slot1 + 1;
    // 1. fragments of step s+1 (its data was made visible by the previous barrier; after the
    //    last step this reads unused LDS, which keeps the step free of branches)
    readF(c1, m1, slot1, af[1 - Q], bfr[1 - Q]);
    // 2. global loads: the input chunk first (so the compiler's merged wait for a chunk store never
    //    covers this step's weight loads), then B for step s+3.  1-tap: the chunk first used at
    //    step s+3.  With a halo: chunk c1 + 1 on the last step of a chunk, taps - 1 steps before
    //    step (c1, taps - 2) stores it (one register set: the previous chunk is stored by then).
    if constexpr (HALO > 0) {
      if (m1 == 0 && c1 + 1 < nchunks) loadA(c1 + 1, ra[0]);
    } else {
      if (m3 == 0 && c3 < nchunks) loadA(c3, ra[Q % RA_SETS]);
    }
    loadB(min(c3, nchunks - 1), c3 < nchunks ? m3 : taps - 1, rb[Q]);
    // 3. MFMAs of step s
#define DCX_MF(i, j, x, y) \
  acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, af[Q][i][x]), \
                                                      __builtin_bit_cast(bf16x8, bfr[Q][j][y]), acc[i][j], 0, 0, 0)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (PROD == 6) {
          DCX_MF(i, j, 2, 0);
          DCX_MF(i, j, 1, 1);
          DCX_MF(i, j, 0, 2);
          DCX_MF(i, j, 1, 0);
          DCX_MF(i, j, 0, 1);
        }
        DCX_MF(i, j, 0, 0);
      }
#undef DCX_MF
    // 4. stage step s+2: weight tile into its ring slot; its input chunk if s+2 opens one
    storeB(slot2, rb[1 - Q]);
    if (m2 == 0 && c2 < nchunks) storeA(c2 & 1, ra[(1 - Q) % RA_SETS]);
    __syncthreads();
    adv(c1, m1);
    adv(c2, m2);
    adv(c3, m3);
    slot = slot1;
  };
  for (;;) {
    prologue_stores();
    // nsteps is even (launcher): without an odd exit the loop header never merges a path on which
    // this iteration's loads are still in flight, which made the waitcnt pass emit vmcnt(0).
#ifdef DCX_CLOCK_DIAG
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
#endif
    for (int s = 0; s < nsteps; s += 2) {
      step(s, std::integral_constant<int, 0>{});
      step(s + 1, std::integral_constant<int, 1>{});
    }
#ifdef DCX_CLOCK_DIAG
    if (threadIdx.x == 0) {
      atomicAdd(&g_clock_diag[0], __builtin_amdgcn_s_memtime() - t0);
      atomicAdd(&g_clock_diag[1], __builtin_amdgcn_s_memrealtime() - r0);
      atomicAdd(&g_clock_diag[2], (unsigned long long)nsteps);
    }
#endif
    // the next tile's first loads go out before this tile's epilogue, which hides their latency
    const int eq0 = q0, eco0 = co0, eb = b, eph = ph;
    const int Ln = L + G;
    const bool more = Ln < total;  // uniform over the workgroup
    if (more) {
      setup(Ln);
      prologue_loads();
    }
    epilogue_lds<BM, BN, WM, WN, (2 * ABUF + 3 * BBUF) / 2, NT, HALO ? 0 : 2>(p, p, acc, eq0, eco0, eb, eph,
                                                                reinterpret_cast<float*>(lds));
    if (!more) break;
    L = Ln;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    __syncthreads();  // the epilogue's LDS reads are done before the next prologue writes LDS
  }
}

// ---------------------------------------------------------------------------------------------
// Ping-pong x6 conv kernel for the dominant shape (256 x 128 tile, tap halo, planes input).
//
// The two waves on each SIMD (wave w and w + 4) belong to different groups: group 0 = waves 0-3
// (tile rows 0-127), group 1 = waves 4-7 (rows 128-255).  Segments are separated by barriers that
// all 8 waves execute; group 0 runs  MFMA(s) | MEM0(s)  and group 1 runs  MEM1(s) | MFMA(s),  so
// in every segment one wave per SIMD issues its 24 MFMAs while its partner reads fragments,
// stores staged tiles and issues global loads, and the matrix pipe no longer idles while both
// waves of a SIMD do their memory work at the same time (conv_gemm_x6w8: ~1/3 of each step).
//
// Segment k = 2s: group 0 MFMA(s), group 1 MEM1(s);  k = 2s+1: group 0 MEM0(s), group 1 MFMA(s).
//   MEM0(s): fragments of step s+1; store its half of step s+2; load its half of step s+3.
//   MEM1(s): fragments of step s;   store its half of step s+1; load its half of step s+2.
// Step t's data is complete after segment 2t-2 and is read in segments 2t-1 (group 0) and 2t
// (group 1), so the weight ring needs only 2 slots (t & 1): step t+2 is written in segments 2t+1
// and 2t+2.  Input tiles are double-buffered by chunk parity and follow the schedule of their
// chunk's first step.  Each group stages half of every tile (both halves with the same maps).
// ---------------------------------------------------------------------------------------------
// AF32 (Cout = 64, fp32 input split while staging, as conv_gemm_x6w4f): 512 x 64 tiles, 8 x 1
// waves with the same 64 x 64 wave tiles, so the staging VALU of one group overlaps the other
// group's MFMAs.
template <int HALO, int BN, bool AF32 = false>
__device__ __forceinline__ void x6pp_tile(const ConvParams& p, const ConvParams& pr, const int wg, const int b, const int ph) {
  // wave tiles 64 x (BN / 2): 24 MFMAs per segment at BN = 128
  static_assert(BN == 128 || BN == 256 || (AF32 && BN == 64), "column tile");
  constexpr int BM = AF32 ? 512 : 256, WN = AF32 ? 1 : 2, WM = 8 / WN;
  constexpr int WR = 64, WC = BN / WN, TM = 2, TN = WC / 32;
  constexpr int XROW = 56;  // padded 112-byte rows
  constexpr int AROWS = BM + HALO;
  constexpr int APC = AF32 ? 4 : 6;  // staged 16-byte pieces per input row per chunk
  constexpr int A_P = AROWS * APC, B_P = BN * 6;        // 16-byte pieces per tile
  constexpr int A_H = A_P / 2, B_H = B_P / 2;           // per group
  constexpr int A_PT = (A_H + 255) / 256, B_PT = (B_H + 255) / 256;
  constexpr int ABUF = AROWS * XROW, BBUF = BN * XROW;
  static_assert(A_P % 2 == 0 && B_P % 2 == 0, "halves");
  __shared__ __attribute__((aligned(16))) unsigned short lds[2 * ABUF + 2 * BBUF];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int group = __builtin_amdgcn_readfirstlane(tid >> 8), gt = tid & 255;
  const int wm = wave / WN, wn = wave % WN;
  const int ntiles = p.Cout / BN;
  const int mt = wg / ntiles, nt = wg - mt * ntiles;
  const int q0 = mt * BM, co0 = nt * BN;
  int clip, c0, nchunks;
  ksplit_slice(p, b, clip, c0, nchunks);  // split-K slice (AF32 launches never split)
  const unsigned short* __restrict__ xb6 = AF32 ? nullptr : p.x6 + (long long)clip * p.x_bstride * 3 + c0 * 48;
  const float* __restrict__ xbf = AF32 ? p.x + (long long)clip * p.x_bstride : nullptr;
  const long long ldx6 = (long long)p.ldx * 3;
  const int wchunks = p.Cin / BK;  // weight layout
  const int taps = p.taps;
  const int nsteps = nchunks * taps;
  const int lo_rel = p.in_step < 0 ? (taps - 1) * p.in_step : 0;
  const int row0 = q0 + p.in_base[ph] + lo_rel;
  const unsigned short* __restrict__ wbase =
      p.w6 + ((long long)ph * taps * wchunks + c0) * p.Cout * 48 + (long long)co0 * 48;
  const long long wslab = (long long)p.Cout * 48;
  const int lin = p.Lin;

  // this thread's staging slots in its group's half of each tile (surplus slots repeat the last)
  int a_row[A_PT], a_k[A_PT], b_off[B_PT], b_lds[B_PT];
#pragma unroll
  for (int i = 0; i < A_PT; ++i) {
    const int idx = group * A_H + min(gt + 256 * i, A_H - 1);
    a_row[i] = idx / APC;
    a_k[i] = idx - a_row[i] * APC;  // AF32: 4-channel group
  }
#pragma unroll
  for (int i = 0; i < B_PT; ++i) {
    const int idx = group * B_H + min(gt + 256 * i, B_H - 1);
    const int col = idx / 6, piece = idx - col * 6;
    b_off[i] = idx * 8;
    b_lds[i] = col * XROW + piece * 8;
  }
  f32x4 ra[A_PT], rb[B_PT];
  auto loadA = [&](int c) {
#pragma unroll
    for (int i = 0; i < A_PT; ++i) {
      const int ir = row0 + a_row[i];
      const bool ok = ir >= 0 && ir < lin;
      if constexpr (AF32) {
        const float* src = ok ? xbf + (long long)ir * p.ldx + c * 16 + a_k[i] * 4 : g_zero_row;
        ra[i] = *reinterpret_cast<const f32x4*>(src);
      } else {
        const unsigned short* src =
            ok ? xb6 + (long long)ir * ldx6 + c * 48 + a_k[i] * 8 : reinterpret_cast<const unsigned short*>(g_zero_row);
        ra[i] = *reinterpret_cast<const f32x4*>(src);
      }
    }
  };
  auto storeA = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_PT; ++i) {
      if constexpr (AF32) {  // silu (optional) and the 3-plane split of 4 channels: three 8-byte stores
        s16x4 hv, mv, lv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          unsigned short hb, mb, lb;
          split3(p.silu_in ? silu_f(ra[i][e]) : ra[i][e], hb, mb, lb);  // silu(0) = 0: padding stays 0
          hv[e] = (short)hb;
          mv[e] = (short)mb;
          lv[e] = (short)lb;
        }
        unsigned short* d = lds + buf * ABUF + a_row[i] * XROW + (a_k[i] >> 1) * 24 + (a_k[i] & 1) * 4;
        *reinterpret_cast<s16x4*>(d) = hv;
        *reinterpret_cast<s16x4*>(d + 8) = mv;
        *reinterpret_cast<s16x4*>(d + 16) = lv;
      } else {
        *reinterpret_cast<f32x4*>(lds + buf * ABUF + a_row[i] * XROW + a_k[i] * 8) = ra[i];
      }
    }
  };
  auto loadB = [&](int c, int m) {
    const unsigned short* src = wbase + ((long long)m * wchunks + c) * wslab;
#pragma unroll
    for (int i = 0; i < B_PT; ++i) rb[i] = *reinterpret_cast<const f32x4*>(src + b_off[i]);
  };
  auto storeB = [&](int slot) {
#pragma unroll
    for (int i = 0; i < B_PT; ++i) *reinterpret_cast<f32x4*>(lds + 2 * ABUF + slot * BBUF + b_lds[i]) = rb[i];
  };

  const int lrow = lane & 31, hoff = (lane >> 5) * 24;
  s16x8 af[TM][3], bfr[TN][3];
  auto readF = [&](int c, int m, int slot) {
    const int off = m * p.in_step - lo_rel;
    const unsigned short* A = lds + (c & 1) * ABUF;
    const unsigned short* Bsm = lds + 2 * ABUF + slot * BBUF;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const unsigned short* ap = A + (wm * WR + i * 32 + lrow + off) * XROW + hoff;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) af[i][pl] = *reinterpret_cast<const s16x8*>(ap + pl * 8);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const unsigned short* bp = Bsm + (wn * WC + j * 32 + lrow) * XROW + hoff;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) bfr[j][pl] = *reinterpret_cast<const s16x8*>(bp + pl * 8);
    }
  };
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  // s_setprio around the cluster keeps hipcc from moving MFMAs across the segment barriers
  // (cdna_hip_programming.md T5), which would collapse the ping-pong
  auto mfma = [&]() {
    __builtin_amdgcn_s_setprio(1);
#define DCX_MF(i, j, x, y) \
  acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, af[i][x]), \
                                                      __builtin_bit_cast(bf16x8, bfr[j][y]), acc[i][j], 0, 0, 0)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        DCX_MF(i, j, 2, 0);
        DCX_MF(i, j, 1, 1);
        DCX_MF(i, j, 0, 2);
        DCX_MF(i, j, 1, 0);
        DCX_MF(i, j, 0, 1);
        DCX_MF(i, j, 0, 0);
      }
#undef DCX_MF
    __builtin_amdgcn_s_setprio(0);
  };
  auto adv = [&](int& c_, int& m_) {
    if (++m_ == taps) { m_ = 0; ++c_; }
  };

  // ---- prologue: both groups stage their halves of A(0), B(0), B(1); A(1) when step 1 opens it
  loadA(0);
  loadB(0, 0);
  storeA(0);
  storeB(0);
  int c1 = 0, m1 = 0;  // position of step 1
  adv(c1, m1);
  loadB(c1, m1);
  storeB(1);
  if (m1 == 0) {  // taps == 1
    loadA(1);
    storeA(1);
  }
  // position of the step this group stores next (group 0: step 2 in MEM0(0); group 1: step 2 in
  // MEM1(1)) and of the step it reads next; both groups start their loads for step 2
  int cw = c1, mw = m1;
  adv(cw, mw);                        // step 2
  int cl = cw, ml = mw;               // next load: step 2
  if (nsteps > 2) {
    loadB(cl, ml);
    if (ml == 0) loadA(cl);
  }
  adv(cl, ml);                        // step 3
  __syncthreads();
#ifdef DCX_CLOCK_DIAG
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
#endif
  int cr = 0, mr = 0;                 // position of the step whose fragments are read next
#ifdef DCX_SEG_DIAG
  unsigned long long sd[6] = {}, tprev = 0;
#endif
  if (group == 0) {
    readF(0, 0, 0);
    adv(cr, mr);                      // group 0 reads step 1 in MEM0(0)
    for (int s = 0; s < nsteps; ++s) {
      DCX_SEGT(ta);
#ifdef DCX_SEG_DIAG
      if (s) sd[5] += ta - tprev;
#endif
      mfma();                         // MFMA(s)
      DCX_SEGT(tb);
      __syncthreads();
      DCX_SEGT(tc);
      // MEM0(s): fragments of step s+1, store step s+2, load step s+3 (issuing the loads before
      // the fragment reads was slower: 2480 vs 2048 cycles per step at k11)
      if (s + 1 < nsteps) readF(cr, mr, (s + 1) & 1);
      DCX_SEGT(tc1);
      if (s + 2 < nsteps) {
        storeB((s + 2) & 1);
        if (mw == 0) storeA(cw & 1);
      }
      DCX_SEGT(tc2);
      if (s + 3 < nsteps) {
        loadB(cl, ml);
        if (ml == 0) loadA(cl);
      }
      adv(cr, mr);
      adv(cw, mw);
      adv(cl, ml);
      DCX_SEGT(td);
      __syncthreads();
#ifdef DCX_SEG_DIAG
      sd[0] += tb - ta;
      sd[1] += tc - tb;
      sd[2] += tc1 - tc;
      sd[3] += tc2 - tc1;
      sd[4] += td - tc2;
      tprev = td;
#endif
    }
  } else {
    for (int s = 0; s < nsteps; ++s) {
      // MEM1(s): fragments of step s, store step s+1 (steps 0, 1 came from the prologue),
      // load step s+2 (step 2 was loaded in the prologue)
      DCX_SEGT(ta);
#ifdef DCX_SEG_DIAG
      if (s) sd[1] += ta - tprev;
#endif
      readF(cr, mr, s & 1);
      DCX_SEGT(ta1);
      if (s >= 1 && s + 1 < nsteps) {
        storeB((s + 1) & 1);
        if (mw == 0) storeA(cw & 1);
        adv(cw, mw);
      }
      DCX_SEGT(ta2);
      if (s >= 1 && s + 2 < nsteps) {
        loadB(cl, ml);
        if (ml == 0) loadA(cl);
        adv(cl, ml);
      }
      adv(cr, mr);
      DCX_SEGT(tb);
      __syncthreads();
      DCX_SEGT(tc);
      mfma();                         // MFMA(s)
      DCX_SEGT(td);
      __syncthreads();
#ifdef DCX_SEG_DIAG
      sd[2] += ta1 - ta;
      sd[3] += ta2 - ta1;
      sd[4] += tb - ta2;
      sd[5] += tc - tb;
      sd[0] += td - tc;
      tprev = td;
#endif
    }
  }
#ifdef DCX_SEG_DIAG
  if ((threadIdx.x & 255) == 0) {
    const int o = group * 6;
#pragma unroll
    for (int i = 0; i < 6; ++i) atomicAdd(&g_seg_diag[o + i], sd[i]);
    if (group == 0) atomicAdd(&g_seg_diag[12], (unsigned long long)nsteps);
  }
#endif
#ifdef DCX_CLOCK_DIAG
  if (threadIdx.x == 0) {
    atomicAdd(&g_clock_diag[0], __builtin_amdgcn_s_memtime() - t0);
    atomicAdd(&g_clock_diag[1], __builtin_amdgcn_s_memrealtime() - r0);
    atomicAdd(&g_clock_diag[2], (unsigned long long)nsteps);
  }
#endif
  epilogue_lds<BM, BN, WM, WN, (2 * ABUF + 2 * BBUF) / 2, 512, HALO ? 0 : 2>(p, pr, acc, q0, co0, b, ph, reinterpret_cast<float*>(lds));
}

// ---------------------------------------------------------------------------------------------
// conv_gemm_x6lm: conv_gemm_x6pp with the global loads moved into the MFMA segments.
//
// Per-segment stamps of conv_gemm_x6pp (tools/seg_diag.py) show its MEM segment, not the MFMA
// segment, setting the pace: at k11 a wave spends ~310 cycles issuing its 12 fragment reads,
// ~180 on its LDS stores and ~570 issuing 2-6 global loads behind them, against ~800 for 24
// MFMAs, so the MFMA wave then waits ~250-450 cycles at the barrier.  Here each wave issues its
// next loads at the head of its MFMA segment, while its SIMD partner is the one using LDS, into
// a second staging register set: step t is loaded in MFMA(t - 3) into set t & 1 and stored by
// group 0 in MEM0(t - 2), by group 1 in MEM1(t - 1) (three segments of latency cover either way).
// The loop is unrolled by two so the register sets are static.  Input-chunk loads (conditional)
// go before the weight loads (unconditional, index clamped at the tail), so the weight loads are
// always the youngest and the stores' vmcnt waits stay counted.
// ---------------------------------------------------------------------------------------------
template <int HALO>
__global__ void __launch_bounds__(512, 2) conv_gemm_x6lm(const ConvParams p) {
  constexpr int BM = 256, BN = 128, WN = 2;
  constexpr int WR = 64, WC = BN / WN, TM = 2, TN = WC / 32;
  constexpr int XROW = 56;  // padded 112-byte rows
  constexpr int AROWS = BM + HALO;
  constexpr int A_P = AROWS * 6, B_P = BN * 6;
  constexpr int A_H = A_P / 2, B_H = B_P / 2;
  constexpr int A_PT = (A_H + 255) / 256, B_PT = (B_H + 255) / 256;
  constexpr int ABUF = AROWS * XROW, BBUF = BN * XROW;
  __shared__ __attribute__((aligned(16))) unsigned short lds[2 * ABUF + 2 * BBUF];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int group = __builtin_amdgcn_readfirstlane(tid >> 8), gt = tid & 255;
  const int wm = wave / WN, wn = wave % WN;
  const int ntiles = p.Cout / BN;
  int wg, b, ph;
  flat_tile(((p.Lq + BM - 1) / BM) * ntiles, p.batch, wg, b, ph);
  const int mt = wg / ntiles, nt = wg - mt * ntiles;
  const int q0 = mt * BM, co0 = nt * BN;
  int clip, c0, nchunks;
  ksplit_slice(p, b, clip, c0, nchunks);  // split-K slice
  const unsigned short* __restrict__ xb6 = p.x6 + (long long)clip * p.x_bstride * 3 + c0 * 48;
  const long long ldx6 = (long long)p.ldx * 3;
  const int wchunks = p.Cin / BK;  // weight layout
  const int taps = p.taps;
  const int nsteps = nchunks * taps;
  const int lo_rel = p.in_step < 0 ? (taps - 1) * p.in_step : 0;
  const int row0 = q0 + p.in_base[ph] + lo_rel;
  const unsigned short* __restrict__ wbase =
      p.w6 + ((long long)ph * taps * wchunks + c0) * p.Cout * 48 + (long long)co0 * 48;
  const long long wslab = (long long)p.Cout * 48;
  const int lin = p.Lin;

  int a_row[A_PT], a_k[A_PT], b_off[B_PT], b_lds[B_PT];
#pragma unroll
  for (int i = 0; i < A_PT; ++i) {
    const int idx = group * A_H + min(gt + 256 * i, A_H - 1);
    a_row[i] = idx / 6;
    a_k[i] = idx - a_row[i] * 6;
  }
#pragma unroll
  for (int i = 0; i < B_PT; ++i) {
    const int idx = group * B_H + min(gt + 256 * i, B_H - 1);
    const int col = idx / 6, piece = idx - col * 6;
    b_off[i] = idx * 8;
    b_lds[i] = col * XROW + piece * 8;
  }
  f32x4 ra[2][A_PT], rb[2][B_PT];
  auto loadA = [&](int c, f32x4(&r)[A_PT]) {
#pragma unroll
    for (int i = 0; i < A_PT; ++i) {
      const int ir = row0 + a_row[i];
      const bool ok = ir >= 0 && ir < lin;
      const unsigned short* src =
          ok ? xb6 + (long long)ir * ldx6 + c * 48 + a_k[i] * 8 : reinterpret_cast<const unsigned short*>(g_zero_row);
      r[i] = *reinterpret_cast<const f32x4*>(src);
    }
  };
  auto storeA = [&](int buf, const f32x4(&r)[A_PT]) {
#pragma unroll
    for (int i = 0; i < A_PT; ++i)
      *reinterpret_cast<f32x4*>(lds + buf * ABUF + a_row[i] * XROW + a_k[i] * 8) = r[i];
  };
  auto loadB = [&](int c, int m, f32x4(&r)[B_PT]) {
    const unsigned short* src = wbase + ((long long)m * wchunks + c) * wslab;
#pragma unroll
    for (int i = 0; i < B_PT; ++i) r[i] = *reinterpret_cast<const f32x4*>(src + b_off[i]);
  };
  auto storeB = [&](int slot, const f32x4(&r)[B_PT]) {
#pragma unroll
    for (int i = 0; i < B_PT; ++i) *reinterpret_cast<f32x4*>(lds + 2 * ABUF + slot * BBUF + b_lds[i]) = r[i];
  };

  const int lrow = lane & 31, hoff = (lane >> 5) * 24;
  s16x8 af[TM][3], bfr[TN][3];
  auto readF = [&](int c, int m, int slot) {
    const int off = m * p.in_step - lo_rel;
    const unsigned short* A = lds + (c & 1) * ABUF;
    const unsigned short* Bsm = lds + 2 * ABUF + slot * BBUF;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const unsigned short* ap = A + (wm * WR + i * 32 + lrow + off) * XROW + hoff;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) af[i][pl] = *reinterpret_cast<const s16x8*>(ap + pl * 8);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const unsigned short* bp = Bsm + (wn * WC + j * 32 + lrow) * XROW + hoff;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) bfr[j][pl] = *reinterpret_cast<const s16x8*>(bp + pl * 8);
    }
  };
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  // MFMA cluster of one step with the staging loads `ld` spread through it: NL loads, one after
  // every 24 / (NL + 1) MFMAs (sched_group_barrier pins the order), so their issue overlaps MFMAs
  // instead of holding back the first one
  auto mfma_with = [&](auto nl_tag, auto&& ld) {
    constexpr int NL = decltype(nl_tag)::value;
    __builtin_amdgcn_s_setprio(1);
    ld();
#define DCX_MF(i, j, x, y) \
  acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, af[i][x]), \
                                                      __builtin_bit_cast(bf16x8, bfr[j][y]), acc[i][j], 0, 0, 0)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        DCX_MF(i, j, 2, 0);
        DCX_MF(i, j, 1, 1);
        DCX_MF(i, j, 0, 2);
        DCX_MF(i, j, 1, 0);
        DCX_MF(i, j, 0, 1);
        DCX_MF(i, j, 0, 0);
      }
#undef DCX_MF
    if constexpr (NL > 0) {
      constexpr int G = 24 / (NL + 1);
#pragma unroll
      for (int k = 0; k < NL; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, G, 0);  // MFMA
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 24 - NL * G, 0);
    }
    __builtin_amdgcn_s_setprio(0);
  };
  auto adv = [&](int& c_, int& m_) {
    if (++m_ == taps) { m_ = 0; ++c_; }
  };
  // loads of step (cl, ml) into register set Q: the input chunk when the step opens one (1-tap:
  // every step, clamped past the end, so unconditional), then the weight tile (clamped past the
  // end, unconditional).  With a halo the input-chunk loads go out before the MFMA cluster and
  // only the weight loads are spread through it.
  int cl, ml;
  constexpr int NL = HALO ? B_PT : A_PT + B_PT;
  auto load_pre = [&](auto qtag) {
    constexpr int Q = decltype(qtag)::value;
    if constexpr (HALO > 0)
      if (ml == 0 && cl < nchunks) loadA(cl, ra[Q]);
  };
  auto load_in = [&](auto qtag) {
    constexpr int Q = decltype(qtag)::value;
    return [&]() {
      if constexpr (HALO == 0) loadA(min(cl, nchunks - 1), ra[Q]);
      loadB(min(cl, nchunks - 1), cl < nchunks ? ml : taps - 1, rb[Q]);
    };
  };
  auto load_step = [&](auto qtag) {  // prologue: plain
    constexpr int Q = decltype(qtag)::value;
    if (ml == 0 && cl < nchunks) loadA(cl, ra[Q]);
    loadB(min(cl, nchunks - 1), cl < nchunks ? ml : taps - 1, rb[Q]);
    adv(cl, ml);
  };

  // ---- prologue: steps 0 and 1 to LDS, step 2 into register set 0
  loadA(0, ra[0]);
  loadB(0, 0, rb[0]);
  storeA(0, ra[0]);
  storeB(0, rb[0]);
  int c1 = 0, m1 = 0;  // position of step 1
  adv(c1, m1);
  loadB(c1, m1, rb[1]);
  if (m1 == 0) loadA(1, ra[1]);  // taps == 1
  storeB(1, rb[1]);
  if (m1 == 0) storeA(1, ra[1]);
  cl = c1;
  ml = m1;
  adv(cl, ml);                   // step 2
  int cw = cl, mw = ml;          // next step this group stores: 2
  load_step(std::integral_constant<int, 0>{});  // step 2 -> set 0; next load: step 3
  __syncthreads();
#ifdef DCX_CLOCK_DIAG
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
#endif
  int cr = 0, mr = 0;
  if (group == 0) {
    readF(0, 0, 0);
    adv(cr, mr);
    // iteration s: MFMA(s) (after loading step s+3 into set (s+1) & 1), then MEM0(s): fragments
    // of step s+1, store step s+2 from set s & 1
    auto iter = [&](int s, auto qtag) {
      constexpr int Q = decltype(qtag)::value;  // s & 1
      load_pre(std::integral_constant<int, 1 - Q>{});
      mfma_with(std::integral_constant<int, NL>{}, load_in(std::integral_constant<int, 1 - Q>{}));
      adv(cl, ml);
      __syncthreads();
      if (s + 1 < nsteps) readF(cr, mr, (s + 1) & 1);
      if (s + 2 < nsteps) {
        storeB((s + 2) & 1, rb[Q]);
        if (mw == 0) storeA(cw & 1, ra[Q]);
      }
      adv(cr, mr);
      adv(cw, mw);
      __syncthreads();
    };
    for (int s = 0; s < nsteps; s += 2) {
      iter(s, std::integral_constant<int, 0>{});
      iter(s + 1, std::integral_constant<int, 1>{});
    }
  } else {
    // iteration s: MEM1(s): fragments of step s, store step s+1 from set (s+1) & 1 (step 1 came
    // from the prologue); then MFMA(s) after loading step s+3 into set (s+1) & 1
    auto iter = [&](int s, auto qtag) {
      constexpr int Q = decltype(qtag)::value;  // s & 1
      readF(cr, mr, s & 1);
      if (s >= 1 && s + 1 < nsteps) {
        storeB((s + 1) & 1, rb[1 - Q]);
        if (mw == 0) storeA(cw & 1, ra[1 - Q]);
      }
      if (s >= 1) adv(cw, mw);
      adv(cr, mr);
      __syncthreads();
      load_pre(std::integral_constant<int, 1 - Q>{});
      mfma_with(std::integral_constant<int, NL>{}, load_in(std::integral_constant<int, 1 - Q>{}));
      adv(cl, ml);
      __syncthreads();
    };
    for (int s = 0; s < nsteps; s += 2) {
      iter(s, std::integral_constant<int, 0>{});
      iter(s + 1, std::integral_constant<int, 1>{});
    }
  }
#ifdef DCX_CLOCK_DIAG
  if (threadIdx.x == 0) {
    atomicAdd(&g_clock_diag[0], __builtin_amdgcn_s_memtime() - t0);
    atomicAdd(&g_clock_diag[1], __builtin_amdgcn_s_memrealtime() - r0);
    atomicAdd(&g_clock_diag[2], (unsigned long long)nsteps);
  }
#endif
  epilogue_lds<BM, BN, 4, WN, (2 * ABUF + 2 * BBUF) / 2, 512, HALO ? 0 : 2>(p, p, acc, q0, co0, b, ph, reinterpret_cast<float*>(lds));
}

template <int HALO, int BN, bool AF32 = false>
__global__ void __launch_bounds__(512, 2) conv_gemm_x6pp(const ConvParams p) {
  constexpr int BM = AF32 ? 512 : 256;
  int wg, b, ph;
  flat_tile(((p.Lq + BM - 1) / BM) * (p.Cout / BN), p.batch, wg, b, ph);
  x6pp_tile<HALO, BN, AF32>(p, p, wg, b, ph);
}

// Grouped split-K launch (round 4, the split-K latency mode): up to 3 independent halo convs (the
// three ResBlocks' convs of one dilation index) in one grid, member k with its own K-slice count
// (ConvParams::ksplit; its clips are virtual: slice * clips + clip).  Member by raw block index, the
// XCD remap inside the member, as conv_gemm_x6dq_group.
__global__ void __launch_bounds__(512, 2) conv_gemm_x6pp_group(const ConvGroup g) {
  const int t = blockIdx.x;
  const int k = t >= g.start[1] ? (t >= g.start[2] ? 2 : 1) : 0;
  const int local = xcd_remap(t - g.start[k], g.start[k + 1] - g.start[k]);
  const int b = local / g.tiles_per_clip[k];
  ConvParams p;  // a private copy of the main-loop fields (pr: the range fields, read in place by the epilogue)
  if (k == 0) p = g.p[0];
  else if (k == 1) p = g.p[1];
  else p = g.p[2];
  const ConvParams& pr = k == 0 ? g.p[0] : k == 1 ? g.p[1] : g.p[2];
  x6pp_tile<64, 128>(p, pr, local - b * g.tiles_per_clip[k], b, 0);
}

template <int HALO>
static hipError_t launch_x6pp(const ConvParams& p, int batch, int phases, hipStream_t s, const char** kname) {
  // (BN = 256 needs 128 accumulator + 72 fragment VGPRs and spills at 2 waves per SIMD).  1-tap
  // convs take conv_gemm_x6lm (loads spread through the MFMA segments): 151 -> 161 TF/s at
  // 1024 -> 4096; with a halo it measured equal at k11 and 4-5 % slower at k3 / taps 2.
  const dim3 grid((unsigned)(((p.Lq + 255) / 256) * (p.Cout / 128) * batch * phases));
  ConvParams q = p;
  q.batch = batch;
  q.phases = phases;
  if constexpr (HALO == 0) {
    if (kname) *kname = "conv_gemm_x6lm<256,128>";
    hipLaunchKernelGGL((conv_gemm_x6lm<0>), grid, dim3(512), 0, s, q);
  } else {
    if (kname) *kname = "conv_gemm_x6pp<256,128,halo>";
    hipLaunchKernelGGL((conv_gemm_x6pp<HALO, 128>), grid, dim3(512), 0, s, q);
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// conv_gemm_x6dm: ping-pong x6 conv on 256 x 256 (or 512 x 128) tiles with LDS-DMA staging.
//
// conv_gemm_x6pp's per-segment stamps put its memory segment (12 fragment reads, register-staged
// LDS stores, global loads: ~1050 cycles at k11) above its MFMA segment (24 MFMAs, ~800), so the
// matrix pipe waited at every barrier.  Here:
//  * staging is LDS-DMA (buffer_load_dwordx4 ... lds): no staging registers and no ds_write
//    pass in the memory segment; each wave issues its pieces and retires them one segment later
//    with a counted vmcnt;
//  * the freed registers buy 64 x 128 wave tiles (256 x 256 block tile): 48 MFMAs per segment
//    against 18 fragment reads (a quarter fewer LDS reads per MFMA than 64 x 64), and each input
//    tile is re-read by half as many column tiles.
// LDS images are lane-linear per DMA instruction (1 KiB = 64 x 16 B): the unpadded 96-byte rows
// of XRow<true> (rows with bit 3 set hold their two K halves swapped, conflict-free fragment
// reads at any tap offset), the swizzle applied on the per-lane SOURCE offsets.  Out-of-range
// input rows (the conv's zero padding) are out of the buffer descriptor's range and load zeros.
// Ring: 3 weight slots (step t in slot t % 3) and 2 input-chunk buffers (chunk parity); step t
// is issued by group 0 in MEM0(t - 3) and by group 1 in MEM1(t - 2), retired at the end of each
// wave's next memory segment, first read in segment 2t - 1 (the schedule of conv_gemm_x6pp).
// ---------------------------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, unsigned short* lds, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)lds, 16, voff, soff, 0, 0);
}
// barrier that keeps the compiler's memory ops on their side and does not drain the DMA queue
__device__ __forceinline__ void seg_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ void wait_dma(int n) {  // n = DMA pieces this wave issued since the ones to retire
#define DCX_W(k) \
  case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
  switch (n) {
    DCX_W(1) DCX_W(2) DCX_W(3) DCX_W(4) DCX_W(5) DCX_W(6) DCX_W(7) DCX_W(8) DCX_W(9) DCX_W(10) DCX_W(11)
    DCX_W(12) DCX_W(13) DCX_W(14) DCX_W(15) DCX_W(16) DCX_W(17) DCX_W(18) DCX_W(19) DCX_W(20) DCX_W(21) DCX_W(22)
    DCX_W(23)
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
#undef DCX_W
}

// BN = 256: 256 x 256 tiles, 64 x 128 wave tiles; BN = 128: 512 x 128 tiles, 128 x 64 wave tiles
// (the same 48 MFMAs and 18 fragment reads per segment).
template <int HALO, int BN>
__global__ void __launch_bounds__(512, 2) conv_gemm_x6dm(const ConvParams p) {
  constexpr int BM = 65536 / BN, WN = 2;
  constexpr int WR = BM / 4, WC = BN / 2, TM = WR / 32, TN = WC / 32;
  constexpr int XS = XRow<true>::kStride;  // 48 ushorts = 96-byte rows
  // DMA instructions (1 KiB each) per group per tile; a group's instructions are dealt round-robin
  // to its 4 waves.  Halo: input chunks double-buffered by chunk parity; 1-tap: every step opens a
  // chunk, so the input tiles ride the weight ring's 3 slots.
  constexpr int A_G = (BM + HALO) * 6 / 128, B_G = BN * 6 / 128;
  constexpr int A_PW = (A_G + 3) / 4, B_PW = (B_G + 3) / 4;
  constexpr int NA = HALO ? 2 : 3;
  constexpr int ABUF = 2 * A_G * 512;  // ushorts
  constexpr int BBUF = BN * XS;
  constexpr int LDS_US = NA * ABUF + 3 * BBUF;
  static_assert((BM + HALO) * 6 % 128 == 0 && 2 * B_G * 512 == BBUF && A_PW + B_PW <= 11, "DMA piece counts");
  static_assert(LDS_US * 2 <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) unsigned short lds[LDS_US];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int group = __builtin_amdgcn_readfirstlane(tid >> 8);
  const int gw = __builtin_amdgcn_readfirstlane((tid >> 6) & 3);
  const int wm = wave >> 1, wn = wave & 1;
  const int ntiles = p.Cout / BN;
  int wg, b, ph;
  flat_tile(((p.Lq + BM - 1) / BM) * ntiles, p.batch, wg, b, ph);
  const int mt = wg / ntiles, nt = wg - mt * ntiles;
  const int q0 = mt * BM, co0 = nt * BN;
  const int nchunks = p.Cin / BK;
  const int taps = p.taps;
  const int nsteps = nchunks * taps;
  const int lo_rel = p.in_step < 0 ? (taps - 1) * p.in_step : 0;
  const int row0 = q0 + p.in_base[ph] + lo_rel;
  const int arow = p.ldx * 6;  // bytes per planes row
  // halo: descriptor over the clip (negative rows wrap past its range: zeros); 1-tap: over the
  // tile's rows only, so clips of any length keep 32-bit offsets (row0 >= 0 without a halo)
  const __amdgpu_buffer_rsrc_t rx =
      HALO ? __builtin_amdgcn_make_buffer_rsrc((void*)(p.x6 + (long long)b * p.x_bstride * 3), 0, p.Lin * arow, 0x00020000)
           : __builtin_amdgcn_make_buffer_rsrc((void*)(p.x6 + ((long long)b * p.x_bstride + (long long)row0 * p.ldx) * 3), 0,
                                               max(0, min(BM, p.Lin - row0)) * arow, 0x00020000);
  const int rbase = HALO ? row0 : 0;  // row of image row 0 relative to the descriptor
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.w6 + (long long)ph * taps * nchunks * p.Cout * 48), 0, taps * nchunks * p.Cout * 96, 0x00020000);

  // per-lane source offsets of this wave's pieces (lane-linear LDS, swizzle on the source); the
  // wave's i-th instruction is its group's instruction i * 4 + gw
  const int a_cnt = (A_G - gw + 3) / 4, b_cnt = (B_G - gw + 3) / 4;  // wave-uniform
  int a_off[A_PW], b_off[B_PW];
#pragma unroll
  for (int i = 0; i < A_PW; ++i) {
    const int P = (group * A_G + i * 4 + gw) * 64 + lane;
    const int row = P / 6, s = P - row * 6;
    const int hl = (s >= 3) ^ ((row >> 3) & 1), pl = s >= 3 ? s - 3 : s;
    a_off[i] = (rbase + row) * arow + (hl * 3 + pl) * 16;  // negative rows: huge unsigned, out of range
  }
#pragma unroll
  for (int i = 0; i < B_PW; ++i) {
    const int P = (group * B_G + i * 4 + gw) * 64 + lane;
    const int col = P / 6, s = P - col * 6;
    const int sg = ((col >> 3) & 1) ? (s >= 3 ? s - 3 : s + 3) : s;
    b_off[i] = (co0 + col) * 96 + sg * 16;
  }
  unsigned short* const a_dst = lds + (group * A_G + gw) * 512;
  unsigned short* const b_dst = lds + NA * ABUF + (group * B_G + gw) * 512;
  auto dmaA = [&](int c, int abuf) {
#pragma unroll
    for (int i = 0; i < A_PW; ++i)
      if (A_G % 4 == 0 || i < a_cnt) dma16(rx, a_dst + abuf * ABUF + i * 2048, a_off[i] + c * 96, 0);
  };
  auto dmaB = [&](int c, int m, int slot) {
    const int soff = (m * nchunks + c) * p.Cout * 96;
#pragma unroll
    for (int i = 0; i < B_PW; ++i)
      if (B_G % 4 == 0 || i < b_cnt) dma16(rw, b_dst + slot * BBUF + i * 2048, b_off[i], soff);
  };
  // DMA of one step (its input chunk first when the step opens one); returns the pieces issued
  auto dma_step = [&](int c, int m, int slot) {
    int n = b_cnt;
    if (m == 0) {
      dmaA(c, HALO ? (c & 1) : slot);
      n += a_cnt;
    }
    dmaB(c, m, slot);
    return n;
  };

  const int lrow = lane & 31, h = lane >> 5;
  s16x8 af[TM][3], bfr[TN][3];
  auto readF = [&](int c, int m, int slot) {
    const int off = m * p.in_step - lo_rel;
    const unsigned short* A = lds + (HALO ? (c & 1) : slot) * ABUF;
    const unsigned short* Bs = lds + NA * ABUF + slot * BBUF;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int r = wm * WR + i * 32 + lrow + off;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) af[i][pl] = *reinterpret_cast<const s16x8*>(A + XRow<true>::off(r, h * 3 + pl));
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = wn * WC + j * 32 + lrow;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) bfr[j][pl] = *reinterpret_cast<const s16x8*>(Bs + XRow<true>::off(col, h * 3 + pl));
    }
  };
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  auto mfma = [&]() {
    __builtin_amdgcn_s_setprio(1);
#define DCX_MF(i, j, x, y) \
  acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, af[i][x]), \
                                                      __builtin_bit_cast(bf16x8, bfr[j][y]), acc[i][j], 0, 0, 0)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        DCX_MF(i, j, 2, 0);
        DCX_MF(i, j, 1, 1);
        DCX_MF(i, j, 0, 2);
        DCX_MF(i, j, 1, 0);
        DCX_MF(i, j, 0, 1);
        DCX_MF(i, j, 0, 0);
      }
#undef DCX_MF
    __builtin_amdgcn_s_setprio(0);
  };
  auto adv = [&](int& c_, int& m_) {
    if (++m_ == taps) { m_ = 0; ++c_; }
  };
  auto inc3 = [](int& slot) { slot = slot == 2 ? 0 : slot + 1; };

  // ---- prologue: steps 0, 1, 2 (both groups their pieces), drained
  int cl = 0, ml = 0;
  for (int t = 0; t < 3; ++t) {
    if (t < nsteps) dma_step(cl, ml, t);
    adv(cl, ml);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  seg_barrier();
#ifdef DCX_CLOCK_DIAG
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
#endif
  // cl, ml: step 3, the next step either group issues
  int cr = 0, mr = 0;
  if (group == 0) {
    readF(0, 0, 0);
    adv(cr, mr);
    int rs = 1, ws = 0;  // slot of the step read next (s + 1), of the step issued next (s + 3)
    for (int s = 0; s < nsteps; ++s) {
      mfma();  // MFMA(s)
      seg_barrier();
      // MEM0(s): fragments of step s + 1, issue step s + 3, retire step s + 2
      if (s + 1 < nsteps) readF(cr, mr, rs);
      int n = 0;
      if (s + 3 < nsteps) n = dma_step(cl, ml, ws);
      wait_dma(n);
      seg_barrier();
      adv(cr, mr);
      adv(cl, ml);
      inc3(rs);
      inc3(ws);
    }
  } else {
    int rs = 0, ws = 0;  // slot of step s, of step s + 2
    for (int s = 0; s < nsteps; ++s) {
      // MEM1(s): fragments of step s, issue step s + 2 (s >= 1), retire step s + 1
      readF(cr, mr, rs);
      int n = 0;
      if (s >= 1 && s + 2 < nsteps) {
        n = dma_step(cl, ml, ws);
        adv(cl, ml);
      }
      wait_dma(n);
      seg_barrier();
      mfma();  // MFMA(s)
      seg_barrier();
      adv(cr, mr);
      inc3(rs);
      if (s >= 1) inc3(ws);
      else ws = 0;  // step 3's slot
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef DCX_CLOCK_DIAG
  if (threadIdx.x == 0) {  // steps counted in units of x6pp's (half the MFMAs)
    atomicAdd(&g_clock_diag[0], __builtin_amdgcn_s_memtime() - t0);
    atomicAdd(&g_clock_diag[1], __builtin_amdgcn_s_memrealtime() - r0);
    atomicAdd(&g_clock_diag[2], 2ull * nsteps);
  }
#endif
  epilogue_lds<BM, BN, 4, WN, LDS_US / 2, 512, HALO ? 0 : 2>(p, p, acc, q0, co0, b, ph, reinterpret_cast<float*>(lds));
}

// ---------------------------------------------------------------------------------------------
// conv_gemm_x6dq: conv_gemm_x6dm on v_mfma_f32_16x16x32_bf16.
//
// The chip holds a lower clock under 32x32x16 MFMA load than under 16x16x32 at the same cycles per
// FLOP (MI355X_MICROARCH.md, DVFS item 7), and x6dm's loop runs at ~95 % MFMA issue, so what is
// left is the clock.  The six products of a K16 step fold into three K32 MFMAs by pairing terms in
// the K dimension: k = (t, c) with t = lane >> 5 selecting the term, c the channel (lane bits 4
// and 0-3 the channel half and row), so one MFMA sums x_t0 * y_t0 + x_t1 * y_t1 over 16 channels:
//   A{h,m} . B{h',m'} = hh' + mm',   A{m,h} . B{h',m'} = mh' + hm',   A{l,h} . B{h',l'} = lh' + hl'.
// Each operand set is one ds_read_b128 whose lanes pick their plane by t: 3 A sets per 16-row
// block, 2 B sets per 16-column block.  A 64 x 128 (128 x 64) wave tile holds 8 x 4 (4 x 8) f32x4
// accumulators; B fragments for the whole tile and the A fragments of RH row blocks fit in
// registers, the MFMA segment reading the later row blocks' A itself behind the MFMAs of the
// earlier ones.  A is then read in both segments of a step, so the input chunk buffer is reused
// one segment later than in x6dm: taps >= 3 (the ResBlock and conv_pre convs).
// LDS images: 16-row blocks, piece-major inside a block: 16-byte unit (r >> 4) * 96 + s * 16 +
// (r & 15) for piece s = half * 3 + plane of row r; every ds_read_b128 then touches 16
// consecutive rows of one piece per lane group (conflict-free at any tap offset).
// ---------------------------------------------------------------------------------------------
// One output tile (wg = row tile * column tiles + column tile, clip b, phase ph).
template <int BN>
__device__ __forceinline__ void x6dq_tile(const ConvParams& p, const ConvParams& pr, const int wg, const int b, const int ph) {
  DCX_TILET(tile_t0);
  constexpr int HALO = 64;
  constexpr int BM = 65536 / BN, WN = 2;
  constexpr int WR = BM / 4, WC = BN / 2, TM = WR / 16, TN = WC / 16;
  constexpr int RH = BN == 256 ? 2 : 4;  // A row blocks held from the memory segment
  constexpr int A_G = (BM + HALO) * 6 / 128, B_G = BN * 6 / 128;
  constexpr int A_PW = (A_G + 3) / 4, B_PW = (B_G + 3) / 4;
  constexpr int ABUF = 2 * A_G * 512;  // ushorts
  constexpr int BBUF = BN * 48;
  constexpr int LDS_US = 2 * ABUF + 3 * BBUF;
  static_assert((BM + HALO) * 6 % 128 == 0 && 2 * B_G * 512 == BBUF && A_PW + B_PW <= 11, "DMA piece counts");
  static_assert(LDS_US * 2 <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) unsigned short lds[LDS_US];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int group = __builtin_amdgcn_readfirstlane(tid >> 8);
  const int gw = __builtin_amdgcn_readfirstlane((tid >> 6) & 3);
  const int wm = wave >> 1, wn = wave & 1;
  const int ntiles = p.Cout / BN;
  const int mt = wg / ntiles, nt = wg - mt * ntiles;
  const int q0 = mt * BM, co0 = nt * BN;
  const int nchunks = p.Cin / BK;
  const int taps = p.taps;
  const int nsteps = nchunks * taps;
  const int lo_rel = p.in_step < 0 ? (taps - 1) * p.in_step : 0;
  const int row0 = q0 + p.in_base[ph] + lo_rel;
  const int arow = p.ldx * 6;
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.x6 + (long long)b * p.x_bstride * 3), 0, p.Lin * arow, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.w6 + (long long)ph * taps * nchunks * p.Cout * 48), 0, taps * nchunks * p.Cout * 96, 0x00020000);

  // DMA pieces: unit u of a tile image -> row (u / 96) * 16 + (u & 15), piece (u % 96) >> 4
  const int a_cnt = (A_G - gw + 3) / 4, b_cnt = (B_G - gw + 3) / 4;
  int a_off[A_PW], b_off[B_PW];
#pragma unroll
  for (int i = 0; i < A_PW; ++i) {
    const int u = (group * A_G + i * 4 + gw) * 64 + lane;
    const int blk = u / 96, rem = u - blk * 96;
    a_off[i] = (row0 + blk * 16 + (rem & 15)) * arow + (rem >> 4) * 16;  // negative rows: out of range
  }
#pragma unroll
  for (int i = 0; i < B_PW; ++i) {
    const int u = (group * B_G + i * 4 + gw) * 64 + lane;
    const int blk = u / 96, rem = u - blk * 96;
    b_off[i] = (co0 + blk * 16 + (rem & 15)) * 96 + (rem >> 4) * 16;
  }
  unsigned short* const a_dst = lds + (group * A_G + gw) * 512;
  unsigned short* const b_dst = lds + 2 * ABUF + (group * B_G + gw) * 512;
  auto dma_step = [&](int c, int m, int slot) {
    int n = b_cnt;
    if (m == 0) {
#pragma unroll
      for (int i = 0; i < A_PW; ++i)
        if (A_G % 4 == 0 || i < a_cnt) dma16(rx, a_dst + (c & 1) * ABUF + i * 2048, a_off[i] + c * 96, 0);
      n += a_cnt;
    }
    const int soff = (m * nchunks + c) * p.Cout * 96;
#pragma unroll
    for (int i = 0; i < B_PW; ++i)
      if (B_G % 4 == 0 || i < b_cnt) dma16(rw, b_dst + slot * BBUF + i * 2048, b_off[i], soff);
    return n;
  };

  // fragment sets: lane picks plane by t = lane >> 5, channel half hf = (lane >> 4) & 1
  const int l15 = lane & 15, hf = (lane >> 4) & 1, t = lane >> 5;
  const int soA0 = (hf * 3 + t) * 256, soA1 = (hf * 3 + (t ? 0 : 1)) * 256, soA2 = (hf * 3 + (t ? 0 : 2)) * 256;
  const int soB0 = (hf * 3 + t) * 256, soB1 = (hf * 3 + (t ? 2 : 0)) * 256;  // bytes (piece stride 256)
  const char* const ldsb = reinterpret_cast<const char*>(lds);
  const int bcol = (wn * WC / 16) * 1536 + l15 * 16 + 4 * ABUF;  // bytes, B image of slot 0
  s16x8 aq[RH][3], bq[TN][2];
  int abase = 0;  // bytes: this lane's row in the A image of the step being read
  auto readA1 = [&](int rb, int k, int set) {
    const char* a = ldsb + abase + rb * 1536 + (set == 0 ? soA0 : set == 1 ? soA1 : soA2);
    aq[k][set] = *reinterpret_cast<const s16x8*>(a);
  };
  auto readA = [&](int rb, int k) {
    readA1(rb, k, 0);
    readA1(rb, k, 1);
    readA1(rb, k, 2);
  };
  auto readF = [&](int c, int m, int slot) {
    const int r = wm * WR + m * p.in_step - lo_rel + l15;
    abase = (c & 1) * ABUF * 2 + (r >> 4) * 1536 + (r & 15) * 16;
    const char* bb = ldsb + bcol + slot * BBUF * 2;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      bq[j][0] = *reinterpret_cast<const s16x8*>(bb + j * 1536 + soB0);
      bq[j][1] = *reinterpret_cast<const s16x8*>(bb + j * 1536 + soB1);
    }
#pragma unroll
    for (int k = 0; k < RH; ++k) readA(k, k);
  };
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // MFMA segment: row block by row block, and within a block operand set by operand set (per
  // accumulator: lh' + hl', then mh' + hm', then hh' + mm'); as soon as a set's MFMAs are issued,
  // its registers take the same set of row block rb + RH (read from the same step's image), so the
  // reads are spread through the segment and land 2..3 sets' worth of MFMAs before their use
  auto mfma = [&]() {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int rb = 0; rb < TM; ++rb) {
      const int k = rb % RH;
#pragma unroll
      for (int set = 2; set >= 0; --set) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[rb][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, aq[k][set]),
                                                               __builtin_bit_cast(bf16x8, bq[j][set == 2 ? 1 : 0]),
                                                               acc[rb][j], 0, 0, 0);
        if (rb + RH < TM) readA1(rb + RH, k, set);
      }
    }
#pragma unroll
    for (int rb = 0; rb < TM; ++rb)
#pragma unroll
      for (int set = 0; set < 3; ++set) {
        __builtin_amdgcn_sched_group_barrier(0x008, TN, 0);
        if (rb + RH < TM) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
    __builtin_amdgcn_s_setprio(0);
  };
  auto adv = [&](int& c_, int& m_) {
    if (++m_ == taps) { m_ = 0; ++c_; }
  };
  auto inc3 = [](int& slot) { slot = slot == 2 ? 0 : slot + 1; };

  int cl = 0, ml = 0;
  for (int tt = 0; tt < 3; ++tt) {
    if (tt < nsteps) dma_step(cl, ml, tt);
    adv(cl, ml);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  seg_barrier();
  DCX_TILET(tile_t1);
#ifdef DCX_CLOCK_DIAG
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
#endif
  int cr = 0, mr = 0;
#ifdef DCX_SEG_DIAG
  unsigned long long sd[4] = {};
#endif
  if (group == 0) {
    readF(0, 0, 0);
    adv(cr, mr);
    int rs = 1, ws = 0;
    for (int s = 0; s < nsteps; ++s) {
      DCX_SEGT(ta);
      mfma();  // MFMA(s)
      DCX_SEGT(tb);
      seg_barrier();
      DCX_SEGT(tc);
      if (s + 1 < nsteps) readF(cr, mr, rs);
      int n = 0;
      if (s + 3 < nsteps) n = dma_step(cl, ml, ws);
      wait_dma(n);
      DCX_SEGT(td);
      seg_barrier();
      DCX_SEGT(te);
#ifdef DCX_SEG_DIAG
      sd[0] += tb - ta; sd[1] += tc - tb; sd[2] += td - tc; sd[3] += te - td;
#endif
      adv(cr, mr);
      adv(cl, ml);
      inc3(rs);
      inc3(ws);
    }
  } else {
    int rs = 0, ws = 0;
    for (int s = 0; s < nsteps; ++s) {
      DCX_SEGT(ta);
      readF(cr, mr, rs);
      int n = 0;
      if (s >= 1 && s + 2 < nsteps) {
        n = dma_step(cl, ml, ws);
        adv(cl, ml);
      }
      wait_dma(n);
      DCX_SEGT(tb);
      seg_barrier();
      DCX_SEGT(tc);
      mfma();  // MFMA(s)
      DCX_SEGT(td);
      seg_barrier();
      DCX_SEGT(te);
#ifdef DCX_SEG_DIAG
      sd[2] += tb - ta; sd[3] += tc - tb; sd[0] += td - tc; sd[1] += te - td;
#endif
      adv(cr, mr);
      inc3(rs);
      if (s >= 1) inc3(ws);
      else ws = 0;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef DCX_SEG_DIAG
  if ((threadIdx.x & 255) == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) atomicAdd(&g_seg_diag[group * 6 + i], sd[i]);
    if (group == 0) atomicAdd(&g_seg_diag[12], (unsigned long long)nsteps);
  }
#endif
#ifdef DCX_CLOCK_DIAG
  if (threadIdx.x == 0) {
    atomicAdd(&g_clock_diag[0], __builtin_amdgcn_s_memtime() - t0);
    atomicAdd(&g_clock_diag[1], __builtin_amdgcn_s_memrealtime() - r0);
    atomicAdd(&g_clock_diag[2], 2ull * nsteps);
  }
#endif
  DCX_TILET(tile_t2);
  epilogue_lds<BM, BN, 4, WN, LDS_US / 2, 512, 0>(p, pr, acc, q0, co0, b, ph, reinterpret_cast<float*>(lds));
#ifdef DCX_TILE_DIAG
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long t3 = __builtin_amdgcn_s_memrealtime();
    const unsigned int k = atomicAdd(&g_tile_cnt, 1u);
    if (k < (unsigned)kTileDiagMax) {
      unsigned long long* o = g_tile_diag + 6ull * k;
      o[0] = tile_t0; o[1] = tile_t1; o[2] = tile_t2; o[3] = t3;
      o[4] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
      o[5] = __builtin_amdgcn_s_getreg((15 << 11) | 20);
    }
  }
#endif
}

template <int BN>
__global__ void __launch_bounds__(512, 2) conv_gemm_x6dq(const ConvParams p) {
  int wg, b, ph;
  flat_tile(((p.Lq + 65536 / BN - 1) / (65536 / BN)) * (p.Cout / BN), p.batch, wg, b, ph);
  x6dq_tile<BN>(p, p, wg, b, ph);
}

// Grouped launch: up to 3 independent convs with the same tiling (the three ResBlocks' convs of one
// dilation index, tap counts 3 / 7 / 11), longest first, so the short ones fill the last round.
template <int BN>
__global__ void __launch_bounds__(512, 2) conv_gemm_x6dq_group(const ConvGroup g) {
  // member by raw block index, so every XCD (block index mod 8) gets its share of each member's
  // tiles; a remap of the whole grid would hand the 11-tap tiles to the first XCDs and the 3-tap
  // ones to the last
  const int t = blockIdx.x;
  const int k = t >= g.start[1] ? (t >= g.start[2] ? 2 : 1) : 0;
  const int local = xcd_remap(t - g.start[k], g.start[k + 1] - g.start[k]);
  const int b = local / g.tiles_per_clip[k];
  // a private copy: the tile body's inline-asm barriers clobber memory, which would make the
  // compiler re-read every field of a kernarg-resident struct after each of them
  ConvParams p;  // a private copy of the main-loop fields (pr: the range fields, read in place by the epilogue)
  if (k == 0) p = g.p[0];
  else if (k == 1) p = g.p[1];
  else p = g.p[2];
  const ConvParams& pr = k == 0 ? g.p[0] : k == 1 ? g.p[1] : g.p[2];
  x6dq_tile<BN>(p, pr, local - b * g.tiles_per_clip[k], b, 0);
}

template <int BN>
static hipError_t launch_x6dq(const ConvParams& p, int batch, int phases, hipStream_t s, const char** kname) {
  constexpr int BM = 65536 / BN;
  const dim3 grid((unsigned)(((p.Lq + BM - 1) / BM) * (p.Cout / BN) * batch * phases));
  ConvParams q = p;
  q.batch = batch;
  q.phases = phases;
  if (kname) *kname = BN == 256 ? "conv_gemm_x6dq<256,256,halo>" : "conv_gemm_x6dq<512,128,halo>";
  hipLaunchKernelGGL((conv_gemm_x6dq<BN>), grid, dim3(512), 0, s, q);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// conv_gemm_x3dq: the fp16 "h3" arithmetic (round 5) on conv_gemm_x6dq's LDS-DMA ping-pong schedule.
//
// An fp32 value is held as two fp16 values, h = fp16(x) and l = fp16(x - h) (dcx_planes.h "h2"
// layout, 22 significant bits), the weights likewise after scaling by 2^w3_shift (the largest |w|
// just below 2^15, so l stays normal for all weights within 2^-18 of it); the accumulators are
// scaled back by 2^-w3_shift before the epilogue.  A product keeps three terms, hh' + hl' + lh'
// (ll' is 2^-22 relative), against x6's six, at the same K32 rate per MFMA
// (v_mfma_f32_16x16x32_f16; the K16 f16 MFMA issues at half rate on gfx950, tools/probe).
// A step is one 32-channel chunk of one tap; per 16 x 16 block three MFMAs, A{h} . B{l'},
// A{l} . B{h'} and A{h} . B{h'}, the lanes of K group kg = lane >> 4 holding channel group kg
// (8 channels) of every operand, so a lane reads h and l of its rows and h' and l' of its columns
// once per step.
// Tiles BM x BN = 128 x 256 (BN = 256) or 256 x 128, 8 waves of 64 x 64 (group 0 the upper half of
// the rows); every fragment of a step (8 A + 8 B ds_read_b128) is read in the memory segment and
// an MFMA segment is 48 MFMAs.  LDS images, piece-major and row-linear: A [piece 8][BM + 64][16 B]
// (two buffers, by chunk parity), B [piece 8][BN][16 B] (3-slot ring), piece = plane * 4 + channel
// group; one 1 KiB DMA instruction fills 64 rows of one piece.  Rows of one piece are 16 B apart,
// so a ds_read_b128 lane group (16 distinct rows mod 16) is conflict-free at any tap offset.
// The A buffer of chunk c + 2 is issued taps - 2 segments after chunk c's last read: taps >= 3.
// ---------------------------------------------------------------------------------------------
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// HALO = 64: convs with a tap halo (taps >= 3), input chunks double-buffered by chunk parity;
// HALO = 0 (conv_gemm_x3dm): one-tap convs, every step opens a chunk, so the input tiles ride the
// weight ring's 3 slots, over a descriptor of the tile's rows only (32-bit offsets at any length).
template <int BN, int HALO>
__device__ __forceinline__ void x3dq_tile(const ConvParams& p, const ConvParams& pr, const int wg, const int b, const int ph) {
  constexpr int BM = 32768 / BN, WN = BN / 64, WM = 8 / WN;
  constexpr int NA = HALO ? 2 : 3;
  constexpr int WR = BM / WM, WC = BN / WN, TM = WR / 16, TN = WC / 16;
  constexpr int AR = BM + HALO;                 // rows of an input image
  constexpr int A_G = AR / 16, B_G = BN / 16;   // 1 KiB DMA instructions per group (A per chunk, B per step)
  constexpr int A_PW = A_G / 4, B_PW = B_G / 4;
  constexpr int ABUF = AR * 128, BBUF = BN * 128;  // bytes
  constexpr int LDS_B = NA * ABUF + 3 * BBUF;
  static_assert(WR == 64 && WC == 64 && A_G % 4 == 0 && B_G % 4 == 0 && AR % 64 == 0, "tile shape");
  static_assert(LDS_B <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) unsigned short lds[LDS_B / 2];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int group = __builtin_amdgcn_readfirstlane(tid >> 8);
  const int gw = __builtin_amdgcn_readfirstlane((tid >> 6) & 3);
  const int wm = wave / WN, wn = wave % WN;
  const int ntiles = p.Cout / BN;
  const int mt = wg / ntiles, nt = wg - mt * ntiles;
  const int q0 = mt * BM, co0 = nt * BN;
  const int nchunks = p.Cin / 32;
  const int taps = p.taps;
  const int nsteps = nchunks * taps;
  const int lo_rel = p.in_step < 0 ? (taps - 1) * p.in_step : 0;
  const int row0 = q0 + p.in_base[ph] + lo_rel;
  const int arow = p.ldx * 4;  // bytes per h2 row
  const __amdgpu_buffer_rsrc_t rx =
      HALO ? __builtin_amdgcn_make_buffer_rsrc((void*)(p.x6 + (long long)b * p.x_bstride * 2), 0, p.Lin * arow, 0x00020000)
           : __builtin_amdgcn_make_buffer_rsrc((void*)(p.x6 + ((long long)b * p.x_bstride + (long long)row0 * p.ldx) * 2), 0,
                                               max(0, min(BM, p.Lin - row0)) * arow, 0x00020000);
  const int rbase = HALO ? row0 : 0;  // row of image row 0 relative to the descriptor
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.w3 + (long long)ph * taps * nchunks * p.Cout * 64), 0, taps * nchunks * p.Cout * 128, 0x00020000);

  // DMA: group instruction k fills 64 rows of piece (k * 64) / rows; the wave's i-th is k = i * 4 + gw.
  // Source of piece pc in an h2 row's chunk: channel group pc & 3 at 32 B, plane pc >> 2 at 16 B.
  int a_off[A_PW], b_off[B_PW];
#pragma unroll
  for (int i = 0; i < A_PW; ++i) {
    const int u = (group * A_G + i * 4 + gw) * 64;
    const int pc = u / AR, row = u - pc * AR + lane;
    a_off[i] = (rbase + row) * arow + (pc & 3) * 32 + (pc >> 2) * 16;  // negative rows: out of range
  }
#pragma unroll
  for (int i = 0; i < B_PW; ++i) {
    const int u = (group * B_G + i * 4 + gw) * 64;
    const int pc = u / BN, col = u - pc * BN + lane;
    b_off[i] = (co0 + col) * 128 + (pc & 3) * 32 + (pc >> 2) * 16;
  }
  unsigned short* const a_dst = lds + (group * A_G + gw) * 512;
  unsigned short* const b_dst = lds + NA * ABUF / 2 + (group * B_G + gw) * 512;
  [[maybe_unused]] bool in_loop = false;  // -DDCX_X3_NODMA (diagnostic): no DMA after the prologue (wrong results)
  auto dma_step = [&](int c, int m, int slot) {
#ifdef DCX_X3_NODMA
    if (in_loop) return 0;
#endif
    int n = B_PW;
    if (m == 0) {
#pragma unroll
      for (int i = 0; i < A_PW; ++i)
        dma16(rx, a_dst + (HALO ? (c & 1) : slot) * (ABUF / 2) + i * 2048, a_off[i] + c * 128, 0);
      n += A_PW;
    }
    const int soff = (m * nchunks + c) * p.Cout * 128;
#pragma unroll
    for (int i = 0; i < B_PW; ++i) dma16(rw, b_dst + slot * (BBUF / 2) + i * 2048, b_off[i], soff);
    return n;
  };

  const int l15 = lane & 15, kg = lane >> 4;
  // piece offsets (bytes): h and l of the lane's channel group
  const int pah = kg * AR * 16, pal = (4 + kg) * AR * 16;
  const int pbh = kg * BN * 16, pbl = (4 + kg) * BN * 16;
  const char* const ldsb = reinterpret_cast<const char*>(lds);
  const int bcol = NA * ABUF + (wn * WC + l15) * 16;
  s16x8 aq[TM][2], bq[TN][2];  // [h, l]
  auto readF = [&](int c, int m, int slot) {
    const char* a = ldsb + (HALO ? (c & 1) : slot) * ABUF + (wm * WR + m * p.in_step - lo_rel + l15) * 16;
    const char* bb = ldsb + bcol + slot * BBUF;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      bq[j][0] = *reinterpret_cast<const s16x8*>(bb + j * 256 + pbh);
      bq[j][1] = *reinterpret_cast<const s16x8*>(bb + j * 256 + pbl);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      aq[i][0] = *reinterpret_cast<const s16x8*>(a + i * 256 + pah);
      aq[i][1] = *reinterpret_cast<const s16x8*>(a + i * 256 + pal);
    }
  };
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // the cross terms first (hl', lh'), then hh'; 16 independent accumulators between dependent MFMAs
  // (priority 1 while issuing MFMAs: without it the C2 step took 212.0 against 192.8 ms, r05k)
  auto mfma = [&]() {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int sa = k == 1 ? 1 : 0, sb = k == 0 ? 1 : 0;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, aq[i][sa]),
                                                             __builtin_bit_cast(f16x8, bq[j][sb]), acc[i][j], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
  };
  auto adv = [&](int& c_, int& m_) {
    if (++m_ == taps) { m_ = 0; ++c_; }
  };
  auto inc3 = [](int& slot) { slot = slot == 2 ? 0 : slot + 1; };

  int cl = 0, ml = 0;
  for (int tt = 0; tt < 3; ++tt) {
    if (tt < nsteps) dma_step(cl, ml, tt);
    adv(cl, ml);
  }
  // the epilogue's range values and the input's unscale, in flight with the prologue's DMA
  const EpiPre epre = epi_range_pre<HALO == 0 ? 3 : 0>(p, pr, b);
  const float unscale = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int,
      __builtin_ldexpf(1.0f, -(p.w3_shift + (pr.x_ash ? pr.x_ash[b] : pr.x_ash_c))))));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  seg_barrier();
  in_loop = true;
  int cr = 0, mr = 0;
#ifdef DCX_SEG_DIAG
  unsigned long long sd[6] = {};
#endif
  if (group == 0) {
    readF(0, 0, 0);
    adv(cr, mr);
    int rs = 1, ws = 0;  // slot of the step read next (s + 1), of the step issued next (s + 3)
    for (int s = 0; s < nsteps; ++s) {
      DCX_SEGT(ta);
      mfma();  // MFMA(s)
      DCX_SEGT(tb);
      seg_barrier();
      DCX_SEGT(tc);
      // MEM0(s): issue step s + 3, fragments of step s + 1, retire step s + 2 (the DMA first: the
      // fragment reads' latency then hides behind the DMA issue, C2 192.8 -> 190.3 ms, r05k)
      int n = 0;
      if (s + 3 < nsteps) n = dma_step(cl, ml, ws);
      DCX_SEGT(tr);
      if (s + 1 < nsteps) readF(cr, mr, rs);
      DCX_SEGT(tq);
      wait_dma(n);
      DCX_SEGT(td);
      seg_barrier();
      DCX_SEGT(te);
#ifdef DCX_SEG_DIAG
      sd[0] += tb - ta; sd[1] += tc - tb; sd[2] += td - tc; sd[3] += te - td; sd[4] += tr - tc; sd[5] += tq - tr;
#endif
      adv(cr, mr);
      adv(cl, ml);
      inc3(rs);
      inc3(ws);
    }
  } else {
    int rs = 0, ws = 0;  // slot of step s, of step s + 2
    for (int s = 0; s < nsteps; ++s) {
      DCX_SEGT(ta);
      // MEM1(s): issue step s + 2 (s >= 1), fragments of step s, retire step s + 1
      int n = 0;
      if (s >= 1 && s + 2 < nsteps) {
        n = dma_step(cl, ml, ws);
        adv(cl, ml);
      }
      DCX_SEGT(tr);
      readF(cr, mr, rs);
      DCX_SEGT(tq);
      wait_dma(n);
      DCX_SEGT(tb);
      seg_barrier();
      DCX_SEGT(tc);
      mfma();  // MFMA(s)
      DCX_SEGT(td);
      seg_barrier();
      DCX_SEGT(te);
#ifdef DCX_SEG_DIAG
      sd[2] += tb - ta; sd[3] += tc - tb; sd[0] += td - tc; sd[1] += te - td; sd[4] += tr - ta; sd[5] += tq - tr;
#endif
      adv(cr, mr);
      inc3(rs);
      if (s >= 1) inc3(ws);
      else ws = 0;  // step 3's slot
    }
  }
#ifdef DCX_SEG_DIAG
  if ((threadIdx.x & 255) == 0) {
#pragma unroll
    for (int i = 0; i < 6; ++i) atomicAdd(&g_seg_diag[group * 6 + i], sd[i]);
    if (group == 0) atomicAdd(&g_seg_diag[12], (unsigned long long)nsteps);
  }
#endif
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // undo the weight and the input's range scaling (powers of two: exact)
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] *= unscale;
  epilogue_lds<BM, BN, WM, WN, LDS_B / 4, 512, HALO == 0 ? 3 : 0>(p, pr, acc, q0, co0, b, ph, reinterpret_cast<float*>(lds), &epre);
}

template <int BN, int HALO>
__global__ void __launch_bounds__(512, 2) conv_gemm_x3dq(const ConvParams p) {
  int wg, b, ph;
  flat_tile(((p.Lq + 32768 / BN - 1) / (32768 / BN)) * (p.Cout / BN), p.batch, wg, b, ph);
  x3dq_tile<BN, HALO>(p, p, wg, b, ph);
}

// grouped launch of up to 3 h3 convs (conv_gemm_x6dq_group's member mapping)
template <int BN>
__global__ void __launch_bounds__(512, 2) conv_gemm_x3dq_group(const ConvGroup g) {
  const int t = blockIdx.x;
  const int k = t >= g.start[1] ? (t >= g.start[2] ? 2 : 1) : 0;
  const int local = xcd_remap(t - g.start[k], g.start[k + 1] - g.start[k]);
  const int b = local / g.tiles_per_clip[k];
  ConvParams p;  // a private copy of the main-loop fields (pr: the range fields, read in place by the epilogue)
  if (k == 0) p = g.p[0];
  else if (k == 1) p = g.p[1];
  else p = g.p[2];
  const ConvParams& pr = k == 0 ? g.p[0] : k == 1 ? g.p[1] : g.p[2];
  x3dq_tile<BN, 64>(p, pr, local - b * g.tiles_per_clip[k], b, 0);
}

// ---------------------------------------------------------------------------------------------
// conv_gemm_x3dw: h3 arithmetic on 256 x 256 tiles (64 x 128 wave tiles, 96 MFMAs per segment).
//
// Segment stamps of x3dq / x3dm (tools/seg_diag_h3.py) put their memory segment, and within it the
// DMA issue, at or above the MFMA segment: a CU takes in about 16 B per cycle by LDS-DMA, and a
// 256 x 128 tile needs (A / taps + B) bytes per 48 MFMAs per wave.  A 256 x 256 tile moves the same
// A and twice the columns per step, and a 64 x 128 wave tile issues twice the MFMAs per fragment
// read.  It fits the LDS with a 2-slot step ring (B 32 KiB per slot; A 40 KiB per chunk, double-
// buffered by chunk parity, or, one-tap, 32 KiB riding the B slot): 144 / 128 KiB.
// Schedule (segment 2s = MFMA0(s) | MEM1(s), 2s + 1 = MEM0(s) | MFMA1(s); step t in slot t % 2):
//   * group 1 reads step s in MEM1(s); group 0 reads step s + 1 in MEM0(s);
//   * group 0 alone issues the DMA: step s + 2 in MEM0(s) (step s's slot, whose last reader was
//     MEM1(s)), and waits for it (vmcnt(0)) at the end of MFMA0(s + 1), before the barrier that
//     opens MEM0(s + 1), its first reader: one segment of MFMAs covers the DMA latency.
//   * A chunk c (halo) is issued with step c * taps into buffer c & 1, whose last reader (chunk
//     c - 2's last step, MEM1((c - 1) * taps - 1)) is at least two segments earlier for taps >= 2.
// Per-lane DMA offsets are one VGPR per operand (row base) plus a wave-uniform add per piece.
// ---------------------------------------------------------------------------------------------
// SPLIT (Knobs::h3_split): the weight pieces of step s + 2 are issued half by group 0 in MEM0(s)
// and half by group 1 in MEM1(s) (one tap: group 0 the input pieces, group 1 all weight pieces), so
// the CU fetches during both segments.  Group 1 may overwrite step s's slot only once all four of its
// waves have read their step-s fragments: each wave, once its reads have returned, bumps an LDS
// counter, and waits for it to reach 4 (s + 2) before issuing: group 0's waves bump it once too,
// after their step-0 reads (made before the loop, in segment 0, the segment in which group 1 refills
// step 0's slot with step 2 -- without them in the count that refill raced those reads and the last
// clip's output differed between runs, tools/determinism_check.py).  Group 1 retires its pieces at
// the end of MEM1(s + 1), before the barrier that opens MEM0(s + 1), their first reader.
// BN = 256: 256 x 256 tiles of 64 x 128 wave tiles (Cout % 256 == 0); BN = 128: 384 x 128 tiles of
// 48 x 128 wave tiles (the C = 128 stage: 72 MFMAs per segment against x3dq's 48).
template <int HALO, bool SPLIT, int BN = 256>
__device__ __forceinline__ void x3dw_tile(const ConvParams& p, const ConvParams& pr, const int wg, const int b, const int ph) {
  constexpr int BM = BN == 256 ? 256 : 384, WN = BN / 128, WM = 8 / WN;
  constexpr int WR = BM / WM, WC = 128, TM = WR / 16, TN = WC / 16;
  constexpr int AR = BM + HALO;                 // rows of an input image
  constexpr int A_N = AR / 8, B_N = BN / 8;     // 1 KiB DMA instructions per A chunk / B step
  constexpr int A_PW = A_N / 4;                 // A pieces per group-0 wave
  constexpr int ABUF = AR * 128, BBUF = BN * 128;  // bytes
  constexpr int NA = 2;                         // A buffers (halo: chunk parity; one tap: step slot)
  constexpr int LDS_B = NA * ABUF + 2 * BBUF;
  static_assert(A_N % 4 == 0 && B_N % 4 == 0 && AR % 64 == 0, "tile shape");
  static_assert(LDS_B + 16 <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) unsigned short lds[LDS_B / 2 + 8];  // + group 1's read counter
  unsigned int* const rd_cnt = reinterpret_cast<unsigned int*>(lds + LDS_B / 2);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int group = __builtin_amdgcn_readfirstlane(tid >> 8);
  const int gw = __builtin_amdgcn_readfirstlane((tid >> 6) & 3);
  const int wm = wave / WN, wn = wave % WN;
  const int ntiles = p.Cout / BN;
  const int mt = wg / ntiles, nt = wg - mt * ntiles;
  const int q0 = mt * BM, co0 = nt * BN;
  const int nchunks = p.Cin / 32;
  const int taps = p.taps;
  const int nsteps = nchunks * taps;
  const int lo_rel = p.in_step < 0 ? (taps - 1) * p.in_step : 0;
  const int row0 = q0 + p.in_base[ph] + lo_rel;
  const int arow = p.ldx * 4;  // bytes per h2 row
  const __amdgpu_buffer_rsrc_t rx =
      HALO ? __builtin_amdgcn_make_buffer_rsrc((void*)(p.x6 + (long long)b * p.x_bstride * 2), 0, p.Lin * arow, 0x00020000)
           : __builtin_amdgcn_make_buffer_rsrc((void*)(p.x6 + ((long long)b * p.x_bstride + (long long)row0 * p.ldx) * 2), 0,
                                               max(0, min(BM, p.Lin - row0)) * arow, 0x00020000);
  const int rbase = HALO ? row0 : 0;  // row of image row 0 relative to the descriptor
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.w3 + (long long)ph * taps * nchunks * p.Cout * 64), 0, taps * nchunks * p.Cout * 128, 0x00020000);

  // DMA (group 0 alone): instruction k fills 64 rows of piece (k * 64) / rows; the wave's i-th is
  // k = i * 4 + gw.  Lane part of the source offset in one VGPR, the rest wave-uniform.  (Group 1
  // issuing half of the weight pieces from inside its MFMA segment, so that the DMA of a step is in
  // flight in both segments, measured slower: C2 194.2-194.7 against 185.3-185.4 ms, r05n; the
  // issue stalls behind group 0's and holds up the MFMAs.)
  const int a_lane = (rbase + lane) * arow;  // negative rows: huge unsigned, out of range (zeros)
  const int b_lane = (co0 + lane) * 128;
  [[maybe_unused]] bool in_loop = false;  // -DDCX_X3_NODMA (diagnostic): no DMA after the prologue (wrong results)
  auto dmaA1 = [&](int c, int slot, int i) {  // the wave's i-th A piece of chunk c
#ifdef DCX_X3_NODMA
    if (in_loop) return;
#endif
    const int k = i * 4 + gw;
    const int u = k * 64, pc = u / AR, row = u - pc * AR;
    const int abuf = HALO ? (c & 1) : slot;
    dma16(rx, lds + abuf * (ABUF / 2) + k * 512, a_lane + row * arow + (pc & 3) * 32 + (pc >> 2) * 16 + c * 128, 0);
  };
  // B instructions [0, B_G0) are group 0's, [B_G0, B_N) group 1's (SPLIT)
#ifndef DCX_X3W_BG0_DIV  // A/B builds: group 0's share of the weight pieces, 1 / DIV (halo convs)
#define DCX_X3W_BG0_DIV 2
#endif
  constexpr int B_G0 = !SPLIT ? B_N : HALO ? B_N / DCX_X3W_BG0_DIV : 0;
  constexpr int B_W0 = B_G0 / 4, B_W1 = (B_N - B_G0) / 4;  // B pieces per wave of group 0 / 1
  auto dmaB1 = [&](int c, int m, int slot, int i) {  // the wave's i-th B piece of step (c, m)
#ifdef DCX_X3_NODMA
    if (in_loop) return;
#endif
    const int k = (group ? B_G0 : 0) + i * 4 + gw;
    const int u = k * 64, pc = u / BN, col = u - pc * BN;
    dma16(rw, lds + NA * ABUF / 2 + slot * (BBUF / 2) + k * 512, b_lane + col * 128 + (pc & 3) * 32 + (pc >> 2) * 16,
          (m * nchunks + c) * p.Cout * 128);
  };
  auto dma_step = [&](int c, int m, int slot) {  // group 0's pieces of a step (its input chunk first)
    if (m == 0) {
#pragma unroll
      for (int i = 0; i < A_PW; ++i) dmaA1(c, slot, i);
    }
#pragma unroll
    for (int i = 0; i < B_W0; ++i) dmaB1(c, m, slot, i);
  };
  auto dma_step1 = [&](int c, int m, int slot) {  // group 1's (SPLIT)
#pragma unroll
    for (int i = 0; i < B_W1; ++i) dmaB1(c, m, slot, i);
  };

  // fragment addresses: one lane base per operand (h piece of the lane's channel group kg); the
  // l piece, row / column blocks and the B slot are immediate offsets
  const int l15 = lane & 15, kg = lane >> 4;
  const char* const ldsb = reinterpret_cast<const char*>(lds);
  const char* const a_rd = ldsb + kg * AR * 16 + (wm * WR + l15) * 16;
  const char* const b_rd = ldsb + NA * ABUF + kg * BN * 16 + (wn * WC + l15) * 16;
  s16x8 aq[TM][2], bq[TN][2];  // [h, l]
  auto readF = [&](int c, int m, int slot) {
    const char* a = a_rd + ((HALO ? (c & 1) : slot) * ABUF + (m * p.in_step - lo_rel) * 16);
    const char* bb = b_rd + slot * BBUF;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      bq[j][0] = *reinterpret_cast<const s16x8*>(bb + j * 256);
      bq[j][1] = *reinterpret_cast<const s16x8*>(bb + j * 256 + 4 * BN * 16);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      aq[i][0] = *reinterpret_cast<const s16x8*>(a + i * 256);
      aq[i][1] = *reinterpret_cast<const s16x8*>(a + i * 256 + 4 * AR * 16);
    }
  };
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mfma = [&]() {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int sa = k == 1 ? 1 : 0, sb = k == 0 ? 1 : 0;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, aq[i][sa]),
                                                             __builtin_bit_cast(f16x8, bq[j][sb]), acc[i][j], 0, 0, 0);
      }
    }
    __builtin_amdgcn_s_setprio(0);
  };
  auto adv = [&](int& c_, int& m_) {
    if (++m_ == taps) { m_ = 0; ++c_; }
  };

  // prologue: steps 0 and 1, drained
  int cl = 0, ml = 0;  // the next step this group issues
  if (SPLIT && tid == 0) *rd_cnt = 0u;
  for (int t = 0; t < 2 && t < nsteps; ++t) {
    if (group == 0) dma_step(cl, ml, t);
    else if (SPLIT) dma_step1(cl, ml, t);
    adv(cl, ml);
  }
  // the epilogue's range values and the input's unscale, in flight with the prologue's DMA
  const EpiPre epre = epi_range_pre<HALO == 0 ? 3 : 0>(p, pr, b);
  const float unscale = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int,
      __builtin_ldexpf(1.0f, -(p.w3_shift + (pr.x_ash ? pr.x_ash[b] : pr.x_ash_c))))));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  seg_barrier();
  in_loop = true;
#ifdef DCX_SEG_DIAG
  unsigned long long sd[6] = {};
#endif
  int cr = 0, mr = 0;
  if (group == 0) {
    readF(0, 0, 0);
    if (SPLIT) {  // step 0's slot is refilled by group 1 in segment 0: count these reads too
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_fetch_add(rd_cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    adv(cr, mr);
    for (int s = 0; s < nsteps; ++s) {
      DCX_SEGT(ta);
      mfma();  // MFMA(s)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // step s + 1 (issued in MEM0(s - 1)) landed
      DCX_SEGT(tb);
      seg_barrier();
      DCX_SEGT(tc);
      // MEM0(s): issue step s + 2 into step s's slot, fragments of step s + 1 (reads first: same
      // times, r05q)
      if (s + 2 < nsteps) {
        dma_step(cl, ml, s & 1);
        adv(cl, ml);
      }
      DCX_SEGT(tr);
      if (s + 1 < nsteps) readF(cr, mr, (s + 1) & 1);
      DCX_SEGT(tq);
      DCX_SEGT(td);
      seg_barrier();
      DCX_SEGT(te);
#ifdef DCX_SEG_DIAG
      sd[0] += tb - ta; sd[1] += tc - tb; sd[2] += td - tc; sd[3] += te - td; sd[4] += tr - tc; sd[5] += tq - tr;
#endif
      adv(cr, mr);
    }
  } else {
    for (int s = 0; s < nsteps; ++s) {
      DCX_SEGT(ta);
      readF(cr, mr, s & 1);  // MEM1(s): fragments of step s
      if (SPLIT) {
        int n = 0;
        if (s + 2 < nsteps) {  // this group's pieces of step s + 2, into step s's slot once read
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          if (lane == 0) __hip_atomic_fetch_add(rd_cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          const unsigned int want = 4u * (unsigned)(s + 2);  // + group 0's four step-0 reads
          while (__hip_atomic_load(rd_cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < want) {
          }
          dma_step1(cl, ml, s & 1);
          adv(cl, ml);
          n = B_W1;
        }
        wait_dma(n);  // step s + 1's pieces (issued in MEM1(s - 1)) landed
      }
      DCX_SEGT(tb);
      seg_barrier();
      DCX_SEGT(tc);
      mfma();  // MFMA(s)
      DCX_SEGT(td);
      seg_barrier();
      DCX_SEGT(te);
#ifdef DCX_SEG_DIAG
      sd[2] += tb - ta; sd[3] += tc - tb; sd[0] += td - tc; sd[1] += te - td; sd[5] += tb - ta;
#endif
      adv(cr, mr);
    }
  }
#ifdef DCX_SEG_DIAG
  if ((threadIdx.x & 255) == 0) {
#pragma unroll
    for (int i = 0; i < 6; ++i) atomicAdd(&g_seg_diag[group * 6 + i], sd[i]);
    if (group == 0) atomicAdd(&g_seg_diag[12], (unsigned long long)nsteps);
  }
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < 6; ++i) atomicAdd(&g_seg_diag8[wave * 6 + i], sd[i]);
    if (wave == 0) atomicAdd(&g_seg_diag8[48], (unsigned long long)nsteps);
  }
#endif
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // undo the weight and the input's range scaling (powers of two: exact)
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] *= unscale;
  epilogue_lds<BM, BN, WM, WN, LDS_B / 4, 512, HALO == 0 ? 3 : 0>(p, pr, acc, q0, co0, b, ph, reinterpret_cast<float*>(lds), &epre);
}

template <int HALO, bool SPLIT, int BN = 256>
__global__ void __launch_bounds__(512, 2) conv_gemm_x3dw(const ConvParams p) {
  constexpr int BM = BN == 256 ? 256 : 384;
  int wg, b, ph;
  flat_tile(((p.Lq + BM - 1) / BM) * (p.Cout / BN), p.batch, wg, b, ph);
  x3dw_tile<HALO, SPLIT, BN>(p, p, wg, b, ph);
}

template <bool SPLIT, int BN = 256>
__global__ void __launch_bounds__(512, 2) conv_gemm_x3dw_group(const ConvGroup g) {
  const int t = blockIdx.x;
  const int k = t >= g.start[1] ? (t >= g.start[2] ? 2 : 1) : 0;
  const int local = xcd_remap(t - g.start[k], g.start[k + 1] - g.start[k]);
  const int b = local / g.tiles_per_clip[k];
  ConvParams p;  // a private copy of the main-loop fields (pr: the range fields, read in place by the epilogue)
  if (k == 0) p = g.p[0];
  else if (k == 1) p = g.p[1];
  else p = g.p[2];
  const ConvParams& pr = k == 0 ? g.p[0] : k == 1 ? g.p[1] : g.p[2];
  x3dw_tile<64, SPLIT, BN>(p, pr, local - b * g.tiles_per_clip[k], b, 0);
}

// Whether conv_gemm_x3dq<bn> (taps >= 3 with a halo) or conv_gemm_x3dm<bn> (one tap) takes an h3
// conv (input in the h2 layout, x_compact == 3).
// wide (conv_gemm_x3dw): taps >= 2 (its input buffer is free two segments before it is refilled)
static bool x3dq_ok(const ConvParams& p, int bn, bool wide = false) {
  const int span = (p.taps - 1) * (p.in_step < 0 ? -p.in_step : p.in_step);
  if (!p.x6 || !p.w3 || p.x_compact != 3 || p.Cin % 32 || p.Cout % bn || p.ksplit > 1) return false;
  const long long arow = (long long)p.ldx * 4;
  if ((long long)p.taps * p.Cin * p.Cout * 4 >= (1LL << 31)) return false;
  if (p.taps == 1) {  // per-tile descriptor: every phase's rows start at or after the tile's
    for (int i = 0; i < kMaxPhases; ++i)
      if (p.in_base[i] < 0) return false;
    return 256LL * arow < (1LL << 31);
  }
  return p.taps >= (wide ? 2 : 3) && span > 0 && span <= 64 && (long long)(p.Lin + 1024) * arow < (1LL << 31);
}
// Tiles of an h3 conv: 256 x 256 (conv_gemm_x3dw) where Cout % 256 == 0, else 256 x 128.  (256 x 128
// against 128 x 256: half the weight DMA per step, C2 205.1 -> 193.2 ms, r05i.)  Knobs::h3_bn
// (DCX_H3_BN, A/B): 128 = the 256 x 128 tiles everywhere, 256 = the 128 x 256 ones at Cout % 256 == 0.
// Returns the column tile, 512 standing for the 256 x 256 kernel.
// 384 stands for the 384 x 128 conv_gemm_x3dw (Cout % 256 != 0, taps >= 2; DCX_H3_BN=128 keeps the
// 256 x 128 conv_gemm_x3dq there where it can, taps >= 3).
static int x3dq_bn(const ConvParams& p) {
  const int k = p.kn ? p.kn->h3_bn : 0;
  if (p.Cout % 256) return (k == 128 && p.taps >= 3) || p.taps < 2 ? 128 : 384;
  return k == 128 ? 128 : k == 256 ? 256 : 512;
}

// ---------------------------------------------------------------------------------------------
// conv_gemm_bf16dm: the DCX_GEMM_BF16 mode's 1x1 convs (one hi * hi' product, the reference's
// enable_bfloat16 autocast) on the LDS-DMA ping-pong schedule of conv_gemm_x6dm.
//
// A step is K32 (two K16 chunks, hi planes only: 4 pieces of 16 B per row), 16x16x32 MFMAs on
// 64 x 128 wave tiles: 32 MFMAs against 12 fragment reads per segment.  A and B ride one 3-slot
// ring (step t in slot t % 3, 16 + 16 KiB per slot), issued by group 0 in MEM0(t - 3) and group 1
// in MEM1(t - 2) and retired one memory segment later.  LDS images: 16-row blocks, piece-major
// (16-byte unit (r >> 4) * 64 + piece * 16 + (r & 15), piece = 8-channel group of the step).
// ---------------------------------------------------------------------------------------------
//
// REG (round 3): launches whose epilogue is bias or GELU with a compact bf16 output only (the
// encoder's pwconv1) swap the MFMA operands, so a lane's 16x16 accumulator holds 4 consecutive
// output channels of one row, and finish the tile straight from registers (8-byte compact stores):
// no LDS staging, no barriers.  The pwconv1 launches had spent 24 us per tile in the LDS-staged
// epilogue against 8 us in their K loop (C = 256).  The swap transposes each 16x16 product (the
// same K products summed per element), so the bits are those of the staged epilogue.
template <bool REG>
__global__ void __launch_bounds__(512, 2) conv_gemm_bf16dm(const ConvParams p) {
  DCX_TILET(tile_t0);
  constexpr int BM = 256, BN = 256, WN = 2, WM = 4;
  constexpr int WR = 64, WC = 128, TM = WR / 16, TN = WC / 16;
  constexpr int A_G = BM * 4 / 128, B_G = BN * 4 / 128;  // DMA instructions per group per step
  constexpr int A_PW = A_G / 4, B_PW = B_G / 4;
  constexpr int ABUF = BM * 4 * 8, BBUF = BN * 4 * 8;    // ushorts
  constexpr int LDS_US = 3 * (ABUF + BBUF);               // 96 KiB
  __shared__ __attribute__((aligned(16))) unsigned short lds[LDS_US];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int group = __builtin_amdgcn_readfirstlane(tid >> 8);
  const int gw = __builtin_amdgcn_readfirstlane((tid >> 6) & 3);
  const int wm = wave / WN, wn = wave % WN;
  const int ntiles = p.Cout / BN;
  int wg, b, ph;
  flat_tile(((p.Lq + BM - 1) / BM) * ntiles, p.batch, wg, b, ph);
  const int mt = wg / ntiles, nt = wg - mt * ntiles;
  const int q0 = mt * BM, co0 = nt * BN;
  const int nsteps = p.Cin / 32;
  // input: planes (hi pieces at 48-byte strides, 6 bytes per element) or compact bf16 (x_compact:
  // one contiguous 64-byte run per row and step); weights: planes w6 or compact wc likewise
  const int xc = p.x_compact == 1 ? 1 : 3;
  const int arow = p.ldx * 2 * xc, a_kq = 16 * xc, a_step = 64 * xc;
  const int row0 = q0 + p.in_base[ph];  // >= 0 for 1x1 convs; the descriptor covers the tile's rows
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.x6 + ((long long)b * p.x_bstride + (long long)row0 * p.ldx) * xc), 0,
      max(0, min(BM, p.Lin - row0)) * arow, 0x00020000);
  const bool wc = p.wc != nullptr;
  const __amdgpu_buffer_rsrc_t rw =
      wc ? __builtin_amdgcn_make_buffer_rsrc((void*)(p.wc + (long long)ph * (p.Cin / 32) * p.Cout * 32), 0,
                                             (p.Cin / 32) * p.Cout * 64, 0x00020000)
         : __builtin_amdgcn_make_buffer_rsrc((void*)(p.w6 + (long long)ph * (p.Cin / 16) * p.Cout * 48), 0,
                                             (p.Cin / 16) * p.Cout * 96, 0x00020000);
  const int b_step = wc ? p.Cout * 64 : p.Cout * 192;

  // DMA pieces (bytes, step 0): unit u -> row (u / 64) * 16 + (u & 15), piece (u % 64) >> 4 = the
  // 8-channel group kq; step s adds s * a_step (input) and s * b_step (weights: two K16 chunks)
  int a_off[A_PW], b_off[B_PW];
#pragma unroll
  for (int i = 0; i < A_PW; ++i) {
    const int u = (group * A_G + i * 4 + gw) * 64 + lane;
    const int r = (u >> 6) * 16 + (u & 15), kq = (u & 63) >> 4;
    a_off[i] = r * arow + kq * a_kq;  // rows past Lin: out of range, zeros
  }
#pragma unroll
  for (int i = 0; i < B_PW; ++i) {
    const int u = (group * B_G + i * 4 + gw) * 64 + lane;
    const int c = (u >> 6) * 16 + (u & 15), kq = (u & 63) >> 4;
    b_off[i] = wc ? (co0 + c) * 64 + kq * 16 : (kq >> 1) * p.Cout * 96 + (co0 + c) * 96 + (kq & 1) * 48;
  }
  unsigned short* const a_dst = lds + (group * A_G + gw) * 512;
  unsigned short* const b_dst = lds + 3 * ABUF + (group * B_G + gw) * 512;
  auto dma_step = [&](int s, int slot) {
#pragma unroll
    for (int i = 0; i < A_PW; ++i) dma16(rx, a_dst + slot * ABUF + i * 2048, a_off[i] + s * a_step, 0);
#pragma unroll
    for (int i = 0; i < B_PW; ++i) dma16(rw, b_dst + slot * BBUF + i * 2048, b_off[i], s * b_step);
    return A_PW + B_PW;
  };

  const int l15 = lane & 15, kq = lane >> 4;
  const char* const ldsb = reinterpret_cast<const char*>(lds);
  const int a_lane = (wm * WR / 16) * 1024 + kq * 256 + l15 * 16;           // bytes in an A image
  const int b_lane = 6 * ABUF + (wn * WC / 16) * 1024 + kq * 256 + l15 * 16;  // bytes, B image of slot 0
  s16x8 af[TM], bq[TN];
  auto readF = [&](int slot) {
#pragma unroll
    for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const s16x8*>(ldsb + slot * ABUF * 2 + a_lane + i * 1024);
#pragma unroll
    for (int j = 0; j < TN; ++j) bq[j] = *reinterpret_cast<const s16x8*>(ldsb + slot * BBUF * 2 + b_lane + j * 1024);
  };
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mfma = [&]() {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        if constexpr (REG)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, bq[j]),
                                                              __builtin_bit_cast(bf16x8, af[i]), acc[i][j], 0, 0, 0);
        else
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af[i]),
                                                              __builtin_bit_cast(bf16x8, bq[j]), acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto inc3 = [](int& slot) { slot = slot == 2 ? 0 : slot + 1; };

  for (int t = 0; t < 3; ++t)
    if (t < nsteps) dma_step(t, t);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  seg_barrier();
  DCX_TILET(tile_t1);
#ifdef DCX_CLOCK_DIAG
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
#endif
  if (group == 0) {
    readF(0);
    int rs = 1, ws = 0;
    for (int s = 0; s < nsteps; ++s) {
      mfma();  // MFMA(s)
      seg_barrier();
      if (s + 1 < nsteps) readF(rs);  // MEM0(s): fragments of step s + 1, issue step s + 3
      int n = 0;
      if (s + 3 < nsteps) n = dma_step(s + 3, ws);
      wait_dma(n);
      seg_barrier();
      inc3(rs);
      inc3(ws);
    }
  } else {
    int rs = 0, ws = 0;
    for (int s = 0; s < nsteps; ++s) {
      readF(rs);  // MEM1(s): fragments of step s, issue step s + 2 (s >= 1)
      int n = 0;
      if (s >= 1 && s + 2 < nsteps) n = dma_step(s + 2, ws);
      wait_dma(n);
      seg_barrier();
      mfma();  // MFMA(s)
      seg_barrier();
      inc3(rs);
      if (s >= 1) inc3(ws);
      else ws = 0;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef DCX_CLOCK_DIAG
  if (threadIdx.x == 0) {  // steps counted in units of 1536 ideal cycles (a K32 step is 1024)
    atomicAdd(&g_clock_diag[0], __builtin_amdgcn_s_memtime() - t0);
    atomicAdd(&g_clock_diag[1], __builtin_amdgcn_s_memrealtime() - r0);
    atomicAdd(&g_clock_diag[2], (unsigned long long)(nsteps * 2 / 3));
  }
#endif
  DCX_TILET(tile_t2);
  if constexpr (REG) {
    // lane l of block (i, j): output channels co0 + wn*WC + 16 j + 4 (l >> 4) + e of row 16 i + (l & 15)
    // of the wave's rows.  epilogue_lds's operations in its order: bias, bf16 rounding, GELU, the
    // RNE compact store.
#ifdef DCX_DIAG_DUP
    if (p.diag_skip == 2) return;  // the timing copy of a launch: main loop only
#endif
    unsigned short* const y6 = p.y6 + (long long)b * p.y_bstride;
    const int cq = co0 + wn * WC + 4 * (lane >> 4);
    f32x4 bias[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j)
      bias[j] = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + cq + 16 * j) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int q = q0 + wm * WR + 16 * i + (lane & 15);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        f32x4 x = acc[i][j] + bias[j];
        if (p.round_bf16) x = round_bf16x4(x);
        if (p.epi == EPI_GELU) {
          if (p.round_bf16) {
            const f32x2 g0 = gelu_bf16_f2(f32x2{x[0], x[1]}), g1 = gelu_bf16_f2(f32x2{x[2], x[3]});
            x = f32x4{g0[0], g0[1], g1[0], g1[1]};  // (the compact store rounds)
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) x[e] = gelu_f(x[e]);
          }
        }
#ifdef DCX_DIAG_DUP
        if (p.diag_skip == 1 && x[0] != -0x1.234p-100f) continue;  // timing copy: computed, not stored
#endif
        if (q < p.Lq) store_bf16x4(y6, q, p.Cout, cq + 16 * j, x[0], x[1], x[2], x[3]);
      }
    }
  } else {
    epilogue_lds<BM, BN, WM, WN, LDS_US / 2, 512>(p, p, acc, q0, co0, b, ph, reinterpret_cast<float*>(lds));
  }
#ifdef DCX_TILE_DIAG
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long t3 = __builtin_amdgcn_s_memrealtime();
    const unsigned int k = atomicAdd(&g_tile_cnt, 1u);
    if (k < (unsigned)kTileDiagMax) {
      unsigned long long* o = g_tile_diag + 6ull * k;
      o[0] = tile_t0; o[1] = tile_t1; o[2] = tile_t2; o[3] = t3;
      o[4] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
      o[5] = __builtin_amdgcn_s_getreg((15 << 11) | 20) | ((unsigned long long)nsteps << 16);  // + K32 steps
    }
  }
#endif
}

// ---------------------------------------------------------------------------------------------
// conv_gemm_bf16dp (round 4): conv_gemm_bf16dm<REG> made persistent, with one step stream across
// tiles.  A workgroup walks its tiles (XCD-grouped logical order, as conv_gemm_x6w8) and the ping-pong
// step schedule never drains: the DMA of the next tile's first steps is issued during the current
// tile's last ones (the ring slot of global step g is g % 3), so a tile costs no prologue.  Each
// group finishes its tile from registers in the memory segment that follows its last MFMA segment,
// while the other group runs an MFMA segment: group 0 in MEM0 of the tile's last step, group 1 in
// MEM1 of the next tile's first step.  The register epilogue (bias, bf16 rounding, GELU, 8-byte RNE
// compact stores) is bf16dm<true>'s, after the segment's fragment reads and DMA wait, so its stores
// only have to have drained by the next memory segment's wait.  Same MFMAs in the same order per
// tile: the bits of conv_gemm_bf16dm<true> (tests/test_gpu_bf16.py::test_persistent_same_bits).
// GELU launches finish from the LDS table of the bf16 GELU (gelu_lut_fill, filled while the first
// steps' DMA is in flight).  Takes compact input and weights (x_compact == 1, wc), bf16 rounding,
// >= 3 K32 steps, one phase.
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(512, 2) conv_gemm_bf16dp(const ConvParams p) {
  constexpr int BM = 256, BN = 256, WN = 2;
  constexpr int WR = 64, WC = 128, TM = WR / 16, TN = WC / 16;
  constexpr int A_G = BM * 4 / 128, B_G = BN * 4 / 128;  // DMA instructions per group per step
  constexpr int A_PW = A_G / 4, B_PW = B_G / 4;
  constexpr int ABUF = BM * 4 * 8, BBUF = BN * 4 * 8;    // ushorts
  constexpr int LDS_US = 3 * (ABUF + BBUF);               // 96 KiB
  // LDS: the GELU table at byte 0, the launch's bias (fp32, Cout <= kBiasMax), the ring
  constexpr int BIAS_US = 2 * kBf16dpBiasMax, RING_US = kGeluLutUs + BIAS_US;
  __shared__ __attribute__((aligned(16))) unsigned short smem[RING_US + LDS_US];
  unsigned short* const lds = smem + RING_US;
  float* const bias_s = reinterpret_cast<float*>(smem + kGeluLutUs);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int group = __builtin_amdgcn_readfirstlane(tid >> 8);
  const int gw = __builtin_amdgcn_readfirstlane((tid >> 6) & 3);
  const int wm = wave / WN, wn = wave % WN;
  const int ntn = p.Cout / BN, mtiles = (p.Lq + BM - 1) / BM;
  const int per_img = mtiles * ntn, total = per_img * p.batch;
  const int G = gridDim.x;  // a multiple of 8
  const int tile_base = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  const int nt_block = tile_base < total ? (total - tile_base + G - 1) / G : 0;  // tiles of this block
  if (nt_block == 0) return;  // whole workgroup, before any barrier
  const bool lut = p.gelu_lut > 0 && p.epi == EPI_GELU;
  const int nsteps = p.Cin / 32;
  const int gtot = nt_block * nsteps;  // steps of the block's stream
  const int arow = p.ldx * 2;          // compact rows
  const int b_step = p.Cout * 64;

  // tile k of this block -> (clip, first row, first column)
  auto tile_of = [&](int k, int& b, int& q0, int& co0) {
    const int L = tile_base + k * G;
    b = L / per_img;
    const int wg = L - b * per_img;
    const int mt = wg / ntn;
    q0 = mt * BM;
    co0 = (wg - mt * ntn) * BN;
  };
  auto rx_of = [&](int b, int q0) {  // descriptor over the tile's rows (rows past Lin read zeros)
    const int row0 = q0 + p.in_base[0];
    return __builtin_amdgcn_make_buffer_rsrc((void*)(p.x6 + (long long)b * p.x_bstride + (long long)row0 * p.ldx), 0,
                                             max(0, min(BM, p.Lin - row0)) * arow, 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.wc, 0, (p.Cin / 32) * p.Cout * 64, 0x00020000);

  int a_off[A_PW], b_off[B_PW];
#pragma unroll
  for (int i = 0; i < A_PW; ++i) {
    const int u = (group * A_G + i * 4 + gw) * 64 + lane;
    const int r = (u >> 6) * 16 + (u & 15), kq = (u & 63) >> 4;
    a_off[i] = r * arow + kq * 16;
  }
#pragma unroll
  for (int i = 0; i < B_PW; ++i) {
    const int u = (group * B_G + i * 4 + gw) * 64 + lane;
    const int c = (u >> 6) * 16 + (u & 15), kq = (u & 63) >> 4;
    b_off[i] = c * 64 + kq * 16;  // + co0 * 64 in the scalar offset
  }
  unsigned short* const a_dst = lds + (group * A_G + gw) * 512;
  unsigned short* const b_dst = lds + 3 * ABUF + (group * B_G + gw) * 512;
  // DMA of global step g (tile g / nsteps of the stream, K32 step g % nsteps)
  int dk = -1, db = 0, dq0 = 0, dco0 = 0;
  __amdgpu_buffer_rsrc_t drx = rw;
  auto dma_step = [&](int g, int slot) __attribute__((always_inline)) {
    const int k = g / nsteps, st = g - k * nsteps;
    if (k != dk) {  // wave-uniform
      dk = k;
      tile_of(k, db, dq0, dco0);
      drx = rx_of(db, dq0);
    }
#pragma unroll
    for (int i = 0; i < A_PW; ++i) dma16(drx, a_dst + slot * ABUF + i * 2048, a_off[i] + st * 64, 0);
#pragma unroll
    for (int i = 0; i < B_PW; ++i) dma16(rw, b_dst + slot * BBUF + i * 2048, b_off[i], st * b_step + dco0 * 64);
    return A_PW + B_PW;
  };

  const int l15 = lane & 15, kq = lane >> 4;
  const char* const ldsb = reinterpret_cast<const char*>(lds);
  const int a_lane = (wm * WR / 16) * 1024 + kq * 256 + l15 * 16;
  const int b_lane = 6 * ABUF + (wn * WC / 16) * 1024 + kq * 256 + l15 * 16;
  s16x8 af[TM], bq[TN];
  auto readF = [&](int slot) {
#pragma unroll
    for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const s16x8*>(ldsb + slot * ABUF * 2 + a_lane + i * 1024);
#pragma unroll
    for (int j = 0; j < TN; ++j) bq[j] = *reinterpret_cast<const s16x8*>(ldsb + slot * BBUF * 2 + b_lane + j * 1024);
  };
  f32x4 acc[TM][TN];
  auto zero = [&]() {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  zero();
  auto mfma = [&]() {  // operands swapped: a lane's accumulator holds 4 consecutive channels of a row
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, bq[j]),
                                                            __builtin_bit_cast(bf16x8, af[i]), acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // the register epilogue of tile k, then the accumulators cleared.  GELU launches: from the table;
  // a wave with an element outside it stores the evaluated epilogue (conv_gemm_bf16dm<true>'s) over it
  auto epilogue = [&](int k) __attribute__((always_inline)) {
    int bb, q0, co0;
    tile_of(k, bb, q0, co0);
    const int cq = co0 + wn * WC + 4 * (lane >> 4);
    const int rq = wm * WR + (lane & 15);  // + 16 i: the lane's rows in the tile
    bool eval = !lut;
    if (lut) {
      // buffer stores over the tile's valid rows (rows past Lq are dropped by the descriptor)
      const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(p.y6 + (long long)bb * p.y_bstride + (long long)q0 * p.Cout), 0, min(BM, p.Lq - q0) * p.Cout * 2,
          0x00020000);
      u16x2 hi = {0, 0};
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const f32x4 bias = *reinterpret_cast<const f32x4*>(bias_s + cq + 16 * j);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const f32x4 x = acc[i][j] + bias;
          typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
          const u32x2 w = {gelu_lut2(smem, f32x2{x[0], x[1]}, hi), gelu_lut2(smem, f32x2{x[2], x[3]}, hi)};
          __builtin_amdgcn_raw_buffer_store_b64(w, ry, ((rq + 16 * i) * p.Cout + cq + 16 * j) * 2, 0, 0);
        }
      }
      eval = __builtin_amdgcn_ballot_w64(max(hi[0], hi[1]) >= p.gelu_lut) != 0;  // wave-uniform
      if (eval) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the table's stores first
    }
    if (eval) {  // conv_gemm_bf16dm<true>'s evaluated epilogue
      unsigned short* const y6 = p.y6 + (long long)bb * p.y_bstride;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const f32x4 bias = *reinterpret_cast<const f32x4*>(bias_s + cq + 16 * j);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int q = q0 + rq + 16 * i;
          f32x4 x = round_bf16x4(acc[i][j] + bias);
          if (p.epi == EPI_GELU) {
            const f32x2 g0 = gelu_bf16_f2(f32x2{x[0], x[1]}), g1 = gelu_bf16_f2(f32x2{x[2], x[3]});
            x = f32x4{g0[0], g0[1], g1[0], g1[1]};  // (the compact store rounds)
          }
          if (q < p.Lq) store_bf16x4(y6, q, p.Cout, cq + 16 * j, x[0], x[1], x[2], x[3]);
        }
      }
    }
    zero();
  };
  auto inc3 = [](int& slot) { slot = slot == 2 ? 0 : slot + 1; };

  // prologue: steps 0, 1, 2 of the stream (both groups their pieces) and the GELU table, drained
  for (int t = 0; t < 3; ++t)
    if (t < gtot) dma_step(t, t);
  if (lut) gelu_lut_fill(smem, tid, 512);
  for (int c = tid; c < p.Cout; c += 512) bias_s[c] = p.bias ? p.bias[c] : 0.0f;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  seg_barrier();
  if (group == 0) {
    readF(0);
    int rs = 1, ws = 0, st = 0, k = 0;  // st: step of the current tile k
    for (int g = 0; g < gtot; ++g) {
      mfma();  // MFMA(g)
      seg_barrier();
      // MEM0(g): fragments of g + 1, issue g + 3, retire g + 2; after a tile's last step, its epilogue
      if (g + 1 < gtot) readF(rs);
      int n = 0;
      if (g + 3 < gtot) n = dma_step(g + 3, ws);
      wait_dma(n);
      if (++st == nsteps) {
        epilogue(k);
        st = 0;
        ++k;
      }
      seg_barrier();
      inc3(rs);
      inc3(ws);
    }
  } else {
    int rs = 0, ws = 0, st = 0, k = 0;
    for (int g = 0;; ++g) {
      // MEM1(g): fragments of g, issue g + 2 (g >= 1), retire g + 1; at a tile's first step (and
      // after the stream), the previous tile's epilogue
      if (g < gtot) readF(rs);
      int n = 0;
      if (g >= 1 && g + 2 < gtot) n = dma_step(g + 2, ws);
      wait_dma(n);
      if (st == 0 && g > 0) epilogue(k - 1);
      if (g == gtot) break;
      seg_barrier();
      mfma();  // MFMA(g)
      seg_barrier();
      inc3(rs);
      if (g >= 1) inc3(ws);
      else ws = 0;
      if (++st == nsteps) {
        st = 0;
        ++k;
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// whether conv_gemm_x6dm takes the conv: planes input, Cout % 256, taps >= 2 with a halo or one
// tap without, and 32-bit buffer offsets for the input rows (with the tile's halo) and the weights
static bool in_base_nonneg(const ConvParams& p) {  // every phase's input row offset (unused entries are 0)
  for (int i = 0; i < kMaxPhases; ++i)
    if (p.in_base[i] < 0) return false;
  return true;
}

static bool x6dm_ok(const ConvParams& p, bool halo, int bn) {
  if (!p.x6 || !p.w6 || p.nprod != 6 || p.Cout % bn || (halo ? p.taps < 2 : p.taps != 1)) return false;
  const long long arow = (long long)p.ldx * 6;
  const long long wbytes = (long long)p.taps * (p.Cin / BK) * p.Cout * 96;
  if (!halo) return in_base_nonneg(p) && 1024 * arow < (1LL << 31) && wbytes < (1LL << 31);  // per-tile descriptor
  return (long long)(p.Lin + 1024) * arow < (1LL << 31) && 1024 * arow < (1LL << 31) && wbytes < (1LL << 31);
}

// Whether the 64K-output tiles of the LDS-DMA kernels (BM x bn) or the 256 x 128 tiles of
// conv_gemm_x6pp / x6lm take a conv.  Both run one workgroup per CU; the smaller tiles take half the
// time at ~0.88 of the rate, so they win when a launch has few tiles (the C5 streaming hop, short
// clips, 1x1 convs with narrow outputs such as the encoder's 4C -> C).  The rule looks at one clip
// (rows x column tiles x phases), never at the batch size: the two families sum in different
// orders, and a clip must give the same bits alone as inside a batch of equal-length clips.
// At C2's batch of 32 the threshold picks what ceil(tiles / CUs) rounds would.
static bool big_tiles_pay(const ConvParams& p, int phases, int bn) {
  const int bm = 65536 / bn;
  return (long long)((p.Lq + bm - 1) / bm) * (p.Cout / bn) * phases >= 16;
}

template <int HALO, int BN>
static hipError_t launch_x6dm(const ConvParams& p, int batch, int phases, hipStream_t s, const char** kname) {
  constexpr int BM = 65536 / BN;
  const dim3 grid((unsigned)(((p.Lq + BM - 1) / BM) * (p.Cout / BN) * batch * phases));
  ConvParams q = p;
  q.batch = batch;
  q.phases = phases;
  if (kname)
    *kname = BN == 256 ? (HALO ? "conv_gemm_x6dm<256,256,halo>" : "conv_gemm_x6dm<256,256>") : "conv_gemm_x6dm<512,128,halo>";
  hipLaunchKernelGGL((conv_gemm_x6dm<HALO, BN>), grid, dim3(512), 0, s, q);
  return hipGetLastError();
}

// Tile order of the VQ prefilters.  From 16 row panels on, groups of 16 row panels x 16 code tiles
// are resident together, 4 x 8 per XCD, so the blocks of an XCD stream the same panels through its
// L2 (ntiles % 16 == 0; grid vq_grid).  Below 16 row panels (short clips, a streaming hop) that
// order would leave most XCDs without work (a single row panel: two of eight), so the tiles are
// dealt round-robin over the blocks, code tiles spread over every XCD.  The order changes no result.
__device__ __forceinline__ void vq_tile(int mtiles, int ntiles, int& mt, int& nt) {
  const int bid = blockIdx.x;
  if (mtiles < 16) {
    mt = bid % mtiles;
    nt = bid / mtiles;
    return;
  }
  const int xc = bid & 7, l = (bid >> 3) & 31, sup = bid >> 8;
  const int nsm = (mtiles + 15) >> 4;
  mt = (sup % nsm) * 16 + (xc & 3) * 4 + (l & 3);
  nt = (sup / nsm) * 16 + (xc >> 2) * 8 + (l >> 2);
}
static unsigned vq_grid(int mtiles, int ntiles) {
  return mtiles < 16 ? (unsigned)(mtiles * ntiles) : (unsigned)(((mtiles + 15) / 16) * (ntiles / 16) * 256);
}

// ---------------------------------------------------------------------------------------------
// VQ prefilter GEMM (x6 mode): approximate x.e from hi*hi + hi*mid + mid*hi of the planes
// (bound in launch_vq_prefilter), per-tile top 2 of (x2 + e2) - 2 x.e (epilogue_top2).
//
// Same 8-wave / 256x128 / 64x64-per-wave shape as conv_gemm_x6w8, but a step covers K = 32 (two
// 16-deep sub-chunks, hi and mid planes only: 8 pieces of 16 B per row in a 144-byte LDS row,
// 36 dwords, conflict-free for b128 reads), so a step is 2 x 12 MFMAs per wave like the convs'.
// Fragments are single-buffered per sub-chunk: sub-chunk 0 of step s+1 is read from LDS while
// sub-chunk 1 of step s is on the matrix cores, and vice versa.  Loads run three steps ahead
// (input tile double buffer, weight ring of 3), stores two.
// ---------------------------------------------------------------------------------------------
// XMID = false: the rows of x are bf16 values (mid plane zero, bf16 mode), so only their hi pieces
// are staged and hi*hi + hi*mid' issued (2 products; the bound of launch_vq_prefilter still holds).
template <int BM, int BN, int WM, int WN, bool XMID>
__global__ void __launch_bounds__(512) vq_prefilter_x3(const ConvParams p) {
  static_assert(WM * WN == 8, "8 waves per workgroup");
  constexpr int WR = BM / WM, WC = BN / WN;
  constexpr int TM = WR / 32, TN = WC / 32;
  constexpr int ROW = 72;  // ushort per LDS row: 8 pieces + 1 pad piece
  constexpr int APC = XMID ? 8 : 4;  // staged pieces per input row per step
  constexpr int A_PT = BM * APC / 512, B_PT = BN * 8 / 512;
  static_assert(BM * APC % 512 == 0 && BN * 8 % 512 == 0, "staging pieces per thread");
  constexpr int ABUF = BM * ROW, BBUF = BN * ROW;
  __shared__ __attribute__((aligned(16))) unsigned short lds[2 * ABUF + 3 * BBUF];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int ntiles = p.Cout / BN;
  // grouped order: 16 row panels x 16 code tiles resident together, 4 x 8 per XCD (ntiles % 16 == 0)
  const int mtiles = (p.Lq + BM - 1) / BM;
  int mt, nt;
  vq_tile(mtiles, ntiles, mt, nt);
  if (mt >= mtiles) return;  // whole workgroup, before any barrier
    const int q0 = mt * BM, co0 = nt * BN;
  const int nsteps = p.Cin / 32;
  const long long ldx6 = (long long)p.ldx * 3;
  const long long wslab = (long long)p.Cout * 48;  // one 16-deep chunk of the split codebook

  // staging slots: piece k of a row = (sub u = k >> 2, half h = (k >> 1) & 1, plane k & 1)
  const unsigned short* a_src[A_PT];
  int a_lds[A_PT];
#pragma unroll
  for (int i = 0; i < A_PT; ++i) {
    const int idx = tid + 512 * i, row = idx / APC, k = XMID ? idx & 7 : (idx & 3) * 2;  // hi pieces only
    const int q = q0 + row;
    const int goff = (k >> 2) * 48 + ((k >> 1) & 1) * 24 + (k & 1) * 8;
    a_src[i] = q < p.Lq ? p.x6 + (long long)q * ldx6 + goff : reinterpret_cast<const unsigned short*>(g_zero_row);
    a_lds[i] = row * ROW + k * 8;
  }
  const int a_step = 96;  // ushort per step along a row (zero-page rows must not advance)
  bool a_live[A_PT];
#pragma unroll
  for (int i = 0; i < A_PT; ++i) a_live[i] = q0 + (tid + 512 * i) / APC < p.Lq;
  long long b_off[B_PT];
  int b_lds[B_PT];
#pragma unroll
  for (int i = 0; i < B_PT; ++i) {
    const int idx = tid + 512 * i, col = idx >> 3, k = idx & 7;
    b_off[i] = (long long)(co0 + col) * 48 + (k >> 2) * wslab + ((k >> 1) & 1) * 24 + (k & 1) * 8;
    b_lds[i] = col * ROW + k * 8;
  }

  f32x4 ra[2][A_PT], rb[2][B_PT];
  auto loadA = [&](int s, f32x4(&r)[A_PT]) {
#pragma unroll
    for (int i = 0; i < A_PT; ++i)
      r[i] = *reinterpret_cast<const f32x4*>(a_src[i] + (a_live[i] ? s * a_step : 0));
  };
  auto loadB = [&](int s, f32x4(&r)[B_PT]) {
    const unsigned short* base = p.w6 + (long long)s * 2 * wslab;
#pragma unroll
    for (int i = 0; i < B_PT; ++i) r[i] = *reinterpret_cast<const f32x4*>(base + b_off[i]);
  };
  auto storeA = [&](int buf, const f32x4(&r)[A_PT]) {
#pragma unroll
    for (int i = 0; i < A_PT; ++i) *reinterpret_cast<f32x4*>(lds + buf * ABUF + a_lds[i]) = r[i];
  };
  auto storeB = [&](int slot, const f32x4(&r)[B_PT]) {
#pragma unroll
    for (int i = 0; i < B_PT; ++i) *reinterpret_cast<f32x4*>(lds + 2 * ABUF + slot * BBUF + b_lds[i]) = r[i];
  };

  const int lrow = lane & 31;
  const int hoff = (lane >> 5) * 16;  // K half: pieces (h, hi), (h, mid)
  s16x8 fa[2][TM][2], fb[2][TN][2];   // [sub][tile][plane]
  auto readSub = [&](int buf, int slot, int u) {
    const unsigned short* A = lds + buf * ABUF + u * 32 + hoff;
    const unsigned short* Bs = lds + 2 * ABUF + slot * BBUF + u * 32 + hoff;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const unsigned short* ap = A + (wm * WR + i * 32 + lrow) * ROW;
      fa[u][i][0] = *reinterpret_cast<const s16x8*>(ap);
      if constexpr (XMID) fa[u][i][1] = *reinterpret_cast<const s16x8*>(ap + 8);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const unsigned short* bp = Bs + (wn * WC + j * 32 + lrow) * ROW;
      fb[u][j][0] = *reinterpret_cast<const s16x8*>(bp);
      fb[u][j][1] = *reinterpret_cast<const s16x8*>(bp + 8);
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  auto mfmaSub = [&](int u) {
    __builtin_amdgcn_s_setprio(1);  // keeps the MFMA cluster together (measured +5 %)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (XMID)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, fa[u][i][1]),
                                                              __builtin_bit_cast(bf16x8, fb[u][j][0]), acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, fa[u][i][0]),
                                                            __builtin_bit_cast(bf16x8, fb[u][j][1]), acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, fa[u][i][0]),
                                                            __builtin_bit_cast(bf16x8, fb[u][j][0]), acc[i][j], 0, 0, 0);
      }
    __builtin_amdgcn_s_setprio(0);
  };

  // prologue: steps 0 and 1 staged, step 2 in flight
  loadA(0, ra[0]);
  loadB(0, rb[0]);
  storeA(0, ra[0]);
  storeB(0, rb[0]);
  const int s1 = min(1, nsteps - 1), s2 = min(2, nsteps - 1);
  loadA(s1, ra[0]);
  loadB(s1, rb[0]);
  storeA(1, ra[0]);
  storeB(1, rb[0]);
  loadA(s2, ra[1]);
  loadB(s2, rb[1]);
  __syncthreads();
  readSub(0, 0, 0);
  readSub(0, 0, 1);

  int slot = 0;
  auto step = [&](int s, auto qtag) {
    constexpr int Q = decltype(qtag)::value;
    const int slot1 = slot == 2 ? 0 : slot + 1, slot2 = slot1 == 2 ? 0 : slot1 + 1;
    const int s3 = min(s + 3, nsteps - 1);
    loadA(s3, ra[Q]);
    loadB(s3, rb[Q]);
    mfmaSub(0);
    readSub((s + 1) & 1, slot1, 0);  // after the last step: reads unused data, no branch
    mfmaSub(1);
    readSub((s + 1) & 1, slot1, 1);
    storeB(slot2, rb[1 - Q]);
    storeA(s & 1, ra[1 - Q]);  // step s+2's tile into the buffer step s used
    __syncthreads();
    slot = slot1;
  };
  // nsteps is even (launcher): no odd exit, so the loop header never merges a path with this
  // step's loads still in flight (which made the waitcnt pass drain everything, vmcnt(0))
#ifdef DCX_CLOCK_DIAG
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
#endif
  for (int s = 0; s < nsteps; s += 2) {
    step(s, std::integral_constant<int, 0>{});
    step(s + 1, std::integral_constant<int, 1>{});
  }
#ifdef DCX_CLOCK_DIAG
  if (threadIdx.x == 0) {  // steps counted in units of 1536 ideal cycles (24 MFMAs x 2 waves per SIMD)
    atomicAdd(&g_clock_diag[0], __builtin_amdgcn_s_memtime() - t0);
    atomicAdd(&g_clock_diag[1], __builtin_amdgcn_s_memrealtime() - r0);
    atomicAdd(&g_clock_diag[2], (unsigned long long)nsteps);
  }
#endif
  epilogue_top2<BM, BN, WM, WN>(p, acc, q0, co0, nt, ntiles, reinterpret_cast<float*>(lds));
}

// ---------------------------------------------------------------------------------------------
// vq_prefilter_dm: the VQ prefilter on the conv_gemm_x6dm schedule.
//
// vq_prefilter_x3 issues its MFMAs about half of the time: with 64 x 64 wave tiles its LDS traffic
// (16 fragment reads and 6 register-staged stores per 24 MFMAs) is close to the LDS bandwidth, and
// moving it to LDS-DMA alone did not help.  Here the tiles are 256 x 256 with 64 x 128 wave tiles
// (12 fragment reads per 24 MFMAs, no ds_write pass), staged by LDS-DMA into a 3-slot ring and
// run on the two-group ping-pong schedule of conv_gemm_x6dm (1-tap: every K16 step brings its own
// input and codebook tiles).  Each input row panel is also re-read by half as many code tiles.
// The products per K16 (m*h', h*m', h*h', in that order, on 32x32x16) and so the error bound of
// launch_vq_prefilter are those of vq_prefilter_x3.
// LDS images: 64-byte rows holding the hi and mid pieces of both K halves (piece = half * 2 +
// plane) in slot piece ^ ((row >> 2) & 3), which keeps every 16-lane group of a b128 fragment read
// on 64 distinct banks; lane-linear per DMA instruction, the swizzle applied on the source.
// Rows past the input end are outside the (per-tile) buffer descriptor and load zeros.
// XMID = false (bf16 mode, mid plane of x zero): the m*h' MFMA is skipped.
// ---------------------------------------------------------------------------------------------
template <bool XMID>
__global__ void __launch_bounds__(512, 2) vq_prefilter_dm(const ConvParams p) {
  constexpr int BM = 256, BN = 256, WN = 2;
  constexpr int WR = BM / 4, WC = BN / 2, TM = WR / 32, TN = WC / 32;
  constexpr int RW = 32;                          // ushorts per LDS row
  constexpr int G_I = BM * 4 / 64 / 2;            // DMA instructions per group per tile (A or B)
  constexpr int PW = G_I / 4;                     // ... per wave
  constexpr int ABUF = BM * RW, BBUF = BN * RW;
  constexpr int LDS_US = 3 * ABUF + 3 * BBUF;
  static_assert(BM == BN && G_I % 4 == 0 && LDS_US * 2 <= 160 * 1024, "tile shape");
  __shared__ __attribute__((aligned(16))) unsigned short lds[LDS_US];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int group = __builtin_amdgcn_readfirstlane(tid >> 8);
  const int gw = __builtin_amdgcn_readfirstlane((tid >> 6) & 3);
  const int wm = wave >> 1, wn = wave & 1;
  // grouped order (as vq_prefilter_x3): 16 row panels x 16 code tiles resident together, 4 x 8 per
  // XCD, so the blocks of one XCD stream the same panels through its L2 (ntiles % 16 == 0)
  const int ntiles = p.Cout / BN, mtiles = (p.Lq + BM - 1) / BM;
  int mt, nt;
  vq_tile(mtiles, ntiles, mt, nt);
  if (mt >= mtiles) return;  // whole workgroup, before any barrier
  const int q0 = mt * BM, co0 = nt * BN;
  const int nsteps = p.Cin / BK;
  // hm (p.x_compact == 2, x6 mode): x_pjt_in in the "hm" layout and the codebook as
  // launch_repack_codebook_bk packs it (p.wc), so each row's / code's four pieces of a K16 step are
  // one contiguous 64-byte run; otherwise planes (two 32-byte runs per 96-byte chunk)
  const bool hm = p.x_compact == 2;
  const int arow = p.ldx * (hm ? 4 : 6);  // bytes per input row
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.x6 + (long long)q0 * p.ldx * (hm ? 2 : 3)), 0, min(BM, p.Lq - q0) * arow, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw =
      hm ? __builtin_amdgcn_make_buffer_rsrc((void*)p.wc, 0, nsteps * p.Cout * 64, 0x00020000)
         : __builtin_amdgcn_make_buffer_rsrc((void*)p.w6, 0, nsteps * p.Cout * 96, 0x00020000);

  int a_off[PW], b_off[PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int u = (group * G_I + i * 4 + gw) * 64 + lane;
    const int row = u >> 2, pc = (u & 3) ^ ((row >> 2) & 3);
    // (half, plane) within a 96-byte K16 chunk, or within the 64-byte hm run
    const int poff = hm ? ((pc >> 1) * 2 + (pc & 1)) * 16 : (pc >> 1) * 48 + (pc & 1) * 16;
    a_off[i] = row * arow + poff;
    b_off[i] = (co0 + row) * (hm ? 128 : 96) + poff;
  }
  // step c's byte offset: planes c * 96 (input) / c * Cout * 96 (codebook); hm: K32 step c >> 1,
  // half (c & 1) of its 128-byte run
  const int a_step = hm ? 128 : 96;
  const int b_step = hm ? p.Cout * 128 : p.Cout * 96;
  unsigned short* const a_dst = lds + (group * G_I + gw) * 512;
  unsigned short* const b_dst = lds + 3 * ABUF + (group * G_I + gw) * 512;
  auto dma_step = [&](int c, int slot) {
    const int ao = hm ? (c >> 1) * a_step + (c & 1) * 64 : c * a_step;
    const int bo = hm ? (c >> 1) * b_step + (c & 1) * 64 : c * b_step;
#pragma unroll
    for (int i = 0; i < PW; ++i) dma16(rx, a_dst + slot * ABUF + i * 2048, a_off[i] + ao, 0);
#pragma unroll
    for (int i = 0; i < PW; ++i) dma16(rw, b_dst + slot * BBUF + i * 2048, b_off[i], bo);
    return 2 * PW;
  };

  const int lrow = lane & 31, h = lane >> 5;
  s16x8 af[TM][2], bfr[TN][2];
  auto readF = [&](int slot) {
    const unsigned short* A = lds + slot * ABUF;
    const unsigned short* Bs = lds + 3 * ABUF + slot * BBUF;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int r = wm * WR + i * 32 + lrow;
#pragma unroll
      for (int pl = 0; pl < 2; ++pl)
        af[i][pl] = *reinterpret_cast<const s16x8*>(A + r * RW + (((h * 2 + pl) ^ ((r >> 2) & 3)) << 3));
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = wn * WC + j * 32 + lrow;
#pragma unroll
      for (int pl = 0; pl < 2; ++pl)
        bfr[j][pl] = *reinterpret_cast<const s16x8*>(Bs + col * RW + (((h * 2 + pl) ^ ((col >> 2) & 3)) << 3));
    }
  };
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  auto mfma = [&]() {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (XMID)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, af[i][1]),
                                                              __builtin_bit_cast(bf16x8, bfr[j][0]), acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, af[i][0]),
                                                            __builtin_bit_cast(bf16x8, bfr[j][1]), acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, af[i][0]),
                                                            __builtin_bit_cast(bf16x8, bfr[j][0]), acc[i][j], 0, 0, 0);
      }
    __builtin_amdgcn_s_setprio(0);
  };
  auto inc3 = [](int& slot) { slot = slot == 2 ? 0 : slot + 1; };

  // ---- prologue: steps 0, 1, 2 (both groups their pieces), drained
  for (int t = 0; t < 3; ++t) dma_step(t, t);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  seg_barrier();
#ifdef DCX_CLOCK_DIAG
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
#endif
  // Segment 2s: group 0 MFMA(s), group 1 MEM1(s); 2s + 1: group 0 MEM0(s), group 1 MFMA(s).
  if (group == 0) {
    readF(0);
    int rs = 1, ws = 0;  // slot of step s + 1 (read next), of step s + 3 (issued next)
    for (int s = 0; s < nsteps; ++s) {
      mfma();  // MFMA(s)
      seg_barrier();
      // MEM0(s): fragments of step s + 1, issue step s + 3, retire step s + 2
      if (s + 1 < nsteps) readF(rs);
      int n = 0;
      if (s + 3 < nsteps) n = dma_step(s + 3, ws);
      wait_dma(n);
      seg_barrier();
      inc3(rs);
      inc3(ws);
    }
  } else {
    int rs = 0, ws = 0;  // slot of step s, of step s + 2
    for (int s = 0; s < nsteps; ++s) {
      // MEM1(s): fragments of step s, issue step s + 2 (s >= 1), retire step s + 1
      readF(rs);
      int n = 0;
      if (s >= 1 && s + 2 < nsteps) n = dma_step(s + 2, ws);
      wait_dma(n);
      seg_barrier();
      mfma();  // MFMA(s)
      seg_barrier();
      inc3(rs);
      if (s >= 1) inc3(ws);
      else ws = 0;  // step 3's slot
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef DCX_CLOCK_DIAG
  if (threadIdx.x == 0) {  // steps counted in units of vq_prefilter_x3's (K32: twice these)
    atomicAdd(&g_clock_diag[0], __builtin_amdgcn_s_memtime() - t0);
    atomicAdd(&g_clock_diag[1], __builtin_amdgcn_s_memrealtime() - r0);
    atomicAdd(&g_clock_diag[2], (unsigned long long)nsteps / 2);
  }
#endif
  epilogue_top2<BM, BN, 4, WN>(p, acc, q0, co0, nt, ntiles, reinterpret_cast<float*>(lds));
}

// ---------------------------------------------------------------------------------------------
// vq_prefilter_bk: the bf16-mode prefilter (x_pjt_in bf16-valued: x = hi) on K32 steps.
//
// vq_prefilter_dm in bf16 mode issued 16 MFMAs per segment against two barriers, staged x's mid
// plane (zero) and read hi/mid pieces at 48-byte strides.  Here a step is K32 (two K16 chunks cc):
// x arrives in the compact bf16 layout (one 64-byte run per row and step) and the codebook as
// launch_repack_codebook_bk packs it (one 128-byte run of hi/mid pieces per code and step), so
// every DMA instruction reads whole cache lines, and a segment issues 32 MFMAs:
//   per cc: acc += x_h . e_m',  acc += x_h . e_h'   (v_mfma_f32_32x32x16_bf16)
// the products of vq_prefilter_dm's bf16 mode, so the bound of launch_vq_prefilter holds as is.
// Ring: 3 slots of 16 KiB (x) + 32 KiB (codebook), the ping-pong schedule of vq_prefilter_dm.
// LDS images (lane-linear per DMA instruction, swizzle applied on the source):
//   x:  64-byte rows, piece p = cc * 2 + hh in slot p ^ ((row >> 2) & 3);
//   e: 128-byte rows, piece p = (cc * 2 + hh) * 2 + plane in slot p ^ ((code >> 1) & 7);
// both conflict-free for the four lane groups of a ds_read_b128 (MI355X_MICROARCH.md §LDS).
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(512, 2) vq_prefilter_bk(const ConvParams p) {
  constexpr int BM = 256, BN = 256, WN = 2;
  constexpr int WR = BM / 4, WC = BN / 2, TM = WR / 32, TN = WC / 32;
  constexpr int ARW = 32, BRW = 64;            // ushorts per LDS row
  constexpr int A_G = BM * 4 / 64 / 2;         // DMA instructions per group per tile (x: 8)
  constexpr int B_G = BN * 8 / 64 / 2;         // (codebook: 16)
  constexpr int A_PW = A_G / 4, B_PW = B_G / 4;  // per wave
  constexpr int ABUF = BM * ARW, BBUF = BN * BRW;
  constexpr int LDS_US = 3 * ABUF + 3 * BBUF;  // 144 KiB
  static_assert(A_G % 4 == 0 && B_G % 4 == 0 && LDS_US * 2 <= 160 * 1024, "tile shape");
  __shared__ __attribute__((aligned(16))) unsigned short lds[LDS_US];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int group = __builtin_amdgcn_readfirstlane(tid >> 8);
  const int gw = __builtin_amdgcn_readfirstlane((tid >> 6) & 3);
  const int wm = wave >> 1, wn = wave & 1;
  // grouped order of vq_prefilter_dm: 16 row panels x 16 code tiles resident together
  const int ntiles = p.Cout / BN, mtiles = (p.Lq + BM - 1) / BM;
  int mt, nt;
  vq_tile(mtiles, ntiles, mt, nt);
  if (mt >= mtiles) return;  // whole workgroup, before any barrier
  const int q0 = mt * BM, co0 = nt * BN;
  const int nsteps = p.Cin / 32;
  const int arow = p.ldx * 2;  // bytes per compact row
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.x6 + (long long)q0 * p.ldx), 0, min(BM, p.Lq - q0) * arow, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)p.wc, 0, nsteps * p.Cout * 128, 0x00020000);

  int a_off[A_PW], b_off[B_PW];
#pragma unroll
  for (int i = 0; i < A_PW; ++i) {
    const int u = (group * A_G + i * 4 + gw) * 64 + lane;
    const int row = u >> 2, pc = (u & 3) ^ ((row >> 2) & 3);
    a_off[i] = row * arow + pc * 16;
  }
#pragma unroll
  for (int i = 0; i < B_PW; ++i) {
    const int u = (group * B_G + i * 4 + gw) * 64 + lane;
    const int code = u >> 3, pc = (u & 7) ^ ((code >> 1) & 7);
    b_off[i] = (co0 + code) * 128 + pc * 16;
  }
  unsigned short* const a_dst = lds + (group * A_G + gw) * 512;
  unsigned short* const b_dst = lds + 3 * ABUF + (group * B_G + gw) * 512;
  auto dma_step = [&](int c, int slot) {
#pragma unroll
    for (int i = 0; i < A_PW; ++i) dma16(rx, a_dst + slot * ABUF + i * 2048, a_off[i] + c * 64, 0);
#pragma unroll
    for (int i = 0; i < B_PW; ++i) dma16(rw, b_dst + slot * BBUF + i * 2048, b_off[i], c * p.Cout * 128);
    return A_PW + B_PW;
  };

  const int lrow = lane & 31, h = lane >> 5;
  s16x8 af[TM][2], bfr[TN][2][2];
  auto readF = [&](int slot) {
    const unsigned short* A = lds + slot * ABUF;
    const unsigned short* Bs = lds + 3 * ABUF + slot * BBUF;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int r = wm * WR + i * 32 + lrow;
#pragma unroll
      for (int cc = 0; cc < 2; ++cc)
        af[i][cc] = *reinterpret_cast<const s16x8*>(A + r * ARW + (((cc * 2 + h) ^ ((r >> 2) & 3)) << 3));
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = wn * WC + j * 32 + lrow;
#pragma unroll
      for (int cc = 0; cc < 2; ++cc)
#pragma unroll
        for (int pl = 0; pl < 2; ++pl)
          bfr[j][cc][pl] = *reinterpret_cast<const s16x8*>(
              Bs + col * BRW + (((((cc * 2 + h) * 2) + pl) ^ ((col >> 1) & 7)) << 3));
    }
  };
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  auto mfma = [&]() {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int cc = 0; cc < 2; ++cc)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, af[i][cc]),
                                                              __builtin_bit_cast(bf16x8, bfr[j][cc][1]), acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, af[i][cc]),
                                                              __builtin_bit_cast(bf16x8, bfr[j][cc][0]), acc[i][j], 0, 0, 0);
        }
    __builtin_amdgcn_s_setprio(0);
  };
  auto inc3 = [](int& slot) { slot = slot == 2 ? 0 : slot + 1; };

  for (int t = 0; t < 3; ++t) dma_step(t, t);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  seg_barrier();
  if (group == 0) {
    readF(0);
    int rs = 1, ws = 0;
    for (int s = 0; s < nsteps; ++s) {
      mfma();  // MFMA(s)
      seg_barrier();
      if (s + 1 < nsteps) readF(rs);  // MEM0(s): fragments of step s + 1, issue step s + 3
      int n = 0;
      if (s + 3 < nsteps) n = dma_step(s + 3, ws);
      wait_dma(n);
      seg_barrier();
      inc3(rs);
      inc3(ws);
    }
  } else {
    int rs = 0, ws = 0;
    for (int s = 0; s < nsteps; ++s) {
      readF(rs);  // MEM1(s): fragments of step s, issue step s + 2 (s >= 1)
      int n = 0;
      if (s >= 1 && s + 2 < nsteps) n = dma_step(s + 2, ws);
      wait_dma(n);
      seg_barrier();
      mfma();  // MFMA(s)
      seg_barrier();
      inc3(rs);
      if (s >= 1) inc3(ws);
      else ws = 0;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  epilogue_top2<BM, BN, 4, WN>(p, acc, q0, co0, nt, ntiles, reinterpret_cast<float*>(lds));
}

// epilogue_top2 for 16x16 accumulator blocks (v_mfma_f32_16x16x32_bf16: lane l holds column
// l & 15 of its block, rows 4 (l >> 4) + r): the same per-row top 2 and lowest index on ties.
template <int BM, int BN, int WM, int WN>
__device__ __forceinline__ void epilogue_top2_q(const ConvParams& p, f32x4 (&acc)[BM / WM / 16][BN / WN / 16], int q0,
                                                int co0, int nt, int ntiles, float* smem) {
  constexpr int WR = BM / WM, WC = BN / WN;
  constexpr int TM = WR / 16, TN = WC / 16;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int lc = lane & 15, r4 = 4 * (lane >> 4);
  float xxv[TM][4], e2v[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) xxv[i][r] = p.x2[min(q0 + wm * WR + i * 16 + r4 + r, p.Lq - 1)];
#pragma unroll
  for (int j = 0; j < TN; ++j) e2v[j] = p.e2[co0 + wn * WC + j * 16 + lc];
  __syncthreads();
  float* rv = smem;                                      // [WN][BM]
  float* rv2 = smem + WN * BM;                           // [WN][BM]
  int* ri = reinterpret_cast<int*>(smem + 2 * WN * BM);  // [WN][BM]
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rloc = wm * WR + i * 16 + r4 + r;
      const float xx = xxv[i][r];
      float v1 = __builtin_inff(), v2 = __builtin_inff();
      int i1 = 0x7fffffff;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        // a lane's codes come in increasing order, so a strict < keeps the lowest index on ties; the
        // second smallest is min(v2, max(v1, d2)) (top2_merge with one new value, in 5 VALU ops)
        const int co = co0 + wn * WC + j * 16 + lc;
        const float d2 = (xx + e2v[j]) + (-2.0f * acc[i][j][r]);
        i1 = d2 < v1 ? co : i1;
        v2 = fminf(v2, fmaxf(v1, d2));
        v1 = fminf(v1, d2);
      }
      top2_row16(v1, i1, v2);
      if (lc == 0) {
        rv[wn * BM + rloc] = v1;
        rv2[wn * BM + rloc] = v2;
        ri[wn * BM + rloc] = i1;
      }
    }
  }
  __syncthreads();
  for (int rloc = tid; rloc < BM; rloc += blockDim.x) {
    const int q = q0 + rloc;
    if (q >= p.Lq) continue;
    float v1 = rv[rloc], v2 = rv2[rloc];
    int i1 = ri[rloc];
#pragma unroll
    for (int w = 1; w < WN; ++w) top2_merge(v1, i1, v2, rv[w * BM + rloc], ri[w * BM + rloc], rv2[w * BM + rloc]);
    const long long o = (long long)q * ntiles + nt;
    p.part_val[o] = v1;
    p.part_val2[o] = v2;
    p.part_idx[o] = i1;
  }
}

// ---------------------------------------------------------------------------------------------
// vq_prefilter_bq: vq_prefilter_bk on v_mfma_f32_16x16x32_bf16 (round 2).
//
// Same operands, LDS images, DMA ring and ping-pong schedule as vq_prefilter_bk; only the MFMA
// shape changes.  The K32 of one 16x16x32 MFMA is split as k = (t, c): t = lane >> 5 picks the
// codebook plane and c (lane bit 4 and the element) the channel inside a K16 chunk, so one MFMA
// sums x_h . e_h' + x_h . e_m' over 16 channels, the two products vq_prefilter_bk issues as two
// 32x32x16 MFMAs.  The product set and the K terms per accumulator are unchanged (each MFMA now
// adds 32 products instead of 16, half as many MFMAs), so launch_vq_prefilter's bound holds as
// for vq_prefilter_bk.  Why: under MFMA load the chip holds a higher clock for 16x16x32 than for
// 32x32x16 at the same cycles per FLOP (MI355X_MICROARCH.md, DVFS; conv_gemm_x6dq).
// Fragment reads (ds_read_b128, per 16-lane group one 16-byte piece of 16 consecutive rows or
// codes) are conflict-free under the swizzles of vq_prefilter_bk.
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(512, 2) vq_prefilter_bq(const ConvParams p) {
  constexpr int BM = 256, BN = 256, WN = 2;
  constexpr int WR = BM / 4, WC = BN / 2, TM = WR / 16, TN = WC / 16;
  constexpr int ARW = 32, BRW = 64;            // ushorts per LDS row
  constexpr int A_G = BM * 4 / 64 / 2;         // DMA instructions per group per tile (x: 8)
  constexpr int B_G = BN * 8 / 64 / 2;         // (codebook: 16)
  constexpr int A_PW = A_G / 4, B_PW = B_G / 4;  // per wave
  constexpr int ABUF = BM * ARW, BBUF = BN * BRW;
  constexpr int LDS_US = 3 * ABUF + 3 * BBUF;  // 144 KiB
  static_assert(A_G % 4 == 0 && B_G % 4 == 0 && LDS_US * 2 <= 160 * 1024, "tile shape");
  __shared__ __attribute__((aligned(16))) unsigned short lds[LDS_US];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int group = __builtin_amdgcn_readfirstlane(tid >> 8);
  const int gw = __builtin_amdgcn_readfirstlane((tid >> 6) & 3);
  const int wm = wave >> 1, wn = wave & 1;
  const int ntiles = p.Cout / BN, mtiles = (p.Lq + BM - 1) / BM;
  int mt, nt;
  vq_tile(mtiles, ntiles, mt, nt);
  if (mt >= mtiles) return;  // whole workgroup, before any barrier
  const int q0 = mt * BM, co0 = nt * BN;
  const int nsteps = p.Cin / 32;
  const int arow = p.ldx * 2;  // bytes per compact row
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.x6 + (long long)q0 * p.ldx), 0, min(BM, p.Lq - q0) * arow, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)p.wc, 0, nsteps * p.Cout * 128, 0x00020000);

  int a_off[A_PW], b_off[B_PW];
#pragma unroll
  for (int i = 0; i < A_PW; ++i) {
    const int u = (group * A_G + i * 4 + gw) * 64 + lane;
    const int row = u >> 2, pc = (u & 3) ^ ((row >> 2) & 3);
    a_off[i] = row * arow + pc * 16;
  }
#pragma unroll
  for (int i = 0; i < B_PW; ++i) {
    const int u = (group * B_G + i * 4 + gw) * 64 + lane;
    const int code = u >> 3, pc = (u & 7) ^ ((code >> 1) & 7);
    b_off[i] = (co0 + code) * 128 + pc * 16;
  }
  unsigned short* const a_dst = lds + (group * A_G + gw) * 512;
  unsigned short* const b_dst = lds + 3 * ABUF + (group * B_G + gw) * 512;
  auto dma_step = [&](int c, int slot) {
#pragma unroll
    for (int i = 0; i < A_PW; ++i) dma16(rx, a_dst + slot * ABUF + i * 2048, a_off[i] + c * 64, 0);
#pragma unroll
    for (int i = 0; i < B_PW; ++i) dma16(rw, b_dst + slot * BBUF + i * 2048, b_off[i], c * p.Cout * 128);
    return A_PW + B_PW;
  };

  // lane roles: row / code l & 15 of a 16-block, channel half hh = (l >> 4) & 1, plane t = l >> 5
  const int l16 = lane & 15, hh = (lane >> 4) & 1, tp = lane >> 5;
  s16x8 af[TM][2], bfr[TN][2];
  auto readF = [&](int slot) {
    const unsigned short* A = lds + slot * ABUF;
    const unsigned short* Bs = lds + 3 * ABUF + slot * BBUF;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int r = wm * WR + i * 16 + l16;
#pragma unroll
      for (int cc = 0; cc < 2; ++cc)
        af[i][cc] = *reinterpret_cast<const s16x8*>(A + r * ARW + (((cc * 2 + hh) ^ ((r >> 2) & 3)) << 3));
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = wn * WC + j * 16 + l16;
#pragma unroll
      for (int cc = 0; cc < 2; ++cc)
        bfr[j][cc] = *reinterpret_cast<const s16x8*>(
            Bs + col * BRW + (((((cc * 2 + hh) * 2) + tp) ^ ((col >> 1) & 7)) << 3));
    }
  };
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mfma = [&]() {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int cc = 0; cc < 2; ++cc)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af[i][cc]),
                                                              __builtin_bit_cast(bf16x8, bfr[j][cc]), acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto inc3 = [](int& slot) { slot = slot == 2 ? 0 : slot + 1; };

  for (int t = 0; t < 3; ++t) dma_step(t, t);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  seg_barrier();
  if (group == 0) {
    readF(0);
    int rs = 1, ws = 0;
    for (int s = 0; s < nsteps; ++s) {
      mfma();  // MFMA(s)
      seg_barrier();
      if (s + 1 < nsteps) readF(rs);  // MEM0(s): fragments of step s + 1, issue step s + 3
      int n = 0;
      if (s + 3 < nsteps) n = dma_step(s + 3, ws);
      wait_dma(n);
      seg_barrier();
      inc3(rs);
      inc3(ws);
    }
  } else {
    int rs = 0, ws = 0;
    for (int s = 0; s < nsteps; ++s) {
      readF(rs);  // MEM1(s): fragments of step s, issue step s + 2 (s >= 1)
      int n = 0;
      if (s >= 1 && s + 2 < nsteps) n = dma_step(s + 2, ws);
      wait_dma(n);
      seg_barrier();
      mfma();  // MFMA(s)
      seg_barrier();
      inc3(rs);
      if (s >= 1) inc3(ws);
      else ws = 0;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  epilogue_top2_q<BM, BN, 4, WN>(p, acc, q0, co0, nt, ntiles, reinterpret_cast<float*>(lds));
}

// 64-byte LDS rows of vq_prefilter_b1: the 16-byte piece q of row r sits in slot q ^ b1_swz(r), with
// b1_swz(r) = (0, 2, 3, 1)[(r >> 2) & 3].  A ds_read_b128 is serviced in four 16-lane groups,
// {0-3, 12-15, 20-27}, {4-11, 16-19, 28-31} and the same + 32 (MI355X_MICROARCH.md §LDS), and lane l
// reads piece l >> 4 of row l & 15: this map gives the 16 lanes of every group 16 distinct bank quads.
// (Round 3's (r >> 2) & 3 paired up two lanes per quad in every group: 2-way conflicts, 46 % of the
// kernel's LDS cycles in PMC, SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE.)
__device__ __forceinline__ int b1_swz(int r) { return (0x1320 >> (((r >> 2) & 3) * 4)) & 3; }

// ---------------------------------------------------------------------------------------------
// vq_prefilter_b1: one bf16 product per term, x_h . e_h', in both arithmetic modes (round 3).
//
// The search only needs a candidate set that provably holds the nearest code; vq_rescore_kernel
// settles it exactly in fp64.  With x = x_h + x_r and e = e_h + d (x_h, e_h the RNE bf16 values),
// x.e - x_h.e_h = x_r.e + x_h.d, so by Cauchy-Schwarz the dropped terms are at most
// |x_r| max|e| + |x_h| max|d|, where max|d| (0.17 % of max|e| on the synthetic codebook) is
// measured once at load and |x_r| per row by row_sqnorm (zero in bf16 mode).  That bound is
// looser than vq_prefilter_dm's (3 products) or vq_prefilter_bq's (2), so more rows go on to the
// rescore (about 60-95 % instead of 10 %, 3-7 candidates each), but the distance GEMM, 99 % of the
// search's MFMA work, issues 1/3 (x6) or 1/2 (bf16) of the products.
//
// One v_mfma_f32_16x16x32_bf16 per 16 x 16 block and K32 step (lanes l >> 4 = 0..3 read the four
// 16-byte pieces of 8 channels).  Both operands arrive as 64-byte runs per row / code and step:
// x_pjt_in compact ([rows][CD] bf16, the project_in epilogue's y_compact == 1 output) and the
// codebook as launch_repack_codebook_b1 packs it ([CD/32][NC][32] bf16).  LDS images: 64-byte
// rows, piece q in slot q ^ b1_swz(row), conflict-free for the four lane groups of a ds_read_b128.  Ring: NS slots of 16 + 16 KiB on the ping-pong schedule
// of vq_prefilter_bk generalised to NS slots: step t is issued by group 0 in MEM0(t - NS) and by
// group 1 in MEM1(t - NS + 1), and each wave retires its pieces NS - 2 memory segments later.
// ---------------------------------------------------------------------------------------------
template <int NS>
__global__ void __launch_bounds__(512, 2) vq_prefilter_b1(const ConvParams p) {
  constexpr int BM = 256, BN = 256, WN = 2;
  constexpr int WR = BM / 4, WC = BN / 2, TM = WR / 16, TN = WC / 16;
  DCX_TILET(tile_t0);
  constexpr int RW = 32;                       // ushorts per LDS row (64 bytes)
  constexpr int A_G = BM * 4 / 64 / 2;         // DMA instructions per group per tile (8)
  constexpr int B_G = BN * 4 / 64 / 2;         // (8)
  constexpr int A_PW = A_G / 4, B_PW = B_G / 4;  // per wave (2 + 2)
  constexpr int P = A_PW + B_PW;
  constexpr int ABUF = BM * RW, BBUF = BN * RW;
  constexpr int LDS_US = NS * (ABUF + BBUF);   // NS * 32 KiB
  static_assert(A_G % 4 == 0 && B_G % 4 == 0 && LDS_US * 2 <= 160 * 1024 && NS >= 3, "tile shape");
  static_assert(P * (NS - 1) <= 23, "wait_dma range");
  __shared__ __attribute__((aligned(16))) unsigned short lds[LDS_US];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int group = __builtin_amdgcn_readfirstlane(tid >> 8);
  const int gw = __builtin_amdgcn_readfirstlane((tid >> 6) & 3);
  const int wm = wave >> 1, wn = wave & 1;
  const int ntiles = p.Cout / BN, mtiles = (p.Lq + BM - 1) / BM;
  int mt, nt;
  vq_tile(mtiles, ntiles, mt, nt);
  if (mt >= mtiles) return;  // whole workgroup, before any barrier
  const int q0 = mt * BM, co0 = nt * BN;
  const int nsteps = p.Cin / 32;
  const int arow = p.ldx * 2;  // bytes per compact row
#ifdef DCX_VQ_DIAG_L2  // timing build: every tile loads row panel 0 and code tile 0 (L2-resident operands)
  const int lq0 = 0, lco0 = 0;
#else
  const int lq0 = q0, lco0 = co0;
#endif
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.x6 + (long long)lq0 * p.ldx), 0, min(BM, p.Lq - lq0) * arow, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)p.wc, 0, nsteps * p.Cout * 64, 0x00020000);

  int a_off[A_PW], b_off[B_PW];
#pragma unroll
  for (int i = 0; i < A_PW; ++i) {
    const int u = (group * A_G + i * 4 + gw) * 64 + lane;
    const int row = u >> 2, pc = (u & 3) ^ b1_swz(row);
    a_off[i] = row * arow + pc * 16;
  }
#pragma unroll
  for (int i = 0; i < B_PW; ++i) {
    const int u = (group * B_G + i * 4 + gw) * 64 + lane;
    const int code = u >> 2, pc = (u & 3) ^ b1_swz(code);
    b_off[i] = (lco0 + code) * 64 + pc * 16;
  }
  unsigned short* const a_dst = lds + (group * A_G + gw) * 512;
  unsigned short* const b_dst = lds + NS * ABUF + (group * B_G + gw) * 512;
  auto dma_step = [&](int c, int slot) {
#pragma unroll
    for (int i = 0; i < A_PW; ++i) dma16(rx, a_dst + slot * ABUF + i * 2048, a_off[i] + c * 64, 0);
#pragma unroll
    for (int i = 0; i < B_PW; ++i) dma16(rw, b_dst + slot * BBUF + i * 2048, b_off[i], c * p.Cout * 64);
  };

  // lane roles: row / code l & 15 of a 16-block, piece (8 channels) q = l >> 4
  const int l16 = lane & 15, pq = lane >> 4;
  s16x8 af[TM], bfr[TN];
  auto readF = [&](int slot) {
    const unsigned short* A = lds + slot * ABUF;
    const unsigned short* Bs = lds + NS * ABUF + slot * BBUF;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int r = wm * WR + i * 16 + l16;
      af[i] = *reinterpret_cast<const s16x8*>(A + r * RW + ((pq ^ b1_swz(r)) << 3));
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = wn * WC + j * 16 + l16;
      bfr[j] = *reinterpret_cast<const s16x8*>(Bs + col * RW + ((pq ^ b1_swz(col)) << 3));
    }
  };
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mfma = [&]() {
#ifdef DCX_VQ_STATICPRIO  // A/B: group 1 at priority 1 throughout, no per-segment flips (MI355X_MICROARCH.md
                          // "Two waves per SIMD" item 4); the MFMA cluster fenced for the scheduler instead
    __builtin_amdgcn_sched_barrier(0);
#else
    __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af[i]),
                                                            __builtin_bit_cast(bf16x8, bfr[j]), acc[i][j], 0, 0, 0);
#ifdef DCX_VQ_STATICPRIO
    __builtin_amdgcn_sched_barrier(0);
#else
    __builtin_amdgcn_s_setprio(0);
#endif
  };
  auto inc = [](int& slot) { slot = slot == NS - 1 ? 0 : slot + 1; };
  // pieces this wave may leave in flight at the end of a memory segment: its shares of the steps
  // after the ones the next two segments read (lo..hi inclusive, clipped to the steps that exist)
  auto in_flight = [&](int lo, int hi) { return P * max(0, min(hi, nsteps - 1) - lo + 1); };

  for (int t = 0; t < NS && t < nsteps; ++t) dma_step(t, t);
  // group 0 reads step 0 now and step 1 in segment 1 (its own MFMA segment 0 comes first)
  wait_dma(group == 0 ? in_flight(2, NS - 1) : in_flight(1, NS - 1));
#ifdef DCX_TILE_DIAG
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (timing build: the prologue's DMA landed)
#endif
  DCX_TILET(tile_t1);
#ifdef DCX_VQ_STATICPRIO
  if (group == 1) __builtin_amdgcn_s_setprio(1);
#endif
  seg_barrier();
#ifdef DCX_SEG_DIAG
  unsigned long long sd[5] = {};  // per step: mfma issue, barrier, reads + DMA issue, DMA wait, barrier
#endif
  if (group == 0) {
    readF(0);
    int rs = 1, ws = 0;
    for (int s = 0; s < nsteps; ++s) {
      DCX_SEGT(ta);
      mfma();  // MFMA(s)
      DCX_SEGT(tb);
      seg_barrier();
      DCX_SEGT(tc);
      if (s + 1 < nsteps) readF(rs);  // MEM0(s): fragments of step s + 1, issue step s + NS
      if (s + NS < nsteps) dma_step(s + NS, ws);
      DCX_SEGT(td);
      wait_dma(in_flight(s + 3, s + NS));
      DCX_SEGT(te);
      seg_barrier();
      DCX_SEGT(tf);
#ifdef DCX_SEG_DIAG
      sd[0] += tb - ta; sd[1] += tc - tb; sd[2] += td - tc; sd[3] += te - td; sd[4] += tf - te;
#endif
      inc(rs);
      inc(ws);
    }
  } else {
    int rs = 0, ws = 0;
    for (int s = 0; s < nsteps; ++s) {
      DCX_SEGT(ta);
      readF(rs);  // MEM1(s): fragments of step s, issue step s + NS - 1 (s >= 1)
      if (s >= 1 && s + NS - 1 < nsteps) dma_step(s + NS - 1, ws);
      DCX_SEGT(tb);
      wait_dma(in_flight(s + 2, s >= 1 ? s + NS - 1 : NS - 1));
      DCX_SEGT(tc);
      seg_barrier();
      DCX_SEGT(td);
      mfma();  // MFMA(s)
      DCX_SEGT(te);
      seg_barrier();
      DCX_SEGT(tf);
#ifdef DCX_SEG_DIAG
      sd[0] += te - td; sd[1] += tf - te; sd[2] += tb - ta; sd[3] += tc - tb; sd[4] += td - tc;
#endif
      inc(rs);
      if (s >= 1) inc(ws);
      else ws = 0;
    }
  }
#ifdef DCX_SEG_DIAG
  if ((threadIdx.x & 255) == 0) {
#pragma unroll
    for (int i = 0; i < 5; ++i) atomicAdd(&g_seg_diag[group * 6 + i], sd[i]);
    if (group == 0) atomicAdd(&g_seg_diag[12], (unsigned long long)nsteps);
  }
#endif
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  DCX_TILET(tile_t2);
  epilogue_top2_q<BM, BN, 4, WN>(p, acc, q0, co0, nt, ntiles, reinterpret_cast<float*>(lds));
#ifdef DCX_TILE_DIAG
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long t3 = __builtin_amdgcn_s_memrealtime();
    const unsigned int k = atomicAdd(&g_tile_cnt, 1u);
    if (k < (unsigned)kTileDiagMax) {
      unsigned long long* o = g_tile_diag + 6ull * k;
      o[0] = tile_t0; o[1] = tile_t1; o[2] = tile_t2; o[3] = t3;
      o[4] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
      o[5] = __builtin_amdgcn_s_getreg((15 << 11) | 20) | ((unsigned long long)nsteps << 16);
    }
  }
#endif
}

// ---------------------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------------------
template <int BM, int BN, int WM, int WN, bool ARGMIN>
static hipError_t launch_f32(const ConvParams& p, int batch, int phases, hipStream_t s) {
  const int mtiles = (p.Lq + BM - 1) / BM;
  const dim3 grid((unsigned)(mtiles * (p.Cout / BN) * batch * phases));
  ConvParams q = p;
  q.batch = batch;
  q.phases = phases;
  hipLaunchKernelGGL((conv_gemm_f32<BM, BN, WM, WN, ARGMIN>), grid, dim3(256), 0, s, q);
  return hipGetLastError();
}

// Persistent launch: as many workgroups as fit on the device at once (occupancy from the
// runtime, once per kernel), a multiple of 8 (XCD grouping), at most the tile count rounded up.
template <int BM, int BN, int WM, int WN, int HALO, int PROD, bool AF32>
static hipError_t launch_x6_persistent(ConvParams p, int batch, int phases, hipStream_t s) {
  auto kern = conv_gemm_x6w8<BM, BN, WM, WN, HALO, false, PROD, AF32>;
  static std::once_flag once;  // workgroups resident per CU (per instantiation, queried once)
  static int per_cu = 0;
  std::call_once(once, [&] {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * WM * WN, 0) != hipSuccess) per_cu = 0;
  });
  if (per_cu < 1) return hipErrorInvalidValue;
  const int resident = device_cus() * per_cu;
  p.batch = batch;
  p.phases = phases;
  const long long total = (long long)((p.Lq + BM - 1) / BM) * (p.Cout / BN) * batch * phases;
  if (total > (1LL << 30)) return hipErrorInvalidValue;
  int g = (int)std::min<long long>(resident, (total + 7) / 8 * 8);
  g = std::max(8, g / 8 * 8);
  hipLaunchKernelGGL(kern, dim3(g), dim3(64 * WM * WN), 0, s, p);
  return hipGetLastError();
}

template <int BM, int BN, int WM, int WN, int HALO, bool ARGMIN>
static hipError_t launch_x6w8(const ConvParams& p, int batch, int phases, hipStream_t s) {
  static_assert(!ARGMIN, "x6 VQ search uses vq_prefilter_x3");
  return p.nprod == 1 ? launch_x6_persistent<BM, BN, WM, WN, HALO, 1, false>(p, batch, phases, s)
                      : launch_x6_persistent<BM, BN, WM, WN, HALO, 6, false>(p, batch, phases, s);
}

// fp32-input variant (Cin <= 64 convs, see conv_gemm_x6w8)
template <int BM, int BN, int WM, int WN, int HALO>
static hipError_t launch_x6w8_af32(const ConvParams& p, int batch, int phases, hipStream_t s) {
  return p.nprod == 1 ? launch_x6_persistent<BM, BN, WM, WN, HALO, 1, true>(p, batch, phases, s)
                      : launch_x6_persistent<BM, BN, WM, WN, HALO, 6, true>(p, batch, phases, s);
}

static int tap_span(const ConvParams& p) { return (p.taps - 1) * (p.in_step < 0 ? -p.in_step : p.in_step); }

hipError_t launch_splitk_epilogue(const ConvParams& p, const float* partials, int splits, long long stride, int batch,
                                  int phases, hipStream_t s) {
  if (splits < 1 || p.Cout % 4 || p.ldy != p.Cout) return hipErrorInvalidValue;
  ConvParams q = p;
  q.batch = batch;
  q.phases = phases;
  const long long total4 = (long long)phases * batch * p.Lq * (p.Cout / 4);
  hipLaunchKernelGGL(splitk_epilogue_kernel, dim3((unsigned)((total4 + 255) / 256)), dim3(256), 0, s, q, partials, splits,
                     stride, total4);
  return hipGetLastError();
}

// conv_gemm_bf16dp's GELU table: ConvParams::gelu_lut = the table offset from which a wave takes the
// evaluated epilogue (2 kGeluN, the table's end).  Knobs::gelu_lut (DCX_GELU_LUT at dcx_create): 0 =
// evaluated always (A/B); a smaller positive limit sends more waves through the evaluated epilogue (tests)
static int gelu_lut_limit(const Knobs& k) {
  if (k.gelu_lut < 0) return 2 * kGeluN;
  return std::min(k.gelu_lut, 2 * kGeluN);
}
static const Knobs kDefaultKnobs{};
static const Knobs& knobs(const ConvParams& p) { return p.kn ? *p.kn : kDefaultKnobs; }

// CU count per device, filled once per device (std::call_once per slot; devices past the table are
// queried each time)
int device_cus() {
  constexpr int kDev = 64;
  static std::once_flag once[kDev];
  static int cus[kDev];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  auto query = [dev] {
    int c = 0;
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c < 8) c = 256;
    return c;
  };
  if (dev < 0 || dev >= kDev) return query();
  std::call_once(once[dev], [&] { cus[dev] = query(); });
  return cus[dev];
}
static int num_cus() { return device_cus(); }

bool bf16dm_takes(int cin, int cout, int lq, int ldx, int phases) {
#ifdef DCX_NO_BF16DM
  return false;
#endif
  ConvParams q{};
  q.Lq = lq;
  q.Cout = cout;
  return cout % 256 == 0 && cin % 32 == 0 && big_tiles_pay(q, phases, 256) && 1024LL * ldx * 6 < (1LL << 31) &&
         (long long)(cin / 16) * cout * 96 < (1LL << 31);
}

template <int BN>
static hipError_t launch_x3dq(const ConvParams& p, int batch, int phases, hipStream_t s, const char** kname) {
  constexpr int BM = 32768 / BN;
  const dim3 grid((unsigned)(((p.Lq + BM - 1) / BM) * (p.Cout / BN) * batch * phases));
  ConvParams q = p;
  q.batch = batch;
  q.phases = phases;
  if (p.taps == 1) {
    if (kname) *kname = BN == 256 ? "conv_gemm_x3dm<128,256>" : "conv_gemm_x3dm<256,128>";
    hipLaunchKernelGGL((conv_gemm_x3dq<BN, 0>), grid, dim3(512), 0, s, q);
  } else {
    if (kname) *kname = BN == 256 ? "conv_gemm_x3dq<128,256,halo>" : "conv_gemm_x3dq<256,128,halo>";
    hipLaunchKernelGGL((conv_gemm_x3dq<BN, 64>), grid, dim3(512), 0, s, q);
  }
  return hipGetLastError();
}

hipError_t launch_conv(const ConvParams& p, int batch, int phases, hipStream_t s, const char** kname) {
  if (p.Cin % BK || p.Cout % 32 || phases < 1 || phases > kMaxPhases) return hipErrorInvalidValue;
  if (p.x_compact == 3) {  // h2 input: the h3 kernels only
    const int bn = x3dq_bn(p);
    if (!x3dq_ok(p, bn == 512 ? 256 : bn == 384 ? 128 : bn, bn >= 384)) return hipErrorInvalidValue;
    if (bn == 384) {  // 384 x 128 tiles (the C = 128 stage)
      const dim3 grid((unsigned)(((p.Lq + 383) / 384) * (p.Cout / 128) * batch * phases));
      ConvParams q = p;
      q.batch = batch;
      q.phases = phases;
      if (kname) *kname = "conv_gemm_x3dw<384,128,halo>";
      if (knobs(p).h3_split) hipLaunchKernelGGL((conv_gemm_x3dw<64, true, 128>), grid, dim3(512), 0, s, q);
      else hipLaunchKernelGGL((conv_gemm_x3dw<64, false, 128>), grid, dim3(512), 0, s, q);
      return hipGetLastError();
    }
    if (bn == 512) {
      const dim3 grid((unsigned)(((p.Lq + 255) / 256) * (p.Cout / 256) * batch * phases));
      ConvParams q = p;
      q.batch = batch;
      q.phases = phases;
      const bool sp = knobs(p).h3_split;
      if (p.taps == 1) {
        if (kname) *kname = "conv_gemm_x3dw<256,256>";
        if (sp) hipLaunchKernelGGL((conv_gemm_x3dw<0, true>), grid, dim3(512), 0, s, q);
        else hipLaunchKernelGGL((conv_gemm_x3dw<0, false>), grid, dim3(512), 0, s, q);
      } else {
        if (kname) *kname = "conv_gemm_x3dw<256,256,halo>";
        if (sp) hipLaunchKernelGGL((conv_gemm_x3dw<64, true>), grid, dim3(512), 0, s, q);
        else hipLaunchKernelGGL((conv_gemm_x3dw<64, false>), grid, dim3(512), 0, s, q);
      }
      return hipGetLastError();
    }
    return bn == 256 ? launch_x3dq<256>(p, batch, phases, s, kname) : launch_x3dq<128>(p, batch, phases, s, kname);
  }
  if (p.w6) {
    if (p.nprod != 6 && p.nprod != 1) return hipErrorInvalidValue;
    // split-K runs on conv_gemm_x6pp / x6lm (the kernels that read ksplit), whatever the tile count
    const bool ks = p.ksplit > 1;
    if (ks && (p.nprod != 6 || !p.x6 || p.Cout % 128 || batch % p.ksplit || p.kunit < 1 || (p.Cin / BK) % p.kunit ||
               (p.Cin / BK) / p.kunit < p.ksplit))
      return hipErrorInvalidValue;
    const bool b1 = p.nprod == 1;  // profile names: conv_gemm_bf16w* for the one-product mode
    const int span = tap_span(p);
    if (span > 64 || (p.Cin / BK) * p.taps % 2) return hipErrorInvalidValue;
    const bool h = span > 0;
    auto name = [&](const char* x6, const char* bf) {
      if (kname) *kname = b1 ? bf : x6;
    };
    if (!p.x6) {  // fp32 input, split while staging: small-Cout tiles only
      if (!p.x || p.Cin > 128 || p.Cout > 64 || p.taps < 2) return hipErrorInvalidValue;
      if (p.Cout == 64) {
#ifndef DCX_NO_PF
        if (!b1) {  // x6: ping-pong, 512 x 64 tiles
          if (kname) *kname = "conv_gemm_x6pf<512,64,halo>";
          ConvParams q = p;
          q.batch = batch;
          q.phases = phases;
          hipLaunchKernelGGL((conv_gemm_x6pp<64, 64, true>), dim3((unsigned)(((p.Lq + 511) / 512) * (p.Cout / 64) * batch * phases)),
                             dim3(512), 0, s, q);
          return hipGetLastError();
        }
#endif
        name("conv_gemm_x6w4f<256,64,halo>", "conv_gemm_bf16w4f<256,64,halo>");
        return launch_x6w8_af32<256, 64, 4, 1, 64>(p, batch, phases, s);
      }
      name("conv_gemm_x6w4f<256,32,halo>", "conv_gemm_bf16w4f<256,32,halo>");
      return launch_x6w8_af32<256, 32, 4, 1, 64>(p, batch, phases, s);
    }
#ifndef DCX_NO_DM
    if (!ks && !h && x6dm_ok(p, false, 256) && big_tiles_pay(p, phases, 256))
      return launch_x6dm<0, 256>(p, batch, phases, s, kname);  // x6 1-tap, Cout % 256
#endif
#ifndef DCX_NO_PP
    if (p.Cout % 128 == 0 && !h && !b1) return launch_x6pp<0>(p, batch, phases, s, kname);  // x6 1-tap
#endif
    const bool dm_b1 = b1 && !h && p.taps == 1 && in_base_nonneg(p) && bf16dm_takes(p.Cin, p.Cout, p.Lq, p.ldx, phases);
    if (p.x_compact && (!dm_b1 || p.x_compact != 1)) return hipErrorInvalidValue;  // only conv_gemm_bf16dm reads it
#ifndef DCX_NO_BF16DM
    if (dm_b1) {
      ConvParams q = p;
      q.batch = batch;
      q.phases = phases;
      q.gelu_lut = gelu_lut_limit(knobs(p));
      const dim3 grid((unsigned)(((p.Lq + 255) / 256) * (p.Cout / 256) * batch * phases));
      // the register epilogue: bias / GELU epilogues with a compact bf16 output only.  With an fp32
      // output too (the VQ blocks' 1x1 convs) or a residual (pwconv2) it measured slower than the
      // staged epilogue, whose 16-byte stores cover 512 contiguous bytes of a row per instruction
      // (C3 bf16dm, A/B: pwconv1 only 52.5 ms, + the fp32-output convs 55.4, + pwconv2 56.6)
      const bool reg = (p.epi == EPI_BIAS || p.epi == EPI_GELU) && p.y6 && p.y_compact == 1 && !p.y && !p.y2 &&
                       !p.y6s && p.mean_mode == MEAN_NONE && phases == 1 && p.out_mul == 1 && knobs(p).bf16_reg_epi;
      // the persistent form (one step stream across tiles) for compact operands; Knobs::bf16_persist = 0
      // (DCX_BF16_PERSIST=0) keeps conv_gemm_bf16dm<true> (A/B, same bits)
      if (reg && p.x_compact == 1 && p.wc && p.round_bf16 && p.Cin / 32 >= 3 && p.Cout <= kBf16dpBiasMax &&
          (long long)std::min(256, p.Lq) * p.Cout * 2 < (1ll << 31) && knobs(p).bf16_persist) {
        if (kname) *kname = "conv_gemm_bf16dp<256,256,reg>";
        const long long tiles = (long long)grid.x;
        const int g = (int)std::min<long long>(num_cus(), (tiles + 7) / 8 * 8);
        hipLaunchKernelGGL(conv_gemm_bf16dp, dim3((unsigned)std::max(8, g / 8 * 8)), dim3(512), 0, s, q);
        return hipGetLastError();
      }
      if (kname) *kname = reg ? "conv_gemm_bf16dm<256,256,reg>" : "conv_gemm_bf16dm<256,256>";
      if (reg) hipLaunchKernelGGL(conv_gemm_bf16dm<true>, grid, dim3(512), 0, s, q);
      else hipLaunchKernelGGL(conv_gemm_bf16dm<false>, grid, dim3(512), 0, s, q);
      return hipGetLastError();
    }
#endif
    if (p.Cout % 128 == 0 && !h) {  // 1-tap: 4-wave 128 x 128 tiles, two workgroups per CU
      name("conv_gemm_x6w4<128,128>", "conv_gemm_bf16w4<128,128>");
      return launch_x6w8<128, 128, 2, 2, 0, false>(p, batch, phases, s);
    }
    if (p.Cout % 128 == 0) {
      const bool pay256 = !ks && big_tiles_pay(p, phases, 256), pay128 = !ks && big_tiles_pay(p, phases, 128);
      (void)pay256;
      (void)pay128;
#ifndef DCX_NO_DQ
      if (p.taps >= 3 && pay256 && x6dm_ok(p, true, 256)) return launch_x6dq<256>(p, batch, phases, s, kname);  // 16x16x32
      if (p.taps >= 3 && pay128 && x6dm_ok(p, true, 128)) return launch_x6dq<128>(p, batch, phases, s, kname);
#endif
#ifndef DCX_NO_DM
      if (pay256 && x6dm_ok(p, true, 256)) return launch_x6dm<64, 256>(p, batch, phases, s, kname);  // LDS-DMA ping-pong
      if (pay128 && x6dm_ok(p, true, 128)) return launch_x6dm<64, 128>(p, batch, phases, s, kname);
#endif
#ifndef DCX_NO_PP
      if (!b1) return launch_x6pp<64>(p, batch, phases, s, kname);  // x6: ping-pong kernel
#endif
      name("conv_gemm_x6w8<256,128,halo>", "conv_gemm_bf16w8<256,128,halo>");
      return launch_x6w8<256, 128, 4, 2, 64, false>(p, batch, phases, s);
    }
    // small Cout: 4-wave 256-row tiles (< 80 KB LDS), two workgroups per CU
    if (p.Cout % 64 == 0) {
      if (h) {
        name("conv_gemm_x6w4<256,64,halo>", "conv_gemm_bf16w4<256,64,halo>");
        return launch_x6w8<256, 64, 4, 1, 64, false>(p, batch, phases, s);
      }
      name("conv_gemm_x6w4<256,64>", "conv_gemm_bf16w4<256,64>");
      return launch_x6w8<256, 64, 4, 1, 0, false>(p, batch, phases, s);
    }
    if (h) {
      name("conv_gemm_x6w4<256,32,halo>", "conv_gemm_bf16w4<256,32,halo>");
      return launch_x6w8<256, 32, 4, 1, 64, false>(p, batch, phases, s);
    }
    name("conv_gemm_x6w4<256,32>", "conv_gemm_bf16w4<256,32>");
    return launch_x6w8<256, 32, 4, 1, 0, false>(p, batch, phases, s);
  }
  if (p.Cout % 128 == 0) {
    if (kname) *kname = "conv_gemm_f32<128,128>";
    return launch_f32<128, 128, 2, 2, false>(p, batch, phases, s);
  }
  if (p.Cout % 64 == 0) {
    if (kname) *kname = "conv_gemm_f32<256,64>";
    return launch_f32<256, 64, 4, 1, false>(p, batch, phases, s);
  }
  if (kname) *kname = "conv_gemm_f32<256,32>";
  return launch_f32<256, 32, 4, 1, false>(p, batch, phases, s);
}

hipError_t launch_conv_group(const ConvParams* ps, int n, int batch, hipStream_t s, const char** kname) {
  if (n < 1 || n > kMaxGroup || batch < 1) return hipErrorInvalidValue;
  const int cout = ps[0].Cout;
  if (ps[0].x_compact == 3) {  // h3 convs: conv_gemm_x3dw_group / x3dq_group (any tile count)
    const int bsel = x3dq_bn(ps[0]);
    const int bn = bsel == 512 ? 256 : bsel == 384 ? 128 : bsel, bm = bsel == 512 ? 256 : bsel == 384 ? 384 : 32768 / bn;
    for (int i = 0; i < n; ++i)
      if (ps[i].Cout != cout || ps[i].x_compact != 3 || ps[i].taps < 3 || x3dq_bn(ps[i]) != bsel ||
          !x3dq_ok(ps[i], bn, bsel >= 384))
        return hipErrorNotSupported;
    int order[kMaxGroup] = {0, 1, 2};
    for (int i = 0; i < n; ++i)
      for (int j = i + 1; j < n; ++j)
        if (ps[order[j]].taps > ps[order[i]].taps) std::swap(order[i], order[j]);
    ConvGroup g{};
    long long start = 0;
    for (int k = 0; k < n; ++k) {
      const ConvParams& p = ps[order[k]];
      g.p[k] = p;
      g.tiles_per_clip[k] = ((p.Lq + bm - 1) / bm) * (cout / bn);
      g.start[k] = (int)start;
      start += (long long)g.tiles_per_clip[k] * batch;
    }
    if (start > (1LL << 30)) return hipErrorInvalidValue;
    for (int k = n; k <= kMaxGroup; ++k) g.start[k] = (int)start;
    if (bsel == 384) {
      if (kname) *kname = "conv_gemm_x3dw_group<384,128,halo>";
      if (knobs(ps[0]).h3_split) hipLaunchKernelGGL((conv_gemm_x3dw_group<true, 128>), dim3((unsigned)start), dim3(512), 0, s, g);
      else hipLaunchKernelGGL((conv_gemm_x3dw_group<false, 128>), dim3((unsigned)start), dim3(512), 0, s, g);
    } else if (bsel == 512) {
      if (kname) *kname = "conv_gemm_x3dw_group<256,256,halo>";
      if (knobs(ps[0]).h3_split) hipLaunchKernelGGL(conv_gemm_x3dw_group<true>, dim3((unsigned)start), dim3(512), 0, s, g);
      else hipLaunchKernelGGL(conv_gemm_x3dw_group<false>, dim3((unsigned)start), dim3(512), 0, s, g);
    } else if (bn == 256) {
      if (kname) *kname = "conv_gemm_x3dq_group<128,256,halo>";
      hipLaunchKernelGGL((conv_gemm_x3dq_group<256>), dim3((unsigned)start), dim3(512), 0, s, g);
    } else {
      if (kname) *kname = "conv_gemm_x3dq_group<256,128,halo>";
      hipLaunchKernelGGL((conv_gemm_x3dq_group<128>), dim3((unsigned)start), dim3(512), 0, s, g);
    }
    return hipGetLastError();
  }
  const int bn = cout % 256 == 0 ? 256 : 128, bm = 65536 / bn;
  // every member must be one launch_conv would give to conv_gemm_x6dq<bn> (same bits either way)
  for (int i = 0; i < n; ++i) {
    const ConvParams& p = ps[i];
    if (p.Cout != cout || cout % 128 || p.Cin % BK || !p.x6 || !p.w6 || p.nprod != 6 || p.x_compact || p.taps < 3 ||
        tap_span(p) == 0 || tap_span(p) > 64 || (p.Cin / BK) * p.taps % 2 || !x6dm_ok(p, true, bn) ||
        !big_tiles_pay(p, 1, bn))
      return hipErrorNotSupported;
  }
  int order[kMaxGroup] = {0, 1, 2};  // longest (most taps) first
  for (int i = 0; i < n; ++i)
    for (int j = i + 1; j < n; ++j)
      if (ps[order[j]].taps > ps[order[i]].taps) std::swap(order[i], order[j]);
  ConvGroup g{};
  long long start = 0;
  for (int k = 0; k < n; ++k) {
    const ConvParams& p = ps[order[k]];
    g.p[k] = p;
    g.tiles_per_clip[k] = ((p.Lq + bm - 1) / bm) * (cout / bn);
    g.start[k] = (int)start;
    start += (long long)g.tiles_per_clip[k] * batch;
  }
  if (start > (1LL << 30)) return hipErrorInvalidValue;
  for (int k = n; k <= kMaxGroup; ++k) g.start[k] = (int)start;
  if (bn == 256) {
    if (kname) *kname = "conv_gemm_x6dq_group<256,256,halo>";
    hipLaunchKernelGGL((conv_gemm_x6dq_group<256>), dim3((unsigned)start), dim3(512), 0, s, g);
  } else {
    if (kname) *kname = "conv_gemm_x6dq_group<512,128,halo>";
    hipLaunchKernelGGL((conv_gemm_x6dq_group<128>), dim3((unsigned)start), dim3(512), 0, s, g);
  }
  return hipGetLastError();
}

hipError_t launch_conv_split_group(const ConvParams* ps, int n, int batch, hipStream_t s, const char** kname) {
  if (n < 1 || n > kMaxGroup || batch < 1) return hipErrorInvalidValue;
  for (int i = 0; i < n; ++i) {  // every member a conv launch_conv would give to conv_gemm_x6pp<64, 128>
    const ConvParams& p = ps[i];
    const int S = std::max(1, p.ksplit);
    const int span = tap_span(p);
    if (!p.x6 || !p.w6 || p.nprod != 6 || p.x_compact || p.Cout % 128 || p.Cin % BK || p.taps < 3 || span == 0 ||
        span > 64 || (p.Cin / BK) * p.taps % 2 || (S > 1 && (p.kunit < 1 || (p.Cin / BK) % p.kunit ||
                                                            (p.Cin / BK) / p.kunit < S)))
      return hipErrorNotSupported;
  }
  int order[kMaxGroup] = {0, 1, 2};  // most work per slice first
  auto work = [&](int i) { return (long long)ps[i].taps * (ps[i].Cin / BK) / std::max(1, ps[i].ksplit); };
  for (int i = 0; i < n; ++i)
    for (int j = i + 1; j < n; ++j)
      if (work(order[j]) > work(order[i])) std::swap(order[i], order[j]);
  ConvGroup g{};
  long long start = 0;
  for (int k = 0; k < n; ++k) {
    const ConvParams& p = ps[order[k]];
    g.p[k] = p;
    g.p[k].batch = batch * std::max(1, p.ksplit);
    g.p[k].phases = 1;
    g.tiles_per_clip[k] = ((p.Lq + 255) / 256) * (p.Cout / 128);
    g.start[k] = (int)start;
    start += (long long)g.tiles_per_clip[k] * g.p[k].batch;
  }
  if (start > (1LL << 30)) return hipErrorInvalidValue;
  for (int k = n; k <= kMaxGroup; ++k) g.start[k] = (int)start;
  if (kname) *kname = "conv_gemm_x6pp_group<256,128,halo>";
  hipLaunchKernelGGL(conv_gemm_x6pp_group, dim3((unsigned)start), dim3(512), 0, s, g);
  return hipGetLastError();
}

hipError_t launch_splitk_epilogue_group(const ConvParams* ps, const float* const* partials, const int* splits,
                                        const long long* strides, int n, int batch, bool chain, hipStream_t s) {
  if (n < 1 || n > kMaxGroup || batch < 1) return hipErrorInvalidValue;
  SplitEpiGroup g{};
  g.chain = chain ? n : 0;
  long long start = 0;
  for (int k = 0; k < n; ++k) {
    const ConvParams& p = ps[k];
    if (splits[k] < 1 || p.Cout % 4 || p.ldy != p.Cout) return hipErrorInvalidValue;
    g.p[k] = p;
    g.p[k].batch = batch;
    g.p[k].phases = 1;
    g.part[k] = partials[k];
    g.splits[k] = splits[k];
    g.stride[k] = strides[k];
    g.total4[k] = (long long)batch * p.Lq * (p.Cout / 4);
    if (chain && (p.Lq != ps[0].Lq || p.Cout != ps[0].Cout)) return hipErrorInvalidValue;
    g.start[k] = (int)start;
    // chain: one range of blocks (member 0's) whose threads finish every member in order; the
    // other members' ranges are empty but start[] still marks which members exist
    start += chain && k > 0 ? 0 : (g.total4[k] + 255) / 256;
  }
  if (start > (1LL << 30)) return hipErrorInvalidValue;
  for (int k = n; k <= kMaxGroup; ++k) g.start[k] = (int)start;
  hipLaunchKernelGGL(splitk_epilogue_group_kernel, dim3((unsigned)start), dim3(256), 0, s, g);
  return hipGetLastError();
}

int vq_argmin_ntiles(int ncodes) { return ncodes / 128; }

// code tile of the x6-mode prefilter: 256 (vq_prefilter_dm) where its shape limits hold, else 128
static bool vq_dm_ok(int ncodes, int dim) {
#ifdef DCX_NO_VQDM
  return false;
#endif
  return ncodes % (256 * 16) == 0 && dim % BK == 0 && dim / BK >= 3 && (long long)dim * 6 * 256 < (1ll << 31) &&
         (long long)(dim / BK) * ncodes * 96 < (1ll << 31);
}
// Code tile of the prefilter launch_vq_prefilter picks: 256 for vq_prefilter_bk / vq_prefilter_dm, 128
// for vq_prefilter_x3 (planes x_pjt_in where vq_prefilter_dm's limits fail).  (Routing searches of one
// row panel, a streaming hop, to the 128-code tiles for twice the workgroups measured 1.55 -> 2.55 ms.)
int vq_prefilter_ntiles(int ncodes, int dim, long long rows, int x_layout) {
  (void)rows;
  if (x_layout == 1 || x_layout == 2) return ncodes / 256;
  return ncodes / (vq_dm_ok(ncodes, dim) ? 256 : 128);
}

hipError_t launch_vq_argmin(const ConvParams& p, int rows, hipStream_t s, const char** kname) {
  if (p.Cin % BK || p.Cout % 128) return hipErrorInvalidValue;
  ConvParams q = p;
  q.Lq = rows;
  q.Lin = rows;
  if (p.w6) return hipErrorInvalidValue;  // x6 mode searches with launch_vq_prefilter + rescore
  if (kname) *kname = "vq_dist_argmin_f32<128,128>";
  return launch_f32<128, 128, 2, 2, true>(q, 1, 1, s);
}

// bf16x3 prefilter of the VQ search (x6 mode).  With x = h + m + l per operand (dcx_planes.h,
// u = 2^-8), dropping h*l', m*m', l*h' and smaller leaves an error <= 3.1 u^2 sum_k |x_k e_k|
// (4.7e-5); fp32 accumulation of 672 MFMA partial sums adds <= 2688 * 2^-24 (1.6e-4, allowing 4
// roundings per MFMA).  By Cauchy-Schwarz sum_k |x_k e_k| <= |x| max|e|, so each approximate
// squared distance is within 2 * kVqPrefilterBound * |x| max|e| + 8 * 2^-24 (|x|^2 + max|e|^2)
// of the exact one; vq_rescore_kernel uses that bound.
bool vq_bk_takes(int ncodes, int dim) {
#ifdef DCX_NO_VQBK
  return false;
#endif
  return ncodes % (256 * 16) == 0 && dim % 32 == 0 && dim / 32 >= 3 && (long long)dim * 2 * 256 < (1ll << 31) &&
         (long long)(dim / 32) * ncodes * 128 < (1ll << 31);
}

bool vq_hm_takes(int ncodes, int dim, long long rows) {
  (void)rows;
  return vq_bk_takes(ncodes, dim) && vq_dm_ok(ncodes, dim);
}

// vq_prefilter_b1's ring depth (slots of 32 KiB; DCX_VQ_NS=3..5 in A/B builds)
#ifndef DCX_VQ_NS
#define DCX_VQ_NS 4
#endif
bool vq_b1_takes(int ncodes, int dim) {
#ifdef DCX_VQ_OLD
  return false;
#endif
  return ncodes % (256 * 16) == 0 && dim % 32 == 0 && dim / 32 >= DCX_VQ_NS && (long long)dim * 2 * 256 < (1ll << 31) &&
         (long long)(dim / 32) * ncodes * 64 < (1ll << 31);
}

// vq_prefilter_b1 (x_layout 1 unless built with DCX_VQ_OLD): x.e - x_h.e_h = x_r.e + x_h.d with
// |x_r.e| <= |x_r| max|e| (the rescore's second term) and |x_h.d| <= |x_h| max|d| <= (1 + 2^-8)|x| dmax;
// fp32 summation of the dim exact products, in whatever order the MFMAs add them, errs by at most
// dim 2^-24 sum_k |x_h,k e_h,k| <= dim 2^-24 (1 + 2^-8)^2 |x| max|e|.  The other kernels: the
// kVqPrefilterBound form of the comment above vq_bk_takes.
double vq_prefilter_cx(int x_layout, int ncodes, int dim, float emax, float dmax) {
  if (x_layout != 1 || !vq_b1_takes(ncodes, dim)) return (double)kVqPrefilterBound * emax;
  return (1.0 + 0x1p-8) * (double)dmax + (double)dim * 0x1p-24 * (1.0 + 0x1p-6) * (double)emax;
}

hipError_t launch_vq_prefilter(const ConvParams& p, int rows, bool x_bf16, hipStream_t s, const char** kname) {
  constexpr int BM = 256, BN = 128;
  if (!p.x6 || !p.part_val2 || rows < 1) return hipErrorInvalidValue;
  ConvParams q = p;
  q.Lq = rows;
  q.Lin = rows;
  q.taps = 1;
#ifndef DCX_VQ_OLD
  if (p.x_compact == 1) {  // compact x_pjt_in (either mode) and the [CD/32][NC][32] hi codebook
    if (!p.wc || !vq_b1_takes(p.Cout, p.Cin)) return hipErrorInvalidValue;
    const int mtiles = (rows + 255) / 256, ntiles = p.Cout / 256;
    const dim3 grid(vq_grid(mtiles, ntiles));
    if (kname) *kname = "vq_prefilter_b1<256,256>";
    hipLaunchKernelGGL(vq_prefilter_b1<DCX_VQ_NS>, grid, dim3(512), 0, s, q);
    return hipGetLastError();
  }
  if (p.x_compact == 2) return hipErrorInvalidValue;
#endif
  if (!p.w6 || p.Cin % BK || p.Cout % (BN * 16)) return hipErrorInvalidValue;
  if (p.x_compact == 2) {  // x6 mode, "hm" x_pjt_in and the repacked codebook: vq_prefilter_dm
    if (x_bf16 || !p.wc || !vq_hm_takes(p.Cout, p.Cin, rows)) return hipErrorInvalidValue;
    const int mtiles = (rows + 255) / 256, ntiles = p.Cout / 256;
    const dim3 grid(vq_grid(mtiles, ntiles));
    if (kname) *kname = "vq_prefilter_dm<256,256>";
    hipLaunchKernelGGL((vq_prefilter_dm<true>), grid, dim3(512), 0, s, q);
    return hipGetLastError();
  }
  if (p.x_compact == 1) {  // bf16 mode, compact x_pjt_in and the repacked codebook
    if (!x_bf16 || !p.wc || !vq_bk_takes(p.Cout, p.Cin)) return hipErrorInvalidValue;
    const int mtiles = (rows + 255) / 256, ntiles = p.Cout / 256;
    const dim3 grid(vq_grid(mtiles, ntiles));
#ifdef DCX_VQ_BK32  // the 32x32x16 form (A/B builds)
    if (kname) *kname = "vq_prefilter_bk<256,256>";
    hipLaunchKernelGGL(vq_prefilter_bk, grid, dim3(512), 0, s, q);
#else
    if (kname) *kname = "vq_prefilter_bq<256,256>";
    hipLaunchKernelGGL(vq_prefilter_bq, grid, dim3(512), 0, s, q);
#endif
    return hipGetLastError();
  }
  if (vq_dm_ok(p.Cout, p.Cin)) {
    const int mtiles = (rows + 255) / 256, ntiles = p.Cout / 256;
    const dim3 grid(vq_grid(mtiles, ntiles));
    if (kname) *kname = x_bf16 ? "vq_prefilter_dm_x2<256,256>" : "vq_prefilter_dm<256,256>";
    if (x_bf16) hipLaunchKernelGGL((vq_prefilter_dm<false>), grid, dim3(512), 0, s, q);
    else hipLaunchKernelGGL((vq_prefilter_dm<true>), grid, dim3(512), 0, s, q);
    return hipGetLastError();
  }
  const int mtiles = (rows + BM - 1) / BM, ntiles = p.Cout / BN;
  const int nsm = (mtiles + 15) / 16;
  dim3 grid(vq_grid(mtiles, ntiles));
  (void)nsm;
  if (p.Cin % 64) return hipErrorInvalidValue;  // even number of K32 steps
  if (x_bf16) {
    if (kname) *kname = "vq_prefilter_x2<256,128>";
    hipLaunchKernelGGL((vq_prefilter_x3<BM, BN, 4, 2, false>), grid, dim3(512), 0, s, q);
  } else {
    if (kname) *kname = "vq_prefilter_x3<256,128>";
    hipLaunchKernelGGL((vq_prefilter_x3<BM, BN, 4, 2, true>), grid, dim3(512), 0, s, q);
  }
  return hipGetLastError();
}

}  // namespace dcx

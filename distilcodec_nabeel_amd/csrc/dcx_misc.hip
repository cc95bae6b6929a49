// Bandwidth-bound kernels of the DistilCodec path (gfx950): row LayerNorms, the fused
// depthwise-conv + LayerNorm front of each ConvNeXt block, the STFT framing / magnitude steps,
// codebook gathers, the VQ partial-argmin reduction, conv_post + tanh, and a batched transpose.
// All use 16-byte accesses along the contiguous channel axis (channels-last layout).
#include "dcx_kernels.h"
#include "dcx_planes.h"

#include <algorithm>

namespace dcx {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// ---------------------------------------------------------------------------------------------
// LayerNorm over the channel axis of each row.  channels_first_form=1 follows the reference's
// custom channels_first LayerNorm `(x-u)/sqrt(s+eps)*w+b` (convnext_utils.py:208-213);
// 0 follows F.layer_norm (`(x-u)*rsqrt(s+eps)*w+b`, convnext_utils.py:205).  Biased variance.
// 2: the channels_first form on a bf16 input under the reference's CUDA autocast (the encoder
// stem, whose Conv1d returns bf16; DCX_GEMM_BF16): `x.mean(1)` and `x - u` run in bf16 (fp32
// arithmetic, bf16 results), `.pow(2)` is on autocast's fp32 list, so s is the fp32 mean of the
// squared bf16 differences and the rest is fp32.
// One wave per row, NV float4 per lane (C = 256*NV).
// ---------------------------------------------------------------------------------------------
template <int NV>
__device__ __forceinline__ void ln_finish(f32x4 (&v)[NV], int C, float eps, int cf, const float* __restrict__ w,
                                          const float* __restrict__ b, float* __restrict__ yrow,
                                          unsigned short* __restrict__ y6, int y6c, long long row, int lane,
                                          int* __restrict__ ash_row, float* __restrict__ amax_row) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  float mean = wave_sum(s) / (float)C;
  if (cf == 2) {  // v := bf16(x - bf16(mean)); the fp32 steps below then see u = 0
    mean = bf16_val(bf16_bits(mean));
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = round_bf16x4(v[i] - mean);
    mean = 0.f;
  }
  float sq = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const f32x4 d = v[i] - mean;
    sq += (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w);
  }
  const float var = wave_sum(sq) / (float)C;
  const float den = sqrtf(var + eps);
  const float rstd = 1.0f / den;
  f32x4 ov[NV];
  float am = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (lane + 64 * i) * 4;
    const f32x4 wv = *reinterpret_cast<const f32x4*>(w + c);
    const f32x4 bv = *reinterpret_cast<const f32x4*>(b + c);
    f32x4 o;
    if (cf) {  // 1, 2
      o = (v[i] - mean) / den * wv + bv;
    } else {
      o = (v[i] - mean) * rstd * wv + bv;
    }
    ov[i] = o;
    am = fmaxf(am, fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fmaxf(fabsf(o.z), fabsf(o.w))));
    if (yrow) *reinterpret_cast<f32x4*>(yrow + c) = o;
  }
  if (!y6) return;
  // h2 (an h3 one-tap consumer): the row scaled by 2^h2_shift(its exact max |o|), the shift and the
  // max recorded per row (dcx_kernels.h)
  float sc = 1.0f;
  if (y6c == 3) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) am = fmaxf(am, __shfl_xor(am, off, 64));
    const int sh = h2_shift(am);
    sc = __builtin_ldexpf(1.0f, sh);
    if (lane == 0) {
      ash_row[row] = sh;
      if (amax_row) amax_row[row] = am;
    }
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (lane + 64 * i) * 4;
    const f32x4 o = ov[i];
    if (y6c == 1) store_bf16x4(y6, row, C, c, o.x, o.y, o.z, o.w);
    else if (y6c == 3) store_h2_4(y6, row, C, c, o.x, o.y, o.z, o.w, sc);
    else store_planes4(y6, row, C, c, o.x, o.y, o.z, o.w);
  }
}

template <int NV>
__global__ void __launch_bounds__(256) ln_rows_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                       unsigned short* __restrict__ y6, int y6c, const float* __restrict__ w,
                                                       const float* __restrict__ b, long long rows, float eps, int cf,
                                                       int* ash_row, float* amax_row) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  constexpr int C = 256 * NV;
  f32x4 v[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = *reinterpret_cast<const f32x4*>(x + row * C + (lane + 64 * i) * 4);
  ln_finish<NV>(v, C, eps, cf, w, b, y ? y + row * C : nullptr, y6, y6c, row, lane, ash_row, amax_row);
}

hipError_t launch_ln_rows(const float* x, float* y, unsigned short* y6, int y6c, const float* w, const float* b,
                          long long rows, int C, float eps, int cf, hipStream_t s, int* ash_row, float* amax_row) {
  if (y6 && y6c == 3 && !ash_row) return hipErrorInvalidValue;
  dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  switch (C) {
    case 256: hipLaunchKernelGGL(ln_rows_kernel<1>, grid, block, 0, s, x, y, y6, y6c, w, b, rows, eps, cf, ash_row, amax_row); break;
    case 512: hipLaunchKernelGGL(ln_rows_kernel<2>, grid, block, 0, s, x, y, y6, y6c, w, b, rows, eps, cf, ash_row, amax_row); break;
    case 768: hipLaunchKernelGGL(ln_rows_kernel<3>, grid, block, 0, s, x, y, y6, y6c, w, b, rows, eps, cf, ash_row, amax_row); break;
    case 1024: hipLaunchKernelGGL(ln_rows_kernel<4>, grid, block, 0, s, x, y, y6, y6c, w, b, rows, eps, cf, ash_row, amax_row); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ConvNeXtBlock front (convnext_utils.py:266-268): depthwise Conv1d k7 p3 (+bias) then
// F.layer_norm over channels.  dww is packed [7][C].  A workgroup (4 waves) owns DW_R consecutive
// rows of one clip: it stages their input rows with the 3-row halo on each side in LDS once (rows
// outside the clip as zeros: the conv's padding), so each input row is read from memory
// (R + 6) / R times instead of 7; each wave then finishes every 4th row (taps from LDS, one wave
// per row for the LayerNorm reduction).  The per-row arithmetic and its order are those of the
// one-wave-per-row form this replaces (taps in order, out-of-range products dropped).
// DW_R = 16 rows per workgroup; 4 when 16-row tiles would leave most CUs idle (a streaming hop).
template <int NV, int DW_R>
__global__ void __launch_bounds__(256) dwconv_ln_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                         unsigned short* __restrict__ y6, int y6c,
                                                         const float* __restrict__ dww, const float* __restrict__ dwb,
                                                         const float* __restrict__ lnw, const float* __restrict__ lnb,
                                                         int L, int tiles, int bf, int* ash_row, float* amax_row) {
  constexpr int C = 256 * NV, C4 = C / 4, ROWS = DW_R + 6;
  __shared__ f32x4 tile[ROWS * C4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int bidx = blockIdx.x / tiles, t0 = (blockIdx.x - bidx * tiles) * DW_R;
  const float* xb = x + (long long)bidx * L * C;
  // stage rows t0 - 3 .. t0 + DW_R + 2 (all loads issued before any LDS store)
  constexpr int PER = (ROWS * C4 + 255) / 256;
  f32x4 st[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int i = threadIdx.x + k * 256;
    const int r = i / C4, c4 = i - r * C4;
    const int tt = t0 - 3 + r;
    const bool ok = i < ROWS * C4 && tt >= 0 && tt < L;
    st[k] = ok ? *reinterpret_cast<const f32x4*>(xb + (long long)tt * C + c4 * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
    if (bf) st[k] = round_bf16x4(st[k]);
  }
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int i = threadIdx.x + k * 256;
    if (i < ROWS * C4) tile[i] = st[k];
  }
  f32x4 wv[NV][7], bv[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (lane + 64 * i) * 4;
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      wv[i][j] = *reinterpret_cast<const f32x4*>(dww + j * C + c);
      if (bf) wv[i][j] = round_bf16x4(wv[i][j]);
    }
    bv[i] = *reinterpret_cast<const f32x4*>(dwb + c);
    if (bf) bv[i] = round_bf16x4(bv[i]);
  }
  __syncthreads();
  for (int rr = wave; rr < DW_R; rr += 4) {
    const int t = t0 + rr;
    if (t >= L) break;  // wave-uniform
    f32x4 v[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c4 = lane + 64 * i;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 7; ++j) {
        const int tt = t + j - 3;
        const f32x4 pr = tile[(rr + j) * C4 + c4] * wv[i][j];
        if (tt >= 0 && tt < L) acc += pr;
      }
      v[i] = acc + bv[i];
      if (bf) v[i] = round_bf16x4(v[i]);
    }
    const long long row = (long long)bidx * L + t;
    ln_finish<NV>(v, C, 1e-6f, 0, lnw, lnb, y ? y + row * C : nullptr, y6, y6c, row, lane, ash_row, amax_row);
  }
}

// dwconv_ln_run (round 3): the same per-row arithmetic without the per-workgroup staging.  One
// wave walks RW consecutive rows of one clip (launches of >= 8192 rows) with the 7-row input
// window in registers (a ring of 7 + D rows: row t + 3 + D is loaded while row t is finished), so
// each input row is read (RW + 6) / RW times and its load overlaps the previous rows' LayerNorms;
// the taps sit in LDS (28 KiB at C = 1024).  The tiled kernel above held 22 fp32 rows in LDS per
// 4-wave workgroup (88 KiB at C = 1024: one workgroup per CU, its loads and its arithmetic never
// overlapping): C3's 19 launches ran at 3.75 TB/s.  The ring slots are static in the unrolled loop
// (slot = row mod S).
template <int NV, int RW, int D>
__global__ void __launch_bounds__(256) dwconv_ln_run_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                             unsigned short* __restrict__ y6, int y6c,
                                                             const float* __restrict__ dww, const float* __restrict__ dwb,
                                                             const float* __restrict__ lnw, const float* __restrict__ lnb,
                                                             int L, int runs, long long nruns, int bf, int* ash_row,
                                                             float* amax_row) {
  constexpr int C = 256 * NV, C4 = C / 4, S = 7 + D;
  __shared__ f32x4 wsh[7 * C4];
  for (int i = threadIdx.x; i < 7 * C4; i += 256) {
    const f32x4 wv = reinterpret_cast<const f32x4*>(dww)[i];
    wsh[i] = bf ? round_bf16x4(wv) : wv;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long long run = (long long)blockIdx.x * 4 + wave;
  if (run >= nruns) return;  // whole wave, after the block's only barrier
  const int bidx = (int)(run / runs), t0 = (int)(run - (long long)bidx * runs) * RW, t1 = min(t0 + RW, L);
  const float* xb = x + (long long)bidx * L * C;
  f32x4 win[S][NV], bv[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    bv[i] = *reinterpret_cast<const f32x4*>(dwb + (lane + 64 * i) * 4);
    if (bf) bv[i] = round_bf16x4(bv[i]);
  }
  auto load_row = [&](f32x4 (&dst)[NV], int tt) {  // row clamped: out-of-range taps are dropped below
    const float* src = xb + (long long)min(max(tt, 0), L - 1) * C;
#pragma unroll
    for (int i = 0; i < NV; ++i) dst[i] = *reinterpret_cast<const f32x4*>(src + (lane + 64 * i) * 4);
  };
  // bf16 mode: a row is rounded where it is first used (tap 6 of row r - 3), not where it is loaded,
  // so the prefetch keeps its distance
  auto round_row = [&](f32x4 (&r)[NV]) {
#pragma unroll
    for (int i = 0; i < NV; ++i) r[i] = round_bf16x4(r[i]);
  };
  // rows t0 - 3 .. t0 + 2 + D in slots 0 .. 5 + D (row r in slot (r - t0 + 3) mod S)
#pragma unroll
  for (int k = 0; k < 6 + D; ++k) load_row(win[k], t0 - 3 + k);
  if (bf) {
#pragma unroll
    for (int k = 0; k < 6; ++k) round_row(win[k]);
  }
  for (int t = t0;; t += S) {
#pragma unroll
    for (int k = 0; k < S; ++k) {
      const int tk = t + k;
      if (tk >= t1) return;  // wave-uniform
      if (bf) round_row(win[(k + 6) % S]);  // row tk + 3, first used now
      if (tk + 3 + D < t1 + 3) load_row(win[(k + S - 1) % S], tk + 3 + D);  // into row tk - 4's slot
      f32x4 v[NV];
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int c4 = lane + 64 * i;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 7; ++j) {
          const int tt = tk + j - 3;
          const f32x4 pr = win[(k + j) % S][i] * wsh[j * C4 + c4];
          if (tt >= 0 && tt < L) acc += pr;
        }
        v[i] = acc + bv[i];
        if (bf) v[i] = round_bf16x4(v[i]);
      }
      const long long row = (long long)bidx * L + tk;
      ln_finish<NV>(v, C, 1e-6f, 0, lnw, lnb, y ? y + row * C : nullptr, y6, y6c, row, lane, ash_row, amax_row);
    }
  }
}

template <int NV>
static void launch_dwconv_ln_nv(const float* x, float* y, unsigned short* y6, int y6c, const float* dww,
                                const float* dwb, const float* lnw, const float* lnb, int batch, int L, int rw, int bf,
                                hipStream_t s, int* ash_row, float* amax_row) {
  const int runs = (L + rw - 1) / rw;
  const long long nruns = (long long)batch * runs;
  const dim3 grid((unsigned)((nruns + 3) / 4)), block(256);
  constexpr int D = NV >= 4 ? 1 : 2;  // rows prefetched beyond the window (registers: 2 waves per SIMD at C = 1024)
  switch (rw) {
    case 32: hipLaunchKernelGGL((dwconv_ln_run_kernel<NV, 32, D>), grid, block, 0, s, x, y, y6, y6c, dww, dwb, lnw, lnb, L, runs, nruns, bf, ash_row, amax_row); break;
    case 16: hipLaunchKernelGGL((dwconv_ln_run_kernel<NV, 16, D>), grid, block, 0, s, x, y, y6, y6c, dww, dwb, lnw, lnb, L, runs, nruns, bf, ash_row, amax_row); break;
    case 8: hipLaunchKernelGGL((dwconv_ln_run_kernel<NV, 8, D>), grid, block, 0, s, x, y, y6, y6c, dww, dwb, lnw, lnb, L, runs, nruns, bf, ash_row, amax_row); break;
    default: hipLaunchKernelGGL((dwconv_ln_run_kernel<NV, 4, D>), grid, block, 0, s, x, y, y6, y6c, dww, dwb, lnw, lnb, L, runs, nruns, bf, ash_row, amax_row); break;
  }
}

hipError_t launch_dwconv_ln(const float* x, float* y, unsigned short* y6, int y6c, const float* dww, const float* dwb,
                            const float* lnw, const float* lnb, int batch, int L, int C, int bf16, const Knobs* kn,
                            hipStream_t s, int* ash_row, float* amax_row) {
  if (y6 && y6c == 3 && !ash_row) return hipErrorInvalidValue;
  const bool tiled = kn && kn->dwconv_tiled;  // A/B and tests: the round-2 tiled kernel (same bits)
  const long long rows = (long long)batch * L;
  // below 8192 rows (a streaming hop: 93 rows) the tiled kernel's 4-row tiles, one row per wave,
  // measured faster than runs of 1 or 4 rows (C5 hop 4.06-4.09 vs 4.09-4.14 ms, A/B)
  if (!tiled && rows >= 8192) {
    // rows per wave: the longest run that still gives >= 2048 waves (8 per CU)
    const int rw = rows >= 2048LL * 32 ? 32 : rows >= 2048LL * 16 ? 16 : rows >= 2048LL * 8 ? 8 : 4;
    if ((long long)batch * ((L + rw - 1) / rw) / 4 >= (1LL << 31)) return hipErrorInvalidValue;
    switch (C) {
      case 256: launch_dwconv_ln_nv<1>(x, y, y6, y6c, dww, dwb, lnw, lnb, batch, L, rw, bf16, s, ash_row, amax_row); break;
      case 512: launch_dwconv_ln_nv<2>(x, y, y6, y6c, dww, dwb, lnw, lnb, batch, L, rw, bf16, s, ash_row, amax_row); break;
      case 768: launch_dwconv_ln_nv<3>(x, y, y6, y6c, dww, dwb, lnw, lnb, batch, L, rw, bf16, s, ash_row, amax_row); break;
      case 1024: launch_dwconv_ln_nv<4>(x, y, y6, y6c, dww, dwb, lnw, lnb, batch, L, rw, bf16, s, ash_row, amax_row); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }

  const bool small = (long long)batch * ((L + 15) / 16) < 512;
  const int R = small ? 4 : 16, tiles = (L + R - 1) / R;
  if ((long long)batch * tiles >= (1LL << 31)) return hipErrorInvalidValue;
  dim3 grid((unsigned)(batch * tiles)), block(256);
  switch (C) {
    case 256: if (small) hipLaunchKernelGGL((dwconv_ln_kernel<1, 4>), grid, block, 0, s, x, y, y6, y6c, dww, dwb, lnw, lnb, L, tiles, bf16, ash_row, amax_row);
      else hipLaunchKernelGGL((dwconv_ln_kernel<1, 16>), grid, block, 0, s, x, y, y6, y6c, dww, dwb, lnw, lnb, L, tiles, bf16, ash_row, amax_row); break;
    case 512: if (small) hipLaunchKernelGGL((dwconv_ln_kernel<2, 4>), grid, block, 0, s, x, y, y6, y6c, dww, dwb, lnw, lnb, L, tiles, bf16, ash_row, amax_row);
      else hipLaunchKernelGGL((dwconv_ln_kernel<2, 16>), grid, block, 0, s, x, y, y6, y6c, dww, dwb, lnw, lnb, L, tiles, bf16, ash_row, amax_row); break;
    case 768: if (small) hipLaunchKernelGGL((dwconv_ln_kernel<3, 4>), grid, block, 0, s, x, y, y6, y6c, dww, dwb, lnw, lnb, L, tiles, bf16, ash_row, amax_row);
      else hipLaunchKernelGGL((dwconv_ln_kernel<3, 16>), grid, block, 0, s, x, y, y6, y6c, dww, dwb, lnw, lnb, L, tiles, bf16, ash_row, amax_row); break;
    case 1024: if (small) hipLaunchKernelGGL((dwconv_ln_kernel<4, 4>), grid, block, 0, s, x, y, y6, y6c, dww, dwb, lnw, lnb, L, tiles, bf16, ash_row, amax_row);
      else hipLaunchKernelGGL((dwconv_ln_kernel<4, 16>), grid, block, 0, s, x, y, y6, y6c, dww, dwb, lnw, lnb, L, tiles, bf16, ash_row, amax_row); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// STFT framing: reflect pad ((win-hop)/2 each side, mel_spec.py:30-37) and cut the padded
// signal into rows of `hop` samples, so frame f = rows f..f+3 (a 4-tap conv over 256 channels).
// ---------------------------------------------------------------------------------------------
__global__ void frame_pad_kernel(const float* __restrict__ audio, float* __restrict__ frames,
                                 unsigned short* __restrict__ frames6, long long n, int rows, int hop, int pad_left) {
  const int b = blockIdx.y;
  const long long total4 = (long long)rows * hop / 4;
  for (long long i4 = (long long)blockIdx.x * blockDim.x + threadIdx.x; i4 < total4;
       i4 += (long long)gridDim.x * blockDim.x) {
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      long long src = i4 * 4 + e - pad_left;
      if (src < 0) src = -src;
      if (src >= n) src = 2 * (n - 1) - src;
      v[e] = audio[(long long)b * n + src];
    }
    const long long i = i4 * 4;
    if (frames) *reinterpret_cast<f32x4*>(frames + (long long)b * rows * hop + i) = f32x4{v[0], v[1], v[2], v[3]};
    if (frames6) {
      const long long row = (long long)b * rows + i / hop;
      store_planes4(frames6, row, hop, (int)(i % hop), v[0], v[1], v[2], v[3]);
    }
  }
}

hipError_t launch_frame_pad(const float* audio, float* frames, unsigned short* frames6, int batch, long long n, int rows,
                            int hop, int pad_left, hipStream_t s) {
  if (hop % 8) return hipErrorInvalidValue;
  const long long total4 = (long long)rows * hop / 4;
  unsigned gx = (unsigned)((total4 + 255) / 256);
  if (gx > 4096) gx = 4096;
  hipLaunchKernelGGL(frame_pad_kernel, dim3(gx, batch), dim3(256), 0, s, audio, frames, frames6, n, rows, hop, pad_left);
  return hipGetLastError();
}

// |STFT| = sqrt(re^2 + im^2 + 1e-6) (mel_spec.py:54-55).  spec columns: [0, nbins) real part of
// bins 0..nbins-1, [nbins, 2*nbins-2) imaginary part of bins 1..nbins-2 (bins 0 and n_fft/2 are
// real for a real signal).  Output row padded with zeros to ld_out.  Optional loglin [rows][nbins]:
// compress(linear) = log(clamp(|STFT|, 1e-5)), the second output of return_linear (mel_spec.py:119-120).
__global__ void spec_mag_kernel(const float* __restrict__ spec, float* __restrict__ mag, unsigned short* __restrict__ mag6,
                                float* __restrict__ loglin, long long rows, int nbins, int ld_out) {
  const long long row = blockIdx.x;
  if (row >= rows) return;
  const int ld_in = 2 * nbins - 2;
  for (int k4 = threadIdx.x * 4; k4 < ld_out; k4 += blockDim.x * 4) {
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = k4 + e;
      o[e] = 0.f;
      if (k < nbins) {
        const float re = spec[row * ld_in + k];
        const float im = (k > 0 && k < nbins - 1) ? spec[row * ld_in + nbins + k - 1] : 0.f;
        o[e] = sqrtf((re * re + im * im) + 1e-6f);
        if (loglin) loglin[row * nbins + k] = logf(fmaxf(o[e], 1e-5f));
      }
    }
    if (mag) *reinterpret_cast<f32x4*>(mag + row * ld_out + k4) = f32x4{o[0], o[1], o[2], o[3]};
    if (mag6) store_planes4(mag6, row, ld_out, k4, o[0], o[1], o[2], o[3]);
  }
}

hipError_t launch_spec_mag(const float* spec, float* mag, unsigned short* mag6, float* loglin, long long rows, int nbins,
                           int ld_out, hipStream_t s) {
  if (ld_out % 8 || ld_out < nbins) return hipErrorInvalidValue;
  hipLaunchKernelGGL(spec_mag_kernel, dim3((unsigned)rows), dim3(256), 0, s, spec, mag, mag6, loglin, rows, nbins, ld_out);
  return hipGetLastError();
}

// silu(x) as fp32 and/or planes (dcx_module_forward's ResBlock / ParallelBlock entries: the
// generator itself produces these in conv epilogues).  Same arithmetic as the epilogues' silu.  The
// h2 layout goes through launch_h2_ranged (its range scale needs the clip's max first).
__global__ void __launch_bounds__(256) silu_act_kernel(const float* __restrict__ x, float* __restrict__ yf,
                                                        unsigned short* __restrict__ y6, long long rows, int C) {
  const long long total4 = rows * C / 4;
  for (long long i4 = (long long)blockIdx.x * 256 + threadIdx.x; i4 < total4; i4 += (long long)gridDim.x * 256) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(x + i4 * 4);
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = v[e] * __builtin_amdgcn_rcpf(1.0f + __expf(-v[e]));
    if (yf) *reinterpret_cast<f32x4*>(yf + i4 * 4) = f32x4{o[0], o[1], o[2], o[3]};
    if (y6) store_planes4(y6, (i4 * 4) / C, C, (int)((i4 * 4) % C), o[0], o[1], o[2], o[3]);
  }
}

hipError_t launch_silu_act(const float* x, float* yf, unsigned short* y6, long long rows, int C, hipStream_t s, int h2) {
  if (C % 8 || rows < 0 || (h2 && y6)) return hipErrorInvalidValue;
  const long long total4 = rows * C / 4;
  if (total4 == 0) return hipSuccess;
  const long long nb = (total4 + 255) / 256;
  const unsigned g = (unsigned)(nb < 8192 ? nb : 8192);
  hipLaunchKernelGGL(silu_act_kernel, dim3(g), dim3(256), 0, s, x, yf, y6, rows, C);
  return hipGetLastError();
}

// launch_h2_ranged (round 6): the range of a tensor handed in by the caller, per clip (blockIdx.y):
// the max |x| over the clip, then the h2 split of f(x) * 2^h2_shift(max(amax, floor)).
__global__ void __launch_bounds__(256) clip_amax_kernel(const float* __restrict__ x, long long n4, float* amax) {
  const int b = blockIdx.y;
  const f32x4* xb = reinterpret_cast<const f32x4*>(x) + (long long)b * n4;
  float m = 0.f;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    const f32x4 v = xb[i];
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
  }
  range_report(m, amax, b, __builtin_inff(), nullptr, range_cur(amax, b));
}

__global__ void __launch_bounds__(256) h2_ranged_kernel(const float* __restrict__ x, float* __restrict__ yf,
                                                         unsigned short* __restrict__ y6, long long L, int C, int silu,
                                                         float floor, const float* __restrict__ amax, int* ash,
                                                         int* rflag) {
  const int b = blockIdx.y;
  const float bound = fmaxf(amax[b], floor);
  const int sh = h2_shift(bound);
  const float sc = __builtin_ldexpf(1.0f, sh);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    ash[b] = sh;
    if (rflag && !(bound <= 3.0e38f)) atomicOr(rflag, RANGE_NONFINITE);
  }
  const long long n4 = L * C / 4, base = (long long)b * L * C;
  for (long long i4 = (long long)blockIdx.x * 256 + threadIdx.x; i4 < n4; i4 += (long long)gridDim.x * 256) {
    const long long i = base + i4 * 4;
    const f32x4 v = *reinterpret_cast<const f32x4*>(x + i);
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = silu ? v[e] * __builtin_amdgcn_rcpf(1.0f + __expf(-v[e])) : v[e];
    if (yf) *reinterpret_cast<f32x4*>(yf + i) = f32x4{o[0], o[1], o[2], o[3]};
    store_h2_4(y6, i / C, C, (int)(i % C), o[0], o[1], o[2], o[3], sc);
  }
}

// launch_h2_rows (round 6): one wave per row, C = 256 NV channels: the row's max |x|, then its h2
// split scaled by 2^h2_shift(max) (the LayerNorm kernels' per-row form, for tensors in fp32)
template <int NV>
__global__ void __launch_bounds__(256) h2_rows_kernel(const float* __restrict__ x, unsigned short* __restrict__ y6,
                                                       long long rows, int* __restrict__ ash_row) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  constexpr int C = 256 * NV;
  f32x4 v[NV];
  float am = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    v[i] = *reinterpret_cast<const f32x4*>(x + row * C + (lane + 64 * i) * 4);
    am = fmaxf(am, fmaxf(fmaxf(fabsf(v[i].x), fabsf(v[i].y)), fmaxf(fabsf(v[i].z), fabsf(v[i].w))));
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) am = fmaxf(am, __shfl_xor(am, off, 64));
  const int sh = h2_shift(am);
  const float sc = __builtin_ldexpf(1.0f, sh);
  if (lane == 0) ash_row[row] = sh;
#pragma unroll
  for (int i = 0; i < NV; ++i) store_h2_4(y6, row, C, (lane + 64 * i) * 4, v[i].x, v[i].y, v[i].z, v[i].w, sc);
}

hipError_t launch_h2_rows(const float* x, unsigned short* y6, long long rows, int C, int* ash_row, hipStream_t s) {
  if (!x || !y6 || !ash_row || rows < 0) return hipErrorInvalidValue;
  if (rows == 0) return hipSuccess;
  dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  switch (C) {
    case 256: hipLaunchKernelGGL(h2_rows_kernel<1>, grid, block, 0, s, x, y6, rows, ash_row); break;
    case 512: hipLaunchKernelGGL(h2_rows_kernel<2>, grid, block, 0, s, x, y6, rows, ash_row); break;
    case 768: hipLaunchKernelGGL(h2_rows_kernel<3>, grid, block, 0, s, x, y6, rows, ash_row); break;
    case 1024: hipLaunchKernelGGL(h2_rows_kernel<4>, grid, block, 0, s, x, y6, rows, ash_row); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// Zeroes n 32-bit words with a kernel, not hipMemsetAsync: inside a hipGraph capture the kernel node
// is ordered like every other launch (round 6: with memset nodes for the range slots, the second
// replay of a captured hop read slots the first had left).
__global__ void __launch_bounds__(256) zero_words_kernel(unsigned* p, long long n) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) p[i] = 0u;
}

hipError_t launch_zero_words(void* p, long long n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (!p) return hipErrorInvalidValue;
  const long long nb = (n + 255) / 256;
  hipLaunchKernelGGL(zero_words_kernel, dim3((unsigned)std::min<long long>(nb, 1024)), dim3(256), 0, s, (unsigned*)p, n);
  return hipGetLastError();
}

hipError_t launch_clip_amax(const float* x, int batch, long long L, int C, float* amax, hipStream_t s) {
  if (C % 4 || L < 0 || batch < 1 || batch > 65535 || !amax) return hipErrorInvalidValue;
  hipError_t e = launch_zero_words(amax, batch, s);
  if (e != hipSuccess) return e;
  const long long n4 = L * C / 4;
  const unsigned gx = (unsigned)std::max<long long>(1, std::min<long long>((n4 + 255) / 256, std::max(1, 4096 / batch)));
  if (n4 > 0) hipLaunchKernelGGL(clip_amax_kernel, dim3(gx, batch), dim3(256), 0, s, x, n4, amax);
  return hipGetLastError();
}

hipError_t launch_h2_ranged(const float* x, float* yf, unsigned short* y6, int batch, long long L, int C, int silu,
                            float floor, float* amax, int* ash, int* rflag, hipStream_t s) {
  if (C % 32 || L < 0 || batch < 1 || batch > 65535 || !y6 || !amax || !ash) return hipErrorInvalidValue;
  hipError_t e = launch_zero_words(amax, batch, s);
  if (e != hipSuccess) return e;
  const long long n4 = L * C / 4;
  const long long nb = (n4 + 255) / 256;
  const unsigned gx = (unsigned)std::max<long long>(1, std::min<long long>(nb, std::max(1, 4096 / batch)));
  if (n4 > 0) hipLaunchKernelGGL(clip_amax_kernel, dim3(gx, batch), dim3(256), 0, s, x, n4, amax);
  hipLaunchKernelGGL(h2_ranged_kernel, dim3(gx, batch), dim3(256), 0, s, x, yf, y6, L, C, silu, floor, amax, ash, rflag);
  return hipGetLastError();
}

// fp32 [rows][C] -> planes, or (compact) bf16 [rows][C] (boundary conversion for tensors handed in
// by the caller; the h2 layout goes through launch_h2_ranged).
__global__ void __launch_bounds__(256) split_planes_kernel(const float* __restrict__ x, unsigned short* __restrict__ y6,
                                                            long long rows, int C, int compact) {
  const long long total4 = rows * C / 4;
  for (long long i4 = (long long)blockIdx.x * blockDim.x + threadIdx.x; i4 < total4;
       i4 += (long long)gridDim.x * blockDim.x) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(x + i4 * 4);
    const long long i = i4 * 4;
    if (compact == 1) store_bf16x4(y6, i / C, C, (int)(i % C), v.x, v.y, v.z, v.w);
    else if (compact == 2) store_hm4(y6, i / C, C, (int)(i % C), v.x, v.y, v.z, v.w);
    else store_planes4(y6, i / C, C, (int)(i % C), v.x, v.y, v.z, v.w);
  }
}

hipError_t launch_split_planes(const float* x, unsigned short* y6, long long rows, int C, int compact, hipStream_t s) {
  if (C % 8 || compact < 0 || compact > 2 || (compact >= 2 && C % 32)) return hipErrorInvalidValue;
  const long long total4 = rows * C / 4;
  unsigned g = (unsigned)((total4 + 255) / 256);
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(split_planes_kernel, dim3(g), dim3(256), 0, s, x, y6, rows, C, compact);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// VQ helpers
// ---------------------------------------------------------------------------------------------
// |x|^2 per row (vector_quantize_pytorch.py:42), accumulated in fp64: rounded once to fp32 (out,
// the prefilter's epilogue) and kept in fp64 (x2d, the rescore).  With xr2, also |x - bf16(x)|^2
// (the residual the one-product prefilter vq_prefilter_b1 drops from x).  Thread 0 also zeroes the
// rescore's pair counter (zero_me), so the search issues no memset node when graph-captured.
__global__ void __launch_bounds__(256) row_sqnorm_kernel(const float* __restrict__ x, long long rows, int C,
                                                          float* __restrict__ out, double* __restrict__ x2d,
                                                          float* __restrict__ xr2, unsigned long long* __restrict__ zero_me) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (zero_me && blockIdx.x == 0 && threadIdx.x == 0) *zero_me = 0;
  if (row >= rows) return;
  double s = 0.0, r = 0.0;
  for (int c = lane * 4; c < C; c += 256) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(x + row * C + c);
    s += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const double d = (double)v[k] - (double)bf16_val(bf16_bits(v[k]));
      r += d * d;
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    s += __shfl_xor(s, off, 64);
    r += __shfl_xor(r, off, 64);
  }
  if (lane == 0) {
    out[row] = (float)s;
    if (x2d) x2d[row] = s;
    if (xr2) xr2[row] = (float)r;
  }
}

hipError_t launch_row_sqnorm(const float* x, long long rows, int C, float* out, double* x2d, float* xr2,
                             unsigned long long* zero_me, hipStream_t s) {
  if (C % 4) return hipErrorInvalidValue;
  hipLaunchKernelGGL(row_sqnorm_kernel, dim3((unsigned)std::max<long long>((rows + 3) / 4, 1)), dim3(256), 0, s, x,
                     rows, C, out, x2d, xr2, zero_me);
  return hipGetLastError();
}

// Combine per-tile (distance, index) partials: smallest distance, lowest index on ties.
__global__ void vq_reduce_kernel(const float* __restrict__ pv, const int* __restrict__ pi, int rows, int ntiles,
                                 int32_t* __restrict__ codes) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float bv = __builtin_inff();
  int bi = 0x7fffffff;
  for (int t = lane; t < ntiles; t += 64) {
    const float v = pv[(long long)row * ntiles + t];
    const int i = pi[(long long)row * ntiles + t];
    if (v < bv || (v == bv && i < bi)) { bv = v; bi = i; }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const float ov = __shfl_xor(bv, off, 64);
    const int oi = __shfl_xor(bi, off, 64);
    if (ov < bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
  }
  if (lane == 0) codes[row] = bi;
}

hipError_t launch_vq_reduce(const float* part_val, const int* part_idx, int rows, int ntiles, int32_t* codes,
                            hipStream_t s) {
  hipLaunchKernelGGL(vq_reduce_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, part_val, part_idx, rows,
                     ntiles, codes);
  return hipGetLastError();
}

// VQ search, second half (x6 and bf16 modes).  From the prefilter's per-tile (smallest, second
// smallest, code of smallest) approximate squared distances of a row:
//   best = smallest approximate value; thr = best + 2 * bound (vq_prefilter_cx's bound);
//   a tile is a candidate if its smallest <= thr, and wholly a candidate if its second <= thr.
// One candidate code: it is the exact argmin; done.  Otherwise every candidate code is rescored
// with an fp64 dot product and fp64 norms, smallest exact distance, lowest index on ties (the
// reference's first-index argmax of -dist).
//
// Three launches (round 3), because with the one-product prefilter most rows have 2-10 candidates
// (up to whole 256-code tiles in x6 mode), and evaluating them serially per row left the rescore
// latency-bound (one workgroup per row: 9.9 ms at C3, 4.3 ms at C2):
//   vq_certify_kernel    one wave per row: certifies, or reserves a contiguous block of
//                        (row, code) pairs in the workspace list (a vector atomicAdd on one
//                        counter), rounded up to chunks of kVqChunk with sentinel padding, and
//                        writes the row's candidates there in tile order;
//   vq_pair_eval_kernel  one wave per chunk: x once into registers, then for each listed code
//                        d = (|x|^2 + |e|^2) - 2 x.e in fp64 (|x|^2 and |e|^2 the fp64 sums of
//                        row_sqnorm and of the load-time codebook pass); the chunk's best (d, code);
//   vq_pair_reduce_kernel one wave per listed row: smallest d over its chunks, lowest code on ties.
// (One wave per pair, x re-read for every candidate, moved 1.6x the bytes: 8.2 ms at C3.)
// A row whose candidates would overflow the list is rescored by its own wave in the certify
// kernel (the same fp64 arithmetic), so the result never depends on the list capacity.
constexpr int kMaxVqTiles = 512;
constexpr int kMaxVqDimVec = 16;  // dim <= 16 * 256
constexpr int kVqChunk = 8;       // candidate pairs per vq_pair_eval_kernel work item

__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
__device__ __forceinline__ bool dless(double d, int c, double bd, int bc) { return d < bd || (d == bd && c < bc); }

// One row of dim = 256 nvec floats as lane-strided float4s.  Every load is issued unconditionally
// (index clamped; the extra ones re-read the last float4 and are dropped by the caller), so all of
// them are in flight at once: loads under `if (u < nvec)` went out one round trip at a time.
__device__ __forceinline__ void load_row(f32x4 (&v)[kMaxVqDimVec], const float* __restrict__ row, int nvec, int lane) {
#pragma unroll
  for (int u = 0; u < kMaxVqDimVec; ++u)
    v[u] = *reinterpret_cast<const f32x4*>(row + min(u, nvec - 1) * 256 + lane * 4);
}
// x.e in fp64 over one wave, both rows streamed in quarters (the in-place path of vq_certify_kernel,
// whose 1024-thread workgroups leave 128 VGPRs per lane)
__device__ __forceinline__ double dot_stream_f64(const float* __restrict__ xrow, const float* __restrict__ crow,
                                                 int nvec, int lane) {
  constexpr int H = kMaxVqDimVec / 4;
  double acc = 0;
#pragma nounroll
  for (int h = 0; h < 4; ++h) {
    f32x4 a[H], e[H];
#pragma unroll
    for (int u = 0; u < H; ++u) {
      const int uu = min(h * H + u, nvec - 1);
      a[u] = *reinterpret_cast<const f32x4*>(xrow + uu * 256 + lane * 4);
      e[u] = *reinterpret_cast<const f32x4*>(crow + uu * 256 + lane * 4);
    }
#pragma unroll
    for (int u = 0; u < H; ++u)
      if (h * H + u < nvec)
        acc += (double)a[u][0] * e[u][0] + (double)a[u][1] * e[u][1] + (double)a[u][2] * e[u][2] +
               (double)a[u][3] * e[u][3];
  }
  return wave_sum_f64(acc);
}
// x.e in fp64 over one wave, x held in registers (every lane returns the sum)
__device__ __forceinline__ double dot_f64(const f32x4 (&xr)[kMaxVqDimVec], const float* __restrict__ crow, int nvec,
                                          int lane) {
  f32x4 e[kMaxVqDimVec];
  load_row(e, crow, nvec, lane);
  double acc = 0;
#pragma unroll
  for (int u = 0; u < kMaxVqDimVec; ++u)
    if (u < nvec)
      acc += (double)xr[u][0] * e[u][0] + (double)xr[u][1] * e[u][1] + (double)xr[u][2] * e[u][2] +
             (double)xr[u][3] * e[u][3];
  return wave_sum_f64(acc);
}

constexpr int kCertifyRows = 16;  // rows (waves) per vq_certify_kernel workgroup: one list atomic per workgroup

__global__ void __launch_bounds__(64 * kCertifyRows) vq_certify_kernel(const float* __restrict__ pv, const int* __restrict__ pi,
                                                         const float* __restrict__ pv2, int ntiles, int tile_codes,
                                                         long long rows, const float* __restrict__ x,
                                                         const float* __restrict__ x2, const double* __restrict__ x2d,
                                                         const float* __restrict__ xr2, int dim,
                                                         const float* __restrict__ code,
                                                         const double* __restrict__ e2d, double cx, float emax,
                                                         float e2max, int32_t* __restrict__ codes,
                                                         int2* __restrict__ pairs, long long cap,
                                                         unsigned long long* __restrict__ npairs, int2* __restrict__ row_list,
                                                         int* __restrict__ stats) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __shared__ int s_n[kCertifyRows];
  __shared__ unsigned long long s_base;
  // rows past the end take part in the workgroup's list reservation with nothing to list
  const bool live = (long long)blockIdx.x * kCertifyRows + wave < rows;
  const long long row = live ? (long long)blockIdx.x * kCertifyRows + wave : rows - 1;
  const float* v1p = pv + row * ntiles;
  const float* v2p = pv2 + row * ntiles;
  const int* i1p = pi + row * ntiles;

  // 1. best approximate value.  The bound takes |x|^2 from row_sqnorm (fp64 sum rounded to fp32,
  // within 2^-24 relative), raised by 2^-20 so it is never below the exact value.
  float bv = __builtin_inff();
  int bi = 0x7fffffff;
  for (int t = lane; t < ntiles; t += 64) {
    const float v = v1p[t];
    const int i = i1p[t];
    if (v < bv || (v == bv && i < bi)) { bv = v; bi = i; }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const float ov = __shfl_xor(bv, off, 64);
    const int oi = __shfl_xor(bi, off, 64);
    if (ov < bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
  }
  const double xxb = (double)x2[row] * (1.0 + 0x1p-20);
  // half-width of the prefilter's error: cx |x| (+ max|e| |x_r| for vq_prefilter_b1, whose x_r = x - bf16(x)
  // comes from row_sqnorm, raised like |x|^2), plus the fp32 rounding of (|x|^2 + |e|^2) - 2 x.e
  const double xrb = xr2 ? (double)xr2[row] * (1.0 + 0x1p-20) : 0.0;
  const double bound = 2.0 * (cx * sqrt(xxb) + (double)emax * sqrt(xrb)) + 8.0 * 0x1p-24 * (xxb + (double)e2max);
  const double thr = (double)bv + 2.0 * bound * (1.0 + 1e-6);

  // 2. candidates inside the bound; each lane counts those of its tiles (t = lane + 64 k): single codes
  // (the tile's smallest only) and whole tiles (its second smallest inside the bound too)
  int cnt = 0, nwhole = 0;
  for (int t = lane; t < ntiles; t += 64) {
    const double v1 = v1p[t], v2 = v2p[t];
    if (v1 <= thr) {
      if (v2 <= thr) ++nwhole;
      else ++cnt;
    }
  }
  int pre = cnt;  // inclusive prefix of the single codes over lanes
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int o = __shfl_up(pre, off, 64);
    if (lane >= off) pre += o;
  }
  int wsum = nwhole;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) wsum += __shfl_xor(wsum, off, 64);
  const int nsingle = __shfl(pre, 63, 64);
  const int total = live ? nsingle + wsum * tile_codes : 0;
  // whole chunks (cap is a multiple too); one atomicAdd per workgroup reserves every row's block
  // (an atomic per row on the one counter serialised 150k times at C3)
  const int rtot = total <= 1 ? 0 : (total + kVqChunk - 1) / kVqChunk * kVqChunk;
  if (lane == 0) s_n[wave] = rtot;
  __syncthreads();
  if (threadIdx.x == 0) {
    int sum = 0;
    for (int w = 0; w < kCertifyRows; ++w) sum += s_n[w];
    s_base = sum ? atomicAdd(npairs, (unsigned long long)sum) : 0;
  }
  __syncthreads();
  if (!live) return;
  if (total <= 1) {  // certified (0 only for non-finite input: keep the prefilter's pick)
    if (lane == 0) {
      codes[row] = bi;
      row_list[row] = make_int2(-1, 0);
    }
    return;
  }
  if (stats && lane == 0) {
    atomicAdd(&stats[0], 1);
    atomicAdd(&stats[1], total);
  }
  unsigned long long base = s_base;
  for (int w = 0; w < wave; ++w) base += s_n[w];
  if (base + rtot <= (unsigned long long)cap) {
    // 3a. list the candidates for vq_pair_eval_kernel: the single codes (each lane its own), then
    // the whole tiles, written by the whole wave (one lane writing 256 entries held its workgroup of
    // 16 rows for ~100 us: 1.7 ms at C2)
    long long o = (long long)base + pre - cnt;
    for (int t = lane; t < ntiles; t += 64) {
      const double v1 = v1p[t], v2 = v2p[t];
      if (v1 <= thr && !(v2 <= thr)) pairs[o++] = make_int2((int)row, i1p[t]);  // the counting predicates
    }
    long long ow = (long long)base + nsingle;
    for (int tb = 0; tb < ntiles; tb += 64) {
      const int t = tb + lane;
      const bool whole = t < ntiles && (double)v1p[t] <= thr && (double)v2p[t] <= thr;
      unsigned long long mask = __ballot(whole);
      while (mask) {
        const int k = __builtin_ctzll(mask);
        mask &= mask - 1;
        for (int j = lane; j < tile_codes; j += 64) pairs[ow + j] = make_int2((int)row, (tb + k) * tile_codes + j);
        ow += tile_codes;
      }
    }
    if (lane < rtot - total) pairs[base + total + lane] = make_int2(-1, -1);
    if (lane == 0) row_list[row] = make_int2((int)base, total);
    return;
  }
  // 3b. list full: rescore here, one candidate at a time.  The part of the reserved block that lies
  // inside the list gets sentinels, so vq_pair_eval_kernel never reads an entry this call did not write.
  for (unsigned long long o = base + lane; o < (unsigned long long)cap; o += 64) pairs[o] = make_int2(-1, -1);
  if (lane == 0) row_list[row] = make_int2(-1, 0);
  const int nvec = dim >> 8;
  const float* xrow = x + row * dim;
  double best = __builtin_inf();
  int bc = 0x7fffffff;
  auto eval = [&](int c) {
    const double d = (x2d[row] + e2d[c]) - 2.0 * dot_stream_f64(xrow, code + (long long)c * dim, nvec, lane);
    if (dless(d, c, best, bc)) { best = d; bc = c; }
  };
  for (int t = 0; t < ntiles; ++t) {
    const double v1 = v1p[t], v2 = v2p[t];
    if (!(v1 <= thr)) continue;
    if (v2 <= thr)
      for (int c = t * tile_codes; c < (t + 1) * tile_codes; ++c) eval(c);
    else
      eval(i1p[t]);
  }
  if (lane == 0) codes[row] = bc;
}

__global__ void __launch_bounds__(256) vq_pair_eval_kernel(const int2* __restrict__ pairs,
                                                           const unsigned long long* __restrict__ npairs,
                                                           long long cap, long long rows, int ncodes,
                                                           const float* __restrict__ x,
                                                           const double* __restrict__ x2d, int dim,
                                                           const float* __restrict__ code,
                                                           const double* __restrict__ e2d, double* __restrict__ cdist,
                                                           int* __restrict__ ccode) {
  const int lane = threadIdx.x & 63;
  const long long nch = (long long)min(*npairs, (unsigned long long)cap) / kVqChunk;
  const long long nw = (long long)gridDim.x * 4;
  const int nvec = dim >> 8;
  for (long long q = (long long)blockIdx.x * 4 + (threadIdx.x >> 6); q < nch; q += nw) {
    const int2 my = lane < kVqChunk ? pairs[q * kVqChunk + lane] : make_int2(-1, -1);
    const int row = __shfl(my.x, 0, 64);
    if (row < 0 || row >= rows) continue;  // a chunk of sentinels (overflowed block)
    f32x4 xr[kMaxVqDimVec];
    load_row(xr, x + (long long)row * dim, nvec, lane);
    const double xx = x2d[row];
    double best = __builtin_inf();
    int bc = 0x7fffffff;
    for (int k = 0; k < kVqChunk; ++k) {
      const int r = __shfl(my.x, k, 64), c = __shfl(my.y, k, 64);
      if (r != row || c < 0 || c >= ncodes) continue;  // padding
      const double d = (xx + e2d[c]) - 2.0 * dot_f64(xr, code + (long long)c * dim, nvec, lane);
      if (dless(d, c, best, bc)) { best = d; bc = c; }
    }
    if (lane == 0) {
      cdist[q] = best;
      ccode[q] = bc;
    }
  }
}

__global__ void __launch_bounds__(256) vq_pair_reduce_kernel(const int2* __restrict__ row_list,
                                                             const double* __restrict__ cdist,
                                                             const int* __restrict__ ccode, long long rows,
                                                             int32_t* __restrict__ codes) {
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int2 rl = row_list[row];
  if (rl.x < 0) return;
  const long long q0 = rl.x / kVqChunk;
  const int nq = (rl.y + kVqChunk - 1) / kVqChunk;
  double best = __builtin_inf();
  int bc = 0x7fffffff;
  for (int j = lane; j < nq; j += 64) {
    const double d = cdist[q0 + j];
    const int c = ccode[q0 + j];
    if (dless(d, c, best, bc)) { best = d; bc = c; }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const double od = __shfl_xor(best, off, 64);
    const int oc = __shfl_xor(bc, off, 64);
    if (dless(od, oc, best, bc)) { best = od; bc = oc; }
  }
  if (lane == 0) codes[row] = bc;
}

static bool rescore_args_ok(const VqRescoreArgs& a) {
  return a.ntiles >= 1 && a.ntiles <= kMaxVqTiles && a.dim % 256 == 0 && a.dim <= 256 * kMaxVqDimVec && a.rows >= 0 &&
         a.rows <= (1ll << 31) - 1 && a.cap >= 0 && a.cap <= 0x7fffffffll && a.cap % kVqChunk == 0 && a.pairs && a.cdist && a.ccode && a.row_list &&
         a.npairs && a.x2d && a.e2d;
}

hipError_t launch_vq_certify(const VqRescoreArgs& a, hipStream_t s) {
  if (!rescore_args_ok(a)) return hipErrorInvalidValue;
  if (a.rows == 0) return hipSuccess;
  hipLaunchKernelGGL(vq_certify_kernel, dim3((unsigned)((a.rows + kCertifyRows - 1) / kCertifyRows)),
                     dim3(64 * kCertifyRows), 0, s, a.part_val, a.part_idx, a.part_val2, a.ntiles, a.tile_codes,
                     a.rows, a.x, a.x2, a.x2d, a.xr2, a.dim, a.codebook, a.e2d, a.cx, a.emax, a.e2max, a.codes, a.pairs,
                     a.cap, a.npairs, a.row_list, a.stats);
  return hipGetLastError();
}

hipError_t launch_vq_pair_eval(const VqRescoreArgs& a, hipStream_t s) {
  if (!rescore_args_ok(a)) return hipErrorInvalidValue;
  if (a.rows == 0) return hipSuccess;
  // the pair count is known on the device only: enough waves to cover the list, at most 8 blocks per CU
  const long long eb = std::min<long long>((a.cap / kVqChunk + 3) / 4, 2048);
  hipLaunchKernelGGL(vq_pair_eval_kernel, dim3((unsigned)std::max<long long>(eb, 1)), dim3(256), 0, s, a.pairs,
                     a.npairs, a.cap, a.rows, a.ntiles * a.tile_codes, a.x, a.x2d, a.dim, a.codebook, a.e2d,
                     a.cdist, a.ccode);
  return hipGetLastError();
}

hipError_t launch_vq_pair_reduce(const VqRescoreArgs& a, hipStream_t s) {
  if (!rescore_args_ok(a)) return hipErrorInvalidValue;
  if (a.rows == 0) return hipSuccess;
  hipLaunchKernelGGL(vq_pair_reduce_kernel, dim3((unsigned)((a.rows + 3) / 4)), dim3(256), 0, s, a.row_list, a.cdist,
                     a.ccode, a.rows, a.codes);
  return hipGetLastError();
}

// out[r] = table[idx[r]] (batched_embedding / einx.get_at).  With masked_row >= 0, index -1 reads
// that row (the decode table's project_out(0) row: the reference masks code -1, residual_vq.py:120-127).
// Other negative indices wrap like torch indexing; anything still outside [0, ntable) reads row 0
// and is counted.
__global__ void __launch_bounds__(256) gather_rows_kernel(const float* __restrict__ table, int ntable,
                                                           const int32_t* __restrict__ idx, long long rows, int width,
                                                           float* __restrict__ out, int32_t* n_invalid, int masked_row) {
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int raw = idx[row];
  int i;
  if (raw == -1 && masked_row >= 0) {
    i = masked_row;  // only code -1 reads the masked row
  } else {
    i = raw < 0 ? raw + ntable : raw;
    if (i < 0 || i >= ntable) {
      if (lane == 0 && n_invalid) atomicAdd(n_invalid, 1);
      i = 0;
    }
  }
  const float* src = table + (long long)i * width;
  float* dst = out + row * width;
  for (int c = lane * 4; c < width; c += 256)
    *reinterpret_cast<f32x4*>(dst + c) = *reinterpret_cast<const f32x4*>(src + c);
}

hipError_t launch_gather_rows(const float* table, int ntable, const int32_t* idx, long long rows, int width, float* out,
                              int32_t* n_invalid, int masked_row, hipStream_t s) {
  if (width % 4) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, table, ntable, idx, rows,
                     width, out, n_invalid, masked_row);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// conv_post (C -> 1, kernel k, "same" padding) + tanh (generators.py:141-145).  The input is
// already silu-activated by the previous stage's epilogue.  Block = 256 output samples; the
// input rows they touch are staged once in LDS (row stride 36 floats: conflict-free b128 reads).
// bf: the reference's CUDA autocast (DCX_GEMM_BF16): bf16 operands (input and weights rounded
// while staging, the caller passes the bias rounded), the conv result rounded to bf16, tanh of it
// rounded to bf16.
// ---------------------------------------------------------------------------------------------
template <int C>
__global__ void __launch_bounds__(256) conv_post_tanh_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                              float bias, float* __restrict__ out, int L, int k, int bf) {
  constexpr int LD = C + 4;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int pad = (k - 1) / 2;
  const int rows = 256 + k - 1;
  float* tile = sm;                 // [rows][LD]
  float* ws = sm + rows * LD;       // [k][C]
  const int b = blockIdx.y;
  const int t0 = blockIdx.x * 256;
  const float* xb = x + (long long)b * L * C;
  for (int i = threadIdx.x; i < rows * (C / 4); i += 256) {
    const int r = i / (C / 4), c4 = i % (C / 4);
    const int t = t0 - pad + r;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (t >= 0 && t < L) v = *reinterpret_cast<const f32x4*>(xb + (long long)t * C + c4 * 4);
    if (bf) v = round_bf16x4(v);
    *reinterpret_cast<f32x4*>(tile + r * LD + c4 * 4) = v;
  }
  for (int i = threadIdx.x; i < k * C; i += 256) ws[i] = bf ? bf16_val(bf16_bits(w[i])) : w[i];
  __syncthreads();
  const int t = t0 + threadIdx.x;
  if (t >= L) return;
  float acc = 0.f;
  for (int j = 0; j < k; ++j) {
    const float* xr = tile + (threadIdx.x + j) * LD;
    const float* wr = ws + j * C;
#pragma unroll
    for (int c = 0; c < C; c += 4) {
      const f32x4 xv = *reinterpret_cast<const f32x4*>(xr + c);
      const f32x4 wv = *reinterpret_cast<const f32x4*>(wr + c);
      acc = fmaf(xv.x, wv.x, acc);
      acc = fmaf(xv.y, wv.y, acc);
      acc = fmaf(xv.z, wv.z, acc);
      acc = fmaf(xv.w, wv.w, acc);
    }
  }
  if (bf)
    out[(long long)b * L + t] = bf16_val(bf16_bits(tanhf(bf16_val(bf16_bits(acc + bias)))));
  else
    out[(long long)b * L + t] = tanhf(acc + bias);
}

hipError_t launch_conv_post_tanh(const float* x, const float* w, float bias, float* out, int batch, int L, int C, int k,
                                 int bf16, hipStream_t s) {
  dim3 grid((unsigned)((L + 255) / 256), batch);
  const size_t lds = (size_t)((256 + k - 1) * (C + 4) + k * C) * sizeof(float);
  switch (C) {
    case 32: hipLaunchKernelGGL(conv_post_tanh_kernel<32>, grid, dim3(256), lds, s, x, w, bias, out, L, k, bf16); break;
    case 64: hipLaunchKernelGGL(conv_post_tanh_kernel<64>, grid, dim3(256), lds, s, x, w, bias, out, L, k, bf16); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// [B][R][C] -> [B][C][R] through a 32x33 LDS tile.
// ---------------------------------------------------------------------------------------------
__global__ void transpose_kernel(const float* __restrict__ in, float* __restrict__ out, long long R, long long C) {
  __shared__ float tile[32][33];
  const int b = blockIdx.z;
  const long long r0 = (long long)blockIdx.y * 32, c0 = (long long)blockIdx.x * 32;
  const float* ib = in + (long long)b * R * C;
  float* ob = out + (long long)b * R * C;
  for (int i = threadIdx.y; i < 32; i += 8) {
    const long long r = r0 + i, c = c0 + threadIdx.x;
    if (r < R && c < C) tile[i][threadIdx.x] = ib[r * C + c];
  }
  __syncthreads();
  for (int i = threadIdx.y; i < 32; i += 8) {
    const long long c = c0 + i, r = r0 + threadIdx.x;
    if (r < R && c < C) ob[c * R + r] = tile[threadIdx.x][i];
  }
}

hipError_t launch_transpose(const float* in, float* out, int batch, long long rows, long long cols, hipStream_t s) {
  dim3 grid((unsigned)((cols + 31) / 32), (unsigned)((rows + 31) / 32), batch);
  hipLaunchKernelGGL(transpose_kernel, grid, dim3(32, 8), 0, s, in, out, rows, cols);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Sample-rate conversion by up / down (the reference resamples with librosa.resample on input
// audio at another rate: distil_codec.py:108-110, 676; meldataset.py:18-20).  Polyphase FIR in the
// form of scipy.signal.resample_poly (upfirdn of the zero-stuffed input, h pre-padded, output
// window starting at `pre`):
//   y[b][i] = sum_m h[t - up * m] * x[b][m],   t = (i + pre) * down,   0 <= t - up * m < hlen, 0 <= m < n_in
// One thread per output sample, fp64 taps and accumulation (20-60 taps per output, the work is
// tiny next to the HBM traffic), fp32 output.
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) resample_poly_kernel(const float* __restrict__ x, long long n_in, long long xs,
                                                            const double* __restrict__ h, int hlen, int up, int down,
                                                            long long pre, float* __restrict__ y, long long n_out,
                                                            long long ys) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n_out) return;
  const float* __restrict__ xb = x + (long long)blockIdx.y * xs;
  const long long t = (i + pre) * down;
  const long long m_hi = min(t / up, n_in - 1);
  const long long m_lo = t - (hlen - 1) <= 0 ? 0 : (t - (hlen - 1) + up - 1) / up;
  double acc = 0.0;
  for (long long m = m_lo; m <= m_hi; ++m) acc = fma(h[t - up * m], (double)xb[m], acc);
  y[(long long)blockIdx.y * ys + i] = (float)acc;
}

hipError_t launch_resample_poly(const float* x, int batch, long long n_in, long long xs, const double* h, int hlen,
                                int up, int down, long long pre, float* y, long long n_out, long long ys,
                                hipStream_t s) {
  const dim3 grid((unsigned)((n_out + 255) / 256), (unsigned)batch);
  hipLaunchKernelGGL(resample_poly_kernel, grid, dim3(256), 0, s, x, n_in, xs, h, hlen, up, down, pre, y, n_out, ys);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Codebook for the bf16-mode VQ prefilter (vq_prefilter_bk): the hi and mid planes of the x6
// codebook ([CD/16][NC][2 halves][3 planes][8], ConvParams::w6 layout) repacked per K32 step as
// [CD/32][NC][8 pieces][8] bf16, piece = (chunk half cc, channel half hh, plane hi/mid) =
// (cc * 2 + hh) * 2 + pl: 128 contiguous bytes per code per step.  One thread per 16-byte piece.
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) repack_codebook_bk_kernel(const unsigned short* __restrict__ cb6, int ncodes,
                                                                 long long pieces, unsigned short* __restrict__ out) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= pieces) return;
  const int pc = (int)(i & 7);
  const long long sn = i >> 3;  // step * ncodes + code
  const long long st = sn / ncodes, n = sn - st * ncodes;
  const int cc = pc >> 2, hh = (pc >> 1) & 1, pl = pc & 1;
  const unsigned short* src = cb6 + ((2 * st + cc) * ncodes + n) * 48 + hh * 24 + pl * 8;
  *reinterpret_cast<uint4*>(out + i * 8) = *reinterpret_cast<const uint4*>(src);
}

hipError_t launch_repack_codebook_bk(const unsigned short* cb6, int ncodes, int dim, unsigned short* out,
                                     hipStream_t s) {
  if (dim % 32) return hipErrorInvalidValue;
  const long long pieces = (long long)(dim / 32) * ncodes * 8;
  hipLaunchKernelGGL(repack_codebook_bk_kernel, dim3((unsigned)((pieces + 255) / 256)), dim3(256), 0, s, cb6, ncodes,
                     pieces, out);
  return hipGetLastError();
}

}  // namespace dcx

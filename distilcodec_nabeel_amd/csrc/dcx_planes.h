// Device helpers for the x6 "planes" representation: an fp32 value x is stored as three bf16
// (hi, mid, lo), round-to-nearest-even each: hi = bf16(x), mid = bf16(x - hi), lo = bf16(x - hi - mid).
// Both differences are exact in fp32 and |x - (hi + mid + lo)| <= 2^-27 |x|.  Layout of a planes
// tensor [rows][C]: per row, per group of 8 channels, 24 bf16 = hi[8] mid[8] lo[8].
#pragma once
#include <hip/hip_runtime.h>

namespace dcx {

typedef short s16x4p __attribute__((ext_vector_type(4)));

// RNE to bf16: v_cvt_pk_bf16_f32 (hipcc pairs adjacent conversions into one instruction); the
// same bits as (u + 0x7FFF + ((u >> 16) & 1)) >> 16 for every non-NaN input, NaN stays NaN.
__device__ __forceinline__ unsigned short bf16_bits(float x) { return __builtin_bit_cast(unsigned short, (__bf16)x); }
__device__ __forceinline__ float bf16_val(unsigned short b) { return __uint_as_float((unsigned)b << 16); }

// four fp32 values rounded to bf16 values (the bf16 mode's torch.autocast rounding points)
typedef float f32x4p __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4p round_bf16x4(f32x4p v) {
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = bf16_val(bf16_bits(v[e]));
  return v;
}

__device__ __forceinline__ void split3(float x, unsigned short& h, unsigned short& m, unsigned short& l) {
  h = bf16_bits(x);
  const float r1 = x - bf16_val(h);
  m = bf16_bits(r1);
  const float r2 = r1 - bf16_val(m);
  l = bf16_bits(r2);
}

// Element (row, c) of a planes tensor with C channels: offset of its hi value (mid +8, lo +16).
__device__ __forceinline__ long long plane_off(long long row, int C, int c) {
  return row * (long long)C * 3 + (c >> 3) * 24 + (c & 7);
}

// Store one value (scalar path, e.g. one MFMA accumulator element per lane).
__device__ __forceinline__ void store_planes1(unsigned short* base, long long row, int C, int c, float v) {
  unsigned short h, m, l;
  split3(v, h, m, l);
  unsigned short* d = base + plane_off(row, C, c);
  d[0] = h;
  d[8] = m;
  d[16] = l;
}

// Store 4 consecutive channels c..c+3 (c % 4 == 0) of one row: three 8-byte stores.
__device__ __forceinline__ void store_planes4(unsigned short* base, long long row, int C, int c, float a, float b,
                                              float cc, float d) {
  s16x4p hv, mv, lv;
  const float v[4] = {a, b, cc, d};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    unsigned short h, m, l;
    split3(v[e], h, m, l);
    hv[e] = (short)h;
    mv[e] = (short)m;
    lv[e] = (short)l;
  }
  unsigned short* dst = base + plane_off(row, C, c);
  *reinterpret_cast<s16x4p*>(dst) = hv;
  *reinterpret_cast<s16x4p*>(dst + 8) = mv;
  *reinterpret_cast<s16x4p*>(dst + 16) = lv;
}

// Compact bf16 layout (DCX_GEMM_BF16 mode, tensors whose consumers read only the hi plane):
// [rows][C] bf16 = hi only, 2 bytes per element.  Store 4 consecutive channels c..c+3 (c % 4 == 0).
__device__ __forceinline__ void store_bf16x4(unsigned short* base, long long row, int C, int c, float a, float b,
                                             float cc, float d) {
  s16x4p hv;
  hv[0] = (short)bf16_bits(a);
  hv[1] = (short)bf16_bits(b);
  hv[2] = (short)bf16_bits(cc);
  hv[3] = (short)bf16_bits(d);
  *reinterpret_cast<s16x4p*>(base + row * (long long)C + c) = hv;
}

// "hm" layout (x6-mode x_pjt_in, read only by vq_prefilter_dm): the hi and mid planes per 32
// channels as [rows][C/32][8 pieces][8] bf16, piece = ((c >> 3) & 3) * 2 + plane (4 B per element),
// the per-K32 layout of launch_repack_codebook_bk.  Store 4 consecutive channels c..c+3 (c % 4 == 0).
__device__ __forceinline__ void store_hm4(unsigned short* base, long long row, int C, int c, float a, float b,
                                          float cc, float d) {
  s16x4p hv, mv;
  const float v[4] = {a, b, cc, d};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    unsigned short h, m, l;
    split3(v[e], h, m, l);
    hv[e] = (short)h;
    mv[e] = (short)m;
  }
  unsigned short* dst = base + row * (long long)C * 2 + (c >> 5) * 64 + ((c >> 3) & 3) * 16 + (c & 7);
  *reinterpret_cast<s16x4p*>(dst) = hv;
  *reinterpret_cast<s16x4p*>(dst + 8) = mv;
}

// 8 consecutive channels c..c+7 (c % 8 == 0) of one row: one 16-byte store per plane.
typedef short s16x8p __attribute__((ext_vector_type(8)));
__device__ __forceinline__ void store_planes8(unsigned short* base, long long row, int C, int c, const float (&v)[8]) {
  s16x8p hv, mv, lv;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    unsigned short h, m, l;
    split3(v[e], h, m, l);
    hv[e] = (short)h;
    mv[e] = (short)m;
    lv[e] = (short)l;
  }
  unsigned short* dst = base + plane_off(row, C, c);
  *reinterpret_cast<s16x8p*>(dst) = hv;
  *reinterpret_cast<s16x8p*>(dst + 8) = mv;
  *reinterpret_cast<s16x8p*>(dst + 16) = lv;
}

__device__ __forceinline__ void store_bf16x8(unsigned short* base, long long row, int C, int c, const float (&v)[8]) {
  s16x8p hv;
#pragma unroll
  for (int e = 0; e < 8; ++e) hv[e] = (short)bf16_bits(v[e]);
  *reinterpret_cast<s16x8p*>(base + row * (long long)C + c) = hv;
}

__device__ __forceinline__ void store_hm8(unsigned short* base, long long row, int C, int c, const float (&v)[8]) {
  s16x8p hv, mv;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    unsigned short h, m, l;
    split3(v[e], h, m, l);
    hv[e] = (short)h;
    mv[e] = (short)m;
  }
  unsigned short* dst = base + row * (long long)C * 2 + (c >> 5) * 64 + ((c >> 3) & 3) * 16;
  *reinterpret_cast<s16x8p*>(dst) = hv;
  *reinterpret_cast<s16x8p*>(dst + 8) = mv;
}

// "h2" layout (the h3 arithmetic of conv_gemm_x3dq): x as two fp16 values, h = fp16(x) (RNE) and
// l = fp16(x - h) (x - h is exact in fp32), 22 significant bits for |x| in [2^-3, 2^16) (l is exact
// to 2^-25 absolute where x - h is subnormal).  Producers scale x by 2^h2_shift(bound) first
// (dcx_kernels.h), so the range is only left when a bound is violated: |x| > 65504 then saturates
// to +-65504 with l = 0 (finite; the producer raises RANGE_OVER), NaN stays NaN.  The hm layout's
// order: [rows][C/32][8 pieces][8] fp16, piece = ((c >> 3) & 3) * 2 + plane, 4 B per element.
// SAT = false (split2h_nc): no saturation, for producers whose scale comes from a rigorous bound
// and that report a violated one themselves (the conv epilogues and pair-kernel images: |x| <= 2^15
// for finite inputs; past it h and l go inf / NaN and the producer has raised the range flag).  The
// three VALU of the clamp were a tenth of those epilogues' per-element work.
template <bool SAT = true>
__device__ __forceinline__ void split2h(float x, unsigned short& h, unsigned short& l) {
  const float xs = !SAT ? x : fabsf(x) > 65504.f ? copysignf(65504.f, x) : x;  // NaN stays NaN
  const _Float16 hh = (_Float16)xs;
  h = __builtin_bit_cast(unsigned short, hh);
  l = __builtin_bit_cast(unsigned short, (_Float16)(xs - (float)hh));
}
__device__ __forceinline__ void split2h_nc(float x, unsigned short& h, unsigned short& l) { split2h<false>(x, h, l); }
// sc: the producer's power-of-two range scale (exact)
template <bool SAT = true>
__device__ __forceinline__ void store_h2_4(unsigned short* base, long long row, int C, int c, float a, float b,
                                           float cc, float d, float sc = 1.0f) {
  s16x4p hv, lv;
  const float v[4] = {a * sc, b * sc, cc * sc, d * sc};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    unsigned short h, l;
    split2h<SAT>(v[e], h, l);
    hv[e] = (short)h;
    lv[e] = (short)l;
  }
  unsigned short* dst = base + row * (long long)C * 2 + (c >> 5) * 64 + ((c >> 3) & 3) * 16 + (c & 7);
  *reinterpret_cast<s16x4p*>(dst) = hv;
  *reinterpret_cast<s16x4p*>(dst + 8) = lv;
}
template <bool SAT = true>
__device__ __forceinline__ void store_h2_8(unsigned short* base, long long row, int C, int c, const float (&v)[8],
                                           float sc = 1.0f) {
  s16x8p hv, lv;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    unsigned short h, l;
    split2h<SAT>(v[e] * sc, h, l);
    hv[e] = (short)h;
    lv[e] = (short)l;
  }
  unsigned short* dst = base + row * (long long)C * 2 + (c >> 5) * 64 + ((c >> 3) & 3) * 16;
  *reinterpret_cast<s16x8p*>(dst) = hv;
  *reinterpret_cast<s16x8p*>(dst + 8) = lv;
}

}  // namespace dcx

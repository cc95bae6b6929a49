// Fused ResBlock1 pairs for the small-channel generator stages (C = 32 and 64).
//
// ResBlock1 (convnext_utils.py:106-113) runs three pairs
//     xt = c2(silu(c1(silu(x))));  x = xt + x
// with c1 dilated (k, d) and c2 undilated (k, 1); ParralelBlock (:137-138) averages three such
// ResBlocks (k = 3 / 7 / 11).  At C = 32 / 64 each conv has K = k * C <= 704, so one conv per launch
// (conv_gemm_x6w4f / x6pf) spent its time staging and splitting its fp32 input and round-tripping
// silu(c1) through HBM rather than in MFMAs (0.30 / 0.47 MFMA busy, 7 SALU + 8 VALU per MFMA).
//
// conv_res_pair runs one pair of all three ResBlocks per launch.  A workgroup owns R output rows of
// one clip and, for each ResBlock in turn:
//   1. S image: silu(state) as x6 planes in LDS, rows [r0 - 8 - 32, r0 + R + 8 + 32) (zero outside
//      the clip = the conv's zero padding), prefetched into registers during the previous c2;
//   2. c1 over the R + 16 rows [r0 - 8, r0 + R + 8) (the c2 halo, (k - 1) / 2 <= 8);
//   3. T image: silu(c1 + b1) planes written over S (zero outside the clip);
//   4. c2 over the R output rows, epilogue state + c2 + b2 to the next state buffer (or, for the
//      last pair, into the ParallelBlock mean, kept in registers across the three ResBlocks in
//      ResBlock order: m = v0; m += v1; m = (m + v2) / 3, then silu(mean) to the next ConvT input).
// The halo makes in-place updates race, so each pair writes a buffer other than the one it reads.
//
// Arithmetic: the x6 products of conv_gemm_x6dq (v_mfma_f32_16x16x32_bf16, the K dimension split
// into (term, channel)), with the weights as the A operand and the activations as B, so each lane's
// accumulator holds 4 consecutive channels of one time row: T-image writes are 8-byte plane stores
// and epilogue loads / stores are 16-byte fp32 accesses.
//   W{h',m'} . X{h,m} = hh' + mm',  W{h',m'} . X{m,h} = mh' + hm',  W{h',l'} . X{l,h} = lh' + hl'.
// Weights stream through a 2-slot LDS ring, one tap (C * C * 6 bytes) per step, prefetched one
// step ahead into registers; the step sequence runs on across convs, ResBlocks and tiles.
// LDS images: piece-major and row-linear, byte ((chunk * 6 + piece) * NS + row) * 16 (piece = half * 3 +
// plane, NS the image rows, a multiple of 16): every ds_read_b128 of 16 consecutive rows of one piece
// is conflict-free at any tap offset, and a tap's row offset is one add per read set (round 5; the
// round-2 layout of 16-row blocks cost ~6 VALU per row block and tap in address arithmetic).  The
// weight slot is the global tap slice [chunk][Cout][96 B] copied as is.
#include <algorithm>
#include <cstdio>

#include "dcx_kernels.h"
#include "dcx_planes.h"

namespace dcx {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float rp_silu(float v) { return v * __builtin_amdgcn_rcpf(1.0f + __expf(-v)); }
// barrier that leaves global loads in flight (only LDS traffic is drained)
__device__ __forceinline__ void rp_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
typedef __attribute__((address_space(3))) void* rp_lds_t;
// retire this wave's weight pieces: all but the n youngest vector-memory ops (the prefetch loads
// issued after the pieces) done
__device__ __forceinline__ void rp_wait(int n) {
#define RP_W(k) \
  case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
  switch (n) {
    RP_W(1) RP_W(2) RP_W(3) RP_W(4) RP_W(5) RP_W(6) RP_W(7) RP_W(8) RP_W(9) RP_W(10) RP_W(11) RP_W(12)
    RP_W(13) RP_W(14) RP_W(15) RP_W(16) RP_W(17) RP_W(18) RP_W(19) RP_W(20) RP_W(21) RP_W(22) RP_W(23) RP_W(24)
    RP_W(25) RP_W(26) RP_W(27) RP_W(28) RP_W(29) RP_W(30) RP_W(31) RP_W(32)
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // n > 32 waits for more: always safe
  }
#undef RP_W
}

#ifdef RP_DIAG_STAMPS
// Diagnostic build only: shader-clock sums per phase of conv_res_pair (wave 0 of every workgroup):
// [0] c1 steps, [1] T image, [2] c2 steps, [3] epilogue, [4] next S image, [5] member-tiles,
// [6] c1 steps counted, [7] c2 steps counted, [8] c1 step MFMA phases, [9] c1 step barrier waits.
__device__ unsigned long long g_rp_diag[32];  // [C == 64][16]
#define RP_T(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#else
#define RP_T(v)
#endif

// output rows per tile: 496 / 176 (C = 32 / 64) by default; the launcher takes fewer rows per tile
// when a launch has too few tiles for the CUs (small batches: the C5 streaming hop), same bits
template <int C>
constexpr int kRpRows = C == 32 ? 496 : 176;
template <int C, int RR = kRpRows<C>>
struct RpGeom {
  static constexpr int R = RR;
  static constexpr int M1 = R + 16;              // c1 rows: [r0 - 8, r0 + R + 8)
  static constexpr int H1 = 32;                  // largest c1 reach (k - 1) / 2 * d
  static constexpr int NS = M1 + 2 * H1;         // S image rows
  static constexpr int NCH = C / 16;             // K16 chunks per tap
  static constexpr int WC = C / 32, WR = 8 / WC; // waves: WR row groups x WC column halves (32 ch)
  static constexpr int NB1 = M1 / 16, RB1 = NB1 / WR;
  static constexpr int NB2 = R / 16, RB2 = (NB2 + WR - 1) / WR;
  static constexpr int PS = NS * 16;             // bytes per piece of one chunk (image layout below)
  static constexpr int IMG = NCH * 6 * PS;       // S image bytes (T reuses its start)
  static constexpr int TPS = C == 32 ? 2 : 1;    // taps per step (weight slot)
  static constexpr int WTAP = C * C * 6;         // one tap of weights
  static constexpr int WSLOT = TPS * WTAP;
  static constexpr int G8 = C / 8;               // 8-channel groups per row
  static constexpr int NIT = (NS * G8 + 511) / 512;
  static constexpr int WP = WSLOT / 1024, WPW = (WP + 7) / 8;  // DMA pieces per slot, per wave
  static constexpr int LDS = IMG + 2 * WSLOT + 2 * kMaxGroup * C * 4;
  static_assert(NB1 % WR == 0 && RB1 == RB2, "row blocks per wave");
  static_assert(WSLOT % 1024 == 0 && LDS <= 160 * 1024, "LDS");
};

// conv_res_pair_h3's geometry: RpGeom's rows and wave layout, h3 images (8 pieces of 16 B per row
// and 32-channel chunk: 4 B per element), so taller tiles fit the LDS
template <int C>
constexpr int kRp3Rows = C == 32 ? 624 : 240;
template <int C, int RR = kRp3Rows<C>>
struct RpGeom3 {
  static constexpr int R = RR;
  static constexpr int M1 = R + 16, H1 = 32, NS = M1 + 2 * H1;
  static constexpr int WC = C / 32, WR = 8 / WC;
  static constexpr int NB1 = M1 / 16, RB1 = NB1 / WR;
  static constexpr int NB2 = R / 16, RB2 = (NB2 + WR - 1) / WR;
  static constexpr int PS = NS * 16;
  static constexpr int NCH = C / 32;            // K32 chunks per tap
  static constexpr int IMG = NCH * 8 * PS;      // S image bytes (T reuses it)
  static constexpr int WTAP = C * C * 4;        // one tap of h3 weights (bytes)
  static constexpr int G8 = C / 8;
  static constexpr int NIT = (NS * G8 + 511) / 512;
  static_assert(NB1 % WR == 0 && RB1 == RB2, "row blocks per wave");
  static_assert(IMG + 2 * kMaxGroup * C * 4 <= 160 * 1024, "LDS");
};

}  // namespace

template <int C, bool MEAN, int RR = kRpRows<C>>
__global__ void __launch_bounds__(512, 1) conv_res_pair(const ResPairParams p) {
  using G = RpGeom<C, RR>;
  constexpr int R = G::R, NCH = G::NCH, WR = G::WR, RB = G::RB1, PS = G::PS, IMG = G::IMG, TPS = G::TPS;
  constexpr int WTAP = G::WTAP, WSLOT = G::WSLOT, G8 = G::G8, NIT = G::NIT, WP = G::WP, WPW = G::WPW, NS = G::NS;
  __shared__ __attribute__((aligned(16))) char lds[G::LDS];
  float* const bias_lds = reinterpret_cast<float*>(lds + IMG + 2 * WSLOT);  // [conv][member][C]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wc = wave % G::WC, wr = wave / G::WC;
  const int l15 = lane & 15, hf = (lane >> 4) & 1, t = lane >> 5;
  const int L = p.L, nmem = p.nmem;
  const int ntl = (L + R - 1) / R;
  const int total = ntl * p.batch;

  // ---- weight ring: LDS-DMA of a step's taps (lane-linear 1 KiB pieces, no staging registers);
  // taps past the conv's last read zeros (outside the buffer descriptor) and are never used ----
  auto issue_w = [&](int m, int conv, int step, int slot) {
#ifdef RP_DIAG_NODMA  // timing build: weights never refilled after the prologue (wrong results)
    if (step > 0 || conv > 0 || m > 0) return;
#endif
    const int k = p.taps[m], j0 = step * TPS;
    const unsigned short* w = (conv ? p.w2[m] : p.w1[m]) + (long long)j0 * (WTAP / 2);
    const __amdgpu_buffer_rsrc_t rw =
        __builtin_amdgcn_make_buffer_rsrc((void*)w, 0, min(TPS, k - j0) * WTAP, 0x00020000);
#pragma unroll
    for (int i = 0; i < WPW; ++i) {
      const int piece = wave + 8 * i;
      if (WP % 8 == 0 || piece < WP)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (rp_lds_t)(lds + IMG + slot * WSLOT + piece * 1024), 16,
                                                 piece * 1024 + lane * 16, 0, 0, 0);
    }
    asm volatile("" ::: "memory");  // later loads stay younger than the pieces (rp_wait counts them)
  };

  // ---- S image fill: state rows -> registers (issue) -> silu, planes, LDS (commit) ----
  f32x4 pf[NIT][2];
  auto issue_fill_item = [&](const float* src, int r0, int k) {
    const int it = min(tid + 512 * k, NS * G8 - 1);  // unconditional (rp_wait counts the loads)
    const int s = ((it >> 3) / G8) * 8 + (it & 7), g8 = (it >> 3) % G8;
    const int a = min(max(r0 - 8 - G::H1 + s, 0), L - 1);
    const f32x4* q = reinterpret_cast<const f32x4*>(src + (long long)a * C + g8 * 8);
    pf[k][0] = q[0];
    pf[k][1] = q[1];
  };
  auto commit_fill = [&](int r0) {
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
      const int it = tid + 512 * k;
      if (!(NIT * 512 == NS * G8 || it < NS * G8)) continue;
      const int s = ((it >> 3) / G8) * 8 + (it & 7), g8 = (it >> 3) % G8;
      const int a = r0 - 8 - G::H1 + s;
      const bool ok = a >= 0 && a < L;
      s16x8 hv, mv, lv;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float sv = rp_silu(pf[k][e >> 2][e & 3]);
        const float v = ok ? sv : 0.f;
        unsigned short h, m, l;
        split3(v, h, m, l);
        hv[e] = (short)h;
        mv[e] = (short)m;
        lv[e] = (short)l;
      }
      char* d = lds + ((g8 >> 1) * 6 + (g8 & 1) * 3) * PS + s * 16;
      *reinterpret_cast<s16x8*>(d) = hv;
      *reinterpret_cast<s16x8*>(d + PS) = mv;
      *reinterpret_cast<s16x8*>(d + 2 * PS) = lv;
    }
  };

  // ---- one step: the step's taps, every chunk, rows of this wave, its 2 column blocks.  hook(i)
  // runs after row block i of the first tap (global loads spread between the MFMAs) ----
  // lane parts of the three activation reads (piece, row within the 16-row block); a tap adds its
  // wave-uniform row offset once, and row block / chunk offsets are instruction immediates
  const int pk0 = ((hf * 3 + t) * NS + l15) * 16, pk1 = ((hf * 3 + (t ? 0 : 1)) * NS + l15) * 16;
  const int pk2 = ((hf * 3 + (t ? 0 : 2)) * NS + l15) * 16;
  auto mfma_step = [&](f32x4 (&acc)[RB][2], int slot, int ntaps, int row0, int rstep, int nrb, auto hook) {
#pragma unroll
    for (int u = 0; u < TPS; ++u) {
      if (u >= ntaps) break;
      const char* wb = lds + IMG + slot * WSLOT + u * WTAP;
      s16x8 wf[NCH][2][2];
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          const char* w = wb + (ch * C + (2 * wc + cb) * 16 + l15) * 96 + hf * 48;
          wf[ch][cb][0] = *reinterpret_cast<const s16x8*>(w + t * 16);        // {h', m'}
          wf[ch][cb][1] = *reinterpret_cast<const s16x8*>(w + (t ? 32 : 0));  // {h', l'}
        }
      const int rowoff = row0 + u * rstep;
      const int tb = (wr * 16 + rowoff) * 16;
      const char *xb0 = lds + pk0 + tb, *xb1 = lds + pk1 + tb, *xb2 = lds + pk2 + tb;
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < RB; ++i) {
        if (i < nrb) {
          const int io = (WR * 16 * i) * 16;
#pragma unroll
          for (int ch = 0; ch < NCH; ++ch) {
            const s16x8 x2 = *reinterpret_cast<const s16x8*>(xb2 + io + ch * 6 * PS);
            const s16x8 x1 = *reinterpret_cast<const s16x8*>(xb1 + io + ch * 6 * PS);
            const s16x8 x0 = *reinterpret_cast<const s16x8*>(xb0 + io + ch * 6 * PS);
#pragma unroll
            for (int cb = 0; cb < 2; ++cb) {
              acc[i][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wf[ch][cb][1]),
                                                                   __builtin_bit_cast(bf16x8, x2), acc[i][cb], 0, 0, 0);
              acc[i][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wf[ch][cb][0]),
                                                                   __builtin_bit_cast(bf16x8, x1), acc[i][cb], 0, 0, 0);
              acc[i][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wf[ch][cb][0]),
                                                                   __builtin_bit_cast(bf16x8, x0), acc[i][cb], 0, 0, 0);
            }
          }
        }
        if (u == 0) hook(i);
      }
      __builtin_amdgcn_s_setprio(0);
    }
  };
  auto no_hook = [](int) {};

  // rows of c2 this wave owns
  const int nrb2 = min(RB, (G::NB2 - wr + WR - 1) / WR);
  int tile = blockIdx.x;
  if (tile >= total) return;  // whole workgroup, before any barrier
  int b = tile / ntl, r0 = (tile - b * ntl) * R;
  // prologue: biases, first ResBlock's S image and first weight step
  if (tid < 2 * nmem * C) {
    const int conv = tid / (nmem * C), m = (tid / C) % nmem, c = tid % C;
    bias_lds[(conv * kMaxGroup + m) * C + c] = (conv ? p.b2[m] : p.b1[m])[c];
  }
  issue_w(0, 0, 0, 0);
#pragma unroll
  for (int k = 0; k < NIT; ++k) issue_fill_item(p.src[0] + (long long)b * p.bstride, r0, k);
  commit_fill(r0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  rp_barrier();
  int slot = 0;
  f32x4 macc[MEAN ? RB : 1][2];
#ifdef RP_DIAG_STAMPS
  unsigned long long dg[16] = {};
#endif
  for (;;) {
    const int next_tile = tile + gridDim.x;
    const bool more = next_tile < total;
    const int nb = more ? next_tile / ntl : 0, nr0 = more ? (next_tile - nb * ntl) * R : 0;
    for (int m = 0; m < nmem; ++m) {
      const int k = p.taps[m], hk = (k - 1) >> 1, d = p.dil[m];
      const int nst = (k + TPS - 1) / TPS;  // steps per conv
      const long long cb0 = (long long)b * p.bstride;
      const bool last_m = m + 1 == nmem;
      const bool has_next = !last_m || more;
      f32x4 acc[RB][2];
      RP_T(ta);
      // ---- c1 over rows [r0 - 8, r0 + R + 8) from the S image
#pragma unroll
      for (int i = 0; i < RB; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int j = 0; j < nst; ++j) {
        if (j + 1 < nst) issue_w(m, 0, j + 1, slot ^ 1);
        else issue_w(m, 1, 0, slot ^ 1);
        RP_T(s1);
        mfma_step(acc, slot, min(TPS, k - j * TPS), G::H1 + (j * TPS - hk) * d, d, RB, no_hook);
        RP_T(s2);
#ifndef RP_DIAG_NOWAIT  // timing build: the next slot's pieces are not waited for (wrong results)
        rp_wait(0);
#endif
        rp_barrier();
#ifdef RP_DIAG_STAMPS
        {
          RP_T(s3);
          dg[8] += s2 - s1;
          dg[9] += s3 - s2;
        }
#endif
        slot ^= 1;
      }
      RP_T(tb);
      // ---- T image: silu(c1 + b1) planes over the S image (zero outside the clip)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const int c0 = (2 * wc + cb) * 16 + 4 * (lane >> 4);
        const f32x4 bias = *reinterpret_cast<const f32x4*>(bias_lds + m * C + c0);
#pragma unroll
        for (int i = 0; i < RB; ++i) {
          const int ir = (wr + WR * i) * 16 + l15, a = r0 - 8 + ir;
          const bool ok = a >= 0 && a < L;
          s16x4 hv, mv, lv;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float sv = rp_silu(acc[i][cb][e] + bias[e]);
            const float v = ok ? sv : 0.f;
            unsigned short h, mm, l;
            split3(v, h, mm, l);
            hv[e] = (short)h;
            mv[e] = (short)mm;
            lv[e] = (short)l;
          }
          char* dst = lds + ((c0 >> 4) * 6 + ((c0 >> 3) & 1) * 3) * PS + ir * 16 + (c0 & 7) * 2;
          *reinterpret_cast<s16x4*>(dst) = hv;
          *reinterpret_cast<s16x4*>(dst + PS) = mv;
          *reinterpret_cast<s16x4*>(dst + 2 * PS) = lv;
        }
      }
      rp_barrier();
      RP_T(tc);
      // ---- c2 over rows [r0, r0 + R) from the T image.  Step 0 loads the residual rows, step 1 (or
      // 0) the next S image's rows (this tile's next ResBlock, or the next tile's first), one row
      // block's share between the MFMAs of each, after the step's weight pieces.  The two steps are
      // peeled out of the loop: a load pending across the loop's back edge made hipcc wait for it.
#pragma unroll
      for (int i = 0; i < RB; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      const float* nsrc = !last_m ? p.src[m + 1] + cb0 : p.src[0] + (long long)nb * p.bstride;
      const int nsr0 = !last_m ? r0 : nr0;
      const int jpf = nst > 1 ? 1 : 0;
      f32x4 res[RB][2];
      auto res_hook = [&](int i) {
        const int q = min(r0 + (wr + WR * i) * 16 + l15, L - 1);
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          const int c0 = (2 * wc + cb) * 16 + 4 * (lane >> 4);
          res[i][cb] = *reinterpret_cast<const f32x4*>(p.src[m] + cb0 + (long long)q * C + c0);
        }
      };
      auto pf_hook = [&](int i) {
        if (!has_next) return;
#pragma unroll
        for (int kk = NIT * i / RB; kk < NIT * (i + 1) / RB; ++kk) issue_fill_item(nsrc, nsr0, kk);
      };
      auto both_hook = [&](int i) {
        res_hook(i);
        pf_hook(i);
      };
      auto c2_issue_w = [&](int j) {
        if (j + 1 < nst) issue_w(m, 1, j + 1, slot ^ 1);
        else if (has_next) issue_w(last_m ? 0 : m + 1, 0, 0, slot ^ 1);
      };
      const int npf = has_next ? 2 * NIT : 0;
      c2_issue_w(0);
      if (jpf == 0) {
        mfma_step(acc, slot, min(TPS, k), 8 - hk, 1, nrb2, both_hook);
        rp_wait(2 * RB + npf);
      } else {
        mfma_step(acc, slot, TPS, 8 - hk, 1, nrb2, res_hook);
        rp_wait(2 * RB);
        rp_barrier();
        slot ^= 1;
        c2_issue_w(1);
        mfma_step(acc, slot, min(TPS, k - TPS), 8 + TPS - hk, 1, nrb2, pf_hook);
        rp_wait(npf);
      }
      rp_barrier();
      slot ^= 1;
      for (int j = jpf + 1; j < nst; ++j) {
        c2_issue_w(j);
        mfma_step(acc, slot, min(TPS, k - j * TPS), 8 + j * TPS - hk, 1, nrb2, no_hook);
#ifndef RP_DIAG_NOWAIT
        rp_wait(0);
#endif
        rp_barrier();
        slot ^= 1;
      }
      RP_T(te);
      // ---- epilogue: state + c2 + b2 (rows past the clip end are dropped)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const int c0 = (2 * wc + cb) * 16 + 4 * (lane >> 4);
        const f32x4 bias = *reinterpret_cast<const f32x4*>(bias_lds + (kMaxGroup + m) * C + c0);
#pragma unroll
        for (int i = 0; i < RB; ++i) {
          if (i >= nrb2) break;
          const int q = r0 + (wr + WR * i) * 16 + l15;
          const f32x4 v = res[i][cb] + (acc[i][cb] + bias);
          if constexpr (!MEAN) {
            if (q < L) *reinterpret_cast<f32x4*>(p.dst[m] + cb0 + (long long)q * C + c0) = v;
          } else if (m == 0) {
            macc[i][cb] = v;
          } else if (!last_m) {
            macc[i][cb] = macc[i][cb] + v;
          } else {
            const f32x4 mv = (macc[i][cb] + v) / 3.0f;
            f32x4 sv;
#pragma unroll
            for (int e = 0; e < 4; ++e) sv[e] = rp_silu(mv[e]);
            if (q < L) *reinterpret_cast<f32x4*>(p.mean_out + cb0 + (long long)q * C + c0) = sv;
          }
        }
      }
      RP_T(tf);
      if (has_next) {
        commit_fill(nsr0);
        rp_barrier();
      }
#ifdef RP_DIAG_STAMPS
      {
        RP_T(tg);
        dg[0] += tb - ta; dg[1] += tc - tb; dg[2] += te - tc; dg[3] += tf - te; dg[4] += tg - tf;
        dg[5] += 1; dg[6] += nst; dg[7] += nst;
      }
#endif
    }
    if (!more) break;
    tile = next_tile;
    b = nb;
    r0 = nr0;
  }
#ifdef RP_DIAG_STAMPS
  if (tid == 0)
    for (int i = 0; i < 16; ++i) atomicAdd(&g_rp_diag[(C == 64 ? 16 : 0) + i], dg[i]);
#endif
}

// Barrier-free tap loops (round 3): conv_res_pair_g.  conv_res_pair's per-step stamps put a c1 tap
// step at 3690 cycles against 2304 of MFMA issue per SIMD (C = 64).  A timing build that never
// refilled the weight ring was no faster, and a 4-slot ring of half-tap units with the next unit's
// fragments prefetched into registers took 2278 cycles per 1152-cycle unit: every barrier of the
// ring costs ~1100 cycles (the 8 waves restart together behind one LDS queue, and the slowest wave
// sets the end), however short the step.  Here each wave loads its weight fragments from global
// memory (L2; the four waves of a column half read the same bytes, so most hit L1) into registers,
// chunk by chunk, one tap ahead: after the MFMAs of chunk ch of tap j, the registers take chunk ch
// of the next tap in the stream (next conv, member or tile).  The tap loops need no barrier; only the
// image hand-offs do (S -> T after c1, T -> the next S after c2).  Arithmetic, summation order and
// layouts are conv_res_pair's, so the results are the same bits.
template <int C, bool MEAN, int RR = kRpRows<C>>
__global__ void __launch_bounds__(512, 1) conv_res_pair_g(const ResPairParams p) {
  using G = RpGeom<C, RR>;
  constexpr int R = G::R, NCH = G::NCH, WR = G::WR, RB = G::RB1, PS = G::PS, IMG = G::IMG;
  constexpr int G8 = G::G8, NIT = G::NIT, NS = G::NS, WTAP = G::WTAP;
  __shared__ __attribute__((aligned(16))) char lds[IMG + 2 * kMaxGroup * C * 4];
  float* const bias_lds = reinterpret_cast<float*>(lds + IMG);  // [conv][member][C]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wc = wave % G::WC, wr = wave / G::WC;
  const int l15 = lane & 15, hf = (lane >> 4) & 1, t = lane >> 5;
  const int L = p.L, nmem = p.nmem;
  const int ntl = (L + R - 1) / R;
  const int total = ntl * p.batch;

  // ---- S image fill (as conv_res_pair) ----
  f32x4 pf[NIT][2];
  auto issue_fill_item = [&](const float* src, int r0, int k) {
    const int it = min(tid + 512 * k, NS * G8 - 1);
    const int s = ((it >> 3) / G8) * 8 + (it & 7), g8 = (it >> 3) % G8;
    const int a = min(max(r0 - 8 - G::H1 + s, 0), L - 1);
    const f32x4* q = reinterpret_cast<const f32x4*>(src + (long long)a * C + g8 * 8);
    pf[k][0] = q[0];
    pf[k][1] = q[1];
  };
  auto commit_fill = [&](int r0) {
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
      const int it = tid + 512 * k;
      if (!(NIT * 512 == NS * G8 || it < NS * G8)) continue;
      const int s = ((it >> 3) / G8) * 8 + (it & 7), g8 = (it >> 3) % G8;
      const int a = r0 - 8 - G::H1 + s;
      const bool ok = a >= 0 && a < L;
      s16x8 hv, mv, lv;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float sv = rp_silu(pf[k][e >> 2][e & 3]);
        const float v = ok ? sv : 0.f;
        unsigned short h, m, l;
        split3(v, h, m, l);
        hv[e] = (short)h;
        mv[e] = (short)m;
        lv[e] = (short)l;
      }
      char* d = lds + ((g8 >> 1) * 6 + (g8 & 1) * 3) * PS + s * 16;
      *reinterpret_cast<s16x8*>(d) = hv;
      *reinterpret_cast<s16x8*>(d + PS) = mv;
      *reinterpret_cast<s16x8*>(d + 2 * PS) = lv;
    }
  };

  // ---- weight fragments of chunk ch of a tap ([chunk][Cout][96 B], the ConvParams::w6 tap slice):
  // [column block][{h',m'} | {h',l'}] ----
  s16x8 wf[NCH][2][2];
  // buffer loads: the lane offsets are loop-invariant VGPRs, the tap base a scalar resource and the
  // chunk / column-block offsets scalar constants, so a reload costs no address arithmetic
  const int wo0 = ((2 * wc) * 16 + l15) * 96 + hf * 48 + t * 16, wo1 = ((2 * wc) * 16 + l15) * 96 + hf * 48 + (t ? 32 : 0);
  auto load_wf = [&](const unsigned short* wtap, int ch) {
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)wtap, 0, WTAP, 0x00020000);
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      const int so = (ch * C + cb * 16) * 96;
      wf[ch][cb][0] = __builtin_bit_cast(s16x8, __builtin_amdgcn_raw_buffer_load_b128(rw, wo0, so, 0));
      wf[ch][cb][1] = __builtin_bit_cast(s16x8, __builtin_amdgcn_raw_buffer_load_b128(rw, wo1, so, 0));
    }
  };
  // the tap after tap j of conv `conv` of member m: the stream runs c1, c2 of each member, then
  // member 0 again (the next tile; past the last tile harmless loads of weights already used)
  auto next_tap = [&](int m, int conv, int j) -> const unsigned short* {
    if (j + 1 < p.taps[m]) return (conv ? p.w2[m] : p.w1[m]) + (long long)(j + 1) * (WTAP / 2);
    if (conv == 0) return p.w2[m];
    return p.w1[m + 1 < nmem ? m + 1 : 0];
  };

  // ---- one tap, chunk-major: the MFMAs of chunk ch for every row block of the wave, then chunk ch
  // of the next tap into the fragment registers; hook() once every reload of the tap is issued (its
  // loads are then younger than the fragments the next tap waits for) ----
  // lane parts of the three activation reads (piece, row within the 16-row block); a tap adds its
  // wave-uniform row offset once, and row block / chunk offsets are instruction immediates
  const int pk0 = ((hf * 3 + t) * NS + l15) * 16, pk1 = ((hf * 3 + (t ? 0 : 1)) * NS + l15) * 16;
  const int pk2 = ((hf * 3 + (t ? 0 : 2)) * NS + l15) * 16;
  auto tap = [&](f32x4 (&acc)[RB][2], int rowoff, int nrb, const unsigned short* wnext, auto hook) {
    const int tb = (wr * 16 + rowoff) * 16;
    const char *xb0 = lds + pk0 + tb, *xb1 = lds + pk1 + tb, *xb2 = lds + pk2 + tb;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
#pragma unroll
      for (int i = 0; i < RB; ++i) {
        if (i < nrb) {
          const int io = (WR * 16 * i) * 16 + ch * 6 * PS;
          const s16x8 x2 = *reinterpret_cast<const s16x8*>(xb2 + io);
          const s16x8 x1 = *reinterpret_cast<const s16x8*>(xb1 + io);
          const s16x8 x0 = *reinterpret_cast<const s16x8*>(xb0 + io);
#pragma unroll
          for (int cb = 0; cb < 2; ++cb) {
            acc[i][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wf[ch][cb][1]),
                                                                 __builtin_bit_cast(bf16x8, x2), acc[i][cb], 0, 0, 0);
            acc[i][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wf[ch][cb][0]),
                                                                 __builtin_bit_cast(bf16x8, x1), acc[i][cb], 0, 0, 0);
            acc[i][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wf[ch][cb][0]),
                                                                 __builtin_bit_cast(bf16x8, x0), acc[i][cb], 0, 0, 0);
          }
        }
      }
      load_wf(wnext, ch);
      // keep the reloads here: left to itself the scheduler sinks all of them to the end of the tap,
      // and the next tap's first MFMAs then wait a whole L2 round trip
      __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_s_setprio(0);
    hook();
  };
  auto no_hook = [] {};

  const int nrb2 = min(RB, (G::NB2 - wr + WR - 1) / WR);
  int tile = blockIdx.x;
  if (tile >= total) return;  // whole workgroup, before any barrier
  int b = tile / ntl, r0 = (tile - b * ntl) * R;
  if (tid < 2 * nmem * C) {
    const int conv = tid / (nmem * C), m = (tid / C) % nmem, c = tid % C;
    bias_lds[(conv * kMaxGroup + m) * C + c] = (conv ? p.b2[m] : p.b1[m])[c];
  }
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) load_wf(p.w1[0], ch);
#pragma unroll
  for (int k = 0; k < NIT; ++k) issue_fill_item(p.src[0] + (long long)b * p.bstride, r0, k);
  commit_fill(r0);
  rp_barrier();
  f32x4 macc[MEAN ? RB : 1][2];
#ifdef RP_DIAG_STAMPS
  unsigned long long dg[16] = {};
#endif
  for (;;) {
    const int next_tile = tile + gridDim.x;
    const bool more = next_tile < total;
    const int nb = more ? next_tile / ntl : 0, nr0 = more ? (next_tile - nb * ntl) * R : 0;
    for (int m = 0; m < nmem; ++m) {
      const int k = p.taps[m], hk = (k - 1) >> 1, d = p.dil[m];
      const long long cb0 = (long long)b * p.bstride;
      const bool last_m = m + 1 == nmem;
      const bool has_next = !last_m || more;
      f32x4 acc[RB][2];
      RP_T(ta);
      // ---- c1 over rows [r0 - 8, r0 + R + 8) from the S image
#pragma unroll
      for (int i = 0; i < RB; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int ts = p.tap_sync;
      for (int j = 0; j < k; ++j) {
        tap(acc, G::H1 + (j - hk) * d, RB, next_tap(m, 0, j), no_hook);
        if (ts && (j + 1) % ts == 0 && j + 1 < k) rp_barrier();  // workgroup-uniform
      }
      RP_T(tb);
      rp_barrier();  // every wave's S reads are done before T overwrites them
      // ---- T image: silu(c1 + b1) planes over the S image (zero outside the clip)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const int c0 = (2 * wc + cb) * 16 + 4 * (lane >> 4);
        const f32x4 bias = *reinterpret_cast<const f32x4*>(bias_lds + m * C + c0);
#pragma unroll
        for (int i = 0; i < RB; ++i) {
          const int ir = (wr + WR * i) * 16 + l15, a = r0 - 8 + ir;
          const bool ok = a >= 0 && a < L;
          s16x4 hv, mv, lv;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float sv = rp_silu(acc[i][cb][e] + bias[e]);
            const float v = ok ? sv : 0.f;
            unsigned short h, mm, l;
            split3(v, h, mm, l);
            hv[e] = (short)h;
            mv[e] = (short)mm;
            lv[e] = (short)l;
          }
          char* dst = lds + ((c0 >> 4) * 6 + ((c0 >> 3) & 1) * 3) * PS + ir * 16 + (c0 & 7) * 2;
          *reinterpret_cast<s16x4*>(dst) = hv;
          *reinterpret_cast<s16x4*>(dst + PS) = mv;
          *reinterpret_cast<s16x4*>(dst + 2 * PS) = lv;
        }
      }
      rp_barrier();
      RP_T(tc);
      // ---- c2 over rows [r0, r0 + R) from the T image.  Tap 0 loads the residual rows, taps 1 and 2
      // the next S image's rows (this tile's next ResBlock, or the next tile's first), each after the
      // tap's fragment reloads (k >= 3, so taps 0..2 exist; they are peeled so that the register
      // arrays are indexed by constants)
#pragma unroll
      for (int i = 0; i < RB; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      const float* nsrc = !last_m ? p.src[m + 1] + cb0 : p.src[0] + (long long)nb * p.bstride;
      const int nsr0 = !last_m ? r0 : nr0;
      f32x4 res[RB][2];
      auto res_hook = [&] {
#pragma unroll
        for (int i = 0; i < RB; ++i) {
          const int q = min(r0 + (wr + WR * i) * 16 + l15, L - 1);
#pragma unroll
          for (int cb = 0; cb < 2; ++cb) {
            const int c0 = (2 * wc + cb) * 16 + 4 * (lane >> 4);
            res[i][cb] = *reinterpret_cast<const f32x4*>(p.src[m] + cb0 + (long long)q * C + c0);
          }
        }
      };
      auto pf_hook0 = [&] {
        if (!has_next) return;
#pragma unroll
        for (int kk = 0; kk < NIT / 2; ++kk) issue_fill_item(nsrc, nsr0, kk);
      };
      auto pf_hook1 = [&] {
        if (!has_next) return;
#pragma unroll
        for (int kk = NIT / 2; kk < NIT; ++kk) issue_fill_item(nsrc, nsr0, kk);
      };
      tap(acc, 8 - hk, nrb2, next_tap(m, 1, 0), res_hook);
      if (ts == 1) rp_barrier();
      tap(acc, 9 - hk, nrb2, next_tap(m, 1, 1), pf_hook0);
      if (ts && 2 % ts == 0) rp_barrier();
      tap(acc, 10 - hk, nrb2, next_tap(m, 1, 2), pf_hook1);
      if (ts && 3 % ts == 0 && 3 < k) rp_barrier();
      for (int j = 3; j < k; ++j) {
        tap(acc, 8 + j - hk, nrb2, next_tap(m, 1, j), no_hook);
        if (ts && (j + 1) % ts == 0 && j + 1 < k) rp_barrier();
      }
      RP_T(te);
      // ---- epilogue: state + c2 + b2 (rows past the clip end are dropped)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const int c0 = (2 * wc + cb) * 16 + 4 * (lane >> 4);
        const f32x4 bias = *reinterpret_cast<const f32x4*>(bias_lds + (kMaxGroup + m) * C + c0);
#pragma unroll
        for (int i = 0; i < RB; ++i) {
          if (i >= nrb2) break;
          const int q = r0 + (wr + WR * i) * 16 + l15;
          const f32x4 v = res[i][cb] + (acc[i][cb] + bias);
          if constexpr (!MEAN) {
            if (q < L) *reinterpret_cast<f32x4*>(p.dst[m] + cb0 + (long long)q * C + c0) = v;
          } else if (m == 0) {
            macc[i][cb] = v;
          } else if (!last_m) {
            macc[i][cb] = macc[i][cb] + v;
          } else {
            const f32x4 mv = (macc[i][cb] + v) / 3.0f;
            f32x4 sv;
#pragma unroll
            for (int e = 0; e < 4; ++e) sv[e] = rp_silu(mv[e]);
            if (q < L) *reinterpret_cast<f32x4*>(p.mean_out + cb0 + (long long)q * C + c0) = sv;
          }
        }
      }
      RP_T(tf);
      if (has_next) {
        rp_barrier();  // every wave's T reads are done before the next S image overwrites them
        commit_fill(nsr0);
        rp_barrier();
      }
#ifdef RP_DIAG_STAMPS
      {
        RP_T(tg);
        dg[0] += tb - ta; dg[1] += tc - tb; dg[2] += te - tc; dg[3] += tf - te; dg[4] += tg - tf;
        dg[5] += 1; dg[6] += k; dg[7] += k;
      }
#endif
    }
    if (!more) break;
    tile = next_tile;
    b = nb;
    r0 = nr0;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last tap's (unused) fragment reloads
#ifdef RP_DIAG_STAMPS
  if (tid == 0)
    for (int i = 0; i < 16; ++i) atomicAdd(&g_rp_diag[(C == 64 ? 16 : 0) + i], dg[i]);
#endif
}

// conv_res_pair_h3 (round 5): conv_res_pair_g in h3 arithmetic (ResPairParams::h3; the fp16 h / l
// split of conv_gemm_x3dq, three products per fp32 product on v_mfma_f32_16x16x32_f16).  A K32 chunk
// of a tap is three MFMAs per 16 x 16 block, W{h'} . X{l}, W{l'} . X{h}, W{h'} . X{h}, the lanes of K
// group kg = lane >> 4 holding channel group kg of both operands: half the MFMAs of x6, two fragment
// reads per block and chunk instead of six, and images of 4 B per element instead of 6 (byte
// ((chunk * 8 + piece) * NS + row) * 16, piece = plane * 4 + channel group).  Weights: the
// ConvParams::w3 tap slices ([chunk][Cout][4][h' 8 | l' 8], scaled by 2^w3_shift per conv); the
// accumulators are scaled back before the bias.  Schedule, tiles and hand-offs are conv_res_pair_g's.
template <int C, bool MEAN, int RR = kRp3Rows<C>, bool RING = false>
__global__ void __launch_bounds__(512, 1) conv_res_pair_h3(const ResPairParams p) {
#ifdef __HIP_DEVICE_COMPILE__  // the body is device code only (its host pass dropped the RING stubs)
  using G = RpGeom3<C, RR>;
  constexpr int R = G::R, WR = G::WR, RB = G::RB1, PS = G::PS;
  constexpr int G8 = G::G8, NIT = G::NIT, NS = G::NS;
  constexpr int NCH = G::NCH, IMG = G::IMG, WTAP = G::WTAP;
  // RING (round 6, Knobs::rp_ring): the weight taps through an LDS ring of NSLOT taps instead of
  // per-wave loads (below)
  constexpr int NSLOT = 4, RINGB = RING ? NSLOT * WTAP : 0, BIASB = 2 * kMaxGroup * C * 4;
  constexpr int NP = C * C / 256, PPW = (NP + 7) / 8;  // 1 KiB pieces per tap, per wave
  static_assert(IMG + RINGB + BIASB + 2 * NSLOT * 4 <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) char lds[IMG + RINGB + BIASB + (RING ? 2 * NSLOT * 4 : 0)];
  float* const bias_lds = reinterpret_cast<float*>(lds + IMG + RINGB);  // [conv][member][C]
  // ring counters: rd_cnt[slot] += 1 per wave once it holds a tap of the slot in registers, full_cnt[slot]
  // += 1 per wave once its pieces of the slot's tap have landed (monotone: use u of a slot is complete at 8 (u + 1))
  unsigned* const rd_cnt = reinterpret_cast<unsigned*>(lds + IMG + RINGB + BIASB);
  unsigned* const full_cnt = rd_cnt + NSLOT;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wc = wave % G::WC, wr = wave / G::WC;
  const int l15 = lane & 15, kg = lane >> 4;
  const int L = p.L, nmem = p.nmem;
  const int ntl = (L + R - 1) / R;
  const int total = ntl * p.batch;

  // ---- S image fill (as conv_res_pair) ----
  f32x4 pf[NIT][2];
  auto issue_fill_item = [&](const float* src, int r0, int k) {
    const int it = min(tid + 512 * k, NS * G8 - 1);
    const int s = ((it >> 3) / G8) * 8 + (it & 7), g8 = (it >> 3) % G8;
    const int a = min(max(r0 - 8 - G::H1 + s, 0), L - 1);
    const f32x4* q = reinterpret_cast<const f32x4*>(src + (long long)a * C + g8 * 8);
    pf[k][0] = q[0];
    pf[k][1] = q[1];
  };
  // sc: the image's range scale, 2^h2_shift(max |state| of the clip) (dcx_kernels.h)
  auto commit_fill = [&](int r0, float sc) {
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
      const int it = tid + 512 * k;
      if (!(NIT * 512 == NS * G8 || it < NS * G8)) continue;
      const int s = ((it >> 3) / G8) * 8 + (it & 7), g8 = (it >> 3) % G8;
      const int a = r0 - 8 - G::H1 + s;
      const bool ok = a >= 0 && a < L;
      s16x8 hv, lv;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float sv = rp_silu(pf[k][e >> 2][e & 3]) * sc;
        const float v = ok ? sv : 0.f;
        unsigned short hh, ll;
        split2h_nc(v, hh, ll);
        hv[e] = (short)hh;
        lv[e] = (short)ll;
      }
      char* d = lds + ((g8 >> 2) * 8 + (g8 & 3)) * PS + s * 16;
      *reinterpret_cast<s16x8*>(d) = hv;
      *reinterpret_cast<s16x8*>(d + 4 * PS) = lv;
    }
  };

  // ---- weight fragments of chunk ch of a tap ([chunk][Cout][128 B], the ConvParams::w3 tap slice):
  // [column block][h' | l'] of the lane's channel group ----
  s16x8 wf[NCH][2][2];
  const int wo0 = ((2 * wc) * 16 + l15) * 128 + kg * 32, wo1 = wo0 + 16;
  [[maybe_unused]] bool wl_off = false;  // -DRP_DIAG_NOWLOAD (timing only, wrong results): no reloads after the prologue
  auto load_wf = [&](const unsigned short* wtap, int ch) {
#ifdef RP_DIAG_NOWLOAD
    if (wl_off) return;
#endif
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)wtap, 0, WTAP, 0x00020000);
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      const int so = (ch * C + cb * 16) * 128;
      wf[ch][cb][0] = __builtin_bit_cast(s16x8, __builtin_amdgcn_raw_buffer_load_b128(rw, wo0, so, 0));
      wf[ch][cb][1] = __builtin_bit_cast(s16x8, __builtin_amdgcn_raw_buffer_load_b128(rw, wo1, so, 0));
    }
  };
  // the tap after tap j of conv `conv` of member m: the stream runs c1, c2 of each member, then
  // member 0 again (the next tile; past the last tile harmless loads of weights already used)
  auto next_tap = [&](int m, int conv, int j) -> const unsigned short* {
    if (RING) return nullptr;
    if (j + 1 < p.taps[m]) return (conv ? p.w2[m] : p.w1[m]) + (long long)(j + 1) * (WTAP / 2);
    if (conv == 0) return p.w2[m];
    return p.w1[m + 1 < nmem ? m + 1 : 0];
  };

  // ---- RING: the weight stream through LDS.  Tap t (counted over the whole kernel: c1 then c2 of
  // each member, tile after tile) sits in slot t % NSLOT as NP pieces of 1 KiB, piece (ch, column
  // block, h' | l') laid out as the fragment read of a wave (lane l: channel l & 15 of the block, K
  // group l >> 4), so every ds_read_b128 of a fragment is one linear 1 KiB piece (conflict-free).
  // Each wave issues pieces w, w + 8, ... of a tap by LDS-DMA, two taps ahead; per tap t it
  //   A. counts itself in rd_cnt[t % NSLOT] once its reads of tap t (made during tap t - 1) returned;
  //   B. waits for its own pieces of tap t + 1 (vmcnt, counted past the younger loads) and counts
  //      itself in full_cnt[(t + 1) % NSLOT];
  //   C. issues its pieces of tap t + 2 into that tap's slot once every wave has counted itself in as
  //      having read the slot's previous tap t + 2 - NSLOT;
  //   and after its chunk-0 MFMAs waits for full_cnt of tap t + 1 before reading it from the ring.
  // A wave counts itself in (A, B) before it waits on anything at a tap, so the slowest wave is never
  // blocked: no deadlock, and the waves stay within two taps of each other.  Replaces per-wave loads
  // of each tap's fragments from L2 / L1 (16 KiB per wave-pair at C = 64, 4x the tap; timing build
  // without them: 21.0 -> 13.5 ms for the C = 64 ParallelBlock, r06e).
  int ring_t = 0;                    // the tap being computed
  int ic_m = 0, ic_conv = 0, ic_j = 0;  // the next tap to issue (ring_t + 2 in the loop)
  int dsrc[PPW];                     // per-lane source offsets of this wave's pieces
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int pc = min(wave + 8 * i, NP - 1);
    const int pl = pc & 1, cbk = (pc >> 1) % (C / 16), ch = (pc >> 1) / (C / 16);
    dsrc[i] = (ch * C + cbk * 16 + l15) * 128 + kg * 32 + pl * 16;
  }
  // members' weights and tap counts picked by uniform selects (an index into the kernel-argument
  // arrays became a vector load that hipcc then waited for with vmcnt(0), DMA in flight included)
  auto mpick = [&](auto a0, auto a1, auto a2, int m) { return m == 0 ? a0 : m == 1 ? a1 : a2; };
  auto ring_issue = [&](int slot) {  // this wave's pieces of the issue cursor's tap, then advance it
    const unsigned short* w1 = mpick(p.w1[0], p.w1[1], p.w1[2], ic_m);
    const unsigned short* w2 = mpick(p.w2[0], p.w2[1], p.w2[2], ic_m);
    const unsigned short* wp = (ic_conv ? w2 : w1) + (long long)ic_j * (WTAP / 2);
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)wp, 0, WTAP, 0x00020000);
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int pc = wave + 8 * i;
      if (NP % 8 == 0 || pc < NP)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (rp_lds_t)(lds + IMG + slot * WTAP + pc * 1024), 16, dsrc[i], 0, 0, 0);
    }
    if (++ic_j == mpick(p.taps[0], p.taps[1], p.taps[2], ic_m)) {
      ic_j = 0;
      if (ic_conv == 0) ic_conv = 1;
      else {
        ic_conv = 0;
        ic_m = ic_m + 1 < nmem ? ic_m + 1 : 0;
      }
    }
  };
  // the counter read is inline asm: as a C++ LDS load hipcc made it wait for the wave's LDS-DMA in
  // flight (vmcnt(0): the pieces of tap t + 2, just issued), which it cannot tell apart from the slot
  auto spin_ge = [&](const unsigned* c, unsigned want) {
    const unsigned a = (unsigned)(size_t)(const __attribute__((address_space(3))) void*)c;
    for (;;) {
      unsigned v;
      asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
      if (__builtin_amdgcn_readfirstlane(v) >= want) break;
      __builtin_amdgcn_s_sleep(1);
    }
  };
  auto count_in = [&](unsigned* c) {  // inline asm for the same reason as spin_ge
    const unsigned a = (unsigned)(size_t)(__attribute__((address_space(3))) void*)c;
    if (lane == 0) asm volatile("ds_add_u32 %0, %1" ::"v"(a), "v"(1u) : "memory");
  };
  const int wrd = lane * 16 + (2 * wc) * 2 * 1024;  // lane part of a fragment read from the ring
  auto read_wf = [&](int slot, int ch) {
    const char* wb = lds + IMG + slot * WTAP + wrd;
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      wf[ch][cb][0] = *reinterpret_cast<const s16x8*>(wb + ((ch * (C / 16) + cb) * 2 + 0) * 1024);
      wf[ch][cb][1] = *reinterpret_cast<const s16x8*>(wb + ((ch * (C / 16) + cb) * 2 + 1) * 1024);
    }
  };

  // ---- one tap, chunk-major: the MFMAs of chunk ch for every row block of the wave, then chunk ch
  // of the next tap into the fragment registers; hook() once every reload of the tap is issued (its
  // loads are then younger than the fragments the next tap waits for) ----
  // lane parts of the two activation reads (h and l pieces of the lane's channel group, row within
  // the 16-row block); a tap adds its wave-uniform row offset once, row block / chunk offsets are
  // instruction immediates
  const int pkh = (kg * NS + l15) * 16, pkl = ((4 + kg) * NS + l15) * 16;
  // RING: hook() first (its nyoung global loads are then the only ones younger than the pieces B
  // waits for; nyoung may undercount, never overcount)
  auto tap = [&](f32x4 (&acc)[RB][2], int rowoff, int nrb, const unsigned short* wnext, int nyoung, auto hook) {
    const int tb = (wr * 16 + rowoff) * 16;
    const char *xbh = lds + pkh + tb, *xbl = lds + pkl + tb;
    const int t = ring_t;
    if constexpr (RING) {
      hook();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // A
      count_in(rd_cnt + t % NSLOT);
      rp_wait(nyoung);  // B
      count_in(full_cnt + (t + 1) % NSLOT);
      spin_ge(rd_cnt + (t + 2) % NSLOT, 8u * (unsigned)((t + 2) / NSLOT));  // C
      ring_issue((t + 2) % NSLOT);
      ring_t = t + 1;
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
#pragma unroll
      for (int i = 0; i < RB; ++i) {
        if (i < nrb) {
          const int io = (WR * 16 * i) * 16 + ch * 8 * PS;
          const s16x8 xl = *reinterpret_cast<const s16x8*>(xbl + io);
          const s16x8 xh = *reinterpret_cast<const s16x8*>(xbh + io);
#pragma unroll
          for (int cb = 0; cb < 2; ++cb) {
            acc[i][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, wf[ch][cb][0]),
                                                                __builtin_bit_cast(f16x8, xl), acc[i][cb], 0, 0, 0);
            acc[i][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, wf[ch][cb][1]),
                                                                __builtin_bit_cast(f16x8, xh), acc[i][cb], 0, 0, 0);
            acc[i][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, wf[ch][cb][0]),
                                                                __builtin_bit_cast(f16x8, xh), acc[i][cb], 0, 0, 0);
          }
        }
      }
      if constexpr (RING) {
        if (ch == 0) spin_ge(full_cnt + (t + 1) % NSLOT, 8u * (unsigned)((t + 1) / NSLOT + 1));
        read_wf((t + 1) % NSLOT, ch);
      } else {
        load_wf(wnext, ch);
      }
      // keep the reloads here: left to itself the scheduler sinks all of them to the end of the tap,
      // and the next tap's first MFMAs then wait a whole L2 round trip
      __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_s_setprio(0);
    if constexpr (!RING) hook();
  };
  auto no_hook = [] {};

  // c2 computes every row block (the waves owning fewer than RB of the R output rows compute rows past
  // them, from image rows inside the image, and drop them in the epilogue): a runtime row-block count
  // put a branch between the MFMAs of every row block (round 6: c2 taps ran 1.2-1.6x as long as c1's)
  const int nrb2 = min(RB, (G::NB2 - wr + WR - 1) / WR);
  // range shifts (round 6): member m's S image of clip bb from the measured max |state|, its T image
  // from the bound g1 max|state| + max|b1| of c1's output (|silu(v)| <= |v|)
  auto s_shift = [&](int m, int bb) { return p.src_amax[m] ? h2_shift(p.src_amax[m][bb]) : 0; };
  auto t_shift = [&](int m, int bb) {
    return p.src_amax[m] ? h2_shift(fmaf(p.g1[m], p.src_amax[m][bb], p.bm1[m])) : 0;
  };
  // the shifts of the tile's clip for every member, read once per tile into scalar registers (read
  // where they are used, each load's wait took every load and DMA in flight with it)
  // (RING: the launcher guarantees src_amax for every member, so the loads are unconditional and
  // issued together); shs0n: member 0's S shift of the next tile's clip
  int shs[kMaxGroup], sht[kMaxGroup], shs0n = 0;
  auto tile_shifts = [&](int bb, int nbb) {
    float a[kMaxGroup];
#pragma unroll
    for (int i = 0; i < kMaxGroup; ++i) a[i] = p.src_amax[i < nmem ? i : 0][bb];
    const float an = p.src_amax[0][nbb];
#pragma unroll
    for (int i = 0; i < kMaxGroup; ++i) {
      shs[i] = __builtin_amdgcn_readfirstlane(h2_shift(a[i]));
      sht[i] = __builtin_amdgcn_readfirstlane(h2_shift(fmaf(p.g1[i], a[i], p.bm1[i])));
    }
    shs0n = __builtin_amdgcn_readfirstlane(h2_shift(an));
  };
  int tile = blockIdx.x;
  if (tile >= total) return;  // whole workgroup, before any barrier
  int b = tile / ntl, r0 = (tile - b * ntl) * R;
  if (tid < 2 * nmem * C) {
    const int conv = tid / (nmem * C), m = (tid / C) % nmem, c = tid % C;
    bias_lds[(conv * kMaxGroup + m) * C + c] = (conv ? p.b2[m] : p.b1[m])[c];
  }
  if constexpr (RING) {
    if (tid < 2 * NSLOT) rd_cnt[tid] = 0u;
    rp_barrier();
    ring_issue(0);
    ring_issue(1);
  } else {
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) load_wf(p.w1[0], ch);
  }
#pragma unroll
  for (int k = 0; k < NIT; ++k) issue_fill_item(p.src[0] + (long long)b * p.bstride, r0, k);
  commit_fill(r0, __builtin_ldexpf(1.0f, s_shift(0, b)));
  if constexpr (RING) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    count_in(full_cnt + 0);  // tap 1's pieces are counted in by B of tap 0
  }
  rp_barrier();
  if constexpr (RING) {
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) read_wf(0, ch);
  }
  wl_off = true;
  f32x4 macc[MEAN ? RB : 1][2];
#ifdef RP_DIAG_STAMPS
  unsigned long long dg[16] = {};
#endif
  for (;;) {
    const int next_tile = tile + gridDim.x;
    const bool more = next_tile < total;
    const int nb = more ? next_tile / ntl : 0, nr0 = more ? (next_tile - nb * ntl) * R : 0;
    if constexpr (RING) tile_shifts(b, nb);
    for (int m = 0; m < nmem; ++m) {
      const int k = p.taps[m], hk = (k - 1) >> 1, d = p.dil[m];
      const long long cb0 = (long long)b * p.bstride;
      const bool last_m = m + 1 == nmem;
      const bool has_next = !last_m || more;
      f32x4 acc[RB][2];
      RP_T(ta);
      // ---- c1 over rows [r0 - 8, r0 + R + 8) from the S image
#pragma unroll
      for (int i = 0; i < RB; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int ts = p.tap_sync;
      for (int j = 0; j < k; ++j) {
        tap(acc, G::H1 + (j - hk) * d, RB, next_tap(m, 0, j), 0, no_hook);
        if (ts && (j + 1) % ts == 0 && j + 1 < k) rp_barrier();  // workgroup-uniform
      }
      RP_T(tb);
      rp_barrier();  // every wave's S reads are done before T overwrites them
      // ---- T image: silu(c1 + b1) as h / l over the S image (zero outside the clip), range-scaled
      const int sh_t = RING ? mpick(sht[0], sht[1], sht[2], m) : t_shift(m, b);
      const float us1 = __builtin_ldexpf(1.0f, -(p.w3_shift1[m] + (RING ? mpick(shs[0], shs[1], shs[2], m) : s_shift(m, b))));
      const float tsc = __builtin_ldexpf(1.0f, sh_t);  // (rigorous bound: no per-element check, epilogue_lds)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const int c0 = (2 * wc + cb) * 16 + 4 * (lane >> 4);
        const f32x4 bias = *reinterpret_cast<const f32x4*>(bias_lds + m * C + c0);
#pragma unroll
        for (int i = 0; i < RB; ++i) {
          const int ir = (wr + WR * i) * 16 + l15, a = r0 - 8 + ir;
          const bool ok = a >= 0 && a < L;
          s16x4 hv, lv;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float pre = acc[i][cb][e] * us1 + bias[e];
            const float sv = rp_silu(pre);
            const float v = ok ? sv * tsc : 0.f;
            unsigned short hh, ll;
            split2h_nc(v, hh, ll);
            hv[e] = (short)hh;
            lv[e] = (short)ll;
          }
          char* dst = lds + ((c0 >> 5) * 8 + ((c0 >> 3) & 3)) * PS + ir * 16 + (c0 & 7) * 2;
          *reinterpret_cast<s16x4*>(dst) = hv;
          *reinterpret_cast<s16x4*>(dst + 4 * PS) = lv;
        }
      }
      rp_barrier();
      RP_T(tc);
      // ---- c2 over rows [r0, r0 + R) from the T image.  Tap 0 loads the residual rows, taps 1 and 2
      // the next S image's rows (this tile's next ResBlock, or the next tile's first), each after the
      // tap's fragment reloads (k >= 3, so taps 0..2 exist; they are peeled so that the register
      // arrays are indexed by constants)
#pragma unroll
      for (int i = 0; i < RB; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      const float* nsrc = !last_m ? p.src[m + 1] + cb0 : p.src[0] + (long long)nb * p.bstride;
      const int nsr0 = !last_m ? r0 : nr0;
      f32x4 res[RB][2];
      float dcur = 0.f;  // this clip's running max |dst| (range_report)
      auto res_hook = [&] {
        if constexpr (!MEAN) dcur = range_cur(p.dst_amax[m], b);  // older than the residual loads
#pragma unroll
        for (int i = 0; i < RB; ++i) {
          const int q = min(r0 + (wr + WR * i) * 16 + l15, L - 1);
#pragma unroll
          for (int cb = 0; cb < 2; ++cb) {
            const int c0 = (2 * wc + cb) * 16 + 4 * (lane >> 4);
            res[i][cb] = *reinterpret_cast<const f32x4*>(p.src[m] + cb0 + (long long)q * C + c0);
          }
        }
      };
      auto pf_hook0 = [&] {
        if (!has_next) return;
#pragma unroll
        for (int kk = 0; kk < NIT / 2; ++kk) issue_fill_item(nsrc, nsr0, kk);
      };
      auto pf_hook1 = [&] {
        if (!has_next) return;
#pragma unroll
        for (int kk = NIT / 2; kk < NIT; ++kk) issue_fill_item(nsrc, nsr0, kk);
      };
      tap(acc, 8 - hk, RB, next_tap(m, 1, 0), RB * 2, res_hook);
      if (ts == 1) rp_barrier();
      tap(acc, 9 - hk, RB, next_tap(m, 1, 1), has_next ? (NIT / 2) * 2 : 0, pf_hook0);
      if (ts && 2 % ts == 0) rp_barrier();
      tap(acc, 10 - hk, RB, next_tap(m, 1, 2), has_next ? (NIT - NIT / 2) * 2 : 0, pf_hook1);
      if (ts && 3 % ts == 0 && 3 < k) rp_barrier();
      for (int j = 3; j < k; ++j) {
        tap(acc, 8 + j - hk, RB, next_tap(m, 1, j), 0, no_hook);
        if (ts && (j + 1) % ts == 0 && j + 1 < k) rp_barrier();
      }
      RP_T(te);
      // ---- epilogue: state + c2 + b2 (rows past the clip end are dropped); its max |.| per clip for
      // the next pair's S image
      const float us2 = __builtin_ldexpf(1.0f, -(p.w3_shift2[m] + sh_t));
      float dmax = 0.f;
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const int c0 = (2 * wc + cb) * 16 + 4 * (lane >> 4);
        const f32x4 bias = *reinterpret_cast<const f32x4*>(bias_lds + (kMaxGroup + m) * C + c0);
#pragma unroll
        for (int i = 0; i < RB; ++i) {
          if (i >= nrb2) break;
          const int q = r0 + (wr + WR * i) * 16 + l15;
          const f32x4 v = res[i][cb] + (acc[i][cb] * us2 + bias);
          if constexpr (!MEAN) {
            if (q < L) {
              *reinterpret_cast<f32x4*>(p.dst[m] + cb0 + (long long)q * C + c0) = v;
              dmax = fmaxf(dmax, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
            }
          } else if (m == 0) {
            macc[i][cb] = v;
          } else if (!last_m) {
            macc[i][cb] = macc[i][cb] + v;
          } else {
            const f32x4 mv = (macc[i][cb] + v) / 3.0f;
            f32x4 sv;
#pragma unroll
            for (int e = 0; e < 4; ++e) sv[e] = rp_silu(mv[e]);
            if (q < L) *reinterpret_cast<f32x4*>(p.mean_out + cb0 + (long long)q * C + c0) = sv;
          }
        }
      }
      if constexpr (!MEAN) {
        if (p.dst_amax[m]) range_report(dmax, p.dst_amax[m], b, __builtin_inff(), nullptr, dcur);  // workgroup-uniform
      }
      RP_T(tf);
      if (has_next) {
        rp_barrier();  // every wave's T reads are done before the next S image overwrites them
        commit_fill(nsr0, __builtin_ldexpf(1.0f, RING ? (last_m ? shs0n : mpick(shs[1], shs[2], shs[2], m))
                                                 : last_m ? s_shift(0, nb) : s_shift(m + 1, b)));
        rp_barrier();
      }
#ifdef RP_DIAG_STAMPS
      {
        RP_T(tg);
        dg[0] += tb - ta; dg[1] += tc - tb; dg[2] += te - tc; dg[3] += tf - te; dg[4] += tg - tf;
        dg[5] += 1; dg[6] += k; dg[7] += k;
      }
#endif
    }
    if (!more) break;
    tile = next_tile;
    b = nb;
    r0 = nr0;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last tap's (unused) fragment reloads
#ifdef RP_DIAG_STAMPS
  if (tid == 0)
    for (int i = 0; i < 16; ++i) atomicAdd(&g_rp_diag[(C == 64 ? 16 : 0) + i], dg[i]);
#endif
#endif
}


// conv_res_pair_w4 (round 5): the barrier-free tap loops of conv_res_pair_g on 4-wave workgroups, TWO
// per CU.  In the 8-wave kernels the two waves of a SIMD belong to one workgroup and go through the
// same phases together: both run their tap loops (sharing the matrix pipe, each covering the other's
// LDS latency only while both are there), then both convert images (VALU only, the matrix pipe idle),
// then both wait at the hand-off barriers for the slowest wave (PMC: 0.40-0.50 MFMA busy; stamps of
// the 8-wave barrier-free kernel: taps at 0.92 of MFMA issue for the leading wave, the lagging wave's
// deficit paid at the next barrier).  Here the partner wave on each SIMD belongs to ANOTHER workgroup,
// with its own LDS image and barriers, so one workgroup's image conversions, epilogue, S-image loads
// and barrier waits run beside the other's MFMAs.  Each workgroup owns R output rows of one clip (its
// image within half the LDS); the S image is filled only over the rows member m's c1 reads (its reach
// (k - 1) / 2 * d), straight from global memory (the other workgroup covers the load latency).  The
// MFMAs, their order per accumulator and the layouts are conv_res_pair_g's, so the bits are the same.
template <int C, int RR>
struct RpGeom4 {
  static constexpr int R = RR;
  static constexpr int M1 = R + 16;               // c1 rows: [r0 - 8, r0 + R + 8)
  static constexpr int H1 = 32;                   // largest c1 reach
  static constexpr int NS = M1 + 2 * H1;          // S image rows
  static constexpr int NCH = C / 16;
  static constexpr int WC = C / 32, WR = 4 / WC;  // waves: WR row groups x WC column halves
  static constexpr int NB1 = M1 / 16, RB = NB1 / WR;
  static constexpr int NB2 = R / 16;
  static constexpr int PS = NS * 16;
  static constexpr int IMG = NCH * 6 * PS;
  static constexpr int G8 = C / 8;
  static constexpr int WTAP = C * C * 6;
  static constexpr int FB = 4;                    // S-image items (8 channels) per thread per load batch
  static constexpr int LDS = IMG + 2 * kMaxGroup * C * 4;
  static_assert(NB1 % WR == 0 && (NB2 + WR - 1) / WR <= RB, "row blocks per wave");
  static_assert(LDS <= 80 * 1024, "two workgroups per CU");
};
template <int C>
constexpr int kRp4Rows = C == 32 ? 304 : 112;

template <int C, bool MEAN, int RR = kRp4Rows<C>>
__global__ void __launch_bounds__(256, 2) conv_res_pair_w4(const ResPairParams p) {
  using G = RpGeom4<C, RR>;
  constexpr int R = G::R, NCH = G::NCH, WR = G::WR, RB = G::RB, PS = G::PS, IMG = G::IMG;
  constexpr int G8 = G::G8, NS = G::NS, WTAP = G::WTAP, FB = G::FB;
  __shared__ __attribute__((aligned(16))) char lds[G::LDS];
  float* const bias_lds = reinterpret_cast<float*>(lds + IMG);  // [conv][member][C]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wc = wave % G::WC, wr = wave / G::WC;
  const int l15 = lane & 15, hf = (lane >> 4) & 1, t = lane >> 5;
  const int L = p.L, nmem = p.nmem;
  const int ntl = (L + R - 1) / R;
  const int total = ntl * p.batch;

  // ---- S image: silu(state) as planes over the 8-row groups covering [H1 - reach, H1 + M1 + reach)
  // (zero outside the clip = the conv's padding); rows outside that range are never read ----
  auto fill = [&](const float* src, int r0, int reach) {
    const int lo = (G::H1 - reach) & ~7;
    const int hi = min(NS, (G::H1 + G::M1 + reach + 7) & ~7);
    const int nit = (hi - lo) * G8;
    for (int base = 0; base < nit; base += 256 * FB) {
      f32x4 v[FB][2];
#pragma unroll
      for (int k = 0; k < FB; ++k) {  // unconditional loads (index clamped): all in flight at once
        const int it = min(base + tid + 256 * k, nit - 1);
        const int s = lo + ((it >> 3) / G8) * 8 + (it & 7), g8 = (it >> 3) % G8;
        const int a = min(max(r0 - 8 - G::H1 + s, 0), L - 1);
        const f32x4* q = reinterpret_cast<const f32x4*>(src + (long long)a * C + g8 * 8);
        v[k][0] = q[0];
        v[k][1] = q[1];
      }
#pragma unroll
      for (int k = 0; k < FB; ++k) {
        const int it = base + tid + 256 * k;
        if (it < nit) {
          const int s = lo + ((it >> 3) / G8) * 8 + (it & 7), g8 = (it >> 3) % G8;
          const int a = r0 - 8 - G::H1 + s;
          const bool ok = a >= 0 && a < L;
          s16x8 hv, mv, lv;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float sv = rp_silu(v[k][e >> 2][e & 3]);
            const float x = ok ? sv : 0.f;
            unsigned short h, m, l;
            split3(x, h, m, l);
            hv[e] = (short)h;
            mv[e] = (short)m;
            lv[e] = (short)l;
          }
          char* d = lds + ((g8 >> 1) * 6 + (g8 & 1) * 3) * PS + s * 16;
          *reinterpret_cast<s16x8*>(d) = hv;
          *reinterpret_cast<s16x8*>(d + PS) = mv;
          *reinterpret_cast<s16x8*>(d + 2 * PS) = lv;
        }
      }
    }
  };

  // ---- weight fragments, one tap ahead (conv_res_pair_g) ----
  s16x8 wf[NCH][2][2];
  // buffer loads: the lane offsets are loop-invariant VGPRs, the tap base a scalar resource and the
  // chunk / column-block offsets scalar constants, so a reload costs no address arithmetic
  const int wo0 = ((2 * wc) * 16 + l15) * 96 + hf * 48 + t * 16, wo1 = ((2 * wc) * 16 + l15) * 96 + hf * 48 + (t ? 32 : 0);
  auto load_wf = [&](const unsigned short* wtap, int ch) {
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)wtap, 0, WTAP, 0x00020000);
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      const int so = (ch * C + cb * 16) * 96;
      wf[ch][cb][0] = __builtin_bit_cast(s16x8, __builtin_amdgcn_raw_buffer_load_b128(rw, wo0, so, 0));
      wf[ch][cb][1] = __builtin_bit_cast(s16x8, __builtin_amdgcn_raw_buffer_load_b128(rw, wo1, so, 0));
    }
  };
  auto next_tap = [&](int m, int conv, int j) -> const unsigned short* {
    if (j + 1 < p.taps[m]) return (conv ? p.w2[m] : p.w1[m]) + (long long)(j + 1) * (WTAP / 2);
    if (conv == 0) return p.w2[m];
    return p.w1[m + 1 < nmem ? m + 1 : 0];
  };
  // lane parts of the three activation reads (piece, row within the 16-row block); a tap adds its
  // wave-uniform row offset once, and row block / chunk offsets are instruction immediates
  const int pk0 = ((hf * 3 + t) * NS + l15) * 16, pk1 = ((hf * 3 + (t ? 0 : 1)) * NS + l15) * 16;
  const int pk2 = ((hf * 3 + (t ? 0 : 2)) * NS + l15) * 16;
  auto tap = [&](f32x4 (&acc)[RB][2], int rowoff, int nrb, const unsigned short* wnext) {
    const int tb = (wr * 16 + rowoff) * 16;
    const char *xb0 = lds + pk0 + tb, *xb1 = lds + pk1 + tb, *xb2 = lds + pk2 + tb;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
#pragma unroll
      for (int i = 0; i < RB; ++i) {
        if (i < nrb) {
          const int io = (WR * 16 * i) * 16 + ch * 6 * PS;
          const s16x8 x2 = *reinterpret_cast<const s16x8*>(xb2 + io);
          const s16x8 x1 = *reinterpret_cast<const s16x8*>(xb1 + io);
          const s16x8 x0 = *reinterpret_cast<const s16x8*>(xb0 + io);
#pragma unroll
          for (int cb = 0; cb < 2; ++cb) {
            acc[i][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wf[ch][cb][1]),
                                                                 __builtin_bit_cast(bf16x8, x2), acc[i][cb], 0, 0, 0);
            acc[i][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wf[ch][cb][0]),
                                                                 __builtin_bit_cast(bf16x8, x1), acc[i][cb], 0, 0, 0);
            acc[i][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wf[ch][cb][0]),
                                                                 __builtin_bit_cast(bf16x8, x0), acc[i][cb], 0, 0, 0);
          }
        }
      }
      load_wf(wnext, ch);
      __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_s_setprio(0);
  };

  const int nrb2 = min(RB, (G::NB2 - wr + WR - 1) / WR);
  int tile = blockIdx.x;
  if (tile >= total) return;  // whole workgroup, before any barrier
  int b = tile / ntl, r0 = (tile - b * ntl) * R;
  for (int i = tid; i < 2 * nmem * C; i += 256) {
    const int conv = i / (nmem * C), m = (i / C) % nmem, c = i % C;
    bias_lds[(conv * kMaxGroup + m) * C + c] = (conv ? p.b2[m] : p.b1[m])[c];
  }
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) load_wf(p.w1[0], ch);
  f32x4 macc[MEAN ? RB : 1][2];
  for (;;) {
    const int next_tile = tile + gridDim.x;
    const bool more = next_tile < total;
    const long long cb0 = (long long)b * p.bstride;
    for (int m = 0; m < nmem; ++m) {
      const int k = p.taps[m], hk = (k - 1) >> 1, d = p.dil[m];
      const bool last_m = m + 1 == nmem;
      fill(p.src[m] + cb0, r0, hk * d);
      rp_barrier();
      // ---- c1 over rows [r0 - 8, r0 + R + 8) from the S image
      f32x4 acc[RB][2];
#pragma unroll
      for (int i = 0; i < RB; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int j = 0; j < k; ++j) tap(acc, G::H1 + (j - hk) * d, RB, next_tap(m, 0, j));
      rp_barrier();  // every wave's S reads are done before T overwrites them
      // ---- T image: silu(c1 + b1) planes over the S image (zero outside the clip)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const int c0 = (2 * wc + cb) * 16 + 4 * (lane >> 4);
        const f32x4 bias = *reinterpret_cast<const f32x4*>(bias_lds + m * C + c0);
#pragma unroll
        for (int i = 0; i < RB; ++i) {
          const int ir = (wr + WR * i) * 16 + l15, a = r0 - 8 + ir;
          const bool ok = a >= 0 && a < L;
          s16x4 hv, mv, lv;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float sv = rp_silu(acc[i][cb][e] + bias[e]);
            const float v = ok ? sv : 0.f;
            unsigned short h, mm, l;
            split3(v, h, mm, l);
            hv[e] = (short)h;
            mv[e] = (short)mm;
            lv[e] = (short)l;
          }
          char* dst = lds + ((c0 >> 4) * 6 + ((c0 >> 3) & 1) * 3) * PS + ir * 16 + (c0 & 7) * 2;
          *reinterpret_cast<s16x4*>(dst) = hv;
          *reinterpret_cast<s16x4*>(dst + PS) = mv;
          *reinterpret_cast<s16x4*>(dst + 2 * PS) = lv;
        }
      }
      rp_barrier();
      // ---- c2 over rows [r0, r0 + R) from the T image; the residual rows are loaded after tap 0's
      // fragment reloads
#pragma unroll
      for (int i = 0; i < RB; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      f32x4 res[RB][2];
      tap(acc, 8 - hk, nrb2, next_tap(m, 1, 0));
#pragma unroll
      for (int i = 0; i < RB; ++i) {
        const int q = min(r0 + (wr + WR * i) * 16 + l15, L - 1);
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          const int c0 = (2 * wc + cb) * 16 + 4 * (lane >> 4);
          res[i][cb] = *reinterpret_cast<const f32x4*>(p.src[m] + cb0 + (long long)q * C + c0);
        }
      }
      for (int j = 1; j < k; ++j) tap(acc, 8 + j - hk, nrb2, next_tap(m, 1, j));
      // ---- epilogue: state + c2 + b2 (rows past the clip end are dropped)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const int c0 = (2 * wc + cb) * 16 + 4 * (lane >> 4);
        const f32x4 bias = *reinterpret_cast<const f32x4*>(bias_lds + (kMaxGroup + m) * C + c0);
#pragma unroll
        for (int i = 0; i < RB; ++i) {
          if (i >= nrb2) break;
          const int q = r0 + (wr + WR * i) * 16 + l15;
          const f32x4 v = res[i][cb] + (acc[i][cb] + bias);
          if constexpr (!MEAN) {
            if (q < L) *reinterpret_cast<f32x4*>(p.dst[m] + cb0 + (long long)q * C + c0) = v;
          } else if (m == 0) {
            macc[i][cb] = v;
          } else if (!last_m) {
            macc[i][cb] = macc[i][cb] + v;
          } else {
            const f32x4 mv = (macc[i][cb] + v) / 3.0f;
            f32x4 sv;
#pragma unroll
            for (int e = 0; e < 4; ++e) sv[e] = rp_silu(mv[e]);
            if (q < L) *reinterpret_cast<f32x4*>(p.mean_out + cb0 + (long long)q * C + c0) = sv;
          }
        }
      }
      rp_barrier();  // every wave's T reads are done before the next S image overwrites them
    }
    if (!more) break;
    tile = next_tile;
    b = tile / ntl;
    r0 = (tile - b * ntl) * R;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last tap's (unused) fragment reloads
}

#ifdef RP_DIAG_STAMPS
extern "C" int dcx_diag_rp(unsigned long long* out32, int reset) {
  if (hipMemcpyFromSymbol(out32, HIP_SYMBOL(g_rp_diag), sizeof(unsigned long long) * 32) != hipSuccess) return -1;
  if (reset) {
    const unsigned long long z[32] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_rp_diag), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}
#endif

hipError_t launch_res_pair(const ResPairParams& p, hipStream_t s, const char** kname) {
  if (p.nmem < 1 || p.nmem > kMaxGroup || p.batch < 1 || p.L < 1 || (p.C != 32 && p.C != 64))
    return hipErrorInvalidValue;
  for (int m = 0; m < p.nmem; ++m) {
    const int hk = (p.taps[m] - 1) / 2;
    if (p.taps[m] < 1 || p.taps[m] % 2 == 0 || hk > 8 || p.dil[m] < 1 || hk * p.dil[m] > 32 || !p.src[m] ||
        !p.w1[m] || !p.w2[m] || !p.b1[m] || !p.b2[m] || (!p.mean_out && !p.dst[m]))
      return hipErrorInvalidValue;
  }
  static const Knobs kDefault{};
  const Knobs& kn = p.kn ? *p.kn : kDefault;
  const int cus = device_cus();
  // C = 32: the barrier-free conv_res_pair_g, C = 64: the step schedule; Knobs (A/B and
  // tests): rp_old runs the step schedule at C = 32 too, rp_g64 the barrier-free kernel at C = 64,
  // rp_w4 conv_res_pair_w4 (two 4-wave workgroups per CU: same bits, measured 2-6 % slower)
  const bool w4 = kn.rp_w4 && !kn.rp_old && !kn.rp_g64 && !p.h3;
  const int slots = w4 ? 2 * cus : cus;
  // rows per tile: the default unless a smaller tile finishes the launch sooner, by rounds of tiles
  // over the workgroup slots times a tile's rows (c1 rows R + 16, c2 rows R, ~64 rows' worth of fixed
  // cost); Knobs::rp_rows forces one of the instantiated sizes.  Every size gives the same bits.
  static constexpr int kW8_32[3] = {496, 240, 112}, kW8_64[3] = {176, 112, 48};
  static constexpr int kH3_32[3] = {624, 240, 112}, kH3_64[3] = {240, 112, 48};
  static constexpr int kW4_32[3] = {304, 112, 48}, kW4_64[3] = {112, 48, 48};
  const int* sizes = p.h3 ? (p.C == 32 ? kH3_32 : kH3_64)
                     : w4 ? (p.C == 32 ? kW4_32 : kW4_64) : (p.C == 32 ? kW8_32 : kW8_64);
  int si = 0;
  long long best = -1;
  for (int i = 0; i < 3; ++i) {
    const int r = sizes[i];
    const long long tiles = (long long)((p.L + r - 1) / r) * p.batch;
    const long long cost = (tiles + slots - 1) / slots * (2LL * r + 16 + 64);
    if (best < 0 || cost < best) {
      best = cost;
      si = i;
    }
  }
  for (int i = 0; i < 3; ++i)
    if (kn.rp_rows && sizes[i] == kn.rp_rows) si = i;
  const int R = sizes[si];
  const long long total = (long long)((p.L + R - 1) / R) * p.batch;
  if (total > (1LL << 30)) return hipErrorInvalidValue;
  const unsigned grid = (unsigned)std::min<long long>(total, slots);  // resident workgroups (LDS)
  ResPairParams q = p;
  q.tap_sync = std::max(0, kn.rp_sync);
  const bool mean = p.mean_out != nullptr;
  // profile names are string literals (no shared buffer between threads)
#define DCX_RP_GO(KERN, CC, RR, NAME, ...)                                                  \
  do {                                                                                      \
    if (kname) *kname = mean ? #KERN "<" #CC ",mean" NAME ">" : #KERN "<" #CC NAME ">";     \
    if (mean) hipLaunchKernelGGL((KERN<CC, true, RR __VA_ARGS__>), dim3(grid), dim3(w4 ? 256 : 512), 0, s, q);   \
    else hipLaunchKernelGGL((KERN<CC, false, RR __VA_ARGS__>), dim3(grid), dim3(w4 ? 256 : 512), 0, s, q);       \
  } while (0)
#define DCX_RP_SIZES(KERN, CC, R0, R1, R2, ...)                \
  do {                                                         \
    if (si == 0) DCX_RP_GO(KERN, CC, R0, "" __VA_ARGS__);                  \
    else if (si == 1) DCX_RP_GO(KERN, CC, R1, ",small" __VA_ARGS__);       \
    else DCX_RP_GO(KERN, CC, R2, ",small" __VA_ARGS__);                    \
  } while (0)
  bool ring_ok = kn.rp_ring != 0;  // the ring kernel reads every member's src_amax unconditionally
  for (int m = 0; m < p.nmem; ++m) ring_ok = ring_ok && p.src_amax[m];
  if (p.h3 && ring_ok) {  // h3 weights, the LDS weight ring (round 6, default)
    if (p.C == 32) DCX_RP_SIZES(conv_res_pair_h3, 32, 624, 240, 112, ",ring", , true);
    else DCX_RP_SIZES(conv_res_pair_h3, 64, 240, 112, 48, ",ring", , true);
  } else if (p.h3) {  // h3 weights: conv_res_pair_h3 (the barrier-free schedule at both widths)
    if (p.C == 32) DCX_RP_SIZES(conv_res_pair_h3, 32, 624, 240, 112);
    else DCX_RP_SIZES(conv_res_pair_h3, 64, 240, 112, 48);
  } else if (w4) {
    if (p.C == 32) DCX_RP_SIZES(conv_res_pair_w4, 32, 304, 112, 48);
    else DCX_RP_SIZES(conv_res_pair_w4, 64, 112, 48, 48);
  } else if (p.C == 32 && !kn.rp_old) {
    DCX_RP_SIZES(conv_res_pair_g, 32, 496, 240, 112);
  } else if (p.C == 64 && !kn.rp_old && kn.rp_g64) {
    DCX_RP_SIZES(conv_res_pair_g, 64, 176, 112, 48);
  } else if (p.C == 32) {
    DCX_RP_SIZES(conv_res_pair, 32, 496, 240, 112);
  } else {
    DCX_RP_SIZES(conv_res_pair, 64, 176, 112, 48);
  }
#undef DCX_RP_SIZES
#undef DCX_RP_GO
  return hipGetLastError();
}

}  // namespace dcx

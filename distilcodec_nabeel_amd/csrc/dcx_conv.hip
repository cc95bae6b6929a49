// Implicit-GEMM 1-D convolution on gfx950 fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// One kernel family serves every contraction on the DistilCodec path:
//   Conv1d k>1 / dilated (stem k7, conv_pre k13, ResBlock1 k3/7/11 x dil 1/3/5),
//   1x1 convs and nn.Linear (taps = 1), ConvTranspose1d as `stride` polyphase convs
//   (phase = blockIdx.z), the STFT as a 4-tap conv over 256-sample rows, the mel matmul,
//   and the VQ distance GEMM (argmin epilogue, never materialising rows x 32768).
//
// GEMM view: rows = output time positions q (M), cols = output channels (N),
// K = taps x Cin.  Channels-last activations make every A-tile row a contiguous Cin slice and
// every store a contiguous Cout slice (coalesced); the weight tile is [Cout][taps*Cin].
//
// MFMA fragment maps (cdna_hip_programming.md §3): for 32x32x2 f32, lane l supplies
// A[i=l&31][k=l>>5] and B[k=l>>5][j=l&31]; C/D: col=l&31, row=(r&3)+8*(r>>2)+4*(l>>5).
// Within each 16-deep K chunk, lane half h owns k = 8h..8h+7 (k-step s uses k = 8h+s), so a
// fragment is two ds_read_b128 of 8 consecutive k.  LDS rows are padded to 20 floats, which
// makes those reads conflict-free (20*i mod 64 distinct over every 16-lane b128 group).
//
// Pipeline: register-staged double buffer, one barrier per K chunk: the global loads for chunk
// k+1 are issued before the MFMAs of chunk k and written to the other LDS buffer after them.
#include "dcx_kernels.h"

namespace dcx {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int BK = 16;    // K chunk per pipeline stage
constexpr int LDSK = 20;  // padded LDS row (floats)

__device__ __forceinline__ float silu_f(float v) { return v / (1.0f + expf(-v)); }
__device__ __forceinline__ float gelu_f(float v) { return 0.5f * v * (1.0f + erff(v * 0.70710678118654752440f)); }

// XCD-aware bijective block remap (cdna_hip_programming.md §5 "XCD swizzle must be bijective"):
// blocks b and b+8 share an XCD, so consecutive logical tiles (same row panel, all column
// tiles) are dealt to the same XCD and share its L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

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
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = wg / ntiles, nt = wg - mt * ntiles;
  const int q0 = mt * BM, co0 = nt * BN;
  const int b = blockIdx.y, ph = blockIdx.z;
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

  const int rhalf = 4 * (lane >> 5);
  if constexpr (!ARGMIN) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int co = co0 + wn * WC + j * 32 + lrow;
        const float bias = p.bias ? p.bias[co] : 0.f;
        const float gam = (p.epi == EPI_GAMMA_RES) ? p.gamma[co] : 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int q = q0 + wm * WR + i * 32 + (r & 3) + 8 * (r >> 2) + rhalf;
          if (q >= p.Lq) continue;
          const long long o = (long long)b * p.y_bstride + (long long)(q * p.out_mul + ph) * p.ldy + co;
          float v = acc[i][j][r] + bias;
          switch (p.epi) {
            case EPI_GELU: v = gelu_f(v); break;
            case EPI_GAMMA_RES: v = p.res[o] + gam * v; break;
            case EPI_RES: v = p.res[o] + v; break;
            case EPI_LOGCLAMP: v = logf(fmaxf(v, 1e-5f)); break;
            default: break;
          }
          if (p.mean_mode == MEAN_FIRST) {
            p.macc[o] = v;
            continue;
          } else if (p.mean_mode == MEAN_MID) {
            p.macc[o] = p.macc[o] + v;
            continue;
          } else if (p.mean_mode == MEAN_LAST) {
            v = (p.macc[o] + v) / 3.0f;
          }
          if (p.y) p.y[o] = v;
          if (p.y2) p.y2[o] = silu_f(v);
        }
      }
  } else {
    // VQ search epilogue: dist = sqrt(clamp((|x|^2 + |e|^2) + (-2 x.e), 0)) exactly in the
    // reference's operation order (vector_quantize_pytorch.py:41-45); per row keep the
    // smallest distance, lowest code index on ties (torch argmax of -dist returns the first).
    __syncthreads();
    float* rv = smem;                                        // [WN][BM]
    int* ri = reinterpret_cast<int*>(smem + WN * BM);        // [WN][BM]
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

template <int BM, int BN, int WM, int WN, bool ARGMIN>
static hipError_t launch_tile(const ConvParams& p, int batch, int phases, hipStream_t s) {
  const int mtiles = (p.Lq + BM - 1) / BM;
  const int ntiles = p.Cout / BN;
  dim3 grid(mtiles * ntiles, batch, phases);
  hipLaunchKernelGGL((conv_gemm_f32<BM, BN, WM, WN, ARGMIN>), grid, dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_conv(const ConvParams& p, int batch, int phases, hipStream_t s, const char** kname) {
  if (p.Cin % BK || p.Cout % 32 || phases < 1 || phases > kMaxPhases) return hipErrorInvalidValue;
  if (p.Cout % 128 == 0) {
    if (kname) *kname = "conv_gemm_f32<128,128>";
    return launch_tile<128, 128, 2, 2, false>(p, batch, phases, s);
  }
  if (p.Cout % 64 == 0) {
    if (kname) *kname = "conv_gemm_f32<256,64>";
    return launch_tile<256, 64, 4, 1, false>(p, batch, phases, s);
  }
  if (kname) *kname = "conv_gemm_f32<256,32>";
  return launch_tile<256, 32, 4, 1, false>(p, batch, phases, s);
}

int vq_argmin_ntiles(int ncodes) { return ncodes / 128; }

hipError_t launch_vq_argmin(const ConvParams& p, int rows, hipStream_t s, const char** kname) {
  if (p.Cin % BK || p.Cout % 128) return hipErrorInvalidValue;
  if (kname) *kname = "vq_dist_argmin_f32<128,128>";
  ConvParams q = p;
  q.Lq = rows;
  q.Lin = rows;
  return launch_tile<128, 128, 2, 2, true>(q, 1, 1, s);
}

}  // namespace dcx

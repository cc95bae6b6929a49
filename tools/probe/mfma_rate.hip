// Microbenchmark: issue cycles per MFMA for the fp16 / bf16 16x16 shapes on gfx950 (one wave per
// SIMD, 4 independent accumulators, back to back).  Build: hipcc -O3 --offload-arch=gfx950 mfma_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

template <int KIND>
__global__ void __launch_bounds__(256) k(float* out, unsigned long long* cyc, int iters) {
  const int lane = threadIdx.x & 63;
  f16x8 a8, b8;
  f16x4 a4, b4;
  bf16x8 c8, d8;
  for (int i = 0; i < 8; ++i) { a8[i] = (_Float16)(0.001f * (lane + i)); b8[i] = (_Float16)(0.002f * (lane - i)); c8[i] = (__bf16)(0.001f * (lane + i)); d8[i] = (__bf16)(0.003f * i); }
  for (int i = 0; i < 4; ++i) { a4[i] = a8[i]; b4[i] = b8[i]; }
  f32x4 acc0 = {0, 0, 0, 0}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if constexpr (KIND == 0) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(c8, d8, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(c8, d8, acc1, 0, 0, 0);
        acc2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(c8, d8, acc2, 0, 0, 0);
        acc3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(c8, d8, acc3, 0, 0, 0);
      } else if constexpr (KIND == 1) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, acc1, 0, 0, 0);
        acc2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, acc2, 0, 0, 0);
        acc3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, acc3, 0, 0, 0);
      } else if constexpr (KIND == 2) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, acc1, 0, 0, 0);
        acc2 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, acc2, 0, 0, 0);
        acc3 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, acc3, 0, 0, 0);
      } else {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s16x4, a4), __builtin_bit_cast(s16x4, b4), acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s16x4, a4), __builtin_bit_cast(s16x4, b4), acc1, 0, 0, 0);
        acc2 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s16x4, a4), __builtin_bit_cast(s16x4, b4), acc2, 0, 0, 0);
        acc3 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s16x4, a4), __builtin_bit_cast(s16x4, b4), acc3, 0, 0, 0);
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 256 + threadIdx.x] = acc0[0] + acc1[1] + acc2[2] + acc3[3];
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, 1024 * 256 * sizeof(float));
  hipMalloc(&cyc, 1024 * sizeof(unsigned long long));
  const char* names[4] = {"16x16x32_bf16", "16x16x32_f16", "16x16x16_f16", "16x16x16_bf16_1k"};
  const int iters = 4096;
  for (int rep = 0; rep < 2; ++rep)
    for (int kind = 0; kind < 4; ++kind) {
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      auto launch = [&] {
        if (kind == 0) hipLaunchKernelGGL(k<0>, dim3(256), dim3(256), 0, 0, out, cyc, iters);
        if (kind == 1) hipLaunchKernelGGL(k<1>, dim3(256), dim3(256), 0, 0, out, cyc, iters);
        if (kind == 2) hipLaunchKernelGGL(k<2>, dim3(256), dim3(256), 0, 0, out, cyc, iters);
        if (kind == 3) hipLaunchKernelGGL(k<3>, dim3(256), dim3(256), 0, 0, out, cyc, iters);
      };
      launch();
      hipEventRecord(e0);
      launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      unsigned long long c;
      hipMemcpy(&c, cyc, sizeof c, hipMemcpyDeviceToHost);
      const double n = 32.0 * iters;  // MFMAs per wave
      const double macs = kind < 2 ? 16 * 16 * 32 : 16 * 16 * 16;
      printf("%-18s %6.2f cycles/MFMA/wave (1 wave per SIMD)  chip %.0f TF\n", names[kind], c / n,
             2.0 * macs * n * 4 * 256 / (ms * 1e-3) / 1e12);
    }
  return 0;
}

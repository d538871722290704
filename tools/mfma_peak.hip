// Calibration: sustained v_mfma_f32_32x32x16_bf16 / 16x16x32 rate with register-only operands,
// every CU busy, 1 or 2 waves per SIMD (cdna_hip_programming.md §5.4 rule 25: measure the roof).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_peak tools/mfma_peak.hip && /tmp/mfma_peak
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int ACC>
__global__ void __launch_bounds__(256) k32(float* out, int iters) {
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (__bf16)(threadIdx.x * 0.001f + i); b[i] = (__bf16)(i * 0.5f); }
  f32x16 c[ACC];
  for (int j = 0; j < ACC; ++j)
    for (int r = 0; r < 16; ++r) c[j][r] = 0.f;
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int j = 0; j < ACC; ++j) c[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c[j], 0, 0, 0);
  float s = 0.f;
  for (int j = 0; j < ACC; ++j)
    for (int r = 0; r < 16; ++r) s += c[j][r];
  if (s == 1234.5f) out[threadIdx.x] = s;
}

// same with an s_barrier every BAR iterations (4 MFMAs per iteration per wave)
template <int BAR>
__global__ void __launch_bounds__(256) k32bar(float* out, int iters) {
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (__bf16)(threadIdx.x * 0.001f + i); b[i] = (__bf16)(i * 0.5f); }
  f32x16 c0, c1, c2, c3;
  for (int r = 0; r < 16; ++r) { c0[r] = 0.f; c1[r] = 0.f; c2[r] = 0.f; c3[r] = 0.f; }
  for (int it = 0; it < iters; ++it) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c3, 0, 0, 0);
    if (BAR > 0 && (it % BAR) == BAR - 1) __builtin_amdgcn_s_barrier();
  }
  float s = 0.f;
  for (int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
  if (s == 1234.5f) out[threadIdx.x] = s;
}

template <int ACC>
__global__ void __launch_bounds__(256) k16(float* out, int iters) {
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (__bf16)(threadIdx.x * 0.001f + i); b[i] = (__bf16)(i * 0.5f); }
  f32x4 c[ACC];
  for (int j = 0; j < ACC; ++j) c[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int j = 0; j < ACC; ++j) c[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c[j], 0, 0, 0);
  float s = 0.f;
  for (int j = 0; j < ACC; ++j)
    for (int r = 0; r < 4; ++r) s += c[j][r];
  if (s == 1234.5f) out[threadIdx.x] = s;
}

template <typename K>
void run(const char* name, K kern, int wgs_per_cu, int flop_per_mfma, int acc, int iters = 4000, int nwg = 0) {
  float* out;
  hipMalloc(&out, 1024 * sizeof(float));
  const int cus = 256;
  dim3 grid(nwg ? nwg : cus * wgs_per_cu), block(256);
  hipLaunchKernelGGL(kern, grid, block, 0, 0, out, 100);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, grid, block, 0, 0, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double flop = 5.0 * grid.x * 4.0 /*waves*/ * iters * acc * (double)flop_per_mfma;
  printf("%-10s waves/SIMD=%d  %.1f TFLOP/s  (%.3f ms)\n", name, wgs_per_cu, flop / (ms * 1e-3) / 1e12, ms / 5);
  hipFree(out);
}

int main() {
  run("32x32x16", k32<4>, 1, 32 * 32 * 16 * 2, 4);
  run("32x32x16", k32<4>, 2, 32 * 32 * 16 * 2, 4);
  run("bar/4mfma", k32bar<1>, 2, 32 * 32 * 16 * 2, 4);
  run("bar/16mfma", k32bar<4>, 2, 32 * 32 * 16 * 2, 4);
  run("bar/64mfma", k32bar<16>, 2, 32 * 32 * 16 * 2, 4);
  run("bar/16mfma", k32bar<4>, 1, 32 * 32 * 16 * 2, 4);
  // attention-like: 3840 short workgroups of 4 waves, 67 x 4 MFMAs each, barrier every 16
  run("short-wg", k32bar<4>, 2, 32 * 32 * 16 * 2, 4, 67, 3840);
  run("long-wg", k32bar<4>, 2, 32 * 32 * 16 * 2, 4, 67 * 15, 256 * 2);
  return 0;
}

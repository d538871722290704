// Exhaustive check over all 65536 bf16 inputs x: do the hardware forms (v_exp_f32 + v_rcp_f32) round to
// the same bf16 as the precise fp32 forms (expf + IEEE division) the reference's bf16 ops compute in fp32?
//   sigmoid(x)  — attention.hip attn_pack_out: rbf(sigmoid(gate)), gate a bf16 value (model.py:157,264)
//   silu(x)     — gemm.hip SwiGLU epilogue: rbf(silu(a)), a = rbf(acc) (model.py:307-308)
// hipcc -O3 -ffp-contract=off --offload-arch=gfx950 tools/sigmoid_exhaustive.hip -o tools/sigmoid_exhaustive.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cmath>
#include <cstring>
#include <vector>

__device__ __forceinline__ float bf2f(uint32_t b) { return __uint_as_float(b << 16); }
__device__ __forceinline__ uint32_t f2bf(float f) {  // RNE, as v_cvt_pk_bf16_f32 for finite values
  const uint32_t u = __float_as_uint(f);
  return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}
// out[f][b] = (precise bf16) | (hardware bf16) << 16 for every input bit pattern b (plain vector stores)
__global__ void check(uint32_t* out) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= 65536u) return;
  const float x = bf2f(b);
  const float sp = 1.0f / (1.0f + expf(-x));
  const float sh = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * -1.44269504088896341f));
  out[b] = f2bf(sp) | (f2bf(sh) << 16);
  const float up = x / (1.0f + expf(-x));  // F.silu in fp32
  const float uh = x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * -1.44269504088896341f));
  out[65536 + b] = f2bf(up) | (f2bf(uh) << 16);
}
int main() {
  uint32_t* d;
  if (hipMalloc(&d, 2 * 65536 * 4) != hipSuccess) return 2;
  hipLaunchKernelGGL(check, dim3(256), dim3(256), 0, 0, d);
  std::vector<uint32_t> h(2 * 65536);
  if (hipMemcpy(h.data(), d, 2 * 65536 * 4, hipMemcpyDeviceToHost) != hipSuccess) return 2;
  const char* names[2] = {"sigmoid", "silu"};
  for (int fn = 0; fn < 2; ++fn) {
    unsigned n = 0, nan_in = 0;
    for (uint32_t b = 0; b < 65536u; ++b) {
      uint32_t u = b << 16; float f; memcpy(&f, &u, 4);
      if (f != f) { ++nan_in; continue; }
      const uint32_t v = h[fn * 65536 + b];
      if ((v & 0xffffu) != (v >> 16)) {
        if (n < 32) printf("  %s 0x%04x (%g): precise 0x%04x hw 0x%04x\n", names[fn], b, f, v & 0xffffu, v >> 16);
        ++n;
      }
    }
    printf("%s: mismatching non-NaN bf16 inputs: %u of %u\n", names[fn], n, 65536u - nan_in);
  }
  hipFree(d);
  return 0;
}

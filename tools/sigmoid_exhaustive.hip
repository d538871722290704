// Exhaustive check over all 65536 bf16 inputs x: do the production hardware forms (common.h; v_exp_f32 +
// v_rcp_f32) round to the same bf16 as the precise fp32 forms (expf + IEEE division) the reference's bf16
// ops compute in fp32?
//   sigmoid(x)  — attention.hip attn_pack_out: rbf(sigmoid(gate)), gate a bf16 value (model.py:157,264);
//                 production takes sigmoid_f for x < -87 (checked here as "sigmoid+fallback")
//   silu(x)     — gemm.hip SwiGLU epilogue: rbf(silu_bf16in(a)), a = rbf(acc) (model.py:307-308)
// hipcc -O3 -ffp-contract=off --offload-arch=gfx950 tools/sigmoid_exhaustive.hip -o tools/sigmoid_exhaustive.bin
#include "../echo-tts_amd/csrc/common.h"

#include <cstdio>
#include <cstring>
#include <vector>

// out[f][b] = (precise bf16) | (production bf16) << 16 for every input bit pattern b (plain vector stores)
__global__ void check(uint32_t* out) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= 65536u) return;
  const float x = bf2f(b);
  const float sp = sigmoid_f(x);
  out[b] = f2bf(sp) | ((uint32_t)f2bf(sigmoid_hw(x)) << 16);
  out[65536 + b] = f2bf(sp) | ((uint32_t)f2bf(x < -87.0f ? sigmoid_f(x) : sigmoid_hw(x)) << 16);
  out[2 * 65536 + b] = f2bf(silu_f(x)) | ((uint32_t)f2bf(silu_bf16in(x)) << 16);
}

int main() {
  uint32_t* d;
  if (hipMalloc(&d, 3 * 65536 * 4) != hipSuccess) return 2;
  hipLaunchKernelGGL(check, dim3(256), dim3(256), 0, 0, d);
  std::vector<uint32_t> h(3 * 65536);
  if (hipMemcpy(h.data(), d, 3 * 65536 * 4, hipMemcpyDeviceToHost) != hipSuccess) return 2;
  const char* names[3] = {"sigmoid_hw", "sigmoid_hw+fallback", "silu_bf16in"};
  int bad = 0;
  for (int fn = 0; fn < 3; ++fn) {
    unsigned n = 0, nan_in = 0;
    for (uint32_t b = 0; b < 65536u; ++b) {
      uint32_t u = b << 16;
      float f;
      memcpy(&f, &u, 4);
      if (f != f) { ++nan_in; continue; }
      const uint32_t v = h[fn * 65536 + b];
      if ((v & 0xffffu) != (v >> 16)) {
        if (n < 32) printf("  %s 0x%04x (%g): precise 0x%04x production 0x%04x\n", names[fn], b, f, v & 0xffffu, v >> 16);
        ++n;
      }
    }
    printf("%s: mismatching non-NaN bf16 inputs: %u of %u\n", names[fn], n, 65536u - nan_in);
    if (fn > 0 && n) bad = 1;
  }
  hipFree(d);
  return bad;
}

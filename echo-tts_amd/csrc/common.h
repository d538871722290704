// Shared device helpers for the gfx950 kernels: bf16 storage, rounding, vector types.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/echo_hip.h"

typedef uint16_t bf16_t;  // bfloat16 storage (no arithmetic on it)
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

__device__ __forceinline__ float bf2f(uint32_t u16) { return __uint_as_float(u16 << 16); }

// Round-to-nearest-even fp32 -> bf16 (hardware v_cvt_pk_bf16_f32; NaN stays NaN).
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}
__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}
__device__ __forceinline__ float rbf(float f) { return bf2f(f2bf(f)); }

// Element-type traits: rounding points of the reference's dtype contract.
template <typename T> struct Elt;
template <> struct Elt<bf16_t> {
  static __device__ __forceinline__ float ld(const bf16_t* p) { return bf2f(*p); }
  static __device__ __forceinline__ void st(bf16_t* p, float v) { *p = f2bf(v); }
  static __device__ __forceinline__ float rnd(float v) { return rbf(v); }
  static constexpr int bytes = 2;
};
template <> struct Elt<float> {
  static __device__ __forceinline__ float ld(const float* p) { return *p; }
  static __device__ __forceinline__ void st(float* p, float v) { *p = v; }
  static __device__ __forceinline__ float rnd(float v) { return v; }
  static constexpr int bytes = 4;
};

// Load/store 8 consecutive elements as fp32 (16 B for bf16, 2x16 B for fp32).
__device__ __forceinline__ void load8(const bf16_t* p, float* o) {
  uint4 u = *(const uint4*)p;
  uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) { o[2 * i] = bf2f(w[i] & 0xffffu); o[2 * i + 1] = bf2f(w[i] >> 16); }
}
__device__ __forceinline__ void load8(const float* p, float* o) {
  float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}
__device__ __forceinline__ void store8(bf16_t* p, const float* v) {
  uint4 u;
  u.x = pack2bf(v[0], v[1]); u.y = pack2bf(v[2], v[3]); u.z = pack2bf(v[4], v[5]); u.w = pack2bf(v[6], v[7]);
  *(uint4*)p = u;
}
__device__ __forceinline__ void store8(float* p, const float* v) {
  *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
  *(float4*)(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}

// Correctly rounded elementwise helpers that the compiler must not contract.
__device__ __forceinline__ float silu_f(float v) { return v / (1.0f + expf(-v)); }
__device__ __forceinline__ float sigmoid_f(float v) { return 1.0f / (1.0f + expf(-v)); }

// Hardware-op forms of sigmoid / SiLU for bf16 INPUTS (v_exp_f32 + v_rcp_f32 instead of expf + IEEE
// division), each checked over all 65536 bf16 inputs on MI355X against the precise fp32 form the
// reference's bf16 ops compute (tools/sigmoid_exhaustive.hip includes this header, so it tests these
// exact functions; profiles/r3_sigmoid_exhaustive.txt).
//
// sigmoid_hw (attention gate, model.py:157,264): rounded to bf16 it equals the rounded precise
// sigmoid for every input except x = -87.5, -88, -88.5, whose sigmoids are fp32 denormals that
// v_rcp_f32 flushes to 0. Callers take the precise path for x < -87 (a wave-uniform rare branch).
__device__ __forceinline__ float sigmoid_hw(float v) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(v * -1.44269504088896341f));
}
// silu_bf16in (SwiGLU epilogue, model.py:307): rbf(silu_bf16in(a)) == rbf(a / (1 + expf(-a))) for
// every bf16 a, by two fix-ups of the hardware form a * rcp(1 + 2^(-a log2 e)):
//  * a < -64: numerator and divisor are scaled by 2^-32 (exact) so that the reciprocal of the huge
//    1 + e^-a stays normal — otherwise v_rcp_f32 flushes it and a in {-87.5, -88, -88.5}, whose
//    SiLUs are normal numbers (~-8.7e-37), come out as -0;
//  * a = 5.9375: its fp32 SiLU, 5.9218745, lies one fp32 ulp below the bf16 rounding midpoint
//    5.921875 that the ~2-ulp hardware form crosses; the exact bf16 result 5.90625 is selected.
__device__ __forceinline__ float silu_bf16in(float a) {
  const float sc = a < -64.0f ? 0x1p-32f : 1.0f;
  const float d = 1.0f + __builtin_amdgcn_exp2f(a * -1.44269504088896341f);
  const float s = (a * sc) * __builtin_amdgcn_rcpf(d * sc);
  return a == 5.9375f ? 5.90625f : s;
}

// ---- in-launch hand-offs between workgroups of one launch (cdna_hip_programming.md Guideline 16: write-through
// (sc1) payload stores drained by every storing wave, one relaxed agent-scope arrival per workgroup, a relaxed
// bounded poll, ONE agent-scope acquire) over the caller-owned counter buffer of echo_set_sync_buffer: word 0 is
// the error flag (a bounded poll gave up: never in a correct run), the [arrivals, departures] pairs start at
// word 16. Every workgroup that waits must be resident at once: the host launches these forms only for grids of
// at most one workgroup per CU.
constexpr int SYNC_ERR = 0, SYNC_CNT0 = 16;
extern uint32_t* g_sync;      // echo_set_sync_buffer (attention.hip); NULL = in-launch hand-offs off
extern int64_t g_sync_words;
// ONE lane, after every storing wave's s_waitcnt vmcnt(0) and a workgroup barrier; the workgroup joins another
// barrier after it before any load of the handed-off bytes
__device__ __forceinline__ void sync_arrive_wait(uint32_t* sync, uint32_t* cnt, uint32_t expect) {
  __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint32_t spins = 0;
  while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < expect) {
    __builtin_amdgcn_s_sleep(2);
    if (++spins == (1u << 22)) {  // bounded: never hang the GPU
      __hip_atomic_store(sync + SYNC_ERR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
// ONE lane of a workgroup that passed sync_arrive_wait on `cnt`: the last of the n departures finds every
// waiter past its poll and re-zeroes the pair (the buffer is zero again when the launch ends)
__device__ __forceinline__ void sync_depart(uint32_t* cnt, uint32_t n) {
  if (__hip_atomic_fetch_add(cnt + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == n - 1) {
    __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(cnt + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// 16-B write-through store at a byte offset of a buffer resource (aux 16 = sc1)
__device__ __forceinline__ void st_sc1_b128(const __amdgpu_buffer_rsrc_t& rs, uint32_t off, float4 v) {
  typedef __attribute__((__vector_size__(4 * sizeof(float)))) float f32v4;
  __builtin_amdgcn_raw_buffer_store_b128((f32v4){v.x, v.y, v.z, v.w}, rs, off, 0, 16);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// LDS-DMA (global_load_lds_dwordx4) through inline asm, SADDR form: global address = 64-bit
// scalar base + 32-bit per-lane byte offset, LDS destination = M0 (+ lane * 16). hipcc does not
// see the DMA, so it inserts no conservative vmcnt(0) in front of LDS reads of the other buffer;
// the caller waits for completion explicitly (s_waitcnt vmcnt). Compiler-inserted waits for
// other vector-memory ops can only over-count younger operations, never under-wait. M0 is
// saved/restored inside the statement (cdna_hip_programming.md §5.7).
__device__ __forceinline__ void glds16s(const void* sbase, uint32_t voff, uint32_t lds_addr) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds_addr) : "memory");
}

__device__ __forceinline__ uint32_t lds_addr_of(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

#define ECHO_LAUNCH_CHECK()                         \
  do {                                              \
    hipError_t _e = hipGetLastError();              \
    if (_e != hipSuccess) return (int)_e;           \
  } while (0)

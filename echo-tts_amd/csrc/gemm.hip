// gemm.hip — C[M,N] = A[M,K] . W[N,K]^T with the fused epilogues of echo_hip.h.
//
// Replaces every nn.Linear on the sampling path (reference model.py:56-62,118-122,
// 177-197,303-305,443,532-540,557) together with the elementwise tails the
// reference runs right after them (SwiGLU, gated residual, bias, SiLU, /6, .float()).
//
// bf16 kernel (gfx950, MFMA v_mfma_f32_16x16x32_bf16):
//   * tile BM x BN x 64, WM x WN waves, each wave TM x TN of 16x16 fragments;
//   * both operands are K-contiguous rows; a K-step stages A and W tiles into LDS
//     with global_load_lds_dwordx4 (one 1 KiB wave-instruction = 8 rows of 128 B),
//     double-buffered, the chunk swizzle `chunk ^ ((row>>1)&7)` applied on the
//     SOURCE address so the lane-linear LDS image is conflict-free for the
//     16-lane ds_read_b128 groups of the fragment reads;
//   * operands are swapped (W fragment = MFMA A, X fragment = MFMA B) so each lane
//     ends with 4 consecutive output columns of one row;
//   * epilogue: bias/round/act in registers, then a per-wave XOR-swizzled LDS tile,
//     read back as 16-B row chunks for coalesced stores and the row-wise tails
//     (residual read, gate) — one HBM pass for the whole fused tail;
//   * block -> tile map: bijective XCD remap then group-M ordering (L2 reuse of W).
// fp32 kernel: plain LDS-tiled FMA GEMM for the fp32 parity mode (same epilogues).
#include "common.h"

// echo_set_policy_rows (shared with attention.hip's split-KV policy)
int g_policy_num = 1, g_policy_den = 1;

namespace {

constexpr int BK = 64;

struct Epi {
  const void* bias; int64_t stride_bias;
  const void* aux; int64_t ld_aux, stride_aux;
  const void* gate; int64_t stride_gate;
  int epi, act; float out_div;
  // ECHO_EPI_HEADNORM
  const void* hn_w; int64_t hn_w_stride; const float* hn_rope;
  int hn_heads, hn_nblk, hn_rope_heads, hn_seq_len, hn_pos0, hn_pos_mult; float hn_eps;
  int gm;  // persistent 256x256 kernel: group-M height (set by launch_ps_ek; tile 18 + diag key 1: override)
  const void* act_alpha;        // ECHO_ACT_SNAKE
  int conv_c, conv_taps, conv_dil;  // causal-conv A addressing (echo_hip.h)
  // RESID + the next AdaLN (EchoGemmArgs.mod_*; the split-K finish kernel only)
  void* mod_out; int64_t ld_mod; const void* mod_shift; const void* mod_scale1; float mod_eps;
  // EK_PARTIAL_FUSED (the split-K finish inside the launch): the output, its row stride, the counter buffer
  void* fin_out; int64_t fin_ldc; uint32_t* sync;
  int abl;  // small-M kernel timing ablations (diagnostics build, echo_gemm_set_diag key 16; results wrong)
};

// Element offset added to A for the K-slice starting at k0 in conv mode (0 otherwise): tap
// t = k0 / conv_c reads rows shifted back by (taps-1-t)*dil, at column k0 - t*conv_c.
__device__ __forceinline__ int64_t tap_delta(const Epi& ep, int k0, int64_t lda) {
  if (ep.conv_taps == 0) return 0;
  const int tap = k0 / ep.conv_c;
  return -((int64_t)tap * ep.conv_c + (int64_t)(ep.conv_taps - 1 - tap) * ep.conv_dil * lda);
}

// GELU (exact erf form, nn.GELU default) and Snake (autoencoder.py:97-102) for the epilogues.
__device__ __forceinline__ float gelu_erf(float x) { return x * 0.5f * (1.0f + erff(x * 0.70710678118654752f)); }
// bf16 Snake with the reference's rounding after each tensor op:
// x + round(round(1/round(a + 1e-9)) * round(round(sin(round(a*x)))^2))
__device__ __forceinline__ float snake_bf16(float x, float a) {
  const float s = rbf(sinf(rbf(a * x)));
  const float r = rbf(1.0f / rbf(a + 1e-9f));
  return rbf(x + rbf(r * rbf(s * s)));
}
__device__ __forceinline__ float snake_f32(float x, float a) {
  const float s = sinf(a * x);
  return x + (1.0f / (a + 1e-9f)) * (s * s);
}

__device__ __forceinline__ float epi_pointwise(float v, const Epi& ep, int n) {
  v = rbf(v);
  if (ep.act == ECHO_ACT_SILU) v = rbf(silu_f(v));
  else if (ep.act == ECHO_ACT_GELU) v = rbf(gelu_erf(v));
  else if (ep.act == ECHO_ACT_SNAKE) v = snake_bf16(v, bf2f(((const bf16_t*)ep.act_alpha)[n]));
  if (ep.out_div != 0.0f) v = rbf(v / ep.out_div);
  return v;
}

// Epilogue kinds, resolved on the host (ek_of) so the hot GEMMs get straight-line code:
// EK_GENERIC handles every Epi combination with runtime flags; the specialised kinds cover the
// decoder's three hot shapes (QKVG store, W13 SwiGLU, Wo/W2 gated residual) without bias/act/div;
// EK_BIAS (store + bias, the decoder's input projection) exists in the persistent kernel only.
enum { EK_GENERIC = 0, EK_STORE = 1, EK_SWIGLU = 2, EK_RESID = 3, EK_HEADNORM = 4, EK_BIAS = 5 };

// x from lane l ^ o (o = 8, 4, 2, 1: within 16-lane rows) without ds_bpermute's LDS round trip:
// DPP row_ror:8 for 8 ((l + 8) mod 16 = l ^ 8), quad_perm for 2 and 1, ds_swizzle (bitmask mode,
// xor 4) for 4 — the same lane pairs as __shfl_xor, so a butterfly sum is bitwise unchanged.
template <int O>
__device__ __forceinline__ float xor_lane16(float x) {
  const int v = __float_as_int(x);
  if constexpr (O == 8) return __int_as_float(__builtin_amdgcn_update_dpp(0, v, 0x128, 0xF, 0xF, false));
  else if constexpr (O == 4) return __int_as_float(__builtin_amdgcn_ds_swizzle(v, 0x101F));
  else if constexpr (O == 2) return __int_as_float(__builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false));
  else return __int_as_float(__builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false));
}

constexpr int largest_divisor_le(int n, int cap) {
  int d = cap < n ? cap : n;
  while (n % d) --d;
  return d;
}

// Epilogue shared by the bf16 kernels (must follow a barrier after the last LDS read):
// stage 1 registers -> per-wave swizzled LDS tile (bf16-rounded, bias/act/div or SwiGLU);
// stage 2 16-B row chunks -> residual/gate tail -> coalesced stores.
template <int TM, int TN, int FM, int FN, int EK>
__device__ __forceinline__ void gemm_epilogue(f32x4 (&acc)[FM][FN], bf16_t* lds, int wid, int wm, int wn, int lane,
                                              int m0, int n0, int M, int N, int z, void* __restrict__ Cv,
                                              int64_t ldc, int64_t sC, const Epi& ep) {
  const bool swiglu = EK == EK_GENERIC ? ep.epi == ECHO_EPI_SWIGLU : EK == EK_SWIGLU;
  const int TNo = swiglu ? TN / 2 : TN;  // staged columns per wave row
  const int CH = TNo / 8;                // 16-B chunks per staged row
  bf16_t* stg = lds + wid * (TM * TN);
  const bf16_t* biasp = (EK == EK_GENERIC && ep.bias) ? (const bf16_t*)ep.bias + z * ep.stride_bias : nullptr;
  const int cq = 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int ml = i * 16 + (lane & 15);
    if (swiglu) {
#pragma unroll
      for (int jj = 0; jj < FN / 2; ++jj) {
        float u[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float a = rbf(acc[i][2 * jj][r]), b = rbf(acc[i][2 * jj + 1][r]);
          u[r] = rbf(silu_bf16in(a)) * b;
        }
        const int c0 = jj * 16 + cq;
        const int ph = ((c0 >> 3) ^ (ml & (CH - 1))) * 8 + (c0 & 7);
        *(uint2*)(stg + ml * TNo + ph) = make_uint2(pack2bf(u[0], u[1]), pack2bf(u[2], u[3]));
      }
    } else {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        float v[4];
        const int nl = j * 16 + cq;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float x = acc[i][j][r];
          if (EK == EK_GENERIC) {
            const int nc = min(n0 + wn * TN + nl + r, N - 1);
            if (biasp) x += bf2f(biasp[nc]);
            x = epi_pointwise(x, ep, nc);
          }
          v[r] = x;  // pack2bf rounds (RNE) exactly once
        }
        const int ph = ((nl >> 3) ^ (ml & (CH - 1))) * 8 + (nl & 7);
        *(uint2*)(stg + ml * TNo + ph) = make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");

  // ---- epilogue, stage 2: row chunks -> fused row-wise tail -> 16-B stores
  const int Nout = swiglu ? N / 2 : N;
  const int nbase = (swiglu ? n0 / 2 : n0) + wn * TNo;
  if constexpr (EK == EK_HEADNORM) {
    // q/k RMSNorm + RoPE of echo_head_norm_rope fused after the store rounding. A 128-column
    // head is one wave's staged tile (TN == 128) or spans the tiles of the G = 128 / TN waves (wm, G p .. G p + G - 1)
    // (TN == 64 / 32; each wave of the group then takes 1 / G of the group's rows). 16 lanes per row, 8 consecutive
    // columns per lane and the same xor-butterfly sum as head_norm_rope_kernel, so results are bitwise equal.
    static_assert((TN == 32 || TN == 64 || TN == 128) && TM % (128 / TN * 4) == 0,
                  "HEADNORM epilogue: 32-, 64- or 128-column wave tiles");
    constexpr int G = 128 / TN;
    constexpr int PR = TM / G;   // rows of the group's tile taken by each wave
    constexpr int CHS = TN / 8;  // 16-B chunks per staged row
    if (G > 1) __syncthreads();  // the partner waves' staged tiles are complete
    const int hcol = n0 + (wn & ~(G - 1)) * TN;  // first column of this wave's head
    const int hidx = hcol >> 7;
    const int blk = hidx / ep.hn_heads, h = hidx - blk * ep.hn_heads;
    const bool norm = blk < ep.hn_nblk;
    const bool rope = norm && h < ep.hn_rope_heads;
    const int ch = lane & 15, rq = lane >> 4;
    const int c = ch & (CHS - 1);
    const bf16_t* src = lds + ((wid & ~(G - 1)) + ch / CHS) * (TM * TN);
    float wv[8];
    if (norm) load8((const bf16_t*)ep.hn_w + blk * ep.hn_w_stride + h * 128 + ch * 8, wv);
    bf16_t* Cp = (bf16_t*)Cv + z * sC + hcol + ch * 8;
    if (hcol >= N) return;
    constexpr int NR = PR / 4;  // 4-row iterations per wave
    // Batched: the LDS reads, RoPE table loads, sums, butterflies and reciprocal square roots of
    // HB row iterations are issued together (independent chains interleave) instead of one
    // row iteration's serial chain at a time; per element the same operations in the same order.
    constexpr int HB = largest_divisor_le(NR, 4);
    for (int it0 = 0; it0 < NR; it0 += HB) {
      float v[HB][8];
#pragma unroll
      for (int b = 0; b < HB; ++b) {
        const int row = (wn & (G - 1)) * PR + (it0 + b) * 4 + rq;
        load8(src + row * TN + ((c ^ (row & (CHS - 1))) * 8), v[b]);
      }
      if (norm) {
        float4 cs[HB][2];
        if (rope) {
#pragma unroll
          for (int b = 0; b < HB; ++b) {
            const int m = m0 + wm * TM + (wn & (G - 1)) * PR + (it0 + b) * 4 + rq;
            const int pos = ep.hn_pos0 + ep.hn_pos_mult * (min(m, M - 1) % ep.hn_seq_len);
            const float4* cp = (const float4*)(ep.hn_rope + ((int64_t)pos * 64 + ch * 4) * 2);
            cs[b][0] = cp[0];
            cs[b][1] = cp[1];
          }
        }
        float ss[HB];
#pragma unroll
        for (int b = 0; b < HB; ++b) {
          ss[b] = 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) ss[b] += v[b][e] * v[b][e];
        }
#pragma unroll
        for (int b = 0; b < HB; ++b) ss[b] += xor_lane16<8>(ss[b]);
#pragma unroll
        for (int b = 0; b < HB; ++b) ss[b] += xor_lane16<4>(ss[b]);
#pragma unroll
        for (int b = 0; b < HB; ++b) ss[b] += xor_lane16<2>(ss[b]);
#pragma unroll
        for (int b = 0; b < HB; ++b) ss[b] += xor_lane16<1>(ss[b]);
#pragma unroll
        for (int b = 0; b < HB; ++b) {
          const float r = 1.0f / sqrtf(ss[b] / 128.0f + ep.hn_eps);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[b][e] = rbf((v[b][e] * r) * wv[e]);
          if (rope) {
            const float cc[4] = {cs[b][0].x, cs[b][0].z, cs[b][1].x, cs[b][1].z};
            const float sn[4] = {cs[b][0].y, cs[b][0].w, cs[b][1].y, cs[b][1].w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float x0 = v[b][2 * e], x1 = v[b][2 * e + 1];
              v[b][2 * e] = (x0 * cc[e]) - (x1 * sn[e]);
              v[b][2 * e + 1] = (x0 * sn[e]) + (x1 * cc[e]);
            }
          }
        }
      }
#pragma unroll
      for (int b = 0; b < HB; ++b) {
        const int m = m0 + wm * TM + (wn & (G - 1)) * PR + (it0 + b) * 4 + rq;
        if (m < M) store8(Cp + (int64_t)m * ldc, v[b]);
      }
    }
    return;
  } else if constexpr (EK != EK_GENERIC) {
    // all of this lane's chunks are read (LDS, and the residual rows) before any store, so
    // the long-latency loads overlap; in-place residual (aux == C) is safe because every
    // element is read and written by the same lane.
    constexpr int CHc = (EK == EK_SWIGLU ? TN / 2 : TN) / 8, RPIc = 64 / CHc, NIT = TM / RPIc;
    // row chunks per batch (registers): all of them, or at most 8 (residual / long tiles) — a divisor of NIT
    constexpr int NB = (EK == EK_RESID || NIT > 16) ? largest_divisor_le(NIT, 8) : NIT;
    const int c = lane % CHc;
    const int n = nbase + c * 8;
    if (n >= Nout) return;
    bf16_t* Cp = (bf16_t*)Cv + z * sC + n;
    float g[8];
    if constexpr (EK == EK_RESID) {
      if (ep.gate) load8((const bf16_t*)ep.gate + z * ep.stride_gate + n, g);
    }
#pragma unroll
    for (int i0 = 0; i0 < NIT; i0 += NB) {
      u32x4 d[NB];
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const int row = (i0 + b) * RPIc + lane / CHc;
        d[b] = *(const u32x4*)(stg + row * CHc * 8 + ((c ^ (row & (CHc - 1))) * 8));
      }
      if constexpr (EK == EK_RESID) {
        const bf16_t* auxp = (const bf16_t*)ep.aux + z * ep.stride_aux + n;
        u32x4 x[NB];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          const int m = min(m0 + wm * TM + (i0 + b) * RPIc + lane / CHc, M - 1);
          x[b] = *(const u32x4*)(auxp + (int64_t)m * ep.ld_aux);
        }
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          float v[8], xf[8];
          const bf16_t* dv = (const bf16_t*)&d[b];
          const bf16_t* xv = (const bf16_t*)&x[b];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            v[e] = bf2f(dv[e]);
            xf[e] = bf2f(xv[e]);
            if (ep.gate) v[e] = rbf(g[e] * v[e]);
            v[e] = xf[e] + v[e];
          }
          d[b] = u32x4{pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]), pack2bf(v[6], v[7])};
        }
      }
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const int m = m0 + wm * TM + (i0 + b) * RPIc + lane / CHc;
        if (m < M) *(u32x4*)(Cp + (int64_t)m * ldc) = d[b];
      }
    }
    return;
  }
  const int RPI = 64 / CH;
  const int c = lane % CH;
  for (int it = 0; it < TM / RPI; ++it) {
    const int row = it * RPI + lane / CH;
    const int m = m0 + wm * TM + row;
    const int n = nbase + c * 8;
    float v[8];
    load8(stg + row * TNo + ((c ^ (row & (CH - 1))) * 8), v);
    if (m >= M || n >= Nout) continue;
    if (ep.epi == 99) { asm volatile("" ::"v"(v[0]), "v"(v[7])); continue; }
    if (ep.epi == ECHO_EPI_RESID) {
      float x[8];
      load8((const bf16_t*)ep.aux + z * ep.stride_aux + (int64_t)m * ep.ld_aux + n, x);
      if (ep.gate) {
        float g[8];
        load8((const bf16_t*)ep.gate + z * ep.stride_gate + n, g);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = rbf(g[e] * v[e]);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = rbf(x[e] + v[e]);
    }
    if (ep.epi == ECHO_EPI_F32OUT)
      store8((float*)Cv + z * sC + (int64_t)m * ldc + n, v);
    else
      store8((bf16_t*)Cv + z * sC + (int64_t)m * ldc + n, v);
  }
}

// NS = 2: one K-tile of lookahead (DMA of tile k+1 during tile k, vmcnt(0) + barrier per tile).
// NS = 3: two tiles of lookahead with a counted vmcnt and a raw barrier (inline-asm DMA, which
// hipcc's waitcnt pass does not drain before the fragment reads) — for the small tiles whose K
// loop is DMA-latency-bound (under-filled launches, row tails); same K order, bitwise equal.
template <int BM, int BN, int WM, int WN, int EK, int NS = 2>
__global__ void __launch_bounds__(64 * WM * WN)
gemm_bf16_kernel(const bf16_t* __restrict__ A, int64_t lda, int64_t sA,
                 const bf16_t* __restrict__ W, int64_t ldw, int64_t sW,
                 void* __restrict__ Cv, int64_t ldc, int64_t sC,
                 int M, int N, int K, int tiles_m, int tiles_n, Epi ep) {
  constexpr int NW = WM * WN;
  constexpr int NT = 64 * NW;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int STAGE = (BM + BN) * BK;  // elements per buffer
  static_assert((BM * 8) % NT == 0 && (BN * 8) % NT == 0, "staging split");
  static_assert(NS == 2 || NS == 3, "stages");
  __shared__ __attribute__((aligned(16))) bf16_t lds[NS * STAGE];

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int z = blockIdx.y;
  A += z * sA;
  W += z * sW;

  // ---- block -> tile: bijective XCD remap, then group-M ordering
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  constexpr int GM = 8;
  const int grp = wg / (GM * tiles_n);
  const int fm = grp * GM;
  const int gm = min(tiles_m - fm, GM);
  const int rem = wg - grp * GM * tiles_n;
  const int tm = fm + rem % gm, tn = rem / gm;
  const int m0 = tm * BM, n0 = tn * BN;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto stage = [&](int kt, int buf) {
    bf16_t* As = lds + buf * STAGE;
    bf16_t* Bs = As + BM * BK;
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < BM * 8 / NT; ++i) {
      const int rb = (i * NW + wid) * 8;
      const int row = rb + (lane >> 3);
      const int gc = (lane & 7) ^ ((row >> 1) & 7);
      const int grow = min(m0 + row, M - 1);
      const bf16_t* src = A + (int64_t)grow * lda + k0 + gc * 8 + tap_delta(ep, k0, lda);
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(As + rb * BK), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < BN * 8 / NT; ++i) {
      const int rb = (i * NW + wid) * 8;
      const int row = rb + (lane >> 3);
      const int gc = (lane & 7) ^ ((row >> 1) & 7);
      const int grow = min(n0 + row, N - 1);
      const bf16_t* src = W + (int64_t)grow * ldw + k0 + gc * 8;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(Bs + rb * BK), 16, 0, 0);
    }
  };

  // NS = 3 staging: SADDR-form asm DMA (32-bit offsets; the host checks the operand extents)
  constexpr int DOPS = (BM + BN) * 8 / NT;  // DMA wave-instructions per stage
  auto stage3 = [&](int kt, int buf) __attribute__((always_inline)) {
    const int k0 = kt * BK;
    const bf16_t* abase = A + tap_delta(ep, k0, lda) + k0;
    const bf16_t* wbase = W + k0;
#pragma unroll
    for (int i = 0; i < BM * 8 / NT; ++i) {
      const int rb = (i * NW + wid) * 8;
      const int row = rb + (lane >> 3);
      const int gc = (lane & 7) ^ ((row >> 1) & 7);
      const uint32_t off = (uint32_t)(((int64_t)min(m0 + row, M - 1) * lda + gc * 8) * 2);
      glds16s(abase, off, __builtin_amdgcn_readfirstlane(lds_addr_of(lds + buf * STAGE + rb * BK)));
    }
#pragma unroll
    for (int i = 0; i < BN * 8 / NT; ++i) {
      const int rb = (i * NW + wid) * 8;
      const int row = rb + (lane >> 3);
      const int gc = (lane & 7) ^ ((row >> 1) & 7);
      const uint32_t off = (uint32_t)(((int64_t)min(n0 + row, N - 1) * ldw + gc * 8) * 2);
      glds16s(wbase, off, __builtin_amdgcn_readfirstlane(lds_addr_of(lds + buf * STAGE + BM * BK + rb * BK)));
    }
  };

  const int nk = K / BK;
  const int frow = lane & 15;
  const int fsw = frow >> 1;
  auto compute = [&](const bf16_t* As) __attribute__((always_inline)) {
    const bf16_t* Bs = As + BM * BK;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ph = ((4 * s + (lane >> 4)) ^ fsw) * 8;
      bf16x8 xf[FM], wf[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) xf[i] = *(const bf16x8*)(As + (wm * TM + i * 16 + frow) * BK + ph);
#pragma unroll
      for (int j = 0; j < FN; ++j) wf[j] = *(const bf16x8*)(Bs + (wn * TN + j * 16 + frow) * BK + ph);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  };
  if constexpr (NS == 3) {
    // tiles 0, 1 in flight; at tile kt: wait for it (tile kt+1 may stay in flight), barrier (tile kt
    // visible, every wave done with tile kt-1's buffer), then DMA tile kt+2 into that buffer
    stage3(0, 0);
    if (nk > 1) stage3(1, 1);
    int cur = 0;
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DOPS) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (kt + 2 < nk) stage3(kt + 2, cur == 0 ? 2 : cur - 1);
      compute(lds + cur * STAGE);
      cur = cur == 2 ? 0 : cur + 1;
    }
    __syncthreads();  // last fragment reads done before the epilogue reuses the LDS
    gemm_epilogue<TM, TN, FM, FN, EK>(acc, lds, wid, wm, wn, lane, m0, n0, M, N, z, Cv, ldc, sC, ep);
    return;
  }
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(kt + 1, cur ^ 1);
    const bf16_t* As = lds + cur * STAGE;
    const bf16_t* Bs = As + BM * BK;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ph = ((4 * s + (lane >> 4)) ^ fsw) * 8;
      bf16x8 xf[FM], wf[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) xf[i] = *(const bf16x8*)(As + (wm * TM + i * 16 + frow) * BK + ph);
#pragma unroll
      for (int j = 0; j < FN; ++j) wf[j] = *(const bf16x8*)(Bs + (wn * TN + j * 16 + frow) * BK + ph);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  gemm_epilogue<TM, TN, FM, FN, EK>(acc, lds, wid, wm, wn, lane, m0, n0, M, N, z, Cv, ldc, sC, ep);
}

// ----------------------------------------------------------------------------- small-M launches
// gemm_bf16_sk_kernel: the decoder GEMMs of under-filled launches (B = 1 sampler steps, blockwise
// blocks: M = 160 ... 1920 rows). There the chip is bound by what each CU pulls from L2 into LDS
// (≈ 70-90 GB/s per CU, MI355X_MICROARCH.md "ring-gemm"/"Indexed rows") — a 64x64 tile needs 4 B per
// 2 x 64 MAC, and a single 4-wave workgroup with one K-tile of lookahead gets well under that rate —
// not by MFMA. So: bigger tiles, one or two workgroups per CU, an NS-stage LDS ring with NS - 1 K-tiles
// of LDS-DMA in flight behind counted vmcnt waits, and, where the tiles alone do not reach every CU,
// K split over gridDim.y = S workgroups (contiguous K-tile ranges [s n / S, (s + 1) n / S)).
//   S = 1: the shared fused epilogue; same fragments, same K order as every other bf16 kernel, so the
//          output is bitwise the one the 256x256 / 320x256 kernels give at large M.
//   EK = EK_PARTIAL: the unit's fp32 accumulators go to the workspace slab ws[s] ([S][M][N], ld N,
//          straight from registers: 16 B per lane), and gemm_splitk_finish_kernel sums the S slabs in
//          order s = 0 .. S-1 and applies the epilogue.
constexpr int EK_PARTIAL = 6;
// EK_PARTIAL_FUSED (gated residual only, round 6): the K-slices of a tile store their slabs write-through, wait for
// each other (per-tile arrival counter in the caller's counter buffer, common.h), and each finishes 1/S of the
// tile's (row, 8-column) units with gemm_splitk_finish_kernel<EK_RESID>'s arithmetic; with ep.mod_out the row
// panel's workgroups then wait for the whole panel and each normalises + modulates a share of its rows, one wave per
// row, with the finish kernel's MOD arithmetic (= adaln_rows_kernel<4>'s). One launch instead of GEMM + finish,
// bitwise the same output. Every workgroup of the launch must be resident at once (host: grid <= CUs).
constexpr int EK_PARTIAL_FUSED = 7;

// vmcnt(n * D) for n = 0 .. 3 (counted waits need immediates)
template <int D>
__device__ __forceinline__ void vm_wait_stages(int n) {
  if (n >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * D) : "memory");
  else if (n == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * D) : "memory");
  else if (n == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// The in-launch split-K finish of EK_PARTIAL_FUSED (see there). ws: the S fp32 slabs [S][M][N]; this workgroup is
// K-slice s of tile (tm, tn) with origin (m0, n0).
template <int BM, int BN, int NT>
__device__ __forceinline__ void sk_fused_finish(const void* ws, int M, int N, int S, int s, int tm, int tn, int tiles_m,
                                                int tiles_n, int m0, int n0, const Epi& ep) {
  uint32_t* sync = ep.sync;
  const bool mod = ep.mod_out != nullptr;
  // publish this K-slice's slab tile (every storing wave drained its write-through stores), wait for the tile's S
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  uint32_t* tcnt = sync + SYNC_CNT0 + 2 * (tm * tiles_n + tn);
  if (threadIdx.x == 0) sync_arrive_wait(sync, tcnt, (uint32_t)S);
  __syncthreads();
  // 1/S of the tile's (row, 8-column) units, gemm_splitk_finish_kernel<EK_RESID>'s arithmetic
  constexpr int CPR = BN / 8, U = BM * CPR;
  const float* ws0 = (const float*)ws;
  const int64_t slab = (int64_t)M * N;
  const __amdgpu_buffer_rsrc_t hr = rsrc_of(ep.fin_out, 0xFFFFFFF0u);
  (void)hr;
  for (int u = s * U / S + (int)threadIdx.x; u < (s + 1) * U / S; u += NT) {
    const int r = u / CPR, c = u - r * CPR;
    const int m = m0 + r, n = n0 + 8 * c;
    if (m >= M) continue;
    float v[8];
    load8(ws0 + (int64_t)m * N + n, v);
    for (int k = 1; k < S; ++k) {
      float w[8];
      load8(ws0 + k * slab + (int64_t)m * N + n, w);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += w[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = rbf(v[e]);
    float x[8];
    load8((const bf16_t*)ep.aux + (int64_t)m * ep.ld_aux + n, x);
    if (ep.gate) {
      float g[8];
      load8((const bf16_t*)ep.gate + n, g);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = rbf(g[e] * v[e]);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = x[e] + v[e];  // the store rounds
    if (mod) {  // the panel's other workgroups read this row: write-through
      const uint4 h = make_uint4(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]), pack2bf(v[6], v[7]));
      st_sc1_b128(hr, (uint32_t)(((int64_t)m * ep.fin_ldc + n) * 2),
                  make_float4(__uint_as_float(h.x), __uint_as_float(h.y), __uint_as_float(h.z), __uint_as_float(h.w)));
    } else {
      store8((bf16_t*)ep.fin_out + (int64_t)m * ep.fin_ldc + n, v);
    }
  }
  if (threadIdx.x == 0) sync_depart(tcnt, (uint32_t)S);
  if (!mod) return;
  // the next AdaLN needs whole rows: wait for every K-slice of every column tile of this row panel
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int pw = tiles_n * S;  // workgroups of the panel
  uint32_t* pcnt = sync + SYNC_CNT0 + 2 * (tiles_m * tiles_n + tm);
  if (threadIdx.x == 0) sync_arrive_wait(sync, pcnt, (uint32_t)pw);
  __syncthreads();
  // one wave per row: rows k, k + pw, ... of the panel for this workgroup's index k; lane l holds the 8-column
  // chunks t = q * 64 + l (q = 0..3), squares summed in (q, e) order, then the wave butterfly (the finish MOD)
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  constexpr int NWV = NT / 64;
  for (int r = tn * S + s + wv * pw; r < BM; r += NWV * pw) {
    const int m = m0 + r;
    if (m >= M) break;
    const bf16_t* hrow = (const bf16_t*)ep.fin_out + (int64_t)m * ep.fin_ldc;
    float h[4][8];
#pragma unroll
    for (int q = 0; q < 4; ++q) load8(hrow + (q * 64 + lane) * 8, h[q]);
    float ss = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 8; ++e) ss += h[q][e] * h[q][e];
    ss = wave_sum(ss);
    const float rr = 1.0f / sqrtf(ss / 2048.0f + ep.mod_eps);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n = (q * 64 + lane) * 8;
      float s1[8], sh[8], o[8];
      load8((const bf16_t*)ep.mod_scale1 + n, s1);
      load8((const bf16_t*)ep.mod_shift + n, sh);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = ((h[q][e] * rr) * s1[e]) + sh[e];
      store8((bf16_t*)ep.mod_out + (int64_t)m * ep.ld_mod + n, o);
    }
  }
  if (threadIdx.x == 0) sync_depart(pcnt, (uint32_t)pw);
}

template <int BM, int BN, int WM, int WN, int EK, int NS>
__global__ void __launch_bounds__(64 * WM * WN)
gemm_bf16_sk_kernel(const bf16_t* __restrict__ A, int64_t lda, const bf16_t* __restrict__ W, int64_t ldw,
                    void* __restrict__ Cv, int64_t ldc, int M, int N, int K, int tiles_m, int tiles_n, Epi ep) {
  constexpr int NW = WM * WN;
  constexpr int NT = 64 * NW;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int STAGE = (BM + BN) * BK;  // elements per ring slot
  // LDS-DMA wave-instructions per slot: 8 rows each; where the rows do not split evenly over the waves the
  // last round wraps to rows already staged (a duplicate DMA of the same bytes to the same LDS address), so
  // every wave issues the same count and the counted waits stay uniform
  constexpr int AI = (BM * 8 + NT - 1) / NT, BI = (BN * 8 + NT - 1) / NT;
  constexpr int DOPS = AI + BI;
  static_assert(BM % 8 == 0 && BN % 8 == 0, "8-row DMA groups");
  static_assert(NS >= 2 && NS <= 5 && DOPS * (NS - 2) <= 63, "ring depth / vmcnt range");
  __shared__ __attribute__((aligned(16))) bf16_t lds[NS * STAGE];

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid / WN, wn = wid % WN;

  // block -> tile as gemm_bf16_kernel (bijective XCD remap, group-M); blockIdx.y = K split
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  constexpr int GM = 8;
  const int grp = wg / (GM * tiles_n);
  const int fm = grp * GM;
  const int gm = min(tiles_m - fm, GM);
  const int rem = wg - grp * GM * tiles_n;
  const int tm = fm + rem % gm, tn = rem / gm;
  const int m0 = tm * BM, n0 = tn * BN;
  const int S = gridDim.y, s = blockIdx.y;
  const int nk_all = K / BK;
  const int kb = (int)((int64_t)s * nk_all / S);
  const int nk = (int)((int64_t)(s + 1) * nk_all / S) - kb;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // SADDR-form DMA of K-tile kb + kt into ring slot `slot` (32-bit offsets: the host checks the extents);
  // part 0 = the A pieces, 1 = the W pieces, 2 = both
  auto stage = [&](int kt, int slot, int part = 2) __attribute__((always_inline)) {
    const int k0 = (kb + kt) * BK;
    const bf16_t* abase = A + k0;
    const bf16_t* wbase = W + k0;
    bf16_t* dst = lds + slot * STAGE;
    if (part != 1) {
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int rb = ((i * NW + wid) * 8) % BM;
      const int row = rb + (lane >> 3);
      const int gc = (lane & 7) ^ ((row >> 1) & 7);
      const uint32_t off = (uint32_t)(((int64_t)min(m0 + row, M - 1) * lda + gc * 8) * 2);
      glds16s(abase, off, __builtin_amdgcn_readfirstlane(lds_addr_of(dst + rb * BK)));
    }
    }
    if (part == 0) return;
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int rb = ((i * NW + wid) * 8) % BN;
      const int row = rb + (lane >> 3);
      const int gc = (lane & 7) ^ ((row >> 1) & 7);
      const uint32_t off = (uint32_t)(((int64_t)min(n0 + row, N - 1) * ldw + gc * 8) * 2);
      glds16s(wbase, off, __builtin_amdgcn_readfirstlane(lds_addr_of(dst + BM * BK + rb * BK)));
    }
  };

  const int frow = lane & 15;
  const int fsw = frow >> 1;
  // snext >= 0: the DMA of K-tile snext is issued inside the compute, its A pieces after the first half's fragment
  // reads and its W pieces after the second half's, under their LDS latency and beside the other wave's MFMAs
  // (issued as one block between the barrier and the compute, each wave's pieces delayed its first fragment reads:
  // profiles/r6_sk_dma_split.txt)
  auto compute = [&](const bf16_t* As, int snext = -1, int sslot = 0) __attribute__((always_inline)) {
    const bf16_t* Bs = As + BM * BK;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ph = ((4 * ks + (lane >> 4)) ^ fsw) * 8;
      bf16x8 xf[FM], wf[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) xf[i] = *(const bf16x8*)(As + (wm * TM + i * 16 + frow) * BK + ph);
#pragma unroll
      for (int j = 0; j < FN; ++j) wf[j] = *(const bf16x8*)(Bs + (wn * TN + j * 16 + frow) * BK + ph);
      if (snext >= 0) stage(snext, sslot, ks);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  };

  // ring: slots hold K-tiles kt mod NS; at tile kt wait for it (the up to NS - 2 younger tiles stay in
  // flight), barrier (tile kt visible; every wave is done reading tile kt - 1's slot), then refill that
  // slot with tile kt + NS - 1 and compute tile kt
  // ECHO_DIAG timing ablations (results wrong): 1 no MFMA / fragment reads, 2 no DMA in the loop, 4 no epilogue,
  // 8 no DMA at all
#ifdef ECHO_DIAG
  const int abl = ep.abl;
#else
  constexpr int abl = 0;
#endif
#pragma unroll
  for (int p = 0; p < NS - 1; ++p)
    if (p < nk && !(abl & 8)) stage(p, p);
  for (int kt = 0; kt < nk; ++kt) {
    vm_wait_stages<DOPS>(min(NS - 2, nk - 1 - kt));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const bool more = kt + NS - 1 < nk && !(abl & 10);
    // 8-wave configs: the next K-tile's DMA issued inside the compute (round 6: 5-9 % faster at the B = 1 shapes);
    // with one wave per SIMD nothing runs beside the issue, and the 4-wave configs stay 9 % faster without it
    if (NW >= 8 && !(abl & 32)) {
      if (!(abl & 1)) compute(lds + (kt % NS) * STAGE, more ? kt + NS - 1 : -1, (kt + NS - 1) % NS);
      else if (more) stage(kt + NS - 1, (kt + NS - 1) % NS);
    } else {  // the 4-wave configs (and diag bit 32, A/B): all of it between the barrier and the compute
      if (more) stage(kt + NS - 1, (kt + NS - 1) % NS);
      if (!(abl & 1)) compute(lds + (kt % NS) * STAGE);
    }
  }
  if (abl & 4) return;

  if constexpr (EK == EK_PARTIAL || EK == EK_PARTIAL_FUSED) {
    // fp32 partial tile -> ws slab s: lane holds row (lane & 15) of each 16-row fragment, 4 consecutive
    // columns 4 (lane >> 4) .. + 3 of each 16-column fragment (FUSED: write-through, byte offsets < 4 GiB)
    float* slab = (float*)Cv + (int64_t)s * M * ldc;
    const __amdgpu_buffer_rsrc_t wsr = rsrc_of(Cv, 0xFFFFFFF0u);
    (void)wsr;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = m0 + wm * TM + i * 16 + frow;
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + wn * TN + j * 16 + 4 * (lane >> 4);
        if (n < N) {
          if constexpr (EK == EK_PARTIAL_FUSED) {
            const f32x4 v = acc[i][j];
            st_sc1_b128(wsr, (uint32_t)((((int64_t)s * M + m) * ldc + n) * 4), make_float4(v[0], v[1], v[2], v[3]));
          } else {
            *(f32x4*)(slab + (int64_t)m * ldc + n) = acc[i][j];
          }
        }
      }
    }
    if constexpr (EK == EK_PARTIAL_FUSED) sk_fused_finish<BM, BN, NT>(Cv, M, N, S, s, tm, tn, tiles_m, tiles_n, m0, n0, ep);
  } else {
    __syncthreads();  // last fragment reads done before the epilogue reuses the LDS
    gemm_epilogue<TM, TN, FM, FN, EK>(acc, lds, wid, wm, wn, lane, m0, n0, M, N, 0, Cv, ldc, 0, ep);
  }
}

// Sum of the S fp32 partial slabs ws[s][M][N] (order s = 0 .. S-1) + the fused epilogue of the split
// launch, with the roundings of gemm_epilogue: one thread per 8 output columns of one row (16 B out);
// EK_HEADNORM: the 16 threads of a (row, 128-column head) are one 16-lane row of the wave (N % 128 == 0),
// so the sum of squares is the xor-butterfly of head_norm_rope_kernel / the fused epilogue.
// MOD (EK_RESID, N == 2048: the workgroup is one row, thread t = columns 8t .. 8t+7): the updated row is
// also normalised and modulated into ep.mod_out with adaln_rows_kernel<4>'s arithmetic — there lane l of
// the row's wave holds the chunks t = c*64 + l (c = 0..3), i.e. the same lane of each of our 4 waves; the
// rounded row goes through LDS so that every lane sums its 32 squares in that kernel's order before the
// same wave butterfly, and r, the products and the rounding are the same expressions (bitwise equal).
template <int EK, bool MOD = false>
__global__ void __launch_bounds__(256)
gemm_splitk_finish_kernel(const float* __restrict__ ws, int S, int M, int N, void* __restrict__ Cv, int64_t ldc,
                          Epi ep) {
  static_assert(!MOD || EK == EK_RESID, "the fused AdaLN follows the residual epilogue");
  const int Nout = EK == EK_SWIGLU ? N / 2 : N;
  const int cpr = Nout / 8;  // 8-column chunks per output row
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)M * cpr) return;
  const int m = (int)(t / cpr), c = (int)(t - (int64_t)m * cpr);
  const int n = c * 8;  // first output column
  const int64_t slab = (int64_t)M * N;
  auto sum8 = [&](int col, float (&v)[8]) __attribute__((always_inline)) {
    const float* p = ws + (int64_t)m * N + col;
    load8(p, v);
    for (int k = 1; k < S; ++k) {
      float w[8];
      load8(p + k * slab, w);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += w[e];
    }
  };
  float v[8];
  if constexpr (EK == EK_SWIGLU) {
    // output column j <- GEMM columns a = (j / 16) * 32 + j % 16 and b = a + 16 (w1 / w3 blocks of 16)
    const int a0 = (n / 16) * 32 + n % 16;
    float a[8], b[8];
    sum8(a0, a);
    sum8(a0 + 16, b);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = rbf(silu_bf16in(rbf(a[e]))) * rbf(b[e]);
  } else {
    sum8(n, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = rbf(v[e]);
  }
  bf16_t* out = (bf16_t*)Cv + (int64_t)m * ldc + n;
  if constexpr (EK == EK_RESID) {
    float x[8];
    load8((const bf16_t*)ep.aux + (int64_t)m * ep.ld_aux + n, x);
    if (ep.gate) {
      float g[8];
      load8((const bf16_t*)ep.gate + n, g);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = rbf(g[e] * v[e]);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = x[e] + v[e];  // store8 rounds
    if constexpr (MOD) {
      __shared__ float row[2048];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[e] = rbf(v[e]);
        row[n + e] = v[e];
      }
      store8(out, v);
      __syncthreads();
      const int lane = threadIdx.x & 63;
      float ss = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float u = row[(q * 64 + lane) * 8 + e];
          ss += u * u;
        }
      ss = wave_sum(ss);
      const float r = 1.0f / sqrtf(ss / 2048.0f + ep.mod_eps);
      float s1[8], sh[8], o[8];
      load8((const bf16_t*)ep.mod_scale1 + n, s1);
      load8((const bf16_t*)ep.mod_shift + n, sh);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = ((v[e] * r) * s1[e]) + sh[e];
      store8((bf16_t*)ep.mod_out + (int64_t)m * ep.ld_mod + n, o);
      return;
    }
  } else if constexpr (EK == EK_HEADNORM) {
    const int hidx = n >> 7, ch = (n >> 3) & 15;
    const int blk = hidx / ep.hn_heads, h = hidx - blk * ep.hn_heads;
    if (blk < ep.hn_nblk) {  // uniform over the 16 lanes of the head
      float wv[8];
      load8((const bf16_t*)ep.hn_w + blk * ep.hn_w_stride + h * 128 + ch * 8, wv);
      float ss = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) ss += v[e] * v[e];
      ss += xor_lane16<8>(ss);
      ss += xor_lane16<4>(ss);
      ss += xor_lane16<2>(ss);
      ss += xor_lane16<1>(ss);
      const float r = 1.0f / sqrtf(ss / 128.0f + ep.hn_eps);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = rbf((v[e] * r) * wv[e]);
      if (h < ep.hn_rope_heads) {
        const int pos = ep.hn_pos0 + ep.hn_pos_mult * (m % ep.hn_seq_len);
        const float4* cp = (const float4*)(ep.hn_rope + ((int64_t)pos * 64 + ch * 4) * 2);
        const float4 c0 = cp[0], c1 = cp[1];
        const float cc[4] = {c0.x, c0.z, c1.x, c1.z};
        const float sn[4] = {c0.y, c0.w, c1.y, c1.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float x0 = v[2 * e], x1 = v[2 * e + 1];
          v[2 * e] = (x0 * cc[e]) - (x1 * sn[e]);
          v[2 * e + 1] = (x0 * sn[e]) + (x1 * cc[e]);
        }
      }
    }
  }
  store8(out, v);
}

// ----------------------------------------------------------------------------- 256x256 ping-pong
// Same tile, operands, LDS image and epilogue as gemm_bf16_kernel<256,256,2,4>, different schedule:
//   * a K-tile is computed in 4 phases, one 64x32 quadrant per wave per phase (16 MFMAs),
//     quadrant order (0,0),(0,1),(1,1),(1,0) so each phase re-reads only 4-8 fragments;
//   * each phase = L segment (fragment ds_reads + this phase's share of the next K-tile's DMA,
//     counted vmcnt, lgkmcnt(0), s_barrier) then C segment (16 MFMAs, s_barrier);
//   * waves 4-7 (wm = 1) run one barrier behind waves 0-3, so on every SIMD one wave
//     computes while its partner loads (the two waves of a SIMD alternate roles);
//   * the next K-tile is staged in 4 chunks ordered by first use (A rows of qm=0, B cols
//     of qn=0, B cols of qn=1, A rows of qm=1), chunk j issued in phase j; every chunk has
//     >= 2 phases in flight (vmcnt keeps the 2 most recent chunks = 4 DMA per wave) and
//     is overwritten only after its last reader's lgkmcnt(0) + barrier (WAR).
// Derivation of the RAW/WAR distances: DESIGN.md "GEMM ping-pong schedule".
__device__ __forceinline__ void vm_wait(int n) {
  if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (n >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__device__ __forceinline__ void pp_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// first row of 8-row group g (0..15) of staging chunk c (128 rows of A or B)
__device__ __forceinline__ int chunk_row(int c, int g) {
  if (c == 0 || c == 3) return (c == 3 ? 64 : 0) + (g < 8 ? g * 8 : 128 + (g - 8) * 8);
  return (g >> 2) * 64 + (c == 2 ? 32 : 0) + (g & 3) * 8;
}

template <int ABL, int EK>  // ABL: timing ablations only (1 no in-loop DMA, 2 no fragment reads, 4 no
                            // epilogue stores, 8 no epilogue); EK: epilogue kind
__global__ void __launch_bounds__(512)
gemm_bf16_pp_kernel(const bf16_t* __restrict__ A, int64_t lda, int64_t sA,
                    const bf16_t* __restrict__ W, int64_t ldw, int64_t sW,
                    void* __restrict__ Cv, int64_t ldc, int64_t sC,
                    int M, int N, int K, int tiles_m, int tiles_n, Epi ep) {
  constexpr int BM = 256, BN = 256, TM = 128, TN = 64, FM = 8, FN = 4;
  constexpr int STAGE = (BM + BN) * BK;
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * STAGE];

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid >> 2, wn = wid & 3;
  const int z = blockIdx.y;
  A += z * sA;
  W += z * sW;
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  constexpr int GM = 8;
  const int grp = wg / (GM * tiles_n);
  const int fm = grp * GM;
  const int gm = min(tiles_m - fm, GM);
  const int rem = wg - grp * GM * tiles_n;
  const int tm = fm + rem % gm, tn = rem / gm;
  const int m0 = tm * BM, n0 = tn * BN;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // per-wave DMA sources/destinations of its two 8-row groups of every chunk (loop-invariant)
  const bf16_t* dsrc[4][2];
  int ddst[4][2];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int rb = chunk_row(c, 2 * wid + h);
      const int row = rb + (lane >> 3);
      const int gc = (lane & 7) ^ ((row >> 1) & 7);
      const bool isA = (c == 0 || c == 3);
      const int grow = isA ? min(m0 + row, M - 1) : min(n0 + row, N - 1);
      dsrc[c][h] = (isA ? A + (int64_t)grow * lda : W + (int64_t)grow * ldw) + gc * 8;
      ddst[c][h] = (isA ? 0 : BM * BK) + rb * BK;
    }
  // chunk c of K-tile kt into buffer kt&1 (two 1 KiB wave-instructions)
  auto dma = [&](int c, int kt) {
    const int64_t td = (c == 0 || c == 3) ? tap_delta(ep, kt * BK, lda) : 0;
#pragma unroll
    for (int h = 0; h < 2; ++h)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(dsrc[c][h] + kt * BK + td),
          (__attribute__((address_space(3))) void*)(lds + (kt & 1) * STAGE + ddst[c][h]), 16, 0, 0);
  };

  const int nk = K / BK;
  // prologue: K-tile 0 whole; phase 0 reads only chunks 0-1, chunks 2-3 retire at its vm_wait(2)
#pragma unroll
  for (int c = 0; c < 4; ++c) dma(c, 0);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  pp_barrier();
  if (wm == 1) pp_barrier();  // waves 4-7 run one barrier (half a phase) behind

  const int frow = lane & 15;
  const int fsw = frow >> 1;
  bf16x8 af[4][2], bfr[2][2];
  for (int kt = 0; kt < nk; ++kt) {
    const bf16_t* As = lds + (kt & 1) * STAGE;
    const bf16_t* Bs = As + BM * BK;
    const bool more = kt + 1 < nk;
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
      const int qm = (ph == 2 || ph == 3) ? 1 : 0;
      const int qn = (ph == 1 || ph == 2) ? 1 : 0;
      // ---- L segment
      if ((ph == 0 || ph == 2) && (!(ABL & 2) || kt == 0)) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int s = 0; s < 2; ++s)
            af[i][s] = *(const bf16x8*)(As + (wm * TM + qm * 64 + i * 16 + frow) * BK +
                                        (((4 * s + (lane >> 4)) ^ fsw) * 8));
      }
      if (ph != 2 && (!(ABL & 2) || kt == 0)) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int s = 0; s < 2; ++s)
            bfr[j][s] = *(const bf16x8*)(Bs + (wn * TN + qn * 32 + j * 16 + frow) * BK +
                                         (((4 * s + (lane >> 4)) ^ fsw) * 8));
      }
      if (more && !(ABL & 1)) dma(ph, kt + 1);
      // outstanding DMA allowed: this phase's and the previous phase's
      const bool prev = ((ph > 0) ? more : (kt > 0)) && !(ABL & 1);
      vm_wait((more && !(ABL & 1) ? 2 : 0) + (prev ? 2 : 0));
      pp_barrier();
      // ---- C segment (this wave's fragment reads retire here, overlapping the barrier wait;
      // the first DMA that overwrites any region read in this phase comes >= 2 phases later)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int s = 0; s < 2; ++s)
            acc[qm * 4 + i][qn * 2 + j] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j][s], af[i][s], acc[qm * 4 + i][qn * 2 + j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      pp_barrier();
    }
  }
  if (wm == 0) pp_barrier();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (ABL & 8) {  // timing ablation: keep acc live, no epilogue
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }
  Epi e2 = ep;
  if (ABL & 4) e2.epi = 99;  // timing ablation: stage 2 loads/stores skipped
  gemm_epilogue<TM, TN, FM, FN, EK>(acc, lds, wid, wm, wn, lane, m0, n0, M, N, z, Cv, ldc, sC, e2);
}

// ----------------------------------------------------------------------------- 2-phase ping-pong
// Same tile, LDS image, chunking and epilogue as gemm_bf16_pp_kernel, but a K-tile is 2 phases of
// 32 MFMAs (half the barriers per MFMA): phase 0 = A rows qm=0 x all 64 B columns of the wave,
// phase 1 = A rows qm=1 x the same B fragments (held in registers, never re-read).
//   * every L segment retires its fragment reads (lgkmcnt(0)) BEFORE its barrier, so a chunk's
//     region is free as soon as the reader's next barrier has passed;
//   * DMA runs 1.5 K-tiles ahead: chunks 0-2 (A qm0 rows + all B) of tile kt+2 are issued in
//     phase 1 of tile kt (their region of buffer kt&1 was last read in phase 0), chunk 3 (A qm1)
//     of tile kt+1 in phase 0 of tile kt (region last read in phase 1 of tile kt-1);
//   * each chunk is waited for 4 segments (2 phases) after issue: steady state vmcnt(8).
template <int N> __device__ __forceinline__ void vm_wait_n() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int EK>
__global__ void __launch_bounds__(512)
gemm_bf16_pp2_kernel(const bf16_t* __restrict__ A, int64_t lda, int64_t sA,
                     const bf16_t* __restrict__ W, int64_t ldw, int64_t sW,
                     void* __restrict__ Cv, int64_t ldc, int64_t sC,
                     int M, int N, int K, int tiles_m, int tiles_n, Epi ep) {
  constexpr int BM = 256, BN = 256, TM = 128, TN = 64, FM = 8, FN = 4;
  constexpr int STAGE = (BM + BN) * BK;
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * STAGE];

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid >> 2, wn = wid & 3;
  const int z = blockIdx.y;
  A += z * sA;
  W += z * sW;
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  constexpr int GM = 8;
  const int grp = wg / (GM * tiles_n);
  const int fm = grp * GM;
  const int gm = min(tiles_m - fm, GM);
  const int rem = wg - grp * GM * tiles_n;
  const int tm = fm + rem % gm, tn = rem / gm;
  const int m0 = tm * BM, n0 = tn * BN;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const bf16_t* dsrc[4][2];
  int ddst[4][2];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int rb = chunk_row(c, 2 * wid + h);
      const int row = rb + (lane >> 3);
      const int gc = (lane & 7) ^ ((row >> 1) & 7);
      const bool isA = (c == 0 || c == 3);
      const int grow = isA ? min(m0 + row, M - 1) : min(n0 + row, N - 1);
      dsrc[c][h] = (isA ? A + (int64_t)grow * lda : W + (int64_t)grow * ldw) + gc * 8;
      ddst[c][h] = (isA ? 0 : BM * BK) + rb * BK;
    }
  auto dma = [&](int c, int kt) {
    const int64_t td = (c == 0 || c == 3) ? tap_delta(ep, kt * BK, lda) : 0;
#pragma unroll
    for (int h = 0; h < 2; ++h)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(dsrc[c][h] + kt * BK + td),
          (__attribute__((address_space(3))) void*)(lds + (kt & 1) * STAGE + ddst[c][h]), 16, 0, 0);
  };

  const int nk = K / BK;
  // prologue: tile 0 whole, chunks 0-2 of tile 1; wait for chunks 0-2 of tile 0
#pragma unroll
  for (int c = 0; c < 4; ++c) dma(c, 0);
  if (nk > 1) {
    dma(0, 1); dma(1, 1); dma(2, 1);
    vm_wait_n<8>();
  } else {
    vm_wait_n<2>();
  }
  pp_barrier();
  if (wm == 1) pp_barrier();  // waves 4-7 run one barrier (one segment) behind

  const int frow = lane & 15;
  const int fsw = frow >> 1;
  bf16x8 af[4][2], bfr[4][2];
  for (int kt = 0; kt < nk; ++kt) {
    const bf16_t* As = lds + (kt & 1) * STAGE;
    const bf16_t* Bs = As + BM * BK;
    const bool n1 = kt + 1 < nk, n2 = kt + 2 < nk;
#pragma unroll
    for (int ph = 0; ph < 2; ++ph) {
      // ---- L segment
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int s = 0; s < 2; ++s)
          af[i][s] = *(const bf16x8*)(As + (wm * TM + ph * 64 + i * 16 + frow) * BK +
                                      (((4 * s + (lane >> 4)) ^ fsw) * 8));
      if (ph == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int s = 0; s < 2; ++s)
            bfr[j][s] = *(const bf16x8*)(Bs + (wn * TN + j * 16 + frow) * BK +
                                         (((4 * s + (lane >> 4)) ^ fsw) * 8));
        if (n1) dma(3, kt + 1);
        // retire chunk 3 of tile kt (issued one phase pair ago)
        if (n1) vm_wait_n<8>(); else vm_wait_n<0>();
      } else {
        if (n2) { dma(0, kt + 2); dma(1, kt + 2); dma(2, kt + 2); }
        // retire chunks 0-2 of tile kt+1
        if (n2) vm_wait_n<8>(); else if (n1) vm_wait_n<2>(); else vm_wait_n<0>();
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      pp_barrier();
      // ---- C segment
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int s = 0; s < 2; ++s)
            acc[ph * 4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j][s], af[i][s], acc[ph * 4 + i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      pp_barrier();
    }
  }
  if (wm == 0) pp_barrier();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (ep.epi == 99) {  // diagnostic (tile 15): no epilogue, accumulators kept live
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }
  gemm_epilogue<TM, TN, FM, FN, EK>(acc, lds, wid, wm, wn, lane, m0, n0, M, N, z, Cv, ldc, sC, ep);
}

// ----------------------------------------------------------------------------- persistent 2-phase
// gemm_bf16_pp2_kernel's K loop (same LDS image, chunking and K order: bitwise-equal results) run
// by one persistent workgroup per CU over tiles blockIdx.x, +gridDim.x, ... The epilogue works
// from the accumulator registers (8-B row segments, no LDS staging) and runs AFTER the next
// tile's prologue DMA has been issued, so the output store burst overlaps the next tile's first
// loads instead of serialising with a workgroup teardown + relaunch.
//   * vmcnt counts loads, stores and LDS-DMA in issue order: the SN epilogue stores of a wave are
//     younger than the next tile's prologue DMA, so the waits of that prologue and of K-tile 0
//     allow SN more operations in flight; the first wait of K-tile 1 retires them.
//   * every wave issues exactly SN stores per tile (raw buffer stores; rows past M fall beyond the
//     buffer's num_records and are dropped by the hardware), so the counted waits hold for any M.
//   * RESID reads the residual + gate of the current tile BEFORE issuing the prologue DMA, and
//     waits for them with vmcnt(14) (the 14 prologue DMA stay in flight).
//   * measured: the stores must be acknowledged before K-tile 1's first wait, and
//     with every CU storing its 128 KB tile at once that costs more than the relaunch it saves.
constexpr int reg_epi_stores(int ek) { return ek == EK_SWIGLU ? 8 : 16; }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t brsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

template <int EK>
__global__ void __launch_bounds__(512)
gemm_bf16_ps_kernel(const bf16_t* __restrict__ A, int64_t lda, int64_t sA,
                    const bf16_t* __restrict__ W, int64_t ldw, int64_t sW,
                    void* __restrict__ Cv, int64_t ldc, int64_t sC,
                    int M, int N, int K, int tiles_m, int tiles_n, Epi ep) {
  static_assert(EK == EK_STORE || EK == EK_SWIGLU || EK == EK_RESID || EK == EK_BIAS || EK == EK_HEADNORM,
                "register epilogue kinds");
  constexpr int BM = 256, BN = 256, TM = 128, TN = 64, FM = 8, FN = 4;
  constexpr int STAGE = (BM + BN) * BK;
  constexpr int SN = reg_epi_stores(EK);
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * STAGE];
  // HEADNORM: per-(row, 8-column chunk) sums of squares of every wave, read by the partner wave that
  // holds the other 64 columns of the head (8 waves x 128 rows x 8 chunks fp32 = 32 KB; with the
  // 128 KB double buffer the workgroup declares all 160 KB of the CU's LDS)
  __shared__ float hnx[EK == EK_HEADNORM ? 8 * TM * 8 : 1];

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid >> 2, wn = wid & 3;
  const int z = blockIdx.y;
  A += z * sA;
  W += z * sW;
  const int ntl = tiles_m * tiles_n;
  const int q8 = ntl >> 3, r8 = ntl & 7;
  // group-M height, chosen on the host (launch_ps_ek; tile 18: diagnostic override)
  const int GM = ep.gm > 0 ? ep.gm : 8;
  // tile t -> origin: gemm_bf16_pp2_kernel's XCD-chunked group-M order with t in place of the
  // block id (t = blockIdx.x + r * gridDim.x keeps t & 7 = the XCD when gridDim.x % 8 == 0)
  auto origin = [&](int t, int& m0, int& n0) __attribute__((always_inline)) {
    const int xcd = t & 7;
    const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (t >> 3);
    const int grp = wg / (GM * tiles_n);
    const int fm = grp * GM;
    const int gm = min(tiles_m - fm, GM);
    const int rem = wg - grp * GM * tiles_n;
    m0 = (fm + rem % gm) * BM;
    n0 = (rem / gm) * BN;
  };

  // per-lane 32-bit byte offsets of the staging rows (SADDR-form DMA: half the VGPRs of pointers)
  uint32_t doff[4][2];
  auto setup = [&](int m0, int n0) __attribute__((always_inline)) {
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int row = chunk_row(c, 2 * wid + h) + (lane >> 3);
        const int gc = (lane & 7) ^ ((row >> 1) & 7);
        const bool isA = (c == 0 || c == 3);
        const int64_t e = isA ? (int64_t)min(m0 + row, M - 1) * lda : (int64_t)min(n0 + row, N - 1) * ldw;
        doff[c][h] = (uint32_t)((e + gc * 8) * 2);
      }
  };
  const uint32_t lds0 = lds_addr_of(lds);
  auto dma = [&](int c, int kt) __attribute__((always_inline)) {
    const bf16_t* base = ((c == 0 || c == 3) ? A + tap_delta(ep, kt * BK, lda) : W) + kt * BK;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int rb = chunk_row(c, 2 * wid + h);
      const uint32_t dst = lds0 + (uint32_t)(((kt & 1) * STAGE + ((c == 0 || c == 3) ? 0 : BM * BK) + rb * BK) * 2);
      glds16s(base, doff[c][h], __builtin_amdgcn_readfirstlane(dst));
    }
  };
  // tile prologue: K-tile 0 whole, chunks 0-2 of K-tile 1 (14 DMA per wave; the host ensures nk >= 2)
  auto prologue = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int c = 0; c < 4; ++c) dma(c, 0);
    dma(0, 1); dma(1, 1); dma(2, 1);
  };

  const int nk = K / BK;
  int t = blockIdx.x;
  if (t >= ntl) return;
  int m0, n0;
  origin(t, m0, n0);
  setup(m0, n0);
  // EK_BIAS: the bias of this lane's accumulator columns (n0 + wn*TN + j*16 + cq + r) of a tile is
  // loaded just before the tile's prologue DMA (older than every DMA the K loop waits for, so the
  // counted waits are unchanged) and consumed after the K loop's final vmcnt(0)
  const int cq = 4 * (lane >> 4);
  uint2 bb[FN], bbn[FN];
  auto load_bias = [&](int n0t, uint2 (&d)[FN]) __attribute__((always_inline)) {
    const bf16_t* bp = (const bf16_t*)ep.bias + z * ep.stride_bias + n0t + wn * TN + cq;
#pragma unroll
    for (int j = 0; j < FN; ++j) d[j] = *(const uint2*)(bp + j * 16);
  };
  if constexpr (EK == EK_BIAS) load_bias(n0, bb);
  prologue();

  // the output's last row ends at column N (N / 2 for SwiGLU, whose output holds half the GEMM's columns): with
  // N there, row M would lie inside num_records whenever ldc < N, and the last tile row past M would be stored
  const __amdgpu_buffer_rsrc_t crs =
      brsrc((bf16_t*)Cv + z * sC, (uint32_t)(((int64_t)(M - 1) * ldc + (EK == EK_SWIGLU ? N / 2 : N)) * 2));
  const int frow = lane & 15;
  const int fsw = frow >> 1;
  bool first = true;
  for (;;) {
    if (first) vm_wait_n<8>(); else vm_wait_n<8 + SN>();
    pp_barrier();
    if (wm == 1) pp_barrier();  // waves 4-7 run one barrier (one segment) behind

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 af[4][2], bfr[4][2];
    for (int kt = 0; kt < nk; ++kt) {
      const bf16_t* As = lds + (kt & 1) * STAGE;
      const bf16_t* Bs = As + BM * BK;
      const bool n1 = kt + 1 < nk, n2 = kt + 2 < nk;
      const bool xs = !first && kt == 0;  // the previous tile's SN stores are still counted
#pragma unroll
      for (int ph = 0; ph < 2; ++ph) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int s = 0; s < 2; ++s)
            af[i][s] = *(const bf16x8*)(As + (wm * TM + ph * 64 + i * 16 + frow) * BK +
                                        (((4 * s + (lane >> 4)) ^ fsw) * 8));
        if (ph == 0) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int s = 0; s < 2; ++s)
              bfr[j][s] = *(const bf16x8*)(Bs + (wn * TN + j * 16 + frow) * BK +
                                           (((4 * s + (lane >> 4)) ^ fsw) * 8));
          if (n1) dma(3, kt + 1);
          if (!n1) vm_wait_n<0>();
          else if (xs) vm_wait_n<8 + SN>();
          else vm_wait_n<8>();
        } else {
          if (n2) { dma(0, kt + 2); dma(1, kt + 2); dma(2, kt + 2); }
          if (n2) { if (xs) vm_wait_n<8 + SN>(); else vm_wait_n<8>(); }
          else if (n1) { if (xs) vm_wait_n<2 + SN>(); else vm_wait_n<2>(); }
          else vm_wait_n<0>();
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        pp_barrier();
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int s = 0; s < 2; ++s)
              acc[ph * 4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j][s], af[i][s], acc[ph * 4 + i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        pp_barrier();
      }
    }
    if (wm == 0) pp_barrier();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // every wave's last fragment reads are done: both LDS buffers are free
    if constexpr (EK == EK_BIAS) {
#pragma unroll
      for (int j = 0; j < FN; ++j) asm volatile("" ::"v"(bb[j].x), "v"(bb[j].y));
    }

    const int tnext = t + gridDim.x;
    const bool more = tnext < ntl;
    // Output layout after one v_permlane16_swap per packed word of a fragment pair (j0, j1) =
    // (2p, 2p+1): lane group g = lane>>4 holds 8 consecutive columns of row m, at column
    // p*32 + (g&1)*16 + (g>>1)*8 of the wave's 64 — 16-B stores, 64 B per row per instruction.
    // N % 256 == 0 (host): no column overhang; rows >= M give byte offsets >= num_records
    // (m*ld >= (M-1)*ld + N), which the buffer unit drops (stores) or reads as 0 (loads).
    const int mb = m0 + wm * TM + (lane & 15);
    const int g4 = lane >> 4;
    const int cpos = (g4 & 1) * 16 + (g4 >> 1) * 8;   // column of this lane's 8 within a 32-column pair
    const int nb = n0 + wn * TN + cpos;
    auto swap_pair = [&](uint2 lo, uint2 hi) __attribute__((always_inline)) -> u32x4 {
      const auto s0 = __builtin_amdgcn_permlane16_swap(lo.x, hi.x, false, false);
      const auto s1 = __builtin_amdgcn_permlane16_swap(lo.y, hi.y, false, false);
      return u32x4{s0[0], s1[0], s0[1], s1[1]};
    };
    u32x4 xr[FM][FN / 2];
    float g[FN / 2][8];
    if constexpr (EK == EK_RESID) {
      const __amdgpu_buffer_rsrc_t ars =
          brsrc((const bf16_t*)ep.aux + z * ep.stride_aux, (uint32_t)(((int64_t)(M - 1) * ep.ld_aux + N) * 2));
#pragma unroll
      for (int ii = 0; ii < FM; ++ii) {
        const uint32_t off = (uint32_t)(((mb + ii * 16) * ep.ld_aux + nb) * 2);
#pragma unroll
        for (int p = 0; p < FN / 2; ++p)
          xr[ii][p] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(ars, off + p * 64, 0, 0));
      }
      if (ep.gate) {
        const bf16_t* gp = (const bf16_t*)ep.gate + z * ep.stride_gate + nb;
#pragma unroll
        for (int p = 0; p < FN / 2; ++p) load8(gp + p * 32, g[p]);
      }
    }
    // HEADNORM (q/k RMSNorm + half RoPE, ECHO_EPI_HEADNORM): the head of this wave's 64 columns (a head is
    // the 128 columns of waves (wm, 2p) and (wm, 2p+1)), its flags, and the norm weights of this lane's 16
    // columns, loaded before the prologue DMA like RESID's residual rows
    const int hidx = (n0 + (wn & ~1) * TN) >> 7;
    const int hblk = EK == EK_HEADNORM ? hidx / ep.hn_heads : 0;
    const int hhd = hidx - hblk * (EK == EK_HEADNORM ? ep.hn_heads : 0);
    const bool hnorm = EK == EK_HEADNORM && hblk < ep.hn_nblk;
    const bool hrope = hnorm && hhd < ep.hn_rope_heads;
    // lane-derived values recomputed from an opaque copy of the lane id, so that the compiler does not
    // hoist them above the K loop (which runs at the 256-VGPR limit)
    int hl = lane;
    if constexpr (EK == EK_HEADNORM) asm volatile("" : "+v"(hl));
    const int hg = hl >> 4, hrow = hl & 15;
    uint2 hw[FN];  // norm weights of this lane's 16 columns, loaded before the prologue DMA
    if constexpr (EK == EK_HEADNORM) {
      if (hnorm) {
        const bf16_t* wp = (const bf16_t*)ep.hn_w + hblk * ep.hn_w_stride + hhd * 128 + (wn & 1) * TN + 4 * hg;
#pragma unroll
        for (int j = 0; j < FN; ++j) hw[j] = *(const uint2*)(wp + j * 16);
      }
    }
    int m0n = 0, n0n = 0;
    if (more) {
      origin(tnext, m0n, n0n);
      setup(m0n, n0n);
      if constexpr (EK == EK_BIAS) load_bias(n0n, bbn);
      prologue();
    }
    if constexpr (EK == EK_RESID) {
      if (more) vm_wait_n<14>(); else vm_wait_n<0>();
    }

    // ---- epilogue from registers: exactly SN buffer stores per wave
    if constexpr (EK == EK_HEADNORM) {
      // Bitwise equal to gemm_epilogue's HEADNORM kind (and to echo_head_norm_rope): v = bf16(acc) (the
      // store rounding); per 8-column chunk c of a head the sum of squares in column order from 0; then
      // the 16-lane butterfly's tree over chunks (c ^ 8, c ^ 4, c ^ 2, c ^ 1; every level adds the same
      // two operands in either lane, so all chunks end with the same value); r = 1 / sqrtf(ss / 128 + eps);
      // v = bf16(v * r * w); RoPE on column pairs in fp32; one rounding at the store.
      // Register layout: acc[i][j][e] = row wm*128 + i*16 + (lane & 15), column wn*64 + j*16 + 4g + e
      // (g = lane >> 4): chunk 2j + (g >> 1) of the wave's 8, its columns 0-3 in lanes g = 0, 2 and 4-7 in
      // lanes g = 1, 3 (the partial sum crosses lane ^ 16 once); chunk c ^ 8 is the partner wave's same
      // chunk (LDS), c ^ 4 and c ^ 2 are this lane's j ^ 2 and j ^ 1, c ^ 1 is lane ^ 32.
      const int g = hg;
      const bool hi16 = (g & 1) != 0;
      uint2 hp[FM][FN];   // the store rounding first: bf16(acc), 2 per register (acc is dead after this)
#pragma unroll
      for (int ii = 0; ii < FM; ++ii)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          hp[ii][j] = make_uint2(pack2bf(acc[ii][j][0], acc[ii][j][1]), pack2bf(acc[ii][j][2], acc[ii][j][3]));
      auto unpack = [](uint2 u, float (&v)[4]) __attribute__((always_inline)) {
        v[0] = bf2f(u.x & 0xffffu); v[1] = bf2f(u.x >> 16); v[2] = bf2f(u.y & 0xffffu); v[3] = bf2f(u.y >> 16);
      };
      // (cos, sin) of this lane's 2 column pairs per j (fp32 table rows, like the reference's complex64
      // freqs, model.py:9-24), 4 rows at a time (64 registers), loaded after the prologue DMA (issuing
      // them before it, or before the sums below, spills: the K loop runs at 256 VGPRs)
      float4 rc[FM / 2][FN];
      auto load_rope = [&](int i0) __attribute__((always_inline)) {
#pragma unroll
        for (int ii = 0; ii < FM / 2; ++ii) {
          const int m = m0 + wm * TM + (i0 + ii) * 16 + hrow;
          const int pos = ep.hn_pos0 + ep.hn_pos_mult * (min(m, M - 1) % ep.hn_seq_len);
          const float* rp = ep.hn_rope + ((int64_t)pos * 64 + (wn & 1) * 32 + 2 * g) * 2;
#pragma unroll
          for (int j = 0; j < FN; ++j) rc[ii][j] = *(const float4*)(rp + j * 16);
        }
      };
      if (hnorm) {
#pragma unroll
        for (int ii = 0; ii < FM; ++ii)
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            float v[4];
            unpack(hp[ii][j], v);
            float h = 0.f;
#pragma unroll
            for (int e = 0; e < 4; ++e) h += v[e] * v[e];   // columns 0-3 (lanes g = 0, 2)
            const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(h), __float_as_uint(h), false, false);
            float c8 = __uint_as_float(hi16 ? sw[0] : sw[1]);   // lane ^ 16's partial
#pragma unroll
            for (int e = 0; e < 4; ++e) c8 += v[e] * v[e];  // columns 4-7 continue it: the chunk's sum
            if (hi16) hnx[(wid * TM + ii * 16 + hrow) * 8 + 2 * j + (g >> 1)] = c8;
          }
      }
      // every wave (all take this path) has written its chunk sums: raw barrier after the LDS writes retire
      // (__syncthreads' fence would also wait for the prologue DMA, vmcnt(0))
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      pp_barrier();
      if (hnorm) {
        float hr[FM];
#pragma unroll
        for (int ii = 0; ii < FM; ++ii) {
          float t1[FN];
          const int ro = ii * 16 + hrow;
#pragma unroll
          for (int j = 0; j < FN; ++j)   // lanes g = 1, 3: this chunk + the partner wave's same chunk (c ^ 8)
            t1[j] = hnx[(wid * TM + ro) * 8 + 2 * j + (g >> 1)] + hnx[((wid ^ 1) * TM + ro) * 8 + 2 * j + (g >> 1)];
          const float t3 = (t1[0] + t1[2]) + (t1[1] + t1[3]);   // c ^ 4 (j ^ 2), then c ^ 2 (j ^ 1)
          const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(t3), __float_as_uint(t3), false, false);
          const float t4 = t3 + __uint_as_float(hl >= 32 ? sw[0] : sw[1]);   // c ^ 1 (lane ^ 32)
          const float r = 1.0f / sqrtf(t4 / 128.0f + ep.hn_eps);
          const auto sr = __builtin_amdgcn_permlane16_swap(__float_as_uint(r), __float_as_uint(r), false, false);
          hr[ii] = hi16 ? r : __uint_as_float(sr[1]);  // lanes g = 0, 2 take lane ^ 16's
        }
        if (more) vm_wait_n<14>(); else vm_wait_n<0>();   // the weights (older than the prologue DMA)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          float wv[4];
          unpack(hw[j], wv);
#pragma unroll
          for (int ii = 0; ii < FM; ++ii) {
            float v[4];
            unpack(hp[ii][j], v);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = (v[e] * hr[ii]) * wv[e];
            hp[ii][j] = make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));   // bf16(v * r * w)
          }
        }
      }
      if (hrope) {
#pragma unroll
        for (int i0 = 0; i0 < FM; i0 += FM / 2) {
          load_rope(i0);
          // all 16 loads in flight together, then one wait (without the pin hipcc sinks each load to
          // its use and waits for it there: 16 serial L2 round trips per half)
#pragma unroll
          for (int ii = 0; ii < FM / 2; ++ii)
#pragma unroll
            for (int j = 0; j < FN; ++j)
              asm volatile("" : "+v"(rc[ii][j].x), "+v"(rc[ii][j].y), "+v"(rc[ii][j].z), "+v"(rc[ii][j].w));
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
          for (int ii = 0; ii < FM / 2; ++ii)
#pragma unroll
            for (int j = 0; j < FN; ++j) {
              float v[4];
              unpack(hp[i0 + ii][j], v);
              const float4 cs = rc[ii][j];
              const float y0 = (v[0] * cs.x) - (v[1] * cs.y), y1 = (v[0] * cs.y) + (v[1] * cs.x);
              const float y2 = (v[2] * cs.z) - (v[3] * cs.w), y3 = (v[2] * cs.w) + (v[3] * cs.z);
              hp[i0 + ii][j] = make_uint2(pack2bf(y0, y1), pack2bf(y2, y3));
            }
        }
      }
#pragma unroll
      for (int ii = 0; ii < FM; ++ii) {
        const uint32_t off = (uint32_t)(((mb + ii * 16) * ldc + nb) * 2);
#pragma unroll
        for (int p = 0; p < FN / 2; ++p)
          __builtin_amdgcn_raw_buffer_store_b128(swap_pair(hp[ii][2 * p], hp[ii][2 * p + 1]), crs, off + p * 64, 0, 0);
      }
    } else if constexpr (EK == EK_SWIGLU) {
      // gate/up column blocks interleaved by 16 (j = 2jj gate, 2jj+1 up), as gemm_epilogue; the
      // two output fragments (jj = 0, 1) form the swapped pair: 8 columns of 32 per lane
      const int nbo = n0 / 2 + wn * (TN / 2) + cpos;
#pragma unroll
      for (int ii = 0; ii < FM; ++ii) {
        uint2 q[2];
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          float u[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float a = rbf(acc[ii][2 * jj][r]), b = rbf(acc[ii][2 * jj + 1][r]);
            u[r] = rbf(silu_bf16in(a)) * b;
          }
          q[jj] = make_uint2(pack2bf(u[0], u[1]), pack2bf(u[2], u[3]));
        }
        const u32x4 o = swap_pair(q[0], q[1]);
        __builtin_amdgcn_raw_buffer_store_b128(o, crs, (uint32_t)(((mb + ii * 16) * ldc + nbo) * 2), 0, 0);
      }
    } else {
#pragma unroll
      for (int ii = 0; ii < FM; ++ii) {
        const uint32_t off = (uint32_t)(((mb + ii * 16) * ldc + nb) * 2);
#pragma unroll
        for (int p = 0; p < FN / 2; ++p) {
          f32x4 c0 = acc[ii][2 * p];
          f32x4 c1 = acc[ii][2 * p + 1];
          if constexpr (EK == EK_BIAS) {
            // acc + bias in fp32, rounded once (gemm_epilogue's generic kind: x += bias; rbf)
            const uint2 b0 = bb[2 * p], b1 = bb[2 * p + 1];
            c0[0] += bf2f(b0.x & 0xffffu); c0[1] += bf2f(b0.x >> 16);
            c0[2] += bf2f(b0.y & 0xffffu); c0[3] += bf2f(b0.y >> 16);
            c1[0] += bf2f(b1.x & 0xffffu); c1[1] += bf2f(b1.x >> 16);
            c1[2] += bf2f(b1.y & 0xffffu); c1[3] += bf2f(b1.y >> 16);
          }
          u32x4 o = swap_pair(make_uint2(pack2bf(c0[0], c0[1]), pack2bf(c0[2], c0[3])),
                              make_uint2(pack2bf(c1[0], c1[1]), pack2bf(c1[2], c1[3])));
          if constexpr (EK == EK_RESID) {
            // out = bf16(x + bf16(g * bf16(acc))): gemm_epilogue's stage-2 rounding points
#pragma unroll
            for (int w = 0; w < 4; ++w) {
              float v0 = bf2f(o[w] & 0xffffu), v1 = bf2f(o[w] >> 16);
              if (ep.gate) { v0 = rbf(g[p][2 * w] * v0); v1 = rbf(g[p][2 * w + 1] * v1); }
              v0 = bf2f(xr[ii][p][w] & 0xffffu) + v0;
              v1 = bf2f(xr[ii][p][w] >> 16) + v1;
              o[w] = pack2bf(v0, v1);
            }
          }
          __builtin_amdgcn_raw_buffer_store_b128(o, crs, off + p * 64, 0, 0);
        }
      }
    }
    if (!more) break;
    t = tnext;
    m0 = m0n;
    n0 = n0n;
    if constexpr (EK == EK_BIAS) {
#pragma unroll
      for (int j = 0; j < FN; ++j) bb[j] = bbn[j];
    }
    first = false;
  }
}

// ----------------------------------------------------------------------------- 320 x 256 tile
// gemm_bf16_t320_kernel<EK_RESID | EK_SWIGLU | EK_HEADNORM>: 320x256x64 tiles for the N = 2048 gated-residual
// GEMMs (Wo, W2), W13 at M = 10240 (SwiGLU: 5.75 rounds of 320-row tiles vs 7.2 of 256-row ones) and the
// blockwise QKVG launches (M = 2560 / 7680: 1 / 3 rounds instead of 1.25 / 3.75), whose
// 256x256 tile count leaves a partial last round at the decoder's M (M = 30720: 960 tiles = 3.75 rounds of
// 256 CUs, M = 10240: 1.25 rounds) while 320-row tiles divide it exactly (768 / 256 tiles = 3 / 1 rounds).
// Same fragments, MFMA and per-element K order as the 256x256 kernels: bitwise-equal results, so the
// B = 16 rows still equal B = 1 runs. 8 waves as 4 (M) x 2 (N), 80 x 128 outputs per wave:
//   phase 0: the wave's 5 x 2 A fragments (held for the K-tile) x its W columns 0-63   (40 MFMA)
//   phase 1: the same A fragments x its W columns 64-127                                (40 MFMA)
// LDS stage = A 320 x 64 | W 256 x 64 (72 KB), 2 stages. DMA chunks (1 KiB wave-instructions, the
// source-side swizzle of the other kernels): cA = all A rows (5 per wave), cW0 = the W rows phase 0 reads
// (2 per wave), cW1 = phase 1's (2 per wave). cA + cW0 of K-tile k+2 are issued in phase 1 of tile k,
// cW1 of tile k+1 in phase 0 of tile k: gemm_bf16_pp2_kernel's schedule and barrier argument with
// c0-c2 -> cA + cW0 and c3 -> cW1, so the steady-state waits are vmcnt(9) (2 + 7 younger pieces).
// Epilogue from registers, row fragment by row fragment (the residual rows of the next one in flight).
//
// PER = 1 (persistent; production for SwiGLU launches of >= 4 tiles per CU, see launch_t320): one workgroup
// per CU walks tiles blockIdx.x, + gridDim.x, ... (gridDim.x a multiple of 8, so t & 7 stays the XCD of the
// block-id map); after a tile's K loop the next tile's prologue DMA is issued BEFORE its epilogue, so the first
// K-tile loads of tile i+1 are in flight under the epilogue math and store burst of tile i (gemm_bf16_ps_kernel's
// scheme). vmcnt counts loads, LDS-DMA and stores in issue order: the SN = t320_sn(EK) stores of a wave are
// younger than the prologue DMA, so the prologue wait and both waits of K-tile 0 allow SN more in flight;
// K-tile 1's first wait (cW1 of K-tile 1, issued after the stores) retires them. Memory operations the compiler
// adds (spill code) are issued after the ops those waits target, so they only make the waits stricter.
// Same K loop, same per-element K order: bitwise equal to PER = 0.
constexpr int t320_sn(int ek) { return ek == EK_SWIGLU ? 10 : 20; }  // stores per wave per tile (FM x 2 / FM x 4)

// The epilogue reads its arguments (C, M, N, the Epi fields) through an opaque copy of the kernarg pointer taken
// after each tile's K loop: otherwise hipcc hoists them out of the tile loop and holds them in SGPRs across the
// K loop (106 SGPRs, spills into VGPRs at the 256-VGPR limit).
struct T320Args {
  const bf16_t* A; int64_t lda; const bf16_t* W; int64_t ldw;
  void* Cv; int64_t ldc;
  int M, N, K, tiles_m, tiles_n;
  Epi ep;
};

template <int EK, int SP = 1, int PER = 0>
__global__ void __launch_bounds__(512) gemm_bf16_t320_kernel(T320Args args) {
  static_assert(EK == EK_RESID || EK == EK_SWIGLU || EK == EK_HEADNORM, "320-row tiles: residual / SwiGLU / head norm");
  static_assert(!(PER && SP), "persistent form: 2 / 7 DMA split only");
  using KA = const __attribute__((address_space(4))) T320Args;
  KA* const kp0 = (KA*)__builtin_amdgcn_kernarg_segment_ptr();
  (void)args;
  // PER: the kernarg pointer through an opaque copy, so that values derived from the arguments at a tile
  // boundary (origin, next-tile bases, epilogue arguments) are recomputed there instead of held across the loop
  auto kargs = [&]() __attribute__((always_inline)) -> KA* {
    uint64_t v = (uint64_t)kp0;
    if constexpr (PER) asm volatile("" : "+s"(v));
    return (KA*)v;
  };
  const int64_t lda = kp0->lda, ldw = kp0->ldw;
  const int K = kp0->K;
  constexpr int BM = 320, BN = 256, TM = 80, TN = 128, FM = 5, FN = 8;
  constexpr int STAGE = (BM + BN) * BK;
  constexpr int SN = t320_sn(EK);
  // + the persistent head-norm form's norm weights: 128 per wave (its head), staged once per tile (2 KiB)
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * STAGE + ((EK == EK_HEADNORM && PER) ? 8 * 128 : 0)];

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int grp = wid >> 2;  // ping-pong group: waves 4-7 run one barrier behind
  // tile t -> origin: XCD-chunked (t & 7 = XCD) group-M order (GM rows of tiles per group: Epi::gm, default 8)
  auto origin = [&](int t, int& m0o, int& n0o) __attribute__((always_inline)) {
    KA* const kq = kargs();
    const int tiles_m = kq->tiles_m, tiles_n = kq->tiles_n;
    const int GM = kq->ep.gm > 0 ? kq->ep.gm : 8;
    const int nwg = tiles_m * tiles_n;
    const int q8 = nwg >> 3, r8 = nwg & 7;
    const int xcd = t & 7;
    const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (t >> 3);
    const int gq = wg / (GM * tiles_n);
    const int fm = gq * GM;
    const int gm = min(tiles_m - fm, GM);
    const int rem = wg - gq * GM * tiles_n;
    m0o = (fm + rem % gm) * BM;
    n0o = (rem / gm) * BN;
  };
  const int nwg = kp0->tiles_m * kp0->tiles_n;
  int tcur = blockIdx.x;
  if (PER && tcur >= nwg) return;
  int m0, n0;
  origin(tcur, m0, n0);

  // per-lane source offsets of an 8-row group (row rb + lane/8, chunk (lane&7) ^ ((row>>1)&7)); the
  // swizzle term depends only on the group's parity (rb/8 odd adds 4)
  // (PER: recomputed from an opaque copy of the lane id at the top of every tile, so that they are dead
  // during the epilogue, which runs at the 256-VGPR limit)
  uint32_t vA[2], vW[2];
  auto lane_offsets = [&]() __attribute__((always_inline)) {
    int ln = lane;
    if constexpr (PER) asm volatile("" : "+v"(ln));
    const int l8 = ln >> 3;
#pragma unroll
    for (int par = 0; par < 2; ++par) {
      const int gc = (ln & 7) ^ ((4 * par + (l8 >> 1)) & 7);
      vA[par] = (uint32_t)((l8 * lda + gc * 8) * 2);
      vW[par] = (uint32_t)((l8 * ldw + gc * 8) * 2);
    }
  };
  lane_offsets();
  const uint32_t lds0 = lds_addr_of(lds);
  const bf16_t* Ab = kp0->A + (int64_t)m0 * lda;
  const bf16_t* Wb = kp0->W + (int64_t)n0 * ldw;
  // chunk c (0 = cA, 1 = cW0, 2 = cW1) of K-tile kt into stage kt & 1 (of the tile Ab / Wb point at)
  auto dma = [&](int c, int kt) __attribute__((always_inline)) {
    const uint32_t st = lds0 + (uint32_t)((kt & 1) * STAGE * 2);
    if (c == 0) {
#pragma unroll
      for (int q = 0; q < 5; ++q) {
        const int rb = (q * 8 + wid) * 8;
        glds16s(Ab + (int64_t)rb * lda + kt * BK, vA[(rb >> 3) & 1], __builtin_amdgcn_readfirstlane(st + rb * BK * 2));
      }
    } else {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int g = h * 8 + wid;
        const int rb = (g < 8 ? g * 8 : 128 + (g - 8) * 8) + (c == 2 ? 64 : 0);
        glds16s(Wb + (int64_t)rb * ldw + kt * BK, vW[(rb >> 3) & 1],
                __builtin_amdgcn_readfirstlane(st + (BM + rb) * BK * 2));
      }
    }
  };

  const int nk = K / BK;
  // SP = 1 (tile 21, A/B): DMA balanced between the two L segments — phase 0 of tile k issues cW0 and cW1 of
  // tile k+1 (4 pieces), phase 1 cA of tile k+2 (5) instead of 2 / 7; cW0 then has one phase of DMA latency
  // instead of two. Waits: phase 0 retires cW1(k) -> vmcnt(9) (cA(k+1) 5 + this phase's 4 younger), phase 1
  // retires cA(k+1) + cW0(k+1) -> vmcnt(7). Measured within +-1 % of the 2 / 7 schedule on every decoder
  // shape (profiles/r3_gemm_t320_dma_balance.txt); round 5, replayed from graphs: -1 / -2 % for the gated residual
  // at 3 tiles per CU (Wo / W2 at M = 30720), production there (launch_t320).
  // prologue: tile 0 (cA, cW0, then cW1) and cA (SP) or cA + cW0 (!SP) of tile 1; the tile loop's first wait
  // retires tile 0's cA + cW0 (PER: the previous tile's SN stores are younger and stay in flight)
  auto prologue = [&]() __attribute__((always_inline)) {
    dma(0, 0); dma(1, 0); dma(2, 0);
    if (nk > 1) {
      dma(0, 1);
      if constexpr (!SP) dma(1, 1);
    }
  };
  prologue();

  // ---- epilogue: out = bf16(x + bf16(g * bf16(acc))) (the persistent kernel's RESID kind). A lane holds
  // rows mb + 16 ii, columns 16 j + 4 (lane >> 4) .. + 3 of the wave's 128; one v_permlane16_swap per
  // packed word of a fragment pair (2p, 2p+1) gives it 8 consecutive columns (16-B accesses).
  auto swap_pair = [&](uint2 lo, uint2 hi) __attribute__((always_inline)) -> u32x4 {
    const auto s0 = __builtin_amdgcn_permlane16_swap(lo.x, hi.x, false, false);
    const auto s1 = __builtin_amdgcn_permlane16_swap(lo.y, hi.y, false, false);
    return u32x4{s0[0], s1[0], s0[1], s1[1]};
  };
  bool first = true;
  for (;;) {
    if (PER && !first) lane_offsets();
    if (nk > 1) {
      if constexpr (SP) vm_wait_n<7>();
      else if (first) vm_wait_n<9>();
      else vm_wait_n<9 + SN>();
    } else {
      if (first) vm_wait_n<2>(); else vm_wait_n<2 + SN>();
    }
    pp_barrier();
    if (grp == 1) pp_barrier();

    // fragment-read lane terms (PER: from an opaque lane copy per tile, dead during the epilogue)
    int lf = lane;
    if constexpr (PER) asm volatile("" : "+v"(lf));
    const int frow = lf & 15, fq = lf >> 4;
    const int fsw = frow >> 1;
    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 af[FM][2], bfr[4][2];
    for (int kt = 0; kt < nk; ++kt) {
      const bf16_t* As = lds + (kt & 1) * STAGE;
      const bf16_t* Bs = As + BM * BK;
      const bool n1 = kt + 1 < nk, n2 = kt + 2 < nk;
      const bool xs = PER && !first && kt == 0;  // the previous tile's SN stores are still counted
#pragma unroll
      for (int ph = 0; ph < 2; ++ph) {
        // ---- L segment
        if (ph == 0) {
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int s = 0; s < 2; ++s)
              af[i][s] = *(const bf16x8*)(As + (wm * TM + i * 16 + frow) * BK + (((4 * s + fq) ^ fsw) * 8));
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int s = 0; s < 2; ++s)
            bfr[j][s] = *(const bf16x8*)(Bs + (wn * TN + ph * 64 + j * 16 + frow) * BK + (((4 * s + fq) ^ fsw) * 8));
        if constexpr (SP) {
          if (ph == 0) {
            if (n1) { dma(1, kt + 1); dma(2, kt + 1); }
            // retire cW1 of tile kt (issued in phase 0 of tile kt-1 / the prologue)
            if (n1) vm_wait_n<9>(); else vm_wait_n<0>();
          } else {
            if (n2) dma(0, kt + 2);
            // retire cA + cW0 of tile kt+1
            if (n2) vm_wait_n<7>(); else if (n1) vm_wait_n<2>(); else vm_wait_n<0>();
          }
        } else {
          if (ph == 0) {
            if (n1) dma(2, kt + 1);
            // retire cW1 of tile kt (issued in phase 0 of tile kt-1 / the prologue)
            if (n1) { if (xs) vm_wait_n<9 + SN>(); else vm_wait_n<9>(); } else vm_wait_n<0>();
          } else {
            if (n2) { dma(0, kt + 2); dma(1, kt + 2); }
            // retire cA + cW0 of tile kt+1
            if (n2) { if (xs) vm_wait_n<9 + SN>(); else vm_wait_n<9>(); }
            else if (n1) { if (xs) vm_wait_n<2 + SN>(); else vm_wait_n<2>(); }
            else vm_wait_n<0>();
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        pp_barrier();
        // ---- C segment
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int s = 0; s < 2; ++s)
              acc[i][ph * 4 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j][s], af[i][s], acc[i][ph * 4 + j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        pp_barrier();
      }
    }
    if (grp == 0) pp_barrier();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    bool more = false;
    int m0n = 0, n0n = 0;
    if constexpr (PER) {
      // every wave's last fragment reads are retired: both LDS stages take the next tile's prologue DMA
      pp_barrier();
      tcur += gridDim.x;
      more = tcur < nwg;
      if (more) {
        origin(tcur, m0n, n0n);
        KA* const kq = kargs();
        Ab = kq->A + (int64_t)m0n * lda;
        Wb = kq->W + (int64_t)n0n * ldw;
        lane_offsets();
        prologue();
      }
    }
    KA* const kp = kargs();
    auto& ep = kp->ep;
    const int M = kp->M, N = kp->N;
    const int64_t ldc = kp->ldc;
    const __amdgpu_buffer_rsrc_t crs =
        brsrc(kp->Cv, (uint32_t)(((int64_t)(M - 1) * ldc + (EK == EK_SWIGLU ? N / 2 : N)) * 2));
    // lane-derived epilogue values from an opaque copy of the lane id (PER: not hoisted out of the tile loop,
    // where they would stay live across the K loop)
    int le = lane;
    if constexpr (PER) asm volatile("" : "+v"(le));
    const int g4 = le >> 4;
    const int cpos = (g4 & 1) * 16 + (g4 >> 1) * 8;
    const int mb = m0 + wm * TM + (le & 15);
    const int nb = n0 + wn * TN + cpos;

    if constexpr (EK == EK_HEADNORM) {
      // q/k RMSNorm + half RoPE (ECHO_EPI_HEADNORM), bitwise equal to the persistent kernel's HEADNORM kind
      // and to echo_head_norm_rope: v = bf16(acc); per 8-column chunk c of the head the sum of squares in
      // column order from 0; then the butterfly's tree over chunks (c ^ 8, c ^ 4, c ^ 2, c ^ 1); r = 1 /
      // sqrtf(ss / 128 + eps); v = bf16(v * r * w); RoPE on column pairs in fp32; one rounding at the store.
      // Here a wave's 128 columns are one whole head: chunk 2j + (g >> 1) of column fragment j (g = lane >> 4),
      // its columns 0-3 in lanes g = 0, 2 and 4-7 in g = 1, 3 (one lane ^ 16 exchange); c ^ 8 is fragment
      // j ^ 4 and c ^ 4, c ^ 2 fragments j ^ 2, j ^ 1 of the same lane; c ^ 1 is lane ^ 32.
      const int hidx = (n0 + wn * TN) >> 7;
      const int hblk = hidx / ep.hn_heads, hhd = hidx - hblk * ep.hn_heads;
      const bool hnorm = hblk < ep.hn_nblk, hrope = hnorm && hhd < ep.hn_rope_heads;
      const bool hi16 = (g4 & 1) != 0;
      auto unpack = [](uint2 u, float (&v)[4]) __attribute__((always_inline)) {
        v[0] = bf2f(u.x & 0xffffu); v[1] = bf2f(u.x >> 16); v[2] = bf2f(u.y & 0xffffu); v[3] = bf2f(u.y >> 16);
      };
      // the store rounding first for the whole tile: bf16(acc), 2 per register (80 VGPRs instead of the 160 of
      // acc, which is dead after this: room for the table loads without spills)
      uint2 hpa[FM][FN];
#pragma unroll
      for (int ii = 0; ii < FM; ++ii)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          hpa[ii][j] = make_uint2(pack2bf(acc[ii][j][0], acc[ii][j][1]), pack2bf(acc[ii][j][2], acc[ii][j][3]));
      // PER: materialised here (hipcc would otherwise sink the packs to their uses and keep acc live)
      if constexpr (PER) {
#pragma unroll
        for (int ii = 0; ii < FM; ++ii)
#pragma unroll
          for (int j = 0; j < FN; ++j) asm volatile("" : "+v"(hpa[ii][j].x), "+v"(hpa[ii][j].y));
      }
      // norm weights: PER stages the wave's 128 (one global load per lane, one latency per tile) in its own 256 B
      // of LDS past the ring and reads them per row fragment, instead of holding 16 registers across the row
      // loop (that live range spilled) or re-reading them from global memory per fragment (a load latency
      // exposed five times per tile)
      const bf16_t* wp = (const bf16_t*)ep.hn_w + hblk * ep.hn_w_stride + hhd * 128 + 4 * g4;
      uint2 hw[FN];
      bf16_t* const hwl = lds + 2 * STAGE + wid * 128;
      if (!PER && hnorm) {
#pragma unroll
        for (int j = 0; j < FN; ++j) hw[j] = *(const uint2*)(wp + j * 16);
      }
      if constexpr (PER) {
        if (hnorm) {
          const uint32_t wv = *(const uint32_t*)((const bf16_t*)ep.hn_w + hblk * ep.hn_w_stride + hhd * 128 + 2 * le);
          *(uint32_t*)(hwl + 2 * le) = wv;
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
      }
#pragma unroll
      for (int ii = 0; ii < FM; ++ii) {
        const int m = mb + ii * 16;
        float4 rc[FN];
        const int pos = ep.hn_pos0 + ep.hn_pos_mult * (min(m, M - 1) % ep.hn_seq_len);
        const float* rp = ep.hn_rope + ((int64_t)pos * 64 + 2 * g4) * 2;
        if (!PER && hrope) {  // (cos, sin) of the lane's 2 column pairs per fragment, in flight during the sums
#pragma unroll
          for (int j = 0; j < FN; ++j) rc[j] = *(const float4*)(rp + j * 16);
        }
        uint2 hp[FN];
#pragma unroll
        for (int j = 0; j < FN; ++j) hp[j] = hpa[ii][j];
        if constexpr (PER) {
          if (hnorm) {
#pragma unroll
            for (int j = 0; j < FN; ++j) hw[j] = *(const uint2*)(hwl + 4 * g4 + j * 16);
          }
        }
        if (hnorm) {
          float c8[FN];
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            float v[4];
            unpack(hp[j], v);
            float h = 0.f;
#pragma unroll
            for (int e = 0; e < 4; ++e) h += v[e] * v[e];   // columns 0-3 (lanes g = 0, 2)
            const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(h), __float_as_uint(h), false, false);
            float c = __uint_as_float(hi16 ? sw[0] : sw[1]);  // lane ^ 16's partial
#pragma unroll
            for (int e = 0; e < 4; ++e) c += v[e] * v[e];  // columns 4-7: the chunk's sum (lanes g = 1, 3)
            c8[j] = c;
          }
          const float t3 = ((c8[0] + c8[4]) + (c8[2] + c8[6])) + ((c8[1] + c8[5]) + (c8[3] + c8[7]));
          const auto s32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(t3), __float_as_uint(t3), false, false);
          const float t4 = t3 + __uint_as_float(le >= 32 ? s32[0] : s32[1]);   // c ^ 1 (lane ^ 32)
          const float r = 1.0f / sqrtf(t4 / 128.0f + ep.hn_eps);
          const auto sr = __builtin_amdgcn_permlane16_swap(__float_as_uint(r), __float_as_uint(r), false, false);
          const float rr = hi16 ? r : __uint_as_float(sr[1]);  // lanes g = 0, 2 take lane ^ 16's
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            float v[4], wv[4];
            unpack(hp[j], v);
            unpack(hw[j], wv);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = (v[e] * rr) * wv[e];
            hp[j] = make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));   // bf16(v * r * w)
          }
          if (hrope) {
#pragma unroll
            for (int j = 0; j < FN; ++j) {
              float v[4];
              unpack(hp[j], v);
              const float4 cs = PER ? *(const float4*)(rp + j * 16) : rc[j];  // PER: loaded at the use
              const float y0 = (v[0] * cs.x) - (v[1] * cs.y), y1 = (v[0] * cs.y) + (v[1] * cs.x);
              const float y2 = (v[2] * cs.z) - (v[3] * cs.w), y3 = (v[2] * cs.w) + (v[3] * cs.z);
              hp[j] = make_uint2(pack2bf(y0, y1), pack2bf(y2, y3));
            }
          }
        }
        const uint32_t off = (uint32_t)((m * ldc + nb) * 2);
#pragma unroll
        for (int p = 0; p < FN / 2; ++p)
          __builtin_amdgcn_raw_buffer_store_b128(swap_pair(hp[2 * p], hp[2 * p + 1]), crs, off + p * 64, 0, 0);
        // PER: one row fragment at a time (hipcc otherwise hoists the next fragments' table loads and spills)
        if constexpr (PER) __builtin_amdgcn_sched_barrier(0);
      }
    } else if constexpr (EK == EK_SWIGLU) {
      // gate / up column blocks interleaved by 16 (fragment 2jo gate, 2jo+1 up of output fragment jo): the
      // persistent kernel's SwiGLU kind; output fragments (2p, 2p+1) form the swapped pair of 8 columns
      const int nbo = n0 / 2 + wn * (TN / 2) + cpos;
#pragma unroll
      for (int ii = 0; ii < FM; ++ii) {
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          uint2 q[2];
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) {
            float u[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float a = rbf(acc[ii][4 * p + 2 * jj][r]), b = rbf(acc[ii][4 * p + 2 * jj + 1][r]);
              u[r] = rbf(silu_bf16in(a)) * b;
            }
            q[jj] = make_uint2(pack2bf(u[0], u[1]), pack2bf(u[2], u[3]));
          }
          __builtin_amdgcn_raw_buffer_store_b128(swap_pair(q[0], q[1]), crs,
                                                 (uint32_t)(((mb + ii * 16) * ldc + nbo + p * 32) * 2), 0, 0);
        }
      }
    } else {
      const __amdgpu_buffer_rsrc_t ars = brsrc(ep.aux, (uint32_t)(((int64_t)(M - 1) * ep.ld_aux + N) * 2));
      u32x4 gv[FN / 2];
      if (ep.gate) {
#pragma unroll
        for (int p = 0; p < FN / 2; ++p) gv[p] = *(const u32x4*)((const bf16_t*)ep.gate + nb + p * 32);
      }
      u32x4 xr[2][FN / 2];
      auto load_x = [&](int ii, u32x4 (&d)[FN / 2]) __attribute__((always_inline)) {
        const uint32_t off = (uint32_t)(((mb + ii * 16) * ep.ld_aux + nb) * 2);
#pragma unroll
        for (int p = 0; p < FN / 2; ++p)
          d[p] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(ars, off + p * 64, 0, 0));
      };
      load_x(0, xr[0]);
#pragma unroll
      for (int ii = 0; ii < FM; ++ii) {
        if (ii + 1 < FM) load_x(ii + 1, xr[(ii + 1) & 1]);
        const uint32_t off = (uint32_t)(((mb + ii * 16) * ldc + nb) * 2);
#pragma unroll
        for (int p = 0; p < FN / 2; ++p) {
          const f32x4 c0 = acc[ii][2 * p], c1 = acc[ii][2 * p + 1];
          u32x4 o = swap_pair(make_uint2(pack2bf(c0[0], c0[1]), pack2bf(c0[2], c0[3])),
                              make_uint2(pack2bf(c1[0], c1[1]), pack2bf(c1[2], c1[3])));
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            float v0 = bf2f(o[w] & 0xffffu), v1 = bf2f(o[w] >> 16);
            if (ep.gate) {
              v0 = rbf(bf2f(gv[p][w] & 0xffffu) * v0);
              v1 = rbf(bf2f(gv[p][w] >> 16) * v1);
            }
            v0 = bf2f(xr[ii & 1][p][w] & 0xffffu) + v0;
            v1 = bf2f(xr[ii & 1][p][w] >> 16) + v1;
            o[w] = pack2bf(v0, v1);
          }
          __builtin_amdgcn_raw_buffer_store_b128(o, crs, off + p * 64, 0, 0);
        }
      }
    }
    if (!more) break;
    m0 = m0n;
    n0 = n0n;
    first = false;
  }
}

// ----------------------------------------------------------------------------- fp32 (parity mode)
constexpr int FT = 64, FK = 16;

__global__ void __launch_bounds__(256)
gemm_f32_kernel(const float* __restrict__ A, int64_t lda, int64_t sA,
                const float* __restrict__ W, int64_t ldw, int64_t sW,
                void* __restrict__ Cv, int64_t ldc, int64_t sC, int M, int N, int K, Epi ep) {
  __shared__ float As[FK][FT + 1], Ws[FK][FT + 1];
  __shared__ float Ct[FT][FT + 1];
  const int z = blockIdx.z;
  A += z * sA;
  W += z * sW;
  const int m0 = blockIdx.y * FT, n0 = blockIdx.x * FT;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  float acc[4][4] = {};
  for (int k0 = 0; k0 < K; k0 += FK) {
    for (int e = threadIdx.x; e < FT * FK; e += 256) {
      const int r = e / FK, kk = e % FK;
      As[kk][r] = A[(int64_t)min(m0 + r, M - 1) * lda + k0 + kk + tap_delta(ep, k0, lda)];
      Ws[kk][r] = W[(int64_t)min(n0 + r, N - 1) * ldw + k0 + kk];
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < FK; ++kk) {
      float a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) { a[i] = As[kk][ty + 16 * i]; b[i] = Ws[kk][tx + 16 * i]; }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a[i], b[j], acc[i][j]);
    }
    __syncthreads();
  }
  const float* bias = ep.bias ? (const float*)ep.bias + z * ep.stride_bias : nullptr;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float v = acc[i][j];
      const int n = n0 + tx + 16 * j;
      if (bias && ep.epi != ECHO_EPI_SWIGLU) v += bias[min(n, N - 1)];
      if (ep.act == ECHO_ACT_SILU) v = silu_f(v);
      else if (ep.act == ECHO_ACT_GELU) v = gelu_erf(v);
      else if (ep.act == ECHO_ACT_SNAKE) v = snake_f32(v, ((const float*)ep.act_alpha)[min(n, N - 1)]);
      if (ep.out_div != 0.0f) v = v / ep.out_div;
      Ct[ty + 16 * i][tx + 16 * j] = v;
    }
  __syncthreads();
  if (ep.epi == ECHO_EPI_SWIGLU) {
    for (int e = threadIdx.x; e < FT * FT / 2; e += 256) {
      const int r = e / (FT / 2), o = e % (FT / 2);
      const int ca = (o / 16) * 32 + (o % 16);
      const int m = m0 + r, n = n0 / 2 + o;
      if (m < M && n < N / 2) ((float*)Cv)[z * sC + (int64_t)m * ldc + n] = silu_f(Ct[r][ca]) * Ct[r][ca + 16];
    }
    return;
  }
  for (int e = threadIdx.x; e < FT * FT; e += 256) {
    const int r = e / FT, cc = e % FT;
    const int m = m0 + r, n = n0 + cc;
    if (m >= M || n >= N) continue;
    float v = Ct[r][cc];
    if (ep.epi == ECHO_EPI_RESID) {
      if (ep.gate) v = ((const float*)ep.gate)[z * ep.stride_gate + n] * v;
      v = ((const float*)ep.aux)[z * ep.stride_aux + (int64_t)m * ep.ld_aux + n] + v;
    }
    ((float*)Cv)[z * sC + (int64_t)m * ldc + n] = v;
  }
}

// fp32 on the f32-input MFMA (v_mfma_f32_32x32x2_f32, exact f32 at the vector rate): 128x128x32
// tiles, 4 waves of 64x64 (2x2 MFMA tiles). The MFMA result is a k-ordered fmaf chain (one rounding
// per product, MI355X guide §3), i.e. the same arithmetic as gemm_f32_kernel's per-thread fmaf loop:
// both kernels are bitwise equal (tested), this one at ~3x the throughput. Operands staged k-major in
// LDS (A[k][m], W[k][n]) so a lane's fragment element (row l&31, k l>>5) is one conflict-free read;
// the next K-tile is prefetched into registers during the current tile's MFMAs. The epilogue
// (bias, SiLU/GELU/Snake, /out_div, SwiGLU, gated residual) is gemm_f32_kernel's on a 128x128 tile.
constexpr int QM = 128, QN = 128, QK = 32, QP = 4;
constexpr int Q_LDS = (2 * QK * (QM + QP) > QM * (QN + 1)) ? 2 * QK * (QM + QP) : QM * (QN + 1);

__global__ void __launch_bounds__(256)
gemm_f32_mfma_kernel(const float* __restrict__ A, int64_t lda, int64_t sA,
                     const float* __restrict__ W, int64_t ldw, int64_t sW,
                     void* __restrict__ Cv, int64_t ldc, int64_t sC, int M, int N, int K, Epi ep) {
  __shared__ __attribute__((aligned(16))) float sm[Q_LDS];
  float(*As)[QM + QP] = (float(*)[QM + QP])sm;
  float(*Ws)[QN + QP] = (float(*)[QN + QP])(sm + QK * (QM + QP));
  const int z = blockIdx.z;
  A += z * sA;
  W += z * sW;
  const int m0 = blockIdx.y * QM, n0 = blockIdx.x * QN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wm = wid >> 1, wn = wid & 1;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
  f32x4 ra[4], rw[4];
  auto gload = [&](int k0) {
    const int64_t td = tap_delta(ep, k0, lda);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + 256 * i, r = e >> 3, c = e & 7;
      ra[i] = *(const f32x4*)(A + (int64_t)min(m0 + r, M - 1) * lda + k0 + c * 4 + td);
      rw[i] = *(const f32x4*)(W + (int64_t)min(n0 + r, N - 1) * ldw + k0 + c * 4);
    }
  };
  gload(0);
  for (int k0 = 0; k0 < K; k0 += QK) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + 256 * i, r = e >> 3, c = e & 7;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        As[c * 4 + j][r] = ra[i][j];
        Ws[c * 4 + j][r] = rw[i][j];
      }
    }
    __syncthreads();
    if (k0 + QK < K) gload(k0 + QK);
#pragma unroll
    for (int kk = 0; kk < QK / 2; ++kk) {
      const int kr = kk * 2 + (lane >> 5), li = lane & 31;
      const float a0 = As[kr][wm * 64 + li], a1 = As[kr][wm * 64 + 32 + li];
      const float b0 = Ws[kr][wn * 64 + li], b1 = Ws[kr][wn * 64 + 32 + li];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
  }
  __syncthreads();
  float(*Ct)[QN + 1] = (float(*)[QN + 1])sm;
  const float* bias = ep.bias ? (const float*)ep.bias + z * ep.stride_bias : nullptr;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int r = wm * 64 + i * 32 + (g & 3) + 8 * (g >> 2) + 4 * (lane >> 5);
        const int cc = wn * 64 + j * 32 + (lane & 31);
        const int n = n0 + cc;
        float v = acc[i][j][g];
        if (bias && ep.epi != ECHO_EPI_SWIGLU) v += bias[min(n, N - 1)];
        if (ep.act == ECHO_ACT_SILU) v = silu_f(v);
        else if (ep.act == ECHO_ACT_GELU) v = gelu_erf(v);
        else if (ep.act == ECHO_ACT_SNAKE) v = snake_f32(v, ((const float*)ep.act_alpha)[min(n, N - 1)]);
        if (ep.out_div != 0.0f) v = v / ep.out_div;
        Ct[r][cc] = v;
      }
  __syncthreads();
  if (ep.epi == ECHO_EPI_SWIGLU) {
    for (int e = tid; e < QM * QN / 2; e += 256) {
      const int r = e / (QN / 2), o = e % (QN / 2);
      const int ca = (o / 16) * 32 + (o % 16);
      const int m = m0 + r, n = n0 / 2 + o;
      if (m < M && n < N / 2) ((float*)Cv)[z * sC + (int64_t)m * ldc + n] = silu_f(Ct[r][ca]) * Ct[r][ca + 16];
    }
    return;
  }
  for (int e = tid; e < QM * QN; e += 256) {
    const int r = e / QN, cc = e % QN;
    const int m = m0 + r, n = n0 + cc;
    if (m >= M || n >= N) continue;
    float v = Ct[r][cc];
    if (ep.epi == ECHO_EPI_RESID) {
      if (ep.gate) v = ((const float*)ep.gate)[z * ep.stride_gate + n] * v;
      v = ((const float*)ep.aux)[z * ep.stride_aux + (int64_t)m * ep.ld_aux + n] + v;
    }
    ((float*)Cv)[z * sC + (int64_t)m * ldc + n] = v;
  }
}

// the MFMA kernel reads 16-B rows chunks: 16-B aligned operands, K-tiles that never straddle a conv tap
bool f32_mfma_ok(const EchoGemmArgs* a) {
  if (a->tile == 19) return false;  // diagnostic: force the scalar fp32 kernel
  if (((uintptr_t)a->A | (uintptr_t)a->W) & 15) return false;
  if (a->lda % 4 || a->ldw % 4 || a->stride_a % 4 || a->stride_w % 4 || a->K % QK) return false;
  if (a->conv_taps > 0 && a->conv_c % QK) return false;
  return true;
}

struct TileCfg { int bm, bn, occ; float eff; };
constexpr TileCfg kTiles[] = {  // eff: per-tile throughput relative to the 2-phase ping-pong 256x256
    {256, 256, 1, 1.00f},  // 1: 8 waves, 128x64 per wave (runs gemm_bf16_pp2_kernel)
    {256, 128, 1, 0.68f},  // 2: 8 waves, 64x64 per wave
    {128, 128, 2, 0.64f},  // 3: 4 waves, 64x64 per wave
    {128, 64, 3, 0.50f},   // 4: 4 waves, 64x32 per wave
    {64, 64, 4, 0.32f},    // 5: 4 waves, 32x32 per wave
};

// estimated cost of config c (0-based) for an MxN GEMM: rounds x per-CU work / efficiency
double tile_cost(int c, int M, int N, int batch) {
  const TileCfg& t = kTiles[c];
  const double tiles = (double)((M + t.bm - 1) / t.bm) * ((N + t.bn - 1) / t.bn) * batch;
  const double rounds = ceil(tiles / (256.0 * t.occ));
  return rounds * t.occ * (double)t.bm * t.bn / t.eff;
}

int g_gemm_ps_grid = 0;     // echo_gemm_set_diag key 6: persistent-kernel workgroup count cap (0 = CUs; A/B)
int g_gemm_fill_min = 128;  // echo_gemm_set_diag key 5: a 256x256 pick below this many tiles switches (A/B)

int pick_tile(int M, int N, int K, int batch) {
  (void)K;
  int best = 1;
  double best_t = 1e300;
  for (int c = 0; c < 5; ++c) {
    const double est = tile_cost(c, M, N, batch);
    if (est < best_t * 0.999) { best_t = est; best = c + 1; }
  }
  // Under-filled launches (fewer tiles than CUs) are latency-bound per workgroup, which the
  // throughput model does not see: take the largest multi-block config that still gives every CU
  // a tile, else the one with the most tiles (tools/bench_gemm.py, e.g. M=1920 N=2048 K=5888:
  // 256x128 86.7 us, 128x64 61.6 us; M=640 N=80: 39.7 -> 14.2 us on 64x64). At half fill or more the
  // big tile still wins (C5 decoder, N=2048 residual: M=7680 / 240 tiles 59.8 vs 74.5 us on 128x128,
  // M=5120 / 160 tiles 48.3 vs 55.9 us; M=2560 / 80 tiles 45.3 vs 33.3 us): its switch is below 128
  auto ntiles = [&](int c) { return (double)((M + kTiles[c].bm - 1) / kTiles[c].bm) * ((N + kTiles[c].bn - 1) / kTiles[c].bn) * batch; };
  if (ntiles(best - 1) < (best == 1 ? g_gemm_fill_min : 256)) {
    for (int c = 2; c < 5; ++c)
      if (ntiles(c) >= 256 || c == 4) return c + 1;
  }
  return best;
}

// Wave-quantisation split of a 256x256 launch: rows [0, M1) as whole rounds of 256x256 tiles,
// rows [M1, M) with the cheapest smaller config. Returns M1 (0 = no split) and the tail config.
int split_rows(int M, int N, int* tail_cfg) {
  const int tn = (N + 255) / 256;
  int per = 256;  // rows of 256-row tiles per full round: multiple of 256 / gcd(256, tn)
  for (int g = tn; g % 2 == 0 && per > 1; g /= 2) per /= 2;
  const int M1 = (M / (256 * per)) * (256 * per);
  if (M1 == 0 || M1 >= M) return 0;
  const double full = tile_cost(0, M, N, 1);
  double best = 1e300;
  // tail candidates: the multi-block-per-CU configs. 256x128 (config 2) leaves half the CUs idle on
  // these tails and measured slowest (M=2048 N=2048, K 2048 / 5888: 37.5 / 85.2 us vs 28.2 / 61.4 us
  // for 128x64, tools/bench_gemm.py), which the round-based cost model does not see
  for (int c = 2; c < 5; ++c) {
    const double e = tile_cost(c, M - M1, N, 1);
    if (e < best) { best = e; *tail_cfg = c + 1; }
  }
  return tile_cost(0, M1, N, 1) + best < 0.9 * full ? M1 : 0;
}

int g_gemm_ns3 = 1;  // echo_gemm_set_diag key 2: 3-stage small tiles on (1) / off (0)

// the 3-stage small-tile kernel addresses A and W with 32-bit byte offsets from a scalar base
bool ns3_ok(const EchoGemmArgs* a) {
  const int64_t lim = (int64_t)1 << 31;
  return (int64_t)a->M * a->lda * 2 < lim && (int64_t)a->N * a->ldw * 2 < lim;
}

template <int BM, int BN, int WM, int WN, int EK>
int launch_bf16_ek(const EchoGemmArgs* a, const Epi& ep, hipStream_t s) {
  const int tm = (a->M + BM - 1) / BM, tn = (a->N + BN - 1) / BN;
  dim3 grid(tm * tn, a->batch);
  // 3 stages for the two smallest configs (48 / 72 KB of LDS) with a specialised epilogue: B = 1
  // decoder GEMMs 6-15 % faster (M = 640 W2 48.0 -> 40.6 us), the C3 W2 row tail 60.8 -> 57.5 us;
  // the generic-epilogue output projection (fp32 out + bias, N = 80) is faster at the 2-stage
  // kernel's higher occupancy (29.3 vs 31.5 us)
  bool ns3 = false;
  if constexpr (BM * BN <= 128 * 64 && EK != EK_GENERIC) {
    if (ns3_ok(a) && g_gemm_ns3) {
      ns3 = true;
      hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, WM, WN, EK, 3>), grid, dim3(64 * WM * WN), 0, s,
                         (const bf16_t*)a->A, a->lda, a->stride_a, (const bf16_t*)a->W, a->ldw, a->stride_w,
                         a->C, a->ldc, a->stride_c, a->M, a->N, a->K, tm, tn, ep);
    }
  }
  if (!ns3) {
    hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, WM, WN, EK>), grid, dim3(64 * WM * WN), 0, s,
                       (const bf16_t*)a->A, a->lda, a->stride_a, (const bf16_t*)a->W, a->ldw, a->stride_w,
                       a->C, a->ldc, a->stride_c, a->M, a->N, a->K, tm, tn, ep);
  }
  ECHO_LAUNCH_CHECK();
  return 0;
}

template <int ABL, int EK>
int launch_pp_ek(const EchoGemmArgs* a, const Epi& ep, hipStream_t s) {
  const int tm = (a->M + 255) / 256, tn = (a->N + 255) / 256;
  hipLaunchKernelGGL((gemm_bf16_pp_kernel<ABL, EK>), dim3(tm * tn, a->batch), dim3(512), 0, s, (const bf16_t*)a->A,
                     a->lda, a->stride_a, (const bf16_t*)a->W, a->ldw, a->stride_w, a->C, a->ldc, a->stride_c,
                     a->M, a->N, a->K, tm, tn, ep);
  ECHO_LAUNCH_CHECK();
  return 0;
}

template <int EK>
int launch_pp2_ek(const EchoGemmArgs* a, const Epi& ep, hipStream_t s) {
  const int tm = (a->M + 255) / 256, tn = (a->N + 255) / 256;
  hipLaunchKernelGGL((gemm_bf16_pp2_kernel<EK>), dim3(tm * tn, a->batch), dim3(512), 0, s, (const bf16_t*)a->A,
                     a->lda, a->stride_a, (const bf16_t*)a->W, a->ldw, a->stride_w, a->C, a->ldc, a->stride_c,
                     a->M, a->N, a->K, tm, tn, ep);
  ECHO_LAUNCH_CHECK();
  return 0;
}

int g_num_cus = 0;  // persistent grid size (hipDeviceProp multiProcessorCount, queried once)

// group-M height of the persistent 256x256 and 320-row kernels (echo_gemm_set_diag key 13; 0 = 4). Each XCD's
// 32 concurrent tiles then cover 4 row panels x 8 column panels: 13.2 MB of A / W panels per XCD round for the
// 320-row tiles (14.5 MB at 8 x 4) — C3 +0.7 % over 8, 16 -1.7 %, 2 / 3 / 5 / 6 between (profiles/r5_gemm_group_m.txt)
int g_gemm_group_m = 0;

template <int EK>
int launch_ps_ek(const EchoGemmArgs* a, const Epi& ep, hipStream_t s) {
  const int tm = (a->M + 255) / 256, tn = (a->N + 255) / 256;
  if (g_num_cus == 0) {
    int dev = 0, n = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return (int)e;
    if (n <= 0) return ECHO_EINVAL;
    g_num_cus = n;
  }
  const int grid = min(tm * tn, g_gemm_ps_grid > 0 ? g_gemm_ps_grid : g_num_cus);
  // group-M height 8. Measured with tile 18 (tools/bench_gemm.py --stagger G): 1, 2, 4 and 16 are
  // 2-6 % slower on QKVG/W13; on the N = 2048 residual GEMMs 4 was within +-2 % of 8 in either
  // direction across two boxes (Wo 245 vs 252 / 235 vs 229 us, W2 591 vs 604 / 579 vs 587 us)
  Epi e = ep;
  if (e.gm <= 0) e.gm = g_gemm_group_m > 0 ? g_gemm_group_m : 4;
  hipLaunchKernelGGL((gemm_bf16_ps_kernel<EK>), dim3(grid, a->batch), dim3(512), 0, s, (const bf16_t*)a->A,
                     a->lda, a->stride_a, (const bf16_t*)a->W, a->ldw, a->stride_w, a->C, a->ldc, a->stride_c,
                     a->M, a->N, a->K, tm, tn, e);
  ECHO_LAUNCH_CHECK();
  return 0;
}

// epilogue kind of a call: the specialised kinds need no bias, no activation and no divisor
int ek_of(const EchoGemmArgs* a) {
  if (a->bias && a->act == ECHO_ACT_NONE && a->out_div == 0.0f && a->epilogue == ECHO_EPI_STORE &&
      a->dtype == ECHO_BF16)
    return EK_BIAS;  // persistent kernel only; the other launchers take it as EK_GENERIC
  if (a->bias || a->act != ECHO_ACT_NONE || a->out_div != 0.0f) return EK_GENERIC;
  switch (a->epilogue) {
    case ECHO_EPI_STORE: return EK_STORE;
    case ECHO_EPI_SWIGLU: return EK_SWIGLU;
    case ECHO_EPI_RESID: return EK_RESID;
    case ECHO_EPI_HEADNORM: return EK_HEADNORM;
    default: return EK_GENERIC;
  }
}

template <int BM, int BN, int WM, int WN>
int launch_bf16(const EchoGemmArgs* a, const Epi& ep, hipStream_t s) {
  switch (ek_of(a)) {
    case EK_STORE: return launch_bf16_ek<BM, BN, WM, WN, EK_STORE>(a, ep, s);
    case EK_SWIGLU: return launch_bf16_ek<BM, BN, WM, WN, EK_SWIGLU>(a, ep, s);
    case EK_RESID: return launch_bf16_ek<BM, BN, WM, WN, EK_RESID>(a, ep, s);
    default: return launch_bf16_ek<BM, BN, WM, WN, EK_GENERIC>(a, ep, s);
  }
}

// persistent kernel: register epilogues only, K >= 128, and 32-bit buffer offsets for C / aux
bool ps_ok(const EchoGemmArgs* a, int ek) {
  if (ek != EK_STORE && ek != EK_SWIGLU && ek != EK_RESID && ek != EK_BIAS && ek != EK_HEADNORM) return false;
  if (ek == EK_HEADNORM && (a->batch != 1 || a->hn_heads <= 0)) return false;
  if (a->K < 128 || a->N % 256) return false;
  const int64_t lim = (int64_t)1 << 30;  // elements: 32-bit byte offsets (rows up to M + 255)
  if ((int64_t)(a->M + 255) * a->ldc >= lim || (int64_t)a->M * a->lda >= lim || (int64_t)a->N * a->ldw >= lim)
    return false;
  if (ek == EK_RESID && (int64_t)(a->M + 255) * a->ld_aux >= lim) return false;
  return true;
}

int launch_ps(const EchoGemmArgs* a, const Epi& ep, hipStream_t s) {
  switch (ek_of(a)) {
    case EK_STORE: return launch_ps_ek<EK_STORE>(a, ep, s);
    case EK_SWIGLU: return launch_ps_ek<EK_SWIGLU>(a, ep, s);
    case EK_RESID: return launch_ps_ek<EK_RESID>(a, ep, s);
    case EK_BIAS: return launch_ps_ek<EK_BIAS>(a, ep, s);
    case EK_HEADNORM: return launch_ps_ek<EK_HEADNORM>(a, ep, s);
    default: return ECHO_EINVAL;
  }
}

int launch_pp2(const EchoGemmArgs* a, const Epi& ep, hipStream_t s) {
  switch (ek_of(a)) {
    case EK_HEADNORM: return launch_pp2_ek<EK_HEADNORM>(a, ep, s);
    case EK_STORE: return launch_pp2_ek<EK_STORE>(a, ep, s);
    case EK_SWIGLU: return launch_pp2_ek<EK_SWIGLU>(a, ep, s);
    case EK_RESID: return launch_pp2_ek<EK_RESID>(a, ep, s);
    default: return launch_pp2_ek<EK_GENERIC>(a, ep, s);
  }
}

template <int ABL>
int launch_pp(const EchoGemmArgs* a, const Epi& ep, hipStream_t s) {
  if (ABL != 0) return launch_pp_ek<ABL, EK_GENERIC>(a, ep, s);
  switch (ek_of(a)) {
    case EK_STORE: return launch_pp_ek<0, EK_STORE>(a, ep, s);
    case EK_SWIGLU: return launch_pp_ek<0, EK_SWIGLU>(a, ep, s);
    case EK_RESID: return launch_pp_ek<0, EK_RESID>(a, ep, s);
    default: return launch_pp_ek<0, EK_GENERIC>(a, ep, s);
  }
}

int cu_count_cached() {
  if (g_num_cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      return 256;
    g_num_cus = n;
  }
  return g_num_cus;
}

// 320x256 tiles (gemm_bf16_t320_kernel): gated residual, SwiGLU or head norm, M % 320 == 0, 32-bit buffer offsets,
// 16-B aligned operands
bool t320_ok(const EchoGemmArgs* a) {
  const int ek = ek_of(a);
  if (a->dtype != ECHO_BF16 || (ek != EK_RESID && ek != EK_SWIGLU && ek != EK_HEADNORM) || a->batch != 1 ||
      a->conv_taps > 0)
    return false;
  if (ek == EK_HEADNORM && a->hn_heads <= 0) return false;
  if (a->M % 320 || a->N % 256 || a->K % 64 || a->K < 128) return false;
  const int64_t lim = (int64_t)1 << 30;
  if ((int64_t)a->M * a->ldc >= lim || (int64_t)a->M * a->lda >= lim || (int64_t)a->N * a->ldw >= lim) return false;
  if (((uintptr_t)a->A | (uintptr_t)a->W | (uintptr_t)a->C) & 15) return false;
  if (a->lda % 8 || a->ldw % 8 || a->ldc % 8) return false;
  if (ek == EK_RESID &&
      ((int64_t)a->M * a->ld_aux >= lim || a->ld_aux % 8 || (((uintptr_t)a->aux | (uintptr_t)a->gate) & 15)))
    return false;
  return true;
}

// PER = 1: one persistent workgroup per CU (grid = min(tiles, CUs rounded down to a multiple of 8))
template <int SP, int PER>
int launch_t320_sp(const EchoGemmArgs* a, const Epi& ep, hipStream_t s) {
  const int tm = a->M / 320, tn = a->N / 256;
  int grid = tm * tn;
  if (PER) {
    const int cus = cu_count_cached() & ~7;
    if (cus >= 8 && grid > cus) grid = cus;
  }
  Epi e2 = ep;
  if (e2.gm <= 0) e2.gm = g_gemm_group_m > 0 ? g_gemm_group_m : 4;
  const T320Args ta{(const bf16_t*)a->A, a->lda, (const bf16_t*)a->W, a->ldw, a->C, a->ldc, a->M, a->N, a->K, tm, tn, e2};
  if (ek_of(a) == EK_SWIGLU)
    hipLaunchKernelGGL((gemm_bf16_t320_kernel<EK_SWIGLU, SP, PER>), dim3(grid), dim3(512), 0, s, ta);
  else if (ek_of(a) == EK_HEADNORM)
    hipLaunchKernelGGL((gemm_bf16_t320_kernel<EK_HEADNORM, SP, PER>), dim3(grid), dim3(512), 0, s, ta);
  else
    hipLaunchKernelGGL((gemm_bf16_t320_kernel<EK_RESID, SP, PER>), dim3(grid), dim3(512), 0, s, ta);
  ECHO_LAUNCH_CHECK();
  return 0;
}
// production 320-row launch: the persistent form for SwiGLU launches of at least 4 tiles per CU (W13: 15 / 5
// tiles per CU at M = 30720 / 10240, -2.5 / -3 %, C3 +0.8 %; profiles/r3_t320_persistent.txt, r3s2_ab_t320p.txt)
// (tile 22 forces one tile per workgroup, 23 the persistent form). One tile per workgroup for the blockwise W13 launch
// (M = 7680: 2 tiles per CU, C5 -0.4 % when persistent) and the gated residual (3 / 1 tiles per CU, K = 5888 for
// W2: no measurable gain). The head-norm epilogue's persistent form (spill-free since round 4: norm weights
// and RoPE rows read at the use) from 8 tiles per CU: QKVG M = 30720 (12 per CU) 764.6 -> 753.0 us, M = 10240
// (4 per CU) 258.5 vs 258.7 (profiles/r4_t320_headnorm_persistent.txt). The gated residual from 2 tiles per CU
// (Wo / W2 at M = 30720: 3 per CU) with the 4 / 5 DMA split (SP = 1): 212.1 -> 209.9 / 512.9 -> 502.9 us, launches
// replayed from a graph, twice; at one round no difference (profiles/r5_sk_large_sweep.txt).
int launch_t320(const EchoGemmArgs* a, const Epi& ep, hipStream_t s) {
  const int64_t tiles = (int64_t)(a->M / 320) * (a->N / 256), cus = cu_count_cached();
  const int ek = ek_of(a);
  const bool per = ((ek == EK_SWIGLU && tiles >= 4 * cus) || (ek == EK_HEADNORM && tiles >= 8 * cus));
  if (!per && ek == EK_RESID && tiles >= 2 * cus) return launch_t320_sp<1, 0>(a, ep, s);
  return per ? launch_t320_sp<0, 1>(a, ep, s) : launch_t320_sp<0, 0>(a, ep, s);
}

// auto pick between 320x256 and 256x256 tiles by whole rounds of the CUs: a 320-row tile does 1.25x the work
// of a 256-row one in ≈1.2x the time (more MFMA per staged byte; HEADNORM: one wave per head, no LDS
// exchange), so 320-row tiles win when ⌈tiles320 / CUs⌉ x 1.2 < ⌈tiles256 / CUs⌉ (tools/bench_gemm.py,
// bench_qkvg.py): the N = 2048 residual at M = 30720 / 10240 (3.6 vs 4, 1.2 vs 2), W13 at M = 30720 / 10240
// (21.6 vs 22, 7.2 vs 8), QKVG + head norm at M = 30720 / 10240 / 7680 / 2560 (14.4 vs 15, 4.8 vs 5,
// 3.6 vs 4, 1.2 vs 2); not W13 at M = 7680 / 2560 (6 vs 6, 2.4 vs 2)
bool t320_pays(const EchoGemmArgs* a, int cus) {
  const int64_t n320 = (int64_t)(a->M / 320) * (a->N / 256);
  const int64_t n256 = (int64_t)((a->M + 255) / 256) * (a->N / 256);
  if (n320 < cus) return false;
  const double r320 = (double)((n320 + cus - 1) / cus) * 1.2, r256 = (double)((n256 + cus - 1) / cus);
  return r320 < 0.99 * r256;
}

// Column split of a 320-row launch whose tile count leaves a partial round (W13, N = 11776 = 46 tile
// columns): the first c1 tile columns as whole rounds of 320x256 tiles, the other N - 256 c1 columns as a
// second launch on the persistent 256x256 kernel (same K order per element: bitwise equal). Cost in
// 256x256 tile-rounds (a 320-row round = 1.2); returns c1, or 0 when no split beats the best single launch
// by 2 % (M = 30720: c1 = 40, 15 x 1.2 + 3 = 21 vs 21.6; M = 10240: 5 x 1.2 + 1 = 7 vs 7.2).
int t320_col_split(const EchoGemmArgs* a, int cus) {
  const int64_t pm = a->M / 320, p256 = (a->M + 255) / 256, tn = a->N / 256;
  auto rounds = [&](int64_t tiles) { return (double)((tiles + cus - 1) / cus); };
  const double one = std::min(pm * tn >= cus ? rounds(pm * tn) * 1.2 : 1e300, rounds(p256 * tn));
  double best = 0.98 * one;
  int c1 = 0;
  for (int64_t c = 1; c < tn; ++c) {
    if (pm * c < cus) continue;
    const double e = rounds(pm * c) * 1.2 + rounds(p256 * (tn - c)) + 0.05;
    if (e < best) { best = e; c1 = (int)c; }
  }
  return c1;
}

int g_gemm_t320 = 0;  // echo_gemm_set_diag key 7: 320-row tiles in the auto pick: 0 = when they need fewer
                      // tile-rounds x 1.2 (t320_pays), 1 = never, 2 = whenever at least one round (A/B)
int g_gemm_gm = 0;  // echo_gemm_set_diag key 1: group-M height of tile 18 (A/B)
int g_gemm_no_rowsplit = 0;  // key 3: no row-tail split of 256x256 launches (A/B)
int g_gemm_no_ps = 0;        // key 4: the 2-phase kernel instead of the persistent one (A/B)
int g_gemm_no_colsplit = 0;  // key 8: no column split of 320-row launches (t320_col_split; A/B)
int g_gemm_no_splitk = 0;    // key 11: never split K (tests that compare B = 1 bitwise with B = 16 rows)
int g_gemm_no_sk = 0;        // key 12: no small-M kernel in the auto pick (A/B)

// ---- small-M kernel family (gemm_bf16_sk_kernel): configs of `tile` 1CS
struct SkCfg { int bm, bn, wm, wn, ns; };
constexpr SkCfg kSk[] = {
    {0, 0, 0, 0, 0},
    {128, 128, 2, 2, 4},  // 1: 128 KB ring, one workgroup per CU
    {128, 64, 2, 2, 4},   // 2: 96 KB
    {64, 64, 2, 2, 4},    // 3: 64 KB, two per CU
    {160, 64, 2, 2, 4},   // 4: 112 KB (the blockwise block's 160 rows in one tile)
    {64, 128, 2, 2, 4},   // 5: 96 KB
    {128, 128, 2, 4, 4},  // 6-9: the same tiles with 8 waves (two per SIMD: one wave's fragment reads
    {128, 64, 2, 4, 4},   //      under the other's MFMAs)
    {64, 64, 2, 4, 4},
    {64, 128, 2, 4, 4},
    {160, 128, 2, 2, 4},  // 10: 144 KB; 11: 156 KB; 12: 144 KB — whole 160-row blocks / wide tiles for the
    {160, 256, 2, 2, 3},  //     weight-streaming launches (QKVG / W13 at 160-640 rows: few, big, K-split
    {128, 256, 2, 2, 3},  //     tiles cut the per-CU re-read of A)
    {128, 256, 2, 4, 3},  // 13: 144 KB, 8 waves
    {160, 128, 2, 2, 2},  // 14: 72 KB, two per CU
    {160, 128, 2, 4, 4},  // 15: 144 KB, 8 waves (160-row blocks: one round at M = 2560, three at 7680, N = 2048)
    {160, 128, 2, 4, 3},  // 16: 108 KB
};
constexpr int kNumSk = 16;
// `tile` 100 + 10 c + S (c = 1 .. kNumSk, S = 1 .. 9): small-M config c with K split S
constexpr bool sk_tile(int t) { return t >= 110 && t < 100 + 10 * (kNumSk + 1) && t % 10 != 0; }
int sk_occ(int c) { return (160 * 1024) / ((kSk[c].bm + kSk[c].bn) * BK * 2 * kSk[c].ns); }

// the fused epilogue straight from the unit's registers is expressible for this wave tile (gemm_epilogue's
// row-chunk loop must divide the wave's rows); otherwise the launch goes through the finish kernel
constexpr bool sk_direct(int tm, int tn, int ek, int wn) {
  // SwiGLU pairs the w1 / w3 16-column blocks inside a wave: its tile needs whole pairs (tn % 32 == 0);
  // head norm: a 128-column head in one wave's tile or in the 64- / 32-column tiles of 2 / 4 waves of one row of the
  // workgroup's waves (wn % (128 / tn) == 0: the head never spans workgroups)
  return ek == EK_SWIGLU     ? (tn % 32 == 0 && tm % (64 / (tn / 16)) == 0)
         : ek == EK_HEADNORM ? ((tn == 32 || tn == 64 || tn == 128) && tm % (128 / tn * 4) == 0 && wn % (128 / tn) == 0)
                             : (ek == EK_STORE || ek == EK_RESID) && tm % (64 / (tn / 8)) == 0;
}

// small-M path applies: bf16, one batch, no conv, a fused kind the finish kernel has, 32-bit DMA offsets
bool sk_ok(const EchoGemmArgs* a) {
  const int ek = ek_of(a);
  if (a->dtype != ECHO_BF16 || a->batch != 1 || a->conv_taps > 0) return false;
  if (ek != EK_STORE && ek != EK_SWIGLU && ek != EK_RESID && ek != EK_HEADNORM) return false;
  if (ek == EK_HEADNORM && (a->N % 128 || a->hn_heads <= 0)) return false;
  if (ek == EK_SWIGLU && a->N % 32) return false;
  if (!ns3_ok(a) || a->K < 128) return false;
  if (((uintptr_t)a->A | (uintptr_t)a->W | (uintptr_t)a->C) & 15) return false;
  if (ek == EK_RESID && ((((uintptr_t)a->aux | (uintptr_t)a->gate) & 15) || a->ld_aux % 8)) return false;
  return true;
}

bool sk_partial(int c, int S, int ek) {
  const int tm = kSk[c].bm / kSk[c].wm, tn = kSk[c].bn / kSk[c].wn;
  return S > 1 || !sk_direct(tm, tn, ek, kSk[c].wn);
}

int64_t sk_ws_bytes(const EchoGemmArgs* a, int c, int S) {
  return sk_partial(c, S, ek_of(a)) ? (int64_t)S * a->M * a->N * 4 : 0;
}

// the small-M plan: config and K split from the POLICY rows (echo_set_policy_rows: the rows the launch
// would have in a one-process run of the whole batch), so that the split — the only choice that changes
// the summation order — is the one-process choice on every rank
int64_t policy_rows(int64_t rows) { return rows * g_policy_num / g_policy_den; }

bool sk_plan(const EchoGemmArgs* a, bool allow_split, int* cfg, int* split) {
  if (g_gemm_no_sk || !sk_ok(a)) return false;
  const int64_t Mp = policy_rows(a->M);
  // Measured with the weights streamed from HBM as in the sampler (profiles/r4_sk_hbm_sweep.txt: every
  // config x split against the round-3 pick and hipBLASLt, 16 rotating weight copies; cache-resident
  // weights, profiles/r4_sk_sweep.txt, hide the difference): the 4-deep LDS-DMA ring keeps enough weight
  // bytes in flight per CU where the round-3 tiles (2-stage, one K-tile ahead) wait on HBM latency.
  //   gated residual, N = 2048 (Wo K = 2048, W2 K = 5888), us:    M = 160      480      640     1920
  //     round-3 pick                                       K 2048  12.0     12.9     15.9     24.6
  //                                                        K 5888  20.4     31.3     31.1     69.7
  //     here                                               K 2048  11.8 8/2 12.5 8/1 15.8 3/1  (r3)
  //                                                        K 5888  17.8 5/4 25.4 6/4 30.2 6/3  58.5 6/1
  //   QKVG + q/k norm + RoPE (N = 8192; round 3: store + head_norm_rope) 22.6 -> 18.9 (5/1),
  //     37.1 -> 27.0 (1/1), 39.5 -> 33.5 (10/1); W13 SwiGLU 24.4 -> 22.8 (6/1) at 160 rows, 39.1 -> 35.4 and
  //     38.1 -> 36.9 (13/1: 128x256 tiles of 8 waves) at 480 / 640; the 1920-row W13 / QKVG keep the round-3
  //     pick (as fast or faster there).
  const int ek = ek_of(a);
  const bool longk = a->K >= 4096;
  int c, S = 1;
  if (ek == EK_RESID && a->N >= 1024 && a->N <= 2048) {
    // (M <= 256, K 5888: config 3 at S = 4 measured 16.6 -> 15.9 us in isolation, replayed from a graph with the
    // activations L2-resident, but 19.0 -> 21.0 us with its finish inside the sampler, where the activations were
    // just written: 64x64 tiles read them from the fabric twice as often; profiles/r5_sk_depth_sweep.txt)
    // (round 6, with the 8-wave configs' in-compute DMA: Wo at 640 rows config 3 -> 9, 16.2 -> 14.2 us; at 1920 rows
    // the 128x64 two-stage tile -> config 6, 23.3 -> 20.9 us; profiles/r6_wo_8wave.txt)
    if (Mp <= 256) { c = longk ? 9 : 8; S = longk ? 4 : 2; }  // W2 at 160 rows: 5 -> 9 (8 waves), 16.8 -> 15.0 us
    else if (Mp <= 512) { c = longk ? 6 : 8; S = longk ? 4 : 1; }
    else if (Mp <= 768) { c = longk ? 6 : 9; S = longk ? 3 : 1; }
    else if (Mp <= 2048) c = 6;
    // the blockwise B = 16 plain step (M = 2560: 256 tiles of 160x128 = one round): 37.9 -> 31.3 us (Wo),
    // 85.6 -> 73.3 (W2) (profiles/r4_sk5_sweep.txt; hipBLASLt's plain store 26.7 / 58.5)
    else if (Mp > 2048 && Mp <= 3072) c = 15;
    else return false;
  } else if (ek == EK_HEADNORM && a->N >= 4096 && Mp <= 768) {
    // round 6: the 8-wave configs now fuse the head norm over four waves' 32-column tiles (gemm_epilogue):
    // 160 / 480 / 640 rows 18.4 -> 17.1 (9), 27.7 -> 23.7 (6), 32.9 -> 28.4 us (16), bitwise equal
    // (profiles/r6_qkvg_8wave.txt; the 4-wave configs 5 / 1 / 10 before)
    c = Mp <= 256 ? 9 : Mp <= 512 ? 6 : 16;
  } else if (ek == EK_SWIGLU && a->N >= 8192 && Mp <= 768) {
    c = Mp <= 256 ? 6 : 13;  // 480 / 640 rows: 39.1 -> 35.4 / 38.1 -> 36.9 us (profiles/r4_sk4_sweep.txt)
  } else {
    return false;
  }
  if (!allow_split || g_gemm_no_splitk) S = 1;
  S = std::max(1, std::min(S, a->K / BK / 2));
  *cfg = c;
  *split = S;
  return true;
}

}  // namespace

template <int BM, int BN, int WM, int WN, int NS, int EK>
int launch_sk_direct(const EchoGemmArgs* a, const Epi& ep, hipStream_t s) {
  constexpr int TM = BM / WM, TN = BN / WN;
  if constexpr (sk_direct(TM, TN, EK, WN)) {
    const int tm = (a->M + BM - 1) / BM, tn = (a->N + BN - 1) / BN;
    hipLaunchKernelGGL((gemm_bf16_sk_kernel<BM, BN, WM, WN, EK, NS>), dim3(tm * tn, 1), dim3(64 * WM * WN), 0, s,
                       (const bf16_t*)a->A, a->lda, (const bf16_t*)a->W, a->ldw, a->C, a->ldc, a->M, a->N, a->K, tm,
                       tn, ep);
    ECHO_LAUNCH_CHECK();
    return 0;
  } else {
    return ECHO_EINVAL;
  }
}

// the split-K finish of a gated residual runs inside the launch (EK_PARTIAL_FUSED) when a counter buffer is set
// (echo_set_sync_buffer), every workgroup fits on the chip at once and the counters and byte offsets fit
int g_sk_abl = 0;  // key 16 (diagnostics build): small-M kernel timing ablations (Epi::abl)
int g_no_fused_finish = 0;  // echo_gemm_set_diag key 14: 1 = never finish split-K inside the launch (A/B)
int g_no_inlaunch_merge = 0;  // key 15: 1 = split-KV attention never merges inside its launch (A/B; attention.hip)

bool sk_fused_ok(const EchoGemmArgs* a, int tm, int tn, int S) {
  return g_sync && !g_no_fused_finish && ek_of(a) == EK_RESID && (S > 1 || a->mod_out) && (int64_t)tm * tn * S <= cu_count_cached() &&
         SYNC_CNT0 + 2 * ((int64_t)tm * tn + tm) <= g_sync_words &&
         (int64_t)S * a->M * a->N * 4 < ((int64_t)1 << 32) - 16 &&
         (int64_t)a->M * a->ldc * 2 < ((int64_t)1 << 32) - 16 && (uintptr_t)a->C % 16 == 0;
}

template <int BM, int BN, int WM, int WN, int NS, bool FUSE_OK = false>
int launch_sk(const EchoGemmArgs* a, const Epi& ep, int S, void* ws, hipStream_t s) {
  const int ek = ek_of(a);
  const int tm = (a->M + BM - 1) / BM, tn = (a->N + BN - 1) / BN;
  const bool mod = ep.mod_out != nullptr;  // caller checked: RESID, N == 2048, partial plan
#ifdef ECHO_DIAG  // measured slower than GEMM + finish kernel: diagnostics build only
  if constexpr (FUSE_OK) {
    if (sk_fused_ok(a, tm, tn, S)) {  // one launch: the K-slices finish the tiles (and the AdaLN) themselves
      Epi ef = ep;
      ef.fin_out = a->C;
      ef.fin_ldc = a->ldc;
      ef.sync = g_sync;
      hipLaunchKernelGGL((gemm_bf16_sk_kernel<BM, BN, WM, WN, EK_PARTIAL_FUSED, NS>), dim3(tm * tn, S),
                         dim3(64 * WM * WN), 0, s, (const bf16_t*)a->A, a->lda, (const bf16_t*)a->W, a->ldw, ws,
                         (int64_t)a->N, a->M, a->N, a->K, tm, tn, ef);
      ECHO_LAUNCH_CHECK();
      return 0;
    }
  }
#endif
  if (!mod && !(S > 1 || !sk_direct(BM / WM, BN / WN, ek, WN))) {
    switch (ek) {
      case EK_STORE: return launch_sk_direct<BM, BN, WM, WN, NS, EK_STORE>(a, ep, s);
      case EK_SWIGLU: return launch_sk_direct<BM, BN, WM, WN, NS, EK_SWIGLU>(a, ep, s);
      case EK_RESID: return launch_sk_direct<BM, BN, WM, WN, NS, EK_RESID>(a, ep, s);
      case EK_HEADNORM: return launch_sk_direct<BM, BN, WM, WN, NS, EK_HEADNORM>(a, ep, s);
      default: return ECHO_EINVAL;
    }
  }
  hipLaunchKernelGGL((gemm_bf16_sk_kernel<BM, BN, WM, WN, EK_PARTIAL, NS>), dim3(tm * tn, S), dim3(64 * WM * WN), 0, s,
                     (const bf16_t*)a->A, a->lda, (const bf16_t*)a->W, a->ldw, ws, (int64_t)a->N, a->M, a->N, a->K,
                     tm, tn, ep);
  ECHO_LAUNCH_CHECK();
  const int nout = ek == EK_SWIGLU ? a->N / 2 : a->N;
  const int64_t threads = (int64_t)a->M * (nout / 8);
  const dim3 g((unsigned)((threads + 255) / 256));
  const float* w = (const float*)ws;
  switch (ek) {
    case EK_STORE: hipLaunchKernelGGL(gemm_splitk_finish_kernel<EK_STORE>, g, dim3(256), 0, s, w, S, a->M, a->N, a->C, a->ldc, ep); break;
    case EK_SWIGLU: hipLaunchKernelGGL(gemm_splitk_finish_kernel<EK_SWIGLU>, g, dim3(256), 0, s, w, S, a->M, a->N, a->C, a->ldc, ep); break;
    case EK_RESID:
      if (mod) hipLaunchKernelGGL((gemm_splitk_finish_kernel<EK_RESID, true>), g, dim3(256), 0, s, w, S, a->M, a->N, a->C, a->ldc, ep);
      else hipLaunchKernelGGL(gemm_splitk_finish_kernel<EK_RESID>, g, dim3(256), 0, s, w, S, a->M, a->N, a->C, a->ldc, ep);
      break;
    case EK_HEADNORM: hipLaunchKernelGGL(gemm_splitk_finish_kernel<EK_HEADNORM>, g, dim3(256), 0, s, w, S, a->M, a->N, a->C, a->ldc, ep); break;
    default: return ECHO_EINVAL;
  }
  ECHO_LAUNCH_CHECK();
  return 0;
}

int launch_sk_cfg(const EchoGemmArgs* a, const Epi& ep, int c, int S, void* ws, hipStream_t s) {
  switch (c) {
    case 1: return launch_sk<128, 128, 2, 2, 4>(a, ep, S, ws, s);
    case 2: return launch_sk<128, 64, 2, 2, 4>(a, ep, S, ws, s);
    case 3: return launch_sk<64, 64, 2, 2, 4, true>(a, ep, S, ws, s);
    case 4: return launch_sk<160, 64, 2, 2, 4>(a, ep, S, ws, s);
    case 5: return launch_sk<64, 128, 2, 2, 4, true>(a, ep, S, ws, s);
    case 6: return launch_sk<128, 128, 2, 4, 4, true>(a, ep, S, ws, s);
    case 7: return launch_sk<128, 64, 2, 4, 4>(a, ep, S, ws, s);
    case 8: return launch_sk<64, 64, 2, 4, 4, true>(a, ep, S, ws, s);
    case 9: return launch_sk<64, 128, 2, 4, 4>(a, ep, S, ws, s);
    case 10: return launch_sk<160, 128, 2, 2, 4>(a, ep, S, ws, s);
    case 11: return launch_sk<160, 256, 2, 2, 3>(a, ep, S, ws, s);
    case 12: return launch_sk<128, 256, 2, 2, 3>(a, ep, S, ws, s);
    case 13: return launch_sk<128, 256, 2, 4, 3>(a, ep, S, ws, s);
    case 14: return launch_sk<160, 128, 2, 2, 2>(a, ep, S, ws, s);
    case 15: return launch_sk<160, 128, 2, 4, 4>(a, ep, S, ws, s);
    case 16: return launch_sk<160, 128, 2, 4, 3>(a, ep, S, ws, s);
    default: return ECHO_EINVAL;
  }
}

// The auto plan of a `tile` == 0 launch (host only). echo_gemm_ws launches what it returns and
// echo_gemm_planned_tile reports it, so the labels bench.py / perf_model.py put on timed launches are the launches
// production makes. Decisions in order: the small-M family (sk_plan), the large-tile pick (256x256 -> the persistent
// kernel, or the 2-phase one for a one-round head norm), an unfused head norm (store + echo_head_norm_rope), fp32,
// the 320-row column split, 320-row tiles, the W13 column split at 1537-2048 rows, the row-tail split.
enum { RT_SK = 1, RT_TILE, RT_HN_SPLIT, RT_F32, RT_T320_COLSPLIT, RT_T320, RT_W13_COLSPLIT, RT_ROWSPLIT };
struct Route {
  int kind = RT_TILE;
  int t = 0;               // large-tile config (RT_TILE) / the 256x256 kernel of a split
  int c = 0, S = 1;        // RT_SK: small-M config and K split
  bool sk_ws = false;      // RT_SK: uses the workspace
  int c1 = 0;              // RT_*_COLSPLIT: tile columns of the first launch
  int M1 = 0, tail = 0;    // RT_ROWSPLIT: rows of the 256x256 rounds, the tail's config
};

Route plan_route(const EchoGemmArgs* a, const void* ws, int64_t ws_bytes) {
  Route r;
  int c = 0, S = 1;
  if (sk_plan(a, ws != nullptr, &c, &S)) {
    const int64_t need = sk_ws_bytes(a, c, S);
    if (need == 0 || (ws && (uintptr_t)ws % 16 == 0 && ws_bytes >= need)) {
      r.kind = RT_SK; r.c = c; r.S = S; r.sk_ws = need > 0;
      return r;
    }
    if (sk_plan(a, false, &c, &S) && sk_ws_bytes(a, c, S) == 0) {  // the best plan without a workspace
      r.kind = RT_SK; r.c = c; r.S = S;
      return r;
    }
  }
  const bool headnorm = a->epilogue == ECHO_EPI_HEADNORM;
  int t = pick_tile(a->M, a->N, a->K, a->batch);
  // Head norm in at most one tile round (the C2 CFG step's QKVG, M = 1920: 256 tiles): the 2-phase kernel with its
  // LDS-staged epilogue, 63.3 -> 60.7 us against the persistent kernel's register epilogue, which gains nothing
  // from persistence in one round (launches replayed from a graph, profiles/r5_sk_1920_sweep.txt; bitwise equal)
  if (t == 1) {
    const int64_t tiles = (int64_t)((a->M + 255) / 256) * ((a->N + 255) / 256) * a->batch;
    const bool one_round_hn = headnorm && tiles <= cu_count_cached();
    t = (a->dtype == ECHO_BF16 && ps_ok(a, ek_of(a)) && !g_gemm_no_ps && !one_round_hn) ? 16 : 13;
  }
  r.t = t;
  // fused on the persistent kernel (t 16, via ps_ok) or the 2-phase one (t 13)
  const bool hn_fused = a->dtype == ECHO_BF16 && ((t == 13 && a->N % 128 == 0) || (t == 16 && ps_ok(a, EK_HEADNORM)));
  if (headnorm && !hn_fused) { r.kind = RT_HN_SPLIT; return r; }
  if (a->dtype == ECHO_F32) { r.kind = RT_F32; return r; }
  const int cus = cu_count_cached();
  if (g_gemm_t320 == 0 && !g_gemm_no_colsplit && a->batch == 1 && !headnorm && t320_ok(a)) {
    const int c1 = t320_col_split(a, cus);
    if (c1 > 0) { r.kind = RT_T320_COLSPLIT; r.c1 = c1; return r; }
  }
  if (g_gemm_t320 != 1 && t320_ok(a)) {
    const int n320 = (a->M / 320) * (a->N / 256);
    if (g_gemm_t320 == 2 ? n320 >= cus : t320_pays(a, cus)) { r.kind = RT_T320; return r; }
  }
  // SwiGLU at 1537..2048 rows (W13 of the B = 1 CFG step, M = 1920: 8 x 46 = 368 tiles, two rounds of the
  // persistent 256x256 kernel): the first ⌊0.94 CUs / row tiles⌋ tile columns there (one round) and the rest on
  // the small-M 128x256 8-wave config (one round of half tiles) — 98.8 -> 88.2 us (profiles/r5_colsplit.txt).
  // Same K order per element: bitwise equal.
  if (!g_gemm_no_colsplit && !g_gemm_no_sk && a->batch == 1 && t == 16 && ek_of(a) == EK_SWIGLU && a->N % 256 == 0) {
    const int tm = (a->M + 255) / 256, tn = a->N / 256;
    const int c1 = (int)(0.94 * cus) / tm;
    if ((tm == 7 || tm == 8) && tm * tn > cus && tm * tn < 2 * cus && c1 > 0 && c1 < tn) {
      EchoGemmArgs rest = *a;
      rest.N = a->N - c1 * 256;
      rest.W = (const bf16_t*)a->W + (int64_t)c1 * 256 * a->ldw;
      rest.C = (bf16_t*)a->C + c1 * 128;
      rest.tile = 100 + 10 * 13 + 1;
      if (sk_ok(&rest)) { r.kind = RT_W13_COLSPLIT; r.c1 = c1; return r; }
    }
  }
  if ((t == 13 || t == 16) && a->batch == 1 && !headnorm && !g_gemm_no_rowsplit) {
    int tail = 0;
    const int M1 = split_rows(a->M, a->N, &tail);
    if (M1 > 0) { r.kind = RT_ROWSPLIT; r.M1 = M1; r.tail = tail; return r; }
  }
  return r;
}

extern int g_adaln_blocks;  // elementwise.hip

extern "C" int echo_gemm_set_diag(int32_t key, int32_t value) {
  if (value < 0) return ECHO_EINVAL;
  if (key == 1) g_gemm_gm = value;
  else if (key == 2) g_gemm_ns3 = value != 0;
  else if (key == 3) g_gemm_no_rowsplit = value != 0;
  else if (key == 4) g_gemm_no_ps = value != 0;
  else if (key == 5) g_gemm_fill_min = value;
  else if (key == 6) g_gemm_ps_grid = value;
  else if (key == 7) { if (value > 2) return ECHO_EINVAL; g_gemm_t320 = value; }
  else if (key == 8) g_gemm_no_colsplit = value != 0;
  else if (key == 9) g_adaln_blocks = value;
  else if (key == 11) g_gemm_no_splitk = value != 0;
  else if (key == 12) g_gemm_no_sk = value != 0;
  else if (key == 13) { if (value < 0 || value > 64) return ECHO_EINVAL; g_gemm_group_m = value; }
  else if (key == 14) g_no_fused_finish = value != 0;
  else if (key == 15) g_no_inlaunch_merge = value != 0;
#ifdef ECHO_DIAG
  else if (key == 16) g_sk_abl = value;
#endif
  else return ECHO_EINVAL;
  return 0;
}

extern "C" int echo_gemm_pick_tile(int32_t M, int32_t N, int32_t K, int32_t batch) {
  const int t = pick_tile(M, N, K, batch);
  return t == 1 ? 13 : t;
}

extern "C" int echo_set_policy_rows(int32_t num, int32_t den) {
  if (num <= 0 || den <= 0 || num < den) return ECHO_EINVAL;
  g_policy_num = num;
  g_policy_den = den;
  return 0;
}

// configs whose launch_sk instantiates the in-launch finish (EK_PARTIAL_FUSED): the residual plans' tiles
bool sk_fuse_cfg(int c) { return c == 3 || c == 5 || c == 6 || c == 8; }

// workspace of a small-M launch: the split slabs, or — a gated residual + next AdaLN whose plan does not split K
// but whose grid fits the chip while a counter buffer is set — the one slab of the in-launch finish (the GEMM +
// modulate pass become one launch)
int64_t sk_ws_bytes_mod(const EchoGemmArgs* a, int c, int S) {
  const int64_t need = sk_ws_bytes(a, c, S);
  if (need > 0 || !a->mod_out || S != 1 || !sk_fuse_cfg(c) || a->N != 2048) return need;
  const int tm = (a->M + kSk[c].bm - 1) / kSk[c].bm, tn = (a->N + kSk[c].bn - 1) / kSk[c].bn;
  return sk_fused_ok(a, tm, tn, 1) ? (int64_t)a->M * a->N * 4 : 0;
}

extern "C" int64_t echo_gemm_ws_bytes(const EchoGemmArgs* a) {
  if (!a || a->M <= 0 || a->N <= 0 || a->K <= 0 || a->K % BK) return 0;
  if (sk_tile(a->tile)) {
    const int c = (a->tile - 100) / 10, S = a->tile % 10;
    if (c < 1 || c > kNumSk || S < 1 || !sk_ok(a)) return 0;
    return sk_ws_bytes_mod(a, c, S);
  }
  int c = 0, S = 1;
  if (a->tile == 0 && sk_plan(a, true, &c, &S)) return sk_ws_bytes_mod(a, c, S);
  return 0;
}

// the launch echo_gemm_ws would make for these arguments with a workspace of ws_bytes (host only; perf_model.py
// labels its timed launches with it): plan_route's decision as a code (echo_hip.h)
extern "C" int32_t echo_gemm_planned_tile(const EchoGemmArgs* a, int64_t ws_bytes) {
  if (!a || a->M <= 0 || a->N <= 0 || a->K <= 0 || a->K % BK) return 0;
  if (a->tile != 0) return a->tile;
  const Route r = plan_route(a, ws_bytes > 0 ? (const void*)(uintptr_t)256 : nullptr, ws_bytes);
  switch (r.kind) {
    case RT_SK: return 100 + 10 * r.c + r.S;
    case RT_T320: return 20;
    // 301-305: past the small-M codes (100 + 10 c + S <= 269), so that no label means two launches
    case RT_T320_COLSPLIT: return 301;
    case RT_W13_COLSPLIT: return 302;
    case RT_ROWSPLIT: return 303;
    case RT_HN_SPLIT: return 304;
    case RT_F32: return 305;
    default: return r.t;
  }
}

extern "C" int echo_gemm(const EchoGemmArgs* a, void* stream) { return echo_gemm_ws(a, nullptr, 0, stream); }

extern "C" int echo_gemm_ws(const EchoGemmArgs* a, void* ws, int64_t ws_bytes, void* stream) {
  if (!a || !a->A || !a->W || !a->C) return ECHO_EINVAL;
  if (a->M <= 0 || a->N <= 0 || a->K <= 0 || a->batch <= 0) return ECHO_ESHAPE;
  if (a->K % 64 || a->N % 16 || a->lda % 8 || a->ldw % 8 || a->ldc % 8) return ECHO_EALIGN;
  if (a->dtype != ECHO_BF16 && a->dtype != ECHO_F32) return ECHO_EDTYPE;
  if (a->epilogue == ECHO_EPI_RESID && !a->aux) return ECHO_EINVAL;
  if (a->epilogue == ECHO_EPI_SWIGLU && (a->N % 32 || a->bias)) return ECHO_EINVAL;
  if (a->epilogue < 0 || a->epilogue > 4) return ECHO_EINVAL;
  // leading dimensions cover the rows they address (conv mode: A rows are conv_c wide)
  if (a->lda < (a->conv_taps > 0 ? a->conv_c : a->K) || a->ldw < a->K ||
      a->ldc < (a->epilogue == ECHO_EPI_SWIGLU ? a->N / 2 : a->N) ||
      (a->epilogue == ECHO_EPI_RESID && a->ld_aux < a->N))
    return ECHO_ESHAPE;
  if (a->act < 0 || a->act > ECHO_ACT_SNAKE || (a->act == ECHO_ACT_SNAKE && !a->act_alpha)) return ECHO_EINVAL;
  if (a->conv_taps < 0 || (a->conv_taps > 0 && (a->conv_c <= 0 || a->conv_dil <= 0 ||
                                                 (int64_t)a->conv_taps * a->conv_c != a->K ||
                                                 a->conv_c % (a->dtype == ECHO_BF16 ? 64 : 16))))
    return ECHO_EINVAL;
  const bool headnorm = a->epilogue == ECHO_EPI_HEADNORM;
  if (headnorm && (a->batch != 1 || !a->hn_w || a->hn_heads <= 0 || a->hn_nblk < 0 || a->hn_seq_len <= 0 ||
                   (int64_t)a->hn_nblk * a->hn_heads * 128 > a->N || (a->hn_rope_heads > 0 && !a->hn_rope) ||
                   a->bias || a->act != ECHO_ACT_NONE || a->out_div != 0.0f))
    return ECHO_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  Epi ep{a->bias, a->stride_bias, a->aux, a->ld_aux, a->stride_aux, a->gate, a->stride_gate,
         a->epilogue, a->act, a->out_div,
         a->hn_w, a->hn_w_stride, a->hn_rope, a->hn_heads, a->hn_nblk, a->hn_rope_heads, a->hn_seq_len,
         a->hn_pos0, a->hn_pos_mult, a->hn_eps, 0, a->act_alpha, a->conv_c, a->conv_taps, a->conv_dil,
         nullptr, 0, nullptr, nullptr, 0.f};
#ifdef ECHO_DIAG
  ep.abl = g_sk_abl;
#endif
  if (a->mod_out) {
    // residual + the next AdaLN: fused into the finish kernel when the small-M plan has one (K split or
    // no direct epilogue) and a row is one finish workgroup (N == 2048); else the GEMM, then
    // echo_adaln_modulate on the rows it wrote (the same kernel arithmetic: bitwise equal)
    if (a->epilogue != ECHO_EPI_RESID || a->batch != 1 || !a->mod_shift || !a->mod_scale1 || a->ldc != a->N ||
        a->ld_mod != a->N)
      return ECHO_EINVAL;
    {  // the normalised rows may not overlap the residual rows they are computed from
      const uintptr_t es = a->dtype == ECHO_F32 ? 4 : 2, bytes = (uintptr_t)a->M * a->N * es;
      const uintptr_t c0 = (uintptr_t)a->C, m0 = (uintptr_t)a->mod_out;
      if (m0 < c0 + bytes && c0 < m0 + bytes) return ECHO_EINVAL;
    }
    const bool aligned = (((uintptr_t)a->mod_out | (uintptr_t)a->mod_shift | (uintptr_t)a->mod_scale1) & 15) == 0;
    int c = 0, S = 1;
    if (sk_tile(a->tile)) {
      c = (a->tile - 100) / 10;
      S = a->tile % 10;
    } else if (a->tile != 0 || !sk_plan(a, ws != nullptr, &c, &S)) {
      c = 0;
    }
    const int64_t need = c >= 1 && c <= kNumSk && sk_ok(a) ? sk_ws_bytes_mod(a, c, S) : 0;
    if (a->dtype == ECHO_BF16 && a->N == 2048 && aligned && need > 0 && a->K / BK >= S && ws &&
        (uintptr_t)ws % 16 == 0 && ws_bytes >= need) {
      Epi em = ep;
      em.mod_out = a->mod_out;
      em.ld_mod = a->ld_mod;
      em.mod_shift = a->mod_shift;
      em.mod_scale1 = a->mod_scale1;
      em.mod_eps = a->mod_eps;
      return launch_sk_cfg(a, em, c, S, ws, s);
    }
    EchoGemmArgs b = *a;
    b.mod_out = nullptr;
    const int rc = echo_gemm_ws(&b, ws, ws_bytes, stream);
    if (rc) return rc;
    return echo_adaln_modulate(a->dtype, a->C, a->mod_out, a->M, a->N, a->mod_shift, a->mod_scale1, 0, 0,
                               a->mod_eps, stream);
  }
  // small-M family (gemm_bf16_sk_kernel) forced by `tile` 1CS
  if (sk_tile(a->tile)) {
    const int c = (a->tile - 100) / 10, S = a->tile % 10;
    if (c < 1 || c > kNumSk || S < 1 || !sk_ok(a) || a->K / BK < S) return ECHO_EINVAL;
    const int64_t need = sk_ws_bytes(a, c, S);
    if (need > 0 && (!ws || (uintptr_t)ws % 16 || ws_bytes < need)) return ECHO_EINVAL;
    return launch_sk_cfg(a, ep, c, S, ws, (hipStream_t)stream);
  }
  // head norm not fused for this shape / dtype: plain store, then the standalone kernel (same results)
  auto hn_split = [&]() -> int {
    EchoGemmArgs b = *a;
    b.epilogue = ECHO_EPI_STORE;
    const int rc = echo_gemm(&b, stream);
    if (rc || a->hn_nblk == 0) return rc;
    return echo_head_norm_rope(a->dtype, a->C, a->ldc, a->M, a->hn_heads, a->hn_nblk, 0,
                               (int64_t)a->hn_heads * 128, a->hn_w, a->hn_w_stride, a->hn_rope, a->hn_rope_heads,
                               a->hn_seq_len, a->hn_pos0, a->hn_pos_mult, a->hn_eps, stream);
  };
  auto run_f32 = [&]() -> int {
    if (f32_mfma_ok(a)) {
      dim3 grid((a->N + QN - 1) / QN, (a->M + QM - 1) / QM, a->batch);
      hipLaunchKernelGGL(gemm_f32_mfma_kernel, grid, dim3(256), 0, s, (const float*)a->A, a->lda, a->stride_a,
                         (const float*)a->W, a->ldw, a->stride_w, a->C, a->ldc, a->stride_c, a->M, a->N,
                         a->K, ep);
    } else {
      dim3 grid((a->N + FT - 1) / FT, (a->M + FT - 1) / FT, a->batch);
      hipLaunchKernelGGL(gemm_f32_kernel, grid, dim3(256), 0, s, (const float*)a->A, a->lda, a->stride_a,
                         (const float*)a->W, a->ldw, a->stride_w, a->C, a->ldc, a->stride_c, a->M, a->N,
                         a->K, ep);
    }
    ECHO_LAUNCH_CHECK();
    return 0;
  };
  // two launches on the same stream: tile columns [0, c1) on 320-row tiles (whole rounds), the rest by the auto pick
  auto t320_colsplit = [&](int c1) -> int {
    const int n1 = c1 * 256;
    EchoGemmArgs h = *a, r = *a;
    h.N = n1;
    h.tile = 20;
    r.N = a->N - n1;
    r.W = (const bf16_t*)a->W + (int64_t)n1 * a->ldw;
    r.C = (bf16_t*)a->C + (a->epilogue == ECHO_EPI_SWIGLU ? n1 / 2 : n1);
    if (a->aux) r.aux = (const bf16_t*)a->aux + n1;
    if (a->gate) r.gate = (const bf16_t*)a->gate + n1;
    if (a->bias) r.bias = (const bf16_t*)a->bias + n1;
    const int rc = echo_gemm(&h, stream);
    return rc ? rc : echo_gemm(&r, stream);
  };
  // W13 at 1537..2048 rows: tile columns [0, c1) on the persistent 256x256 kernel, the rest on small-M config 13
  auto w13_colsplit = [&](int c1) -> int {
    const int n1 = c1 * 256;
    EchoGemmArgs h = *a, r = *a;
    h.N = n1;
    h.tile = 16;
    r.N = a->N - n1;
    r.W = (const bf16_t*)a->W + (int64_t)n1 * a->ldw;
    r.C = (bf16_t*)a->C + n1 / 2;
    r.tile = 100 + 10 * 13 + 1;
    const int rc = echo_gemm(&h, stream);
    return rc ? rc : echo_gemm(&r, stream);
  };
  // two launches on the same stream: full rounds of the 256x256 kernel, then the row tail
  auto rowsplit = [&](int M1, int tail_cfg, int t) -> int {
    EchoGemmArgs h = *a, r = *a;
    h.M = M1;
    h.tile = t;
    r.M = a->M - M1;
    r.tile = tail_cfg;
    r.A = (const bf16_t*)a->A + (int64_t)M1 * a->lda;
    r.C = (a->epilogue == ECHO_EPI_F32OUT ? (void*)((float*)a->C + (int64_t)M1 * a->ldc)
                                           : (void*)((bf16_t*)a->C + (int64_t)M1 * a->ldc));
    if (a->aux) r.aux = (const bf16_t*)a->aux + (int64_t)M1 * a->ld_aux;
    const int rc = echo_gemm(&h, stream);
    return rc ? rc : echo_gemm(&r, stream);
  };
  auto run_tile = [&](int t) -> int {
    switch (t) {
      case 1: return launch_bf16<256, 256, 2, 4>(a, ep, s);
      case 2: return launch_bf16<256, 128, 4, 2>(a, ep, s);
      case 3: return launch_bf16<128, 128, 2, 2>(a, ep, s);
      case 4: return launch_bf16<128, 64, 2, 2>(a, ep, s);
      case 5: return launch_bf16<64, 64, 2, 2>(a, ep, s);
      case 6: return launch_pp<0>(a, ep, s);
#ifdef ECHO_DIAG
      // timing ablations of the 4-phase kernel (results wrong): diagnostics build only
      case 7: return launch_pp<1>(a, ep, s);
      case 8: return launch_pp<2>(a, ep, s);
      case 9: return launch_pp<3>(a, ep, s);
      case 10: return launch_pp<4>(a, ep, s);
      case 11: return launch_pp<8>(a, ep, s);
      case 12: return launch_pp<11>(a, ep, s);
      case 15:  // no epilogue (ep.epi = 99 above)
#endif
      case 13: return launch_pp2(a, ep, s);
      case 16: return ps_ok(a, ek_of(a)) ? launch_ps(a, ep, s) : launch_pp2(a, ep, s);
      case 18: return ps_ok(a, ek_of(a)) ? launch_ps(a, ep, s) : ECHO_EINVAL;  // group-M override (diag key 1)
      default: return ECHO_EINVAL;
    }
  };
  const bool misaligned = ((uintptr_t)a->A | (uintptr_t)a->W | (uintptr_t)a->C) & 15;
  if (a->tile == 0) {  // the auto plan (plan_route; echo_gemm_planned_tile reports the same decision)
    const Route r = plan_route(a, ws, ws_bytes);
    if (r.kind == RT_SK) return launch_sk_cfg(a, ep, r.c, r.S, r.sk_ws ? ws : nullptr, s);
    if (r.kind == RT_HN_SPLIT) return hn_split();
    if (r.kind == RT_F32) return run_f32();
    if (a->dtype != ECHO_BF16) return ECHO_EDTYPE;
    if (misaligned) return ECHO_EALIGN;
    switch (r.kind) {
      case RT_T320_COLSPLIT: return t320_colsplit(r.c1);
      case RT_T320: return launch_t320(a, ep, s);
      case RT_W13_COLSPLIT: return w13_colsplit(r.c1);
      case RT_ROWSPLIT: return rowsplit(r.M1, r.tail, r.t);
      default: return run_tile(r.t);
    }
  }
  // forced tile (tests, tools/bench_gemm.py)
  if (a->tile == 18) ep.gm = g_gemm_gm;
#ifdef ECHO_DIAG
  if (a->tile == 15) ep.epi = 99;  // diagnostic: no epilogue (diagnostics build only)
#endif
  const int t = a->tile;
  // fused on the persistent kernel (t 16/18, N % 256 == 0, via ps_ok), the 2-phase one (t 13) or 320-row tiles
  const bool hn_fused = a->dtype == ECHO_BF16 && ((t == 13 && a->N % 128 == 0) ||
                                                   ((t == 16 || t == 18) && ps_ok(a, EK_HEADNORM)) ||
                                                   ((t >= 20 && t <= 23) && t320_ok(a)));
  if (headnorm && !hn_fused) return hn_split();
  if (a->dtype == ECHO_F32) return run_f32();
  if (a->dtype != ECHO_BF16) return ECHO_EDTYPE;
  if (misaligned) return ECHO_EALIGN;
  if (t == 20) return t320_ok(a) ? launch_t320(a, ep, s) : ECHO_EINVAL;  // 320-row tiles (auto DMA split)
  if (t == 21) return t320_ok(a) ? launch_t320_sp<1, 0>(a, ep, s) : ECHO_EINVAL;  // 4 / 5 DMA split (A/B)
  if (t == 22) return t320_ok(a) ? launch_t320_sp<0, 0>(a, ep, s) : ECHO_EINVAL;  // one tile per workgroup
  if (t == 23) return t320_ok(a) ? launch_t320_sp<0, 1>(a, ep, s) : ECHO_EINVAL;  // persistent
  return run_tile(t);
}

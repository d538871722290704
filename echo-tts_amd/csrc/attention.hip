// attention.hip — segmented joint attention with fused sigmoid gate.
//
// Replaces JointAttention.forward's KV concat + SDPA + gating
// (reference model.py:237-264) and SelfAttention's SDPA + gating (model.py:144-157).
// The reference concatenates [self | latent | text | speaker] keys and masks them
// with a bool mask; every mask it builds is a prefix per segment
// (inference.py:204-207,284-287, model.py:243-244), so this kernel walks up to four
// segments in place with per-row valid lengths and never touches masked keys
// (bit-identical to masking them: exp(-inf) = 0). CFG rows share one physical
// copy of the text/speaker KV through `batch_mod`.
//
// bf16 kernel: one workgroup = 4 waves = 128 queries of one (row, head); each wave
// owns 32 queries. Scores are computed transposed, S^T = K.Q^T with
// v_mfma_f32_32x32x16_bf16, so each lane holds 16 keys of ONE query: the row max
// is 15 fmax + one cross-half shuffle. P feeds the PV product straight from the
// accumulator registers (bf16-packed) as the B operand of O^T = V^T.P, and V^T
// fragments come from a row-major LDS tile via ds_read_b64_tr_b16. K and V tiles
// (64 keys x 128) use one XOR image (chunk ^ ((r&3)<<2 | (r>>2)&3)) that is
// conflict-free for both the K row reads and the V transposed reads.
#include "common.h"

namespace {

__device__ __forceinline__ int swz(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }

__device__ __forceinline__ int remap_xcd(int bid, int nwg) {
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
}

// LDS-DMA (global_load_lds_dwordx4) issued through inline asm: hipcc does not see it, so it
// cannot insert a conservative vmcnt(0) in front of the ds_reads of the OTHER buffer (it did
// for the V transposed reads). Completion is waited for explicitly (vmcnt(0) + barrier at the
// end of each tile). M0 is saved/restored inside the statement (cdna_hip_programming.md §5.7).
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_addr) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_addr) : "memory");
}

__device__ __forceinline__ uint32_t lds_addr_of(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

constexpr int QB = 128;  // queries per workgroup
constexpr int KT = 64;   // keys per tile

struct SegInfo {
  const bf16_t* kb;
  const bf16_t* vb;
  int64_t ld;
  int kend, causal, first;  // first = index of the segment's first tile in the flat tile list
};

__global__ void __launch_bounds__(256, 2) attn_bf16_kernel(EchoAttnArgs a) {
  // [buffer][K | V][64 keys x 128] — one array (keeps hipcc from draining DMA before ds_reads)
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * 2 * KT * 128];

  const int nqb = (a.n_q + QB - 1) / QB;
  const int L = remap_xcd(blockIdx.x, gridDim.x);
  const int qb = L % nqb;
  const int head = (L / nqb) % a.heads;
  const int row = L / (nqb * a.heads);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h2 = lane >> 5, ql = lane & 31;
  const int q0 = qb * QB;
  const int qi = q0 + w * 32 + ql;
  const int qc = min(qi, a.n_q - 1);

  const bf16_t* qp = (const bf16_t*)a.q + row * a.q_ld_batch + (int64_t)qc * a.q_ld_tok + head * 128;
  bf16x8 qf[8];
#pragma unroll
  for (int ds = 0; ds < 8; ++ds) qf[ds] = *(const bf16x8*)(qp + 16 * ds + 8 * h2);
  // consume Q here so hipcc waits for it once, not inside the tile loop (where its counted
  // waits would land on the asm DMA of the next tile)
#pragma unroll
  for (int ds = 0; ds < 8; ++ds) asm volatile("" ::"v"(qf[ds]));

  // flat list of 64-key tiles over the (up to 4) segments; per-segment fields are kept in
  // named scalars (no runtime-indexed arrays: those go to scratch)
  SegInfo s0{}, s1{}, s2{}, s3{};
  int ntiles = 0;
  auto init_seg = [&](int sg, SegInfo& d) {
    d.first = ntiles;
    if (sg < a.nseg && a.seg[sg].k) {
      const EchoKVSegment& S = a.seg[sg];
      const int len = S.len ? S.len[row] : S.capacity;
      int kend = min(len, S.capacity);
      if (S.causal) kend = min(kend, q0 + QB);
      kend = max(kend, 0);
      const int b = row % S.batch_mod;
      d.kb = (const bf16_t*)S.k + b * S.ld_batch + head * 128;
      d.vb = (const bf16_t*)S.v + b * S.ld_batch + head * 128;
      d.ld = S.ld_tok;
      d.kend = kend;
      d.causal = S.causal;
      ntiles += (kend + KT - 1) / KT;
    }
  };
  init_seg(0, s0);
  init_seg(1, s1);
  init_seg(2, s2);
  init_seg(3, s3);
  auto pick = [&](int ti) -> SegInfo {
    return ti >= s3.first && s3.kend > 0 ? s3 : ti >= s2.first && s2.kend > 0 ? s2
         : ti >= s1.first && s1.kend > 0 ? s1 : s0;
  };

  // DMA of tile ti into buffer `buf`: 64 rows x 256 B for K and V = 32 wave-instructions
  // of 1 KiB (4 rows each); lane-linear LDS image, XOR swizzle applied on the source chunk.
  const int dr = lane >> 4, dp = lane & 15;
  auto dma_tile = [&](int ti, int buf) {
    const SegInfo d = pick(ti);
    const int t0 = (ti - d.first) * KT;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = (i * 4 + w) * 4 + dr;  // tile row 0..63 written by this lane
      const int64_t tok = min(t0 + r, d.kend - 1);
      const int c = dp ^ swz(r);
      const int dst = ((i * 4 + w) * 4) * 128;
      const uint32_t kdst = __builtin_amdgcn_readfirstlane(lds_addr_of(lds + (buf * 2) * KT * 128 + dst));
      const uint32_t vdst = __builtin_amdgcn_readfirstlane(lds_addr_of(lds + (buf * 2 + 1) * KT * 128 + dst));
      glds16(d.kb + tok * d.ld + c * 8, kdst);
      glds16(d.vb + tok * d.ld + c * 8, vdst);
    }
  };

  f32x16 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;
  const float sl2 = a.scale * 1.4426950408889634f;
  const int g = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;

  if (ntiles > 0) dma_tile(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int ti = 0; ti < ntiles; ++ti) {
    const int cur = ti & 1;
    if (ti + 1 < ntiles) dma_tile(ti + 1, cur ^ 1);  // lands while this tile computes
    const bf16_t* Ks = lds + (cur * 2) * KT * 128;
    const bf16_t* Vs = Ks + KT * 128;
    const SegInfo d = pick(ti);
    const int t0 = (ti - d.first) * KT;
    const int kend = d.kend;
    const bool full = (t0 + KT <= kend) && !d.causal;

    // ---- S^T = K . Q^T for two 32-key sub-tiles
    f32x16 st[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int r = 0; r < 16; ++r) st[kk][r] = 0.f;
      const int kr_ = kk * 32 + ql;
#pragma unroll
      for (int ds = 0; ds < 8; ++ds) {
        const int c = 2 * ds + h2;
        const bf16x8 kf = *(const bf16x8*)(Ks + kr_ * 128 + ((c ^ swz(kr_)) * 8));
        st[kk] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ds], st[kk], 0, 0, 0);
      }
    }
    // ---- mask (partial tiles only), online softmax (lane = query, registers = keys).
    // The running max is kept on RAW scores (scale > 0 preserves the argmax); one FMA per score
    // forms the exp2 argument s*c - m*c; raw v_exp_f32 (results < 2^-126 flush to 0).
    float mx = -INFINITY;
    if (!full) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = t0 + kk * 32 + (r & 3) + 8 * (r >> 2) + 4 * h2;
          const bool ok = key < kend && (!d.causal || key <= qi);
          st[kk][r] = ok ? st[kk][r] : -INFINITY;
        }
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int r = 0; r < 16; r += 2) mx = fmaxf(mx, fmaxf(st[kk][r], st[kk][r + 1]));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_run, mx);
    const float msc = m_new == -INFINITY ? 0.f : -m_new * sl2;
    float psum = 0.f;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(st[kk][r], sl2, msc));
        st[kk][r] = pv;
        psum += pv;
      }
    if (__any(m_new != m_run)) {  // otherwise alpha == 1 exactly for every lane
      const float alpha = __builtin_amdgcn_exp2f(__builtin_fmaf(m_run, sl2, msc));
      l_run *= alpha;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
    }
    l_run += psum;
    m_run = m_new;

    // ---- O^T += V^T . P  (P from the accumulators, V^T by transposed LDS reads)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        bf16x8 pf;
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[j] = (__bf16)st[kk][8 * s2 + j];
        const int key0 = kk * 32 + 16 * s2 + 4 * h2;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const int ch = 4 * dt + 2 * (g & 1) + (p4 >> 1);
          const int r0 = key0 + q4, r1 = key0 + 8 + q4;
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(Vs + r0 * 128 + ((ch ^ swz(r0)) * 8) + (p4 & 1) * 4));
          const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(Vs + r1 * 128 + ((ch ^ swz(r1)) * 8) + (p4 & 1) * 4));
          typedef __attribute__((ext_vector_type(8))) short s16x8;
          const s16x8 v8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, v8), pf, o[dt], 0, 0, 0);
        }
      }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // next tile landed (this wave's share)
    __syncthreads();                                    // ... and everyone's; buffer `cur` free
  }

  // ---- epilogue: normalise, round, gate, store (4 consecutive d per register group)
  const float lt = l_run + __shfl_xor(l_run, 32, 64);
  const float inv = 1.0f / lt;
  if (qi >= a.n_q) return;
  bf16_t* op = (bf16_t*)a.out + row * a.o_ld_batch + (int64_t)qi * a.o_ld_tok + head * 128;
  const bf16_t* gp = a.gate ? (const bf16_t*)a.gate + row * a.g_ld_batch + (int64_t)qi * a.g_ld_tok + head * 128
                            : nullptr;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int rg = 0; rg < 4; ++rg) {
      const int d = dt * 32 + 8 * rg + 4 * h2;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = rbf(o[dt][4 * rg + e] * inv);
      if (gp) {
        const uint2 gg = *(const uint2*)(gp + d);
        const float gv[4] = {bf2f(gg.x & 0xffffu), bf2f(gg.x >> 16), bf2f(gg.y & 0xffffu), bf2f(gg.y >> 16)};
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = rbf(v[e] * rbf(sigmoid_f(gv[e])));
      }
      *(uint2*)(op + d) = make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
    }
}

// ----------------------------------------------------------------------------- fp32 (parity mode)
constexpr int FQ = 64, FKT = 32;

__global__ void __launch_bounds__(64) attn_f32_kernel(EchoAttnArgs a) {
  __shared__ float Ks[FKT][128], Vs[FKT][128];
  const int nqb = (a.n_q + FQ - 1) / FQ;
  const int L = blockIdx.x;
  const int qb = L % nqb, head = (L / nqb) % a.heads, row = L / (nqb * a.heads);
  const int tid = threadIdx.x;
  const int qi = qb * FQ + tid, qc = min(qi, a.n_q - 1);
  const float* qp = (const float*)a.q + row * a.q_ld_batch + (int64_t)qc * a.q_ld_tok + head * 128;
  float q[128], o[128];
#pragma unroll
  for (int d = 0; d < 128; ++d) { q[d] = qp[d]; o[d] = 0.f; }
  float m = -INFINITY, l = 0.f;
#pragma unroll
  for (int sg = 0; sg < 4; ++sg) {
    if (sg >= a.nseg) break;
    const EchoKVSegment S = a.seg[sg];
    if (!S.k) continue;
    const int len = S.len ? S.len[row] : S.capacity;
    int kend = min(len, S.capacity);
    if (S.causal) kend = min(kend, qb * FQ + FQ);
    if (kend <= 0) continue;
    const int b = row % S.batch_mod;
    const float* kb = (const float*)S.k + b * S.ld_batch + head * 128;
    const float* vb = (const float*)S.v + b * S.ld_batch + head * 128;
    for (int t0 = 0; t0 < kend; t0 += FKT) {
      __syncthreads();
      for (int e = tid; e < FKT * 32; e += 64) {
        const int r = e / 32, c = (e % 32) * 4;
        const int64_t tok = min(t0 + r, kend - 1);
        *(float4*)&Ks[r][c] = *(const float4*)(kb + tok * S.ld_tok + c);
        *(float4*)&Vs[r][c] = *(const float4*)(vb + tok * S.ld_tok + c);
      }
      __syncthreads();
      for (int kk = 0; kk < FKT; ++kk) {
        const int key = t0 + kk;
        if (key >= kend || (S.causal && key > qi)) continue;
        float s = 0.f;
#pragma unroll
        for (int d = 0; d < 128; ++d) s = fmaf(q[d], Ks[kk][d], s);
        s *= a.scale;
        const float mn = fmaxf(m, s);
        const float al = expf(m - mn), p = expf(s - mn);
        l = l * al + p;
#pragma unroll
        for (int d = 0; d < 128; ++d) o[d] = o[d] * al + p * Vs[kk][d];
        m = mn;
      }
    }
  }
  if (qi >= a.n_q) return;
  float* op = (float*)a.out + row * a.o_ld_batch + (int64_t)qi * a.o_ld_tok + head * 128;
  const float* gp = a.gate ? (const float*)a.gate + row * a.g_ld_batch + (int64_t)qi * a.g_ld_tok + head * 128
                           : nullptr;
#pragma unroll
  for (int d = 0; d < 128; ++d) {
    float v = o[d] / l;
    if (gp) v = v * sigmoid_f(gp[d]);
    op[d] = v;
  }
}

}  // namespace

extern "C" int echo_attention(const EchoAttnArgs* a, void* stream) {
  if (!a || !a->q || !a->out) return ECHO_EINVAL;
  if (a->rows <= 0 || a->n_q <= 0 || a->heads <= 0 || a->nseg < 1 || a->nseg > 4) return ECHO_ESHAPE;
  bool any = false;
  for (int s = 0; s < a->nseg; ++s) {
    const EchoKVSegment& S = a->seg[s];
    if (!S.k) continue;
    if (!S.v || S.batch_mod <= 0 || S.capacity <= 0) return ECHO_EINVAL;
    if (S.ld_tok % 8 || S.ld_batch % 8) return ECHO_EALIGN;
    any = true;
  }
  if (!any) return ECHO_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (a->dtype == ECHO_BF16) {
    if (a->q_ld_tok % 8 || a->o_ld_tok % 4) return ECHO_EALIGN;
    const int nqb = (a->n_q + QB - 1) / QB;
    hipLaunchKernelGGL(attn_bf16_kernel, dim3(nqb * a->heads * a->rows), dim3(256), 0, s, *a);
  } else if (a->dtype == ECHO_F32) {
    const int nqb = (a->n_q + FQ - 1) / FQ;
    hipLaunchKernelGGL(attn_f32_kernel, dim3(nqb * a->heads * a->rows), dim3(64), 0, s, *a);
  } else {
    return ECHO_EDTYPE;
  }
  ECHO_LAUNCH_CHECK();
  return 0;
}

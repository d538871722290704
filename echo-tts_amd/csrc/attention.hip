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

#include <type_traits>

// q / gate row of output row `row` (EchoAttnArgs.q_batch_mod: row groups that share one q copy)
#define ECHO_QROW(a, row) ((a).q_batch_mod > 0 ? (row) % (a).q_batch_mod : (row))

namespace {

template <class Args>  // EchoAttnArgs, or the split kernel's kernarg-segment view of it
__device__ void attn_combine_unit(const Args& a, const float* __restrict__ ws, int nsp, int rh, int qi, int c8);

__device__ __forceinline__ int swz(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }

// max of three fp32 values in one v_max3_f32 (scores are finite or -inf: no NaN handling needed)
__device__ __forceinline__ float max3_f(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// x of lane l combined with x of lane l ^ 32 through v_permlane32_swap (VALU) instead of __shfl_xor's
// ds_bpermute (an LDS round trip on the QK -> softmax critical path): swap(x, x) gives every lane both
// halves' values; max and + are exact and commutative, so the result equals the __shfl_xor form
__device__ __forceinline__ float halves_max(float x) {
  const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
}
__device__ __forceinline__ float halves_sum(float x) {
  const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
}

__device__ __forceinline__ int remap_xcd(int bid, int nwg) {
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
}

constexpr int KT = 64;   // keys per tile

// Diagnostics only (echo_attention_variant ablation bit 128, tools/attn_timeline.py): s_memrealtime
// stamps [entry, prologue landed, tile loop done, exit, ntiles, XCD] written by wave 0, lane 0.
__device__ uint64_t* g_attn_stamps;
__device__ __forceinline__ uint64_t rt_now() { return __builtin_amdgcn_s_memrealtime(); }
// bit 512: per-tile phase stamps (s_memtime, shader cycles) of workgroup 0's waves, stored after the
// per-workgroup area: [wave][tile < 64][6] = tile start, scores ready, softmax done, PV issued,
// DMA landed, barrier passed
__device__ __forceinline__ void phase_stamp(uint64_t* at) {
  __builtin_amdgcn_sched_barrier(0);
  const uint64_t t = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) *at = t;
  __builtin_amdgcn_sched_barrier(0);
}

// value select (a ?: between two named variables is an lvalue: clang selects their ADDRESSES,
// which keeps SROA from promoting them and sends them to scratch)
template <class T>
__device__ __forceinline__ T sel4(int sg, T a0, T a1, T a2, T a3) {
  return sg == 3 ? a3 : sg == 2 ? a2 : sg == 1 ? a1 : a0;
}

// ---- shared epilogue of the bf16 kernels: O / l, round, * round(sigmoid(gate)), round, store.
// A lane holds query qi, columns 8k + 4*h2 .. +3 of each 8-column group k (k = 4*dt + rg). Each
// pair of groups (k, k+1) is packed to bf16 and exchanged across the wave halves with
// v_permlane32_swap (cdna_hip_programming.md T21): lanes 0-31 then hold columns 8k .. 8k+7, lanes
// 32-63 columns 8k+8 .. 8k+15, so gate loads and output stores are 16 B per lane (8 + 8 instead of
// 16 + 16 8-B accesses; the store tail is issue-bound). Same roundings as the reference
// (model.py:255-264: SDPA out bf16, sigmoid(gate) bf16, product bf16).
// normalise by 1/l, round to bf16, pack: v4[pk] = this lane's 8 columns 16*pk + 8*h2 of query ql
__device__ __forceinline__ void attn_pack_o(const f32x16 (&o)[4], float inv, uint4 (&v4)[8]) {
  uint32_t w[16][2];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int dt = k >> 2, rg = k & 3;
    w[k][0] = pack2bf(rbf(o[dt][4 * rg + 0] * inv), rbf(o[dt][4 * rg + 1] * inv));
    w[k][1] = pack2bf(rbf(o[dt][4 * rg + 2] * inv), rbf(o[dt][4 * rg + 3] * inv));
  }
#pragma unroll
  for (int pk = 0; pk < 8; ++pk) {
    const auto x = __builtin_amdgcn_permlane32_swap(w[2 * pk][0], w[2 * pk + 1][0], false, false);
    const auto y = __builtin_amdgcn_permlane32_swap(w[2 * pk][1], w[2 * pk + 1][1], false, false);
    v4[pk] = make_uint4(x[0], y[0], x[1], y[1]);
  }
}

// out = round(round(o / l) * round(sigmoid(gate))) (model.py:255-264 roundings) on element-aligned
// packed bf16 (v4: normalised O, g4: gates, any common layout). The precise path is needed only for
// gates below -87 (bf16 bits above 0xC2AE as unsigned 16-bit: negative, magnitude > 87; NaNs also
// land there): one packed-u16 max over the lane's 64 gates decides, for the whole wave.
__device__ __forceinline__ void attn_gate(uint4 (&v4)[8], const uint4 (&g4)[8]) {
  typedef __attribute__((ext_vector_type(2))) unsigned short u16x2;
  u16x2 gmax = {0, 0};
#pragma unroll
  for (int pk = 0; pk < 8; ++pk) {
    gmax = __builtin_elementwise_max(gmax, __builtin_bit_cast(u16x2, g4[pk].x));
    gmax = __builtin_elementwise_max(gmax, __builtin_bit_cast(u16x2, g4[pk].y));
    gmax = __builtin_elementwise_max(gmax, __builtin_bit_cast(u16x2, g4[pk].z));
    gmax = __builtin_elementwise_max(gmax, __builtin_bit_cast(u16x2, g4[pk].w));
  }
  const bool tiny = gmax[0] > 0xC2AEu || gmax[1] > 0xC2AEu;
  auto gated = [&](bool precise) __attribute__((always_inline)) {
#pragma unroll
    for (int pk = 0; pk < 8; ++pk) {
      const uint32_t vv[4] = {v4[pk].x, v4[pk].y, v4[pk].z, v4[pk].w};
      const uint32_t gg[4] = {g4[pk].x, g4[pk].y, g4[pk].z, g4[pk].w};
      uint32_t r[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float g0 = bf2f(gg[e] & 0xffffu), g1 = bf2f(gg[e] >> 16);
        const float s0 = precise ? sigmoid_f(g0) : sigmoid_hw(g0);
        const float s1 = precise ? sigmoid_f(g1) : sigmoid_hw(g1);
        r[e] = pack2bf(rbf(bf2f(vv[e] & 0xffffu) * rbf(s0)), rbf(bf2f(vv[e] >> 16) * rbf(s1)));
      }
      v4[pk] = make_uint4(r[0], r[1], r[2], r[3]);
    }
  };
  if (__builtin_expect(__any(tiny), 0)) gated(true);
  else gated(false);
}

__device__ __forceinline__ void attn_pack_out(const f32x16 (&o)[4], float inv, int h2, bool valid, const bf16_t* gp,
                                              uint4 (&v4)[8]) {
  attn_pack_o(o, inv, v4);
  if (!valid || !gp) return;
  const int c0 = 8 * h2;  // this lane's 8 columns of each 16-column pair
  uint4 g4[8];
#pragma unroll
  for (int pk = 0; pk < 8; ++pk) g4[pk] = *(const uint4*)(gp + 16 * pk + c0);
  attn_gate(v4, g4);
}

__device__ __forceinline__ void attn_bstore(const uint4& v, __amdgpu_buffer_rsrc_t rs, uint32_t off) {
  typedef __attribute__((__vector_size__(4 * sizeof(unsigned int)))) unsigned int u32v4;
  __builtin_amdgcn_raw_buffer_store_b128(u32v4{v.x, v.y, v.z, v.w}, rs, off, 0, 0);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t attn_rsrc(const void* p, uint32_t bytes);
__device__ __forceinline__ void attn_bstore(const uint4& v, __amdgpu_buffer_rsrc_t rs, uint32_t off);

// row-layout output of one wave (attn_bf16_kernel's epilogue): lane (rl, cc) = (lane / 16, lane % 16)
// stores rows 4*pk + rl, columns 8*cc .. 8*cc + 7 of the wave's 32-row tile at `ob` (row stride
// ld elements); rows >= nv fall outside the buffer range and are dropped (always 8 instructions)
__device__ __forceinline__ void attn_store_rows(const uint4 (&v4)[8], bf16_t* ob, int nv, int64_t ld, int lane) {
  const __amdgpu_buffer_rsrc_t rs = attn_rsrc(ob, (uint32_t)(((int64_t)(min(nv, 32) - 1) * ld + 128) * 2));
  const uint32_t lo = (uint32_t)(((lane >> 4) * ld + (lane & 15) * 8) * 2), step = (uint32_t)(ld * 8);
#pragma unroll
  for (int pk = 0; pk < 8; ++pk) attn_bstore(v4[pk], rs, lo + pk * step);
}

__device__ __forceinline__ uint4 attn_bload(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
  typedef __attribute__((__vector_size__(4 * sizeof(unsigned int)))) unsigned int u32v4;
  const u32v4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
  return make_uint4(v[0], v[1], v[2], v[3]);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t attn_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

// 8-B write-through store of the in-launch split-KV merge's (m, l) pair (common.h: the 16-B form, the protocol)
__device__ __forceinline__ void st_sc1_b64(float* p, float2 v) {
  const uint64_t bits = ((uint64_t)__float_as_uint(v.y) << 32) | __float_as_uint(v.x);
  __hip_atomic_store((uint64_t*)p, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// 8 16-B stores per valid lane (a wave with any valid lane issues exactly 8 store instructions)
__device__ __forceinline__ void attn_write_out(const uint4 (&v4)[8], bf16_t* op, int h2, bool valid) {
  if (!valid) return;
#pragma unroll
  for (int pk = 0; pk < 8; ++pk) *(uint4*)(op + 16 * pk + 8 * h2) = v4[pk];
}

__device__ __forceinline__ void attn_store_out(const f32x16 (&o)[4], float inv, int qi, int h2, bool valid,
                                               bf16_t* op, const bf16_t* gp) {
  (void)qi;
  uint4 v4[8];
  attn_pack_out(o, inv, h2, valid, gp, v4);
  attn_write_out(v4, op, h2, valid);
}

// ---- shared by the bf16 kernels: per-workgroup segment table and tile cursors.
// Segment fields live in named scalars (struct copies / runtime-indexed arrays of them go to
// scratch; kernel-argument references copy the whole argument block to scratch), filled straight
// from the kernel arguments; needs a, row, head, q0, QB, KTT in scope.
#define ECHO_SEG_TABLE()                                                                       \
  const bf16_t *kb0 = nullptr, *kb1 = nullptr, *kb2 = nullptr, *kb3 = nullptr;                 \
  const bf16_t *vb0 = nullptr, *vb1 = nullptr, *vb2 = nullptr, *vb3 = nullptr;                 \
  int64_t ld0 = 0, ld1 = 0, ld2 = 0, ld3 = 0;                                                  \
  int ke0 = 0, ke1 = 0, ke2 = 0, ke3 = 0, ca0 = 0, ca1 = 0, ca2 = 0, ca3 = 0;                  \
  int ntiles = 0;                                                                              \
  ECHO_SEG_ENTRY(0)                                                                            \
  ECHO_SEG_ENTRY(1)                                                                            \
  ECHO_SEG_ENTRY(2)                                                                            \
  ECHO_SEG_ENTRY(3)
#define ECHO_SEG_ENTRY(SG)                                                                     \
  if (SG < a.nseg && a.seg[SG].k) {                                                            \
    const int len_ = a.seg[SG].len ? a.seg[SG].len[row] : a.seg[SG].capacity;                  \
    int kend_ = min(len_, a.seg[SG].capacity);                                                 \
    if (a.seg[SG].causal) kend_ = min(kend_, q0 + QB);                                         \
    kend_ = max(kend_, 0);                                                                     \
    const int b_ = row % a.seg[SG].batch_mod;                                                  \
    kb##SG = (const bf16_t*)a.seg[SG].k + b_ * a.seg[SG].ld_batch + head * 128;                \
    vb##SG = (const bf16_t*)a.seg[SG].v + b_ * a.seg[SG].ld_batch + head * 128;                \
    ld##SG = a.seg[SG].ld_tok;                                                                 \
    ke##SG = kend_;                                                                            \
    ca##SG = a.seg[SG].causal;                                                                 \
    ntiles += (kend_ + KTT - 1) / KTT;                                                         \
  }

// Tile cursor over the flat tile list [segment 0 tiles | segment 1 tiles | ...]: scalar state
// advanced one tile per call (each cursor visits tiles in order); segment fields are re-selected
// only when a segment ends.
struct Cursor {
  int seg, left, t0, kend, causal, ld;
  const bf16_t *kb, *vb;
};
#define ECHO_CURSOR_ADVANCE()                                                                  \
  auto advance = [&](Cursor& c) __attribute__((always_inline)) {                               \
    if (c.left == 0) {                                                                         \
      do { ++c.seg; } while (c.seg < 3 && sel4(c.seg, ke0, ke1, ke2, ke3) <= 0);               \
      c.kb = sel4(c.seg, kb0, kb1, kb2, kb3);                                                  \
      c.vb = sel4(c.seg, vb0, vb1, vb2, vb3);                                                  \
      c.ld = (int)sel4(c.seg, ld0, ld1, ld2, ld3);                                             \
      c.kend = sel4(c.seg, ke0, ke1, ke2, ke3);                                                \
      c.causal = sel4(c.seg, ca0, ca1, ca2, ca3);                                              \
      c.t0 = 0;                                                                                \
      c.left = (c.kend + KTT - 1) / KTT;                                                       \
    } else {                                                                                   \
      c.t0 += KTT;                                                                             \
    }                                                                                          \
    --c.left;                                                                                  \
  };

struct SegInfo {
  const bf16_t* kb;
  const bf16_t* vb;
  int64_t ld;
  int kend, causal, first;  // first = index of the segment's first tile in the flat tile list
};

// ABL: timing ablations only (echo_attention_variant, tools/bench_attn.py; results are wrong):
// 1 = no in-loop DMA, 2 = no softmax VALU, 4 = no PV (MFMA + V reads), 8 = no QK (MFMA + K reads)
// NW waves x 32 queries per workgroup (QB = 32 NW). K/V staging: ST = 2 or 3 -> ST-stage LDS ring
// filled by LDS-DMA (tile t+ST-1 issued at tile t); ST = 0 -> register staging (cdna_hip_programming.md
// T14): tile t+2 is loaded into VGPRs at the top of tile t and written (swizzled) into the free LDS
// buffer at the top of tile t+1, so 2 LDS buffers give a 2-tile lookahead.
//
// PS = 1 (variant 8; production for 1-3 items per slot until the row-layout epilogue made the plain
// grid faster): persistent form of the production schedule — gridDim.x workgroups walk the (q block, row,
// head) items item = blockIdx.x + k * gridDim.x (same XCD for every k when gridDim.x % 8 == 0). An
// item's gated output is stored after the NEXT item's Q loads and first K/V DMA have been issued, and
// only those are waited for (vmcnt counts loads, LDS-DMA and stores in issue order), so the store
// tail of one item overlaps the prologue of the next instead of a workgroup teardown + relaunch.
//
// SP = 1: split-KV form for launches with fewer items than CUs (B = 1 sampler steps, blockwise
// blocks). Item = (q block, split, row, head); split s of nsp walks tiles [s*n/nsp, (s+1)*n/nsp) of
// the item's flat tile list and stores its UNNORMALISED partial (O fp32, m in exp2 units, l) to
// `ws` (layout: attn_split_ws_bytes); attn_combine_kernel merges the splits, normalises, gates and
// stores. Same tile math; only the summation order over keys differs from SP = 0 (fp32-close).
// SP = 2: the same split, merged inside the launch (no attn_combine_kernel): each split publishes its partial
// with write-through (sc1) stores, every storing wave drains, one lane adds to the item's arrival counter in
// `sync` and polls it (relaxed, bounded) until all nsp splits have arrived, then ONE agent-scope acquire and
// the workgroup merges its 1/nsp share of the item's (query, 8-column) units with attn_combine_unit — the
// combine kernel's arithmetic, so the output is bitwise the SP = 1 + combine result (cdna_hip_programming.md
// Guideline 16, R1 / counter form). Needs every split of an item resident at once: the host launches it only
// for grids of at most one workgroup per CU. The last split to depart resets the item's two counters, so
// `sync` (caller-owned, zero at first use) is zero again when the launch ends.
template <int ABL, int NW, int ST, int KTT = 64, int PS = 0, int SP = 0>
__global__ void __launch_bounds__(64 * NW, NW <= 4 ? (KTT == 32 ? 3 : 2) : 1)
    attn_bf16_kernel(EchoAttnArgs a_arg, float* ws, int nsp, uint32_t* sync) {
  static_assert(!PS || (ABL == 0 && ST == 2), "persistent form: production schedule only");
  static_assert(!SP || (ABL == 0 && ST == 2 && !PS && NW == 4), "split-KV form: production schedule only");
  constexpr int QB = 32 * NW;
  constexpr int DPT = KTT / (4 * NW);  // DMA wave-instructions per wave per K (or V) tile
  const uint64_t ts0 = (ABL & 128) ? rt_now() : 0;
  constexpr int NKK = KTT / 32;        // 32-key sub-tiles per tile
  // [stage][K | V][64 keys x 128] — one array (keeps hipcc from draining DMA before ds_reads)
  constexpr int NBUF = ST == 0 ? 2 : ST;
  __shared__ __attribute__((aligned(16))) bf16_t lds[NBUF * 2 * KTT * 128];

  // the arguments are read through the kernarg segment pointer; in the persistent form it is
  // laundered per item, so hipcc re-reads them instead of hoisting the ~50 scalars of the segment
  // table out of the item loop (where they spill)
  using KArgs = const __attribute__((address_space(4))) EchoAttnArgs;
  KArgs* const kargs = (KArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  (void)a_arg;
  const int nqb = (kargs->n_q + QB - 1) / QB;
  const int nitems = PS ? nqb * kargs->rows * kargs->heads : (int)blockIdx.x + 1;
  (void)ws;
  (void)nsp;
  (void)sync;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h2 = lane >> 5, ql = lane & 31;
  uint4 pend[8];  // PS: the previous item's gated output, not yet stored
  bf16_t* pend_op = nullptr;
  bool pend_valid = false, pend_any = false;
  int item = blockIdx.x;
  do {
  KArgs* kap = kargs;
  if constexpr (PS) asm volatile("" : "+s"(kap));
  KArgs& a = *kap;
  const int L = remap_xcd(item, PS ? nitems : (int)gridDim.x);
  const int qb = L % nqb;
  // rows fastest: each XCD's contiguous block range then covers every row type (cond /
  // uncond-text / uncond-speaker rows have different key counts), and the CFG rows that share
  // one text/speaker K/V copy land on the same XCD
  const int Lr = SP ? L / (nqb * nsp) : L / nqb;
  const int sp = SP ? (L / nqb) % nsp : 0;
  const int row = Lr % a.rows;
  const int head = Lr / a.rows;
  const int q0 = qb * QB;
  const int qi = q0 + w * 32 + ql;
  const int qc = min(qi, a.n_q - 1);

  const bf16_t* qp = (const bf16_t*)a.q + ECHO_QROW(a, row) * a.q_ld_batch + (int64_t)qc * a.q_ld_tok + head * 128;
  bf16x8 qf[8];
#pragma unroll
  for (int ds = 0; ds < 8; ++ds) qf[ds] = *(const bf16x8*)(qp + 16 * ds + 8 * h2);
  // consume Q here so hipcc waits for it once, not inside the tile loop (where its counted
  // waits would land on the asm DMA of the next tile); PS: after the pending stores are issued
  if constexpr (!PS) {
#pragma unroll
    for (int ds = 0; ds < 8; ++ds) asm volatile("" ::"v"(qf[ds]));
  }

  // flat list of 64-key tiles over the (up to 4) segments; per-segment fields are kept in
  // named scalars (no runtime-indexed arrays: those go to scratch)
  ECHO_SEG_TABLE()

  ECHO_CURSOR_ADVANCE()
  Cursor dmc{-1, 0, 0, 0, 0, 0, nullptr, nullptr};  // DMA / load side
  Cursor cpc{-1, 0, 0, 0, 0, 0, nullptr, nullptr};  // compute side
  if constexpr (SP) {
    // this split's tile range of the flat list (scalar cursor walk; <= ~20 tiles)
    const int tb = sp * ntiles / nsp, te = (sp + 1) * ntiles / nsp;
    for (int i = 0; i < tb; ++i) { advance(dmc); advance(cpc); }
    ntiles = te - tb;
  }

  // DMA of the next tile (dmc) into buffer `buf`: 64 rows x 256 B for K and V = 32
  // wave-instructions of 1 KiB (4 rows each); lane-linear LDS image, XOR swizzle applied on the
  // source chunk; rows past the segment's valid length are clamped to its last row.
  const int dr = lane >> 4, dp = lane & 15;
  auto dma_tile = [&](int buf) __attribute__((always_inline)) {
    advance(dmc);
    const int last = dmc.kend - 1 - dmc.t0;
    const bf16_t* kbase = dmc.kb + (int64_t)dmc.t0 * dmc.ld;
    const bf16_t* vbase = dmc.vb + (int64_t)dmc.t0 * dmc.ld;
#pragma unroll
    for (int i = 0; i < DPT; ++i) {
      const int r = (i * NW + w) * 4 + dr;  // tile row 0..63 written by this lane
      const uint32_t voff = (uint32_t)(min(r, last) * dmc.ld + ((dp ^ swz(r)) * 8)) * 2u;
      const int dst = ((i * NW + w) * 4) * 128;
      const uint32_t kdst = __builtin_amdgcn_readfirstlane(lds_addr_of(lds + (buf * 2) * KTT * 128 + dst));
      const uint32_t vdst = __builtin_amdgcn_readfirstlane(lds_addr_of(lds + (buf * 2 + 1) * KTT * 128 + dst));
      glds16s(kbase, voff, kdst);
      glds16s(vbase, voff, vdst);
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

  // register staging: thread t moves 16-B chunks c = t + i*64*NW (row c>>4, chunk c&15) of K and V
  u32x4 kreg[DPT], vreg[DPT];
  auto load_tile = [&]() {
    advance(dmc);
#pragma unroll
    for (int i = 0; i < DPT; ++i) {
      const int c = tid + i * 64 * NW;
      const int64_t tok = dmc.t0 + min(c >> 4, dmc.kend - 1 - dmc.t0);
      kreg[i] = *(const u32x4*)(dmc.kb + tok * dmc.ld + (c & 15) * 8);
      vreg[i] = *(const u32x4*)(dmc.vb + tok * dmc.ld + (c & 15) * 8);
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int i = 0; i < DPT; ++i) {
      const int c = tid + i * 64 * NW;
      const int r = c >> 4;
      const int off = r * 128 + (((c & 15) ^ swz(r)) * 8);
      *(u32x4*)(lds + (buf * 2) * KTT * 128 + off) = kreg[i];
      *(u32x4*)(lds + (buf * 2 + 1) * KTT * 128 + off) = vreg[i];
    }
  };

  if constexpr (ST == 0) {
    if (ntiles > 0) { load_tile(); store_tile(0); }
    if (ntiles > 1) load_tile();
  } else {
    // prologue: tiles 0 .. ST-2 in flight, wait for tile 0
#pragma unroll
    for (int p = 0; p < ST - 1; ++p)
      if (p < ntiles) dma_tile(p);
    if (ST == 3 && ntiles > 1) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * DPT) : "memory");
    } else if (PS && pend_any) {
      // the previous item's 8 stores go behind Q + tile 0 and stay in flight
      asm volatile("" ::: "memory");
      attn_write_out(pend, pend_op, h2, pend_valid);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  if constexpr (PS) {
#pragma unroll
    for (int ds = 0; ds < 8; ++ds) asm volatile("" ::"v"(qf[ds]));
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();  // raw: __syncthreads' release fence would wait for the stores
  } else {
    __syncthreads();
  }

  const uint64_t ts1 = (ABL & 128) ? rt_now() : 0;
  int cur = 0;
  if (ABL & 64) ntiles = 0;
  uint64_t* ph = ((ABL & 512) && blockIdx.x == 0) ? g_attn_stamps + (int64_t)gridDim.x * 6 + w * 64 * 6 : nullptr;
  // one tile; `cur` (the LDS buffer of tile ti) is a literal in the 2-buffer schedules, so every
  // fragment address is a per-lane base + an immediate offset (no per-tile address arithmetic)
  auto tile_body = [&](int ti, int cur) __attribute__((always_inline)) {
    if ((ABL & 512) && ph && ti < 64) phase_stamp(ph + ti * 6 + 0);
    if constexpr (ST == 0) {
      // buffer cur^1 held tile ti-1: every wave passed the barrier after reading it
      if (ti + 1 < ntiles && !(ABL & 1)) store_tile(cur ^ 1);
      if (ti + 2 < ntiles && !(ABL & 1)) load_tile();
    } else {
      // tile ti+ST-1 into the stage tile ti-1 used (all waves passed the barrier after reading it)
      if (ti + ST - 1 < ntiles && !(ABL & 1)) dma_tile(cur == 0 ? ST - 1 : cur - 1);
    }
    const bf16_t* Ks = lds + (cur * 2) * KTT * 128;
    const bf16_t* Vs = Ks + KTT * 128;
    advance(cpc);
    const int t0 = cpc.t0, kend = cpc.kend;
    const bool full = (t0 + KTT <= kend) && !cpc.causal;

    // ---- S^T = K . Q^T for two 32-key sub-tiles
    f32x16 st[NKK];
    if (ABL & 256) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) {
#pragma unroll
      for (int r = 0; r < 16; ++r) st[kk][r] = 0.f;
      const int kr_ = kk * 32 + ql;
      if (ABL & 8) {
        for (int r = 0; r < 16; ++r) st[kk][r] = bf2f(qf[r & 7][r >> 3]);
        continue;
      }
#pragma unroll
      for (int ds = 0; ds < 8; ++ds) {
        const int c = 2 * ds + h2;
        const bf16x8 kf = *(const bf16x8*)(Ks + kr_ * 128 + ((c ^ swz(kr_)) * 8));
        st[kk] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ds], st[kk], 0, 0, 0);
      }
    }
    if (!(ABL & 8)) {
      // K fragment reads run 4 MFMAs ahead (hipcc otherwise waits on each read right before its
      // MFMA: 16 serialised LDS latencies, ≈2.7k cycles per tile measured with ablation 512)
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 2);
#pragma unroll
      for (int i = 0; i < 8 * NKK; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 2);
        if (i + 4 < 8 * NKK) __builtin_amdgcn_sched_group_barrier(0x100, 1, 2);
      }
    }
    if (ABL & 256) __builtin_amdgcn_s_setprio(0);
    // ---- mask (partial tiles only), online softmax (lane = query, registers = keys).
    // The running max is kept on RAW scores (scale > 0 preserves the argmax); one FMA per score
    // forms the exp2 argument s*c - m*c; raw v_exp_f32 (results < 2^-126 flush to 0).
    if ((ABL & 512) && ph && ti < 64) {  // a VALU read of the last QK result waits for the MFMA chain
      float dmy;
      asm volatile("v_mov_b32 %0, %1" : "=v"(dmy) : "v"(st[NKK - 1][15]));
      phase_stamp(ph + ti * 6 + 1);
    }
    float mx = -INFINITY;
    if (!(ABL & 2)) {
    if (!full && cpc.causal) {
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = t0 + kk * 32 + (r & 3) + 8 * (r >> 2) + 4 * h2;
          const bool ok = key < kend && (!cpc.causal || key <= qi);
          st[kk][r] = ok ? st[kk][r] : -INFINITY;
        }
    } else if (!full) {
      // prefix mask of a non-causal segment: key t0 + c + 4*h2 is visible iff 4*h2 < (kend - t0) - c,
      // one compare of a per-lane constant with a scalar per score
      const int lim = kend - t0, hb = 4 * h2;
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int c = kk * 32 + (r & 3) + 8 * (r >> 2);
          st[kk][r] = hb < lim - c ? st[kk][r] : -INFINITY;
        }
    }
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) {
      // v_max3 chain: hipcc's fmaxf first canonicalises every MFMA output (one v_max each)
      float m = max3_f(st[kk][0], st[kk][1], st[kk][2]);
#pragma unroll
      for (int r = 3; r < 15; r += 2) m = max3_f(m, st[kk][r], st[kk][r + 1]);
      mx = max3_f(mx, m, st[kk][15]);
    }
    mx = halves_max(mx);
    // deferred running max (cdna_hip_programming.md T13): the max moves only when some lane's
    // tile max exceeds it by more than 8 in exp2 units, so P <= 2^8 (fp32 O and l have the
    // range, a bf16 P the same relative precision) and the O rescale runs on a few tiles instead
    // of nearly every tile; it is applied before this tile's P is formed (textbook order)
    if (__any(m_run == -INFINITY || (mx - m_run) * sl2 > 8.0f)) {
      const float m_new = fmaxf(m_run, mx);
      const float alpha =
          __builtin_amdgcn_exp2f(__builtin_fmaf(m_run, sl2, m_new == -INFINITY ? 0.f : -m_new * sl2));
      l_run *= alpha;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
      m_run = m_new;
    }
    const float msc = m_run == -INFINITY ? 0.f : -m_run * sl2;
    float psum = 0.f;
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(st[kk][r], sl2, msc));
        st[kk][r] = pv;
        psum += pv;
      }
    l_run += psum;
    }
    if ((ABL & 512) && ph && ti < 64) phase_stamp(ph + ti * 6 + 2);

    if (ABL & 256) __builtin_amdgcn_s_setprio(1);
    // ---- O^T += V^T . P  (P from the accumulators, V^T by transposed LDS reads)
#pragma unroll
    for (int kk = 0; kk < ((ABL & 4) ? 0 : NKK); ++kk)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        bf16x8 pf;
        if (ABL & 32) {
          pf = qf[kk * 2 + s2];
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) pf[j] = (__bf16)st[kk][8 * s2 + j];
        }
        const int key0 = kk * 32 + 16 * s2 + 4 * h2;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const int ch = 4 * dt + 2 * (g & 1) + (p4 >> 1);
          const int r0 = key0 + q4, r1 = key0 + 8 + q4;
          typedef __attribute__((ext_vector_type(8))) short s16x8;
          s16x8 v8;
          if (ABL & 16) {
            v8 = __builtin_bit_cast(s16x8, qf[4 + dt]);
          } else {
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(Vs + r0 * 128 + ((ch ^ swz(r0)) * 8) + (p4 & 1) * 4));
          const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(Vs + r1 * 128 + ((ch ^ swz(r1)) * 8) + (p4 & 1) * 4));
          v8 = s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          }
          o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, v8), pf, o[dt], 0, 0, 0);
        }
      }
    if (!(ABL & 4) && !(ABL & 16)) {
      // V^T transposed reads (2 per MFMA) run 2 MFMAs ahead
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 3);
#pragma unroll
      for (int i = 0; i < 8 * NKK; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 3);
        if (i + 2 < 8 * NKK) __builtin_amdgcn_sched_group_barrier(0x100, 2, 3);
      }
    }
    if (ABL & 256) __builtin_amdgcn_s_setprio(0);
    if ((ABL & 512) && ph && ti < 64) phase_stamp(ph + ti * 6 + 3);
    if constexpr (ST == 0) {
      __syncthreads();  // tile ti+1 was written at the top of this tile
    } else {
      // tile ti+1 landed (this wave's share; later tiles may stay in flight) ... and everyone's
      if (ST == 3 && ti + 2 < ntiles && !(ABL & 1)) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * DPT) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if ((ABL & 512) && ph && ti < 64) phase_stamp(ph + ti * 6 + 4);
      __syncthreads();
      if ((ABL & 512) && ph && ti < 64) phase_stamp(ph + ti * 6 + 5);
    }
  };
  if constexpr (ST == 3) {
    for (int ti = 0; ti < ntiles; ++ti) {
      tile_body(ti, cur);
      cur = cur == ST - 1 ? 0 : cur + 1;
    }
  } else {
    for (int ti = 0; ti < ntiles; ti += 2) {
      tile_body(ti, 0);
      if (ti + 1 >= ntiles) break;
      tile_body(ti + 1, 1);
    }
  }

  const uint64_t ts2 = (ABL & 128) ? rt_now() : 0;
  if ((ABL & 128) && threadIdx.x == 0) {
    uint64_t* st = g_attn_stamps + (int64_t)blockIdx.x * 6;
    st[0] = ts0; st[1] = ts1; st[2] = ts2; st[4] = ntiles; st[5] = blockIdx.x & 7;
  }
  // ---- epilogue: normalise, round, gate, store (widened 16-B accesses, attn_store_out)
  const float lt = halves_sum(l_run);
  const float inv = 1.0f / lt;
  {
    const bool valid = qi < a.n_q;
    bf16_t* op = (bf16_t*)a.out + row * a.o_ld_batch + (int64_t)qc * a.o_ld_tok + head * 128;
    const bf16_t* gp = a.gate ? (const bf16_t*)a.gate + ECHO_QROW(a, row) * a.g_ld_batch + (int64_t)qc * a.g_ld_tok + head * 128
                              : nullptr;
    if constexpr (SP) {
      // partial O at chunk c = d / 4 (32 chunks of 4 floats), laid out [chunk][query] so the 32
      // lanes of a half-wave store 512 contiguous bytes per instruction
      const int64_t it = ((int64_t)sp * a.rows + row) * a.heads + head;
      const int64_t ml_off = (int64_t)nsp * a.rows * a.heads * 128 * a.n_q;  // (m, l) pairs after every O
      const __amdgpu_buffer_rsrc_t wsr = rsrc_of(ws, 0xFFFFFFF0u);  // SP = 2: the O partials' byte offsets
      (void)wsr;
      if (valid) {
        float* wo = ws + it * 128 * a.n_q;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
          for (int rg = 0; rg < 4; ++rg) {
            const int c = dt * 8 + 2 * rg + h2;
            const float4 v = make_float4(o[dt][4 * rg], o[dt][4 * rg + 1], o[dt][4 * rg + 2], o[dt][4 * rg + 3]);
            if constexpr (SP == 2) {
              st_sc1_b128(wsr, (uint32_t)(((it * 128 + (int64_t)c * 4) * a.n_q + (int64_t)qi * 4) * 4), v);
            } else {
              *(float4*)(wo + ((int64_t)c * a.n_q + qi) * 4) = v;
            }
          }
        if (h2 == 0) {
          float* wml = ws + ml_off + (it * a.n_q + qi) * 2;
          const float2 v = make_float2(m_run == -INFINITY ? -INFINITY : m_run * sl2, lt);
          if constexpr (SP == 2) st_sc1_b64(wml, v); else *(float2*)wml = v;
        }
      }
      (void)inv;
      if constexpr (SP == 2) {
        // publish: every storing wave drains its write-through stores, then one arrival per workgroup
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const int rh = row * a.heads + head;
        uint32_t* cnt = sync + SYNC_CNT0 + 2 * ((int64_t)rh * nqb + qb);  // [arrivals, departures] of this item
        if (tid == 0) sync_arrive_wait(sync, cnt, (uint32_t)nsp);
        __syncthreads();
        // this split's share of the item's QB x 16 (query, 8-column) units, 16 queries x 16 chunks per pass
        constexpr int U = QB * 16;
        const int u0 = sp * U / nsp, u1 = (sp + 1) * U / nsp;
        for (int u = u0 + tid; u < u1; u += 64 * NW) {
          const int qq = q0 + (u & 15) + 16 * (u >> 8), c8 = (u >> 4) & 15;
          if (qq < a.n_q) attn_combine_unit(a, ws, nsp, rh, qq, c8);
        }
        if (tid == 0) sync_depart(cnt, (uint32_t)nsp);
      }
    } else if constexpr (PS) {
      // (the persistent form keeps the per-lane epilogue: the row form's LDS transposition needs a
      // barrier before the next item's DMA and spills around the item loop — 179 vs 154 us, R = 16)
      attn_pack_out(o, inv, h2, valid, gp, pend);
      pend_op = op;
      pend_valid = valid;
      pend_any = __any(valid);
    } else if constexpr ((ABL & 2048) != 0) {
      attn_store_out(o, inv, qi, h2, valid, op, gp);  // ablation 2048: the per-lane (32 rows x 32 B) form
    } else {
      // row-layout epilogue: the wave's 32 x 128 tile is transposed through its own 8 KB of LDS
      // (free: every wave passed the last tile's barrier after its final LDS reads, and no DMA is
      // in flight), so every gate load and output store instruction covers 4 whole 256-B rows
      // instead of 32 rows x 32 B (cdna_hip_programming.md attention rules: "O staged through LDS
      // and stored as whole rows"). Lane (rl, cc) = (lane / 16, lane % 16) holds rows 4*pk + rl,
      // columns 8*cc .. 8*cc + 7. Rows past n_q: gate loads and stores fall outside the buffer ranges
      // (loads return 0, stores are dropped).
      const int nv = a.n_q - (q0 + w * 32);  // wave-uniform
      if (nv > 0) {
        const int rl = lane >> 4, cc = lane & 15;
        const int64_t qw = q0 + w * 32;
        uint4 g4[8];
        auto load_gates = [&]() __attribute__((always_inline)) {
          // rows past n_q read as 0 (outside the buffer range); their outputs are dropped below
          const __amdgpu_buffer_rsrc_t gr =
              attn_rsrc((const bf16_t*)a.gate + ECHO_QROW(a, row) * a.g_ld_batch + qw * a.g_ld_tok + head * 128,
                        (uint32_t)(((int64_t)(min(nv, 32) - 1) * a.g_ld_tok + 128) * 2));
          const uint32_t glo = (uint32_t)((rl * a.g_ld_tok + cc * 8) * 2), gst = (uint32_t)(a.g_ld_tok * 8);
#pragma unroll
          for (int pk = 0; pk < 8; ++pk) g4[pk] = attn_bload(gr, glo + pk * gst);
        };
        if (gp) load_gates();  // in flight during the transposition
        uint4 v4[8];
        attn_pack_o(o, inv, v4);
        bf16_t* sw = lds + w * 32 * 128;
#pragma unroll
        for (int pk = 0; pk < 8; ++pk) *(uint4*)(sw + ql * 128 + (((2 * pk + h2) ^ (ql & 15)) * 8)) = v4[pk];
#pragma unroll
        for (int pk = 0; pk < 8; ++pk) {
          const int r = pk * 4 + rl;
          v4[pk] = *(const uint4*)(sw + r * 128 + ((cc ^ (r & 15)) * 8));
        }
        if (gp) attn_gate(v4, g4);
        attn_store_rows(v4, (bf16_t*)a.out + row * a.o_ld_batch + qw * a.o_ld_tok + head * 128, nv, a.o_ld_tok, lane);
      }
    }
  }
  if ((ABL & 128) && threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    g_attn_stamps[(int64_t)blockIdx.x * 6 + 3] = rt_now();
  }
  if constexpr (!PS) break;
  item += gridDim.x;
  } while (item < nitems);  // item loop
  if constexpr (PS) {
    if (pend_any) attn_write_out(pend, pend_op, h2, pend_valid);
  }
}

// ----------------------------------------------------------------------------- asm-owned pipeline
// attn_pl_kernel: attn_bf16_kernel<0, 4, 2>'s math in the same order (bitwise-equal output), with the
// tile loop software-pipelined by hand (cdna_hip_programming.md T15) over registers the compiler does
// not own: amdgpu_num_vgpr(96) caps hipcc at v0..v95 and the tile bodies (attn_pl.inc, generated by
// tools/gen_attn_pl.py) keep O, two score buffers and the K / V^T fragment rings in v96..v255. Per tile t:
//   X(t): softmax of tile t (fma, exp2, row sum, bf16 pack of P in place)  ||  QK of tile t+1 (16 MFMA)
//   Y(t): PV of tile t (16 MFMA)  ||  prefix mask (partial tiles) + row max of tile t+1
// then the deferred-max decision for t+1 (rare O rescale), the wave's DMA wait and ONE barrier.
// hipcc's own allocation of the production kernel copies O (32 v_mov_b64) and the scores (32 v_mov_b32)
// across the rescale / mask branch joins on every tile; here no loop state crosses a compiler join.
// K and V have separate 2-slot rings ([K0 | K1 | V0 | V1], 16 KB each): K(t+2) and V(t+1) are issued
// at the top of iteration t into the slots that K(t) and V(t-1) left (read before the previous
// barrier) and waited for at its end. Non-causal segments only (decoder attention); the host routes
// causal launches (speaker / latent encoders) to attn_bf16_kernel.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
#include "attn_pl.inc"

// ABL (timing ablations, variants 12-16; results wrong): 1 no loop DMA, 2 no X body, 4 no Y body,
// 8 no end-of-tile wait + barrier, 16 no tile loop.
// NW: waves per workgroup (4: 128 queries, two workgroups per CU; 8: 256 queries, one workgroup per CU, each
// K/V tile staged once for twice the queries — variant 20, slower: DESIGN.md §3).
// Measured and removed (round 5 prune; numbers in DESIGN.md §3 / §7): K / V rings of 3 + 2, 3 + 3, 4 + 4 and
// 2 + 3 slots with counted waits across the barrier; V(t+1)'s DMA between the X and Y bodies; CFG-adjacent
// and longest-first block orders; the split-KV form of this kernel (2-4 % slower than attn_bf16_kernel's).
template <int ABL, int NW = 4>
__global__ void __launch_bounds__(64 * NW, NW == 8 ? 1 : 2) __attribute__((amdgpu_num_vgpr(96)))
    attn_pl_kernel(EchoAttnArgs a_arg) {
  constexpr int QB = 32 * NW, DPT = 16 / NW, KTT = KT, NK = 2, NV = 2;
  __shared__ __attribute__((aligned(16))) bf16_t lds[(NK + NV) * KT * 128];  // K slots | V slots

  using KArgs = const __attribute__((address_space(4))) EchoAttnArgs;
  KArgs& a = *(KArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  (void)a_arg;
  const int nqb = (a.n_q + QB - 1) / QB;
  const int L = remap_xcd(blockIdx.x, gridDim.x);
  const int qb = L % nqb;
  const int Lr = L / nqb;  // rows fastest (see attn_bf16_kernel)
  const int row = Lr % a.rows, head = Lr / a.rows;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h2 = lane >> 5, ql = lane & 31;
  const int q0 = qb * QB;
  const int qc = min(q0 + w * 32 + ql, a.n_q - 1);

  const bf16_t* qp = (const bf16_t*)a.q + ECHO_QROW(a, row) * a.q_ld_batch + (int64_t)qc * a.q_ld_tok + head * 128;
  bf16x8 qf[8];
#pragma unroll
  for (int ds = 0; ds < 8; ++ds) qf[ds] = *(const bf16x8*)(qp + 16 * ds + 8 * h2);

  ECHO_SEG_TABLE()
  ECHO_CURSOR_ADVANCE()
  Cursor kc{-1, 0, 0, 0, 0, 0, nullptr, nullptr};  // K DMA (NK - 1 tiles ahead of the QK)
  Cursor vc{-1, 0, 0, 0, 0, 0, nullptr, nullptr};  // V DMA (NV - 1 tiles ahead of the PV)
  Cursor mc{-1, 0, 0, 0, 0, 0, nullptr, nullptr};  // the tile whose scores are masked / maxed

  const int dr = lane >> 4, dp = lane & 15;
  // one tile's share of this wave (DPT pieces) into slot `slot` of the K (part 0) or V (part 1) ring
  auto dma_part = [&](Cursor& c, int part, int slot) __attribute__((always_inline)) {
    advance(c);
    const int last = c.kend - 1 - c.t0;
    const bf16_t* base = (part ? c.vb : c.kb) + (int64_t)c.t0 * c.ld;
#pragma unroll
    for (int i = 0; i < DPT; ++i) {
      const int r = (i * NW + w) * 4 + dr;
      const uint32_t voff = (uint32_t)(min(r, last) * c.ld + ((dp ^ swz(r)) * 8)) * 2u;
      const uint32_t dst = __builtin_amdgcn_readfirstlane(
          lds_addr_of(lds + (part * NK + slot) * KT * 128 + ((i * NW + w) * 4) * 128));
      glds16s(base, voff, dst);
    }
  };

  // per-lane LDS byte addresses of the fragment reads (slot / sub-tile offsets are immediates):
  // K row kk*32 + ql, chunk (2 ds + h2) ^ swz; V^T rows r0 = 4 h2 + q4 (+ 8) of chunk 4 dt + ...
  const uint32_t lbase = lds_addr_of(lds);
  uint32_t ka[8], va[8];
#pragma unroll
  for (int ds = 0; ds < 8; ++ds) ka[ds] = lbase + (uint32_t)(ql * 128 + (((2 * ds + h2) ^ swz(ql)) * 8)) * 2u;
  {
    const int g = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
    const int r0 = 4 * h2 + q4, r1 = r0 + 8;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int ch = 4 * dt + 2 * (g & 1) + (p4 >> 1);
      va[2 * dt] = lbase + (uint32_t)NK * KT * 128 * 2 + (uint32_t)(r0 * 128 + ((ch ^ swz(r0)) * 8) + (p4 & 1) * 4) * 2u;
      va[2 * dt + 1] = lbase + (uint32_t)NK * KT * 128 * 2 + (uint32_t)(r1 * 128 + ((ch ^ swz(r1)) * 8) + (p4 & 1) * 4) * 2u;
    }
  }

  float m_run = -INFINITY, l_run = 0.f;
  const float sl2 = a.scale * 1.4426950408889634f;
  const int hb = 4 * h2;
  // waves whose 32 queries all lie past n_q (the last q block of a 160-query blockwise launch has one
  // active wave of four) issue their DMA share and take the barriers but skip every tile body (a scalar
  // branch around opaque asm: the active waves' code is unchanged)
  const bool wact = q0 + w * 32 < a.n_q;
  // prefix mask of the next tile (cursor mc advanced to it) if it is partial
  auto mask_tile = [&](auto par) __attribute__((always_inline)) {
    constexpr int P = decltype(par)::value;
    advance(mc);
    const int lim = mc.kend - mc.t0;
    if (lim < KTT) {
      if constexpr (P == 0) pl_mask_0(lim, hb); else pl_mask_1(lim, hb);
    }
  };
  // the deferred running-max decision of attn_bf16_kernel for a tile with lane max mx
  auto decide = [&](float mx) __attribute__((always_inline)) {
    mx = halves_max(mx);
    if (__any(m_run == -INFINITY || (mx - m_run) * sl2 > 8.0f)) {
      const float m_new = fmaxf(m_run, mx);
      const float alpha =
          __builtin_amdgcn_exp2f(__builtin_fmaf(m_run, sl2, m_new == -INFINITY ? 0.f : -m_new * sl2));
      l_run *= alpha;
      pl_rescale(alpha);
      m_run = m_new;
    }
  };

  pl_zero_o();
  // prologue: K(0), V(0), K(1) — needed before tile 0's loop iteration; scores, mask and max of tile 0
  if (ntiles > 0) { dma_part(kc, 0, 0); dma_part(vc, 1, 0); }
  if (ntiles > 1) dma_part(kc, 0, 1);
  // Q and the prologue DMA in flight together: one wait (hipcc's vmcnt(0) for Q covers the DMA issued after it)
#pragma unroll
  for (int ds = 0; ds < 8; ++ds) asm volatile("" ::"v"(qf[ds]));
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  if (ntiles > 0) {
    if (wact) {
      pl_qk_cs<0, 0>(qf, ka);
      mask_tile(std::integral_constant<int, 0>{});
      float mx, ma;
      pl_max_0(mx, ma);
      decide(mx);
    } else {
      advance(mc);
    }
  }
  asm volatile("s_barrier" ::: "memory");  // every wave's K(0) reads are done: slot 0 takes K(NK)

  auto iter = [&](int t, auto unr) __attribute__((always_inline)) {
    constexpr int P = decltype(unr)::value;  // t & 1: the score buffer of tile t
    constexpr int KS = 1 - P;                // K slot of tile t + 1 (its QK runs in X(t))
    constexpr int VS = P;                    // V slot of tile t (its PV runs in Y(t))
    if (t + 2 < ntiles && !(ABL & 1)) dma_part(kc, 0, P);      // K(t+2) -> K slot t & 1 (K(t) was read in X(t-1))
    if (t + 1 < ntiles && !(ABL & 1)) dma_part(vc, 1, 1 - P);  // V(t+1) -> V slot (t+1) & 1 (V(t-1) read in Y(t-1))
    const float msc = m_run == -INFINITY ? 0.f : -m_run * sl2;
    float ps;
    if (!wact) {
      if (t + 1 < ntiles) advance(mc);
    } else if (t + 1 < ntiles) {
      ps = 0.f;
      if constexpr (!(ABL & 2)) pl_x_cs<P, KS>(qf, ka, sl2, msc, ps);
      l_run += ps;
      mask_tile(std::integral_constant<int, 1 - P>{});
      float mx = 0.f, ma;
      if constexpr (!(ABL & 4)) pl_y_cs<P, VS>(va, mx, ma);
      decide(mx);
    } else {
      if constexpr (P == 0) pl_xl_0(sl2, msc, ps); else pl_xl_1(sl2, msc, ps);
      l_run += ps;
      pl_yl_cs<P, VS>(va);
    }
    // K(t+2) and V(t+1) must have landed (every wave's share, then the barrier)
    if constexpr (!(ABL & 8)) asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  };
  if (ABL & 16) ntiles = 0;
  for (int t = 0; t < ntiles; t += 2) {
    iter(t, std::integral_constant<int, 0>{});
    if (t + 1 >= ntiles) break;
    iter(t + 1, std::integral_constant<int, 1>{});
  }

  // ---- epilogue (attn_bf16_kernel's row layout): normalise, round, transpose through LDS, gate, store
  const float lt = halves_sum(l_run);
  const float inv = 1.0f / lt;
  const int nv = a.n_q - (q0 + w * 32);  // wave-uniform
  if (nv > 0) {
    uint4 v4[8];
    auto pack_dt = [&](const float (&od)[16], int dt) __attribute__((always_inline)) {
      uint32_t wd[4][2];
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        wd[rg][0] = pack2bf(rbf(od[4 * rg + 0] * inv), rbf(od[4 * rg + 1] * inv));
        wd[rg][1] = pack2bf(rbf(od[4 * rg + 2] * inv), rbf(od[4 * rg + 3] * inv));
      }
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const auto x = __builtin_amdgcn_permlane32_swap(wd[2 * k][0], wd[2 * k + 1][0], false, false);
        const auto y = __builtin_amdgcn_permlane32_swap(wd[2 * k][1], wd[2 * k + 1][1], false, false);
        v4[2 * dt + k] = make_uint4(x[0], y[0], x[1], y[1]);
      }
    };
    const int rl = lane >> 4, cc = lane & 15;
    const int64_t qw = q0 + w * 32;
    uint4 g4[8];
    if (a.gate) {  // in flight during the pack and the transposition
      const __amdgpu_buffer_rsrc_t gr =
          attn_rsrc((const bf16_t*)a.gate + ECHO_QROW(a, row) * a.g_ld_batch + qw * a.g_ld_tok + head * 128,
                    (uint32_t)(((int64_t)(min(nv, 32) - 1) * a.g_ld_tok + 128) * 2));
      const uint32_t glo = (uint32_t)((rl * a.g_ld_tok + cc * 8) * 2), gst = (uint32_t)(a.g_ld_tok * 8);
#pragma unroll
      for (int pk = 0; pk < 8; ++pk) g4[pk] = attn_bload(gr, glo + pk * gst);
    }
    {
      float od[16];
      pl_get_o_0(od); pack_dt(od, 0);
      pl_get_o_1(od); pack_dt(od, 1);
      pl_get_o_2(od); pack_dt(od, 2);
      pl_get_o_3(od); pack_dt(od, 3);
    }
    bf16_t* sw = lds + w * 32 * 128;  // free: no DMA in flight, every wave passed the last barrier
#pragma unroll
    for (int pk = 0; pk < 8; ++pk) *(uint4*)(sw + ql * 128 + (((2 * pk + h2) ^ (ql & 15)) * 8)) = v4[pk];
#pragma unroll
    for (int pk = 0; pk < 8; ++pk) {
      const int r = pk * 4 + rl;
      v4[pk] = *(const uint4*)(sw + r * 128 + ((cc ^ (r & 15)) * 8));
    }
    if (a.gate) attn_gate(v4, g4);
    attn_store_rows(v4, (bf16_t*)a.out + row * a.o_ld_batch + qw * a.o_ld_tok + head * 128, nv, a.o_ld_tok, lane);
  }
}

// ----------------------------------------------------------------------------- one wave per SIMD, 64 rows
// A wave-uniform 64-bit value moved into SGPRs. readfirstlane returns int: each half goes through uint32_t before
// the widening, or a low word with bit 31 set sign-extends over the high word (a wild tile address).
__device__ __forceinline__ uint64_t uniform_u64(uint64_t x) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32));
  return ((uint64_t)hi << 32) | (uint64_t)lo;
}

// attn_w64_kernel: the structure of cdna_hip_programming.md's "4-wave, one-wave-per-SIMD" attention: each wave
// owns 64 queries (q blocks A = qw .. qw+31, B = qw+32 .. qw+63 of the item's 64 NW) and the whole 512-register
// file (map: tools/gen_attn_w64.py), so every K / V^T fragment read from LDS feeds two MFMAs. NW = 4: one
// 256-query workgroup per CU (each K / V tile staged once for 256 queries: half attn_pl_kernel's LDS-DMA per
// query); NW = 2: two 128-query workgroups per CU. 80 KiB of LDS per workgroup: a 3-slot K ring, a 2-slot V ring. The tile bodies (attn_w64.inc) software-pipeline
// each wave on its own: X(t) = softmax(t) || QK(t+1) with the DMA of V(t+1) and K(t+3) in its MFMA gaps,
// Y(t) = PV(t) || row max(t+1). Per 32-query block the math, its order and every rounding are
// attn_bf16_kernel<0, 4, 2>'s (the deferred-max decision is taken per block, as there): bitwise equal.
// Non-causal launches only. ABL (timing ablations, results wrong): 1 = no DMA in the tile loop, 8 = no end-of-tile
// DMA wait (the barrier stays), 16 = no tile loop.
// Measured slower than attn_pl_kernel: diagnostics build only (ECHO_DIAG=1), the product ABI refuses it.
#ifdef ECHO_DIAG
#include "attn_w64.inc"

template <int ABL, int NW>
__global__ void __launch_bounds__(64 * NW, 1) __attribute__((amdgpu_num_vgpr(128))) attn_w64_kernel(EchoAttnArgs a_arg) {
  static_assert(NW == 2 || NW == 4, "2 or 4 waves");
  using WB = std::conditional_t<NW == 2, W2, W4>;
  constexpr int QB = 64 * NW, KTT = KT;
  __shared__ __attribute__((aligned(16))) bf16_t lds[5 * KT * 128];  // K slots 0-2 | V slots 0-1 (80 KiB)
  using KArgs = const __attribute__((address_space(4))) EchoAttnArgs;
  KArgs& a = *(KArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  (void)a_arg;
  const int nqb = (a.n_q + QB - 1) / QB;
  const int L = remap_xcd(blockIdx.x, gridDim.x);
  const int qb = L % nqb;
  const int Lr = L / nqb;  // rows fastest (see attn_bf16_kernel)
  const int row = Lr % a.rows, head = Lr / a.rows;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h2 = lane >> 5, ql = lane & 31;
  const int q0 = qb * QB;
  const int qw = q0 + 64 * w;  // q block A = qw .. qw + 31, B = qw + 32 .. qw + 63 (rows past n_q: clamped loads)
  {
    const int qca = min(qw + ql, a.n_q - 1), qcb = min(qw + 32 + ql, a.n_q - 1);
    const bf16_t* qbase = (const bf16_t*)a.q + ECHO_QROW(a, row) * a.q_ld_batch + head * 128;
    WB::load_q((uint32_t)(((int64_t)qca * a.q_ld_tok + 8 * h2) * 2), (uint32_t)(((int64_t)qcb * a.q_ld_tok + 8 * h2) * 2),
             qbase);
  }

  ECHO_SEG_TABLE()
  ECHO_CURSOR_ADVANCE()
  Cursor kc{-1, 0, 0, 0, 0, 0, nullptr, nullptr};  // K DMA (3 tiles ahead of the QK)
  Cursor vc{-1, 0, 0, 0, 0, 0, nullptr, nullptr};  // V DMA (1 tile ahead of the PV)
  Cursor mc{-1, 0, 0, 0, 0, 0, nullptr, nullptr};  // the tile whose scores are masked / maxed

  // LDS-DMA lane terms: piece i of the wave covers tile rows 8 i + r0 (r0 = 4 w + lane / 16), its lane reads the
  // source chunk (lane % 16) ^ swz(row) (cx0 / cx1: even / odd i), into the wave's 1 KiB of the piece's 2 KiB
  const int dr = lane >> 4, dp = lane & 15;
  const uint32_t r0 = (uint32_t)(4 * w + dr);
  const uint32_t cx0 = (uint32_t)((dp ^ ((dr << 2) | w)) * 16), cx1 = (uint32_t)((dp ^ ((dr << 2) | (2 + w))) * 16);
  const uint32_t lbase = lds_addr_of(lds);
  const uint32_t lw = __builtin_amdgcn_readfirstlane(lbase + (uint32_t)w * 1024u);
  struct Dma {
    const void* base;
    uint32_t last, ld2;
  };
  auto next_dma = [&](Cursor& c, int part) __attribute__((always_inline)) {
    advance(c);
    // wave-uniform by construction; readfirstlane lets the asm's "s" operands take them when hipcc cannot prove it
    const uint64_t pb = (uint64_t)(uintptr_t)((part ? c.vb : c.kb) + (int64_t)c.t0 * c.ld);
    Dma d;
    d.base = (const void*)uniform_u64(pb);
    d.last = __builtin_amdgcn_readfirstlane((uint32_t)(c.kend - 1 - c.t0));
    d.ld2 = __builtin_amdgcn_readfirstlane((uint32_t)c.ld * 2u);
    return d;
  };

  // per-lane LDS byte addresses of the fragment reads (slot / sub-tile offsets are immediates of the bodies)
  uint32_t ka[8], va[8];
#pragma unroll
  for (int ds = 0; ds < 8; ++ds) ka[ds] = lbase + (uint32_t)(ql * 128 + (((2 * ds + h2) ^ swz(ql)) * 8)) * 2u;
  {
    const int g = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
    const int rr0 = 4 * h2 + q4, rr1 = rr0 + 8;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int ch = 4 * dt + 2 * (g & 1) + (p4 >> 1);
      va[2 * dt] = lbase + 3u * KT * 128 * 2 + (uint32_t)(rr0 * 128 + ((ch ^ swz(rr0)) * 8) + (p4 & 1) * 4) * 2u;
      va[2 * dt + 1] = lbase + 3u * KT * 128 * 2 + (uint32_t)(rr1 * 128 + ((ch ^ swz(rr1)) * 8) + (p4 & 1) * 4) * 2u;
    }
  }

  float ma_run = -INFINITY, la = 0.f, mb_run = -INFINITY, lb = 0.f;
  const float sl2 = a.scale * 1.4426950408889634f;
  const int hb = 4 * h2;
  auto mask_tile = [&](auto par) __attribute__((always_inline)) {
    constexpr int P = decltype(par)::value;
    advance(mc);
    const int lim = mc.kend - mc.t0;
    if (lim < KTT) {
      if constexpr (P == 0) WB::mask_0(lim, hb); else WB::mask_1(lim, hb);
    }
  };
  // attn_bf16_kernel's deferred running-max decision, per 32-query block
  auto decide = [&](float& m_run, float& l_run, float mx, auto blk) __attribute__((always_inline)) {
    mx = halves_max(mx);
    if (__any(m_run == -INFINITY || (mx - m_run) * sl2 > 8.0f)) {
      const float m_new = fmaxf(m_run, mx);
      const float alpha =
          __builtin_amdgcn_exp2f(__builtin_fmaf(m_run, sl2, m_new == -INFINITY ? 0.f : -m_new * sl2));
      l_run *= alpha;
      if constexpr (decltype(blk)::value == 0) WB::rescale_0(alpha); else WB::rescale_1(alpha);
      m_run = m_new;
    }
  };

  WB::zero_o();
  // prologue: K(0), V(0), K(1), K(2) after the Q loads; Q, K(0), V(0), K(1) waited (K(2)'s 16 / NW pieces may stay
  // in flight)
  if (ntiles > 0) {
    Dma d = next_dma(kc, 0);
    WB::template dma_cs<0, 0>(r0, cx0, cx1, lw, d.last, d.ld2, d.base);
    d = next_dma(vc, 1);
    WB::template dma_cs<1, 0>(r0, cx0, cx1, lw, d.last, d.ld2, d.base);
  }
  if (ntiles > 1) {
    const Dma d = next_dma(kc, 0);
    WB::template dma_cs<0, 1>(r0, cx0, cx1, lw, d.last, d.ld2, d.base);
  }
  if (ntiles > 2) {
    const Dma d = next_dma(kc, 0);
    WB::template dma_cs<0, 2>(r0, cx0, cx1, lw, d.last, d.ld2, d.base);
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(16 / NW) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  }
  if (ntiles > 0) {
    WB::qk_0_0(ka);
    mask_tile(std::integral_constant<int, 0>{});
    float mxa, mxb;
    WB::max_0(mxa, mxb);
    decide(ma_run, la, mxa, std::integral_constant<int, 0>{});
    decide(mb_run, lb, mxb, std::integral_constant<int, 1>{});
  }
  asm volatile("s_barrier" ::: "memory");  // every wave's K(0) reads are done: slot 0 takes K(3)

  auto iter = [&](int t, auto unr) __attribute__((always_inline)) {
    constexpr int U = decltype(unr)::value;  // t mod 6
    constexpr int P = U & 1;                 // score buffer of tile t (its V slot too)
    constexpr int KS = (U + 1) % 3;          // K slot of tile t + 1 (its QK runs in X(t))
    constexpr int KD = U % 3;                // K slot that takes K(t + 3) (K(t) was read in X(t - 1))
    const float msa = ma_run == -INFINITY ? 0.f : -ma_run * sl2;
    const float msb = mb_run == -INFINITY ? 0.f : -mb_run * sl2;
    float psa = 0.f, psb = 0.f;
    if (t + 1 < ntiles) {
      // X(t): V(t+1) -> V slot 1 - P (V(t-1) was read in Y(t-1))
      const Dma dv = next_dma(vc, 1);
      if constexpr ((ABL & 1) != 0) {
        if constexpr (P == 0 && KS == 0) WB::xa_0_0(ka, sl2, msa, msb, psa, psb);
        else if constexpr (P == 0 && KS == 1) WB::xa_0_1(ka, sl2, msa, msb, psa, psb);
        else if constexpr (P == 0) WB::xa_0_2(ka, sl2, msa, msb, psa, psb);
        else if constexpr (KS == 0) WB::xa_1_0(ka, sl2, msa, msb, psa, psb);
        else if constexpr (KS == 1) WB::xa_1_1(ka, sl2, msa, msb, psa, psb);
        else WB::xa_1_2(ka, sl2, msa, msb, psa, psb);
        (void)dv;
      } else {
        if constexpr (P == 0 && KS == 0) WB::x_0_0(ka, sl2, msa, msb, psa, psb, r0, cx0, cx1, lw, dv.last, dv.ld2, dv.base);
        else if constexpr (P == 0 && KS == 1) WB::x_0_1(ka, sl2, msa, msb, psa, psb, r0, cx0, cx1, lw, dv.last, dv.ld2, dv.base);
        else if constexpr (P == 0) WB::x_0_2(ka, sl2, msa, msb, psa, psb, r0, cx0, cx1, lw, dv.last, dv.ld2, dv.base);
        else if constexpr (KS == 0) WB::x_1_0(ka, sl2, msa, msb, psa, psb, r0, cx0, cx1, lw, dv.last, dv.ld2, dv.base);
        else if constexpr (KS == 1) WB::x_1_1(ka, sl2, msa, msb, psa, psb, r0, cx0, cx1, lw, dv.last, dv.ld2, dv.base);
        else WB::x_1_2(ka, sl2, msa, msb, psa, psb, r0, cx0, cx1, lw, dv.last, dv.ld2, dv.base);
      }
      mask_tile(std::integral_constant<int, 1 - P>{});
      // Y(t): K(t+3) -> K slot KD, issued last in the iteration so that it may stay in flight across the barrier
      float mxa, mxb;
      const bool kdma = t + 3 < ntiles && !(ABL & 1);
      if (kdma) {
        const Dma dk = next_dma(kc, 0);
        WB::template y_cs<P, KD>(va, sl2, msa, msb, psa, psb, mxa, mxb, r0, cx0, cx1, lw, dk.last, dk.ld2, dk.base);
      } else {
        WB::template y_cs<P, -1>(va, sl2, msa, msb, psa, psb, mxa, mxb, r0, cx0, cx1, lw, 0u, 0u, nullptr);
      }
      la += psa;
      lb += psb;
      decide(ma_run, la, mxa, std::integral_constant<int, 0>{});
      decide(mb_run, lb, mxb, std::integral_constant<int, 1>{});
      // V(t+1) and K(t+2) (issued before it) must have landed; K(t+3), issued last (16 / NW pieces), may stay in flight
      if constexpr ((ABL & 8) != 0) asm volatile("s_barrier" ::: "memory");
      else if (kdma) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(16 / NW) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    } else {
      if constexpr (P == 0) WB::xl_0(sl2, msa, msb, psa, psb); else WB::xl_1(sl2, msa, msb, psa, psb);
      if constexpr (P == 0) WB::yl_0(va, sl2, msa, msb, psa, psb); else WB::yl_1(va, sl2, msa, msb, psa, psb);
      la += psa;
      lb += psb;
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    }
  };
  if (ABL & 16) ntiles = 0;
  for (int t = 0; t < ntiles; t += 6) {
    iter(t, std::integral_constant<int, 0>{});
    if (t + 1 >= ntiles) break;
    iter(t + 1, std::integral_constant<int, 1>{});
    if (t + 2 >= ntiles) break;
    iter(t + 2, std::integral_constant<int, 2>{});
    if (t + 3 >= ntiles) break;
    iter(t + 3, std::integral_constant<int, 3>{});
    if (t + 4 >= ntiles) break;
    iter(t + 4, std::integral_constant<int, 4>{});
    if (t + 5 >= ntiles) break;
    iter(t + 5, std::integral_constant<int, 5>{});
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");  // (ablations / ntiles == 0: nothing may be in flight)

  // ---- epilogue per q block (attn_pl_kernel's row layout): normalise, round, transpose through LDS, gate, store
  auto store_block = [&](auto blk, float l_run) __attribute__((always_inline)) {
    constexpr int J = decltype(blk)::value;
    const float inv = 1.0f / halves_sum(l_run);
    const int nv = a.n_q - (qw + 32 * J);  // wave-uniform
    if (nv <= 0) return;
    uint4 v4[8];
    auto pack_dt = [&](const float (&od)[16], int dt) __attribute__((always_inline)) {
      uint32_t wd[4][2];
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        wd[rg][0] = pack2bf(rbf(od[4 * rg + 0] * inv), rbf(od[4 * rg + 1] * inv));
        wd[rg][1] = pack2bf(rbf(od[4 * rg + 2] * inv), rbf(od[4 * rg + 3] * inv));
      }
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const auto x = __builtin_amdgcn_permlane32_swap(wd[2 * k][0], wd[2 * k + 1][0], false, false);
        const auto y = __builtin_amdgcn_permlane32_swap(wd[2 * k][1], wd[2 * k + 1][1], false, false);
        v4[2 * dt + k] = make_uint4(x[0], y[0], x[1], y[1]);
      }
    };
    const int rl = lane >> 4, cc = lane & 15;
    const int64_t qv = qw + 32 * J;
    uint4 g4[8];
    if (a.gate) {  // in flight during the pack and the transposition
      const __amdgpu_buffer_rsrc_t gr =
          attn_rsrc((const bf16_t*)a.gate + ECHO_QROW(a, row) * a.g_ld_batch + qv * a.g_ld_tok + head * 128,
                    (uint32_t)(((int64_t)(min(nv, 32) - 1) * a.g_ld_tok + 128) * 2));
      const uint32_t glo = (uint32_t)((rl * a.g_ld_tok + cc * 8) * 2), gst = (uint32_t)(a.g_ld_tok * 8);
#pragma unroll
      for (int pk = 0; pk < 8; ++pk) g4[pk] = attn_bload(gr, glo + pk * gst);
    }
    {
      float od[16];
      if constexpr (J == 0) {
        WB::get_o_0_0(od); pack_dt(od, 0);
        WB::get_o_0_1(od); pack_dt(od, 1);
        WB::get_o_0_2(od); pack_dt(od, 2);
        WB::get_o_0_3(od); pack_dt(od, 3);
      } else {
        WB::get_o_1_0(od); pack_dt(od, 0);
        WB::get_o_1_1(od); pack_dt(od, 1);
        WB::get_o_1_2(od); pack_dt(od, 2);
        WB::get_o_1_3(od); pack_dt(od, 3);
      }
    }
    bf16_t* sw = lds + (2 * w + J) * 32 * 128;  // free: no DMA in flight, every wave passed the last barrier
#pragma unroll
    for (int pk = 0; pk < 8; ++pk) *(uint4*)(sw + ql * 128 + (((2 * pk + h2) ^ (ql & 15)) * 8)) = v4[pk];
#pragma unroll
    for (int pk = 0; pk < 8; ++pk) {
      const int r = pk * 4 + rl;
      v4[pk] = *(const uint4*)(sw + r * 128 + ((cc ^ (r & 15)) * 8));
    }
    if (a.gate) attn_gate(v4, g4);
    attn_store_rows(v4, (bf16_t*)a.out + row * a.o_ld_batch + qv * a.o_ld_tok + head * 128, nv, a.o_ld_tok, lane);
  };
  store_block(std::integral_constant<int, 0>{}, la);
  store_block(std::integral_constant<int, 1>{}, lb);
}
#endif  // ECHO_DIAG

// one (query qi, 8 output columns c8) unit of (row, head) rh of the split-KV combine
template <class Args>
__device__ void attn_combine_unit(const Args& a, const float* __restrict__ ws, int nsp, int rh, int qi, int c8) {
  const int row = rh / a.heads, head = rh % a.heads;
  const int64_t per_split = (int64_t)a.rows * a.heads * 128 * a.n_q;
  const float* ml = ws + nsp * per_split;
  // the gate and, for up to 4 splits (every policy split count), every split's (m, l) and partial O are loaded
  // before any of them is used: one memory round trip instead of one per split; the arithmetic below runs in
  // the same order either way
  uint4 g4 = make_uint4(0, 0, 0, 0);
  if (a.gate)
    g4 = *(const uint4*)((const bf16_t*)a.gate + ECHO_QROW(a, row) * a.g_ld_batch + (int64_t)qi * a.g_ld_tok +
                         head * 128 + 8 * c8);
  constexpr int NB = 4;
  float2 mlb[NB];
  float4 lob[NB], hib[NB];
  if (nsp <= NB) {
#pragma unroll
    for (int s = 0; s < NB; ++s) {
      if (s < nsp) {
        const int64_t it = (int64_t)s * a.rows * a.heads + rh;
        const float* wo = ws + it * 128 * a.n_q;
        mlb[s] = *(const float2*)(ml + (it * a.n_q + qi) * 2);
        lob[s] = *(const float4*)(wo + ((int64_t)(2 * c8) * a.n_q + qi) * 4);
        hib[s] = *(const float4*)(wo + ((int64_t)(2 * c8 + 1) * a.n_q + qi) * 4);
      }
    }
  }
  float mx = -INFINITY;
  if (nsp <= NB) {
#pragma unroll
    for (int s = 0; s < NB; ++s)
      if (s < nsp) mx = fmaxf(mx, mlb[s].x);
  } else {
    for (int s = 0; s < nsp; ++s) mx = fmaxf(mx, ml[(((int64_t)s * a.rows * a.heads + rh) * a.n_q + qi) * 2]);
  }
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, l = 0.f;
  auto add = [&](float2 m_l, float4 lo, float4 hi) __attribute__((always_inline)) {
    if (m_l.x == -INFINITY) return;  // split without a visible key for this query
    const float wgt = __builtin_amdgcn_exp2f(m_l.x - mx);
    acc[0] += wgt * lo.x; acc[1] += wgt * lo.y; acc[2] += wgt * lo.z; acc[3] += wgt * lo.w;
    acc[4] += wgt * hi.x; acc[5] += wgt * hi.y; acc[6] += wgt * hi.z; acc[7] += wgt * hi.w;
    l += wgt * m_l.y;
  };
  if (nsp <= NB) {
#pragma unroll
    for (int s = 0; s < NB; ++s)
      if (s < nsp) add(mlb[s], lob[s], hib[s]);
  } else {
    for (int s = 0; s < nsp; ++s) {
      const int64_t it = (int64_t)s * a.rows * a.heads + rh;
      const float* wo = ws + it * 128 * a.n_q;
      add(*(const float2*)(ml + (it * a.n_q + qi) * 2), *(const float4*)(wo + ((int64_t)(2 * c8) * a.n_q + qi) * 4),
          *(const float4*)(wo + ((int64_t)(2 * c8 + 1) * a.n_q + qi) * 4));
    }
  }
  const float inv = 1.0f / l;
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = rbf(acc[e] * inv);
  if (a.gate) {
    const uint32_t gg[4] = {g4.x, g4.y, g4.z, g4.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float g0 = bf2f(gg[e] & 0xffffu), g1 = bf2f(gg[e] >> 16);  // sigmoid_hw: see attn_pack_out
      v[2 * e] = rbf(v[2 * e] * rbf(g0 < -87.0f ? sigmoid_f(g0) : sigmoid_hw(g0)));
      v[2 * e + 1] = rbf(v[2 * e + 1] * rbf(g1 < -87.0f ? sigmoid_f(g1) : sigmoid_hw(g1)));
    }
  }
  *(uint4*)((bf16_t*)a.out + row * a.o_ld_batch + (int64_t)qi * a.o_ld_tok + head * 128 + 8 * c8) =
      make_uint4(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]), pack2bf(v[6], v[7]));
}

__global__ void __launch_bounds__(256) attn_combine_kernel(EchoAttnArgs a, const float* __restrict__ ws, int nsp) {
  const int nqb = (a.n_q + 15) / 16;
  const int qb = blockIdx.x % nqb, rh = blockIdx.x / nqb;  // rh = row * heads + head
  const int qi = qb * 16 + (threadIdx.x & 15), c8 = threadIdx.x >> 4;
  if (qi >= a.n_q) return;
  attn_combine_unit(a, ws, nsp, rh, qi, c8);
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
  const float* qp = (const float*)a.q + ECHO_QROW(a, row) * a.q_ld_batch + (int64_t)qc * a.q_ld_tok + head * 128;
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
  const float* gp = a.gate ? (const float*)a.gate + ECHO_QROW(a, row) * a.g_ld_batch + (int64_t)qi * a.g_ld_tok + head * 128
                           : nullptr;
#pragma unroll
  for (int d = 0; d < 128; ++d) {
    float v = o[d] / l;
    if (gp) v = v * sigmoid_f(gp[d]);
    op[d] = v;
  }
}

}  // namespace

namespace {

int check_attn_args(const EchoAttnArgs* a) {
  if (!a || !a->q || !a->out) return ECHO_EINVAL;
  if (a->rows <= 0 || a->n_q <= 0 || a->heads <= 0 || a->nseg < 1 || a->nseg > 4) return ECHO_ESHAPE;
  if (a->q_batch_mod < 0 || a->q_batch_mod > a->rows) return ECHO_ESHAPE;
  bool any = false;
  for (int s = 0; s < a->nseg; ++s) {
    const EchoKVSegment& S = a->seg[s];
    if (!S.k) continue;
    if (!S.v || S.batch_mod <= 0 || S.capacity <= 0) return ECHO_EINVAL;
    if (S.ld_tok % 8 || S.ld_batch % 8) return ECHO_EALIGN;
    any = true;
  }
  if (!any) return ECHO_EINVAL;
  // bf16: 16-B Q loads, 16-B gate loads and output stores (attn_store_out)
  if (a->dtype == ECHO_BF16 &&
      (a->q_ld_tok % 8 || a->q_ld_batch % 8 || a->o_ld_tok % 8 || a->o_ld_batch % 8 || (uintptr_t)a->q % 16 ||
       (uintptr_t)a->out % 16 || (a->gate && (a->g_ld_tok % 8 || a->g_ld_batch % 8 || (uintptr_t)a->gate % 16))))
    return ECHO_EALIGN;
  if (a->dtype != ECHO_BF16 && a->dtype != ECHO_F32) return ECHO_EDTYPE;
  return 0;
}

int attn_grid(const EchoAttnArgs* a, int qb) { return ((a->n_q + qb - 1) / qb) * a->heads * a->rows; }

bool any_causal(const EchoAttnArgs* a) {
  for (int s = 0; s < a->nseg; ++s)
    if (a->seg[s].k && a->seg[s].causal) return true;
  return false;
}

int g_attn_pl = 1;  // echo_attention_set_pipeline: 0 = attn_bf16_kernel for every launch (A/B)

#ifdef ECHO_DIAG
// persistent grid: two workgroups per CU (a multiple of 8, so an item's XCD is its block's XCD)
int attn_ps_grid(int nitems) {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      return -1;
    cus = n;
  }
  return min(nitems, (2 * cus + 7) / 8 * 8);
}
#endif


// Measurement variants of the bf16 kernel (tools/bench_attn.py; DESIGN.md §7 lists what each
// showed). The product library keeps variant 0 (the compiler-scheduled production kernel, the bitwise
// reference of the others) and 11 (attn_pl_kernel, production for non-causal launches) with ablation 0;
// everything else is in the diagnostics build only (ECHO_DIAG=1) and refused with ECHO_EINVAL here:
// 1/2 8 waves with a 2/3-slot ring, 3/4 register-staged K/V with 4/8 waves, 6/7 32-key tiles with a
// 2/3-slot ring, 8 the persistent form of 0, 9 two waves (64 queries) per workgroup, 10 = 0 with the
// per-lane epilogue (round-2 form before the row-layout epilogue), 30/40 attn_w64_kernel, the ablation
// bits of attn_bf16_kernel (128: s_memrealtime stamps) and the asm kernels' ablations 12-22 / 31-43.
int launch_attn_variant(const EchoAttnArgs* a, int cfg, int abl, hipStream_t s) {
  const int qb = (cfg == 1 || cfg == 2 || cfg == 4) ? 256 : 128;
  const dim3 grid(attn_grid(a, qb));
  if (cfg == 0 && abl == 0) {
    hipLaunchKernelGGL((attn_bf16_kernel<0, 4, 2>), grid, dim3(256), 0, s, *a, (float*)nullptr, 1, (uint32_t*)nullptr);
    ECHO_LAUNCH_CHECK();
    return 0;
  }
  if (cfg == 11) {  // asm-owned software pipeline (production for non-causal launches)
    if (abl || any_causal(a)) return ECHO_EINVAL;
    hipLaunchKernelGGL(attn_pl_kernel<0>, grid, dim3(256), 0, s, *a);
    ECHO_LAUNCH_CHECK();
    return 0;
  }
#ifndef ECHO_DIAG
  (void)qb;
  return ECHO_EINVAL;
#else
#define ECHO_ATTN_LAUNCH(A, NW, ST, ...) \
  hipLaunchKernelGGL((attn_bf16_kernel<A, NW, ST, ##__VA_ARGS__>), grid, dim3(64 * NW), 0, s, *a, (float*)nullptr, 1, (uint32_t*)nullptr)
#define ECHO_ATTN_ABLS(NW, ST)                        \
  switch (abl) {                                      \
    case 0: ECHO_ATTN_LAUNCH(0, NW, ST); break;       \
    case 128: ECHO_ATTN_LAUNCH(128, NW, ST); break;   \
    case 1: ECHO_ATTN_LAUNCH(1, NW, ST); break;       \
    case 2: ECHO_ATTN_LAUNCH(2, NW, ST); break;       \
    case 3: ECHO_ATTN_LAUNCH(3, NW, ST); break;       \
    case 4: ECHO_ATTN_LAUNCH(4, NW, ST); break;       \
    case 6: ECHO_ATTN_LAUNCH(6, NW, ST); break;       \
    case 7: ECHO_ATTN_LAUNCH(7, NW, ST); break;       \
    case 8: ECHO_ATTN_LAUNCH(8, NW, ST); break;       \
    case 13: ECHO_ATTN_LAUNCH(13, NW, ST); break;     \
    case 19: ECHO_ATTN_LAUNCH(19, NW, ST); break;     \
    case 35: ECHO_ATTN_LAUNCH(35, NW, ST); break;     \
    case 51: ECHO_ATTN_LAUNCH(51, NW, ST); break;     \
    case 64: ECHO_ATTN_LAUNCH(64, NW, ST); break;     \
    case 256: ECHO_ATTN_LAUNCH(256, NW, ST); break;   \
    case 640: ECHO_ATTN_LAUNCH(640, NW, ST); break;   \
    case 641: ECHO_ATTN_LAUNCH(641, NW, ST); break;   \
    default: return ECHO_EINVAL;                      \
  }
  switch (cfg) {
    case 0: ECHO_ATTN_ABLS(4, 2); break;
    case 1: ECHO_ATTN_ABLS(8, 2); break;
    case 2: ECHO_ATTN_ABLS(8, 3); break;
    case 3: ECHO_ATTN_ABLS(4, 0); break;
    case 4: ECHO_ATTN_ABLS(8, 0); break;
    case 8: {  // persistent form: two workgroups per CU
      if (abl) return ECHO_EINVAL;
      const int ps_grid = attn_ps_grid(grid.x);
      if (ps_grid <= 0) return ECHO_EINVAL;
      hipLaunchKernelGGL((attn_bf16_kernel<0, 4, 2, 64, 1>), dim3(ps_grid), dim3(256), 0, s, *a, (float*)nullptr, 1, (uint32_t*)nullptr);
      break;
    }
    case 6: if (abl) return ECHO_EINVAL; ECHO_ATTN_LAUNCH(0, 4, 2, 32); break;
    case 9:  // 2 waves x 32 queries per workgroup
      if (abl) return ECHO_EINVAL;
      hipLaunchKernelGGL((attn_bf16_kernel<0, 2, 2>), dim3(attn_grid(a, 64)), dim3(128), 0, s, *a, (float*)nullptr, 1, (uint32_t*)nullptr);
      break;
    case 7: if (abl) return ECHO_EINVAL; ECHO_ATTN_LAUNCH(0, 4, 3, 32); break;
    case 10: if (abl) return ECHO_EINVAL; ECHO_ATTN_LAUNCH(2048, 4, 2); break;  // per-lane epilogue
    case 30:  // one wave per SIMD, 64 queries per wave, two waves per workgroup (measured slower)
      if (abl || any_causal(a)) return ECHO_EINVAL;
      hipLaunchKernelGGL((attn_w64_kernel<0, 2>), grid, dim3(128), 0, s, *a);
      break;
    case 40:  // four waves x 64 queries (256-query workgroups)
      if (abl || any_causal(a)) return ECHO_EINVAL;
      hipLaunchKernelGGL((attn_w64_kernel<0, 4>), dim3(attn_grid(a, 256)), dim3(256), 0, s, *a);
      break;
    // ablations of the asm-owned kernels (timing only, results wrong; DESIGN.md §3 lists what each showed):
    // attn_pl_kernel ABL bits 12-18, 8 waves x 32 queries 20-22, attn_w64_kernel 31-33 / 41-43 (16 no tile loop,
    // 1 no loop DMA, 8 no end-of-tile wait)
    case 12: hipLaunchKernelGGL(attn_pl_kernel<1>, grid, dim3(256), 0, s, *a); break;
    case 13: hipLaunchKernelGGL(attn_pl_kernel<2>, grid, dim3(256), 0, s, *a); break;
    case 14: hipLaunchKernelGGL(attn_pl_kernel<4>, grid, dim3(256), 0, s, *a); break;
    case 15: hipLaunchKernelGGL(attn_pl_kernel<8>, grid, dim3(256), 0, s, *a); break;
    case 16: hipLaunchKernelGGL(attn_pl_kernel<16>, grid, dim3(256), 0, s, *a); break;
    case 17: hipLaunchKernelGGL(attn_pl_kernel<6>, grid, dim3(256), 0, s, *a); break;
    case 18: hipLaunchKernelGGL(attn_pl_kernel<7>, grid, dim3(256), 0, s, *a); break;
    case 31: case 32: case 33:
      if (any_causal(a)) return ECHO_EINVAL;
      if (cfg == 31) hipLaunchKernelGGL((attn_w64_kernel<16, 2>), grid, dim3(128), 0, s, *a);
      else if (cfg == 32) hipLaunchKernelGGL((attn_w64_kernel<1, 2>), grid, dim3(128), 0, s, *a);
      else hipLaunchKernelGGL((attn_w64_kernel<8, 2>), grid, dim3(128), 0, s, *a);
      break;
    case 41: case 42: case 43: {
      if (any_causal(a)) return ECHO_EINVAL;
      const dim3 g4(attn_grid(a, 256));
      if (cfg == 41) hipLaunchKernelGGL((attn_w64_kernel<16, 4>), g4, dim3(256), 0, s, *a);
      else if (cfg == 42) hipLaunchKernelGGL((attn_w64_kernel<1, 4>), g4, dim3(256), 0, s, *a);
      else hipLaunchKernelGGL((attn_w64_kernel<8, 4>), g4, dim3(256), 0, s, *a);
      break;
    }
    case 20: case 21: case 22: {
      if (any_causal(a)) return ECHO_EINVAL;
      const dim3 g8(attn_grid(a, 256));
      if (cfg == 20) hipLaunchKernelGGL((attn_pl_kernel<0, 8>), g8, dim3(512), 0, s, *a);
      else if (cfg == 21) hipLaunchKernelGGL((attn_pl_kernel<16, 8>), g8, dim3(512), 0, s, *a);
      else hipLaunchKernelGGL((attn_pl_kernel<6, 8>), g8, dim3(512), 0, s, *a);
      break;
    }
    default: return ECHO_EINVAL;
  }
#undef ECHO_ATTN_ABLS
#undef ECHO_ATTN_LAUNCH
  ECHO_LAUNCH_CHECK();
  return 0;
#endif  // ECHO_DIAG
}

}  // namespace

extern "C" int echo_attention(const EchoAttnArgs* a, void* stream) {
  const int rc = check_attn_args(a);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  if (a->dtype == ECHO_BF16) {
    // one workgroup per item. The persistent form (variant 8, bitwise equal; its store tail overlaps
    // the next item's prologue) won for 1-3 items per workgroup slot with the per-lane epilogue
    // (R = 16: 152.7 -> 146.9 us); with the row-layout epilogue the plain grid is faster there too
    // (R = 16: 149.7 vs 153.7 us, n_q = 160: 47.7 vs 48.3, one box; profiles/r2_attn_cmp.txt).
    // (fewer items than CUs, B = 1: 64-query workgroups — variant 9, bitwise equal — are slower,
    // R = 3: 43.2 -> 54.1 us, R = 1: 38.7 -> 47.1 us: the per-workgroup tile chain stays as long and
    // each wave issues twice the DMA; that case takes split-KV chains, echo_attention_split)
    // non-causal launches (every decoder attention) run the asm-owned pipeline (attn_pl_kernel, bitwise
    // equal to attn_bf16_kernel<0, 4, 2>); causal ones (speaker / latent encoders) the compiler-scheduled kernel
#ifdef ECHO_DIAG
    if (g_attn_pl == 2 && !any_causal(a))
      hipLaunchKernelGGL((attn_w64_kernel<0, 4>), dim3(attn_grid(a, 256)), dim3(256), 0, s, *a);
    else
#endif
    if (g_attn_pl && !any_causal(a))
      hipLaunchKernelGGL(attn_pl_kernel<0>, dim3(attn_grid(a, 128)), dim3(256), 0, s, *a);
    else
      hipLaunchKernelGGL((attn_bf16_kernel<0, 4, 2>), dim3(attn_grid(a, 128)), dim3(256), 0, s, *a, (float*)nullptr, 1, (uint32_t*)nullptr);
  } else {
    hipLaunchKernelGGL(attn_f32_kernel, dim3(attn_grid(a, FQ)), dim3(64), 0, s, *a);
  }
  ECHO_LAUNCH_CHECK();
  return 0;
}

extern int g_policy_num, g_policy_den;  // echo_set_policy_rows (gemm.hip)

namespace {
int g_attn_split_override = -1;  // echo_attention_set_split: force nsplit (diagnostics), -1 = policy
int cu_count() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      return 256;
    cus = n;
  }
  return cus;
}
}  // namespace

extern "C" int64_t echo_attention_split_ws_bytes(const EchoAttnArgs* a, int32_t nsplit) {
  if (!a || nsplit < 2 || a->rows <= 0 || a->heads <= 0 || a->n_q <= 0) return 0;
  return (int64_t)nsplit * a->rows * a->heads * a->n_q * (128 + 2) * (int64_t)sizeof(float);
}

extern "C" int32_t echo_attention_pick_split(const EchoAttnArgs* a) {
  if (check_attn_args(a) || a->dtype != ECHO_BF16) return 1;
  int tiles = 0;  // upper bound of an item's flat tile list (capacities; lens are on the device)
  for (int s = 0; s < a->nseg; ++s)
    if (a->seg[s].k) tiles += (a->seg[s].capacity + KT - 1) / KT;
  int nsp;
  if (g_attn_split_override >= 0) {
    nsp = g_attn_split_override;
  } else {
    // measured (tools/bench_attn.py --splits, MI355X, 256 CUs; us for split counts 1 / 2 / 3 / 4):
    //   640 queries, R = 3 (240 items): 38.5 / 44.0 / 50.1 / 52.7  -> never
    //   640 queries, R = 1 ( 80 items): 35.7 / 30.0 / 29.7 / 31.8  -> 3
    //   160 queries, R = 3 ( 96 items): 28.7 / 25.1 / 26.5 / 27.1  -> 2
    //   160 queries, R = 1 ( 32 items): 27.9 / 21.7 / 21.0 / 21.0  -> 3-4
    // the per-workgroup prologue (Q + first K/V tile) and the partials' round trip through L2/HBM
    // (nsplit x the output in fp32) bound the gain: split only launches that leave half the CUs idle
    // items of the launch as a one-process run of the whole batch would have them (echo_set_policy_rows)
    const int nitems = (int)((int64_t)attn_grid(a, 128) * g_policy_num / g_policy_den), cus = cu_count();
    nsp = nitems * 2 > cus ? 1 : nitems * 8 >= cus * 3 ? 2 : nitems * 8 > cus ? 3 : 4;
    nsp = min(nsp, tiles / 3);
  }
  return max(1, min(nsp, min(tiles, 16)));
}

extern "C" int echo_attention_set_pipeline(int32_t on) {
#ifdef ECHO_DIAG
  if (on < 0 || on > 2) return ECHO_EINVAL;  // 2: attn_w64_kernel (diagnostics build only)
#else
  if (on < 0 || on > 1) return ECHO_EINVAL;
#endif
  g_attn_pl = on;
  return 0;
}

extern "C" int echo_attention_set_split(int32_t nsplit) {
  if (nsplit < -1 || nsplit > 16) return ECHO_EINVAL;
  g_attn_split_override = nsplit;
  return 0;
}

uint32_t* g_sync = nullptr;  // echo_set_sync_buffer: caller-owned counters of in-launch merges (0 words = off)
int64_t g_sync_words = 0;

// The in-launch hand-offs (the split-KV merge here, the split-K finish in gemm.hip) were measured slower than the
// kernel boundaries they remove (C5 B = 1 68.0 -> 55.4 audio-s/s), so they exist in the
// diagnostics build only (ECHO_DIAG=1); the product library refuses a counter buffer.
extern "C" int echo_set_sync_buffer(uint32_t* sync, int64_t words) {
  if ((sync == nullptr) != (words == 0) || words < 0 || (uintptr_t)sync % 64) return ECHO_EINVAL;
#ifndef ECHO_DIAG
  if (sync) return ECHO_EINVAL;
#endif
  g_sync = sync;
  g_sync_words = words;
  return 0;
}

extern int g_no_inlaunch_merge;  // echo_gemm_set_diag key 15 (gemm.hip)

extern "C" int32_t echo_attention_merge_in_launch(const EchoAttnArgs* a, int32_t nsplit) {
  if (!g_sync || g_no_inlaunch_merge || !a || nsplit < 2 || nsplit > 16 || a->rows <= 0 || a->heads <= 0 || a->n_q <= 0) return 0;
  const int64_t items = (int64_t)attn_grid(a, 128);
  // every split of an item must be resident at once: at most one workgroup per CU; counters must fit
  return items * nsplit <= cu_count() && SYNC_CNT0 + 2 * items <= g_sync_words &&
         echo_attention_split_ws_bytes(a, nsplit) < ((int64_t)1 << 32) - 16;
}

extern "C" int echo_attention_split(const EchoAttnArgs* a, int32_t nsplit, void* ws, int64_t ws_bytes, void* stream) {
  const int rc = check_attn_args(a);
  if (rc) return rc;
  if (nsplit <= 1) return echo_attention(a, stream);
  if (a->dtype != ECHO_BF16) return ECHO_EDTYPE;
  if (nsplit > 16) return ECHO_EINVAL;
  if (!ws || (uintptr_t)ws % 16 || ws_bytes < echo_attention_split_ws_bytes(a, nsplit)) return ECHO_EINVAL;
  hipStream_t s = (hipStream_t)stream;
#ifdef ECHO_DIAG
  if (echo_attention_merge_in_launch(a, nsplit)) {  // one launch: the splits merge themselves (SP = 2)
    hipLaunchKernelGGL((attn_bf16_kernel<0, 4, 2, 64, 0, 2>), dim3(attn_grid(a, 128) * nsplit), dim3(256), 0, s, *a,
                       (float*)ws, (int)nsplit, g_sync);
    ECHO_LAUNCH_CHECK();
    return 0;
  }
#endif
  hipLaunchKernelGGL((attn_bf16_kernel<0, 4, 2, 64, 0, 1>), dim3(attn_grid(a, 128) * nsplit), dim3(256), 0, s, *a,
                     (float*)ws, (int)nsplit, (uint32_t*)nullptr);
  ECHO_LAUNCH_CHECK();
  hipLaunchKernelGGL(attn_combine_kernel, dim3(a->rows * a->heads * ((a->n_q + 15) / 16)), dim3(256), 0, s, *a,
                     (const float*)ws, (int)nsplit);
  ECHO_LAUNCH_CHECK();
  return 0;
}

extern "C" int echo_attention_variant(const EchoAttnArgs* a, int32_t variant, int32_t ablation, uint64_t* stamps,
                                      void* stream) {
  const int rc = check_attn_args(a);
  if (rc) return rc;
  if (a->dtype != ECHO_BF16) return ECHO_EDTYPE;
  if ((ablation & 640) && (!stamps || variant > 4)) return ECHO_EINVAL;  // stamps: attn_bf16_kernel variants
#ifndef ECHO_DIAG
  if (ablation) return ECHO_EINVAL;  // ablations and stamps: diagnostics build only
#endif
  if (ablation & 640) {
    if (hipMemcpyToSymbolAsync(HIP_SYMBOL(g_attn_stamps), &stamps, sizeof(stamps), 0, hipMemcpyHostToDevice,
                               (hipStream_t)stream) != hipSuccess)
      return ECHO_EINVAL;
  }
  return launch_attn_variant(a, variant, ablation, (hipStream_t)stream);
}

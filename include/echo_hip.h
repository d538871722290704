/*
 * echo_hip.h — C ABI of the MI355X-native Echo-TTS sampling path.
 *
 * The reference path is pure Python/PyTorch: its "FFI" is the
 * set of torch ops the DiT forward issues. Each entry point below replaces one
 * group of those ops (file:line cited per function) and is bound from Python
 * with ctypes (echo-tts_amd/_lib.py; the binding a maintainer would add to the
 * reference is shown in INTEGRATION.md).
 *
 * Conventions (all functions):
 *   - plain device pointers + sizes; no torch types;
 *   - `dtype` selects the element type of activations/weights:
 *       ECHO_BF16 (0) = bfloat16 storage, ECHO_F32 (1) = float32;
 *   - `stream` is a hipStream_t (NULL = default stream); nothing here
 *     synchronises the host, so every call is capturable in a hipGraph;
 *   - return 0 on success, a negative ECHO_E* code on invalid arguments
 *     (checked on the host before launch), or a positive hipError_t.
 *   - lengths/masks are prefix lengths: a key mask of the reference
 *     (model.py:246-261) must be a prefix to be expressible (host checks it).
 */
#ifndef ECHO_HIP_H
#define ECHO_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ECHO_BF16 = 0, ECHO_F32 = 1 };
enum { ECHO_OK = 0, ECHO_EINVAL = -1, ECHO_EDTYPE = -2, ECHO_ESHAPE = -3, ECHO_EALIGN = -4 };

/* GEMM epilogues (applied in this order; see echo-tts_amd/csrc/gemm.hip):
 *   v = acc (+ bias[n]);  v = round(v)                       F.linear (model.py:56-62,303-305,...)
 *   act == ECHO_ACT_SILU: v = round(silu(v))                 nn.SiLU in cond_module (model.py:532-538)
 *   act == ECHO_ACT_GELU: v = round(gelu_erf(v))             ConvNeXt pwconv1 + nn.GELU (autoencoder.py:366-367)
 *   act == ECHO_ACT_SNAKE: v = snake(v, act_alpha[n]) with the reference's bf16 rounding after
 *                    every op (fp32: none)                   Snake1d after a conv (autoencoder.py:97-102,886)
 *   out_div != 0:         v = round(v / out_div)             SpeakerEncoder `x / 6.` (model.py:462)
 *   ECHO_EPI_SWIGLU: W rows interleaved in blocks of 16 (w1,w3,w1,w3,...);
 *                    out[m][n] = round(round(silu(a)) * b)   MLP.forward (model.py:307-308)
 *   ECHO_EPI_RESID:  out = round(aux[m][n] + round(gate[n] * v))   gated residual (model.py:385,388)
 *                    (gate NULL: out = round(aux + v); aux may alias out)
 *   ECHO_EPI_F32OUT: out (float32) = v                       out_proj(...).float() (model.py:602-604)
 *   ECHO_EPI_HEADNORM: out = v, then columns [0, hn_nblk*hn_heads*128) get the per-head
 *                    RMSNorm (+ RoPE on heads < hn_rope_heads) of echo_head_norm_rope with
 *                    col0 = 0, col_stride = hn_heads*128 — q_norm/k_norm + RoPE right after
 *                    the fused QKV(G) projection (model.py:138-142,199-202,221-232); batch == 1
 */
enum { ECHO_EPI_STORE = 0, ECHO_EPI_SWIGLU = 1, ECHO_EPI_RESID = 2, ECHO_EPI_F32OUT = 3, ECHO_EPI_HEADNORM = 4 };
enum { ECHO_ACT_NONE = 0, ECHO_ACT_SILU = 1, ECHO_ACT_GELU = 2, ECHO_ACT_SNAKE = 3 };

typedef struct {
  int32_t dtype;
  int32_t M, N, K;          /* C[M,N] = A[M,K] . W[N,K]^T ; K % 64 == 0, N % 16 == 0 */
  int32_t batch;            /* grid.y batches, strides in elements */
  const void* A; int64_t lda; int64_t stride_a;
  const void* W; int64_t ldw; int64_t stride_w;
  void* C; int64_t ldc; int64_t stride_c;
  const void* bias; int64_t stride_bias;          /* [N] or NULL */
  const void* aux; int64_t ld_aux; int64_t stride_aux;  /* RESID residual input */
  const void* gate; int64_t stride_gate;          /* RESID per-column gate or NULL */
  int32_t epilogue, act;
  float out_div;
  int32_t tile;             /* 0 = auto; else forced config id (tests/tuning) */
  /* ECHO_EPI_HEADNORM parameters (meaning as in echo_head_norm_rope) */
  const void* hn_w; int64_t hn_w_stride; const float* hn_rope;
  int32_t hn_heads, hn_nblk, hn_rope_heads, hn_seq_len, hn_pos0, hn_pos_mult;
  float hn_eps;
  /* ECHO_ACT_SNAKE per-column alpha [N] (output dtype) */
  const void* act_alpha;
  /* Causal 1-D convolution as a GEMM (conv_taps > 0): K = conv_taps * conv_c and A is the
   * channels-last activation x (row stride lda) read as the virtual matrix
   *   A'[t][tap*conv_c + c] = x[t - (conv_taps-1-tap)*conv_dil][c]
   * i.e. CausalConvNet (autoencoder.py:264-289) with W[co][tap*conv_c + ci] = w[co][ci][tap].
   * Rows before t = 0 are read from memory: the caller keeps >= (conv_taps-1)*conv_dil zero rows
   * ahead of A. conv_c % 64 == 0 (bf16) / % 16 == 0 (fp32). */
  int32_t conv_c, conv_taps, conv_dil;
  /* ECHO_EPI_RESID only, mod_out != NULL: also the NEXT LowRankAdaLN normalisation of the updated rows,
   *   mod_out[m][n] = round(((out[m][n] * rsqrt(mean_n(out[m][:]^2) + mod_eps)) * mod_scale1[n]) + mod_shift[n])
   * (echo_adaln_modulate's arithmetic on the residual stream this GEMM just wrote; model.py:76-81 of the next
   * AdaLN). Needs batch == 1 and contiguous rows (ldc == ld_mod == N). Fused into the split-K finish kernel
   * of under-filled bf16 launches (N == 2048: one workgroup per row), a separate echo_adaln_modulate pass
   * after the GEMM otherwise; bitwise the same either way. */
  void* mod_out; int64_t ld_mod;
  const void* mod_shift; const void* mod_scale1;
  float mod_eps;
} EchoGemmArgs;

/* Replaces every nn.Linear of the DiT and its encoders (F.linear, model.py:56-62,
 * 118-122,177-197,303-305,443,532-540,557) plus the fused elementwise tails above. */
int echo_gemm(const EchoGemmArgs* args, void* stream);

/* Tile configuration echo_gemm picks for a shape when args->tile == 0 (1..5). */
int echo_gemm_pick_tile(int32_t M, int32_t N, int32_t K, int32_t batch);

/* Under-filled launches (the B = 1 and blockwise decoder GEMMs, M <= a few thousand rows) can split K
 * over S workgroups that each store an fp32 partial tile; a second kernel sums the S partials in order
 * and applies the fused epilogue. That needs a device workspace of echo_gemm_ws_bytes(args) bytes
 * (0: the plan for these arguments does not split K) passed to echo_gemm_ws. echo_gemm(args, stream)
 * is echo_gemm_ws(args, NULL, 0, stream): it never splits K. Same results as echo_gemm except that a
 * split launch sums K in S contiguous partial sums (fp32; the unsplit kernels all share one K order).
 * The workspace is only touched by the launched kernels (stream-ordered, capturable). */
int64_t echo_gemm_ws_bytes(const EchoGemmArgs* args);
/* Host-only query: the launch echo_gemm_ws(args, ws, ws_bytes, .) would make (the same host routine decides both;
 * bench.py's per-launch labels): 100 + 10 c + S = the small-M config c with K split S ways; 2..5 the smaller tile
 * configs; 13 the 2-phase 256x256 kernel; 16 the persistent 256x256 kernel; 20 320-row tiles; 301 the 320-row column
 * split (whole rounds of 320-row tile columns, the rest by the auto pick); 302 the W13 column split at 1537-2048 rows
 * (persistent 256x256 kernel + small-M config 13); 303 the row-tail split (256x256 rounds + a smaller-tile tail);
 * 304 store + echo_head_norm_rope (head norm not fused for the shape); 305 fp32 (round 6: 301-305, past the small-M
 * codes, which reach 269); a forced `tile` is returned as is. */
int32_t echo_gemm_planned_tile(const EchoGemmArgs* args, int64_t ws_bytes);
int echo_gemm_ws(const EchoGemmArgs* args, void* ws, int64_t ws_bytes, void* stream);

/* Split decisions (GEMM split-K here, split-KV in echo_attention_pick_split) depend on the launch's
 * row count. A process that runs `den` of the `num` prompts of a sharded batch (echo_tts_amd.distributed)
 * sets num / den so that every such decision is taken for the rows the whole batch would have in one
 * process: each rank then runs the same kernels, with the same summation order, as a one-process run of
 * the whole batch (bitwise-equal gathered output). 1 / 1 (default) = decide on the launch's own rows. */
int echo_set_policy_rows(int32_t num, int32_t den);

/* Diagnostic knobs for tools/bench_gemm.py (not used by the product path). key 1: the persistent
 * 256x256 kernel's group-M height for `tile` = 18. key 2: 0 turns the 3-stage pipeline of the two smallest tile configs off (A/B
 * timing; both schedules give bitwise-equal results). key 3: 1 = no row-tail split of auto-picked
 * 256x256 launches; key 4: 1 = the 2-phase kernel instead of the persistent one for auto-picked
 * 256x256 launches; key 5: tile count below which an auto-picked 256x256 launch switches to a
 * smaller tile (default 128); key 6: cap on the persistent kernel's workgroup count (0 = one per CU);
 * key 7: 320x256 tiles for the gated residual / SwiGLU / head norm (0 = when they need fewer 1.2x
 * tile-rounds than 256x256 tiles, 1 = never, 2 = whenever they fill at least one round); key 8: 1 = no
 * column split of auto-picked launches: neither the 320-row one (W13 at M = 320 k: 320-row tiles on whole rounds
 * of tile columns, the rest on the persistent 256x256 kernel) nor the W13 one at 1537-2048 rows (one round of the
 * persistent 256x256 kernel, the rest on small-M config 13); key 9: block cap of the wave-per-row AdaLN kernel (0 = 8192);
 * (`tile` 22 / 23 force one 320-row tile per workgroup / the persistent 320-row kernel for any epilogue;
 * A/B timing, all bitwise-equal; key 10 is retired.)
 * key 11: 1 = never split K in echo_gemm_ws (the B = 1 runs that tests compare bitwise with B = 16 rows);
 * key 12: 1 = no small-M kernel in the auto pick (the round-3 small tiles; A/B);
 * key 13: group-M height of the persistent 256x256 and 320-row kernels' tile order (0 = 4; 1..64; bitwise-equal).
 * key 14 / 15: 1 = no in-launch split-K finish / split-KV merge (A/B of echo_set_sync_buffer's hand-offs; no effect in
 * the product library, which has none); key 16 (diagnostics build only, refused here): timing ablations of the
 * small-M kernel (bits: 1 no MFMA, 2 no DMA in the K loop, 4 no epilogue, 8 no DMA at all; results wrong; 32 the
 * round-5 DMA issue order, results right).
 * `tile` 100 + 10*C + S (C = small-M config 1..16, S = split 1..9) forces a small-M launch (tools/bench_gemm.py).
 * The timing-ablation tiles 7-12 and 15 (results wrong) exist in the diagnostics build (ECHO_DIAG=1) only. */
int echo_gemm_set_diag(int32_t key, int32_t value);

/* One key/value segment of the joint attention (model.py:246-253): rows of
 * `len[row]` valid tokens (prefix), head h at element offset h*128. */
typedef struct {
  const void* k; const void* v;
  int64_t ld_tok;     /* elements between consecutive tokens */
  int64_t ld_batch;   /* elements between batch entries */
  int32_t batch_mod;  /* batch entry used by decoder row r: r % batch_mod */
  int32_t capacity;   /* tokens stored per batch entry (loads are clamped to it) */
  const int32_t* len; /* [rows] valid prefix lengths (device), NULL = capacity */
  int32_t causal;     /* key j visible to query i iff j <= i (encoder self-attention) */
} EchoKVSegment;

typedef struct {
  int32_t dtype;
  int32_t rows, n_q, heads, nseg;
  const void* q; int64_t q_ld_tok, q_ld_batch;
  const void* gate; int64_t g_ld_tok, g_ld_batch;  /* out *= sigmoid(gate) (model.py:157,264); NULL = none */
  void* out; int64_t o_ld_tok, o_ld_batch;
  float scale;              /* softmax scale, 1/sqrt(128) */
  EchoKVSegment seg[4];     /* [self | latent | text | speaker] */
  int32_t q_batch_mod;      /* q and gate of output row r are row r % q_batch_mod (0 = row r): the CFG
                               batch's identical layer-0 row groups (inference.py:516) read one copy */
} EchoAttnArgs;

/* Replaces the KV concat + F.scaled_dot_product_attention + sigmoid gate of
 * JointAttention.forward (model.py:237-264) and SelfAttention.forward (model.py:144-157). */
int echo_attention(const EchoAttnArgs* args, void* stream);

/* Split-KV form of echo_attention for launches that leave most CUs idle (B = 1 sampler steps,
 * blockwise blocks): each (128-query block, row, head) item's key tiles are split over `nsplit`
 * workgroups that store unnormalised partials (O fp32, running max, row sum) into `ws`, and a
 * combine pass merges
 * them, normalises, gates and stores `out` (same roundings as echo_attention;
 * only the fp32 summation order over keys differs). nsplit <= 1 runs echo_attention.
 * `ws`: device, 16-B aligned, >= echo_attention_split_ws_bytes(args, nsplit) bytes.
 * Replaces the same reference lines as echo_attention (model.py:237-264, 144-157). */
int echo_attention_split(const EchoAttnArgs* args, int32_t nsplit, void* ws, int64_t ws_bytes, void* stream);
int64_t echo_attention_split_ws_bytes(const EchoAttnArgs* args, int32_t nsplit);
/* In-launch hand-offs (round 6) — DIAGNOSTICS BUILD (ECHO_DIAG=1) ONLY: measured slower end to end than the
 * kernel boundaries they remove (profiles/r6_inlaunch_ab.jsonl), so the product library
 * refuses a non-NULL buffer with ECHO_EINVAL and echo_attention_merge_in_launch answers 0 there.
 * `sync`: a caller-owned device buffer of `words` uint32 (64-B aligned, zero before
 * its first use, never used by two launches that can run at the same time — e.g. one per captured plan / stream)
 * holding the arrival counters of merges done inside one launch; every such launch leaves it zero again.
 * NULL / 0 (default) = off. While it is set, echo_attention_split merges the splits inside its launch when every
 * split of every item can be resident at once (at most one workgroup per CU) — one kernel instead of the split
 * kernel + combine pass — and split-K gated-residual GEMMs whose grid fits finish inside their launch (one kernel
 * instead of GEMM + finish pass); bitwise the same output. Process-global (like echo_set_policy_rows); a captured graph
 * keeps the pointer set when it was captured. Word 0 becomes non-zero if a bounded wait ever gave up (never in a
 * correct run: tests read it). */
int echo_set_sync_buffer(uint32_t* sync, int64_t words);
/* Host-only: 1 if echo_attention_split(args, nsplit, ...) would merge inside its launch with the current buffer. */
int32_t echo_attention_merge_in_launch(const EchoAttnArgs* args, int32_t nsplit);
/* Host policy: the split count echo_attention_split should use for these shapes (1 = none). */
int32_t echo_attention_pick_split(const EchoAttnArgs* args);
/* Diagnostics: force the policy's answer (0/1 = never split, 2..16), -1 = back to the policy. */
int echo_attention_set_split(int32_t nsplit);
/* Diagnostics: 1 (default) = non-causal bf16 launches run the asm-owned software-pipelined kernel
 * (attn_pl_kernel, bitwise equal to the compiler-scheduled one), 0 = the compiler-scheduled kernel for
 * every launch (A/B measurements); 2 = attn_w64_kernel (one wave per SIMD, 64 queries per wave; measured
 * slower) in the diagnostics build (ECHO_DIAG=1) only — the product library refuses 2 with ECHO_EINVAL. */
int echo_attention_set_pipeline(int32_t on);

/* Diagnostics only (tools/bench_attn.py, tools/attn_timeline.py; never on the sampling path):
 * measurement variants of the bf16 attention kernel. variant 0 = the production kernel;
 * ablation != 0 removes parts of the work (results are then WRONG, timing only); ablation bit 128
 * records per-workgroup s_memrealtime stamps into `stamps` (device, [workgroups][6] uint64:
 * entry, prologue landed, tile loop done, exit, tiles, XCD); bit 512 (with 128) additionally
 * records per-tile phase cycles of workgroup 0 after that area ([4 waves][64][6]).
 * The product library accepts variant 0 and 11 (attn_pl_kernel) with ablation 0 and refuses everything
 * else with ECHO_EINVAL; the diagnostics build (ECHO_DIAG=1) has every variant and ablation.
 * Variants/bits: csrc/attention.hip. */
int echo_attention_variant(const EchoAttnArgs* args, int32_t variant, int32_t ablation, uint64_t* stamps,
                           void* stream);

/* RMSNorm(x)*w in fp32, cast back (model.py:99-104). Row stride in elements. */
int echo_rmsnorm(int32_t dtype, const void* x, int64_t ldx, const void* w, void* y, int64_t ldy,
                 int32_t rows, int32_t dim, float eps, void* stream);

/* LowRankAdaLN normalisation tail: y = round((x*rsqrt(mean x^2+eps))*scale1 + shift)
 * with precomputed scale1 = round(scale+1) and shift (model.py:76-83). Row r uses the
 * vectors at offset (r / rows_per_vec) * vec_stride (rows_per_vec <= 0: one vector). */
int echo_adaln_modulate(int32_t dtype, const void* x, void* y, int32_t rows, int32_t dim,
                        const void* shift, const void* scale1, int32_t rows_per_vec,
                        int64_t vec_stride, float eps, void* stream);

/* Per-head RMSNorm (+ RoPE on heads [0, rope_heads)) applied in place to `nblk`
 * column blocks of `heads*128` elements: block b starts at column col0 + b*col_stride
 * and uses norm weight w + b*w_stride ([heads,128]). Position of row i is
 * pos0 + pos_mult*(i % seq_len); rope table = float2 (cos,sin) [positions][64].
 * Covers q_norm/k_norm + _apply_rotary_half / apply_rotary_emb (model.py:138-142,
 * 221-232,274,281,289-291). rope_heads = 0 disables RoPE. */
int echo_head_norm_rope(int32_t dtype, void* x, int64_t ldx, int32_t rows, int32_t heads,
                        int32_t nblk, int64_t col0, int64_t col_stride, const void* w, int64_t w_stride,
                        const float* rope, int32_t rope_heads, int32_t seq_len, int32_t pos0,
                        int32_t pos_mult, float eps, void* stream);

/* Timestep embedding [cos|sin](float(t_s) * freqs) cast to dtype (model.py:27-43).
 * t: [S] floats already rounded to the model dtype; freqs: [half] fp32; out [S, 2*half]. */
int echo_timestep_embedding(int32_t dtype, const float* t, const float* freqs, void* out,
                            int32_t S, int32_t half, void* stream);

/* y = round(silu(x)) elementwise over a [rows, cols] block with strides (model.py:72-74). */
int echo_silu(int32_t dtype, const void* x, int64_t ldx, void* y, int64_t ldy, int32_t rows,
              int32_t cols, void* stream);

/* AdaLN table finish: raw [n_ada][S][3][D] (shift, scale, gate after the low-rank
 * refinement) -> table [S][n_ada][3][D] with (shift, round(scale+1), round(tanh(gate)))
 * (model.py:72-81). */
int echo_adaln_finish(int32_t dtype, const void* raw, void* table, int32_t n_ada, int32_t S,
                      int32_t D, void* stream);

/* Sampler state -> model input: out[c*B*N + i][0:C] = round(x[i][0:C]), zero-padded to
 * ld_out columns, for c in [0, copies) (torch.cat([x,x,x]).to(dtype), inference.py:516,533). */
int echo_latent_to_input(int32_t dtype, const float* x, void* out, int32_t rows, int32_t C,
                         int32_t ld_out, int32_t copies, void* stream);

/* Fused CFG combine + temporal score rescale + Euler update on the fp32 state
 * (inference.py:526-530,431-443,542-543,558). v: [R][n] with R = 3 (cfg) or 1 blocks
 * of n = B*N*80 elements. Scalars precomputed on the host in fp32 exactly as the
 * reference computes them. */
typedef struct {
  int32_t has_cfg; float cfg_text, cfg_speaker;
  int32_t rescale; float omt, ratio, inv_omt;   /* 1-t, ratio, 1/(1-t) */
  float dt;                                     /* t_next - t */
} EchoStepArgs;
int echo_euler_step(float* x, const float* v, int64_t n, const EchoStepArgs* a, void* stream);

/* Byte-embedding gather: out[i] = table[ids[i]] (nn.Embedding, model.py:403,420). */
int echo_embed(int32_t dtype, const int32_t* ids, const void* table, void* out, int32_t n,
               int32_t dim, void* stream);

/* In-place x[r][0:cols] = round(x * scale) on a strided block (KV speaker scaling,
 * Tensor.mul_ on bf16, inference.py:420-428). */
int echo_scale_rows(int32_t dtype, void* x, int64_t ldx, int32_t rows, int32_t cols, float scale,
                    void* stream);

/* fp32 -> dtype cast of n elements (speaker_latent.to(dtype), inference.py:483). */
int echo_cast_from_f32(int32_t dtype, const float* x, void* y, int64_t n, void* stream);

/* ---- Fish-S1-DAC output path (csrc/codec.hip). Activations are
 * channels-last [batch][rows][C]; s* arguments are per-item strides in elements. */

/* ae_decode's PCA inverse (inference.py:233): out[r][d] = (lat[r]/scale) . comps[:, d] + mean[d],
 * fp32 math, stored in dtype. lat [rows, K] fp32, comps [K, D] fp32, mean [D] fp32. */
int echo_pca_inverse(int32_t dtype, const float* lat, const float* comps, const float* mean, float scale,
                     void* out, int32_t rows, int32_t K, int32_t D, void* stream);
/* Snake1d (autoencoder.py:97-108): y = x + (alpha+1e-9)^-1 sin(alpha x)^2 per channel; C % 8 == 0. */
int echo_snake(int32_t dtype, const void* x, int64_t ldx, int64_t sx, void* y, int64_t ldy, int64_t sy,
               const void* alpha, int32_t rows, int32_t C, int32_t batch, void* stream);
/* ConvNeXtBlock head (autoencoder.py:360-364): causal depthwise conv k7 + bias (w_dw [C][7]), then
 * LayerNorm over C (eps) with ln_w / ln_b. Rows t < 0 of the conv read as zero. C <= 2048. */
int echo_dwconv_layernorm(int32_t dtype, const void* x, int64_t ldx, int64_t sx, void* y, int64_t ldy, int64_t sy,
                          const void* w_dw, const void* b_dw, const void* ln_w, const void* ln_b, int32_t rows,
                          int32_t C, int32_t batch, float eps, void* stream);
/* RMSNorm of the AE transformer (autoencoder.py:720-731): cast(x * rsqrt(mean(x^2)+eps)) * w. */
int echo_ae_rmsnorm(int32_t dtype, const void* x, int64_t ldx, const void* w, void* y, int64_t ldy, int32_t rows,
                    int32_t dim, float eps, void* stream);
/* apply_rotary_emb (autoencoder.py:815-826) in place on interleaved pairs of [rows][heads*hd];
 * table bf16 [npos][hd/2][2] (cos, sin), position = row % seq_len. */
int echo_rope_pairs(int32_t dtype, void* x, int64_t ld, int32_t rows, int32_t heads, int32_t hd,
                    const void* table_bf16, int32_t seq_len, void* stream);
/* Window-limited causal attention (autoencoder.py:663-706,762-773): qkv [batch*T][3*heads*64]
 * (q | k | v, row stride ld), out [batch*T][heads*64]; query t sees keys max(0,t-window+1)..t.
 * head_dim == 64, any window (128 for pre/post_module, 512 for the encoder transformer). */
int echo_window_attention(int32_t dtype, const void* qkv, int64_t ld, void* out, int64_t ldo, int32_t batch,
                          int32_t T, int32_t heads, int32_t head_dim, int32_t window, void* stream);
/* Decoder tail (autoencoder.py:995-996 + .float()): y[t] = tanh(conv_k7(s)[t] + bias) on the
 * Snake'd input s (>= 6 zero rows before t = 0 in its buffer); w [7][C] tap-major; y fp32. */
int echo_conv_out_tanh(int32_t dtype, const void* s, int64_t lds, int64_t ss, const void* w, const void* bias,
                       float* y, int64_t sy, int32_t rows, int32_t C, int32_t batch, void* stream);
/* find_flattening_point (inference.py:315-330) of x [L][D] fp32 -> *out (device int32). */
int echo_flattening_point(const float* x, int32_t L, int32_t D, int32_t window, float std_threshold, float target,
                          int32_t* out, void* stream);

/* ---- Fish-S1-DAC input path (csrc/codec.hip). */

/* Encoder input conv (autoencoder.py:913, CausalWNConv1d(1, C, 7)): x [batch][L] audio (dtype,
 * per-item stride sx) -> y rows [batch][L][C] (row stride ldy, item stride sy). */
int echo_conv_in(int32_t dtype, const void* x, int64_t sx, const void* w, const void* bias, void* y, int64_t ldy,
                 int64_t sy, int32_t L, int32_t C, int32_t batch, void* stream);

/* Residual-VQ weights in dtype, weight norm folded: stage 0 = semantic quantizer, 1.. = residual
 * quantizers (autoencoder.py:376-427). codebook_sizes[q] entries per stage, tables concatenated. */
typedef struct EchoRvqWeights {
  const void* w_in;    /* [nq][codebook_dim][D]  in_proj (WN conv k1) */
  const void* b_in;    /* [nq][codebook_dim] */
  const void* cbn;     /* F.normalize(codebook) rows, [sum sizes][codebook_dim] */
  const void* csq;     /* cbn.pow(2).sum(1) as the reference rounds it, [sum sizes] */
  const void* cb;      /* raw codebook rows (embedding lookup), [sum sizes][codebook_dim] */
  const void* w_out;   /* [nq][D][codebook_dim]  out_proj (WN conv k1) */
  const void* b_out;   /* [nq][D] */
  int32_t codebook_sizes[16];
  int32_t nq;
  int32_t codebook_dim; /* 8 */
} EchoRvqWeights;

/* DownsampleResidualVectorQuantize code path + DAC.encode_zq + ae_encode's PCA projection
 * (autoencoder.py:451-471,130-157,1117-1126; inference.py:223-229), one workgroup per frame:
 * z [rows][D] (pre_module output, rows = batch*T, D == 1024) -> codes [batch][nq][T] int32,
 * zq [rows][D] (dtype, optional: NULL), lat [rows][npca] fp32 = ((zq - mean) @ comps^T) * scale. */
int echo_rvq_encode(int32_t dtype, const void* z, int64_t ldz, int32_t rows, int32_t T, int32_t D,
                    const EchoRvqWeights* w, int32_t* codes, void* zq, int64_t ldq, const float* comps,
                    const float* mean, float scale, float* lat, int32_t npca, void* stream);

/* Library identification (build stamp) — for load checks. */
const char* echo_version(void);

/* ABI revision of the argument structs in this header. Bumped whenever a struct's layout changes
 * (4: EchoAttnArgs gained the trailing q_batch_mod; 5: EchoGemmArgs gained the mod_* fields of the fused
 * residual + AdaLN). A binding built against an older header must
 * refuse to run: check echo_abi_version() == ECHO_ABI_VERSION and the struct sizes below at load. */
#define ECHO_ABI_VERSION 6
int32_t echo_abi_version(void);
/* sizeof() of an argument struct as this library was compiled: 0 EchoGemmArgs, 1 EchoAttnArgs,
 * 2 EchoKVSegment, 3 EchoStepArgs, 4 EchoRvqWeights; -1 for an unknown id. */
int64_t echo_abi_struct_size(int32_t which);

#ifdef __cplusplus
}
#endif
#endif /* ECHO_HIP_H */

// torch_ops.cpp — PyTorch-ROCm custom-op registration of the Echo-TTS sampling path
// (TORCH_LIBRARY(echo_hip)).
//
// Every op validates its tensors on the host (TORCH_CHECK -> Python RuntimeError), derives the
// plain pointers / strides of the C ABI (include/echo_hip.h) and launches on the current HIP stream
// of the tensors' device. No op synchronises the host, so all of them are capturable in a hipGraph.
// Functional ops allocate their outputs through the PyTorch caching allocator; the `*_out` / `*_`
// forms write into caller-owned buffers (the engine's static workspace). The CPU dispatch key is
// registered to fail loudly: the sampling path has no CPU fallback. Fake (meta) kernels live in
// echo-tts_amd/ops.py (torch.library.register_fake), so torch.compile can trace through the ops.
//
// Reference ops each entry replaces (file:line of /root/reference):
//   gemm / gemm_out        every nn.Linear + fused tails   model.py:56-62,118-122,177-197,303-308,385-388,602-604
//   gemm_resid_norm_out    gated residual + next AdaLN     model.py:385,388 + 76-81
//   joint_attention(_out)  KV concat + SDPA + sigmoid gate model.py:237-264, 144-157; inference.py:409-417
//   rmsnorm(_out)          RMSNorm                         model.py:99-104
//   norm_modulate(_out)    LowRankAdaLN normalisation tail model.py:76-83
//   head_norm_rope_        q/k norm + RoPE                 model.py:138-142,221-232,274-291
//   timestep_embedding     get_timestep_embedding          model.py:27-43
//   silu(_out)             nn.SiLU / F.silu               model.py:72-74,532-538
//   adaln_finish(_out)     (scale+1), tanh(gate)           model.py:72-81
//   latent_to_input(_out)  torch.cat([x]*3).to(dtype)      inference.py:516,533
//   euler_cfg_step(_)      CFG combine + rescale + Euler   inference.py:526-530,431-443,558
//   embed(_out)            nn.Embedding (text bytes)       model.py:403,420
//   scale_rows_            _multiply_kv_cache mul_          inference.py:420-428
//   cast_from_f32(_out)    speaker_latent.to(dtype)        inference.py:483
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <string>
#include <vector>

#include "echo_hip.h"

namespace {

using at::Tensor;
using c10::optional;

const char* err_name(int rc) {
  switch (rc) {
    case ECHO_EINVAL: return "ECHO_EINVAL";
    case ECHO_EDTYPE: return "ECHO_EDTYPE";
    case ECHO_ESHAPE: return "ECHO_ESHAPE";
    case ECHO_EALIGN: return "ECHO_EALIGN";
    default: return "hipError";
  }
}

void check_rc(int rc, const char* what) {
  TORCH_CHECK(rc == 0, what, " failed: ", err_name(rc), " (", rc, ")");
}

void* stream_of(const Tensor& t) { return (void*)c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

void need_dev(const Tensor& ref, const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "echo_hip: ", name, " must be a device tensor (no CPU fallback)");
  TORCH_CHECK(t.device() == ref.device(), "echo_hip: ", name, " is on ", t.device(), ", expected ", ref.device());
}

void need_dev(const Tensor& ref, const optional<Tensor>& t, const char* name) {
  if (t.has_value() && t->defined()) need_dev(ref, *t, name);
}

const void* ptr(const optional<Tensor>& t) { return (t.has_value() && t->defined()) ? t->data_ptr() : nullptr; }

int32_t dt_of(const Tensor& t, const char* name) {
  if (t.scalar_type() == at::kBFloat16) return ECHO_BF16;
  if (t.scalar_type() == at::kFloat) return ECHO_F32;
  TORCH_CHECK(false, "echo_hip: ", name, " has unsupported dtype ", t.scalar_type(), " (bfloat16 or float32)");
}

// (batch, rows, cols, ld, batch_stride) of a 2-D / 3-D row-major view with a contiguous last dim
struct Mat {
  int64_t batch, rows, cols, ld, sb;
};

Mat mat(const Tensor& t, const char* name) {
  TORCH_CHECK(t.dim() == 2 || t.dim() == 3, "echo_hip: ", name, " must be 2-D or 3-D, got ", t.sizes());
  TORCH_CHECK(t.stride(-1) == 1 || t.size(-1) == 1, "echo_hip: ", name, " must have a contiguous last dim");
  if (t.dim() == 2) return {1, t.size(0), t.size(1), t.stride(0), 0};
  return {t.size(0), t.size(1), t.size(2), t.stride(1), t.stride(0)};
}

int32_t i32(int64_t v, const char* what) {
  TORCH_CHECK(v >= INT32_MIN && v <= INT32_MAX, "echo_hip: ", what, " out of int32 range");
  return (int32_t)v;
}

// ------------------------------------------------------------------------------------------ GEMM

struct GemmSpec {
  int64_t M, N, K, batch, n_out;
  bool f32out;
};

// hn = [heads, nblk, w_stride, rope_heads, seq_len, pos0, pos_mult]; conv = [] or [taps, dilation]
GemmSpec gemm_spec(const Tensor& a, const Tensor& w, int64_t epilogue, at::IntArrayRef conv) {
  TORCH_CHECK(a.scalar_type() == w.scalar_type(), "echo_hip.gemm: a/w dtype mismatch");
  const Mat A = mat(a, "a"), Wm = mat(w, "w");
  int64_t K = A.cols;
  if (!conv.empty()) {
    TORCH_CHECK(conv.size() == 2 && conv[0] > 0 && conv[1] > 0, "echo_hip.gemm: conv = [taps, dilation]");
    K = A.cols * conv[0];
    TORCH_CHECK(a.storage_offset() >= (conv[0] - 1) * conv[1] * A.ld,
                "echo_hip.gemm: conv input needs (taps-1)*dilation rows of its buffer before row 0");
  }
  TORCH_CHECK(Wm.cols == K, "echo_hip.gemm: K mismatch ", K, " vs ", Wm.cols);
  const int64_t batch = std::max(A.batch, Wm.batch);
  TORCH_CHECK((A.batch == 1 || A.batch == batch) && (Wm.batch == 1 || Wm.batch == batch),
              "echo_hip.gemm: batch mismatch");
  TORCH_CHECK(epilogue >= ECHO_EPI_STORE && epilogue <= ECHO_EPI_HEADNORM, "echo_hip.gemm: bad epilogue ", epilogue);
  const int64_t n_out = epilogue == ECHO_EPI_SWIGLU ? Wm.rows / 2 : Wm.rows;
  return {A.rows, Wm.rows, K, batch, n_out, epilogue == ECHO_EPI_F32OUT};
}

// the next AdaLN fused behind a gated residual (gemm_resid_norm_out)
struct ModArgs {
  const Tensor& xn;
  const Tensor& shift;
  const Tensor& scale1;
  double eps;
};

void gemm_launch(const Tensor& a, const Tensor& w, const Tensor& out, const optional<Tensor>& bias,
                 int64_t epilogue, const optional<Tensor>& aux, const optional<Tensor>& gate, int64_t act,
                 double out_div, int64_t tile, const optional<Tensor>& hn_w, const optional<Tensor>& hn_rope,
                 at::IntArrayRef hn, double hn_eps, const optional<Tensor>& act_alpha, at::IntArrayRef conv,
                 const ModArgs* mod = nullptr) {
  need_dev(a, a, "a");
  need_dev(a, w, "w");
  need_dev(a, out, "out");
  need_dev(a, bias, "bias");
  need_dev(a, aux, "aux");
  need_dev(a, gate, "gate");
  need_dev(a, hn_w, "hn_w");
  need_dev(a, hn_rope, "hn_rope");
  need_dev(a, act_alpha, "act_alpha");
  const bool headnorm = !hn.empty();
  TORCH_CHECK(!headnorm || epilogue == ECHO_EPI_STORE || epilogue == ECHO_EPI_HEADNORM,
              "echo_hip.gemm: head norm replaces the store epilogue");
  if (headnorm) epilogue = ECHO_EPI_HEADNORM;
  const GemmSpec s = gemm_spec(a, w, epilogue, conv);
  const Mat A = mat(a, "a"), Wm = mat(w, "w"), O = mat(out, "out");
  const auto odt = s.f32out ? at::kFloat : a.scalar_type();
  TORCH_CHECK(O.rows == s.M && O.cols == s.n_out && out.scalar_type() == odt, "echo_hip.gemm: out ", out.sizes(),
              "/", out.scalar_type(), " != [", s.M, ", ", s.n_out, "]/", odt);
  TORCH_CHECK(O.batch == s.batch || (s.batch == 1 && out.dim() == 2), "echo_hip.gemm: out batch mismatch");
  EchoGemmArgs g{};
  g.dtype = dt_of(a, "a");
  g.M = i32(s.M, "M");
  g.N = i32(s.N, "N");
  g.K = i32(s.K, "K");
  g.batch = i32(s.batch, "batch");
  g.A = a.data_ptr();
  g.lda = A.ld;
  g.stride_a = a.dim() == 3 ? A.sb : 0;
  g.W = w.data_ptr();
  g.ldw = Wm.ld;
  g.stride_w = w.dim() == 3 ? Wm.sb : 0;
  g.C = out.data_ptr();
  g.ldc = O.ld;
  g.stride_c = out.dim() == 3 ? O.sb : 0;
  if (bias.has_value() && bias->defined()) {
    const Tensor& b = *bias;
    TORCH_CHECK(b.scalar_type() == a.scalar_type() && b.size(-1) == s.N && b.stride(-1) == 1 && b.dim() <= 2,
                "echo_hip.gemm: bias must be [(B,)N] of the model dtype");
    g.bias = b.data_ptr();
    g.stride_bias = b.dim() == 2 ? b.stride(0) : 0;
  }
  if (epilogue == ECHO_EPI_RESID) {
    TORCH_CHECK(aux.has_value() && aux->defined(), "echo_hip.gemm: RESID needs aux");
    const Mat X = mat(*aux, "aux");
    TORCH_CHECK(X.rows == s.M && X.cols == s.n_out && aux->scalar_type() == a.scalar_type(),
                "echo_hip.gemm: aux shape/dtype");
    g.aux = aux->data_ptr();
    g.ld_aux = X.ld;
    g.stride_aux = aux->dim() == 3 ? X.sb : 0;
    if (gate.has_value() && gate->defined()) {
      const Tensor& gt = *gate;
      TORCH_CHECK(gt.size(-1) == s.N && gt.stride(-1) == 1 && gt.scalar_type() == a.scalar_type() && gt.dim() <= 2,
                  "echo_hip.gemm: gate must be [(B,)N]");
      g.gate = gt.data_ptr();
      g.stride_gate = gt.dim() == 2 ? gt.stride(0) : 0;
    }
  }
  g.epilogue = (int32_t)epilogue;
  g.act = i32(act, "act");
  g.out_div = (float)out_div;
  g.tile = i32(tile, "tile");
  if (act == ECHO_ACT_SNAKE) {
    TORCH_CHECK(act_alpha.has_value() && act_alpha->defined() && act_alpha->scalar_type() == a.scalar_type() &&
                    act_alpha->numel() == s.N && act_alpha->is_contiguous(),
                "echo_hip.gemm: ACT_SNAKE needs a contiguous alpha [N] of the model dtype");
    g.act_alpha = act_alpha->data_ptr();
  }
  if (!conv.empty()) {
    g.conv_c = i32(A.cols, "conv_c");
    g.conv_taps = i32(conv[0], "taps");
    g.conv_dil = i32(conv[1], "dilation");
  }
  if (headnorm) {
    TORCH_CHECK(hn.size() == 7, "echo_hip.gemm: hn = [heads, nblk, w_stride, rope_heads, seq_len, pos0, pos_mult]");
    TORCH_CHECK(hn_w.has_value() && hn_w->defined() && hn_w->scalar_type() == a.scalar_type(),
                "echo_hip.gemm: head-norm weight must be the model dtype");
    TORCH_CHECK(!(hn_rope.has_value() && hn_rope->defined()) || hn_rope->scalar_type() == at::kFloat,
                "echo_hip.gemm: rope table must be float32");
    g.hn_w = hn_w->data_ptr();
    g.hn_heads = i32(hn[0], "hn heads");
    g.hn_nblk = i32(hn[1], "hn nblk");
    g.hn_w_stride = hn[2];
    g.hn_rope = (const float*)ptr(hn_rope);
    g.hn_rope_heads = i32(hn[3], "hn rope_heads");
    g.hn_seq_len = i32(hn[4], "hn seq_len");
    g.hn_pos0 = i32(hn[5], "hn pos0");
    g.hn_pos_mult = i32(hn[6], "hn pos_mult");
    g.hn_eps = (float)hn_eps;
  }
  if (mod) {
    need_dev(a, mod->xn, "xn");
    need_dev(a, mod->shift, "shift");
    need_dev(a, mod->scale1, "scale1");
    TORCH_CHECK(epilogue == ECHO_EPI_RESID && s.batch == 1 && out.is_contiguous() && mod->xn.is_contiguous() &&
                    mod->xn.sizes() == out.sizes() && mod->xn.scalar_type() == a.scalar_type(),
                "echo_hip.gemm_resid_norm: one batch, contiguous h / xn of equal shape and the model dtype");
    {
      const uintptr_t nb = (uintptr_t)out.numel() * out.element_size();
      const uintptr_t h0 = (uintptr_t)out.data_ptr(), x0 = (uintptr_t)mod->xn.data_ptr();
      TORCH_CHECK(x0 >= h0 + nb || h0 >= x0 + nb, "echo_hip.gemm_resid_norm: xn overlaps h");
    }
    for (const Tensor* v : {&mod->shift, &mod->scale1})
      TORCH_CHECK(v->dim() == 1 && v->numel() == s.N && v->is_contiguous() && v->scalar_type() == a.scalar_type(),
                  "echo_hip.gemm_resid_norm: shift / scale1 must be contiguous [N] of the model dtype");
    g.mod_out = mod->xn.data_ptr();
    g.ld_mod = s.N;
    g.mod_shift = mod->shift.data_ptr();
    g.mod_scale1 = mod->scale1.data_ptr();
    g.mod_eps = (float)mod->eps;
  }
  c10::DeviceGuard guard(a.device());
  // under-filled launches may split K (echo_gemm_ws_bytes > 0): the fp32 partial slabs come from the
  // caching allocator (graph-private pool under hipGraph capture)
  const int64_t wsb = echo_gemm_ws_bytes(&g);
  if (wsb > 0) {
    Tensor ws = at::empty({(wsb + 3) / 4}, a.options().dtype(at::kFloat));
    check_rc(echo_gemm_ws(&g, ws.data_ptr(), wsb, stream_of(a)), "echo_hip.gemm");
  } else {
    check_rc(echo_gemm(&g, stream_of(a)), "echo_hip.gemm");
  }
}

Tensor gemm(const Tensor& a, const Tensor& w, const optional<Tensor>& bias, int64_t epilogue,
            const optional<Tensor>& aux, const optional<Tensor>& gate, int64_t act, double out_div, int64_t tile,
            const optional<Tensor>& hn_w, const optional<Tensor>& hn_rope, at::IntArrayRef hn, double hn_eps,
            const optional<Tensor>& act_alpha, at::IntArrayRef conv) {
  const GemmSpec s = gemm_spec(a, w, hn.empty() ? epilogue : (int64_t)ECHO_EPI_HEADNORM, conv);
  auto opts = a.options().dtype(s.f32out ? at::kFloat : a.scalar_type());
  Tensor out = (s.batch == 1 && a.dim() == 2) ? at::empty({s.M, s.n_out}, opts) : at::empty({s.batch, s.M, s.n_out}, opts);
  gemm_launch(a, w, out, bias, epilogue, aux, gate, act, out_div, tile, hn_w, hn_rope, hn, hn_eps, act_alpha, conv);
  return out;
}

void gemm_out(const Tensor& a, const Tensor& w, const Tensor& out, const optional<Tensor>& bias, int64_t epilogue,
              const optional<Tensor>& aux, const optional<Tensor>& gate, int64_t act, double out_div, int64_t tile,
              const optional<Tensor>& hn_w, const optional<Tensor>& hn_rope, at::IntArrayRef hn, double hn_eps,
              const optional<Tensor>& act_alpha, at::IntArrayRef conv) {
  gemm_launch(a, w, out, bias, epilogue, aux, gate, act, out_div, tile, hn_w, hn_rope, hn, hn_eps, act_alpha, conv);
}

// h = round(h + round(gate * (a @ w^T))), then xn = round(rmsnorm(h) * scale1 + shift): a gated residual
// (model.py:385,388) followed by the next LowRankAdaLN's normalisation (model.py:76-81) — fused into one
// finish kernel on under-filled launches, the two kernels otherwise (bitwise equal)
void gemm_resid_norm_out(const Tensor& a, const Tensor& w, const Tensor& h, const optional<Tensor>& gate,
                         const Tensor& shift, const Tensor& scale1, double eps, const Tensor& xn, int64_t tile) {
  const ModArgs m{xn, shift, scale1, eps};
  gemm_launch(a, w, h, c10::nullopt, ECHO_EPI_RESID, h, gate, 0, 0.0, tile, c10::nullopt, c10::nullopt, {}, 0.0,
              c10::nullopt, {}, &m);
}

// ------------------------------------------------------------------------------------- attention

std::pair<int64_t, int64_t> head_view(const Tensor& t, const char* name) {
  TORCH_CHECK(t.dim() == 4 && t.size(3) == 128 && t.stride(3) == 1 && (t.stride(2) == 128 || t.size(2) == 1),
              "echo_hip.joint_attention: ", name, " must be [B, L, H, 128] with contiguous heads, got ", t.sizes(),
              " strides ", t.strides());
  return {t.stride(1), t.stride(0)};
}

EchoAttnArgs attn_args(const Tensor& q, const optional<Tensor>& gate, at::TensorList seg_k, at::TensorList seg_v,
                       const c10::List<optional<Tensor>>& seg_len, at::IntArrayRef seg_batch_mod,
                       at::IntArrayRef seg_causal, const Tensor& out, double scale) {
  const size_t ns = seg_k.size();
  TORCH_CHECK(ns >= 1 && ns <= 4, "echo_hip.joint_attention: 1-4 segments");
  TORCH_CHECK(seg_v.size() == ns && seg_len.size() == ns && seg_batch_mod.size() == ns && seg_causal.size() == ns,
              "echo_hip.joint_attention: per-segment lists must have equal lengths");
  need_dev(q, q, "q");
  need_dev(q, out, "out");
  need_dev(q, gate, "gate");
  EchoAttnArgs a{};
  a.dtype = dt_of(q, "q");
  // out rows may be a multiple of q's: output row r reads q / gate row r % q.size(0)
  // (the identical CFG row groups of layer 0 share one q copy, EchoAttnArgs.q_batch_mod)
  TORCH_CHECK(q.dim() == 4 && out.dim() == 4 && q.size(0) > 0 && out.size(0) % q.size(0) == 0 &&
                  out.sizes().slice(1) == q.sizes().slice(1) && out.scalar_type() == q.scalar_type(),
              "echo_hip.joint_attention: out must match q (rows: a multiple of q's)");
  a.rows = i32(out.size(0), "rows");
  a.q_batch_mod = out.size(0) == q.size(0) ? 0 : i32(q.size(0), "q rows");
  a.n_q = i32(q.size(1), "n_q");
  a.heads = i32(q.size(2), "heads");
  a.nseg = (int32_t)ns;
  a.q = q.data_ptr();
  std::tie(a.q_ld_tok, a.q_ld_batch) = head_view(q, "q");
  a.out = out.data_ptr();
  std::tie(a.o_ld_tok, a.o_ld_batch) = head_view(out, "out");
  if (gate.has_value() && gate->defined()) {
    TORCH_CHECK(gate->sizes() == q.sizes() && gate->scalar_type() == q.scalar_type(),
                "echo_hip.joint_attention: gate must match q");
    a.gate = gate->data_ptr();
    std::tie(a.g_ld_tok, a.g_ld_batch) = head_view(*gate, "gate");
  }
  a.scale = (float)scale;
  for (size_t i = 0; i < ns; ++i) {
    const Tensor &k = seg_k[i], &v = seg_v[i];
    need_dev(q, k, "segment k");
    need_dev(q, v, "segment v");
    TORCH_CHECK(k.scalar_type() == q.scalar_type() && v.scalar_type() == q.scalar_type(),
                "echo_hip.joint_attention: segment dtype");
    const auto kv = head_view(k, "k"), vv = head_view(v, "v");
    TORCH_CHECK(kv == vv && k.sizes() == v.sizes() && k.size(2) == q.size(2),
                "echo_hip.joint_attention: k/v of a segment must share shape and strides");
    EchoKVSegment& s = a.seg[i];
    s.k = k.size(1) == 0 ? nullptr : k.data_ptr();
    s.v = v.data_ptr();
    s.ld_tok = kv.first;
    s.ld_batch = kv.second;
    s.batch_mod = i32(seg_batch_mod[i] > 0 ? seg_batch_mod[i] : k.size(0), "batch_mod");
    TORCH_CHECK(s.batch_mod <= k.size(0), "echo_hip.joint_attention: batch_mod exceeds segment batch");
    s.capacity = i32(k.size(1), "capacity");
    const optional<Tensor> len = seg_len.get(i);
    if (len.has_value() && len->defined()) {
      need_dev(q, *len, "segment lens");
      TORCH_CHECK(len->scalar_type() == at::kInt && len->numel() >= out.size(0) && len->is_contiguous(),
                  "echo_hip.joint_attention: lens must be contiguous int32 [rows]");
      s.len = (const int32_t*)len->data_ptr();
    }
    s.causal = seg_causal[i] ? 1 : 0;
  }
  return a;
}

void joint_attention_out(const Tensor& q, const optional<Tensor>& gate, at::TensorList seg_k, at::TensorList seg_v,
                         const c10::List<optional<Tensor>>& seg_len, at::IntArrayRef seg_batch_mod,
                         at::IntArrayRef seg_causal, const Tensor& out, double scale) {
  EchoAttnArgs a = attn_args(q, gate, seg_k, seg_v, seg_len, seg_batch_mod, seg_causal, out, scale);
  c10::DeviceGuard guard(q.device());
  // launches that would leave most CUs idle run the split-KV form; its workspace comes from the
  // caching allocator (graph-private pool under hipGraph capture)
  const int32_t nsp = echo_attention_pick_split(&a);
  if (nsp > 1) {
    const int64_t bytes = echo_attention_split_ws_bytes(&a, nsp);
    Tensor ws = at::empty({(bytes + 3) / 4}, q.options().dtype(at::kFloat));
    check_rc(echo_attention_split(&a, nsp, ws.data_ptr(), bytes, stream_of(q)), "echo_hip.joint_attention");
  } else {
    check_rc(echo_attention(&a, stream_of(q)), "echo_hip.joint_attention");
  }
}

Tensor joint_attention(const Tensor& q, const optional<Tensor>& gate, at::TensorList seg_k, at::TensorList seg_v,
                       const c10::List<optional<Tensor>>& seg_len, at::IntArrayRef seg_batch_mod,
                       at::IntArrayRef seg_causal, double scale) {
  Tensor out = at::empty(q.sizes(), q.options());
  joint_attention_out(q, gate, seg_k, seg_v, seg_len, seg_batch_mod, seg_causal, out, scale);
  return out;
}

void attention_variant_out(const Tensor& q, const optional<Tensor>& gate, at::TensorList seg_k, at::TensorList seg_v,
                           const c10::List<optional<Tensor>>& seg_len, at::IntArrayRef seg_batch_mod,
                           at::IntArrayRef seg_causal, const Tensor& out, double scale, int64_t variant,
                           int64_t ablation, const optional<Tensor>& stamps) {
  EchoAttnArgs a = attn_args(q, gate, seg_k, seg_v, seg_len, seg_batch_mod, seg_causal, out, scale);
  need_dev(q, stamps, "stamps");
  c10::DeviceGuard guard(q.device());
  check_rc(echo_attention_variant(&a, i32(variant, "variant"), i32(ablation, "ablation"), (uint64_t*)ptr(stamps),
                                  stream_of(q)),
           "echo_hip.attention_variant");
}

// -------------------------------------------------------------------------------- norms and glue

void rmsnorm_out(const Tensor& x, const Tensor& w, double eps, const Tensor& out) {
  need_dev(x, x, "x");
  need_dev(x, w, "w");
  need_dev(x, out, "out");
  TORCH_CHECK(x.dim() == 2 && out.dim() == 2 && x.stride(1) == 1 && out.stride(1) == 1,
              "echo_hip.rmsnorm: x/out must be 2-D row-major views");
  TORCH_CHECK(out.sizes() == x.sizes() && out.scalar_type() == x.scalar_type() && w.scalar_type() == x.scalar_type() &&
                  w.numel() == x.size(1) && w.is_contiguous(),
              "echo_hip.rmsnorm: shapes/dtypes");
  c10::DeviceGuard guard(x.device());
  check_rc(echo_rmsnorm(dt_of(x, "x"), x.data_ptr(), x.stride(0), w.data_ptr(), out.data_ptr(), out.stride(0),
                        i32(x.size(0), "rows"), i32(x.size(1), "dim"), (float)eps, stream_of(x)),
           "echo_hip.rmsnorm");
}

Tensor rmsnorm(const Tensor& x, const Tensor& w, double eps) {
  Tensor out = at::empty(x.sizes(), x.options());
  rmsnorm_out(x, w, eps, out);
  return out;
}

// shift/scale1: [D] (one vector for all rows) or [V, D] (rows split evenly over V vectors)
void norm_modulate_out(const Tensor& x, const Tensor& shift, const Tensor& scale1, double eps, const Tensor& out) {
  need_dev(x, x, "x");
  need_dev(x, shift, "shift");
  need_dev(x, scale1, "scale1");
  need_dev(x, out, "out");
  TORCH_CHECK(x.is_contiguous() && out.is_contiguous() && out.sizes() == x.sizes() &&
                  out.scalar_type() == x.scalar_type(),
              "echo_hip.norm_modulate: contiguous x/out of equal shape and dtype");
  const int64_t D = x.size(-1), rows = x.numel() / D;
  TORCH_CHECK(shift.sizes() == scale1.sizes() && shift.strides() == scale1.strides() && shift.size(-1) == D &&
                  shift.stride(-1) == 1 && shift.dim() <= 2 && shift.scalar_type() == x.scalar_type() &&
                  scale1.scalar_type() == x.scalar_type(),
              "echo_hip.norm_modulate: shift/scale1 must be [D] or [V, D] with equal strides");
  int64_t rpv = 0, vstride = 0;
  if (shift.dim() == 2 && shift.size(0) > 1) {
    TORCH_CHECK(rows % shift.size(0) == 0, "echo_hip.norm_modulate: rows not divisible by vector count");
    rpv = rows / shift.size(0);
    vstride = shift.stride(0);
  }
  c10::DeviceGuard guard(x.device());
  check_rc(echo_adaln_modulate(dt_of(x, "x"), x.data_ptr(), out.data_ptr(), i32(rows, "rows"), i32(D, "dim"),
                               shift.data_ptr(), scale1.data_ptr(), i32(rpv, "rows_per_vec"), vstride, (float)eps,
                               stream_of(x)),
           "echo_hip.norm_modulate");
}

Tensor norm_modulate(const Tensor& x, const Tensor& shift, const Tensor& scale1, double eps) {
  Tensor out = at::empty(x.sizes(), x.options());
  norm_modulate_out(x, shift, scale1, eps, out);
  return out;
}

void head_norm_rope_(const Tensor& x, const Tensor& w, double eps, int64_t heads, int64_t nblk, int64_t col0,
                     int64_t col_stride, int64_t w_stride, const optional<Tensor>& rope, int64_t rope_heads,
                     int64_t seq_len, int64_t pos0, int64_t pos_mult) {
  need_dev(x, x, "x");
  need_dev(x, w, "w");
  need_dev(x, rope, "rope");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "echo_hip.head_norm_rope_: x must be a 2-D row-major view");
  TORCH_CHECK(w.scalar_type() == x.scalar_type(), "echo_hip.head_norm_rope_: weight dtype");
  TORCH_CHECK(col0 + (nblk - 1) * col_stride + heads * 128 <= x.size(1), "echo_hip.head_norm_rope_: columns exceed x");
  TORCH_CHECK(!(rope.has_value() && rope->defined()) || rope->scalar_type() == at::kFloat,
              "echo_hip.head_norm_rope_: rope table must be float32");
  c10::DeviceGuard guard(x.device());
  check_rc(echo_head_norm_rope(dt_of(x, "x"), x.data_ptr(), x.stride(0), i32(x.size(0), "rows"), i32(heads, "heads"),
                               i32(nblk, "nblk"), col0, col_stride, w.data_ptr(), w_stride, (const float*)ptr(rope),
                               i32(rope_heads, "rope_heads"), i32(seq_len, "seq_len"), i32(pos0, "pos0"),
                               i32(pos_mult, "pos_mult"), (float)eps, stream_of(x)),
           "echo_hip.head_norm_rope_");
}

Tensor timestep_embedding(const Tensor& t, const Tensor& freqs, at::ScalarType dtype) {
  need_dev(freqs, t, "t");
  need_dev(freqs, freqs, "freqs");
  TORCH_CHECK(t.scalar_type() == at::kFloat && freqs.scalar_type() == at::kFloat && t.is_contiguous() &&
                  freqs.is_contiguous(),
              "echo_hip.timestep_embedding: t and freqs must be contiguous float32");
  Tensor out = at::empty({t.numel(), 2 * freqs.numel()}, freqs.options().dtype(dtype));
  c10::DeviceGuard guard(t.device());
  check_rc(echo_timestep_embedding(dt_of(out, "out"), (const float*)t.data_ptr(), (const float*)freqs.data_ptr(),
                                   out.data_ptr(), i32(t.numel(), "S"), i32(freqs.numel(), "half"), stream_of(t)),
           "echo_hip.timestep_embedding");
  return out;
}

void silu_out(const Tensor& x, const Tensor& out) {
  need_dev(x, x, "x");
  need_dev(x, out, "out");
  TORCH_CHECK(x.dim() == 2 && out.dim() == 2 && x.stride(1) == 1 && out.stride(1) == 1 && out.sizes() == x.sizes() &&
                  out.scalar_type() == x.scalar_type(),
              "echo_hip.silu: 2-D row-major x/out of equal shape");
  c10::DeviceGuard guard(x.device());
  check_rc(echo_silu(dt_of(x, "x"), x.data_ptr(), x.stride(0), out.data_ptr(), out.stride(0), i32(x.size(0), "rows"),
                     i32(x.size(1), "cols"), stream_of(x)),
           "echo_hip.silu");
}

Tensor silu(const Tensor& x) {
  Tensor out = at::empty(x.sizes(), x.options());
  silu_out(x, out);
  return out;
}

// raw [n_ada, S, 3, D] -> table [S, n_ada, 3, D]
void adaln_finish_out(const Tensor& raw, const Tensor& table) {
  need_dev(raw, raw, "raw");
  need_dev(raw, table, "table");
  TORCH_CHECK(raw.dim() == 4 && raw.size(2) == 3 && raw.is_contiguous() && table.is_contiguous() &&
                  table.dim() == 4 && table.size(0) == raw.size(1) && table.size(1) == raw.size(0) &&
                  table.size(2) == 3 && table.size(3) == raw.size(3) && table.scalar_type() == raw.scalar_type(),
              "echo_hip.adaln_finish: raw [n_ada, S, 3, D] -> table [S, n_ada, 3, D]");
  c10::DeviceGuard guard(raw.device());
  check_rc(echo_adaln_finish(dt_of(raw, "raw"), raw.data_ptr(), table.data_ptr(), i32(raw.size(0), "n_ada"),
                             i32(raw.size(1), "S"), i32(raw.size(3), "D"), stream_of(raw)),
           "echo_hip.adaln_finish");
}

Tensor adaln_finish(const Tensor& raw) {
  Tensor t = at::empty({raw.size(1), raw.size(0), 3, raw.size(3)}, raw.options());
  adaln_finish_out(raw, t);
  return t;
}

// x fp32 [..., C] (rows = numel / C) -> out [copies * rows, ld] model dtype, zero-padded
void latent_to_input_out(const Tensor& x, int64_t copies, const Tensor& out) {
  need_dev(x, x, "x");
  need_dev(x, out, "out");
  TORCH_CHECK(x.scalar_type() == at::kFloat && x.is_contiguous(), "echo_hip.latent_to_input: x must be contiguous fp32");
  const int64_t C = x.size(-1), rows = x.numel() / C;
  TORCH_CHECK(out.dim() == 2 && out.is_contiguous() && out.size(0) >= copies * rows && out.size(1) >= C,
              "echo_hip.latent_to_input: out must be contiguous [>= copies*rows, >= C]");
  c10::DeviceGuard guard(x.device());
  check_rc(echo_latent_to_input(dt_of(out, "out"), (const float*)x.data_ptr(), out.data_ptr(), i32(rows, "rows"),
                                i32(C, "C"), i32(out.size(1), "ld"), i32(copies, "copies"), stream_of(x)),
           "echo_hip.latent_to_input");
}

Tensor latent_to_input(const Tensor& x, int64_t copies, int64_t ld, at::ScalarType dtype) {
  const int64_t rows = x.numel() / x.size(-1);
  Tensor out = at::empty({copies * rows, ld}, x.options().dtype(dtype));
  latent_to_input_out(x, copies, out);
  return out;
}

void euler_cfg_step_(const Tensor& x, const Tensor& v, int64_t has_cfg, double cfg_text, double cfg_speaker,
                     int64_t rescale, double omt, double ratio, double inv_omt, double dt) {
  need_dev(x, x, "x");
  need_dev(x, v, "v");
  TORCH_CHECK(x.scalar_type() == at::kFloat && v.scalar_type() == at::kFloat && x.is_contiguous() && v.is_contiguous(),
              "echo_hip.euler_cfg_step_: contiguous fp32 x and v");
  TORCH_CHECK(v.numel() >= (has_cfg ? 3 : 1) * x.numel(), "echo_hip.euler_cfg_step_: v has too few elements");
  EchoStepArgs a{(int32_t)(has_cfg != 0), (float)cfg_text, (float)cfg_speaker, (int32_t)(rescale != 0),
                 (float)omt, (float)ratio, (float)inv_omt, (float)dt};
  c10::DeviceGuard guard(x.device());
  check_rc(echo_euler_step((float*)x.data_ptr(), (const float*)v.data_ptr(), x.numel(), &a, stream_of(x)),
           "echo_hip.euler_cfg_step_");
}

Tensor euler_cfg_step(const Tensor& x, const Tensor& v, int64_t has_cfg, double cfg_text, double cfg_speaker,
                      int64_t rescale, double omt, double ratio, double inv_omt, double dt) {
  Tensor y = x.clone(at::MemoryFormat::Contiguous);
  euler_cfg_step_(y, v, has_cfg, cfg_text, cfg_speaker, rescale, omt, ratio, inv_omt, dt);
  return y;
}

void embed_out(const Tensor& ids, const Tensor& table, const Tensor& out) {
  need_dev(table, ids, "ids");
  need_dev(table, table, "table");
  need_dev(table, out, "out");
  TORCH_CHECK(ids.scalar_type() == at::kInt && ids.is_contiguous() && table.dim() == 2 && table.is_contiguous() &&
                  out.is_contiguous() && out.numel() == ids.numel() * table.size(1) &&
                  out.scalar_type() == table.scalar_type(),
              "echo_hip.embed: int32 ids, 2-D table, out [n, dim]");
  c10::DeviceGuard guard(table.device());
  check_rc(echo_embed(dt_of(table, "table"), (const int32_t*)ids.data_ptr(), table.data_ptr(), out.data_ptr(),
                      i32(ids.numel(), "n"), i32(table.size(1), "dim"), stream_of(table)),
           "echo_hip.embed");
}

Tensor embed(const Tensor& ids, const Tensor& table) {
  Tensor out = at::empty({ids.numel(), table.size(1)}, table.options());
  embed_out(ids, table, out);
  return out;
}

void scale_rows_(const Tensor& x, int64_t cols, double scale) {
  need_dev(x, x, "x");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && cols <= x.size(1), "echo_hip.scale_rows_: 2-D row-major view");
  c10::DeviceGuard guard(x.device());
  check_rc(echo_scale_rows(dt_of(x, "x"), x.data_ptr(), x.stride(0), i32(x.size(0), "rows"), i32(cols, "cols"),
                           (float)scale, stream_of(x)),
           "echo_hip.scale_rows_");
}

void cast_from_f32_out(const Tensor& x, const Tensor& out) {
  need_dev(x, x, "x");
  need_dev(x, out, "out");
  TORCH_CHECK(x.scalar_type() == at::kFloat && x.is_contiguous() && out.is_contiguous() && out.numel() == x.numel(),
              "echo_hip.cast_from_f32: contiguous fp32 x, out of equal numel");
  c10::DeviceGuard guard(x.device());
  check_rc(echo_cast_from_f32(dt_of(out, "out"), (const float*)x.data_ptr(), out.data_ptr(), x.numel(), stream_of(x)),
           "echo_hip.cast_from_f32");
}

Tensor cast_from_f32(const Tensor& x, at::ScalarType dtype) {
  Tensor out = at::empty(x.sizes(), x.options().dtype(dtype));
  cast_from_f32_out(x, out);
  return out;
}

int64_t gemm_pick_tile(int64_t M, int64_t N, int64_t K, int64_t batch) {
  return echo_gemm_pick_tile(i32(M, "M"), i32(N, "N"), i32(K, "K"), i32(batch, "batch"));
}

std::string version() { return std::string(echo_version()); }

// CPU dispatch: loud refusal instead of the dispatcher's generic NotImplementedError
[[noreturn]] void no_cpu(const c10::OperatorHandle& op, torch::jit::Stack*) {
  TORCH_CHECK(false, op.schema().name(), ": echo_tts_amd ops need device tensors (no CPU fallback)");
}

}  // namespace

#define GEMM_ARGS                                                                                           \
  "Tensor? bias=None, int epilogue=0, Tensor? aux=None, Tensor? gate=None, int act=0, float out_div=0., " \
  "int tile=0, Tensor? hn_w=None, Tensor? hn_rope=None, int[] hn=[], float hn_eps=0., "                    \
  "Tensor? act_alpha=None, int[] conv=[]"
#define ATTN_ARGS "Tensor q, Tensor? gate, Tensor[] seg_k, Tensor[] seg_v, Tensor?[] seg_len, int[] seg_batch_mod, " \
                  "int[] seg_causal"

TORCH_LIBRARY(echo_hip, m) {
  m.def("gemm(Tensor a, Tensor w, " GEMM_ARGS ") -> Tensor");
  m.def("gemm_out(Tensor a, Tensor w, Tensor(a!) out, " GEMM_ARGS ") -> ()");
  m.def("gemm_resid_norm_out(Tensor a, Tensor w, Tensor(a!) h, Tensor? gate, Tensor shift, Tensor scale1, "
        "float eps, Tensor(b!) xn, int tile=0) -> ()");
  m.def("joint_attention(" ATTN_ARGS ", float scale=0.08838834764831845) -> Tensor");
  m.def("joint_attention_out(" ATTN_ARGS ", Tensor(a!) out, float scale=0.08838834764831845) -> ()");
  m.def("attention_variant_out(" ATTN_ARGS ", Tensor(a!) out, float scale, int variant, int ablation, "
        "Tensor(b!)? stamps) -> ()");
  m.def("rmsnorm(Tensor x, Tensor w, float eps) -> Tensor");
  m.def("rmsnorm_out(Tensor x, Tensor w, float eps, Tensor(a!) out) -> ()");
  m.def("norm_modulate(Tensor x, Tensor shift, Tensor scale1, float eps) -> Tensor");
  m.def("norm_modulate_out(Tensor x, Tensor shift, Tensor scale1, float eps, Tensor(a!) out) -> ()");
  m.def("head_norm_rope_(Tensor(a!) x, Tensor w, float eps, int heads, int nblk, int col0, int col_stride, "
        "int w_stride, Tensor? rope, int rope_heads, int seq_len, int pos0, int pos_mult) -> ()");
  m.def("timestep_embedding(Tensor t, Tensor freqs, ScalarType dtype) -> Tensor");
  m.def("silu(Tensor x) -> Tensor");
  m.def("silu_out(Tensor x, Tensor(a!) out) -> ()");
  m.def("adaln_finish(Tensor raw) -> Tensor");
  m.def("adaln_finish_out(Tensor raw, Tensor(a!) table) -> ()");
  m.def("latent_to_input(Tensor x, int copies, int ld, ScalarType dtype) -> Tensor");
  m.def("latent_to_input_out(Tensor x, int copies, Tensor(a!) out) -> ()");
  m.def("euler_cfg_step(Tensor x, Tensor v, int has_cfg, float cfg_text, float cfg_speaker, int rescale, "
        "float omt, float ratio, float inv_omt, float dt) -> Tensor");
  m.def("euler_cfg_step_(Tensor(a!) x, Tensor v, int has_cfg, float cfg_text, float cfg_speaker, int rescale, "
        "float omt, float ratio, float inv_omt, float dt) -> ()");
  m.def("embed(Tensor ids, Tensor table) -> Tensor");
  m.def("embed_out(Tensor ids, Tensor table, Tensor(a!) out) -> ()");
  m.def("scale_rows_(Tensor(a!) x, int cols, float scale) -> ()");
  m.def("cast_from_f32(Tensor x, ScalarType dtype) -> Tensor");
  m.def("cast_from_f32_out(Tensor x, Tensor(a!) out) -> ()");
  m.def("gemm_pick_tile(int M, int N, int K, int batch) -> int", &gemm_pick_tile);
  m.def("version() -> str", &version);
}

TORCH_LIBRARY_IMPL(echo_hip, CUDA, m) {
  m.impl("gemm", &gemm);
  m.impl("gemm_out", &gemm_out);
  m.impl("gemm_resid_norm_out", &gemm_resid_norm_out);
  m.impl("joint_attention", &joint_attention);
  m.impl("joint_attention_out", &joint_attention_out);
  m.impl("attention_variant_out", &attention_variant_out);
  m.impl("rmsnorm", &rmsnorm);
  m.impl("rmsnorm_out", &rmsnorm_out);
  m.impl("norm_modulate", &norm_modulate);
  m.impl("norm_modulate_out", &norm_modulate_out);
  m.impl("head_norm_rope_", &head_norm_rope_);
  m.impl("timestep_embedding", &timestep_embedding);
  m.impl("silu", &silu);
  m.impl("silu_out", &silu_out);
  m.impl("adaln_finish", &adaln_finish);
  m.impl("adaln_finish_out", &adaln_finish_out);
  m.impl("latent_to_input", &latent_to_input);
  m.impl("latent_to_input_out", &latent_to_input_out);
  m.impl("euler_cfg_step", &euler_cfg_step);
  m.impl("euler_cfg_step_", &euler_cfg_step_);
  m.impl("embed", &embed);
  m.impl("embed_out", &embed_out);
  m.impl("scale_rows_", &scale_rows_);
  m.impl("cast_from_f32", &cast_from_f32);
  m.impl("cast_from_f32_out", &cast_from_f32_out);
}

TORCH_LIBRARY_IMPL(echo_hip, CPU, m) {
  for (const char* name : {"gemm", "gemm_out", "gemm_resid_norm_out", "joint_attention", "joint_attention_out", "attention_variant_out",
                           "rmsnorm", "rmsnorm_out", "norm_modulate", "norm_modulate_out", "head_norm_rope_",
                           "timestep_embedding", "silu", "silu_out", "adaln_finish", "adaln_finish_out",
                           "latent_to_input", "latent_to_input_out", "euler_cfg_step", "euler_cfg_step_", "embed",
                           "embed_out", "scale_rows_", "cast_from_f32", "cast_from_f32_out"})
    m.impl(name, torch::CppFunction::makeFromBoxedFunction<&no_cpu>());
}

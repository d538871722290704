// codec.hip — the non-GEMM kernels of the Fish-S1-DAC output path.
//
// ae_decode (reference inference.py:232-235) runs its convolutions, linears and transposed
// convolutions as echo_gemm calls (causal conv = GEMM over a tap-shifted view of the channels-last
// activation, gemm.hip); the kernels here are the rest: PCA inverse, Snake, the ConvNeXt depthwise
// conv + LayerNorm, RMSNorm (cast-then-weight form), interleaved-pair RoPE, window-limited causal
// attention (head_dim 64), the output conv + tanh, and the crop heuristic's flattening point.
// Activations are channels-last [item][row][channel]; bf16 results are rounded where the
// reference's bf16 ops round (one rounding per torch op), fp32 results are not.
#include "common.h"

namespace {

template <typename T> __device__ __forceinline__ float ldf(const T* p);
template <> __device__ __forceinline__ float ldf<bf16_t>(const bf16_t* p) { return bf2f(*p); }
template <> __device__ __forceinline__ float ldf<float>(const float* p) { return *p; }
template <typename T> __device__ __forceinline__ void stf(T* p, float v);
template <> __device__ __forceinline__ void stf<bf16_t>(bf16_t* p, float v) { *p = f2bf(v); }
template <> __device__ __forceinline__ void stf<float>(float* p, float v) { *p = v; }
template <typename T> __device__ __forceinline__ float rnd(float v) { return Elt<T>::rnd(v); }

// snake (autoencoder.py:97-102): x + (alpha + 1e-9)^-1 * sin(alpha * x)^2, rounded after every
// tensor op in bf16 (as the reference's bf16 module computes it), unrounded in fp32.
template <typename T> __device__ __forceinline__ float snake1(float x, float a) {
  const float s = rnd<T>(sinf(rnd<T>(a * x)));
  const float r = rnd<T>(1.0f / rnd<T>(a + 1e-9f));
  return rnd<T>(x + rnd<T>(r * rnd<T>(s * s)));
}

// ---- PCA inverse (inference.py:233): out = ((lat / scale) @ comps + mean) cast to T
template <typename T>
__global__ void __launch_bounds__(256) pca_inverse_kernel(const float* __restrict__ lat, const float* __restrict__ comps,
                                                          const float* __restrict__ mean, float scale, T* __restrict__ out,
                                                          int rows, int K, int D) {
  const int d = blockIdx.x * 256 + threadIdx.x;
  const int r = blockIdx.y;
  if (d >= D) return;
  const float* l = lat + (int64_t)r * K;
  float acc = 0.f;
  for (int k = 0; k < K; ++k) acc = acc + (l[k] / scale) * comps[(int64_t)k * D + d];
  stf<T>(out + (int64_t)r * D + d, acc + mean[d]);
}

// ---- Snake over [batch][rows][C] (C % 8 == 0), 8 channels per thread
template <typename T>
__global__ void __launch_bounds__(256) snake_kernel(const T* __restrict__ x, int64_t ldx, int64_t sx,
                                                    T* __restrict__ y, int64_t ldy, int64_t sy,
                                                    const T* __restrict__ alpha, int rows, int C) {
  const int per_row = C / 8;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)rows * per_row) return;
  const int r = (int)(i / per_row), c = (int)(i % per_row) * 8;
  const T* xp = x + blockIdx.y * sx + (int64_t)r * ldx + c;
  T* yp = y + blockIdx.y * sy + (int64_t)r * ldy + c;
  float v[8], a[8];
  load8(xp, v);
  load8(alpha + c, a);
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = snake1<T>(v[e], a[e]);
  store8(yp, v);
}

// ---- ConvNeXt head (autoencoder.py:360-364): causal depthwise conv k7 (+bias) then LayerNorm
// over C (eps 1e-6) with weight/bias; one 256-thread block per row, C <= 2048, C % 8 == 0.
template <typename T>
__global__ void __launch_bounds__(256) dwconv_ln_kernel(const T* __restrict__ x, int64_t ldx, int64_t sx,
                                                        T* __restrict__ y, int64_t ldy, int64_t sy,
                                                        const T* __restrict__ wdw, const T* __restrict__ bdw,
                                                        const T* __restrict__ lnw, const T* __restrict__ lnb,
                                                        int C, float eps) {
  __shared__ float red[8];
  const int t = blockIdx.x;
  const T* xb = x + blockIdx.y * sx;
  constexpr int MAXC = 1;  // 256 threads x 8 channels = 2048
  float h[8];
  const int c = threadIdx.x * 8;
  const bool on = c < C;
  float s1 = 0.f;
  if (on) {
#pragma unroll
    for (int e = 0; e < 8; ++e) h[e] = 0.f;
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      const int tt = t - 6 + j;
      if (tt < 0) continue;
      float xv[8];
      load8(xb + (int64_t)tt * ldx + c, xv);
#pragma unroll
      for (int e = 0; e < 8; ++e) h[e] = h[e] + ldf<T>(wdw + (int64_t)(c + e) * 7 + j) * xv[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      h[e] = rnd<T>(h[e] + ldf<T>(bdw + c + e));
      s1 += h[e];
    }
  }
  (void)MAXC;
  // two-pass LayerNorm statistics (fp32): mean, then E[(h-mean)^2]
  s1 = wave_sum(s1);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s1;
  __syncthreads();
  const float mean = (red[0] + red[1] + red[2] + red[3]) / (float)C;
  float s2 = 0.f;
  if (on) {
#pragma unroll
    for (int e = 0; e < 8; ++e) { const float d = h[e] - mean; s2 += d * d; }
  }
  s2 = wave_sum(s2);
  if ((threadIdx.x & 63) == 0) red[4 + (threadIdx.x >> 6)] = s2;
  __syncthreads();
  const float var = (red[4] + red[5] + red[6] + red[7]) / (float)C;
  const float rstd = 1.0f / sqrtf(var + eps);
  if (!on) return;
  float o[8], w[8], b[8];
  load8(lnw + c, w);
  load8(lnb + c, b);
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = (h[e] - mean) * rstd * w[e] + b[e];
  store8(y + blockIdx.y * sy + (int64_t)t * ldy + c, o);
}

// ---- RMSNorm of the AE transformer (autoencoder.py:720-731): the fp32 normalised row is cast to
// T BEFORE the weight multiply (a T op). One block per row, dim % 8 == 0, dim <= 2048.
template <typename T>
__global__ void __launch_bounds__(256) ae_rmsnorm_kernel(const T* __restrict__ x, int64_t ldx, const T* __restrict__ w,
                                                         T* __restrict__ y, int64_t ldy, int dim, float eps) {
  __shared__ float red[4];
  const int c = threadIdx.x * 8;
  const bool on = c < dim;
  float v[8];
  float ss = 0.f;
  if (on) {
    load8(x + blockIdx.x * ldx + c, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) ss += v[e] * v[e];
  }
  ss = wave_sum(ss);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  const float r = 1.0f / sqrtf((red[0] + red[1] + red[2] + red[3]) / (float)dim + eps);
  if (!on) return;
  float wv[8], o[8];
  load8(w + c, wv);
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = rnd<T>(v[e] * r) * wv[e];
  store8(y + blockIdx.x * ldy + c, o);
}

// ---- RoPE on interleaved pairs (apply_rotary_emb, autoencoder.py:815-826): fp32 math on the
// bf16 (cos, sin) table [pos][hd/2][2], pos = row % seq_len; in place on [rows][heads*hd] (ld).
template <typename T>
__global__ void __launch_bounds__(256) rope_pairs_kernel(T* __restrict__ x, int64_t ld, int rows, int heads, int hd,
                                                         const bf16_t* __restrict__ table, int seq_len) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int half = hd / 2;
  if (i >= (int64_t)rows * heads * half) return;
  const int p = (int)(i % half);
  const int h = (int)((i / half) % heads);
  const int r = (int)(i / ((int64_t)half * heads));
  const int pos = r % seq_len;
  T* q = x + (int64_t)r * ld + h * hd + 2 * p;
  const float x0 = ldf<T>(q), x1 = ldf<T>(q + 1);
  const float c = bf2f(table[((int64_t)pos * half + p) * 2]), s = bf2f(table[((int64_t)pos * half + p) * 2 + 1]);
  stf<T>(q, x0 * c - x1 * s);
  stf<T>(q + 1, x1 * c + x0 * s);
}

// ---- window-limited causal attention, head_dim 64 (Attention.forward with the
// WindowLimitedTransformer mask, autoencoder.py:663-706,762-773): query t sees keys
// [max(0, t-window+1), t] of its own item. One block = 64 queries of one (item, head), 4 lanes per
// query (16 dims each). The block's key range [q0-window+1, q0+63] is walked in chunks of AKC keys
// staged in LDS as fp32 (any window: 128 for pre/post_module, 512 for the encoder transformer);
// every query visits its keys in increasing order with an online fp32 softmax.
constexpr int AQ = 64, AHD = 64, AKC = 128;
template <typename T>
__global__ void __launch_bounds__(256) window_attn_kernel(const T* __restrict__ qkv, int64_t ld, T* __restrict__ out,
                                                          int64_t ldo, int T_, int heads, int window, float scale) {
  __shared__ float ks[AKC][AHD];
  __shared__ float vs[AKC][AHD];
  const int q0 = blockIdx.x * AQ;
  const int h = blockIdx.y;
  const int b = blockIdx.z;
  const int kbeg = max(0, q0 - window + 1);
  const int kend = min(T_ - 1, q0 + AQ - 1);
  const T* base = qkv + (int64_t)b * T_ * ld;
  const int kc = heads * AHD;
  const int ql = threadIdx.x >> 2, part = threadIdx.x & 3;
  const int t = q0 + ql;
  const int tq = min(t, T_ - 1);
  float q[16], acc[16];
  const T* qp = base + (int64_t)tq * ld + h * AHD + part * 16;
#pragma unroll
  for (int d = 0; d < 16; ++d) { q[d] = ldf<T>(qp + d); acc[d] = 0.f; }
  float m = -INFINITY, l = 0.f;
  const int jlo = max(0, tq - window + 1), jhi = tq;
  for (int c0 = kbeg; c0 <= kend; c0 += AKC) {
    const int nk = min(AKC, kend - c0 + 1);
    __syncthreads();
    for (int e = threadIdx.x; e < nk * AHD; e += 256) {
      const int j = e / AHD, d = e % AHD;
      const T* row = base + (int64_t)(c0 + j) * ld + h * AHD + d;
      ks[j][d] = ldf<T>(row + kc);
      vs[j][d] = ldf<T>(row + 2 * kc);
    }
    __syncthreads();
    const int j0 = max(jlo, c0) - c0, j1 = min(jhi, c0 + nk - 1) - c0;
    for (int j = j0; j <= j1; ++j) {
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < 16; ++d) s += q[d] * ks[j][part * 16 + d];
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
      s *= scale;
      const float mn = fmaxf(m, s);
      const float corr = __expf(m - mn);
      const float p = __expf(s - mn);
      l = l * corr + p;
#pragma unroll
      for (int d = 0; d < 16; ++d) acc[d] = acc[d] * corr + p * vs[j][part * 16 + d];
      m = mn;
    }
  }
  if (t >= T_) return;
  T* op = out + ((int64_t)b * T_ + t) * ldo + h * AHD + part * 16;
  const float inv = 1.0f / l;
#pragma unroll
  for (int d = 0; d < 16; ++d) stf<T>(op + d, acc[d] * inv);
}

// ---- encoder input conv (Encoder.block[0], autoencoder.py:913): causal WN conv k7, 1 -> C
// channels, on the raw audio [batch][L] (AE dtype): y[t][o] = b[o] + sum_k w[o][k] x[t-6+k]
// (x[<0] = 0), rounded once; written channels-last into the conv buffer rows.
template <typename T>
__global__ void __launch_bounds__(256) conv_in_kernel(const T* __restrict__ x, int64_t sx, const T* __restrict__ w,
                                                      const T* __restrict__ bias, T* __restrict__ y, int64_t ldy,
                                                      int64_t sy, int L, int C) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)L * C) return;
  const int t = (int)(i / C), o = (int)(i % C);
  const T* xb = x + blockIdx.y * sx;
  float acc = 0.f;
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    const int tt = t - 6 + k;
    if (tt >= 0) acc += ldf<T>(w + o * 7 + k) * ldf<T>(xb + tt);
  }
  stf<T>(y + blockIdx.y * sy + (int64_t)t * ldy + o, acc + ldf<T>(bias + o));
}

// ---- residual VQ encode + from_codes + PCA projection, one workgroup per latent frame.
// DownsampleResidualVectorQuantize.forward's code path (autoencoder.py:451-471): the semantic VQ,
// then the RVQ stages on the running residual; each VectorQuantize.forward (:130-137):
//   z_e = in_proj(r) (WN conv k1, D -> 8);   e = F.normalize(z_e) (x / max(|x|, 1e-12));
//   dist_j = |e|^2 - 2 e.c_j + |c_j|^2 over the l2-normalised codebook; code = first argmin;
//   q = out_proj(z_e + (cb[code] - z_e));   r -= q.
// Then DAC.encode_zq (:1117-1126): z_q = out_proj(cb[code_0]) + sum_i out_proj(cb[code_i]) and
// ae_encode's PCA (inference.py:226-228): lat = ((float(z_q) - mean) @ comps^T) * scale.
// Every value the reference materialises is rounded to T (bf16 mode) where it would be.
// Thread t owns channels [4t, 4t+4) of D = 1024; reductions: wave shuffles + LDS across 4 waves.
constexpr int VQ_D = 1024, VQ_CD = 8, VQ_MAXQ = 16, VQ_MAXPCA = 128;
struct RvqArgs {
  const void* w_in;    // [nq][8][D]
  const void* b_in;    // [nq][8]
  const void* cbn;     // normalised codebooks, concatenated [sum sizes][8]
  const void* csq;     // |cbn_j|^2 per entry (reference rounding), [sum sizes]
  const void* cb;      // raw codebooks [sum sizes][8]
  const void* w_out;   // [nq][D][8]
  const void* b_out;   // [nq][D]
  int cb_off[VQ_MAXQ + 1];
  int nq;
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T>
__global__ void __launch_bounds__(256) rvq_encode_kernel(const T* __restrict__ z, int64_t ldz, RvqArgs a,
                                                         int32_t* __restrict__ codes, int T_, T* __restrict__ zq_out,
                                                         int64_t ldq, const float* __restrict__ comps,
                                                         const float* __restrict__ mean, float scale,
                                                         float* __restrict__ lat, int npca) {
  __shared__ float red[4][VQ_MAXPCA];
  __shared__ float e_s[VQ_CD], st_s[VQ_CD];
  __shared__ float bd[4];
  __shared__ int bi[4];
  const int row = blockIdx.x;  // b * T_ + t
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int c0 = tid * 4;
  const T* w_in = (const T*)a.w_in;
  const T* b_in = (const T*)a.b_in;
  const T* cbn = (const T*)a.cbn;
  const T* csq = (const T*)a.csq;
  const T* cb = (const T*)a.cb;
  const T* w_out = (const T*)a.w_out;
  const T* b_out = (const T*)a.b_out;
  float r[4], zs[4], zr[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) { r[i] = ldf<T>(z + (int64_t)row * ldz + c0 + i); zs[i] = 0.f; zr[i] = 0.f; }
  for (int q = 0; q < a.nq; ++q) {
    // z_e = in_proj(r): 8 dot products of length D
    float p[VQ_CD];
#pragma unroll
    for (int o = 0; o < VQ_CD; ++o) {
      const T* wr = w_in + ((int64_t)q * VQ_CD + o) * VQ_D + c0;
      float acc = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) acc += ldf<T>(wr + i) * r[i];
      p[o] = wave_sum(acc);
    }
    if (lane == 0)
#pragma unroll
      for (int o = 0; o < VQ_CD; ++o) red[wv][o] = p[o];
    __syncthreads();
    if (tid == 0) {
      float ze[VQ_CD], n2 = 0.f;
#pragma unroll
      for (int o = 0; o < VQ_CD; ++o) {
        ze[o] = rnd<T>(red[0][o] + red[1][o] + red[2][o] + red[3][o] + ldf<T>(b_in + q * VQ_CD + o));
        n2 += ze[o] * ze[o];
      }
      const float n = fmaxf(rnd<T>(sqrtf(n2)), 1e-12f);
#pragma unroll
      for (int o = 0; o < VQ_CD; ++o) { e_s[o] = rnd<T>(ze[o] / n); st_s[o] = ze[o]; }
    }
    __syncthreads();
    float e[VQ_CD], esq = 0.f;
#pragma unroll
    for (int o = 0; o < VQ_CD; ++o) { e[o] = e_s[o]; esq += e[o] * e[o]; }
    esq = rnd<T>(esq);
    // nearest normalised codebook entry: first index of the minimum distance
    const int off = a.cb_off[q], size = a.cb_off[q + 1] - off;
    float best = INFINITY;
    int bidx = 0x7fffffff;
    for (int j = tid; j < size; j += 256) {
      const T* cj = cbn + (int64_t)(off + j) * VQ_CD;
      float dot = 0.f;
#pragma unroll
      for (int o = 0; o < VQ_CD; ++o) dot += e[o] * ldf<T>(cj + o);
      const float d = rnd<T>(rnd<T>(esq - 2.0f * rnd<T>(dot)) + ldf<T>(csq + off + j));
      if (d < best) { best = d; bidx = j; }  // j increases per thread: keeps the first minimum
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ob = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bidx, o, 64);
      if (ob < best || (ob == best && oi < bidx)) { best = ob; bidx = oi; }
    }
    if (lane == 0) { bd[wv] = best; bi[wv] = bidx; }
    __syncthreads();
    int code = bi[0];
    float cd = bd[0];
#pragma unroll
    for (int w = 1; w < 4; ++w)
      if (bd[w] < cd || (bd[w] == cd && bi[w] < code)) { cd = bd[w]; code = bi[w]; }
    if (tid == 0) codes[((int64_t)(row / T_) * a.nq + q) * T_ + (row % T_)] = code;
    // straight-through input and out_proj for the residual; raw code vector for from_codes
    float stv[VQ_CD], cv[VQ_CD];
    const T* craw = cb + (int64_t)(off + code) * VQ_CD;
#pragma unroll
    for (int o = 0; o < VQ_CD; ++o) {
      cv[o] = ldf<T>(craw + o);
      stv[o] = rnd<T>(st_s[o] + rnd<T>(cv[o] - st_s[o]));
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const T* wr = w_out + ((int64_t)q * VQ_D + c0 + i) * VQ_CD;
      const float bo = ldf<T>(b_out + (int64_t)q * VQ_D + c0 + i);
      float a1 = 0.f, a2 = 0.f;
#pragma unroll
      for (int o = 0; o < VQ_CD; ++o) {
        const float wo = ldf<T>(wr + o);
        a1 += wo * stv[o];
        a2 += wo * cv[o];
      }
      const float qv = rnd<T>(a1 + bo), qc = rnd<T>(a2 + bo);
      r[i] = rnd<T>(r[i] - qv);
      if (q == 0) zs[i] = qc;
      else zr[i] = (q == 1) ? qc : rnd<T>(zr[i] + qc);
    }
    __syncthreads();  // red / e_s / bd reused by the next stage
  }
  float zq[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    zq[i] = a.nq > 1 ? rnd<T>(zs[i] + zr[i]) : zs[i];
    if (zq_out) stf<T>(zq_out + (int64_t)row * ldq + c0 + i, zq[i]);
  }
  // PCA projection: npca dot products of length D in fp32
  for (int j0 = 0; j0 < npca; j0 += VQ_MAXPCA) {
    const int nj = min(VQ_MAXPCA, npca - j0);
    for (int j = 0; j < nj; ++j) {
      const float* cr = comps + (int64_t)(j0 + j) * VQ_D + c0;
      float acc = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) acc += (zq[i] - mean[c0 + i]) * cr[i];
      acc = wave_sum(acc);
      if (lane == 0) red[wv][j] = acc;
    }
    __syncthreads();
    for (int j = tid; j < nj; j += 256)
      lat[(int64_t)row * npca + j0 + j] = (red[0][j] + red[1][j] + red[2][j] + red[3][j]) * scale;
    __syncthreads();
  }
}

// ---- output conv + tanh (Decoder tail, autoencoder.py:995-996): y[t] = tanh(b + sum over 7 taps
// and C channels of w[tap][c] * s[t-6+tap][c]) on the Snake'd input s (zero rows before t = 0 are
// read from the buffer's pad); the conv result is rounded to T, tanh computed and rounded, then
// widened to fp32 (.float(), inference.py:235).
template <typename T>
__global__ void __launch_bounds__(256) conv_out_tanh_kernel(const T* __restrict__ s, int64_t lds_, int64_t ss,
                                                            const T* __restrict__ w, const T* __restrict__ bias,
                                                            float* __restrict__ y, int64_t sy, int rows, int C) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= rows) return;
  const T* sb = s + blockIdx.y * ss;
  float acc = 0.f;
  for (int tap = 0; tap < 7; ++tap) {
    const T* row = sb + (int64_t)(t - 6 + tap) * lds_;
    const T* wr = w + tap * C;
    for (int c = 0; c < C; c += 8) {
      float a[8], b[8];
      load8(row + c, a);
      load8(wr + c, b);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc += a[e] * b[e];
    }
  }
  const float v = rnd<T>(acc + ldf<T>(bias));
  y[blockIdx.y * sy + t] = rnd<T>(tanhf(v));
}

// ---- find_flattening_point (inference.py:315-330): window i covers rows i..i+W-1 of
// [data ; W zero rows]; first i with unbiased std < thr and |mean - target| < 0.1, else L.
// Double-precision sums (torch's CPU std/mean accumulate fp32 input in double).
__global__ void __launch_bounds__(256) flatten_kernel(const float* __restrict__ x, int L, int D, int W, float thr,
                                                      float target, int* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= L) return;
  double s = 0.0, q = 0.0;
  for (int r = i; r < min(i + W, L); ++r)
    for (int d = 0; d < D; ++d) {
      const double v = x[(int64_t)r * D + d];
      s += v;
      q += v * v;
    }
  const double n = (double)W * D;
  const double mean = s / n;
  const double var = (q - s * mean) / (n - 1.0);
  const double sd = sqrt(var > 0.0 ? var : 0.0);
  if (sd < (double)thr && fabs(mean - (double)target) < 0.1) atomicMin(out, i);
}

__global__ void fill_int_kernel(int* p, int v) { *p = v; }

}  // namespace

#define ECHO_DISPATCH(dtype, KERNEL_CALL_BF16, KERNEL_CALL_F32) \
  do {                                                           \
    if ((dtype) == ECHO_BF16) { KERNEL_CALL_BF16; }              \
    else if ((dtype) == ECHO_F32) { KERNEL_CALL_F32; }           \
    else return ECHO_EDTYPE;                                     \
  } while (0)

extern "C" int echo_pca_inverse(int32_t dtype, const float* lat, const float* comps, const float* mean,
                                float scale, void* out, int32_t rows, int32_t K, int32_t D, void* stream) {
  if (!lat || !comps || !mean || !out || rows < 0 || K <= 0 || D <= 0 || scale == 0.0f) return ECHO_EINVAL;
  if (rows == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  dim3 g((D + 255) / 256, rows);
  ECHO_DISPATCH(dtype,
      hipLaunchKernelGGL(pca_inverse_kernel<bf16_t>, g, dim3(256), 0, s, lat, comps, mean, scale, (bf16_t*)out, rows, K, D),
      hipLaunchKernelGGL(pca_inverse_kernel<float>, g, dim3(256), 0, s, lat, comps, mean, scale, (float*)out, rows, K, D));
  ECHO_LAUNCH_CHECK();
  return 0;
}

extern "C" int echo_snake(int32_t dtype, const void* x, int64_t ldx, int64_t sx, void* y, int64_t ldy, int64_t sy,
                          const void* alpha, int32_t rows, int32_t C, int32_t batch, void* stream) {
  if (!x || !y || !alpha || rows < 0 || C <= 0 || C % 8 || batch <= 0 || ldx % 8 || ldy % 8) return ECHO_EINVAL;
  if (rows == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int64_t n = (int64_t)rows * (C / 8);
  dim3 g((unsigned)((n + 255) / 256), batch);
  ECHO_DISPATCH(dtype,
      hipLaunchKernelGGL(snake_kernel<bf16_t>, g, dim3(256), 0, s, (const bf16_t*)x, ldx, sx, (bf16_t*)y, ldy, sy,
                         (const bf16_t*)alpha, rows, C),
      hipLaunchKernelGGL(snake_kernel<float>, g, dim3(256), 0, s, (const float*)x, ldx, sx, (float*)y, ldy, sy,
                         (const float*)alpha, rows, C));
  ECHO_LAUNCH_CHECK();
  return 0;
}

extern "C" int echo_dwconv_layernorm(int32_t dtype, const void* x, int64_t ldx, int64_t sx, void* y, int64_t ldy,
                                     int64_t sy, const void* w_dw, const void* b_dw, const void* ln_w,
                                     const void* ln_b, int32_t rows, int32_t C, int32_t batch, float eps,
                                     void* stream) {
  if (!x || !y || !w_dw || !b_dw || !ln_w || !ln_b || rows < 0 || C <= 0 || C % 8 || C > 2048 || batch <= 0 ||
      ldx % 8 || ldy % 8)
    return ECHO_EINVAL;
  if (rows == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  dim3 g(rows, batch);
  ECHO_DISPATCH(dtype,
      hipLaunchKernelGGL(dwconv_ln_kernel<bf16_t>, g, dim3(256), 0, s, (const bf16_t*)x, ldx, sx, (bf16_t*)y, ldy, sy,
                         (const bf16_t*)w_dw, (const bf16_t*)b_dw, (const bf16_t*)ln_w, (const bf16_t*)ln_b, C, eps),
      hipLaunchKernelGGL(dwconv_ln_kernel<float>, g, dim3(256), 0, s, (const float*)x, ldx, sx, (float*)y, ldy, sy,
                         (const float*)w_dw, (const float*)b_dw, (const float*)ln_w, (const float*)ln_b, C, eps));
  ECHO_LAUNCH_CHECK();
  return 0;
}

extern "C" int echo_ae_rmsnorm(int32_t dtype, const void* x, int64_t ldx, const void* w, void* y, int64_t ldy,
                               int32_t rows, int32_t dim, float eps, void* stream) {
  if (!x || !w || !y || rows < 0 || dim <= 0 || dim % 8 || dim > 2048 || ldx % 8 || ldy % 8) return ECHO_EINVAL;
  if (rows == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  ECHO_DISPATCH(dtype,
      hipLaunchKernelGGL(ae_rmsnorm_kernel<bf16_t>, dim3(rows), dim3(256), 0, s, (const bf16_t*)x, ldx,
                         (const bf16_t*)w, (bf16_t*)y, ldy, dim, eps),
      hipLaunchKernelGGL(ae_rmsnorm_kernel<float>, dim3(rows), dim3(256), 0, s, (const float*)x, ldx,
                         (const float*)w, (float*)y, ldy, dim, eps));
  ECHO_LAUNCH_CHECK();
  return 0;
}

extern "C" int echo_rope_pairs(int32_t dtype, void* x, int64_t ld, int32_t rows, int32_t heads, int32_t hd,
                               const void* table_bf16, int32_t seq_len, void* stream) {
  if (!x || !table_bf16 || rows < 0 || heads <= 0 || hd <= 0 || hd % 2 || seq_len <= 0) return ECHO_EINVAL;
  if (rows == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int64_t n = (int64_t)rows * heads * (hd / 2);
  dim3 g((unsigned)((n + 255) / 256));
  ECHO_DISPATCH(dtype,
      hipLaunchKernelGGL(rope_pairs_kernel<bf16_t>, g, dim3(256), 0, s, (bf16_t*)x, ld, rows, heads, hd,
                         (const bf16_t*)table_bf16, seq_len),
      hipLaunchKernelGGL(rope_pairs_kernel<float>, g, dim3(256), 0, s, (float*)x, ld, rows, heads, hd,
                         (const bf16_t*)table_bf16, seq_len));
  ECHO_LAUNCH_CHECK();
  return 0;
}

extern "C" int echo_window_attention(int32_t dtype, const void* qkv, int64_t ld, void* out, int64_t ldo,
                                     int32_t batch, int32_t T, int32_t heads, int32_t head_dim, int32_t window,
                                     void* stream) {
  if (!qkv || !out || batch <= 0 || T < 0 || heads <= 0 || head_dim != AHD || window <= 0) return ECHO_EINVAL;
  if (T == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  dim3 g((T + AQ - 1) / AQ, heads, batch);
  const float scale = 1.0f / sqrtf((float)head_dim);
  ECHO_DISPATCH(dtype,
      hipLaunchKernelGGL(window_attn_kernel<bf16_t>, g, dim3(256), 0, s, (const bf16_t*)qkv, ld, (bf16_t*)out, ldo, T,
                         heads, window, scale),
      hipLaunchKernelGGL(window_attn_kernel<float>, g, dim3(256), 0, s, (const float*)qkv, ld, (float*)out, ldo, T,
                         heads, window, scale));
  ECHO_LAUNCH_CHECK();
  return 0;
}

extern "C" int echo_conv_out_tanh(int32_t dtype, const void* s_in, int64_t lds_, int64_t ss, const void* w,
                                  const void* bias, float* y, int64_t sy, int32_t rows, int32_t C, int32_t batch,
                                  void* stream) {
  if (!s_in || !w || !bias || !y || rows < 0 || C <= 0 || C % 8 || batch <= 0 || lds_ % 8) return ECHO_EINVAL;
  if (rows == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  dim3 g((rows + 255) / 256, batch);
  ECHO_DISPATCH(dtype,
      hipLaunchKernelGGL(conv_out_tanh_kernel<bf16_t>, g, dim3(256), 0, s, (const bf16_t*)s_in, lds_, ss,
                         (const bf16_t*)w, (const bf16_t*)bias, y, sy, rows, C),
      hipLaunchKernelGGL(conv_out_tanh_kernel<float>, g, dim3(256), 0, s, (const float*)s_in, lds_, ss,
                         (const float*)w, (const float*)bias, y, sy, rows, C));
  ECHO_LAUNCH_CHECK();
  return 0;
}

extern "C" int echo_flattening_point(const float* x, int32_t L, int32_t D, int32_t window, float std_threshold,
                                     float target, int32_t* out, void* stream) {
  if (!x || !out || L < 0 || D <= 0 || window <= 0) return ECHO_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(fill_int_kernel, dim3(1), dim3(1), 0, s, (int*)out, L);
  if (L > 0)
    hipLaunchKernelGGL(flatten_kernel, dim3((L + 255) / 256), dim3(256), 0, s, x, L, D, window, std_threshold,
                       target, (int*)out);
  ECHO_LAUNCH_CHECK();
  return 0;
}

extern "C" int echo_conv_in(int32_t dtype, const void* x, int64_t sx, const void* w, const void* bias, void* y,
                            int64_t ldy, int64_t sy, int32_t L, int32_t C, int32_t batch, void* stream) {
  if (!x || !w || !bias || !y || L < 0 || C <= 0 || batch <= 0 || ldy < C) return ECHO_EINVAL;
  if (L == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int64_t n = (int64_t)L * C;
  dim3 g((unsigned)((n + 255) / 256), batch);
  ECHO_DISPATCH(dtype,
      hipLaunchKernelGGL(conv_in_kernel<bf16_t>, g, dim3(256), 0, s, (const bf16_t*)x, sx, (const bf16_t*)w,
                         (const bf16_t*)bias, (bf16_t*)y, ldy, sy, L, C),
      hipLaunchKernelGGL(conv_in_kernel<float>, g, dim3(256), 0, s, (const float*)x, sx, (const float*)w,
                         (const float*)bias, (float*)y, ldy, sy, L, C));
  ECHO_LAUNCH_CHECK();
  return 0;
}

extern "C" int echo_rvq_encode(int32_t dtype, const void* z, int64_t ldz, int32_t rows, int32_t T, int32_t D,
                               const EchoRvqWeights* wts, int32_t* codes, void* zq, int64_t ldq, const float* comps,
                               const float* mean, float scale, float* lat, int32_t npca, void* stream) {
  if (!z || !wts || !codes || !comps || !mean || !lat || rows < 0 || T <= 0 || rows % T || D != VQ_D ||
      ldz < D || (zq && ldq < D) || npca <= 0 || wts->nq <= 0 || wts->nq > VQ_MAXQ || wts->codebook_dim != VQ_CD ||
      !wts->w_in || !wts->b_in || !wts->cbn || !wts->csq || !wts->cb || !wts->w_out || !wts->b_out)
    return ECHO_EINVAL;
  if (rows == 0) return 0;
  RvqArgs a;
  a.w_in = wts->w_in; a.b_in = wts->b_in; a.cbn = wts->cbn; a.csq = wts->csq; a.cb = wts->cb;
  a.w_out = wts->w_out; a.b_out = wts->b_out; a.nq = wts->nq;
  a.cb_off[0] = 0;
  for (int q = 0; q < wts->nq; ++q) {
    if (wts->codebook_sizes[q] <= 0) return ECHO_EINVAL;
    a.cb_off[q + 1] = a.cb_off[q] + wts->codebook_sizes[q];
  }
  hipStream_t s = (hipStream_t)stream;
  ECHO_DISPATCH(dtype,
      hipLaunchKernelGGL(rvq_encode_kernel<bf16_t>, dim3(rows), dim3(256), 0, s, (const bf16_t*)z, ldz, a, codes, T,
                         (bf16_t*)zq, ldq, comps, mean, scale, lat, npca),
      hipLaunchKernelGGL(rvq_encode_kernel<float>, dim3(rows), dim3(256), 0, s, (const float*)z, ldz, a, codes, T,
                         (float*)zq, ldq, comps, mean, scale, lat, npca));
  ECHO_LAUNCH_CHECK();
  return 0;
}

/* asan_host.c — host-side AddressSanitizer driver for the C ABI (include/echo_hip.h).
 *
 * tests/test_asan_host.py builds every csrc/*.hip with `hipcc --offload-host-only` (host code
 * only: argument validation, shape policies, launch setup) and `-Xarch_host -fsanitize=address`,
 * links this driver against it and runs it on the CPU. Every call here stays on the host: the
 * pure policies (tile pick, split-KV pick, workspace size, knobs) over a sweep of shapes, and every
 * entry point with arguments that must be refused BEFORE any launch (NULL pointers, bad dtypes,
 * bad shapes, misalignment). A launch would need the device code this build leaves out, so each
 * refusal is also checked to come back as the documented negative ECHO_E* code.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/echo_hip.h"

static int failures = 0;
#define EXPECT_NEG(call)                                                             \
  do {                                                                               \
    int rc_ = (call);                                                                \
    if (rc_ >= 0) { fprintf(stderr, "line %d: expected refusal: %s -> %d\n", __LINE__, #call, rc_); ++failures; } \
  } while (0)

static EchoAttnArgs attn_args(int rows, int B, int n_q, void* fake) {
  EchoAttnArgs a;
  memset(&a, 0, sizeof a);
  a.dtype = ECHO_BF16; a.rows = rows; a.n_q = n_q; a.heads = 16; a.nseg = 3; a.scale = 0.0883883f;
  a.q = a.out = a.gate = fake;
  a.q_ld_tok = a.o_ld_tok = a.g_ld_tok = 4 * 16 * 128;
  a.q_ld_batch = a.o_ld_batch = a.g_ld_batch = (int64_t)n_q * 4 * 16 * 128;
  const int cap[3] = {n_q, 448, 160}, bm[3] = {rows, B, B};
  for (int i = 0; i < 3; ++i) {
    a.seg[i].k = a.seg[i].v = fake;
    a.seg[i].ld_tok = 2 * 16 * 128;
    a.seg[i].ld_batch = (int64_t)cap[i] * 2 * 16 * 128;
    a.seg[i].batch_mod = bm[i];
    a.seg[i].capacity = cap[i];
  }
  return a;
}

int main(void) {
  /* a host buffer stands in for device pointers: nothing below may dereference it */
  char* fake = (char*)malloc(4096);
  void* f = fake + 256;
  printf("%s\n", echo_version());

  /* GEMM tile policy over the decoder / encoder / codec shape sweep */
  const int Ms[] = {1, 63, 64, 160, 480, 640, 1920, 2560, 5120, 7680, 10240, 30720, 65536};
  const int Ns[] = {16, 64, 80, 1024, 2048, 4096, 8192, 11776, 49152};
  const int Ks[] = {64, 128, 1280, 2048, 5888};
  long sum = 0;
  for (size_t i = 0; i < sizeof Ms / sizeof *Ms; ++i)
    for (size_t j = 0; j < sizeof Ns / sizeof *Ns; ++j)
      for (size_t k = 0; k < sizeof Ks / sizeof *Ks; ++k)
        for (int b = 1; b <= 3; b += 2) sum += echo_gemm_pick_tile(Ms[i], Ns[j], Ks[k], b);
  printf("tile-pick sweep checksum %ld\n", sum);

  /* split-KV policy + workspace size over row counts and query lengths */
  for (int rows = 1; rows <= 48; ++rows)
    for (int nq = 1; nq <= 640; nq += 53) {
      EchoAttnArgs a = attn_args(rows, rows >= 3 ? rows / 3 : 1, nq, f);
      const int ns = echo_attention_pick_split(&a);
      if (ns < 1 || ns > 16) { fprintf(stderr, "pick_split %d\n", ns); ++failures; }
      if (ns > 1 && echo_attention_split_ws_bytes(&a, ns) <= 0) ++failures;
    }
  if (echo_attention_split_ws_bytes(NULL, 3) != 0) ++failures;
  EXPECT_NEG(echo_attention_set_split(99));
  EXPECT_NEG(echo_gemm_set_diag(1, -1));
  if (echo_attention_set_split(-1) != 0) ++failures;

  /* GEMM refusals */
  EchoGemmArgs g;
  memset(&g, 0, sizeof g);
  EXPECT_NEG(echo_gemm(NULL, NULL));
  EXPECT_NEG(echo_gemm(&g, NULL));
  g.dtype = ECHO_BF16; g.M = 128; g.N = 128; g.K = 100; g.batch = 1;  /* K % 64 != 0 */
  g.A = g.W = g.C = f; g.lda = g.ldw = g.ldc = 128;
  EXPECT_NEG(echo_gemm(&g, NULL));
  g.K = 128; g.dtype = 7;
  EXPECT_NEG(echo_gemm(&g, NULL));
  g.dtype = ECHO_BF16; g.lda = 64;  /* lda < K */
  EXPECT_NEG(echo_gemm(&g, NULL));
  g.lda = 128; g.A = fake + 1;      /* misaligned */
  EXPECT_NEG(echo_gemm(&g, NULL));
  g.A = f; g.epilogue = 99;
  EXPECT_NEG(echo_gemm(&g, NULL));
  g.epilogue = ECHO_EPI_RESID; g.aux = NULL;  /* residual without aux */
  EXPECT_NEG(echo_gemm(&g, NULL));

  /* attention refusals */
  EchoAttnArgs a = attn_args(3, 1, 640, f);
  EchoAttnArgs b = a;
  EXPECT_NEG(echo_attention(NULL, NULL));
  b.nseg = 5; EXPECT_NEG(echo_attention(&b, NULL));
  b = a; b.seg[0].v = NULL; EXPECT_NEG(echo_attention(&b, NULL));
  b = a; b.q_ld_tok = 7; EXPECT_NEG(echo_attention(&b, NULL));
  b = a; b.dtype = 9; EXPECT_NEG(echo_attention(&b, NULL));
  b = a; b.out = fake + 2; EXPECT_NEG(echo_attention(&b, NULL));
  EXPECT_NEG(echo_attention_split(&a, 3, NULL, 0, NULL));          /* no workspace */
  EXPECT_NEG(echo_attention_split(&a, 3, fake + 4, 1 << 30, NULL));  /* misaligned workspace */
  EXPECT_NEG(echo_attention_split(&a, 3, f, 16, NULL));             /* too small */
  EXPECT_NEG(echo_attention_split(&a, 17, f, 1LL << 40, NULL));
  EXPECT_NEG(echo_attention_variant(&a, 99, 0, NULL, NULL));

  /* elementwise / codec refusals (NULL pointers, bad shapes, bad dtypes) */
  EXPECT_NEG(echo_rmsnorm(ECHO_BF16, NULL, 0, NULL, NULL, 0, 0, 0, 1e-6f, NULL));
  EXPECT_NEG(echo_adaln_modulate(ECHO_BF16, NULL, NULL, 0, 0, NULL, NULL, 0, 0, 1e-6f, NULL));
  EXPECT_NEG(echo_timestep_embedding(ECHO_BF16, NULL, NULL, NULL, 0, 0, NULL));
  EXPECT_NEG(echo_silu(ECHO_BF16, NULL, 0, NULL, 0, 0, 0, NULL));
  EXPECT_NEG(echo_adaln_finish(ECHO_BF16, NULL, NULL, 0, 0, 0, NULL));
  EXPECT_NEG(echo_euler_step(NULL, NULL, 0, NULL, NULL));
  EXPECT_NEG(echo_embed(ECHO_BF16, NULL, NULL, NULL, 0, 0, NULL));
  EXPECT_NEG(echo_scale_rows(ECHO_BF16, NULL, 0, 0, 0, 1.0f, NULL));
  EXPECT_NEG(echo_cast_from_f32(ECHO_BF16, NULL, NULL, 0, NULL));
  EXPECT_NEG(echo_cast_from_f32(5, (const float*)f, f, 16, NULL));

  free(fake);
  if (failures) {
    fprintf(stderr, "%d failures\n", failures);
    return 1;
  }
  printf("asan host driver: ok\n");
  return 0;
}

/*
 * omr_oracle.c — CPU restatement of omr_core's detect / encode path (TEST INFRASTRUCTURE ONLY).
 * See omr_oracle.h for the pinned conventions and the parity status ("unpinned" at the bit
 * level against the reference; pinned by golden vectors + the reference's functional KATs).
 *
 * Written for clarity, not speed: plain loops over u64 residues, Shoup twiddles in the NTT,
 * external-product sums kept exactly in 128 bits and reduced once, and an 80-bit long-double
 * quotient estimate for other products (all self-checked by the golden-vector tests).
 */
#include "omr_oracle.h"

#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef unsigned __int128 u128;

/* ------------------------------------------------------------------------------------------
 * Modular arithmetic
 * ---------------------------------------------------------------------------------------- */
static inline uint64_t addmod(uint64_t a, uint64_t b, uint64_t q) {
  uint64_t r = a + b;
  return r >= q ? r - q : r;
}
static inline uint64_t submod(uint64_t a, uint64_t b, uint64_t q) {
  return a >= b ? a - b : a + q - b;
}
static inline uint64_t negmod(uint64_t a, uint64_t q) { return a ? q - a : 0; }
/* a, b < q < 2^51 */
static inline uint64_t mulmod(uint64_t a, uint64_t b, uint64_t q) {
  u128 p = (u128)a * b;
  uint64_t qe = (uint64_t)((long double)a * (long double)b / (long double)q);
  int64_t r = (int64_t)((uint64_t)p - qe * q);
  while (r < 0) r += (int64_t)q;
  while (r >= (int64_t)q) r -= (int64_t)q;
  return (uint64_t)r;
}
static uint64_t powmod(uint64_t b, uint64_t e, uint64_t q) {
  uint64_t r = 1;
  b %= q;
  while (e) {
    if (e & 1) r = mulmod(r, b, q);
    b = mulmod(b, b, q);
    e >>= 1;
  }
  return r;
}
static inline uint64_t shoup_pre(uint64_t w, uint64_t q) { return (uint64_t)(((u128)w << 64) / q); }
static inline uint64_t mul_shoup(uint64_t a, uint64_t w, uint64_t ws, uint64_t q) {
  uint64_t qe = (uint64_t)(((u128)a * ws) >> 64);
  uint64_t r = a * w - qe * q;
  return r >= q ? r - q : r;
}

/* ------------------------------------------------------------------------------------------
 * Negacyclic NTT over Z_q[X]/(X^N+1) — the convention pinned in omr_oracle.h.
 * Replaces the concrete-ntt transform behind NttTable (parameters/mod.rs:174-181,238-245).
 * ---------------------------------------------------------------------------------------- */
typedef struct {
  uint64_t q;
  int N, L;
  uint64_t psi, ninv, ninvs;
  uint64_t *w, *ws, *iw, *iws; /* w[k] = psi^brv(k), iw[k] = psi^-brv(k) */
} ntt_tab;

static ntt_tab g_tab[3];

static uint32_t brv(uint32_t x, int bits) {
  uint32_t r = 0;
  for (int i = 0; i < bits; ++i) r |= ((x >> i) & 1u) << (bits - 1 - i);
  return r;
}

static void tab_init(ntt_tab *t, uint64_t q, int N, uint64_t g) {
  t->q = q;
  t->N = N;
  t->L = 0;
  while ((1 << t->L) < N) t->L++;
  t->psi = powmod(g, (q - 1) / (2 * (uint64_t)N), q);
  uint64_t ipsi = powmod(t->psi, q - 2, q);
  t->w = malloc(sizeof(uint64_t) * N);
  t->ws = malloc(sizeof(uint64_t) * N);
  t->iw = malloc(sizeof(uint64_t) * N);
  t->iws = malloc(sizeof(uint64_t) * N);
  for (int k = 0; k < N; ++k) {
    uint32_t e = brv((uint32_t)k, t->L);
    t->w[k] = powmod(t->psi, e, q);
    t->ws[k] = shoup_pre(t->w[k], q);
    t->iw[k] = powmod(ipsi, e, q);
    t->iws[k] = shoup_pre(t->iw[k], q);
  }
  t->ninv = powmod((uint64_t)N, q - 2, q);
  t->ninvs = shoup_pre(t->ninv, q);
}

__attribute__((constructor)) static void oref_init_tables(void) {
  tab_init(&g_tab[1], OREF_Q1, OREF_N1, 7);  /* smallest primitive root of q1 */
  tab_init(&g_tab[2], OREF_Q2, OREF_N2, 22); /* smallest primitive root of q2 */
}

/* Cooley-Tukey, natural order in, bit-reversed evaluation order out. */
static void ntt_fwd(const ntt_tab *t, uint64_t *a) {
  const int N = t->N;
  const uint64_t q = t->q;
  for (int m = 1, h = N / 2; m < N; m <<= 1, h >>= 1) {
    for (int i = 0; i < m; ++i) {
      const uint64_t W = t->w[m + i], Ws = t->ws[m + i];
      for (int j = 2 * i * h; j < 2 * i * h + h; ++j) {
        uint64_t U = a[j], V = mul_shoup(a[j + h], W, Ws, q);
        a[j] = addmod(U, V, q);
        a[j + h] = submod(U, V, q);
      }
    }
  }
}
/* Gentleman-Sande, bit-reversed in, natural out, scaled by N^-1. */
static void ntt_inv(const ntt_tab *t, uint64_t *a) {
  const int N = t->N;
  const uint64_t q = t->q;
  for (int m = N / 2, h = 1; m >= 1; m >>= 1, h <<= 1) {
    for (int i = 0; i < m; ++i) {
      const uint64_t W = t->iw[m + i], Ws = t->iws[m + i];
      for (int j = 2 * i * h; j < 2 * i * h + h; ++j) {
        uint64_t U = a[j], V = a[j + h];
        a[j] = addmod(U, V, q);
        a[j + h] = mul_shoup(submod(U, V, q), W, Ws, q);
      }
    }
  }
  for (int j = 0; j < N; ++j) a[j] = mul_shoup(a[j], t->ninv, t->ninvs, q);
}

void oref_ntt_forward(int level, uint64_t *a) { ntt_fwd(&g_tab[level], a); }
void oref_ntt_inverse(int level, uint64_t *a) { ntt_inv(&g_tab[level], a); }

/* ------------------------------------------------------------------------------------------
 * Gadget decomposition: NonPowOf2ApproxSignedBasis::new(q, logB, Some(k)) — mod.rs:55,81,89.
 * ---------------------------------------------------------------------------------------- */
typedef struct {
  uint64_t q;
  int logB, d, drop;
} basis_t;
static const basis_t g_basis[4] = {
    {0, 0, 0, 0},
    {OREF_Q1, OREF_LOGB1, OREF_D1, OREF_DROP1},
    {OREF_Q2, OREF_LOGB2, OREF_D2, OREF_DROP2},
    {OREF_Q2, OREF_LOGBT, OREF_DT, 0},
};

static inline void decompose(const basis_t *bs, uint64_t x, int64_t *dg) {
  const int64_t q = (int64_t)bs->q;
  int64_t y = x > (bs->q - 1) / 2 ? (int64_t)x - q : (int64_t)x;
  if (bs->drop) y = (y + (1LL << (bs->drop - 1))) >> bs->drop; /* floor (arithmetic shift) */
  const int64_t B = 1LL << bs->logB;
  for (int k = 0; k < bs->d - 1; ++k) {
    int64_t c = (y + B / 2) >> bs->logB;
    dg[k] = y - c * B;
    y = c;
  }
  dg[bs->d - 1] = y;
}

int oref_decompose(int which, uint64_t x, int64_t *digits) {
  decompose(&g_basis[which], x, digits);
  return g_basis[which].d;
}

/* ------------------------------------------------------------------------------------------
 * Small helpers
 * ---------------------------------------------------------------------------------------- */
uint64_t oref_modswitch_q1_to_qi(uint64_t v) {
  /* lwe_modulus_switch(q1 -> 4096), detector.rs:571-575: round half up */
  return ((2ull * OREF_QI * v + OREF_Q1) / (2ull * OREF_Q1)) % OREF_QI;
}

/* LookUpTable::negacyclic_lut for slices, lut.rs:12-27 */
static void negacyclic_lut(const uint64_t *vals, int nvals, int N, int log_t, uint64_t *lut) {
  const int hd = N >> log_t;
  const int nchunks = N / hd;
  memset(lut, 0, sizeof(uint64_t) * N);
  for (int c = 0; c < nchunks; ++c) {
    int idx = (c + 1) / 2; /* interleave(v, v[1..]) = v0, v1, v1, v2, v2, ... */
    uint64_t v = idx < nvals ? vals[idx] : 0;
    for (int j = 0; j < hd; ++j) lut[c * hd + j] = v;
  }
}

void oref_first_level_lut(uint64_t *lut) {
  /* detector.rs:457-476: output plain modulus 32 -> log = 4; input plain modulus 8 */
  const uint64_t q = OREF_Q1;
  const uint64_t one = ((q >> 4) + 1) >> 1;
  const uint64_t vals[5] = {one, 0, 0, 0, q - one};
  negacyclic_lut(vals, 5, OREF_N1, 3, lut);
}

void oref_second_level_lut(uint64_t *lut) {
  /* detector.rs:479-503: scale_one = round_half_up(q2 / 257); data[2*clue_count] = scale_one */
  const uint64_t q = OREF_Q2;
  const uint64_t one = (2 * q + OREF_P) / (2 * OREF_P);
  uint64_t vals[OREF_TI];
  memset(vals, 0, sizeof(vals));
  vals[2 * OREF_CLUES] = one;
  negacyclic_lut(vals, OREF_TI, OREF_N2, 5, lut);
}

/* X^r * p over Z_q[X]/(X^N+1), r in [0, 2N) */
static void mul_monomial(const ntt_tab *t, const uint64_t *p, uint32_t r, uint64_t *out) {
  const uint32_t N = (uint32_t)t->N;
  for (uint32_t i = 0; i < N; ++i) {
    uint32_t e = i + r;
    if (e < N)
      out[e] = p[i];
    else if (e < 2 * N)
      out[e - N] = negmod(p[i], t->q);
    else
      out[e - 2 * N] = p[i];
  }
}
void oref_negacyclic_mul_monomial(int level, const uint64_t *p, uint32_t r, uint64_t *out) {
  mul_monomial(&g_tab[level], p, r % (2u * (uint32_t)g_tab[level].N), out);
}

/* sigma_g: p(X) -> p(X^g), g odd */
static void automorphism(const uint64_t *p, uint32_t g, uint64_t *out) {
  const uint32_t N = OREF_N2;
  for (uint32_t i = 0; i < N; ++i) {
    uint32_t e = (uint32_t)(((uint64_t)i * g) % (2 * N));
    if (e < N)
      out[e] = p[i];
    else
      out[e - N] = negmod(p[i], OREF_Q2);
  }
}
void oref_automorphism(const uint64_t *p, uint32_t g, uint64_t *out) { automorphism(p, g, out); }

/* ------------------------------------------------------------------------------------------
 * ChaCha (djb variant: 64-bit block counter in words 12-13, 64-bit stream id in 14-15), the
 * core of rand_chacha's ChaCha12Rng = rand 0.8 StdRng.
 * ---------------------------------------------------------------------------------------- */
#define ROTL32(v, n) (((v) << (n)) | ((v) >> (32 - (n))))
#define QR(a, b, c, d)                                                                        \
  a += b; d ^= a; d = ROTL32(d, 16); c += d; b ^= c; b = ROTL32(b, 12);                       \
  a += b; d ^= a; d = ROTL32(d, 8);  c += d; b ^= c; b = ROTL32(b, 7);

void oref_chacha_block(int rounds, const uint32_t key[8], uint64_t counter, uint64_t stream,
                       uint32_t out[16]) {
  uint32_t in[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                     key[0], key[1], key[2], key[3], key[4], key[5], key[6], key[7],
                     (uint32_t)counter, (uint32_t)(counter >> 32),
                     (uint32_t)stream, (uint32_t)(stream >> 32)};
  uint32_t x[16];
  memcpy(x, in, sizeof(x));
  for (int r = 0; r < rounds; r += 2) {
    QR(x[0], x[4], x[8], x[12]);
    QR(x[1], x[5], x[9], x[13]);
    QR(x[2], x[6], x[10], x[14]);
    QR(x[3], x[7], x[11], x[15]);
    QR(x[0], x[5], x[10], x[15]);
    QR(x[1], x[6], x[11], x[12]);
    QR(x[2], x[7], x[8], x[13]);
    QR(x[3], x[4], x[9], x[14]);
  }
  for (int i = 0; i < 16; ++i) out[i] = x[i] + in[i];
}

/* ------------------------------------------------------------------------------------------
 * Context: NTT-domain copies of the evaluation keys (DetectionKey, key_gen/detection.rs:9-16)
 * ---------------------------------------------------------------------------------------- */
#define BSK1_GGSW (2 * OREF_D1 * 2 * OREF_N1)
#define BSK2_GGSW (2 * OREF_D2 * 2 * OREF_N2)
#define KSK_ROW (OREF_NI + 1)
#define TK_STEP (OREF_DT * 2 * OREF_N2)

struct oref_ctx {
  uint64_t *bsk1; /* [512][8][2][1024] NTT domain */
  uint32_t *ksk;  /* [1024][27][671] */
  uint64_t *bsk2; /* [670][12][2][2048] NTT domain */
  uint64_t *tk;   /* [11][25][2][2048] NTT domain */
  uint64_t lut1[OREF_N1], lut2[OREF_N2];
  uint64_t ninv2;
};

oref_ctx *oref_create(const uint32_t *bsk1, const uint32_t *ksk, const uint64_t *bsk2,
                      const uint64_t *tk) {
  oref_ctx *c = calloc(1, sizeof(oref_ctx));
  const size_t n1 = (size_t)OREF_N0 * BSK1_GGSW, n2 = (size_t)OREF_NI * BSK2_GGSW;
  const size_t nk = (size_t)OREF_N1 * OREF_KS_DIGITS * KSK_ROW;
  const size_t nt = (size_t)OREF_TRACE_STEPS * TK_STEP;
  c->bsk1 = malloc(n1 * sizeof(uint64_t));
  c->bsk2 = malloc(n2 * sizeof(uint64_t));
  c->ksk = malloc(nk * sizeof(uint32_t));
  c->tk = malloc(nt * sizeof(uint64_t));
  for (size_t i = 0; i < n1; ++i) c->bsk1[i] = bsk1[i];
  for (size_t i = 0; i < n1; i += OREF_N1) ntt_fwd(&g_tab[1], c->bsk1 + i);
  for (size_t i = 0; i < n2; ++i) c->bsk2[i] = bsk2[i];
  for (size_t i = 0; i < n2; i += OREF_N2) ntt_fwd(&g_tab[2], c->bsk2 + i);
  memcpy(c->ksk, ksk, nk * sizeof(uint32_t));
  for (size_t i = 0; i < nt; ++i) c->tk[i] = tk[i];
  for (size_t i = 0; i < nt; i += OREF_N2) ntt_fwd(&g_tab[2], c->tk + i);
  oref_first_level_lut(c->lut1);
  oref_second_level_lut(c->lut2);
  c->ninv2 = g_tab[2].ninv;
  return c;
}

void oref_destroy(oref_ctx *c) {
  if (!c) return;
  free(c->bsk1);
  free(c->bsk2);
  free(c->ksk);
  free(c->tk);
  free(c);
}

/* ------------------------------------------------------------------------------------------
 * External product RLWE x GGSW and binary blind rotation
 * (BlindRotationKey::blind_rotate, called at detector.rs:555 and :623)
 * ---------------------------------------------------------------------------------------- */
static void ext_product(int level, const uint64_t *ca, const uint64_t *cb, const uint64_t *ggsw,
                        uint64_t *oa, uint64_t *ob) {
  const ntt_tab *t = &g_tab[level];
  const basis_t *bs = &g_basis[level];
  const int N = t->N, d = bs->d;
  const uint64_t q = t->q;
  /* the 2d products per coefficient are summed exactly in 128 bits (each < 2^100, 12 of them
   * < 2^104) and reduced once */
  u128 *acc_a = calloc((size_t)N, sizeof(u128));
  u128 *acc_b = calloc((size_t)N, sizeof(u128));
  uint64_t *dig = malloc(sizeof(uint64_t) * (size_t)N * d);
  int64_t tmp[32];
  for (int p = 0; p < 2; ++p) {
    const uint64_t *src = p == 0 ? ca : cb;
    for (int j = 0; j < N; ++j) {
      decompose(bs, src[j], tmp);
      for (int k = 0; k < d; ++k) dig[(size_t)k * N + j] = tmp[k] < 0 ? (uint64_t)(tmp[k] + (int64_t)q) : (uint64_t)tmp[k];
    }
    for (int k = 0; k < d; ++k) {
      uint64_t *D = dig + (size_t)k * N;
      ntt_fwd(t, D);
      const uint64_t *ga = ggsw + ((size_t)(p * d + k) * 2 + 0) * N;
      const uint64_t *gb = ggsw + ((size_t)(p * d + k) * 2 + 1) * N;
      for (int j = 0; j < N; ++j) {
        acc_a[j] += (u128)D[j] * ga[j];
        acc_b[j] += (u128)D[j] * gb[j];
      }
    }
  }
  for (int j = 0; j < N; ++j) {
    oa[j] = (uint64_t)(acc_a[j] % q);
    ob[j] = (uint64_t)(acc_b[j] % q);
  }
  ntt_inv(t, oa);
  ntt_inv(t, ob);
  free(acc_a);
  free(acc_b);
  free(dig);
}

/* lwe_a values are already mod 2N. out: (a, b) coefficient domain, 2N u64. */
static void blind_rotate(int level, const uint64_t *lut, const uint32_t *lwe_a, uint32_t lwe_b,
                         int n, const uint64_t *bsk, uint64_t *out) {
  const ntt_tab *t = &g_tab[level];
  const int N = t->N;
  const size_t ggsw_sz = (size_t)2 * g_basis[level].d * 2 * N;
  uint64_t *acc_a = out, *acc_b = out + N;
  uint64_t *ta = malloc(sizeof(uint64_t) * N * 4), *tb = ta + N, *ra = tb + N, *rb = ra + N;
  memset(acc_a, 0, sizeof(uint64_t) * N);
  mul_monomial(t, lut, (2u * N - lwe_b % (2u * N)) % (2u * N), acc_b); /* X^{-b} * LUT */
  for (int i = 0; i < n; ++i) {
    const uint32_t ai = lwe_a[i] % (2u * N);
    if (ai == 0) continue; /* (X^0 - 1) * ACC = 0: the external product is exactly 0 */
    mul_monomial(t, acc_a, ai, ta);
    mul_monomial(t, acc_b, ai, tb);
    for (int j = 0; j < N; ++j) {
      ta[j] = submod(ta[j], acc_a[j], t->q);
      tb[j] = submod(tb[j], acc_b[j], t->q);
    }
    ext_product(level, ta, tb, bsk + (size_t)i * ggsw_sz, ra, rb);
    for (int j = 0; j < N; ++j) {
      acc_a[j] = addmod(acc_a[j], ra[j], t->q);
      acc_b[j] = addmod(acc_b[j], rb[j], t->q);
    }
  }
  free(ta);
}

/* ------------------------------------------------------------------------------------------
 * Detect stages (detector.rs:135-166)
 * ---------------------------------------------------------------------------------------- */
/* CmLweCiphertext::extract_all (RLWE-mode common-mask LWE), detector.rs:514 */
void oref_extract_clue(const uint16_t *clue_a, const uint16_t *clue_b, int i, uint16_t *lwe_a,
                       uint16_t *lwe_b) {
  for (int j = 0; j < OREF_N0; ++j) {
    if (j <= i)
      lwe_a[j] = clue_a[i - j] & (OREF_Q0 - 1);
    else
      lwe_a[j] = (uint16_t)((OREF_Q0 - clue_a[OREF_N0 + i - j]) & (OREF_Q0 - 1));
  }
  *lwe_b = clue_b[i] & (OREF_Q0 - 1);
}

uint32_t oref_clue_phase(const uint16_t *clue_a, const uint16_t *clue_b, int i, const uint8_t *s0) {
  uint16_t a[OREF_N0], b;
  oref_extract_clue(clue_a, clue_b, i, a, &b);
  uint32_t acc = b;
  for (int j = 0; j < OREF_N0; ++j) acc += (uint32_t)(OREF_Q0 - (a[j] * s0[j]) % OREF_Q0);
  return acc % OREF_Q0;
}

void oref_br1(const oref_ctx *ctx, const uint16_t *lwe_a, uint16_t lwe_b, uint64_t *rlwe_out) {
  uint32_t a[OREF_N0];
  for (int j = 0; j < OREF_N0; ++j) a[j] = lwe_a[j]; /* q0 == 2*N1: no modulus switch (:519-529) */
  blind_rotate(1, ctx->lut1, a, lwe_b, OREF_N0, ctx->bsk1, rlwe_out);
}

/* first_level_bootstrapping, detector.rs:533-597 */
void oref_first_level(const oref_ctx *ctx, const uint16_t *clue_a, const uint16_t *clue_b,
                      uint32_t *lwe_int) {
  const uint64_t q = OREF_Q1;
  uint64_t sum[2 * OREF_N1], r[2 * OREF_N1];
  memset(sum, 0, sizeof(sum));
  for (int c = 0; c < OREF_CLUES; ++c) {
    uint16_t la[OREF_N0], lb;
    oref_extract_clue(clue_a, clue_b, c, la, &lb);
    oref_br1(ctx, la, lb, r);
    for (int j = 0; j < 2 * OREF_N1; ++j) sum[j] = addmod(sum[j], r[j], q); /* :556 */
  }
  /* extract_lwe_locally (coefficient 0), :561 */
  uint64_t ea[OREF_N1];
  ea[0] = sum[0];
  for (int j = 1; j < OREF_N1; ++j) ea[j] = negmod(sum[OREF_N1 - j], q);
  uint64_t eb = sum[OREF_N1];
  /* NonPowOf2LweKeySwitchingKey::key_switch, :560-563 */
  uint64_t ka[OREF_NI];
  memset(ka, 0, sizeof(ka));
  uint64_t kb = eb;
  for (int i = 0; i < OREF_N1; ++i) {
    for (int j = 0; j < OREF_KS_DIGITS; ++j) {
      if (!((ea[i] >> j) & 1)) continue;
      const uint32_t *row = ctx->ksk + ((size_t)i * OREF_KS_DIGITS + j) * KSK_ROW;
      for (int c = 0; c < OREF_NI; ++c) ka[c] = submod(ka[c], row[c], q);
      kb = submod(kb, row[OREF_NI], q);
    }
  }
  /* lwe_modulus_switch q1 -> 4096 (:571-575), then b += clue_count * 4096/32 (:577-594) */
  for (int c = 0; c < OREF_NI; ++c) lwe_int[c] = (uint32_t)oref_modswitch_q1_to_qi(ka[c]);
  lwe_int[OREF_NI] =
      (uint32_t)((oref_modswitch_q1_to_qi(kb) + OREF_CLUES * (OREF_QI / OREF_TI)) % OREF_QI);
}

/* second_level_bootstrapping, detector.rs:599-624 (4096 == 2*N2: no modulus switch) */
void oref_br2(const oref_ctx *ctx, const uint32_t *lwe_int, uint64_t *rlwe_out) {
  blind_rotate(2, ctx->lut2, lwe_int, lwe_int[OREF_NI], OREF_NI, ctx->bsk2, rlwe_out);
}

/* hom_trace, detector.rs:626-639 */
void oref_trace(const oref_ctx *ctx, const uint64_t *rlwe_in, uint64_t *ntt_out) {
  const ntt_tab *t = &g_tab[2];
  const uint64_t q = OREF_Q2;
  const int N = OREF_N2;
  uint64_t *a = malloc(sizeof(uint64_t) * N * 8);
  uint64_t *b = a + N, *sa = b + N, *sb = sa + N, *A = sb + N, *B = A + N, *D = B + N;
  int64_t dg[OREF_DT];
  uint64_t *dig = malloc(sizeof(uint64_t) * N * OREF_DT);
  for (int j = 0; j < N; ++j) {
    a[j] = mulmod(rlwe_in[j], ctx->ninv2, q); /* mul_shoup_scalar_assign(n_inv), :635-636 */
    b[j] = mulmod(rlwe_in[N + j], ctx->ninv2, q);
  }
  for (int k = 0; k < OREF_TRACE_STEPS; ++k) {
    const uint32_t g = (uint32_t)(N >> k) + 1;
    automorphism(a, g, sa);
    automorphism(b, g, sb);
    for (int j = 0; j < N; ++j) {
      decompose(&g_basis[3], sa[j], dg);
      for (int l = 0; l < OREF_DT; ++l)
        dig[(size_t)l * N + j] = dg[l] < 0 ? (uint64_t)(dg[l] + (int64_t)q) : (uint64_t)dg[l];
    }
    memset(A, 0, sizeof(uint64_t) * N);
    memset(B, 0, sizeof(uint64_t) * N);
    for (int l = 0; l < OREF_DT; ++l) {
      memcpy(D, dig + (size_t)l * N, sizeof(uint64_t) * N);
      ntt_fwd(t, D);
      const uint64_t *ka = ctx->tk + ((size_t)k * OREF_DT + l) * 2 * N;
      const uint64_t *kb = ka + N;
      for (int j = 0; j < N; ++j) {
        A[j] = addmod(A[j], mulmod(D[j], ka[j], q), q);
        B[j] = addmod(B[j], mulmod(D[j], kb[j], q), q);
      }
    }
    ntt_inv(t, A);
    ntt_inv(t, B);
    for (int j = 0; j < N; ++j) {
      a[j] = addmod(a[j], A[j], q);
      b[j] = addmod(b[j], addmod(sb[j], B[j], q), q);
    }
  }
  ntt_fwd(t, a); /* to_ntt_rlwe, :638 */
  ntt_fwd(t, b);
  memcpy(ntt_out, a, sizeof(uint64_t) * N);
  memcpy(ntt_out + N, b, sizeof(uint64_t) * N);
  free(dig);
  free(a);
}

void oref_detect(const oref_ctx *ctx, const uint16_t *clue_a, const uint16_t *clue_b,
                 uint64_t *out) {
  uint32_t lwe[OREF_NI + 1];
  uint64_t *r = malloc(sizeof(uint64_t) * 2 * OREF_N2);
  oref_first_level(ctx, clue_a, clue_b, lwe);
  oref_br2(ctx, lwe, r);
  oref_trace(ctx, r, out);
  free(r);
}

void oref_detect_batch(const oref_ctx *ctx, const uint16_t *clue_a, const uint16_t *clue_b,
                       size_t D, uint64_t *out, int nthreads) {
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
#endif
  for (long m = 0; m < (long)D; ++m)
    oref_detect(ctx, clue_a + (size_t)m * OREF_N0, clue_b + (size_t)m * OREF_CLUES,
                out + (size_t)m * 2 * OREF_N2);
  (void)nthreads;
}

/* ------------------------------------------------------------------------------------------
 * Digest encoding (detector.rs:223-453)
 * ---------------------------------------------------------------------------------------- */
void oref_get_retrieval_params(size_t all, size_t pertinent, oref_retrieval_params *rp) {
  /* RetrievalParams::new(p=257 (non-pow2), N=2048, all, pertinent, 130, 25, 2) */
  const uint64_t p = OREF_P;
  uint32_t pw = 0;
  uint64_t acc = 1;
  while (acc * p <= all) { acc *= p; pw++; } /* ilog(all, p) */
  if (acc < all) pw++;                        /* p^pow < all -> pow += 1 */
  if (pw == 0) pw = 1;
  rp->index_slots_per_bucket = pw;
  rp->slots_per_bucket = pw + 1;
  rp->slots_per_segment = rp->slots_per_bucket * 130;
  rp->segment_per_cipher = OREF_N2 / rp->slots_per_segment;
  rp->max_encode_indices_cipher_count = 25 / rp->segment_per_cipher;
  rp->combination_count = (uint32_t)pertinent + 5;
  rp->cmb_count_per_cipher = 2;
  rp->cmb_cipher_count = (rp->combination_count + 1) / 2;
}

uint32_t oref_bucket(uint64_t seed, uint32_t ct, uint64_t i, uint32_t s) {
  const uint32_t key[8] = {(uint32_t)seed, (uint32_t)(seed >> 32), 0x6f6d7262u /* "omrb" */, ct,
                           0, 0, 0, 0};
  uint32_t w[16];
  oref_chacha_block(12, key, i, 0x62756b74u /* "bukt" */, w);
  return (uint32_t)(((uint64_t)w[s & 15] * 130u) >> 32);
}

static inline uint64_t centered_lift(uint64_t v) {
  /* v < half_p ? v : q - p + v, detector.rs:294,309,431 */
  return v < (OREF_P + 1) / 2 ? v : OREF_Q2 - OREF_P + v;
}

void oref_encode_indices(const uint64_t *pv, size_t D, size_t off, size_t all, uint64_t seed,
                         uint32_t ct, uint64_t *out) {
  oref_retrieval_params rp;
  oref_get_retrieval_params(all, 0, &rp);
  const int N = OREF_N2;
  const uint64_t q = OREF_Q2;
  uint64_t P[OREF_N2];
  memset(out, 0, sizeof(uint64_t) * 2 * N);
  for (size_t m = 0; m < D; ++m) {
    const uint64_t gi = off + m;
    memset(P, 0, sizeof(P));
    for (uint32_t s = 0; s < rp.segment_per_cipher; ++s) {
      const uint32_t bucket = oref_bucket(seed, ct, gi, s);
      const uint32_t addr = s * rp.slots_per_segment + bucket * rp.slots_per_bucket;
      uint64_t v = gi;
      uint32_t k = 0;
      while (v) {
        uint64_t dgt = v % OREF_P;
        P[addr + k] = centered_lift(dgt);
        v = (v - dgt) / OREF_P;
        k++;
      }
      P[addr + rp.index_slots_per_bucket] = 1;
    }
    ntt_fwd(&g_tab[2], P);
    const uint64_t *pa = pv + m * 2 * N, *pb = pa + N;
    for (int j = 0; j < N; ++j) {
      out[j] = addmod(out[j], mulmod(pa[j], P[j], q), q);
      out[N + j] = addmod(out[N + j], mulmod(pb[j], P[j], q), q);
    }
  }
}

void oref_encode_payloads(const uint64_t *pv, const uint16_t *payloads, size_t D, size_t off,
                          size_t all, const uint16_t *weights, uint32_t n_ct, uint32_t per_ct,
                          uint64_t *out) {
  const int N = OREF_N2;
  const uint64_t q = OREF_Q2;
  uint64_t P[OREF_N2];
  memset(out, 0, sizeof(uint64_t) * 2 * N * n_ct);
  for (uint32_t c = 0; c < n_ct; ++c) {
    uint64_t *o = out + (size_t)c * 2 * N;
    for (size_t m = 0; m < D; ++m) {
      const uint64_t gi = off + m;
      memset(P, 0, sizeof(P));
      for (uint32_t j = 0; j < per_ct; ++j) {
        const uint32_t w = weights[(size_t)(c * per_ct + j) * all + gi];
        for (int l = 0; l < OREF_PAYLOAD_LEN; ++l) {
          uint32_t v = ((uint32_t)payloads[m * OREF_PAYLOAD_LEN + l] * w) % OREF_P;
          P[j * OREF_PAYLOAD_LEN + l] = centered_lift(v);
        }
      }
      ntt_fwd(&g_tab[2], P);
      const uint64_t *pa = pv + m * 2 * N, *pb = pa + N;
      for (int j = 0; j < N; ++j) {
        o[j] = addmod(o[j], mulmod(pa[j], P[j], q), q);
        o[N + j] = addmod(o[N + j], mulmod(pb[j], P[j], q), q);
      }
    }
  }
}

uint64_t oref_payload_weights(const uint8_t seed[32], size_t count, uint16_t *out) {
  uint32_t key[8];
  for (int i = 0; i < 8; ++i)
    key[i] = (uint32_t)seed[4 * i] | ((uint32_t)seed[4 * i + 1] << 8) |
             ((uint32_t)seed[4 * i + 2] << 16) | ((uint32_t)seed[4 * i + 3] << 24);
  uint32_t buf[16];
  uint64_t block = 0, rejected = 0;
  int pos = 16;
  size_t n = 0;
  while (n < count) {
    if (pos == 16) {
      oref_chacha_block(12, key, block++, 0, buf);
      pos = 0;
    }
    const uint32_t v = buf[pos++];
    const uint64_t m = (uint64_t)v * OREF_P; /* UniformInt<u16>::sample, range 257, zone 2^32-2 */
    if ((uint32_t)m > 0xFFFFFFFEu) {
      rejected++;
      continue;
    }
    out[n++] = (uint16_t)(m >> 32);
  }
  return rejected;
}

/* ------------------------------------------------------------------------------------------
 * Client-side helpers (retriever.rs, omd.rs)
 * ---------------------------------------------------------------------------------------- */
void oref_decrypt_ntt(const int8_t *s2, const uint64_t *ct, uint64_t *out) {
  const int N = OREF_N2;
  const uint64_t q = OREF_Q2;
  uint64_t S[OREF_N2];
  for (int j = 0; j < N; ++j) S[j] = s2[j] < 0 ? q - (uint64_t)(-s2[j]) : (uint64_t)s2[j];
  ntt_fwd(&g_tab[2], S);
  for (int j = 0; j < N; ++j) out[j] = submod(ct[N + j], mulmod(ct[j], S[j], q), q);
  ntt_inv(&g_tab[2], out);
}

uint32_t oref_decode_coeff(uint64_t c) {
  uint64_t t = (2 * c * OREF_P + OREF_Q2) / (2 * OREF_Q2);
  return (uint32_t)(t >= OREF_P ? t - OREF_P : t);
}

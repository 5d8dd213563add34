/*
 * omr_oracle.h — CPU restatement of the InstantOMR detect path (TEST INFRASTRUCTURE ONLY).
 *
 * This library is the parity oracle for the MI355X detector. Only tests/, the smoke check in
 * __graft_entry__.py and the cpu_baseline leg of bench.py may load it; the product path
 * (tfhe-omr_amd/) never links or calls it.
 *
 * Parity status: the reference's arithmetic lives in the un-vendored primus-fhe crates
 * (git branch omr2, commit unpinned), so bit-level parity against the
 * reference is UNPINNED. Every bit-level convention the reference leaves to primus-fhe is
 * fixed here (see "Conventions" below) and the oracle is pinned by (1) Python big-integer
 * golden vectors for each primitive (tests/golden/), (2) the reference's own functional KATs:
 * omd.rs:48-58 (decrypt(detect(pertinent)) == [1,0,..,0], else all 0) and
 * omr_time_analyze.rs:215-235 (end-to-end index/payload recovery), and (3) the reference's
 * constant tables (LUT values detector.rs:457-503, retrieval layout retrieval_params.rs:50-106,
 * INV_MOD_257 matrix.rs:27-41).
 *
 * Conventions (shared with include/omr_gpu.h):
 *  - RLWE ciphertext (a, b) with b = a*s + e + m over Z_q[X]/(X^N+1); decrypt m = b - a*s.
 *  - LWE ciphertext (a, b) with b = <a,s> + e + m.
 *  - NTT: psi = g^((q-1)/2N), g the smallest primitive root of q (g=7 for q1, g=22 for q2).
 *    Forward NTT output index j holds a(psi^(2*brv(j)+1)) (bit-reversed evaluation order).
 *  - GGSW(m), gadget g_k = 2^(drop + k*logB), k<d:
 *      row k      = (alpha_k + m*g_k, alpha_k*s + e_k)        (a-gadget rows)
 *      row d + k  = (alpha'_k, alpha'_k*s + e'_k + m*g_k)     (b-gadget rows)
 *  - Approximate signed decomposition of x in [0,q): centre x into [-(q-1)/2,(q-1)/2],
 *    y = floor((x + 2^(drop-1)) / 2^drop) (drop>0), then d-1 balanced digits
 *    c = floor((y + B/2)/B), d_k = y - c*B in [-B/2, B/2), y = c; top digit d_{d-1} = y.
 *  - Blind rotation (binary key): ACC = (0, X^{-b}*LUT); for i: ACC += ((X^{a_i}-1)*ACC) [x] BSK_i.
 *  - LWE key switch (27 binary digits, unsigned): out = (0,b) - sum_{i,j} bit_j(a_i) * KSK[i][j],
 *    KSK[i][j] = LWE_{s_int}(s1_i * 2^j).
 *  - Modulus switch q1 -> 4096: round-half-up of v*4096/q1.
 *  - Trace: c *= N^{-1}; for k = 0..10: g = (N>>k)+1, c += KS_k(sigma_g(c)),
 *    TK[k][j] = (alpha, alpha*s + e - sigma_g(s)*4^j), KS_k(a',b') = (sum d_j alpha, b' + sum d_j beta).
 */
#ifndef OMR_ORACLE_H
#define OMR_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Parameter set: omr_core/src/parameters/mod.rs:39-105 */
#define OREF_N0 512          /* clue LWE dimension, mod.rs:40-46 */
#define OREF_Q0 2048         /* clue modulus */
#define OREF_T0 8            /* clue plaintext modulus */
#define OREF_CLUES 7         /* mod.rs:48 */
#define OREF_Q1 134215681ull /* FirstLevelField, mod.rs:18 */
#define OREF_N1 1024
#define OREF_LOGB1 5
#define OREF_D1 4
#define OREF_DROP1 7
#define OREF_KS_DIGITS 27    /* KS log_basis=1 over 27-bit q1, mod.rs:58-66 */
#define OREF_NI 670          /* intermediate LWE, mod.rs:68-74 */
#define OREF_QI 4096
#define OREF_TI 32
#define OREF_Q2 1125899906826241ull /* SecondLevelField, mod.rs:21 */
#define OREF_N2 2048
#define OREF_LOGB2 7
#define OREF_D2 6
#define OREF_DROP2 8
#define OREF_LOGBT 2
#define OREF_DT 25           /* trace basis (q2, 2, None), mod.rs:84-90 */
#define OREF_TRACE_STEPS 11
#define OREF_P 257           /* output plain modulus, mod.rs:93 */
#define OREF_PAYLOAD_LEN 612 /* payload.rs:8 */

/* ---- primitives (exported for golden-vector tests) ---- */
/* level: 1 -> (q1, N1), 2 -> (q2, N2) */
void oref_ntt_forward(int level, uint64_t *a);
void oref_ntt_inverse(int level, uint64_t *a);
/* which: 1 = BR1 basis, 2 = BR2 basis, 3 = trace basis. Returns digit count. */
int oref_decompose(int which, uint64_t x, int64_t *digits);
uint64_t oref_modswitch_q1_to_qi(uint64_t v);
void oref_first_level_lut(uint64_t *lut);  /* N1 entries */
void oref_second_level_lut(uint64_t *lut); /* N2 entries */
void oref_negacyclic_mul_monomial(int level, const uint64_t *p, uint32_t r, uint64_t *out);
void oref_automorphism(const uint64_t *p, uint32_t g, uint64_t *out); /* level 2 */
void oref_chacha_block(int rounds, const uint32_t key[8], uint64_t counter, uint64_t stream,
                       uint32_t out[16]);

/* ---- detect path ---- */
typedef struct oref_ctx oref_ctx;
/* Keys in the canonical coefficient-domain layout (include/omr_gpu.h):
 * bsk1 u32 [512][8][2][1024], ksk u32 [1024][27][671], bsk2 u64 [670][12][2][2048],
 * tk u64 [11][25][2][2048]. The context keeps NTT-domain copies. */
oref_ctx *oref_create(const uint32_t *bsk1, const uint32_t *ksk, const uint64_t *bsk2,
                      const uint64_t *tk);
void oref_destroy(oref_ctx *ctx);

/* Stage functions (detector.rs:505-639). clue_a: 512 u16 (mod 2048), clue_b: 7 u16. */
void oref_extract_clue(const uint16_t *clue_a, const uint16_t *clue_b, int i, uint16_t *lwe_a,
                       uint16_t *lwe_b);
void oref_br1(const oref_ctx *ctx, const uint16_t *lwe_a, uint16_t lwe_b, uint64_t *rlwe_out);
void oref_first_level(const oref_ctx *ctx, const uint16_t *clue_a, const uint16_t *clue_b,
                      uint32_t *lwe_int /* 671: a[670], b; mod 4096 */);
void oref_br2(const oref_ctx *ctx, const uint32_t *lwe_int, uint64_t *rlwe_out);
void oref_trace(const oref_ctx *ctx, const uint64_t *rlwe_in, uint64_t *ntt_out);
void oref_detect(const oref_ctx *ctx, const uint16_t *clue_a, const uint16_t *clue_b,
                 uint64_t *out /* 2*2048 NTT domain: a then b */);
/* D messages, OpenMP over messages with nthreads threads (<=0: all). */
void oref_detect_batch(const oref_ctx *ctx, const uint16_t *clue_a, const uint16_t *clue_b,
                       size_t D, uint64_t *out, int nthreads);

/* ---- digest encoding (detector.rs:223-453) ---- */
/* RetrievalParams::new(257, 2048, D, pertinent, 130, 25, 2) — retrieval_params.rs:50-106 */
typedef struct {
  uint32_t index_slots_per_bucket, slots_per_bucket, slots_per_segment, segment_per_cipher,
      max_encode_indices_cipher_count, combination_count, cmb_count_per_cipher, cmb_cipher_count;
} oref_retrieval_params;
void oref_get_retrieval_params(size_t all_payloads_count, size_t pertinent_count,
                           oref_retrieval_params *rp);
/* Bucket of segment s for global message i in index ciphertext ct (seeded replacement for the
 * reference's thread_rng, detector.rs:262,278). */
uint32_t oref_bucket(uint64_t seed, uint32_t ct, uint64_t i, uint32_t s);
/* pv: D NTT-domain RLWE (2*2048 u64 each) for global indices [offset, offset+D). */
void oref_encode_indices(const uint64_t *pv, size_t D, size_t global_offset,
                         size_t all_payloads_count, uint64_t seed, uint32_t ct,
                         uint64_t *out /* 2*2048 */);
/* weights: u16 [cmb_cipher_count*cmb_per_ct][all_payloads_count] (oref_payload_weights). */
void oref_encode_payloads(const uint64_t *pv, const uint16_t *payloads, size_t D,
                          size_t global_offset, size_t all_payloads_count, const uint16_t *weights,
                          uint32_t n_ct, uint32_t cmb_per_ct, uint64_t *out /* n_ct*2*2048 */);
/* StdRng::from_seed(seed) (ChaCha12) + Uniform<u16>(0,257): detector.rs:376-387 and
 * retriever.rs:215-226; count draws into out. Returns number of rejected samples. */
uint64_t oref_payload_weights(const uint8_t seed[32], size_t count, uint16_t *out);

/* ---- key and clue generation (omr_oracle_keygen.c: key_gen/secret.rs:46-178,
 *      key_gen/clue.rs:27-34; seeded ChaCha12 streams documented there) ---- */
typedef struct {
  uint8_t s0[OREF_N0];    /* clue LWE key, binary */
  int8_t s1[OREF_N1];     /* first-level RLWE key, ternary */
  uint8_t s_int[OREF_NI]; /* intermediate LWE key, binary */
  int8_t s2[OREF_N2];     /* second-level RLWE key, ternary */
  uint16_t pk_a[OREF_N0], pk_b[OREF_N0]; /* LwePublicKeyRlweMode (A, B = A s0 + E) */
} oref_secret_pack;
void oref_keygen_secret(uint64_t seed, oref_secret_pack *sk);
/* Keys in the layout of oref_create; OpenMP over key rows with nthreads threads. */
void oref_keygen_detection_key(const oref_secret_pack *sk, uint64_t seed, uint32_t *bsk1, uint32_t *ksk,
                               uint64_t *bsk2, uint64_t *tk, int nthreads);
/* Clues for global message indices [first, first + count): clue_a u16 [count][512],
 * clue_b u16 [count][7]. */
void oref_gen_clues(const oref_secret_pack *sk, uint64_t seed, uint64_t first, size_t count,
                    uint16_t *clue_a, uint16_t *clue_b, int nthreads);

/* ---- client-side helpers for KATs (retriever.rs, omd.rs) ---- */
/* s2: ternary secret (int8, 2048). ct: NTT-domain (a,b). out: coefficient-domain phase. */
void oref_decrypt_ntt(const int8_t *s2, const uint64_t *ct, uint64_t *out);
/* round(c * 257 / q2) mod 257, half up (retriever.rs:84-89) */
uint32_t oref_decode_coeff(uint64_t c);
/* LWE phase of a clue under s0: b_i - <a^(i), s0> mod 2048 */
uint32_t oref_clue_phase(const uint16_t *clue_a, const uint16_t *clue_b, int i, const uint8_t *s0);

#ifdef __cplusplus
}
#endif
#endif

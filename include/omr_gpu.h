/*
 * omr_gpu.h — C ABI of the MI355X-native InstantOMR detector (libomr_gpu.so).
 *
 * This is the drop-in boundary for the detect path of xiangxiecrypto/tfhe-omr. Each entry
 * point names the reference interface it replaces (file:line under omr_core/src/). A Rust
 * caller binds these with `extern "C"` declarations; Python tests and
 * bench.py bind them with ctypes. Plain C: no exceptions cross the boundary, every call
 * returns an omr_status and omr_last_error() returns the thread-local message of the last
 * failure.
 *
 * Data conventions (identical to the parity oracle, oracle/omr_oracle.h):
 *  - RLWE (a, b), b = a*s + e + m over Z_q[X]/(X^N+1). LWE (a, b), b = <a,s> + e + m.
 *  - NTT domain: index j holds p(psi^(2*brv(j)+1)), psi = g^((q-1)/2N), g = 7 (q1), 22 (q2).
 *  - Keys cross the boundary in the COEFFICIENT domain, canonical residues in [0, q):
 *      bsk1      u32 [512][8][2][1024]   GGSW_{s1}(s0_i), rows 0..3 a-gadget, 4..7 b-gadget
 *      ksk       u32 [1024][27][671]     LWE_{s_int}(s1_i * 2^j): a[670], b
 *      bsk2      u64 [670][12][2][2048]  GGSW_{s2}(s_int_i), rows 0..5 a-gadget, 6..11 b-gadget
 *      trace_key u64 [11][25][2][2048]   step k (g = 2048/2^k + 1), digit j:
 *                                        (alpha, alpha*s2 + e - sigma_g(s2) * 4^j)
 *    GGSW(m) row k = (alpha_k + m*g_k, alpha_k*s + e_k); row d+k = (alpha', alpha'*s + e' + m*g_k),
 *    gadget g_k = 2^(drop + k*logB): BR1 (logB 5, d 4, drop 7), BR2 (logB 7, d 6, drop 8).
 *  - A clue (CmLweCiphertext<u16>) is mask a[512] and bodies b[7], values mod 2048.
 *  - A pertinency ciphertext (NttRlweCiphertext<SecondLevelField>) is u64 [2][2048] (a then b),
 *    NTT domain, canonical residues mod q2.
 */
#ifndef OMR_GPU_H
#define OMR_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Parameter set: omr_core/src/parameters/mod.rs:39-105 */
#define OMR_N0 512
#define OMR_Q0 2048
#define OMR_CLUE_COUNT 7
#define OMR_Q1 134215681u
#define OMR_N1 1024
#define OMR_KS_DIGITS 27
#define OMR_NI 670
#define OMR_QI 4096
#define OMR_Q2 1125899906826241ull
#define OMR_N2 2048
#define OMR_TRACE_STEPS 11
#define OMR_TRACE_DIGITS 25
#define OMR_P 257
#define OMR_PAYLOAD_LEN 612

typedef enum {
  OMR_OK = 0,
  OMR_ERR_INVALID_ARGUMENT = 1,
  OMR_ERR_DEVICE = 2,
  OMR_ERR_OUT_OF_MEMORY = 3,
  OMR_ERR_NOT_INVERTIBLE = 4 /* OmrError::InvertibleMatrix, error.rs:5-8 */
} omr_status;

/* Message of the last failing call on this thread ("" if none). */
const char *omr_last_error(void);
/* Library / build identification, e.g. "omr_gpu 0.1 gfx950". */
const char *omr_version(void);

/* ---------------------------------------------------------------------------------------
 * Key generation (CPU) — KeyGen::generate_secret_key (key_gen/mod.rs:21-27),
 * SecretKeyPack::new (key_gen/secret.rs:46-95), generate_sender (:110), generate_detection_key
 * (:118-178). Deterministic from a 64-bit seed (counter-based ChaCha12 streams per key row),
 * so every rank of a multi-GPU job derives identical keys.
 * ------------------------------------------------------------------------------------- */
typedef struct omr_secret_key_pack omr_secret_key_pack;

omr_status omr_keygen_secret(uint64_t seed, omr_secret_key_pack **out);
void omr_secret_destroy(omr_secret_key_pack *sk);
/* Secret material for client-side checks: s0 (512 bits), s1 (1024 ternary), s_int (670 bits),
 * s2 (2048 ternary). Any pointer may be NULL. */
omr_status omr_secret_export(const omr_secret_key_pack *sk, uint8_t *s0, int8_t *s1,
                             uint8_t *s_int, int8_t *s2);
/* DetectionKey in the coefficient-domain layout above. nthreads <= 0: all host cores. */
omr_status omr_keygen_detection_key(const omr_secret_key_pack *sk, uint64_t seed, uint32_t *bsk1,
                                    uint32_t *ksk, uint64_t *bsk2, uint64_t *trace_key,
                                    int nthreads);
/* Sender::gen_clues (sender.rs:27-32, key_gen/clue.rs:27-34): `count` clues (7 encryptions of 0
 * under the pack's RLWE-mode public key) for global message indices [first, first+count).
 * clue_a u16 [count][512], clue_b u16 [count][7]. */
omr_status omr_gen_clues(const omr_secret_key_pack *sk, uint64_t seed, uint64_t first,
                         size_t count, uint16_t *clue_a, uint16_t *clue_b, int nthreads);
/* Device generators: the same streams as omr_gen_clues /
 * omr_keygen_detection_key, bit-identical output, written to device buffers of the current HIP
 * device on `stream` (a hipStream_t; NULL = default stream). Both return after the stream has
 * completed the work. */
omr_status omr_gen_clues_device(const omr_secret_key_pack *sk, uint64_t seed, uint64_t first,
                                size_t count, uint16_t *d_clue_a, uint16_t *d_clue_b, void *stream);
omr_status omr_keygen_detection_key_device(const omr_secret_key_pack *sk, uint64_t seed,
                                           uint32_t *d_bsk1, uint32_t *d_ksk, uint64_t *d_bsk2,
                                           uint64_t *d_trace_key, void *stream);

/* ---------------------------------------------------------------------------------------
 * Retrieval layout — RetrievalParams::new(257, 2048, all, pertinent, 130, 25, 2)
 * (parameters/retrieval_params.rs:50-106; arguments as in key_gen/secret.rs:189-209).
 * ------------------------------------------------------------------------------------- */
typedef struct {
  uint32_t index_slots_per_bucket, slots_per_bucket, slots_per_segment, segment_per_cipher,
      max_encode_indices_cipher_count, combination_count, cmb_count_per_cipher, cmb_cipher_count;
} omr_retrieval_params;
omr_status omr_get_retrieval_params(size_t all_payloads_count, size_t pertinent_count,
                                    omr_retrieval_params *out);
/* Payload weights: StdRng::from_seed(seed) + Uniform<u16>(0,257), drawn in the reference's
 * order (detector.rs:376-387): out[j*all + i] for combination j < combination_count, the rest
 * zero; out has cmb_cipher_count*cmb_count_per_cipher*all entries. */
omr_status omr_payload_weights(const uint8_t seed[32], size_t all_payloads_count,
                               uint32_t combination_count, uint32_t cmb_cipher_count,
                               uint32_t cmb_count_per_cipher, uint16_t *out);

/* ---------------------------------------------------------------------------------------
 * Retriever (client side, CPU): Retriever::decode_digest (retriever.rs:188-260).
 * ------------------------------------------------------------------------------------- */
/* Decrypt + decode n NttRlweCiphertexts (u64 [n][2][2048], NTT domain) under the pack's s2:
 * out[m][j] = round_half_up(phase_j * 257 / q2) mod 257 (retriever.rs:84-96). */
omr_status omr_decrypt_decode(const omr_secret_key_pack *sk, const uint64_t *ct, size_t n,
                              uint32_t *out);
/* decode_pertinent_indices over the index digest ciphertexts in order, stopping once
 * pertinent_count distinct indices are known (retriever.rs:63-130, :197-201). Writes up to cap
 * indices in increasing order and the number found (the caller compares it with the count). */
omr_status omr_retrieve_indices(const omr_secret_key_pack *sk, const uint64_t *idx_cts,
                                uint32_t n_ct, size_t all_payloads_count, size_t pertinent_count,
                                size_t *indices, size_t cap, size_t *found);
/* decode_combined_payloads + solve_matrix_mod_257 (retriever.rs:203-258, matrix.rs:164-247):
 * payloads u16 [n_indices][612] of the sorted retrieved indices, from the payload digest
 * ciphertexts and the board's weights (omr_payload_weights, same seed as the detector).
 * `combination_count` is the board's RetrievalParams::combination_count (the reference's matrix
 * has that many rows whatever the number of indices found, retriever.rs:196, :215-239); 0 takes
 * the count of a board whose pertinent count is n_indices. OMR_ERR_NOT_INVERTIBLE when the system
 * is singular. */
omr_status omr_retrieve_payloads(const omr_secret_key_pack *sk, const uint64_t *pay_cts,
                                 uint32_t n_ct, size_t all_payloads_count, uint32_t combination_count,
                                 const uint16_t *weights, const size_t *indices, size_t n_indices,
                                 uint16_t *payloads);

/* ---------------------------------------------------------------------------------------
 * Detector — one context per GPU; calls on one context are serialised; contexts are
 * independent. Detector::new (detector.rs:85-110) uploads the keys and converts them to the
 * device layout; the LUTs (:457-503) are built inside. The key view may point to host memory
 * or to device memory of `device` (e.g. from omr_keygen_detection_key_device).
 * ------------------------------------------------------------------------------------- */
typedef struct omr_ctx omr_ctx;

typedef struct {
  const uint32_t *bsk1;
  const uint32_t *ksk;
  const uint64_t *bsk2;
  const uint64_t *trace_key;
} omr_detection_key_view;

omr_status omr_ctx_create(const omr_detection_key_view *key, int device, omr_ctx **out);
void omr_ctx_destroy(omr_ctx *ctx);
/* Kernel names of this build's detect pipeline: "br1=<name> ks=<name> br2=<name>". */
const char *omr_detect_kernels(void);
/* Messages per internal detect chunk (memory/latency knob: 36 KiB of scratch per message);
 * 0 = the default 16,384. */
omr_status omr_ctx_set_batch(omr_ctx *ctx, size_t batch);
/* Chunks of at most `max_messages` messages run the latency kernels (each level-1 rotation
 * spread over more waves, each level-2 message over two CUs that exchange partial products
 * through global memory every step, or over two wave groups of one CU when the cooperative
 * launch of the two-CU grid is refused, and each message's trace over five CUs that all-reduce
 * their digit partials, or one CU when that launch is refused: lower single-message latency,
 * bit-identical output); larger chunks run the throughput kernels. Default 64; 0 = always
 * throughput. The multi-CU grids are launched with hipLaunchCooperativeKernel, so their
 * workgroups are co-resident; if a hand-off still does not complete, the kernel ends, its output
 * is invalid and the error is reported by omr_ctx_check (after the caller's stream sync), by the
 * host entry points, and by the next detect call on the context (which then returns
 * OMR_ERR_DEVICE without running). */
omr_status omr_ctx_set_latency_threshold(omr_ctx *ctx, size_t max_messages);
/* Synchronises `hip_stream` (NULL: the whole device) and reports a pending device-side
 * failure of an earlier call on the context (the two-CU hand-off timeout above) as
 * OMR_ERR_DEVICE, clearing it; OMR_OK when every call completed correctly. Callers of the
 * device entry points use it where they would otherwise only synchronise. */
omr_status omr_ctx_check(omr_ctx *ctx, void *hip_stream);
/* Exactness of the FFT external products. The level-1 rotations and the throughput
 * level-2 rotation compute each external product with FP64 FFTs and round every coefficient to the
 * integer it equals (the reference computes it with an exact NTT: detector.rs:553-557, :623 via
 * concrete-ntt, omr_core/Cargo.toml:38-45). With the guard on, the detect kernels run guarded
 * variants (same output, slower) that record the largest |y - rint(y)| over every rounded
 * coefficient: observed[0] level 1, observed[1] level 2, since context creation or the last reset.
 * apriori[l] is the proven bound E on |computed - exact| of every such coefficient for this key
 * (from kappa[l], the largest stored key-spectrum magnitude, computed at context creation): if
 * E < 0.5 the rounding is exact for every input; a run with observed < 1 - E is exact (an error
 * |e| in [0.5, E] would show a margin >= 1 - E). Any pointer may be NULL; reset != 0 zeroes the
 * observed margins after reading them. The read synchronises the device. */
omr_status omr_ctx_set_rounding_guard(omr_ctx *ctx, int enable);
omr_status omr_ctx_rounding_margin(omr_ctx *ctx, double observed[2], double apriori[2],
                                   double kappa[2], int reset);
/* The exactness contract. A level whose a priori bound E >= 0.5 runs its guarded
 * kernels on EVERY launch of the context, whatever omr_ctx_set_rounding_guard says; after each
 * such launch the observed margin m of that launch is compared with 1 - E on the device:
 *  - level 2: a launch with m >= 1 - E2 is re-run on the exact modular NTT (the latency family's
 *    br2l_kernel + trace), in the same stream order, so its outputs are exact;
 *  - level 1: a launch with m >= 1 - E1 is re-run on the exact modular NTT (br1n_fallback_kernel,
 *    br1_ntt.hpp) in the same stream order, so its outputs are exact.
 * guarded[l] != 0 when level l + 1 is guarded on every launch (automatically or by the user);
 * breaches[l] counts the launches of level l + 1 whose margin reached the threshold. Any pointer
 * may be NULL. Reading breaches synchronises the device. */
omr_status omr_ctx_exactness(omr_ctx *ctx, int guarded[2], uint64_t breaches[2]);
/* Level 1 on the exact modular NTT for every launch of the context (br1n_kernel: the reference's
 * own arithmetic, concrete-ntt in BlindRotationKey::blind_rotate, detector.rs:553-557), instead of the
 * FFT kernels; enable = 0 restores them. Outputs are bit-identical either way -- a cross-check of
 * the FFT path at any size, about 3x slower at level 1. */
omr_status omr_ctx_set_exact_level1(omr_ctx *ctx, int enable);
/* Diagnostics: `count` stored key-spectrum values (complex, re/im pairs) starting at value `first`
 * of level 1 (BSK1, [512][8][2][512], /512) or level 2 (BSK2 limbs, [670][12][2][2][1024], /1024),
 * in the kernels' storage order (register-major slots). */
omr_status omr_ctx_key_spectrum(omr_ctx *ctx, int level, size_t first, size_t count, double *out);
/* Diagnostics (host only, no GPU): the double-double twiddles of the key transform of `level`
 * (n - 1 entries, stage s node i at (1 << s) - 1 + i; per entry re.hi, re.lo, im.hi, im.lo). */
omr_status omr_fft_twiddles_dd(int level, double *out);
/* Encode workgroups fold ceil(D / max_chunks) messages each (at least 32, or 128 from D = 16,384),
 * so a call keeps at most `max_chunks` partial digests per ciphertext (32 KiB each); 0 = the
 * default 4,096. A memory knob: the digests are identical for every setting. */
omr_status omr_ctx_set_encode_chunks(omr_ctx *ctx, size_t max_chunks);

/* Detector::detect (detector.rs:135-166), batched like `par_iter().map(detect)` in
 * examples/omr.rs:160-164. Host buffers: clue_a u16 [D][512], clue_b u16 [D][7],
 * out u64 [D][2][2048] (NTT domain). */
omr_status omr_detect_batch(omr_ctx *ctx, const uint16_t *clue_a, const uint16_t *clue_b,
                            size_t D, uint64_t *out);
/* Detector::detect (detector.rs:135-138) for one message: clue_a u16 [512], clue_b u16 [7],
 * out u64 [2][2048]. Safe to call from many host threads at once on one context, as the
 * reference's `clues.par_iter().map(|c| detector.detect(c))` does on a shared &Detector
 * (examples/omr.rs:160-164): concurrent calls are coalesced into batched launches (whichever
 * caller finds no launch in progress takes every queued request, up to max_messages, as one
 * omr_detect_batch), so many callers reach batch throughput; a lone caller gets single-message
 * latency. Each caller returns when its own output is written. */
omr_status omr_detect(omr_ctx *ctx, const uint16_t *clue_a, const uint16_t *clue_b, uint64_t *out);
/* Coalescing knobs of omr_detect: at most max_messages per combined launch (0 = 65,536), and a
 * window (microseconds, default 0) a launching caller waits for more requests first. */
omr_status omr_ctx_set_coalescing(omr_ctx *ctx, size_t max_messages, long window_us);
/* omr_detect calls served and combined launches run so far on the context. */
omr_status omr_ctx_coalescing_stats(omr_ctx *ctx, size_t *calls, size_t *launches);
/* Same on device buffers, enqueued on `hip_stream` (NULL = HIP's null stream, which orders with
 * the other blocking streams, as in every HIP API); returns once enqueued. Calls on one context may use different streams: they share the
 * context's scratch, so a call's kernels wait (hipStreamWaitEvent) for those of the previous
 * call on another stream; the caller orders its own buffers. */
omr_status omr_detect_batch_device(omr_ctx *ctx, const uint16_t *d_clue_a,
                                   const uint16_t *d_clue_b, size_t D, uint64_t *d_out,
                                   void *hip_stream);

/* Detector::detect_with_time_info (detector.rs:169-221): device time per stage of the last detect
 * call, milliseconds, summed over its messages like DetectTimeInfo (detector.rs:51-57):
 *   total_ms        total_detect_time                      = first_level + second_level + trace
 *   first_level_ms  total_first_level_bootstrapping_time   7 rotations + sum + key switch + mod switch
 *   second_level_ms total_second_level_bootstrapping_time  level-2 blind rotation
 *   trace_ms        total_trace_time                       hom_trace + NTT
 *   key_switch_ms   the sum + key-switch + mod-switch part of first_level_ms (two_level_bs.rs:62-73)
 * Timing modes (omr_ctx_enable_timing): 0 off; 1 stage events around the production kernels —
 * the throughput path fuses the trace into the level-2 kernel, so there trace_ms is 0,
 * second_level_ms includes it and trace_separate is 0; 2 the reference's split: the throughput
 * path runs the level-2 rotation and the trace as two launches (same output, slightly slower),
 * trace_separate = 1. The latency kernels always run the trace as its own launch. */
typedef struct {
  float total_ms, first_level_ms, second_level_ms, trace_ms, key_switch_ms;
  size_t messages;
  int trace_separate;
} omr_detect_timing;
omr_status omr_ctx_enable_timing(omr_ctx *ctx, int mode);
omr_status omr_last_timing(omr_ctx *ctx, omr_detect_timing *t);
/* omr_detect_batch in timing mode 2 and omr_last_timing as one call under the context's lock
 * (concurrent callers cannot switch timing off under each other or read another call's times);
 * the context's timing mode is left as it was. */
omr_status omr_detect_with_time_info(omr_ctx *ctx, const uint16_t *clue_a, const uint16_t *clue_b,
                                     size_t D, uint64_t *out, omr_detect_timing *t);

/* Detector::encode_pertinent_indices (detector.rs:223-339) for index ciphertext `ct` over the
 * messages with global indices [global_offset, global_offset+D) of an all_payloads_count board.
 * Buckets come from a seeded counter-based stream (the reference uses thread_rng, :262) so
 * that shards agree. out u64 [2][2048] (NTT domain), a partial digest summed mod q2 across
 * shards. */
omr_status omr_encode_indices(omr_ctx *ctx, const uint64_t *pv, size_t D, size_t global_offset,
                              size_t all_payloads_count, uint64_t seed, uint32_t ct,
                              uint64_t *out);
omr_status omr_encode_indices_device(omr_ctx *ctx, const uint64_t *d_pv, size_t D,
                                     size_t global_offset, size_t all_payloads_count,
                                     uint64_t seed, uint32_t first_ct, uint32_t n_ct,
                                     uint64_t *d_out /* [n_ct][2][2048] */, void *hip_stream);
/* Detector::encode_pertinent_payloads (detector.rs:341-453). weights: omr_payload_weights()
 * output for the whole board; payloads u16 [D][612]; out u64 [n_ct][2][2048]. */
omr_status omr_encode_payloads(omr_ctx *ctx, const uint64_t *pv, const uint16_t *payloads,
                               size_t D, size_t global_offset, size_t all_payloads_count,
                               const uint16_t *weights, uint32_t n_ct, uint32_t cmb_per_ct,
                               uint64_t *out);
omr_status omr_encode_payloads_device(omr_ctx *ctx, const uint64_t *d_pv,
                                      const uint16_t *d_payloads, size_t D, size_t global_offset,
                                      size_t all_payloads_count, const uint16_t *d_weights,
                                      uint32_t n_ct, uint32_t cmb_per_ct, uint64_t *d_out,
                                      void *hip_stream);

/* ---------------------------------------------------------------------------------------
 * Stage entry points (for parity tests and per-stage benchmarks, benches/two_level_bs.rs).
 * Host buffers.
 * ------------------------------------------------------------------------------------- */
/* First level (detector.rs:533-597) for D messages: out u32 [D][671] (a[670], b mod 4096). */
omr_status omr_first_level(omr_ctx *ctx, const uint16_t *clue_a, const uint16_t *clue_b,
                           size_t D, uint32_t *lwe_int);
/* One level-1 blind rotation per LWE (a u16 [n][512], b u16 [n]): out u64 [n][2][1024]. */
omr_status omr_blind_rotate_level1(omr_ctx *ctx, const uint16_t *lwe_a, const uint16_t *lwe_b,
                                   size_t n, uint64_t *out);
/* Negacyclic product a * k mod (X^1024 + 1, q1) of n pairs through the level-1 FFT external-
 * product path (device_fft.hpp): a u32 [n][1024] with digit-sized centred values (|a| <= 17),
 * k u32 [n][1024] canonical; out u64 [n][1024] canonical. */
omr_status omr_fft1_mul(omr_ctx *ctx, const uint32_t *a, const uint32_t *k, size_t n,
                        uint64_t *out);
/* Second level + trace (detector.rs:599-639) on LWE(670, 4096) inputs: out u64 [n][2][2048]. */
omr_status omr_second_level(omr_ctx *ctx, const uint32_t *lwe_int, size_t n, uint64_t *out);
/* Level-2 blind rotation only (no trace): out u64 [n][2][2048] coefficient domain. */
omr_status omr_blind_rotate_level2(omr_ctx *ctx, const uint32_t *lwe_int, size_t n,
                                   uint64_t *out);
/* Forward / inverse NTT of n polynomials (level 1: N=1024 mod q1, level 2: N=2048 mod q2). */
omr_status omr_ntt(int level, int inverse, uint64_t *polys, size_t n, int device);

#ifdef __cplusplus
}
#endif
#endif

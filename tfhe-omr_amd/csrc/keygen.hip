// Host-side key generation, clue generation and digest-layout helpers (CPU).
//
// Mirrors omr_core's KeyGen / SecretKeyPack / Sender (key_gen/mod.rs:16-27,
// key_gen/secret.rs:46-209, key_gen/clue.rs:27-34, sender.rs:27-32) and the seeded weight
// stream of Detector::encode_pertinent_payloads (detector.rs:376-387). Every random draw comes
// from a ChaCha12 stream keyed by (seed, domain) whose stream id is the key row (or the global
// message index for clues), so results do not depend on thread count or sharding.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "host_ring.hpp"
#include "rng.hpp"

namespace omr {

static thread_local std::string g_last_error;

omr_status set_error(omr_status st, const std::string &msg) {
  g_last_error = msg;
  return st;
}

}  // namespace omr

// ==========================================================================================
// SecretKeyPack (key_gen/secret.rs:17-95)
// ==========================================================================================

using namespace omr;

extern "C" const char *omr_last_error(void) { return omr::g_last_error.c_str(); }
extern "C" const char *omr_version(void) { return "omr_gpu 0.1 gfx950"; }

extern "C" omr_status omr_keygen_secret(uint64_t seed, omr_secret_key_pack **out) {
  if (!out) return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_keygen_secret: out is NULL");
  auto sk = std::make_unique<omr_secret_key_pack>();
  sk->seed = seed;
  {
    Stream s(seed, DOM_S0, 0);
    for (int i = 0; i < N0; ++i) sk->s0[i] = (uint8_t)s.bit();
  }
  {
    Stream s(seed, DOM_S1, 0);
    for (int i = 0; i < N1; ++i) sk->s1[i] = (int8_t)s.ternary();
  }
  {
    Stream s(seed, DOM_SINT, 0);
    for (int i = 0; i < NI; ++i) sk->sint[i] = (uint8_t)s.bit();
  }
  {
    Stream s(seed, DOM_S2, 0);
    for (int i = 0; i < N2; ++i) sk->s2[i] = (int8_t)s.ternary();
  }
  {  // public key: B = A * s0 + E over Z_2048[X]/(X^512+1)
    Stream sa(seed, DOM_PK_A, 0), se(seed, DOM_PK_E, 0);
    Gaussian g(SIGMA_CLUE);
    int32_t b[N0];
    for (int i = 0; i < N0; ++i) sk->pk_a[i] = (uint16_t)(sa.next32() & (Q0 - 1));
    for (int i = 0; i < N0; ++i) b[i] = (int32_t)g.sample(se);
    for (int t = 0; t < N0; ++t) {
      if (!sk->s0[t]) continue;
      for (int i = 0; i < N0; ++i) {
        int e = i + t;
        if (e < N0) b[e] += sk->pk_a[i];
        else b[e - N0] -= sk->pk_a[i];
      }
    }
    for (int i = 0; i < N0; ++i) sk->pk_b[i] = (uint16_t)(((b[i] % Q0) + Q0) % Q0);
  }
  auto ntt_of = [](const int8_t *s, int N, uint64_t q, const auto &tab, std::vector<uint64_t> &v,
                   std::vector<uint64_t> &vs) {
    v.resize(N);
    vs.resize(N);
    for (int i = 0; i < N; ++i) v[i] = to_mod(s[i], q);
    tab.fwd(v.data());
    for (int i = 0; i < N; ++i) vs[i] = tab.pre(v[i]);
  };
  ntt_of(sk->s1, N1, Q1, ntt1(), sk->s1_ntt, sk->s1_ntts);
  ntt_of(sk->s2, N2, Q2, ntt2(), sk->s2_ntt, sk->s2_ntts);
  *out = sk.release();
  return OMR_OK;
}

extern "C" void omr_secret_destroy(omr_secret_key_pack *sk) { delete sk; }

extern "C" omr_status omr_secret_export(const omr_secret_key_pack *sk, uint8_t *s0, int8_t *s1,
                                        uint8_t *s_int, int8_t *s2) {
  if (!sk) return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_secret_export: sk is NULL");
  if (s0) memcpy(s0, sk->s0, sizeof(sk->s0));
  if (s1) memcpy(s1, sk->s1, sizeof(sk->s1));
  if (s_int) memcpy(s_int, sk->sint, sizeof(sk->sint));
  if (s2) memcpy(s2, sk->s2, sizeof(sk->s2));
  return OMR_OK;
}

namespace omr {
namespace {
// RLWE encryption of zero with mask alpha, plus m*g in component `comp` of coefficient 0:
// row = (alpha + [comp==0] m g, alpha*s + e + [comp==1] m g). Writes canonical residues.
template <typename T>
void ggsw_row(Stream &st, const Gaussian &gauss, const HostNtt &tab, const std::vector<uint64_t> &s_ntt,
              const std::vector<uint64_t> &s_ntts, uint64_t mg, int comp, T *out_a, T *out_b,
              const int8_t *sigma_s = nullptr, uint64_t sigma_scale = 0) {
  const int N = tab.N;
  const uint64_t q = tab.q;
  std::vector<uint64_t> a(N), t(N);
  for (int j = 0; j < N; ++j) a[j] = st.uniform(q);
  for (int j = 0; j < N; ++j) t[j] = a[j];
  tab.fwd(t.data());
  for (int j = 0; j < N; ++j) t[j] = tab.mul(t[j], s_ntt[j], s_ntts[j]);
  tab.inv(t.data());  // alpha * s
  for (int j = 0; j < N; ++j) {
    uint64_t b = t[j] + to_mod(gauss.sample(st), q);
    b = b >= q ? b - q : b;
    if (sigma_s && sigma_s[j]) {  // - sigma_g(s) * scale
      uint64_t c = mulmod(sigma_scale, (uint64_t)(sigma_s[j] < 0 ? q - 1 : 1), q);
      b = b >= c ? b - c : b + q - c;
    }
    t[j] = b;
  }
  if (mg) {
    if (comp == 0) a[0] = (a[0] + mg) % q;
    else t[0] = (t[0] + mg) % q;
  }
  for (int j = 0; j < N; ++j) {
    out_a[j] = (T)a[j];
    out_b[j] = (T)t[j];
  }
}
}  // namespace
}  // namespace omr

// DetectionKey (key_gen/secret.rs:118-178).
extern "C" omr_status omr_keygen_detection_key(const omr_secret_key_pack *sk, uint64_t seed,
                                               uint32_t *bsk1, uint32_t *ksk, uint64_t *bsk2,
                                               uint64_t *tk, int nthreads) {
  if (!sk || !bsk1 || !ksk || !bsk2 || !tk)
    return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_keygen_detection_key: NULL argument");
  const Gaussian g1(SIGMA_BR1), gks(SIGMA_KS), g2(SIGMA_BR2), gt(SIGMA_TRACE);
  // BSK1: BlindRotationKey::generate(s0, NTT(s1), basis(q1,5,4), sigma 3.1859), :124-131
  parallel_for((size_t)N0 * 2 * D1, nthreads, [&](size_t row) {
    const size_t i = row / (2 * D1);
    const int r = (int)(row % (2 * D1));
    Stream st(seed, DOM_BSK1, row);
    const int k = r < D1 ? r : r - D1;
    const uint64_t mg = sk->s0[i] ? (1ull << (DROP1 + k * LOGB1)) : 0;
    uint32_t *o = bsk1 + row * 2 * N1;
    ggsw_row<uint32_t>(st, g1, ntt1(), sk->s1_ntt, sk->s1_ntts, mg, r < D1 ? 0 : 1, o, o + N1);
  });
  // KSK: NonPowOf2LweKeySwitchingKey::generate(s1 (-1 -> q1-1), s_int, ...), :133-147
  parallel_for((size_t)N1 * KS_DIGITS, nthreads, [&](size_t row) {
    const size_t i = row / KS_DIGITS;
    const int j = (int)(row % KS_DIGITS);
    Stream st(seed, DOM_KSK, row);
    uint32_t *o = ksk + row * (NI + 1);
    uint64_t b = 0;
    for (int c = 0; c < NI; ++c) {
      uint64_t a = st.uniform(Q1);
      o[c] = (uint32_t)a;
      if (sk->sint[c]) b += a;
    }
    b %= Q1;
    b = (b + to_mod(gks.sample(st), Q1)) % Q1;
    const uint64_t m = mulmod(to_mod(sk->s1[i], Q1), (1ull << j) % Q1, Q1);
    o[NI] = (uint32_t)((b + m) % Q1);
  });
  // BSK2: BlindRotationKey::generate(s_int, NTT(s2), basis(q2,7,6), sigma 0.3908), :149-156
  parallel_for((size_t)NI * 2 * D2, nthreads, [&](size_t row) {
    const size_t i = row / (2 * D2);
    const int r = (int)(row % (2 * D2));
    Stream st(seed, DOM_BSK2, row);
    const int k = r < D2 ? r : r - D2;
    const uint64_t mg = sk->sint[i] ? (1ull << (DROP2 + k * LOGB2)) : 0;
    uint64_t *o = bsk2 + row * 2 * N2;
    ggsw_row<uint64_t>(st, g2, ntt2(), sk->s2_ntt, sk->s2_ntts, mg, r < D2 ? 0 : 1, o, o + N2);
  });
  // TraceKey::new(s2, NTT(s2), basis(q2,2,None), sigma 0.3908), :158-165
  parallel_for((size_t)TRACE_STEPS * DT, nthreads, [&](size_t row) {
    const int k = (int)(row / DT), j = (int)(row % DT);
    const uint32_t g = (uint32_t)(N2 >> k) + 1;
    int8_t sg[N2];
    for (int i = 0; i < N2; ++i) {
      uint32_t e = (uint32_t)(((uint64_t)i * g) % (2 * N2));
      if (e < (uint32_t)N2) sg[e] = sk->s2[i];
      else sg[e - N2] = (int8_t)-sk->s2[i];
    }
    Stream st(seed, DOM_TK, row);
    uint64_t *o = tk + row * 2 * N2;
    ggsw_row<uint64_t>(st, gt, ntt2(), sk->s2_ntt, sk->s2_ntts, 0, 1, o, o + N2, sg,
                       (1ull << (2 * j)) % Q2);
  });
  return OMR_OK;
}

// Sender::gen_clues: ClueKey::gen_clues -> LwePublicKeyRlweMode::encrypt_multi_messages(&[0;7]).
// u = A*r + e1, v = B*r + e2 (+ Delta*m = 0), r binary; clue = (u, v[0..7]).
extern "C" omr_status omr_gen_clues(const omr_secret_key_pack *sk, uint64_t seed, uint64_t first,
                                    size_t count, uint16_t *clue_a, uint16_t *clue_b,
                                    int nthreads) {
  if (!sk || !clue_a || !clue_b)
    return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_gen_clues: NULL argument");
  const Gaussian g(SIGMA_CLUE);
  parallel_for(count, nthreads, [&](size_t m) {
    Stream st(seed, DOM_CLUE, first + m);
    uint8_t r[N0];
    for (int w = 0; w < N0 / 32; ++w) {
      uint32_t v = st.next32();
      for (int b = 0; b < 32; ++b) r[w * 32 + b] = (uint8_t)((v >> b) & 1u);
    }
    int32_t u[N0];
    for (int i = 0; i < N0; ++i) u[i] = (int32_t)g.sample(st);
    for (int t = 0; t < N0; ++t) {
      if (!r[t]) continue;
      const uint16_t *A = sk->pk_a;
      for (int i = 0; i < N0 - t; ++i) u[i + t] += A[i];
      for (int i = N0 - t; i < N0; ++i) u[i + t - N0] -= A[i];
    }
    uint16_t *ca = clue_a + m * N0;
    for (int i = 0; i < N0; ++i) ca[i] = (uint16_t)(((u[i] % Q0) + Q0) % Q0);
    for (int i = 0; i < CLUES; ++i) {
      int32_t v = (int32_t)g.sample(st);
      for (int t = 0; t <= i; ++t)
        if (r[t]) v += sk->pk_b[i - t];
      for (int t = i + 1; t < N0; ++t)
        if (r[t]) v -= sk->pk_b[N0 + i - t];
      clue_b[m * CLUES + i] = (uint16_t)(((v % Q0) + Q0) % Q0);
    }
  });
  return OMR_OK;
}

extern "C" omr_status omr_get_retrieval_params(size_t all, size_t pertinent,
                                               omr_retrieval_params *rp) {
  if (!rp || all == 0) return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_get_retrieval_params");
  uint32_t pw = 0;
  uint64_t acc = 1;
  while (acc * (uint64_t)P <= all) {
    acc *= (uint64_t)P;
    ++pw;
  }
  if (acc < all) ++pw;
  if (pw == 0) pw = 1;
  rp->index_slots_per_bucket = pw;
  rp->slots_per_bucket = pw + 1;
  rp->slots_per_segment = rp->slots_per_bucket * BUCKETS;
  rp->segment_per_cipher = N2 / rp->slots_per_segment;
  rp->max_encode_indices_cipher_count = SEGMENTS / rp->segment_per_cipher;
  rp->combination_count = (uint32_t)pertinent + 5;  // non-power-of-two p (retrieval_params.rs:85-89)
  rp->cmb_count_per_cipher = 2;
  rp->cmb_cipher_count = (rp->combination_count + 1) / 2;
  return OMR_OK;
}

extern "C" omr_status omr_payload_weights(const uint8_t seed[32], size_t all, uint32_t combos,
                                          uint32_t n_ct, uint32_t per_ct, uint16_t *out) {
  if (!seed || !out || (size_t)n_ct * per_ct < combos)
    return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_payload_weights");
  uint32_t key[8];
  for (int i = 0; i < 8; ++i)
    key[i] = (uint32_t)seed[4 * i] | ((uint32_t)seed[4 * i + 1] << 8) |
             ((uint32_t)seed[4 * i + 2] << 16) | ((uint32_t)seed[4 * i + 3] << 24);
  const size_t count = (size_t)combos * all;
  uint32_t buf[16];
  uint64_t block = 0;
  int pos = 16;
  size_t n = 0;
  while (n < count) {
    if (pos == 16) {
      chacha_block(12, key, block++, 0, buf);
      pos = 0;
    }
    const uint64_t m = (uint64_t)buf[pos++] * (uint64_t)P;
    if ((uint32_t)m > 0xFFFFFFFEu) continue;  // UniformInt<u16> rejection zone
    out[n++] = (uint16_t)(m >> 32);
  }
  memset(out + count, 0, ((size_t)n_ct * per_ct * all - count) * sizeof(uint16_t));
  return OMR_OK;
}

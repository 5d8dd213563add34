// Client-side digest decoding (host, CPU): Retriever::decode_digest (retriever.rs:188-260) with
// decode_pertinent_indices (:63-130), decode_combined_payloads (:318-362) and
// solve_matrix_mod_257 (matrix.rs:164-247). Used by clients of the detector, by bench.py's
// end-to-end check and by the multi-GPU driver; needs only the secret key pack.
#include <set>
#include <string>
#include <vector>

#include "host_ring.hpp"

using namespace omr;

namespace {

// b - a * NTT(s2) in the NTT domain, inverse NTT, round(c * p / q2) half up, mod p
// (retriever.rs:84-96). ct: u64 [2][N2] (a, b), NTT domain.
void decrypt_decode_one(const omr_secret_key_pack *sk, const uint64_t *ct, uint32_t p, uint32_t *out) {
  const HostNtt &T = ntt2();
  std::vector<uint64_t> ph(N2);
  const uint64_t *a = ct, *b = ct + N2;
  for (int j = 0; j < N2; ++j) {
    const uint64_t as = T.mul(a[j] % Q2, sk->s2_ntt[j], sk->s2_ntts[j]);
    const uint64_t bj = b[j] % Q2;
    ph[j] = bj >= as ? bj - as : bj + Q2 - as;
  }
  T.inv(ph.data());
  for (int j = 0; j < N2; ++j) {
    uint64_t t = (uint64_t)(((u128)ph[j] * (2 * p) + Q2) / ((u128)2 * Q2));
    out[j] = (uint32_t)(t >= p ? t - p : t);
  }
}

}  // namespace

extern "C" omr_status omr_decrypt_decode(const omr_secret_key_pack *sk, const uint64_t *ct, size_t n,
                                         uint32_t *out) {
  if (!sk || (n && (!ct || !out)))
    return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_decrypt_decode: NULL argument");
  parallel_for(n, 0, [&](size_t m) { decrypt_decode_one(sk, ct + m * 2 * N2, P, out + m * N2); });
  return OMR_OK;
}

extern "C" omr_status omr_retrieve_indices(const omr_secret_key_pack *sk, const uint64_t *idx_cts,
                                           uint32_t n_ct, size_t all_payloads_count,
                                           size_t pertinent_count, size_t *indices, size_t cap,
                                           size_t *found) {
  if (!sk || !found || (n_ct && !idx_cts) || (cap && !indices))
    return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_retrieve_indices: NULL argument");
  omr_retrieval_params rp;
  omr_status st = omr_get_retrieval_params(all_payloads_count, pertinent_count, &rp);
  if (st != OMR_OK) return st;
  const size_t spb = rp.slots_per_bucket, sps = rp.slots_per_segment;
  std::set<size_t> set;
  std::vector<uint32_t> dec(N2);
  // decode_digest stops at the first ciphertext after which every pertinent index is known
  for (uint32_t c = 0; c < n_ct; ++c) {
    decrypt_decode_one(sk, idx_cts + (size_t)c * 2 * N2, P, dec.data());
    for (size_t s0 = 0; s0 + sps <= (size_t)N2; s0 += sps)
      for (size_t b0 = s0; b0 + spb <= s0 + sps; b0 += spb) {
        if (dec[b0 + spb - 1] != 1) continue;  // bucket marker
        size_t v = 0;
        for (size_t k = spb - 1; k-- > 0;) v = v * P + dec[b0 + k];  // base-257 digits, LSD first
        set.insert(v);
      }
    if (set.size() == pertinent_count) break;
  }
  *found = set.size();
  size_t i = 0;
  for (size_t v : set) {
    if (i >= cap) break;
    indices[i++] = v;
  }
  return OMR_OK;
}

extern "C" omr_status omr_retrieve_payloads(const omr_secret_key_pack *sk, const uint64_t *pay_cts,
                                            uint32_t n_ct, size_t all_payloads_count,
                                            uint32_t combination_count, const uint16_t *weights,
                                            const size_t *indices,
                                            size_t n_indices, uint16_t *payloads) {
  if (!sk || !pay_cts || !weights || (n_indices && (!indices || !payloads)))
    return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_retrieve_payloads: NULL argument");
  omr_retrieval_params rp;
  omr_status st = omr_get_retrieval_params(all_payloads_count, n_indices, &rp);
  if (st != OMR_OK) return st;
  const size_t rows = combination_count ? combination_count : rp.combination_count, cols = n_indices,
               per = rp.cmb_count_per_cipher;
  if (n_indices == 0) return OMR_OK;
  if ((size_t)n_ct * per < rows)
    return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_retrieve_payloads: too few payload ciphertexts");
  if (rows < cols)  // matrix.rs:171 asserts num_rows >= num_cols
    return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_retrieve_payloads: fewer combinations than indices");
  for (size_t i = 0; i < n_indices; ++i)
    if (indices[i] >= all_payloads_count)
      return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_retrieve_payloads: index out of range");
  // decode_combined_payloads: combination j lives in ciphertext j / per, slots (j % per) * 612..
  std::vector<std::vector<uint32_t>> rhs(rows, std::vector<uint32_t>(PAYLOAD_LEN));
  std::vector<uint32_t> dec((size_t)n_ct * N2);
  parallel_for(n_ct, 0, [&](size_t c) { decrypt_decode_one(sk, pay_cts + c * 2 * N2, P, &dec[c * N2]); });
  for (size_t j = 0; j < rows; ++j)
    for (int b = 0; b < PAYLOAD_LEN; ++b) rhs[j][b] = dec[(j / per) * N2 + (j % per) * PAYLOAD_LEN + b];
  // matrix[j][k] = weight of combination j for the k-th retrieved index (retriever.rs:220-238)
  std::vector<std::vector<uint32_t>> m(rows, std::vector<uint32_t>(cols));
  for (size_t j = 0; j < rows; ++j)
    for (size_t k = 0; k < cols; ++k) m[j][k] = weights[j * all_payloads_count + indices[k]] % P;
  auto inv = [](uint32_t v) {  // v^(p-2) mod p
    uint32_t r = 1, b = v % P;
    for (uint32_t e = P - 2; e; e >>= 1, b = b * b % P)
      if (e & 1) r = r * b % P;
    return r;
  };
  // forward elimination with the first non-zero pivot, then back substitution (matrix.rs)
  for (size_t i = 0; i < cols; ++i) {
    size_t piv = rows;
    for (size_t j = i; j < rows; ++j)
      if (m[j][i] != 0) {
        piv = j;
        break;
      }
    if (piv == rows) return set_error(OMR_ERR_NOT_INVERTIBLE, "Matrix is not invertible");
    std::swap(m[i], m[piv]);
    std::swap(rhs[i], rhs[piv]);
    if (m[i][i] != 1) {
      const uint32_t iv = inv(m[i][i]);
      for (size_t k = i; k < cols; ++k) m[i][k] = m[i][k] * iv % P;
      for (auto &x : rhs[i]) x = x * iv % P;
    }
    for (size_t j = i + 1; j < rows; ++j) {
      const uint32_t c = m[j][i];
      if (!c) continue;
      for (size_t k = i; k < cols; ++k) m[j][k] = (m[j][k] + P * P - c * m[i][k]) % P;
      for (int b = 0; b < PAYLOAD_LEN; ++b) rhs[j][b] = (rhs[j][b] + P * P - c * rhs[i][b]) % P;
    }
  }
  for (size_t i = cols; i-- > 1;)
    for (size_t j = 0; j < i; ++j) {
      const uint32_t c = m[j][i];
      if (!c) continue;
      for (int b = 0; b < PAYLOAD_LEN; ++b) rhs[j][b] = (rhs[j][b] + P * P - c * rhs[i][b]) % P;
      m[j][i] = 0;
    }
  for (size_t k = 0; k < cols; ++k)
    for (int b = 0; b < PAYLOAD_LEN; ++b) payloads[k * PAYLOAD_LEN + b] = (uint16_t)rhs[k][b];
  return OMR_OK;
}

// Host-side ring arithmetic shared by key generation (keygen.hip) and the client-side
// retriever (retriever.hip): exact negacyclic NTTs mod q1 / q2 (the device convention,
// include/omr_gpu.h), a thread pool helper and the secret key pack.
#pragma once

#include <algorithm>
#include <thread>
#include <vector>

#include "common.hpp"

namespace omr {

typedef unsigned __int128 u128;

// ------------------------------------------------------------------------------------------
// Host negacyclic NTT (same convention as the device path and oracle/omr_oracle.h).
// ------------------------------------------------------------------------------------------
inline uint64_t mulmod(uint64_t a, uint64_t b, uint64_t q) { return (uint64_t)((u128)a * b % q); }
inline uint64_t powmod(uint64_t b, uint64_t e, uint64_t q) {
  uint64_t r = 1;
  b %= q;
  while (e) {
    if (e & 1) r = mulmod(r, b, q);
    b = mulmod(b, b, q);
    e >>= 1;
  }
  return r;
}
inline uint32_t bitrev(uint32_t x, int bits) { return __builtin_bitreverse32(x) >> (32 - bits); }

struct HostNtt {
  uint64_t q;
  int N, L;
  std::vector<uint64_t> w, ws, iw, iws;
  uint64_t ninv, ninvs;
  HostNtt(uint64_t q_, int N_, uint64_t g) : q(q_), N(N_), L(__builtin_ctz(N_)) {
    uint64_t psi = powmod(g, (q - 1) / (2 * (uint64_t)N), q), ipsi = powmod(psi, q - 2, q);
    w.resize(N); ws.resize(N); iw.resize(N); iws.resize(N);
    for (int k = 0; k < N; ++k) {
      uint32_t e = bitrev((uint32_t)k, L);
      w[k] = powmod(psi, e, q);
      iw[k] = powmod(ipsi, e, q);
      ws[k] = pre(w[k]);
      iws[k] = pre(iw[k]);
    }
    ninv = powmod((uint64_t)N, q - 2, q);
    ninvs = pre(ninv);
  }
  uint64_t pre(uint64_t v) const { return (uint64_t)(((u128)v << 64) / q); }
  uint64_t mul(uint64_t a, uint64_t v, uint64_t vs) const {
    uint64_t qe = (uint64_t)(((u128)a * vs) >> 64);
    uint64_t r = a * v - qe * q;
    return r >= q ? r - q : r;
  }
  void fwd(uint64_t *a) const {
    for (int m = 1, h = N / 2; m < N; m <<= 1, h >>= 1)
      for (int i = 0; i < m; ++i)
        for (int j = 2 * i * h; j < 2 * i * h + h; ++j) {
          uint64_t U = a[j], V = mul(a[j + h], w[m + i], ws[m + i]);
          uint64_t s = U + V;
          a[j] = s >= q ? s - q : s;
          a[j + h] = U >= V ? U - V : U + q - V;
        }
  }
  void inv(uint64_t *a) const {
    for (int m = N / 2, h = 1; m >= 1; m >>= 1, h <<= 1)
      for (int i = 0; i < m; ++i)
        for (int j = 2 * i * h; j < 2 * i * h + h; ++j) {
          uint64_t U = a[j], V = a[j + h];
          uint64_t s = U + V;
          a[j] = s >= q ? s - q : s;
          a[j + h] = mul(U >= V ? U - V : U + q - V, iw[m + i], iws[m + i]);
        }
    for (int j = 0; j < N; ++j) a[j] = mul(a[j], ninv, ninvs);
  }
};

inline const HostNtt &ntt1() {
  static HostNtt t(Q1, N1, 7);
  return t;
}
inline const HostNtt &ntt2() {
  static HostNtt t(Q2, N2, 22);
  return t;
}

template <typename F>
inline void parallel_for(size_t n, int nthreads, F f) {
  if (nthreads <= 0)  // default: host cores, capped at 16 (the GPU box's CPU share)
    nthreads = (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
  nthreads = (int)std::min<size_t>((size_t)nthreads, std::max<size_t>(1, n));
  if (nthreads == 1) {
    for (size_t i = 0; i < n; ++i) f(i);
    return;
  }
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t)
    th.emplace_back([=, &f] {
      for (size_t i = (size_t)t; i < n; i += (size_t)nthreads) f(i);
    });
  for (auto &x : th) x.join();
}

inline uint64_t to_mod(int64_t v, uint64_t q) {
  int64_t r = v % (int64_t)q;
  return (uint64_t)(r < 0 ? r + (int64_t)q : r);
}


}  // namespace omr

struct omr_secret_key_pack {
  uint64_t seed;
  uint8_t s0[omr::N0];     // clue LWE key, binary (LweSecretKeyType::Binary, mod.rs:44)
  int8_t s1[omr::N1];      // first-level RLWE key, ternary (mod.rs:53)
  uint8_t sint[omr::NI];   // intermediate LWE key, binary (mod.rs:72)
  int8_t s2[omr::N2];      // second-level RLWE key, ternary (mod.rs:79)
  uint16_t pk_a[omr::N0];  // RLWE-mode clue public key (LwePublicKeyRlweMode, secret.rs:99-107)
  uint16_t pk_b[omr::N0];
  std::vector<uint64_t> s1_ntt, s1_ntts, s2_ntt, s2_ntts;  // NTT(s) + Shoup companions
};

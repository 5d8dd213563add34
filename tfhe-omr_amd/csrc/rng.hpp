// Seeded random streams shared by the host key/clue generators (keygen.hip) and the device
// generators (keygen_gpu.hip). Every draw comes from a ChaCha12 stream keyed by (seed, domain)
// whose stream id is the key row or the global message index, so a row or a clue is the same
// whichever thread, device or shard produces it.
#pragma once

#include <algorithm>
#include <cmath>
#include <vector>

#include "common.hpp"

namespace omr {

enum Domain : uint32_t {
  DOM_S0 = 1, DOM_S1 = 2, DOM_SINT = 3, DOM_S2 = 4, DOM_PK_A = 5, DOM_PK_E = 6,
  DOM_BSK1 = 10, DOM_KSK = 11, DOM_BSK2 = 12, DOM_TK = 13, DOM_CLUE = 20,
};

class Stream {
 public:
  Stream(uint64_t seed, uint32_t domain, uint64_t stream) : stream_(stream) {
    key_[0] = (uint32_t)seed;
    key_[1] = (uint32_t)(seed >> 32);
    key_[2] = 0x6b657967u;  // "keyg"
    key_[3] = domain;
    for (int i = 4; i < 8; ++i) key_[i] = 0;
  }
  uint32_t next32() {
    if (pos_ == 16) {
      chacha_block(12, key_, ctr_++, stream_, buf_);
      pos_ = 0;
    }
    return buf_[pos_++];
  }
  uint64_t next64() {
    uint64_t lo = next32();
    return lo | ((uint64_t)next32() << 32);
  }
  uint64_t uniform(uint64_t q) {  // rejection sampling on the bit length of q
    int bits = 64 - __builtin_clzll(q - 1);
    uint64_t mask = bits == 64 ? ~0ull : ((1ull << bits) - 1);
    for (;;) {
      uint64_t v = next64() & mask;
      if (v < q) return v;
    }
  }
  int ternary() {
    for (;;) {
      uint32_t v = next32();
      if (v < 0xFFFFFFFFu - (0xFFFFFFFFu % 3)) return (int)(v % 3) - 1;  // {-1, 0, 1}
    }
  }
  int bit() { return (int)(next32() & 1u); }

 private:
  uint32_t key_[8];
  uint64_t stream_;
  uint64_t ctr_ = 0;
  uint32_t buf_[16];
  int pos_ = 16;
};

// Rounded Gaussian by cumulative distribution table over |x| (deterministic, integer search).
class Gaussian {
 public:
  explicit Gaussian(double sigma) {
    int K = std::max(16, (int)std::ceil(sigma * 13.0) + 2);
    std::vector<long double> w(K + 1);
    long double Z = 0;
    for (int k = 0; k <= K; ++k) {
      w[k] = (k == 0 ? 1.0L : 2.0L) * std::exp(-(long double)k * k / (2.0L * sigma * sigma));
      Z += w[k];
    }
    long double acc = 0;
    table_.resize(K + 1);
    for (int k = 0; k <= K; ++k) {
      acc += w[k] / Z;
      long double t = acc * 9223372036854775808.0L;  // 2^63
      table_[k] = t >= 9223372036854775807.0L ? ~0ull >> 1 : (uint64_t)t;
    }
    table_[K] = ~0ull >> 1;
  }
  const std::vector<uint64_t> &table() const { return table_; }
  int64_t sample(Stream &s) const {
    uint64_t u = s.next64() >> 1;
    size_t k = std::upper_bound(table_.begin(), table_.end(), u) - table_.begin();
    if (k >= table_.size()) k = table_.size() - 1;
    if (k == 0) return 0;
    return (s.next32() & 1u) ? -(int64_t)k : (int64_t)k;
  }

 private:
  std::vector<uint64_t> table_;
};

}  // namespace omr

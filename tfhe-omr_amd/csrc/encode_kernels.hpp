// Digest encoding kernels: encode_pertinent_indices (detector.rs:223-339) and
// encode_pertinent_payloads (detector.rs:341-453). Each workgroup folds a chunk of messages into
// one partial RLWE digest in registers; a second kernel sums the chunk partials mod q2 (the
// reference's rayon `.reduce(add_element_wise)`, :333-336 / :445-448).
#pragma once

#include "kernels.hpp"

namespace omr {

struct EncodeLayout {  // RetrievalParams (retrieval_params.rs:50-106)
  int index_slots, slots_per_bucket, slots_per_segment, segment_per_cipher;
};

__device__ __forceinline__ double centred_lift(uint32_t v) {
  // v < half_p ? v : q - p + v  (detector.rs:294,431), as a centred residue
  return v < (uint32_t)(P + 1) / 2 ? (double)v : (double)v - (double)P;
}

// grid (chunks, n_ct); partial [n_ct][chunks][2][N2] canonical u64.
__global__ __launch_bounds__(ENC_T) void encode_indices_kernel(
    const uint64_t *__restrict__ pv, int D, uint64_t offset, EncodeLayout ly, uint64_t seed,
    uint32_t first_ct, int per_wg, const double *__restrict__ tw, uint64_t *__restrict__ partial) {
  using M = Mod<2>;
  constexpr int T = ENC_T, E = ENC_E, N = N2;
  using NTT = WgNtt<M, T, E>;
  __shared__ double xch[NTT::LDS_DOUBLES];
  __shared__ uint8_t buckets[ENC_T][8];
  const int tid = threadIdx.x;
  const int chunk = blockIdx.x, cti = blockIdx.y;
  const uint32_t ct = first_ct + cti;
  const int m0 = chunk * per_wg;
  const int mcount = min(per_wg, D - m0);
  double accA[E], accB[E];
#pragma unroll
  for (int e = 0; e < E; ++e) accA[e] = accB[e] = 0.0;
  // per_wg may exceed ENC_T (large D): the bucket choices are staged ENC_T messages at a time
#pragma unroll 1
  for (int mb = 0; mb < mcount; mb += ENC_T) {
    const int cnt = min(ENC_T, mcount - mb);
    __syncthreads();  // every thread has finished reading the previous block's buckets
    if (tid < cnt) {
      uint32_t w[16];
      bucket_words(seed, ct, offset + m0 + mb + tid, w);
      for (int s = 0; s < ly.segment_per_cipher && s < 8; ++s) buckets[tid][s] = (uint8_t)bucket_of(w[s]);
    }
    __syncthreads();
#pragma unroll 1
    for (int mi = mb; mi < mb + cnt; ++mi) {
      const uint64_t gi = offset + m0 + mi;
      double x[E];
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int pos = tid + e * T;
        const int s = pos / ly.slots_per_segment;
        double v = 0.0;
        if (s < ly.segment_per_cipher) {
          const int within = pos - s * ly.slots_per_segment;
          const int bk = within / ly.slots_per_bucket;
          const int slot = within - bk * ly.slots_per_bucket;
          if (bk == buckets[mi - mb][s]) {
            if (slot == ly.index_slots) {
              v = 1.0;
            } else {
              uint64_t t = gi;  // base-257 digit `slot` of gi (little endian)
              for (int q = 0; q < slot; ++q) t /= (uint64_t)P;
              v = centred_lift((uint32_t)(t % (uint64_t)P));
            }
          }
        }
        x[e] = v;
      }
      NTT::fwd(x, xch, tw, tid);
      const uint64_t *pa = pv + (size_t)(m0 + mi) * 2 * N + tid * E;
      const uint64_t *pb = pa + N;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        accA[e] = red<M>(accA[e] + mm<M>(from_u64<M>(pa[e]), x[e]));
        accB[e] = red<M>(accB[e] + mm<M>(from_u64<M>(pb[e]), x[e]));
      }
    }
  }
  uint64_t *o = partial + ((size_t)cti * gridDim.x + chunk) * 2 * N + tid * E;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    o[e] = to_u64<M>(canon<M>(accA[e]));
    o[N + e] = to_u64<M>(canon<M>(accB[e]));
  }
}

// grid (chunks, n_ct). weights [n_ct*per_ct][all] u16 (global index), payloads [D][612] u16.
__global__ __launch_bounds__(ENC_T) void encode_payloads_kernel(
    const uint64_t *__restrict__ pv, const uint16_t *__restrict__ payloads, int D, uint64_t offset,
    uint64_t all, const uint16_t *__restrict__ weights, int per_ct, int per_wg,
    const double *__restrict__ tw, uint64_t *__restrict__ partial) {
  using M = Mod<2>;
  constexpr int T = ENC_T, E = ENC_E, N = N2;
  using NTT = WgNtt<M, T, E>;
  __shared__ double xch[NTT::LDS_DOUBLES];
  const int tid = threadIdx.x;
  const int chunk = blockIdx.x, c = blockIdx.y;
  const int m0 = chunk * per_wg;
  const int mcount = min(per_wg, D - m0);
  double accA[E], accB[E];
#pragma unroll
  for (int e = 0; e < E; ++e) accA[e] = accB[e] = 0.0;
#pragma unroll 1
  for (int mi = 0; mi < mcount; ++mi) {
    const int m = m0 + mi;
    const uint64_t gi = offset + m;
    double x[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int pos = tid + e * T;
      const int j = pos / PAYLOAD_LEN;
      double v = 0.0;
      if (j < per_ct) {
        const int l = pos - j * PAYLOAD_LEN;
        const uint32_t w = weights[(size_t)(c * per_ct + j) * all + gi];
        v = centred_lift(((uint32_t)payloads[(size_t)m * PAYLOAD_LEN + l] * w) % (uint32_t)P);
      }
      x[e] = v;
    }
    NTT::fwd(x, xch, tw, tid);
    const uint64_t *pa = pv + (size_t)m * 2 * N + tid * E;
    const uint64_t *pb = pa + N;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      accA[e] = red<M>(accA[e] + mm<M>(from_u64<M>(pa[e]), x[e]));
      accB[e] = red<M>(accB[e] + mm<M>(from_u64<M>(pb[e]), x[e]));
    }
  }
  uint64_t *o = partial + ((size_t)c * gridDim.x + chunk) * 2 * N + tid * E;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    o[e] = to_u64<M>(canon<M>(accA[e]));
    o[N + e] = to_u64<M>(canon<M>(accB[e]));
  }
}

// out[c][t] = sum_chunk partial[c][chunk][t] mod q2: every partial is canonical (< q2), so the
// running sum stays canonical with one conditional subtraction per term, for any chunk count.
__global__ void reduce_partials_kernel(const uint64_t *__restrict__ partial, int chunks,
                                       int n_ct, uint64_t *__restrict__ out) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (size_t)n_ct * 2 * N2) return;
  const size_t c = idx / (2 * N2), t = idx % (2 * N2);
  uint64_t s = 0;
  for (int k = 0; k < chunks; ++k) {
    s += partial[((size_t)c * chunks + k) * 2 * N2 + t];
    s = s >= Q2 ? s - Q2 : s;
  }
  out[idx] = s;
}

}  // namespace omr

// Device key and clue generation from the same seeded ChaCha12
// streams as the host generators (rng.hpp, keygen.hip), so every clue and every key row is
// bit-identical to theirs whichever device, shard or thread count produces it:
//   omr_gen_clues_device             Sender::gen_clues (sender.rs:27-32, key_gen/clue.rs:27-34)
//   omr_keygen_detection_key_device  SecretKeyPack::generate_detector (key_gen/secret.rs:118-178)
//
// Stream consumption is data dependent (rejection-sampled uniforms, Gaussians that draw a sign
// word only when non-zero), so each workgroup first expands its stream into LDS with every
// thread computing ChaCha blocks, then:
//   * uniforms: draw j is speculatively taken from words (2j, 2j+1); a workgroup vote detects a
//     rejection (probability 1.5e-5 per draw mod q1, 1.5e-11 mod q2) and only then one thread
//     compacts the draws sequentially;
//   * Gaussians: every thread evaluates the sample that would start at each word position
//     (value and words used, packed), then one thread walks the chain of start positions.
// RLWE rows then compute a*s with the device NTT (kernels.hpp) — the product mod q is unique,
// so the result equals the host's exact-integer NTT product.
#include <string>
#include <vector>

#include "host_ring.hpp"
#include "kernels.hpp"
#include "rng.hpp"

using namespace omr;

namespace {

#define HIP_TRY(expr)                                                                     \
  do {                                                                                    \
    hipError_t _e = (expr);                                                               \
    if (_e != hipSuccess)                                                                 \
      return set_error(OMR_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

constexpr int CDT_LDS = 64;  // CDT tables up to this size are searched from LDS
constexpr int SLACK = 32;    // rejected uniform draws a row may absorb before it reports overrun

// Fill w[0, 16 * nblk) with the words of Stream(seed, dom, stream) (rng.hpp).
__device__ void fill_words(uint32_t *w, int nblk, uint64_t seed, uint32_t dom, uint64_t stream) {
  const uint32_t key[8] = {(uint32_t)seed, (uint32_t)(seed >> 32), 0x6b657967u, dom, 0, 0, 0, 0};
  for (int b = threadIdx.x; b < nblk; b += blockDim.x) {
    uint32_t o[16];
    chacha_block(12, key, (uint64_t)b, stream, o);
#pragma unroll
    for (int i = 0; i < 16; ++i) w[16 * b + i] = o[i];
  }
}

// Gaussian::sample started at word p (rng.hpp): upper_bound of next64() >> 1 in the CDT, sign
// from one more word when non-zero. Returns (sample << 2) | words used.
__device__ __forceinline__ int gauss_packed(const uint32_t *w, int p, const uint64_t *tab, int n) {
  const uint64_t u = ((((uint64_t)w[p + 1]) << 32) | w[p]) >> 1;
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (tab[mid] <= u) lo = mid + 1;
    else hi = mid;
  }
  const int k = lo >= n ? n - 1 : lo;
  if (k == 0) return 2;
  return (((w[p + 2] & 1u) ? -k : k) * 4) | 3;
}

// Replace w[p0, p0 + span) by the packed sample starting at each position (all threads), so
// that one thread can then walk the chain in one LDS read per sample.
__device__ void pack_gaussians(uint32_t *w, int nw, int p0, int span, const uint64_t *tab, int n) {
  constexpr int MAXK = 32;
  int v[MAXK];
  const int T = blockDim.x;
#pragma unroll
  for (int k = 0; k < MAXK; ++k) {
    const int p = p0 + threadIdx.x + k * T;
    v[k] = (k * T < span && p < p0 + span && p + 2 < nw) ? gauss_packed(w, p, tab, n) : 0;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < MAXK; ++k) {
    const int p = p0 + threadIdx.x + k * T;
    if (k * T < span && p < p0 + span && p + 2 < nw) w[p] = (uint32_t)v[k];
  }
  __syncthreads();
}

// ------------------------------------------------------------------------------------------
// Clues: u = A*r + e1, v = B*r + e2 over Z_2048[X]/(X^512+1), r binary (keygen.hip
// omr_gen_clues). One 64-thread workgroup per message.
// ------------------------------------------------------------------------------------------
constexpr int CLUE_WORDS = 16 * 101;  // 16 (r) + 3 * 519 Gaussian words at most, + slack

__global__ __launch_bounds__(64) void gen_clues_kernel(const uint16_t *__restrict__ pk,
                                                       const uint64_t *__restrict__ cdt, int cdt_n,
                                                       uint64_t seed, uint64_t first, size_t count,
                                                       uint16_t *__restrict__ clue_a,
                                                       uint16_t *__restrict__ clue_b) {
  __shared__ uint32_t w[CLUE_WORDS];
  __shared__ int32_t A[N0], B[N0], es[N0 + CLUES];
  __shared__ uint64_t tab[CDT_LDS];
  const size_t m = blockIdx.x;
  const int tid = threadIdx.x;
  if (m >= count) return;
  for (int i = tid; i < N0; i += 64) {
    A[i] = pk[i];
    B[i] = pk[N0 + i];
  }
  for (int i = tid; i < cdt_n; i += 64) tab[i] = cdt[i];
  fill_words(w, CLUE_WORDS / 16, seed, DOM_CLUE, first + m);
  __syncthreads();
  pack_gaussians(w, CLUE_WORDS, 16, 3 * (N0 + CLUES), tab, cdt_n);
  if (tid == 0) {
    int p = 16;
    for (int i = 0; i < N0 + CLUES; ++i) {
      const int v = (int)w[p];
      es[i] = v >> 2;
      p += v & 3;
    }
  }
  __syncthreads();
  // r = words 0..15, bit b of word k is r[32k + b]
  int acc[N0 / 64];
#pragma unroll
  for (int j = 0; j < N0 / 64; ++j) acc[j] = es[tid + 64 * j];
  int accb = tid < CLUES ? es[N0 + tid] : 0;
  for (int k = 0; k < N0 / 32; ++k) {
    uint32_t bits = __builtin_amdgcn_readfirstlane(w[k]);
    while (bits) {
      const int t = 32 * k + __builtin_ctz(bits);
      bits &= bits - 1;
#pragma unroll
      for (int j = 0; j < N0 / 64; ++j) {
        const int d = tid + 64 * j - t;  // u[o] += A[o - t] (o >= t), -= A[o - t + 512]
        const int a = A[d & (N0 - 1)];
        acc[j] += d >= 0 ? a : -a;
      }
      if (tid < CLUES) {
        const int d = tid - t;
        const int b = B[d & (N0 - 1)];
        accb += d >= 0 ? b : -b;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < N0 / 64; ++j) clue_a[m * N0 + tid + 64 * j] = (uint16_t)(acc[j] & (Q0 - 1));
  if (tid < CLUES) clue_b[m * CLUES + tid] = (uint16_t)(accb & (Q0 - 1));
}

// ------------------------------------------------------------------------------------------
// RLWE key rows (keygen.hip ggsw_row): a uniform, b = a*s + e (- sigma_scale * sigma_g(s)),
// plus mg in coefficient 0 of component comp. 256 threads per row.
// ------------------------------------------------------------------------------------------
struct RowJob {
  uint64_t seed;
  uint32_t domain;
  int rows;                     // rows in this launch
  int dsplit;                   // comp = (row % (2 dsplit)) >= dsplit
  const uint64_t *mg;           // [rows] gadget value added in coefficient 0 (0: none)
  const double *s_hat;          // NTT(s), centred, device NTT order
  const double *tw, *itw;       // device NTT twiddles (kernels.hpp convention)
  double ninv;                  // N^-1 mod q, centred
  const uint64_t *cdt;          // Gaussian CDT (<= CDT_LDS entries)
  int cdt_n;
  const int8_t *sigma_s;        // trace key: [TRACE_STEPS][N] sigma_g(s); null otherwise
  const uint64_t *sigma_scale;  // trace key: [rows] 2^(2j) mod q
  int *overrun;                 // set when a row rejects more than SLACK uniform draws
};

template <int LEVEL, typename OUT>
__global__ __launch_bounds__(256) void rlwe_rows_kernel(RowJob job, OUT *__restrict__ out) {
  using M = Mod<LEVEL>;
  constexpr int N = M::N, T = 256, E = N / T;
  constexpr uint64_t Q = LEVEL == 1 ? Q1 : Q2;
  constexpr uint64_t MASK = LEVEL == 1 ? (1ull << 27) - 1 : (1ull << 50) - 1;  // bit length of q
  using NTT = WgNtt<M, T, E>;
  constexpr int NW = 5 * N + 2 * SLACK + 16;
  static_assert(NW % 16 == 0 && NTT::LDS_DOUBLES * 2 <= NW, "word buffer doubles as NTT space");
  static_assert(Q - 1 <= MASK && MASK < 2 * Q, "mask = bit length of q (Stream::uniform)");
  __shared__ uint32_t w[NW];
  __shared__ int32_t es[N];
  __shared__ uint64_t tab[CDT_LDS];
  __shared__ int g0s;
  const int row = blockIdx.x, tid = threadIdx.x;
  if (row >= job.rows) return;
  OUT *oa = out + (size_t)row * 2 * N, *ob = oa + N;
  for (int i = tid; i < job.cdt_n; i += T) tab[i] = job.cdt[i];
  fill_words(w, NW / 16, job.seed, job.domain, (uint64_t)row);
  __syncthreads();
  // uniforms: draw j from words (2j, 2j+1) unless some draw is rejected
  uint64_t a[E];
  int rej = 0;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int j = tid + e * T;
    a[e] = ((((uint64_t)w[2 * j + 1]) << 32) | w[2 * j]) & MASK;
    rej |= a[e] >= Q;
  }
  if (__syncthreads_or(rej)) {
    if (tid == 0) {  // sequential rejection sampling (Stream::uniform) into the output row
      int d = 0, cnt = 0;
      while (cnt < N && d < N + SLACK) {
        const uint64_t v = ((((uint64_t)w[2 * d + 1]) << 32) | w[2 * d]) & MASK;
        ++d;
        if (v < Q) oa[cnt++] = (OUT)v;
      }
      if (cnt < N) atomicOr(job.overrun, 1);
      g0s = 2 * d;
    }
    __threadfence_block();
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; ++e) a[e] = (uint64_t)oa[tid + e * T];
  } else if (tid == 0) {
    g0s = 2 * N;
  }
  __syncthreads();
  const int g0 = g0s;
  pack_gaussians(w, NW, g0, 3 * N, tab, job.cdt_n);
  if (tid == 0) {
    int p = g0;
    for (int i = 0; i < N; ++i) {
      const int v = (int)w[p];
      es[i] = v >> 2;
      p += v & 3;
    }
  }
  __syncthreads();  // the word buffer becomes the NTT exchange space
  // a * s = INTT(NTT(a) . NTT(s)) / N, coefficient tid + e T on return
  double *lds = reinterpret_cast<double *>(w);
  double x[E];
#pragma unroll
  for (int e = 0; e < E; ++e) x[e] = from_u64<M>(a[e]);
  NTT::fwd(x, lds, job.tw, tid);
#pragma unroll
  for (int e = 0; e < E; ++e) x[e] = canon<M>(mm<M>(canon<M>(x[e]), job.s_hat[tid * E + e]));
  NTT::inv(x, lds, job.itw, tid);
  const bool comp1 = (row % (2 * job.dsplit)) >= job.dsplit;
  const uint64_t mg = job.mg ? job.mg[row] : 0;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int j = tid + e * T;
    uint64_t b = to_u64<M>(canon<M>(mm<M>(canon<M>(x[e]), job.ninv)));
    b += es[j] < 0 ? Q - (uint64_t)(-es[j]) : (uint64_t)es[j];
    b = b >= Q ? b - Q : b;
    if (job.sigma_s) {  // - sigma_g(s) * 2^(2j)
      const int sg = job.sigma_s[(size_t)(row / DT) * N + j];
      const uint64_t sc = job.sigma_scale[row];
      if (sg) {
        const uint64_t c = sg < 0 ? Q - sc : sc;
        b = b >= c ? b - c : b + Q - c;
      }
    }
    uint64_t av = a[e];
    if (j == 0 && mg) {
      if (comp1) b = (b + mg) % Q;
      else av = (av + mg) % Q;
    }
    oa[j] = (OUT)av;
    ob[j] = (OUT)b;
  }
}

// ------------------------------------------------------------------------------------------
// Key-switching key rows (keygen.hip): LWE(670) of s1[i] * 2^j under s_int. 64 threads per row.
// ------------------------------------------------------------------------------------------
constexpr int KSK_WORDS = 16 * 88;  // 2 (670 + SLACK) + 3 words, whole blocks
static_assert(2 * (NI + SLACK) + 3 <= KSK_WORDS, "KSK word buffer");

__global__ __launch_bounds__(64) void ksk_rows_kernel(uint64_t seed, const uint8_t *__restrict__ sint,
                                                      const int8_t *__restrict__ s1,
                                                      const uint64_t *__restrict__ cdt, int cdt_n,
                                                      int rows, uint32_t *__restrict__ out,
                                                      int *overrun) {
  constexpr uint64_t MASK = (1ull << 27) - 1;
  __shared__ uint32_t w[KSK_WORDS];
  __shared__ uint64_t part[64];
  const int row = blockIdx.x, tid = threadIdx.x;
  if (row >= rows) return;
  uint32_t *o = out + (size_t)row * (NI + 1);
  fill_words(w, KSK_WORDS / 16, seed, DOM_KSK, (uint64_t)row);
  __syncthreads();
  int rej = 0;
  uint64_t sum = 0;
  for (int c = tid; c < NI; c += 64) {
    const uint64_t v = ((((uint64_t)w[2 * c + 1]) << 32) | w[2 * c]) & MASK;
    rej |= v >= Q1;
    if (v < Q1) {
      o[c] = (uint32_t)v;
      if (sint[c]) sum += v;
    }
  }
  part[tid] = sum;
  const bool slow = __syncthreads_or(rej);
  if (tid == 0) {
    int g0 = 2 * NI;
    sum = 0;
    if (slow) {  // sequential rejection sampling (Stream::uniform)
      int d = 0, cnt = 0;
      while (cnt < NI && d < NI + SLACK) {
        const uint64_t v = ((((uint64_t)w[2 * d + 1]) << 32) | w[2 * d]) & MASK;
        ++d;
        if (v < Q1) {
          o[cnt] = (uint32_t)v;
          if (sint[cnt]) sum += v;
          ++cnt;
        }
      }
      if (cnt < NI) atomicOr(overrun, 1);
      g0 = 2 * d;
    } else {
      for (int t = 0; t < 64; ++t) sum += part[t];
    }
    const int e = (int)gauss_packed(w, g0, cdt, cdt_n) >> 2;
    uint64_t b = sum % Q1;
    b = (b + (e < 0 ? Q1 - (uint64_t)(-e) : (uint64_t)e)) % Q1;
    const uint64_t s = s1[row / KS_DIGITS] < 0 ? Q1 - 1 : (uint64_t)s1[row / KS_DIGITS];
    const uint64_t m = s * ((1ull << (row % KS_DIGITS)) % Q1) % Q1;
    o[NI] = (uint32_t)((b + m) % Q1);
  }
}

template <typename T>
struct DevMem {
  T *p = nullptr;
  ~DevMem() {
    if (p) (void)hipFree(p);
  }
  hipError_t put(const T *src, size_t n, hipStream_t st) {
    hipError_t e = hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T));
    if (e != hipSuccess || n == 0) return e;
    return hipMemcpyAsync(p, src, n * sizeof(T), hipMemcpyHostToDevice, st);
  }
  template <class V>
  hipError_t put(const V &v, hipStream_t st) {
    return put(v.data(), v.size(), st);
  }
};

double centred_d(uint64_t v, uint64_t q) { return v > (q - 1) / 2 ? (double)v - (double)q : (double)v; }

std::vector<double> centred_vec(const std::vector<uint64_t> &v, uint64_t q) {
  std::vector<double> r(v.size());
  for (size_t i = 0; i < v.size(); ++i) r[i] = centred_d(v[i], q);
  return r;
}

}  // namespace

extern "C" omr_status omr_gen_clues_device(const omr_secret_key_pack *sk, uint64_t seed, uint64_t first,
                                           size_t count, uint16_t *d_clue_a, uint16_t *d_clue_b,
                                           void *stream) {
  if (!sk || (count && (!d_clue_a || !d_clue_b)))
    return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_gen_clues_device: NULL argument");
  if (count == 0) return OMR_OK;
  hipStream_t st = (hipStream_t)stream;
  const Gaussian g(SIGMA_CLUE);
  if (g.table().size() > (size_t)CDT_LDS)
    return set_error(OMR_ERR_DEVICE, "omr_gen_clues_device: CDT table too large");
  std::vector<uint16_t> pk(sk->pk_a, sk->pk_a + N0);
  pk.insert(pk.end(), sk->pk_b, sk->pk_b + N0);
  DevMem<uint16_t> dpk;
  DevMem<uint64_t> dcdt;
  HIP_TRY(dpk.put(pk, st));
  HIP_TRY(dcdt.put(g.table(), st));
  constexpr size_t CHUNK = 1u << 20;
  for (size_t off = 0; off < count; off += CHUNK) {
    const size_t n = std::min(CHUNK, count - off);
    gen_clues_kernel<<<(unsigned)n, 64, 0, st>>>(dpk.p, dcdt.p, (int)g.table().size(), seed, first + off, n,
                                                d_clue_a + off * N0, d_clue_b + off * CLUES);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipStreamSynchronize(st));
  return OMR_OK;
}

extern "C" omr_status omr_keygen_detection_key_device(const omr_secret_key_pack *sk, uint64_t seed,
                                                      uint32_t *d_bsk1, uint32_t *d_ksk,
                                                      uint64_t *d_bsk2, uint64_t *d_tk, void *stream) {
  if (!sk || !d_bsk1 || !d_ksk || !d_bsk2 || !d_tk)
    return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_keygen_detection_key_device: NULL argument");
  hipStream_t st = (hipStream_t)stream;
  const Gaussian g1(SIGMA_BR1), gks(SIGMA_KS), g2(SIGMA_BR2), gt(SIGMA_TRACE);
  for (const Gaussian *g : {&g1, &g2, &gt})
    if (g->table().size() > (size_t)CDT_LDS)
      return set_error(OMR_ERR_DEVICE, "omr_keygen_detection_key_device: CDT table too large");
  const HostNtt &T1 = ntt1(), &T2 = ntt2();
  // per-row gadget values (BlindRotationKey::generate: s_i * B^k * 2^drop in component k / D + k)
  std::vector<uint64_t> mg1((size_t)N0 * 2 * D1), mg2((size_t)NI * 2 * D2);
  for (size_t row = 0; row < mg1.size(); ++row) {
    const int r = (int)(row % (2 * D1)), k = r < D1 ? r : r - D1;
    mg1[row] = sk->s0[row / (2 * D1)] ? (1ull << (DROP1 + k * LOGB1)) : 0;
  }
  for (size_t row = 0; row < mg2.size(); ++row) {
    const int r = (int)(row % (2 * D2)), k = r < D2 ? r : r - D2;
    mg2[row] = sk->sint[row / (2 * D2)] ? (1ull << (DROP2 + k * LOGB2)) : 0;
  }
  // trace key: sigma_g(s2) per automorphism, 2^(2j) per digit (TraceKey::new)
  std::vector<int8_t> sgs((size_t)TRACE_STEPS * N2);
  std::vector<uint64_t> tscale((size_t)TRACE_STEPS * DT);
  for (int k = 0; k < TRACE_STEPS; ++k) {
    const uint32_t g = (uint32_t)(N2 >> k) + 1;
    for (int i = 0; i < N2; ++i) {
      const uint32_t e = (uint32_t)(((uint64_t)i * g) % (2 * N2));
      if (e < (uint32_t)N2) sgs[(size_t)k * N2 + e] = sk->s2[i];
      else sgs[(size_t)k * N2 + e - N2] = (int8_t)-sk->s2[i];
    }
    for (int j = 0; j < DT; ++j) tscale[(size_t)k * DT + j] = (1ull << (2 * j)) % Q2;
  }
  DevMem<double> dtw1, ditw1, dtw2, ditw2, ds1, ds2;
  DevMem<uint64_t> dmg1, dmg2, dscale, dc1, dcks, dc2, dct;
  DevMem<int8_t> dsgs, dsk1;
  DevMem<uint8_t> dsint;
  DevMem<int> dover;
  const int zero = 0;
  HIP_TRY(dtw1.put(centred_vec(T1.w, Q1), st));
  HIP_TRY(ditw1.put(centred_vec(T1.iw, Q1), st));
  HIP_TRY(dtw2.put(centred_vec(T2.w, Q2), st));
  HIP_TRY(ditw2.put(centred_vec(T2.iw, Q2), st));
  HIP_TRY(ds1.put(centred_vec(sk->s1_ntt, Q1), st));
  HIP_TRY(ds2.put(centred_vec(sk->s2_ntt, Q2), st));
  HIP_TRY(dmg1.put(mg1, st));
  HIP_TRY(dmg2.put(mg2, st));
  HIP_TRY(dscale.put(tscale, st));
  HIP_TRY(dsgs.put(sgs, st));
  HIP_TRY(dsk1.put(sk->s1, N1, st));
  HIP_TRY(dsint.put(sk->sint, NI, st));
  HIP_TRY(dc1.put(g1.table(), st));
  HIP_TRY(dcks.put(gks.table(), st));
  HIP_TRY(dc2.put(g2.table(), st));
  HIP_TRY(dct.put(gt.table(), st));
  HIP_TRY(dover.put(&zero, 1, st));
  RowJob j1{seed, DOM_BSK1, N0 * 2 * D1, D1, dmg1.p, ds1.p, dtw1.p, ditw1.p,
            centred_d(T1.ninv, Q1), dc1.p, (int)g1.table().size(), nullptr, nullptr, dover.p};
  rlwe_rows_kernel<1, uint32_t><<<j1.rows, 256, 0, st>>>(j1, d_bsk1);
  HIP_TRY(hipGetLastError());
  ksk_rows_kernel<<<N1 * KS_DIGITS, 64, 0, st>>>(seed, dsint.p, dsk1.p, dcks.p, (int)gks.table().size(),
                                                 N1 * KS_DIGITS, d_ksk, dover.p);
  HIP_TRY(hipGetLastError());
  RowJob j2{seed, DOM_BSK2, NI * 2 * D2, D2, dmg2.p, ds2.p, dtw2.p, ditw2.p,
            centred_d(T2.ninv, Q2), dc2.p, (int)g2.table().size(), nullptr, nullptr, dover.p};
  rlwe_rows_kernel<2, uint64_t><<<j2.rows, 256, 0, st>>>(j2, d_bsk2);
  HIP_TRY(hipGetLastError());
  RowJob jt{seed, DOM_TK, TRACE_STEPS * DT, 1, nullptr, ds2.p, dtw2.p, ditw2.p,
            centred_d(T2.ninv, Q2), dct.p, (int)gt.table().size(), dsgs.p, dscale.p, dover.p};
  rlwe_rows_kernel<2, uint64_t><<<jt.rows, 256, 0, st>>>(jt, d_tk);
  HIP_TRY(hipGetLastError());
  int over = 0;
  HIP_TRY(hipMemcpyAsync(&over, dover.p, sizeof(int), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (over)
    return set_error(OMR_ERR_DEVICE, "omr_keygen_detection_key_device: uniform stream overrun");
  return OMR_OK;
}

// Detector context: device-resident keys and tables, batch orchestration and the C ABI of
// include/omr_gpu.h for the detect / encode path.
//
// Detector::new (detector.rs:85-110) -> omr_ctx_create: uploads the coefficient-domain keys,
// converts them on the GPU (BSK1 to the FFT domain x 1/512, BSK2 and the trace key to centred
// FP64 NTT-domain rows with N^-1 folded into the external-product keys, the KSK to int8 limbs)
// and builds the LUTs (:457-503). Detector::detect (:135-166) for a batch of messages -> four
// launches per chunk: br1f_kernel (7 blind rotations per message), sum7_kernel, ks_mfma_kernel,
// br2f_kernel (level-2 rotation on the exact FFT + the trace).
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "br1_ntt.hpp"
#include "br2_fft.hpp"
#include "detect_kernels.hpp"
#include "encode_kernels.hpp"
#include "key_spectra.hpp"
#include "latency_kernels.hpp"

using namespace omr;

#define HIP_TRY(expr)                                                                     \
  do {                                                                                    \
    hipError_t _e = (expr);                                                               \
    if (_e != hipSuccess)                                                                 \
      return set_error(OMR_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

namespace {

typedef unsigned __int128 u128;

uint64_t h_mulmod(uint64_t a, uint64_t b, uint64_t q) { return (uint64_t)((u128)a * b % q); }
uint64_t h_powmod(uint64_t b, uint64_t e, uint64_t q) {
  uint64_t r = 1;
  b %= q;
  while (e) {
    if (e & 1) r = h_mulmod(r, b, q);
    b = h_mulmod(b, b, q);
    e >>= 1;
  }
  return r;
}
double centred(uint64_t v, uint64_t q) { return v > (q - 1) / 2 ? (double)v - (double)q : (double)v; }
uint32_t h_brv(uint32_t x, int bits) { return __builtin_bitreverse32(x) >> (32 - bits); }

// psi^brv(k), psi^-brv(k) as centred doubles (the convention of include/omr_gpu.h).
void twiddles(uint64_t q, int N, uint64_t g, std::vector<double> &tw, std::vector<double> &itw) {
  const int L = __builtin_ctz(N);
  const uint64_t psi = h_powmod(g, (q - 1) / (2 * (uint64_t)N), q);
  const uint64_t ipsi = h_powmod(psi, q - 2, q);
  tw.resize(N);
  itw.resize(N);
  for (int k = 0; k < N; ++k) {
    const uint32_t e = h_brv((uint32_t)k, L);
    tw[k] = centred(h_powmod(psi, e, q), q);
    itw[k] = centred(h_powmod(ipsi, e, q), q);
  }
}

// LookUpTable::negacyclic_lut (lut.rs:12-27): chunk c of N >> log_t coefficients holds
// v[(c+1)/2] (itertools::interleave(v, v[1..])).
std::vector<double> negacyclic_lut(const std::vector<uint64_t> &v, int N, int log_t, uint64_t q) {
  std::vector<double> lut(N, 0.0);
  const int hd = N >> log_t;
  for (int c = 0; c < N / hd; ++c) {
    const size_t idx = (size_t)(c + 1) / 2;
    const uint64_t val = idx < v.size() ? v[idx] : 0;
    for (int j = 0; j < hd; ++j) lut[c * hd + j] = centred(val, q);
  }
  return lut;
}

// FFT twiddles of Fft512 (device_fft.hpp, WgFft): node i of stage s -> w^(eps(s, i) / 2),
// w = exp(i pi / 2n), n = 512, eps(0, 0) = n, eps(s+1, 2i) = eps(s, i) / 2,
// eps(s+1, 2i+1) = eps(s, i) / 2 + 2n (mod 4n). Layout (WgFft::TW_*): [0, 7) T_1..T_7 of the
// pass-0 radix-8 block (A = node(0, 0), B = node(1, 0), C = node(2, 0), T = (C, B, BC, A, AC, AB,
// ABC)), inverse only; [7, 11) the tangent forms (cos, tan) of pass 0's A, B, C, w8 C = node(2, 2);
// 11 + 2 blk + (A, B) the tangent forms of the pass-1 radix-4 block blk (A = node(3, blk),
// B = node(4, 2 blk)); 27 + (t - 1) 32 + hi the pass-2 T_t (A = node(5, hi), B = node(6, 2 hi),
// C = node(7, 4 hi)), inverse only; 251 + 32 k + hi the tangent forms of pass 2's A, B, C, w8 C;
// 379 + 64 e1 + lane the tangent form of the pass-3 (stage 8) even-sibling node
// ((lane & 31) << 3 | (lane >> 5) << 2 | e1 << 1). Each entry is an exact angle (sum of the nodes'
// integer half-eps) evaluated in long double and rounded once (tan = sin / cos in long double).
std::vector<double2> fft_twiddles() {
  using F = Fft512;
  const int L = 9, n = 1 << L;
  std::vector<double2> tw(n, make_double2(1.0, 0.0));
  std::vector<std::vector<long>> half(L);  // half[s][i] = eps(s, i) / 2
  std::vector<long> eps{n};
  for (int s = 0; s < L; ++s) {
    std::vector<long> next;
    for (long e : eps) {
      half[s].push_back(e / 2);
      next.push_back((e / 2) % (4 * n));
      next.push_back((e / 2 + 2 * n) % (4 * n));
    }
    eps.swap(next);
  }
  auto angle = [&](long h) {
    return 3.14159265358979323846264338327950288L * (long double)(h % (8 * n)) / (long double)(2 * n);
  };
  auto at = [&](long h) { return make_double2((double)cosl(angle(h)), (double)sinl(angle(h))); };
  auto ct = [&](long h) {  // no node of the tree lies on an axis, so cos != 0
    const long double c = cosl(angle(h)), s = sinl(angle(h));
    return make_double2((double)c, (double)(s / c));
  };
  auto radix8 = [&](int s0, int hi, auto put) {
    const long a = half[s0][hi], b = half[s0 + 1][2 * hi], c = half[s0 + 2][4 * hi];
    const long h[8] = {0, c, b, b + c, a, a + c, a + b, a + b + c};
    for (int t = 1; t < 8; ++t) put(t, at(h[t]));
  };
  auto radix8_ct = [&](int s0, int hi, auto put) {
    const long h[4] = {half[s0][hi], half[s0 + 1][2 * hi], half[s0 + 2][4 * hi], half[s0 + 2][4 * hi + 2]};
    for (int k = 0; k < 4; ++k) put(k, ct(h[k]));
  };
  radix8(0, 0, [&](int t, double2 v) { tw[F::TW_P0I + t - 1] = v; });
  radix8_ct(0, 0, [&](int k, double2 v) { tw[F::TW_P0F + k] = v; });
  for (int blk = 0; blk < 8; ++blk) {
    tw[F::TW_P1 + 2 * blk] = ct(half[3][blk]);
    tw[F::TW_P1 + 2 * blk + 1] = ct(half[4][2 * blk]);
  }
  for (int hi = 0; hi < 32; ++hi) {
    radix8(5, hi, [&](int t, double2 v) { tw[F::TW_P2I + (t - 1) * 32 + hi] = v; });
    radix8_ct(5, hi, [&](int k, double2 v) { tw[F::TW_P2F + k * 32 + hi] = v; });
  }
  for (int e1 = 0; e1 < 2; ++e1)
    for (int lane = 0; lane < 64; ++lane)
      tw[F::TW_P3 + 64 * e1 + lane] = ct(half[8][((lane & 31) << 3) | ((lane >> 5) << 2) | (e1 << 1)]);
  return tw;
}

// Fft1024 twiddles (br2_fft.hpp): pass p = 1..4, block hi -> (B, A, AB) at tw_off(p) + 3 hi (the
// inverse), then the forward's tangent forms (cos, tan) of (A, B) at TW_LEN + ct_off(p) + 2 hi, with
// A = W(2p, hi), B = W(2p + 1, 2 hi) of the tree with n = 1024 (eps(0, 0) = n, w = e^{i pi / 2n});
// each entry an exact angle evaluated in long double and rounded once.
std::vector<double2> fft2_twiddles() {
  const int L = 10, n = 1 << L;
  std::vector<std::vector<long>> half(L);
  std::vector<long> eps{n};
  for (int s = 0; s < L; ++s) {
    std::vector<long> next;
    for (long e : eps) {
      half[s].push_back(e / 2);
      next.push_back((e / 2) % (4 * n));
      next.push_back((e / 2 + 2 * n) % (4 * n));
    }
    eps.swap(next);
  }
  auto at = [&](long h) {
    const long double ang = 3.14159265358979323846264338327950288L * (long double)(h % (8 * n)) / (long double)(2 * n);
    return make_double2((double)cosl(ang), (double)sinl(ang));
  };
  auto ct = [&](long h) {  // tangent form (cos, tan); no node of the tree lies on an axis
    const long double ang = 3.14159265358979323846264338327950288L * (long double)(h % (8 * n)) / (long double)(2 * n);
    const long double c = cosl(ang), s = sinl(ang);
    return make_double2((double)c, (double)(s / c));
  };
  std::vector<double2> tw(Fft1024::TW_LEN + Fft1024::CT_LEN);
  int off = 0;
  for (int p = 1; p <= 4; ++p)
    for (int hi = 0; hi < (1 << (2 * p)); ++hi) {
      const long a = half[2 * p][hi], b = half[2 * p + 1][2 * hi];
      tw[off++] = at(b);
      tw[off++] = at(a);
      tw[off++] = at(a + b);
      tw[Fft1024::TW_LEN + Fft1024::ct_off(p) + 2 * hi] = ct(a);
      tw[Fft1024::TW_LEN + Fft1024::ct_off(p) + 2 * hi + 1] = ct(b);
    }
  return tw;
}

// ---- exact twiddles of the double-double key transforms (key_spectra.hpp) ----
// exp(i pi h / 2n) in double-double: quadrant and complement reduction on the integer h, then
// Taylor series of sin / cos on [0, pi/4] (terms below 2^-110 dropped): accurate to a few 2^-104.
DD dd_div_d(DD a, double b) {
  const double q1 = a.hi / b, p = q1 * b, pe = std::fma(q1, b, -p);
  return dd_quick(q1, ((a.hi - p) - pe + a.lo) / b);
}
void dd_sincos(DD x, DD &sn, DD &cs) {  // 0 <= x <= pi / 4
  const DD x2 = dd_mul(x, x);
  DD ts = x, tc = {1.0, 0.0};
  sn = x;
  cs = tc;
  for (int k = 1; k < 20; ++k) {
    ts = dd_div_d(dd_mul(ts, x2), (double)((2 * k) * (2 * k + 1)));
    tc = dd_div_d(dd_mul(tc, x2), (double)((2 * k - 1) * (2 * k)));
    sn = dd_add(sn, k & 1 ? dd_neg(ts) : ts);
    cs = dd_add(cs, k & 1 ? dd_neg(tc) : tc);
  }
}
CDD dd_expi(long h, long n) {
  const DD PI = {3.141592653589793116, 1.2246467991473532e-16};
  const long r = ((h % (4 * n)) + 4 * n) % (4 * n);  // angle pi r / 2n, period 4n
  const long quad = r / n, rho = r % n;               // quad * pi/2 + pi rho / 2n
  const bool comp = 2 * rho > n;                      // beyond pi/4: use the complement
  const long m = comp ? n - rho : rho;
  DD sn, cs;
  dd_sincos(dd_mul(PI, DD{(double)m / (2.0 * (double)n), 0.0}), sn, cs);
  DD c = comp ? sn : cs, s = comp ? cs : sn;  // cos, sin of pi rho / 2n
  for (long q = 0; q < quad; ++q) {             // rotate by pi/2: (c, s) -> (-s, c)
    const DD t = c;
    c = dd_neg(s);
    s = t;
  }
  return {c, s};
}
// tree twiddles W(s, i) = w^(eps(s, i) / 2), stage s node i at (1 << s) - 1 + i (dd_tree_fft)
std::vector<CDD> dd_tree_twiddles(int L) {
  const long n = 1L << L;
  std::vector<CDD> tw;
  std::vector<long> eps{n};
  for (int s = 0; s < L; ++s) {
    std::vector<long> next;
    for (long e : eps) {
      tw.push_back(dd_expi(e / 2, n));
      next.push_back((e / 2) % (4 * n));
      next.push_back((e / 2 + 2 * n) % (4 * n));
    }
    eps.swap(next);
  }
  return tw;
}

// A priori bound on |computed - exact| of every rounded coefficient of one external product
// (DESIGN.md §3a). For one CMUX step and one output spectrum, with n complex points, D =
// sqrt(2n) d_max the 2-norm bound of a digit polynomial, kappa_r the largest |K^| of GGSW row r
// (row_max_abs_kernel), the rows accumulated in the order r(0), r(1), ... by two fmas each:
//   E = n D (1 + 2^-30) [(delta_fwd + delta_inv + u (1 + 2^-40)) sum_r kappa_r + sqrt(2) u sum_k (2R - 2k) kappa_r(k)]
// the forward digit transforms within delta_fwd and the inverse within delta_inv relative 2-norm
// error (forward in tangent form, 4u per radix-2 stage: level 1 37u (9 stages), level 2 41u (10);
// inverse: level 1 32u -- 8u per premultiplied radix-8 pass, 5u per Gentleman-Sande stage of P1 and
// P3 --, level 2 26u -- 5u per premultiplied radix-4 pass --, rounded up), the sequential fma accumulation, and
// the double-double keys' |K^ - K| <= u |K|. The maximum over every step and output spectrum.
// kmax: [steps][rows][outputs] (level 1: [512][8][2]; level 2: [670][12][2 out][2 limb], the limbs
// as two more "outputs"). Level 3: level 2 as br2y_kernel (the latency path) accumulates it: each
// 256-thread group chains its three rows (its j-th at weight 2 (3 - j)), then two additions (the
// two groups' partials, the partner workgroup's) add 1 each: weight 8 - 2 j for digit 3 g + j.
// Level 4: the fused FFT trace (br2f_trace): 11 steps, 25 rows (digits |d| <= 3) accumulated in
// order, the trace key's rows [11 * 25][2 out][2 limb] as kmax.
double apriori_bound(int level, const std::vector<double> &kmax) {
  const double u = 0x1p-53;
  const bool y = level == 3, tr = level == 4;
  if (y || tr) level = 2;
  const int n = level == 1 ? 512 : 1024, R = level == 1 ? 2 * D1 : tr ? DT : 2 * D2, O = level == 1 ? 2 : 4;
  const int steps = level == 1 ? N0 : tr ? TRACE_STEPS : NI;
  // accumulation order of the kernels' MAC: br1f / br1l rows 0..7; br2f digits in issue order
  // g = 2 j + w, row p D2 + j + 3 w (br2_fft.hpp)
  const int order2[12] = {0, 3, 1, 4, 2, 5, 6, 9, 7, 10, 8, 11};
  // largest digit: level 1 16, level 2 64, the trace's balanced base-4 digits 2 (the top one 3)
  const double D = std::sqrt(2.0 * n) * (level == 1 ? 16.0 : tr ? 3.0 : 64.0);
  const double dft = level == 1 ? 37 + 32 : 41 + 26;  // delta_fwd + delta_inv, in units of u
  const double cf = dft * u + u * (1 + 0x1p-40), cw = std::sqrt(2.0) * u;
  double worst = 0.0;
  for (int i = 0; i < steps; ++i)
    for (int o = 0; o < O; ++o) {
      double s = 0.0, w = 0.0;
      for (int k = 0; k < R; ++k) {
        const int r = level == 1 || tr ? k : order2[k];
        const double kap = kmax[((size_t)i * R + r) * O + o];
        s += kap;
        w += (y ? 8.0 - 2.0 * ((r % D2) % 3) : 2.0 * R - 2.0 * k) * kap;
      }
      worst = std::max(worst, cf * s + cw * w);
    }
  return (double)n * D * worst * (1 + 0x1p-30);
}

}  // namespace

#ifndef OMR_DEFAULT_LATENCY_MAX
#define OMR_DEFAULT_LATENCY_MAX 64  // chunks up to this many messages run the latency kernels
#endif

struct omr_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  double2 *bsk1f = nullptr;  // level-1 FFT-domain keys [512][8][2][512] complex, x 1/512
  double2 *bsk1l = nullptr;  // the same in br1l_kernel's layout [512][8 slot][8 row][2][64 lane]
  double *bsk1n = nullptr;   // BSK1 in the NTT domain x 1/1024 [512][8][2][1024] (br1_ntt.hpp: level 1's exact path)
  // the coefficient-domain BSK1 kept on the host (32 MB) until bsk1n is built: bsk1n (64 MB of HBM)
  // is converted lazily, only when level 1 is guarded or run exactly (ensure_bsk1n)
  std::vector<uint32_t> bsk1_host;
  double2 *fft1 = nullptr;   // level-1 FFT twiddles
  double *bsk2 = nullptr, *tk = nullptr;  // BSK2 NTT domain (latency kernels), trace key
  double2 *bsk2f = nullptr;                // BSK2 as FFT-domain 25-bit limbs (br2f_kernel), x 1/1024
  double2 *tkf = nullptr;                  // the trace key the same way (br2f_kernel's fused trace)
  double2 *fft2 = nullptr;                 // Fft1024 twiddles
  uint32_t *kskb = nullptr;  // int8 limbs of the KSK, [1024][4][672][32] (matrix-core key switch)
  double *tables = nullptr;  // tw1 itw1 tw2 itw2 lut1 lut2 tw2c
  uint16_t *trace_tabs = nullptr;
  DeviceTables tb{};
  size_t batch = OMR_DEFAULT_BATCH, batch_cap = 0;
  size_t enc_max_chunks = OMR_ENC_MAX_CHUNKS;  // chunk partials per encode ciphertext (omr_ctx_set_encode_chunks)
  uint32_t *ext = nullptr, *lwe1t = nullptr, *lwe_int = nullptr;
  // chunks of at most latency_max messages run the latency kernels (latency_kernels.hpp)
  size_t latency_max = OMR_DEFAULT_LATENCY_MAX;
  int *ks_part = nullptr;  // split key-switch partial sums, [KS_SPLIT][64][672][4]
  // two-CU level-2 latency kernel (br2x_kernel, cooperative launch): partial hand-off slots
  // [n][2][2][N2], flags [n][2], a timeout flag x_err that every launch copies to the pinned host
  // word x_err_host on its stream (read by omr_ctx_check and at the start of the next call)
  double *x_slots = nullptr;
  uint32_t *x_flags = nullptr;
  int *x_err = nullptr, *x_err_host = nullptr;
  size_t x_cap = 0;
  // multi-CU trace of the latency path (trace_x_kernel): partial slots [n][TRACE_X][2][2][N2],
  // flags [n][TRACE_X]
  double *t_slots = nullptr;
  uint32_t *t_flags = nullptr;
  size_t t_cap = 0;
  int num_cu = 0;
  bool coop = false;  // hipDeviceAttributeCooperativeLaunch
  // rounding-margin guard (exactness.hpp): guarded kernel variants for level l when the user set
  // the guard or the key's a priori bound E_l >= 0.5 (guard_auto, the exactness contract); margin:
  // the GUARD_WORDS guard words (bits of the largest |y - rint(y)|, per launch and cumulative, and
  // the breach counts); kappa: largest stored key spectrum magnitude per level; apriori: the bound it
  // gives (apriori_bound); thr = 1 - apriori, the certificate threshold of one launch
  bool guard = false, guard_auto[2] = {false, false};
  // omr_ctx_set_exact_level1: every level-1 launch on the exact modular NTT (br1n_kernel)
  bool exact1 = false;
  unsigned long long *margin = nullptr;
  double kappa[2] = {0.0, 0.0}, apriori[2] = {0.0, 0.0}, thr[2] = {1.0, 1.0};
  // the fused trace on the FFT (br2f_trace) when its a priori bound (apriori_bound level 4) is below
  // 0.5; otherwise br2f_kernel stops at the rotation and trace_kernel's NTT runs (never on a real key)
  double apriori_t = 1.0;
  bool trace_fft = false;
  // the latency path's level 2 on the FFT (br2y_kernel with its key-prefetch helpers; the default
  // since round 5, 6.6 vs 7.6-7.9 ms for br2x at one message; OMR_BR2Y=0 at context creation: br2x)
  // when its accumulation order's bound (apriori_bound level 3) proves it exact and the level is
  // not guarded; br2x_kernel's NTT otherwise
  double apriori_y = 1.0;
  bool br2y = true;
  bool no_prefetch = false;  // OMR_PREFETCH=0: the latency kernels launch no key-prefetch helpers
  bool no_fast_handoff = false;  // OMR_FAST_HANDOFF=0: br2y keeps the sc1 hand-off on one XCD too
  // host-API staging
  uint16_t *s_clue_a = nullptr, *s_clue_b = nullptr;
  uint64_t *s_out = nullptr;
  size_t staged = 0;
  // encode workspace
  uint64_t *partial = nullptr;
  size_t partial_cap = 0;
  // The scratch above is shared by every call on the context, while device-buffer calls only
  // enqueue on the caller's stream: the last stream that used it records scratch_free, and a call
  // on another stream waits for that event before its first kernel.
  hipEvent_t scratch_free = nullptr;
  hipStream_t scratch_stream = nullptr;
  // omr_detect_batch stages the host input in pieces of `batch` messages: their stage times are
  // summed here so omr_last_timing covers the whole call (device-buffer calls read the events)
  omr_detect_timing host_timing{};
  bool host_timing_valid = false;
  // timing: mode 0 off, 1 stage events around the production kernels, 2 trace as its own launch
  int timing = 0;
  std::vector<hipEvent_t> events;  // EV_PER_CHUNK per chunk
  size_t timed_messages = 0, timed_chunks = 0;
  bool timed_split = false;  // the timed call ran the trace as its own launch in every chunk
  std::mutex mu;
  // omr_detect: concurrent single-message calls are combined into batched launches (a leader
  // takes every queued request, runs them as one detect, and wakes their callers)
  struct DetectReq {
    const uint16_t *a, *b;
    uint64_t *out;
    omr_status st;
    std::string err;
    bool done;
  };
  std::mutex qmu;
  std::condition_variable qcv;
  std::vector<DetectReq *> queue;
  bool leader = false;
  size_t coalesce_max = 65536;   // messages per combined launch
  long coalesce_window_us = 0;   // a leader waits this long for more requests before launching
  size_t coalesced_calls = 0, coalesced_launches = 0;
};

#define OMR_BR1_NAME "br1f_kernel"
#define OMR_KS_NAME "ks_mfma_kernel"
#define OMR_BR2_NAME "br2f_kernel"

namespace {

bool guarded(const omr_ctx *c, int level) { return c->guard || c->guard_auto[level]; }

// Frees a device allocation made by this library (a failure here leaves nothing to recover).
template <typename T>
void dev_free(T *&p) {
  if (p) (void)hipFree((void *)p);
  p = nullptr;
}

// Scoped device allocation (freed on every return path).
template <typename T>
struct DevBufHost {
  T *p = nullptr;
  ~DevBufHost() { dev_free(p); }
};

// Scratch reuse across streams (see omr_ctx::scratch_free). Callers hold c->mu.
omr_status scratch_acquire(omr_ctx *c, hipStream_t st) {
  if (c->scratch_stream && c->scratch_stream != st) HIP_TRY(hipStreamWaitEvent(st, c->scratch_free, 0));
  return OMR_OK;
}
omr_status scratch_release(omr_ctx *c, hipStream_t st) {
  HIP_TRY(hipEventRecord(c->scratch_free, st));
  c->scratch_stream = st;
  return OMR_OK;
}
// Reallocating scratch: every stream that used it must be done first.
omr_status scratch_idle(omr_ctx *c) {
  if (c->scratch_stream) HIP_TRY(hipEventSynchronize(c->scratch_free));
  return OMR_OK;
}

omr_status ensure_batch(omr_ctx *c, size_t B) {
  if (B <= c->batch_cap) return OMR_OK;
  omr_status s;
  if ((s = scratch_idle(c)) != OMR_OK) return s;
  dev_free(c->ext);
  dev_free(c->lwe1t);
  dev_free(c->lwe_int);
  c->batch_cap = 0;
  HIP_TRY(hipMalloc(&c->ext, B * CLUES * (N1 + 1) * sizeof(uint32_t)));
  HIP_TRY(hipMalloc(&c->lwe1t, B * (N1 + 1) * sizeof(uint32_t)));
  HIP_TRY(hipMalloc(&c->lwe_int, B * (NI + 1) * sizeof(uint32_t)));
  if (!c->ks_part) HIP_TRY(hipMalloc(&c->ks_part, (size_t)KS_SPLIT * 64 * KSM_COLS * KSM_LIMBS * sizeof(int)));
  c->batch_cap = B;
  return OMR_OK;
}

omr_status ensure_partial(omr_ctx *c, size_t elems) {
  if (elems <= c->partial_cap) return OMR_OK;
  omr_status s;
  if ((s = scratch_idle(c)) != OMR_OK) return s;
  dev_free(c->partial);
  c->partial_cap = 0;
  HIP_TRY(hipMalloc(&c->partial, elems * sizeof(uint64_t)));
  c->partial_cap = elems;
  return OMR_OK;
}

template <int LEVEL, typename IN, typename OUT>
omr_status convert_keys(const IN *host, size_t npoly, OUT *dev, double scale, const double *tw,
                        hipStream_t st) {
  constexpr int N = Mod<LEVEL>::N;
  constexpr int T = LEVEL == 1 ? BR1_T : BR2_T;
  const size_t chunk = 4096;  // polynomials per upload
  IN *tmp = nullptr;
  HIP_TRY(hipMalloc(&tmp, chunk * N * sizeof(IN)));
  for (size_t p0 = 0; p0 < npoly; p0 += chunk) {
    const size_t n = std::min(chunk, npoly - p0);
    HIP_TRY(hipMemcpyAsync(tmp, host + p0 * N, n * N * sizeof(IN), hipMemcpyDefault, st));
    key_to_ntt_kernel<LEVEL, IN, OUT><<<n, T, 0, st>>>(tmp, dev + p0 * N, n, scale, tw);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(st));
  }
  dev_free(tmp);
  return OMR_OK;
}

// ---- BSK2 rows -> the CmuxNtt forward order, x scale (the blind rotation's key layout) ----
__global__ __launch_bounds__(256) static void key_to_cmux_kernel(const uint64_t *in, double *out, size_t npoly,
                                                        double scale, const double *tw2c) {
  using M = Mod<2>;
  using NTT = CmuxNtt;
  __shared__ double lds[NTT::LDS_DOUBLES];
  __shared__ double tws[NTT::N];
  const size_t poly = blockIdx.x;
  const int tid = threadIdx.x;
  if (poly >= npoly) return;
  const uint64_t *src = in + poly * NTT::N;
  double x[NTT::E];
#pragma unroll
  for (int e = 0; e < NTT::E; ++e) {
    x[e] = from_u64<M>(src[tid + e * NTT::T]);
    tws[tid + e * NTT::T] = tw2c[tid + e * NTT::T];
  }
  __syncthreads();
  NTT::fwd<0>(x, lds, tws, tid);
  double *dst = out + poly * NTT::N + tid * NTT::E;
#pragma unroll
  for (int e = 0; e < NTT::E; ++e) dst[e] = canon<M>(mm<M>(canon<M>(x[e]), scale));
}

omr_status convert_keys_cmux(const uint64_t *host, size_t npoly, double *dev, double scale, const double *tw2c,
                             hipStream_t st) {
  const size_t chunk = 4096;  // polynomials per upload
  uint64_t *tmp = nullptr;
  HIP_TRY(hipMalloc(&tmp, chunk * N2 * sizeof(uint64_t)));
  for (size_t p0 = 0; p0 < npoly; p0 += chunk) {
    const size_t n = std::min(chunk, npoly - p0);
    HIP_TRY(hipMemcpyAsync(tmp, host + p0 * N2, n * N2 * sizeof(uint64_t), hipMemcpyDefault, st));
    key_to_cmux_kernel<<<n, CmuxNtt::T, 0, st>>>(tmp, dev + p0 * N2, n, scale, tw2c);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(st));
  }
  dev_free(tmp);
  return OMR_OK;
}

// BSK1 / BSK2 -> FFT-domain key spectra in double-double, rounded once (key_spectra.hpp).
template <int LEVEL, typename IN>
omr_status convert_keys_dd(const IN *host, size_t npoly, double2 *dev, hipStream_t st) {
  constexpr int N = LEVEL == 1 ? N1 : N2;
  const auto twv = dd_tree_twiddles(LEVEL == 1 ? 9 : 10);
  DevBufHost<CDD> tw;
  HIP_TRY(hipMalloc(&tw.p, twv.size() * sizeof(CDD)));
  HIP_TRY(hipMemcpy(tw.p, twv.data(), twv.size() * sizeof(CDD), hipMemcpyHostToDevice));
  const size_t chunk = 4096;  // polynomials per upload
  DevBufHost<IN> tmp;
  HIP_TRY(hipMalloc(&tmp.p, chunk * N * sizeof(IN)));
  for (size_t p0 = 0; p0 < npoly; p0 += chunk) {
    const size_t n = std::min(chunk, npoly - p0);
    HIP_TRY(hipMemcpyAsync(tmp.p, host + p0 * N, n * N * sizeof(IN), hipMemcpyDefault, st));
    key_spectrum_dd_kernel<LEVEL><<<(unsigned)(n * (LEVEL == 1 ? 1 : 2)), KDD_T, 0, st>>>(
        tmp.p, dev + p0 * (LEVEL == 1 ? Fft512::N : 2 * Fft1024::n), n, tw.p);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(st));
  }
  return OMR_OK;
}

bool latency_path(const omr_ctx *c, size_t n) { return n <= c->latency_max; }

// The two-CU kernel's bounded hand-off wait: a workgroup whose partner never published leaves its
// loop and sets x_err; each launch then copies x_err to the pinned x_err_host on its stream. This
// reports (and clears) an error whose copy has landed: callers sync the stream first for a
// definitive answer (omr_ctx_check, the host entry points), or call it before enqueueing new work
// (the device entry points) so a failed earlier call is never attributed to a later one.
omr_status take_handoff_error(omr_ctx *c) {
  if (!c->x_err_host || !__atomic_load_n(c->x_err_host, __ATOMIC_ACQUIRE)) return OMR_OK;
  HIP_TRY(hipDeviceSynchronize());  // no launch may still be copying the flag
  (void)__atomic_exchange_n(c->x_err_host, 0, __ATOMIC_ACQ_REL);
  HIP_TRY(hipMemset(c->x_err, 0, sizeof(int)));
  return set_error(OMR_ERR_DEVICE,
                   "level-2 two-CU hand-off timed out: the output of an earlier detect call on this "
                   "context is invalid");
}

// Zero the per-launch guard word of `level` before a guarded launch.
omr_status guard_begin(omr_ctx *c, int level, hipStream_t st) {
  HIP_TRY(hipMemsetAsync(c->margin + 2 + level, 0, sizeof(unsigned long long), st));
  return OMR_OK;
}
// After a guarded launch and its conditional exact re-run: fold the launch's margin into the
// cumulative word and count a breach.
omr_status guard_end(omr_ctx *c, int level, hipStream_t st) {
  guard_fold_kernel<<<1, 64, 0, st>>>(c->margin, level, c->thr[level]);
  HIP_TRY(hipGetLastError());
  return OMR_OK;
}

// Level 1's exact-NTT key (br1n_kernel / br1n_fallback_kernel), built on first need: when level 1
// is guarded (the exactness contract's re-run target) or run exactly. Callers hold c->mu (or own c).
omr_status ensure_bsk1n(omr_ctx *c) {
  if (c->bsk1n) return OMR_OK;
  if (c->bsk1_host.size() != BSK1_ELEMS)
    return set_error(OMR_ERR_DEVICE, "ensure_bsk1n: the coefficient-domain BSK1 is gone");
  HIP_TRY(hipMalloc(&c->bsk1n, BSK1_ELEMS * sizeof(double)));
  const double ninv1 = centred(h_powmod(N1, Q1 - 2, Q1), Q1);
  omr_status s;
  if ((s = convert_keys<1, uint32_t, double>(c->bsk1_host.data(), BSK1_ELEMS / N1, c->bsk1n, ninv1, c->tb.tw1,
                                             c->stream)) != OMR_OK) {
    dev_free(c->bsk1n);
    return s;
  }
  std::vector<uint32_t>().swap(c->bsk1_host);
  return OMR_OK;
}

// LWE key switch + modulus switch of B messages (lwe1t [1025][B] -> out [B][671]). Up to 64
// messages (the latency path) the input coefficients are split over KS_SPLIT workgroup slices.
omr_status launch_ks(omr_ctx *c, int B, uint32_t *out, hipStream_t st) {
  if (latency_path(c, (size_t)B) && B <= 64) {
    ks_mfma_split_kernel<<<dim3(1, KSM_COLS / 32, KS_SPLIT), 64, 0, st>>>(c->lwe1t, c->kskb, c->ks_part, B, 64);
    HIP_TRY(hipGetLastError());
    ks_combine_kernel<<<(B * (NI + 1) + 255) / 256, 256, 0, st>>>(c->ks_part, c->lwe1t, out, B, 64);
  } else {
    ks_mfma_kernel<<<dim3((B + 63) / 64, KSM_COLS / 32), 64, 0, st>>>(c->lwe1t, c->kskb, out, B);
  }
  HIP_TRY(hipGetLastError());
  return OMR_OK;
}

// Level-1 blind rotations of n (message, clue) pairs (mode 0: clue g % 7 of message g / 7 ->
// extracted LWE; mode 1: explicit LWEs -> full RLWE), BR1F_WPG rotations per workgroup.
// `msgs`: the messages of the chunk (selects the latency kernels, one workgroup per rotation).
omr_status launch_br1(omr_ctx *c, size_t n, const uint16_t *ca, const uint16_t *cb,
                      const uint16_t *la, const uint16_t *lb, uint32_t *ext, uint64_t *rlwe, int mode,
                      hipStream_t st, size_t msgs) {
  if (c->exact1) {  // the reference's arithmetic for every rotation (omr_ctx_set_exact_level1)
    br1n_kernel<<<(unsigned)n, 64, 0, st>>>(ca, cb, la, lb, c->bsk1n, c->tb, ext, rlwe, mode, n);
    HIP_TRY(hipGetLastError());
    return OMR_OK;
  }
  const unsigned g1 = (unsigned)((n + BR1F_WPG - 1) / BR1F_WPG);
  const bool g = guarded(c, 0);
  omr_status s;
  if (g && (s = guard_begin(c, 0, st)) != OMR_OK) return s;
  if (latency_path(c, msgs)) {
    if (g)
      br1l_guard_kernel<<<(unsigned)n, 64 * BR1L_WAVES, 0, st>>>(ca, cb, la, lb, c->bsk1l, c->tb, ext, rlwe, mode,
                                                                  c->margin + 2);
    else
      br1l_kernel<<<(unsigned)n, 64 * BR1L_WAVES, 0, st>>>(ca, cb, la, lb, c->bsk1l, c->tb, ext, rlwe, mode);
  } else if (g) {
    br1f_guard_kernel<<<g1, 64 * BR1F_WPG, 0, st>>>(ca, cb, la, lb, c->bsk1f, c->tb, ext, rlwe, mode, n,
                                                    c->margin + 2);
  } else {
    br1f_kernel<<<g1, 64 * BR1F_WPG, 0, st>>>(ca, cb, la, lb, c->bsk1f, c->tb, ext, rlwe, mode, n);
  }
  HIP_TRY(hipGetLastError());
  if (!g) return OMR_OK;
  // the exactness contract: a guarded launch whose margin reached 1 - E1 is recomputed on the exact
  // NTT in the same stream order (every workgroup leaves at once otherwise)
  br1n_fallback_kernel<<<(unsigned)n, 64, 0, st>>>(ca, cb, la, lb, c->bsk1n, c->tb, ext, rlwe, mode, n,
                                                   c->margin + 2, c->thr[0]);
  HIP_TRY(hipGetLastError());
  return guard_end(c, 0, st);
}

// br2x_kernel over 2 n workgroups as a cooperative launch (co-residency guaranteed, or the launch
// is refused); false when refused, so the caller falls back to br2l_kernel.
omr_status launch_br2x(omr_ctx *c, size_t n, const uint32_t *lwe_int, uint64_t *out, hipStream_t st,
                       bool *launched) {
  *launched = false;
  if (!c->coop || 2 * n > (size_t)c->num_cu) return OMR_OK;  // one 150 KB-LDS workgroup per CU
  if (n > c->x_cap) {
    omr_status s;
    if ((s = scratch_idle(c)) != OMR_OK) return s;
    dev_free(c->x_slots);
    dev_free(c->x_flags);
    c->x_cap = 0;
    HIP_TRY(hipMalloc(&c->x_slots, n * 8 * N2 * sizeof(double)));  // br2y: [n][2][2 slot][2 limb][2][1024]
    HIP_TRY(hipMalloc(&c->x_flags, n * 4 * sizeof(uint32_t)));  // br2y: + the workers' XCD ids
    c->x_cap = n;
  }
  HIP_TRY(hipMemsetAsync(c->x_flags, 0, n * 4 * sizeof(uint32_t), st));
  const double *bsk2 = c->bsk2;
  DeviceTables tb = c->tb;
  double *slots = c->x_slots;
  uint32_t *flags = c->x_flags;
  int *err = c->x_err;
  void *args[] = {(void *)&lwe_int, (void *)&bsk2, (void *)&tb, (void *)&slots, (void *)&flags, (void *)&err,
                  (void *)&out};
  // br2y_kernel (FFT) when the bound of its accumulation order proves it exact and level 2 is not
  // guarded; br2x_kernel's exact NTT otherwise (same arguments apart from the key form)
  const bool y = c->br2y && !guarded(c, 1) && c->apriori_y < 0.5;
  const double2 *bskf = c->bsk2f, *twg = c->fft2;
  // br2y: message m in column m of a grid w8 = n rounded up to 8 columns wide, its mask / body
  // workers in rows 0 / 1, plus 2 BR2Y_H rows of key prefetchers (br2_fft.hpp) when every workgroup
  // still gets a CU of its own
  const int nmsg = (int)n, w8 = (nmsg + 7) / 8 * 8, allow_fast = c->no_fast_handoff ? 0 : 1;
  const int rows = (size_t)w8 * (2 + 2 * BR2Y_H) <= (size_t)c->num_cu && !c->no_prefetch ? 2 + 2 * BR2Y_H : 2;
  if (y && (size_t)w8 * rows > (size_t)c->num_cu) return OMR_OK;  // one workgroup per CU: br2l instead
  void *args_y[] = {(void *)&lwe_int, (void *)&bskf, (void *)&twg, (void *)&tb, (void *)&slots, (void *)&flags,
                    (void *)&err, (void *)&out, (void *)&nmsg, (void *)&w8, (void *)&allow_fast};
  const void *kern = y ? reinterpret_cast<const void *>(&br2y_kernel) : reinterpret_cast<const void *>(&br2x_kernel);
  const hipError_t e = hipLaunchCooperativeKernel(kern, dim3(y ? (unsigned)(w8 * rows) : (unsigned)(2 * n)),
                                                  dim3(y ? BR2Y_T : BR2L_T), y ? args_y : args, 0, st);
  if (e == hipErrorCooperativeLaunchTooLarge || e == hipErrorNotSupported || e == hipErrorInvalidConfiguration) {
    (void)hipGetLastError();  // refused: nothing was enqueued
    return OMR_OK;
  }
  if (e != hipSuccess) return set_error(OMR_ERR_DEVICE, std::string("br2x cooperative launch: ") + hipGetErrorString(e));
  HIP_TRY(hipMemcpyAsync(c->x_err_host, c->x_err, sizeof(int), hipMemcpyDeviceToHost, st));
  *launched = true;
  return OMR_OK;
}

// The latency path's trace over TRACE_X CUs per message (trace_x_kernel) as a cooperative launch;
// false when refused (the caller then runs trace_kernel, one workgroup per message).
omr_status launch_trace_x(omr_ctx *c, size_t n, uint64_t *io, hipStream_t st, bool *launched) {
  *launched = false;
  if (!c->coop || TRACE_X * n > 2 * (size_t)c->num_cu) return OMR_OK;
  if (n > c->t_cap) {
    omr_status s;
    if ((s = scratch_idle(c)) != OMR_OK) return s;
    dev_free(c->t_slots);
    dev_free(c->t_flags);
    c->t_cap = 0;
    HIP_TRY(hipMalloc(&c->t_slots, n * TRACE_X * 4 * N2 * sizeof(double)));
    HIP_TRY(hipMalloc(&c->t_flags, n * TRACE_X * sizeof(uint32_t)));
    c->t_cap = n;
  }
  HIP_TRY(hipMemsetAsync(c->t_flags, 0, n * TRACE_X * sizeof(uint32_t), st));
  const double *tk = c->tk;
  DeviceTables tb = c->tb;
  double *slots = c->t_slots;
  uint32_t *flags = c->t_flags;
  int *err = c->x_err;
  void *args[] = {(void *)&io, (void *)&tk, (void *)&tb, (void *)&slots, (void *)&flags, (void *)&err};
  const hipError_t e = hipLaunchCooperativeKernel(reinterpret_cast<const void *>(&trace_x_kernel),
                                                  dim3((unsigned)(TRACE_X * n)), dim3(BR2_T), args, 0, st);
  if (e == hipErrorCooperativeLaunchTooLarge || e == hipErrorNotSupported || e == hipErrorInvalidConfiguration) {
    (void)hipGetLastError();
    return OMR_OK;
  }
  if (e != hipSuccess) return set_error(OMR_ERR_DEVICE, std::string("trace_x cooperative launch: ") + hipGetErrorString(e));
  HIP_TRY(hipMemcpyAsync(c->x_err_host, c->x_err, sizeof(int), hipMemcpyDeviceToHost, st));
  *launched = true;
  return OMR_OK;
}

// Level-2 blind rotation (+ trace, mode 0) of n LWE(670, 4096) ciphertexts. `mid` (optional) is
// recorded between the rotation and the trace; with split_trace (timing mode 2) the throughput
// path runs them as two launches so that the event separates them.
omr_status launch_br2(omr_ctx *c, size_t n, const uint32_t *lwe_int, uint64_t *out, int mode,
                      hipStream_t st, bool split_trace = false, hipEvent_t mid = nullptr) {
  if (latency_path(c, n)) {  // two CUs (or two 4-wave groups) per message, then the trace in place
    bool two_cu = false;
    omr_status s;
    if ((s = launch_br2x(c, n, lwe_int, out, st, &two_cu)) != OMR_OK) return s;
    if (!two_cu) br2l_kernel<<<(unsigned)n, BR2L_T, 0, st>>>(lwe_int, c->bsk2, c->tb, out);
    split_trace = true;
  } else {
    // br2f_kernel (the rotation, coefficient domain), then the trace as its own launch: on the FFT
    // (trace_fft_kernel) when its a priori bound allows, else the NTT (trace_kernel). The exactness
    // contract: a guarded pair notes both kernels' rounding margins in level 2's word, and a launch
    // pair whose margin reaches the threshold is re-run on the exact NTT (br2l_fallback_kernel and
    // trace_fallback_kernel: every workgroup leaves at once otherwise).
    const bool g = guarded(c, 1);
    omr_status s;
    if (g && (s = guard_begin(c, 1, st)) != OMR_OK) return s;
    if (g)
      br2f_guard_kernel<<<(unsigned)n, Fft1024::T, 0, st>>>(lwe_int, c->bsk2f, c->fft2, c->tb, out, c->margin + 3);
    else
      br2f_kernel<<<(unsigned)n, Fft1024::T, 0, st>>>(lwe_int, c->bsk2f, c->fft2, c->tb, out);
    HIP_TRY(hipGetLastError());
    if (mid) HIP_TRY(hipEventRecord(mid, st));
    if (mode == 0) {
      if (!c->trace_fft)
        trace_kernel<<<(unsigned)n, BR2_T, 0, st>>>(out, c->tk, c->tb);
      else if (g)
        trace_fft_guard_kernel<<<(unsigned)n, Fft1024::T, 0, st>>>(out, c->tkf, c->fft2, c->tb, c->margin + 3);
      else
        trace_fft_kernel<<<(unsigned)n, Fft1024::T, 0, st>>>(out, c->tkf, c->fft2, c->tb);
      HIP_TRY(hipGetLastError());
    }
    if (g) {
      br2l_fallback_kernel<<<(unsigned)n, BR2L_T, 0, st>>>(lwe_int, c->bsk2, c->tb, out, c->margin + 3, c->thr[1]);
      HIP_TRY(hipGetLastError());
      if (mode == 0)
        trace_fallback_kernel<<<(unsigned)n, BR2_T, 0, st>>>(out, c->tk, c->tb, c->margin + 3, c->thr[1]);
      HIP_TRY(hipGetLastError());
      if ((s = guard_end(c, 1, st)) != OMR_OK) return s;
    }
    return OMR_OK;
  }
  HIP_TRY(hipGetLastError());
  if (mid) HIP_TRY(hipEventRecord(mid, st));
  if (split_trace && mode == 0) {
    bool multi = false;
#ifndef OMR_NO_TRACE_X
    if (latency_path(c, n)) {
      omr_status s;
      if ((s = launch_trace_x(c, n, out, st, &multi)) != OMR_OK) return s;
    }
#endif
    if (!multi) trace_kernel<<<(unsigned)n, BR2_T, 0, st>>>(out, c->tk, c->tb);
    HIP_TRY(hipGetLastError());
  }
  return OMR_OK;
}

}  // namespace

// Scale the even (alpha) rows of the trace key by N^-1 in place.
__global__ void scale_even_rows_kernel(double *rows, size_t npoly, double s) {
  using M = Mod<2>;
  const size_t poly = (size_t)blockIdx.x * 2;
  if (poly >= npoly) return;
  double *p = rows + poly * N2;
  for (int j = threadIdx.x; j < N2; j += blockDim.x) p[j] = canon<M>(mm<M>(p[j], s));
}

extern "C" omr_status omr_ctx_create(const omr_detection_key_view *key, int device, omr_ctx **out) {
  if (!key || !out || !key->bsk1 || !key->ksk || !key->bsk2 || !key->trace_key)
    return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_ctx_create: NULL key component");
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev)
    return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_ctx_create: no such device");
  HIP_TRY(hipSetDevice(device));
  auto *c = new omr_ctx();
  c->device = device;
  HIP_TRY(hipDeviceGetAttribute(&c->num_cu, hipDeviceAttributeMultiprocessorCount, device));
  {
    int coop = 0;
    HIP_TRY(hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, device));
    // OMR_COOPERATIVE=0: never use the cooperative multi-CU latency kernels (br2l_kernel and
    // trace_kernel run instead, bit-identical); see DESIGN.md §5a on the exit-time fault of
    // processes that made cooperative launches under rocprofv3
    const char *env = getenv("OMR_COOPERATIVE");
    c->coop = coop != 0 && !(env && env[0] == '0');
    const char *ey = getenv("OMR_BR2Y");
    c->br2y = !(ey && ey[0] == '0');
    const char *ep = getenv("OMR_PREFETCH");
    c->no_prefetch = ep && ep[0] == '0';
    const char *eh = getenv("OMR_FAST_HANDOFF");
    c->no_fast_handoff = eh && eh[0] == '0';
  }
  auto fail = [&](omr_status st) {
    omr_ctx_destroy(c);
    return st;
  };
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->scratch_free, hipEventDisableTiming) != hipSuccess)
    return fail(set_error(OMR_ERR_DEVICE, "hipStreamCreate / hipEventCreate failed"));
  // the context's error word (a two-CU hand-off timeout) and its pinned copy
  if (hipMalloc(&c->x_err, sizeof(int)) != hipSuccess || hipMemset(c->x_err, 0, sizeof(int)) != hipSuccess ||
      hipHostMalloc((void **)&c->x_err_host, sizeof(int), hipHostMallocDefault) != hipSuccess)
    return fail(set_error(OMR_ERR_OUT_OF_MEMORY, "omr_ctx_create: error word"));
  *c->x_err_host = 0;
  // tables
  std::vector<double> tw1, itw1, tw2, itw2;
  twiddles(Q1, N1, 7, tw1, itw1);
  twiddles(Q2, N2, 22, tw2, itw2);
  const uint64_t one1 = ((Q1 >> 4) + 1) >> 1;  // detector.rs:457-476
  auto lut1 = negacyclic_lut({one1, 0, 0, 0, Q1 - one1}, N1, 3, Q1);
  std::vector<uint64_t> v2(TI, 0);
  v2[2 * CLUES] = (2 * Q2 + P) / (2 * P);  // round_half_up(q2/257), detector.rs:479-503
  auto lut2 = negacyclic_lut(v2, N2, 5, Q2);
  std::vector<double> tw2c(tw2);  // CmuxNtt: stage-9/10 twiddles at their lane-contiguous positions
  for (int st = 9; st <= 10; ++st)
    for (int t = 0; t < CmuxNtt::T; ++t)
      for (int e = 0; e < CmuxNtt::E; ++e)
        if (!(e & (st == 9 ? 4 : 2)))
          tw2c[(1 << st) + cmux_tw_off(3, st, t, e)] = tw2[(1 << st) + (cmux_idx(3, t, e) >> (11 - st))];
  std::vector<double> tabs;
  for (auto *v : {&tw1, &itw1, &tw2, &itw2, &lut1, &lut2, &tw2c}) tabs.insert(tabs.end(), v->begin(), v->end());
  std::vector<uint16_t> ttab(2 * TRACE_STEPS * N2);
  for (int k = 0; k < TRACE_STEPS; ++k) {
    const uint32_t g = (uint32_t)(N2 >> k) + 1;
    for (int i = 0; i < N2; ++i) {  // sigma_g: coefficient i -> position i*g mod 2N
      const uint32_t e = (uint32_t)(((uint64_t)i * g) % (2 * N2));
      if (e < (uint32_t)N2) ttab[k * N2 + e] = (uint16_t)i;
      else ttab[k * N2 + (e - N2)] = (uint16_t)(i + N2);
    }
    for (int t = 0; t < N2; ++t) {  // NTT domain: value at t comes from t' with eps(t') = g*eps(t)
      const uint32_t eps = 2 * h_brv((uint32_t)t, 11) + 1;
      const uint32_t e2 = (uint32_t)(((uint64_t)eps * g) % (2 * N2));
      ttab[(TRACE_STEPS + k) * N2 + t] = (uint16_t)h_brv((e2 - 1) / 2, 11);
    }
  }
  if (hipMalloc(&c->tables, tabs.size() * sizeof(double)) != hipSuccess ||
      hipMalloc(&c->trace_tabs, ttab.size() * sizeof(uint16_t)) != hipSuccess)
    return fail(set_error(OMR_ERR_OUT_OF_MEMORY, "omr_ctx_create: tables"));
  if (hipMemcpy(c->tables, tabs.data(), tabs.size() * sizeof(double), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(c->trace_tabs, ttab.data(), ttab.size() * sizeof(uint16_t), hipMemcpyHostToDevice) != hipSuccess)
    return fail(set_error(OMR_ERR_DEVICE, "omr_ctx_create: table upload"));
  c->tb.tw1 = c->tables;
  c->tb.itw1 = c->tables + N1;
  c->tb.tw2 = c->tables + 2 * N1;
  c->tb.itw2 = c->tables + 2 * N1 + N2;
  c->tb.lut1 = c->tables + 2 * N1 + 2 * N2;
  c->tb.lut2 = c->tables + 3 * N1 + 2 * N2;
  c->tb.tw2c = c->tables + 3 * N1 + 3 * N2;
  c->tb.trace_src = c->trace_tabs;
  c->tb.trace_perm = c->trace_tabs + TRACE_STEPS * N2;
  const auto ftw = fft_twiddles();
  if (hipMalloc(&c->fft1, ftw.size() * sizeof(double2)) != hipSuccess)
    return fail(set_error(OMR_ERR_OUT_OF_MEMORY, "omr_ctx_create: tables"));
  if (hipMemcpy(c->fft1, ftw.data(), ftw.size() * sizeof(double2), hipMemcpyHostToDevice) != hipSuccess)
    return fail(set_error(OMR_ERR_DEVICE, "omr_ctx_create: table upload"));
  c->tb.fft1 = c->fft1;
  const auto ftw2 = fft2_twiddles();
  if (hipMalloc(&c->fft2, ftw2.size() * sizeof(double2)) != hipSuccess)
    return fail(set_error(OMR_ERR_OUT_OF_MEMORY, "omr_ctx_create: tables"));
  if (hipMemcpy(c->fft2, ftw2.data(), ftw2.size() * sizeof(double2), hipMemcpyHostToDevice) != hipSuccess)
    return fail(set_error(OMR_ERR_DEVICE, "omr_ctx_create: table upload"));

  // keys
  if (hipMalloc(&c->bsk1f, BSK1_ELEMS / 2 * sizeof(double2)) != hipSuccess ||
      hipMalloc(&c->bsk1l, BSK1_ELEMS / 2 * sizeof(double2)) != hipSuccess ||
      hipMalloc(&c->bsk2, BSK2_ELEMS * sizeof(double)) != hipSuccess ||
      hipMalloc(&c->bsk2f, BSK2_ELEMS * sizeof(double2)) != hipSuccess ||
      hipMalloc(&c->tk, TK_ELEMS * sizeof(double)) != hipSuccess ||
      hipMalloc(&c->tkf, TK_ELEMS * sizeof(double2)) != hipSuccess ||
      hipMalloc(&c->kskb, KSKB_WORDS * sizeof(uint32_t)) != hipSuccess)
    return fail(set_error(OMR_ERR_OUT_OF_MEMORY, "omr_ctx_create: key buffers"));
  const double ninv2 = centred(h_powmod(N2, Q2 - 2, Q2), Q2);
  omr_status st;
  if ((st = convert_keys_dd<1>(key->bsk1, BSK1_ELEMS / N1, c->bsk1f, c->stream)) != OMR_OK) return fail(st);
  bsk1_latency_layout_kernel<<<(unsigned)(BSK1_ELEMS / 2 / 256), 256, 0, c->stream>>>(c->bsk1f, c->bsk1l,
                                                                                     BSK1_ELEMS / 2);
  if (hipGetLastError() != hipSuccess) return fail(set_error(OMR_ERR_DEVICE, "omr_ctx_create: BSK1 layout"));
  c->bsk1_host.resize(BSK1_ELEMS);  // for ensure_bsk1n (the view may point to host or device memory)
  if (hipMemcpy(c->bsk1_host.data(), key->bsk1, BSK1_ELEMS * sizeof(uint32_t), hipMemcpyDefault) != hipSuccess)
    return fail(set_error(OMR_ERR_DEVICE, "omr_ctx_create: BSK1 copy"));
  if ((st = convert_keys_cmux(key->bsk2, BSK2_ELEMS / N2, c->bsk2, ninv2, c->tb.tw2c, c->stream)) != OMR_OK)
    return fail(st);
  if ((st = convert_keys_dd<2>(key->bsk2, BSK2_ELEMS / N2, c->bsk2f, c->stream)) != OMR_OK) return fail(st);
  if ((st = convert_keys_dd<2>(key->trace_key, TK_ELEMS / N2, c->tkf, c->stream)) != OMR_OK) return fail(st);
  {  // kappa_r per key row (the a priori bound's key constants) and the guard's margin words
    const size_t rows1 = BSK1_ELEMS / 2 / Fft512::N, rows2 = BSK2_ELEMS / Fft1024::n, rowst = TK_ELEMS / Fft1024::n;
    DevBufHost<double> km;
    if (hipMalloc(&c->margin, GUARD_WORDS * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc(&km.p, (rows1 + rows2 + rowst) * sizeof(double)) != hipSuccess)
      return fail(set_error(OMR_ERR_OUT_OF_MEMORY, "omr_ctx_create: margin words"));
    const bool ok = hipMemsetAsync(c->margin, 0, GUARD_WORDS * sizeof(unsigned long long), c->stream) == hipSuccess;
    if (ok) {
      row_max_abs_kernel<<<(unsigned)rows1, 256, 0, c->stream>>>(c->bsk1f, Fft512::N, km.p);
      row_max_abs_kernel<<<(unsigned)rows2, 256, 0, c->stream>>>(c->bsk2f, Fft1024::n, km.p + rows1);
      row_max_abs_kernel<<<(unsigned)rowst, 256, 0, c->stream>>>(c->tkf, Fft1024::n, km.p + rows1 + rows2);
    }
    std::vector<double> k1(rows1), k2(rows2), kt(rowst);
    if (!ok || hipGetLastError() != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess ||
        hipMemcpy(k1.data(), km.p, rows1 * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(k2.data(), km.p + rows1, rows2 * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(kt.data(), km.p + rows1 + rows2, rowst * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess)
      return fail(set_error(OMR_ERR_DEVICE, "omr_ctx_create: key spectrum maxima"));
    c->kappa[0] = *std::max_element(k1.begin(), k1.end());
    c->kappa[1] = *std::max_element(k2.begin(), k2.end());
    c->apriori[0] = apriori_bound(1, k1);
    c->apriori[1] = apriori_bound(2, k2);
    c->apriori_y = apriori_bound(3, k2);
    c->apriori_t = apriori_bound(4, kt);
    c->trace_fft = c->apriori_t < 0.5;
    // the exactness contract: a level whose bound does not prove every rounding exact is guarded
    // on every launch and checked against 1 - E (omr_ctx_exactness)
    for (int l = 0; l < 2; ++l) {
      c->guard_auto[l] = !(c->apriori[l] < 0.5);
      c->thr[l] = 1.0 - c->apriori[l];
    }
    // the fused FFT trace shares level 2's guard word and threshold
    if (c->trace_fft) c->thr[1] = 1.0 - std::max(c->apriori[1], c->apriori_t);
  }
  if (c->guard_auto[0] && (st = ensure_bsk1n(c)) != OMR_OK) return fail(st);
  if ((st = convert_keys<2, uint64_t, double>(key->trace_key, TK_ELEMS / N2, c->tk, 1.0, c->tb.tw2,
                                              c->stream)) != OMR_OK)
    return fail(st);
  scale_even_rows_kernel<<<(TK_ELEMS / N2 + 1) / 2, 256, 0, c->stream>>>(c->tk, TK_ELEMS / N2, ninv2);
  {  // the KSK goes to the device once, as the int8 limbs of the matrix-core key switch (88 MB)
    uint32_t *ksk = nullptr;
    const bool ok = hipMalloc(&ksk, (KSK_ELEMS + 64) * sizeof(uint32_t)) == hipSuccess &&
                    hipMemcpyAsync(ksk, key->ksk, KSK_ELEMS * sizeof(uint32_t), hipMemcpyDefault, c->stream) == hipSuccess &&
                    hipMemsetAsync(ksk + KSK_ELEMS, 0, 64 * sizeof(uint32_t), c->stream) == hipSuccess;
    if (ok) ksk_to_i8_kernel<<<(unsigned)((KSKB_WORDS + 255) / 256), 256, 0, c->stream>>>(ksk, c->kskb);
    const bool done = ok && hipGetLastError() == hipSuccess && hipStreamSynchronize(c->stream) == hipSuccess;
    dev_free(ksk);
    if (!done) return fail(set_error(OMR_ERR_DEVICE, "omr_ctx_create: KSK upload"));
  }
  if ((st = ensure_batch(c, c->batch)) != OMR_OK) return fail(st);
  *out = c;
  return OMR_OK;
}

extern "C" void omr_ctx_destroy(omr_ctx *c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->scratch_stream) (void)hipEventSynchronize(c->scratch_free);
  dev_free(c->bsk1f);
  dev_free(c->bsk1l);
  dev_free(c->bsk1n);
  dev_free(c->fft1);
  dev_free(c->bsk2);
  dev_free(c->bsk2f);
  dev_free(c->tkf);
  dev_free(c->fft2);
  dev_free(c->tk);
  dev_free(c->kskb);
  dev_free(c->tables);
  dev_free(c->trace_tabs);
  dev_free(c->ext);
  dev_free(c->lwe1t);
  dev_free(c->lwe_int);
  dev_free(c->s_clue_a);
  dev_free(c->s_clue_b);
  dev_free(c->s_out);
  dev_free(c->partial);
  dev_free(c->ks_part);
  dev_free(c->x_slots);
  dev_free(c->x_flags);
  dev_free(c->t_slots);
  dev_free(c->t_flags);
  dev_free(c->margin);
  dev_free(c->x_err);
  if (c->x_err_host) (void)hipHostFree(c->x_err_host);
  for (auto e : c->events) (void)hipEventDestroy(e);
  if (c->scratch_free) (void)hipEventDestroy(c->scratch_free);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

// Names of the detect-path kernels this build launches (bench.py / profile summaries).
extern "C" const char *omr_detect_kernels(void) {
  return "br1=" OMR_BR1_NAME " ks=" OMR_KS_NAME " br2=" OMR_BR2_NAME;
}

extern "C" omr_status omr_ctx_set_batch(omr_ctx *c, size_t batch) {
  if (!c) return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_ctx_set_batch: NULL ctx");
  std::lock_guard<std::mutex> lk(c->mu);
  c->batch = batch ? batch : OMR_DEFAULT_BATCH;
  HIP_TRY(hipSetDevice(c->device));
  return ensure_batch(c, c->batch);
}

extern "C" omr_status omr_ctx_set_encode_chunks(omr_ctx *c, size_t max_chunks) {
  if (!c) return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_ctx_set_encode_chunks: NULL ctx");
  std::lock_guard<std::mutex> lk(c->mu);
  c->enc_max_chunks = max_chunks ? max_chunks : OMR_ENC_MAX_CHUNKS;
  return OMR_OK;
}

extern "C" omr_status omr_ctx_set_latency_threshold(omr_ctx *c, size_t max_messages) {
  if (!c) return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_ctx_set_latency_threshold: NULL ctx");
  std::lock_guard<std::mutex> lk(c->mu);
  c->latency_max = max_messages;
  return OMR_OK;
}

extern "C" omr_status omr_ctx_enable_timing(omr_ctx *c, int mode) {
  if (!c || mode < 0 || mode > 2) return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_ctx_enable_timing: bad argument");
  std::lock_guard<std::mutex> lk(c->mu);
  c->timing = mode;
  return OMR_OK;
}

extern "C" omr_status omr_ctx_set_rounding_guard(omr_ctx *c, int enable) {
  if (!c) return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_ctx_set_rounding_guard: NULL ctx");
  std::lock_guard<std::mutex> lk(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  omr_status s;
  if (enable && (s = ensure_bsk1n(c)) != OMR_OK) return s;  // a guarded level-1 launch may re-run exactly
  c->guard = enable != 0;
  return OMR_OK;
}

extern "C" omr_status omr_ctx_set_exact_level1(omr_ctx *c, int enable) {
  if (!c) return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_ctx_set_exact_level1: NULL ctx");
  std::lock_guard<std::mutex> lk(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  omr_status s;
  if (enable && (s = ensure_bsk1n(c)) != OMR_OK) return s;
  c->exact1 = enable != 0;
  return OMR_OK;
}

extern "C" omr_status omr_ctx_rounding_margin(omr_ctx *c, double observed[2], double apriori[2], double kappa[2],
                                              int reset) {
  if (!c) return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_ctx_rounding_margin: NULL ctx");
  std::lock_guard<std::mutex> lk(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipDeviceSynchronize());  // every guarded launch on any stream has published
  unsigned long long w[2];
  HIP_TRY(hipMemcpy(w, c->margin, sizeof(w), hipMemcpyDeviceToHost));
  for (int l = 0; l < 2; ++l) {
    if (observed) observed[l] = __builtin_bit_cast(double, w[l]);
    if (apriori) apriori[l] = c->apriori[l];
    if (kappa) kappa[l] = c->kappa[l];
  }
  if (reset) HIP_TRY(hipMemset(c->margin, 0, 2 * sizeof(unsigned long long)));
  return OMR_OK;
}

extern "C" omr_status omr_ctx_exactness(omr_ctx *c, int guarded_out[2], uint64_t breaches[2]) {
  if (!c) return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_ctx_exactness: NULL ctx");
  std::lock_guard<std::mutex> lk(c->mu);
  if (guarded_out)
    for (int l = 0; l < 2; ++l) guarded_out[l] = guarded(c, l) ? 1 : 0;
  if (breaches) {
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipDeviceSynchronize());
    unsigned long long w[2];
    HIP_TRY(hipMemcpy(w, c->margin + 4, sizeof(w), hipMemcpyDeviceToHost));
    breaches[0] = w[0];
    breaches[1] = w[1];
  }
  return OMR_OK;
}

extern "C" omr_status omr_fft_twiddles_dd(int level, double *out) {
  if ((level != 1 && level != 2) || !out) return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_fft_twiddles_dd: bad argument");
  const auto tw = dd_tree_twiddles(level == 1 ? 9 : 10);
  for (size_t i = 0; i < tw.size(); ++i) {
    out[4 * i] = tw[i].re.hi;
    out[4 * i + 1] = tw[i].re.lo;
    out[4 * i + 2] = tw[i].im.hi;
    out[4 * i + 3] = tw[i].im.lo;
  }
  return OMR_OK;
}

extern "C" omr_status omr_ctx_key_spectrum(omr_ctx *c, int level, size_t first, size_t count, double *out) {
  const size_t total = level == 1 ? BSK1_ELEMS / 2 : BSK2_ELEMS;  // double2 values
  if (!c || !out || (level != 1 && level != 2) || first > total || count > total - first)
    return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_ctx_key_spectrum: bad argument");
  std::lock_guard<std::mutex> lk(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipMemcpy(out, (level == 1 ? c->bsk1f : c->bsk2f) + first, count * sizeof(double2), hipMemcpyDeviceToHost));
  return OMR_OK;
}

extern "C" omr_status omr_ctx_check(omr_ctx *c, void *stream) {
  if (!c) return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_ctx_check: NULL ctx");
  std::lock_guard<std::mutex> lk(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  if (stream) {
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  } else {  // the null stream and the context's own (non-blocking) stream
    HIP_TRY(hipDeviceSynchronize());
  }
  return take_handoff_error(c);
}

namespace {

constexpr int EV_PER_CHUNK = 5;

// Detect D messages of device buffers on st, in chunks of c->batch: per chunk br1f (7 rotations
// per message) -> sum7 -> key switch -> br2 + trace. Stage events per chunk: [0] br1 start,
// [1] br1 end, [2] key switch end, [3] level-2 rotation end, [4] trace end (the trace is its own
// launch on both kernel families since round 5: trace_fft_kernel / trace_x_kernel).
omr_status detect_device(omr_ctx *c, const uint16_t *ca, const uint16_t *cb, size_t D,
                         uint64_t *out, hipStream_t st) {
  omr_status s;
  if ((s = take_handoff_error(c)) != OMR_OK) return s;  // an earlier call's output is invalid
  if ((s = ensure_batch(c, std::min(D, c->batch))) != OMR_OK) return s;
  const size_t nchunks = (D + c->batch - 1) / c->batch;
  const bool split = c->timing == 2;
  if (c->timing) {
    while (c->events.size() < nchunks * EV_PER_CHUNK) {
      hipEvent_t e;
      HIP_TRY(hipEventCreate(&e));
      c->events.push_back(e);
    }
    c->timed_messages = D;
    c->timed_chunks = nchunks;
    c->timed_split = true;
  }
  if ((s = scratch_acquire(c, st)) != OMR_OK) return s;
  for (size_t ch = 0; ch < nchunks; ++ch) {
    const size_t off = ch * c->batch;
    const int B = (int)std::min(c->batch, D - off);
    hipEvent_t *ev = c->timing ? &c->events[ch * EV_PER_CHUNK] : nullptr;
    if (ev) HIP_TRY(hipEventRecord(ev[0], st));
    if ((s = launch_br1(c, (size_t)B * CLUES, ca + off * N0, cb + off * CLUES, nullptr, nullptr,
                        c->ext, nullptr, 0, st, (size_t)B)) != OMR_OK)
      return s;
    if (ev) HIP_TRY(hipEventRecord(ev[1], st));
    const size_t n7 = (size_t)B * (N1 + 1);
    sum7_kernel<<<(unsigned)((n7 + 255) / 256), 256, 0, st>>>(c->ext, c->lwe1t, B);
    if ((s = launch_ks(c, B, c->lwe_int, st)) != OMR_OK) return s;
    if (ev) HIP_TRY(hipEventRecord(ev[2], st));
    if ((s = launch_br2(c, (size_t)B, c->lwe_int, out + off * 2 * N2, 0, st, split, ev ? ev[3] : nullptr)) != OMR_OK)
      return s;
    if (ev) HIP_TRY(hipEventRecord(ev[4], st));
  }
  return scratch_release(c, st);
}

omr_status stage_buffers(omr_ctx *c, size_t B) {
  if (B <= c->staged) return OMR_OK;
  dev_free(c->s_clue_a);
  dev_free(c->s_clue_b);
  dev_free(c->s_out);
  c->staged = 0;
  HIP_TRY(hipMalloc(&c->s_clue_a, B * N0 * sizeof(uint16_t)));
  HIP_TRY(hipMalloc(&c->s_clue_b, B * CLUES * sizeof(uint16_t)));
  HIP_TRY(hipMalloc(&c->s_out, B * 2 * N2 * sizeof(uint64_t)));
  c->staged = B;
  return OMR_OK;
}

}  // namespace

extern "C" omr_status omr_detect_batch_device(omr_ctx *c, const uint16_t *ca, const uint16_t *cb,
                                              size_t D, uint64_t *out, void *stream) {
  if (!c || (D && (!ca || !cb || !out)))
    return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_detect_batch_device: NULL argument");
  if (D == 0) return OMR_OK;
  std::lock_guard<std::mutex> lk(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  c->host_timing_valid = false;
  return detect_device(c, ca, cb, D, out, (hipStream_t)stream);  // NULL: HIP's null stream
}

namespace {
omr_status collect_timing(omr_ctx *c, omr_detect_timing *t);
}

namespace {
// omr_detect_batch with c->mu held.
omr_status detect_host_locked(omr_ctx *c, const uint16_t *ca, const uint16_t *cb, size_t D, uint64_t *out) {
  HIP_TRY(hipSetDevice(c->device));
  omr_status s;
  const size_t B = std::min(D, c->batch);
  if ((s = stage_buffers(c, B)) != OMR_OK) return s;
  omr_detect_timing acc{};
  acc.trace_separate = 1;
  c->host_timing_valid = false;
  for (size_t off = 0; off < D; off += B) {
    const size_t n = std::min(B, D - off);
    HIP_TRY(hipMemcpyAsync(c->s_clue_a, ca + off * N0, n * N0 * sizeof(uint16_t), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->s_clue_b, cb + off * CLUES, n * CLUES * sizeof(uint16_t), hipMemcpyHostToDevice, c->stream));
    if ((s = detect_device(c, c->s_clue_a, c->s_clue_b, n, c->s_out, c->stream)) != OMR_OK) return s;
    HIP_TRY(hipMemcpyAsync(out + off * 2 * N2, c->s_out, n * 2 * N2 * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if ((s = take_handoff_error(c)) != OMR_OK) return s;
    if (c->timing) {
      omr_detect_timing t;
      if ((s = collect_timing(c, &t)) != OMR_OK) return s;
      acc.first_level_ms += t.first_level_ms;
      acc.key_switch_ms += t.key_switch_ms;
      acc.second_level_ms += t.second_level_ms;
      acc.trace_ms += t.trace_ms;
      acc.total_ms += t.total_ms;
      acc.messages += t.messages;
      acc.trace_separate &= t.trace_separate;
    }
  }
  if (c->timing) {
    c->host_timing = acc;
    c->host_timing_valid = true;
  }
  return OMR_OK;
}
}  // namespace

extern "C" omr_status omr_detect_batch(omr_ctx *c, const uint16_t *ca, const uint16_t *cb, size_t D,
                                       uint64_t *out) {
  if (!c || (D && (!ca || !cb || !out)))
    return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_detect_batch: NULL argument");
  if (D == 0) return OMR_OK;
  std::lock_guard<std::mutex> lk(c->mu);
  return detect_host_locked(c, ca, cb, D, out);
}

// Detector::detect (detector.rs:135-138) for one message, callable from many host threads at once
// (the reference's `clues.par_iter().map(|c| detector.detect(c))`, examples/omr.rs:160-164, on a
// shared &Detector): the requests queue on the context; whichever caller finds no launch in
// progress becomes the leader, optionally waits coalesce_window_us for more, gathers up to
// coalesce_max queued clues into one omr_detect_batch (latency kernels up to the threshold,
// throughput kernels above), scatters the outputs and wakes their callers; the next leader takes
// what queued meanwhile. Every caller gets its batch's status and error message.
extern "C" omr_status omr_detect(omr_ctx *c, const uint16_t *ca, const uint16_t *cb, uint64_t *out) {
  if (!c || !ca || !cb || !out) return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_detect: NULL argument");
  omr_ctx::DetectReq r{ca, cb, out, OMR_OK, std::string(), false};
  std::unique_lock<std::mutex> lk(c->qmu);
  c->queue.push_back(&r);
  c->qcv.notify_all();  // a leader inside its window may be waiting for a full batch
  while (!r.done) {
    if (c->leader) {
      c->qcv.wait(lk);
      continue;
    }
    c->leader = true;
    if (c->coalesce_window_us > 0 && c->queue.size() < c->coalesce_max)
      c->qcv.wait_for(lk, std::chrono::microseconds(c->coalesce_window_us),
                      [&] { return c->queue.size() >= c->coalesce_max; });
    const size_t n = std::min(c->queue.size(), c->coalesce_max);
    std::vector<omr_ctx::DetectReq *> batch(c->queue.begin(), c->queue.begin() + (long)n);
    c->queue.erase(c->queue.begin(), c->queue.begin() + (long)n);
    lk.unlock();
    // gather, launch, scatter: nothing may throw out of this extern "C" function, and the leader
    // flag must be cleared whatever happens (a staging allocation of up to coalesce_max messages
    // can fail): a failure becomes the batch's status
    omr_status st;
    std::string err;
    try {
      std::vector<uint16_t> ga(n * N0), gb(n * CLUES);
      std::vector<uint64_t> go(n * 2 * N2);
      for (size_t k = 0; k < n; ++k) {
        memcpy(&ga[k * N0], batch[k]->a, N0 * sizeof(uint16_t));
        memcpy(&gb[k * CLUES], batch[k]->b, CLUES * sizeof(uint16_t));
      }
      {
        std::lock_guard<std::mutex> dl(c->mu);
        st = detect_host_locked(c, ga.data(), gb.data(), n, go.data());
      }
      if (st == OMR_OK)
        for (size_t k = 0; k < n; ++k) memcpy(batch[k]->out, &go[k * 2 * N2], 2 * N2 * sizeof(uint64_t));
      else
        err = omr_last_error();
    } catch (const std::bad_alloc &) {
      st = OMR_ERR_OUT_OF_MEMORY;
      err = "omr_detect: host staging of the coalesced batch failed";
    } catch (...) {
      st = OMR_ERR_DEVICE;
      err = "omr_detect: unexpected failure while running the coalesced batch";
    }
    lk.lock();
    for (auto *q : batch) {
      q->st = st;
      q->err = err;
      q->done = true;
    }
    c->coalesced_calls += n;
    c->coalesced_launches += 1;
    c->leader = false;
    c->qcv.notify_all();
  }
  return r.st == OMR_OK ? OMR_OK : set_error(r.st, r.err);
}

extern "C" omr_status omr_ctx_set_coalescing(omr_ctx *c, size_t max_messages, long window_us) {
  if (!c || window_us < 0) return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_ctx_set_coalescing: bad argument");
  std::lock_guard<std::mutex> lk(c->qmu);
  c->coalesce_max = max_messages ? max_messages : 65536;
  c->coalesce_window_us = window_us;
  return OMR_OK;
}

extern "C" omr_status omr_ctx_coalescing_stats(omr_ctx *c, size_t *calls, size_t *launches) {
  if (!c) return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_ctx_coalescing_stats: NULL ctx");
  std::lock_guard<std::mutex> lk(c->qmu);
  if (calls) *calls = c->coalesced_calls;
  if (launches) *launches = c->coalesced_launches;
  return OMR_OK;
}

namespace {
// Stage times of the last detect_device call from its per-chunk events (DetectTimeInfo's split:
// first level includes the key switch, detector.rs:183-191).
omr_status collect_timing(omr_ctx *c, omr_detect_timing *t) {
  memset(t, 0, sizeof(*t));
  if (!c->timing || c->timed_messages == 0) return OMR_OK;
  for (size_t ch = 0; ch < c->timed_chunks; ++ch) {  // the chunk count of the timed call
    hipEvent_t *ev = &c->events[ch * EV_PER_CHUNK];
    HIP_TRY(hipEventSynchronize(ev[4]));
    float a = 0, b = 0, d = 0, e = 0;
    HIP_TRY(hipEventElapsedTime(&a, ev[0], ev[1]));
    HIP_TRY(hipEventElapsedTime(&b, ev[1], ev[2]));
    HIP_TRY(hipEventElapsedTime(&d, ev[2], ev[3]));
    HIP_TRY(hipEventElapsedTime(&e, ev[3], ev[4]));
    t->first_level_ms += a + b;
    t->key_switch_ms += b;
    t->second_level_ms += d;
    t->trace_ms += e;
  }
  t->total_ms = t->first_level_ms + t->second_level_ms + t->trace_ms;
  t->messages = c->timed_messages;
  t->trace_separate = c->timed_split ? 1 : 0;
  return OMR_OK;
}
}  // namespace

extern "C" omr_status omr_last_timing(omr_ctx *c, omr_detect_timing *t) {
  if (!c || !t) return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_last_timing: NULL argument");
  std::lock_guard<std::mutex> lk(c->mu);
  if (c->host_timing_valid) {
    *t = c->host_timing;
    return OMR_OK;
  }
  HIP_TRY(hipSetDevice(c->device));
  return collect_timing(c, t);
}

extern "C" omr_status omr_detect_with_time_info(omr_ctx *c, const uint16_t *ca, const uint16_t *cb, size_t D,
                                                uint64_t *out, omr_detect_timing *t) {
  if (!c || !t || (D && (!ca || !cb || !out)))
    return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_detect_with_time_info: NULL argument");
  memset(t, 0, sizeof(*t));
  t->trace_separate = 1;
  if (D == 0) return OMR_OK;
  std::lock_guard<std::mutex> lk(c->mu);
  const int mode = c->timing;
  c->timing = 2;
  omr_status s = detect_host_locked(c, ca, cb, D, out);
  if (s == OMR_OK) *t = c->host_timing;
  c->timing = mode;
  c->host_timing_valid = mode != 0 && s == OMR_OK;
  return s;
}

// ------------------------------------------------------------------------------------------
// Encode (detector.rs:223-453)
// ------------------------------------------------------------------------------------------
namespace {
// Messages per encode workgroup: at least 32 (128 from D = 16,384), and at most max_chunks
// (default 4,096) chunk partials per ciphertext (scratch n_ct x chunks x 32 KiB: 3.7 GB for 28
// ciphertexts at D = 2^20); above ENC_T messages the index kernel stages its buckets in blocks.
int encode_per_wg(size_t D, size_t max_chunks) {
  const size_t base = D >= 16384 ? 128 : 32;
  return (int)std::max(base, (D + max_chunks - 1) / max_chunks);
}
}  // namespace

extern "C" omr_status omr_encode_indices_device(omr_ctx *c, const uint64_t *pv, size_t D,
                                                size_t offset, size_t all, uint64_t seed,
                                                uint32_t first_ct, uint32_t n_ct, uint64_t *out,
                                                void *stream) {
  if (!c || !out || (D && !pv) || n_ct == 0 || offset + D > all || D > (size_t)INT32_MAX)
    return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_encode_indices_device: bad argument");
  std::lock_guard<std::mutex> lk(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;  // NULL: HIP's null stream
  omr_retrieval_params rp;
  omr_status s;
  if ((s = omr_get_retrieval_params(all, 0, &rp)) != OMR_OK) return s;
  if (D == 0) {
    HIP_TRY(hipMemsetAsync(out, 0, (size_t)n_ct * 2 * N2 * sizeof(uint64_t), st));
    return OMR_OK;
  }
  const int per_wg = encode_per_wg(D, c->enc_max_chunks);
  const int chunks = (int)((D + per_wg - 1) / per_wg);
  if ((s = ensure_partial(c, (size_t)n_ct * chunks * 2 * N2)) != OMR_OK) return s;
  if ((s = scratch_acquire(c, st)) != OMR_OK) return s;
  EncodeLayout ly{(int)rp.index_slots_per_bucket, (int)rp.slots_per_bucket,
                  (int)rp.slots_per_segment, (int)rp.segment_per_cipher};
  encode_indices_kernel<<<dim3(chunks, n_ct), ENC_T, 0, st>>>(pv, (int)D, offset, ly, seed, first_ct,
                                                              per_wg, c->tb.tw2, c->partial);
  HIP_TRY(hipGetLastError());
  const size_t tot = (size_t)n_ct * 2 * N2;
  reduce_partials_kernel<<<(unsigned)((tot + 255) / 256), 256, 0, st>>>(c->partial, chunks, (int)n_ct, out);
  HIP_TRY(hipGetLastError());
  return scratch_release(c, st);
}

extern "C" omr_status omr_encode_payloads_device(omr_ctx *c, const uint64_t *pv,
                                                 const uint16_t *payloads, size_t D, size_t offset,
                                                 size_t all, const uint16_t *weights, uint32_t n_ct,
                                                 uint32_t per_ct, uint64_t *out, void *stream) {
  if (!c || !out || (D && (!pv || !payloads || !weights)) || n_ct == 0 || per_ct == 0 ||
      per_ct * PAYLOAD_LEN > (uint32_t)N2 || offset + D > all || D > (size_t)INT32_MAX)
    return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_encode_payloads_device: bad argument");
  std::lock_guard<std::mutex> lk(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;  // NULL: HIP's null stream
  if (D == 0) {
    HIP_TRY(hipMemsetAsync(out, 0, (size_t)n_ct * 2 * N2 * sizeof(uint64_t), st));
    return OMR_OK;
  }
  const int per_wg = encode_per_wg(D, c->enc_max_chunks);
  const int chunks = (int)((D + per_wg - 1) / per_wg);
  omr_status s;
  if ((s = ensure_partial(c, (size_t)n_ct * chunks * 2 * N2)) != OMR_OK) return s;
  if ((s = scratch_acquire(c, st)) != OMR_OK) return s;
  encode_payloads_kernel<<<dim3(chunks, n_ct), ENC_T, 0, st>>>(pv, payloads, (int)D, offset, all,
                                                               weights, (int)per_ct, per_wg,
                                                               c->tb.tw2, c->partial);
  HIP_TRY(hipGetLastError());
  const size_t tot = (size_t)n_ct * 2 * N2;
  reduce_partials_kernel<<<(unsigned)((tot + 255) / 256), 256, 0, st>>>(c->partial, chunks, (int)n_ct, out);
  HIP_TRY(hipGetLastError());
  return scratch_release(c, st);
}

namespace {
template <typename T>
struct DevBuf {
  T *p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  hipError_t alloc(size_t n) { return hipMalloc(&p, n * sizeof(T)); }
};
}  // namespace

extern "C" omr_status omr_encode_indices(omr_ctx *c, const uint64_t *pv, size_t D, size_t offset,
                                         size_t all, uint64_t seed, uint32_t ct, uint64_t *out) {
  if (!c || !out || (D && !pv)) return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_encode_indices");
  HIP_TRY(hipSetDevice(c->device));
  DevBuf<uint64_t> dpv, dout;
  HIP_TRY(dpv.alloc(std::max<size_t>(D, 1) * 2 * N2));
  HIP_TRY(dout.alloc(2 * N2));
  HIP_TRY(hipMemcpy(dpv.p, pv, D * 2 * N2 * sizeof(uint64_t), hipMemcpyHostToDevice));
  omr_status s = omr_encode_indices_device(c, dpv.p, D, offset, all, seed, ct, 1, dout.p, c->stream);
  if (s != OMR_OK) return s;
  HIP_TRY(hipStreamSynchronize(c->stream));
  HIP_TRY(hipMemcpy(out, dout.p, 2 * N2 * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return OMR_OK;
}

extern "C" omr_status omr_encode_payloads(omr_ctx *c, const uint64_t *pv, const uint16_t *payloads,
                                          size_t D, size_t offset, size_t all,
                                          const uint16_t *weights, uint32_t n_ct, uint32_t per_ct,
                                          uint64_t *out) {
  if (!c || !out || (D && (!pv || !payloads || !weights)))
    return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_encode_payloads");
  HIP_TRY(hipSetDevice(c->device));
  const size_t wn = (size_t)n_ct * per_ct * all;
  DevBuf<uint64_t> dpv, dout;
  DevBuf<uint16_t> dpay, dw;
  HIP_TRY(dpv.alloc(std::max<size_t>(D, 1) * 2 * N2));
  HIP_TRY(dpay.alloc(std::max<size_t>(D, 1) * PAYLOAD_LEN));
  HIP_TRY(dw.alloc(std::max<size_t>(wn, 1)));
  HIP_TRY(dout.alloc((size_t)n_ct * 2 * N2));
  HIP_TRY(hipMemcpy(dpv.p, pv, D * 2 * N2 * sizeof(uint64_t), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(dpay.p, payloads, D * PAYLOAD_LEN * sizeof(uint16_t), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(dw.p, weights, wn * sizeof(uint16_t), hipMemcpyHostToDevice));
  omr_status s = omr_encode_payloads_device(c, dpv.p, dpay.p, D, offset, all, dw.p, n_ct, per_ct,
                                            dout.p, c->stream);
  if (s != OMR_OK) return s;
  HIP_TRY(hipStreamSynchronize(c->stream));
  HIP_TRY(hipMemcpy(out, dout.p, (size_t)n_ct * 2 * N2 * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return OMR_OK;
}

// ------------------------------------------------------------------------------------------
// Stage entry points (parity tests, per-stage benchmarks)
// ------------------------------------------------------------------------------------------
extern "C" omr_status omr_first_level(omr_ctx *c, const uint16_t *ca, const uint16_t *cb, size_t D,
                                      uint32_t *lwe_int) {
  if (!c || !ca || !cb || !lwe_int || D == 0 || D > c->batch)
    return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_first_level: bad argument (D <= batch)");
  std::lock_guard<std::mutex> lk(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  omr_status s;
  if ((s = stage_buffers(c, D)) != OMR_OK || (s = ensure_batch(c, D)) != OMR_OK) return s;
  hipStream_t st = c->stream;
  if ((s = scratch_acquire(c, st)) != OMR_OK) return s;
  HIP_TRY(hipMemcpyAsync(c->s_clue_a, ca, D * N0 * sizeof(uint16_t), hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemcpyAsync(c->s_clue_b, cb, D * CLUES * sizeof(uint16_t), hipMemcpyHostToDevice, st));
  const int B = (int)D;
  if ((s = launch_br1(c, (size_t)B * CLUES, c->s_clue_a, c->s_clue_b, nullptr, nullptr, c->ext,
                      nullptr, 0, st, (size_t)B)) != OMR_OK)
    return s;
  const size_t n7 = (size_t)B * (N1 + 1);
  sum7_kernel<<<(unsigned)((n7 + 255) / 256), 256, 0, st>>>(c->ext, c->lwe1t, B);
  {
    omr_status ks;
    if ((ks = launch_ks(c, B, c->lwe_int, st)) != OMR_OK) return ks;
  }
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(lwe_int, c->lwe_int, D * (NI + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  if ((s = scratch_release(c, st)) != OMR_OK) return s;
  HIP_TRY(hipStreamSynchronize(st));
  return OMR_OK;
}

extern "C" omr_status omr_fft1_mul(omr_ctx *c, const uint32_t *a, const uint32_t *k, size_t n,
                                   uint64_t *out) {
  if (!c || !a || !k || !out || n == 0)
    return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_fft1_mul: bad argument");
  std::lock_guard<std::mutex> lk(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  DevBuf<uint32_t> da, dk;
  DevBuf<uint64_t> dout;
  HIP_TRY(da.alloc(n * N1));
  HIP_TRY(dk.alloc(n * N1));
  HIP_TRY(dout.alloc(n * N1));
  HIP_TRY(hipMemcpy(da.p, a, n * N1 * sizeof(uint32_t), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(dk.p, k, n * N1 * sizeof(uint32_t), hipMemcpyHostToDevice));
  fft1_mul_kernel<<<(unsigned)n, 64, 0, c->stream>>>(da.p, dk.p, dout.p, c->fft1);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(c->stream));
  HIP_TRY(hipMemcpy(out, dout.p, n * N1 * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return OMR_OK;
}

extern "C" omr_status omr_blind_rotate_level1(omr_ctx *c, const uint16_t *la, const uint16_t *lb,
                                              size_t n, uint64_t *out) {
  if (!c || !la || !lb || !out || n == 0)
    return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_blind_rotate_level1: bad argument");
  std::lock_guard<std::mutex> lk(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  DevBuf<uint16_t> da, db;
  DevBuf<uint64_t> dout;
  HIP_TRY(da.alloc(n * N0));
  HIP_TRY(db.alloc(n));
  HIP_TRY(dout.alloc(n * 2 * N1));
  HIP_TRY(hipMemcpy(da.p, la, n * N0 * sizeof(uint16_t), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(db.p, lb, n * sizeof(uint16_t), hipMemcpyHostToDevice));
  // a pending hand-off error belongs to an earlier detect call: report it before this launch (as
  // detect_device does) instead of discarding a valid level-1 output after it
  omr_status s;
  if ((s = take_handoff_error(c)) != OMR_OK) return s;
  // the guarded sequence (guard_begin, guard kernel, br1n_fallback, guard_fold) uses the context's
  // per-launch margin word, shared with every other call: serialise it with them like any scratch
  if ((s = scratch_acquire(c, c->stream)) != OMR_OK) return s;
  if ((s = launch_br1(c, n, nullptr, nullptr, da.p, db.p, nullptr, dout.p, 1, c->stream, n)) != OMR_OK) return s;
  if ((s = scratch_release(c, c->stream)) != OMR_OK) return s;
  HIP_TRY(hipStreamSynchronize(c->stream));
  HIP_TRY(hipMemcpy(out, dout.p, n * 2 * N1 * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return OMR_OK;
}

static omr_status second_level_impl(omr_ctx *c, const uint32_t *lwe, size_t n, uint64_t *out,
                                    int mode) {
  if (!c || !lwe || !out || n == 0)
    return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_second_level: bad argument");
  std::lock_guard<std::mutex> lk(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  DevBuf<uint32_t> dl;
  DevBuf<uint64_t> dout;
  HIP_TRY(dl.alloc(n * (NI + 1)));
  HIP_TRY(dout.alloc(n * 2 * N2));
  HIP_TRY(hipMemcpy(dl.p, lwe, n * (NI + 1) * sizeof(uint32_t), hipMemcpyHostToDevice));
  omr_status ls;
  if ((ls = take_handoff_error(c)) != OMR_OK) return ls;
  if ((ls = scratch_acquire(c, c->stream)) != OMR_OK) return ls;  // the hand-off slots are scratch
  if ((ls = launch_br2(c, n, dl.p, dout.p, mode, c->stream)) != OMR_OK) return ls;
  if ((ls = scratch_release(c, c->stream)) != OMR_OK) return ls;
  HIP_TRY(hipStreamSynchronize(c->stream));
  if ((ls = take_handoff_error(c)) != OMR_OK) return ls;
  HIP_TRY(hipMemcpy(out, dout.p, n * 2 * N2 * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return OMR_OK;
}

extern "C" omr_status omr_second_level(omr_ctx *c, const uint32_t *lwe, size_t n, uint64_t *out) {
  return second_level_impl(c, lwe, n, out, 0);
}
extern "C" omr_status omr_blind_rotate_level2(omr_ctx *c, const uint32_t *lwe, size_t n,
                                              uint64_t *out) {
  return second_level_impl(c, lwe, n, out, 1);
}

extern "C" omr_status omr_ntt(int level, int inverse, uint64_t *polys, size_t n, int device) {
  if ((level != 1 && level != 2) || !polys || n == 0)
    return set_error(OMR_ERR_INVALID_ARGUMENT, "omr_ntt: bad argument");
  HIP_TRY(hipSetDevice(device));
  const uint64_t q = level == 1 ? Q1 : Q2;
  const int N = level == 1 ? N1 : N2;
  std::vector<double> tw, itw;
  twiddles(q, N, level == 1 ? 7 : 22, tw, itw);
  DevBuf<double> dt;
  DevBuf<uint64_t> dp;
  HIP_TRY(dt.alloc(2 * N));
  HIP_TRY(dp.alloc(n * N));
  HIP_TRY(hipMemcpy(dt.p, tw.data(), N * sizeof(double), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(dt.p + N, itw.data(), N * sizeof(double), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(dp.p, polys, n * N * sizeof(uint64_t), hipMemcpyHostToDevice));
  const double ninv = centred(h_powmod(N, q - 2, q), q);
  if (level == 1)
    ntt_u64_kernel<1><<<(unsigned)n, BR1_T>>>(dp.p, n, inverse, ninv, dt.p, dt.p + N);
  else
    ntt_u64_kernel<2><<<(unsigned)n, BR2_T>>>(dp.p, n, inverse, ninv, dt.p, dt.p + N);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(polys, dp.p, n * N * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return OMR_OK;
}

#ifdef OMR_PHASE_TRACE
// Debug builds only (tools/phase_trace.py): copy the latency kernels' phase timestamps.
extern "C" int omr_debug_phase_read(unsigned long long *host, size_t n) {
  const size_t cap = sizeof(omr::omr_phase_buf) / sizeof(unsigned long long);
  if (n > cap) n = cap;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(omr::omr_phase_buf), n * sizeof(unsigned long long)) == hipSuccess
             ? (int)n
             : -1;
}
#endif

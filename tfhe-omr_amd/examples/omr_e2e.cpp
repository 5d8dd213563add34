// omr_e2e — the reference's end-to-end example (omr_core/examples/omr.rs:30-235) driven through
// the C ABI of include/omr_gpu.h from native code: key generation, clue generation (pertinent
// messages from sender A, the rest from sender B), detect on the GPU, encode_pertinent_indices /
// encode_pertinent_payloads, client-side retrieval, and a check that exactly the pertinent
// indices and their payloads come back.
//
//   omr_e2e [-p payload_count] [-d device] [-s seed] [--host-only]
//
// --host-only runs the CPU parts of the ABI (keys, clues, weights, retrieval parameters) without
// a GPU (used by the CPU test suite).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <random>
#include <string>
#include <vector>

#include "omr_gpu.h"

namespace {

constexpr size_t N0 = 512, CLUES = 7, N2 = 2048, PAYLOAD = 612;
constexpr size_t BSK1 = 512ull * 8 * 2 * 1024, KSK = 1024ull * 27 * 671, BSK2 = 670ull * 12 * 2 * 2048,
                 TK = 11ull * 25 * 2 * 2048;

using clk = std::chrono::steady_clock;
double secs(clk::time_point a) { return std::chrono::duration<double>(clk::now() - a).count(); }

#define CHECK(expr)                                                                    \
  do {                                                                                 \
    omr_status st_ = (expr);                                                           \
    if (st_ != OMR_OK) {                                                               \
      std::fprintf(stderr, "%s failed (%d): %s\n", #expr, (int)st_, omr_last_error()); \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

}  // namespace

int main(int argc, char **argv) {
  size_t D = 4096;
  int device = 0;
  uint64_t seed = 2025;
  bool host_only = false;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if ((a == "-p" || a == "--payload-count") && i + 1 < argc) D = std::max<size_t>(1, std::stoull(argv[++i]));
    else if ((a == "-d" || a == "--device") && i + 1 < argc) device = std::atoi(argv[++i]);
    else if ((a == "-s" || a == "--seed") && i + 1 < argc) seed = std::stoull(argv[++i]);
    else if (a == "--host-only") host_only = true;
    else {
      std::fprintf(stderr, "usage: %s [-p payload_count] [-d device] [-s seed] [--host-only]\n", argv[0]);
      return 2;
    }
  }
  std::printf("%s; all payloads count: %zu\n", omr_version(), D);

  // KeyGen::generate_secret_key x2, generate_detector (omr.rs:76-83)
  auto t = clk::now();
  omr_secret_key_pack *pa = nullptr, *pb = nullptr;
  CHECK(omr_keygen_secret(seed ^ 0xA, &pa));
  CHECK(omr_keygen_secret(seed ^ 0xB, &pb));
  std::vector<uint32_t> bsk1(BSK1), ksk(KSK);
  std::vector<uint64_t> bsk2(BSK2), tk(TK);
  CHECK(omr_keygen_detection_key(pa, seed ^ 0xD, bsk1.data(), ksk.data(), bsk2.data(), tk.data(), 0));
  std::printf("keygen time: %.3f s\n", secs(t));

  // pertinent = first min(D, 50) of a shuffle (omr.rs:103-113)
  const size_t pert_count = std::min<size_t>(D, 50);
  std::vector<size_t> order(D);
  std::iota(order.begin(), order.end(), 0);
  std::mt19937_64 rng(seed);
  std::shuffle(order.begin(), order.end(), rng);
  std::vector<size_t> pert(order.begin(), order.begin() + pert_count);
  std::sort(pert.begin(), pert.end());
  std::vector<char> is_pert(D, 0);
  for (size_t i : pert) is_pert[i] = 1;

  // Sender::gen_clues for every message (omr.rs:126-135)
  t = clk::now();
  std::vector<uint16_t> ca(D * N0), cb(D * CLUES), xa(D * N0), xb(D * CLUES);
  CHECK(omr_gen_clues(pa, seed + 1, 0, D, ca.data(), cb.data(), 0));
  CHECK(omr_gen_clues(pb, seed + 2, 0, D, xa.data(), xb.data(), 0));
  for (size_t m = 0; m < D; ++m)
    if (!is_pert[m]) {
      std::copy_n(&xa[m * N0], N0, &ca[m * N0]);
      std::copy_n(&xb[m * CLUES], CLUES, &cb[m * CLUES]);
    }
  std::printf("gen clues time: %.3f s\n", secs(t));

  // Payload::random (omr.rs:140-146)
  std::vector<uint16_t> payloads(D * PAYLOAD);
  for (auto &b : payloads) b = (uint16_t)(rng() & 0xff);

  omr_retrieval_params rp;
  CHECK(omr_get_retrieval_params(D, pert_count, &rp));
  uint8_t wseed[32];
  for (int i = 0; i < 32; ++i) wseed[i] = (uint8_t)(rng() & 0xff);
  std::vector<uint16_t> weights((size_t)rp.cmb_cipher_count * rp.cmb_count_per_cipher * D);
  CHECK(omr_payload_weights(wseed, D, rp.combination_count, rp.cmb_cipher_count, rp.cmb_count_per_cipher,
                            weights.data()));
  std::printf("retrieval params: %u index ct, %u payload ct (%u combinations)\n",
              rp.max_encode_indices_cipher_count, rp.cmb_cipher_count, rp.combination_count);
  if (host_only) {
    std::printf("host-only: keys, clues, weights and parameters OK\n");
    omr_secret_destroy(pa);
    omr_secret_destroy(pb);
    return 0;
  }

  // Detector::new + detect over the board (omr.rs:160-164)
  omr_ctx *ctx = nullptr;
  omr_detection_key_view view{bsk1.data(), ksk.data(), bsk2.data(), tk.data()};
  CHECK(omr_ctx_create(&view, device, &ctx));
  std::vector<uint64_t> pv(D * 2 * N2);
  t = clk::now();
  CHECK(omr_detect_batch(ctx, ca.data(), cb.data(), D, pv.data()));
  const double td = secs(t);
  std::printf("detect time: %.3f s (%.3f ms per message, host buffers)\n", td, td * 1e3 / D);

  // encode_pertinent_indices x max_encode_indices_cipher_count, encode_pertinent_payloads
  t = clk::now();
  const uint32_t n_idx = rp.max_encode_indices_cipher_count, n_pay = rp.cmb_cipher_count;
  std::vector<uint64_t> idx_ct((size_t)n_idx * 2 * N2), pay_ct((size_t)n_pay * 2 * N2);
  for (uint32_t c = 0; c < n_idx; ++c)
    CHECK(omr_encode_indices(ctx, pv.data(), D, 0, D, seed + 3, c, &idx_ct[(size_t)c * 2 * N2]));
  std::printf("encode indices time: %.3f s\n", secs(t));
  t = clk::now();
  CHECK(omr_encode_payloads(ctx, pv.data(), payloads.data(), D, 0, D, weights.data(), n_pay,
                            rp.cmb_count_per_cipher, pay_ct.data()));
  std::printf("encode pertinent payloads time: %.3f s\n", secs(t));

  // Retriever::decode_digest (omr.rs:216-218)
  t = clk::now();
  std::vector<size_t> found(pert_count + 64);
  size_t nfound = 0;
  CHECK(omr_retrieve_indices(pa, idx_ct.data(), n_idx, D, pert_count, found.data(), found.size(), &nfound));
  found.resize(std::min(nfound, found.size()));
  std::vector<uint16_t> solved(found.size() * PAYLOAD);
  CHECK(omr_retrieve_payloads(pa, pay_ct.data(), n_pay, D, rp.combination_count, weights.data(), found.data(), found.size(),
                              solved.data()));
  std::printf("decode time: %.3f s\n", secs(t));

  int fails = found == pert ? 0 : 1;
  if (fails) std::printf("Fail: %zu indices recovered, %zu pertinent\n", found.size(), pert.size());
  for (size_t k = 0; k < found.size() && !fails; ++k)
    if (!std::equal(&solved[k * PAYLOAD], &solved[(k + 1) * PAYLOAD], &payloads[found[k] * PAYLOAD])) {
      std::printf("Fail %zu\n", found[k]);
      ++fails;
    }
  std::printf(fails ? "FAILED\n" : "All done: %zu pertinent indices and payloads recovered\n", found.size());
  omr_ctx_destroy(ctx);
  omr_secret_destroy(pa);
  omr_secret_destroy(pb);
  return fails ? 1 : 0;
}

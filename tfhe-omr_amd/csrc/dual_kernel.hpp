// Level 1 of one chunk and level 2 of the previous chunk in one launch (round 5).
//
// The two blind rotations bind differently: br1f_kernel issues VALU on ~79 % of
// SIMD cycles, br2f_kernel on ~61 % and waits on latency the rest. Alone, one workgroup per CU
// keeps 67 % of level 1's throughput and 59 % of level 2's (profiles/r05v: LDS padded to one
// workgroup per CU), so a CU that runs one workgroup of each can outrun the two levels back to
// back: each fills the other's stalls. dual_kernel is one grid of n1 + n2 workgroups (n1 level-1
// items of BR1F_WPG rotations, n2 level-2 messages) whose LDS pool is the larger of the two
// bodies' (80 KB: two workgroups per CU). Each workgroup picks its role at entry: the one with
// fewer workgroups active on its CU (a per-CU pair of counters, keyed by the XCD id and HW_ID's
// CU / SH / SE fields; the placement decides speed only), then takes the next item of that role's
// queue, or of the other role's when that one is empty -- the grid has exactly one workgroup per
// item, so every workgroup gets one. The bodies are br1f_body / br2f_body unchanged (mode 0:
// extracted LWEs; the coefficient-domain rotation, traced by the launch after), so the outputs
// are bit-identical to the sequential launches.
// ctl: [0] level-1 queue, [1] level-2 queue, [2 + key] this CU's active workgroups (level 1 in the
// low 16 bits, level 2 in the high 16); zeroed before every launch.
#pragma once

#include "br1_fft.hpp"
#include "br2_fft.hpp"

namespace omr {

constexpr size_t DUAL_LDS_BYTES = BR2_LDS_BYTES > BR1_LDS_BYTES ? BR2_LDS_BYTES : BR1_LDS_BYTES;
constexpr int DUAL_CU_KEYS = 8 << 8;  // (XCC_ID: 3 bits) << 8 | HW_ID[15:8]
constexpr int DUAL_CTL_WORDS = 2 + DUAL_CU_KEYS;

__device__ __forceinline__ unsigned dual_cu_key() {
  const unsigned xcc = (unsigned)__builtin_amdgcn_s_getreg(6164) & 7u;  // hwreg(HW_REG_XCC_ID, 0, 4)
  const unsigned hw = (unsigned)__builtin_amdgcn_s_getreg(0x3a04);      // hwreg(HW_REG_HW_ID, 8, 8)
  return (xcc << 8) | (hw & 0xffu);
}

__global__ __launch_bounds__(256, 2) void dual_kernel(
    const uint16_t *__restrict__ clue_a, const uint16_t *__restrict__ clue_b, const double2 *__restrict__ bsk1f,
    uint32_t *__restrict__ ext, size_t nrot, unsigned n1, const uint32_t *__restrict__ lwe_int,
    const double2 *__restrict__ bsk2f, const double2 *__restrict__ twg, uint64_t *__restrict__ out, unsigned n2,
    DeviceTables tb, unsigned *ctl) {
  static_assert(64 * BR1F_WPG == Fft1024::T, "both roles run 256-thread workgroups");
  static_assert(BR1_LDS_XCH == 0 && BR2_LDS_X == 0, "the pool's 8 KB alignment serves br1f_digits");
  __shared__ __attribute__((aligned(8192))) double2 pool[DUAL_LDS_BYTES / sizeof(double2)];
  unsigned *pick = reinterpret_cast<unsigned *>(pool);
  unsigned *cnt = ctl + 2 + dual_cu_key();
  if (threadIdx.x == 0) {
    unsigned v = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), r;
    for (;;) {  // the role with fewer active workgroups on this CU (ties: level 2, the longer one)
      r = (v >> 16) <= (v & 0xffffu) ? 1u : 0u;
      if (__hip_atomic_compare_exchange_strong(cnt, &v, v + (r ? 0x10000u : 1u), __ATOMIC_RELAXED,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        break;
    }
    unsigned it = atomicAdd(ctl + r, 1u);
    if (it >= (r ? n2 : n1)) {  // this role's queue is empty: the other's has an item left
      atomicAdd(cnt, r ? 1u - 0x10000u : 0x10000u - 1u);
      r ^= 1u;
      it = atomicAdd(ctl + r, 1u);
    }
    pick[0] = r;
    pick[1] = it;
  }
  __syncthreads();
  const unsigned role = __builtin_amdgcn_readfirstlane(pick[0]), item = __builtin_amdgcn_readfirstlane(pick[1]);
  __syncthreads();  // pick[] read before the body reuses the pool
  if (role == 0)
    br1f_body<false>(clue_a, clue_b, nullptr, nullptr, bsk1f, tb, ext, nullptr, 0, nrot, nullptr,
                     reinterpret_cast<char *>(pool), item);
  else
    br2f_body<false>(lwe_int, bsk2f, twg, tb, out, nullptr, pool, item);
  if (threadIdx.x == 0) atomicSub(cnt, role ? 0x10000u : 1u);
}

}  // namespace omr

// Batched move selection for the policy players (K12; reference AlphaGo/ai.py:57-66 and
// policy.py:15-25): restrict the network distribution to the sensible moves, apply the
// temperature in log space (p^beta, beta = 1/T) and sample — or take the argmax for greedy rows.
//
// One 64-wide wavefront per position. Sampling is Gumbel-max: argmax_i(beta*log p_i + g_i) with
// g_i = -log(-log u_i) ~ Gumbel(0, 1) draws exactly from p_i^beta / sum_j p_j^beta over the mask,
// the same distribution as the reference's renormalise + temperature + choice, in one pass and
// without a prefix sum. u_i comes from a counter-based hash of (seed, row, point), so results are
// reproducible for a given seed and independent of the launch geometry.
//
//   rag_sample_moves: probs fp32 [B][P] (row stride P), mask uint8 [B][ms] (1 = candidate, first
//   P entries used), greedy uint8 [B] or null, beta, seed -> moves int32 [B] (flat point, -1 when
//   the row has no candidate). Greedy ties resolve to the lowest index (python max() over the
//   x-major legal-move list).
#include "common.h"

using namespace rag;

namespace {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// Order-preserving float -> uint32 (larger float <-> larger integer).
__device__ __forceinline__ uint32_t sortable(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

// Candidate rank as one 64-bit integer, maximised over the row: bit 63 = tier (positive
// probability), bits 32..62 = the key (31 most significant bits of its sortable form), low 32 =
// ~index (ties -> lowest index). Zero-probability candidates (tier 0) only win — uniformly, by
// their Gumbel noise — when every candidate has probability zero.
__global__ void __launch_bounds__(256) sample_moves_kernel(const float* __restrict__ probs,
                                                           const uint8_t* __restrict__ mask,
                                                           int ms, const uint8_t* __restrict__ greedy,
                                                           int B, int P, float beta, uint64_t seed,
                                                           const uint64_t* __restrict__ seed_dev,
                                                           int* __restrict__ moves) {
  if (seed_dev) seed ^= seed_dev[0];  // a captured graph's per-replay seed (self-play plies)
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= B) return;
  const bool gr = greedy != nullptr && greedy[row] != 0;
  const float* p = probs + (size_t)row * P;
  const uint8_t* mk = mask + (size_t)row * ms;
  uint64_t best = 0;
  for (int k = 0; k * 64 < P; ++k) {
    const int i = k * 64 + lane;
    const bool cand = i < P && mk[i] != 0;
    const float pi = cand ? p[i] : 0.f;
    float key;
    uint64_t tier;
    if (gr) {
      key = pi;
      tier = 1;
    } else {
      const uint64_t h = mix64(seed ^ mix64(((uint64_t)row << 20) + (uint64_t)i + 1));
      const float u = ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);  // (0, 1)
      const float g = -__logf(-__logf(u));
      tier = pi > 0.f ? 1 : 0;
      key = pi > 0.f ? beta * __logf(pi) + g : g;
    }
    const uint64_t r = (tier << 63) | ((uint64_t)(sortable(key) >> 1) << 32) |
                       (uint64_t)(0xffffffffu - (uint32_t)i);
    if (cand && r > best) best = r;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t ob = __shfl_xor(best, o, 64);
    best = ob > best ? ob : best;
  }
  if (lane == 0) moves[row] = best ? (int)(0xffffffffu - (uint32_t)(best & 0xffffffffu)) : -1;
}

}  // namespace

// seed_dev: null, or a device uint64 XORed into `seed` at run time (so a captured HIP graph can
// draw fresh moves on every replay from a host-written pinned copy).
RAG_API int rag_sample_moves(const float* probs, const uint8_t* mask, int ms,
                             const uint8_t* greedy, int B, int P, float beta, uint64_t seed,
                             const uint64_t* seed_dev, int* moves, hipStream_t stream) {
  if (B <= 0) return 0;
  if (ms < P || P <= 0) return -1;
  sample_moves_kernel<<<(B + 3) / 4, 256, 0, stream>>>(probs, mask, ms, greedy, B, P, beta, seed,
                                                       seed_dev, moves);
  return (int)hipGetLastError();
}

// Fast rollout policy: a linear softmax over cheap local features of each candidate
// move, used to play positions to the end for MCTS leaf evaluation (the lambda-mixed "z" term).
//
// Features of candidate a for the player c to move (all 0/1):
//   RF_RESPONSE   a is in the 8-neighbourhood of the last move
//   RF_SAVE_ATARI a touches an own group in atari and gains liberties (>=2 empty nbrs or capture)
//   RF_CAPTURE    a touches an opponent group in atari
//   RF_SELF_ATARI a leaves its own group with <= 1 liberty and captures nothing
//   RF_NEAR2      a is within Manhattan distance 2 of the last move (outside the 8-neighbourhood)
//   RF_OWN_NEAR   a is in the 8-neighbourhood of the second-to-last move (own previous move)
//   RF_EDGE       a is on the first line
// plus a 3x3 pattern weight indexed by the colours of the 8 surrounding points relative to c
// (0 empty, 1 own, 2 opponent, 3 off-board; 2 bits each, clockwise from north => 65536 entries).
//
// Candidates: empty, not an own single-point eye (eyeish + at most one bad diagonal in the
// centre, none on the edge), legal (suicide / ko checked on the sampled move only). The same
// feature definitions run on the GPU in csrc/hip/rollout.hip.
#pragma once
#include <cstdint>
#include <vector>

#include "../engine/go_engine.hpp"

namespace rag {

enum RolloutFeature : int {
  RF_RESPONSE = 0, RF_SAVE_ATARI, RF_CAPTURE, RF_SELF_ATARI, RF_NEAR2, RF_OWN_NEAR, RF_EDGE,
  RF_COUNT
};
constexpr int RP_PATTERNS = 1 << 16;

// Seed of a position-keyed rollout: a function of the stones and the player to move only, so
// every search that reaches a position plays the same rollout from it (search/efficiency.py
// compares search designs with such rollouts: the only difference left is the tree's shape).
inline uint64_t position_key_seed(uint64_t hash, int player) {
  return hash * 0xD6E8FEB86659FD93ull ^ (uint64_t)(player + 2) * 0xA0761D6478BD642Full;
}

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull) {}
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  float uniform() { return (next() >> 40) * (1.0f / 16777216.0f); }
};

// 8-neighbourhood tables per board size (clockwise from north; -1 = off board).
struct Ring8 {
  int S;
  int16_t nb[MAXP][8];
  static const Ring8* get(int S);
};

struct RolloutPolicy {
  float w[RF_COUNT];
  std::vector<float> pattern;  // RP_PATTERNS
  RolloutPolicy();

  // Candidate moves with their feature bitmask (bit f = feature f) and pattern index.
  int candidates(const Board& b, int* moves, uint8_t* fbits, int32_t* pat) const;
  // Softmax sample of a legal candidate (PASS if none). Temperature 1.
  int sample(const Board& b, Rng& rng, int* scratch_moves, float* scratch_p) const;
  // Play b (light copy) to the end or `limit` moves; returns the winner (BLACK/WHITE/0).
  int rollout(Board& b, Rng& rng, int limit) const;
};

bool rollout_is_own_eye(const Board& b, int p, int c);

}  // namespace rag

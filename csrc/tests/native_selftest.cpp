// Stand-alone self-test of the native runtime, built without Python so it can run under the
// sanitizers: ThreadSanitizer for the multi-threaded search (thread pools, async
// rollout waves) and Address/UndefinedBehaviorSanitizer for the engine, features, ladders and
// the tree. Driven by tests/test_sanitizers.py:
//   g++ -std=c++17 -O1 -g -fsanitize=thread  ... && ./selftest
//   g++ -std=c++17 -O1 -g -fsanitize=address,undefined ... && ./selftest
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <random>
#include <vector>

#include "../engine/go_engine.hpp"
#include "../engine/thread_pool.hpp"
#include "../mcts/rollout.hpp"
#include "../mcts/search.hpp"

using namespace rag;

#define CHECK(c)                                                          \
  do {                                                                    \
    if (!(c)) {                                                           \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                       \
    }                                                                     \
  } while (0)

static std::shared_ptr<const Zobrist> zob(int S) {
  auto z = std::make_shared<Zobrist>();
  std::mt19937_64 r(0);
  for (int i = 0; i < S * S; ++i) {
    z->white.push_back(r());
    z->black.push_back(r());
  }
  return z;
}

int main() {
  const int S = 9;
  auto z = zob(S);
  RolloutPolicy rp;
  // 1. random games with features + ladders on every position
  std::vector<Board> positions;
  {
    Rng rng(7);
    std::vector<int> mv(MAXP);
    std::vector<float> pr(MAXP);
    for (int g = 0; g < 6; ++g) {
      Board b(S, 7.5, g % 2 == 0, z);
      for (int k = 0; k < 70 && !b.end_of_game(); ++k) {
        const int a = rp.sample(b, rng, mv.data(), pr.data());
        if (a >= 0 && !b.is_legal(a)) continue;
        b.do_move(a, 0);
        positions.push_back(b);
      }
    }
  }
  const int fids[] = {F_BOARD, F_ONES, F_TURNS_SINCE, F_LIBERTIES, F_CAPTURE_SIZE,
                      F_SELF_ATARI_SIZE, F_LIBERTIES_AFTER, F_LADDER_CAPTURE, F_LADDER_ESCAPE,
                      F_SENSIBLENESS, F_ZEROS, F_LEGAL, F_COLOR};
  int planes = 0;
  for (int f : fids) planes += feature_planes(f);
  std::vector<uint8_t> out(planes * S * S);
  for (const Board& b : positions) {
    extract_features(b, fids, (int)(sizeof(fids) / sizeof(fids[0])), out.data());
    Board c(b);
    c.set_light(true);
    for (int p = 0; p < S * S; ++p)
      if (c.color(p) == EMPTY) (void)c.is_ladder_capture(p, -1, 80);
  }
  // 1b. the journaled ladder reader on the shared pool == the copying reader
  {
    std::vector<uint8_t> got(positions.size() * 2 * S * S);
    shared_pool(4).run((int)positions.size(), [&](int i) {
      thread_local LadderReader reader;
      uint8_t* o = got.data() + (size_t)i * 2 * S * S;
      ladder_planes(positions[i], o, o + S * S, &reader);
    });
    for (size_t i = 0; i < positions.size(); ++i) {
      const Board& b = positions[i];
      for (int p = 0; p < S * S; ++p) {
        const bool e = b.color(p) == EMPTY;
        CHECK(got[i * 2 * S * S + p] == (e && b.is_ladder_capture(p, -1, 80)));
        CHECK(got[i * 2 * S * S + S * S + p] == (e && b.is_ladder_escape(p, -1, 80)));
      }
    }
  }
  // 2. multi-threaded rollouts
  {
    mcts_detail::Pool pool(4);
    std::vector<int> winners(positions.size());
    pool.run((int)positions.size(), [&](int i) {
      Board b(positions[i]);
      b.set_enforce_superko(false);
      Rng rng(100 + i);
      winners[i] = rp.rollout(b, rng, 400);
    });
    for (int w : winners) CHECK(w >= -1 && w <= 1);
  }
  // 3. APV search with asynchronous CPU rollout waves overlapping value backups
  {
    Board root(S, 7.5, false, z);
    Search s(root, 4);
    s.lambda = 0.5f;
    std::vector<float> values(64, 0.f);
    for (int wave = 0; wave < 12; ++wave) {
      auto w1 = s.select(16);
      if (w1.first < 0) continue;
      s.start_rollouts(w1.first);
      s.backup_value(w1.first, nullptr, 0, values.data());
      auto w2 = s.select(16);  // selected while w1's rollouts are still running
      if (w2.first >= 0) {
        s.start_rollouts(w2.first);
        s.backup_value(w2.first, nullptr, 0, values.data());
        s.finish_rollouts(w2.first);
      }
      s.finish_rollouts(w1.first);
    }
    CHECK(s.pending_waves() == 0);
    CHECK(s.root_visits() > 100);
    const int mv = s.best_move();
    CHECK(mv >= -1 && mv < S * S);
    CHECK(s.advance(mv) || true);
    auto w = s.select(8);
    CHECK(w.first >= 0);
    s.backup_value(w.first, nullptr, 0, values.data());
    s.finish_rollouts(w.first);
  }
  // 4. parallel descents (descend_parallel): distinct leaves per wave, virtual loss balanced
  {
    Board root(S, 7.5, false, z);
    Search s(root, 4);
    s.lambda = 0.5f;
    s.parallel_select_min = 8;
    std::vector<float> values(64, 0.1f);
    for (int wave = 0; wave < 10; ++wave) {
      auto w = s.select(48);
      if (w.first < 0) continue;
      std::vector<int> ids;
      for (const Leaf& L : s.wave(w.first).leaves) ids.push_back(L.path.back());
      std::sort(ids.begin(), ids.end());
      CHECK(std::adjacent_find(ids.begin(), ids.end()) == ids.end());
      s.start_rollouts(w.first);
      s.backup_value(w.first, nullptr, 0, values.data());
      s.finish_rollouts(w.first);
    }
    CHECK(s.pending_waves() == 0);
    CHECK(s.root_visits() > 200);
  }
  std::printf("native selftest ok: %zu positions\n", positions.size());
  return 0;
}

// Packing native boards into the inputs of the GPU feature / rollout kernels, shared by the
// search (csrc/mcts/search.hpp) and the self-play game batch (gamebatch.cpp).
#pragma once

#include <algorithm>
#include <cstdint>

#include "go_engine.hpp"

namespace rag {

// Output views: a null pointer skips that output; `stride` is the distance in bytes between
// consecutive boards (rows), so outputs may be columns of one record array.
struct PackOut {
  int8_t* colors = nullptr;    // [P]
  int16_t* ages = nullptr;     // [P] stone ages (-1 empty, clamped to 32767)
  int32_t* meta4 = nullptr;    // player, ko, superko flag, 0
  int32_t* meta8 = nullptr;    // rollout kernel meta (see write_meta8)
  uint8_t* illegal = nullptr;  // [P] positional-superko-illegal points (superko boards)
  uint8_t* ladders = nullptr;  // [2][P] ladder capture / escape planes
  size_t s_colors = 0, s_ages = 0, s_meta4 = 0, s_meta8 = 0, s_illegal = 0, s_ladders = 0;
};

// Rollout-kernel meta of a board: player to move, ko, last move, second-to-last move, black
// passes, white passes, moves played, end-of-game flag.
inline void write_meta8(const Board& b, int32_t* m) {
  m[0] = b.current_player();
  m[1] = b.ko();
  m[2] = b.last1();
  m[3] = b.last2();
  m[4] = b.passes_black();
  m[5] = b.passes_white();
  m[6] = b.nmoves();
  m[7] = b.end_of_game() ? 1 : 0;
}

// Row i of every requested output from board b.
inline void pack_board(const Board& b, int i, const PackOut& o) {
  const int P = b.npoints();
  auto row = [&](auto* base, size_t stride) {
    using T = std::remove_pointer_t<decltype(base)>;
    return reinterpret_cast<T*>(reinterpret_cast<char*>(base) + (size_t)i * stride);
  };
  if (o.colors) {
    int8_t* c = row(o.colors, o.s_colors);
    for (int p = 0; p < P; ++p) c[p] = (int8_t)b.color(p);
  }
  if (o.ages) {
    int16_t* a = row(o.ages, o.s_ages);
    for (int p = 0; p < P; ++p) a[p] = (int16_t)std::min(b.stone_age(p), 32767);
  }
  if (o.meta4) {
    int32_t* m = row(o.meta4, o.s_meta4);
    m[0] = b.current_player();
    m[1] = b.ko();
    m[2] = b.enforce_superko() ? 1 : 0;
    m[3] = 0;
  }
  if (o.meta8) write_meta8(b, row(o.meta8, o.s_meta8));
  if (o.illegal) {
    uint8_t* il = row(o.illegal, o.s_illegal);
    for (int p = 0; p < P; ++p)
      il[p] = (b.enforce_superko() && b.color(p) == EMPTY && p != b.ko() && !b.is_suicide(p) &&
               b.is_positional_superko(p))
                  ? 1 : 0;
  }
  if (o.ladders) {
    thread_local LadderReader reader;
    uint8_t* l0 = row(o.ladders, o.s_ladders);
    ladder_planes(b, l0, l0 + P, &reader);
  }
}

}  // namespace rag

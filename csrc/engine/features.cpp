// Native feature-plane extraction — behavioural contract: AlphaGo/preprocessing/preprocessing.py
// of the reference (get_board ... get_legal, preprocessing.py:14-205) plus the "color" plane the
// reference's value net expects (value.py:16).
//
// One pass computes the legal-move list once and fills every requested plane; the python
// reference recomputes legal moves and walks python sets per feature.
#include <algorithm>
#include <cstring>

#include "go_engine.hpp"

namespace rag {

int feature_planes(int fid) {
  switch (fid) {
    case F_BOARD: return 3;
    case F_ONES: return 1;
    case F_TURNS_SINCE: return 8;
    case F_LIBERTIES: return 8;
    case F_CAPTURE_SIZE: return 8;
    case F_SELF_ATARI_SIZE: return 8;
    case F_LIBERTIES_AFTER: return 8;
    case F_LADDER_CAPTURE: return 1;
    case F_LADDER_ESCAPE: return 1;
    case F_SENSIBLENESS: return 1;
    case F_ZEROS: return 1;
    case F_LEGAL: return 1;
    case F_COLOR: return 1;
    default: throw std::invalid_argument("unknown feature id");
  }
}

namespace {

// simulated liberties / group after playing p (preprocessing.py:89-169)
struct AfterMove {
  int libs;
  int size;
};

AfterMove simulate(const Board& b, int p) {
  const Geometry& g = b.geom();
  const int W = g.W;
  const int me = b.current_player();
  Bitset libs, grp, captured;
  libs.clear(W);
  grp.clear(W);
  captured.clear(W);
  for (int i = 0; i < g.nnbr[p]; ++i) {
    int n = g.nbr[p][i];
    if (b.color(n) == EMPTY) libs.set(n);
  }
  grp.set(p);
  int heads[4];
  int nh = b.groups_around(p, heads);
  bool any_cap = false;
  std::vector<int> stones;
  for (int i = 0; i < nh; ++i) {
    int h = heads[i];
    if (b.color(h) == me) {
      Bitset l;
      b.liberty_set(h, l);
      libs.or_with(l, W);
      b.group_stones(h, stones);
      for (int s : stones) grp.set(s);
    } else if (b.liberty_count(h) == 1) {
      b.group_stones(h, stones);
      for (int s : stones) captured.set(s);
      any_cap = true;
    }
  }
  if (any_cap) {
    grp.for_each(W, [&](int s) {
      for (int i = 0; i < g.nnbr[s]; ++i) {
        int n = g.nbr[s][i];
        if (captured.test(n)) libs.set(n);
      }
    });
  }
  libs.reset(p);
  return {libs.count(W), grp.count(W)};
}

}  // namespace

void extract_features(const Board& b, const int* fids, int nf, uint8_t* out) {
  const int S = b.size();
  const int P = S * S;
  int total = 0;
  for (int i = 0; i < nf; ++i) total += feature_planes(fids[i]);
  std::memset(out, 0, (size_t)total * P);

  bool need_legal = false;
  for (int i = 0; i < nf; ++i) {
    int f = fids[i];
    need_legal |= (f == F_CAPTURE_SIZE || f == F_SELF_ATARI_SIZE || f == F_LIBERTIES_AFTER ||
                   f == F_LADDER_CAPTURE || f == F_LADDER_ESCAPE || f == F_SENSIBLENESS ||
                   f == F_LEGAL);
  }
  std::vector<int> non_eye, eyes, legal;
  if (need_legal) {
    b.legal_moves(non_eye, eyes);
    legal = non_eye;
    legal.insert(legal.end(), eyes.begin(), eyes.end());
  }
  const int me = b.current_player();
  bool have_after = false;
  std::vector<AfterMove> after;
  std::vector<uint8_t> ladders;

  uint8_t* o = out;
  for (int i = 0; i < nf; ++i) {
    const int f = fids[i];
    switch (f) {
      case F_BOARD:
        for (int p = 0; p < P; ++p) {
          int c = b.color(p);
          if (c == me)
            o[p] = 1;
          else if (c == -me)
            o[P + p] = 1;
          else
            o[2 * P + p] = 1;
        }
        break;
      case F_ONES:
        std::memset(o, 1, P);
        break;
      case F_ZEROS:
        break;
      case F_COLOR:
        if (me == BLACK) std::memset(o, 1, P);
        break;
      case F_TURNS_SINCE:
        for (int p = 0; p < P; ++p) {
          int a = b.stone_age(p);
          if (a >= 0) o[std::min(a, 7) * P + p] = 1;
        }
        break;
      case F_LIBERTIES:
        for (int p = 0; p < P; ++p) {
          int l = b.liberty_count(p);
          if (l >= 1 && l <= 8) o[(l - 1) * P + p] = 1;
          if (l >= 8) o[7 * P + p] = 1;
        }
        break;
      case F_CAPTURE_SIZE:
        for (int p : legal) {
          int heads[4];
          int nh = b.groups_around(p, heads);
          int n = 0;
          for (int k = 0; k < nh; ++k)
            if (b.liberty_count(heads[k]) == 1 && b.color(heads[k]) != me)
              n += b.group_size(heads[k]);
          o[std::min(n, 7) * P + p] = 1;
        }
        break;
      case F_SELF_ATARI_SIZE:
      case F_LIBERTIES_AFTER:
        if (!have_after) {
          after.resize(legal.size());
          for (size_t k = 0; k < legal.size(); ++k) after[k] = simulate(b, legal[k]);
          have_after = true;
        }
        for (size_t k = 0; k < legal.size(); ++k) {
          const int p = legal[k];
          if (f == F_SELF_ATARI_SIZE) {
            if (after[k].libs == 1) o[std::min(after[k].size - 1, 7) * P + p] = 1;
          } else {
            int idx = std::min(7, after[k].libs - 1);
            if (idx < 0) idx += 8;  // python negative index semantics of planes[-1]
            o[idx * P + p] = 1;
          }
        }
        break;
      case F_LADDER_CAPTURE:
      case F_LADDER_ESCAPE:
        // both planes come from one pass of the journaled reader (ladder.cpp); it answers
        // illegal points with 0 like the per-point reference calls
        if (ladders.empty()) {
          ladders.resize(2 * (size_t)P);
          ladder_planes(b, ladders.data(), ladders.data() + P);
        }
        std::memcpy(o, ladders.data() + (f == F_LADDER_CAPTURE ? 0 : P), P);
        break;
      case F_SENSIBLENESS:
        for (int p : non_eye) o[p] = 1;
        break;
      case F_LEGAL:
        for (int p : legal) o[p] = 1;
        break;
      default:
        throw std::invalid_argument("unknown feature id");
    }
    o += (size_t)feature_planes(f) * P;
  }
}

}  // namespace rag

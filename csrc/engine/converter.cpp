// Native SGF -> training-position converter: one SGF game text in, the feature
// planes of every non-pass move and the moves out. The Python converter
// (rocalphago_amd/features/converter.py) runs many games of a batch on the shared thread pool
// through this and writes whole 64-row LZF chunks.
//
// Behavioural contract: GameConverter.convert_game of the reference
// (AlphaGo/preprocessing/game_converter.py:32-40) over its SGF replay (AlphaGo/util.py:21-63,
// 100-128), as implemented in Python by features/converter.py + utils/go_util.py:
//   * the root node's SZ / AB / AW / PL set up the board (AB/AW stones are played with do_move,
//     then PL picks the player to move);
//   * every later main-line node is a W move (checked first), a B move, or a setup node: an AB-only
//     node on a board with no history places handicap stones, any other AB/AW stones are played;
//   * the planes of a position are taken BEFORE its move is played, pass moves ('' or 'tt') are
//     played but yield no position;
//   * an illegal move ends the game; like the reference's generator (whose consumer stores a
//     position before the replay tries its move) the position of the illegal move is kept.
// Anything this parser does not reproduce byte-for-byte (a parse error, a board size other than
// the requested one, a non-ASCII byte outside a property value, an unusual coordinate) returns
// kFallback, and the caller converts that game with the Python implementation, which raises and
// reports exactly as the reference does.
#include <cstring>
#include <string>
#include <vector>

#include "go_engine.hpp"

namespace rag {

namespace {

struct SgfNode {
  std::vector<std::pair<std::string, std::vector<std::string>>> props;
  const std::vector<std::string>* get(const char* id) const {
    for (auto& p : props)
      if (p.first == id) return &p.second;
    return nullptr;
  }
};

// Recursive-descent SGF parser with the grammar of io/sgf.py. Returns false on any error (the
// caller falls back to the Python parser for its exact error). Collects the main line of the
// first game: the first game tree's nodes, then the first variation's, recursively.
class SgfParser {
 public:
  SgfParser(const char* s, size_t n) : s_(s), n_(n) {}

  bool main_line(std::vector<SgfNode>& out) {
    ws();
    bool first = true;
    while (i_ < n_) {
      if (s_[i_] != '(') {
        if (!first) break;  // trailing garbage after the last game
        return false;
      }
      if (!tree(first ? &out : nullptr, true)) return false;
      first = false;
      ws();
    }
    return !first && !out.empty();
  }

 private:
  static bool is_ws(char c) {
    return c == ' ' || c == '\t' || c == '\r' || c == '\n' || c == '\x0b' || c == '\x0c';
  }
  static bool is_alpha(unsigned char c) {
    return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z');
  }
  void ws() {
    while (i_ < n_ && is_ws(s_[i_])) ++i_;
  }
  // `out` collects nodes while on the main line (null elsewhere); `main` = this tree is on it
  bool tree(std::vector<SgfNode>* out, bool main) {
    ws();
    if (i_ >= n_ || s_[i_] != '(') return false;
    ++i_;
    ws();
    int nodes = 0;
    while (i_ < n_ && s_[i_] == ';') {
      ++i_;
      SgfNode nd;
      if (!node(nd)) return false;
      if (out && main) out->push_back(std::move(nd));
      ++nodes;
      ws();
    }
    if (!nodes) return false;
    bool first_var = true;
    while (i_ < n_ && s_[i_] == '(') {
      if (!tree(out, main && first_var)) return false;
      first_var = false;
      ws();
    }
    ws();
    if (i_ >= n_ || s_[i_] != ')') return false;
    ++i_;
    return true;
  }
  bool node(SgfNode& nd) {
    while (true) {
      ws();
      if (i_ >= n_) break;
      const unsigned char c = (unsigned char)s_[i_];
      if (c >= 0x80) return false;  // python's isalpha() on non-ASCII: leave it to python
      if (!is_alpha(c)) break;
      std::string ident;
      while (i_ < n_ && (unsigned char)s_[i_] < 0x80 && is_alpha((unsigned char)s_[i_])) {
        if (s_[i_] >= 'A' && s_[i_] <= 'Z') ident.push_back(s_[i_]);
        ++i_;
      }
      if (i_ < n_ && (unsigned char)s_[i_] >= 0x80) return false;
      std::vector<std::string> vals;
      ws();
      while (i_ < n_ && s_[i_] == '[') {
        std::string v;
        if (!value(v)) return false;
        vals.push_back(std::move(v));
        ws();
      }
      if (vals.empty()) return false;
      bool merged = false;
      for (auto& p : nd.props)
        if (p.first == ident) {
          p.second.insert(p.second.end(), vals.begin(), vals.end());
          merged = true;
        }
      if (!merged) nd.props.emplace_back(ident, std::move(vals));
    }
    return true;
  }
  bool value(std::string& v) {
    ++i_;  // '['
    while (true) {
      if (i_ >= n_) return false;
      const char c = s_[i_];
      if (c == '\\') {
        ++i_;
        if (i_ < n_ && s_[i_] != '\n') v.push_back(s_[i_]);
        ++i_;
        continue;
      }
      if (c == ']') {
        ++i_;
        return true;
      }
      v.push_back(c);
      ++i_;
    }
  }
  const char* s_;
  size_t n_, i_ = 0;
};

enum Status : int { kOk = 0, kIllegal = 1, kFallback = 3 };

// (col, row) of an SGF point value; 1 = pass, 0 = point, -1 = anything unusual (fallback).
int parse_point(const std::string& v, int& x, int& y) {
  if (v.empty() || v == "tt") return 1;
  if (v.size() < 2) return -1;
  auto idx = [](char c) {
    if (c >= 'a' && c <= 'z') return c - 'a';
    if (c >= 'A' && c <= 'Z') return c - 'A';
    return -1;
  };
  x = idx(v[0]);
  y = idx(v[1]);
  return (x < 0 || y < 0) ? -1 : 0;
}

// AB / AW values, 'aa:cc' rectangles expanded (go_util._expand_point_list); false = fallback
bool point_list(const std::vector<std::string>& vals, std::vector<std::pair<int, int>>& out) {
  for (const std::string& v : vals) {
    const size_t colon = v.find(':');
    if (colon == std::string::npos) {
      int x, y;
      if (parse_point(v, x, y) != 0) return false;
      out.emplace_back(x, y);
      continue;
    }
    int x0, y0, x1, y1;
    if (parse_point(v.substr(0, colon), x0, y0) != 0 ||
        parse_point(v.substr(colon + 1), x1, y1) != 0)
      return false;
    for (int x = std::min(x0, x1); x <= std::max(x0, x1); ++x)
      for (int y = std::min(y0, y1); y <= std::max(y0, y1); ++y) out.emplace_back(x, y);
  }
  return true;
}

int flat(int x, int y, int S) { return (x >= S || y >= S) ? -3 : x * S + y; }

}  // namespace

// The replay shared by both entry points: on_position(board) sees every position that yields a
// training row (before its move is played).
template <class OnPosition>
int replay_sgf(const char* text, size_t len, int bd_size, const std::shared_ptr<const Zobrist>& zob,
               std::vector<uint8_t>& actions, OnPosition&& on_position) {
  actions.clear();
  std::vector<SgfNode> line;
  SgfParser parser(text, len);
  if (!parser.main_line(line)) return kFallback;
  const SgfNode& root = line[0];
  int S = 19;
  if (const auto* sz = root.get("SZ")) {
    const std::string v = (*sz)[0].substr(0, (*sz)[0].find(':'));
    if (v.empty() || v.size() > 3 || v.find_first_not_of("0123456789") != std::string::npos)
      return kFallback;
    S = std::stoi(v);
  }
  if (S != bd_size) return kFallback;  // size-mismatch / setup-error ordering: python decides
  try {
    Board b(S, 7.5, false, zob);
    std::vector<std::pair<int, int>> pts;
    for (const char* key : {"AB", "AW"}) {
      const auto* v = root.get(key);
      if (!v) continue;
      pts.clear();
      if (!point_list(*v, pts)) return kFallback;
      for (auto& p : pts) b.do_move(flat(p.first, p.second, S), key[1] == 'B' ? BLACK : WHITE);
    }
    const auto* pl = root.get("PL");
    b.set_current_player(pl && (*pl)[0] != "B" ? WHITE : BLACK);
    for (size_t k = 1; k < line.size(); ++k) {
      const SgfNode& nd = line[k];
      const auto* w = nd.get("W");
      const auto* bl = w ? nullptr : nd.get("B");
      if (!w && !bl) {  // setup node
        const auto* ab = nd.get("AB");
        const auto* aw = nd.get("AW");
        if (ab && !aw && b.history().empty()) {
          pts.clear();
          if (!point_list(*ab, pts)) return kFallback;
          std::vector<int> h;
          for (auto& p : pts) h.push_back(flat(p.first, p.second, S));
          b.place_handicaps(h);
        } else {
          for (const char* key : {"AB", "AW"}) {
            const auto* v = nd.get(key);
            if (!v) continue;
            pts.clear();
            if (!point_list(*v, pts)) return kFallback;
            for (auto& p : pts)
              b.do_move(flat(p.first, p.second, S), key[1] == 'B' ? BLACK : WHITE);
          }
        }
        continue;
      }
      const std::string& v = (w ? *w : *bl)[0];
      int x = 0, y = 0;
      const int kind = parse_point(v, x, y);
      if (kind < 0) return kFallback;
      const int color = w ? WHITE : BLACK;
      if (kind == 0) {  // the position before the move
        on_position(b);
        actions.push_back((uint8_t)x);
        actions.push_back((uint8_t)y);
        b.do_move(flat(x, y, S), color);
      } else {
        b.do_move(PASS, color);
      }
    }
  } catch (const IllegalMoveError&) {
    return kIllegal;
  } catch (const std::exception&) {
    return kFallback;
  }
  return kOk;
}

int convert_sgf_game(const char* text, size_t len, int bd_size,
                     const std::shared_ptr<const Zobrist>& zob, const int* fids, int nf,
                     std::vector<uint8_t>& states, std::vector<uint8_t>& actions) {
  states.clear();
  const int P = bd_size * bd_size;
  int planes = 0;
  for (int i = 0; i < nf; ++i) planes += feature_planes(fids[i]);
  return replay_sgf(text, len, bd_size, zob, actions, [&](const Board& b) {
    const size_t at = states.size();
    states.resize(at + (size_t)planes * P);
    extract_features(b, fids, nf, states.data() + at);
  });
}

// Replay only: a copy of the board at every training position (the batch converter then
// extracts the planes of all positions of all games in one fine-grained parallel loop, so a
// long game does not serialise the tail of a batch).
int replay_sgf_positions(const char* text, size_t len, int bd_size,
                         const std::shared_ptr<const Zobrist>& zob, std::vector<Board>& boards,
                         std::vector<uint8_t>& actions) {
  boards.clear();
  return replay_sgf(text, len, bd_size, zob, actions,
                    [&](const Board& b) { boards.push_back(b); });
}

}  // namespace rag

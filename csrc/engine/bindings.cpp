// pybind11 module `rocalphago_amd._rocgo`: Go engine, feature extraction, LZF codec, search.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <thread>

#include "go_engine.hpp"
#include "thread_pool.hpp"

namespace py = pybind11;
using namespace rag;

namespace rag {
size_t lzf_decompress(const uint8_t* in, size_t n, uint8_t* out, size_t cap);
size_t lzf_compress(const uint8_t* in, size_t n, uint8_t* out, size_t cap);
void register_search(py::module_& m);
int convert_sgf_game(const char* text, size_t len, int bd_size,
                     const std::shared_ptr<const Zobrist>& zob, const int* fids, int nf,
                     std::vector<uint8_t>& states, std::vector<uint8_t>& actions);
int replay_sgf_positions(const char* text, size_t len, int bd_size,
                         const std::shared_ptr<const Zobrist>& zob, std::vector<Board>& boards,
                         std::vector<uint8_t>& actions);
void register_rollout(py::module_& m);
void register_master(py::module_& m);
void register_gamebatch(py::module_& m);

std::shared_ptr<const Zobrist> make_zobrist(py::array_t<uint64_t, py::array::c_style> w,
                                           py::array_t<uint64_t, py::array::c_style> b) {
  auto z = std::make_shared<Zobrist>();
  z->white.assign(w.data(), w.data() + w.size());
  z->black.assign(b.data(), b.data() + b.size());
  return z;
}
}  // namespace rag

namespace {

py::array_t<int8_t> board_array(const Board& b) {
  const int S = b.size();
  py::array_t<int8_t> a({S, S});
  auto r = a.mutable_unchecked<2>();
  for (int x = 0; x < S; ++x)
    for (int y = 0; y < S; ++y) r(x, y) = (int8_t)b.color(x * S + y);
  return a;
}

std::vector<int> to_fids(const std::vector<int>& f) { return f; }

int total_planes(const std::vector<int>& fids) {
  int t = 0;
  for (int f : fids) t += feature_planes(f);
  return t;
}

void parallel_for(int n, int nthreads, const std::function<void(int)>& fn) {
  if (nthreads <= 1 || n <= 1) {
    for (int i = 0; i < n; ++i) fn(i);
    return;
  }
  shared_pool(std::min(nthreads, 64)).run(n, fn);
}

}  // namespace

PYBIND11_MODULE(_rocgo, m) {
  m.doc() = "RocAlphaGo-MI355X native engine (rules, features, LZF, search)";
  static py::exception<IllegalMoveError> exc(m, "IllegalMove");
  py::register_exception_translator([](std::exception_ptr p) {
    try {
      if (p) std::rethrow_exception(p);
    } catch (const IllegalMoveError& e) {
      exc(e.what());
    }
  });

  py::class_<Zobrist, std::shared_ptr<Zobrist>>(m, "Zobrist");
  m.def("make_zobrist", [](py::array_t<uint64_t, py::array::c_style> w,
                           py::array_t<uint64_t, py::array::c_style> b) {
    return std::const_pointer_cast<Zobrist>(make_zobrist(w, b));
  });

  py::class_<Board>(m, "Board")
      .def(py::init([](int size, double komi, bool superko, std::shared_ptr<Zobrist> z) {
        return Board(size, komi, superko, z);
      }))
      .def("copy", [](const Board& b) { return Board(b); })
      .def("do_move", &Board::do_move, py::arg("a"), py::arg("color") = 0)
      .def("play_unchecked", &Board::play_unchecked)
      .def("is_legal", &Board::is_legal)
      .def("is_suicide", &Board::is_suicide)
      .def("is_positional_superko", &Board::is_positional_superko)
      .def("is_eyeish", &Board::is_eyeish)
      .def("is_eye",
           [](const Board& b, int p, int owner, std::vector<int> stack) {
             return b.is_eye_stack(p, owner, stack);
           })
      .def("is_ladder_capture", &Board::is_ladder_capture, py::arg("a"), py::arg("prey") = -1,
           py::arg("remaining") = 80)
      .def("is_ladder_escape", &Board::is_ladder_escape, py::arg("a"), py::arg("prey") = -1,
           py::arg("remaining") = 80)
      .def("legal_moves",
           [](const Board& b) {
             std::vector<int> ne, ey;
             b.legal_moves(ne, ey);
             return py::make_tuple(ne, ey);
           })
      .def("get_winner", &Board::get_winner)
      .def("score",
           [](const Board& b) {
             double bl, wh;
             b.score(bl, wh);
             return py::make_tuple(wh, bl);
           })
      .def("place_handicaps", &Board::place_handicaps)
      .def("board", &board_array)
      .def("liberty_counts",
           [](const Board& b) {
             const int S = b.size();
             py::array_t<int64_t> a({S, S});
             auto r = a.mutable_unchecked<2>();
             for (int x = 0; x < S; ++x)
               for (int y = 0; y < S; ++y) r(x, y) = b.liberty_count(x * S + y);
             return a;
           })
      .def("stone_ages",
           [](const Board& b) {
             const int S = b.size();
             py::array_t<int64_t> a({S, S});
             auto r = a.mutable_unchecked<2>();
             for (int x = 0; x < S; ++x)
               for (int y = 0; y < S; ++y) r(x, y) = b.stone_age(x * S + y);
             return a;
           })
      .def("group_heads",
           [](const Board& b) {
             const int S = b.size();
             py::array_t<int32_t> a({S * S});
             auto r = a.mutable_unchecked<1>();
             for (int p = 0; p < S * S; ++p) r(p) = b.group_head(p);
             return a;
           })
      .def("group",
           [](const Board& b, int p) {
             std::vector<int> s;
             b.group_stones(p, s);
             return s;
           })
      .def("liberty_set",
           [](const Board& b, int p) {
             Bitset bs;
             b.liberty_set(p, bs);
             std::vector<int> v;
             bs.for_each(b.geom().W, [&](int i) { v.push_back(i); });
             return v;
           })
      .def("groups_around",
           [](const Board& b, int p) {
             int h[4];
             int n = b.groups_around(p, h);
             return std::vector<int>(h, h + n);
           })
      .def("color_at", &Board::color)
      .def("liberty_count", &Board::liberty_count)
      .def("features",
           [](const Board& b, const std::vector<int>& fids) {
             const int S = b.size();
             py::array_t<uint8_t> a({total_planes(fids), S, S});
             extract_features(b, fids.data(), (int)fids.size(), a.mutable_data());
             return a;
           })
      .def_property_readonly("size", &Board::size)
      .def_property("current_player", &Board::current_player, &Board::set_current_player)
      .def_property("ko", &Board::ko, &Board::set_ko)
      .def_property("komi", &Board::komi, &Board::set_komi)
      .def_property("enforce_superko", &Board::enforce_superko, &Board::set_enforce_superko)
      .def_property("end_of_game", &Board::end_of_game, &Board::set_end_of_game)
      .def_property_readonly("black_prisoners", &Board::black_prisoners)
      .def_property_readonly("white_prisoners", &Board::white_prisoners)
      .def("set_prisoners", &Board::set_prisoners)
      .def_property_readonly("passes_black", &Board::passes_black)
      .def_property_readonly("passes_white", &Board::passes_white)
      .def("set_passes", &Board::set_passes)
      .def_property_readonly("hash", &Board::hash)
      .def_property_readonly("history",
                             [](const Board& b) {
                               const auto& h = b.history();
                               return std::vector<int>(h.begin(), h.end());
                             })
      .def_property_readonly("move_count", &Board::move_count)
      .def_property_readonly("last_moves", [](const Board& b) { return py::make_tuple(b.last1(), b.last2()); })
      .def_property_readonly("handicaps",
                             [](const Board& b) {
                               const auto& h = b.handicaps();
                               return std::vector<int>(h.begin(), h.end());
                             })
      .def_property_readonly("previous_hashes", [](const Board& b) { return b.previous_hashes(); });

  m.def(
      "batch_features",
      [](const std::vector<const Board*>& boards, const std::vector<int>& fids, int nthreads) {
        if (boards.empty()) throw std::invalid_argument("empty batch");
        const int S = boards[0]->size();
        for (auto* b : boards)
          if (b->size() != S) throw std::invalid_argument("all states must have the same size");
        const int F = total_planes(fids);
        const int B = (int)boards.size();
        py::array_t<uint8_t> a({B, F, S, S});
        uint8_t* base = a.mutable_data();
        const size_t stride = (size_t)F * S * S;
        {
          py::gil_scoped_release nogil;
          parallel_for(B, nthreads, [&](int i) {
            extract_features(*boards[i], fids.data(), (int)fids.size(), base + i * stride);
          });
        }
        return a;
      },
      py::arg("boards"), py::arg("fids"), py::arg("nthreads") = 8);

  // Inputs of the GPU feature kernel (csrc/hip/features.hip): colours, stone ages, meta
  // (player, ko), positional-superko-illegal points (only for boards that enforce superko) and,
  // when asked, the two ladder planes (native search, threaded) for legal points.
  m.def(
      "gpu_feature_inputs",
      [](const std::vector<const Board*>& boards, bool ladders, int nthreads) {
        if (boards.empty()) throw std::invalid_argument("empty batch");
        const int S = boards[0]->size(), P = S * S, B = (int)boards.size();
        for (auto* b : boards)
          if (b->size() != S) throw std::invalid_argument("all states must have the same size");
        py::array_t<int8_t> colors({B, P});
        py::array_t<int16_t> ages({B, P});
        py::array_t<int32_t> meta({B, 4});
        py::array_t<uint8_t> illegal({B, P});
        py::array_t<uint8_t> lad({ladders ? B : 0, 2, P});
        int8_t* c = colors.mutable_data();
        int16_t* a = ages.mutable_data();
        int32_t* mt = meta.mutable_data();
        uint8_t* il = illegal.mutable_data();
        uint8_t* ld = lad.mutable_data();
        bool any_superko = false;
        for (auto* b : boards) any_superko |= b->enforce_superko();
        {
          py::gil_scoped_release nogil;
          parallel_for(B, nthreads, [&](int i) {
            const Board& b = *boards[i];
            for (int p = 0; p < P; ++p) {
              c[(size_t)i * P + p] = (int8_t)b.color(p);
              a[(size_t)i * P + p] = (int16_t)std::min(b.stone_age(p), 32767);
              il[(size_t)i * P + p] = 0;
            }
            mt[i * 4 + 0] = b.current_player();
            mt[i * 4 + 1] = b.ko();
            mt[i * 4 + 2] = b.enforce_superko() ? 1 : 0;
            mt[i * 4 + 3] = 0;
            if (b.enforce_superko())
              for (int p = 0; p < P; ++p)
                if (b.color(p) == EMPTY && p != b.ko() && !b.is_suicide(p) &&
                    b.is_positional_superko(p))
                  il[(size_t)i * P + p] = 1;
            if (ladders) {
              thread_local LadderReader reader;
              uint8_t* l0 = ld + (size_t)i * 2 * P;
              ladder_planes(b, l0, l0 + P, &reader);
            }
          });
        }
        return py::make_tuple(colors, ages, meta, any_superko ? py::object(illegal) : py::none(),
                              ladders ? py::object(lad) : py::none());
      },
      py::arg("boards"), py::arg("ladders") = true, py::arg("nthreads") = 8);

  // Ladder planes [2, P] (capture, escape) of one board: the journaled single-copy reader
  // (default, ladder.cpp) or, with copying=True, the reference-shaped recursive reader that copies
  // the board at every ply (go_engine.cpp) — kept as the differential oracle.
  m.def(
      "ladder_planes",
      [](const Board& b, bool copying) {
        const int P = b.npoints();
        py::array_t<uint8_t> out({2, P});
        uint8_t* o = out.mutable_data();
        if (copying) {
          for (int p = 0; p < P; ++p) {
            o[p] = o[P + p] = 0;
            if (b.color(p) != EMPTY) continue;
            o[p] = b.is_ladder_capture(p, -1, 80) ? 1 : 0;
            o[P + p] = b.is_ladder_escape(p, -1, 80) ? 1 : 0;
          }
        } else {
          ladder_planes(b, o, o + P);
        }
        return out;
      },
      py::arg("board"), py::arg("copying") = false);

  // Bulk SGF conversion (converter.cpp): games converted in parallel on the shared pool.
  // Converts a batch of SGF texts in parallel (dynamic scheduling over games). Returns
  // (status int32 [n], rows int64 [n], states uint8 [sum rows, F, S, S], actions uint8
  // [sum rows, 2]): the games' rows in batch order in ONE block (filled by a parallel copy), so
  // the writer appends it without any per-game concatenation. Status 0 ok, 1 illegal move
  // (positions up to and including it), 3 = convert this game in python (no rows).
  m.def(
      "convert_games",
      [](const std::vector<py::bytes>& texts, const std::vector<int>& fids, int bd_size,
         py::array_t<uint64_t, py::array::c_style> zw, py::array_t<uint64_t, py::array::c_style> zb,
         int nthreads, int chunk_rows, int lead) -> py::tuple {
        auto zob = make_zobrist(zw, zb);
        static const bool timing = std::getenv("RAG_CONVERT_TIMING") != nullptr;
        auto tnow = [] { return std::chrono::steady_clock::now(); };
        auto t_0 = tnow();
        const int n = (int)texts.size();
        std::vector<std::string> buf(n);
        for (int i = 0; i < n; ++i) buf[i] = texts[i];
        std::vector<std::vector<Board>> bd(n);
        std::vector<std::vector<uint8_t>> ac(n);
        py::array_t<int32_t> status(n);
        py::array_t<int64_t> rows(n);
        int32_t* sp = status.mutable_data();
        int64_t* rp = rows.mutable_data();
        {  // 1: parse + replay every game (boards copied at the training positions)
          py::gil_scoped_release nogil;
          parallel_for(n, nthreads, [&](int i) {
            sp[i] = replay_sgf_positions(buf[i].data(), buf[i].size(), bd_size, zob, bd[i], ac[i]);
            if (sp[i] == 3) {
              bd[i].clear();
              ac[i].clear();
            }
            rp[i] = (int64_t)(ac[i].size() / 2);
          });
        }
        auto t_1 = tnow();
        const int F = total_planes(fids), P = bd_size * bd_size;
        const size_t row_bytes = (size_t)F * P;
        std::vector<int64_t> off(n + 1, 0);
        for (int i = 0; i < n; ++i) off[i + 1] = off[i] + rp[i];
        const int64_t total = off[n];
        // chunk_rows > 0 (the HDF5 writer's fused path): rows [lead, lead + k * chunk_rows) are
        // never materialised -- each whole chunk is extracted into a thread-local buffer and
        // LZF-compressed while it is cache-hot; only the `lead` rows that complete the writer's
        // pending chunk and the tail after the last whole chunk come back as planes
        const int64_t L = chunk_rows > 0 ? std::min<int64_t>(std::max(lead, 0), total) : total;
        const int64_t nfull = chunk_rows > 0 ? (total - L) / chunk_rows : 0;
        const int64_t T = total - L - nfull * (int64_t)std::max(chunk_rows, 0);
        const int64_t kept = L + T;
        py::array_t<uint8_t> sa({(py::ssize_t)kept, (py::ssize_t)F, (py::ssize_t)bd_size,
                                 (py::ssize_t)bd_size});
        py::array_t<uint8_t> aa({(py::ssize_t)total, (py::ssize_t)2});
        uint8_t* sd = sa.mutable_data();
        uint8_t* ad = aa.mutable_data();
        for (int i = 0; i < n; ++i)
          if (rp[i]) std::memcpy(ad + (size_t)off[i] * 2, ac[i].data(), (size_t)rp[i] * 2);
        std::vector<int> game_of((size_t)total);
        for (int i = 0; i < n; ++i)
          for (int64_t r = off[i]; r < off[i + 1]; ++r) game_of[(size_t)r] = i;
        const int nf = (int)fids.size();
        auto extract_row = [&](int64_t r, uint8_t* dst) {
          const int g = game_of[(size_t)r];
          extract_features(bd[g][(size_t)(r - off[g])], fids.data(), nf, dst);
        };
        std::vector<std::string> comp((size_t)nfull);
        std::vector<uint8_t> ok((size_t)nfull, 0);
        {  // 2: planes of every position (compressed whole chunks first: the larger tasks)
          py::gil_scoped_release nogil;
          const size_t cbytes = (size_t)std::max(chunk_rows, 0) * row_bytes;
          parallel_for((int)(nfull + kept), nthreads, [&](int t) {
            if (t < nfull) {
              thread_local std::vector<uint8_t> tmp;
              tmp.resize(cbytes);
              const int64_t r0 = L + (int64_t)t * chunk_rows;
              for (int k = 0; k < chunk_rows; ++k) extract_row(r0 + k, tmp.data() + k * row_bytes);
              std::string& o = comp[(size_t)t];
              o.resize(cbytes + 64);
              size_t len = lzf_compress(tmp.data(), cbytes, (uint8_t*)&o[0], cbytes);
              if (len) {
                o.resize(len);
                ok[(size_t)t] = 1;
              } else {  // incompressible: the raw chunk (stored with the filter skipped)
                o.assign((const char*)tmp.data(), cbytes);
              }
              return;
            }
            const int64_t k = t - nfull;  // kept row: lead rows, then the tail
            const int64_t r = k < L ? k : L + nfull * chunk_rows + (k - L);
            extract_row(r, sd + (size_t)k * row_bytes);
          });
        }
        auto t_2 = tnow();
        {  // the position boards go on the pool too (12k+ board destructors per batch)
          py::gil_scoped_release nogil;
          parallel_for(n, nthreads, [&](int i) { std::vector<Board>().swap(bd[i]); });
        }
        auto t_3 = tnow();
        auto report = [&] {
          if (!timing) return;
          auto ms = [](auto a, auto b) {
            return std::chrono::duration<double, std::milli>(b - a).count();
          };
          std::fprintf(stderr, "convert_games n=%d rows=%lld replay %.2f ms planes %.2f ms free %.2f "
                       "ms wrap %.2f ms\n", n, (long long)total, ms(t_0, t_1), ms(t_1, t_2),
                       ms(t_2, t_3), ms(t_3, tnow()));
        };
        if (chunk_rows <= 0) {
          report();
          return py::make_tuple(status, rows, sa, aa);
        }
        py::list chunks;
        for (int64_t t = 0; t < nfull; ++t)
          chunks.append(py::make_tuple(py::bytes(comp[(size_t)t]), (bool)ok[(size_t)t]));
        report();
        return py::make_tuple(status, rows, sa, aa, chunks, (py::ssize_t)L);
      },
      py::arg("texts"), py::arg("fids"), py::arg("bd_size"), py::arg("zobrist_white"),
      py::arg("zobrist_black"), py::arg("nthreads") = 8, py::arg("chunk_rows") = 0,
      py::arg("lead") = 0);

  // Leaf boards rebuilt from shipped arrays (distributed search workers; Board::from_arrays).
  m.def(
      "boards_from_arrays",
      [](py::array_t<int8_t, py::array::c_style> colors, py::object ages,
         py::array_t<int32_t, py::array::c_style> meta8, int S, double komi,
         py::array_t<uint64_t, py::array::c_style> zw, py::array_t<uint64_t, py::array::c_style> zb) {
        const int P = S * S;
        const int n = (int)(colors.size() / P);
        if (colors.size() != (py::ssize_t)n * P || meta8.size() < (py::ssize_t)n * 8)
          throw std::invalid_argument("colors [n, S*S] and meta8 [n, 8] expected");
        py::array_t<int16_t, py::array::c_style | py::array::forcecast> ag;
        const int16_t* ap = nullptr;
        if (!ages.is_none()) {
          ag = py::array_t<int16_t, py::array::c_style | py::array::forcecast>(ages);
          if (ag.size() != (py::ssize_t)n * P) throw std::invalid_argument("ages [n, S*S]");
          ap = ag.data();
        }
        auto zob = make_zobrist(zw, zb);
        std::vector<Board> out;
        out.reserve(n);
        for (int i = 0; i < n; ++i)
          out.push_back(Board::from_arrays(S, komi, zob, colors.data() + (size_t)i * P,
                                           ap ? ap + (size_t)i * P : nullptr,
                                           meta8.data() + (size_t)i * 8));
        return out;
      },
      py::arg("colors"), py::arg("ages"), py::arg("meta8"), py::arg("size"), py::arg("komi"),
      py::arg("zobrist_white"), py::arg("zobrist_black"));

  m.def("feature_planes", &feature_planes);

  m.def("lzf_decompress", [](py::bytes data, size_t out_size) {
    std::string in = data;
    std::string out(out_size, '\0');
    size_t n = lzf_decompress((const uint8_t*)in.data(), in.size(), (uint8_t*)out.data(), out_size);
    if (n != out_size) throw std::runtime_error("lzf: corrupt stream or size mismatch");
    return py::bytes(out);
  });
  m.def("lzf_compress", [](py::bytes data) -> py::object {
    std::string in = data;
    std::string out(in.size() + 64, '\0');
    size_t n = lzf_compress((const uint8_t*)in.data(), in.size(), (uint8_t*)out.data(), in.size());
    if (n == 0) return py::none();  // incompressible: caller stores the raw chunk
    out.resize(n);
    return py::bytes(out);
  });

  // Compress k equal-size chunks (a contiguous uint8 block [k, chunk]) in parallel on the shared
  // pool: one bytes object per chunk, None where a chunk does not compress (h5lite.WDataset
  // bulk appends).
  m.def(
      "lzf_compress_chunks",
      [](py::array_t<uint8_t, py::array::c_style> block, size_t chunk, int nthreads) {
        if (chunk == 0 || block.size() % chunk) throw std::invalid_argument("bad chunk size");
        const int k = (int)(block.size() / chunk);
        const uint8_t* src = block.data();
        std::vector<std::string> out(k);
        std::vector<size_t> len(k, 0);
        {
          py::gil_scoped_release nogil;
          parallel_for(k, nthreads, [&](int i) {
            out[i].resize(chunk + 64);
            len[i] = lzf_compress(src + (size_t)i * chunk, chunk, (uint8_t*)&out[i][0], chunk);
          });
        }
        py::list res;
        for (int i = 0; i < k; ++i) {
          if (len[i] == 0) {
            res.append(py::none());
          } else {
            out[i].resize(len[i]);
            res.append(py::bytes(out[i]));
          }
        }
        return res;
      },
      py::arg("block"), py::arg("chunk"), py::arg("nthreads") = 8);

  register_search(m);
  register_gamebatch(m);
  register_rollout(m);
  register_master(m);
}

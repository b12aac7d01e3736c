// The multi-GPU search's native half (the reference's ParallelMCTS is an empty
// stub, AlphaGo/mcts.py:219-220, and its search one sequential tree, AlphaGo/mcts.py:191-206).
//
// One tree, on rank 0; every GPU of the node evaluates leaves of it. The tree lives in host
// memory and so do the leaves' inputs and results, so between the processes of one node they
// travel through a POSIX shared-memory *channel* — no device staging, no collective per round:
//
//   * per evaluating rank, a ring of `nslots` slots. A slot carries one wave: the master writes
//     its leaves as move paths from the root (Search::write_paths, a few dozen bytes per leaf)
//     and bumps the slot's request sequence number; the rank rebuilds the boards from its own
//     copy of the root (Search::load_paths), runs features + both networks + rollouts on its
//     GPU, writes priors / values / sensible masks into the slot and bumps the value sequence,
//     and later the rollout results and the rollout sequence;
//   * the master loop (run_master) never blocks on one rank: it keeps up to `depth` waves per
//     rank waiting for values and up to `nslots` per rank holding virtual loss until their
//     rollouts return, selects the next wave for any rank with room (one parallel descent, no
//     leaf boards: Search::select(B, false)), and backs up whatever came back — straight from
//     the shared slots (no copies).
//
// Sequence numbers are 32-bit atomics in the shared mapping (lock-free, address-free); data is
// published by a release store of the sequence and read after an acquire load of it. A slot is
// reused only after its rollouts were backed up, in ring order (values and rollouts of one rank
// come back in the order the rank received its waves).
#pragma once

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstring>
#include <deque>
#include <stdexcept>
#include <string>
#include <vector>

#include "search.hpp"

namespace rag {

constexpr uint64_t kChanMagic = 0x52414743484e4c31ull;  // "RAGCHNL1"

struct alignas(64) ChanHead {
  uint64_t magic;
  uint32_t nranks, nslots, cap, P, PW, stride;
  uint64_t slot_bytes, total_bytes;
  alignas(64) std::atomic<uint32_t> cmd_seq;
  int32_t cmd, arg;
  alignas(64) std::atomic<uint32_t> abort;
  char why[120];
  alignas(64) uint32_t ring[256];  // per rank: the master's next slot (kept across searches)
  // the search's root as its game record (written by the master before the search's first
  // request): [moves, handicaps, size, superko, 2 x komi, hash, player to move, -] and the
  // handicap stones followed by the moves (PASS = -1); an evaluating rank that did not get the
  // position replays it (search/distributed.py)
  alignas(64) int64_t root_meta[8];
  int16_t root_moves[4096];
};

struct alignas(64) SlotHead {
  std::atomic<uint32_t> req_seq;  // master: a wave was posted
  uint32_t n, wave, seed;
  uint64_t root_hash;
  alignas(64) std::atomic<uint32_t> val_seq;  // rank: priors / values / sensible of req_seq
  alignas(64) std::atomic<uint32_t> z_seq;    // rank: rollout results of req_seq
};

static_assert(std::atomic<uint32_t>::is_always_lock_free, "shared atomics must be lock-free");

inline size_t align64(size_t x) { return (x + 63) & ~size_t(63); }

class ShmChannel {
 public:
  enum : int { CMD_NONE = 0, CMD_MOVE = 1, CMD_STOP = 2 };

  // Layout of one slot's body (after its SlotHead), 64-byte aligned sections.
  struct Layout {
    size_t paths, priors, values, sens, z, bytes;
  };
  static Layout layout(uint32_t cap, uint32_t P, uint32_t PW, uint32_t stride) {
    Layout L;
    size_t o = align64(sizeof(SlotHead));
    L.paths = o;
    o = align64(o + (size_t)cap * stride * sizeof(int16_t));
    L.priors = o;
    o = align64(o + (size_t)cap * PW * sizeof(float));
    L.values = o;
    o = align64(o + (size_t)cap * sizeof(float));
    L.sens = o;
    o = align64(o + (size_t)cap * P);
    L.z = o;
    o = align64(o + (size_t)cap * sizeof(float));
    L.bytes = o;
    return L;
  }

  ShmChannel(const std::string& name, bool create, uint32_t nranks = 0, uint32_t nslots = 0,
             uint32_t cap = 0, uint32_t P = 0, uint32_t PW = 0, uint32_t stride = 0)
      : name_(name) {
    if (create) {
      L_ = layout(cap, P, PW, stride);
      const size_t total = align64(sizeof(ChanHead)) + (size_t)nranks * nslots * L_.bytes;
      int fd = open_fd(name, O_CREAT | O_EXCL | O_RDWR);
      if (fd < 0) throw std::runtime_error("cannot create the search channel " + name);
      // the pages are reserved now: a full /dev/shm fails here, not as SIGBUS on a later store
      if (ftruncate(fd, (off_t)total) != 0 || posix_fallocate(fd, 0, (off_t)total) != 0) {
        close(fd);
        unlink_name(name);
        throw std::runtime_error("no room for the search channel " + name + " (" +
                                 std::to_string(total >> 20) + " MB)");
      }
      base_ = (char*)mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
      close(fd);
      if (base_ == MAP_FAILED) {
        unlink_name(name);
        throw std::runtime_error("mmap of the search channel failed");
      }
      bytes_ = total;
      owner_ = true;
      std::memset(base_, 0, align64(sizeof(ChanHead)));
      ChanHead* h = head();
      h->nranks = nranks;
      h->nslots = nslots;
      h->cap = cap;
      h->P = P;
      h->PW = PW;
      h->stride = stride;
      h->slot_bytes = L_.bytes;
      h->total_bytes = total;
      for (uint32_t i = 0; i < nranks * nslots; ++i) {
        SlotHead* s = slot(i / nslots, i % nslots);
        s->req_seq.store(0);
        s->val_seq.store(0);
        s->z_seq.store(0);
      }
      std::atomic_thread_fence(std::memory_order_seq_cst);
      __atomic_store_n(&h->magic, kChanMagic, __ATOMIC_RELEASE);
    } else {
      int fd = open_fd(name, O_RDWR);
      if (fd < 0) throw std::runtime_error("cannot attach the search channel " + name);
      struct stat st;
      if (fstat(fd, &st) != 0 || (size_t)st.st_size < sizeof(ChanHead)) {
        close(fd);
        throw std::runtime_error("search channel too small: " + name);
      }
      bytes_ = (size_t)st.st_size;
      base_ = (char*)mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
      close(fd);
      if (base_ == MAP_FAILED) throw std::runtime_error("mmap of the search channel failed");
      ChanHead* h = head();
      if (__atomic_load_n(&h->magic, __ATOMIC_ACQUIRE) != kChanMagic ||
          h->total_bytes != bytes_)
        throw std::runtime_error("not a search channel (or not initialised): " + name);
      L_ = layout(h->cap, h->P, h->PW, h->stride);
    }
  }
  ~ShmChannel() {
    if (base_ && base_ != MAP_FAILED) munmap(base_, bytes_);
    if (owner_) unlink_name(name_);
  }
  // "/name": a POSIX shared-memory object (/dev/shm); any other name: a file path (a node whose
  // /dev/shm is too small for the channel maps a file instead, search/distributed.py)
  static int open_fd(const std::string& name, int flags) {
    if (!name.empty() && name[0] == '/' && name.find('/', 1) == std::string::npos)
      return shm_open(name.c_str(), flags, 0600);
    return ::open(name.c_str(), flags, 0600);
  }
  static void unlink_name(const std::string& name) {
    if (!name.empty() && name[0] == '/' && name.find('/', 1) == std::string::npos)
      shm_unlink(name.c_str());
    else
      ::unlink(name.c_str());
  }
  ShmChannel(const ShmChannel&) = delete;
  ShmChannel& operator=(const ShmChannel&) = delete;

  ChanHead* head() const { return reinterpret_cast<ChanHead*>(base_); }
  uint32_t nranks() const { return head()->nranks; }
  uint32_t nslots() const { return head()->nslots; }
  uint32_t cap() const { return head()->cap; }
  uint32_t P() const { return head()->P; }
  uint32_t PW() const { return head()->PW; }
  uint32_t stride() const { return head()->stride; }
  const std::string& name() const { return name_; }
  void unlink() {
    if (owner_) unlink_name(name_);
    owner_ = false;
  }

  char* body(uint32_t r, uint32_t k) const {
    if (r >= nranks() || k >= nslots()) throw std::out_of_range("channel slot");
    return base_ + align64(sizeof(ChanHead)) + ((size_t)r * nslots() + k) * L_.bytes;
  }
  SlotHead* slot(uint32_t r, uint32_t k) const { return reinterpret_cast<SlotHead*>(body(r, k)); }
  int16_t* paths(uint32_t r, uint32_t k) const { return (int16_t*)(body(r, k) + L_.paths); }
  float* priors(uint32_t r, uint32_t k) const { return (float*)(body(r, k) + L_.priors); }
  float* values(uint32_t r, uint32_t k) const { return (float*)(body(r, k) + L_.values); }
  uint8_t* sens(uint32_t r, uint32_t k) const { return (uint8_t*)(body(r, k) + L_.sens); }
  float* z(uint32_t r, uint32_t k) const { return (float*)(body(r, k) + L_.z); }
  int64_t* root_meta() const { return head()->root_meta; }
  int16_t* root_moves() const { return head()->root_moves; }

  // ---- control
  void post_cmd(int cmd, int arg) {
    ChanHead* h = head();
    h->cmd = cmd;
    h->arg = arg;
    h->cmd_seq.fetch_add(1, std::memory_order_release);
  }
  void set_abort(const std::string& why) {
    ChanHead* h = head();
    if (h->abort.exchange(1) == 0) {
      std::strncpy(h->why, why.c_str(), sizeof(h->why) - 1);
      h->why[sizeof(h->why) - 1] = 0;
    }
  }
  bool aborted() const { return head()->abort.load(std::memory_order_acquire) != 0; }
  std::string why() const { return std::string(head()->why); }
  void check() const {
    if (aborted()) throw std::runtime_error("search channel aborted: " + why());
  }

  // Evaluating rank: wait until slot k of rank r carries a request newer than `last_req`
  // (returns 1), the command sequence moved past `last_cmd` (2), or `timeout_us` passed (0).
  int wait_request(uint32_t r, uint32_t k, uint32_t last_req, uint32_t last_cmd,
                   int64_t timeout_us) const {
    const SlotHead* s = slot(r, k);
    const ChanHead* h = head();
    Backoff b(timeout_us);
    while (true) {
      if (s->req_seq.load(std::memory_order_acquire) != last_req) return 1;
      if (h->cmd_seq.load(std::memory_order_acquire) != last_cmd) return 2;
      check();
      if (!b.pause()) return 0;
    }
  }
  void post_values(uint32_t r, uint32_t k) {
    SlotHead* s = slot(r, k);
    s->val_seq.store(s->req_seq.load(std::memory_order_relaxed), std::memory_order_release);
  }
  void post_z(uint32_t r, uint32_t k) {
    SlotHead* s = slot(r, k);
    s->z_seq.store(s->req_seq.load(std::memory_order_relaxed), std::memory_order_release);
  }

  // Spin briefly, then sleep in growing steps (<= 100 us), until the deadline.
  struct Backoff {
    explicit Backoff(int64_t timeout_us)
        : t0(std::chrono::steady_clock::now()), limit(timeout_us) {}
    bool pause() {
      ++k;
      if (k < 64) {
        __builtin_ia32_pause();
        return true;
      }
      const int64_t el = std::chrono::duration_cast<std::chrono::microseconds>(
                             std::chrono::steady_clock::now() - t0)
                             .count();
      if (limit >= 0 && el >= limit) return false;
      struct timespec ts{0, 1000L * std::min<int64_t>(100, 5 + (k - 64) / 8)};
      nanosleep(&ts, nullptr);
      return true;
    }
    std::chrono::steady_clock::time_point t0;
    int64_t limit;
    int64_t k = 0;
  };

 private:
  std::string name_;
  char* base_ = nullptr;
  size_t bytes_ = 0;
  bool owner_ = false;
  Layout L_{};
};

// ------------------------------------------------------------------ the master loop
struct MasterConfig {
  std::vector<int> batch;  // leaves per wave, per rank (0: the rank evaluates nothing)
  int depth = 2;           // waves per rank waiting for their values
  int nslots = 8;          // waves per rank holding virtual loss (<= the channel's slots)
  long budget = 0;         // simulations to add to the root
  uint32_t seed = 1;
  double stall_s = 120.0;  // no result from any rank for this long: abort
};

struct MasterStats {
  long waves = 0, sims = 0, rollout_waves = 0, empty_selects = 0;
  double t_select = 0, t_ship = 0, t_value = 0, t_rollout = 0, t_idle = 0, wall = 0;
  std::vector<long> leaves;  // per rank
  long max_inflight = 0;     // most leaves holding virtual loss at once
};

inline MasterStats run_master(Search& s, ShmChannel& ch, const MasterConfig& cfg) {
  using clk = std::chrono::steady_clock;
  auto secs = [](clk::time_point a, clk::time_point b) {
    return std::chrono::duration<double>(b - a).count();
  };
  const int R = (int)ch.nranks();
  if ((int)cfg.batch.size() != R) throw std::invalid_argument("one wave size per rank");
  const int nslots = std::min<int>(cfg.nslots, ch.nslots());
  const int depth = std::max(1, std::min(cfg.depth, nslots));
  const int stride = (int)ch.stride();
  const int P = s.root_board().npoints();
  if ((int)ch.P() != P) throw std::invalid_argument("channel board size differs from the tree's");
  for (int b : cfg.batch)
    if (b < 0 || b > (int)ch.cap()) throw std::invalid_argument("wave larger than a slot");
  // descents never outgrow a record
  if (s.max_depth > stride - 1) s.max_depth = stride - 1;
  const bool rollouts = s.lambda > 0.f;
  const uint64_t root_hash = s.root_board().hash();

  struct Entry {
    int slot, wid, n;
    bool value_done;
  };
  std::vector<std::deque<Entry>> q(R);
  if (R > 256) throw std::invalid_argument("at most 256 ranks");
  std::vector<int> next_slot(R, 0), vpend(R, 0);
  for (int r = 0; r < R; ++r) next_slot[r] = (int)(ch.head()->ring[r] % (uint32_t)nslots);
  // a rank whose last wave found no leaf (all in flight) is asked again only after a backup
  std::vector<uint8_t> blocked(R, 0);
  std::vector<uint32_t> seq(R * nslots, 0);
  for (int r = 0; r < R; ++r)
    for (int k = 0; k < nslots; ++k) seq[r * nslots + k] = ch.slot(r, k)->req_seq.load();
  MasterStats st;
  st.leaves.assign(R, 0);
  const long target = (long)s.root_visits() + cfg.budget;
  long queued = 0, holding = 0;
  int stall = 0, rr = 0;
  const auto t_start = clk::now();
  auto last_progress = t_start;
  ShmChannel::Backoff idle(-1);
  while (true) {
    ch.check();
    bool progress = false;
    // ---- results: value backups (in order per rank), then rollout backups (ring order)
    for (int r = 0; r < R; ++r) {
      for (Entry& e : q[r]) {
        if (e.value_done) continue;
        const SlotHead* sh = ch.slot(r, e.slot);
        if (sh->val_seq.load(std::memory_order_acquire) != seq[r * nslots + e.slot]) break;
        const auto t0 = clk::now();
        s.backup_value(e.wid, ch.priors(r, e.slot), (int)ch.PW(), ch.values(r, e.slot),
                       ch.sens(r, e.slot));
        st.t_value += secs(t0, clk::now());
        e.value_done = true;
        std::fill(blocked.begin(), blocked.end(), 0);
        --vpend[r];
        queued -= e.n;
        st.sims += e.n;
        progress = true;
      }
      while (!q[r].empty() && q[r].front().value_done) {
        Entry& e = q[r].front();
        if (rollouts) {
          const SlotHead* sh = ch.slot(r, e.slot);
          if (sh->z_seq.load(std::memory_order_acquire) != seq[r * nslots + e.slot]) break;
          const auto t0 = clk::now();
          s.backup_rollout(e.wid, ch.z(r, e.slot));
          st.t_rollout += secs(t0, clk::now());
          ++st.rollout_waves;
        }
        holding -= e.n;
        q[r].pop_front();
        std::fill(blocked.begin(), blocked.end(), 0);
        progress = true;
      }
    }
    // ---- new waves for every rank with room, round-robin start (nothing in flight: retry
    // blocked ranks, the stall counter ends a search whose tree has no leaf left)
    if (holding == 0) std::fill(blocked.begin(), blocked.end(), 0);
    for (int i = 0; i < R; ++i) {
      const int r = (rr + i) % R;
      while (!blocked[r] && cfg.batch[r] > 0 && vpend[r] < depth && (int)q[r].size() < nslots &&
             (long)s.root_visits() + queued < target) {
        const long want = std::min<long>(cfg.batch[r], target - s.root_visits() - queued);
        const auto t0 = clk::now();
        const std::pair<int, int> sel = s.select((int)want, false);
        const auto t1 = clk::now();
        st.t_select += secs(t0, t1);
        if (sel.second == 0) {
          ++st.empty_selects;
          ++stall;
          blocked[r] = 1;
          break;
        }
        stall = 0;
        const int k = next_slot[r];
        next_slot[r] = (k + 1) % nslots;
        SlotHead* sh = ch.slot(r, k);
        s.write_paths(sel.first, 0, sel.second, ch.paths(r, k), stride);
        sh->n = (uint32_t)sel.second;
        sh->wave = (uint32_t)st.waves;
        sh->seed = cfg.seed * 2654435761u + (uint32_t)st.waves;
        sh->root_hash = root_hash;
        const uint32_t nseq = seq[r * nslots + k] + 1;
        seq[r * nslots + k] = nseq;
        sh->req_seq.store(nseq, std::memory_order_release);
        st.t_ship += secs(t1, clk::now());
        q[r].push_back(Entry{k, sel.first, sel.second, false});
        ++vpend[r];
        queued += sel.second;
        holding += sel.second;
        st.max_inflight = std::max(st.max_inflight, holding);
        st.leaves[r] += sel.second;
        ++st.waves;
        progress = true;
      }
    }
    rr = (rr + 1) % R;
    bool empty = true;
    for (int r = 0; r < R; ++r) empty = empty && q[r].empty();
    if (empty && ((long)s.root_visits() >= target || stall > 3)) break;
    const auto now = clk::now();
    if (progress) {
      last_progress = now;
      idle = ShmChannel::Backoff(-1);
    } else {
      if (secs(last_progress, now) > cfg.stall_s) {
        ch.set_abort("master: no result from the evaluating ranks for " +
                     std::to_string((int)cfg.stall_s) + " s");
        ch.check();
      }
      const auto t0 = clk::now();
      idle.pause();
      st.t_idle += secs(t0, clk::now());
    }
  }
  for (int r = 0; r < R; ++r) ch.head()->ring[r] = (uint32_t)next_slot[r];
  st.wall = secs(t_start, clk::now());
  return st;
}

}  // namespace rag

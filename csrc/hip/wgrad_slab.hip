// Weight gradient of the 192-filter 3x3 trunk convolution, "all n, all taps" slab formulation.
//
// Same identity as wgrad.hip: with G and X sharing one padded geometry (halo 1, WP = S + 2),
// every tap is a constant shift in the flattened padded row space,
//
//     dW[tap][n][c] = sum_r G[r][n] * X[r + (ky-1)*WP + (kx-1)][c],
//
// and G is zero on halo rows, so the sum runs over all padded rows with no masking.
//
// wgrad.hip's 64(n) x 64(c) tiles re-stage every G row for each of 3 c-tiles and every X row for
// each of 3 n-tiles: ~39 B/clk/CU of L2 -> LDS traffic, above what an L2 gather sustains. Here a
// 768-thread block owns ALL 192 n x 32 c x 9 taps (216 MFMA tiles, 18 per wave) for a chunk of
// 64-row stages. Per stage it stages the 64 G rows (all 192 channels) and one 112-row X slab of
// its 32 channels that covers every tap's shifted window: ~18 B/clk/CU at the MFMA rate.
//
// LDS layouts (no padding; kNBUF-stage ring of 31 KB stages):
//   * G [64][192]: fragments are transposed reads (ds_read_b64_tr_b16) of 8 rows x 32 B per
//     32-lane half. Rows are 384 B (= 32 words mod 64 banks), so the 32-byte unit index is XORed
//     with row bits 1..2: the 8 rows of a half then hit 8 distinct 8-word bank windows.
//   * X [112][32]: rows are 64 B and a tap shifts the start row arbitrarily; XOR of the 16-byte
//     chunk's bit 1 with row bit 2 makes any 8 consecutive rows hit 8 distinct windows (rows r and
//     r+4 share r mod 4 and differ in bit 2).
// The MFMA k index is permuted (krow) exactly as in wgrad.hip, identically for both operands.
//
// Partials: by default each block stores its 9 x 192 x 32 accumulators as bf16 in the MFMA C
// layout ([chunk][ctile][tap][a][wave][lane][4]: one contiguous 8-byte store per lane and tile,
// 512 B per wave instruction) and wgrad_slab_reduce_kernel sums the chunks in fp32 and scatters
// to OIHW. The slab round trip (42 chunks x 1.33 MB in fp32) was ~1/4 of the wgrad time; bf16
// halves it. Each partial already sums 42 x 64 rows in fp32, so the rounding is one bf16 ulp per
// partial on a gradient that bf16 autocast training would round to bf16 as a whole.
// RAG_WGRAD_PART=fp32 keeps the fp32 part[chunk][tap][n][c] slabs + wgrad_reduce_kernel.
#include <cstring>

#include "common.h"
#include "wgrad_part.h"

using namespace rag;

namespace {

constexpr int kRows = 64;                       // padded rows per stage (two MFMA k-steps)
constexpr int kN = 192;                         // output channels (all of them) of the default
constexpr int kC = 32;                          // input channels per block
constexpr int kXRows = 112;                     // X slab rows (7 glds x 16 rows)
constexpr int kXWaves = kXRows / 16;            // waves that stage X

// Per-width layout: a block owns all N (192 | 128) output channels with N / 16 waves.
template <int N>
struct WS {
  static constexpr int GChunks = N / 8;         // 16-byte chunks per G row
  static constexpr int GElems = kRows * N;
  static constexpr int Stage = GElems + kXRows * kC;
  static constexpr int Waves = N / 16;
  static constexpr int Blk = 9 * N * kC;        // accumulators per block (fp16 partial slab)
  static_assert(kRows * GChunks == Waves * 2 * 64, "two G glds per wave");
  static_assert(Waves >= kXWaves, "seven waves stage the X slab");
  // G rows of 384 B (N = 192) are 32 words mod 64 banks: XOR the 32-byte unit with row bits 1..2;
  // rows of 256 B (N = 128) all start at bank 0: XOR it with row bits 0..2. Either way the 8 rows
  // of a transposed-read half hit 8 distinct 8-word bank windows.
  __device__ static int swz_g(int row) {
    return N == 192 ? ((row >> 1) & 3) << 1 : (row & 7) << 1;
  }
};

__device__ __forceinline__ int swz_x(int row) { return ((row >> 2) & 1) << 1; }
__device__ __forceinline__ int krow(int g, int q) { return (g & 1) * 4 + q + (g >> 1) * 8; }

// vmcnt(N) with N = `young` stages of this wave's loads (PER glds each) left in flight
template <int PER>
__device__ __forceinline__ void wait_young(int young) {
  switch (young) {
    case 0: asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(PER) : "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(2 * PER) : "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(3 * PER) : "memory"); break;
  }
}

// kNBUF-stage LDS ring, kNBUF-1 stages in flight. ALL LDS (staging and the bias reduction) lives
// in the one __shared__ array: a second __shared__ object made hipcc drain every in-flight
// global_load_lds (s_waitcnt vmcnt(0)) before the first ds_read of each stage (guide §5,
// "Projection GEMM" item 4(a); seen in this kernel's .s).
constexpr int kBlkElems = 9 * kN * kC;  // accumulators per block at the default width

// inverse block scales follow the fp16 partials of all nblk blocks in the workspace
__host__ __device__ inline float* part_scale(float* part, int nblk, int blk = kBlkElems) {
  return reinterpret_cast<float*>(reinterpret_cast<char*>(part) +
                                  (size_t)nblk * blk * sizeof(_Float16));
}

// Wave -> tile map (kMAP): the block's 12 n-frags x 2 c-frags x 9 taps = 216 MFMA tiles, 18 per
// wave. kMAP 0: 2 n-frags x 1 c-frag x 9 taps per wave (11 transposed fragment reads per k-step);
// kMAP 1: 6 n-frags x 1 c-frag x 3 taps (one kernel row; 9 reads per k-step, -18 % LDS reads).
template <int kMAP, int N = kN, int KS = 3> struct WMap {
  static_assert(kMAP == 0 || (N == 192 && KS == 3), "map 1 is the 192-channel 3x3 layout");
  static constexpr int NA = kMAP ? 6 : 2;  // n-frags per wave
  static constexpr int NT = kMAP ? 3 : (KS == 3 ? 9 : KS);  // taps per wave (5x5: one row)
  static constexpr int G = N / 32;         // map 0: wave groups along n
  __device__ static int nf0(int w) { return kMAP ? (w & 1) * 6 : (w % G) * 2; }
  __device__ static int cf(int w) { return kMAP ? (w >> 1) & 1 : w / G; }
  __device__ static int tap(int w, int i) { return kMAP ? (w >> 2) * 3 + i : i; }
};

// BNX (ResnetPolicy BN prologue, K13): X is the BN input x and the layer input is
// U = ReLU(xcoef[0][col] * x + xcoef[2][col]) (zero on halo rows). Each X-staging wave turns its
// own 16-byte chunk of every staged X slab into U in place, software-pipelined over a 4-stage ring
// so that no LDS latency sits in front of a barrier: at the end of step s it waits for stage s+2's
// loads (stage s+3 stays in flight) and issues the ds_read of its chunk; in step s+1, once the
// first k-step's fragment reads have drained (that wait covers the chunk too), it applies the BN +
// ReLU and ds_writes it back -- the slot is next read in step s+2. U is never stored in HBM.
// (Transforming stage s+1 right before barrier s+1 cost +14 %; loading the chunk to registers
// instead of LDS-DMA made the compiler drain all loads: +60 %.)
// KS = 5 (the 5x5 input layer / ResnetPolicy's first unit, halo 2): a block owns ONE kernel row
// ky (5 taps) of its c-tile, blocks ordered (chunk, c-tile, ky) so the G stages of a chunk are
// re-read from one XCD's L2; its X slab starts ky rows down (64 + 4 rows of the 112 staged).
// Partials per block: 5 x N x 32 in the map-0 C layout ("c-tile" = c-tile * 5 + ky for the
// reduction); the N bias columns are split over those 5 * ntc pseudo c-tiles. fp16 partials only.
template <int kNBUF, bool kBF, int kMAP, int N = kN, bool BNX = false, int KS = 3>
__global__ void __launch_bounds__(64 * WS<N>::Waves)
wgrad_slab_kernel(const bf16* __restrict__ G, const bf16* __restrict__ X,
                  float* __restrict__ part, float* __restrict__ bpart, int R, int WP, int GC,
                  int CIN, int spc, int CINP, const float* __restrict__ xcoef = nullptr,
                  int S = 0, int pair5 = 0, int prio = 0,
                  unsigned* __restrict__ ticket_reset = nullptr) {
  using L = WS<N>;
  static_assert(KS == 3 || (KS == 5 && kBF && kMAP == 0 && !BNX), "5x5: fp16 map-0 partials");
  constexpr int kGrp = KS == 3 ? 1 : KS;  // blocks per (chunk, c-tile): kernel rows
  constexpr int kStage = L::Stage, kGElems = L::GElems, kGChunks = L::GChunks;
  constexpr int kWaves = L::Waves, kBlk = KS == 3 ? L::Blk : L::Blk / 9 * KS,
                kThreads = 64 * kWaves;
  static_assert(!BNX || kNBUF == 4, "the BN prologue pipeline assumes a 4-stage ring");
  // BNX: a [2][64] float table of the column coefficients follows the staging ring (one
  // __shared__ object: see above)
  __shared__ __attribute__((aligned(16))) bf16 lds[kNBUF * kStage + (BNX ? 256 : 0)];
  static_assert(kNBUF * kStage * 2 >= kWaves * 64 * 4, "bias scratch fits the staging array");

  const int lane = lane_id();
  const int w = wave_id();
  const int tid = threadIdx.x;
  const int ntc = CINP / kC;
  // pair5 (5x5, <= 48 real of 64 input channels): c-tile 1 has one real c-fragment, so its
  // blocks take TWO kernel rows -- waves of c-fragment group 1 compute c-fragment 0 of row ky+1
  // (its X window lies WP rows further down the same 112-row slab): 5 + 3 blocks per chunk
  // instead of 10
  // a deferred reduction of these partials claims its units through the handle's counters in a
  // later launch of this stream: zero them here, whatever the previous claiming launch left
  if (ticket_reset && blockIdx.x == 0 && tid < 2) ticket_reset[tid] = 0u;
  const bool pr = KS == 5 && pair5;
  const int ptc = pr ? 8 : ntc * kGrp;  // (pseudo) c-tiles per chunk
  const int wid = xcd_remap(blockIdx.x, gridDim.x);  // the c-tiles of a chunk share one XCD
  const int chunk = wid / ptc;
  const int pct = wid - chunk * ptc;  // pseudo c-tile: c-tile * kGrp + ky (pr: see above)
  const bool pblk = pr && pct >= 5;
  const int ctile = pblk ? 1 : pct / kGrp;
  const int ky = pblk ? 2 * (pct - 5) : pct - ctile * kGrp;  // the slab's kernel row
  const int c0 = ctile * kC;
  const int steps = (R + kRows - 1) / kRows;
  const int sbeg = chunk * spc;
  int nsteps = steps - sbeg;
  nsteps = nsteps < spc ? nsteps : spc;
  nsteps = nsteps > 0 ? nsteps : 0;
  // X slab row 0 <-> stage row 0 shifted by tap (0, 0) (5x5: by tap (ky, 0))
  const int xshift = KS == 3 ? -(WP + 1) : (ky - 2) * WP - 2;

  // staging: G instruction i = 2w + k covers chunk slots [64 i, 64 i + 64) of the [64][24] tile;
  // X instruction w (< 7) covers slab rows [16 w, 16 w + 16)
  int grow[2], gcol[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int slot = (2 * w + k) * 64 + lane;
    const int row = slot / kGChunks;
    const int pc = slot - row * kGChunks;
    grow[k] = row;
    gcol[k] = (pc ^ L::swz_g(row)) * 8;
  }
  const int xrow = w * 16 + (lane >> 2);
  const int xcol = c0 + (((lane & 3) ^ swz_x(xrow)) * 8);
  const bool xw = w < kXWaves;

  float* tab = reinterpret_cast<float*>(lds + kNBUF * kStage);
  if constexpr (BNX) {
    if (tid < S) {
      tab[tid] = xcoef[tid];
      tab[64 + tid] = xcoef[2 * S + tid];
    }
    __syncthreads();
  }
  auto stage = [&](int s, int buf, int part = 3) {  // part: 1 the G pieces, 2 the X piece
    const int r0 = (sbeg + s) * kRows;
    bf16* lg = lds + buf * kStage;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (!(part & 1)) break;
      int r = r0 + grow[k];
      r = r < R ? r : R - 1;  // past the end: the last padded row is halo (zero)
      glds16(G + (size_t)r * GC + gcol[k], lg + (2 * w + k) * 512);
    }
    if (xw && (part & 2)) {
      int r = r0 + xshift + xrow;
      r = r < 0 ? 0 : (r < R ? r : R - 1);  // only ever paired with zero (halo) G rows
      glds16(X + (size_t)r * CIN + xcol, lg + kGElems + w * 512);
    }
  };
  // BNX: this lane's chunk of stage s's X slab (landed): xfetch issues the LDS reads (chunk and
  // column coefficients), xstore applies U = ReLU(cx x + cc) and writes it back in place
  const int WP2 = WP * WP;
  bf16x8 xv;
  float xcx = 0.f, xcc = 0.f;
  auto xslot = [&](int s) {
    return reinterpret_cast<bf16x8*>(lds + (s % kNBUF) * kStage + kGElems + w * 512 + lane * 8);
  };
  auto xfetch = [&](int s) {
    const int r = (sbeg + s) * kRows + xshift + xrow;
    xcx = 0.f;
    xcc = 0.f;
    if (r >= 0 && r < R) {
      const int rem = r % WP2, ii = rem / WP, jj = rem - (rem / WP) * WP;
      if (ii >= 1 && ii <= S && jj >= 1 && jj <= S) {
        xcx = tab[jj - 1];
        xcc = tab[64 + jj - 1];
      }
    }
    xv = *xslot(s);
  };
  auto xstore = [&](int s) {
    bf16x8 v = xv;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (bf16)fmaxf(fmaf(xcx, (float)v[e], xcc), 0.f);
    *xslot(s) = v;
  };

  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int kr = krow(g, q);
  using M = WMap<kMAP, N, KS>;
  constexpr int NA = M::NA, NT = M::NT;
  const int nf0 = M::nf0(w);  // this wave's NA 16-channel n fragments
  const int cf = pblk ? 0 : M::cf(w);    // its 16-channel c fragment
  const int dky = pblk ? M::cf(w) : 0;   // pr: its kernel row is ky + dky
  const bool idle = ky + dky >= KS;      // pr: the last pair block's second row does not exist
  int goff[NA];
#pragma unroll
  for (int a = 0; a < NA; ++a)
    goff[a] = kr * N + ((((nf0 + a) * 2 + (p >> 1)) ^ L::swz_g(kr)) * 8) + 4 * (p & 1);
  int xoff[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    const int t = M::tap(w, i);
    const int xr = KS == 3 ? kr + (t / 3) * WP + (t % 3) : kr + t + dky * WP;  // 5x5: t = kx
    xoff[i] = kGElems + xr * kC + (((cf * 2 + (p >> 1)) ^ swz_x(xr)) * 8) + 4 * (p & 1);
  }

  f32x4 acc[NT][NA];
#pragma unroll
  for (int i = 0; i < NT; ++i)
#pragma unroll
    for (int a = 0; a < NA; ++a) acc[i][a] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool do_bias = bpart != nullptr;
  const int bcol = pct * 32 + (tid & 31);  // bias columns: this (pseudo) c-tile's 32 of the N
  const int brow = tid >> 5;                 // rows brow, brow + kThreads / 32, ...
  float bsum = 0.f;

#pragma unroll
  for (int k = 0; k < kNBUF - 1; ++k)
    if (k < nsteps) stage(k, k);
  if constexpr (BNX) {
    if (xw && nsteps > 0) {  // stage 0 before the first barrier, stage 1's chunk fetched
      wait_young<3>(nsteps - 1 < 2 ? nsteps - 1 : 2);
      xfetch(0);
      xstore(0);
      if (nsteps > 1) {
        wait_young<3>(nsteps - 2 < 1 ? nsteps - 2 : 1);
        xfetch(1);
      }
    }
  }
  // prio bits 0-1: MFMA priority mode; bit 2 (RAG_WGRAD_LATE): stage s+kNBUF-1 after the first
  // k-step's MFMAs instead of right after the barrier (the LDS-DMA issues otherwise sit in front
  // of every wave's first fragment reads of the stage)
  // 0: after the barrier, 1: after k-step 0, 2: after k-step 1, 3: G after k-step 0, X after 1
  const int late = (prio >> 2) & 3;
  prio &= 3;
  if (prio == 2 && w >= kWaves - 4) __builtin_amdgcn_s_setprio(1);  // the last-dispatched waves
  for (int s = 0; s < nsteps; ++s) {
    // retire stage s; up to kNBUF-2 younger stages (2 or 3 glds of this wave each) stay in flight
    int young = nsteps - 1 - s;
    young = young < kNBUF - 2 ? young : kNBUF - 2;
    if (xw)
      wait_young<3>(young);
    else
      wait_young<2>(young);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (!late && s + kNBUF - 1 < nsteps) stage(s + kNBUF - 1, (s + kNBUF - 1) % kNBUF);
    const bf16* lb = lds + (s % kNBUF) * kStage;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ro = kk * 32;  // rows; bits 1..2 unchanged, so the swizzles are unchanged
      bf16x8 fa[NA], fb[NT];
#pragma unroll
      for (int a = 0; a < NA; ++a)
        fa[a] = tr_frag(lb + goff[a] + ro * N, lb + goff[a] + (ro + 16) * N);
#pragma unroll
      for (int i = 0; i < NT; ++i)
        fb[i] = tr_frag(lb + xoff[i] + ro * kC, lb + xoff[i] + (ro + 16) * kC);
      lds_reads_done();
      if constexpr (BNX) {
        if (kk == 0 && xw && s + 1 < nsteps) xstore(s + 1);  // fetched at the end of step s-1
      }
      if (prio == 0) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int a = 0; a < NA; ++a) acc[i][a] = mfma16(fa[a], fb[i], acc[i][a]);
      if (prio == 0) __builtin_amdgcn_s_setprio(0);
      if (s + kNBUF - 1 < nsteps) {
        if (late == kk + 1) stage(s + kNBUF - 1, (s + kNBUF - 1) % kNBUF);
        if (late == 3) stage(s + kNBUF - 1, (s + kNBUF - 1) % kNBUF, kk == 0 ? 1 : 2);
      }
    }
    if constexpr (BNX) {
      // stage s+2 landed (s+3 stays in flight): fetch this lane's chunk for step s+1's xstore
      if (xw && s + 2 < nsteps) {
        wait_young<3>(s + 3 < nsteps ? 1 : 0);
        xfetch(s + 2);
      }
    }
    if (do_bias && bcol < N) {
      for (int r = brow; r < kRows; r += kThreads / 32)
        bsum += (float)lb[r * N + (((bcol >> 3) ^ L::swz_g(r)) << 3) + (bcol & 7)];
    }
  }

  if (idle) {  // nothing to report (the reduction skips these slots)
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int a = 0; a < NA; ++a) acc[i][a] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if (kBF) {
    // scaled fp16 partials in the MFMA C layout: [chunk][ctile][i * NA + a][wave][lane][4];
    // the block's max |acc| picks a power-of-two scale into [2^14, 2^15) (wgrad_part.h)
    float mx = 0.f;
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int a = 0; a < NA; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) mx = fmaxf(mx, fabsf(acc[i][a][r]));
    mx = warp_max(mx);
    float* red = reinterpret_cast<float*>(lds);
    __syncthreads();  // every wave is done reading the staging ring
    if (lane == 0) red[w] = mx;
    __syncthreads();
    mx = red[0];
#pragma unroll
    for (int k = 1; k < kWaves; ++k) mx = fmaxf(mx, red[k]);
    // floor the exponent: a block of (near-)denormal partials must not scale by 2^(14-e) beyond
    // float range (inf * value, NaN * 0); below 2^-100 its fp16 values are 0 anyway
    const int e = mx > 0.f ? max(ilogbf(mx), -100) : 0;
    const float up = ldexpf(1.f, 14 - e);
    if (tid == 0) part_scale(part, gridDim.x, kBlk)[wid] = ldexpf(1.f, e - 14);
    f16* dst = reinterpret_cast<f16*>(part) + (size_t)wid * kBlk + (w * 64 + lane) * 4;
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int a = 0; a < NA; ++a) {
        f16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (f16)(acc[i][a][r] * up);
        *reinterpret_cast<f16x4*>(dst + (i * NA + a) * (kWaves * 256)) = o;
      }
  } else {
  // partial slab part[chunk][tap][n][c]; C layout: col = lane&15, row = 4*(lane>>4) + r
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    float* dst = part + ((size_t)(chunk * 9 + M::tap(w, i)) * N) * CINP;
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      const int n = (nf0 + a) * 16 + g * 4;
      const int cc = c0 + cf * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) dst[(size_t)(n + r) * CINP + cc] = acc[i][a][r];
    }
  }
  }
  if (do_bias) {
    float* bred = reinterpret_cast<float*>(lds);
    __syncthreads();  // every wave is done reading the staging ring
    bred[tid] = bsum;
    __syncthreads();
    if (tid < 32 && bcol < N) {
      float v = 0.f;
      for (int k = 0; k < kThreads / 32; ++k) v += bred[k * 32 + tid];
      bpart[(size_t)chunk * N + bcol] = v;
    }
  }
}

// Sums the fp16 partial slabs of wgrad_slab_kernel<.., true> over chunks in fp32 and scatters
// to OIHW dW [COUT][CIN][3][3] (+ the fp32 bias partials). A 256-thread block owns 64 "octs"
// (8 consecutive partial elements = two lanes' 4-value C fragments); its 4 waves split the chunks
// (wave s sums chunks s, s+4, ...: a 16-byte load per chunk, U in flight) and combine through
// LDS. 4x the threads of one-thread-per-oct, so the ~28 MB of partials stream at HBM rate.
constexpr int kRedSplit = 4;
static_assert(kBlkElems == ws_blk(kN) && kC == kWsC, "wgrad_part.h layout constants");
template <int U>
__global__ void __launch_bounds__(256)
wgrad_slab_reduce_kernel(WgradRed red) {
  __shared__ float part_sums[kRedSplit - 1][64][9];  // 9: odd stride, conflict-free
  const size_t slab = (size_t)red.ntc * red.blk;  // elements per chunk
  const int octs = (int)(slab / 8);
  const int oblocks = (octs + 63) / 64;
  const int tid = threadIdx.x;
  if ((int)blockIdx.x >= oblocks) {  // bias blocks
    const int n = ((int)blockIdx.x - oblocks) * 256 + tid;
    if (!red.db || !red.bpart || n >= red.COUT) return;
    float v = 0.f;
    for (int k = 0; k < red.nchunks; ++k) v += red.bpart[(size_t)k * red.n + n];
    red.db[n] = red.accumulate ? red.db[n] + v : v;
    return;
  }
  const int lo = tid & 63, sp = tid >> 6;
  int q = blockIdx.x * 64 + lo;
  const bool live = q < octs;
  q = live ? q : octs - 1;
  const uint4* p = reinterpret_cast<const uint4*>(red.part) + q;
  const float* sc = red.scale + (q * 8) / red.blk;  // + chunk * ntc
  const size_t st = slab / 8;
  float s[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = 0.f;
  int k = sp;
  for (; k + (U - 1) * kRedSplit < red.nchunks; k += U * kRedSplit) {
    uint4 a[U];
#pragma unroll
    for (int j = 0; j < U; ++j) a[j] = p[(size_t)(k + j * kRedSplit) * st];
#pragma unroll
    for (int j = 0; j < U; ++j) wslab_add8(s, a[j], sc[(k + j * kRedSplit) * red.ntc]);
  }
  for (; k < red.nchunks; k += kRedSplit) wslab_add8(s, p[(size_t)k * st], sc[k * red.ntc]);
  if (sp > 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) part_sums[sp - 1][lo][j] = s[j];
  }
  __syncthreads();
  if (sp > 0 || !live) return;
#pragma unroll
  for (int r = 0; r < kRedSplit - 1; ++r)
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] += part_sums[r][lo][j];
  wslab_store_oct(red, q, s);
}

}  // namespace

// Applicability: 3x3, G and X both halo 1, 192 output channels, CINP == 192 (its six 32-channel
// c-tiles also split the 192 bias columns), and the X slab covering every tap window of a stage
// (64 + 2*WP + 2 <= 112). RAG_WGRAD_SLAB=0 disables it.
bool rag_wgrad_slab_bf16();
bool rag_wgrad_slab_ok(int S, int H, int HG, int GC, int COUTP, int CINP, int KS) {
  static const bool on = [] {
    const char* e = getenv("RAG_WGRAD_SLAB");
    return !(e && e[0] == '0');
  }();
  const int WP = S + 2 * H;
  if (!on || (COUTP != 192 && COUTP != 128) || GC % 8 || GC < COUTP || CINP % kC) return false;
  if (KS == 3)
    return H == 1 && HG == 1 && CINP == COUTP && kRows + 2 * WP + 2 <= kXRows;
  // 5x5: per-row blocks; the 5 * CINP / 32 pseudo c-tiles must cover the COUTP bias columns
  return KS == 5 && rag_wgrad_slab_bf16() && H == 2 && HG == 2 &&
         5 * CINP >= COUTP && kRows + 4 <= kXRows;
}

// Chunks of 64-row stages: one resident block per CU (256) over all c-tiles.
int rag_wgrad_slab_nchunks(int R, int CINP, int* spc, int KS, int pair5) {
  const int steps = (R + kRows - 1) / kRows;
  int nc = 256 / (KS == 5 && pair5 ? 8 : CINP / kC * (KS == 5 ? 5 : 1));
  nc = nc < steps ? nc : steps;
  nc = nc > 0 ? nc : 1;
  const int s = (steps + nc - 1) / nc;
  if (spc) *spc = s;
  return (steps + s - 1) / s;
}

static int g_wslab_bf = -1;    // block-scaled fp16 partial slabs unless RAG_WGRAD_PART=fp32
static int g_wslab_map = -1;   // wave -> tile map (WMap), RAG_WGRAD_MAP

static int wslab_map() {
  if (g_wslab_map < 0) {
    const char* e = getenv("RAG_WGRAD_MAP");
    g_wslab_map = e ? (atoi(e) != 0) : 1;
  }
  return g_wslab_map;
}

RAG_API int rag_wgrad_slab_map(int m) {
  const int old = g_wslab_map;
  g_wslab_map = m;
  return old;
}

RAG_API int rag_wgrad_slab_part_bf16(int on) {
  const int old = g_wslab_bf;
  g_wslab_bf = on;
  return old;
}

bool rag_wgrad_slab_bf16() {
  if (g_wslab_bf < 0) {
    const char* e = getenv("RAG_WGRAD_PART");
    g_wslab_bf = (e && strcmp(e, "fp32") == 0) ? 0 : 1;
  }
  return g_wslab_bf != 0;
}

WgradRed rag_wgrad_slab_red(const void* part, const float* bpart, float* dW, float* db,
                            int nchunks, int CINP, int COUTP, int COUT, int CIN, int accumulate,
                            int KS, int pair5) {
  WgradRed r{};  // ticket null: a static split unless the deferral hands it claim counters
  r.part = (const f16*)part;
  r.bpart = bpart;
  r.dW = dW;
  r.db = db;
  r.nchunks = nchunks;
  r.kgrp = KS == 5 ? 5 : 1;
  r.taps = KS * KS;
  r.pair5 = KS == 5 && pair5;
  r.ntc = r.pair5 ? 8 : CINP / kC * r.kgrp;  // (pseudo) c-tiles per chunk
  r.COUT = COUT;
  r.CIN = CIN;
  r.accumulate = accumulate;
  r.n = COUTP;  // the block's (pseudo) c-tiles also split the N bias columns
  r.waves = COUTP / 16;
  r.blk = KS == 5 ? 5 * COUTP * kC : ws_blk(COUTP);
  r.scale = part_scale((float*)part, nchunks * r.ntc, r.blk);
  r.map = (COUTP == kN && KS == 3) ? wslab_map() : 0;
  return r;
}

// Where the slab kernels issue a stage's LDS-DMA (prio bits 2-3): after the first k-step's MFMAs
// -- SL 110.2-110.7k -> 113.5-114.0k positions/s on one box against right after the stage
// barrier (profiles/dma_placement_r4.txt; "after the second" measured no better) -- and the
// per-segment priority flips around the MFMAs (prio bits 0-1 = 0; none / static: no faster).
constexpr int kWslabPrio = 1 << 2;

int rag_launch_wgrad_slab_reduce(const WgradRed& r, hipStream_t stream) {
  const int octs = (int)((size_t)r.ntc * r.blk / 8);
  const int blocks = (octs + 63) / 64 + (r.n + 255) / 256;
  wgrad_slab_reduce_kernel<4><<<blocks, 256, 0, stream>>>(r);
  return (int)hipGetLastError();
}

int rag_launch_wgrad_slab(const bf16* G, const bf16* X, float* part, float* bpart, int R, int WP,
                          int GC, int CIN, int spc, int CINP, int nchunks, hipStream_t stream,
                          const float* xcoef, int S, int KS, int COUTP, int pair5,
                          unsigned* ticket_reset) {
  const bool bf = rag_wgrad_slab_bf16();
  if (!bf) ticket_reset = nullptr;  // fp32 partials are never deferred
  if (KS == 5) {  // per-row blocks, fp16 partials, map 0
    if (!bf || xcoef) return -5;
    if (pair5 && CINP != 2 * kC) return -5;
    const dim3 g5(nchunks * (pair5 ? 8 : (CINP / kC) * 5));
    if (COUTP == 192)
      wgrad_slab_kernel<3, true, 0, 192, false, 5><<<g5, 768, 0, stream>>>(
          G, X, part, bpart, R, WP, GC, CIN, spc, CINP, nullptr, 0, pair5, kWslabPrio,
          ticket_reset);
    else if (COUTP == 128)
      wgrad_slab_kernel<3, true, 0, 128, false, 5><<<g5, 512, 0, stream>>>(
          G, X, part, bpart, R, WP, GC, CIN, spc, CINP, nullptr, 0, pair5, kWslabPrio,
          ticket_reset);
    else
      return -5;
    return (int)hipGetLastError();
  }
  const dim3 grid(nchunks * (CINP / kC));
  if (xcoef) {  // BN prologue: 128 channels, fp16 partials
    if (CINP != 128 || !bf || S > 64) return -5;
    wgrad_slab_kernel<4, true, 0, 128, true><<<grid, 512, 0, stream>>>(G, X, part, bpart, R, WP,
                                                                       GC, CIN, spc, CINP, xcoef,
                                                                       S, 0, kWslabPrio,
                                                                       ticket_reset);
    return (int)hipGetLastError();
  }
  if (CINP == 128) {  // 8 waves, map 0
    if (bf)
      wgrad_slab_kernel<3, true, 0, 128><<<grid, 512, 0, stream>>>(G, X, part, bpart, R, WP, GC,
                                                                   CIN, spc, CINP, nullptr, 0, 0,
                                                                   kWslabPrio, ticket_reset);
    else
      wgrad_slab_kernel<3, false, 0, 128><<<grid, 512, 0, stream>>>(G, X, part, bpart, R, WP, GC,
                                                                    CIN, spc, CINP);
    return (int)hipGetLastError();
  }
  // 192 channels: a 3-stage ring (4 / 5 measured no faster, deleted round 5); A/B axes: the
  // fp32 partial slabs (RAG_WGRAD_PART=fp32) and the wave -> tile map (RAG_WGRAD_MAP=0)
#define RAG_WSLAB(BF, MP)                                                                       \
  wgrad_slab_kernel<3, BF, MP><<<grid, 64 * WS<kN>::Waves, 0, stream>>>(                       \
      G, X, part, bpart, R, WP, GC, CIN, spc, CINP, nullptr, 0, 0, kWslabPrio, ticket_reset)
  const int mp = wslab_map();
  if (bf && mp) RAG_WSLAB(true, 1);
  else if (bf) RAG_WSLAB(true, 0);
  else if (mp) RAG_WSLAB(false, 1);
  else RAG_WSLAB(false, 0);
#undef RAG_WSLAB
  return (int)hipGetLastError();
}

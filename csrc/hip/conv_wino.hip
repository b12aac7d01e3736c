// Winograd F(2,3) along the board width: the 3x3 trunk convolution (forward and dgrad) with a
// third fewer MFMAs than the direct implicit GEMM (conv_tap.hip).
//
// Math (one board row, a pair of output columns j = 2t, 2t+1; padded input d_s = X[row][2t + s],
// s = 0..3; weights g_kx of one kernel row ky; reference op: policy.py's Convolution2D stack):
//   V0 = d0 - d2   V1 = d1 + d2   V2 = d2 - d1   V3 = d1 - d3            (input transform)
//   U0 = g0        U1 = (g0+g1+g2)/2   U2 = (g0-g1+g2)/2   U3 = g2        (weights, packed)
//   M_q = sum_{ky, c} V_q[row i+ky][t][c] * U_{ky,q}[n][c]                 (four GEMMs, K = 3C)
//   y(2t) = M0 + M1 + M2      y(2t+1) = M1 - M2 - M3
// 12 GEMM taps (ky, q) per output pair instead of 18 direct taps per two pixels: 2/3 of the MFMA
// work. The transform mixes only +-1 terms (one bf16 rounding of V, exact U up to the bf16
// rounding of (g0+-g1+g2)/2); tests/test_wino.py pins it against fp32 F.conv2d.
//
// Accumulators: the loop runs the q = 1 and q = 2 GEMMs first into A and B (M1, M2), turns them
// into (M1 + M2, M1 - M2) in registers, then accumulates q = 0 into A and q = 3 into B with
// V3' = d3 - d1 = -V3: A = y(2t), B = y(2t+1). Two accumulator sets per output pair = one per
// pixel, the same register budget as the direct kernel, so one block still covers a whole board.
//
// Block: one 19x19 board (190 output pairs, padded to 192 = 4 wave rows x 48) x 192 output
// channels (2 wave columns x 96), 8 waves in two ping-pong groups of 4 (conv_tap_pp_kernel's
// structure: per K-step two raw s_barriers X / Y; group 0 reads fragments while group 1 runs its
// MFMAs and the other way round). Smaller boards pack several per block (nb boards, host side).
// K-steps: 2 phases x (C/32) chunks x 2 slots x 3 ky = 72 for C = 192, 18 MFMAs (48 x 96 x 32)
// per wave per step from 3 V fragments + 6 weight fragments.
//
// Per 32-channel chunk-phase k (phase = k / chunks, chunk = k % chunks):
//   * raw slab: the block's padded input rows (board rows x 21 columns, 64 B each), staged by
//     group 0 with LDS-DMA two chunk-phases ahead (double buffered);
//   * V slab: V for the two slots of the phase, [vrow = (board row) x 10 + t][32 ch], built from
//     the raw slab one chunk-phase ahead by every wave (2 or 4 LDS reads, the +- in fp32, one
//     16-byte store per slot), double buffered. A fragment of 16 consecutive output pairs reads
//     16 consecutive V rows (no halo columns in between, unlike the pixel slab of the direct
//     kernel, whose fragments straddle board-row ends): the row-bit-2 swizzle keeps it
//     conflict-free;
//   * weights: one [192 n][32 c] tile per step through a 3-deep ring, staged by group 1.
// LDS: 4 x 14 KB (V) + 2 x 32 KB (raw) + 3 x 12 KB (weights) = 156 KB -> one block per CU.
#include "common.h"
#include "wgrad_part.h"

using namespace rag;

namespace {

constexpr int kWK = 32;                  // channels per chunk (MFMA K)
constexpr int kWMT = 3, kWNT = 6;        // fragments per wave along pairs / output channels
constexpr int kWP = 64 * kWMT;           // 192 output pairs per block (4 wave rows)
constexpr int kWN = 32 * kWNT;           // 192 output channels per block (2 wave columns)
constexpr int kVRows = 224;              // V slab rows (a 19x19 board: 21 x 10 = 210)
constexpr int kRRows = 512;              // raw slab rows (a 19x19 board: 21 x 21 + 1 = 442)
constexpr int kWRing = 3;                // weight tiles in flight / being read
constexpr int kVSlot = kVRows * kWK;
constexpr int kRSlab = kRRows * kWK;
constexpr int kWTile = kWN * kWK;
constexpr int kOffR = 4 * kVSlot;        // V: [2 chunk-phase buffers][2 slots]
constexpr int kOffW = kOffR + 2 * kRSlab;
constexpr int kLoopLds = kOffW + kWRing * kWTile;
constexpr int kEpRow = kWN + 8;          // bf16 per row of the epilogue image
constexpr int kEpImg = 2 * kWP * kEpRow; // one image row per output pixel (pair, column)
constexpr int kLdsElems = kLoopLds > kEpImg ? kLoopLds : kEpImg;
constexpr int kRawPieces = kRRows / 64;  // 16-row LDS-DMA pieces per group-0 wave per chunk
constexpr int kWPieces = kWN / 64;       // weight pieces per group-1 wave per step
constexpr int kRedU = 14;                // chunk loads in flight per reduce thread
static_assert(kLdsElems * 2 <= 160 * 1024, "LDS budget");
static_assert(kRawPieces == 8, "raw pieces are issued two per step over steps 0..3");

__device__ __forceinline__ int swz4w(int row) { return ((row >> 2) & 1) << 1; }

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ bf16x8 vsum(const bf16x8& a, const bf16x8& b) {
  bf16x8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = (bf16)((float)a[e] + (float)b[e]);
  return o;
}
__device__ __forceinline__ bf16x8 vdiff(const bf16x8& a, const bf16x8& b) {
  bf16x8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = (bf16)((float)a[e] - (float)b[e]);
  return o;
}

// X: padded input [B][S+2][S+2][KIN] (halo 1). U: Winograd weights [12 = (ky, q)][NOUT][KIN].
// Y: padded output (halo HO, YC channels); mask: the dgrad ReLU mask (halo HM) or null.
// Block (x, y): boards [x * nb, x * nb + nb), output channels [192 y, 192 y + 192).
// DIAG (timing builds, WRONG results): bit 0 no transform in the loop, bit 1 no raw staging,
// bit 2 no weight staging, bit 3 no MFMAs, bit 4 no fragment reads, bit 5 no epilogue stores;
// bit 6 (results correct): per-wave s_memtime segment sums of the loop into `stamps`.
template <int DIAG = 0>
__global__ void __launch_bounds__(512, 1)
conv_wino_kernel(const bf16* __restrict__ X, const bf16* __restrict__ U,
                 const float* __restrict__ bias, bf16* __restrict__ Y,
                 const bf16* __restrict__ mask, int B, int S, int KIN, int NOUT, int HO, int YC,
                 int relu, int HM, int nb, WgradRed red, long long* stamps = nullptr) {
  __shared__ __attribute__((aligned(16))) bf16 lds[kLdsElems];
  long long seg[6] = {0, 0, 0, 0, 0, 0};
  auto now = [&]() -> long long {
    if constexpr ((DIAG & 64) != 0) return __builtin_amdgcn_s_memtime();
    return 0;
  };
  const int lane = lane_id();
  const int w = wave_id();
  const int grp = w >> 2;  // waves w and w + 4 share a SIMD
  const int wl = w & 3;
  const int wm = grp * 2 + (wl & 1), wn = wl >> 1;
  const int frow = lane & 15, fq = lane >> 4;
  const int WI = S + 2, TJ = (S + 1) >> 1;
  const int PB = S * TJ;    // output pairs per board
  const int VPB = WI * TJ;  // V rows per board
  const int RPB = WI * WI;  // raw rows per board
  const int b0 = blockIdx.x * nb;
  const int n0 = blockIdx.y * kWN;
  const long total_rows = (long)B * RPB;
  const int cchunks = KIN / kWK;
  const int NK = 2 * cchunks;      // chunk-phases
  const int nsteps = 6 * NK;

  // ---- per-lane fragment offsets
  int vb[kWMT];  // V row of this lane's output pair (tap ky adds ky * TJ)
#pragma unroll
  for (int i = 0; i < kWMT; ++i) {
    int m = wm * (16 * kWMT) + i * 16 + frow;
    m = m < nb * PB ? m : nb * PB - 1;  // pad pairs read a valid row, their output is dropped
    const int bl = m / PB, rem = m - bl * PB;
    const int ii = rem / TJ, t = rem - ii * TJ;
    vb[i] = (bl * WI + ii) * TJ + t;
  }
  // weight fragment j: tile row wn * 96 + 16 j + frow; the swizzle depends on row bit 2 only
  // (= frow bit 2), so fragment j sits at a constant 16 * 32 * j elements from fragment 0
  const int boff0 = (wn * (16 * kWNT) + frow) * kWK + ((fq ^ swz4w(frow)) * 8);
  // ---- transform units of this thread (the same for every chunk-phase): V row, 8-channel group,
  // raw row of d0
  const int NU = nb * VPB * 4;
  // (named scalars, not arrays: a runtime-indexed array went to scratch)
  int tv0, tk0, tr0, tv1, tk1, tr1;
  auto unit = [&](int it, int& tv, int& tk, int& tr) {
    const int u = threadIdx.x + it * 512;
    const int v = u >> 2;
    tk = u & 3;
    tv = u < NU ? v : -1;
    const int bl = v / VPB, rem = v - bl * VPB;
    const int r = rem / TJ, t = rem - r * TJ;
    tr = (bl * WI + r) * WI + 2 * t;
  };
  unit(0, tv0, tk0, tr0);
  unit(1, tv1, tk1, tr1);
  // Both of this thread's units of V(kk) from raw(kk) in one pass: all LDS reads first, then
  // the arithmetic, then the stores (one unit at a time was a dependent read -> add -> write
  // chain of ~1000 cycles per call).
  auto transform2 = [&](int kk) {
    int v0 = tv0, k0 = tk0, r0 = tr0, v1 = tv1, k1 = tk1, r1 = tr1;
    asm volatile("" : "+v"(v0), "+v"(k0), "+v"(r0), "+v"(v1), "+v"(k1), "+v"(r1));
    if (v0 < 0) return;         // (boards of S = 2: NU < 512)
    const bool has1 = v1 >= 0;  // unit 1 may be past the end
    if (!has1) {
      v1 = v0;
      k1 = k0;
      r1 = r0;
    }
    const bf16* raw = lds + kOffR + (kk & 1) * kRSlab;
    auto ld = [&](int row, int k8) {
      return *reinterpret_cast<const bf16x8*>(raw + row * kWK + ((k8 ^ swz4w(row)) * 8));
    };
    bf16x8 a0, b0v, a1, b1;
    if (kk < cchunks) {  // phase 1: V1 = d1 + d2, V2 = d2 - d1
      const bf16x8 p1 = ld(r0 + 1, k0), p2 = ld(r0 + 2, k0);
      const bf16x8 q1 = ld(r1 + 1, k1), q2 = ld(r1 + 2, k1);
      a0 = vsum(p1, p2);
      b0v = vdiff(p2, p1);
      a1 = vsum(q1, q2);
      b1 = vdiff(q2, q1);
    } else {  // phase 2: V0 = d0 - d2, V3' = d3 - d1
      const bf16x8 p0 = ld(r0, k0), p1 = ld(r0 + 1, k0), p2 = ld(r0 + 2, k0),
                   p3 = ld(r0 + 3, k0);
      const bf16x8 q0 = ld(r1, k1), q1 = ld(r1 + 1, k1), q2 = ld(r1 + 2, k1),
                   q3 = ld(r1 + 3, k1);
      a0 = vdiff(p0, p2);
      b0v = vdiff(p3, p1);
      a1 = vdiff(q0, q2);
      b1 = vdiff(q3, q1);
    }
    bf16* vs = lds + (kk & 1) * 2 * kVSlot;
    const int o0 = v0 * kWK + ((k0 ^ swz4w(v0)) * 8);
    const int o1 = v1 * kWK + ((k1 ^ swz4w(v1)) * 8);
    *reinterpret_cast<bf16x8*>(vs + o0) = a0;
    *reinterpret_cast<bf16x8*>(vs + kVSlot + o0) = b0v;
    if (has1) {
      *reinterpret_cast<bf16x8*>(vs + o1) = a1;
      *reinterpret_cast<bf16x8*>(vs + kVSlot + o1) = b1;
    }
  };

  // ---- staging: raw slab (group 0), weight tiles (group 1)
  // Every LDS-DMA source is a wave-uniform base (SGPRs) plus this lane's 32-bit byte offset,
  // so a piece issues as `global_load_lds_dwordx4 v_off, s[base]` with one VALU add: with
  // per-lane 64-bit addresses (and the raw rows' clamp) each 1 KB piece cost 150-220 cycles of
  // the issuing wave (s_memtime segments), and hoisted they were 11 live pointers (spills).
  // Lane (lrow, lcol) of piece p stages row 64 p + 16 wl + lrow, 16-byte chunk lcol ^ swz
  // (the swizzle depends on row bit 2 only, the same for every piece).
  const int lrow = lane >> 2, lcol = lane & 3;
  const int prow0 = wl * 16 + lrow;
  const uint32_t loff_r = (uint32_t)(prow0 * KIN + ((lcol ^ swz4w(prow0)) * 8)) * 2u;
  const uint32_t piece_r = (uint32_t)(64 * KIN) * 2u;  // bytes between pieces
  // the block's raw rows run past the tensor's end only in the last block(s): clamp there only
  const int rowlim = (int)(total_rows - (long)b0 * RPB) - 1;  // last valid raw row of the block
  const bool raw_fits = rowlim >= kRRows - 1;
  auto stage_raw = [&](int kk, int p0, int p1) {  // pieces p0 .. p1-1 of raw(kk)
    if ((DIAG & 2) && kk >= 2) return;
    bf16* dst = lds + kOffR + (kk & 1) * kRSlab + wl * 16 * kWK;
    const int c = kk % cchunks;
    const char* xb = reinterpret_cast<const char*>(X + ((long)b0 * RPB) * KIN + c * kWK);
#pragma unroll
    for (int p = 0; p < kRawPieces; ++p) {
      if (p < p0 || p >= p1) continue;
      if (raw_fits) {
        glds16(xb + (loff_r + p * piece_r), dst + p * 64 * kWK);
      } else {
        const int r = prow0 + 64 * p;
        const int rc = r < rowlim ? r : rowlim;
        glds16(xb + (uint32_t)(rc * KIN + ((lcol ^ swz4w(r)) * 8)) * 2u, dst + p * 64 * kWK);
      }
    }
  };
  const long tap_stride = (long)NOUT * KIN;
  const uint32_t loff_w = loff_r;  // weight rows: the same lane -> (row, chunk) map
  // step s -> chunk-phase kk, slot (0: accumulator A, 1: B), ky
  auto stage_w = [&](int s) {
    if ((DIAG & 4) && s >= 2) return;
    const int kk = s / 6, u = s - kk * 6;
    const int slot = u / 3, ky = u - slot * 3;
    const int q = kk < cchunks ? 1 + slot : 3 * slot;  // phase 1: q = 1, 2; phase 2: q = 0, 3
    bf16* dst = lds + kOffW + (s % kWRing) * kWTile + wl * 16 * kWK;
    const char* ub = reinterpret_cast<const char*>(
        U + (ky * 4 + q) * tap_stride + (long)n0 * KIN + (kk % cchunks) * kWK);
#pragma unroll
    for (int k = 0; k < kWPieces; ++k) glds16(ub + (loff_w + k * piece_r), dst + k * 64 * kWK);
  };

  f32x4 accA[kWNT][kWMT], accB[kWNT][kWMT];
#pragma unroll
  for (int j = 0; j < kWNT; ++j)
#pragma unroll
    for (int i = 0; i < kWMT; ++i) {
      accA[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
      accB[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  bf16x8 xa[kWMT], wb[kWNT];
  auto read_frags = [&](int s) {
    if constexpr ((DIAG & 16) != 0) {
      asm volatile("" : "+v"(xa[0]), "+v"(wb[0]));
      return;
    }
    const int kk = s / 6, u = s - kk * 6;
    const int slot = u / 3, ky = u - slot * 3;
    const bf16* vs = lds + ((kk & 1) * 2 + slot) * kVSlot;
    const bf16* wt = lds + kOffW + (s % kWRing) * kWTile;
    const int sh = ky * TJ;
#pragma unroll
    for (int i = 0; i < kWMT; ++i) {
      // opaque per step: hoisted, the (fragment, ky) addresses were loop-invariant registers
      asm volatile("" : "+v"(vb[i]));
      const int r = vb[i] + sh;
      xa[i] = *reinterpret_cast<const bf16x8*>(vs + r * kWK + ((fq ^ swz4w(r)) * 8));
    }
#pragma unroll
    for (int j = 0; j < kWNT; ++j)
      wb[j] = *reinterpret_cast<const bf16x8*>(wt + boff0 + j * 16 * kWK);
    lds_reads_done();  // retire the burst (and any transform writes) before the next barrier
  };
  auto mfmas = [&](int u) {  // u = the step's index within its chunk-phase (a constant)
    if constexpr ((DIAG & 8) != 0) {
      asm volatile("" : "+v"(xa[0]), "+v"(wb[0]), "+v"(xa[1]), "+v"(wb[1]));
      return;
    }
    if (u < 3) {
#pragma unroll
      for (int j = 0; j < kWNT; ++j)
#pragma unroll
        for (int i = 0; i < kWMT; ++i) accA[j][i] = mfma16(wb[j], xa[i], accA[j][i]);
    } else {
#pragma unroll
      for (int j = 0; j < kWNT; ++j)
#pragma unroll
        for (int i = 0; i < kWMT; ++i) accB[j][i] = mfma16(wb[j], xa[i], accB[j][i]);
    }
  };
  auto butterfly = [&]() {  // (M1, M2) -> (M1 + M2, M1 - M2)
#pragma unroll
    for (int j = 0; j < kWNT; ++j)
#pragma unroll
      for (int i = 0; i < kWMT; ++i) {
        const f32x4 a = accA[j][i], b = accB[j][i];
        accA[j][i] = a + b;
        accB[j][i] = a - b;
      }
  };
  // after this wave's MFMAs of step s: the butterfly at the phase boundary, and the transform
  // units of V(kk + 1) at steps u = 1 and 3 of chunk-phase kk
  auto after_mfmas = [&](int kk, int u) {
    if (u == 5 && kk == NK / 2 - 1) butterfly();
    if (kk + 1 < NK && !(DIAG & 1) && u == 1) transform2(kk + 1);
  };

  // ---- prologue: raw(0), raw(1) and V(0) (every wave), B(0), B(1)
  if (grp == 0) {
    stage_raw(0, 0, kRawPieces);
    stage_raw(1, 0, kRawPieces);
    wait_vm<kRawPieces>();  // raw(0) landed (raw(1)'s pieces are younger)
  } else {
    stage_w(0);
    stage_w(1);
  }
  __builtin_amdgcn_s_barrier();  // raw(0) visible
  asm volatile("" ::: "memory");
  transform2(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (grp == 0)
    wait_vm<0>();           // raw(1)
  else
    wait_vm<kWPieces>();    // B(0) (B(1) younger)

  if (grp == 0) {
#pragma unroll 1
    for (int kk = 0; kk < NK; ++kk)
#pragma unroll
    for (int u = 0; u < 6; ++u) {  // unrolled: the slot (accumulator) and ky are constants
      const int s = kk * 6 + u;
      const long long c0 = now();
      __builtin_amdgcn_s_barrier();  // X_s
      asm volatile("" ::: "memory");
      const long long c1 = now();
      if (u < 4 && kk + 2 < NK) stage_raw(kk + 2, 2 * u, 2 * u + 2);
      const long long c2 = now();
      read_frags(s);
      const long long c3 = now();
      __builtin_amdgcn_s_barrier();  // Y_s
      asm volatile("" ::: "memory");
      const long long c4 = now();
      mfmas(u);
      const long long c5 = now();
      after_mfmas(kk, u);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // transform writes before X_{s+1}
      if (u == 5 && kk + 2 < NK) wait_vm<0>();           // raw(kk+2) before chunk-phase kk+1
      if constexpr ((DIAG & 64) != 0) {  // X wait, staging, reads, Y wait, MFMA issue, post
        const long long c6 = now();
        seg[0] += c1 - c0; seg[1] += c2 - c1; seg[2] += c3 - c2;
        seg[3] += c4 - c3; seg[4] += c5 - c4; seg[5] += c6 - c5;
      }
    }
  } else {
    __builtin_amdgcn_s_setprio(1);  // static priority for the younger half
#pragma unroll 1
    for (int kk = 0; kk < NK; ++kk)
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      const int s = kk * 6 + u;
      const long long c0 = now();
      __builtin_amdgcn_s_barrier();  // X_s
      asm volatile("" ::: "memory");
      const long long c1 = now();
      long long c2 = c1;
      if (s > 0) {  // step s - 1, beside group 0's reads of step s
        mfmas(u == 0 ? 5 : u - 1);
        c2 = now();
        after_mfmas(u == 0 ? kk - 1 : kk, u == 0 ? 5 : u - 1);
      }
      const long long c3 = now();
      __builtin_amdgcn_s_barrier();  // Y_s
      asm volatile("" ::: "memory");
      const long long c4 = now();
      read_frags(s);  // beside group 0's MFMAs of step s (also retires the transform writes)
      const long long c5 = now();
      if (s + 2 < nsteps) {
        stage_w(s + 2);
        wait_vm<kWPieces>();  // B(s+1) complete before X_{s+1}: B(s+2) is younger
      } else {
        wait_vm<0>();
      }
      if constexpr ((DIAG & 64) != 0) {  // X wait, MFMA issue, transform, Y wait, reads, stage
        const long long c6 = now();
        seg[0] += c1 - c0; seg[1] += c2 - c1; seg[2] += c3 - c2;
        seg[3] += c4 - c3; seg[4] += c5 - c4; seg[5] += c6 - c5;
      }
    }
    mfmas(5);
    __builtin_amdgcn_s_setprio(0);
  }
  if constexpr ((DIAG & 64) != 0) {
    if (lane == 0 && stamps) {
      long long* o = stamps + ((size_t)blockIdx.x * 8 + w) * 6;
#pragma unroll
      for (int k = 0; k < 6; ++k) o[k] = seg[k];
    }
  }

  // ---- epilogue: bias (+ ReLU) -> bf16 image [pair][column][channel] in LDS, then whole
  // 384-byte pixel rows out with the dgrad mask applied
  __syncthreads();  // every wave is past its last LDS read
#pragma unroll
  for (int j = 0; j < kWNT; ++j) {
    const int n = wn * (16 * kWNT) + j * 16 + fq * 4;
    float4 bb = {0.f, 0.f, 0.f, 0.f};
    if (bias) bb = *reinterpret_cast<const float4*>(bias + n0 + n);
#pragma unroll
    for (int i = 0; i < kWMT; ++i) {
      const int m = wm * (16 * kWMT) + i * 16 + frow;
      bf16x4 oa, ob;
      const float va[4] = {accA[j][i][0] + bb.x, accA[j][i][1] + bb.y, accA[j][i][2] + bb.z,
                           accA[j][i][3] + bb.w};
      const float vb4[4] = {accB[j][i][0] + bb.x, accB[j][i][1] + bb.y, accB[j][i][2] + bb.z,
                            accB[j][i][3] + bb.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        oa[r] = (bf16)(relu ? fmaxf(va[r], 0.f) : va[r]);
        ob[r] = (bf16)(relu ? fmaxf(vb4[r], 0.f) : vb4[r]);
      }
      *reinterpret_cast<bf16x4*>(lds + (2 * m) * kEpRow + n) = oa;
      *reinterpret_cast<bf16x4*>(lds + (2 * m + 1) * kEpRow + n) = ob;
    }
  }
  __syncthreads();
  {
    const int nbl = B - b0 < nb ? B - b0 : nb;
    const int S2 = S * S, WO = S + 2 * HO, WMK = S + 2 * HM;
    constexpr int kChunks = kWN / 8;  // 16-byte chunks per pixel row
    const int total = nbl * S2 * kChunks;
    for (int c = threadIdx.x; c < total; c += 512) {
      const int pix = c / kChunks, k8 = (c - pix * kChunks) * 8;
      const int bl = pix / S2, rem = pix - bl * S2;
      const int i = rem / S, j = rem - i * S;
      const int m = bl * PB + i * TJ + (j >> 1);
      bf16x8 v = *reinterpret_cast<const bf16x8*>(lds + (2 * m + (j & 1)) * kEpRow + k8);
      const int b = b0 + bl;
      if (mask) {
        const bf16x8 mk = *reinterpret_cast<const bf16x8*>(
            mask + (size_t)((b * WMK + i + HM) * WMK + j + HM) * YC + n0 + k8);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = ((float)mk[e] > 0.f) ? v[e] : (bf16)0.f;
      }
      if constexpr ((DIAG & 32) != 0) {
        if ((float)v[0] == 12345.f) Y[0] = v[1];
        continue;
      }
      *reinterpret_cast<bf16x8*>(Y + (size_t)((b * WO + i + HO) * WO + j + HO) * YC + n0 + k8) = v;
    }
  }
  // a deferred wgrad reduction riding in this launch (every block claims units of it)
  if (red.ticket) wslab_reduce_dynamic<kRedU>(red, reinterpret_cast<int*>(lds));
}

// Winograd weights of 3x3 layers from the fp32 OIHW masters: forward Uf [12][COUTP][CINP]
// (tap (ky, q) = ky * 4 + q) and dgrad Ub [12][CINP][COUTP] (the same transform of the flipped,
// transposed kernel W[n][c][2-ky][2-kx]). Block = one 64 (n) x 64 (c) tile of one kernel row ky
// of one layer (blockIdx.y): the row's three taps go through LDS so both layouts are written
// coalesced (Uf along c, Ub along n).
constexpr int kWinoPackFields = 8;  // W, COUT, CIN, COUTP, CINP, Uf, Ub (or 0), unused
__global__ void __launch_bounds__(256) wino_pack_kernel(const int64_t* __restrict__ table) {
  const int64_t* t = table + (size_t)blockIdx.y * kWinoPackFields;
  const float* W = (const float*)t[0];
  const int COUT = (int)t[1], CIN = (int)t[2], COUTP = (int)t[3], CINP = (int)t[4];
  bf16* Uf = (bf16*)t[5];
  bf16* Ub = (bf16*)t[6];
  const int ntn = (COUTP + 63) / 64, ntc = (CINP + 63) / 64;
  const int g = blockIdx.x / 3, ky = blockIdx.x - g * 3;
  if (g >= ntn * ntc) return;
  const int ct = g % ntc, nt = g / ntc;
  __shared__ float tl[3][64][65];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const long tap_stride = (long)COUTP * CINP;
#pragma unroll 4
  for (int i = 0; i < 16; ++i) {
    const int nl = ty + 4 * i;
    const int n = nt * 64 + nl, c = ct * 64 + tx;
    float g0 = 0.f, g1 = 0.f, g2 = 0.f;
    if (n < COUT && c < CIN) {
      const float* p = W + ((size_t)(n * CIN + c) * 3 + ky) * 3;
      g0 = p[0];
      g1 = p[1];
      g2 = p[2];
    }
    tl[0][nl][tx] = g0;
    tl[1][nl][tx] = g1;
    tl[2][nl][tx] = g2;
    if (n < COUTP && c < CINP) {
      const size_t o = (size_t)n * CINP + c;
      Uf[(ky * 4 + 0) * tap_stride + o] = (bf16)g0;
      Uf[(ky * 4 + 1) * tap_stride + o] = (bf16)(0.5f * (g0 + g1 + g2));
      Uf[(ky * 4 + 2) * tap_stride + o] = (bf16)(0.5f * (g0 - g1 + g2));
      Uf[(ky * 4 + 3) * tap_stride + o] = (bf16)g2;
    }
  }
  if (!Ub) return;
  __syncthreads();
  const int kyb = 2 - ky;  // dgrad kernel row; its kx is flipped: (h0, h1, h2) = (g2, g1, g0)
#pragma unroll 4
  for (int i = 0; i < 16; ++i) {
    const int cl = ty + 4 * i;
    const int c = ct * 64 + cl, n = nt * 64 + tx;
    if (c < CINP && n < COUTP) {
      const float h0 = tl[2][tx][cl], h1 = tl[1][tx][cl], h2 = tl[0][tx][cl];
      const size_t o = (size_t)c * COUTP + n;
      Ub[(kyb * 4 + 0) * tap_stride + o] = (bf16)h0;
      Ub[(kyb * 4 + 1) * tap_stride + o] = (bf16)(0.5f * (h0 + h1 + h2));
      Ub[(kyb * 4 + 2) * tap_stride + o] = (bf16)(0.5f * (h0 - h1 + h2));
      Ub[(kyb * 4 + 3) * tap_stride + o] = (bf16)h2;
    }
  }
}

// Boards per block: as many as fit the 192 pair rows, the V slab and the raw slab.
int wino_boards_per_block(int S) {
  const int WI = S + 2, TJ = (S + 1) / 2;
  const int PB = S * TJ, VPB = WI * TJ, RPB = WI * WI;
  int nb = kWP / PB;
  if (nb * VPB > kVRows) nb = kVRows / VPB;
  if (nb * RPB + 1 > kRRows) nb = (kRRows - 1) / RPB;
  return nb;
}

}  // namespace

// True if conv_wino can run this layer: 3x3, input halo 1, input channels a multiple of 32 (at
// most 12 chunks: nothing indexes past them), output channels a multiple of 192, a board that
// fits the block's slabs.
RAG_API int rag_conv_wino_ok(int S, int HI, int KIN, int NOUT, int KS) {
  return KS == 3 && HI == 1 && KIN % kWK == 0 && KIN >= kWK && NOUT % kWN == 0 && S >= 2 &&
         wino_boards_per_block(S) >= 1;
}

// Winograd 3x3 conv (forward or dgrad): X [B][S+2][S+2][KIN] bf16, U [12][NOUT][KIN] bf16
// (rag_wino_pack), Y padded with halo HO and YC >= NOUT channels, mask (dgrad) with halo HM.
// `pending`: a deferred wgrad reduction handle (conv.hip PendingRed) or null.
int rag_conv_wino_launch(const void* X, const void* W, const float* bias, void* Y,
                         const void* mask, int B, int S, int KIN, int NOUT, int HO, int YC,
                         int relu, int HM, hipStream_t stream, const WgradRed* red) {
  if (!rag_conv_wino_ok(S, 1, KIN, NOUT, 3) || YC < NOUT || B <= 0) return -1;
  const int nb = wino_boards_per_block(S);
  WgradRed r{};
  if (red) r = *red;
  const dim3 grid((B + nb - 1) / nb, NOUT / kWN);
  conv_wino_kernel<0><<<grid, 512, 0, stream>>>((const bf16*)X, (const bf16*)W, bias, (bf16*)Y,
                                             (const bf16*)mask, B, S, KIN, NOUT, HO, YC, relu,
                                             HM, nb, r);
  return (int)hipGetLastError();
}

RAG_API int rag_conv_wino(const void* X, const void* W, const float* bias, void* Y,
                          const void* mask, int B, int S, int KIN, int NOUT, int HO, int YC,
                          int relu, int HM, hipStream_t stream) {
  return rag_conv_wino_launch(X, W, bias, Y, mask, B, S, KIN, NOUT, HO, YC, relu, HM, stream,
                              nullptr);
}

static long long* g_wino_stamps = nullptr;
// Per-wave loop segment cycle sums of the last DIAG-64 launch: [block][wave][6] int64.
RAG_API int rag_conv_wino_stamps(long long* host, int nblocks) {
  if (!g_wino_stamps) return -1;
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  return (int)hipMemcpy(host, g_wino_stamps, (size_t)nblocks * 8 * 6 * sizeof(long long),
                        hipMemcpyDeviceToHost);
}

// Timing-diagnostic launches (WRONG results): diag = the kernel's DIAG bits.
RAG_API int rag_conv_wino_diag(int diag, const void* X, const void* W, const float* bias, void* Y,
                               const void* mask, int B, int S, int KIN, int NOUT, int HO, int YC,
                               int relu, int HM, hipStream_t stream) {
  if (!rag_conv_wino_ok(S, 1, KIN, NOUT, 3) || YC < NOUT || B <= 0) return -1;
  const int nb = wino_boards_per_block(S);
  WgradRed r{};
  const dim3 grid((B + nb - 1) / nb, NOUT / kWN);
  const bf16 *x = (const bf16*)X, *w = (const bf16*)W, *mk = (const bf16*)mask;
  bf16* y = (bf16*)Y;
#define RAG_WD(D)                                                                              \
  case D:                                                                                      \
    conv_wino_kernel<D><<<grid, 512, 0, stream>>>(x, w, bias, y, mk, B, S, KIN, NOUT, HO, YC, \
                                                  relu, HM, nb, r, stamps);                  \
    break;
  static long long* stamps = nullptr;
  if ((diag & 64) && !stamps && hipMalloc(&stamps, 4096 * 8 * 6 * sizeof(long long)) != hipSuccess)
    return -3;
  if ((diag & 64) && grid.x > 4096) return -1;
  g_wino_stamps = stamps;
  switch (diag) {
    RAG_WD(1) RAG_WD(2) RAG_WD(4) RAG_WD(8) RAG_WD(16) RAG_WD(32) RAG_WD(3) RAG_WD(7) RAG_WD(24)
    RAG_WD(63) RAG_WD(64)
    default: return -1;
  }
#undef RAG_WD
  return (int)hipGetLastError();
}

// table: kWinoPackFields int64 per layer (W, COUT, CIN, COUTP, CINP, Uf, Ub or 0, 0).
RAG_API int rag_wino_pack(const int64_t* table, int nlayers, int max_tiles, hipStream_t stream) {
  if (nlayers <= 0 || max_tiles <= 0) return -1;
  const dim3 grid((unsigned)(3 * max_tiles), (unsigned)nlayers);
  wino_pack_kernel<<<grid, 256, 0, stream>>>(table);
  return (int)hipGetLastError();
}

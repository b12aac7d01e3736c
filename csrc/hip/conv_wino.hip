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
// work. The transform mixes only +-1 terms (one bf16 rounding of V, one of U = G g);
// tests/test_wino.py pins it against fp32 F.conv2d.
//
// Accumulators: two sets A, B per wave. Phase 1 runs the q = 1 and q = 2 GEMMs into A and B
// (M1, M2), a register butterfly makes them (M1 + M2, M1 - M2), phase 2 accumulates q = 0 into A
// and q = 3 into B with V3' = d3 - d1 = -V3: A = y(2t), B = y(2t+1). Two sets per output pair =
// one accumulator per pixel, the direct kernel's register budget: one block covers a whole
// 19x19 board (190 output pairs, padded to 192) x 192 output channels; smaller boards pack
// several per block (nb, host side).
//
// Block: 8 waves, wave (wm, wn) = 96 pairs (6 fragments) x 48 channels (3 fragments) of both
// sets. K-step (chunk-phase k, ky), 36 per C = 192 layer: per set 6 V fragments from LDS and 3
// weight fragments from registers, 18 MFMA 16x16x32 -> 36 MFMAs per wave per step.
//   * weights never touch LDS: they are packed fragment-major (every 16 x 32 MFMA operand one
//     contiguous 1 KB, rag_wino_pack) and each wave loads its fragments for step s+1 straight
//     into registers right after its step-s MFMAs have read them (L1 serves the two waves that
//     share a column). The first version staged them through an LDS ring with LDS-DMA: ~150 -
//     220 issue cycles per 1 KB piece (s_memtime segments) for 12 KB per 144 MFMAs, more than
//     the MFMAs themselves;
//   * V slab per chunk-phase, [2 sets][vrow = (board row) x 10 + t][32 ch] in LDS, double
//     buffered (56 KB): built one chunk-phase ahead by every thread from raw input rows loaded
//     straight from L2 into registers (two units per thread, loads one step ahead of their
//     +- and 16-byte LDS stores). A fragment of 16 consecutive output pairs reads 16
//     consecutive V rows (no halo columns in between, unlike the direct kernel's pixel slab):
//     the row-bit-2 swizzle keeps it conflict-free;
//   * one barrier per chunk-phase (the V buffer flip); no per-step barriers, the two waves of
//     a SIMD overlap freely.
#include "common.h"
#include "pack.h"
#include "wgrad_part.h"

using namespace rag;

namespace {

constexpr int kWK = 32;                  // channels per chunk (MFMA K)
constexpr int kWP = 192;                 // output pairs per block (a 19x19 board: 190)
constexpr int kVRows = 224;              // V slab rows (a 19x19 board: 21 x 10 = 210)
constexpr int kRRows = 512;              // raw rows a block may touch (19x19: 21 x 21 + 1)
constexpr int kVSlot = kVRows * kWK;
constexpr int kLoopLds = 4 * kVSlot;     // [2 chunk-phase buffers][2 sets]
constexpr int kRedU = 14;                // chunk loads in flight per reduce thread

// Output-tile geometry per block width WN (output channels per block): 8 waves = MW wave rows
// along the 192 pairs x (8 / MW) wave columns along WN; per wave MT pair fragments x NT channel
// fragments of both accumulator sets, its V fragments read in RG groups.
//   WN = 192 (the north-star trunk): 2 x 4 waves of 96 pairs x 48 channels (18 MFMAs per 6 V
//            fragment reads per set and step, 144 accumulator registers);
//   WN = 128 (CNNPolicy's default width): 4 x 2 waves of 48 pairs x 64 channels (12 MFMAs per
//            3 V reads: the 96 x 32 tile of the 192 layout would read twice as much LDS per MFMA).
//   PAIRS = 96 (half a 19x19 board per block, WN = 192): 2 x 4 waves of 48 pairs x 48 channels
//            -- batches of ~128 boards, whose one-board blocks would leave half the chip idle,
//            run two blocks per board (V rows of the half plus two halo rows built by each).
template <int WN, int PAIRS> struct WinoGeo;
template <> struct WinoGeo<192, 192> {
  static constexpr int MW = 2, MT = 6, NT = 3, RG = 2;
};
template <> struct WinoGeo<128, 192> {
  static constexpr int MW = 4, MT = 3, NT = 4, RG = 1;
};
template <> struct WinoGeo<192, 96> {
  static constexpr int MW = 2, MT = 3, NT = 3, RG = 1;
};
template <int WN, int PAIRS> struct WinoTile : WinoGeo<WN, PAIRS> {
  using G = WinoGeo<WN, PAIRS>;
  static_assert(G::MW * 16 * G::MT == PAIRS && (8 / G::MW) * 16 * G::NT == WN, "wave tiling");
  static constexpr int EpRow = WN + 8;            // bf16 per row of the epilogue image
  static constexpr int EpImg = 2 * PAIRS * EpRow;  // one image row per output pixel (pair, col)
  static constexpr int Lds = kLoopLds > EpImg ? kLoopLds : EpImg;
  static_assert(Lds * 2 <= 160 * 1024, "LDS budget");
};
constexpr int kHalfPairs = 96;

__device__ __forceinline__ int swz4w(int row) { return ((row >> 2) & 1) << 1; }

template <int V> struct IntC {
  static constexpr int value = V;
};

// a + s * b of 8 bf16 (s = +-1), rounded once: one 32-bit word (two elements) at a time, so the
// transform never holds more than a few fp32 temporaries next to the 144 accumulators
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <int SGN>
__device__ __forceinline__ bf16x8 vaddsub(const bf16x8& a, const bf16x8& b) {
  const u32x4 ua = __builtin_bit_cast(u32x4, a), ub = __builtin_bit_cast(u32x4, b);
  u32x4 o;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const float a0 = __uint_as_float(ua[w] << 16), a1 = __uint_as_float(ua[w] & 0xffff0000u);
    const float b0 = __uint_as_float(ub[w] << 16), b1 = __uint_as_float(ub[w] & 0xffff0000u);
    const bf16x2 r = {(bf16)(SGN > 0 ? a0 + b0 : a0 - b0), (bf16)(SGN > 0 ? a1 + b1 : a1 - b1)};
    o[w] = __builtin_bit_cast(uint32_t, r);
  }
  return __builtin_bit_cast(bf16x8, o);
}
__device__ __forceinline__ bf16x8 vsum(const bf16x8& a, const bf16x8& b) { return vaddsub<1>(a, b); }
__device__ __forceinline__ bf16x8 vdiff(const bf16x8& a, const bf16x8& b) { return vaddsub<-1>(a, b); }
// The same with the BN prologue (ResnetPolicy): the raw values are BN inputs x and
// the transform runs on U = ReLU(cx x + cc) of each column (cx = cc = 0 on halo pixels: U = 0),
// kept in fp32 up to the one rounding of V
template <int SGN>
__device__ __forceinline__ bf16x8 vaddsub_bn(const bf16x8& a, const bf16x8& b, float cxa,
                                             float cca, float cxb, float ccb) {
  const u32x4 ua = __builtin_bit_cast(u32x4, a), ub = __builtin_bit_cast(u32x4, b);
  u32x4 o;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const float a0 = fmaxf(fmaf(cxa, __uint_as_float(ua[w] << 16), cca), 0.f);
    const float a1 = fmaxf(fmaf(cxa, __uint_as_float(ua[w] & 0xffff0000u), cca), 0.f);
    const float b0 = fmaxf(fmaf(cxb, __uint_as_float(ub[w] << 16), ccb), 0.f);
    const float b1 = fmaxf(fmaf(cxb, __uint_as_float(ub[w] & 0xffff0000u), ccb), 0.f);
    const bf16x2 r = {(bf16)(SGN > 0 ? a0 + b0 : a0 - b0), (bf16)(SGN > 0 ? a1 + b1 : a1 - b1)};
    o[w] = __builtin_bit_cast(uint32_t, r);
  }
  return __builtin_bit_cast(bf16x8, o);
}

// Fused BatchNorm of the 128-channel residual trunk (BNM template argument of conv_wino_kernel):
//   BNM 1 (forward): X is the BN input x, the layer input U = ReLU(coef[0][col] x + coef[2][col])
//          is built in the transform (never stored); `res` (or null) is added to the output; with
//          spart, the block's (sum y, sum y^2) per board column of the stored output;
//   BNM 2 (dgrad): the ReLU mask of U is recomputed from mask = x and coef; with spart,
//          (sum dU, sum dU (x - smean)) per column of the masked output.
// spart: [gridDim.x][2][S] fp32 partials (one row pair per block = per board) for bn.hip's
// finalize, as conv_tap_pp_kernel's BNP / mcoef / spart forms on the direct kernel.
struct WinoBN {
  const float* coef;
  const bf16* res;
  float* spart;
  const float* smean;
};

// X: padded input [B][S+2][S+2][KIN] (halo 1). U: Winograd weights, fragment-major
// [12 = (ky, q)][KIN / 32][NOUT / 16][64 lanes][8] (rag_wino_pack). Y: padded output (halo HO,
// YC channels); mask: the dgrad ReLU mask (halo HM) or null.
// Block (x, y): boards [x * nb, x * nb + nb), output channels [192 y, 192 y + 192).
// SINGLE: one board per block (19x19): the V row of output pair m is m itself (pad pairs 190,
// 191 read rows < 224 whose outputs are dropped), so no per-fragment row table is kept.
template <int WN, bool SINGLE, int PAIRS = kWP, int BNM = 0>
__global__ void __launch_bounds__(512, 1)
conv_wino_kernel(const bf16* __restrict__ X, const bf16* __restrict__ U,
                 const float* __restrict__ bias, bf16* __restrict__ Y,
                 const bf16* __restrict__ mask, int B, int S, int KIN, int NOUT, int HO, int YC,
                 int relu, int HM, int nb, WgradRed red, WinoBN bn = WinoBN{}) {
  using T = WinoTile<WN, PAIRS>;
  constexpr int kWMT = T::MT, kWNT = T::NT, kWN = WN, kEpRow = T::EpRow;
  constexpr bool HALF = PAIRS == kHalfPairs;  // two blocks per board (SINGLE geometry)
  static_assert(!HALF || SINGLE, "half-board blocks: one board");
  static_assert(BNM == 0 || (SINGLE && !HALF && WN == 128), "fused BN: the 128-wide one-board tile");
  // + a [2][64] float column-statistics accumulator past the loop ring / epilogue image
  __shared__ __attribute__((aligned(16))) bf16 lds[T::Lds + (BNM ? 256 : 0)];
  float* sred = reinterpret_cast<float*>(lds + T::Lds);
  if constexpr (BNM != 0) {
    if (bn.spart && threadIdx.x < 128) sred[threadIdx.x] = 0.f;  // published by the first barrier
  }
  const int lane = lane_id();
  const int w = wave_id();
  const int wm = w % T::MW, wn = w / T::MW;
  const int frow = lane & 15, fq = lane >> 4;
  const int WI = S + 2, TJ = (S + 1) >> 1;
  const int PB = S * TJ;    // output pairs per board
  const int VPB = WI * TJ;  // V rows per board
  const int RPB = WI * WI;  // raw rows per board
  const int b0 = HALF ? (int)(blockIdx.x >> 1) : (int)blockIdx.x * nb;
  const int n0 = blockIdx.y * kWN;
  // HALF: this block's output pairs are [p0, p0 + 96) of the board; its V rows start at padded
  // row i0 (V row of pair p at ky: p - i0 TJ + ky TJ)
  const int p0 = HALF ? (int)(blockIdx.x & 1) * kHalfPairs : 0;
  const int i0 = HALF ? p0 / TJ : 0;
  const int voff = p0 - i0 * TJ;
  const long total_rows = (long)B * RPB;
  const int cchunks = KIN / kWK;
  const int NK = 2 * cchunks;  // chunk-phases

  // ---- V rows of this lane's output pairs (tap ky adds ky * TJ)
  int vb[SINGLE ? 1 : kWMT];
#pragma unroll
  for (int i = 0; i < (SINGLE ? 1 : kWMT); ++i) {
    int m = wm * (16 * kWMT) + i * 16 + frow;
    if (SINGLE) {
      vb[i] = m + voff;
      continue;
    }
    m = m < nb * PB ? m : nb * PB - 1;  // pad pairs read a valid row, their output is dropped
    const int bl = m / PB, rem = m - bl * PB;
    const int ii = rem / TJ, t = rem - ii * TJ;
    vb[i] = (bl * WI + ii) * TJ + t;
  }

  // ---- global loads are buffer loads: a wave-uniform descriptor (SGPRs), a 32-bit lane offset
  // and a uniform SGPR offset, one VGPR per address instead of 64-bit pointers (the kernel sat
  // at 256 VGPRs and its scratch reloads, being VMEM, forced vmcnt(0) waits on every weight
  // load in flight); the descriptor's range check also replaces the raw rows' clamp.
  auto rsrc = [](const void* p, long bytes) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    const int nb = __builtin_amdgcn_readfirstlane((int)(bytes < 0x7fffffffL ? bytes : 0x7fffffffL));
    return __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0, nb, 0x00020000);
  };
  // weight fragments: fragment (tap, chunk, nf) is 512 contiguous bf16, lane l's 8 at 8 l
  const int NF = NOUT / 16;
  const auto urs = rsrc(U, 12L * NOUT * KIN * 2);
  const uint32_t uoff = (uint32_t)((((n0 >> 4) + wn * kWNT) * 512 + lane * 8) * 2);
  auto wfrag = [&](int tap, int c, int j) {
    const int so = ((tap * cchunks + c) * NF + j) * 1024;
    return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(urs, uoff, so, 0));
  };
  // taps: set A q = 1 (phase 1) / 0 (phase 2), set B q = 2 / 3; tap (ky, q) = 4 ky + q

  // ---- transform units of this thread (the same for every chunk-phase): V row, 8-channel
  // group, raw row of d0 (named scalars: a runtime-indexed array went to scratch)
  // packed: V row (bits 0-9), 8-channel group (10-11), raw row of d0 (12-30), -1 = no unit
  // (HALF: the V rows of padded rows i0 .. (last pair's row) + 2 only)
  const int NU = HALF ? ((p0 + kHalfPairs - 1) / TJ - i0 + 3) * TJ * 4 : nb * VPB * 4;
  auto unit = [&](int it) {
    const int u = threadIdx.x + it * 512;
    const int v = u >> 2;
    const int bl = v / VPB, rem = v - bl * VPB;
    const int r = rem / TJ, t = rem - r * TJ;
    const int rr = (bl * WI + r + i0) * WI + 2 * t;
    return u < NU ? (v | ((u & 3) << 10) | (rr << 12)) : -1;
  };
  const int tu0 = unit(0), tu1 = unit(1);
  // BNM 1: per transform unit, the BN coefficients of its four raw columns d0..d3 (zero on halo
  // pixels and for a missing unit, so U = 0 there)
  float bcx[2][4], bcc[2][4];
  if constexpr (BNM == 1) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int pk = q ? tu1 : tu0;
      const int v = pk < 0 ? 0 : (pk & 1023);
      const int r = v / TJ, t = v - r * TJ;  // padded row r, pair column t (one board)
      const bool rin = pk >= 0 && r >= 1 && r <= S;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int pc = 2 * t + s;  // padded column of d_s
        const bool in = rin && pc >= 1 && pc <= S;
        bcx[q][s] = in ? bn.coef[pc - 1] : 0.f;
        bcc[q][s] = in ? bn.coef[2 * S + pc - 1] : 0.f;
      }
    }
  }
  // raw rows of this block's boards (out of range, i.e. the last block's +1 row, reads 0)
  const auto xrs = rsrc(X + (long)b0 * RPB * KIN, (total_rows - (long)b0 * RPB) * KIN * 2);
  // The transform of V(kk) runs as four "ops" per thread and chunk-phase, two raw-pixel loads
  // each: op 2u + h of unit u (h = set): phase 1 loads (d1, d2) for both sets (V1 = d1 + d2,
  // V2 = d2 - d1), phase 2 (d0, d2) for set A (V0 = d0 - d2) and (d3, d1) for set B
  // (V3' = d3 - d1). An op's loads go out one MFMA block before its +- and store.
  // Every global load in the loop is issued unconditionally (a missing unit or a chunk-phase
  // past the end loads a valid dummy row and skips only its LDS store): with loads under
  // branches hipcc's counter analysis fell back to `s_waitcnt vmcnt(0)`, so each transform
  // store and each set's first MFMA waited for every load in flight, the next step's weights
  // included.
  // two ops in flight (op o in register pair o & 1): an op's loads go out two MFMA blocks
  // before its +- and store, ~0.5 us: the raw rows of a layer written by the previous launch
  // come from HBM / MALL, and one block's distance cost up to 7 us per launch in the step
  bf16x8 da0, db0, da1, db1;
  auto op_unit = [&](int o, int& v, int& k8, int& rr) {
    int pk = (o >> 1) ? tu1 : tu0;
    asm volatile("" : "+v"(pk));
    v = pk < 0 ? -1 : (pk & 1023);
    pk = pk < 0 ? 0 : pk;
    k8 = (pk >> 10) & 3;
    rr = pk >> 12;
  };
  // P1: the V being built belongs to phase 1 (compile time: a runtime phase test put both
  // arithmetic paths and a join into the loop, and hipcc's counters and registers with them)
  auto op_load = [&](auto p1c, int kk, auto oc) {  // kk may be NK (past the end): a dummy
    constexpr bool P1 = decltype(p1c)::value;
    constexpr int o = decltype(oc)::value, h = o & 1;
    int v, k8, rr;
    op_unit(o, v, k8, rr);
    const int ra = P1 ? 1 : (h ? 3 : 0), rb = P1 ? 2 : (h ? 1 : 2);
    const int so = (kk % cchunks) * kWK * 2;
    const uint32_t o0 = (uint32_t)((rr + ra) * KIN + k8 * 8) * 2u;
    const uint32_t o1 = (uint32_t)((rr + rb) * KIN + k8 * 8) * 2u;
    const bf16x8 a = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(xrs, o0, so, 0));
    const bf16x8 b = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(xrs, o1, so, 0));
    if constexpr (h) {
      da1 = a;
      db1 = b;
    } else {
      da0 = a;
      db0 = b;
    }
  };
  auto op_store = [&](auto p1c, int kk, auto oc) {  // branch-free: no unit -> the last V row
    constexpr bool P1 = decltype(p1c)::value;
    constexpr int o = decltype(oc)::value, h = o & 1;
    int v, k8, rr;
    op_unit(o, v, k8, rr);
    v = v < 0 ? kVRows - 1 : v;
    bf16* vs = lds + (kk & 1) * 2 * kVSlot + h * kVSlot;
    const bf16x8 da = h ? da1 : da0, db = h ? db1 : db0;
    bf16x8 val;
    if constexpr (BNM == 1) {
      constexpr int q = o >> 1, ra = P1 ? 1 : (h ? 3 : 0), rb = P1 ? 2 : (h ? 1 : 2);
      if constexpr (P1 && h)
        val = vaddsub_bn<-1>(db, da, bcx[q][rb], bcc[q][rb], bcx[q][ra], bcc[q][ra]);
      else
        val = vaddsub_bn<P1 ? 1 : -1>(da, db, bcx[q][ra], bcc[q][ra], bcx[q][rb], bcc[q][rb]);
    } else {
      val = P1 ? (h ? vdiff(db, da) : vsum(da, db)) : vdiff(da, db);
    }
    *reinterpret_cast<bf16x8*>(vs + v * kWK + ((k8 ^ swz4w(v)) * 8)) = val;
  };

  f32x4 accA[kWNT][kWMT], accB[kWNT][kWMT];
#pragma unroll
  for (int j = 0; j < kWNT; ++j)
#pragma unroll
    for (int i = 0; i < kWMT; ++i) {
      accA[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
      accB[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  // V fragments are read in two halves of three (12 registers instead of 24: with all six
  // live, hipcc spilled the transform's raw loads and waited for them at once)
  constexpr int kH = kWMT / T::RG;  // V fragments per read group
  bf16x8 xa[kH], wA[kWNT], wB[kWNT];
  auto read_v = [&](int kk, int ky, int set, int h) {
    const bf16* vs = lds + ((kk & 1) * 2 + set) * kVSlot;
    const int sh = ky * TJ;
    if constexpr (SINGLE) {
      int r0 = vb[0];
      asm volatile("" : "+v"(r0));  // not hoisted: per-(fragment, ky) addresses, 18 registers
      r0 += sh + h * kH * 16;
      const int sw0 = (fq ^ swz4w(r0)) * 8;  // rows r0 + 16 i share row bit 2
#pragma unroll
      for (int i = 0; i < kH; ++i)
        xa[i] = *reinterpret_cast<const bf16x8*>(vs + (r0 + i * 16) * kWK + sw0);
    } else {
#pragma unroll
      for (int i = 0; i < kH; ++i) {
        int v = vb[h * kH + i];
        asm volatile("" : "+v"(v));
        const int r = v + sh;
        xa[i] = *reinterpret_cast<const bf16x8*>(vs + r * kWK + ((fq ^ swz4w(r)) * 8));
      }
    }
  };

  // ---- prologue: this XCD's L2 warmed with the layer's weights (block x runs on XCD x % 8:
  // its blocks each touch one slice; in the step every launch finds its weights cold, and the
  // in-loop weight loads, one MFMA block ahead, then waited on HBM), step (0, 0)'s weights, V(0)
  uint32_t warm = 0;
  {
    const int lin = blockIdx.y * gridDim.x + blockIdx.x;
    const int per_xcd = (gridDim.x * gridDim.y + 7) >> 3;
    const uint32_t slice = (uint32_t)((12L * NOUT * KIN * 2 + per_xcd - 1) / per_xcd);
    const uint32_t base = (uint32_t)((lin >> 3) % per_xcd) * slice;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t off = (uint32_t)(threadIdx.x + k * 512) * 16u;
      const uint32_t o = off < slice ? base + off : 0xfffffff0u;  // out of range: reads 0
      warm ^= (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(urs, o, 0, 0);
    }
  }
#pragma unroll
  for (int j = 0; j < kWNT; ++j) {
    wA[j] = wfrag(1, 0, j);
    wB[j] = wfrag(2, 0, j);
  }
  op_load(IntC<1>{}, 0, IntC<0>{});  // V(0) (phase 1)
  op_store(IntC<1>{}, 0, IntC<0>{});
  op_load(IntC<1>{}, 0, IntC<1>{});
  op_store(IntC<1>{}, 0, IntC<1>{});
  op_load(IntC<1>{}, 0, IntC<2>{});
  op_store(IntC<1>{}, 0, IntC<2>{});
  op_load(IntC<1>{}, 0, IntC<3>{});
  op_store(IntC<1>{}, 0, IntC<3>{});
  asm volatile("" ::"v"(warm));  // (the warming loads are not dead)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  // one chunk-phase: CUR = phase of kk (its taps), NXT = phase of kk + 1 (the V built and the
  // weights prefetched during kk)
  auto chunk_phase = [&](int kk, auto curc, auto nxtc) {
    constexpr bool CUR1 = decltype(curc)::value, NXT1 = decltype(nxtc)::value;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      // next step's weights: (kk, ky + 1) or (kk + 1, 0); past the end: a dummy (the last
      // step's again)
      const bool nxt1 = ky < 2 ? CUR1 : NXT1;
      int nkk = ky < 2 ? kk : kk + 1, nky = ky < 2 ? ky + 1 : 0;
      if (nkk >= NK) {
        nkk = NK - 1;
        nky = 2;
      }
      const int nc = nkk % cchunks;
      const int ntA = nky * 4 + (nxt1 ? 1 : 0), ntB = nky * 4 + (nxt1 ? 2 : 3);
      // transform ops of V(kk + 1) in the six (ky, set) slots: slot t stores op t-2 and loads
      // op t (loads in slots 0..3, stores in 2..5; in the last chunk-phase they fill the idle
      // buffer, read by nobody)
      if (ky == 1) op_store(nxtc, kk + 1, IntC<0>{});
      if (ky == 2) op_store(nxtc, kk + 1, IntC<2>{});
      __builtin_amdgcn_sched_barrier(0);
      if (ky == 0) op_load(nxtc, kk + 1, IntC<0>{});
      if (ky == 1) op_load(nxtc, kk + 1, IntC<2>{});
      __builtin_amdgcn_sched_barrier(0);
      // ---- set A
#pragma unroll
      for (int h = 0; h < T::RG; ++h) {
        read_v(kk, ky, 0, h);
#pragma unroll
        for (int j = 0; j < kWNT; ++j) {
#pragma unroll
          for (int i = 0; i < kH; ++i)
            accA[j][h * kH + i] = mfma16(wA[j], xa[i], accA[j][h * kH + i]);
          if (h == T::RG - 1) wA[j] = wfrag(ntA, nc, j);
        }
      }
      // (scheduling fences: hipcc otherwise reads set B's fragments into a second register set
      // while set A's MFMAs still hold the first, and the kernel spills)
      __builtin_amdgcn_sched_barrier(0);
      if (ky == 1) op_store(nxtc, kk + 1, IntC<1>{});
      if (ky == 2) op_store(nxtc, kk + 1, IntC<3>{});
      __builtin_amdgcn_sched_barrier(0);  // the old op's registers free before the new loads
      if (ky == 0) op_load(nxtc, kk + 1, IntC<1>{});
      if (ky == 1) op_load(nxtc, kk + 1, IntC<3>{});
      __builtin_amdgcn_sched_barrier(0);
      // ---- set B
#pragma unroll
      for (int h = 0; h < T::RG; ++h) {
        read_v(kk, ky, 1, h);
#pragma unroll
        for (int j = 0; j < kWNT; ++j) {
#pragma unroll
          for (int i = 0; i < kH; ++i)
            accB[j][h * kH + i] = mfma16(wB[j], xa[i], accB[j][h * kH + i]);
          if (h == T::RG - 1) wB[j] = wfrag(ntB, nc, j);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // V(kk + 1) complete and V(kk) read by every wave before the buffers flip
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

#pragma unroll 1
  for (int kk = 0; kk < cchunks - 1; ++kk) chunk_phase(kk, IntC<1>{}, IntC<1>{});
  chunk_phase(cchunks - 1, IntC<1>{}, IntC<0>{});
  // (M1, M2) -> (M1 + M2, M1 - M2)
#pragma unroll
  for (int j = 0; j < kWNT; ++j)
#pragma unroll
    for (int i = 0; i < kWMT; ++i) {
      const f32x4 a = accA[j][i], b = accB[j][i];
      accA[j][i] = a + b;
      accB[j][i] = a - b;
    }
#pragma unroll 1
  for (int kk = cchunks; kk < NK; ++kk) chunk_phase(kk, IntC<0>{}, IntC<0>{});

  // ---- epilogue: bias (+ ReLU) -> bf16 image [pair][column][channel] in LDS, then whole
  // 384-byte pixel rows out with the dgrad mask applied
  __syncthreads();
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
  if constexpr (BNM != 0) {
    // one board: 16 consecutive threads own one pixel row of 128 channels (512 = 32 rows per
    // pass, every thread runs the same passes so the row reductions' shuffles see whole waves)
    const int S2 = S * S, WO = S + 2 * HO, WMK = S + 2 * HM;
    constexpr int kChunks = kWN / 8;
    const int total = S2 * kChunks, nit = (total + 511) / 512;
    const bool st = bn.spart != nullptr;
    for (int it = 0; it < nit; ++it) {
      const int e = threadIdx.x + it * 512;
      const bool valid = e < total;
      const int pix = valid ? e / kChunks : 0, k8 = (e % kChunks) * 8;
      const int i = pix / S, j = pix - (pix / S) * S;
      float s0 = 0.f, s1 = 0.f;
      if (valid) {
        const int m = i * TJ + (j >> 1);
        bf16x8 v = *reinterpret_cast<const bf16x8*>(lds + (2 * m + (j & 1)) * kEpRow + k8);
        const size_t yo = (size_t)((b0 * WO + i + HO) * WO + j + HO) * YC + n0 + k8;
        if constexpr (BNM == 1) {
          if (bn.res) {  // the residual unit's skip (bias (+ ReLU) already in the image)
            const bf16x8 r = *reinterpret_cast<const bf16x8*>(bn.res + yo);
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = (bf16)((float)v[q] + (float)r[q]);
          }
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const float f = (float)v[q];
            s0 += f;
            s1 = fmaf(f, f, s1);
          }
        } else {
          const bf16x8 mk = *reinterpret_cast<const bf16x8*>(
              mask + (size_t)((b0 * WMK + i + HM) * WMK + j + HM) * YC + n0 + k8);
          const float cx = bn.coef[j], cc = bn.coef[2 * S + j];
          const float mu = bn.smean ? bn.smean[j] : 0.f;
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const float xm = (float)mk[q];
            v[q] = fmaf(cx, xm, cc) > 0.f ? v[q] : (bf16)0.f;
            const float d = (float)v[q];
            s0 += d;
            s1 = fmaf(d, xm - mu, s1);  // backward: sum dU (x - mean)
          }
        }
        *reinterpret_cast<bf16x8*>(Y + yo) = v;
      }
      if (st) {
#pragma unroll
        for (int o = kChunks / 2; o > 0; o >>= 1) {
          s0 += __shfl_xor(s0, o, 64);
          s1 += __shfl_xor(s1, o, 64);
        }
        if ((threadIdx.x & (kChunks - 1)) == 0 && valid) {
          atomicAdd(sred + j, s0);
          atomicAdd(sred + 64 + j, s1);
        }
      }
    }
    if (st) {
      __syncthreads();
      if ((int)threadIdx.x < 2 * S) {
        const int q = threadIdx.x / S, c = threadIdx.x - q * S;
        bn.spart[((size_t)blockIdx.x * 2 + q) * S + c] = sred[q * 64 + c];
      }
    }
  } else {
    const int nbl = B - b0 < nb ? B - b0 : nb;
    const int S2 = S * S, WO = S + 2 * HO, WMK = S + 2 * HM;
    constexpr int kChunks = kWN / 8;  // 16-byte chunks per pixel row
    // HALF: the pixels of pairs [p0, min(p0 + 96, PB)) (2 per pair, the last column odd S)
    const int pe = p0 + kHalfPairs < PB ? p0 + kHalfPairs : PB;
    const int pixb = HALF ? (p0 / TJ) * S + 2 * (p0 % TJ) : 0;
    const int pixe = HALF ? (pe / TJ) * S + 2 * (pe % TJ) : 0;
    const int total = HALF ? ((pixe < S2 ? pixe : S2) - pixb) * kChunks : nbl * S2 * kChunks;
    for (int e = threadIdx.x; e < total; e += 512) {
      const int pix = e / kChunks + pixb, k8 = (e - (e / kChunks) * kChunks) * 8;
      const int bl = HALF ? 0 : pix / S2, rem = pix - bl * S2;
      const int i = rem / S, j = rem - i * S;
      const int m = bl * PB + i * TJ + (j >> 1) - p0;
      bf16x8 v = *reinterpret_cast<const bf16x8*>(lds + (2 * m + (j & 1)) * kEpRow + k8);
      const int b = b0 + bl;
      if (mask) {
        const bf16x8 mk = *reinterpret_cast<const bf16x8*>(
            mask + (size_t)((b * WMK + i + HM) * WMK + j + HM) * YC + n0 + k8);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = ((float)mk[q] > 0.f) ? v[q] : (bf16)0.f;
      }
      *reinterpret_cast<bf16x8*>(Y + (size_t)((b * WO + i + HO) * WO + j + HO) * YC + n0 + k8) = v;
    }
  }
  // a deferred wgrad reduction riding in this launch (every block claims units of it)
  if (red.ticket) wslab_reduce_dynamic<kRedU>(red, reinterpret_cast<int*>(lds));
}

// Winograd weights of 3x3 layers from the fp32 OIHW masters (pack.h wino_pack_block: table
// layout, fragment order, tiling).
// (at most 128 VGPRs, pack.h pack_rsrc: four blocks per CU, the SL trunk's 792 in one round)
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4)))
wino_pack_kernel(const int64_t* __restrict__ table, SgdFold sgd) {
  __shared__ float tl[kWinoPackLds];
  wino_pack_block(table, (int)blockIdx.y, (int)blockIdx.x, sgd, tl);
}

// The rest of a flat parameter buffer after a folded repack: plain SGD over up to two element
// ranges [a0, a0 + n0), [a1, a1 + n1) of p (gradients sgd.goff elements further).
struct SgdRest {
  float* p;
  long a0, n0, a1, n1;
};

// The whole weight update of a fused trunk step in ONE launch (round 6: rag_wino_pack +
// rag_pack_trunk + sgd_kernel were three launches, 38 us per SL step, each mostly its own
// latency chain): grid rows [0, trows) are the pack_trunk rows (nfull + 1 bias row), the next
// row (when rest.n0 + rest.n1 > 0) steps the rest of the flat buffer, the last nwino rows are
// wino_pack rows. The pack_trunk rows come first: blocks dispatch in grid order, and a 5x5
// layer's tile is the longest chain of the launch (two load rounds of 16 taps); behind 792
// wino_pack blocks (232 VGPRs: two blocks per CU) it started only in their second round.
// Dynamic LDS: the larger of the two tiles (pack_trunk sized for the trunk's largest kernel).
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4)))
pack_step_kernel(const int64_t* __restrict__ wtable, int nwino,
                 const int64_t* __restrict__ ttable, int nrows, int nfull, int max_taps,
                 SgdFold sgd, SgdRest rest) {
  extern __shared__ float lds_dyn[];
  int y = (int)blockIdx.y;
  const int bx = (int)blockIdx.x, gx = (int)gridDim.x;
  const int trows = nfull + (nrows > nfull ? 1 : 0);
  if (y < trows) {
    pack_trunk_block(ttable, y, nrows, nfull, sgd, bx, gx, max_taps, lds_dyn);
    return;
  }
  y -= trows;
  const long n = rest.n0 + rest.n1;
  if (n > 0 && y == 0) {
    for (long i = (long)bx * 256 + threadIdx.x; i < n; i += (long)gx * 256) {
      float* w = rest.p + (i < rest.n0 ? rest.a0 + i : rest.a1 + (i - rest.n0));
      *w = sgd.update(*w, w[sgd.goff]);
    }
    return;
  }
  y -= n > 0 ? 1 : 0;
  if (y < nwino) wino_pack_block(wtable, y, bx, sgd, lds_dyn);
}

// Boards per block: as many as fit the 192 pair rows and the V slab.
int wino_boards_per_block(int S) {
  const int WI = S + 2, TJ = (S + 1) / 2;
  const int PB = S * TJ, VPB = WI * TJ, RPB = WI * WI;
  int nb = kWP / PB;
  if (nb * VPB > kVRows) nb = kVRows / VPB;
  if (nb * RPB + 1 > kRRows) nb = (kRRows - 1) / RPB;  // (32-bit raw offsets stay small)
  return nb;
}

// Output channels per block for a layer of NOUT channels: 192-multiples take 192-wide tiles,
// exactly 128 the 128-wide one (one board per block only), else 0 (no Winograd kernel).
int wino_tile(int NOUT, int S) {
  if (NOUT % 192 == 0) return 192;
  if (NOUT == 128 && wino_boards_per_block(S) == 1) return 128;
  return 0;
}

}  // namespace

// True if conv_wino can run this layer: 3x3, input halo 1, input channels a multiple of 32 (at
// most 12 chunks: nothing indexes past them), output channels a multiple of 192 or exactly 128,
// a board that fits the block's slabs.
RAG_API int rag_conv_wino_ok(int S, int HI, int KIN, int NOUT, int KS) {
  return KS == 3 && HI == 1 && KIN % kWK == 0 && KIN >= kWK && S >= 2 &&
         wino_boards_per_block(S) >= 1 && wino_tile(NOUT, S) > 0;
}

// True if conv_wino should take a layer of this batch rather than the direct kernel (given
// rag_conv_wino_ok): one board per block (multi-board blocks of small boards are not measured
// faster yet) and a grid of 512-thread blocks, one per CU, whose last wave fills at least 7/8 of
// the CUs. The Winograd kernel's time is one fixed cost per wave (50.5 us at 19x19, 192 -> 192
// on MI355X) against the direct kernel's per-pixel cost (57 us per 256 boards), so a ragged
// last wave gives the gain back.
// Half-board blocks (96 pairs, 192-wide tiles): boards of more than 96 and at most 192 pairs.
static bool wino_half_ok(int S, int NOUT) {
  const int TJ = (S + 1) / 2;
  return NOUT % 192 == 0 && wino_boards_per_block(S) == 1 && S * TJ > kHalfPairs;
}
static int wino_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 0;
    cus = n;
  }
  return cus;
}
// 1: one-board blocks, 2: half-board blocks, 0: neither (the direct kernel).
// A grid of at most one wave of blocks (one per CU) costs one block's time whatever its size, and
// that beats the direct kernel at every batch: 192 -> 192 at 19x19 (benchmarks/wino_bench.py
// --batch sweep, one box) one-board blocks 41-45 us for B = 32..200 against 45-55 us direct,
// half-board blocks 29-35 us for B <= 128 (their 2B blocks still one wave). Several waves: a
// ragged last wave gives the gain back, so the Winograd grid must fill 7/8 of its last wave.
static int wino_mode(int B, int S, int KIN, int NOUT) {
  if (!rag_conv_wino_ok(S, 1, KIN, NOUT, 3) || B <= 0 || wino_boards_per_block(S) != 1) return 0;
  const int cus = wino_cus();
  if (!cus) return 0;
  auto fills = [&](long blocks) {
    const long waves = (blocks + cus - 1) / cus;
    return blocks * 8 >= waves * cus * 7;
  };
  const long full = (long)B * (NOUT / wino_tile(NOUT, S));
  const bool half = wino_half_ok(S, NOUT);
  if (full <= cus) return half && 2 * full <= cus ? 2 : 1;
  if (fills(full)) return 1;
  if (half && fills(2 * full)) return 2;
  return 0;
}
RAG_API int rag_conv_wino_prefer(int B, int S, int KIN, int NOUT) {
  return wino_mode(B, S, KIN, NOUT) != 0;
}
RAG_API int rag_conv_wino_mode(int B, int S, int KIN, int NOUT) {
  return wino_mode(B, S, KIN, NOUT);
}

// Winograd 3x3 conv (forward or dgrad): X [B][S+2][S+2][KIN] bf16, U the layer's fragment-major
// Winograd weights (rag_wino_pack), Y padded with halo HO and YC >= NOUT channels, mask (dgrad) with halo HM.
// `pending`: a deferred wgrad reduction handle (conv.hip PendingRed) or null.
// half (192-wide tiles only): run half-board blocks whenever the shape has them (wino_half_ok),
// not only when the one-board grid would leave a ragged wave -- for launches that share the chip
// with long resident kernels (the search's GPU rollouts hold a 128-VGPR wave on most CUs: a
// one-board block needs 2 x 244 VGPRs on every SIMD, a half-board block 2 x 165).
int rag_conv_wino_launch(const void* X, const void* W, const float* bias, void* Y,
                         const void* mask, int B, int S, int KIN, int NOUT, int HO, int YC,
                         int relu, int HM, hipStream_t stream, const WgradRed* red, int half) {
  if (!rag_conv_wino_ok(S, 1, KIN, NOUT, 3) || YC < NOUT || B <= 0) return -1;
  const int nb = wino_boards_per_block(S);
  WgradRed r{};
  if (red) r = *red;
  const int wt = wino_tile(NOUT, S);
  const dim3 grid((B + nb - 1) / nb, NOUT / wt);
  if (wt == 192 && ((half && wino_half_ok(S, NOUT)) || wino_mode(B, S, KIN, NOUT) == 2))
    conv_wino_kernel<192, true, kHalfPairs><<<dim3(2 * B, NOUT / wt), 512, 0, stream>>>(
        (const bf16*)X, (const bf16*)W, bias, (bf16*)Y, (const bf16*)mask, B, S, KIN, NOUT, HO,
        YC, relu, HM, 1, r);
  else if (wt == 128)
    conv_wino_kernel<128, true><<<grid, 512, 0, stream>>>((const bf16*)X, (const bf16*)W, bias,
                                                          (bf16*)Y, (const bf16*)mask, B, S, KIN,
                                                          NOUT, HO, YC, relu, HM, nb, r);
  else if (nb == 1)
    conv_wino_kernel<192, true><<<grid, 512, 0, stream>>>((const bf16*)X, (const bf16*)W, bias,
                                                          (bf16*)Y, (const bf16*)mask, B, S, KIN,
                                                          NOUT, HO, YC, relu, HM, nb, r);
  else
    conv_wino_kernel<192, false><<<grid, 512, 0, stream>>>((const bf16*)X, (const bf16*)W, bias,
                                                           (bf16*)Y, (const bf16*)mask, B, S, KIN,
                                                           NOUT, HO, YC, relu, HM, nb, r);
  return (int)hipGetLastError();
}

// The fused-BN forms (WinoBN, ResnetPolicy's 128-channel trunk): the 128-wide one-board tile at
// batches whose grid fills the chip.
static bool wino_bn_ok(int B, int S, int KIN, int NOUT) {
  return NOUT == 128 && KIN == 128 && S <= 64 && wino_tile(NOUT, S) == 128 &&
         wino_mode(B, S, KIN, NOUT) == 1;
}
RAG_API int rag_conv_wino_bn_ok(int B, int S, int KIN, int NOUT) {
  return wino_bn_ok(B, S, KIN, NOUT);
}

// Forward (coef: BN prologue on X, res optional) or dgrad (mcoef: mask = the BN input x) form;
// spart [B][2][S] optional, smean with mcoef only. -5 if the shape or the argument set has no
// kernel.
int rag_conv_wino_bn_launch(const void* X, const void* W, const float* bias, void* Y,
                            const void* mask, const void* res, int B, int S, int KIN, int NOUT,
                            int HO, int YC, int relu, int HM, hipStream_t stream,
                            const WgradRed* red, const float* coef, const float* mcoef,
                            float* spart, const float* smean) {
  if (!wino_bn_ok(B, S, KIN, NOUT) || YC < NOUT || (coef != nullptr) == (mcoef != nullptr) ||
      (mcoef && (!mask || res)) || (smean && !mcoef))
    return -5;
  WgradRed r{};
  if (red) r = *red;
  if (coef)
    conv_wino_kernel<128, true, kWP, 1><<<B, 512, 0, stream>>>(
        (const bf16*)X, (const bf16*)W, bias, (bf16*)Y, nullptr, B, S, KIN, NOUT, HO, YC, relu,
        HM, 1, r, WinoBN{coef, (const bf16*)res, spart, nullptr});
  else
    conv_wino_kernel<128, true, kWP, 2><<<B, 512, 0, stream>>>(
        (const bf16*)X, (const bf16*)W, bias, (bf16*)Y, (const bf16*)mask, B, S, KIN, NOUT, HO,
        YC, relu, HM, 1, r, WinoBN{mcoef, nullptr, spart, smean});
  return (int)hipGetLastError();
}

RAG_API int rag_conv_wino(const void* X, const void* W, const float* bias, void* Y,
                          const void* mask, int B, int S, int KIN, int NOUT, int HO, int YC,
                          int relu, int HM, hipStream_t stream) {
  return rag_conv_wino_launch(X, W, bias, Y, mask, B, S, KIN, NOUT, HO, YC, relu, HM, stream,
                              nullptr, 0);
}

// table: kWinoPackFields int64 per layer (W, COUT, CIN, COUTP, CINP, Uf or 0, Ub or 0, Wd or 0).
// goff / lr / wd / sgd_on: the optimizer step folded in (rag_pack_trunk)
RAG_API int rag_wino_pack(const int64_t* table, int nlayers, int max_tiles, hipStream_t stream,
                          int64_t goff, float lr, float wd, int sgd_on) {
  if (nlayers <= 0 || max_tiles <= 0) return -1;
  // 32 x 16 tiles: at most 8 per 64 x 64 tile of the widest layer (wino_pack_kernel)
  const dim3 grid((unsigned)(8 * max_tiles), (unsigned)nlayers);
  wino_pack_kernel<<<grid, 256, 0, stream>>>(table, SgdFold{(long)goff, lr, wd, sgd_on});
  return (int)hipGetLastError();
}

// One launch for a fused trunk's whole weight update (pack_step_kernel): the pack_trunk rows of
// `ttable` (nrows, nfull: rag_pack_trunk's table and split; kernels up to max_taps taps, at most
// 49), the Winograd rows of `wtable` (nwino, rag_wino_pack's table; 0 = none), on a grid `width`
// blocks wide (at least 8 per 64 x 64 tile of the widest Winograd layer, and the widest
// pack_trunk layer's 16 x 16 tiles), and -- with the fold -- plain SGD over up to two ranges
// [a0, a0 + n0), [a1, a1 + n1) of the flat buffer `flat`.
RAG_API int rag_pack_step(const int64_t* wtable, int nwino, const int64_t* ttable, int nrows,
                          int nfull, int max_taps, int width, hipStream_t stream, int64_t goff,
                          float lr, float wd, int sgd_on, float* flat, int64_t a0, int64_t n0,
                          int64_t a1, int64_t n1) {
  if (nwino < 0 || nrows < 0 || nfull < 0 || nfull > nrows || width <= 0 || max_taps < 1 ||
      max_taps > kPTaps || n0 < 0 || n1 < 0 || (nwino > 0 && !wtable) || (nrows > 0 && !ttable))
    return -1;
  const bool rest = sgd_on && n0 + n1 > 0;
  if (rest && !flat) return -1;
  const int trows = nfull + (nrows > nfull ? 1 : 0);
  const int rows = nwino + trows + (rest ? 1 : 0);
  if (rows == 0) return 0;
  const int l1 = kWinoPackLds, l2 = pack_trunk_lds(max_taps);
  const size_t lds = (size_t)(nfull > 0 && l2 > l1 ? l2 : l1) * sizeof(float);
  const SgdRest r{flat, (long)a0, rest ? (long)n0 : 0L, (long)a1, rest ? (long)n1 : 0L};
  pack_step_kernel<<<dim3((unsigned)width, (unsigned)rows), 256, lds, stream>>>(
      wtable, nwino, ttable, nrows, nfull, max_taps, SgdFold{(long)goff, lr, wd, sgd_on}, r);
  return (int)hipGetLastError();
}

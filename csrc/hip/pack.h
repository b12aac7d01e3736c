// Per-block bodies of the weight-repack kernels, shared by their own launches (conv.hip
// pack_trunk_kernel, conv_wino.hip wino_pack_kernel) and by the one launch that packs a whole
// trunk after an optimizer step (conv_wino.hip pack_step_kernel). Each body takes its block
// coordinates and its LDS tile as arguments; every early return is block-uniform. The bodies
// are force-inlined: as called functions (hipcc's choice for a body called from two kernels)
// they ran with a stack frame and reached their LDS tile through generic (flat) pointers.
#pragma once
#include "common.h"

namespace rag {

// Buffer resource over a block-uniform fp32 base (the packing kernels' master tiles): 32-bit
// element offsets instead of a 64-bit address per load keep the 32-36 loads a thread has in
// flight within 128 VGPRs (with flat addresses hipcc gave the Winograd repack 232 VGPRs, i.e.
// two blocks per CU and its 792 blocks in two rounds). An offset of kPackOob reads 0.
constexpr uint32_t kPackOob = 0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t pack_rsrc(const float* p) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo),
                                           (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ float pack_ld(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
__device__ __forceinline__ void pack_st(__amdgpu_buffer_rsrc_t r, uint32_t off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, off, 0, 0);
}

// ---- direct GEMM layouts (pack_trunk). `table` holds kPackFields int64 per layer: W, b (or 0),
// COUT, CIN, KS, COUTP, CINP, Wf (or 0), Wb (or 0), bias_out (or 0), first element index.
// A block packs 16 (n) x 16 (c) tiles of one layer, all its taps, grid-strided over the layer's
// tiles. A tile's OIHW masters are 16 runs of 16 * taps contiguous floats, read (and with the SGD
// fold stepped and written back) coalesced, every load before any store; they go through LDS so
// that both bf16 layouts are written along their contiguous dimension: the forward layout
// [tap][n][c] along c, the dgrad layout [tap'][c][n] along n. (Until round 6: one block per tap
// of a 64 x 64 tile, whose lanes read 1 of every taps floats: 15-17 us per SL step for the 5x5
// layer alone, and scattered 4-byte master writes from 25 blocks per cache line with the fold.)
constexpr int kPackFields = 11;
constexpr int kPT = 16, kPTaps = 49;  // tile edge; taps of the largest kernel packed (7x7)

// LDS floats a pack_trunk block needs for kernels of `taps` taps
__host__ __device__ constexpr int pack_trunk_lds(int taps) { return taps * kPT * (kPT + 1); }

// Grid row `y` of a pack_trunk launch: rows [0, nfull) pack weights, row nfull (if nrows > nfull)
// pads the biases of the bias-only rows [nfull, nrows), one block each.
__device__ __forceinline__ void pack_trunk_block(const int64_t* __restrict__ table, int y,
                                                 int nrows, int nfull, SgdFold sgd, int bx,
                                                 int gx, int max_taps, float* __restrict__ tl) {
  // the padded bias of a layer (its fp32 master stepped first with sgd.on)
  auto pack_bias = [&](float* b, int COUT, int COUTP, float* bo) {
    for (int n = threadIdx.x; n < COUTP; n += blockDim.x) {
      const float v = (b && n < COUT) ? sgd.step(b + n) : 0.f;
      if (bo) bo[n] = v;
    }
  };
  if (y == nfull) {  // the bias-only rows (after the nfull packed ones): one block each
    for (int r = nfull + bx; r < nrows; r += gx) {
      const int64_t* t = table + (size_t)r * kPackFields;
      pack_bias((float*)t[1], (int)t[2], (int)t[5], (float*)t[9]);
    }
    return;
  }
  const int64_t* t = table + (size_t)y * kPackFields;
  float* W = (float*)t[0];
  float* b = (float*)t[1];
  const int COUT = (int)t[2], CIN = (int)t[3], KS = (int)t[4], COUTP = (int)t[5],
            CINP = (int)t[6];
  bf16* Wf = (bf16*)t[7];
  bf16* Wb = (bf16*)t[8];
  float* bo = (float*)t[9];
  if (bx == 0) pack_bias(b, COUT, COUTP, bo);
  if (!Wf && !Wb) return;  // bias-only row (a Winograd layer: its wino_pack row packs the weights)
  const int taps = KS * KS;
  if (taps > max_taps) return;  // (the host never builds such a row: see the launchers)
  const int ntc = (CINP + kPT - 1) / kPT, ntiles = ((COUTP + kPT - 1) / kPT) * ntc;
  const int row = kPT * taps;  // contiguous masters per output channel of a tile
  const int tid = threadIdx.x;
  for (int tile = bx; tile < ntiles; tile += gx) {
    const int n0 = (tile / ntc) * kPT, c0 = (tile % ntc) * kPT;
    // element tid + 256 i of the tile (i < taps), in chunks of 16 per thread: each chunk's
    // loads all go out before its stores
    // the tile's masters from W + (n0 CIN + c0) taps: row r, element e at r CIN taps + e
    const float* wt = W + (size_t)(n0 * CIN + c0) * taps;
    const auto rw = pack_rsrc(wt), rg = pack_rsrc(wt + (sgd.on ? sgd.goff : 0));
    for (int i0 = 0; i0 < taps; i0 += 16) {
      float v[16], gr[16];
      // element k of the chunk: its offset (recomputed after the loads rather than held)
      auto offset = [&](int k) {
        const int i = i0 + k, idx = tid + 256 * i, r = idx / row, e = idx - r * row;
        const bool in = i < taps && n0 + r < COUT && c0 + e / taps < CIN;
        return in ? (uint32_t)((r * CIN * taps + e) * 4) : kPackOob;
      };
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const uint32_t o = offset(k);
        v[k] = pack_ld(rw, o);
        gr[k] = sgd.on ? pack_ld(rg, o) : 0.f;
      }
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int i = i0 + k, idx = tid + 256 * i, r = idx / row, e = idx - r * row;
        if (i >= taps) break;
        const int cl = e / taps, tap = e - cl * taps;
        const uint32_t o = offset(k);
        if (sgd.on && o != kPackOob) {
          v[k] = sgd.update(v[k], gr[k]);
          pack_st(rw, o, v[k]);
        }
        tl[(tap * kPT + r) * (kPT + 1) + cl] = v[k];
      }
    }
    __syncthreads();
    for (int it = tid; it < taps * kPT * kPT; it += 256) {
      const int tap = it / (kPT * kPT), q = it - tap * kPT * kPT;
      if (Wf) {  // c fastest
        const int cl = q % kPT, r = q / kPT, n = n0 + r, c = c0 + cl;
        if (n < COUTP && c < CINP)
          Wf[((size_t)tap * COUTP + n) * CINP + c] = (bf16)tl[(tap * kPT + r) * (kPT + 1) + cl];
      }
      if (Wb) {  // n fastest
        const int r = q % kPT, cl = q / kPT, n = n0 + r, c = c0 + cl;
        if (n < COUTP && c < CINP)
          Wb[((size_t)(taps - 1 - tap) * CINP + c) * COUTP + n] =
              (bf16)tl[(tap * kPT + r) * (kPT + 1) + cl];
      }
    }
    __syncthreads();  // tl is reused by the next tile
  }
}

// ---- Winograd weights of 3x3 layers (wino_pack) from the fp32 OIHW masters: forward Uf
// (N = COUTP, K = CINP) and dgrad Ub (N = CINP, K = COUTP: the same transform of the flipped,
// transposed kernel W[n][c][2-ky][2-kx]), tap (ky, q) = ky * 4 + q, each stored fragment-major
// [12][K / 32][N / 16][64][8]: element (n, k) of a tap at lane (n % 16) + 16 ((k % 32) / 8),
// position k % 8 of fragment (k / 32, n / 16), as a 16x16x32 MFMA A operand reads it.
// Wd (or 0): the direct dgrad layout [tap'][CINP][COUTP] (tap' = 8 - (3 ky + kx), pack_trunk's Wb)
// from the same LDS tile, for layers whose dgrad runs the direct kernel: the fp32 weights are
// read once per step instead of once more by pack_trunk.
constexpr int kWinoPackFields = 8;  // W, COUT, CIN, COUTP, CINP, Uf, Ub (or 0), Wd (or 0)
// One block per 32 (n) x 16 (c) tile of a layer, all 9 taps: the tile's OIHW masters are 32 rows
// of 16 x 9 = 144 contiguous floats, read (and with the SGD fold stepped and written back) with
// coalesced accesses, staged transposed in LDS, then written out as the forward / dgrad
// Winograd fragments and the direct dgrad layout. (The first version gave each block one kernel
// row of a 64 x 64 tile: 3 of every 9 floats per lane. With the fold its scattered 4-byte master
// writes, three blocks per cache line, took 41-43 us per SL step against 11.5 us unfolded.)
constexpr int kPackN = 32, kPackC = 16, kPackRow = kPackC * 9;
constexpr int kWinoPackLds = 9 * kPackN * (kPackC + 1);  // LDS floats of a wino_pack block

__device__ __forceinline__ void wino_pack_block(const int64_t* __restrict__ table, int y, int bx,
                                       SgdFold sgd, float* __restrict__ lds) {
  const int64_t* t = table + (size_t)y * kWinoPackFields;
  float* W = (float*)t[0];
  const int COUT = (int)t[1], CIN = (int)t[2], COUTP = (int)t[3], CINP = (int)t[4];
  bf16* Uf = (bf16*)t[5];
  bf16* Ub = (bf16*)t[6];
  bf16* Wd = (bf16*)t[7];
  const int ntc = (CINP + kPackC - 1) / kPackC, ntn = (COUTP + kPackN - 1) / kPackN;
  if (bx >= ntn * ntc) return;
  const int n0 = (bx / ntc) * kPackN, c0 = (bx % ntc) * kPackC;
  float(*tl)[kPackN][kPackC + 1] = reinterpret_cast<float(*)[kPackN][kPackC + 1]>(lds);
  const int tid = threadIdx.x;
  constexpr int kPer = kPackN * kPackRow / 256;  // 18 floats per thread
  // ---- masters (and gradients): every load before any store; the tile's masters from
  // W + (n0 CIN + c0) 9: row r, element e at r CIN 9 + e
  const float* wt = W + (size_t)(n0 * CIN + c0) * 9;
  const auto rw = pack_rsrc(wt), rg = pack_rsrc(wt + (sgd.on ? sgd.goff : 0));
  float v[kPer], gr[kPer];
  uint32_t off[kPer];
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int idx = tid + 256 * i, r = idx / kPackRow, e = idx - r * kPackRow;
    const int n = n0 + r, c = c0 + e / 9;
    off[i] = (n < COUT && c < CIN) ? (uint32_t)((r * CIN * 9 + e) * 4) : kPackOob;
    v[i] = pack_ld(rw, off[i]);
    gr[i] = sgd.on ? pack_ld(rg, off[i]) : 0.f;
  }
  if (sgd.on) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      if (off[i] != kPackOob) {
        v[i] = sgd.update(v[i], gr[i]);
        pack_st(rw, off[i], v[i]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int idx = tid + 256 * i, r = idx / kPackRow, e = idx - r * kPackRow;
    const int cl = e / 9, tap = e - cl * 9;
    tl[tap][r][cl] = v[i];
  }
  __syncthreads();
  const long tap_stride = (long)COUTP * CINP;
  // fragment-major offset of (n, k) in a [N][K] tap
  auto fm = [](int n, int k, int N) {
    return ((size_t)((k >> 5) * (N >> 4) + (n >> 4)) * 64 + (n & 15) + 16 * ((k & 31) >> 3)) * 8 +
           (k & 7);
  };
  // ---- forward Winograd weights: U_q of (n, c) at kernel row ky (c fastest across lanes)
  if (Uf) {
    for (int it = tid; it < 3 * kPackN * kPackC; it += 256) {
      const int cl = it % kPackC, r = (it / kPackC) % kPackN, ky = it / (kPackC * kPackN);
      const int n = n0 + r, c = c0 + cl;
      if (n >= COUTP || c >= CINP) continue;
      const float g0 = tl[3 * ky][r][cl], g1 = tl[3 * ky + 1][r][cl], g2 = tl[3 * ky + 2][r][cl];
      const size_t o = fm(n, c, COUTP);
      Uf[(ky * 4 + 0) * tap_stride + o] = (bf16)g0;
      Uf[(ky * 4 + 1) * tap_stride + o] = (bf16)(0.5f * (g0 + g1 + g2));
      Uf[(ky * 4 + 2) * tap_stride + o] = (bf16)(0.5f * (g0 - g1 + g2));
      Uf[(ky * 4 + 3) * tap_stride + o] = (bf16)g2;
    }
  }
  // ---- dgrad: N = cin, K = cout (n fastest across lanes); dgrad kernel row 2 - ky with its kx
  // flipped: (h0, h1, h2) = (g2, g1, g0)
  for (int it = tid; it < 3 * kPackN * kPackC; it += 256) {
    const int r = it % kPackN, cl = (it / kPackN) % kPackC, ky = it / (kPackC * kPackN);
    const int n = n0 + r, c = c0 + cl;
    if (n >= COUTP || c >= CINP) continue;
    const float h0 = tl[3 * ky + 2][r][cl], h1 = tl[3 * ky + 1][r][cl], h2 = tl[3 * ky][r][cl];
    if (Wd) {
#pragma unroll
      for (int kx = 0; kx < 3; ++kx)
        Wd[((size_t)(8 - (3 * ky + kx)) * CINP + c) * COUTP + n] = (bf16)tl[3 * ky + kx][r][cl];
    }
    if (Ub) {
      const int kyb = 2 - ky;
      const size_t o = fm(c, n, CINP);
      Ub[(kyb * 4 + 0) * tap_stride + o] = (bf16)h0;
      Ub[(kyb * 4 + 1) * tap_stride + o] = (bf16)(0.5f * (h0 + h1 + h2));
      Ub[(kyb * 4 + 2) * tap_stride + o] = (bf16)(0.5f * (h0 - h1 + h2));
      Ub[(kyb * 4 + 3) * tap_stride + o] = (bf16)h2;
    }
  }
}

}  // namespace rag

// Convolution weight gradient, "all taps per block" formulation (gfx950).
//
// When the layer input X and the output gradient G share one padded geometry (halo H >= ks/2 on
// both, WP = S + 2H), every tap of the convolution is a constant row shift in the flattened padded
// row space r = (b*WP + y)*WP + x:
//
//     dW[tap][n][c] = sum_r G[r][n] * X[r + (ky-h)*WP + (kx-h)][c]        (h = ks/2)
//
// G is zero on its halo rows, so the sum can run over ALL padded rows with no per-pixel masking.
// One block owns a 64(n) x 64(c) output tile for RG kernel rows (RG*ks taps) and a chunk of
// 64-row stages; per stage it stages 64 G rows and one X slab that covers every tap's shifted
// window, so X is read once per stage for all taps (instead of once per tap).
//
// Fragments come from LDS with ds_read_b64_tr_b16 (the reduction dim "pixels" is the row dim of
// both tiles). LDS rows are 160 bytes (64 channels + 16 pad): row starts then fall on banks
// r*40 mod 64, which are eight distinct 8-word windows for any 8 consecutive rows. The MFMA k
// index is permuted so that each 32-lane half of a transposed read touches 8 consecutive rows;
// this keeps every read bank-conflict free for ANY tap shift with no XOR swizzle, so all LDS
// addresses are a per-lane base plus an immediate.
#include "common.h"

using namespace rag;

namespace {

constexpr int kRS = 80;                      // LDS row stride (elements): 64 data + 16 pad
constexpr int kRowChunks = kRS / 8;          // 16-byte chunks per LDS row
constexpr int kBK = 64;                      // padded rows per stage
constexpr int kGInst = kBK * kRowChunks / 64;  // 10 glds instructions for the G tile
constexpr int kInst = 28;                    // glds per stage (7 per wave)
constexpr int kXRowsLoaded = (kInst - kGInst) * 64 / kRowChunks;  // 115 full X rows
constexpr int kXRowsAlloc = 116;
constexpr int kStageElems = (kBK + kXRowsAlloc) * kRS;
constexpr int kPerWave = kInst / 4;
static_assert(kGInst * 64 == kBK * kRowChunks, "G tile must fill whole instructions");
static_assert(kInst % 4 == 0, "uniform per-wave load count");

// k-row of MFMA fragment element (lane group g, element 4*hf + q): see header comment.
__device__ __forceinline__ int krow(int g, int q) { return (g & 1) * 4 + q + (g >> 1) * 8; }

template <int KS, int RG, int NBUF>
__global__ void __launch_bounds__(256, NBUF == 2 ? 2 : 1)
wgrad_taps_kernel(const bf16* __restrict__ G, const bf16* __restrict__ X,
                  float* __restrict__ part, float* __restrict__ bpart, int R, int WP, int GC,
                  int CIN, int spc, int COUTP, int CINP) {
  constexpr int NT = RG * KS;  // taps owned by this block
  constexpr int HK = KS / 2;
  __shared__ __attribute__((aligned(16))) bf16 lds[NBUF * kStageElems];

  const int lane = lane_id();
  const int w = wave_id();
  const int wn = w & 1, wc = w >> 1;
  const int ntn = COUTP / 64, ntc = CINP / 64;
  constexpr int NGRP = KS / RG;
  const int per_chunk = NGRP * ntn * ntc;
  const int wid = xcd_remap(blockIdx.x, gridDim.x);
  const int chunk = wid / per_chunk;
  int rem = wid - chunk * per_chunk;
  const int grp = rem / (ntn * ntc);
  rem -= grp * ntn * ntc;
  const int tn = rem / ntc, tc = rem - (rem / ntc) * ntc;
  const int n0 = tn * 64, c0 = tc * 64;
  const int ky0 = grp * RG;
  // X slab row 0 corresponds to shift (ky0-h)*WP - h relative to the G stage row 0
  const int xshift0 = (ky0 - HK) * WP - HK;

  const int steps = (R + kBK - 1) / kBK;
  const int sbeg = chunk * spc;
  int nsteps = steps - sbeg;
  nsteps = nsteps < spc ? nsteps : spc;

  // staging: instruction i = w + 4k covers chunk slots [64 i, 64 i + 64) of the stage
  int srow[kPerWave], scol[kPerWave];
#pragma unroll
  for (int k = 0; k < kPerWave; ++k) {
    const int i = w + 4 * k;
    int slot = i * 64 + lane;
    if (i >= kGInst) slot -= kGInst * 64;
    const int row = slot / kRowChunks;
    int ch = slot - row * kRowChunks;
    if (ch >= 8) ch -= 8;  // pad chunk: load a valid duplicate, never read
    srow[k] = row;
    scol[k] = ch * 8;
  }
  // Running per-lane source offsets (elements), advanced by one stage per issue; stages are
  // issued strictly in order. Only stages that touch the ends of the row range take the
  // clamped path.
  int soff[kPerWave];
#pragma unroll
  for (int k = 0; k < kPerWave; ++k) {
    const int i = w + 4 * k;
    soff[k] = i < kGInst ? (sbeg * kBK + srow[k]) * GC + n0 + scol[k]
                         : (sbeg * kBK + xshift0 + srow[k]) * CIN + c0 + scol[k];
  }
  auto stage = [&](int s, int buf) {
    const int r0 = (sbeg + s) * kBK;
    bf16* lb = lds + buf * kStageElems;
    const bool inside = r0 + xshift0 >= 0 && r0 + xshift0 + kXRowsLoaded <= R && r0 + kBK <= R;
    if (inside) {
#pragma unroll
      for (int k = 0; k < kPerWave; ++k) {
        const int i = w + 4 * k;  // wave-uniform
        glds16((i < kGInst ? G : X) + soff[k], lb + i * 512);
      }
    } else {
#pragma unroll
      for (int k = 0; k < kPerWave; ++k) {
        const int i = w + 4 * k;  // wave-uniform
        if (i < kGInst) {
          int r = r0 + srow[k];
          r = r < R ? r : R - 1;  // past the end: the last padded row is halo (zero)
          glds16(G + (size_t)r * GC + n0 + scol[k], lb + i * 512);
        } else {
          int r = r0 + xshift0 + srow[k];
          r = r < 0 ? 0 : (r < R ? r : R - 1);  // only ever paired with zero G rows
          glds16(X + (size_t)r * CIN + c0 + scol[k], lb + i * 512);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < kPerWave; ++k) soff[k] += w + 4 * k < kGInst ? kBK * GC : kBK * CIN;
  };

  f32x4 acc[NT][2][2];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int c = 0; c < 2; ++c) acc[t][a][c] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int kr = krow(g, q);
  // per-lane LDS element offsets (buffer 0); the rest are immediates
  const int gbase = kr * kRS + wn * 32 + 4 * p;
  int xbase[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int ky = t / KS, kx = t - (t / KS) * KS;
    xbase[t] = kBK * kRS + (kr + ky * WP + kx) * kRS + wc * 32 + 4 * p;
  }
  const bool do_bias = (bpart != nullptr) && grp == 0 && tc == 0;
  float bsum = 0.f;

  if (nsteps > 0) stage(0, 0);
  if (NBUF == 3 && nsteps > 1) stage(1, 1);
  for (int s = 0; s < nsteps; ++s) {
    if (NBUF == 3 && s + 1 < nsteps)
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" :: "n"(kPerWave) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int pf = NBUF - 1;
    if (s + pf < nsteps) stage(s + pf, (s + pf) % NBUF);
    const bf16* lb = lds + (s % NBUF) * kStageElems;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      // fragments are read in tap groups of TG (registers: 9 taps x 2 would spill at 2 blocks/CU)
      constexpr int TG = (NT > 5 && NT % 3 == 0) ? 3 : NT;
      bf16x8 fa[2];
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const bf16* p0 = lb + gbase + (32 * hh) * kRS + a * 16;
        fa[a] = tr_frag(p0, p0 + 16 * kRS);
      }
#pragma unroll
      for (int t0 = 0; t0 < NT; t0 += TG) {
        bf16x8 fb[TG][2];
#pragma unroll
        for (int u = 0; u < TG; ++u)
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            const bf16* p0 = lb + xbase[t0 + u] + (32 * hh) * kRS + c * 16;
            fb[u][c] = tr_frag(p0, p0 + 16 * kRS);
          }
        lds_reads_done();
#pragma unroll
        for (int u = 0; u < TG; ++u)
#pragma unroll
          for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int c = 0; c < 2; ++c)
              acc[t0 + u][a][c] = mfma16(fa[a], fb[u][c], acc[t0 + u][a][c]);
      }
    }
    if (do_bias && (int)threadIdx.x < 64) {
      const int c = threadIdx.x;
#pragma unroll 8
      for (int r = 0; r < kBK; ++r) bsum += (float)lb[r * kRS + c];
    }
  }

  // partial slab part[chunk][tap][n][c]; C layout: col = lane&15, row = 4*(lane>>4) + r
  const int taps = KS * KS;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int tap = ky0 * KS + t;
    float* dst = part + ((size_t)(chunk * taps + tap) * COUTP) * CINP;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int n = n0 + wn * 32 + a * 16 + g * 4;
        const int cc = c0 + wc * 32 + c * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) dst[(size_t)(n + r) * CINP + cc] = acc[t][a][c][r];
      }
  }
  if (do_bias && (int)threadIdx.x < 64) bpart[(size_t)chunk * COUTP + n0 + threadIdx.x] = bsum;
}

// LDS ring depth 2 (prefetch distance 1, two blocks per CU; 3 stages at one block per CU
// measured no faster, deleted round 5).
template <int KS, int RG>
void launch(const bf16* G, const bf16* X, float* part, float* bpart, int R, int WP, int GC,
            int CIN, int spc, int COUTP, int CINP, int nchunks, hipStream_t st) {
  dim3 grid(nchunks * (KS / RG) * (COUTP / 64) * (CINP / 64));
  wgrad_taps_kernel<KS, RG, 2><<<grid, 256, 0, st>>>(G, X, part, bpart, R, WP, GC, CIN, spc,
                                                     COUTP, CINP);
}

}  // namespace

// Does one stage's X slab (kXRowsLoaded rows) cover every shifted window of RG kernel rows?
bool rag_wgrad_taps_fits(int WP, int KS, int RG) {
  return kBK + (RG - 1) * WP + (KS - 1) <= kXRowsLoaded;
}

// Concurrent blocks the taps kernel is sized for (2 per CU with 2 LDS buffers).
int rag_wgrad_taps_target_blocks() { return 512; }

int rag_launch_wgrad_taps(const bf16* G, const bf16* X, float* part, float* bpart, int R, int WP,
                          int GC, int CIN, int spc, int COUTP, int CINP, int KS, int RG,
                          int nchunks, hipStream_t stream) {
  if (COUTP % 64 || CINP % 64 || GC % 8 || CIN % 8) return -1;
  if (!rag_wgrad_taps_fits(WP, KS, RG)) return -1;
  if (KS == 3 && RG == 3) launch<3, 3>(G, X, part, bpart, R, WP, GC, CIN, spc, COUTP, CINP, nchunks, stream);
  else if (KS == 3 && RG == 1) launch<3, 1>(G, X, part, bpart, R, WP, GC, CIN, spc, COUTP, CINP, nchunks, stream);
  else if (KS == 1 && RG == 1) launch<1, 1>(G, X, part, bpart, R, WP, GC, CIN, spc, COUTP, CINP, nchunks, stream);
  else if (KS == 5 && RG == 1) launch<5, 1>(G, X, part, bpart, R, WP, GC, CIN, spc, COUTP, CINP, nchunks, stream);
  else if (KS == 7 && RG == 1) launch<7, 1>(G, X, part, bpart, R, WP, GC, CIN, spc, COUTP, CINP, nchunks, stream);
  else return -2;
  return (int)hipGetLastError();
}

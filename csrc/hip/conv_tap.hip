// Tap-shared input slab implicit-GEMM 3x3 convolution for the 192-filter trunk (forward and dgrad).
//
// conv_pipe (conv_fwd.hip) stages a fresh 192-pixel x 32-channel A tile for every (tap, chunk)
// step: each pixel's channels are fetched nine times per layer. Here a block keeps conv_pipe's
// 192 (pixels) x 192 (channels) output tile and its 4 waves of 96 x 96, but for every 32-channel
// chunk it stages ONE slab holding the padded input rows of all nine taps (<= 298 rows for any
// 192-pixel run of 19x19 boards, staged as 320 rows of 64 B), and only the 192 x 32 weight tile is
// staged per (chunk, tap) step:
//   * pixel m = (b, i, j) reads padded row P(m) + ky*WI + kx, P(m) = (b*WI + i + s)*WI + j + s;
//     slab row = P(m) - P(m0) + ky*WI + kx: a lane keeps its fixed pixel offsets and adds the
//     (wave-uniform) tap offset per step;
//   * the 64-byte slab rows are swizzled on row bit 2 (chunk bit 1): a 16-lane ds_read_b128
//     group reads 16 rows that are consecutive except at a board-row wrap, which the row-bit-2
//     swizzle keeps conflict-free for any start row (conv_slab.hip's derivation);
//   * staging per chunk drops from 9 x 12 KB (A) + 9 x 12 KB (B) to 20 KB + 9 x 12 KB;
//   * pipeline: 3-slot weight ring, 2 slabs; loads for step s+2 are issued after the barrier of
//     step s, the next chunk's slab after the barrier of the chunk's first tap; counted
//     `s_waitcnt vmcnt(N)` (each wave issues 3 weight and 5 slab loads) + raw s_barrier.
// LDS: 2 x 20 KB + 3 x 12 KB = 76 KB -> two blocks per CU, like conv_pipe.
#include <algorithm>

#include "common.h"
#include "wgrad_part.h"

using namespace rag;

extern thread_local int g_conv_cin_real;  // conv.hip: real input channels of this launch

namespace {

constexpr int kBK = 32;
constexpr int kMT = 6, kNT = 6;       // 16-row fragments per wave along M / N
constexpr int kBM = 32 * kMT;         // 192 pixels
constexpr int kBN = 32 * kNT;         // 192 output channels
constexpr int kSlabRows = 320;        // >= 298 (worst 192-pixel run, 19x19, halo 1, 3x3)
constexpr int kSlab = kSlabRows * kBK;
constexpr int kBTile = kBN * kBK;
constexpr int kLds = 2 * kSlab + 3 * kBTile;
constexpr int kAL = kSlabRows / 64;   // slab glds per wave (16 rows each)
constexpr int kBL = kBN / 64;         // weight glds per wave

__device__ __forceinline__ int swz4(int row) { return ((row >> 2) & 1) << 1; }

template <int V> struct IntC {
  static constexpr int value = V;
};

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// epilogue (as conv_pipe): lane owns channels n..n+3 of pixel m for every (j, i) tile
// BN column statistics of a conv output (BN fusion, ResnetPolicy): `sred` is an LDS [2][64] float
// accumulator of this block (sum, sum of squares per board column of the stored bf16 values).
// The four lanes of a pixel (fq) are combined by shuffles, then one lane per pixel adds to LDS.
__device__ __forceinline__ void stats_add_pixel(float* sred, int valid, int col, float s0,
                                                float s1, int fq) {
  s0 += __shfl_xor(s0, 16, 64);
  s1 += __shfl_xor(s1, 16, 64);
  s0 += __shfl_xor(s0, 32, 64);
  s1 += __shfl_xor(s1, 32, 64);
  if (fq == 0 && valid) {
    atomicAdd(sred + col, s0);
    atomicAdd(sred + 64 + col, s1);
  }
}

template <int NT = kNT, int MT = kMT>
__device__ __forceinline__ void epilogue(const f32x4 (&acc)[NT][MT], int mw, int nw, int M,
                                         int S, int WO, int HO, int YC, int HM,
                                         const float* __restrict__ bias,
                                         const bf16* __restrict__ res, int relu,
                                         const bf16* __restrict__ mask, bf16* __restrict__ Y,
                                         int frow, int fq, float* sred = nullptr) {
  const int S2 = S * S;
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int m = mw + i * 16 + frow;
    if (sred) {  // uniform: every lane takes part in the shuffles
      float s0 = 0.f, s1 = 0.f;
      int col = 0;
      if (m < M) {
        const int rem = m % S2;
        col = rem % S;
        const size_t orow = (size_t)(((m / S2) * WO + rem / S + HO) * WO + col + HO) * YC;
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const int n = nw + j * 16 + fq * 4;
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = acc[j][i][r];
          if (bias) {
            const float4 bb = *reinterpret_cast<const float4*>(bias + n);
            v[0] += bb.x;
            v[1] += bb.y;
            v[2] += bb.z;
            v[3] += bb.w;
          }
          if (res) {
            const bf16x4 rv = *reinterpret_cast<const bf16x4*>(res + orow + n);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += (float)rv[r];
          }
          bf16x4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            o[r] = (bf16)(relu ? fmaxf(v[r], 0.f) : v[r]);
            const float q = (float)o[r];
            s0 += q;
            s1 = fmaf(q, q, s1);
          }
          *reinterpret_cast<bf16x4*>(Y + orow + n) = o;
        }
      }
      stats_add_pixel(sred, m < M, col, s0, s1, fq);
      continue;
    }
    if (m >= M) continue;
    const int b = m / S2;
    const int rem = m - b * S2;
    const int pi = rem / S;
    const int pj = rem - pi * S;
    const size_t orow = (size_t)((b * WO + pi + HO) * WO + pj + HO) * YC;
    const int WMK = S + 2 * HM;
    const size_t mrow = (size_t)((b * WMK + pi + HM) * WMK + pj + HM) * YC;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int n = nw + j * 16 + fq * 4;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[j][i][r];
      if (bias) {
        const float4 bb = *reinterpret_cast<const float4*>(bias + n);
        v[0] += bb.x;
        v[1] += bb.y;
        v[2] += bb.z;
        v[3] += bb.w;
      }
      if (res) {
        const bf16x4 rv = *reinterpret_cast<const bf16x4*>(res + orow + n);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += (float)rv[r];
      }
      if (relu) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
      }
      if (mask) {
        const bf16x4 mk = *reinterpret_cast<const bf16x4*>(mask + mrow + n);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = ((float)mk[r] > 0.f) ? v[r] : 0.f;
      }
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (bf16)v[r];
      *reinterpret_cast<bf16x4*>(Y + orow + n) = o;
    }
  }
}

// Block-level epilogue through LDS (no residual): every wave writes its bias (+ReLU) tile as bf16
// into an LDS image [BM pixels][192 + 8 channels] (the 16-byte pad makes the 16 pixel rows of a
// ds_write_b64 lane group land on distinct banks), then the whole block writes pixel rows of
// 192 channels (384 contiguous bytes in the channels-last activation) with 16-byte lane chunks,
// applying the dgrad ReLU mask from equally coalesced reads. The register epilogue above writes
// 16 pixels x 32 bytes per store instruction; this one writes whole rows.
#ifndef RAG_EP_PREFETCH
#define RAG_EP_PREFETCH 512  // the ping-pong epilogue's mask prefetch (0: the per-chunk loads)
#endif
constexpr int kEpRow = kBN + 8;  // bf16 per LDS image row (192 channels; NT = 4: 136)
template <int BM, int NT = kNT, int MT = kMT, int NTHR = 0>
__device__ __forceinline__ void epilogue_lds(const f32x4 (&acc)[NT][MT], bf16* __restrict__ img,
                                             int mwl, int nwl, int m0, int n0, int M, int S,
                                             int WO, int HO, int YC, int HM,
                                             const float* __restrict__ bias, int relu,
                                             const bf16* __restrict__ mask,
                                             bf16* __restrict__ Y, int frow, int fq,
                                             const float* __restrict__ mcoef = nullptr,
                                             float* sred = nullptr,
                                             const float* __restrict__ smean = nullptr) {
  constexpr int EpRow = 32 * NT + 8;
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int n = nwl + j * 16 + fq * 4;
    float4 bb = {0.f, 0.f, 0.f, 0.f};
    if (bias) bb = *reinterpret_cast<const float4*>(bias + n0 + n);
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      float v[4] = {acc[j][i][0] + bb.x, acc[j][i][1] + bb.y, acc[j][i][2] + bb.z,
                    acc[j][i][3] + bb.w};
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (bf16)(relu ? fmaxf(v[r], 0.f) : v[r]);
      *reinterpret_cast<bf16x4*>(img + (mwl + i * 16 + frow) * EpRow + n) = o;
    }
  }
  const int S2 = S * S, WMK = S + 2 * HM;
  constexpr int kChunks = 32 * NT / 8;  // 16-byte chunks per pixel row
  // NTHR (the block size, when the caller fixes it): every mask chunk of this thread is loaded
  // here, before the barrier, all in flight at once, instead of one dependent load per row
  // chunk inside the store loop (dgrad: the mask read was that loop's latency chain)
  constexpr int kIt = NTHR > 0 ? (BM * kChunks + NTHR - 1) / NTHR : 1;
  bf16x8 mkp[kIt];
  if constexpr (NTHR > 0) {
    if (mask) {
#pragma unroll
      for (int it = 0; it < kIt; ++it) {
        const int c = threadIdx.x + it * NTHR;
        const int row = c / kChunks, k8 = (c - row * kChunks) * 8;
        const int m = m0 + row;
        if (c < BM * kChunks && m < M) {
          const int b = m / S2;
          const int rem = m - b * S2;
          const int pi = rem / S, pj = rem - pi * S;
          mkp[it] = *reinterpret_cast<const bf16x8*>(
              mask + (size_t)((b * WMK + pi + HM) * WMK + pj + HM) * YC + n0 + k8);
        }
      }
    }
  }
  __syncthreads();
  // with statistics (128-channel tiles only): kChunks consecutive threads own one pixel row
  // (kChunks | 64, and BM * kChunks a multiple of the block size, so every thread runs the same
  // iterations)
  if constexpr (64 % kChunks == 0) if (sred) {
    const int step = NTHR > 0 ? NTHR : (int)blockDim.x;
    const int nit = NTHR > 0 ? kIt : (BM * kChunks - (int)threadIdx.x + step - 1) / step;
#pragma unroll
    for (int it = 0; it < nit; ++it) {
      const int c = threadIdx.x + it * step;
      if (NTHR > 0 && c >= BM * kChunks) break;
      const int row = c / kChunks, k8 = (c - row * kChunks) * 8;
      const int m = m0 + row;
      float s0 = 0.f, s1 = 0.f;
      int pj = 0;
      if (m < M) {
        const int b = m / S2;
        const int rem = m - b * S2;
        const int pi = rem / S;
        pj = rem - pi * S;
        bf16x8 v = *reinterpret_cast<const bf16x8*>(img + row * EpRow + k8);
        if (mask) {
          bf16x8 mk;
          if constexpr (NTHR > 0)
            mk = mkp[it];
          else
            mk = *reinterpret_cast<const bf16x8*>(
                mask + (size_t)((b * WMK + pi + HM) * WMK + pj + HM) * YC + n0 + k8);
          const float cx = mcoef ? mcoef[pj] : 0.f, cc = mcoef ? mcoef[2 * S + pj] : 0.f;
          const float mu = smean ? smean[pj] : 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float xm = (float)mk[e];
            const bool on = mcoef ? fmaf(cx, xm, cc) > 0.f : xm > 0.f;
            v[e] = on ? v[e] : (bf16)0.f;
            const float d = (float)v[e];
            s0 += d;
            s1 = fmaf(d, xm - mu, s1);  // backward: sum dy * (x - mean)
          }
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float q = (float)v[e];
            s0 += q;
            s1 = fmaf(q, q, s1);  // forward: sum x^2
          }
        }
        *reinterpret_cast<bf16x8*>(Y + (size_t)((b * WO + pi + HO) * WO + pj + HO) * YC + n0 +
                                   k8) = v;
      }
#pragma unroll
      for (int o = kChunks / 2; o > 0; o >>= 1) {
        s0 += __shfl_xor(s0, o, 64);
        s1 += __shfl_xor(s1, o, 64);
      }
      if ((threadIdx.x & (kChunks - 1)) == 0 && m < M) {
        atomicAdd(sred + pj, s0);
        atomicAdd(sred + 64 + pj, s1);
      }
    }
    return;
  }  // if (sred)
  const int step = NTHR > 0 ? NTHR : (int)blockDim.x;
  const int nit = NTHR > 0 ? kIt : (BM * kChunks - (int)threadIdx.x + step - 1) / step;
#pragma unroll
  for (int it = 0; it < nit; ++it) {
    const int c = threadIdx.x + it * step;
    if (NTHR > 0 && c >= BM * kChunks) break;
    const int row = c / kChunks, k8 = (c - row * kChunks) * 8;
    const int m = m0 + row;
    if (m >= M) continue;
    const int b = m / S2;
    const int rem = m - b * S2;
    const int pi = rem / S, pj = rem - pi * S;
    bf16x8 v = *reinterpret_cast<const bf16x8*>(img + row * EpRow + k8);
    if (mask) {
      bf16x8 mk;
      if constexpr (NTHR > 0)
        mk = mkp[it];
      else
        mk = *reinterpret_cast<const bf16x8*>(
            mask + (size_t)((b * WMK + pi + HM) * WMK + pj + HM) * YC + n0 + k8);
      if (mcoef) {
        // the layer input U = ReLU(cx[col] * x + cc[col]) was never stored (BN prologue): the
        // mask is recomputed from the BN input x and the column coefficients
        const float cx = mcoef[pj], cc = mcoef[2 * S + pj];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaf(cx, (float)mk[e], cc) > 0.f ? v[e] : (bf16)0.f;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = ((float)mk[e] > 0.f) ? v[e] : (bf16)0.f;
      }
    }
    *reinterpret_cast<bf16x8*>(Y + (size_t)((b * WO + pi + HO) * WO + pj + HO) * YC + n0 + k8) =
        v;
  }
}

// Blocks [nconv, gridDim.x) are not convolution tiles: they run a deferred wgrad partial-slab
// reduction (wgrad_part.h) in the block slots the convolution grid leaves free.
constexpr int kRedU = 14;  // chunk loads in flight per reduce thread
__global__ void __launch_bounds__(256, 2)
conv_tap_kernel(const bf16* __restrict__ X, const bf16* __restrict__ Wt,
                const float* __restrict__ bias, bf16* __restrict__ Y,
                const bf16* __restrict__ mask, const bf16* __restrict__ res, int M, int S,
                int WI, int shift, int WO, int HO, int CIN, int WROWS, int YC, int relu, int HM,
                long total_rows, int nconv, WgradRed red, int ep_lds) {
  static_assert(kLds >= kBM * kEpRow, "the LDS ring must hold the epilogue image");
  __shared__ __attribute__((aligned(16))) bf16 lds[kLds];
  if ((int)blockIdx.x >= nconv) {
    wslab_reduce_blocks<kRedU>(red, (int)blockIdx.x - nconv, (int)gridDim.x - nconv);
    return;
  }
  const int lane = lane_id();
  const int w = wave_id();
  const int wm = w & 1, wn = w >> 1;
  const int nblk_m = (M + kBM - 1) / kBM;
  const int bid = xcd_remap(blockIdx.x, nconv);
  const int bm = bid % nblk_m, bn = bid / nblk_m;
  const int m0 = bm * kBM;
  const int n0 = bn * kBN;
  const int S2 = S * S;
  auto prow = [&](int m) {
    const int b = m / S2;
    const int rem = m - b * S2;
    const int i = rem / S;
    const int j = rem - i * S;
    return (long)(b * WI + i + shift) * WI + j + shift;
  };
  const long base = prow(m0);

  // staging sources (elements): slab rows (w + 4k)*16 + lane/4, weight rows likewise
  const bf16* asrc[kAL];
#pragma unroll
  for (int k = 0; k < kAL; ++k) {
    const int r = (w + 4 * k) * 16 + (lane >> 2);
    long g = base + r;
    g = g < total_rows ? g : total_rows - 1;
    asrc[k] = X + g * CIN + (((lane & 3) ^ swz4(r)) * 8);
  }
  const bf16* bsrc[kBL];
#pragma unroll
  for (int k = 0; k < kBL; ++k) {
    const int r = (w + 4 * k) * 16 + (lane >> 2);
    bsrc[k] = Wt + (long)(n0 + r) * CIN + (((lane & 3) ^ swz4(r)) * 8);
  }
  const long tap_stride = (long)WROWS * CIN;
  auto stage_a = [&](int q) {
    bf16* dst = lds + (q & 1) * kSlab;
#pragma unroll
    for (int k = 0; k < kAL; ++k) glds16(asrc[k] + q * kBK, dst + (w + 4 * k) * 16 * kBK);
  };
  auto stage_b = [&](int s) {  // step s = chunk * 9 + tap
    const int q = s / 9, t = s - q * 9;
    bf16* dst = lds + 2 * kSlab + (s % 3) * kBTile;
#pragma unroll
    for (int k = 0; k < kBL; ++k)
      glds16(bsrc[k] + t * tap_stride + q * kBK, dst + (w + 4 * k) * 16 * kBK);
  };

  const int frow = lane & 15;
  const int fq = lane >> 4;
  // slab row of each A fragment row for tap (0, 0); tap (ky, kx) adds ky*WI + kx
  int prel[kMT];
#pragma unroll
  for (int i = 0; i < kMT; ++i) {
    int m = m0 + wm * (16 * kMT) + i * 16 + frow;
    m = m < M ? m : M - 1;
    prel[i] = (int)(prow(m) - base);
  }
  int boffs[kNT];
#pragma unroll
  for (int j = 0; j < kNT; ++j) {
    const int row = wn * (16 * kNT) + j * 16 + frow;
    boffs[j] = row * kBK + ((fq ^ swz4(row)) * 8);
  }

  f32x4 acc[kNT][kMT];
#pragma unroll
  for (int j = 0; j < kNT; ++j)
#pragma unroll
    for (int i = 0; i < kMT; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int cchunks = CIN / kBK;
  const int nsteps = 9 * cchunks;
  stage_a(0);
  stage_b(0);
  stage_b(1);

  for (int q = 0; q < cchunks; ++q) {
    const bool more = q + 1 < cchunks;
    const bf16* slab = lds + (q & 1) * kSlab;
    int ky = 0, kx = 0;
#pragma unroll 1
    for (int t = 0; t < 9; ++t) {
      const int s = q * 9 + t;
      // loads younger than the ones step s needs: B(s+1) (3 per wave) and, at taps 1-2, the next
      // chunk's slab (5 per wave, issued after B(q*9+2) at tap 0)
      if (t == 0 || t >= 3) {
        if (t == 8 && !more)
          wait_vm<0>();
        else
          wait_vm<kBL>();
      } else {
        if (more)
          wait_vm<kBL + kAL>();
        else
          wait_vm<kBL>();
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (s + 2 < nsteps) stage_b(s + 2);
      if (t == 0 && more) stage_a(q + 1);
      const bf16* bt = lds + 2 * kSlab + (s % 3) * kBTile;
      const int toff = ky * WI + kx;
      bf16x8 xa[kMT], wb[kNT];
#pragma unroll
      for (int i = 0; i < kMT; ++i) {
        const int r = prel[i] + toff;
        xa[i] = *reinterpret_cast<const bf16x8*>(slab + r * kBK + ((fq ^ swz4(r)) * 8));
      }
#pragma unroll
      for (int j = 0; j < kNT; ++j) wb[j] = *reinterpret_cast<const bf16x8*>(bt + boffs[j]);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int j = 0; j < kNT; ++j)
#pragma unroll
        for (int i = 0; i < kMT; ++i) acc[j][i] = mfma16(wb[j], xa[i], acc[j][i]);
      __builtin_amdgcn_s_setprio(0);
      if (++kx == 3) {
        kx = 0;
        ++ky;
      }
    }
  }

  if (ep_lds && !res) {
    __syncthreads();  // every wave is past its last LDS read: the ring becomes the output image
    epilogue_lds<kBM>(acc, lds, wm * (16 * kMT), wn * (16 * kNT), m0, n0, M, S, WO, HO, YC, HM,
                      bias, relu, mask, Y, frow, fq);
  } else {
    epilogue(acc, m0 + wm * (16 * kMT), n0 + wn * (16 * kNT), M, S, WO, HO, YC, HM, bias, res,
             relu, mask, Y, frow, fq);
  }
}


// ---------------------------------------------------------------------------------------------
// 8-wave variant: one 512-thread block per CU owns 384 pixels x 192 channels (waves 4 (M) x 2 (N)
// of 96 x 96, the same wave tile), so every weight tile is staged once per 384 pixels instead of
// once per 192, and the weight ring is NB deep (NB-1 steps in flight, against the ~1 us LDS-DMA
// latency under load: MI355X_MICROARCH.md 'ldsdma-fill'). Slab: <= 554 rows for any 384-pixel
// run, staged as 640 rows (5 glds per wave). Weight tile: 12 glds per step, 2 for waves 0-3 and
// 1 for waves 4-7 (the counted waits use each wave's own count).
constexpr int k8BM = 384;
constexpr int k8SlabRows = 640;
constexpr int k8Slab = k8SlabRows * kBK;
constexpr int k8AL = k8SlabRows / 128;

__device__ __forceinline__ void wait_vm_rt(int n) {
  switch (n) {
    case 0: wait_vm<0>(); break;
    case 1: wait_vm<1>(); break;
    case 2: wait_vm<2>(); break;
    case 3: wait_vm<3>(); break;
    case 4: wait_vm<4>(); break;
    case 5: wait_vm<5>(); break;
    case 6: wait_vm<6>(); break;
    case 7: wait_vm<7>(); break;
    case 8: wait_vm<8>(); break;
    case 9: wait_vm<9>(); break;
    case 10: wait_vm<10>(); break;
    case 11: wait_vm<11>(); break;
    case 12: wait_vm<12>(); break;
    case 13: wait_vm<13>(); break;
    case 14: wait_vm<14>(); break;
    case 15: wait_vm<15>(); break;
    case 16: wait_vm<16>(); break;
    case 17: wait_vm<17>(); break;
    case 18: wait_vm<18>(); break;
    case 19: wait_vm<19>(); break;
    default: wait_vm<20>(); break;
  }
}

template <int NB>
__global__ void __launch_bounds__(512)
conv_tap8_kernel(const bf16* __restrict__ X, const bf16* __restrict__ Wt,
                 const float* __restrict__ bias, bf16* __restrict__ Y,
                 const bf16* __restrict__ mask, const bf16* __restrict__ res, int M, int S,
                 int WI, int shift, int WO, int HO, int CIN, int WROWS, int YC, int relu, int HM,
                 long total_rows) {
  constexpr int kL = 2 * k8Slab + NB * kBTile;
  __shared__ __attribute__((aligned(16))) bf16 lds[kL];
  const int lane = lane_id();
  const int w = wave_id();
  const int wm = w & 3, wn = w >> 2;
  const int nblk_m = (M + k8BM - 1) / k8BM;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int bm = bid % nblk_m, bn = bid / nblk_m;
  const int m0 = bm * k8BM;
  const int n0 = bn * kBN;
  const int S2 = S * S;
  auto prow = [&](int m) {
    const int b = m / S2;
    const int rem = m - b * S2;
    const int i = rem / S;
    const int j = rem - i * S;
    return (long)(b * WI + i + shift) * WI + j + shift;
  };
  const long base = prow(m0);

  const bf16* asrc[k8AL];
#pragma unroll
  for (int k = 0; k < k8AL; ++k) {
    const int r = (w + 8 * k) * 16 + (lane >> 2);
    long g = base + r;
    g = g < total_rows ? g : total_rows - 1;
    asrc[k] = X + g * CIN + (((lane & 3) ^ swz4(r)) * 8);
  }
  // weight rows: instruction i = w (all waves) and i = 8 + w (waves 0-3) of the 12 per step
  const int bl = w < 4 ? 2 : 1;
  const bf16* bsrc[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = w + 8 * k;
    const int r = (i < 12 ? i : 0) * 16 + (lane >> 2);
    bsrc[k] = Wt + (long)(n0 + r) * CIN + (((lane & 3) ^ swz4(r)) * 8);
  }
  const long tap_stride = (long)WROWS * CIN;
  auto stage_a = [&](int q) {
    bf16* dst = lds + (q & 1) * k8Slab;
#pragma unroll
    for (int k = 0; k < k8AL; ++k) glds16(asrc[k] + q * kBK, dst + (w + 8 * k) * 16 * kBK);
  };
  auto stage_b = [&](int s) {
    const int q = s / 9, t = s - q * 9;
    bf16* dst = lds + 2 * k8Slab + (s % NB) * kBTile;
    const long off = t * tap_stride + q * kBK;
    glds16(bsrc[0] + off, dst + w * 16 * kBK);
    if (w < 4) glds16(bsrc[1] + off, dst + (8 + w) * 16 * kBK);
  };

  const int frow = lane & 15;
  const int fq = lane >> 4;
  int prel[kMT];
#pragma unroll
  for (int i = 0; i < kMT; ++i) {
    int m = m0 + wm * (16 * kMT) + i * 16 + frow;
    m = m < M ? m : M - 1;
    prel[i] = (int)(prow(m) - base);
  }
  int boffs[kNT];
#pragma unroll
  for (int j = 0; j < kNT; ++j) {
    const int row = wn * (16 * kNT) + j * 16 + frow;
    boffs[j] = row * kBK + ((fq ^ swz4(row)) * 8);
  }

  f32x4 acc[kNT][kMT];
#pragma unroll
  for (int j = 0; j < kNT; ++j)
#pragma unroll
    for (int i = 0; i < kMT; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int cchunks = CIN / kBK;
  const int nsteps = 9 * cchunks;
  constexpr int D = NB - 1;  // weight tiles in flight ahead of the current step
  stage_a(0);
#pragma unroll
  for (int k = 0; k < D; ++k)
    if (k < nsteps) stage_b(k);

  for (int q = 0; q < cchunks; ++q) {
    const bool more = q + 1 < cchunks;
    const bf16* slab = lds + (q & 1) * k8Slab;
    int ky = 0, kx = 0;
#pragma unroll 1
    for (int t = 0; t < 9; ++t) {
      const int s = q * 9 + t;
      // younger than B(s): B(s+1 .. s+D-1) and, at taps 1..D, the next chunk's slab (issued at
      // tap 0 after B(q*9+D))
      int yb = nsteps - 1 - s;
      yb = yb < D - 1 ? yb : D - 1;
      wait_vm_rt(yb * bl + ((more && t >= 1 && t <= D) ? k8AL : 0));
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (s + D < nsteps) stage_b(s + D);
      if (t == 0 && more) stage_a(q + 1);
      const bf16* bt = lds + 2 * k8Slab + (s % NB) * kBTile;
      const int toff = ky * WI + kx;
      bf16x8 xa[kMT], wb[kNT];
#pragma unroll
      for (int i = 0; i < kMT; ++i) {
        const int r = prel[i] + toff;
        xa[i] = *reinterpret_cast<const bf16x8*>(slab + r * kBK + ((fq ^ swz4(r)) * 8));
      }
#pragma unroll
      for (int j = 0; j < kNT; ++j) wb[j] = *reinterpret_cast<const bf16x8*>(bt + boffs[j]);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int j = 0; j < kNT; ++j)
#pragma unroll
        for (int i = 0; i < kMT; ++i) acc[j][i] = mfma16(wb[j], xa[i], acc[j][i]);
      __builtin_amdgcn_s_setprio(0);
      if (++kx == 3) {
        kx = 0;
        ++ky;
      }
    }
  }
  epilogue(acc, m0 + wm * (16 * kMT), n0 + wn * (16 * kNT), M, S, WO, HO, YC, HM, bias, res, relu,
           mask, Y, frow, fq);
}

// ---------------------------------------------------------------------------------------------
// 8-wave variant of the same 192 x 192 block tile: waves 2 (M) x 4 (N) of 96 x 48, capped at 128
// VGPRs so two blocks give FOUR waves per SIMD (conv_tap_kernel: two). Each wave reads 6 slab + 3
// weight fragments for 18 MFMAs per step; the LDS layout, swizzles, staging ring and counted
// waits are conv_tap_kernel's, with the 20 slab / 12 weight glds of a step split 3+2 / 2+1
// between waves 0-3 and 4-7 (each wave waits on its own count).
constexpr int k16NT = 3;

__global__ void __launch_bounds__(512, 4)  // 4 waves per SIMD (EU): <= 128 VGPRs
conv_tap16_kernel(const bf16* __restrict__ X, const bf16* __restrict__ Wt,
                  const float* __restrict__ bias, bf16* __restrict__ Y,
                  const bf16* __restrict__ mask, const bf16* __restrict__ res, int M, int S,
                  int WI, int shift, int WO, int HO, int CIN, int WROWS, int YC, int relu, int HM,
                  long total_rows) {
  __shared__ __attribute__((aligned(16))) bf16 lds[kLds];
  const int lane = lane_id();
  const int w = wave_id();
  const bool lo4 = w < 4;
  const int wm = w & 1, wn = w >> 1;
  const int nblk_m = (M + kBM - 1) / kBM;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int bm = bid % nblk_m, bn = bid / nblk_m;
  const int m0 = bm * kBM;
  const int n0 = bn * kBN;
  const int S2 = S * S;
  auto prow = [&](int m) {
    const int b = m / S2;
    const int rem = m - b * S2;
    const int i = rem / S;
    const int j = rem - i * S;
    return (long)(b * WI + i + shift) * WI + j + shift;
  };
  const long base = prow(m0);

  // slab glds i = w + 8k (k = 0, 1, and 2 for waves 0-3): rows 16 i .. 16 i + 15; weight glds
  // i = w + 8k (k = 0, and 1 for waves 0-3). Source addresses are recomputed at each issue (a few
  // VALU per glds) instead of held in 64-bit registers, to stay within 128 VGPRs.
  const int lrow = lane >> 2;
  const int lcol = lane & 3;
  const long tap_stride = (long)WROWS * CIN;
  auto stage_a = [&](int q) {
    bf16* dst = lds + (q & 1) * kSlab;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      if (k == 2 && !lo4) break;
      const int r = (w + 8 * k) * 16 + lrow;
      long g = base + r;
      g = g < total_rows ? g : total_rows - 1;
      glds16(X + g * CIN + ((lcol ^ swz4(r)) * 8) + q * kBK, dst + (w + 8 * k) * 16 * kBK);
    }
  };
  auto stage_b = [&](int s) {  // step s = chunk * 9 + tap
    const int q = s / 9, t = s - q * 9;
    bf16* dst = lds + 2 * kSlab + (s % 3) * kBTile;
    const bf16* src = Wt + t * tap_stride + q * kBK;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (k == 1 && !lo4) break;
      const int r = (w + 8 * k) * 16 + lrow;
      glds16(src + (long)(n0 + r) * CIN + ((lcol ^ swz4(r)) * 8), dst + (w + 8 * k) * 16 * kBK);
    }
  };

  const int frow = lane & 15;
  const int fq = lane >> 4;
  int prel[kMT];
#pragma unroll
  for (int i = 0; i < kMT; ++i) {
    int m = m0 + wm * (16 * kMT) + i * 16 + frow;
    m = m < M ? m : M - 1;
    prel[i] = (int)(prow(m) - base);
  }
  int boffs[k16NT];
#pragma unroll
  for (int j = 0; j < k16NT; ++j) {
    const int row = wn * (16 * k16NT) + j * 16 + frow;
    boffs[j] = row * kBK + ((fq ^ swz4(row)) * 8);
  }

  f32x4 acc[k16NT][kMT];
#pragma unroll
  for (int j = 0; j < k16NT; ++j)
#pragma unroll
    for (int i = 0; i < kMT; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int cchunks = CIN / kBK;
  const int nsteps = 9 * cchunks;
  stage_a(0);
  stage_b(0);
  stage_b(1);

  for (int q = 0; q < cchunks; ++q) {
    const bool more = q + 1 < cchunks;
    const bf16* slab = lds + (q & 1) * kSlab;
    int ky = 0, kx = 0;
#pragma unroll 1
    for (int t = 0; t < 9; ++t) {
      const int s = q * 9 + t;
      // as conv_tap_kernel: younger than B(s) are B(s+1) and, at taps 1-2, the next slab
      const bool last = t == 8 && !more;
      const bool with_a = more && (t == 1 || t == 2);
      if (lo4) {
        if (last) wait_vm<0>(); else if (with_a) wait_vm<5>(); else wait_vm<2>();
      } else {
        if (last) wait_vm<0>(); else if (with_a) wait_vm<3>(); else wait_vm<1>();
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (s + 2 < nsteps) stage_b(s + 2);
      if (t == 0 && more) stage_a(q + 1);
      const bf16* bt = lds + 2 * kSlab + (s % 3) * kBTile;
      const int toff = ky * WI + kx;
      bf16x8 xa[kMT], wb[k16NT];
#pragma unroll
      for (int i = 0; i < kMT; ++i) {
        const int r = prel[i] + toff;
        xa[i] = *reinterpret_cast<const bf16x8*>(slab + r * kBK + ((fq ^ swz4(r)) * 8));
      }
#pragma unroll
      for (int j = 0; j < k16NT; ++j) wb[j] = *reinterpret_cast<const bf16x8*>(bt + boffs[j]);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int j = 0; j < k16NT; ++j)
#pragma unroll
        for (int i = 0; i < kMT; ++i) acc[j][i] = mfma16(wb[j], xa[i], acc[j][i]);
      __builtin_amdgcn_s_setprio(0);
      if (++kx == 3) {
        kx = 0;
        ++ky;
      }
    }
  }

  epilogue<k16NT>(acc, m0 + wm * (16 * kMT), n0 + wn * (16 * k16NT), M, S, WO, HO, YC, HM, bias,
                  res, relu, mask, Y, frow, fq);
}

// ---------------------------------------------------------------------------------------------
// Ping-pong 8-wave kernel (conv_tap_pp_kernel): one 512-thread block per CU owns 384 pixels x 192
// channels with the same 96 x 96 wave tiles, split into two wave GROUPS that alternate roles at
// every barrier so that the two waves sharing a SIMD (wave w and w + 4) never want the matrix pipe
// at the same time:
//
//   phase A(s):  group 0 reads step s's fragments (and issues the staging loads)
//                group 1 runs the MFMAs of step s - 1
//   ---- s_barrier ----
//   phase B(s):  group 0 runs the MFMAs of step s
//                group 1 reads step s's fragments
//   ---- s_barrier ----
//
// Each wave still holds ONE fragment set (read(s) is always after its own MFMA(s-1)), so no second
// register set is needed; the pipe alternates between the two partners' 36-MFMA segments while
// the other partner's LDS reads / DMA issue run beside them. Group 0 (waves 0-3, pixels 0-191)
// issues every global->LDS load (3 weight glds per step, 10 slab glds per chunk per wave), so
// only its waves wait on vmcnt; group 1 (waves 4-7, pixels 192-383) only reads LDS and multiplies.
// LDS: 2 slabs x 640 rows (>= 554 for any 384-pixel run) + NB weight slots: 80 + NB x 12 KB.
// Hazards (RAW / WAR) are ordered by the two barriers per step: B(s) is retired by group 0's
// counted wait before X_s and read by group 0 in A(s) and group 1 in B(s); slot (s+D) % NB is
// rewritten after X_s, when its previous tile's last reader (group 1 in B(s+D-NB)) has passed
// X_{s+D-NB+1} (D <= NB-1); every read burst ends with lgkmcnt(0) before the wave's next barrier.
constexpr int kPPBM = 384;
constexpr int kPPSlabRows = 640;
constexpr int kPPSlab = kPPSlabRows * kBK;
constexpr int kPPAL = kPPSlabRows / 64;  // slab glds per loader wave (4 loader waves x 16 rows)
constexpr int kPPSlabRows5 = 768;        // 5x5 taps (12 glds per loader wave)
constexpr int kPPSlabRows192 = 320;      // 192-pixel blocks (MT = 3, 5 glds per loader wave)
constexpr int kPPSlabRows192x5 = 448;    // 192-pixel blocks, 5x5 taps (<= 424 rows at 19x19)

// DIAG (diagnostic builds only, wrong results): bit 0 = no staging inside the loop, bit 1 = no
// fragment reads (MFMAs on stale registers), bit 2 = clock stamps (s_memtime / s_memrealtime of
// wave 0 around the main loop into `stamps`).
// BNP (ResnetPolicy, K13): the input slab is X = the BN input x, and the loader waves turn each
// staged slab into U = ReLU(cx[col] * x + cc[col]) in place (zero on halo rows) before the barrier
// that publishes it, with bnc = the BN's [3][S] column coefficients; U is never written to HBM.
// mcoef: the dgrad form of the same fusion (mask = U > 0 recomputed from x, see epilogue_lds).
// spart: this block's BN column statistics of the output ([blockIdx][2][S] partials for
// bn.hip's finalize): (sum, sum of squares) of the stored output in the forward, or with smean
// (the BN's mean) (sum dU, sum dU * (x - mean)) of the masked dgrad output, x = `mask`. They
// replace the separate statistics passes over the activation.
// SPREAD: the loader group issues the next chunk's slab loads a few per step over taps
// 0 .. TAPS-2 instead of all of them at tap 0 (the tap-0 read phase otherwise carries ~10 DMA
// issues and holds the partner group at the next barrier).
// WG0: of the PPBL weight slices of a step, the last WG0 are staged by the loader group 0 right
// after its MFMA segment (balancing the two groups' non-MFMA phases; group 1 stages the rest).
// PRIO: one static s_setprio 1 for group 1 (the second-dispatched half) and no per-segment
// priority flips (MI355X_MICROARCH.md, "Two waves per SIMD", item 4).
// PAIR (5x5 input layer with <= 48 real input channels padded to 64): the second 32-channel
// chunk holds only 16 real channels, so its steps pair two taps -- lanes of k-quads 0/1 read
// channels 32..47 of tap t, quads 2/3 the same channels of tap t+1 (channels 48..63 of tap 24,
// zero padding, for the last, unpaired tap) -- 25 + 13 = 38 K-steps instead of 50.
// K2 (the 128-channel 3x3 layers, NT = 4): each barrier pair covers two K-steps. A wave's 24
// MFMAs per step are shorter than its 10 fragment reads plus two barriers (the loop ran ~890
// cycles per phase for 384 MFMA cycles), so both groups hold two steps' fragments (80 VGPRs
// beside the 96 accumulators) and a phase is 48 MFMAs against 20 reads. The weight ring is
// NB = 6 tiles (two being read, two landed, two in flight); the next chunk's slab is issued at
// tap 1 (the super-step holding tap 0 may still read the chunk before, tap 8) and completes --
// and, with BNP, is transformed over taps 4..7 -- before the super-step that reads its tap 0.
// RS (register staging): the loop's staging goes through VGPRs instead of LDS-DMA. A
// global_load_lds piece costs 100-230 issue cycles inside a read phase (segment accounting:
// group 1's 2-3 weight pieces + wait took 427-519 cycles per step, group 0's slab pieces ~250);
// a global_load_dwordx4 issues in a few cycles and its ds_write_b128 lands a step later.
// RS = 1: group 1 loads the weight tile of step s+2 into registers after its fragment reads of
// step s and writes it to the ring at step s+1; RS = 2: also the next chunk's slab, two pieces
// per tap loaded after group 0's MFMA issue at taps 0..4 and written (BNP: transformed in
// registers, no LDS round trip) a tap later. Chunk 0's slab stays LDS-DMA (prologue).
template <int NB, int DIAG = 0, int ISSUE = 0, int NT = kNT, bool BNP = false, int KS = 3,
          int MT = kMT, int SPREAD = 0, int WG0 = 0, int PRIO = 0, int PAIR = 0, int K2 = 0,
          int RS = 0>
__global__ void __launch_bounds__(512, MT == kMT ? 1 : 4)
conv_tap_pp_kernel(const bf16* __restrict__ X, const bf16* __restrict__ Wt,
                   const float* __restrict__ bias, bf16* __restrict__ Y,
                   const bf16* __restrict__ mask, const bf16* __restrict__ res, int M, int S,
                   int WI, int shift, int WO, int HO, int CIN, int WROWS, int YC, int relu, int HM,
                   long total_rows, int nconv, WgradRed red, const float* __restrict__ bnc = nullptr,
                   const float* __restrict__ mcoef = nullptr, float* __restrict__ spart = nullptr,
                   const float* __restrict__ smean = nullptr, long long* stamps = nullptr) {
  constexpr int BN = 32 * NT, BTile = BN * kBK, PPBL = BN / 64, EpRow = BN + 8;
  constexpr int PB1 = PPBL - WG0;  // weight slices per step staged by group 1
  constexpr bool PR = PAIR && KS == 5;
  static_assert(!PAIR || (KS == 5 && !BNP && !ISSUE), "tap pairing: the 5x5 input layer");
  static_assert(WG0 >= 0 && PB1 >= 1 && (WG0 == 0 || (!BNP && !ISSUE)), "WG0 split");
  static_assert(!K2 || (KS == 3 && MT == kMT && NB >= 6 && !DIAG && !ISSUE && !SPREAD && !WG0 &&
                        !PAIR), "two K-steps per barrier pair: the plain 3x3 ping-pong");
  static_assert(!RS || (!ISSUE && !WG0 && !PAIR && !K2 && !(DIAG & 3)), "register staging");
  constexpr int TAPS = KS * KS;  // 9 (3x3) or 25 (the 5x5 layers: SL input, ResNet unit 0)
  // slab rows: 640 cover any 384-pixel run's 9-tap window (554), 768 its 25-tap one (748)
  // MT = 3: 192-pixel blocks (sub-chip grids, e.g. 128-game self-play passes): <= 298 rows
  constexpr int SR = KS == 3 ? (MT == kMT ? kPPSlabRows : kPPSlabRows192)
                             : (MT == kMT ? kPPSlabRows5 : kPPSlabRows192x5);
  constexpr int BM = 64 * MT;  // 4 wave rows of MT fragments
  static_assert(MT == kMT || (MT == 3 && !BNP), "192-pixel blocks: no BN prologue");
  constexpr int SLAB = SR * kBK, AL = SR / 64;
  static_assert(!BNP || KS == 3, "the BN prologue is a 3x3 path");
  static_assert(BN % 64 == 0, "the loader waves stage 64-row weight slices");
  constexpr int kLoop = 2 * SLAB + NB * BTile;
  constexpr int kL = kLoop > BM * EpRow ? kLoop : BM * EpRow;  // loop ring | epilogue image
  // weight tiles staged ahead of the current step (issued in the MFMA segment, the slot's last
  // reader is one phase further back: NB tiles ahead are safe)
  constexpr int D = (ISSUE == 1 || ISSUE == 2) ? NB : NB - 1;
  // + a [2][64] float BN-statistics accumulator past the ring / epilogue image
  __shared__ __attribute__((aligned(16))) bf16 lds[kL + 256];
  // claimed reductions (red.ticket) ride only in 128-wide launches: the 192-wide kernels keep
  // the static split and none of the claim code (SL -1 % with it compiled in, same-box A/B)
  constexpr bool kClaim = NT == 4;
  if ((int)blockIdx.x >= nconv) {
    if (kClaim && red.ticket)
      wslab_reduce_dynamic<kRedU>(red, reinterpret_cast<int*>(lds));
    else
      wslab_reduce_blocks<kRedU>(red, (int)blockIdx.x - nconv, (int)gridDim.x - nconv);
    return;
  }
  float* sred = spart ? reinterpret_cast<float*>(lds + kL) : nullptr;
  if (spart) {
    if (threadIdx.x < 128) sred[threadIdx.x] = 0.f;
    __syncthreads();
  }
  long long r_entry = 0;
  if constexpr (DIAG & 4) r_entry = __builtin_amdgcn_s_memrealtime();
  const int lane = lane_id();
  const int w = wave_id();
  const int grp = w >> 2;  // wave-uniform: waves w and w + 4 share a SIMD
  const int wl = w & 3;
  const int wm = grp * 2 + (wl & 1), wn = wl >> 1;
  const int nblk_m = (M + BM - 1) / BM;
  const int bid = xcd_remap(blockIdx.x, nconv);
  const int bm = bid % nblk_m, bn = bid / nblk_m;
  const int m0 = bm * BM;
  const int n0 = bn * BN;
  const int S2 = S * S;
  auto prow = [&](int m) {
    const int b = m / S2;
    const int rem = m - b * S2;
    const int i = rem / S;
    const int j = rem - i * S;
    return (long)(b * WI + i + shift) * WI + j + shift;
  };
  const long base = prow(m0);
  const long tap_stride = (long)WROWS * CIN;
  const int lrow = lane >> 2, lcol = lane & 3;

  // group 0's weight sources (row (wl + 4k)*16 + lane/4 of the 192-row tile)
  // BNP: per staged slab row of this lane (fixed across chunks: column BN), the coefficients of
  // U = ReLU(cx * x + cc); zero on halo / past-the-end rows, so U = 0 there
  float pcx[BNP ? AL : 1], pcc[BNP ? AL : 1];
  if constexpr (BNP) {
    const long WI2 = (long)WI * WI;
    const int hi = shift + 1;  // 3x3: the input halo
#pragma unroll
    for (int k = 0; k < AL; ++k) {
      const long g = base + (wl + 4 * k) * 16 + lrow;
      const long b = g / WI2;
      const int rem = (int)(g - b * WI2);
      const int ii = rem / WI, jj = rem - (rem / WI) * WI;
      const bool in = g < total_rows && ii >= hi && ii < hi + S && jj >= hi && jj < hi + S;
      pcx[k] = in ? bnc[jj - hi] : 0.f;
      pcc[k] = in ? bnc[2 * S + jj - hi] : 0.f;
    }
  }
  // after this wave's own slab(q) loads completed: its 16 bytes of staged rows k0 .. k1-1 -> U.
  // The next chunk's slab is transformed two rows per step over taps 4..8 of the current chunk
  // (its loads, issued at tap 0, have landed by tap 4), behind group 0's MFMA issue, so the LDS
  // round trips never sit in front of a barrier (all ten at tap 8 cost +10 % kernel time).
  auto bn_slab = [&](int q, int k0, int k1) {
    if constexpr (BNP) {
      bf16* dst = lds + (q & 1) * SLAB;
#pragma unroll
      for (int k = 0; k < AL; ++k) {
        if (k < k0 || k >= k1) continue;
        bf16x8* p = reinterpret_cast<bf16x8*>(dst + (wl + 4 * k) * 16 * kBK + lane * 8);
        bf16x8 v = *p;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (bf16)fmaxf(fmaf(pcx[k], (float)v[e], pcc[k]), 0.f);
        *p = v;
      }
    }
  };
  const bf16* bsrc[PPBL];  // (32-bit offsets instead: SL -0.5 %, profiles/conv_phase_experiments_r4.txt)
#pragma unroll
  for (int k = 0; k < PPBL; ++k) {
    const int r = (wl + 4 * k) * 16 + lrow;
    bsrc[k] = Wt + (long)(n0 + r) * CIN + ((lcol ^ swz4(r)) * 8);
  }
  auto stage_a = [&](int q, int k0 = 0, int k1 = 1 << 20) {  // chunk q, pieces k0 .. k1-1
    bf16* dst = lds + (q & 1) * SLAB;
#pragma unroll
    for (int k = 0; k < AL; ++k) {
      if (k < k0 || k >= k1) continue;
      const int r = (wl + 4 * k) * 16 + lrow;
      long g = base + r;
      g = g < total_rows ? g : total_rows - 1;
      glds16(X + g * CIN + ((lcol ^ swz4(r)) * 8) + q * kBK, dst + (wl + 4 * k) * 16 * kBK);
    }
  };
  // step s -> (chunk q, tap t); PR: steps TAPS.. are chunk 1's tap pairs (2p, 2p + 1)
  auto decode = [&](int s, int& q, int& t) {
    if (PR && s >= TAPS) {
      q = 1;
      t = 2 * (s - TAPS);
    } else {
      q = s / TAPS;
      t = s - q * TAPS;
    }
  };
  // PR: this lane's staged weight piece is virtual 16-byte chunk v = lcol ^ swz (the same for
  // every slice: the slice rows differ by multiples of 16); v >= 2 of a paired step comes from
  // the next tap's channels 32 + 8 (v - 2)
  const bool vhi = ((lcol ^ swz4(lrow)) >= 2);
  auto stage_b = [&](int s, int k0 = 0, int k1 = 1 << 20) {  // step s = chunk * 9 + tap
    int q, t;
    decode(s, q, t);
    bf16* dst = lds + 2 * SLAB + (s % NB) * BTile;
    long off = t * tap_stride + q * kBK;
    if (PR && q == 1 && vhi && t + 1 < TAPS) off += tap_stride - 16;
#pragma unroll
    for (int k = 0; k < PPBL; ++k)
      if (k >= k0 && k < k1) glds16(bsrc[k] + off, dst + (wl + 4 * k) * 16 * kBK);
  };

  const int frow = lane & 15;
  const int fq = lane >> 4;
  int prel[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    int m = m0 + wm * (16 * MT) + i * 16 + frow;
    m = m < M ? m : M - 1;
    prel[i] = (int)(prow(m) - base);
  }
  int boffs[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int row = wn * (16 * NT) + j * 16 + frow;
    boffs[j] = row * kBK + ((fq ^ swz4(row)) * 8);
  }

  f32x4 acc[NT][MT];
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int i = 0; i < MT; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int cchunks = CIN / kBK;
  const int nsteps = PR ? TAPS + (TAPS + 1) / 2 : TAPS * cchunks;  // PR: cchunks == 2
  bf16x8 xa[MT], wb[NT];
  bf16x8 xa2[K2 ? MT : 1], wb2[K2 ? NT : 1];  // K2: the second step's fragments
  auto read_into = [&](int s, bf16x8* xa, bf16x8* wb) {
    int q, t;
    decode(s, q, t);
    const bf16* slab = lds + (q & 1) * SLAB;
    const bf16* bt = lds + 2 * SLAB + (s % NB) * BTile;
    int tl = t, ch = fq;  // PR: k-quads 2/3 of a paired step read the next tap's chunks 0/1
    if (PR && q == 1 && fq >= 2 && t + 1 < TAPS) {
      tl = t + 1;
      ch = fq & 1;
    }
    const int ky = tl / KS, kx = tl - ky * KS;
    const int toff = ky * WI + kx;
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int r = prel[i] + toff;
      xa[i] = *reinterpret_cast<const bf16x8*>(slab + r * kBK + ((ch ^ swz4(r)) * 8));
    }
#pragma unroll
    for (int j = 0; j < NT; ++j) wb[j] = *reinterpret_cast<const bf16x8*>(bt + boffs[j]);
  };
  auto read_frags = [&](int s) {
    if constexpr (DIAG & 2) {
      asm volatile("" : "+v"(xa[0]), "+v"(wb[0]));
      return;
    }
    read_into(s, xa, wb);
    lds_reads_done();  // retire this burst before the wave's next barrier (WAR on the LDS)
  };
  // K2: the fragments of steps s (and s + 1 when has1), one retire for both bursts
  auto read_pair = [&](int s, bool has1) {
    read_into(s, xa, wb);
    if (has1) read_into(s + 1, xa2, wb2);
    lds_reads_done();
  };
  auto mfmas_pair = [&](bool has1) {
    if constexpr (!PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int i = 0; i < MT; ++i) acc[j][i] = mfma16(wb[j], xa[i], acc[j][i]);
    if (has1) {
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int i = 0; i < MT; ++i) acc[j][i] = mfma16(wb2[j], xa2[i], acc[j][i]);
    }
    if constexpr (!PRIO) __builtin_amdgcn_s_setprio(0);
  };
  auto mfmas = [&]() {
    if constexpr (!PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int i = 0; i < MT; ++i) acc[j][i] = mfma16(wb[j], xa[i], acc[j][i]);
    if constexpr (!PRIO) __builtin_amdgcn_s_setprio(0);
  };
  // MFMA segment with staging loads issued between its MFMA rows (ISSUE = 1)
  auto mfmas_staged = [&](int sb) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int j = 0; j < NT; ++j) {
#pragma unroll
      for (int i = 0; i < MT; ++i) acc[j][i] = mfma16(wb[j], xa[i], acc[j][i]);
      if (j < PPBL && sb >= 0) {
        int q, t;
        decode(sb, q, t);
        bf16* dst = lds + 2 * SLAB + (sb % NB) * BTile;
        glds16(bsrc[j] + t * tap_stride + q * kBK, dst + (wl + 4 * j) * 16 * kBK);
      }
    }
    __builtin_amdgcn_s_setprio(0);
  };

  long long t0 = 0, r0 = 0;
  if constexpr (DIAG & 4) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  if constexpr (DIAG & 2) {  // random-looking operands (zeros would let the clock rise)
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) xa[i][e] = (bf16)(((lane * 37 + i * 11 + e * 5) % 29) * 0.07f - 1.f);
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) wb[j][e] = (bf16)(((lane * 13 + j * 7 + e * 3) % 31) * 0.06f - 0.9f);
  }
  // DIAG & 8: per-wave cycle accounting of the loop's segments (s_memtime), lane 0 of waves 0 / 4
  long long acc_t[5] = {0, 0, 0, 0, 0};
  auto now = [&]() -> long long {
    if constexpr (DIAG & 8) return __builtin_amdgcn_s_memtime();
    return 0;
  };
  // Staging split between the groups, each in its own read phase: group 0 stages the slab (10 glds
  // per wave per chunk, at tap 0), group 1 the weight tiles (3 glds per wave per step, after its
  // fragment reads). Each group waits only for its own loads, before the barrier that precedes
  // the first read of that data (always group 0's, at the next X barrier).
  if constexpr (K2) {
    const int nsup = (nsteps + 1) / 2;
    if (grp == 0) {
      stage_a(0);
      wait_vm<0>();
      bn_slab(0, 0, AL);
#pragma unroll 1
      for (int u = 0; u < nsup; ++u) {
        const int s0 = 2 * u;
        const bool has1 = s0 + 1 < nsteps;
        __builtin_amdgcn_s_barrier();  // X_u
        asm volatile("" ::: "memory");
#pragma unroll
        for (int h = 0; h < 2; ++h) {  // slab(q+1) at tap 1: its buffer's last reader is tap 8
          int q, t;
          decode(s0 + h, q, t);
          if ((h == 0 || has1) && t == 1 && q + 1 < cchunks) stage_a(q + 1);
        }
        read_pair(s0, has1);
        __builtin_amdgcn_s_barrier();  // Y_u
        asm volatile("" ::: "memory");
        mfmas_pair(has1);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          if (h == 1 && !has1) break;
          int q, t;
          decode(s0 + h, q, t);
          if (q + 1 >= cchunks) continue;
          if constexpr (BNP) {
            // slab(q+1), issued at tap 1, transformed over taps 4..7: done before the super-step
            // holding tap 8 (which may also hold the next chunk's tap 0)
            if (t >= 4 && t <= 7) {
              if (t == 4) wait_vm<0>();
              bn_slab(q + 1, (t - 4) * AL / 4, (t - 3) * AL / 4);
              asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            }
          } else {
            if (t == 7) wait_vm<0>();
          }
        }
      }
    } else {
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
      constexpr int DA = NB - 2;  // steps staged ahead of the super-step being read
#pragma unroll
      for (int k = 0; k < DA; ++k)
        if (k < nsteps) stage_b(k, 0, PB1);
      {  // B(0), B(1) complete
        const int last = nsteps - 1 < DA - 1 ? nsteps - 1 : DA - 1;
        const int need = nsteps - 1 < 1 ? nsteps - 1 : 1;
        wait_vm_rt((last - need) * PB1);
      }
      bool had1 = false;
#pragma unroll 1
      for (int u = 0; u < nsup; ++u) {
        const int s0 = 2 * u;
        const bool has1 = s0 + 1 < nsteps;
        __builtin_amdgcn_s_barrier();  // X_u
        asm volatile("" ::: "memory");
        if (u > 0) mfmas_pair(had1);  // super-step u - 1, beside group 0's reads of u
        __builtin_amdgcn_s_barrier();  // Y_u
        asm volatile("" ::: "memory");
        read_pair(s0, has1);  // beside group 0's MFMAs of u
        had1 = has1;
        if (s0 + DA < nsteps) stage_b(s0 + DA, 0, PB1);
        if (s0 + DA + 1 < nsteps) stage_b(s0 + DA + 1, 0, PB1);
        // B(s0 + 2), B(s0 + 3) complete before X_{u+1}: younger are the steps up to s0 + DA + 1
        const int lastc = s0 + DA + 1 < nsteps - 1 ? s0 + DA + 1 : nsteps - 1;
        const int need = s0 + 3 < nsteps - 1 ? s0 + 3 : nsteps - 1;
        const int yb = lastc - need;
        wait_vm_rt(yb > 0 ? yb * PB1 : 0);
      }
      mfmas_pair(had1);
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
    }
  } else if constexpr (RS > 0) {
    constexpr int SLT = (AL + 1) / 2;  // RS = 2: slab piece pairs, loaded at taps 0 .. SLT-1
    static_assert(RS < 2 || SLT + 1 < TAPS, "slab pieces land before the chunk's last tap");
    if (grp == 0) {
      stage_a(0);
      wait_vm<0>();
      bn_slab(0, 0, AL);
      bf16x8 sreg[2];
      // pieces 2p, 2p+1 of chunk q's slab -> sreg
      auto slab_get = [&](int q, int p) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int k = 2 * p + e;
          if (k >= AL) continue;
          const int r = (wl + 4 * k) * 16 + lrow;
          long g = base + r;
          g = g < total_rows ? g : total_rows - 1;
          sreg[e] = *reinterpret_cast<const bf16x8*>(X + g * CIN + ((lcol ^ swz4(r)) * 8) +
                                                      q * kBK);
        }
      };
      // sreg -> the slab buffer of chunk q (BNP: U = ReLU(cx x + cc) of the piece's row). The
      // piece index is a template constant (a switch on the pair), so pcx / pcc stay registers
      // (a runtime-indexed form was rewritten by the compiler into scratch accesses).
      auto put_piece = [&](bf16* dst, auto kc) {
        constexpr int k = decltype(kc)::value;
        if constexpr (k < AL) {
          bf16x8 v = sreg[k & 1];
          if constexpr (BNP) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = (bf16)fmaxf(fmaf(pcx[k], (float)v[e], pcc[k]), 0.f);
          }
          *reinterpret_cast<bf16x8*>(dst + (wl + 4 * k) * 16 * kBK + lane * 8) = v;
        }
      };
      auto slab_put = [&](int q, int p) {
        bf16* dst = lds + (q & 1) * SLAB;
        static_assert(AL <= 12, "slab_put covers six piece pairs");
        switch (p) {
          case 0: put_piece(dst, IntC<0>{}); put_piece(dst, IntC<1>{}); break;
          case 1: put_piece(dst, IntC<2>{}); put_piece(dst, IntC<3>{}); break;
          case 2: put_piece(dst, IntC<4>{}); put_piece(dst, IntC<5>{}); break;
          case 3: put_piece(dst, IntC<6>{}); put_piece(dst, IntC<7>{}); break;
          case 4: put_piece(dst, IntC<8>{}); put_piece(dst, IntC<9>{}); break;
          default: put_piece(dst, IntC<10>{}); put_piece(dst, IntC<11>{}); break;
        }
      };
#pragma unroll 1
      for (int s = 0; s < nsteps; ++s) {
        int q, t;
        decode(s, q, t);
        const bool more = q + 1 < cchunks;
        const long long c1 = now();
        __builtin_amdgcn_s_barrier();  // X_s
        asm volatile("" ::: "memory");
        const long long c2 = now();
        if constexpr (RS == 1) {  // slab by LDS-DMA, as the default loop
          if constexpr (SPREAD && !BNP) {
            if (t < TAPS - 1 && more) stage_a(q + 1, t * AL / (TAPS - 1), (t + 1) * AL / (TAPS - 1));
          } else {
            if (t == 0 && more) stage_a(q + 1);
          }
        }
        read_frags(s);
        const long long c3 = now();
        __builtin_amdgcn_s_barrier();  // Y_s
        asm volatile("" ::: "memory");
        const long long c4 = now();
        mfmas();
        const long long c5 = now();
        if constexpr (RS == 1) {
          if constexpr (BNP) {
            if (t >= 4 && more) {
              if (t == 4) wait_vm<0>();
              bn_slab(q + 1, 2 * (t - 4), 2 * (t - 4) + 2);
            }
          } else {
            if (t == TAPS - 1 && more) wait_vm<0>();
          }
        } else if (more) {
          // behind the MFMA issue: last tap's pieces -> LDS, this tap's pieces -> registers
          if (t >= 1 && t <= SLT) slab_put(q + 1, t - 1);
          if (t < SLT) slab_get(q + 1, t);
        }
        const long long c6 = now();
        if constexpr (DIAG & 8) {
          acc_t[0] += c2 - c1;
          acc_t[1] += c3 - c2;
          acc_t[2] += c4 - c3;
          acc_t[3] += c5 - c4;
          acc_t[4] += c6 - c5;
        }
      }
    } else {
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
      bf16x8 wreg[PB1];
      auto w_get = [&](int s) {
        int q, t;
        decode(s, q, t);
        const long off = t * tap_stride + q * kBK;
#pragma unroll
        for (int k = 0; k < PB1; ++k) wreg[k] = *reinterpret_cast<const bf16x8*>(bsrc[k] + off);
      };
      auto w_put = [&](int s) {
        bf16* dst = lds + 2 * SLAB + (s % NB) * BTile;
#pragma unroll
        for (int k = 0; k < PB1; ++k)
          *reinterpret_cast<bf16x8*>(dst + (wl + 4 * k) * 16 * kBK + lane * 8) = wreg[k];
      };
      w_get(0);
      w_put(0);
      if (nsteps > 1) w_get(1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // B(0) in the ring before X_0
#pragma unroll 1
      for (int s = 0; s < nsteps; ++s) {
        const long long c0 = now();
        __builtin_amdgcn_s_barrier();  // X_s
        asm volatile("" ::: "memory");
        const long long c1 = now();
        if (s > 0) mfmas();  // step s - 1, beside group 0's reads of step s
        const long long c2 = now();
        __builtin_amdgcn_s_barrier();  // Y_s
        asm volatile("" ::: "memory");
        const long long c3 = now();
        read_into(s, xa, wb);  // beside group 0's MFMAs of step s
        const long long c4 = now();
        // B(s+1) (loaded a step ago) -> its ring slot (last read at step s+1-NB); B(s+2) -> regs;
        // the fragment-read retire below also retires the ds_write before X_{s+1}
        if (s + 1 < nsteps) w_put(s + 1);
        if (s + 2 < nsteps) w_get(s + 2);
        lds_reads_done();
        const long long c5 = now();
        if constexpr (DIAG & 8) {
          acc_t[0] += c1 - c0;
          acc_t[1] += c2 - c1;
          acc_t[2] += c3 - c2;
          acc_t[3] += c4 - c3;
          acc_t[4] += c5 - c4;
        }
      }
      mfmas();
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
    }
  } else if (grp == 0) {
    stage_a(0);
    if constexpr (WG0 > 0) {
#pragma unroll
      for (int k = 0; k < D; ++k)
        if (k < nsteps) stage_b(k, PB1, PPBL);
    }
    wait_vm<0>();
    bn_slab(0, 0, AL);
#pragma unroll 1
    for (int s = 0; s < nsteps; ++s) {
      int q, t;
      decode(s, q, t);
      const bool more = q + 1 < cchunks;
      const long long c1 = now();
      __builtin_amdgcn_s_barrier();  // X_s
      asm volatile("" ::: "memory");
      const long long c2 = now();
      int slab_now = 0;  // slab pieces this wave issues in this step (younger than B(s+1)'s)
      if constexpr (!(DIAG & 1)) {
        if constexpr (SPREAD == 1 && !BNP) {
          // pieces [t*AL/(TAPS-1), (t+1)*AL/(TAPS-1)) at taps 0 .. TAPS-2; all retired by the
          // wait after the last tap's MFMAs, as before
          if (t < TAPS - 1 && more) {
            const int k0 = t * AL / (TAPS - 1), k1 = (t + 1) * AL / (TAPS - 1);
            stage_a(q + 1, k0, k1);
            slab_now = k1 - k0;
          }
        } else if constexpr (SPREAD == 0 || BNP) {
          if (t == 0 && more) {
            stage_a(q + 1);
            slab_now = AL;
          }
        }
      }
      if constexpr (SPREAD == 3 && !BNP && !(DIAG & 3)) {
        // SPREAD = 3: the same pieces issued between this step's fragment reads and their retire
        // (the LDS-DMA issue overlaps the reads' latency instead of delaying them)
        read_into(s, xa, wb);
        if (t < TAPS - 1 && more) stage_a(q + 1, t * AL / (TAPS - 1), (t + 1) * AL / (TAPS - 1));
        lds_reads_done();
      } else {
        read_frags(s);
      }
      const long long c3 = now();
      __builtin_amdgcn_s_barrier();  // Y_s
      asm volatile("" ::: "memory");
      const long long c4 = now();
      mfmas();
      const long long c5 = now();
      if constexpr (SPREAD == 2 && !BNP && !(DIAG & 1)) {
        // SPREAD = 2: the same pieces issued behind this step's MFMA issue instead of in front of
        // its fragment reads (as the wgrad slab kernel's stage placement, RAG_WGRAD_LATE)
        if (t < TAPS - 1 && more) stage_a(q + 1, t * AL / (TAPS - 1), (t + 1) * AL / (TAPS - 1));
      }
      if constexpr (BNP) {
        // slab(q+1) complete at tap 4, transformed over taps 4..8 (this wave's reads of step s+1
        // drain the writes before the next chunk's X barrier)
        if (t >= 4 && more) {
          if (t == 4) wait_vm<0>();
          bn_slab(q + 1, 2 * (t - 4), 2 * (t - 4) + 2);
        }
      } else {
        if constexpr (WG0 > 0 && !(DIAG & 1)) {
          // this group's slices of B(s+D), then B(s+1)'s (issued a step ago) complete before
          // X_{s+1}: younger are this step's slab pieces and the slices just issued
          int young = slab_now;
          if (s + D < nsteps) {
            stage_b(s + D, PB1, PPBL);
            young += WG0;
          }
          if (s + 1 < nsteps) wait_vm_rt(young);
        }
        if (t == TAPS - 1 && more) wait_vm<0>();  // slab(q+1) complete before the next chunk
      }
      const long long c6 = now();
      if constexpr (DIAG & 8) {  // X wait, stage+read, Y wait, MFMA issue, vm wait
        acc_t[0] += c2 - c1;
        acc_t[1] += c3 - c2;
        acc_t[2] += c4 - c3;
        acc_t[3] += c5 - c4;
        acc_t[4] += c6 - c5;
      }
    }
  } else {
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);  // static: the younger half
#pragma unroll
    for (int k = 0; k < D; ++k)
      if (k < nsteps) stage_b(k, 0, PB1);
    wait_vm_rt((nsteps - 1 < D - 1 ? nsteps - 1 : D - 1) * PB1);  // B(0) complete
#pragma unroll 1
    for (int s = 0; s < nsteps; ++s) {
      const long long c0 = now();
      __builtin_amdgcn_s_barrier();  // X_s
      asm volatile("" ::: "memory");
      const long long c1 = now();
      if constexpr (ISSUE == 1 && !(DIAG & 1)) {
        // step s - 1's MFMAs carry the loads of B(s - 1 + D)
        if (s > 0) mfmas_staged(s - 1 + D < nsteps ? s - 1 + D : -1);
      } else if constexpr (ISSUE == 2 && !(DIAG & 1)) {
        // ISSUE = 2: B(s - 1 + D) issued right behind step s - 1's MFMA issue (the placement that
        // paid in the wgrad slab kernel), not after this group's fragment reads
        if (s > 0) {
          mfmas();
          if (s - 1 + D < nsteps) stage_b(s - 1 + D, 0, PB1);
        }
      } else {
        if (s > 0) mfmas();          // step s - 1, beside group 0's reads of step s
      }
      const long long c2 = now();
      __builtin_amdgcn_s_barrier();  // Y_s
      asm volatile("" ::: "memory");
      const long long c3 = now();
      if constexpr (ISSUE == 3 && !(DIAG & 3)) {
        // ISSUE = 3: B(s+D) issued between this group's fragment reads and their retire
        read_into(s, xa, wb);
        if (s + D < nsteps) stage_b(s + D, 0, PB1);
        lds_reads_done();
      } else {
        read_frags(s);               // beside group 0's MFMAs of step s
      }
      const long long c4 = now();
      if constexpr (!(DIAG & 1)) {
        if constexpr (ISSUE == 1 || ISSUE == 2) {
          // B(s+1) complete before X_{s+1}: issued so far are B(.. min(s-1+D, nsteps-1))
          int last = s - 1 + D < nsteps - 1 ? s - 1 + D : nsteps - 1;
          const int yb = last - (s + 1);
          wait_vm_rt(yb > 0 ? yb * PPBL : 0);
        } else {
          if constexpr (ISSUE != 3) {
            if (s + D < nsteps) stage_b(s + D, 0, PB1);
          }
          // B(s+1) complete before X_{s+1}: younger are B(s+2 .. min(s+D, nsteps-1))
          int yb = nsteps - 2 - s;
          yb = yb < D - 1 ? yb : D - 1;
          wait_vm_rt(yb > 0 ? yb * PB1 : 0);
        }
      }
      const long long c5 = now();
      if constexpr (DIAG & 8) {  // X wait, MFMA issue, Y wait, read, stage + vm wait
        acc_t[0] += c1 - c0;
        acc_t[1] += c2 - c1;
        acc_t[2] += c3 - c2;
        acc_t[3] += c4 - c3;
        acc_t[4] += c5 - c4;
      }
    }
    mfmas();
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
  }
  if constexpr (DIAG & 8) {
    if (lane == 0 && (w == 0 || w == 4) && stamps) {
      long long* o = stamps + 6 * 4096 + (size_t)blockIdx.x * 10 + (w == 4 ? 5 : 0);
#pragma unroll
      for (int k = 0; k < 5; ++k) o[k] = acc_t[k];
    }
  }
  long long t1 = 0, r1 = 0;
  if constexpr (DIAG & 4) {
    t1 = __builtin_amdgcn_s_memtime();
    r1 = __builtin_amdgcn_s_memrealtime();
  }
  if (res) {
    epilogue(acc, m0 + wm * (16 * MT), n0 + wn * (16 * NT), M, S, WO, HO, YC, HM, bias, res,
             relu, mask, Y, frow, fq, sred);
  } else {
    __syncthreads();  // every wave is past its last LDS read: the ring becomes the output image
    // (the 128-wide kernels keep the per-chunk loads: CNNPolicy-128 162.0 vs 165.9k with them)
    epilogue_lds<BM, NT, MT, NT == kNT ? RAG_EP_PREFETCH : 0>(acc, lds, wm * (16 * MT), wn * (16 * NT), m0, n0,
                                              M, S, WO, HO, YC, HM, bias, relu, mask, Y, frow,
                                              fq, mcoef, sred, smean);
  }
  if (spart) {  // the block's column partials
    __syncthreads();
    if ((int)threadIdx.x < 2 * S) {
      const int q = threadIdx.x / S, wc = threadIdx.x - q * S;
      spart[((size_t)blockIdx.x * 2 + q) * S + wc] = sred[q * 64 + wc];
    }
  }
  // a deferred wgrad reduction riding in this launch: the tile done, help finish it
  if constexpr (kClaim) {
    if (red.ticket && gridDim.x > nconv) wslab_reduce_dynamic<kRedU>(red, reinterpret_cast<int*>(lds));
  }
  if constexpr (DIAG & 4) {
    // per block: loop cycles, loop ticks, then absolute ticks at entry / loop start / loop end /
    // exit (wave 0; 100 MHz)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const long long r2 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && stamps) {
      long long* o = stamps + 6 * blockIdx.x;
      o[0] = t1 - t0;
      o[1] = r1 - r0;
      o[2] = r_entry;
      o[3] = r0;
      o[4] = r1;
      o[5] = r2;
    }
  }
}

int g_tap_mode = -1;  // -1: read RAG_CONV_TAP on first use (default on)
int g_conv_k2 = -1;   // -1: read RAG_CONV_K2 on first use (128-channel 3x3 ping-pong variant)
int g_conv_rs = -1;   // -1: read RAG_CONV_RS on first use (register staging, 3x3 ping-pong)
int conv_rs() {
  if (g_conv_rs < 0) {
    const char* e = getenv("RAG_CONV_RS");
    g_conv_rs = e ? atoi(e) : 0;
  }
  return g_conv_rs;
}
int g_ep_lds_override = -1;  // rag_conv_ep_lds(): A/B switch of conv_tap_kernel's epilogue

// Worst-case slab extent of a bm-pixel run (host check of the kernels' slab-row assumptions).
int max_slab_rows(int S, int WI, int shift, int bm, int KS = 3) {
  const int S2 = S * S;
  auto prow = [&](long m) {
    const long b = m / S2, rem = m - b * S2, i = rem / S, j = rem - i * S;
    return (b * WI + i + shift) * WI + j + shift;
  };
  long mx = 0;
  for (long m0 = 0; m0 < (long)S2 * bm + bm; m0 += bm)
    mx = std::max(mx, prow(m0 + bm - 1) + (KS - 1) * (WI + 1) - prow(m0) + 1);
  return (int)mx;
}

long long* g_stamps = nullptr;
}  // namespace

// Diagnostic launches of the ping-pong kernel (results are WRONG for diag 1-3): diag bit 0 = no
// staging, bit 1 = no fragment reads; every diag launch records per-block (cycles, 100 MHz ticks)
// of the main loop, read back with rag_conv_diag_stamps; bit 4 = the 128-channel kernel. 3x3
// forward/dgrad shapes only.
RAG_API int rag_conv_pp_diag(int diag, const void* X, const void* W, const float* bias, void* Y,
                             const void* mask, int B, int S, int HI, int HO, int CIN, int COUTP,
                             int YC, int relu, int HM, hipStream_t stream) {
  if (!g_stamps && hipMalloc(&g_stamps, 16 * 4096 * sizeof(long long)) != hipSuccess) return -3;
  const int M = B * S * S, WI = S + 2 * HI, WO = S + 2 * HO, shift = HI - 1;
  const bool n128 = diag & 16;  // the 128-channel kernel (NT = 4, 3-deep ring)
  const int rsd = (diag >> 5) & 3;  // bits 5-6: register staging (timing builds 4 / 12 only)
  const int BNW = n128 ? 128 : kBN;
  const int nconv = ((M + kPPBM - 1) / kPPBM) * (COUTP / BNW);
  if (nconv > 4096 || COUTP % BNW || CIN % kBK) return -1;
  const long total = (long)B * WI * WI;
  const bf16 *x = (const bf16*)X, *w = (const bf16*)W, *mk = (const bf16*)mask;
  bf16* y = (bf16*)Y;
  WgradRed r{};
#define RAG_PPD(D)                                                                               \
  if (n128)                                                                                      \
    conv_tap_pp_kernel<3, D, 0, 4><<<nconv, 512, 0, stream>>>(                                   \
        x, w, bias, y, mk, nullptr, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM, total,    \
        nconv, r, nullptr, nullptr, nullptr, nullptr, g_stamps);                                 \
  else                                                                                           \
    conv_tap_pp_kernel<4, D><<<nconv, 512, 0, stream>>>(x, w, bias, y, mk, nullptr, M, S, WI,    \
                                                        shift, WO, HO, CIN, COUTP, YC, relu, HM, \
                                                        total, nconv, r, nullptr, nullptr,       \
                                                        nullptr, nullptr, g_stamps)
#define RAG_PPDR(D, RSV)                                                                          \
  if (n128)                                                                                      \
    conv_tap_pp_kernel<3, D, 0, 4, false, 3, kMT, 0, 0, 0, 0, 0, RSV><<<nconv, 512, 0, stream>>>( \
        x, w, bias, y, mk, nullptr, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM, total,    \
        nconv, r, nullptr, nullptr, nullptr, nullptr, g_stamps);                                 \
  else                                                                                           \
    conv_tap_pp_kernel<3, D, 0, kNT, false, 3, kMT, 0, 0, 1, 0, 0, RSV>                          \
        <<<nconv, 512, 0, stream>>>(x, w, bias, y, mk, nullptr, M, S, WI, shift, WO, HO, CIN,    \
                                    COUTP, YC, relu, HM, total, nconv, r, nullptr, nullptr,      \
                                    nullptr, nullptr, g_stamps)
  if (rsd) {
    if ((diag & 3) != 0) return -1;
    if (rsd == 1) {
      if (diag & 8) { RAG_PPDR(12, 1); } else { RAG_PPDR(4, 1); }
    } else {
      if (diag & 8) { RAG_PPDR(12, 2); } else { RAG_PPDR(4, 2); }
    }
    return (int)hipGetLastError();
  }
#undef RAG_PPDR
  switch (diag & 11) {
    case 0: RAG_PPD(4); break;
    case 1: RAG_PPD(5); break;
    case 2: RAG_PPD(6); break;
    case 3: RAG_PPD(7); break;
    default: RAG_PPD(12); break;  // 8: segment accounting of the full kernel
  }
#undef RAG_PPD
  return (int)hipGetLastError();
}

RAG_API int rag_conv_diag_stamps(long long* host, int nblocks) {
  if (!g_stamps) return -1;
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  return (int)hipMemcpy(host, g_stamps, 6 * nblocks * sizeof(long long), hipMemcpyDeviceToHost);
}

RAG_API int rag_conv_diag_segments(long long* host, int nblocks) {
  if (!g_stamps) return -1;
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  return (int)hipMemcpy(host, g_stamps + 6 * 4096, 10 * nblocks * sizeof(long long),
                        hipMemcpyDeviceToHost);
}

RAG_API int rag_conv_ep_lds(int on) {
  const int old = g_ep_lds_override;
  g_ep_lds_override = on;
  return old;
}

RAG_API int rag_conv_rs(int v) {
  const int old = g_conv_rs;
  g_conv_rs = v;
  return old;
}

RAG_API int rag_conv_k2(int v) {
  const int old = g_conv_k2;
  g_conv_k2 = v;
  return old;
}

RAG_API int rag_conv_tap_mode(int mode) {
  const int old = g_tap_mode;
  g_tap_mode = mode;
  return old;
}

// Returns true if the tap-slab kernel handled the launch: 3x3, 192-multiple output channels,
// input channels a multiple of 32, and every 192-pixel run's nine-tap slab fits kSlabRows.
// Returns true if a tap-slab kernel handled the launch: 3x3, 192-multiple output channels,
// input channels a multiple of 32, and every pixel run's nine-tap slab fits the kernel's slab.
// Mode (RAG_CONV_TAP / rag_conv_tap_mode): 0 off, 1 = 4-wave 192-pixel kernel (round-2 default),
// 2 / 3 = 8-wave 384-pixel kernel with a 4- / 5-deep weight ring (measured slower: docs/KERNELS.md),
// 4 = 8-wave 192-pixel kernel, four waves per SIMD (conv_tap16_kernel), 5 / 6 / 7 = ping-pong
// 8-wave 384-pixel kernel with a 4- / 3- / 5-deep weight ring (conv_tap_pp_kernel; 6 = round 3),
// 8 / 9 = the same with the weight loads issued inside the MFMA segment (measured slower),
// 10 = mode 6 with the next chunk's slab loads spread over the taps, 11 = 10 + one weight slice
// staged by the loader group, 12 = 10 + static priority for the second wave group (default),
// 13 = 11 + 12, 14 = 6 + static priority, 15 = 12 with a 4-deep ring (3x3 192-channel layers;
// the other shapes run the mode-6 kernels).
int rag_launch_wgrad_slab_reduce(const WgradRed& r, hipStream_t stream);  // wgrad_slab.hip

// bnc / mcoef (BN prologue / mask coefficients, conv_tap_pp_kernel BNP): only the 128-channel
// ping-pong path takes them; with either set, any other shape returns false.
bool rag_conv_tap_bn_ok(int M, int S, int WI, int shift, int CIN, int COUTP, int KS);

bool rag_conv_tap_launch(const bf16* x, const bf16* w, const float* bias, bf16* y,
                         const bf16* mk, const bf16* res, int M, int S, int WI, int shift, int WO,
                         int HO, int CIN, int COUTP, int YC, int KS, int relu, int HM, long total_rows,
                         hipStream_t stream, const WgradRed* red, const float* bnc,
                         const float* mcoef, float* spart, const float* smean) {
  if ((bnc || mcoef || spart) &&
      ((mcoef && res) || !rag_conv_tap_bn_ok(M, S, WI, shift, CIN, COUTP, KS)))
    return false;
  if (g_tap_mode < 0) {
    const char* e = getenv("RAG_CONV_TAP");
    // ping-pong, 3-deep ring, slab loads spread over the chunk's taps, static priority for the
    // second wave group (mode 12): SL 111.7-111.9k -> 113.6-113.9k positions/s on one box
    // (profiles/conv_variants_r4b.txt)
    g_tap_mode = e ? atoi(e) : 12;
  }
  // 192-multiple widths: 96 x 96 wave tiles (NT = 6); 128-multiple widths (ResnetPolicy's and
  // the reference CNNPolicy's default 128 filters) only on the ping-pong kernel, 96 x 64 (NT = 4)
  const bool w192 = COUTP % kBN == 0, w128 = !w192 && COUTP % 128 == 0;
  if (!g_tap_mode || !(KS == 3 || KS == 5) || !(w192 || w128) || CIN % kBK || CIN < kBK)
    return false;
  if (KS == 5) {
    // 5x5 (the SL input layer, ResnetPolicy's first unit): the ping-pong kernel over 25 taps,
    // when the grid fills the chip and every 384-pixel run's 25-tap slab fits 640 rows
    static int key5 = -1, rows5 = 0;
    const int k5 = S * 4096 + WI * 8 + shift;
    if (k5 != key5) {
      rows5 = max_slab_rows(S, WI, shift, kPPBM, KS);
      key5 = k5;
    }
    const char* e = getenv("RAG_PP_MIN_BLOCKS");
    const int pmin = e ? atoi(e) : 200;
    const int nconv = ((M + kPPBM - 1) / kPPBM) * (COUTP / (w192 ? kBN : 128));
    static const bool pp5 = [] {  // RAG_CONV_PP5=0: the 5x5 layers stay on conv_pipe
      const char* v = getenv("RAG_CONV_PP5");
      return !(v && v[0] == '0');
    }();
    if (!pp5 || bnc || mcoef || spart || g_tap_mode < 5 || g_tap_mode > 20) return false;
    // <= 48 real input channels in a 64-channel layout (the caller's hint, rag_conv_igemm_cin):
    // chunk 1 steps pair two taps (PAIR; RAG_CONV_PAIR5=0 disables)
    static const bool pair_on = [] {
      const char* v = getenv("RAG_CONV_PAIR5");
      return !(v && v[0] == '0');
    }();
    const bool pair5 = pair_on && CIN == 64 && g_conv_cin_real > 0 && g_conv_cin_real <= 48;
    if (nconv < pmin) {
      // sub-chip grids (128-game self-play passes): 192-pixel blocks, as the 3x3 layers
      static int key5b = -1, rows5b = 0;
      if (k5 != key5b) {
        rows5b = max_slab_rows(S, WI, shift, kBM, KS);
        key5b = k5;
      }
      const int n192 = ((M + kBM - 1) / kBM) * (COUTP / kBN);
      if (!w192 || n192 < pmin || rows5b > kPPSlabRows192x5) return false;
      int nred = 0;
      WgradRed r{};
      if (red) {
        r = *red;
        r.ticket = nullptr;  // claimed reduction: 128-wide launches only (SL -1.3 %)
        nred = std::max(8, (256 - n192 % 256) % 256);
      }
      if (pair5)
        conv_tap_pp_kernel<3, 0, 0, 6, false, 5, 3, 0, 0, 0, 1><<<n192 + nred, 512, 0, stream>>>(
            x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM,
            total_rows, n192, r);
      else
        conv_tap_pp_kernel<3, 0, 0, 6, false, 5, 3><<<n192 + nred, 512, 0, stream>>>(
            x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM,
            total_rows, n192, r);
      return true;
    }
    if (rows5 > kPPSlabRows5) return false;
    int nred = 0;
    WgradRed r{};
    if (red) {
      r = *red;
      if (w192) r.ticket = nullptr;  // claimed reduction: 128-wide launches only
      nred = std::max(8, (256 - nconv % 256) % 256);
    }
    // (the spread / static-priority 3x3 variants measured slower on the 5x5 layer: 52.9-53.7
    // vs 49.9 us, profiles/conv_variants_r4b.txt; every mode runs the plain ping-pong here)
    // RAG_CONV5_VAR (A/B of the paired 192-filter input layer): 1 static priority, 2 spread
    // slab + static priority, 3 a 4-deep weight ring
    static const int v5 = [] {
      const char* e = getenv("RAG_CONV5_VAR");
      return e ? atoi(e) : 0;
    }();
#define RAG_PP5(NBV, SPV, PRV)                                                                   \
  conv_tap_pp_kernel<NBV, 0, 0, 6, false, 5, kMT, SPV, 0, PRV, 1><<<nconv + nred, 512, 0, stream>>>( \
      x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM, total_rows, nconv, r)
    if (w192 && pair5) {
      if (v5 == 1) RAG_PP5(3, 0, 1);
      else if (v5 == 2) RAG_PP5(3, 1, 1);
      else if (v5 == 3) RAG_PP5(4, 0, 0);
      else RAG_PP5(3, 0, 0);
    }
#undef RAG_PP5
    else if (w192)
      conv_tap_pp_kernel<3, 0, 0, 6, false, 5><<<nconv + nred, 512, 0, stream>>>(
          x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM, total_rows,
          nconv, r);
    else if (pair5)  // 128 filters (ResnetPolicy's input layer)
      conv_tap_pp_kernel<3, 0, 0, 4, false, 5, kMT, 0, 0, 0, 1><<<nconv + nred, 512, 0,
                                                                   stream>>>(
          x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM, total_rows,
          nconv, r);
    else
      conv_tap_pp_kernel<3, 0, 0, 4, false, 5><<<nconv + nred, 512, 0, stream>>>(
          x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM, total_rows,
          nconv, r);
    return true;
  }
  static int cached_key = -1, cached_rows = 0, cached_rows8 = 0;
  const int key = S * 4096 + WI * 8 + shift;
  if (key != cached_key) {
    cached_rows = max_slab_rows(S, WI, shift, kBM);
    cached_rows8 = max_slab_rows(S, WI, shift, k8BM);
    cached_key = key;
  }
  if ((g_tap_mode == 2 || g_tap_mode == 3) && w192 && cached_rows8 <= k8SlabRows) {
    if (red) rag_launch_wgrad_slab_reduce(*red, stream);
    const int nblk_m = (M + k8BM - 1) / k8BM;
    dim3 grid(nblk_m * (COUTP / kBN));
    if (g_tap_mode == 3)
      conv_tap8_kernel<5><<<grid, 512, 0, stream>>>(x, w, bias, y, mk, res, M, S, WI, shift, WO,
                                                    HO, CIN, COUTP, YC, relu, HM, total_rows);
    else
      conv_tap8_kernel<4><<<grid, 512, 0, stream>>>(x, w, bias, y, mk, res, M, S, WI, shift, WO,
                                                    HO, CIN, COUTP, YC, relu, HM, total_rows);
    return true;
  }
  // Small batches (self-play plies, short search waves): fewer 384-pixel blocks than CUs leave
  // most of the chip idle, so the 192-pixel kernel (twice the blocks) runs them instead.
  static const int pp_min = [] {
    const char* e = getenv("RAG_PP_MIN_BLOCKS");
    return e ? atoi(e) : 200;  // B = 256 at 19x19 is 241 blocks: stays on the ping-pong kernel
  }();
  if (w128) {
    const int nconv = ((M + kPPBM - 1) / kPPBM) * (COUTP / 128);
    if (g_tap_mode < 5 || g_tap_mode > 20 || cached_rows8 > kPPSlabRows || nconv < pp_min)
      return false;  // small batches: conv_pipe
    int nred = 0;
    WgradRed r{};
    if (red) {
      r = *red;
      // claimed reduction (r.ticket): CNNPolicy-128 164.9 -> 169.2 k positions/s
      nred = std::max(8, (256 - nconv % 256) % 256);
    }
    if (g_conv_k2 < 0) {
      const char* e = getenv("RAG_CONV_K2");
      g_conv_k2 = e ? atoi(e) : 0;
    }
    // K2 (two K-steps per barrier pair, rag_conv_k2): 1 = plain, 2 = + static group-1 priority;
    // RS (register staging, rag_conv_rs): 1 = weights, 2 = weights + slab
#define RAG_PP128(BNPV, PRIOV, K2V, RSV, BNC)                                                     \
  conv_tap_pp_kernel<K2V ? 6 : 3, 0, 0, 4, BNPV, 3, kMT, 0, 0, PRIOV, 0, K2V, RSV>                \
      <<<nconv + nred, 512, 0, stream>>>(x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN,   \
                                         COUTP, YC, relu, HM, total_rows, nconv, r, BNC, mcoef,  \
                                         spart, smean)
    const int rs = conv_rs();
    if (bnc) {
      if (rs == 1) RAG_PP128(true, 0, 0, 1, bnc);
      else if (rs == 2) RAG_PP128(true, 0, 0, 2, bnc);
      else if (g_conv_k2 == 1) RAG_PP128(true, 0, 1, 0, bnc);
      else if (g_conv_k2 == 2) RAG_PP128(true, 1, 1, 0, bnc);
      else RAG_PP128(true, 0, 0, 0, bnc);
    } else {
      if (rs == 1) RAG_PP128(false, 0, 0, 1, nullptr);
      else if (rs == 2) RAG_PP128(false, 0, 0, 2, nullptr);
      else if (g_conv_k2 == 1) RAG_PP128(false, 0, 1, 0, nullptr);
      else if (g_conv_k2 == 2) RAG_PP128(false, 1, 1, 0, nullptr);
      else RAG_PP128(false, 0, 0, 0, nullptr);
    }
#undef RAG_PP128
    return true;
  }
  const bool pp_fills = ((M + kPPBM - 1) / kPPBM) * (COUTP / kBN) >= pp_min;
  static const bool pp192_all = [] {  // RAG_CONV_PP192=2: 192-pixel blocks everywhere (A/B)
    const char* v = getenv("RAG_CONV_PP192");
    return v && v[0] == '2';
  }();
  if ((g_tap_mode >= 5 && g_tap_mode <= 20) && cached_rows8 <= kPPSlabRows && pp_fills &&
      !pp192_all) {
    // ping-pong kernel: one block per CU; reduce blocks fill the CUs its last round leaves free
    const int nconv = ((M + kPPBM - 1) / kPPBM) * (COUTP / kBN);
    int nred = 0;
    WgradRed r{};
    if (red) {
      r = *red;
      r.ticket = nullptr;  // claimed reduction: 128-wide launches only (SL -1.3 %)
      nred = std::max(8, (256 - nconv % 256) % 256);
    }
    if (g_tap_mode == 5)
      conv_tap_pp_kernel<4><<<nconv + nred, 512, 0, stream>>>(
          x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM, total_rows,
          nconv, r);
    else if (g_tap_mode == 7)
      conv_tap_pp_kernel<5><<<nconv + nred, 512, 0, stream>>>(
          x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM, total_rows,
          nconv, r);
    else if (g_tap_mode == 8)
      conv_tap_pp_kernel<3, 0, 1><<<nconv + nred, 512, 0, stream>>>(
          x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM, total_rows,
          nconv, r);
    else if (g_tap_mode == 9)
      conv_tap_pp_kernel<4, 0, 1><<<nconv + nred, 512, 0, stream>>>(
          x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM, total_rows,
          nconv, r);
    else if (g_tap_mode == 10)
      conv_tap_pp_kernel<3, 0, 0, kNT, false, 3, kMT, 1><<<nconv + nred, 512, 0, stream>>>(
          x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM, total_rows,
          nconv, r);
    else if (g_tap_mode == 11)
      conv_tap_pp_kernel<3, 0, 0, kNT, false, 3, kMT, 1, 1><<<nconv + nred, 512, 0, stream>>>(
          x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM, total_rows,
          nconv, r);
    else if (g_tap_mode == 12 && conv_rs() == 1)
      conv_tap_pp_kernel<3, 0, 0, kNT, false, 3, kMT, 1, 0, 1, 0, 0, 1>
          <<<nconv + nred, 512, 0, stream>>>(x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN,
                                             COUTP, YC, relu, HM, total_rows, nconv, r);
    else if (g_tap_mode == 12 && conv_rs() == 2)
      conv_tap_pp_kernel<3, 0, 0, kNT, false, 3, kMT, 0, 0, 1, 0, 0, 2>
          <<<nconv + nred, 512, 0, stream>>>(x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN,
                                             COUTP, YC, relu, HM, total_rows, nconv, r);
    else if (g_tap_mode == 18)
      conv_tap_pp_kernel<3, 0, 0, kNT, false, 3, kMT, 3, 0, 1><<<nconv + nred, 512, 0, stream>>>(
          x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM, total_rows,
          nconv, r);
    else if (g_tap_mode == 19)
      conv_tap_pp_kernel<3, 0, 3, kNT, false, 3, kMT, 1, 0, 1><<<nconv + nred, 512, 0, stream>>>(
          x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM, total_rows,
          nconv, r);
    else if (g_tap_mode == 20)
      conv_tap_pp_kernel<3, 0, 3, kNT, false, 3, kMT, 3, 0, 1><<<nconv + nred, 512, 0, stream>>>(
          x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM, total_rows,
          nconv, r);
    else if (g_tap_mode == 17)
      conv_tap_pp_kernel<3, 0, 2, kNT, false, 3, kMT, 1, 0, 1><<<nconv + nred, 512, 0, stream>>>(
          x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM, total_rows,
          nconv, r);
    else if (g_tap_mode == 16)
      conv_tap_pp_kernel<3, 0, 0, kNT, false, 3, kMT, 2, 0, 1><<<nconv + nred, 512, 0, stream>>>(
          x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM, total_rows,
          nconv, r);
    else if (g_tap_mode == 12)
      conv_tap_pp_kernel<3, 0, 0, kNT, false, 3, kMT, 1, 0, 1><<<nconv + nred, 512, 0, stream>>>(
          x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM, total_rows,
          nconv, r);
    else if (g_tap_mode == 13)
      conv_tap_pp_kernel<3, 0, 0, kNT, false, 3, kMT, 1, 1, 1><<<nconv + nred, 512, 0, stream>>>(
          x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM, total_rows,
          nconv, r);
    else if (g_tap_mode == 14)
      conv_tap_pp_kernel<3, 0, 0, kNT, false, 3, kMT, 0, 0, 1><<<nconv + nred, 512, 0, stream>>>(
          x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM, total_rows,
          nconv, r);
    else if (g_tap_mode == 15)
      conv_tap_pp_kernel<4, 0, 0, kNT, false, 3, kMT, 1, 0, 1><<<nconv + nred, 512, 0, stream>>>(
          x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM, total_rows,
          nconv, r);
    else
      conv_tap_pp_kernel<3><<<nconv + nred, 512, 0, stream>>>(
          x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM, total_rows,
          nconv, r);
    return true;
  }
  // Grids too small for 384-pixel blocks (the 128-game passes of self-play: 121 blocks) but that
  // fill the chip with 192-pixel ones: the ping-pong kernel with 48 x 96 wave tiles (MT = 3) -- two
  // waves per SIMD, where conv_tap_kernel below runs ONE 4-wave block per CU, one wave per SIMD,
  // with nothing to hide its LDS reads behind. RAG_CONV_PP192=0: conv_tap_kernel.
  static const bool pp192 = [] {
    const char* v = getenv("RAG_CONV_PP192");
    return !(v && v[0] == '0');
  }();
  const int n192 = ((M + kBM - 1) / kBM) * (COUTP / kBN);
  if (pp192 && g_tap_mode >= 5 && g_tap_mode <= 20 && n192 >= pp_min &&
      cached_rows <= kPPSlabRows192) {
    int nred = 0;
    WgradRed r{};
    if (red) {
      r = *red;
      r.ticket = nullptr;  // claimed reduction: 128-wide launches only (SL -1.3 %)
      nred = std::max(8, (256 - n192 % 256) % 256);
    }
    conv_tap_pp_kernel<3, 0, 0, kNT, false, 3, 3><<<n192 + nred, 512, 0, stream>>>(
        x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM, total_rows,
        n192, r);
    return true;
  }
  if (cached_rows > kSlabRows) return false;
  const int nblk_m = (M + kBM - 1) / kBM;
  dim3 grid(nblk_m * (COUTP / kBN));
  if (g_tap_mode == 4) {
    if (red) rag_launch_wgrad_slab_reduce(*red, stream);
    conv_tap16_kernel<<<grid, 512, 0, stream>>>(x, w, bias, y, mk, res, M, S, WI, shift, WO, HO,
                                                CIN, COUTP, YC, relu, HM, total_rows);
    return true;
  }
  // reduce blocks: the slots two-blocks-per-CU leave free on 256 CUs (30 at B = 256), at least 8
  const int nconv = (int)grid.x;
  int nred = 0;
  WgradRed r{};
  if (red) {
    r = *red;
    r.ticket = nullptr;  // claimed reduction: 128-wide launches only (SL -1.3 %)
    nred = std::min(64, std::max(8, 2 * 256 - nconv));
  }
  static const int ep_lds = [] {  // RAG_EP_LDS=0: the register epilogue (A/B)
    const char* e = getenv("RAG_EP_LDS");
    return e ? atoi(e) : 1;
  }();
  conv_tap_kernel<<<nconv + nred, 256, 0, stream>>>(x, w, bias, y, mk, res, M, S, WI, shift, WO,
                                                    HO, CIN, COUTP, YC, relu, HM, total_rows,
                                                    nconv, r, g_ep_lds_override >= 0
                                                                  ? g_ep_lds_override : ep_lds);
  return true;
}

bool rag_conv_tap_bn_ok(int M, int S, int WI, int shift, int CIN, int COUTP, int KS) {
  if (g_tap_mode < 0) {
    const char* e = getenv("RAG_CONV_TAP");
    g_tap_mode = e ? atoi(e) : 12;
  }
  const char* e = getenv("RAG_PP_MIN_BLOCKS");
  const int pp_min = e ? atoi(e) : 200;
  const int nconv = ((M + kPPBM - 1) / kPPBM) * (COUTP / 128);
  return g_tap_mode >= 5 && g_tap_mode <= 20 && KS == 3 && COUTP % kBN != 0 && COUTP % 128 == 0 &&
         CIN % kBK == 0 && CIN >= kBK && nconv >= pp_min &&
         max_slab_rows(S, WI, shift, kPPBM) <= kPPSlabRows;
}

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
                long total_rows, int nconv, WgradRed red) {
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

  if (!res) {
    __syncthreads();  // every wave is past its last LDS read: the ring becomes the output image
    epilogue_lds<kBM>(acc, lds, wm * (16 * kMT), wn * (16 * kNT), m0, n0, M, S, WO, HO, YC, HM,
                      bias, relu, mask, Y, frow, fq);
  } else {
    epilogue(acc, m0 + wm * (16 * kMT), n0 + wn * (16 * kNT), M, S, WO, HO, YC, HM, bias, res,
             relu, mask, Y, frow, fq);
  }
}


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
// PRIO: one static s_setprio 1 for group 1 (the second-dispatched half) and no per-segment
// priority flips (MI355X_MICROARCH.md, "Two waves per SIMD", item 4).
// PAIR (5x5 input layer with <= 48 real input channels padded to 64): the second 32-channel
// chunk holds only 16 real channels, so its steps pair two taps -- lanes of k-quads 0/1 read
// channels 32..47 of tap t, quads 2/3 the same channels of tap t+1 (channels 48..63 of tap 24,
// zero padding, for the last, unpaired tap) -- 25 + 13 = 38 K-steps instead of 50.
// (Variants measured and deleted in round 5 -- in-loop weight issue (ISSUE 1-3), loader-group
// weight slices (WG0), spread placements 2/3, two K-steps per barrier pair (K2), register
// staging (RS), diagnostic timing builds: docs/KERNELS.md "Deleted variants".)
template <int NB, int NT = kNT, bool BNP = false, int KS = 3, int MT = kMT, int SPREAD = 0,
          int PRIO = 0, int PAIR = 0>
__global__ void __launch_bounds__(512, MT == kMT ? 1 : 4)
conv_tap_pp_kernel(const bf16* __restrict__ X, const bf16* __restrict__ Wt,
                   const float* __restrict__ bias, bf16* __restrict__ Y,
                   const bf16* __restrict__ mask, const bf16* __restrict__ res, int M, int S,
                   int WI, int shift, int WO, int HO, int CIN, int WROWS, int YC, int relu, int HM,
                   long total_rows, int nconv, WgradRed red, const float* __restrict__ bnc = nullptr,
                   const float* __restrict__ mcoef = nullptr, float* __restrict__ spart = nullptr,
                   const float* __restrict__ smean = nullptr) {
  constexpr int BN = 32 * NT, BTile = BN * kBK, PPBL = BN / 64, EpRow = BN + 8;
  constexpr bool PR = PAIR && KS == 5;
  static_assert(!PAIR || (KS == 5 && !BNP), "tap pairing: the 5x5 input layer");
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
  // weight tiles staged ahead of the current step (the slot's last reader is one phase back)
  constexpr int D = NB - 1;
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
    read_into(s, xa, wb);
    lds_reads_done();  // retire this burst before the wave's next barrier (WAR on the LDS)
  };
  auto mfmas = [&]() {
    if constexpr (!PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int i = 0; i < MT; ++i) acc[j][i] = mfma16(wb[j], xa[i], acc[j][i]);
    if constexpr (!PRIO) __builtin_amdgcn_s_setprio(0);
  };

  // Staging split between the groups, each in its own read phase: group 0 stages the slab (10 glds
  // per wave per chunk, at tap 0), group 1 the weight tiles (3 glds per wave per step, after its
  // fragment reads). Each group waits only for its own loads, before the barrier that precedes
  // the first read of that data (always group 0's, at the next X barrier).
  if (grp == 0) {
    stage_a(0);
    wait_vm<0>();
    bn_slab(0, 0, AL);
#pragma unroll 1
    for (int s = 0; s < nsteps; ++s) {
      int q, t;
      decode(s, q, t);
      const bool more = q + 1 < cchunks;
      __builtin_amdgcn_s_barrier();  // X_s
      asm volatile("" ::: "memory");
      if constexpr (SPREAD && !BNP) {
        // pieces [t*AL/(TAPS-1), (t+1)*AL/(TAPS-1)) at taps 0 .. TAPS-2; all retired by the
        // wait after the last tap's MFMAs
        if (t < TAPS - 1 && more) stage_a(q + 1, t * AL / (TAPS - 1), (t + 1) * AL / (TAPS - 1));
      } else {
        if (t == 0 && more) stage_a(q + 1);
      }
      read_frags(s);
      __builtin_amdgcn_s_barrier();  // Y_s
      asm volatile("" ::: "memory");
      mfmas();
      if constexpr (BNP) {
        // slab(q+1) complete at tap 4, transformed over taps 4..8 (this wave's reads of step s+1
        // drain the writes before the next chunk's X barrier)
        if (t >= 4 && more) {
          if (t == 4) wait_vm<0>();
          bn_slab(q + 1, 2 * (t - 4), 2 * (t - 4) + 2);
        }
      } else {
        if (t == TAPS - 1 && more) wait_vm<0>();  // slab(q+1) complete before the next chunk
      }
    }
  } else {
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);  // static: the younger half
#pragma unroll
    for (int k = 0; k < D; ++k)
      if (k < nsteps) stage_b(k);
    wait_vm_rt((nsteps - 1 < D - 1 ? nsteps - 1 : D - 1) * PPBL);  // B(0) complete
#pragma unroll 1
    for (int s = 0; s < nsteps; ++s) {
      __builtin_amdgcn_s_barrier();  // X_s
      asm volatile("" ::: "memory");
      if (s > 0) mfmas();            // step s - 1, beside group 0's reads of step s
      __builtin_amdgcn_s_barrier();  // Y_s
      asm volatile("" ::: "memory");
      read_frags(s);                 // beside group 0's MFMAs of step s
      if (s + D < nsteps) stage_b(s + D);
      // B(s+1) complete before X_{s+1}: younger are B(s+2 .. min(s+D, nsteps-1))
      int yb = nsteps - 2 - s;
      yb = yb < D - 1 ? yb : D - 1;
      wait_vm_rt(yb > 0 ? yb * PPBL : 0);
    }
    mfmas();
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
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
}

// Dispatch mode (RAG_CONV_TAP / rag_conv_tap_mode, read on first use): 0 = none of these kernels
// (conv_pipe / the caller's fallback), 6 = the plain ping-pong kernel (round 3: all slab loads at
// tap 0, per-segment priority flips) as the A/B alternative, 12 (default) = slab loads spread
// over a chunk's taps + one static priority for the second wave group: SL 111.7-111.9k ->
// 113.6-113.9k positions/s on one box (profiles/conv_variants_r4b.txt). The 128-wide, 5x5 and
// sub-chip kernels are the same in both modes.
int g_tap_mode = -1;
// Fewer 384-pixel blocks than this leave most of the chip idle: the 192-pixel kernels run them
// (B = 256 at 19x19 is 241 blocks and stays on the 384-pixel kernel).
constexpr int kPPMinBlocks = 200;

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

int tap_mode() {
  if (g_tap_mode < 0) {
    const char* e = getenv("RAG_CONV_TAP");
    g_tap_mode = e ? atoi(e) : 12;
  }
  return g_tap_mode;
}

// The reduce-block slots a launch of `nconv` one-per-CU blocks leaves free on 256 CUs (>= 8),
// and the launch's copy of the pending reduction: the 192-wide kernels keep the static split
// (their claim code measured SL -1.3 %), the 128-wide ones claim units dynamically.
int reduce_slots(int nconv, const WgradRed* red, WgradRed& r, bool claim) {
  if (!red) return 0;
  r = *red;
  if (!claim) r.ticket = nullptr;
  return std::max(8, (256 - nconv % 256) % 256);
}
}  // namespace

RAG_API int rag_conv_tap_mode(int mode) {
  const int old = g_tap_mode;
  g_tap_mode = mode;
  return old;
}

int rag_launch_wgrad_slab_reduce(const WgradRed& r, hipStream_t stream);  // wgrad_slab.hip

// bnc / mcoef (BN prologue / mask coefficients, conv_tap_pp_kernel BNP): only the 128-channel
// ping-pong path takes them; with either set, any other shape returns false.
bool rag_conv_tap_bn_ok(int M, int S, int WI, int shift, int CIN, int COUTP, int KS);

// Returns true if one of this file's kernels handled the launch: 3x3 or 5x5, 192- or
// 128-multiple output channels, input channels a multiple of 32, and every pixel run's tap
// window fits the kernel's slab. Per (taps, width) class: the 384-pixel ping-pong kernel
// (3x3 192: default / plain A/B; 128: with or without the BN prologue; 5x5: tap-paired input
// layer or plain) when the grid fills the chip, else its 192-pixel form (MT = 3), else (3x3 192,
// small grids) the 4-wave conv_tap_kernel.
bool rag_conv_tap_launch(const bf16* x, const bf16* w, const float* bias, bf16* y,
                         const bf16* mk, const bf16* res, int M, int S, int WI, int shift, int WO,
                         int HO, int CIN, int COUTP, int YC, int KS, int relu, int HM, long total_rows,
                         hipStream_t stream, const WgradRed* red, const float* bnc,
                         const float* mcoef, float* spart, const float* smean) {
  if ((bnc || mcoef || spart) &&
      ((mcoef && res) || !rag_conv_tap_bn_ok(M, S, WI, shift, CIN, COUTP, KS)))
    return false;
  const int mode = tap_mode();
  // 192-multiple widths: 96 x 96 wave tiles (NT = 6); 128-multiple widths (ResnetPolicy's and
  // the reference CNNPolicy's default 128 filters) only on the ping-pong kernel, 96 x 64 (NT = 4)
  const bool w192 = COUTP % kBN == 0, w128 = !w192 && COUTP % 128 == 0;
  if (!mode || !(KS == 3 || KS == 5) || !(w192 || w128) || CIN % kBK || CIN < kBK) return false;
  WgradRed r{};
#define RAG_PP_ARGS(NCONV)                                                                      \
  x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM, total_rows, NCONV, r
  if (KS == 5) {
    // 5x5 (the SL input layer, ResnetPolicy's first unit): the ping-pong kernel over 25 taps,
    // when the grid fills the chip and every 384-pixel run's 25-tap slab fits 768 rows
    static int key5 = -1, rows5 = 0, rows5b = 0;
    const int k5 = S * 4096 + WI * 8 + shift;
    if (k5 != key5) {
      rows5 = max_slab_rows(S, WI, shift, kPPBM, KS);
      rows5b = max_slab_rows(S, WI, shift, kBM, KS);
      key5 = k5;
    }
    if (bnc || mcoef || spart) return false;
    const int nconv = ((M + kPPBM - 1) / kPPBM) * (COUTP / (w192 ? kBN : 128));
    // <= 48 real input channels in a 64-channel layout (the caller's hint, rag_conv_igemm_cin):
    // chunk 1 steps pair two taps
    const bool pair5 = CIN == 64 && g_conv_cin_real > 0 && g_conv_cin_real <= 48;
    if (nconv < kPPMinBlocks) {
      // sub-chip grids (128-game self-play passes): 192-pixel blocks, as the 3x3 layers, at
      // every such batch (a block's time is the launch's: the self-play tail's plies of < 107
      // games ran conv_pipe at 45.6 us against 32.5 us for this kernel at 128 games,
      // profiles/rl_selfplay_r5.txt)
      const int n192 = ((M + kBM - 1) / kBM) * (COUTP / kBN);
      if (!w192 || rows5b > kPPSlabRows192x5) return false;
      const int nred = reduce_slots(n192, red, r, false);
      if (pair5)
        conv_tap_pp_kernel<3, 6, false, 5, 3, 0, 0, 1><<<n192 + nred, 512, 0, stream>>>(
            RAG_PP_ARGS(n192));
      else
        conv_tap_pp_kernel<3, 6, false, 5, 3><<<n192 + nred, 512, 0, stream>>>(RAG_PP_ARGS(n192));
      return true;
    }
    if (rows5 > kPPSlabRows5) return false;
    const int nred = reduce_slots(nconv, red, r, !w192);
    if (w192 && pair5)
      conv_tap_pp_kernel<3, 6, false, 5, kMT, 0, 0, 1><<<nconv + nred, 512, 0, stream>>>(
          RAG_PP_ARGS(nconv));
    else if (w192)
      conv_tap_pp_kernel<3, 6, false, 5><<<nconv + nred, 512, 0, stream>>>(RAG_PP_ARGS(nconv));
    else if (pair5)  // 128 filters (ResnetPolicy's input layer)
      conv_tap_pp_kernel<3, 4, false, 5, kMT, 0, 0, 1><<<nconv + nred, 512, 0, stream>>>(
          RAG_PP_ARGS(nconv));
    else
      conv_tap_pp_kernel<3, 4, false, 5><<<nconv + nred, 512, 0, stream>>>(RAG_PP_ARGS(nconv));
    return true;
  }
  static int cached_key = -1, cached_rows = 0, cached_rows8 = 0;
  const int key = S * 4096 + WI * 8 + shift;
  if (key != cached_key) {
    cached_rows = max_slab_rows(S, WI, shift, kBM);
    cached_rows8 = max_slab_rows(S, WI, shift, kPPBM);
    cached_key = key;
  }
  if (w128) {
    const int nconv = ((M + kPPBM - 1) / kPPBM) * (COUTP / 128);
    if (cached_rows8 > kPPSlabRows || nconv < kPPMinBlocks) return false;  // small: conv_pipe
    // claimed reduction (r.ticket): CNNPolicy-128 164.9 -> 169.2 k positions/s
    const int nred = reduce_slots(nconv, red, r, true);
    if (bnc)
      conv_tap_pp_kernel<3, 4, true><<<nconv + nred, 512, 0, stream>>>(RAG_PP_ARGS(nconv), bnc,
                                                                        mcoef, spart, smean);
    else
      conv_tap_pp_kernel<3, 4, false><<<nconv + nred, 512, 0, stream>>>(
          RAG_PP_ARGS(nconv), nullptr, mcoef, spart, smean);
    return true;
  }
  const int nconv = ((M + kPPBM - 1) / kPPBM) * (COUTP / kBN);
  if (cached_rows8 <= kPPSlabRows && nconv >= kPPMinBlocks) {
    // ping-pong kernel: one block per CU; reduce blocks fill the CUs its last round leaves free
    const int nred = reduce_slots(nconv, red, r, false);
    if (mode == 6)
      conv_tap_pp_kernel<3><<<nconv + nred, 512, 0, stream>>>(RAG_PP_ARGS(nconv));
    else
      conv_tap_pp_kernel<3, kNT, false, 3, kMT, 1, 1><<<nconv + nred, 512, 0, stream>>>(
          RAG_PP_ARGS(nconv));
    return true;
  }
  // Grids too small for 384-pixel blocks (the 128-game passes of self-play: 121 blocks) but that
  // fill the chip with 192-pixel ones: the ping-pong kernel with 48 x 96 wave tiles (MT = 3) -- two
  // waves per SIMD, where conv_tap_kernel below runs ONE 4-wave block per CU, one wave per SIMD,
  // with nothing to hide its LDS reads behind.
  const int n192 = ((M + kBM - 1) / kBM) * (COUTP / kBN);
  if (n192 >= kPPMinBlocks && cached_rows <= kPPSlabRows192) {
    const int nred = reduce_slots(n192, red, r, false);
    conv_tap_pp_kernel<3, kNT, false, 3, 3><<<n192 + nred, 512, 0, stream>>>(RAG_PP_ARGS(n192));
    return true;
  }
#undef RAG_PP_ARGS
  if (cached_rows > kSlabRows) return false;
  // reduce blocks: the slots two-blocks-per-CU leave free on 256 CUs (30 at B = 256), at least 8
  const int nc = ((M + kBM - 1) / kBM) * (COUTP / kBN);
  int nred = 0;
  if (red) {
    r = *red;
    r.ticket = nullptr;
    nred = std::min(64, std::max(8, 2 * 256 - nc));
  }
  conv_tap_kernel<<<nc + nred, 256, 0, stream>>>(x, w, bias, y, mk, res, M, S, WI, shift, WO, HO,
                                                 CIN, COUTP, YC, relu, HM, total_rows, nc, r);
  return true;
}

bool rag_conv_tap_bn_ok(int M, int S, int WI, int shift, int CIN, int COUTP, int KS) {
  const int nconv = ((M + kPPBM - 1) / kPPBM) * (COUTP / 128);
  return tap_mode() && KS == 3 && COUTP % kBN != 0 && COUTP % 128 == 0 && CIN % kBK == 0 &&
         CIN >= kBK && nconv >= kPPMinBlocks && max_slab_rows(S, WI, shift, kPPBM) <= kPPSlabRows;
}

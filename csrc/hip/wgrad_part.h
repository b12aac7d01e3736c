// Block-scaled fp16 partial slabs of wgrad_slab_kernel (wgrad_slab.hip) and their chunk reduction, shared by
// the standalone reduce kernel and the reduce blocks fused into the next dgrad launch
// (conv_tap.hip).
//
// Partials are fp16 with one power-of-two scale per block (block floating point: the block's
// largest |partial| maps into [2^14, 2^15), 11 mantissa bits instead of bf16's 8 at the same
// bytes); scale[chunk * ntc + ctile] holds the inverse factor.
// Layout per chunk: [ctile][slot][wave][lane][4] fp16, slot = i * NA + a (WMap: wave w owns NA
// n-frags starting at nf0(w), c-frag cf(w) and NT taps tap(w, i)); an "oct" is 8 consecutive
// elements = the 4-value C fragments of two adjacent lanes.
#pragma once
#include "common.h"

namespace rag {

// A block owns all N output channels (N = 192: 12 waves, N = 128: 8 waves, one wave per 16 of
// them) x one 32-channel c-tile x 9 taps.
constexpr int kWsC = 32;                    // input channels per block (c-tile)
__host__ __device__ constexpr int ws_blk(int n) { return 9 * n * kWsC; }  // accumulators / block

// Everything a chunk reduction needs (passed by value into kernels).
typedef _Float16 f16;
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

struct WgradRed {
  const f16* part;     // [nchunks][ntc * blk] scaled fp16 partials
  const float* scale;  // [nchunks * ntc] inverse block scales
  const float* bpart;  // [nchunks][n] fp32 bias partials (or null)
  float* dW;           // OIHW [COUT][CIN][3][3]
  float* db;           // [COUT] (or null)
  int nchunks, ntc, COUT, CIN, accumulate, map;
  int n, waves, blk;   // block channels (192 | 128), waves (n / 16), accumulators per block
  int taps, kgrp;      // KS * KS; blocks per c-tile (5x5: one kernel row each, else 1)
  int pair5;           // 5x5 with <= 48 of 64 channels: pseudo c-tiles 5..7 = c-tile 1, rows 2p, 2p+1
  // [2] device counters (claim ticket, finished blocks), zero between launches: kernels that
  // support it claim the reduction in block-sized units (wslab_reduce_dynamic); null = static
  unsigned* ticket;
};

__device__ __forceinline__ void wslab_add8(float (&s)[8], const uint4& v, float sc) {
  const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const f16x2 h = __builtin_bit_cast(f16x2, u[j]);
    s[2 * j] += sc * (float)h[0];
    s[2 * j + 1] += sc * (float)h[1];
  }
}

// Scatter the chunk sum of oct q to OIHW dW.
__device__ __forceinline__ void wslab_store_oct(const WgradRed& r, int q, const float (&s)[8]) {
  const int e = q * 8;
  const int pct = e / r.blk;  // (pseudo) c-tile: c-tile * kgrp + kernel row
  const int loc = e - pct * r.blk;
  const bool pblk = r.pair5 && pct >= 5;
  const int ctile = pblk ? 1 : pct / r.kgrp;
  int ky = pblk ? 2 * (pct - 5) : pct - ctile * r.kgrp;
  const int lane0 = (loc >> 2) & 63;
  const int wv = (loc >> 8) % r.waves;
  const int slot = (loc >> 8) / r.waves;  // i * NA + a
  int nb, cb, t;
  if (r.map) {
    const int a = slot % 6, i = slot / 6;
    t = (wv >> 2) * 3 + i;
    nb = ((wv & 1) * 6 + a) * 16;
    cb = ctile * kWsC + ((wv >> 1) & 1) * 16;
  } else {  // map 0: wave wv owns n-frags 2 (wv % g), +1 and c-frag wv / g, g = n / 32
    const int a = slot & 1, g = r.n >> 5;
    if (pblk) {  // the wave group picks the kernel row, the c-fragment is c-tile 1's first
      ky += wv / g;
      if (ky >= 5) return;
      cb = kWsC;
    } else {
      cb = ctile * kWsC + (wv / g) * 16;
    }
    t = ky * 5 + (slot >> 1);  // 3x3: ky = 0, slot >> 1 = tap; 5x5: the block's row ky, kx
    nb = ((wv % g) * 2 + a) * 16;
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int lane = lane0 + h;
    const int c = cb + (lane & 15);
    if (c >= r.CIN) continue;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int n = nb + (lane >> 4) * 4 + k;
      if (n >= r.COUT) continue;
      const size_t o = ((size_t)n * r.CIN + c) * r.taps + t;
      r.dW[o] = r.accumulate ? r.dW[o] + s[h * 4 + k] : s[h * 4 + k];
    }
  }
}

// Reduce blocks fused into another kernel: block b of nb handles octs b*T + tid, stepping nb*T,
// each summed over all chunks with U 16-byte loads in flight; block 0 also sums the bias.
// One oct: its chunk sum (U 16-byte loads in flight) scattered to dW.
template <int U>
__device__ __forceinline__ void wslab_reduce_oct(const WgradRed& r, int q) {
  const size_t st = (size_t)r.ntc * r.blk / 8;  // uint4 stride between chunks
  float s[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = 0.f;
  const uint4* p = reinterpret_cast<const uint4*>(r.part) + q;
  const float* sc = r.scale + (q * 8) / r.blk;  // + chunk * ntc
  int k = 0;
  for (; k + U <= r.nchunks; k += U) {
    uint4 a[U];
#pragma unroll
    for (int j = 0; j < U; ++j) a[j] = p[(size_t)(k + j) * st];
#pragma unroll
    for (int j = 0; j < U; ++j) wslab_add8(s, a[j], sc[(k + j) * r.ntc]);
  }
  for (; k < r.nchunks; ++k) wslab_add8(s, p[(size_t)k * st], sc[k * r.ntc]);
  wslab_store_oct(r, q, s);
}

__device__ __forceinline__ void wslab_reduce_bias(const WgradRed& r, int tid, int T) {
  for (int n = tid; n < r.COUT; n += T) {
    float v = 0.f;
    for (int k = 0; k < r.nchunks; ++k) v += r.bpart[(size_t)k * r.n + n];
    r.db[n] = r.accumulate ? r.db[n] + v : v;
  }
}

template <int U>
__device__ __forceinline__ void wslab_reduce_blocks(const WgradRed& r, int b, int nb) {
  const int T = blockDim.x, tid = threadIdx.x;
  const int octs = r.ntc * r.blk / 8;
  for (int q = b * T + tid; q < octs; q += nb * T) wslab_reduce_oct<U>(r, q);
  if (b == 0 && r.db && r.bpart) wslab_reduce_bias(r, tid, T);
}

// The reduction claimed in units of blockDim.x octs (the last unit: the bias) through the
// r.ticket counter, by EVERY block of the launch: the riding reduce blocks from the start (in the
// CU slots the convolution grid leaves free), the convolution blocks after their epilogue. With
// a static split the few riding blocks did all of it and were the launch's tail (128-channel
// dgrad: 50 vs 38 us without a reduction). Each block exits after its first failed claim, then
// counts itself finished; the last one resets both counters (the claim's returned value orders
// it before the count). The slab launch that writes the partials zeroes them as well, so a
// claiming launch in which some block never got here cannot leave the next reduction a stale
// ticket (which would skip it). smem: one int of LDS, free at the call.
template <int U>
__device__ __forceinline__ void wslab_reduce_dynamic(const WgradRed& r, int* smem) {
  const int T = blockDim.x, tid = threadIdx.x;
  const int octs = r.ntc * r.blk / 8;
  const int units = (octs + T - 1) / T;
  const int nunits = units + ((r.db && r.bpart) ? 1 : 0);
  __syncthreads();  // smem may still be read by the caller's last LDS phase
  while (true) {
    if (tid == 0) smem[0] = (int)atomicAdd(&r.ticket[0], 1u);
    __syncthreads();
    const int u = smem[0];
    __syncthreads();
    if (u >= nunits) break;
    if (u < units) {
      const int q = u * T + tid;
      if (q < octs) wslab_reduce_oct<U>(r, q);
    } else {
      wslab_reduce_bias(r, tid, T);
    }
  }
  if (tid == 0) {
    const unsigned done = atomicAdd(&r.ticket[1], 1u);
    if (done == gridDim.x - 1) {
      atomicExch(&r.ticket[0], 0u);
      atomicExch(&r.ticket[1], 0u);
    }
  }
}

}  // namespace rag

// Network heads on gfx950 — kernels K03/K04 (policy head + fused softmax cross-entropy /
// REINFORCE loss) and the 1x1-conv part of K11 (value head), forward and backward.
//
// Policy head (reference policy.py:124-136 + nn_util.py:118-133):
//   z[b,p] = sum_k w[k] * h[b,p,k] + b0 + bias[p];  prob = softmax_p(z)
// One workgroup per board: pixel dot products (16-byte channel loads), logits kept in LDS, block
// max/sum reductions, then probabilities, per-sample loss, dL/dz and top-1 hit written in the same
// pass. Loss modes: 0 = none (inference), 1 = categorical cross-entropy (Keras, mean over batch),
// 2 = REINFORCE log_loss (Keras: -y log clip(p), averaged over the S*S classes and the batch;
// reinforcement_policy_trainer.py:89-94), each sample scaled by an optional signed weight.
#include "common.h"

using namespace rag;

namespace {

constexpr int kHeadThreads = 256;
// policy_head_fwd: 1024 threads, 8 per pixel: a 19x19 board's 361 dot products take three
// coalesced passes (one lane per pixel and 384 threads: 18.3 us for B = 256, now 13.5 us; the
// kernel is latency-bound, one block per board)
constexpr int kHeadFwdThreads = 1024;

__device__ __forceinline__ float block_reduce(float v, float* sh, bool is_max) {
  v = is_max ? warp_max(v) : warp_sum(v);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  float r = sh[0];
  const int nw = blockDim.x >> 6;
  for (int k = 1; k < nw; ++k) r = is_max ? fmaxf(r, sh[k]) : r + sh[k];
  return r;
}

__global__ void __launch_bounds__(kHeadFwdThreads)
policy_head_fwd_kernel(const bf16* __restrict__ H, const float* __restrict__ w, const float* b0,
                       const float* __restrict__ pbias, float* __restrict__ probs,
                       const int64_t* __restrict__ labels, const float* __restrict__ sweight,
                       float* __restrict__ loss, float* __restrict__ dz, float* __restrict__ hit,
                       const float* __restrict__ pass_w, const float* __restrict__ pass_b,
                       float* __restrict__ zout, float* __restrict__ dpass,
                       float* __restrict__ acc, int S, int KP, int K, int mode, float gscale,
                       float* __restrict__ dzsum = nullptr) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* z = smem;                        // S*S logits (+ the pass logit)
  float* ws = smem + ((S * S + 4) & ~3);  // KP weights
  __shared__ float red[16];
  const int b = blockIdx.x;
  const int S2 = S * S, WP = S + 2;
  for (int k = threadIdx.x; k < KP; k += blockDim.x) ws[k] = k < K ? w[k] : 0.f;
  __syncthreads();
  const float bias0 = b0 ? *b0 : 0.f;
  // 8 lanes per pixel, each a 16-byte slice of every 128-byte channel segment: a wave's load
  // instruction reads 8 pixels x 128 contiguous bytes (one lane per pixel read 384-byte rows in
  // 16-byte steps, one dependent load after another: 18 us for B = 256), then a 3-step
  // cross-lane sum
  {
    const int sub = threadIdx.x & 7;
    for (int p0 = threadIdx.x >> 3; p0 < ((S2 + 7) & ~7); p0 += blockDim.x >> 3) {
      const int p = p0 < S2 ? p0 : S2 - 1;
      const int i = p / S, j = p - (p / S) * S;
      const bf16* row = H + ((size_t)(b * WP + i + 1) * WP + j + 1) * KP;
      float acc = 0.f;
#pragma unroll 4
      for (int c = sub * 8; c < KP; c += 64) {
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(row + c);
#pragma unroll
        for (int t = 0; t < 8; ++t) acc += (float)v[t] * ws[c + t];
      }
      acc += __shfl_xor(acc, 1);
      acc += __shfl_xor(acc, 2);
      acc += __shfl_xor(acc, 4);
      if (sub == 0 && p0 < S2) z[p] = acc + bias0 + (pbias ? pbias[p] : 0.f);
    }
  }
  __syncthreads();
  // optional pass logit (PassLogit layer): W . z + b over the position logits, the
  // softmax then runs over C = S*S + 1 classes with pass last
  const bool has_pass = pass_w != nullptr;
  const int C = S2 + (has_pass ? 1 : 0);
  if (has_pass) {
    float pd = 0.f;
    for (int p = threadIdx.x; p < S2; p += blockDim.x) {
      pd += pass_w[p] * z[p];
      if (zout) zout[(size_t)b * S2 + p] = z[p];
    }
    pd = block_reduce(pd, red, false);
    if (threadIdx.x == 0) z[S2] = pd + *pass_b;
    __syncthreads();
  }
  float mx = -INFINITY;
  int amax = 0;
  for (int p = threadIdx.x; p < C; p += blockDim.x)
    if (z[p] > mx) {
      mx = z[p];
      amax = p;
    }
  const float gmax = block_reduce(mx, red, true);
  float se = 0.f;
  for (int p = threadIdx.x; p < C; p += blockDim.x) se += __expf(z[p] - gmax);
  const float sum = block_reduce(se, red, false);
  const float inv = 1.f / sum;
  const int64_t lab = (mode && labels) ? labels[b] : -1;
  const float sw = sweight ? sweight[b] : 1.f;
  const float cls = (mode == 2) ? 1.f / (float)C : 1.f;
  // dL/d(pass logit): it also flows back into every position logit through W
  float dp = 0.f;
  if (has_pass) {
    const float pp = __expf(z[S2] - gmax) * inv;
    dp = (pp - (lab == S2 ? 1.f : 0.f)) * sw * cls * gscale;
    if (threadIdx.x == 0) {
      probs[(size_t)b * C + S2] = pp;
      if (mode && dpass) dpass[b] = dp;
    }
  }
  float dsum = 0.f;
  for (int p = threadIdx.x; p < S2; p += blockDim.x) {
    const float pr = __expf(z[p] - gmax) * inv;
    probs[(size_t)b * C + p] = pr;
    if (mode && dz) {
      const float y = (p == lab) ? 1.f : 0.f;
      const float d = (pr - y) * sw * cls * gscale + (has_pass ? dp * pass_w[p] : 0.f);
      dz[(size_t)b * S2 + p] = d;
      dsum += d;
    }
  }
  if (mode && dz && dzsum) {  // the board's sum of dz (block-uniform branch), for db0
    dsum = block_reduce(dsum, red, false);
    if (threadIdx.x == 0) dzsum[b] = dsum;
  }
  if (mode && threadIdx.x == 0 && lab >= 0) {
    float pl = __expf(z[lab] - gmax) * inv;
    pl = fminf(fmaxf(pl, 1e-7f), 1.f - 1e-7f);
    const float lb = -__logf(pl) * sw * cls;
    if (loss) loss[b] = lb;
    if (acc) atomicAdd(&acc[0], lb);  // running metric sums (training loops read them lazily)
  } else if (mode && threadIdx.x == 0 && loss) {
    loss[b] = 0.f;  // unlabelled board: the backward's metric reduce sums loss[:B] as is
  }
  // top-1 hit (ties -> lowest index, like argmax)
  if (mode && hit) {
    // reduce (value, index) pair: first the max value is known (gmax); find lowest index == gmax
    int cand = (mx == gmax) ? amax : 0x7fffffff;
    for (int o = 32; o > 0; o >>= 1) cand = min(cand, __shfl_xor(cand, o, 64));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = __int_as_float(cand);
    __syncthreads();
    if (threadIdx.x == 0) {
      int best = 0x7fffffff;
      for (int k = 0; k < (int)(blockDim.x >> 6); ++k) best = min(best, __float_as_int(red[k]));
      hit[b] = (best == lab) ? 1.f : 0.f;
      if (acc && best == lab) atomicAdd(&acc[1], 1.f);
    }
  }
}

// Backward of the 1x1 K->1 head conv (+ per-position bias), two launches without contended
// atomics:
//  (1) per block of pixels: dH[b,p,k] = dz[b,p] * w[k] * (H[b,p,k] > 0)  (fused ReLU derivative
//      of the last trunk layer) and the block's partial dw: dwpart[blk,k] = sum_p dz * H[., k].
//      The PPI pixel lanes of a block combine their dw partials through an LDS array (plain
//      stores + one column sum; LDS atomics on 192 addresses serialised ~2k adds per block).
//  (2) column sums with coalesced row reads: dw[k] = sum_blk dwpart[blk,k],
//      dpbias[p] = sum_b dz[b,p], db0 = sum_p dpbias[p].
constexpr int kHeadBwdBlocks = 256;  // <= one block per CU: dwpart stays 256 rows
template <int CH>  // CH = KP / 8 sixteen-byte channel chunks per pixel row
__global__ void __launch_bounds__(kHeadThreads)
head_bwd_kernel(const bf16* __restrict__ H, const float* __restrict__ w,
                const float* __restrict__ dz, bf16* __restrict__ dH, float* __restrict__ dwpart,
                float* __restrict__ db0, int npix, int pix_per_block, int S, int K,
                int relu_mask) {
  constexpr int KP = CH * 8;
  constexpr int PPI = kHeadThreads / CH;  // pixels per block iteration
  __shared__ float ws[KP];
  __shared__ __attribute__((aligned(16))) float dwl[PPI][KP];
  for (int k = threadIdx.x; k < KP; k += blockDim.x) ws[k] = k < K ? w[k] : 0.f;
  if (blockIdx.x == 0 && threadIdx.x == 0 && db0) *db0 = 0.f;
  __syncthreads();
  const int S2 = S * S, WP = S + 2;
  const int ch = threadIdx.x % CH, sub = threadIdx.x / CH;
  float wl[8], dwacc[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    wl[t] = ws[ch * 8 + t];
    dwacc[t] = 0.f;
  }
  const int pbeg = blockIdx.x * pix_per_block;
  const int pend = min(npix, pbeg + pix_per_block);
  if (sub < PPI) {
    // 8 pixels per batch: all loads issued before any use (memory-level parallelism)
    constexpr int U = 8;
    for (int P0 = pbeg + sub; P0 < pend; P0 += U * PPI) {
      size_t off[U];
      float g[U];
      bf16x8 hv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int P = min(P0 + u * PPI, pend - 1);
        const int b = P / S2, p = P - (P / S2) * S2;
        const int i = p / S, j = p - (p / S) * S;
        off[u] = ((size_t)(b * WP + i + 1) * WP + j + 1) * KP + ch * 8;
        g[u] = (P0 + u * PPI < pend) ? dz[P] : 0.f;
        hv[u] = *reinterpret_cast<const bf16x8*>(H + off[u]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        bf16x8 o;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const float hf = (float)hv[u][t];
          float d = g[u] * wl[t];
          if (relu_mask && !(hf > 0.f)) d = 0.f;
          o[t] = (bf16)d;
          dwacc[t] += g[u] * hf;
        }
        if (dH && P0 + u * PPI < pend) *reinterpret_cast<bf16x8*>(dH + off[u]) = o;
      }
    }
    float4* dst = reinterpret_cast<float4*>(&dwl[sub][ch * 8]);
    dst[0] = make_float4(dwacc[0], dwacc[1], dwacc[2], dwacc[3]);
    dst[1] = make_float4(dwacc[4], dwacc[5], dwacc[6], dwacc[7]);
  }
  __syncthreads();
  for (int k = threadIdx.x; k < KP; k += blockDim.x) {
    float v = 0.f;
#pragma unroll
    for (int r = 0; r < PPI; ++r) v += dwl[r][k];
    dwpart[(size_t)blockIdx.x * KP + k] = v;
  }
}

// Column sums of a row-major [rows][ld] fp32 matrix over 64-column tiles: 1024 threads = 64
// columns x 16 row lanes (each row segment is one coalesced 256-byte read), 16-way LDS combine.
// Blocks [0, ceil(K/64)): dw[k] = sum_blk dwpart[blk][k]; the rest: dpbias[p] = sum_b dz[b][p]
// and db0 += the block's sum of its dpbias columns.
__global__ void __launch_bounds__(1024)
head_bwd_reduce_kernel(const float* __restrict__ dwpart, const float* __restrict__ dz,
                       float* __restrict__ dw, float* __restrict__ db0,
                       float* __restrict__ dpbias, int nblk, int B, int S2, int KP, int K,
                       const float* __restrict__ mloss = nullptr,
                       const float* __restrict__ mhit = nullptr, float* __restrict__ acc = nullptr,
                       const float* __restrict__ dzsum = nullptr) {
  __shared__ float red[16][65];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int kt = (K + 63) / 64;
  if ((int)blockIdx.x == (int)gridDim.x - 1) {
    // the last block: db0 = sum of all dz (fixed summation order, so the step is bit-for-bit
    // reproducible -- per-block atomics made it depend on block timing), and the forward's
    // running metrics acc[0] += sum loss, acc[1] += sum hit (instead of two contended device
    // atomics per board in the head forward)
    float d = 0.f, a = 0.f, h = 0.f;
    if (db0 && dzsum) {  // the head forward's per-board sums
      for (int i = threadIdx.x; i < B; i += blockDim.x) d += dzsum[i];
    } else if (db0) {
      // all of dz (the value head: no per-board sums): 16-byte loads, four in flight per
      // thread on independent sums (one dependent 4-byte load at a time took 24 us for
      // 256 x 361 values -- the whole value-net step's longest small kernel)
      const size_t n = (size_t)B * S2, n4 = (reinterpret_cast<uintptr_t>(dz) & 15) ? 0 : n / 4;
      const float4* d4 = reinterpret_cast<const float4*>(dz);
      const size_t bt = blockDim.x;
      float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
      size_t i = threadIdx.x;
      for (; i + 3 * bt < n4; i += 4 * bt) {
        const float4 a = d4[i], b = d4[i + bt], c = d4[i + 2 * bt], e = d4[i + 3 * bt];
        s0 += (a.x + a.y) + (a.z + a.w);
        s1 += (b.x + b.y) + (b.z + b.w);
        s2 += (c.x + c.y) + (c.z + c.w);
        s3 += (e.x + e.y) + (e.z + e.w);
      }
      for (; i < n4; i += bt) {
        const float4 a = d4[i];
        s0 += (a.x + a.y) + (a.z + a.w);
      }
      for (size_t j = n4 * 4 + threadIdx.x; j < n; j += bt) s1 += dz[j];
      d = (s0 + s1) + (s2 + s3);
    }
    if (acc)
      for (int i = threadIdx.x; i < B; i += blockDim.x) {
        a += mloss[i];
        h += mhit[i];
      }
    d = warp_sum(d);
    a = warp_sum(a);
    h = warp_sum(h);
    if (tx == 0) {
      red[ty][0] = d;
      red[ty][1] = a;
      red[ty][2] = h;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      float sd = 0.f, sa = 0.f, sh = 0.f;
      for (int k = 0; k < (int)(blockDim.x >> 6); ++k) {
        sd += red[k][0];
        sa += red[k][1];
        sh += red[k][2];
      }
      if (db0) *db0 = sd;
      if (acc) {
        acc[0] += sa;
        acc[1] += sh;
      }
    }
    return;
  }
  const bool isw = (int)blockIdx.x < kt;
  const int col = (isw ? (int)blockIdx.x : (int)blockIdx.x - kt) * 64 + tx;
  const int ncol = isw ? K : S2;
  const int rows = isw ? nblk : B;
  const int ld = isw ? KP : S2;
  const float* src = isw ? dwpart : dz;
  float s = 0.f;
  if (col < ncol) {
    constexpr int U = 4;
    int r = ty;
    for (; r + 16 * (U - 1) < rows; r += 16 * U) {
      float a[U];
#pragma unroll
      for (int u = 0; u < U; ++u) a[u] = src[(size_t)(r + 16 * u) * ld + col];
#pragma unroll
      for (int u = 0; u < U; ++u) s += a[u];
    }
    for (; r < rows; r += 16) s += src[(size_t)r * ld + col];
  }
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0) {
    float v = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) v += red[r][tx];
    if (col < ncol) {
      if (isw) {
        dw[col] = v;
      } else if (dpbias) {
        dpbias[col] = v;
      }
    }
  }
}

// z[b,p] = sum_k w[k]*h[b,p,k] + b0 (value-head 1x1 conv, no softmax). 8 lanes per pixel
// (coalesced 128-byte channel segments, as policy_head_fwd_kernel), each lane's NM x 8 weights
// in registers for the whole grid-stride loop: the first version loaded w[c + t] per element
// and pixel (24 loads per lane per pixel for K = 192), 23 us for a B = 256 batch against the
// ~8 us its 35 MB of reads need. NM = 0: any K (weights read per pixel).
template <int NM>
__global__ void __launch_bounds__(kHeadThreads)
head_linear_kernel(const bf16* __restrict__ H, const float* __restrict__ w, const float* b0,
                   float* __restrict__ z, int B, int S, int KP, int K) {
  const int S2 = S * S, WP = S + 2;
  const int total = B * S2;
  const int sub = threadIdx.x & 7;
  float wr[NM > 0 ? NM : 1][8];
  if constexpr (NM > 0) {
#pragma unroll
    for (int m = 0; m < NM; ++m)
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const int c = m * 64 + sub * 8 + t;
        wr[m][t] = c < K ? w[c] : 0.f;
      }
  }
  const float bias = b0 ? *b0 : 0.f;
  const int groups = (int)((gridDim.x * blockDim.x) >> 3);
  // every lane of an 8-lane group runs the same iterations (the shuffles stay inside it)
  for (int idx = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 3); idx < total;
       idx += groups) {
    const int b = idx / S2, p = idx - b * S2;
    const int i = p / S, j = p - i * S;
    const bf16* row = H + ((size_t)(b * WP + i + 1) * WP + j + 1) * KP;
    float acc = 0.f;
    if constexpr (NM > 0) {
#pragma unroll
      for (int m = 0; m < NM; ++m) {
        const int c = m * 64 + sub * 8;
        if (c < K) {  // (K a multiple of 8: a lane's 8 channels are all in or all out)
          const bf16x8 v = *reinterpret_cast<const bf16x8*>(row + c);
#pragma unroll
          for (int t = 0; t < 8; ++t) acc = fmaf((float)v[t], wr[m][t], acc);
        }
      }
    } else {
      for (int c = sub * 8; c < K; c += 64) {
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(row + c);
#pragma unroll
        for (int t = 0; t < 8; ++t)
          if (c + t < K) acc += (float)v[t] * w[c + t];
      }
    }
    acc += __shfl_xor(acc, 1);
    acc += __shfl_xor(acc, 2);
    acc += __shfl_xor(acc, 4);
    if (sub == 0) z[idx] = acc + bias;
  }
}


// Value-net MLP tail for inference: out[b] = tanh(act(z[b] . W1 + b1) . W2 + b2).
// z [B, P] fp32, W1 [P, H] row-major, W2 [H]. Replaces two library GEMM launches whose single
// 256x256 macro-tile put the whole B = 256 leaf batch on one workgroup (~110 us).
// Pass 1: a block owns kMlpRows boards x 64 output columns; its 4 waves split the P reduction
// (lanes = columns, so every W1 read is one coalesced 256-byte row segment; 8 waves measured
// 10.5 us vs 16.7 us for 4 on a B = 256 leaf batch), the wave partials
// are summed through LDS, then act(h) * W2 is reduced over the 64 columns into
// part[b][column tile]. Pass 2 sums the column tiles and applies tanh. B = 256, H = 256 gives
// 256 blocks (one per CU) instead of one.
constexpr int kMlpRows = 4;
constexpr int kMlpCols = 64;
constexpr int kMlpWaves = 8;

__global__ void __launch_bounds__(64 * kMlpWaves)
value_mlp_part_kernel(const float* __restrict__ z, const float* __restrict__ W1,
                      const float* __restrict__ b1, const float* __restrict__ W2,
                      float* __restrict__ part, float* __restrict__ hout, int B, int P, int H,
                      int act) {
  extern __shared__ float zs[];  // [kMlpRows][P], then [kMlpWaves][kMlpRows][64] partials
  float* red = zs + kMlpRows * P;
  const int ntile = (H + kMlpCols - 1) / kMlpCols;
  const int tile = blockIdx.x % ntile;
  const int b0 = (blockIdx.x / ntile) * kMlpRows;
  const int nr = B - b0 < kMlpRows ? B - b0 : kMlpRows;
  for (int i = threadIdx.x; i < kMlpRows * P; i += 64 * kMlpWaves) {
    const int r = i / P;
    zs[i] = r < nr ? z[(size_t)(b0 + r) * P + (i - r * P)] : 0.f;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = tile * kMlpCols + lane;
  const int kper = (P + kMlpWaves - 1) / kMlpWaves;
  const int k0 = wave * kper, k1 = k0 + kper < P ? k0 + kper : P;
  float acc[kMlpRows];
#pragma unroll
  for (int r = 0; r < kMlpRows; ++r) acc[r] = 0.f;
  if (j < H) {
    const float* wc = W1 + j;
    int k = k0;
    for (; k + 3 < k1; k += 4) {
      const float w0 = wc[(size_t)k * H], w1 = wc[(size_t)(k + 1) * H],
                  w2 = wc[(size_t)(k + 2) * H], w3 = wc[(size_t)(k + 3) * H];
#pragma unroll
      for (int r = 0; r < kMlpRows; ++r) {
        const float* zr = zs + r * P + k;
        acc[r] += zr[0] * w0 + zr[1] * w1 + zr[2] * w2 + zr[3] * w3;
      }
    }
    for (; k < k1; ++k) {
      const float w0 = wc[(size_t)k * H];
#pragma unroll
      for (int r = 0; r < kMlpRows; ++r) acc[r] += zs[r * P + k] * w0;
    }
  }
#pragma unroll
  for (int r = 0; r < kMlpRows; ++r) red[(wave * kMlpRows + r) * 64 + lane] = acc[r];
  __syncthreads();
  if (wave < kMlpRows) {  // wave r finishes board r
    const int r = wave;
    float h = 0.f;
    for (int w = 0; w < kMlpWaves; ++w) h += red[(w * kMlpRows + r) * 64 + lane];
    float v = 0.f;
    if (j < H) {
      h += b1[j];
      if (hout && r < nr) hout[(size_t)(b0 + r) * H + j] = h;  // pre-activation, for training
      if (act == 1) h = h > 0.f ? h : 0.f;
      else if (act == 2) h = tanhf(h);
      v = h * W2[j];
    }
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0 && r < nr) part[(size_t)(b0 + r) * ntile + tile] = v;
  }
}

__global__ void value_mlp_out_kernel(const float* __restrict__ part, const float* __restrict__ b2,
                                     float* __restrict__ out, int B, int ntile) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float s = *b2;
  for (int t = 0; t < ntile; ++t) s += part[(size_t)b * ntile + t];
  out[b] = tanhf(s);
}

// PassLogit weight gradients: dW[j] = sum_b zout[b, j] * dpass[b] (one lane per point,
// coalesced over j; the batch loop is 4-way unrolled), db = sum_b dpass[b] (block 0, wave
// reduction). Overwrites dW / db.
constexpr int kPassThreads = 128;

__global__ void __launch_bounds__(kPassThreads)
pass_grads_kernel(const float* __restrict__ z, const float* __restrict__ dpass,
                  float* __restrict__ dW, float* __restrict__ db, int B, int P) {
  const int j = blockIdx.x * kPassThreads + threadIdx.x;
  if (j < P) {
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int b = 0;
    for (; b + 4 <= B; b += 4) {
      a0 += z[(size_t)b * P + j] * dpass[b];
      a1 += z[(size_t)(b + 1) * P + j] * dpass[b + 1];
      a2 += z[(size_t)(b + 2) * P + j] * dpass[b + 2];
      a3 += z[(size_t)(b + 3) * P + j] * dpass[b + 3];
    }
    for (; b < B; ++b) a0 += z[(size_t)b * P + j] * dpass[b];
    dW[j] = (a0 + a1) + (a2 + a3);
  }
  if (blockIdx.x == 0) {
    __shared__ float red[kPassThreads / 64];
    float s = 0.f;
    for (int b = threadIdx.x; b < B; b += kPassThreads) s += dpass[b];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
      float t = 0.f;
      for (int w = 0; w < kPassThreads / 64; ++w) t += red[w];
      *db = t;
    }
  }
}

}  // namespace

RAG_API int rag_pass_grads(const float* zout, const float* dpass, float* dW, float* db, int B,
                           int P, hipStream_t stream) {
  if (B <= 0 || P <= 0) return -1;
  pass_grads_kernel<<<(P + kPassThreads - 1) / kPassThreads, kPassThreads, 0, stream>>>(
      zout, dpass, dW, db, B, P);
  return (int)hipGetLastError();
}

RAG_API int rag_policy_head_fwd(const void* H, const float* w, const float* b0,
                                const float* pbias, float* probs, const int64_t* labels,
                                const float* sweight, float* loss, float* dz, float* hit,
                                float* acc, int B, int S, int KP, int K, int mode, float gscale,
                                hipStream_t stream) {
  // acc (optional, float[2]): += sum of the batch's losses, += number of top-1 hits
  const size_t sm = (size_t)(((S * S + 4) & ~3) + KP) * sizeof(float);
  policy_head_fwd_kernel<<<B, kHeadFwdThreads, sm, stream>>>((const bf16*)H, w, b0, pbias, probs,
                                                          labels, sweight, loss, dz, hit, nullptr,
                                                          nullptr, nullptr, nullptr, acc, S, KP,
                                                          K, mode, gscale);
  return (int)hipGetLastError();
}

// As rag_policy_head_fwd, plus dzsum [B]: each board's sum of dz (the head bias gradient's
// per-board term, summed in a fixed order by rag_head_bwd_m).
RAG_API int rag_policy_head_fwd_s(const void* H, const float* w, const float* b0,
                                  const float* pbias, float* probs, const int64_t* labels,
                                  const float* sweight, float* loss, float* dz, float* hit,
                                  float* acc, float* dzsum, int B, int S, int KP, int K, int mode,
                                  float gscale, hipStream_t stream) {
  const size_t sm = (size_t)(((S * S + 4) & ~3) + KP) * sizeof(float);
  policy_head_fwd_kernel<<<B, kHeadFwdThreads, sm, stream>>>((const bf16*)H, w, b0, pbias, probs,
                                                          labels, sweight, loss, dz, hit, nullptr,
                                                          nullptr, nullptr, nullptr, acc, S, KP,
                                                          K, mode, gscale, dzsum);
  return (int)hipGetLastError();
}

// With a pass logit (pass_w [S*S], pass_b [1]): probs [B, S*S + 1], labels may be S*S (pass),
// zout [B, S*S] receives the position logits and dpass [B] dL/d(pass logit) for the PassLogit
// weight gradients (dW = dpass^T zout, db = sum dpass); dz already carries dpass * pass_w.
RAG_API int rag_policy_head_pass_fwd(const void* H, const float* w, const float* b0,
                                     const float* pbias, const float* pass_w,
                                     const float* pass_b, float* probs, const int64_t* labels,
                                     const float* sweight, float* loss, float* dz, float* hit,
                                     float* zout, float* dpass, float* acc, int B, int S, int KP,
                                     int K, int mode, float gscale, hipStream_t stream) {
  if (!pass_w || !pass_b) return -1;
  const size_t sm = (size_t)(((S * S + 4) & ~3) + KP) * sizeof(float);
  policy_head_fwd_kernel<<<B, kHeadFwdThreads, sm, stream>>>((const bf16*)H, w, b0, pbias, probs,
                                                          labels, sweight, loss, dz, hit, pass_w,
                                                          pass_b, zout, dpass, acc, S, KP, K,
                                                          mode, gscale);
  return (int)hipGetLastError();
}

// mloss / mhit / acc (optional): the head forward's per-board loss and top-1 hit (written with
// a null acc), summed into the running metrics acc[0..1] by one extra reduce block.
RAG_API int rag_head_bwd_m(const void* H, const float* w, const float* dz, void* dH, float* dw,
                           float* db0, float* dpbias, float* work, int B, int S, int KP, int K,
                           int relu_mask, const float* mloss, const float* mhit, float* acc,
                           const float* dzsum, hipStream_t stream) {
  // work: >= rag_head_bwd_workspace(B, S, KP) floats
  const int npix = B * S * S;
  int nblk = (npix + 47) / 48;
  if (nblk > kHeadBwdBlocks) nblk = kHeadBwdBlocks;
  const int ppb = (npix + nblk - 1) / nblk;
#define RAG_HB(C)                                                                             \
  case C:                                                                                     \
    head_bwd_kernel<C><<<nblk, kHeadThreads, 0, stream>>>((const bf16*)H, w, dz, (bf16*)dH,   \
                                                          work, db0, npix, ppb, S, K,         \
                                                          relu_mask);                         \
    break;
  switch (KP / 8) {
    RAG_HB(4) RAG_HB(8) RAG_HB(12) RAG_HB(16) RAG_HB(24) RAG_HB(32) RAG_HB(48) RAG_HB(64)
    default: return -1;
  }
#undef RAG_HB
  const int rblocks = (K + 63) / 64 + (S * S + 63) / 64;
  head_bwd_reduce_kernel<<<rblocks + 1, 1024, 0, stream>>>(
      work, dz, dw, db0, dpbias, nblk, B, S * S, KP, K, mloss, mhit, acc, dzsum);
  return (int)hipGetLastError();
}

RAG_API int rag_head_bwd(const void* H, const float* w, const float* dz, void* dH, float* dw,
                         float* db0, float* dpbias, float* work, int B, int S, int KP, int K,
                         int relu_mask, hipStream_t stream) {
  return rag_head_bwd_m(H, w, dz, dH, dw, db0, dpbias, work, B, S, KP, K, relu_mask, nullptr,
                        nullptr, nullptr, nullptr, stream);
}

RAG_API size_t rag_head_bwd_workspace(int B, int S, int KP) {
  const int npix = B * S * S;
  int nblk = (npix + 47) / 48;
  if (nblk > kHeadBwdBlocks) nblk = kHeadBwdBlocks;
  return (size_t)nblk * KP;
}

RAG_API int rag_head_linear(const void* H, const float* w, const float* b0, float* z, int B,
                            int S, int KP, int K, hipStream_t stream) {
  const int total = B * S * S;
  int blocks = (int)(((size_t)total * 8 + kHeadThreads - 1) / kHeadThreads);  // 8 lanes / pixel
  blocks = blocks < 8192 ? blocks : 8192;
  const int nm = K % 8 == 0 ? (K + 63) / 64 : 0;
#define RAG_HL(NM) \
  head_linear_kernel<NM><<<blocks, kHeadThreads, 0, stream>>>((const bf16*)H, w, b0, z, B, S, KP, K)
  if (nm == 1) RAG_HL(1);
  else if (nm == 2) RAG_HL(2);
  else if (nm == 3) RAG_HL(3);
  else if (nm == 4) RAG_HL(4);
  else RAG_HL(0);
#undef RAG_HL
  return (int)hipGetLastError();
}

RAG_API size_t rag_value_mlp_workspace(int B, int H) {
  return (size_t)B * ((H + kMlpCols - 1) / kMlpCols);
}

RAG_API int rag_value_mlp_fwd(const float* z, const float* W1, const float* b1, const float* W2,
                              const float* b2, float* out, float* work, float* hout, int B,
                              int P, int H, int act, hipStream_t stream) {
  // work: >= rag_value_mlp_workspace(B, H) floats
  if (B <= 0) return 0;
  static_assert(kMlpRows <= kMlpWaves, "one wave per board in the epilogue");
  const size_t sm = ((size_t)kMlpRows * P + kMlpWaves * kMlpRows * 64) * sizeof(float);
  if (sm > 64 * 1024) return -1;
  const int ntile = (H + kMlpCols - 1) / kMlpCols;
  const int nblk = (B + kMlpRows - 1) / kMlpRows * ntile;
  value_mlp_part_kernel<<<nblk, 64 * kMlpWaves, sm, stream>>>(z, W1, b1, W2, work, hout, B, P, H,
                                                              act);
  // out == null (training): the column partials in `work` feed rag_value_mlp_bwd instead
  if (out) value_mlp_out_kernel<<<(B + 255) / 256, 256, 0, stream>>>(work, b2, out, B, ntile);
  return (int)hipGetLastError();
}

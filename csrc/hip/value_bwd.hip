// Value-net MLP head, training direction (SURVEY C11/C12 value head: Dense(S*S -> H) + act,
// Dense(H -> 1) + tanh, MSE loss; reference AlphaGo/models/value.py:43-93 builds the Keras graph).
//
// The forward pass is value_mlp_part_kernel (head.hip) with `hout` = the pre-activation
// h = z W1 + b1 and `part` = the per-64-column partial sums of act(h) . W2. This file turns them
// into every gradient of the head in two launches, all fp32:
//   1. value_tail_bwd_kernel   one block per board: v = tanh(b2 + sum(part)), the (optionally
//                              sample-weighted) squared error, ds = dL/d(pre-tanh),
//                              dh = ds * W2 * act'(h)                       -> dh [B, H], ds [B]
//   2. value_grads_kernel      one grid with three independent parts:
//                              dW1 [P, H] = z^T dh     (M = P, N = H, K = B)
//                              dz  [B, P] = dh W1^T    (M = B, N = P, K = H)
//                              column sums db1 = sum_b dh, dW2 = sum_b ds * act(h),
//                              db2 = sum_b ds
// Replaces ~15 library/elementwise launches of the autograd tail (fused.py ValuePlan.fwd_bwd).
//
// Loss (Keras 'mse' with sample weights, quirk-compatible with the generic executor):
//   L = mean_b( (v_b - y_b)^2 * w_b ),  w_b = sw_b / mean_b(sw_b != 0)   (w_b = 1 without sw)
#include "common.h"

namespace rag {
namespace {

constexpr int kTailThreads = 256;

__device__ __forceinline__ float act_f(float h, int act) {
  if (act == 1) return h > 0.f ? h : 0.f;
  if (act == 2) return tanhf(h);
  return h;
}

__device__ __forceinline__ float act_grad(float h, int act) {
  if (act == 1) return h > 0.f ? 1.f : 0.f;
  if (act == 2) {
    const float t = tanhf(h);
    return 1.f - t * t;
  }
  return 1.f;
}

__device__ __forceinline__ float block_sum(float v, float* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();  // red may still be read by a previous call
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float s = 0.f;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w];
  return s;
}

__global__ void __launch_bounds__(kTailThreads)
value_tail_bwd_kernel(const float* __restrict__ part, int ntile, const float* __restrict__ hpre,
                      const float* __restrict__ W2, const float* __restrict__ b2,
                      const float* __restrict__ y, const float* __restrict__ sw,
                      float* __restrict__ dh, float* __restrict__ ds_out,
                      float* __restrict__ loss, float* __restrict__ vout, int B, int H, int act) {
  __shared__ float red[kTailThreads / 64];
  const int b = blockIdx.x;
  float wb = 1.f;
  if (sw) {  // w_b = sw_b / fraction of non-zero sample weights
    float cnt = 0.f;
    for (int i = threadIdx.x; i < B; i += kTailThreads) cnt += sw[i] != 0.f ? 1.f : 0.f;
    cnt = block_sum(cnt, red);
    const float frac = cnt / (float)B;
    wb = sw[b] / (frac > 1e-12f ? frac : 1e-12f);
  }
  float s = *b2;
  for (int t = 0; t < ntile; ++t) s += part[(size_t)b * ntile + t];
  const float v = tanhf(s);
  const float diff = v - y[b];
  const float invB = 1.f / (float)B;
  const float ds = 2.f * diff * wb * invB * (1.f - v * v);
  for (int j = threadIdx.x; j < H; j += kTailThreads) {
    const float h = hpre[(size_t)b * H + j];
    dh[(size_t)b * H + j] = ds * W2[j] * act_grad(h, act);
  }
  if (threadIdx.x == 0) {
    ds_out[b] = ds;
    loss[b] = diff * diff * wb * invB;
    if (vout) vout[b] = v;
  }
}

// ---- one launch for every batch reduction of the head -------------------------------------
// Blocks [0, g1): tiles of dW1 = z^T dh; [g1, g1 + g2): tiles of dz = dh W1^T;
// the last ncol blocks: column sums db1 = sum_b dh, dW2 = sum_b ds act(h), db2 = sum_b ds.
// The pieces are independent and each is latency-bound at this size (M, N ~ 256..361,
// K = B or H ~ 256), so one grid overlaps their memory round trips: three launches measured
// 11.6 + 11.6 + 4.5 us.
//
// GEMM tile: C[m, n] = sum_k A(m, k) B(k, n) with general element strides (fp32), 32 x 32
// outputs per block, 256 threads each owning a 2 x 2 sub-tile strided by 16 (a wave reads 4
// broadcast A values and 16 consecutive B values per k: conflict-free). K is staged 128 deep;
// the next chunk's 32 loads are issued into registers before the current chunk is multiplied.
// Loads are unconditional from clamped addresses and masked after (a guarded load compiles to a
// branch + wait per element and serialises them). Staging walks the unit-stride axis fastest so
// both operand layouts load coalesced.
constexpr int kGT = 32, kGK = 128;
constexpr int kPer = kGT * kGK / 256;  // 16 elements of each operand per thread and chunk

struct Gemm {
  const float* A;
  long sam, sak;
  const float* B;
  long sbk, sbn;
  float* C;
  long ldc;
  int M, N, K, tiles_n;
};

struct ColSum {
  const float* hpre;
  const float* dh;
  const float* ds;
  float *db1, *dW2, *db2;
  int B, H, act;
};

__device__ __forceinline__ void gemm_load(const Gemm& g, int m0, int n0, int k0, float* av,
                                          float* bv) {
  const int tid = threadIdx.x;
  const bool a_mfast = g.sam == 1, b_nfast = g.sbn == 1;
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int e = tid + 256 * i;  // 0 .. 4095 = 32 x 128
    const int am = a_mfast ? (e & 31) : (e >> 7), ak = a_mfast ? (e >> 5) : (e & 127);
    const int bn = b_nfast ? (e & 31) : (e >> 7), bk = b_nfast ? (e >> 5) : (e & 127);
    const int gm = m0 + am, gk = k0 + ak, gn = n0 + bn, gk2 = k0 + bk;
    const bool va = gm < g.M && gk < g.K, vb = gn < g.N && gk2 < g.K;
    const float a = g.A[va ? gm * g.sam + gk * g.sak : 0];
    const float b = g.B[vb ? gk2 * g.sbk + gn * g.sbn : 0];
    av[i] = va ? a : 0.f;
    bv[i] = vb ? b : 0.f;
  }
}

__device__ void gemm_tile(const Gemm& g, int tile, float (*As)[kGT + 1],
                          float (*Bs)[kGT + 1]) {
  const int tid = threadIdx.x;
  const int m0 = (tile / g.tiles_n) * kGT, n0 = (tile % g.tiles_n) * kGT;
  const int tm = tid >> 4, tn = tid & 15;
  const bool a_mfast = g.sam == 1, b_nfast = g.sbn == 1;
  float acc[2][2] = {{0.f, 0.f}, {0.f, 0.f}};
  float av[kPer], bv[kPer];
  gemm_load(g, m0, n0, 0, av, bv);
  for (int k0 = 0; k0 < g.K; k0 += kGK) {
    if (k0) __syncthreads();  // previous chunk fully consumed
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = tid + 256 * i;
      const int am = a_mfast ? (e & 31) : (e >> 7), ak = a_mfast ? (e >> 5) : (e & 127);
      const int bn = b_nfast ? (e & 31) : (e >> 7), bk = b_nfast ? (e >> 5) : (e & 127);
      As[ak][am] = av[i];
      Bs[bk][bn] = bv[i];
    }
    __syncthreads();
    if (k0 + kGK < g.K) gemm_load(g, m0, n0, k0 + kGK, av, bv);  // in flight during the FMAs
    const int kn = g.K - k0 < kGK ? g.K - k0 : kGK;
#pragma unroll 8
    for (int k = 0; k < kn; ++k) {
      const float a0 = As[k][tm], a1 = As[k][tm + 16];
      const float b0 = Bs[k][tn], b1 = Bs[k][tn + 16];
      acc[0][0] += a0 * b0;
      acc[0][1] += a0 * b1;
      acc[1][0] += a1 * b0;
      acc[1][1] += a1 * b1;
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int gm = m0 + tm + 16 * i;
    if (gm >= g.M) continue;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int gn = n0 + tn + 16 * j;
      if (gn < g.N) g.C[gm * g.ldc + gn] = acc[i][j];
    }
  }
}

// lanes = 64 columns, the 4 waves split the batch, 8 rows in flight per lane; block 0 of the
// column sums also reduces ds for db2
__device__ void colsum_block(const ColSum& c, int blk, float* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = blk * 64 + lane;
  float s1 = 0.f, s2 = 0.f;
  if (j < c.H) {
    int b = wave;
    for (; b + 28 < c.B; b += 32) {
      float d[8], h[8], g[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const size_t o = (size_t)(b + 4 * u) * c.H + j;
        d[u] = c.dh[o];
        h[u] = c.hpre[o];
        g[u] = c.ds[b + 4 * u];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        s1 += d[u];
        s2 += g[u] * act_f(h[u], c.act);
      }
    }
    for (; b < c.B; b += 4) {
      s1 += c.dh[(size_t)b * c.H + j];
      s2 += c.ds[b] * act_f(c.hpre[(size_t)b * c.H + j], c.act);
    }
  }
  float* r1 = red;            // [4][64]
  float* r2 = red + 4 * 64;   // [4][64]
  r1[wave * 64 + lane] = s1;
  r2[wave * 64 + lane] = s2;
  __syncthreads();
  if (wave == 0 && j < c.H) {
    c.db1[j] = r1[lane] + r1[64 + lane] + r1[128 + lane] + r1[192 + lane];
    c.dW2[j] = r2[lane] + r2[64 + lane] + r2[128 + lane] + r2[192 + lane];
  }
  if (blk == 0) {
    float t = 0.f;
    for (int b = threadIdx.x; b < c.B; b += 256) t += c.ds[b];
    t = block_sum(t, red + 8 * 64);
    if (threadIdx.x == 0) *c.db2 = t;
  }
}

__global__ void __launch_bounds__(256)
value_grads_kernel(Gemm g1, int nb1, Gemm g2, int nb2, ColSum cs) {
  __shared__ float As[kGK][kGT + 1];
  __shared__ float Bs[kGK][kGT + 1];
  const int blk = blockIdx.x;
  if (blk < nb1) {
    gemm_tile(g1, blk, As, Bs);
  } else if (blk < nb1 + nb2) {
    gemm_tile(g2, blk - nb1, As, Bs);
  } else {
    colsum_block(cs, blk - nb1 - nb2, &As[0][0]);  // 8 * 64 + 4 floats of scratch
  }
}

Gemm make_gemm(const float* A, long sam, long sak, const float* B, long sbk, long sbn, float* C,
               long ldc, int M, int N, int K, int* nblocks) {
  Gemm g{A, sam, sak, B, sbk, sbn, C, ldc, M, N, K, (N + kGT - 1) / kGT};
  *nblocks = C ? ((M + kGT - 1) / kGT) * g.tiles_n : 0;
  return g;
}

}  // namespace
}  // namespace rag

using namespace rag;

RAG_API size_t rag_value_mlp_bwd_workspace(int B, int H) { return (size_t)B * H + B; }

// part: the value_mlp forward workspace (B x ceil(H/64) partial sums), hpre: its `hout`.
// work >= rag_value_mlp_bwd_workspace(B, H) floats. dz may be null (no input gradient).
RAG_API int rag_value_mlp_bwd(const float* z, const float* W1, const float* W2, const float* b2,
                              const float* hpre, const float* part, const float* y,
                              const float* sw, float* work, float* loss, float* vout, float* dW1,
                              float* db1, float* dW2, float* db2, float* dz, int B, int P, int H,
                              int act, hipStream_t stream) {
  if (B <= 0) return 0;
  if (P <= 0 || H <= 0 || act < 0 || act > 2) return -1;
  float* dh = work;
  float* ds = work + (size_t)B * H;
  const int ntile = (H + 63) / 64;
  value_tail_bwd_kernel<<<B, kTailThreads, 0, stream>>>(part, ntile, hpre, W2, b2, y, sw, dh, ds,
                                                        loss, vout, B, H, act);
  int nb1 = 0, nb2 = 0;
  // dW1[p, j] = sum_b z[b, p] dh[b, j]
  const Gemm g1 = make_gemm(z, 1, P, dh, H, 1, dW1, H, P, H, B, &nb1);
  // dz[b, p] = sum_j dh[b, j] W1[p, j]
  const Gemm g2 = make_gemm(dh, H, 1, W1, 1, H, dz, P, B, P, H, &nb2);
  const ColSum cs{hpre, dh, ds, db1, dW2, db2, B, H, act};
  const int ncol = (H + 63) / 64;
  value_grads_kernel<<<nb1 + nb2 + ncol, 256, 0, stream>>>(g1, nb1, g2, nb2, cs);
  return (int)hipGetLastError();
}

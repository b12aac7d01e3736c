// Column BatchNorm + ReLU for the residual policy network (ResnetPolicy, reference
// AlphaGo/models/policy.py:211-244; Keras-1 learning phase nn_util.py:48-54).
//
// The reference applies Keras-1 BatchNormalization with its default axis=-1 to 'th' (B, C, H, W)
// tensors, so there is ONE statistic per board COLUMN w (S of them), reduced over (b, c, h). We
// keep that for checkpoint parity. On the padded channels-last layout [B][S+2H][S+2H][CP] the
// interior of one board row (b, h) is a contiguous run of S*CP bf16, and a 16-byte vector p of it
// covers column w = p / (CP/8): each thread owns fixed vectors of a row and walks rows, so its
// running sums always belong to the same columns (no atomics, deterministic).
//
//   rag_bn_train_fwd   batch statistics -> mean/rstd, the affine (scale, shift) of the fused
//                      BN+ReLU apply, and the running-average update (momentum, Keras-1 style)
//   rag_bn_infer_coef  (scale, shift) from the running statistics (inference learning phase)
//   rag_bn_bwd_coef    dgamma/dbeta and the per-column coefficients of dL/dx
//   rag_bn_apply       out = act(c0[w]*x + c1[w]*dy + c2[w] + res) over the interior, zero padded
//                      channels: forward BN+ReLU (c1 = 0), the final ReLU (no coefficients) and
//                      the BN backward with the residual gradient added (act = identity)
// All are HBM-bound streaming kernels (one or two reads + one write of a 29 MB activation at
// B=256, K=128); the conv epilogue does the residual sum of the forward (conv.hip `res`).
#include "common.h"

using namespace rag;

namespace {

constexpr int kT = 256;
constexpr int kKV = 4;  // vectors per thread per row: S*CP/8 <= 1024

__device__ __forceinline__ void load8(const bf16* p, float (&v)[8]) {
  const bf16x8 x = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = (float)x[e];
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Column finish from the two column sums (s0, s1). MODE 0: training forward, 1: backward,
// 2: inference (no sums).
struct BNArgs {
  double N;
  float eps, momentum;
  const float* gamma;
  const float* beta;
  float* rmean;
  float* rvar;
  float* stats;
  float* coef;
  float* dgamma;
  float* dbeta;
};

template <int MODE>
__device__ void bn_finish_col(const BNArgs& a, int S, int w, double s0, double s1) {
  const float ga = a.gamma ? a.gamma[w] : 1.f;
  if (MODE == 0) {
    const double mean = s0 / a.N;
    const double var = fmax(s1 / a.N - mean * mean, 0.0);
    const float rstd = (float)(1.0 / sqrt(var + (double)a.eps));
    a.stats[w] = (float)mean;
    a.stats[S + w] = rstd;
    a.coef[w] = ga * rstd;                                                     // x
    a.coef[S + w] = 0.f;                                                       // dy
    a.coef[2 * S + w] = (a.beta ? a.beta[w] : 0.f) - (float)mean * ga * rstd;  // const
    if (a.rmean) {
      a.rmean[w] = a.momentum * a.rmean[w] + (1.f - a.momentum) * (float)mean;
      a.rvar[w] = a.momentum * a.rvar[w] + (1.f - a.momentum) * (float)var;
    }
  } else if (MODE == 2) {
    const float rstd = 1.f / sqrtf(a.rvar[w] + a.eps);
    a.coef[w] = ga * rstd;
    a.coef[S + w] = 0.f;
    a.coef[2 * S + w] = (a.beta ? a.beta[w] : 0.f) - a.rmean[w] * ga * rstd;
  } else {
    // dx = ga*rstd*dy - k1*(dbeta + xhat*dgamma),  k1 = ga*rstd/N,  xhat = (x-mean)*rstd
    const float mean = a.stats[w], rstd = a.stats[S + w];
    const float db = (float)s0, dg = (float)(s1 * rstd);
    if (a.dgamma) a.dgamma[w] = dg;
    if (a.dbeta) a.dbeta[w] = db;
    const float k1 = (float)(ga * rstd / a.N);
    const float cx = -k1 * dg * rstd;
    a.coef[w] = cx;
    a.coef[S + w] = ga * rstd;
    a.coef[2 * S + w] = -k1 * db - cx * mean;
  }
}

// MODE 0: per-column (sum x, sum x^2); MODE 1: (sum dy, sum dy*(x-mean)).
// (Folding the finalize into the last block to finish -- agent-scope release fence + completion
// counter -- measured 95 us per launch instead of 7-12 us: every block's fence writes back its
// XCD's L2. Two launches it is.)
template <int MODE>
__global__ void __launch_bounds__(kT) bn_reduce_kernel(const bf16* __restrict__ X, int hx,
                                                        const bf16* __restrict__ DY, int hd,
                                                        const float* __restrict__ stats,
                                                        float* __restrict__ part, int R, int S,
                                                        int CP, int rows_per_blk) {
  __shared__ float red[2][kT * kKV];
  const int t = threadIdx.x;
  const int CPV = CP / 8;
  const int V = S * CPV;
  const int WX = S + 2 * hx, WD = S + 2 * hd;
  float a0[kKV], a1[kKV], mu[kKV];
#pragma unroll
  for (int k = 0; k < kKV; ++k) {
    a0[k] = 0.f;
    a1[k] = 0.f;
    const int p = t + kT * k;
    mu[k] = (MODE == 1 && p < V) ? stats[p / CPV] : 0.f;
  }
  const int r0 = blockIdx.x * rows_per_blk;
  const int r1 = min(R, r0 + rows_per_blk);
  for (int r = r0; r < r1; ++r) {
    const int b = r / S, h = r - (r / S) * S;
    const bf16* xrow = X + ((size_t)(b * WX + h + hx) * WX + hx) * CP;
    const bf16* drow = MODE == 1 ? DY + ((size_t)(b * WD + h + hd) * WD + hd) * CP : nullptr;
#pragma unroll
    for (int k = 0; k < kKV; ++k) {
      const int p = t + kT * k;
      if (p >= V) continue;
      float x[8];
      load8(xrow + (size_t)p * 8, x);
      if (MODE == 0) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          a0[k] += x[e];
          a1[k] = fmaf(x[e], x[e], a1[k]);
        }
      } else {
        float d[8];
        load8(drow + (size_t)p * 8, d);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          a0[k] += d[e];
          a1[k] = fmaf(d[e], x[e] - mu[k], a1[k]);
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < kKV; ++k) {
    red[0][t + kT * k] = a0[k];
    red[1][t + kT * k] = a1[k];
  }
  __syncthreads();
  if (t < 2 * S) {
    const int w = t >> 1, q = t & 1;
    float s = 0.f;
    for (int p = w * CPV; p < (w + 1) * CPV; ++p) s += red[q][p];
    part[((size_t)blockIdx.x * 2 + q) * S + w] = s;
  }
}

// One block per column w: 256 threads stride over the nblk partials (double accumulation),
// wave shuffles + LDS combine them, thread 0 finishes the column.
template <int MODE>
__global__ void __launch_bounds__(kT) bn_finalize_kernel(const float* __restrict__ part, int nblk,
                                                          int S, BNArgs a) {
  __shared__ double red[2][kT / 64];
  const int w = blockIdx.x;
  const int t = threadIdx.x, g = t >> 6, lane = t & 63;
  double s0 = 0.0, s1 = 0.0;
  for (int i = t; i < nblk; i += kT) {
    s0 += part[((size_t)i * 2) * S + w];
    s1 += part[((size_t)i * 2 + 1) * S + w];
  }
  s0 = wave_sum_d(s0);
  s1 = wave_sum_d(s1);
  if (lane == 0) {
    red[0][g] = s0;
    red[1][g] = s1;
  }
  __syncthreads();
  if (t) return;
  s0 = red[0][0] + red[0][1] + red[0][2] + red[0][3];
  s1 = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  bn_finish_col<MODE>(a, S, w, s0, s1);
}

// Inference coefficients from the running statistics: one thread per column.
__global__ void bn_infer_kernel(BNArgs a, int S) {
  const int w = threadIdx.x;
  if (w < S) bn_finish_col<2>(a, S, w, 0.0, 0.0);
}

// out = act(c0[w]*x + c1[w]*dy + c2[w] + res) over the interior, grid-stride (coef may be LDS)
__device__ __forceinline__ void bn_apply_body(const bf16* __restrict__ X, int hx,
                                              const bf16* __restrict__ DY, int hd, const bf16* RES,
                                              int hr, bf16* O, int ho, const float* coef, int relu,
                                              int B, int S, int C, int CP) {
  const int CPV = CP / 8;
  const int total = B * S * S * CPV;  // < 2^31 (checked by the launcher)
  const int WX = S + 2 * hx, WD = S + 2 * hd, WR = S + 2 * hr, WO = S + 2 * ho;
  for (int i = blockIdx.x * kT + threadIdx.x; i < total; i += gridDim.x * kT) {
    const int cv = i % CPV;
    const int pix = i / CPV;
    const int w = pix % S;
    const int bh = pix / S;
    const int h = bh % S;
    const int b = bh / S;
    const int c0 = cv * 8;
    bf16x8 o;
    if (c0 >= C) {
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (bf16)0.f;
    } else {
      float x[8];
      load8(X + ((size_t)(b * WX + h + hx) * WX + w + hx) * CP + c0, x);
      const float cx = coef ? coef[w] : 1.f;
      const float cd = coef ? coef[S + w] : 0.f;
      const float cc = coef ? coef[2 * S + w] : 0.f;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaf(cx, x[e], cc);
      if (DY) {
        float d[8];
        load8(DY + ((size_t)(b * WD + h + hd) * WD + w + hd) * CP + c0, d);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaf(cd, d[e], v[e]);
      }
      if (RES) {
        float r[8];
        load8(RES + ((size_t)(b * WR + h + hr) * WR + w + hr) * CP + c0, r);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += r[e];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float y = relu ? fmaxf(v[e], 0.f) : v[e];
        o[e] = (bf16)((c0 + e) < C ? y : 0.f);
      }
    }
    *reinterpret_cast<bf16x8*>(O + ((size_t)(b * WO + h + ho) * WO + w + ho) * CP + c0) = o;
  }
}

__global__ void __launch_bounds__(kT) bn_apply_kernel(
    const bf16* __restrict__ X, int hx, const bf16* __restrict__ DY, int hd,
    const bf16* RES, int hr, bf16* O, int ho,  // RES may alias O (in-place skip gradient)
    const float* __restrict__ coef, int relu, int B, int S, int C, int CP) {
  bn_apply_body(X, hx, DY, hd, RES, hr, O, ho, coef, relu, B, S, C, CP);
}

// The backward BN apply with its finalize folded in: every block sums the nblk backward partials
// [nblk][2][S] (the dgrad epilogues' (sum dU, sum dU (x - mean))) itself -- 8 slices of 32
// column lanes, double, the same order in every block, so all blocks derive bit-identical
// coefficients -- into LDS; block 0 also writes dgamma / dbeta. Saves the finalize launch per BN
// (19 per ResnetPolicy step); the grid is capped so the partial reads stay a few MB of L2.
constexpr int kApplyPartBlocks = 1024;
__global__ void __launch_bounds__(kT) bn_apply_part_kernel(
    const float* __restrict__ part, int nblk, BNArgs a, const bf16* __restrict__ X, int hx,
    const bf16* __restrict__ DY, int hd, const bf16* RES, int hr, bf16* O, int ho, int B, int S,
    int C, int CP) {
  __shared__ double red[2][8][32];
  __shared__ float cf[3 * 64];
  const int t = threadIdx.x, w = t & 31, sl = t >> 5;
  double s0 = 0.0, s1 = 0.0;
  if (w < S) {
#pragma unroll 4
    for (int i = sl; i < nblk; i += 8) {
      s0 += part[((size_t)i * 2) * S + w];
      s1 += part[((size_t)i * 2 + 1) * S + w];
    }
  }
  red[0][sl][w] = s0;
  red[1][sl][w] = s1;
  __syncthreads();
  if (t < S) {
    double a0 = 0.0, a1 = 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      a0 += red[0][k][t];
      a1 += red[1][k][t];
    }
    BNArgs b = a;
    b.coef = cf;
    if (blockIdx.x != 0) {
      b.dgamma = nullptr;
      b.dbeta = nullptr;
    }
    bn_finish_col<1>(b, S, t, a0, a1);
  }
  __syncthreads();
  bn_apply_body(X, hx, DY, hd, RES, hr, O, ho, cf, 0, B, S, C, CP);
}

int reduce_blocks(int R) { return R < 1024 ? R : 1024; }

}  // namespace

// Floats of workspace rag_bn_train_fwd / rag_bn_bwd_coef need (per-block partials).
RAG_API int rag_bn_workspace(int B, int S) { return reduce_blocks(B * S) * 2 * S; }

RAG_API int rag_bn_train_fwd(const void* X, int hx, int B, int S, int C, int CP,
                             const float* gamma, const float* beta, float* rmean, float* rvar,
                             float eps, float momentum, float* stats, float* coef, float* work,
                             hipStream_t stream) {
  if (CP % 8 || S * CP / 8 > kT * kKV || S > 64 || C > CP) return -1;
  const int R = B * S, nblk = reduce_blocks(R);
  const int rpb = (R + nblk - 1) / nblk;
  const BNArgs a{(double)B * S * C, eps, momentum, gamma, beta, rmean, rvar, stats, coef,
                 nullptr, nullptr};
  bn_reduce_kernel<0><<<nblk, kT, 0, stream>>>((const bf16*)X, hx, nullptr, 0, nullptr,
                                               work, R, S, CP, rpb);
  bn_finalize_kernel<0><<<S, kT, 0, stream>>>(work, nblk, S, a);
  return (int)hipGetLastError();
}

RAG_API int rag_bn_infer_coef(const float* gamma, const float* beta, float* rmean, float* rvar,
                              float eps, int S, float* coef, hipStream_t stream) {
  if (S > 64) return -1;
  const BNArgs a{1.0, eps, 0.f, gamma, beta, rmean, rvar, nullptr, coef, nullptr, nullptr};
  bn_infer_kernel<<<1, 64, 0, stream>>>(a, S);
  return (int)hipGetLastError();
}

RAG_API int rag_bn_bwd_coef(const void* X, int hx, const void* DY, int hd, int B, int S, int C,
                            int CP, const float* gamma, const float* stats, float* dgamma,
                            float* dbeta, float* coef, float* work, hipStream_t stream) {
  if (CP % 8 || S * CP / 8 > kT * kKV || S > 64 || C > CP) return -1;
  const int R = B * S, nblk = reduce_blocks(R);
  const int rpb = (R + nblk - 1) / nblk;
  const BNArgs a{(double)B * S * C, 0.f, 0.f, gamma, nullptr, nullptr, nullptr, (float*)stats,
                 coef, dgamma, dbeta};
  bn_reduce_kernel<1><<<nblk, kT, 0, stream>>>((const bf16*)X, hx, (const bf16*)DY, hd, stats,
                                               work, R, S, CP, rpb);
  bn_finalize_kernel<1><<<S, kT, 0, stream>>>(work, nblk, S, a);
  return (int)hipGetLastError();
}

// Finalize from per-block partials [nblk][2][S] that another kernel produced (the BN-fused conv
// epilogues, conv_tap.hip `spart`): forward (sum x, sum x^2) -> stats / coef / running averages,
// backward (sum dy, sum dy (x - mean)) -> dgamma / dbeta / the dL/dx coefficients.
RAG_API int rag_bn_finalize_fwd(const float* part, int nblk, int B, int S, int C,
                                const float* gamma, const float* beta, float* rmean, float* rvar,
                                float eps, float momentum, float* stats, float* coef,
                                hipStream_t stream) {
  if (S > 64) return -1;
  const BNArgs a{(double)B * S * C, eps, momentum, gamma, beta, rmean, rvar, stats, coef,
                 nullptr, nullptr};
  bn_finalize_kernel<0><<<S, kT, 0, stream>>>(part, nblk, S, a);
  return (int)hipGetLastError();
}

RAG_API int rag_bn_finalize_bwd(const float* part, int nblk, int B, int S, int C,
                                const float* gamma, const float* stats, float* dgamma,
                                float* dbeta, float* coef, hipStream_t stream) {
  if (S > 64) return -1;
  const BNArgs a{(double)B * S * C, 0.f, 0.f, gamma, nullptr, nullptr, nullptr, (float*)stats,
                 coef, dgamma, dbeta};
  bn_finalize_kernel<1><<<S, kT, 0, stream>>>(part, nblk, S, a);
  return (int)hipGetLastError();
}

RAG_API int rag_bn_apply(const void* X, int hx, const void* DY, int hd, const void* RES, int hr,
                         void* O, int ho, const float* coef, int relu, int B, int S, int C, int CP,
                         hipStream_t stream) {
  if (CP % 8 || C > CP || (size_t)B * S * S * (CP / 8) >= (1u << 31)) return -1;
  const size_t total = (size_t)B * S * S * (CP / 8);
  size_t nb = (total + kT - 1) / kT;
  if (nb > 8192) nb = 8192;
  bn_apply_kernel<<<(int)nb, kT, 0, stream>>>((const bf16*)X, hx, (const bf16*)DY, hd,
                                              (const bf16*)RES, hr, (bf16*)O, ho, coef, relu, B,
                                              S, C, CP);
  return (int)hipGetLastError();
}

// rag_bn_finalize_bwd + rag_bn_apply(dy, coef) in one launch: out = dL/dx (+ RES) of a BN whose
// backward statistics are the per-block partials `part` [nblk][2][S]; dgamma / dbeta as the
// finalize. S <= 32.
RAG_API int rag_bn_apply_bwd_part(const float* part, int nblk, const float* gamma,
                                  const float* stats, float* dgamma, float* dbeta, const void* X,
                                  int hx, const void* DY, int hd, const void* RES, int hr, void* O,
                                  int ho, int B, int S, int C, int CP, hipStream_t stream) {
  if (S > 32 || CP % 8 || C > CP || (size_t)B * S * S * (CP / 8) >= (1u << 31) || !DY)
    return -1;
  const BNArgs a{(double)B * S * C, 0.f, 0.f, gamma, nullptr, nullptr, nullptr, (float*)stats,
                 nullptr, dgamma, dbeta};
  const size_t total = (size_t)B * S * S * (CP / 8);
  size_t nb = (total + kT - 1) / kT;
  if (nb > kApplyPartBlocks) nb = kApplyPartBlocks;
  bn_apply_part_kernel<<<(int)nb, kT, 0, stream>>>(part, nblk, a, (const bf16*)X, hx,
                                                   (const bf16*)DY, hd, (const bf16*)RES, hr,
                                                   (bf16*)O, ho, B, S, C, CP);
  return (int)hipGetLastError();
}

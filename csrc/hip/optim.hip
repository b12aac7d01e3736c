// Fused optimizer kernels (K07) — Keras-1 SGD semantics (supervised_policy_trainer.py:249,
// reinforcement_policy_trainer.py:185): lr_t = lr / (1 + decay * iterations) is computed on the
// host; here   v = momentum * v - lr_t * (g + wd * p);  p += nesterov ? momentum * v - lr_t * g' : v
// over one flat fp32 parameter buffer (all layers, a single launch), vectorised 4-wide.
#include "common.h"

namespace {

__global__ void sgd_kernel(float* __restrict__ p, const float* __restrict__ g,
                           float* __restrict__ v, int64_t n, float lr, float momentum, float wd,
                           int nesterov) {
  const int64_t n4 = n / 4;
  float4* p4 = reinterpret_cast<float4*>(p);
  const float4* g4 = reinterpret_cast<const float4*>(g);
  float4* v4 = reinterpret_cast<float4*>(v);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    float4 pp = p4[i];
    float4 gg = g4[i];
    float* pe = reinterpret_cast<float*>(&pp);
    float* ge = reinterpret_cast<float*>(&gg);
    if (v) {
      float4 vv = v4[i];
      float* ve = reinterpret_cast<float*>(&vv);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float gk = ge[k] + wd * pe[k];
        ve[k] = momentum * ve[k] - lr * gk;
        pe[k] += nesterov ? momentum * ve[k] - lr * gk : ve[k];
      }
      v4[i] = vv;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) pe[k] -= lr * (ge[k] + wd * pe[k]);
    }
    p4[i] = pp;
  }
  // tail
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const int64_t i = n4 * 4 + threadIdx.x;
    const float gk = g[i] + wd * p[i];
    if (v) {
      v[i] = momentum * v[i] - lr * gk;
      p[i] += nesterov ? momentum * v[i] - lr * gk : v[i];
    } else {
      p[i] -= lr * gk;
    }
  }
}

}  // namespace

RAG_API int rag_sgd(float* p, const float* g, float* v, int64_t n, float lr, float momentum,
                    float wd, int nesterov, hipStream_t stream) {
  if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)v) & 15) return -1;
  int64_t blocks = (n / 4 + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  sgd_kernel<<<(int)blocks, 256, 0, stream>>>(p, g, v, n, lr, momentum, wd, nesterov);
  return (int)hipGetLastError();
}

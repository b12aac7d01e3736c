// Per-step SL batch preparation in one launch: for each of the B sampled rows a
// random dihedral transform (one of the trainer's allowed symmetries) and the transformed target
// index. Replaces the random draw, the symmetry lookup and the two label gathers (four small
// library kernels per step).
#include "common.h"

namespace {

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

// tf_out[i] = sym[h(seed, step, i) % nsym]; lab_out[i] = tf_table[tf_out[i]][labels[index[i]]]
__global__ void sl_batch_kernel(const int64_t* __restrict__ index,
                                const int64_t* __restrict__ labels,
                                const int64_t* __restrict__ tf_table, int P,
                                const int* __restrict__ sym, int nsym, uint32_t seed,
                                uint32_t step, int* __restrict__ tf_out,
                                int64_t* __restrict__ lab_out, int B) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  const uint32_t h = mix32(seed ^ mix32(step * 0x9E3779B9u + (uint32_t)i * 0x85EBCA6Bu + 1u));
  const int t = sym[h % (uint32_t)nsym];
  tf_out[i] = t;
  lab_out[i] = tf_table[(size_t)t * P + labels[index[i]]];
}

// The value-net step's batch: tf_out[i] as sl_batch, y_out[i] = values[index[i]] (the outcome
// is invariant under the board's symmetries).
__global__ void value_batch_kernel(const int64_t* __restrict__ index,
                                   const float* __restrict__ values,
                                   const int* __restrict__ sym, int nsym, uint32_t seed,
                                   uint32_t step, int* __restrict__ tf_out,
                                   float* __restrict__ y_out, int B) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  const uint32_t h = mix32(seed ^ mix32(step * 0x9E3779B9u + (uint32_t)i * 0x85EBCA6Bu + 1u));
  tf_out[i] = sym[h % (uint32_t)nsym];
  y_out[i] = values[index[i]];
}

}  // namespace

RAG_API int rag_value_batch(const int64_t* index, const float* values, const int* sym, int nsym,
                            unsigned seed, unsigned step, int* tf_out, float* y_out, int B,
                            hipStream_t stream) {
  if (B <= 0) return 0;
  if (nsym <= 0) return -1;
  value_batch_kernel<<<(B + 255) / 256, 256, 0, stream>>>(index, values, sym, nsym, seed, step,
                                                          tf_out, y_out, B);
  return (int)hipGetLastError();
}

RAG_API int rag_sl_batch(const int64_t* index, const int64_t* labels, const int64_t* tf_table,
                         int P, const int* sym, int nsym, unsigned seed, unsigned step,
                         int* tf_out, int64_t* lab_out, int B, hipStream_t stream) {
  if (B <= 0) return 0;
  if (nsym <= 0 || P <= 0) return -1;
  sl_batch_kernel<<<(B + 255) / 256, 256, 0, stream>>>(index, labels, tf_table, P, sym, nsym,
                                                       seed, step, tf_out, lab_out, B);
  return (int)hipGetLastError();
}

// Shared definitions for the gfx950 (CDNA4 / MI355X) kernels of RocAlphaGo-MI355X.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define RAG_API extern "C" __attribute__((visibility("default")))

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;

#define LDS_PTR(T) __attribute__((address_space(3))) T*

namespace rag {

__device__ __forceinline__ float bf2f(bf16 v) { return (float)v; }
__device__ __forceinline__ bf16 f2bf(float v) { return (bf16)v; }

// 16-byte global -> LDS direct copy (global_load_lds_dwordx4). LDS destination is
// wave-uniform `lds_base` + lane*16; the global source is per lane.
__device__ __forceinline__ void glds16(const void* gsrc, void* lds_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gsrc,
                                   (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Row swizzle for [row][32 x bf16] (64-byte) LDS tiles read as 16x16x32 MFMA fragments with
// ds_read_b128 (lane reads row lane&15, 16-byte chunk lane>>4). Swapping chunk bit 1 on rows
// with bit 3 set makes all four 16-lane ds_read_b128 groups conflict-free (derivation in
// docs/KERNELS.md). Involution: applied to the global source on staging and on the read.
__device__ __forceinline__ int swz64(int row) { return ((row >> 3) & 1) << 1; }

// Row swizzle (16-byte chunk XOR) for [row][CH x 16B] LDS tiles read with ds_read_tr16_b64 as
// 16x16x32 fragments: a 32-lane half reads rows {8g+q (+4)}, g,q in 0..3, 32 bytes each, so rows
// r and r+8 (and, for some row lengths, r+2) alias onto the same banks. The XOR makes the eight
// 32-byte windows of a half disjoint (conflict-free) for every row length used (derivation in
// docs/KERNELS.md); it only permutes even chunk pairs, so 32-byte windows stay contiguous.
template <int CH>
__device__ __forceinline__ int swz_tr(int r) {
  if constexpr (CH % 16 == 0) {
    return 2 * (r & 3) + 8 * ((r >> 3) & 1);
  } else if constexpr (CH % 8 == 0) {
    return 2 * ((r >> 1) & 1) + 4 * ((r >> 3) & 1);
  } else if constexpr (CH % 4 == 0) {
    return 2 * ((r >> 3) & 1);
  } else {
    return 0;
  }
}

// Transposed 16x16x32 fragment read (2 x ds_read_b64_tr_b16) as inline asm. Through the
// __builtin_amdgcn_ds_read_tr16_b64 builtin hipcc cannot tell these LDS reads from in-flight
// global_load_lds writes and drains them all (s_waitcnt vmcnt(0)) before the first read of every
// staging step (seen in wgrad_slab's .s), which serialises a multi-stage LDS ring. The caller
// retires the reads with lds_reads_done() before their MFMAs (guide §5.4 rule 18: the
// sched_barrier keeps hipcc from hoisting the MFMAs above the asm wait).
__device__ __forceinline__ uint32_t lds_addr(const bf16* p) {
  return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((LDS_PTR(const bf16))p));
}
__device__ __forceinline__ bf16x8 tr_frag(const bf16* p0, const bf16* p1) {
  bf16x4 lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(lds_addr(p0)));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hi) : "v"(lds_addr(p1)));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
__device__ __forceinline__ void lds_reads_done() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ int wave_id() {
  return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
}
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Bijective XCD-aware remap of a 1-D block index (guide T1): consecutive tiles land on one XCD.
__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
  const int q = nblk / 8, r = nblk % 8;
  const int xcd = bid % 8, idx = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// SGD folded into the weight packing (pack.h pack_trunk_block / wino_pack_block):
// a packing kernel that reads fp32 master w also reads its gradient g = w[goff] (the model's
// flat gradient buffer mirrors the parameter buffer), writes back w - lr (g + wd w) and packs
// the updated value; on = 0: plain packing.
struct SgdFold {
  long goff;
  float lr, wd;
  int on;
  // the update itself (sgd_kernel's arithmetic, so a fold is bit-exact against it)
  __device__ __forceinline__ float update(float v, float g) const { return v - lr * (g + wd * v); }
  __device__ __forceinline__ float step(float* w) const {
    const float v = *w;
    if (!on) return v;
    const float u = update(v, w[goff]);
    *w = u;
    return u;
  }
};

}  // namespace rag

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

using namespace rag;

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

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__global__ void __launch_bounds__(256, 2)
conv_tap_kernel(const bf16* __restrict__ X, const bf16* __restrict__ Wt,
                const float* __restrict__ bias, bf16* __restrict__ Y,
                const bf16* __restrict__ mask, const bf16* __restrict__ res, int M, int S,
                int WI, int shift, int WO, int HO, int CIN, int WROWS, int YC, int relu, int HM,
                long total_rows) {
  __shared__ __attribute__((aligned(16))) bf16 lds[kLds];
  const int lane = lane_id();
  const int w = wave_id();
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

  // epilogue (as conv_pipe): lane owns channels n..n+3 of pixel m for every (j, i) tile
#pragma unroll
  for (int i = 0; i < kMT; ++i) {
    const int m = m0 + wm * (16 * kMT) + i * 16 + frow;
    if (m >= M) continue;
    const int b = m / S2;
    const int rem = m - b * S2;
    const int pi = rem / S;
    const int pj = rem - pi * S;
    const size_t orow = (size_t)((b * WO + pi + HO) * WO + pj + HO) * YC;
    const int WMK = S + 2 * HM;
    const size_t mrow = (size_t)((b * WMK + pi + HM) * WMK + pj + HM) * YC;
#pragma unroll
    for (int j = 0; j < kNT; ++j) {
      const int n = n0 + wn * (16 * kNT) + j * 16 + fq * 4;
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

int g_tap_mode = -1;  // -1: read RAG_CONV_TAP on first use (default on)

// Worst-case slab extent of a kBM-pixel run (host check of the kernel's kSlabRows assumption).
int max_slab_rows(int S, int WI, int shift) {
  const int S2 = S * S;
  auto prow = [&](long m) {
    const long b = m / S2, rem = m - b * S2, i = rem / S, j = rem - i * S;
    return (b * WI + i + shift) * WI + j + shift;
  };
  long mx = 0;
  for (long m0 = 0; m0 < 4L * S2 + kBM; m0 += kBM)
    mx = std::max(mx, prow(m0 + kBM - 1) + 2 * WI + 2 - prow(m0) + 1);
  return (int)mx;
}

}  // namespace

RAG_API int rag_conv_tap_mode(int mode) {
  const int old = g_tap_mode;
  g_tap_mode = mode;
  return old;
}

// Returns true if the tap-slab kernel handled the launch: 3x3, 192-multiple output channels,
// input channels a multiple of 32, and every 192-pixel run's nine-tap slab fits kSlabRows.
bool rag_conv_tap_launch(const bf16* x, const bf16* w, const float* bias, bf16* y,
                         const bf16* mk, const bf16* res, int M, int S, int WI, int shift, int WO,
                         int HO, int CIN, int COUTP, int YC, int KS, int relu, int HM, long total_rows,
                         hipStream_t stream) {
  if (g_tap_mode < 0) {
    const char* e = getenv("RAG_CONV_TAP");
    g_tap_mode = e ? atoi(e) : 1;
  }
  if (!g_tap_mode || KS != 3 || COUTP % kBN || CIN % kBK || CIN < kBK) return false;
  static int cached_key = -1, cached_rows = 0;
  const int key = S * 4096 + WI * 8 + shift;
  if (key != cached_key) {
    cached_rows = max_slab_rows(S, WI, shift);
    cached_key = key;
  }
  if (cached_rows > kSlabRows) return false;
  const int nblk_m = (M + kBM - 1) / kBM;
  dim3 grid(nblk_m * (COUTP / kBN));
  conv_tap_kernel<<<grid, 256, 0, stream>>>(x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN,
                                            COUTP, YC, relu, HM, total_rows);
  return true;
}

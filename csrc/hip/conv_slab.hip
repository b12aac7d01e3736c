// Slab-staged implicit-GEMM 3x3 convolution for the 192-filter 19x19 trunk (forward and dgrad).
//
// conv_pipe (conv_fwd.hip) stages a fresh 192-pixel x 32-channel A tile for every (tap, chunk)
// step, so each pixel's channels are fetched from L2 nine times per layer: ~42 B/clk/CU of staging
// against the ~30-35 B/clk/CU an L2 gather sustains — the kernel is L2-bound, not MFMA-bound.
//
// Here one workgroup owns one whole board and all 192 output channels:
//   * pixels are "virtual rows" of the padded plane: output (i, j) is row u = i*WI + j
//     (WI = S + 2), and tap (ky, kx) reads padded input row u + ky*WI + kx — a constant shift, so
//     one slab of input rows per 32-channel chunk serves all nine taps;
//   * the slab (576 rows x 32 ch, double-buffered) is staged once per chunk; only the 192 x 32
//     weight tile changes per step (3-slot ring). Staging drops to ~13 B/clk/CU;
//   * 12 waves as 2 (M) x 6 (N): each wave owns 208 virtual rows (13 fragments) x 32 channels and
//     issues 26 MFMA 16x16x32 per step. 416 virtual rows cover the 397 needed (361 real pixels);
//   * fragment start rows are arbitrary (row shift ky*WI + kx), so the 64-byte rows are swizzled
//     on row bit 2 (chunk bit 1): for any start row the 16-lane ds_read_b128 groups read rows
//     {r..r+3, r+12..r+15} with one chunk and {r+4..r+11} with the other, and adding 4 or 12 flips
//     bit 2, so every group covers all 16 (row mod 4, chunk) bank slots — conflict-free;
//   * counted vmcnt waits + raw s_barrier as in conv_pipe (every wave issues the same loads).
// LDS: 2 x 36 KB slabs + 3 x 12 KB weight tiles = 108 KB -> one 768-thread block per CU.
#include "common.h"

using namespace rag;

namespace {

constexpr int kBK = 32;
constexpr int kN = 192;        // output channels per block (all of them)
constexpr int kMF = 13;        // 16-row fragments per wave along M
constexpr int kWM = 16 * kMF;  // 208 virtual rows per wave
constexpr int kBM = 2 * kWM;   // 416 virtual rows per block
constexpr int kNF = 2;         // 16-channel fragments per wave along N
constexpr int kWaves = 12;
constexpr int kSlabRows = 576;  // 36 glds x 16 rows: 3 per wave; >= 416 + 2*WI + 2
constexpr int kSlab = kSlabRows * kBK;
constexpr int kBTile = kN * kBK;
constexpr int kLds = 2 * kSlab + 3 * kBTile;

__device__ __forceinline__ int swz4(int row) { return ((row >> 2) & 1) << 1; }

__device__ __forceinline__ void wait_vm(int n) {
  if (n >= 4)
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (n == 3)
    asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if (n >= 1)
    asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__global__ void __launch_bounds__(768)
conv_slab_kernel(const bf16* __restrict__ X, const bf16* __restrict__ Wt,
                 const float* __restrict__ bias, bf16* __restrict__ Y,
                 const bf16* __restrict__ mask, const bf16* __restrict__ res, int S, int CIN,
                 int WROWS, int WO, int HO, int YC, int relu, int HM, long total_rows) {
  __shared__ __attribute__((aligned(16))) bf16 lds[kLds];
  const int lane = lane_id();
  const int w = wave_id();
  const int wm = w / 6, wn = w - (w / 6) * 6;
  const int b = blockIdx.x;
  const int WI = S + 2;
  const long row0 = (long)b * WI * WI;

  // staging sources: slab rows (w*3 + k)*16 + lane/4, weight rows w*16 + lane/4
  const bf16* asrc[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int r = (w * 3 + k) * 16 + (lane >> 2);
    long g = row0 + r;
    g = g < total_rows ? g : total_rows - 1;
    asrc[k] = X + g * CIN + (((lane & 3) ^ swz4(r)) * 8);
  }
  const int brow = w * 16 + (lane >> 2);
  const bf16* bsrc = Wt + (long)brow * CIN + (((lane & 3) ^ swz4(brow)) * 8);

  const int cchunks = CIN / kBK;
  const int nsteps = 9 * cchunks;

  auto stage_a = [&](int q) {
    bf16* dst = lds + (q & 1) * kSlab;
#pragma unroll
    for (int k = 0; k < 3; ++k) glds16(asrc[k] + q * kBK, dst + (w * 3 + k) * 16 * kBK);
  };
  auto stage_b = [&](int s) {
    const int q = s / 9, t = s - q * 9;
    bf16* dst = lds + 2 * kSlab + (s % 3) * kBTile;
    glds16(bsrc + (long)t * WROWS * CIN + q * kBK, dst + w * 16 * kBK);
  };

  f32x4 acc[kNF][kMF];
#pragma unroll
  for (int g = 0; g < kNF; ++g)
#pragma unroll
    for (int f = 0; f < kMF; ++f) acc[g][f] = f32x4{0.f, 0.f, 0.f, 0.f};

  stage_a(0);
  stage_b(0);
  if (nsteps > 1) stage_b(1);

  const int frow = lane & 15;
  const int fq = lane >> 4;
  int boffs[kNF];
#pragma unroll
  for (int g = 0; g < kNF; ++g) {
    const int row = wn * 32 + g * 16 + frow;
    boffs[g] = row * kBK + ((fq ^ swz4(row)) * 8);
  }
  const int R0 = wm * kWM + frow;

  for (int s = 0; s < nsteps; ++s) {
    const int q = s / 9, t = s - q * 9;
    // loads issued after stage_b(s) that may stay in flight: stage_b(s+1) and a slab issued
    // at step s-1 or s-2 (the slab of chunk c+1 is issued at step 9c, after stage_b(9c+2))
    int young = s + 1 < nsteps ? 1 : 0;
    if (s >= 2 && (s - 2) % 9 == 0 && (s - 2) / 9 + 1 < cchunks) young += 3;
    if (s >= 1 && (s - 1) % 9 == 0 && (s - 1) / 9 + 1 < cchunks) young += 3;
    wait_vm(young);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (s + 2 < nsteps) stage_b(s + 2);
    if (t == 0 && q + 1 < cchunks) stage_a(q + 1);

    const int ky = t / 3, kx = t - ky * 3;
    const bf16* slab = lds + (q & 1) * kSlab;
    const bf16* bt = lds + 2 * kSlab + (s % 3) * kBTile;
    bf16x8 wb[kNF];
#pragma unroll
    for (int g = 0; g < kNF; ++g) wb[g] = *reinterpret_cast<const bf16x8*>(bt + boffs[g]);
    const int r0 = R0 + ky * WI + kx;
    const bf16* abase = slab + r0 * kBK + ((fq ^ swz4(r0)) * 8);  // swz4(r0 + 16f) == swz4(r0)
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int f = 0; f < kMF; ++f) {
      const bf16x8 xa = *reinterpret_cast<const bf16x8*>(abase + f * 16 * kBK);
#pragma unroll
      for (int g = 0; g < kNF; ++g) acc[g][f] = mfma16(wb[g], xa, acc[g][f]);
    }
    __builtin_amdgcn_s_setprio(0);
  }

  // epilogue: lane owns channels n..n+3 of virtual row u for every (g, f) fragment
  const int WMK = S + 2 * HM;
#pragma unroll
  for (int f = 0; f < kMF; ++f) {
    const int u = wm * kWM + f * 16 + frow;
    const int pi = u / WI, pj = u - (u / WI) * WI;
    if (pi >= S || pj >= S) continue;
    const size_t orow = (size_t)(((long)b * WO + pi + HO) * WO + pj + HO) * YC;
    const size_t mrow = (size_t)(((long)b * WMK + pi + HM) * WMK + pj + HM) * YC;
#pragma unroll
    for (int g = 0; g < kNF; ++g) {
      const int n = wn * 32 + g * 16 + fq * 4;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[g][f][r];
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

}  // namespace

// Measured on MI355X (B = 256, kernel_bench): fwd 80.9 us vs conv_pipe 76.6 us, dgrad 86.6 vs
// 88.0 us, SL step 3.25 vs 3.20 ms. The staging cut does not pay: both kernels run ~1/3 of the
// nominal MFMA rate at the power-limited clock, and the slab's 416 virtual rows per 361 pixels
// add 15 % MFMA work. So it is opt-in: RAG_CONV_SLAB=1 (or rag_conv_slab_mode(1)).
static int g_slab_mode = -2;  // -2: read RAG_CONV_SLAB on first use

RAG_API int rag_conv_slab_mode(int mode) {
  const int old = g_slab_mode;
  g_slab_mode = mode;
  return old;
}

// Returns true if the slab kernel handled the launch: enabled, 3x3, halo-1 input, 19x19 boards,
// exactly 192 output channels, CIN % 32 == 0.
bool rag_conv_slab_launch(const bf16* x, const bf16* w, const float* bias, bf16* y,
                          const bf16* mk, const bf16* res, int B, int S, int HI, int WO, int HO,
                          int CIN, int COUTP, int YC, int KS, int relu, int HM,
                          hipStream_t stream) {
  if (g_slab_mode == -2) {
    const char* e = getenv("RAG_CONV_SLAB");
    g_slab_mode = e ? atoi(e) : 0;
  }
  if (g_slab_mode != 1) return false;
  if (KS != 3 || HI != 1 || S != 19 || COUTP != kN || CIN % kBK || CIN < kBK) return false;
  const int WI = S + 2;
  if ((S - 1) * WI + S > kBM || kBM + 2 * WI + 2 > kSlabRows) return false;
  const long total_rows = (long)B * WI * WI;
  conv_slab_kernel<<<B, 64 * kWaves, 0, stream>>>(x, w, bias, y, mk, res, S, CIN, COUTP, WO, HO,
                                                 YC, relu, HM, total_rows);
  return true;
}

// Pipelined implicit-GEMM convolution (forward and dgrad) for gfx950.
//
// Same math and layouts as conv_igemm_kernel (conv.hip): C[m][n] = sum_{tap,c} X[row(m,tap)][c] *
// W[tap][n][c] over the padded channels-last activations, bias + ReLU (or the dgrad ReLU mask of
// the layer input) fused in the epilogue. What changes is the K loop:
//
//   * a ring of 3 LDS stages filled by global_load_lds (16 B per lane, LDS-direct) with the loads
//     of stage s+2 issued right after the barrier of stage s, so two K-steps of loads are always
//     in flight behind the MFMAs;
//   * every wave issues the same number of loads per stage (A: BM*BK*2/1024/4, B: BN*BK*2/1024/4),
//     so one counted `s_waitcnt vmcnt(PER_STAGE)` retires exactly stage s, followed by a raw
//     s_barrier (never __syncthreads: its implicit vmcnt(0) would drain the prefetch);
//   * BK = 32 with the st_16x32-style chunk swizzle of conv.hip (conflict-free ds_read_b128).
//
// Block = 128 pixels x BN output channels (BN = 64/128/192), 4 waves as 2 (m) x 2 (n); each wave
// owns 64 x BN/2 and issues 4 x BN/32 MFMA 16x16x32 per K-step. 60 KB of LDS per block -> two
// blocks per CU.
#include "common.h"

using namespace rag;

namespace {

constexpr int kBK = 32;
constexpr int kNBUF = 3;
// K-loop order: 0 = tap outer / channel chunk inner (A/B, rag_conv_order), 1 (default: 3-8 %
// faster) = channel chunk outer / tap inner
int g_conv_order = 1;

template <int KS, int NT, int MT>
__global__ void __launch_bounds__(256, 2)
conv_pipe_kernel(const bf16* __restrict__ X, const bf16* __restrict__ Wt,
                 const float* __restrict__ bias, bf16* __restrict__ Y,
                 const bf16* __restrict__ mask, const bf16* __restrict__ res, int M, int S, int WI, int shift, int WO, int HO,
                 int CIN, int WROWS, int YC, int relu, int HM, int cmajor) {
  constexpr int kBM = 32 * MT;  // 2 waves along M, MT 16-row fragments each
  constexpr int WM = 16 * MT;
  constexpr int BN = 32 * NT;
  constexpr int WN = 16 * NT;
  constexpr int STAGE = (kBM + BN) * kBK;
  constexpr int AINST = kBM / 16;  // 1 KB glds per 16 rows of 64 B
  constexpr int BINST = BN / 16;
  static_assert(AINST % 4 == 0 && BINST % 4 == 0, "uniform per-wave load count");
  constexpr int AK = AINST / 4, BK4 = BINST / 4;
  constexpr int PER_STAGE = AK + BK4;
  __shared__ __attribute__((aligned(16))) bf16 lds[kNBUF * STAGE];

  const int lane = lane_id();
  const int w = wave_id();
  const int wm = w & 1, wn = w >> 1;
  const int nblk_m = (M + kBM - 1) / kBM;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int bm = bid % nblk_m, bn = bid / nblk_m;
  const int m0 = bm * kBM;
  const int n0 = bn * BN;
  const int S2 = S * S;

  int abase[AK];
#pragma unroll
  for (int k = 0; k < AK; ++k) {
    const int row = (w + 4 * k) * 16 + (lane >> 2);
    int m = m0 + row;
    m = m < M ? m : M - 1;
    const int b = m / S2;
    const int rem = m - b * S2;
    const int i = rem / S;
    const int j = rem - i * S;
    abase[k] = ((b * WI + i + shift) * WI + j + shift) * CIN + (((lane & 3) ^ swz64(row)) * 8);
  }
  int bbase[BK4];
#pragma unroll
  for (int k = 0; k < BK4; ++k) {
    const int row = (w + 4 * k) * 16 + (lane >> 2);
    bbase[k] = (n0 + row) * CIN + (((lane & 3) ^ swz64(row)) * 8);
  }

  const int cchunks = CIN / kBK;
  const int nsteps = KS * KS * cchunks;

  // stages are issued strictly in order: a scalar (tap, channel-chunk) iterator replaces the
  // per-stage divisions
  int it_c0 = 0, it_tap = 0, it_kx = 0, it_ky = 0;
  auto stage = [&](int buf, int /*s*/) {
    const int aoff = (it_ky * WI + it_kx) * CIN + it_c0;
    const int boff = it_tap * WROWS * CIN + it_c0;
    bf16* la = lds + buf * STAGE;
#pragma unroll
    for (int k = 0; k < AK; ++k) glds16(X + abase[k] + aoff, la + (w + 4 * k) * 16 * kBK);
    bf16* lb = la + kBM * kBK;
#pragma unroll
    for (int k = 0; k < BK4; ++k) glds16(Wt + bbase[k] + boff, lb + (w + 4 * k) * 16 * kBK);
    if (cmajor) {  // channel chunk outer, tap inner: the 9 taps of a chunk re-read one ~L1-sized
                   // footprint of input rows back to back
      ++it_tap;
      if (++it_kx == KS) {
        it_kx = 0;
        if (++it_ky == KS) {
          it_ky = 0;
          it_tap = 0;
          it_c0 += kBK;
        }
      }
    } else {
      it_c0 += kBK;
      if (it_c0 == CIN) {
        it_c0 = 0;
        ++it_tap;
        if (++it_kx == KS) {
          it_kx = 0;
          ++it_ky;
        }
      }
    }
  };

  f32x4 acc[NT][MT];
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int i = 0; i < MT; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  stage(0, 0);
  if (nsteps > 1) stage(1, 1);

  const int frow = lane & 15;
  const int fq = lane >> 4;
  // per-lane fragment offsets (elements, buffer 0)
  int aoffs[MT], boffs[NT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int row = wm * WM + i * 16 + frow;
    aoffs[i] = row * kBK + ((fq ^ swz64(row)) * 8);
  }
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int row = wn * WN + j * 16 + frow;
    boffs[j] = kBM * kBK + row * kBK + ((fq ^ swz64(row)) * 8);
  }

  int buf = 0;
  for (int s = 0; s < nsteps; ++s) {
    if (s + 1 < nsteps)
      asm volatile("s_waitcnt vmcnt(%0)" :: "n"(PER_STAGE) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (s + 2 < nsteps) {
      int nb = buf + 2;
      nb = nb >= kNBUF ? nb - kNBUF : nb;
      stage(nb, s + 2);
    }
    const bf16* lb = lds + buf * STAGE;
    bf16x8 xa[MT], wb[NT];
#pragma unroll
    for (int i = 0; i < MT; ++i) xa[i] = *reinterpret_cast<const bf16x8*>(lb + aoffs[i]);
#pragma unroll
    for (int j = 0; j < NT; ++j) wb[j] = *reinterpret_cast<const bf16x8*>(lb + boffs[j]);
    __builtin_amdgcn_s_setprio(1);  // the MFMA burst goes first on the shared pipe
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int i = 0; i < MT; ++i) acc[j][i] = mfma16(wb[j], xa[i], acc[j][i]);
    __builtin_amdgcn_s_setprio(0);
    buf = buf + 1 == kNBUF ? 0 : buf + 1;
  }

  // epilogue: lane owns channels n..n+3 of pixel m for every (j, i) tile
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int m = m0 + wm * WM + i * 16 + frow;
    if (m >= M) continue;
    const int b = m / S2;
    const int rem = m - b * S2;
    const int pi = rem / S;
    const int pj = rem - pi * S;
    const size_t orow = (size_t)((b * WO + pi + HO) * WO + pj + HO) * YC;
    const int WMK = S + 2 * HM;  // the mask (layer input) may use its own halo
    const size_t mrow = (size_t)((b * WMK + pi + HM) * WMK + pj + HM) * YC;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int n = n0 + wn * WN + j * 16 + fq * 4;
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
      if (res) {  // residual (ResNet sum-merge), laid out like Y
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

template <int KS>
bool launch_ks(int nt, int mt, dim3 grid, hipStream_t st, const bf16* X, const bf16* W,
               const float* bias, bf16* Y, const bf16* mask, const bf16* res, int M, int S,
               int WI, int shift, int WO, int HO, int CIN, int WROWS, int YC, int relu, int HM) {
#define RAG_PIPE(N, T)                                                                        \
  if (nt == N && mt == T) {                                                                   \
    conv_pipe_kernel<KS, N, T><<<grid, 256, 0, st>>>(X, W, bias, Y, mask, res, M, S, WI,    \
                                                         shift, WO, HO, CIN, WROWS, YC, relu,  \
                                                         HM, g_conv_order);                    \
    return true;                                                                              \
  }
  RAG_PIPE(2, 4) RAG_PIPE(2, 6) RAG_PIPE(2, 8) RAG_PIPE(4, 4)
  RAG_PIPE(4, 6) RAG_PIPE(4, 8) RAG_PIPE(6, 4) RAG_PIPE(6, 6)
#undef RAG_PIPE
  return false;
}

// Pixel-tile height (MT 16-row fragments per wave, BM = 32*MT): the candidate that fills the
// 512 resident-block slots (2 per CU) best — e.g. K=128 at B=256 (M=92416): MT=4 gives 722
// blocks (two rounds, the second 41% full), MT=6 gives 482 blocks (one round, 94% full); on a
// tie (within 2 %) the taller tile.
int pick_mt(int M, int nt, int ntiles_n) {
  const int cands[3] = {4, 6, 8};
  const int ncand = nt == 6 ? 2 : 3;
  int best = 4;
  double best_eff = -1.0;
  for (int i = 0; i < ncand; ++i) {
    const int mt = cands[i];
    const long nblk = (long)((M + 32 * mt - 1) / (32 * mt)) * ntiles_n;
    const long rounds = (nblk + 511) / 512;
    const double eff = (double)nblk / (double)(rounds * 512);
    // the taller tile wins unless it fills the slots >2 % worse (more reuse per staged weight
    // tile: at B=512 the 5x5 layer took 165 us with MT=4 vs ~2 x 64 us per 256 with MT=6)
    if (eff > best_eff - 0.02) {
      best_eff = eff;
      best = mt;
    }
  }
  return best;
}

}  // namespace

// Returns true if the pipelined kernel handled the launch (COUTP multiple of 64; any KS in
// {1,3,5,7}); false leaves it to the generic kernel in conv.hip.
bool rag_conv_pipe_launch(const bf16* x, const bf16* w, const float* bias, bf16* y,
                          const bf16* mk, const bf16* res, int M, int S, int WI, int shift,
                          int WO, int HO, int CIN, int COUTP, int YC, int KS, int relu, int HM, hipStream_t stream) {
  const int nt = COUTP % 192 == 0 ? 6 : (COUTP % 128 == 0 ? 4 : (COUTP % 64 == 0 ? 2 : 0));
  if (!nt) return false;
  const int ntn = COUTP / (32 * nt);
  const int mt = pick_mt(M, nt, ntn);
  const int bm = 32 * mt;
  const int nblk_m = (M + bm - 1) / bm;
  dim3 grid(nblk_m * ntn);
  switch (KS) {
    case 1: return launch_ks<1>(nt, mt, grid, stream, x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM);
    case 3: return launch_ks<3>(nt, mt, grid, stream, x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM);
    case 5: return launch_ks<5>(nt, mt, grid, stream, x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM);
    case 7: return launch_ks<7>(nt, mt, grid, stream, x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM);
    default: return false;
  }
}

// K-loop order of conv_pipe (see g_conv_order); returns the previous setting.
RAG_API int rag_conv_order(int order) {
  const int old = g_conv_order;
  g_conv_order = order;
  return old;
}

// Implicit-GEMM convolutions for 19x19 Go boards on gfx950 (MI355X) — kernels K01/K02/K05/K06/K08.
//
// Activation layout ("padded channels-last"): bf16 [B][S+2H][S+2H][C] with an all-zero halo of
// width H (H=1 for 3x3 and 1x1 layers, H=2 for the 5x5 input layer) and C padded to a multiple
// of 32. A 'same' convolution then needs no boundary test: output pixel (i,j) reads input rows
// ((b*W + i + ky + shift) * W + j + kx + shift), shift = H - KS/2. The halo is written once
// (buffers are zero-initialised) and never touched by any kernel.
//
// GEMM view:  Y[m, n] = sum_{tap, c} X[row(m, tap), c] * Wf[tap, n, c]
//             m = b*S*S + i*S + j (B*361 rows), n = output channel, K = taps * C.
// The same kernel computes dgrad with tap-flipped, transposed weights Wb[tap', c, n] and an
// epilogue mask (input > 0) that applies the producing layer's ReLU derivative in place.
//
// Tiling (conv_igemm): 256 threads = 4 waves (2 along M x 2 along N); block tile 128 pixels x
// 32*NT channels; wave tile 64 x 16*NT as 4 x NT MFMA 16x16x32 bf16 tiles. K step = one tap x 32
// channels. Both operands are staged global->LDS with global_load_lds_dwordx4 (per-lane gathered
// source rows, lane-linear LDS image, swizzle applied on the source address), double-buffered.
// The MFMA is issued as C^T = W * X^T so each lane owns 4 consecutive output channels of one
// pixel: the epilogue (bias, ReLU, ReLU-mask, bf16 pack) stores 8 bytes per lane.
#include <mutex>

#include "common.h"
#include "pack.h"
#include "wgrad_part.h"

using namespace rag;

namespace {

constexpr int kBM = 128;  // pixels per block
constexpr int kBK = 32;   // K per step (one MFMA)

template <int KS, int NT>
__global__ void __launch_bounds__(256, 3)
conv_igemm_kernel(const bf16* __restrict__ X, const bf16* __restrict__ Wt,
                  const float* __restrict__ bias, bf16* __restrict__ Y,
                  const bf16* __restrict__ mask, const bf16* __restrict__ res, int M, int S, int WI, int shift, int WO, int HO,
                  int CIN, int WROWS, int YC, int relu, int HM) {
  constexpr int BN = 32 * NT;
  constexpr int WN = 16 * NT;
  constexpr int STAGE = (kBM + BN) * kBK;  // bf16 elements per stage
  __shared__ __attribute__((aligned(16))) bf16 lds[2 * STAGE];

  const int lane = lane_id();
  const int w = wave_id();
  const int wm = w & 1, wn = w >> 1;
  const int m0 = blockIdx.x * kBM;
  const int n0 = blockIdx.y * BN;
  const int S2 = S * S;

  // per-lane gather rows for the A (pixel) tile: instructions w and w+4, 16 rows each
  int abase[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int row = (w + 4 * k) * 16 + (lane >> 2);
    int m = m0 + row;
    m = m < M ? m : M - 1;
    const int b = m / S2;
    const int rem = m - b * S2;
    const int i = rem / S;
    const int j = rem - i * S;
    abase[k] = ((b * WI + i + shift) * WI + j + shift) * CIN + (((lane & 3) ^ swz64(row)) * 8);
  }
  constexpr int BINST = BN / 16;  // wave-instructions per B tile
  int bbase[(BINST + 3) / 4];
#pragma unroll
  for (int k = 0; k < (BINST + 3) / 4; ++k) {
    const int row = (w + 4 * k) * 16 + (lane >> 2);
    bbase[k] = (n0 + row) * CIN + (((lane & 3) ^ swz64(row)) * 8);
  }

  const int cchunks = CIN / kBK;
  const int nsteps = KS * KS * cchunks;

  auto stage = [&](int buf, int s) {
    const int tap = s / cchunks;
    const int c0 = (s - tap * cchunks) * kBK;
    const int ky = tap / KS, kx = tap - (tap / KS) * KS;
    const int aoff = (ky * WI + kx) * CIN + c0;
    bf16* la = lds + buf * STAGE;
#pragma unroll
    for (int k = 0; k < 2; ++k) glds16(X + abase[k] + aoff, la + (w + 4 * k) * 16 * kBK);
    bf16* lb = la + kBM * kBK;
    const int boff = tap * WROWS * CIN + c0;
#pragma unroll
    for (int k = 0; k < (BINST + 3) / 4; ++k) {
      const int inst = w + 4 * k;
      if (inst < BINST) glds16(Wt + bbase[k] + boff, lb + inst * 16 * kBK);
    }
  };

  f32x4 acc[NT][4];
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int frow = lane & 15;
  const int fq = lane >> 4;
  for (int s = 0; s < nsteps; ++s) {
    const int cur = s & 1;
    if (s + 1 < nsteps) stage(cur ^ 1, s + 1);
    const bf16* la = lds + cur * STAGE;
    const bf16* lb = la + kBM * kBK;
    bf16x8 xa[4], wb[NT];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wm * 64 + i * 16 + frow;
      xa[i] = *reinterpret_cast<const bf16x8*>(la + row * kBK + ((fq ^ swz64(row)) * 8));
    }
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int row = wn * WN + j * 16 + frow;
      wb[j] = *reinterpret_cast<const bf16x8*>(lb + row * kBK + ((fq ^ swz64(row)) * 8));
    }
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[j][i] = mfma16(wb[j], xa[i], acc[j][i]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // epilogue: lane owns channels n..n+3 of pixel m for every (j, i) tile
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wm * 64 + i * 16 + frow;
    if (m >= M) continue;
    const int b = m / S2;
    const int rem = m - b * S2;
    const int pi = rem / S;
    const int pj = rem - pi * S;
    const size_t orow = (size_t)((b * WO + pi + HO) * WO + pj + HO) * YC;
    const int WM = S + 2 * HM;  // the mask (layer input) may use its own halo
    const size_t mrow = (size_t)((b * WM + pi + HM) * WM + pj + HM) * YC;
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

// ---------------------------------------------------------------------------------- wgrad
// dW[tap][n][c] = sum_m G[m][n] * X[row(m,tap)][c]   (G = gradient w.r.t. pre-activation)
// Block = (pixel chunk, (n,c) tile, tap). Per step: 32 pixels of G and of the tap-shifted X are
// staged row-major ([pixel][channel], the natural layout) by global_load_lds; fragments along
// the pixel (K) axis are read with ds_read_tr16_b64 (hardware transpose). fp32 partials go to a
// per-chunk slab (plain stores), reduced by wgrad_reduce_kernel, which also emits OIHW layout.
// Software pipeline: 64-pixel stages (two MFMA k-steps), 3 LDS buffers, loads for stage s+2
// issued right after the barrier of stage s; every wave issues the same number of
// global_load_lds per stage, so a single counted `s_waitcnt vmcnt(PER_STAGE)` retires exactly
// stage s while s+1 stays in flight, followed by a raw s_barrier (never __syncthreads, whose
// implicit vmcnt(0) would drain the prefetch).
template <int KS, int NTN, int NTC>
__global__ void __launch_bounds__(256, 1)
conv_wgrad_kernel(const bf16* __restrict__ G, const bf16* __restrict__ X,
                  float* __restrict__ part, float* __restrict__ bpart, int M, int S, int WI,
                  int shift, int WG, int HG, int GC, int CIN, int steps_per_chunk, int COUTP,
                  int CINP, int ntile_c) {
  constexpr int BKP = 64;  // pixels per stage
  constexpr int NBUF = 3;
  constexpr int BNN = 32 * NTN, BNC = 32 * NTC;
  constexpr int WNN = 16 * NTN, WNC = 16 * NTC;
  constexpr int GROW = BNN, XROW = BNC;  // elements per LDS row
  constexpr int STAGE = BKP * (GROW + XROW);
  constexpr int GCH = BNN / 8, XCH = BNC / 8;  // 16B chunks per row
  constexpr int GINST = BKP * GCH / 64, XINST = BKP * XCH / 64;
  static_assert(GINST % 4 == 0 && XINST % 4 == 0, "uniform per-wave load count");
  constexpr int GK = GINST / 4, XK = XINST / 4;
  constexpr int PER_STAGE = GK + XK;  // glds per wave per stage
  __shared__ __attribute__((aligned(16))) bf16 lds[NBUF * STAGE];

  const int lane = lane_id();
  const int w = wave_id();
  const int wa = w & 1, wb = w >> 1;  // wa along n, wb along c
  // 1-D grid, XCD-aware: the taps x tiles blocks that share one pixel chunk get consecutive
  // work ids on the same XCD, so its G/X rows come from HBM once and then hit that XCD's L2.
  const int taps = KS * KS;
  const int ntile_n = COUTP / BNN;
  const int per_chunk = taps * ntile_n * ntile_c;
  const int wid = xcd_remap(blockIdx.x, gridDim.x);
  const int chunk = wid / per_chunk;
  const int wrem = wid - chunk * per_chunk;
  const int tile = wrem / taps;
  const int tap = wrem - tile * taps;
  const int tn = tile / ntile_c, tc = tile - (tile / ntile_c) * ntile_c;
  const int n0 = tn * BNN, c0 = tc * BNC;
  const int ky = tap / KS, kx = tap - (tap / KS) * KS;
  const int mbeg = chunk * steps_per_chunk * BKP;

  // per-lane pixel coordinates of its staged rows, advanced by BKP pixels per stage
  int gm[GK], gb[GK], gi[GK], gj[GK], goff[GK];
  int xm[XK], xb[XK], xi[XK], xj[XK], xoff[XK];
  auto init_pix = [&](int m, int& b, int& i, int& j) {
    const int S2 = S * S;
    const int mm = m < M ? m : M - 1;
    b = mm / S2;
    const int r = mm - b * S2;
    i = r / S;
    j = r - i * S;
  };
  auto adv = [&](int& b, int& i, int& j) {
    j += BKP;
    while (j >= S) { j -= S; ++i; }
    while (i >= S) { i -= S; ++b; }
  };
#pragma unroll
  for (int k = 0; k < GK; ++k) {
    const int idx = (w + 4 * k) * 64 + lane;
    const int row = idx / GCH;
    goff[k] = n0 + ((idx - row * GCH) ^ swz_tr<GCH>(row)) * 8;
    gm[k] = mbeg + row;
    init_pix(gm[k], gb[k], gi[k], gj[k]);
  }
#pragma unroll
  for (int k = 0; k < XK; ++k) {
    const int idx = (w + 4 * k) * 64 + lane;
    const int row = idx / XCH;
    xoff[k] = c0 + ((idx - row * XCH) ^ swz_tr<XCH>(row)) * 8;
    xm[k] = mbeg + row;
    init_pix(xm[k], xb[k], xi[k], xj[k]);
  }

  auto stage = [&](int buf) {
    bf16* lg = lds + buf * STAGE;
    bf16* lx = lg + BKP * GROW;
#pragma unroll
    for (int k = 0; k < GK; ++k) {
      // rows past M read padded row 0 (a halo pixel: zero) and contribute nothing
      const size_t src = gm[k] < M
          ? (size_t)((gb[k] * WG + gi[k] + HG) * WG + gj[k] + HG) * GC + goff[k] : 0;
      glds16(G + src, lg + (w + 4 * k) * 512);
      gm[k] += BKP;
      if (gm[k] < M) adv(gb[k], gi[k], gj[k]);
    }
#pragma unroll
    for (int k = 0; k < XK; ++k) {
      const size_t src = (size_t)((xb[k] * WI + xi[k] + ky + shift) * WI + xj[k] + kx +
                                  shift) * CIN + xoff[k];
      glds16(X + src, lx + (w + 4 * k) * 512);
      xm[k] += BKP;
      if (xm[k] < M) adv(xb[k], xi[k], xj[k]);
    }
  };

  f32x4 acc[NTN][NTC];
#pragma unroll
  for (int a = 0; a < NTN; ++a)
#pragma unroll
    for (int c = 0; c < NTC; ++c) acc[a][c] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;
  const bool do_bias = (bpart != nullptr) && tap == 0 && tc == 0;

  const int mleft = M - mbeg;
  int nsteps = (mleft + BKP - 1) / BKP;
  nsteps = nsteps < steps_per_chunk ? nsteps : steps_per_chunk;
  nsteps = nsteps > 0 ? nsteps : 0;

  if (nsteps > 0) stage(0);
  if (nsteps > 1) stage(1);
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  for (int s = 0; s < nsteps; ++s) {
    // retire stage s (stage s+1 may stay in flight), then make it visible to all waves
    if (s + 1 < nsteps)
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" :: "n"(PER_STAGE) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (s + 2 < nsteps) stage((s + 2) % NBUF);
    const bf16* lg = lds + (s % NBUF) * STAGE;
    const bf16* lx = lg + BKP * GROW;
#pragma unroll
    for (int h = 0; h < 2; ++h) {  // two MFMA k-steps of 32 pixels
      const int rb = h * 32;
      bf16x8 fa[NTN], fb[NTC];
#pragma unroll
      for (int a = 0; a < NTN; ++a) {
        const int col = wa * WNN + a * 16 + 4 * p;
        const int r0 = rb + 8 * g + q, r1 = r0 + 4;
        const bf16* p0 = lg + r0 * GROW + (((col >> 3) ^ swz_tr<GCH>(r0)) << 3) + (col & 7);
        const bf16* p1 = lg + r1 * GROW + (((col >> 3) ^ swz_tr<GCH>(r1)) << 3) + (col & 7);
        fa[a] = tr_frag(p0, p1);
      }
#pragma unroll
      for (int c = 0; c < NTC; ++c) {
        const int col = wb * WNC + c * 16 + 4 * p;
        const int r0 = rb + 8 * g + q, r1 = r0 + 4;
        const bf16* p0 = lx + r0 * XROW + (((col >> 3) ^ swz_tr<XCH>(r0)) << 3) + (col & 7);
        const bf16* p1 = lx + r1 * XROW + (((col >> 3) ^ swz_tr<XCH>(r1)) << 3) + (col & 7);
        fb[c] = tr_frag(p0, p1);
      }
      lds_reads_done();
#pragma unroll
      for (int a = 0; a < NTN; ++a)
#pragma unroll
        for (int c = 0; c < NTC; ++c) acc[a][c] = mfma16(fa[a], fb[c], acc[a][c]);
    }
    if (do_bias && (int)threadIdx.x < BNN) {
      const int c = threadIdx.x;
#pragma unroll 8
      for (int r = 0; r < BKP; ++r)
        bsum += (float)lg[r * GROW + (((c >> 3) ^ swz_tr<GCH>(r)) << 3) + (c & 7)];
    }
  }

  // write the partial slab part[chunk][tap][n][c] (fp32, plain stores)
  float* dst = part + ((size_t)(chunk * taps + tap) * COUTP) * CINP;
#pragma unroll
  for (int a = 0; a < NTN; ++a)
#pragma unroll
    for (int c = 0; c < NTC; ++c) {
      const int n = n0 + wa * WNN + a * 16 + g * 4;
      const int cc = c0 + wb * WNC + c * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) dst[(size_t)(n + r) * CINP + cc] = acc[a][c][r];
    }
  if (do_bias && (int)threadIdx.x < BNN) bpart[(size_t)chunk * COUTP + n0 + threadIdx.x] = bsum;
}

// Sum the partial slabs -> OIHW fp32 weight gradient (unpadded) and bias gradient. One thread
// per float4 quad of the [tap][n][c] slab walks the chunks (4 loads in flight): every chunk read
// is a coalesced stream. Measured against a variant that splits the chunks over 4 waves of a
// block (more blocks, 16 loads in flight per quad): that one was 15-20 % slower on MI355X.
template <int U>
__global__ void wgrad_reduce_kernel(const float* __restrict__ part, const float* __restrict__ bpart,
                                    float* __restrict__ dW, float* __restrict__ db, int nchunks,
                                    int taps, int COUT, int CIN, int COUTP, int CINP, int KS,
                                    int accumulate) {
  const size_t slab = (size_t)taps * COUTP * CINP;
  const int quads = (int)(slab / 4);
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < quads + COUTP;
       q += gridDim.x * blockDim.x) {
    if (q < quads) {
      const size_t off = (size_t)q * 4;
      const int c = (int)(off % CINP);
      const int tn = (int)(off / CINP);
      const int n = tn % COUTP, tap = tn / COUTP;
      if (n >= COUT || c >= CIN) continue;
      const float4* p = reinterpret_cast<const float4*>(part + off);
      const size_t st = slab / 4;
      float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0;
      int k = 0;
      for (; k + U - 1 < nchunks; k += U) {
        float4 a[U];
#pragma unroll
        for (int j = 0; j < U; ++j) a[j] = p[(k + j) * st];
#pragma unroll
        for (int j = 0; j < U; j += 2) {
          s0.x += a[j].x; s0.y += a[j].y; s0.z += a[j].z; s0.w += a[j].w;
          s1.x += a[j + 1].x; s1.y += a[j + 1].y; s1.z += a[j + 1].z; s1.w += a[j + 1].w;
        }
      }
      for (; k < nchunks; ++k) {
        const float4 a = p[k * st];
        s0.x += a.x; s0.y += a.y; s0.z += a.z; s0.w += a.w;
      }
      const float v[4] = {s0.x + s1.x, s0.y + s1.y, s0.z + s1.z, s0.w + s1.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (c + j >= CIN) break;
        const size_t o = ((size_t)n * CIN + c + j) * taps + tap;  // OIHW
        dW[o] = accumulate ? dW[o] + v[j] : v[j];
      }
    } else if (db && bpart) {
      const int n = q - quads;
      if (n >= COUT) continue;
      float s = 0.f;
      for (int k = 0; k < nchunks; ++k) s += bpart[(size_t)k * COUTP + n];
      db[n] = accumulate ? db[n] + s : s;
    }
  }
}

// OIHW fp32 master weights -> bf16 forward [tap][COUTP][CINP] and dgrad [tap'][CINP][COUTP]
__global__ void pack_weights_kernel(const float* __restrict__ W, bf16* __restrict__ Wf,
                                    bf16* __restrict__ Wb, int COUT, int CIN, int KS, int COUTP,
                                    int CINP) {
  const int taps = KS * KS;
  const int total = taps * COUTP * CINP;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += gridDim.x * blockDim.x) {
    const int c = idx % CINP;
    const int n = (idx / CINP) % COUTP;
    const int tap = idx / (CINP * COUTP);
    float v = 0.f;
    if (n < COUT && c < CIN) v = W[((size_t)n * CIN + c) * taps + tap];
    Wf[idx] = (bf16)v;
    if (Wb) Wb[((size_t)(taps - 1 - tap) * CINP + c) * COUTP + n] = (bf16)v;
  }
}

__device__ __forceinline__ void dihedral(int t, int n, int i, int j, int& si, int& sj) {
  // source coordinate of output (i, j) under transform t (np.rot90 / flips, reference order
  // noop, rot90, rot180, rot270, fliplr, flipud, diag1, diag2)
  switch (t) {
    case 1: si = j; sj = n - 1 - i; break;
    case 2: si = n - 1 - i; sj = n - 1 - j; break;
    case 3: si = n - 1 - j; sj = i; break;
    case 4: si = i; sj = n - 1 - j; break;
    case 5: si = n - 1 - i; sj = j; break;
    case 6: si = j; sj = i; break;
    case 7: si = n - 1 - j; sj = n - 1 - i; break;
    default: si = i; sj = j; break;
  }
}

// uint8 feature planes [B][F][S][S] (optionally gathered by index and dihedral-transformed)
// -> padded channels-last bf16 [B][S+2H][S+2H][CP]   (K08 fused with layout conversion)
// One thread per (pixel, 8-channel group): 8x the threads of a per-pixel loop, so the byte
// gathers of one pixel's planes are in flight together and a wave's 16-byte stores are contiguous.
// FS = planes per position in F (>= NF: e.g. the policy net reads the first 48 of the search's
// shared 49-plane policy+value input in place).
template <typename T>
__global__ void pack_input_kernel(const T* __restrict__ F, const int64_t* __restrict__ index,
                                  const int* __restrict__ tf, bf16* __restrict__ X, int B, int NF,
                                  int FS, int S, int H, int CP) {
  const int S2 = S * S;
  const int G = CP / 8;
  const int total = B * S2 * G;
  const int WP = S + 2 * H;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const int idx = t / G;
    const int c8 = (t - idx * G) * 8;
    const int b = idx / S2;
    const int rem = idx - b * S2;
    const int i = rem / S, j = rem - (rem / S) * S;
    int si = i, sj = j;
    if (tf) dihedral(tf[b], S, i, j, si, sj);
    const int64_t sb = index ? index[b] : b;
    const T* src = F + (size_t)sb * FS * S2 + si * S + sj;
    bf16* dst = X + ((size_t)(b * WP + i + H) * WP + j + H) * CP;
    bf16x8 v;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = c8 + k;
      v[k] = (bf16)(c < NF ? (float)src[(size_t)c * S2] : 0.f);
    }
    *reinterpret_cast<bf16x8*>(dst + c8) = v;
  }
}

// As pack_input_kernel, one block per position: the position's NF planes (one contiguous
// NF * S2 run of F) are read coalesced into LDS as bf16 first, then each thread builds 16-byte
// (pixel, 8-channel) stores from LDS. The per-thread gather of pack_input_kernel reads 8 bytes
// at a 361-byte stride per store (14.7 us for B = 256, 48 planes); this reads F once, in order.
constexpr int kPackInMaxC = 64, kPackInMaxS2 = 361;
constexpr int kPackInThreads = 512;  // one block per position: short per-thread load chains
template <typename T>
__global__ void __launch_bounds__(kPackInThreads)
pack_input_lds_kernel(const T* __restrict__ F, const int64_t* __restrict__ index,
                      const int* __restrict__ tf, bf16* __restrict__ X, int NF, int FS, int S,
                      int H, int CP) {
  __shared__ bf16 st[kPackInMaxC * kPackInMaxS2];
  const int S2 = S * S;
  const int b = blockIdx.x;
  const int64_t sb = index ? index[b] : b;
  const T* src = F + (size_t)sb * FS * S2;
  const int n = NF * S2;
  if (sizeof(T) == 1 && (reinterpret_cast<uintptr_t>(src) & 3) == 0) {
    // 4 planes bytes per load (uint8 planes of a 4-byte aligned position)
    const uint32_t* s4 = reinterpret_cast<const uint32_t*>(src);
    const int n4 = n >> 2;
#pragma unroll 4
    for (int e = threadIdx.x; e < n4; e += kPackInThreads) {
      const uint32_t w = s4[e];
#pragma unroll
      for (int k = 0; k < 4; ++k) st[4 * e + k] = (bf16)(float)((w >> (8 * k)) & 0xff);
    }
    for (int e = 4 * n4 + threadIdx.x; e < n; e += kPackInThreads) st[e] = (bf16)(float)src[e];
  } else {
#pragma unroll 4
    for (int e = threadIdx.x; e < n; e += kPackInThreads) st[e] = (bf16)(float)src[e];
  }
  __syncthreads();
  const int G = CP / 8, WP = S + 2 * H;
  const int t = tf ? tf[b] : 0;
  for (int e = threadIdx.x; e < S2 * G; e += kPackInThreads) {
    const int p = e / G, c8 = (e - p * G) * 8;
    const int i = p / S, j = p - i * S;
    int si = i, sj = j;
    if (t) dihedral(t, S, i, j, si, sj);
    const int q = si * S + sj;
    bf16x8 v;
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = c8 + k < NF ? st[(c8 + k) * S2 + q] : (bf16)0.f;
    *reinterpret_cast<bf16x8*>(X + ((size_t)(b * WP + i + H) * WP + j + H) * CP + c8) = v;
  }
}

// Bit-packed positions (one 64-bit word per point, bit f = plane f; 2.9 KB per 19x19 position
// instead of 17 KB of uint8 planes, so a GPU-resident buffer holds ~6x more positions) ->
// padded bf16 trunk input, with the same index gather and dihedral transform.
__global__ void pack_input_bits_kernel(const uint64_t* __restrict__ Fb,
                                       const int64_t* __restrict__ index,
                                       const int* __restrict__ tf, bf16* __restrict__ X, int B,
                                       int NF, int S, int H, int CP) {
  const int S2 = S * S;
  const int G = CP / 8;
  const int total = B * S2 * G;
  const int WP = S + 2 * H;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const int idx = t / G;
    const int c8 = (t - idx * G) * 8;
    const int b = idx / S2;
    const int rem = idx - b * S2;
    const int i = rem / S, j = rem - (rem / S) * S;
    int si = i, sj = j;
    if (tf) dihedral(tf[b], S, i, j, si, sj);
    const int64_t sb = index ? index[b] : b;
    const uint64_t word = Fb[(size_t)sb * S2 + si * S + sj];
    bf16* dst = X + ((size_t)(b * WP + i + H) * WP + j + H) * CP;
    bf16x8 v;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = c8 + k;
      v[k] = (bf16)((c < NF && ((word >> c) & 1ull)) ? 1.f : 0.f);
    }
    *reinterpret_cast<bf16x8*>(dst + c8) = v;
  }
}

// padded channels-last bf16 -> NCHW fp32 (tests / debugging / generic consumers)
__global__ void unpack_kernel(const bf16* __restrict__ X, float* __restrict__ out, int B, int C,
                              int S, int H, int CP) {
  const int S2 = S * S;
  const int WP = S + 2 * H;
  const int total = B * C * S2;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += gridDim.x * blockDim.x) {
    const int p = idx % S2;
    const int c = (idx / S2) % C;
    const int b = idx / (S2 * C);
    const int i = p / S, j = p % S;
    out[idx] = (float)X[((size_t)(b * WP + i + H) * WP + j + H) * CP + c];
  }
}

// NCHW fp32 -> padded channels-last bf16 (gradient / activation import)
__global__ void pack_nchw_kernel(const float* __restrict__ in, bf16* __restrict__ X, int B, int C,
                                 int S, int H, int CP) {
  const int S2 = S * S;
  const int WP = S + 2 * H;
  const int total = B * S2 * CP;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += gridDim.x * blockDim.x) {
    const int c = idx % CP;
    const int p = (idx / CP) % S2;
    const int b = idx / (CP * S2);
    const int i = p / S, j = p % S;
    const float v = c < C ? in[((size_t)b * C + c) * S2 + p] : 0.f;
    X[((size_t)(b * WP + i + H) * WP + j + H) * CP + c] = (bf16)v;
  }
}

template <int KS>
void launch_igemm_ks(int nt, dim3 grid, hipStream_t st, const bf16* X, const bf16* W,
                     const float* bias, bf16* Y, const bf16* mask, const bf16* res, int M, int S, int WI,
                     int shift, int WO, int HO, int CIN, int WROWS, int YC, int relu, int HM) {
  switch (nt) {
#define RAG_NT(N)                                                                              \
  case N:                                                                                      \
    conv_igemm_kernel<KS, N><<<grid, 256, 0, st>>>(X, W, bias, Y, mask, res, M, S, WI, shift, WO, \
                                                   HO, CIN, WROWS, YC, relu, HM);             \
    break;
    RAG_NT(1) RAG_NT(2) RAG_NT(3) RAG_NT(4) RAG_NT(6)
#undef RAG_NT
  }
}

int pick_nt(int coutp) {
  if (coutp % 192 == 0) return 6;
  if (coutp % 128 == 0) return 4;
  if (coutp % 96 == 0) return 3;
  if (coutp % 64 == 0) return 2;
  return 1;
}

}  // namespace

// ============================================================================= C ABI
bool rag_conv_pipe_launch(const bf16* x, const bf16* w, const float* bias, bf16* y,
                          const bf16* mk, const bf16* res, int M, int S, int WI, int shift,
                          int WO, int HO, int CIN, int COUTP, int YC, int KS, int relu, int HM,
                          hipStream_t stream);  // conv_fwd.hip
bool rag_conv_tap_launch(const bf16* x, const bf16* w, const float* bias, bf16* y,
                         const bf16* mk, const bf16* res, int M, int S, int WI, int shift, int WO,
                         int HO, int CIN, int COUTP, int YC, int KS, int relu, int HM,
                         long total_rows, hipStream_t stream, const WgradRed* red,
                         const float* bnc, const float* mcoef, float* spart,
                         const float* smean);  // conv_tap.hip
bool rag_conv_tap_bn_ok(int M, int S, int WI, int shift, int CIN, int COUTP, int KS);
bool rag_wgrad_slab_ok(int S, int H, int HG, int GC, int COUTP, int CINP, int KS);

// Conv forward / dgrad.  X: padded input (halo HI, CIN channels, CIN % 32 == 0).  W: packed
// bf16 weights [taps][WROWS][CIN].  Y: padded output (halo HO, YC channels, COUTP % 32 == 0,
// COUTP <= YC).  bias: fp32 [COUTP] or null.  mask: the dgrad ReLU mask (layer input), null or
// laid out like Y but with its own halo HM.  res: null or a residual added before the activation
// (ResNet sum-merge), laid out like Y (may alias Y: each element is read then written by one lane).
// Deferred wgrad reduction (rag_conv_wgrad_deferred): the fp16 partial-slab reduction of one
// layer waits in a caller-owned handle (PendingRed: the trainer's trunk owns one) and rides along
// the next conv_tap launch that the caller hands the same handle, on the same stream, as extra
// blocks (that launch fills 482 of 512 block slots at B = 256, so the reduction runs in otherwise
// idle slots instead of as a 14 us kernel of its own). Launches without the handle never see it;
// a launch with the handle on another stream, a second deferral or rag_wgrad_flush(handle)
// launches the pending reduction as a standalone kernel. No process-wide state: two trainers (or
// a trainer and a search) may interleave their launches on one stream.
int rag_launch_wgrad_slab_reduce(const WgradRed& r, hipStream_t stream);  // wgrad_slab.hip
struct PendingRed {
  int valid;
  hipStream_t stream;
  WgradRed r;
  unsigned* dticket;  // the handle's [2] device claim counters (allocated on first deferral)
};

RAG_API size_t rag_wgrad_pending_bytes() { return sizeof(PendingRed); }

// The handle's claim counters, allocated (and zeroed) when the handle is created rather than on
// its first deferral (hipMalloc synchronises the device in the middle of a step), and freed
// with it (ops.PendingReduction.__del__).
RAG_API int rag_wgrad_pending_init(void* h) {
  PendingRed* p = static_cast<PendingRed*>(h);
  if (!p) return -1;
  if (!p->dticket) {
    if (hipMalloc(&p->dticket, 2 * sizeof(unsigned)) != hipSuccess) return -3;
    if (hipMemset(p->dticket, 0, 2 * sizeof(unsigned)) != hipSuccess) return -3;
  }
  return 0;
}
RAG_API int rag_wgrad_pending_free(void* h) {
  PendingRed* p = static_cast<PendingRed*>(h);
  if (!p || !p->dticket) return 0;
  const hipError_t e = hipFree(p->dticket);
  p->dticket = nullptr;
  return e == hipSuccess ? 0 : -3;
}

// Take the handle's reduction if there is one: returns false if it was empty.
static bool take_pending(void* h, WgradRed* r, hipStream_t* st) {
  PendingRed* p = static_cast<PendingRed*>(h);
  if (!p || !p->valid) return false;
  *r = p->r;
  *st = p->stream;
  p->valid = 0;
  return true;
}

static int flush_pending(void* h, hipStream_t stream) {
  WgradRed r;
  hipStream_t st;
  if (!take_pending(h, &r, &st)) return 0;
  return rag_launch_wgrad_slab_reduce(r, stream ? stream : st);
}

RAG_API int rag_wgrad_flush(hipStream_t stream, void* pending) {
  return flush_pending(pending, stream);
}

// BN prologue fusion (ResnetPolicy): true if rag_conv_igemm_bn / rag_conv_wgrad*_bn can run a
// layer of this shape with its input given as the BN input x plus [3][S] column coefficients.
RAG_API int rag_conv_bn_fusable(int B, int S, int HI, int CIN, int COUTP, int KS) {
  return KS == 3 && HI == 1 && CIN == COUTP &&
         rag_conv_tap_bn_ok(B * S * S, S, S + 2 * HI, HI - 1, CIN, COUTP, KS) &&
         rag_wgrad_slab_ok(S, HI, HI, COUTP, COUTP, CIN, KS);
}

static int conv_igemm_impl(const void* X, const void* W, const float* bias, void* Y,
                           const void* mask, const void* resid, int B, int S, int HI, int HO,
                           int CIN, int COUTP, int YC, int KS, int relu, int HM,
                           hipStream_t stream, void* pending, const float* bnc,
                           const float* mcoef, float* spart = nullptr,
                           const float* smean = nullptr);

namespace {
// Real input channels of the launch in progress (0 = unknown: the padded CIN is all real);
// set by rag_conv_igemm_cin for the launch it makes, read by the tap kernels' dispatch.
}  // namespace
thread_local int g_conv_cin_real = 0;

// `pending`: null, or the caller's deferred-reduction handle (see PendingRed above).
RAG_API int rag_conv_igemm(const void* X, const void* W, const float* bias, void* Y,
                           const void* mask, const void* resid, int B, int S, int HI, int HO,
                           int CIN, int COUTP, int YC, int KS, int relu, int HM,
                           hipStream_t stream, void* pending) {
  return conv_igemm_impl(X, W, bias, Y, mask, resid, B, S, HI, HO, CIN, COUTP, YC, KS, relu, HM,
                         stream, pending, nullptr, nullptr);
}

// As rag_conv_igemm, telling the dispatch how many of the CIN (padded) input channels are real:
// a 5x5 layer with <= 48 of 64 skips the zero channels' MFMAs (conv_tap.hip, PAIR).
RAG_API int rag_conv_igemm_cin(const void* X, const void* W, const float* bias, void* Y,
                               const void* mask, const void* resid, int B, int S, int HI, int HO,
                               int CIN, int COUTP, int YC, int KS, int relu, int HM,
                               hipStream_t stream, void* pending, int cin_real) {
  g_conv_cin_real = cin_real;
  const int rc = conv_igemm_impl(X, W, bias, Y, mask, resid, B, S, HI, HO, CIN, COUTP, YC, KS,
                                 relu, HM, stream, pending, nullptr, nullptr);
  g_conv_cin_real = 0;
  return rc;
}

// As rag_conv_igemm with the BN prologue: X is the BN input x and the layer input is
// U = ReLU(bnc[0][col] * x + bnc[2][col]) (forward), and/or the dgrad ReLU mask is recomputed
// from `mask` = x and mcoef (no residual then). -5 if the shape has no fused kernel
// (rag_conv_bn_fusable).
// spart (optional): the output's BN column statistics as per-block partials [nblk][2][S] for
// rag_bn_finalize (nblk = rag_conv_bn_stat_blocks); smean: the BN mean for the backward form.
RAG_API int rag_conv_igemm_bn(const void* X, const void* W, const float* bias, void* Y,
                              const void* mask, const void* resid, int B, int S, int HI, int HO,
                              int CIN, int COUTP, int YC, int relu, int HM, hipStream_t stream,
                              void* pending, const float* bnc, const float* mcoef, float* spart,
                              const float* smean) {
  if ((!bnc && !mcoef && !spart) || (mcoef && resid) || (smean && !mcoef)) return -5;
  return conv_igemm_impl(X, W, bias, Y, mask, resid, B, S, HI, HO, CIN, COUTP, YC, 3, relu, HM,
                         stream, pending, bnc, mcoef, spart, smean);
}

// Winograd F(2,3) 3x3 convolution (conv_wino.hip): forward or dgrad with the layer's Winograd
// weights [12][NOUT][KIN] (rag_wino_pack). A deferred wgrad reduction in `pending` rides along
// the launch (every block claims units of it after its epilogue) when it has claim counters and
// the grid is one-dimensional; otherwise it goes out on its own first.
int rag_conv_wino_launch(const void* X, const void* W, const float* bias, void* Y,
                         const void* mask, int B, int S, int KIN, int NOUT, int HO, int YC,
                         int relu, int HM, hipStream_t stream, const WgradRed* red, int half);
// The pending reduction of `pending` for a Winograd launch of NOUT channels on `stream`: it rides
// (returned in *pend, *red = pend) when it has claim counters and the grid is one-dimensional,
// else it goes out on its own now. Returns that launch's error code (0).
static int wino_pending(void* pending, hipStream_t stream, int NOUT, WgradRed* pend,
                        const WgradRed** red) {
  hipStream_t pend_stream = nullptr;
  *red = nullptr;
  if (!take_pending(pending, pend, &pend_stream)) return 0;
  if (pend_stream == stream && pend->ticket && (NOUT == 192 || NOUT == 128)) {  // 1-D grids
    *red = pend;
    return 0;
  }
  return rag_launch_wgrad_slab_reduce(*pend, pend_stream);
}

RAG_API int rag_conv_wino_p(const void* X, const void* W, const float* bias, void* Y,
                            const void* mask, int B, int S, int KIN, int NOUT, int HO, int YC,
                            int relu, int HM, hipStream_t stream, void* pending, int half) {
  WgradRed pend;
  const WgradRed* red = nullptr;
  if (const int rc = wino_pending(pending, stream, NOUT, &pend, &red)) return rc;
  return rag_conv_wino_launch(X, W, bias, Y, mask, B, S, KIN, NOUT, HO, YC, relu, HM, stream,
                              red, half);
}

// Winograd 3x3 conv with the fused BatchNorm of the residual trunk (conv_wino.hip WinoBN):
// forward with `coef` (X = the BN input, U = ReLU(coef[0][col] x + coef[2][col]) built in the
// transform; `resid` optional) or dgrad with `mcoef` (mask = x); `spart` [B][2][S] per-board
// column statistics (forward: sum y, sum y^2; dgrad with smean: sum dU, sum dU (x - mean)).
// -5 when rag_conv_wino_bn_ok is false for the shape or the argument set has no kernel.
int rag_conv_wino_bn_launch(const void* X, const void* W, const float* bias, void* Y,
                            const void* mask, const void* res, int B, int S, int KIN, int NOUT,
                            int HO, int YC, int relu, int HM, hipStream_t stream,
                            const WgradRed* red, const float* coef, const float* mcoef,
                            float* spart, const float* smean);
RAG_API int rag_conv_wino_bn_ok(int B, int S, int KIN, int NOUT);
RAG_API int rag_conv_wino_bn(const void* X, const void* W, const float* bias, void* Y,
                             const void* mask, const void* resid, int B, int S, int KIN, int NOUT,
                             int HO, int YC, int relu, int HM, hipStream_t stream, void* pending,
                             const float* coef, const float* mcoef, float* spart,
                             const float* smean) {
  if (!rag_conv_wino_bn_ok(B, S, KIN, NOUT) || YC < NOUT || (coef != nullptr) == (mcoef != nullptr) ||
      (mcoef && (!mask || resid)) || (smean && !mcoef))
    return -5;  // (checked before the pending reduction is taken)
  WgradRed pend;
  const WgradRed* red = nullptr;
  if (const int rc = wino_pending(pending, stream, NOUT, &pend, &red)) return rc;
  return rag_conv_wino_bn_launch(X, W, bias, Y, mask, resid, B, S, KIN, NOUT, HO, YC, relu, HM,
                                 stream, red, coef, mcoef, spart, smean);
}

// Partial rows rag_conv_igemm_bn writes to `spart` (one per convolution block).
RAG_API int rag_conv_bn_stat_blocks(int B, int S, int COUTP) {
  return ((B * S * S + 383) / 384) * (COUTP / 128);
}

static int conv_igemm_impl(const void* X, const void* W, const float* bias, void* Y,
                           const void* mask, const void* resid, int B, int S, int HI, int HO,
                           int CIN, int COUTP, int YC, int KS, int relu, int HM,
                           hipStream_t stream, void* pending, const float* bnc,
                           const float* mcoef, float* spart, const float* smean) {
  if (CIN % 32 || COUTP % 32 || YC < COUTP || HI < KS / 2) return -1;
  const int M = B * S * S;
  const int nt = pick_nt(COUTP);
  dim3 grid((M + kBM - 1) / kBM, COUTP / (32 * nt));
  const int WI = S + 2 * HI, WO = S + 2 * HO, shift = HI - KS / 2;
  const bf16* x = (const bf16*)X;
  const bf16* w = (const bf16*)W;
  bf16* y = (bf16*)Y;
  const bf16* mk = (const bf16*)mask;
  const bf16* res = (const bf16*)resid;
  WgradRed pend;
  hipStream_t pend_stream = nullptr;
  const WgradRed* red = nullptr;
  if (take_pending(pending, &pend, &pend_stream)) {
    if (pend_stream == stream) {
      red = &pend;  // rides along this launch (or goes out on its own just below)
    } else {
      const int rc = rag_launch_wgrad_slab_reduce(pend, pend_stream);
      if (rc) return rc;
    }
  }
  if (bnc || mcoef || spart) {  // BN fusion: the 128-channel ping-pong kernel or nothing
    if (rag_conv_tap_launch(x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, KS,
                            relu, HM, (long)B * WI * WI, stream, red, bnc, mcoef, spart, smean))
      return (int)hipGetLastError();
    if (red) rag_launch_wgrad_slab_reduce(*red, stream);
    return -5;
  }
  if (rag_conv_tap_launch(x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN,
                                      COUTP, YC, KS, relu, HM, (long)B * WI * WI, stream, red,
                                      nullptr, nullptr, nullptr, nullptr))
    return (int)hipGetLastError();
  if (red) {  // not a tap-slab launch: the reduction goes out on its own first
    const int rc = rag_launch_wgrad_slab_reduce(*red, stream);
    if (rc) return rc;
  }
  if (rag_conv_pipe_launch(x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN,
                                       COUTP, YC, KS, relu, HM, stream))
    return (int)hipGetLastError();
  switch (KS) {
    case 1: launch_igemm_ks<1>(nt, grid, stream, x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM); break;
    case 3: launch_igemm_ks<3>(nt, grid, stream, x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM); break;
    case 5: launch_igemm_ks<5>(nt, grid, stream, x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM); break;
    case 7: launch_igemm_ks<7>(nt, grid, stream, x, w, bias, y, mk, res, M, S, WI, shift, WO, HO, CIN, COUTP, YC, relu, HM); break;
    default: return -2;
  }
  return (int)hipGetLastError();
}

// Workspace (floats) needed by rag_conv_wgrad for the partial slabs.
int rag_launch_wgrad_taps(const bf16* G, const bf16* X, float* part, float* bpart, int R, int WP,
                          int GC, int CIN, int spc, int COUTP, int CINP, int KS, int RG,
                          int nchunks, hipStream_t stream);  // wgrad.hip
bool rag_wgrad_taps_fits(int WP, int KS, int RG);  // wgrad.hip
int rag_wgrad_taps_target_blocks();  // wgrad.hip
bool rag_wgrad_slab_ok(int S, int H, int HG, int GC, int COUTP, int CINP, int KS);  // wgrad_slab.hip
int rag_wgrad_slab_nchunks(int R, int CINP, int* spc, int KS, int pair5 = 0);     // wgrad_slab.hip
bool rag_wgrad_slab_bf16();                                                        // wgrad_slab.hip
WgradRed rag_wgrad_slab_red(const void* part, const float* bpart, float* dW, float* db,
                            int nchunks, int CINP, int COUTP, int COUT, int CIN, int accumulate,
                            int KS, int pair5);
int rag_launch_wgrad_slab_reduce(const WgradRed& r, hipStream_t stream);        // wgrad_slab.hip
int rag_launch_wgrad_slab(const bf16* G, const bf16* X, float* part, float* bpart, int R, int WP,
                          int GC, int CIN, int spc, int CINP, int nchunks, hipStream_t stream,
                          const float* xcoef, int S, int KS, int COUTP, int pair5,
                          unsigned* ticket_reset);

namespace {
// all-taps variant applicability and plan (see wgrad.hip)
struct TapsPlan {
  bool ok;
  int rg, nchunks, spc;
};
TapsPlan taps_plan(int B, int S, int H, int HG, int COUTP, int CINP, int KS) {
  TapsPlan p{false, 1, 1, 1};
  if (H != HG || H < KS / 2 || COUTP % 64 || CINP % 64) return p;
  const int WP = S + 2 * H;
  const int rg = (KS == 3) ? 3 : 1;
  if (!rag_wgrad_taps_fits(WP, KS, rg)) return p;
  const int R = B * WP * WP;
  const int steps = (R + 63) / 64;
  const int per_chunk = (KS / rg) * (COUTP / 64) * (CINP / 64);
  int nc = rag_wgrad_taps_target_blocks() / per_chunk;  // one full wave of resident blocks
  if (nc > steps) nc = steps;
  if (nc < 1) nc = 1;
  p.ok = true;
  p.rg = rg;
  p.spc = (steps + nc - 1) / nc;
  p.nchunks = (steps + p.spc - 1) / p.spc;
  return p;
}
int gather_nchunks(int B, int S, int COUTP, int CINP, int KS) {
  const int M = B * S * S;
  const int taps = KS * KS;
  const int ntn = COUTP % 192 == 0 ? 6 : (COUTP % 128 == 0 ? 4 : (COUTP % 64 == 0 ? 2 : 1));
  const int ntc = CINP % 96 == 0 ? 3 : (CINP % 64 == 0 ? 2 : 1);
  const int tiles = taps * (COUTP / (32 * ntn)) * (CINP / (32 * ntc));
  const int msteps = (M + 63) / 64;
  int nc = (512 + tiles - 1) / tiles;
  if (nc > msteps) nc = msteps;
  if (nc < 1) nc = 1;
  return nc;
}
}  // namespace

// Upper bound (floats) of the wgrad workspace over both kernel variants and halos <= 3.
RAG_API size_t rag_conv_wgrad_workspace(int B, int S, int COUTP, int CINP, int KS, int* nchunks) {
  const int taps = KS * KS;
  int nc = gather_nchunks(B, S, COUTP, CINP, KS);
  for (int H = 1; H <= 3; ++H) {
    TapsPlan tp = taps_plan(B, S, H, H, COUTP, CINP, KS);
    if (tp.ok && tp.nchunks > nc) nc = tp.nchunks;
  }
  for (int H = 1; H <= 2; ++H) {
    if (rag_wgrad_slab_ok(S, H, H, COUTP, COUTP, CINP, KS)) {
      for (int pr = 0; pr <= 1; ++pr) {  // the 5x5 row-paired grid has more chunks
        const int sn = rag_wgrad_slab_nchunks(B * (S + 2 * H) * (S + 2 * H), CINP, nullptr, KS,
                                              pr);
        if (sn > nc) nc = sn;
      }
    }
  }
  if (nchunks) *nchunks = nc;
  return (size_t)nc * taps * COUTP * CINP + (size_t)nc * COUTP;
}

template <int KS>
static void launch_wgrad_ks(int ntn, int ntc, dim3 grid, hipStream_t st, const bf16* G,
                            const bf16* X, float* part, float* bpart, int M, int S, int WI,
                            int shift, int WG, int HG, int GC, int CIN, int spc, int COUTP,
                            int CINP, int ntile_c) {
#define RAG_WG(A, C)                                                                          \
  if (ntn == A && ntc == C) {                                                                 \
    conv_wgrad_kernel<KS, A, C><<<grid, 256, 0, st>>>(G, X, part, bpart, M, S, WI, shift, WG, \
                                                      HG, GC, CIN, spc, COUTP, CINP, ntile_c);\
    return;                                                                                   \
  }
  RAG_WG(6, 3) RAG_WG(6, 2) RAG_WG(6, 1) RAG_WG(4, 3) RAG_WG(4, 2) RAG_WG(4, 1)
  RAG_WG(2, 3) RAG_WG(2, 2) RAG_WG(2, 1) RAG_WG(1, 3) RAG_WG(1, 2) RAG_WG(1, 1)
#undef RAG_WG
}

// Weight + bias gradient. G: dL/d(pre-activation) in padded layout (halo 1, GC channels).
// X: the layer input (halo HI, CINP channels). dW: OIHW fp32 [COUT][CIN][KS][KS]. db: [COUT].
static int conv_wgrad_impl(const void* G, const void* X, float* dW, float* db, float* work,
                           int B, int S, int HI, int HG, int GC, int COUT, int COUTP, int CIN,
                           int CINP, int KS, int accumulate, hipStream_t stream,
                           hipStream_t reduce_stream, void* pending,
                           const float* xcoef = nullptr) {
  {  // a pending reduction reads the partial slabs this wgrad is about to overwrite
    const int rc = flush_pending(pending, nullptr);
    if (rc) return rc;
  }
  const bool defer = pending != nullptr;
  if (COUTP % 32 || CINP % 32) return -1;
  const int taps = KS * KS;
  const bf16* g = (const bf16*)G;
  const bf16* x = (const bf16*)X;
  TapsPlan tp = taps_plan(B, S, HI, HG, COUTP, CINP, KS);
  int nchunks;
  float* part = work;
  float* bpart;
  bool bf16_part = false;
  const bool slab = rag_wgrad_slab_ok(S, HI, HG, GC, COUTP, CINP, KS);
  if (xcoef && !(slab && KS == 3 && rag_wgrad_slab_bf16() && CINP == 128)) return -5;
  // 5x5 with <= 48 real of 64 input channels (the SL input layer): c-tile 1's blocks pair two
  // kernel rows instead of computing a zero c-fragment
  const int pair5 = KS == 5 && CINP == 64 && CIN <= 48 && !xcoef ? 1 : 0;
  if (slab) {
    bf16_part = rag_wgrad_slab_bf16();
    const int WP = S + 2 * HI;
    const int R = B * WP * WP;
    int spc = 1;
    nchunks = rag_wgrad_slab_nchunks(R, CINP, &spc, KS, pair5);
    bpart = db ? work + (size_t)nchunks * taps * COUTP * CINP : nullptr;
    // a reduction deferred on this stream gets claim counters, zeroed by this launch (so a
    // claiming launch that ended early cannot leave the next one a stale ticket)
    unsigned* ticket_reset = nullptr;
    if (defer && bf16_part && !(reduce_stream && reduce_stream != stream)) {
      PendingRed* p = static_cast<PendingRed*>(pending);
      if (!p->dticket && hipMalloc(&p->dticket, 2 * sizeof(unsigned)) != hipSuccess) return -3;
      ticket_reset = p->dticket;
    }
    const int rc = rag_launch_wgrad_slab(g, x, part, bpart, R, WP, GC, CINP, spc, CINP, nchunks,
                                         stream, xcoef, S, KS, COUTP, pair5, ticket_reset);
    if (rc) return rc;
  } else if (tp.ok) {
    nchunks = tp.nchunks;
    bpart = db ? work + (size_t)nchunks * taps * COUTP * CINP : nullptr;
    const int WP = S + 2 * HI;
    const int rc = rag_launch_wgrad_taps(g, x, part, bpart, B * WP * WP, WP, GC, CINP, tp.spc,
                                         COUTP, CINP, KS, tp.rg, nchunks, stream);
    if (rc) return rc;
  } else {
    nchunks = gather_nchunks(B, S, COUTP, CINP, KS);
    const int M = B * S * S;
    const int ntn = COUTP % 192 == 0 ? 6 : (COUTP % 128 == 0 ? 4 : (COUTP % 64 == 0 ? 2 : 1));
    const int ntc = CINP % 96 == 0 ? 3 : (CINP % 64 == 0 ? 2 : 1);
    const int ntile_n = COUTP / (32 * ntn), ntile_c = CINP / (32 * ntc);
    const int msteps = (M + 63) / 64;
    const int spc = (msteps + nchunks - 1) / nchunks;
    bpart = db ? work + (size_t)nchunks * taps * COUTP * CINP : nullptr;
    dim3 grid(nchunks * ntile_n * ntile_c * taps);
    const int WI = S + 2 * HI, shift = HI - KS / 2, WG = S + 2 * HG;
    switch (KS) {
      case 1: launch_wgrad_ks<1>(ntn, ntc, grid, stream, g, x, part, bpart, M, S, WI, shift, WG, HG, GC, CINP, spc, COUTP, CINP, ntile_c); break;
      case 3: launch_wgrad_ks<3>(ntn, ntc, grid, stream, g, x, part, bpart, M, S, WI, shift, WG, HG, GC, CINP, spc, COUTP, CINP, ntile_c); break;
      case 5: launch_wgrad_ks<5>(ntn, ntc, grid, stream, g, x, part, bpart, M, S, WI, shift, WG, HG, GC, CINP, spc, COUTP, CINP, ntile_c); break;
      case 7: launch_wgrad_ks<7>(ntn, ntc, grid, stream, g, x, part, bpart, M, S, WI, shift, WG, HG, GC, CINP, spc, COUTP, CINP, ntile_c); break;
      default: return -2;
    }
  }
  // The slab reduce is bandwidth-bound while the next kernels (dgrad) are MFMA-bound: with a
  // separate reduce stream it runs concurrently with them, ordered after this wgrad by an event.
  hipStream_t rs = stream;
  if (reduce_stream && reduce_stream != stream) {
    static hipEvent_t ring[16];
    static int next = 0;
    hipEvent_t& ev = ring[next];
    next = (next + 1) & 15;
    if (!ev && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return -3;
    if (hipEventRecord(ev, stream) != hipSuccess) return -3;
    if (hipStreamWaitEvent(reduce_stream, ev, 0) != hipSuccess) return -3;
    rs = reduce_stream;
  }
  if (bf16_part) {
    const WgradRed r = rag_wgrad_slab_red(part, bpart, dW, db, nchunks, CINP, COUTP, COUT, CIN,
                                          accumulate, KS, slab ? pair5 : 0);
    if (defer && rs == stream) {
      PendingRed* p = static_cast<PendingRed*>(pending);
      p->r = r;
      // the riding reduce blocks claim units dynamically (launches that keep the static split
      // clear the ticket) through the handle's counters, which the slab launch above zeroed
      p->r.ticket = p->dticket;
      p->stream = stream;
      p->valid = 1;
      return 0;
    }
    return rag_launch_wgrad_slab_reduce(r, rs);
  }
  const int total = taps * COUTP * CINP / 4 + COUTP;
  const int blocks = (total + 255) / 256;  // 4 chunk loads in flight per thread (8 / 16: same)
  wgrad_reduce_kernel<4><<<blocks, 256, 0, rs>>>(part, bpart, dW, db, nchunks, taps, COUT, CIN,
                                                 COUTP, CINP, KS, accumulate);
  return (int)hipGetLastError();
}

RAG_API int rag_conv_wgrad(const void* G, const void* X, float* dW, float* db, float* work,
                           int B, int S, int HI, int HG, int GC, int COUT, int COUTP, int CIN,
                           int CINP, int KS, int accumulate, hipStream_t stream,
                           hipStream_t reduce_stream) {
  return conv_wgrad_impl(G, X, dW, db, work, B, S, HI, HG, GC, COUT, COUTP, CIN, CINP, KS,
                         accumulate, stream, reduce_stream, nullptr);
}

// As rag_conv_wgrad, but an fp16 partial-slab reduction is left pending in the caller's handle
// for the next conv launch given that handle on `stream`; dW / db are complete once that launch
// (or rag_wgrad_flush(handle)) ran. A reduction already pending in the handle is launched first.
RAG_API int rag_conv_wgrad_deferred(const void* G, const void* X, float* dW, float* db,
                                    float* work, int B, int S, int HI, int HG, int GC, int COUT,
                                    int COUTP, int CIN, int CINP, int KS, int accumulate,
                                    hipStream_t stream, void* pending) {
  if (!pending) return -4;
  return conv_wgrad_impl(G, X, dW, db, work, B, S, HI, HG, GC, COUT, COUTP, CIN, CINP, KS,
                         accumulate, stream, nullptr, pending);
}

// As rag_conv_wgrad_deferred with the BN prologue: X is the BN input x and the layer input is
// U = ReLU(xcoef[0][col] * x + xcoef[2][col]) (-5 if the shape has no fused kernel).
RAG_API int rag_conv_wgrad_deferred_bn(const void* G, const void* X, float* dW, float* db,
                                       float* work, int B, int S, int HI, int HG, int GC, int COUT,
                                       int COUTP, int CIN, int CINP, int KS, int accumulate,
                                       hipStream_t stream, void* pending, const float* xcoef) {
  if (!xcoef) return -5;
  return conv_wgrad_impl(G, X, dW, db, work, B, S, HI, HG, GC, COUT, COUTP, CIN, CINP, KS,
                         accumulate, stream, nullptr, pending, xcoef);
}

RAG_API int rag_pack_weights(const float* W, void* Wf, void* Wb, int COUT, int CIN, int KS,
                             int COUTP, int CINP, hipStream_t stream) {
  const int total = KS * KS * COUTP * CINP;
  const int blocks = (total + 255) / 256 < 2048 ? (total + 255) / 256 : 2048;
  pack_weights_kernel<<<blocks, 256, 0, stream>>>(W, (bf16*)Wf, (bf16*)Wb, COUT, CIN, KS, COUTP,
                                                  CINP);
  return (int)hipGetLastError();
}

// One launch that repacks every layer of a trunk after an optimizer step: for each layer the
// bf16 forward / dgrad GEMM layouts of its OIHW fp32 weights and the padded fp32 bias (pack.h
// pack_trunk_block: table layout, tiling). The whole SL-style step's repack (with the Winograd
// layers and the rest of the optimizer step) is one launch instead: conv_wino.hip rag_pack_step.
namespace {
__global__ void __launch_bounds__(256) pack_trunk_kernel(const int64_t* __restrict__ table,
                                                         int nrows, int nfull, SgdFold sgd) {
  __shared__ float tl[pack_trunk_lds(kPTaps)];  // [tap][n][c]
  pack_trunk_block(table, (int)blockIdx.y, nrows, nfull, sgd, (int)blockIdx.x, (int)gridDim.x,
                   kPTaps, tl);
}
}  // namespace

// lr, wd, goff (elements from a master weight to its gradient), sgd_on: the optimizer step
// folded into the packing (each master element is stepped by exactly one thread)
RAG_API int rag_pack_trunk(const int64_t* table, int nrows, int nfull, int64_t total,
                           hipStream_t stream, int64_t goff, float lr, float wd, int sgd_on) {
  // total: the grid width (blocks per layer row; each grid-strides over its layer's 16x16 tiles).
  // Rows [0, nfull) pack weights (one grid row each); rows [nfull, nrows) only pad their bias
  // (Winograd layers: rag_wino_pack packs the weights) and share one grid row: the 11 bias-only
  // rows of the SL trunk were 11 x 200 blocks that exited at once.
  if (nrows <= 0 || nfull < 0 || nfull > nrows || total <= 0 || total % 8) return -1;
  const dim3 grid((unsigned)total, (unsigned)(nfull + (nrows > nfull ? 1 : 0)));
  pack_trunk_kernel<<<grid, 256, 0, stream>>>(table, nrows, nfull,
                                              SgdFold{(long)goff, lr, wd, sgd_on});
  return (int)hipGetLastError();
}

RAG_API int rag_pack_input_u8(const uint8_t* F, const int64_t* index, const int* tf, void* X,
                              int B, int NF, int FS, int S, int H, int CP, hipStream_t stream) {
  if (FS < NF) return -1;
  if (NF <= kPackInMaxC && S * S <= kPackInMaxS2 && CP <= kPackInMaxC && B > 0) {
    pack_input_lds_kernel<uint8_t><<<B, kPackInThreads, 0, stream>>>(F, index, tf, (bf16*)X, NF, FS,
                                                                     S, H, CP);
    return (int)hipGetLastError();
  }
  const int total = B * S * S * (CP / 8);
  const int blocks = (total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192;
  pack_input_kernel<uint8_t><<<blocks, 256, 0, stream>>>(F, index, tf, (bf16*)X, B, NF, FS, S, H,
                                                         CP);
  return (int)hipGetLastError();
}

RAG_API int rag_pack_input_bits(const uint64_t* Fb, const int64_t* index, const int* tf, void* X,
                                int B, int NF, int S, int H, int CP, hipStream_t stream) {
  if (NF > 64) return -1;
  const int total = B * S * S * (CP / 8);
  const int blocks = (total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192;
  pack_input_bits_kernel<<<blocks, 256, 0, stream>>>(Fb, index, tf, (bf16*)X, B, NF, S, H, CP);
  return (int)hipGetLastError();
}

RAG_API int rag_pack_input_f32(const float* F, const int64_t* index, const int* tf, void* X,
                               int B, int NF, int FS, int S, int H, int CP, hipStream_t stream) {
  if (FS < NF) return -1;
  if (NF <= kPackInMaxC && S * S <= kPackInMaxS2 && CP <= kPackInMaxC && B > 0) {
    pack_input_lds_kernel<float><<<B, kPackInThreads, 0, stream>>>(F, index, tf, (bf16*)X, NF, FS,
                                                                   S, H, CP);
    return (int)hipGetLastError();
  }
  const int total = B * S * S * (CP / 8);
  const int blocks = (total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192;
  pack_input_kernel<float><<<blocks, 256, 0, stream>>>(F, index, tf, (bf16*)X, B, NF, FS, S, H, CP);
  return (int)hipGetLastError();
}

RAG_API int rag_unpack(const void* X, float* out, int B, int C, int S, int H, int CP,
                       hipStream_t stream) {
  const int total = B * C * S * S;
  const int blocks = (total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096;
  unpack_kernel<<<blocks, 256, 0, stream>>>((const bf16*)X, out, B, C, S, H, CP);
  return (int)hipGetLastError();
}

RAG_API int rag_pack_nchw(const float* in, void* X, int B, int C, int S, int H, int CP,
                          hipStream_t stream) {
  const int total = B * S * S * CP;
  const int blocks = (total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096;
  pack_nchw_kernel<<<blocks, 256, 0, stream>>>(in, (bf16*)X, B, C, S, H, CP);
  return (int)hipGetLastError();
}

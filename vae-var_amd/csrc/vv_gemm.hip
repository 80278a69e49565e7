// fp32 GEMM on gfx950 MFMA (v_mfma_f32_32x32x2_f32): C = epi(A . B^T), B = nn.Linear weight [N][K].
//
// Every nn.Linear of the Swin-U-Net (networks_old/utils/swinblock.py:105,115 qkv/proj, :18-20 fc1/fc2,
// networks_old/transformer.py:73 PatchMerging.reduction, :103 PatchExpand.expand, :435 concat_back_dim,
// :552 Enc_net.proj, :596 Dec_net.proj) runs through this one kernel, forward with W [N][K] and the
// input-gradient backward with the pre-transposed W^T [K][N].
//
// Tile: BM x BN x 32, 256 threads = 4 waves as WM x WN, each wave TM x TN MFMA tiles of 32x32.
// k mapping inside a 32-deep k-tile: MFMA step s (0..15), lane half h uses k = 16h + s, so each lane
// reads 4 consecutive k of its row with one ds_read_b128 (rows padded to 36 floats: conflict-free).
// Double-buffered LDS, register-staged global prefetch of tile t+1 during the MFMAs of tile t,
// one barrier per k-tile.
#include "vv_kernels.h"

#include <algorithm>

namespace vv {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float dgelu_f(float x) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
  const float pdf = 0.39894228040143268f * expf(-0.5f * x * x);
  return cdf + x * pdf;
}

constexpr int KALIGN = 32;  // K, ksplit granularity accepted by gemm_nt (covers every BK variant)

// GEMM epilogue. 32x32: acc[a][b][r] -> row (r&3) + 8(r>>2) + 4h, col lane&31; 16x16: row 4h + r,
// col lane&15 (h = lane>>4). Everything an element needs (bias, output row, residual, pre-activation) is
// loaded for the whole fragment first, so the stores are not serialised behind one dependent load each;
// FULL tiles skip all bounds checks.
template <int BM, int BN, int WM, int WN, int EPI, int MF, bool FULL, typename ACC>
__device__ __forceinline__ void epilogue(const GemmArgs& args, const GemmGroup& G, ACC& acc, int m0, int n0, int wm,
                                         int wn, int rin, int hh) {
  constexpr int TM = BM / WM / MF;
  constexpr int TN = BN / WN / MF;
  constexpr int NR = MF == 32 ? 16 : 4;
  const int M = args.M, N = args.N;
  float bv[TN];
  int colv[TN];
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    colv[b] = n0 + wn * TN * MF + b * MF + rin;
    const int cc = FULL ? colv[b] : min(colv[b], N - 1);
    bv[b] = G.bias ? G.bias[cc] : 0.0f;
  }
#pragma unroll
  for (int a = 0; a < TM; ++a) {
    int ov[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int row = m0 + wm * TM * MF + a * MF + (MF == 32 ? (r & 3) + 8 * (r >> 2) + 4 * hh : 4 * hh + r);
      const int rc = FULL ? row : min(row, M - 1);
      ov[r] = args.crow ? args.crow[rc] : rc;
    }
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int col = FULL ? colv[b] : min(colv[b], N - 1);
      float ex[NR];
      if constexpr (EPI == EPI_RESID) {
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          const int rr = args.rmod > 0 ? ov[r] % args.rmod : ov[r];
          ex[r] = G.R[(size_t)rr * args.ldr + col];
        }
      } else if constexpr (EPI == EPI_DGELU) {
#pragma unroll
        for (int r = 0; r < NR; ++r) ex[r] = G.aux[(size_t)ov[r] * args.ldaux + col];
      }
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        if (!FULL) {
          const int row = m0 + wm * TM * MF + a * MF + (MF == 32 ? (r & 3) + 8 * (r >> 2) + 4 * hh : 4 * hh + r);
          if (row >= M || colv[b] >= N) continue;
        }
        const int o = ov[r];
        float v = acc[a][b][r] + bv[b];
        if constexpr (EPI == EPI_GELU) {
          G.aux[(size_t)o * args.ldaux + col] = v;
          v = gelu_f(v);
        } else if constexpr (EPI == EPI_RESID) {
          v = ex[r] + v;
        } else if constexpr (EPI == EPI_DGELU) {
          v = acc[a][b][r] * dgelu_f(ex[r]);
        }
        G.C[(size_t)o * args.ldc + col] = v;
      }
    }
  }
}

// XCD-aware tile order: the dispatcher deals consecutive workgroups round-robin over the 8 XCDs; remap so
// XCD x gets a contiguous range of logical tiles (M-major), i.e. a band of A rows that its 4 MB L2 serves
// to all of its CUs (cdna_hip_programming.md T1, bijective form for tile counts not divisible by 8).
__device__ __forceinline__ int xcd_remap(int bid, int nt) {
  const int q = nt >> 3, r = nt & 7, x = bid & 7, l = bid >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + l;
}

// Grouped tile order for the split kernels: logical tile t walks the GM m-blocks of its group first, then
// the n-blocks, so a contiguous range of logical tiles (what xcd_remap hands one XCD) covers a compact
// GM x (range/GM) block of the output and its A/B panels are re-read from that XCD's L2, not the fabric.
constexpr int kGroupM = 8;
__device__ __forceinline__ void tile_mn(int t, int ntm, int ntn, int& mb, int& nb) {
  const int g = t / (kGroupM * ntn), m0 = g * kGroupM;
  const int gm = min(kGroupM, ntm - m0), r = t - g * kGroupM * ntn;
  mb = m0 + r % gm;
  nb = r / gm;
}

template <int BM, int BN, int BK, int WM, int WN, int EPI, bool XCD, int MF, int DEPTH>
__global__ __launch_bounds__(64 * WM * WN) void k_gemm_nt(GemmArgs args) {
  constexpr int NT = 64 * WM * WN;
  constexpr int LS = BK + 4;        // LDS row stride (floats): rows land on distinct 16-B slots
  constexpr int TPR = BK / 4;       // threads per staged row (float4 each)
  constexpr int RPP = NT / TPR;     // rows per staging pass
  constexpr int TM = BM / WM / MF;   // MFMA tiles per wave
  constexpr int TN = BN / WN / MF;
  constexpr int AI = BM / RPP;
  constexpr int BI = BN / RPP;
  constexpr int KG = 64 / MF;        // lane groups along k: 2 (32x32x2) or 4 (16x16x4)
  constexpr int HALF = BK / KG;      // lane group h takes k in [h*HALF, (h+1)*HALF)
  typedef float accv __attribute__((ext_vector_type(MF == 32 ? 16 : 4)));
  static_assert(AI >= 1 && BI >= 1 && AI * RPP == BM && BI * RPP == BN, "staging shape");
  static_assert(TM >= 1 && TN >= 1, "wave tile");
  extern __shared__ __attribute__((aligned(16))) float smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const GemmGroup G = args.g[blockIdx.z];
  const int M = args.M, N = args.N, K = args.K, ksplit = args.ksplit;
  const int ntn = (N + BN - 1) / BN;
  const int ntiles = ntn * ((M + BM - 1) / BM);
  const int nkt = K / BK;
  int tile, kb = 0, ke = nkt, part = -1;
  if ((int)blockIdx.x < args.tdp || args.tsplit <= 1) {
    tile = XCD ? xcd_remap(blockIdx.x, ntiles) : blockIdx.x;
  } else {
    part = blockIdx.x - args.tdp;  // tail item: tile tdp + part / S, k-chunk part % S
    const int S = args.tsplit, c = part % S;
    tile = args.tdp + part / S;
    kb = (c * nkt) / S;
    ke = ((c + 1) * nkt) / S;
  }
  const int m0 = (tile / ntn) * BM, n0 = (tile % ntn) * BN;
  const int lr = tid / TPR, lc = (tid % TPR) * 4;

  const float* a1p[AI];
  const float* a2p[AI];
  const float* bp[BI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int r = min(m0 + lr + RPP * i, M - 1);
    const int ar = args.arow ? args.arow[r] : r;
    a1p[i] = G.A + (size_t)ar * args.lda + lc;
    a2p[i] = G.A2 ? G.A2 + (size_t)r * args.lda2 + lc - ksplit : a1p[i];
  }
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int n = min(n0 + lr + RPP * i, N - 1);
    bp[i] = G.B + (size_t)n * (args.ldb ? args.ldb : K) + lc;
  }

  // register staging sets (named, statically indexed): DEPTH 1 = tile t+1 in flight during tile t,
  // DEPTH 2 = tiles t+1 (landed, written to LDS after the compute) and t+2 (in flight)
  f4 ra0[AI], rb0[BI], ra1[AI], rb1[BI];
  auto gload = [&](int k0, f4 (&ra)[AI], f4 (&rb)[BI]) {
    if (k0 < ksplit) {
#pragma unroll
      for (int i = 0; i < AI; ++i) ra[i] = *reinterpret_cast<const f4*>(a1p[i] + k0);
    } else {
#pragma unroll
      for (int i = 0; i < AI; ++i) ra[i] = *reinterpret_cast<const f4*>(a2p[i] + k0);
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) rb[i] = *reinterpret_cast<const f4*>(bp[i] + k0);
  };
  auto sstore = [&](int buf, const f4 (&ra)[AI], const f4 (&rb)[BI]) {
    float* As = smem + buf * (BM + BN) * LS;
    float* Bs = As + BM * LS;
#pragma unroll
    for (int i = 0; i < AI; ++i) *reinterpret_cast<f4*>(As + (lr + RPP * i) * LS + lc) = ra[i];
#pragma unroll
    for (int i = 0; i < BI; ++i) *reinterpret_cast<f4*>(Bs + (lr + RPP * i) * LS + lc) = rb[i];
  };

  const int wm = wave / WN, wn = wave % WN;
  const int rin = lane & (MF - 1), hh = lane / MF;
  constexpr int NR = MF == 32 ? 16 : 4;
  accv acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < NR; ++r) acc[a][b][r] = 0.0f;

  auto compute = [&](int buf) {
    const float* As = smem + buf * (BM + BN) * LS + (wm * TM * MF + rin) * LS + hh * HALF;
    const float* Bs = smem + buf * (BM + BN) * LS + BM * LS + (wn * TN * MF + rin) * LS + hh * HALF;
#pragma unroll
    for (int kq = 0; kq < HALF / 4; ++kq) {
      f4 af[TM], bf[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) af[a] = *reinterpret_cast<const f4*>(As + a * MF * LS + kq * 4);
#pragma unroll
      for (int b = 0; b < TN; ++b) bf[b] = *reinterpret_cast<const f4*>(Bs + b * MF * LS + kq * 4);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b) {
            if constexpr (MF == 32)
              acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a][s], bf[b][s], acc[a][b], 0, 0, 0);
            else
              acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[a][s], bf[b][s], acc[a][b], 0, 0, 0);
          }
    }
  };

  const int nk = ke - kb;
  if constexpr (DEPTH == 1) {
    gload(kb * BK, ra0, rb0);
    sstore(0, ra0, rb0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) gload((kb + kt + 1) * BK, ra0, rb0);
      compute(cur);
      if (kt + 1 < nk) sstore(cur ^ 1, ra0, rb0);
      __syncthreads();
    }
  } else {
    static_assert(DEPTH == 1 || DEPTH == 2, "depth");
    // prologue: tile 0 -> LDS buffer 0, tile 1 -> registers set 1
    gload(kb * BK, ra0, rb0);
    if (nk > 1) gload((kb + 1) * BK, ra1, rb1);
    sstore(0, ra0, rb0);
    __syncthreads();
    // steady state, unrolled by two so each register set is named statically
    for (int kt = 0; kt < nk; kt += 2) {
      // even step: compute buf 0 (tile kt); set 1 holds tile kt+1; load tile kt+2 into set 0
      if (kt + 2 < nk) gload((kb + kt + 2) * BK, ra0, rb0);
      compute(0);
      if (kt + 1 < nk) sstore(1, ra1, rb1);
      __syncthreads();
      if (kt + 1 >= nk) break;
      // odd step: compute buf 1 (tile kt+1); set 0 holds tile kt+2; load tile kt+3 into set 1
      if (kt + 3 < nk) gload((kb + kt + 3) * BK, ra1, rb1);
      compute(1);
      if (kt + 2 < nk) sstore(0, ra0, rb0);
      __syncthreads();
    }
  }

  // epilogue: 32x32: acc[a][b][r] -> row (r&3) + 8(r>>2) + 4h, col lane&31;
  //           16x16: row 4h + r, col lane&15 (h = lane>>4)
  // Everything an element needs (bias, output row, residual, pre-activation) is loaded for the whole
  // fragment first, so the stores are not serialised behind one dependent load each.
  if (part >= 0) {
    // tail chunk: raw fp32 partial, register-major [TM*TN*NR][NT] so the fixup reads it coalesced
    float* w = args.ws + ((size_t)blockIdx.z * (gridDim.x - args.tdp) + part) * (size_t)(TM * TN * NR * NT);
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b)
#pragma unroll
        for (int r = 0; r < NR; ++r) w[(size_t)((a * TN + b) * NR + r) * NT + tid] = acc[a][b][r];
    return;
  }
  if (m0 + BM <= M && n0 + BN <= N)
    epilogue<BM, BN, WM, WN, EPI, MF, true>(args, G, acc, m0, n0, wm, wn, rin, hh);
  else
    epilogue<BM, BN, WM, WN, EPI, MF, false>(args, G, acc, m0, n0, wm, wn, rin, hh);
}

// Tail fixup: sums the tsplit k-chunk partials of each tail tile in chunk order (deterministic) and applies
// the same epilogue as the main kernel. grid = (tail tiles, 1, groups), same block shape as the main kernel.
template <int BM, int BN, int WM, int WN, int EPI, int MF, bool GROUPED = false>
__global__ __launch_bounds__(64 * WM * WN) void k_gemm_fixup(GemmArgs args) {
  constexpr int NT = 64 * WM * WN;
  constexpr int TM = BM / WM / MF;
  constexpr int TN = BN / WN / MF;
  constexpr int NR = MF == 32 ? 16 : 4;
  constexpr int NREG = TM * TN * NR;
  typedef float accv __attribute__((ext_vector_type(MF == 32 ? 16 : 4)));
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const GemmGroup G = args.g[blockIdx.z];
  const int M = args.M, N = args.N;
  const int ntn = (N + BN - 1) / BN;
  const int S = args.tsplit;
  const int tile = args.tdp + blockIdx.x;
  int mb = tile / ntn, nb = tile % ntn;
  if (GROUPED) tile_mn(tile, (M + BM - 1) / BM, ntn, mb, nb);
  const int m0 = mb * BM, n0 = nb * BN;
  const size_t items = (size_t)gridDim.x * S;
  const float* w = args.ws + ((size_t)blockIdx.z * items + (size_t)blockIdx.x * S) * (size_t)(NREG * NT);
  accv acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const size_t j = (size_t)((a * TN + b) * NR + r) * NT + tid;
        float v = w[j];
        for (int c = 1; c < S; ++c) v += w[(size_t)c * NREG * NT + j];
        acc[a][b][r] = v;
      }
  const int wm = wave / WN, wn = wave % WN;
  const int rin = lane & (MF - 1), hh = lane / MF;
  if (m0 + BM <= M && n0 + BN <= N)
    epilogue<BM, BN, WM, WN, EPI, MF, true>(args, G, acc, m0, n0, wm, wn, rin, hh);
  else
    epilogue<BM, BN, WM, WN, EPI, MF, false>(args, G, acc, m0, n0, wm, wn, rin, hh);
}

// ---------------------------------------------------------------------------------------------------------
// fp32 GEMM as six bf16 MFMA products (v_mfma_f32_32x32x16_bf16, 16x the f32 MFMA rate on gfx950).
//
// Each fp32 operand is split exactly into three bf16 planes, x = h + m + l (each residual is exact in fp32
// and 3 x 8 significant bits cover fp32's 24), and
//   a.b = h_a h_b + h_a m_b + m_a h_b + h_a l_b + l_a h_b + m_a m_b  (+ terms ~2^-24 |a b|, dropped)
// is accumulated in fp32 by the MFMA; products of bf16 values are exact in fp32, so the result carries
// fp32-level error (measured against fp64: tests/test_gpu_kernels.py::test_gemm_split_accuracy) at
// 16/6 = 2.67x the fp32-MFMA arithmetic rate.
//
// Weights (B) are split once at load time into three bf16 planes (split_planes, round-to-nearest; per row
// [h | m | l] x K, so any row block of a registered weight, e.g. one source of a torch.cat, has planes) and
// staged by plain 16-B copies; activations (A) are split while staging the k-tile into LDS by truncation
// (h = x & 0xffff0000, m = (x - h) & 0xffff0000, l = x - h - m: four VALU ops and 1.5 byte-permutes per
// element, once per workgroup, never per MFMA). LDS: per buffer 3 planes x (BM + BN) rows x 32 bf16 (64-B
// rows), 16-B chunk c of row r stored at chunk c ^ ((r >> 2) & 3): the ds_read_b128 lane groups of a 32-row
// fragment ({0-3,12-15,20-27}, ...) land on 16 distinct 16-B slots and every 128-B write window (two
// consecutive rows) on 32 distinct banks (MI355X_MICROARCH.md §LDS).
// Fragment (32x32x16): lane l reads row l&31, k = 8(l>>5) .. +7 of one plane; A and B share the k map.
// Same tile/item scheme (data-parallel rounds + split-K tail + fixup) and epilogues as k_gemm_nt.
typedef __bf16 bf8v __attribute__((ext_vector_type(8)));
typedef unsigned int u2v __attribute__((ext_vector_type(2)));
typedef unsigned int u4v __attribute__((ext_vector_type(4)));

// 4 fp32 -> h, m, l bf16 planes (4 elements each, packed in 2 dwords), truncation split
__device__ __forceinline__ void split3t(const f4& x, u2v& h, u2v& m, u2v& l) {
  unsigned xb[4], mb[4], lb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    xb[i] = __float_as_uint(x[i]);
    const float r1 = x[i] - __uint_as_float(xb[i] & 0xffff0000u);
    mb[i] = __float_as_uint(r1);
    lb[i] = __float_as_uint(r1 - __uint_as_float(mb[i] & 0xffff0000u));
  }
  h[0] = __builtin_amdgcn_perm(xb[1], xb[0], 0x07060302u);
  h[1] = __builtin_amdgcn_perm(xb[3], xb[2], 0x07060302u);
  m[0] = __builtin_amdgcn_perm(mb[1], mb[0], 0x07060302u);
  m[1] = __builtin_amdgcn_perm(mb[3], mb[2], 0x07060302u);
  l[0] = __builtin_amdgcn_perm(lb[1], lb[0], 0x07060302u);
  l[1] = __builtin_amdgcn_perm(lb[3], lb[2], 0x07060302u);
}

__global__ void k_split_planes(const float* __restrict__ src, unsigned short* __restrict__ dst, size_t n, int K) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float x = src[i];
    const __bf16 h = (__bf16)x;
    const float r1 = x - (float)h;
    const __bf16 m = (__bf16)r1;
    const __bf16 l = (__bf16)(r1 - (float)m);
    const size_t row = i / K, k = i % K;
    unsigned short* d = dst + row * 3 * K + k;
    d[0] = __builtin_bit_cast(unsigned short, h);
    d[K] = __builtin_bit_cast(unsigned short, m);
    d[2 * K] = __builtin_bit_cast(unsigned short, l);
  }
}

hipError_t split_planes(const float* src, unsigned short* dst, size_t n, int K, hipStream_t s) {
  if (!n) return hipSuccess;
  if (K <= 0 || n % K) return hipErrorInvalidValue;
  const int blocks = (int)std::min<size_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(k_split_planes, dim3(blocks), dim3(256), 0, s, src, dst, n, K);
  return hipGetLastError();
}

template <int BM, int BN, int WM, int WN, int EPI, bool BPRE, int DEPTH, int NBUF, bool APRE = false>
__global__ __launch_bounds__(64 * WM * WN) void k_gemm_bs(GemmArgs args) {
  constexpr int BK = 32;
  constexpr int NT = 64 * WM * WN;
  constexpr int LSB = BK;                   // bf16 per LDS row (XOR-swizzled 16-B chunks)
  constexpr int PLANE = (BM + BN) * LSB;    // bf16 per plane (A rows then B rows)
  constexpr int TPR = BK / 4;               // fp32 staging: threads per row (float4 each)
  constexpr int RPP = NT / TPR;
  constexpr int TM = BM / WM / 32;
  constexpr int TN = BN / WN / 32;
  constexpr int AI = APRE ? 1 : BM / RPP;   // fp32 A staging (split in the kernel)
  constexpr int AQ = BM * 4 / NT;           // plane A staging: 16-B chunks per thread per plane
  constexpr int BI = BPRE ? 1 : BN / RPP;   // fp32 B staging (no planes)
  constexpr int BQ = BN * 4 / NT;           // plane B staging: 16-B chunks per thread per plane
  typedef float accv __attribute__((ext_vector_type(16)));
  static_assert(APRE ? (AQ >= 1 && AQ * NT == BM * 4) : (AI >= 1 && AI * RPP == BM), "A staging shape");
  static_assert(BPRE ? (BQ >= 1 && BQ * NT == BN * 4) : (BI >= 1 && BI * RPP == BN), "B staging shape");
  static_assert(TM >= 1 && TN >= 1, "wave tile");
  extern __shared__ __attribute__((aligned(16))) unsigned short lds16[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const GemmGroup G = args.g[blockIdx.z];
  const int M = args.M, N = args.N, K = args.K, ksplit = args.ksplit;
  const int ntn = (N + BN - 1) / BN, ntm = (M + BM - 1) / BM;
  const int nkt = K / BK;
  int tile, kb = 0, ke = nkt, part = -1;
  if (args.tsplit <= 1) {
    tile = xcd_remap(blockIdx.x, ntm * ntn);
  } else if ((int)blockIdx.x < args.tdp) {
    tile = xcd_remap(blockIdx.x, args.tdp);
  } else {
    part = blockIdx.x - args.tdp;
    const int S = args.tsplit, c = part % S;
    tile = args.tdp + part / S;
    kb = (c * nkt) / S;
    ke = ((c + 1) * nkt) / S;
  }
  int mb, nb;
  tile_mn(tile, ntm, ntn, mb, nb);
  const int m0 = mb * BM, n0 = nb * BN;
  const int lr = tid / TPR, lc = (tid % TPR) * 4;
  // LDS element offset of (row, k) within a plane: 16-B chunk k/8 XOR-swizzled by (row >> 2) & 3
  auto swz = [](int row, int k) { return row * LSB + ((((k >> 3) ^ (row >> 2)) & 3) << 3) + (k & 7); };

  const float* a1p[AI];
  const float* a2p[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int r = min(m0 + lr + RPP * i, M - 1);
    const int ar = args.arow ? args.arow[r] : r;
    a1p[i] = G.A + (size_t)ar * args.lda + lc;
    a2p[i] = G.A2 ? G.A2 + (size_t)r * args.lda2 + lc - ksplit : a1p[i];
  }
  const unsigned short* aq[AQ > 0 ? AQ : 1];
  if constexpr (APRE) {
#pragma unroll
    for (int i = 0; i < AQ; ++i) {
      const int c = tid + NT * i;
      const int r = min(m0 + c / 4, M - 1);
      const int ar = args.arow ? args.arow[r] : r;
      aq[i] = G.Ap + (size_t)ar * 3 * args.lda + (c % 4) * 8;
    }
  }
  const float* bp[BI];
  const unsigned short* bq[BQ > 0 ? BQ : 1];
  if constexpr (BPRE) {
#pragma unroll
    for (int i = 0; i < BQ; ++i) {
      const int c = tid + NT * i;
      const int n = min(n0 + c / 4, N - 1);
      bq[i] = G.Bp + (size_t)n * 3 * K + (c % 4) * 8;
    }
  } else {
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int n = min(n0 + lr + RPP * i, N - 1);
      bp[i] = G.B + (size_t)n * (args.ldb ? args.ldb : K) + lc;
    }
  }
  const size_t ps = K;  // planes of one B row: [h | m | l] x K

  struct Stg {
    f4 ra[AI], rb[BI];
    u4v rq[BQ > 0 ? BQ : 1][3];
    u4v qa[AQ > 0 ? AQ : 1][3];
  };
  auto gload = [&](int k0, Stg& st) {
    if constexpr (APRE) {
#pragma unroll
      for (int i = 0; i < AQ; ++i)
#pragma unroll
        for (int p = 0; p < 3; ++p) st.qa[i][p] = *reinterpret_cast<const u4v*>(aq[i] + p * args.lda + k0);
    } else if (k0 < ksplit) {
#pragma unroll
      for (int i = 0; i < AI; ++i) st.ra[i] = *reinterpret_cast<const f4*>(a1p[i] + k0);
    } else {
#pragma unroll
      for (int i = 0; i < AI; ++i) st.ra[i] = *reinterpret_cast<const f4*>(a2p[i] + k0);
    }
    if constexpr (BPRE) {
#pragma unroll
      for (int i = 0; i < BQ; ++i)
#pragma unroll
        for (int p = 0; p < 3; ++p) st.rq[i][p] = *reinterpret_cast<const u4v*>(bq[i] + p * ps + k0);
    } else {
#pragma unroll
      for (int i = 0; i < BI; ++i) st.rb[i] = *reinterpret_cast<const f4*>(bp[i] + k0);
    }
  };
  auto sstore = [&](int buf, const Stg& st) {
    unsigned short* P = lds16 + buf * 3 * PLANE;
    u2v h, m, l;
    if constexpr (APRE) {
#pragma unroll
      for (int i = 0; i < AQ; ++i) {
        const int c = tid + NT * i;
        const int o = swz(c / 4, (c % 4) * 8);
#pragma unroll
        for (int p = 0; p < 3; ++p) *reinterpret_cast<u4v*>(P + p * PLANE + o) = st.qa[i][p];
      }
    }
#pragma unroll
    for (int i = 0; i < (APRE ? 0 : AI); ++i) {
      split3t(st.ra[i], h, m, l);
      const int o = swz(lr + RPP * i, lc);
      *reinterpret_cast<u2v*>(P + o) = h;
      *reinterpret_cast<u2v*>(P + PLANE + o) = m;
      *reinterpret_cast<u2v*>(P + 2 * PLANE + o) = l;
    }
    if constexpr (BPRE) {
#pragma unroll
      for (int i = 0; i < BQ; ++i) {
        const int c = tid + NT * i;
        const int o = swz(BM + c / 4, (c % 4) * 8);
#pragma unroll
        for (int p = 0; p < 3; ++p) *reinterpret_cast<u4v*>(P + p * PLANE + o) = st.rq[i][p];
      }
    } else {
#pragma unroll
      for (int i = 0; i < BI; ++i) {
        split3t(st.rb[i], h, m, l);
        const int o = swz(BM + lr + RPP * i, lc);
        *reinterpret_cast<u2v*>(P + o) = h;
        *reinterpret_cast<u2v*>(P + PLANE + o) = m;
        *reinterpret_cast<u2v*>(P + 2 * PLANE + o) = l;
      }
    }
  };

  const int wm = wave / WN, wn = wave % WN;
  const int rin = lane & 31, hh = lane >> 5;
  accv acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.0f;

  auto compute = [&](int buf) {
    const unsigned short* P = lds16 + buf * 3 * PLANE;
    // fragment rows start at multiples of 32, so the swizzle term is (rin >> 2) & 3 for every fragment.
    // All fragments of the k-tile are read first (one LDS latency per k-tile), then the MFMAs run back to
    // back; without the sched_barrier the compiler re-uses fragment registers and waits on every read.
    const unsigned short* As = P + (wm * TM * 32 + rin) * LSB;
    const unsigned short* Bs = P + (BM + wn * TN * 32 + rin) * LSB;
    bf8v fa[2][TM][3], fb[2][TN][3];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ck = ((2 * s + hh) ^ ((rin >> 2) & 3)) * 8;
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int p = 0; p < 3; ++p) fa[s][a][p] = *reinterpret_cast<const bf8v*>(As + p * PLANE + a * 32 * LSB + ck);
#pragma unroll
      for (int b = 0; b < TN; ++b)
#pragma unroll
        for (int p = 0; p < 3; ++p) fb[s][b][p] = *reinterpret_cast<const bf8v*>(Bs + p * PLANE + b * 32 * LSB + ck);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          // smallest terms first
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][a][2], fb[s][b][0], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][a][0], fb[s][b][2], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][a][1], fb[s][b][1], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][a][1], fb[s][b][0], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][a][0], fb[s][b][1], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][a][0], fb[s][b][0], acc[a][b], 0, 0, 0);
        }
  };

  const int nk = ke - kb;
  if constexpr (NBUF == 1) {
    // one LDS buffer (several workgroups per CU): store -> barrier -> compute -> barrier; the next tile's
    // global loads (DEPTH tiles ahead) are in flight during the compute
    Stg s0, s1;
    gload(kb * BK, s0);
    if (DEPTH == 2 && nk > 1) gload((kb + 1) * BK, s1);
    for (int kt = 0; kt < nk; kt += DEPTH) {
      sstore(0, s0);
      __syncthreads();
      if (kt + DEPTH < nk) gload((kb + kt + DEPTH) * BK, s0);
      compute(0);
      __syncthreads();
      if constexpr (DEPTH == 2) {
        if (kt + 1 >= nk) break;
        sstore(0, s1);
        __syncthreads();
        if (kt + 3 < nk) gload((kb + kt + 3) * BK, s1);
        compute(0);
        __syncthreads();
      }
    }
  } else if constexpr (DEPTH == 1) {
    Stg s0;
    gload(kb * BK, s0);
    sstore(0, s0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) gload((kb + kt + 1) * BK, s0);
      compute(cur);
      if (kt + 1 < nk) sstore(cur ^ 1, s0);
      __syncthreads();
    }
  } else {
    // two LDS buffers, two register sets: tile t+1's loads were issued two computes before its store
    Stg s0, s1;
    gload(kb * BK, s0);
    if (nk > 1) gload((kb + 1) * BK, s1);
    sstore(0, s0);
    __syncthreads();
    for (int kt = 0; kt < nk; kt += 2) {
      if (kt + 2 < nk) gload((kb + kt + 2) * BK, s0);
      compute(0);
      if (kt + 1 < nk) sstore(1, s1);
      __syncthreads();
      if (kt + 1 >= nk) break;
      if (kt + 3 < nk) gload((kb + kt + 3) * BK, s1);
      compute(1);
      if (kt + 2 < nk) sstore(0, s0);
      __syncthreads();
    }
  }

  if (part >= 0) {
    float* w = args.ws + ((size_t)blockIdx.z * (gridDim.x - args.tdp) + part) * (size_t)(TM * TN * 16 * NT);
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) w[(size_t)((a * TN + b) * 16 + r) * NT + tid] = acc[a][b][r];
    return;
  }
  if (m0 + BM <= M && n0 + BN <= N)
    epilogue<BM, BN, WM, WN, EPI, 32, true>(args, G, acc, m0, n0, wm, wn, rin, hh);
  else
    epilogue<BM, BN, WM, WN, EPI, 32, false>(args, G, acc, m0, n0, wm, wn, rin, hh);
}

template <int BM, int BN, int WM, int WN, int EPI, bool BPRE, int DEPTH, int NBUF, bool APRE = false>
static hipError_t launch_bs_k(const GemmArgs& a, hipStream_t s, dim3 grid, size_t lds, int tail) {
  static bool init = false;
  if (!init) {
    hipError_t e = hipFuncSetAttribute((const void*)k_gemm_bs<BM, BN, WM, WN, EPI, BPRE, DEPTH, NBUF, APRE>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    init = true;
  }
  hipLaunchKernelGGL((k_gemm_bs<BM, BN, WM, WN, EPI, BPRE, DEPTH, NBUF, APRE>), grid, dim3(64 * WM * WN), lds, s, a);
  if (tail)
    hipLaunchKernelGGL((k_gemm_fixup<BM, BN, WM, WN, EPI, 32, true>), dim3(tail, 1, a.ngroups), dim3(64 * WM * WN),
                       0, s, a);
  return hipGetLastError();
}

template <int BM, int BN, int WM, int WN, int DEPTH = 1, int NBUF = 2>
static hipError_t launch_bs(const GemmArgs& a, hipStream_t s) {
  constexpr int BK = 32;
  if (a.K % BK || a.ksplit % BK) return hipErrorInvalidValue;
  const size_t lds = NBUF * 3 * (BM + BN) * BK * sizeof(unsigned short);
  const int T = ((a.N + BN - 1) / BN) * ((a.M + BM - 1) / BM);
  const int tail = a.tsplit > 1 ? T - a.tdp : 0;
  dim3 grid(tail ? a.tdp + tail * a.tsplit : T, 1, a.ngroups);
  bool pre = true, apre = true;
  for (int g = 0; g < a.ngroups; ++g) {
    pre = pre && a.g[g].Bp;
    apre = apre && a.g[g].Ap;
  }
  if (pre && apre && a.epi == EPI_STORE) return launch_bs_k<BM, BN, WM, WN, EPI_STORE, true, DEPTH, NBUF, true>(a, s, grid, lds, tail);
  switch (a.epi * 2 + (pre ? 1 : 0)) {
#define VV_EPI(E)                                                                    \
  case 2 * E: return launch_bs_k<BM, BN, WM, WN, E, false, DEPTH, NBUF>(a, s, grid, lds, tail); \
  case 2 * E + 1: return launch_bs_k<BM, BN, WM, WN, E, true, DEPTH, NBUF>(a, s, grid, lds, tail);
    VV_EPI(EPI_STORE)
    VV_EPI(EPI_GELU)
    VV_EPI(EPI_RESID)
    VV_EPI(EPI_DGELU)
#undef VV_EPI
    default:
      return hipErrorInvalidValue;
  }
}

template <int BM, int BN, int BK, int WM, int WN, bool XCD = false, int MF = 32, int DEPTH = 1>
static hipError_t launch_tile(const GemmArgs& a, hipStream_t s) {
  constexpr int LS = BK + 4;
  if (a.K % BK || a.ksplit % BK) return hipErrorInvalidValue;
  const size_t lds = 2 * (BM + BN) * LS * sizeof(float);
  const int T = ((a.N + BN - 1) / BN) * ((a.M + BM - 1) / BM);
  const int tail = a.tsplit > 1 ? T - a.tdp : 0;
  dim3 grid(tail ? a.tdp + tail * a.tsplit : T, 1, a.ngroups);
  switch (a.epi) {
#define VV_EPI(E)                                                                                   \
  case E: {                                                                                         \
    static bool init = false;                                                                       \
    if (!init) {                                                                                    \
      hipError_t e = hipFuncSetAttribute((const void*)k_gemm_nt<BM, BN, BK, WM, WN, E, XCD, MF, DEPTH>,             \
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);     \
      if (e != hipSuccess) return e;                                                                \
      init = true;                                                                                  \
    }                                                                                               \
    hipLaunchKernelGGL((k_gemm_nt<BM, BN, BK, WM, WN, E, XCD, MF, DEPTH>), grid, dim3(64 * WM * WN), lds, s, a);   \
    if (tail)                                                                                       \
      hipLaunchKernelGGL((k_gemm_fixup<BM, BN, WM, WN, E, MF>), dim3(tail, 1, a.ngroups), dim3(64 * WM * WN), 0, \
                         s, a);                                                                     \
    return hipGetLastError();                                                                       \
  }
    VV_EPI(EPI_STORE)
    VV_EPI(EPI_GELU)
    VV_EPI(EPI_RESID)
    VV_EPI(EPI_DGELU)
#undef VV_EPI
    default:
      return hipErrorInvalidValue;
  }
}

// tile variants (index = tile hint)
static hipError_t launch_variant(int t, const GemmArgs& a, hipStream_t s) {
  switch (t) {
    case 0: return launch_tile<128, 128, 32, 2, 2>(a, s);
    case 1: return launch_tile<128, 64, 32, 2, 2>(a, s);
    case 2: return launch_tile<64, 64, 32, 2, 2>(a, s);
    case 3: return launch_tile<64, 64, 16, 2, 2>(a, s);
    case 4: return launch_tile<32, 64, 32, 1, 2>(a, s);
    case 5: return launch_tile<64, 32, 32, 2, 1>(a, s);
    case 6: return launch_tile<64, 128, 32, 2, 2>(a, s);
    case 7: return launch_tile<32, 64, 16, 1, 2>(a, s);
    case 8: return launch_tile<64, 64, 64, 2, 2>(a, s);
    case 9: return launch_tile<64, 64, 32, 2, 2, true>(a, s);     // 2 with the XCD remap
    case 10: return launch_tile<64, 64, 32, 2, 2, false, 16>(a, s);   // 16x16x4 MFMA
    case 11: return launch_tile<128, 64, 32, 2, 2, false, 16>(a, s);
    case 12: return launch_tile<64, 128, 32, 2, 2, false, 16>(a, s);
    case 13: return launch_tile<128, 128, 32, 2, 2, false, 16>(a, s);
    case 14: return launch_tile<64, 64, 16, 2, 2, false, 16>(a, s);
    case 15: return launch_tile<32, 64, 32, 1, 2, false, 16>(a, s);
    case 16: return launch_tile<64, 64, 32, 2, 2, false, 32, 2>(a, s);    // 2-deep register prefetch
    case 17: return launch_tile<64, 128, 32, 2, 2, false, 32, 2>(a, s);
    case 18: return launch_tile<32, 64, 32, 1, 2, false, 32, 2>(a, s);
    case 19: return launch_tile<64, 64, 64, 2, 2, false, 32, 2>(a, s);
    case 20: return launch_tile<64, 64, 16, 2, 2, false, 32, 2>(a, s);
    // bf16x6 split (fp32-accurate) variants
    case 21: return launch_bs<128, 128, 2, 4>(a, s);
    case 22: return launch_bs<128, 128, 2, 2>(a, s);
    case 23: return launch_bs<128, 64, 2, 2>(a, s);
    case 24: return launch_bs<64, 64, 2, 2>(a, s);
    case 25: return launch_bs<64, 128, 2, 2>(a, s);
    case 26: return launch_bs<128, 64, 2, 1>(a, s);
    case 27: return launch_bs<128, 128, 2, 4, 2, 2>(a, s);   // 2-deep register prefetch
    case 28: return launch_bs<128, 128, 2, 4, 1, 1>(a, s);   // one LDS buffer: 2 WGs / CU
    case 29: return launch_bs<64, 64, 2, 2, 2, 2>(a, s);
    case 30: return launch_bs<128, 64, 2, 2, 2, 2>(a, s);
    case 31: return launch_bs<128, 128, 2, 2, 1, 1>(a, s);
    case 32: return launch_bs<128, 128, 2, 4, 2, 1>(a, s);
    case 33: return launch_bs<64, 128, 2, 2, 2, 2>(a, s);
    default: return hipErrorInvalidValue;
  }
}

static long tiles_of(const GemmArgs& a, int bm, int bn) {
  return (long)((a.M + bm - 1) / bm) * ((a.N + bn - 1) / bn) * a.ngroups;
}

// tile choice (measured on MI355X, tools/gemm_bench.py; 4 WGs/CU resident): high-occupancy 64x64 tiles beat
// larger tiles on every decoder shape at M = 2048 / 8192; 32x64 when 64x64 leaves CUs idle

static int g_num_cu = 0;
static int g_math = GEMM_SPLIT;
void set_gemm_math(int m) { g_math = m; }
int gemm_math() { return g_math; }

struct SplitArena {
  const float* base;
  size_t n;
  const unsigned short* planes;
};
static SplitArena g_split[16];
static int g_nsplit = 0;

void register_split_arena(const float* base, size_t n, const unsigned short* planes) {
  unregister_split_arena(base);
  if (g_nsplit < 16) g_split[g_nsplit++] = {base, n, planes};
}
void unregister_split_arena(const float* base) {
  for (int i = 0; i < g_nsplit; ++i)
    if (g_split[i].base == base) {
      g_split[i] = g_split[--g_nsplit];
      return;
    }
}
static const unsigned short* split_planes_of(const float* B) {
  for (int i = 0; i < g_nsplit; ++i)
    if (B >= g_split[i].base && B < g_split[i].base + g_split[i].n) return g_split[i].planes + 3 * (size_t)(B - g_split[i].base);
  return nullptr;
}
constexpr size_t kWsFloats = (size_t)1 << 21;  // 8 MB: tail partials of up to 512 chunks of a 64x64 tile

size_t gemm_ws_floats() { return kWsFloats; }

// tile choice (measured on MI355X, tools/gemm_bench.py, tools/gemm_split_check.py)
static int pick_tile(const GemmArgs& a) {
  if (g_math == GEMM_SPLIT) {
    // 128x128 with 64x64 per wave, one LDS buffer (2 WGs / CU) when it fills the chip; else 64x64
    if (tiles_of(a, 128, 128) >= 256) return 31;
    return 24;
  }
  // f32 MFMA: high-occupancy 64x64 tiles beat larger tiles on every decoder shape at M = 2048 / 8192;
  // 32x64 when 64x64 leaves CUs idle
  if (tiles_of(a, 64, 64) >= 512) return 2;
  return 4;
}

// tile edge of each variant (for the tail split)
static void variant_tile(int t, int& bm, int& bn, int& bk) {
  static const int tab[][3] = {{128, 128, 32}, {128, 64, 32}, {64, 64, 32}, {64, 64, 16}, {32, 64, 32}, {64, 32, 32},
                               {64, 128, 32}, {32, 64, 16}, {64, 64, 64}, {64, 64, 32}, {64, 64, 32}, {128, 64, 32},
                               {64, 128, 32}, {128, 128, 32}, {64, 64, 16}, {32, 64, 32}, {64, 64, 32}, {64, 128, 32},
                               {32, 64, 32}, {64, 64, 64}, {64, 64, 16}, {128, 128, 32}, {128, 128, 32},
                               {128, 64, 32}, {64, 64, 32}, {64, 128, 32}, {128, 64, 32}, {128, 128, 32},
                               {128, 128, 32}, {64, 64, 32}, {128, 64, 32}, {128, 128, 32}, {128, 128, 32},
                               {64, 128, 32}};
  bm = tab[t][0];
  bn = tab[t][1];
  bk = tab[t][2];
}

hipError_t gemm_nt(const GemmArgs& a_in, hipStream_t s, int tile_hint, float* ws) {
  GemmArgs a = a_in;
  if (a.M <= 0 || a.N <= 0 || a.ngroups <= 0 || a.ngroups > kMaxGroups) return hipErrorInvalidValue;
  if (a.K % KALIGN != 0 || a.ksplit % KALIGN != 0 || a.ksplit <= 0 || a.ksplit > a.K) return hipErrorInvalidValue;
  if ((a.lda & 3) || (a.lda2 & 3) || (a.K & 3) || (a.ldb & 3) || (a.ldb && a.ldb < a.K)) return hipErrorInvalidValue;
  const int t = tile_hint >= 0 ? tile_hint : pick_tile(a);
  if (t < 0 || t > 33) return hipErrorInvalidValue;
  // data-parallel rounds of whole tiles + the remaining tiles split along K over the idle CUs
  if (!g_num_cu) {
    int dev = 0;
    hipDeviceProp_t p;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&p, dev) == hipSuccess) g_num_cu = p.multiProcessorCount;
    if (g_num_cu <= 0) g_num_cu = 256;
  }
  a.tdp = 0;
  a.tsplit = 1;
  a.ws = ws;
  for (int g = 0; g < a.ngroups; ++g) {
    a.g[g].Bp = (t >= 21 && (!a.ldb || a.ldb == a.K)) ? split_planes_of(a.g[g].B) : nullptr;
    a.g[g].Ap = (t >= 21 && !a.g[g].A2 && !a.g[g].Ap) ? split_planes_of(a.g[g].A) : a.g[g].Ap;
  }
  if (ws && a.ngroups == 1) {
    int bm, bn, bk;
    variant_tile(t, bm, bn, bk);
    const int T = ((a.N + bn - 1) / bn) * ((a.M + bm - 1) / bm);
    const int P = g_num_cu, nkt = a.K / bk;
    const int tdp = (T / P) * P, tail = T - tdp;
    if (tdp > 0 && tail > 0 && tail <= P / 2) {
      // chunks of >= 12 k-tiles: below that the fixup launch and partial traffic cost more than the tail
      int S = std::min(P / tail, nkt / 12);
      const size_t tile_f = (size_t)bm * bn;
      while (S > 1 && (size_t)tail * S * tile_f > kWsFloats) --S;
      if (S > 1) {
        a.tdp = tdp;
        a.tsplit = S;
      }
    }
  }
  const int ph = prof_begin(s);
  const hipError_t e = launch_variant(t, a, s);
  // algorithmic: 2MNK flops; bytes = A + B + C (+R/aux) once each
  const double G = a.ngroups;
  double bytes = 4.0 * G * ((double)a.M * a.K + (double)a.N * a.K + (double)a.M * a.N);
  if (a.epi == EPI_RESID || a.epi == EPI_GELU || a.epi == EPI_DGELU) bytes += 4.0 * G * (double)a.M * a.N;
  prof_end(ph, s, PC_GEMM, 2.0 * G * a.M * a.N * a.K, bytes);
  return e;
}

}  // namespace vv

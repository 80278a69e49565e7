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
#include "vv_gelu.h"
#include "vv_kernels.h"
#include "vv_lanes.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <mutex>
#include <utility>
#include <vector>

namespace vv {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float gelu_f(float x) { return gelu_fast(x); }  // vv_gelu.h
__device__ __forceinline__ float dgelu_f(float x) { return dgelu_fast(x); }

constexpr int KALIGN = 32;  // K, ksplit granularity accepted by gemm_nt (covers every BK variant)

// dynamic-LDS limit of a kernel, set once per (kernel, device): hipFuncSetAttribute acts on the current device
hipError_t set_lds_limit(const void* k, size_t lds) {
  static std::mutex mu;
  static std::vector<std::pair<const void*, int>> done;
  int dev = 0;
  if (hipError_t e = hipGetDevice(&dev)) return e;
  std::lock_guard<std::mutex> lk(mu);
  for (auto& d : done)
    if (d.first == k && d.second == dev) return hipSuccess;
  if (hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)) return e;
  done.emplace_back(k, dev);
  return hipSuccess;
}

// compute units of the current device (cached per device)
int device_cus() {
  static std::mutex mu;
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  std::lock_guard<std::mutex> lk(mu);
  if (!cus[dev]) {
    hipDeviceProp_t p;
    cus[dev] = (hipGetDeviceProperties(&p, dev) == hipSuccess && p.multiProcessorCount > 0) ? p.multiProcessorCount : 256;
  }
  return cus[dev];
}


// GEMM epilogue. 32x32: acc[a][b][r] -> row (r&3) + 8(r>>2) + 4h, col lane&31; 16x16: row 4h + r,
// col lane&15 (h = lane>>4). Everything an element needs (bias, output row, residual, pre-activation) is
// loaded for the whole fragment first, so the stores are not serialised behind one dependent load each;
// FULL tiles skip all bounds checks. The optional bias and row-map loads are issued unconditionally (from a
// dummy address, G.A, when the pointer is null) and selected afterwards: a load under a branch leaves the
// compiler unable to count outstanding memory operations, and it then waits for ALL of them (vmcnt(0)) --
// the next tile's prefetched A in a persistent kernel, and in partial tiles every previous store.
// Plane-writing forms of GELU / DGELU (tile 48 only, GemmArgs.opl): the value v of each element is stored as the
// fp16x3 planes of the next GEMM's A, h = fp16(v s), l = fp16(v s - h) (k_rowsplit's arithmetic), with the row
// scale s = 2^e chosen from the bound U_r (GemmArgs.opl) so that 2 U_r s < 2^15: every tile of a row derives the
// same s from the same inputs, so no row maximum crosses tiles. s only moves the planes' exponent, so the planes
// equal k_rowsplit's (up to the power of two the consumer undoes) unless an l part falls below fp16's normal range.
constexpr int EPI_GELU_PL = 4, EPI_DGELU_PL = 5;

template <int BM, int BN, int WM, int WN, int EPI_, int MF, bool FULL, typename ACC>
__device__ __forceinline__ void epilogue(const GemmArgs& args, const GemmGroup& G, ACC& acc, int m0, int n0, int wm,
                                         int wn, int rin, int hh) {
  constexpr bool PL = EPI_ == EPI_GELU_PL || EPI_ == EPI_DGELU_PL;
  constexpr int EPI = EPI_ == EPI_GELU_PL ? EPI_GELU : EPI_ == EPI_DGELU_PL ? EPI_DGELU : EPI_;
  constexpr int TM = BM / WM / MF;
  constexpr int TN = BN / WN / MF;
  constexpr int NR = MF == 32 ? 16 : 4;
  const int M = args.M, N = args.N;
  float ubw = 0.f, ubb = 0.f;  // f K max|B|, f max|bias|
  if constexpr (PL) {
    const float tw = *args.obw, tb = *(args.obb ? args.obb : args.obw);
    constexpr float f = EPI == EPI_GELU ? 1.0f : 1.25f;
    ubw = f * (float)args.K * tw;
    ubb = args.obb ? f * tb : 0.0f;
  }
  float bv[TN];
  int colv[TN];
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    colv[b] = n0 + wn * TN * MF + b * MF + rin;
    const int cc = FULL ? colv[b] : min(colv[b], N - 1);
    const float t = *(G.bias ? G.bias + cc : G.A);
    bv[b] = G.bias ? t : 0.0f;
  }
#pragma unroll
  for (int a = 0; a < TM; ++a) {
    int ov[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int row = m0 + wm * TM * MF + a * MF + (MF == 32 ? (r & 3) + 8 * (r >> 2) + 4 * hh : 4 * hh + r);
      const int rc = FULL ? row : min(row, M - 1);
      const int t = *(args.crow ? args.crow + rc : reinterpret_cast<const int*>(G.A));
      ov[r] = args.crow ? t : rc;
    }
    float so[NR];  // plane forms: the row scales (GEMM row = output row: no crow)
    if constexpr (PL) {
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const float ia = __uint_as_float((254u << 23) - __float_as_uint(args.escale[ov[r]]));  // max|A_r| < 2^15 ia
        const unsigned mx = __float_as_uint(2.0f * (ubw * (32768.0f * ia) + ubb));
        so[r] = __uint_as_float((268u - max(mx >> 23, 15u)) << 23);
      }
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
          if (G.aux) G.aux[(size_t)o * args.ldaux + col] = v;  // the pre-activation, for a backward only
          v = gelu_f(v);
        } else if constexpr (EPI == EPI_RESID) {
          v = ex[r] + v;
        } else if constexpr (EPI == EPI_DGELU) {
          v = acc[a][b][r] * dgelu_f(ex[r]);
        }
        if constexpr (PL) {
          const float x = v * so[r];
          const _Float16 hv = (_Float16)x;
          const _Float16 lv = (_Float16)(x - (float)hv);
          unsigned short* pp = args.opl + (size_t)o * 2 * N + 2 * (col & ~31) + (col & 31);  // chunk-interleaved
          pp[0] = __builtin_bit_cast(unsigned short, hv);
          pp[32] = __builtin_bit_cast(unsigned short, lv);
          if (colv[b] == 0) args.ors[o] = so[r];
        } else {
          G.C[(size_t)o * args.ldc + col] = v;
        }
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
// gm > 0: the launch's group size (GemmArgs.gm, chosen per shape by gemm_nt); the kernels without it use kGroupM
__device__ __forceinline__ void tile_mn(int t, int ntm, int ntn, int& mb, int& nb, int GM = kGroupM) {
  GM = GM > 0 ? GM : kGroupM;
  const int g = t / (GM * ntn), m0 = g * GM;
  const int gm = min(GM, ntm - m0), r = t - g * GM * ntn;
  mb = m0 + r % gm;
  nb = r / gm;
}

template <int BM, int BN, int BK, int WM, int WN, int EPI, int MF>
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
    tile = blockIdx.x;
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

  // register staging: tile t+1 is in flight during the MFMAs of tile t
  f4 ra0[AI], rb0[BI];
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
  if (GROUPED) tile_mn(tile, (M + BM - 1) / BM, ntn, mb, nb, args.gm);
  const int m0 = mb * BM, n0 = nb * BN;
  const size_t items = (size_t)gridDim.x * S;
  const float* w = args.ws + ((size_t)blockIdx.z * items + (size_t)blockIdx.x * S) * (size_t)(NREG * NT);
  // all NREG loads of one chunk in flight together, chunks summed in order (bit-identical to a per-register
  // chain, one memory latency per chunk instead of one per register and chunk)
  accv acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < NR; ++r) acc[a][b][r] = w[(size_t)((a * TN + b) * NR + r) * NT + tid];
  for (int c = 1; c < S; ++c) {
    const float* wc = w + (size_t)c * NREG * NT;
    accv t[TM][TN];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b)
#pragma unroll
        for (int r = 0; r < NR; ++r) t[a][b][r] = wc[(size_t)((a * TN + b) * NR + r) * NT + tid];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) acc[a][b] += t[a][b];
  }
  const int wm = wave / WN, wn = wave % WN;
  const int rin = lane & (MF - 1), hh = lane / MF;
  if (m0 + BM <= M && n0 + BN <= N)
    epilogue<BM, BN, WM, WN, EPI, MF, true>(args, G, acc, m0, n0, wm, wn, rin, hh);
  else
    epilogue<BM, BN, WM, WN, EPI, MF, false>(args, G, acc, m0, n0, wm, wn, rin, hh);
}

// Split-K tail fixup, one workgroup per (tail tile, 32x32 sub-block (a, b)): each thread sums the S chunk
// partials of its 16 accumulator registers of that sub-block in chunk order (deterministic) and runs the
// epilogue on them; TM*TN times the parallelism of k_gemm_fixup for tiles with several sub-blocks per wave.
template <int BM, int BN, int WM, int WN, int EPI>
__global__ __launch_bounds__(64 * WM * WN) void k_gemm_fixup_sub(GemmArgs args) {
  constexpr int NT = 64 * WM * WN, TM = BM / WM / 32, TN = BN / WN / 32, NREG = TM * TN * 16;
  typedef float accv __attribute__((ext_vector_type(16)));
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const GemmGroup G = args.g[blockIdx.z];
  const int M = args.M, N = args.N;
  const int ntn = (N + BN - 1) / BN, ntm = (M + BM - 1) / BM;
  const int S = args.tsplit;
  const int tile = args.tdp + blockIdx.x;
  int mb, nb;
  tile_mn(tile, ntm, ntn, mb, nb, args.gm);
  const int a = blockIdx.y / TN, b = blockIdx.y % TN;
  const int wm = wave / WN, wn = wave % WN;
  const size_t items = (size_t)gridDim.x * S;
  const float* w = args.ws + ((size_t)blockIdx.z * items + (size_t)blockIdx.x * S) * (size_t)(NREG * NT);
  accv acc[1][1];
  const size_t j0 = (size_t)((a * TN + b) * 16) * NT + tid;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[0][0][r] = w[j0 + (size_t)r * NT];
  for (int c = 1; c < S; ++c) {  // one chunk's 16 loads in flight together, chunks summed in order
    const float* wc = w + (size_t)c * NREG * NT + j0;
    accv t;
#pragma unroll
    for (int r = 0; r < 16; ++r) t[r] = wc[(size_t)r * NT];
    acc[0][0] += t;
  }
  const int m0 = mb * BM + wm * TM * 32 + a * 32, n0 = nb * BN + wn * TN * 32 + b * 32;
  const int rin = lane & 31, hh = lane >> 5;
  if (m0 + 32 <= M && n0 + 32 <= N)
    epilogue<32, 32, 1, 1, EPI, 32, true>(args, G, acc, m0, n0, 0, 0, rin, hh);
  else
    epilogue<32, 32, 1, 1, EPI, 32, false>(args, G, acc, m0, n0, 0, 0, rin, hh);
}

// The same for the 16x16-MFMA layout (k_gemm_h3m / k_gemm_h4, 4 x 4 fragments of 16x16 per wave): one workgroup
// per (tail tile, fragment row a of every wave); each thread sums the S chunk partials of its 16 registers of the
// 16 x 64 strip (a, b = 0..3) in chunk order and runs the epilogue on the strip.
template <int BM, int BN, int WM, int WN, int EPI>
__global__ __launch_bounds__(64 * WM * WN) void k_gemm_fixup_sub16(GemmArgs args) {
  constexpr int NT = 64 * WM * WN, TM = BM / WM / 16, TN = BN / WN / 16, NREG = TM * TN * 4;
  typedef float accv __attribute__((ext_vector_type(4)));
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const GemmGroup G = args.g[blockIdx.z];
  const int M = args.M, N = args.N;
  const int ntn = (N + BN - 1) / BN, ntm = (M + BM - 1) / BM;
  const int S = args.tsplit;
  const int tile = args.tdp + blockIdx.x;
  int mb, nb;
  tile_mn(tile, ntm, ntn, mb, nb, args.gm);
  const int a = blockIdx.y;
  const int wm = wave / WN, wn = wave % WN;
  const size_t items = (size_t)gridDim.x * S;
  const float* w = args.ws + ((size_t)blockIdx.z * items + (size_t)blockIdx.x * S) * (size_t)(NREG * NT);
  accv acc[1][TN];
  const size_t j0 = (size_t)(a * TN * 4) * NT + tid;
#pragma unroll
  for (int b = 0; b < TN; ++b)
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[0][b][r] = w[j0 + (size_t)(b * 4 + r) * NT];
  for (int c = 1; c < S; ++c) {  // one chunk's loads in flight together, chunks summed in order
    const float* wc = w + (size_t)c * NREG * NT + j0;
    accv t[TN];
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) t[b][r] = wc[(size_t)(b * 4 + r) * NT];
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[0][b] += t[b];
  }
  const int m0 = mb * BM + wm * TM * 16 + a * 16, n0 = nb * BN + wn * TN * 16;
  const int rin = lane & 15, hh = lane >> 4;
  if (m0 + 16 <= M && n0 + TN * 16 <= N)
    epilogue<16, TN * 16, 1, 1, EPI, 16, true>(args, G, acc, m0, n0, 0, 0, rin, hh);
  else
    epilogue<16, TN * 16, 1, 1, EPI, 16, false>(args, G, acc, m0, n0, 0, 0, rin, hh);
}

// Tile 49's split-K fixup for a plain GEMM (r06: gemm_nt's N = 1152 split GEMMs on 64 tiles x 4 chunks = 256
// workgroups, as gemm_ln's): workgroup (tile, a) sums the S chunk partials of fragment row a of every wave in chunk
// order (k_gemm_h5 wrote element (row 32 wave + 16 a + 4 hh + r, column 16 b + rin) at ((a 9 + b) 4 + r) 512 + 64 wave
// + lane of partial tile S + c) and runs the GEMM's epilogue on the 16 x 144 rows of each wave
template <int EPI>
__global__ __launch_bounds__(512) void k_gemm_fixup49(GemmArgs args) {
  constexpr int TN = 9, PS = 2 * TN * 4 * 512;  // floats per partial
  typedef float accv __attribute__((ext_vector_type(4)));
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const GemmGroup G = args.g[0];
  const int M = args.M, N = args.N, ntn = (N + 143) / 144, ntm = (M + 255) / 256, S = args.tsplit;
  const int tile = blockIdx.x, a = blockIdx.y;
  int mb, nb;
  tile_mn(tile, ntm, ntn, mb, nb, args.gm);
  const float* w = args.ws + (size_t)tile * S * PS + (size_t)(a * TN * 4) * 512 + tid;
  accv acc[1][TN];
#pragma unroll
  for (int b = 0; b < TN; ++b)
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[0][b][r] = w[(size_t)(b * 4 + r) * 512];
  for (int c = 1; c < S; ++c) {  // one chunk's loads in flight together, chunks summed in order
    accv t[TN];
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) t[b][r] = w[(size_t)c * PS + (size_t)(b * 4 + r) * 512];
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[0][b] += t[b];
  }
  const int m0 = mb * 256 + wave * 32 + a * 16, n0 = nb * 144;
  const int rin = lane & 15, hh = lane >> 4;
  if (m0 + 16 <= M && n0 + 144 <= N)
    epilogue<16, 144, 1, 1, EPI, 16, true>(args, G, acc, m0, n0, 0, 0, rin, hh);
  else
    epilogue<16, 144, 1, 1, EPI, 16, false>(args, G, acc, m0, n0, 0, 0, rin, hh);
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

template <int BM, int BN, int WM, int WN, int EPI, bool BPRE, int NBUF, bool APRE = false>
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
  tile_mn(tile, ntm, ntn, mb, nb, args.gm);
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
  Stg s0;
  gload(kb * BK, s0);
  if constexpr (NBUF == 1) {
    // one LDS buffer (several workgroups per CU): store -> barrier -> compute -> barrier; the next tile's
    // global loads are in flight during the compute
    for (int kt = 0; kt < nk; ++kt) {
      sstore(0, s0);
      __syncthreads();
      if (kt + 1 < nk) gload((kb + kt + 1) * BK, s0);
      compute(0);
      __syncthreads();
    }
  } else if constexpr (NBUF == 2) {
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
    // NBUF 3 (r05, tile 26): the same two LDS buffers, but two register stages, so a k-tile's global loads are
    // issued two k-tiles before its LDS store (short-K launches: one k-tile's MFMAs, 12 per wave, do not cover a
    // load's latency). Unrolled by two so that the stages keep fixed registers.
    Stg s1;
    if (nk > 1) gload((kb + 1) * BK, s1);
    sstore(0, s0);
    __syncthreads();
    for (int kt = 0; kt < nk; kt += 2) {
      // s1 holds k-tile kt + 1, s0 is free
      if (kt + 2 < nk) gload((kb + kt + 2) * BK, s0);
      compute(0);
      if (kt + 1 < nk) sstore(1, s1);
      __syncthreads();
      if (kt + 1 >= nk) break;
      // s0 holds k-tile kt + 2, s1 is free
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

template <int BM, int BN, int WM, int WN, int EPI, bool BPRE, int NBUF, bool APRE = false>
static hipError_t launch_bs_k(const GemmArgs& a, hipStream_t s, dim3 grid, size_t lds, int tail) {
  if (hipError_t e = set_lds_limit((const void*)k_gemm_bs<BM, BN, WM, WN, EPI, BPRE, NBUF, APRE>, lds)) return e;
  hipLaunchKernelGGL((k_gemm_bs<BM, BN, WM, WN, EPI, BPRE, NBUF, APRE>), grid, dim3(64 * WM * WN), lds, s, a);
  if (tail)
    hipLaunchKernelGGL((k_gemm_fixup_sub<BM, BN, WM, WN, EPI>),
                       dim3(tail, (BM / WM / 32) * (BN / WN / 32), a.ngroups), dim3(64 * WM * WN), 0, s, a);
  return hipGetLastError();
}

template <int BM, int BN, int WM, int WN, int NBUF = 2>
static hipError_t launch_bs(const GemmArgs& a, hipStream_t s) {
  constexpr int BK = 32;
  if (a.K % BK || a.ksplit % BK) return hipErrorInvalidValue;
  const size_t lds = (NBUF < 2 ? NBUF : 2) * 3 * (BM + BN) * BK * sizeof(unsigned short);
  const int T = ((a.N + BN - 1) / BN) * ((a.M + BM - 1) / BM);
  const int tail = a.tsplit > 1 ? T - a.tdp : 0;
  dim3 grid(tail ? a.tdp + tail * a.tsplit : T, 1, a.ngroups);
  bool pre = true, apre = true;
  for (int g = 0; g < a.ngroups; ++g) {
    pre = pre && a.g[g].Bp;
    apre = apre && a.g[g].Ap;
  }
  if (pre && apre && a.epi == EPI_STORE) return launch_bs_k<BM, BN, WM, WN, EPI_STORE, true, NBUF, true>(a, s, grid, lds, tail);
  switch (a.epi * 2 + (pre ? 1 : 0)) {
#define VV_EPI(E)                                                                    \
  case 2 * E: return launch_bs_k<BM, BN, WM, WN, E, false, NBUF>(a, s, grid, lds, tail); \
  case 2 * E + 1: return launch_bs_k<BM, BN, WM, WN, E, true, NBUF>(a, s, grid, lds, tail);
    VV_EPI(EPI_STORE)
    VV_EPI(EPI_GELU)
    VV_EPI(EPI_RESID)
    VV_EPI(EPI_DGELU)
#undef VV_EPI
    default:
      return hipErrorInvalidValue;
  }
}

template <int BM, int BN, int BK, int WM, int WN, int EPI>
static hipError_t launch_tile_k(const GemmArgs& a, hipStream_t s, dim3 grid, size_t lds, int tail) {
  if (hipError_t e = set_lds_limit((const void*)k_gemm_nt<BM, BN, BK, WM, WN, EPI, 32>, lds)) return e;
  hipLaunchKernelGGL((k_gemm_nt<BM, BN, BK, WM, WN, EPI, 32>), grid, dim3(64 * WM * WN), lds, s, a);
  if (tail) hipLaunchKernelGGL((k_gemm_fixup<BM, BN, WM, WN, EPI, 32>), dim3(tail, 1, a.ngroups), dim3(64 * WM * WN), 0, s, a);
  return hipGetLastError();
}

template <int BM, int BN, int BK, int WM, int WN>
static hipError_t launch_tile(const GemmArgs& a, hipStream_t s) {
  constexpr int LS = BK + 4;
  if (a.K % BK || a.ksplit % BK) return hipErrorInvalidValue;
  const size_t lds = 2 * (BM + BN) * LS * sizeof(float);
  const int T = ((a.N + BN - 1) / BN) * ((a.M + BM - 1) / BM);
  const int tail = a.tsplit > 1 ? T - a.tdp : 0;
  dim3 grid(tail ? a.tdp + tail * a.tsplit : T, 1, a.ngroups);
  switch (a.epi) {
    case EPI_STORE: return launch_tile_k<BM, BN, BK, WM, WN, EPI_STORE>(a, s, grid, lds, tail);
    case EPI_GELU: return launch_tile_k<BM, BN, BK, WM, WN, EPI_GELU>(a, s, grid, lds, tail);
    case EPI_RESID: return launch_tile_k<BM, BN, BK, WM, WN, EPI_RESID>(a, s, grid, lds, tail);
    case EPI_DGELU: return launch_tile_k<BM, BN, BK, WM, WN, EPI_DGELU>(a, s, grid, lds, tail);
    default: return hipErrorInvalidValue;
  }
}

// ---------------------------------------------------------------------------------------------------------
// Pipelined split GEMM: 128x128x32 tile, 4 waves of 64x64, two LDS buffers, ONE barrier per k-tile.
// Iteration kt reads all fragments of tile kt from buf[kt&1] and, while its 48 MFMAs run, splits tile kt+1
// (already in registers since iteration kt-1) into buf[(kt+1)&1] and issues the global loads of tile kt+2;
// sched_group_barrier interleaves the split VALU, the LDS writes and the loads between the MFMAs so the matrix
// pipe is never waiting for the staging (k_gemm_bs serialises them: split, barrier, MFMAs, barrier).
template <int EPI, bool APRE>
__global__ __launch_bounds__(256, 1) void k_gemm_bs2(GemmArgs args) {
  constexpr int BM = 128, BN = 128, BK = 32, NT = 256, WN = 2, TM = 2, TN = 2;
  constexpr int LSB = BK, PLANE = (BM + BN) * LSB;
  constexpr int TPR = BK / 4, RPP = NT / TPR;   // fp32 A staging: 8 threads per row, 32 rows per pass
  constexpr int AI = APRE ? 1 : BM / RPP;       // 4
  constexpr int AQ = BM * 4 / NT;               // 2 (16-B chunks per thread per plane)
  constexpr int BQ = BN * 4 / NT;               // 2
  typedef float accv __attribute__((ext_vector_type(16)));
  extern __shared__ __attribute__((aligned(16))) unsigned short lds16[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
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
  tile_mn(tile, ntm, ntn, mb, nb, args.gm);
  const int m0 = mb * BM, n0 = nb * BN;
  const int lr = tid / TPR, lc = (tid % TPR) * 4;
  auto swz = [](int row, int k) { return row * LSB + ((((k >> 3) ^ (row >> 2)) & 3) << 3) + (k & 7); };

  const float* a1p[AI];
  const float* a2p[AI];
  const unsigned short* aq[AQ];
  if constexpr (APRE) {
#pragma unroll
    for (int i = 0; i < AQ; ++i) {
      const int c = tid + NT * i;
      const int r = min(m0 + c / 4, M - 1);
      const int ar = args.arow ? args.arow[r] : r;
      aq[i] = G.Ap + (size_t)ar * 3 * args.lda + (c % 4) * 8;
    }
  } else {
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int r = min(m0 + lr + RPP * i, M - 1);
      const int ar = args.arow ? args.arow[r] : r;
      a1p[i] = G.A + (size_t)ar * args.lda + lc;
      a2p[i] = G.A2 ? G.A2 + (size_t)r * args.lda2 + lc - ksplit : a1p[i];
    }
  }
  const unsigned short* bq[BQ];
#pragma unroll
  for (int i = 0; i < BQ; ++i) {
    const int c = tid + NT * i;
    const int n = min(n0 + c / 4, N - 1);
    bq[i] = G.Bp + (size_t)n * 3 * K + (c % 4) * 8;
  }

  f4 ra[AI];
  u4v qa[AQ][3], rq[BQ][3];
  auto gload = [&](int k0) {
    if constexpr (APRE) {
#pragma unroll
      for (int i = 0; i < AQ; ++i)
#pragma unroll
        for (int p = 0; p < 3; ++p) qa[i][p] = *reinterpret_cast<const u4v*>(aq[i] + p * args.lda + k0);
    } else if (k0 < ksplit) {
#pragma unroll
      for (int i = 0; i < AI; ++i) ra[i] = *reinterpret_cast<const f4*>(a1p[i] + k0);
    } else {
#pragma unroll
      for (int i = 0; i < AI; ++i) ra[i] = *reinterpret_cast<const f4*>(a2p[i] + k0);
    }
#pragma unroll
    for (int i = 0; i < BQ; ++i)
#pragma unroll
      for (int p = 0; p < 3; ++p) rq[i][p] = *reinterpret_cast<const u4v*>(bq[i] + p * K + k0);
  };
  auto sstore = [&](int buf) {
    unsigned short* P = lds16 + buf * 3 * PLANE;
    if constexpr (APRE) {
#pragma unroll
      for (int i = 0; i < AQ; ++i) {
        const int c = tid + NT * i;
        const int o = swz(c / 4, (c % 4) * 8);
#pragma unroll
        for (int p = 0; p < 3; ++p) *reinterpret_cast<u4v*>(P + p * PLANE + o) = qa[i][p];
      }
    } else {
      u2v h, m, l;
#pragma unroll
      for (int i = 0; i < AI; ++i) {
        split3t(ra[i], h, m, l);
        const int o = swz(lr + RPP * i, lc);
        *reinterpret_cast<u2v*>(P + o) = h;
        *reinterpret_cast<u2v*>(P + PLANE + o) = m;
        *reinterpret_cast<u2v*>(P + 2 * PLANE + o) = l;
      }
    }
#pragma unroll
    for (int i = 0; i < BQ; ++i) {
      const int c = tid + NT * i;
      const int o = swz(BM + c / 4, (c % 4) * 8);
#pragma unroll
      for (int p = 0; p < 3; ++p) *reinterpret_cast<u4v*>(P + p * PLANE + o) = rq[i][p];
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

  const int nk = ke - kb;
  gload(kb * BK);
  sstore(0);
  if (nk > 1) gload((kb + 1) * BK);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const unsigned short* P = lds16 + (kt & 1) * 3 * PLANE;
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
    // 48 MFMA slots, each followed by a small, fixed piece of the staging work (source order is kept by
    // sched_barrier): slots 0-15 split one element of tile kt+1's A chunk, 16-19 pack + write a chunk's planes,
    // 20-25 write the B planes, 26-35 issue tile kt+2's global loads. Branch-free: on the last two iterations
    // the staging re-reads the last k-tile and writes a buffer nobody reads again.
    unsigned short* Pn = lds16 + ((kt + 1) & 1) * 3 * PLANE;
    const int k2 = min(kb + kt + 2, ke - 1) * BK;
    unsigned xb[AI][4], mbv[AI][4], lbv[AI][4];
#pragma unroll
    for (int i = 0; i < 48; ++i) {
      // MFMA i: step s, product p (smallest first), chain (a, b) fastest -> consecutive MFMAs independent
      const int st = i / 24, pr = (i % 24) / 4, a = (i % 4) / 2, b = i % 2;
      const bf8v& xa = fa[st][a][pr == 0 ? 2 : pr == 1 ? 0 : pr == 2 ? 1 : pr == 3 ? 1 : 0];
      const bf8v& xbv = fb[st][b][pr == 0 ? 0 : pr == 1 ? 2 : pr == 2 ? 1 : pr == 3 ? 0 : pr == 4 ? 1 : 0];
      const bf8v& xa2 = (pr == 4 || pr == 5) ? fa[st][a][0] : xa;
      acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xa2, xbv, acc[a][b], 0, 0, 0);
      if constexpr (!APRE) {
        if (i < 16) {
          const int c = i / 4, e = i % 4;
          const unsigned xv = __float_as_uint(ra[c][e]);
          const float r1 = ra[c][e] - __uint_as_float(xv & 0xffff0000u);
          xb[c][e] = xv;
          mbv[c][e] = __float_as_uint(r1);
          lbv[c][e] = __float_as_uint(r1 - __uint_as_float(mbv[c][e] & 0xffff0000u));
        } else if (i < 20) {
          const int c = i - 16;
          u2v h, m, l;
          h[0] = __builtin_amdgcn_perm(xb[c][1], xb[c][0], 0x07060302u);
          h[1] = __builtin_amdgcn_perm(xb[c][3], xb[c][2], 0x07060302u);
          m[0] = __builtin_amdgcn_perm(mbv[c][1], mbv[c][0], 0x07060302u);
          m[1] = __builtin_amdgcn_perm(mbv[c][3], mbv[c][2], 0x07060302u);
          l[0] = __builtin_amdgcn_perm(lbv[c][1], lbv[c][0], 0x07060302u);
          l[1] = __builtin_amdgcn_perm(lbv[c][3], lbv[c][2], 0x07060302u);
          const int o = swz(lr + RPP * c, lc);
          *reinterpret_cast<u2v*>(Pn + o) = h;
          *reinterpret_cast<u2v*>(Pn + PLANE + o) = m;
          *reinterpret_cast<u2v*>(Pn + 2 * PLANE + o) = l;
        }
      } else {
        if (i < 6) {
          const int c = tid + NT * (i / 3);
          *reinterpret_cast<u4v*>(Pn + (i % 3) * PLANE + swz(c / 4, (c % 4) * 8)) = qa[i / 3][i % 3];
        }
      }
      if (i >= 20 && i < 26) {
        const int q = (i - 20) / 3, p = (i - 20) % 3;
        const int c = tid + NT * q;
        *reinterpret_cast<u4v*>(Pn + p * PLANE + swz(BM + c / 4, (c % 4) * 8)) = rq[q][p];
      }
      if (i >= 26 && i < 26 + (APRE ? 3 * AQ : AI)) {
        const int j = i - 26;
        if constexpr (APRE) {
          qa[j / 3][j % 3] = *reinterpret_cast<const u4v*>(aq[j / 3] + (j % 3) * args.lda + k2);
        } else {
          ra[j] = *reinterpret_cast<const f4*>((k2 < ksplit ? a1p[j] : a2p[j]) + k2);
        }
      }
      if (i >= 36 && i < 42) {
        const int q = (i - 36) / 3, p = (i - 36) % 3;
        rq[q][p] = *reinterpret_cast<const u4v*>(bq[q] + p * K + k2);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
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
    epilogue<BM, BN, 2, WN, EPI, 32, true>(args, G, acc, m0, n0, wm, wn, rin, hh);
  else
    epilogue<BM, BN, 2, WN, EPI, 32, false>(args, G, acc, m0, n0, wm, wn, rin, hh);
}

template <int EPI, bool APRE>
static hipError_t launch_bs2_k(const GemmArgs& a, hipStream_t s, dim3 grid, size_t lds, int tail) {
  if (hipError_t e = set_lds_limit((const void*)k_gemm_bs2<EPI, APRE>, lds)) return e;
  hipLaunchKernelGGL((k_gemm_bs2<EPI, APRE>), grid, dim3(256), lds, s, a);
  if (tail)
    hipLaunchKernelGGL((k_gemm_fixup_sub<128, 128, 2, 2, EPI>), dim3(tail, 4, a.ngroups), dim3(256), 0, s, a);
  return hipGetLastError();
}

// requires pre-split B planes for every group (registered weights); falls back to k_gemm_bs otherwise
static hipError_t launch_bs2(const GemmArgs& a, hipStream_t s) {
  if (a.K % 32 || a.ksplit % 32) return hipErrorInvalidValue;
  bool pre = true, apre = true;
  for (int g = 0; g < a.ngroups; ++g) {
    pre = pre && a.g[g].Bp;
    apre = apre && a.g[g].Ap;
  }
  if (!pre) return launch_bs<128, 128, 2, 2, 1>(a, s);
  const size_t lds = 2 * 3 * 256 * 32 * sizeof(unsigned short);
  const int T = ((a.N + 127) / 128) * ((a.M + 127) / 128);
  const int tail = a.tsplit > 1 ? T - a.tdp : 0;
  dim3 grid(tail ? a.tdp + tail * a.tsplit : T, 1, a.ngroups);
  if (apre && a.epi == EPI_STORE) return launch_bs2_k<EPI_STORE, true>(a, s, grid, lds, tail);
  switch (a.epi) {
    case EPI_STORE: return launch_bs2_k<EPI_STORE, false>(a, s, grid, lds, tail);
    case EPI_GELU: return launch_bs2_k<EPI_GELU, false>(a, s, grid, lds, tail);
    case EPI_RESID: return launch_bs2_k<EPI_RESID, false>(a, s, grid, lds, tail);
    case EPI_DGELU: return launch_bs2_k<EPI_DGELU, false>(a, s, grid, lds, tail);
    default: return hipErrorInvalidValue;
  }
}

// ---------------------------------------------------------------------------------------------------------
// fp32 GEMM as three fp16 MFMA products (GEMM_SPLIT16; v_mfma_f32_32x32x16_f16, half the MFMAs of the bf16x6
// split for the same fp32-level error).
//
// An fp16 pair carries 22 significant bits (x = h + l + O(2^-22 x)) but only a 5-bit exponent, so each operand
// row is first scaled by a power of two that puts its maximum in [2^14, 2^15): B (weights) at load time
// (k_split16_rows), A (activations) by k_rowscale just before the GEMM (one pass over A, max over the whole
// logical row incl. the A2 part and the arow gather). Then
//   a.b = (h_a h_b + h_a l_b + l_a h_b) 2^-(e_a + e_b)      (dropped: l_a l_b and the residuals, ~2^-22 |a b|)
// Products of fp16 values are exact in fp32; both scales are applied once, after the k loop. A is split while
// the k-tile is staged (h = fp16(a 2^e), l = fp16(a 2^e - h), round-to-nearest, the residual exact in fp32).
// Tile 128x128x32, 4 waves of 64x64, two LDS buffers with the same swizzle as k_gemm_bs2, ONE barrier per
// k-tile: the MFMAs of tile kt run while tile kt+1 (in registers) is split into the other buffer and tile kt+2
// is loaded; same split-K tail and epilogues.
typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef _Float16 h4v __attribute__((ext_vector_type(4)));

// s[r] = 2^(141 - exponent(max_k |A(r,k)|)) for the logical rows of a GEMM (one wave per row; grid.z = group)
__global__ __launch_bounds__(256) void k_rowscale(GemmArgs args, float* __restrict__ out) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= args.M) return;
  const GemmGroup G = args.g[blockIdx.z];
  const int ar = args.arow ? args.arow[r] : r;
  const float* a = G.A + (size_t)ar * args.lda;
  auto amax = [](const f4& v) {
    return max(max(__float_as_uint(fabsf(v[0])), __float_as_uint(fabsf(v[1]))),
               max(__float_as_uint(fabsf(v[2])), __float_as_uint(fabsf(v[3]))));
  };
  unsigned mx = 0;
  int k = lane * 4;
  // four independent row loads in flight per lane (K = 1152: 4.5 float4 per lane)
  for (; k + 768 < args.ksplit; k += 1024) {
    const f4 v0 = *reinterpret_cast<const f4*>(a + k);
    const f4 v1 = *reinterpret_cast<const f4*>(a + k + 256);
    const f4 v2 = *reinterpret_cast<const f4*>(a + k + 512);
    const f4 v3 = *reinterpret_cast<const f4*>(a + k + 768);
    mx = max(mx, max(max(amax(v0), amax(v1)), max(amax(v2), amax(v3))));
  }
  for (; k < args.ksplit; k += 256) mx = max(mx, amax(*reinterpret_cast<const f4*>(a + k)));
  if (G.A2) {
    const float* a2 = G.A2 + (size_t)r * args.lda2;
    for (int k = lane * 4; k < args.K - args.ksplit; k += 256) {
      const f4 v = *reinterpret_cast<const f4*>(a2 + k);
      mx = max(mx, max(max(__float_as_uint(fabsf(v[0])), __float_as_uint(fabsf(v[1]))),
                       max(__float_as_uint(fabsf(v[2])), __float_as_uint(fabsf(v[3])))));
    }
  }
  mx = lane_max<64>(mx);
  if (lane == 0) out[(size_t)blockIdx.z * args.M + r] = __uint_as_float((268u - max(mx >> 23, 15u)) << 23);
}

// k_rowscale with every load of the row issued at once (NV float4 per lane, NV = ceil(K / 256), indices past the
// row end clamped: duplicates do not change a max): one memory round trip per row instead of one per group of
// four float4 -- the kernel runs two waves per SIMD at 2048 rows, so it is latency-bound. Bit-identical.
template <int NV>
__global__ __launch_bounds__(256) void k_rowscale_n(GemmArgs args, float* __restrict__ out) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= args.M) return;
  const GemmGroup G = args.g[blockIdx.z];
  const int ar = args.arow ? args.arow[r] : r;
  const float* a1 = G.A + (size_t)ar * args.lda;
  const float* a2 = G.A2 ? G.A2 + (size_t)r * args.lda2 - args.ksplit : a1;
  f4 v[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int k = min(lane * 4 + 256 * i, args.K - 4);
    v[i] = *reinterpret_cast<const f4*>((k < args.ksplit ? a1 : a2) + k);
  }
  unsigned mx = 0;
#pragma unroll
  for (int i = 0; i < NV; ++i)
    mx = max(mx, max(max(__float_as_uint(fabsf(v[i][0])), __float_as_uint(fabsf(v[i][1]))),
                     max(__float_as_uint(fabsf(v[i][2])), __float_as_uint(fabsf(v[i][3])))));
  mx = lane_max<64>(mx);
  if (lane == 0) out[(size_t)blockIdx.z * args.M + r] = __uint_as_float((268u - max(mx >> 23, 15u)) << 23);
}

static void launch_rowscale(const GemmArgs& a, float* out, hipStream_t s) {
  const dim3 grid((a.M + 3) / 4, 1, a.ngroups);
  const int nv = (a.K + 255) / 256;
  switch (nv <= 5 ? (nv <= 2 ? 2 : 5) : nv <= 9 ? 9 : nv <= 14 ? 14 : nv <= 18 ? 18 : 0) {
    case 2: hipLaunchKernelGGL(k_rowscale_n<2>, grid, dim3(256), 0, s, a, out); break;
    case 5: hipLaunchKernelGGL(k_rowscale_n<5>, grid, dim3(256), 0, s, a, out); break;
    case 9: hipLaunchKernelGGL(k_rowscale_n<9>, grid, dim3(256), 0, s, a, out); break;
    case 14: hipLaunchKernelGGL(k_rowscale_n<14>, grid, dim3(256), 0, s, a, out); break;
    case 18: hipLaunchKernelGGL(k_rowscale_n<18>, grid, dim3(256), 0, s, a, out); break;
    default: hipLaunchKernelGGL(k_rowscale, grid, dim3(256), 0, s, a, out); break;
  }
}

// out[z][r] = scales[z][arow[r]]: the producer's per-physical-row scales in the gathered GEMM's row order
__global__ __launch_bounds__(256) void k_gather_scales(const float* __restrict__ scales, const int* __restrict__ arow,
                                                       float* __restrict__ out, int M) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r < M) out[(size_t)blockIdx.z * M + r] = scales[(size_t)blockIdx.z * M + arow[r]];
}

// BM = 128: 4 waves (2 x 2 of 64x64), 64 KB of LDS, two workgroups per CU. BM = 256: 8 waves (4 x 2 of 64x64),
// 96 KB, one workgroup per CU: the same two waves per SIMD, but each B k-tile feeds 256 rows, so a CU stages 48 KB
// (global loads and LDS stores) per 2 x 24 MFMAs per SIMD instead of 64 KB.
template <int EPI, int BM>
__global__ __launch_bounds__(2 * BM, 1) void k_gemm_h3(GemmArgs args, const float* __restrict__ ascale) {
  constexpr int BN = 128, BK = 32, NT = 2 * BM, WN = 2, WM = BM / 64, TM = 2, TN = 2;
  constexpr int LSB = BK, PLANE = (BM + BN) * LSB;  // unsigned shorts
  constexpr int BUF = 2 * PLANE;                    // fp16 planes h, l of the A and B rows
  constexpr int TPR = BK / 4, RPP = NT / TPR, AI = BM / RPP, BQ = BN * 4 / NT;  // 8, 32, 4, 2
  typedef float accv __attribute__((ext_vector_type(16)));
  extern __shared__ __attribute__((aligned(16))) unsigned short lds16[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
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
    // split items in chunk-major order, contiguous per XCD (xcd_remap): one XCD runs the same k-chunk of
    // neighbouring tiles, so the A / B k-slices it shares stay in its L2; part = the item's partial slot
    const int items = gridDim.x - args.tdp, S = args.tsplit, tt = items / S;
    const int L = xcd_remap(blockIdx.x - args.tdp, items), c = L / tt, tl = L - c * tt;
    part = tl * S + c;
    tile = args.tdp + tl;
    kb = (c * nkt) / S;
    ke = ((c + 1) * nkt) / S;
  }
  int mb, nb;
  tile_mn(tile, ntm, ntn, mb, nb, args.gm);
  const int m0 = mb * BM, n0 = nb * BN;
  const int lr = tid / TPR, lc = (tid % TPR) * 4;
  auto swz = [](int row, int k) { return row * LSB + ((((k >> 3) ^ (row >> 2)) & 3) << 3) + (k & 7); };
  const float* rs = ascale + (size_t)blockIdx.z * M;

  const float* a1p[AI];
  const float* a2p[AI];
  float sa[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int r = min(m0 + lr + RPP * i, M - 1);
    const int ar = args.arow ? args.arow[r] : r;
    a1p[i] = G.A + (size_t)ar * args.lda + lc;
    a2p[i] = G.A2 ? G.A2 + (size_t)r * args.lda2 + lc - ksplit : a1p[i];
    sa[i] = rs[r];
  }
  const unsigned short* bq[BQ];
#pragma unroll
  for (int i = 0; i < BQ; ++i) {
    const int c = tid + NT * i;
    const int n = min(n0 + c / 4, N - 1);
    bq[i] = G.Bh + (size_t)n * 2 * K + (c % 4) * 8;
  }

  f4 ra[AI];
  u4v rq[BQ][2];
  auto aload = [&](int i, int k0) { ra[i] = *reinterpret_cast<const f4*>((k0 < ksplit ? a1p[i] : a2p[i]) + k0); };
  auto bload = [&](int q, int p, int k0) { rq[q][p] = *reinterpret_cast<const u4v*>(bq[q] + 2 * k0 + p * 32); };
  auto asplit = [&](unsigned short* P, int i) {
    const int o = swz(lr + RPP * i, lc);
    h4v hv, lv;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float v = ra[i][e] * sa[i];
      hv[e] = (_Float16)v;
      lv[e] = (_Float16)(v - (float)hv[e]);
    }
    *reinterpret_cast<h4v*>(P + o) = hv;
    *reinterpret_cast<h4v*>(P + PLANE + o) = lv;
  };
  auto bstore = [&](unsigned short* P, int q, int p) {
    const int c = tid + NT * q;
    *reinterpret_cast<u4v*>(P + p * PLANE + swz(BM + c / 4, (c % 4) * 8)) = rq[q][p];
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

  const int nk = ke - kb;
#pragma unroll
  for (int i = 0; i < AI; ++i) aload(i, kb * BK);
#pragma unroll
  for (int q = 0; q < BQ; ++q)
#pragma unroll
    for (int p = 0; p < 2; ++p) bload(q, p, kb * BK);
#pragma unroll
  for (int i = 0; i < AI; ++i) asplit(lds16, i);
#pragma unroll
  for (int q = 0; q < BQ; ++q)
#pragma unroll
    for (int p = 0; p < 2; ++p) bstore(lds16, q, p);
  {
    const int k1 = min(kb + 1, ke - 1) * BK;
#pragma unroll
    for (int i = 0; i < AI; ++i) aload(i, k1);
#pragma unroll
    for (int q = 0; q < BQ; ++q)
#pragma unroll
      for (int p = 0; p < 2; ++p) bload(q, p, k1);
  }
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const unsigned short* P = lds16 + (kt & 1) * BUF;
    const unsigned short* As = P + (wm * TM * 32 + rin) * LSB;
    const unsigned short* Bs = P + (BM + wn * TN * 32 + rin) * LSB;
    h8v fa[2][TM][2], fb[2][TN][2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ck = ((2 * s + hh) ^ ((rin >> 2) & 3)) * 8;
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int p = 0; p < 2; ++p) fa[s][a][p] = *reinterpret_cast<const h8v*>(As + p * PLANE + a * 32 * LSB + ck);
#pragma unroll
      for (int b = 0; b < TN; ++b)
#pragma unroll
        for (int p = 0; p < 2; ++p) fb[s][b][p] = *reinterpret_cast<const h8v*>(Bs + p * PLANE + b * 32 * LSB + ck);
    }
    __builtin_amdgcn_sched_barrier(0);
    unsigned short* Pn = lds16 + ((kt + 1) & 1) * BUF;
    const int k2 = min(kb + kt + 2, ke - 1) * BK;
    // 24 MFMA slots: step s, product (l h, h l, h h: smallest first), chain (a, b) fastest. Branch-free staging:
    // on the last two iterations it re-reads the last k-tile and writes a buffer nobody reads again.
#pragma unroll
    for (int i = 0; i < 24; ++i) {
      const int st = i / 12, pr = (i % 12) / 4, a = (i % 4) / 2, b = i % 2;
      const h8v& xa = fa[st][a][pr == 0 ? 1 : 0];
      const h8v& xb = fb[st][b][pr == 1 ? 1 : 0];
      acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xa, xb, acc[a][b], 0, 0, 0);
      if (i < 2 * AI && (i & 1)) asplit(Pn, i / 2);
      if (i >= 8 && i < 8 + 2 * BQ) bstore(Pn, (i - 8) / 2, (i - 8) % 2);
      if (i >= 12 && i < 12 + AI) aload(i - 12, k2);
      if (i >= 16 && i < 16 + 2 * BQ) bload((i - 16) / 2, (i - 16) % 2, k2);
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
  }

  // undo the scales: rows of A (2^-e_a), rows of B = columns of C (2^-e_b)
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int col = min(n0 + wn * TN * 32 + b * 32 + rin, N - 1);
    const float sb = G.Bs[(size_t)col * (K / 32)];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int row = min(m0 + wm * TM * 32 + a * 32 + 8 * j + 4 * hh + q, M - 1);
          const float ia = __uint_as_float((254u << 23) - __float_as_uint(rs[row]));   // 2^-e_a
          acc[a][b][4 * j + q] *= ia * sb;
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

// The same fp16x3 kernel on v_mfma_f32_16x16x32_f16 (4 x 4 tiles of 16x16 per 64x64 wave tile, 48 MFMAs of 16
// cycles per k-tile): equal cycles per FLOP, but the chip holds a higher clock under the 16x16 form
// (MI355X_MICROARCH.md DVFS item 7). Tiles 46 (BM 128) and 47 (BM 256).
template <int EPI, int BM>
__global__ __launch_bounds__(2 * BM, 1) void k_gemm_h3m(GemmArgs args, const float* __restrict__ ascale) {
  constexpr int BN = 128, BK = 32, NT = 2 * BM, WN = 2, WM = BM / 64, TM = 4, TN = 4;  // 16x16 tiles per wave
  constexpr int LSB = BK, PLANE = (BM + BN) * LSB;  // unsigned shorts
  constexpr int BUF = 2 * PLANE;                    // fp16 planes h, l of the A and B rows
  constexpr int TPR = BK / 4, RPP = NT / TPR, AI = BM / RPP, BQ = BN * 4 / NT;  // 8, 32, 4, 2
  typedef float accv __attribute__((ext_vector_type(4)));
  extern __shared__ __attribute__((aligned(16))) unsigned short lds16[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
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
    // split items in chunk-major order, contiguous per XCD (xcd_remap): one XCD runs the same k-chunk of
    // neighbouring tiles, so the A / B k-slices it shares stay in its L2; part = the item's partial slot
    const int items = gridDim.x - args.tdp, S = args.tsplit, tt = items / S;
    const int L = xcd_remap(blockIdx.x - args.tdp, items), c = L / tt, tl = L - c * tt;
    part = tl * S + c;
    tile = args.tdp + tl;
    kb = (c * nkt) / S;
    ke = ((c + 1) * nkt) / S;
  }
  int mb, nb;
  tile_mn(tile, ntm, ntn, mb, nb, args.gm);
  const int m0 = mb * BM, n0 = nb * BN;
  const int lr = tid / TPR, lc = (tid % TPR) * 4;
  // 16-B chunk c of row r at chunk c ^ h((r >> 2) & 3), h = {0, 2, 3, 1}: the four lane groups of a ds_read_b128
  // of a 16x16x32 fragment (rows lane & 15, chunk lane >> 4) land on 16 distinct 16-B slots
  auto hsw = [](int q) { return (0x78 >> (2 * (q & 3))) & 3; };  // 0, 2, 3, 1
  auto swz = [&](int row, int k) { return row * LSB + ((((k >> 3) ^ hsw(row >> 2)) & 3) << 3) + (k & 7); };
  const float* rs = ascale + (size_t)blockIdx.z * M;

  const float* a1p[AI];
  const float* a2p[AI];
  float sa[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int r = min(m0 + lr + RPP * i, M - 1);
    const int ar = args.arow ? args.arow[r] : r;
    a1p[i] = G.A + (size_t)ar * args.lda + lc;
    a2p[i] = G.A2 ? G.A2 + (size_t)r * args.lda2 + lc - ksplit : a1p[i];
    sa[i] = rs[r];
  }
  const unsigned short* bq[BQ];
#pragma unroll
  for (int i = 0; i < BQ; ++i) {
    const int c = tid + NT * i;
    const int n = min(n0 + c / 4, N - 1);
    bq[i] = G.Bh + (size_t)n * 2 * K + (c % 4) * 8;
  }

  f4 ra[AI];
  u4v rq[BQ][2];
  auto aload = [&](int i, int k0) { ra[i] = *reinterpret_cast<const f4*>((k0 < ksplit ? a1p[i] : a2p[i]) + k0); };
  auto bload = [&](int q, int p, int k0) { rq[q][p] = *reinterpret_cast<const u4v*>(bq[q] + 2 * k0 + p * 32); };
  auto asplit = [&](unsigned short* P, int i) {
    const int o = swz(lr + RPP * i, lc);
    h4v hv, lv;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float v = ra[i][e] * sa[i];
      hv[e] = (_Float16)v;
      lv[e] = (_Float16)(v - (float)hv[e]);
    }
    *reinterpret_cast<h4v*>(P + o) = hv;
    *reinterpret_cast<h4v*>(P + PLANE + o) = lv;
  };
  auto bstore = [&](unsigned short* P, int q, int p) {
    const int c = tid + NT * q;
    *reinterpret_cast<u4v*>(P + p * PLANE + swz(BM + c / 4, (c % 4) * 8)) = rq[q][p];
  };

  const int wm = wave / WN, wn = wave % WN;
  const int rin = lane & 15, hh = lane >> 4;
  accv acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[a][b][r] = 0.0f;

  const int nk = ke - kb;
#pragma unroll
  for (int i = 0; i < AI; ++i) aload(i, kb * BK);
#pragma unroll
  for (int q = 0; q < BQ; ++q)
#pragma unroll
    for (int p = 0; p < 2; ++p) bload(q, p, kb * BK);
#pragma unroll
  for (int i = 0; i < AI; ++i) asplit(lds16, i);
#pragma unroll
  for (int q = 0; q < BQ; ++q)
#pragma unroll
    for (int p = 0; p < 2; ++p) bstore(lds16, q, p);
  {
    const int k1 = min(kb + 1, ke - 1) * BK;
#pragma unroll
    for (int i = 0; i < AI; ++i) aload(i, k1);
#pragma unroll
    for (int q = 0; q < BQ; ++q)
#pragma unroll
      for (int p = 0; p < 2; ++p) bload(q, p, k1);
  }
  __syncthreads();

  const int ck = ((hh ^ hsw(rin >> 2)) & 3) * 8;  // fragment rows start at multiples of 16
  for (int kt = 0; kt < nk; ++kt) {
    const unsigned short* P = lds16 + (kt & 1) * BUF;
    const unsigned short* As = P + (wm * TM * 16 + rin) * LSB + ck;
    const unsigned short* Bs = P + (BM + wn * TN * 16 + rin) * LSB + ck;
    h8v fa[TM][2], fb[TN][2];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int p = 0; p < 2; ++p) fa[a][p] = *reinterpret_cast<const h8v*>(As + p * PLANE + a * 16 * LSB);
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int p = 0; p < 2; ++p) fb[b][p] = *reinterpret_cast<const h8v*>(Bs + p * PLANE + b * 16 * LSB);
    __builtin_amdgcn_sched_barrier(0);
    unsigned short* Pn = lds16 + ((kt + 1) & 1) * BUF;
    const int k2 = min(kb + kt + 2, ke - 1) * BK;
    // 48 v_mfma_f32_16x16x32_f16 slots (the whole 32-deep k-tile each): product (l h, h l, h h: smallest first),
    // then (a, b); the staging of the 32x32 kernel runs on the even slots
#pragma unroll
    for (int i = 0; i < 48; ++i) {
      const int pr = i / 16, a = (i % 16) / 4, b = i % 4;
      const h8v& xa = fa[a][pr == 0 ? 1 : 0];
      const h8v& xb = fb[b][pr == 1 ? 1 : 0];
      acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa, xb, acc[a][b], 0, 0, 0);
      if ((i & 1) == 0) {
        const int j = i >> 1;
        if (j < 2 * AI && (j & 1)) asplit(Pn, j / 2);
        if (j >= 8 && j < 8 + 2 * BQ) bstore(Pn, (j - 8) / 2, (j - 8) % 2);
        if (j >= 12 && j < 12 + AI) aload(j - 12, k2);
        if (j >= 16 && j < 16 + 2 * BQ) bload((j - 16) / 2, (j - 16) % 2, k2);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
  }

  // undo the scales: rows of A (2^-e_a), rows of B = columns of C (2^-e_b); 16x16 tile: row 4 hh + r, col rin
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int col = min(n0 + wn * TN * 16 + b * 16 + rin, N - 1);
    const float sb = G.Bs[(size_t)col * (K / 32)];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = min(m0 + wm * TM * 16 + a * 16 + 4 * hh + r, M - 1);
        const float ia = __uint_as_float((254u << 23) - __float_as_uint(rs[row]));   // 2^-e_a
        acc[a][b][r] *= ia * sb;
      }
  }

  if (part >= 0) {
    float* w = args.ws + ((size_t)blockIdx.z * (gridDim.x - args.tdp) + part) * (size_t)(TM * TN * 4 * NT);
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) w[(size_t)((a * TN + b) * 4 + r) * NT + tid] = acc[a][b][r];
    return;
  }
  if (m0 + BM <= M && n0 + BN <= N)
    epilogue<BM, BN, WM, WN, EPI, 16, true>(args, G, acc, m0, n0, wm, wn, rin, hh);
  else
    epilogue<BM, BN, WM, WN, EPI, 16, false>(args, G, acc, m0, n0, wm, wn, rin, hh);
}

// ---------------------------------------------------------------------------------------------------------
// fp16x3 on pre-split operands, both staged by LDS-DMA (tile 48).
//
// k_rowsplit writes A once per GEMM as fp16 planes in GEMM row order (the arow gather and the A2 concat applied),
// row r scaled by 2^e and stored chunk-interleaved: [h(k 0..31) | l(k 0..31) | h(k 32..63) | l(k 32..63) | ...] (the same scale and split arithmetic as k_rowscale + the in-loop split of
// k_gemm_h3m, so the products are bit-identical), exactly B's plane layout. k_gemm_h4 then streams both operands
// HBM/L2 -> LDS with global_load_lds_dwordx4 (no VGPR staging, no ds_write, no VALU split in the loop) through a
// three-stage ring (3 x 48 KB of 160 KB), keeping two k-tiles in flight across the one raw s_barrier per k-tile
// (counted vmcnt(6), never 0 in the loop: cdna_hip_programming.md "Pipelining across barriers"). The LDS image is
// lane-linear per DMA instruction; the bank swizzle of the 16x16x32 fragment reads (chunk c of row r at
// c ^ h((r >> 2) & 3)) is applied to each lane's global source address instead (rule 21). The fragments of k-tile
// t+1 are read under the second half of k-tile t's 48 MFMAs (two register sets). Geometry, MFMA order, split-K
// tail and epilogue are those of k_gemm_h3m<EPI, 256>, so C is bit-identical to tile 47.

// one wave per logical row: max |A| of the row -> scale 2^(141 - e) (k_rowscale's formula), then the scaled row
// split into fp16 h = fp16(v), l = fp16(v - h) and stored as chunk-interleaved planes of row r; NV float4 per lane
template <int NV>
__global__ __launch_bounds__(256) void k_rowsplit(GemmArgs args, float* __restrict__ rs, unsigned short* __restrict__ pl) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= args.M) return;
  const GemmGroup G = args.g[blockIdx.z];
  const int K = args.K;
  const int ar = args.arow ? args.arow[r] : r;
  const float* a1 = G.A + (size_t)ar * args.lda;
  const float* a2 = G.A2 ? G.A2 + (size_t)r * args.lda2 - args.ksplit : a1;
  f4 v[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int k = min(lane * 4 + 256 * i, K - 4);
    v[i] = *reinterpret_cast<const f4*>((k < args.ksplit ? a1 : a2) + k);
  }
  unsigned mx = 0;
#pragma unroll
  for (int i = 0; i < NV; ++i)
    mx = max(mx, max(max(__float_as_uint(fabsf(v[i][0])), __float_as_uint(fabsf(v[i][1]))),
                     max(__float_as_uint(fabsf(v[i][2])), __float_as_uint(fabsf(v[i][3])))));
  mx = lane_max<64>(mx);
  const float s = __uint_as_float((268u - max(mx >> 23, 15u)) << 23);
  const size_t zr = (size_t)blockIdx.z * args.M + r;
  if (lane == 0) rs[zr] = s;
  unsigned short* ph = pl + zr * 2 * (size_t)K;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int k = lane * 4 + 256 * i;
    if (k >= K) break;
    h4v hv, lv;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float x = v[i][e] * s;
      hv[e] = (_Float16)x;
      lv[e] = (_Float16)(x - (float)hv[e]);
    }
    *reinterpret_cast<h4v*>(ph + 2 * (k & ~31) + (k & 31)) = hv;  // chunk-interleaved planes
    *reinterpret_cast<h4v*>(ph + 2 * (k & ~31) + 32 + (k & 31)) = lv;
  }
}

typedef __attribute__((address_space(3))) void* lds_ptr_t;


template <int EPI>
__global__ __launch_bounds__(512, 1) void k_gemm_h4(GemmArgs args, const float* __restrict__ ascale,
                                                    const unsigned short* __restrict__ apl) {
  constexpr int BM = 256, BN = 128, BK = 32, NT = 512, WN = 2, WM = 4, TM = 4, TN = 4;
  constexpr int STG = (BM + BN) * 2 * BK;                  // [row][h 32 | l 32] halfs: 24576 halfs = 48 KB per stage
  typedef float accv __attribute__((ext_vector_type(4)));
  extern __shared__ __attribute__((aligned(16))) unsigned short lds16[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const GemmGroup G = args.g[blockIdx.z];
  const int M = args.M, N = args.N, K = args.K;
  const int ntn = (N + BN - 1) / BN, ntm = (M + BM - 1) / BM;
  const int nkt = K / BK;
  int tile = 0, kb = 0, ke = nkt, part = -1;
  if (args.tsplit <= 1) {
    tile = xcd_remap(blockIdx.x, ntm * ntn);
  } else if ((int)blockIdx.x < args.tdp) {
    tile = xcd_remap(blockIdx.x, args.tdp);
  } else {
    const int items = gridDim.x - args.tdp, S = args.tsplit, tt = items / S;
    const int L = xcd_remap(blockIdx.x - args.tdp, items), c = L / tt, tl = L - c * tt;
    part = tl * S + c;
    tile = args.tdp + tl;
    kb = (c * nkt) / S;
    ke = ((c + 1) * nkt) / S;
  }
  int mb, nb;
  tile_mn(tile, ntm, ntn, mb, nb, args.gm);
  const int m0 = mb * BM, n0 = nb * BN;
  const float* rs = ascale + (size_t)blockIdx.z * M;
  // this lane's 16 A row scales (gathered through arow from the producer's physical-row scales when agather: no
  // k_gather_scales launch), loaded after the k loop (before it: +2 % kernel time, profiles/r04/ab_r04s)
  float rsv[4][4];

  // Planes are chunk-interleaved in memory (per row and 32-deep k-tile: h 64 B | l 64 B, one 128-B line) and in
  // LDS ([row][128 B], A rows then B rows). One DMA instruction fills 8 rows: lane i writes LDS bytes 16 i, row
  // i >> 3, slot i & 7, which holds the row's 16-B chunk (i & 7) ^ ((row >> 1) & 7) -- the swizzle under which the
  // 16 rows x one chunk of a fragment read land on 16 distinct 16-B slots of the 256-B bank row (rule 21: applied
  // to the source address, the LDS image stays lane-linear). Wave w stages A pieces w + 8 j (rows 8 (w + 8 j) ..,
  // j < 4) and B pieces w + 8 j (j < 2).
  const int prow = lane >> 3, pslot = lane & 7;
  const unsigned short* asrc[4];
  const unsigned short* bsrc[2];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = 8 * (wave + 8 * j) + prow;
    int gr = min(m0 + row, M - 1);
    if (args.apre && args.arow) gr = args.arow[gr];  // producer planes are in physical row order
    asrc[j] = apl + ((size_t)blockIdx.z * M + gr) * 2 * K + 8 * (pslot ^ ((row >> 1) & 7));
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = 8 * (wave + 8 * j) + prow;
    const int gn = min(n0 + row, N - 1);
    bsrc[j] = G.Bh + (size_t)gn * 2 * K + 8 * (pslot ^ ((row >> 1) & 7));
  }
  // DMA piece q (0..3: A pieces, 4..5: B pieces) of k-tile kt into stage buffer buf
  auto piece = [&](int kt, int buf, int q) {
    unsigned short* S = lds16 + buf * STG;
    const int k2 = 2 * kt * BK;  // halfs of the row before k-tile kt
    if (q < 4) {
      __builtin_amdgcn_global_load_lds((const void*)(asrc[q] + k2), (lds_ptr_t)(S + 8 * (wave + 8 * q) * 64), 16, 0,
                                       0);
    } else {
      __builtin_amdgcn_global_load_lds((const void*)(bsrc[q - 4] + k2),
                                       (lds_ptr_t)(S + (BM + 8 * (wave + 8 * (q - 4))) * 64), 16, 0, 0);
    }
  };
  auto stage = [&](int kt, int buf) {
#pragma unroll
    for (int q = 0; q < 6; ++q) piece(kt, buf, q);
  };

  const int wm = wave / WN, wn = wave % WN;
  const int rin = lane & 15, hh = lane >> 4;
  // fragment (row rin of a 16-row block, k-chunk hh) of plane p: LDS 16-B slot (4 p + hh) ^ ((rin >> 1) & 7)
  const int ck0 = (hh ^ ((rin >> 1) & 7)) * 8, ck1 = ((4 + hh) ^ ((rin >> 1) & 7)) * 8;
  const int aoff = (wm * TM * 16 + rin) * 64, boff = (BM + wn * TN * 16 + rin) * 64;
  auto frags = [&](int buf, h8v (&fa)[TM][2], h8v (&fb)[TN][2]) {
    const unsigned short* S = lds16 + buf * STG;
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int p = 0; p < 2; ++p)
        fa[a][p] = *reinterpret_cast<const h8v*>(S + aoff + a * 16 * 64 + (p ? ck1 : ck0));
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int p = 0; p < 2; ++p)
        fb[b][p] = *reinterpret_cast<const h8v*>(S + boff + b * 16 * 64 + (p ? ck1 : ck0));
  };

  accv acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[a][b][r] = 0.0f;

  // 48 MFMA slots of one k-tile. Slot order: the 16 (l h), then (h l) for b = 0, 1, [barrier], (h l) for b = 2, 3,
  // then the 16 (h h). Every accumulator still gets l h, h l, h h in that order (k_gemm_h3m's per-accumulator order,
  // so C is unchanged), but A's l-plane fragments and B's l-plane fragments b = 0, 1 die in the first half.
  auto mfma1 = [&](const h8v (&fa)[TM][2], const h8v (&fb)[TN][2], int i) {
    int pr, a, b;
    if (i < 16) {
      pr = 0, a = i / 4, b = i % 4;
    } else if (i < 32) {
      pr = 1, b = (i - 16) / 4, a = (i - 16) % 4;
    } else {
      pr = 2, a = (i - 32) / 4, b = (i - 32) % 4;
    }
    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[a][pr == 0 ? 1 : 0], fb[b][pr == 1 ? 1 : 0], acc[a][b], 0, 0,
                                                       0);
  };
  // fragment read j (0..15) of k-tile buffer buf, in the order the next k-tile's slots need them: A l-plane
  // (a = 0..3), B h-plane, A h-plane, B l-plane
  auto read1 = [&](int buf, int j, h8v (&na)[TM][2], h8v (&nbv)[TN][2]) {
    const unsigned short* S = lds16 + buf * STG;
    if (j < 4)
      na[j][1] = *reinterpret_cast<const h8v*>(S + aoff + j * 16 * 64 + ck1);
    else if (j < 8)
      nbv[j - 4][0] = *reinterpret_cast<const h8v*>(S + boff + (j - 4) * 16 * 64 + ck0);
    else if (j < 12)
      na[j - 8][0] = *reinterpret_cast<const h8v*>(S + aoff + (j - 8) * 16 * 64 + ck0);
    else
      nbv[j - 12][1] = *reinterpret_cast<const h8v*>(S + boff + (j - 12) * 16 * 64 + ck1);
  };
  // One k-tile t (fragments in cur): the DMA of k-tile t + 2 (clamped: the last two iterations re-stage the last
  // k-tile into a buffer nobody reads again) is issued as 6 pieces, one every 8 MFMA slots; after the first 24 slots
  // wait for my k-tile t + 1 pieces (the 3 first-half pieces of t + 2 may stay in flight) and barrier (everyone's
  // t + 1 landed; everyone's reads of the buffer t + 2 overwrites, k-tile t - 1, retired before the previous
  // barrier); then k-tile t + 1's 16 fragment reads, one beside each of the next 16 MFMA slots (a burst of 16
  // ds_read_b128 per wave stalls the wave's MFMA issue behind the LDS queue).
  const int nk = ke - kb;
  auto step = [&](int t, const h8v (&fa)[TM][2], const h8v (&fb)[TN][2], h8v (&na)[TM][2], h8v (&nbv)[TN][2]) {
    const int sk = min(kb + t + 2, ke - 1), sb = (t + 2) % 3, rb = (t + 1) % 3;
#pragma unroll
    for (int i = 0; i < 24; ++i) {
      if ((i & 7) == 0) {
        piece(sk, sb, i / 8);
        __builtin_amdgcn_sched_barrier(0);
      }
      mfma1(fa, fb, i);
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 24; i < 48; ++i) {
      if ((i & 7) == 0) piece(sk, sb, 3 + (i - 24) / 8);
      if (i - 24 < 16) read1(rb, i - 24, na, nbv);
      __builtin_amdgcn_sched_barrier(0);
      mfma1(fa, fb, i);
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };

  h8v fa0[TM][2], fb0[TN][2], fa1[TM][2], fb1[TN][2];
  stage(kb, 0);
  stage(min(kb + 1, ke - 1), 1);
  asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  frags(0, fa0, fb0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  int t = 0;
  for (; t + 1 < nk; t += 2) {
    step(t, fa0, fb0, fa1, fb1);
    step(t + 1, fa1, fb1, fa0, fb0);
  }
  if (t < nk) step(t, fa0, fb0, fa1, fb1);
  // drain the DMAs still in flight before the workgroup can exit (their LDS must not be reassigned under them)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = min(m0 + wm * TM * 16 + a * 16 + 4 * hh + r, M - 1);
      rsv[a][r] = rs[args.agather ? args.arow[row] : row];
    }
  // undo the scales: rows of A (2^-e_a), rows of B = columns of C (2^-e_b); 16x16 tile: row 4 hh + r, col rin
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int col = min(n0 + wn * TN * 16 + b * 16 + rin, N - 1);
    const float sb = G.Bs[(size_t)col * (K / 32)];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float ia = __uint_as_float((254u << 23) - __float_as_uint(rsv[a][r]));   // 2^-e_a
        acc[a][b][r] *= ia * sb;
      }
  }

  if (part >= 0) {
    float* w = args.ws + ((size_t)blockIdx.z * (gridDim.x - args.tdp) + part) * (size_t)(TM * TN * 4 * NT);
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) w[(size_t)((a * TN + b) * 4 + r) * NT + tid] = acc[a][b][r];
    return;
  }
  if (m0 + BM <= M && n0 + BN <= N)
    epilogue<BM, BN, WM, WN, EPI, 16, true>(args, G, acc, m0, n0, wm, wn, rin, hh);
  else
    epilogue<BM, BN, WM, WN, EPI, 16, false>(args, G, acc, m0, n0, wm, wn, rin, hh);
}

// Row-wise epilogue of a full tile staged in LDS (tile 49): a wave's 32 x BN fp32 results, written to LDS from the
// accumulators, are read back as pairs of float4 chunks of rows (8 consecutive columns per lane and item), so bias /
// aux are float4 loads, aux and C float4 stores and the fp16x3 planes 16-byte stores of 8 halfs (the register
// epilogue stores 2 bytes per plane and element). Same per-element arithmetic as epilogue() (results bit-identical);
// rows in GEMM order (no crow), no residual.
template <int BN, int EPI_>
__device__ __forceinline__ void epilogue_rows(const GemmArgs& args, const GemmGroup& G, const float* E, int LS, int r0,
                                              int n0, int lane) {
  constexpr bool PL = EPI_ == EPI_GELU_PL || EPI_ == EPI_DGELU_PL;
  constexpr int EPI = EPI_ == EPI_GELU_PL ? EPI_GELU : EPI_ == EPI_DGELU_PL ? EPI_DGELU : EPI_;
  constexpr int CP = BN / 8, NI = 32 * CP / 64, B3 = 3;  // 8-column items per row / per lane; batch of loads
  static_assert(BN % 8 == 0 && NI % B3 == 0, "item batches");
  const int N = args.N;
  float ubw = 0.f, ubb = 0.f;
  if constexpr (PL) {
    const float tw = *args.obw, tb = *(args.obb ? args.obb : args.obw);
    constexpr float f = EPI == EPI_GELU ? 1.0f : 1.25f;
    ubw = f * (float)args.K * tw;
    ubb = args.obb ? f * tb : 0.0f;
  }
#pragma unroll
  for (int i0 = 0; i0 < NI; i0 += B3) {
    f4 v[B3][2], bv[B3][2], ex[B3][2];
    float sc[B3];
#pragma unroll
    for (int j = 0; j < B3; ++j) {
      const int e = lane + 64 * (i0 + j), rr = e / CP, col = 8 * (e - rr * CP);
      const int gr = r0 + rr, gc = n0 + col;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        v[j][h] = *reinterpret_cast<const f4*>(E + rr * LS + col + 4 * h);
        const f4 t = *reinterpret_cast<const f4*>(G.bias ? G.bias + gc + 4 * h : G.A);  // unconditional (dummy address)
        bv[j][h] = G.bias ? t : f4{0.f, 0.f, 0.f, 0.f};
        if constexpr (EPI == EPI_DGELU)
          ex[j][h] = *reinterpret_cast<const f4*>(G.aux + (size_t)gr * args.ldaux + gc + 4 * h);
      }
      if constexpr (PL) {
        const float ia = __uint_as_float((254u << 23) - __float_as_uint(args.escale[gr]));
        const unsigned mx = __float_as_uint(2.0f * (ubw * (32768.0f * ia) + ubb));
        sc[j] = __uint_as_float((268u - max(mx >> 23, 15u)) << 23);
      }
    }
#pragma unroll
    for (int j = 0; j < B3; ++j) {
      const int e = lane + 64 * (i0 + j), rr = e / CP, col = 8 * (e - rr * CP);
      const int gr = r0 + rr, gc = n0 + col;
      f4 o[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float xs[4], ys[4];  // GELU / GELU' four at a time (vv_gelu.h gelu4: the four chains interleave)
#pragma unroll
        for (int q = 0; q < 4; ++q) xs[q] = EPI == EPI_DGELU ? ex[j][h][q] : v[j][h][q] + bv[j][h][q];
        if constexpr (EPI == EPI_GELU) gelu4(xs, ys);
        if constexpr (EPI == EPI_DGELU) dgelu4(xs, ys);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          o[h][q] = EPI == EPI_GELU ? ys[q] : EPI == EPI_DGELU ? v[j][h][q] * ys[q] : v[j][h][q] + bv[j][h][q];
        if constexpr (EPI == EPI_GELU) {
          if (G.aux) {
            f4 pre;
#pragma unroll
            for (int q = 0; q < 4; ++q) pre[q] = v[j][h][q] + bv[j][h][q];
            *reinterpret_cast<f4*>(G.aux + (size_t)gr * args.ldaux + gc + 4 * h) = pre;  // the pre-activation
          }
        }
        if constexpr (!PL) *reinterpret_cast<f4*>(G.C + (size_t)gr * args.ldc + gc + 4 * h) = o[h];
      }
      if constexpr (PL) {
        h8v hv, lv;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float x = o[q >> 2][q & 3] * sc[j];
          hv[q] = (_Float16)x;
          lv[q] = (_Float16)(x - (float)hv[q]);
        }
        unsigned short* pp = args.opl + (size_t)gr * 2 * N + 2 * (gc & ~31) + (gc & 31);  // chunk-interleaved
        *reinterpret_cast<h8v*>(pp) = hv;
        *reinterpret_cast<h8v*>(pp + 32) = lv;
        if (gc == 0) args.ors[gr] = sc[j];
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------------------
// Tile 49: the tile-48 operands (fp16x3 planes, both by LDS-DMA through a 3-stage ring) on 256 x 144 tiles, so that
// the N = 4608 GEMMs at 2048 rows (fc1 forward, the fc2 input gradient) are exactly 8 x 32 = 256 tiles: one round
// on 256 CUs with no split-K tail and no fixup launch (tile 48: 288 tiles = 256 + a 32-tile tail split 3 ways + a
// fixup). 8 waves of 32 rows x 144 columns (2 x 9 fragments of 16 x 16, 54 v_mfma_f32_16x16x32_f16 per k-tile).
// Every accumulator receives l h, h l, h h of each k-tile in that order, as in tile 48, so C is bit-identical to
// tile 48's data-parallel tiles.
//
// LDS stage = [A 256 rows | B 144 rows] x 128 B (h 32 | l 32 halfs per row and k-tile) = 51,200 B; 3 stages.
// DMA pieces (1 KiB = 8 rows each): A 32 (4 per wave), B 18 (2 per wave, a third for waves 0 and 1).
// Per k-tile t (frags of t: A in registers, B column blocks in groups of three, two groups ahead of use):
//   group 0 (blocks 0..2): the reads of group 1 go out after block 0's MFMAs, the first A pieces of k-tile t + 2
//   beside them; group 1 (blocks 3..5): the reads of group 2 after block 3, the last A piece; block 6, then wait for
//   my k-tile t + 1 pieces (vmcnt(4): only the 4 younger A pieces of t + 2 may stay in flight) and my reads, and
//   s_barrier: everyone's t + 1 pieces landed, everyone's reads of buffer t % 3 retired; blocks 7, 8 beside the reads
//   of k-tile t + 1's A fragments and group 0, and the B pieces of k-tile t + 2.
// The compiler waits lgkmcnt(0) before the first MFMA of each group (it does not count in-order LDS reads across these
// loops), so the reads outstanding at those waits are two groups old (r04 schedule measurements: DESIGN §3e).
// Buffer (t + 2) % 3 = (t - 1) % 3 was last read before the barrier of k-tile t - 1, so the DMA of t + 2 may start
// anywhere in k-tile t.
// AG: A's row scales gathered through arow from the producer's physical rows (h4_gather; a compile-time form: as a
// runtime condition the index changed the code of every tile-49 launch and cost 5 % of the closure, r06)
template <int EPI, bool AG = false>
__global__ __launch_bounds__(512, 1) void k_gemm_h5(GemmArgs args, const float* __restrict__ ascale,
                                                    const unsigned short* __restrict__ apl) {
  constexpr int BM = 256, BN = 144, BK = 32, WM = 8, WN = 1, TM = 2, TN = 9;
  constexpr int STG = (BM + BN) * 2 * BK;  // halfs per stage
  typedef float accv __attribute__((ext_vector_type(4)));
  extern __shared__ __attribute__((aligned(16))) unsigned short lds16[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const GemmGroup G = args.g[blockIdx.z];
  const int M = args.M, N = args.N, K = args.K;
  const int ntn = (N + BN - 1) / BN, ntm = (M + BM - 1) / BM;
  // data-parallel, or (r06, gemm_ln) every tile split S = args.tsplit ways along K: chunk-major and XCD-contiguous as
  // tile 48's split (an XCD's workgroups stream the same k-slice of A and B), partials to ws for the fused fixup
  int tile, kb = 0, part = -1, nk = K / BK;
  if (args.tsplit <= 1) {
    tile = xcd_remap(blockIdx.x, ntm * ntn);
  } else {
    const int S = args.tsplit, tt = ntm * ntn, L = xcd_remap(blockIdx.x, tt * S), c = L / tt;
    tile = L - c * tt;
    part = tile * S + c;
    kb = (c * nk) / S;
    nk = ((c + 1) * nk) / S - kb;
  }
  int mb, nb;
  tile_mn(tile, ntm, ntn, mb, nb, args.gm);
  const int m0 = mb * BM, n0 = nb * BN;
  const float* rs = ascale + (size_t)blockIdx.z * M;

  const int prow = lane >> 3, pslot = lane & 7;
  const unsigned short* asrc[4];
  const unsigned short* bsrc[3];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = 8 * (wave + 8 * j) + prow;
    int gr = min(m0 + row, M - 1);
    if (args.apre && args.arow) gr = args.arow[gr];  // producer planes are in physical row order
    asrc[j] = apl + ((size_t)blockIdx.z * M + gr) * 2 * K + 8 * (pslot ^ ((row >> 1) & 7));
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int row = 8 * min(wave + 8 * j, 17) + prow;  // pieces 16, 17: waves 0, 1 only
    const int gn = min(n0 + row, N - 1);
    bsrc[j] = G.Bh + (size_t)gn * 2 * K + 8 * (pslot ^ ((row >> 1) & 7));
  }
  const bool b3 = wave < 2;  // wave-uniform
  auto apiece = [&](int kt, int buf, int j) {
    unsigned short* S = lds16 + buf * STG;
    __builtin_amdgcn_global_load_lds((const void*)(asrc[j] + 2 * kt * BK), (lds_ptr_t)(S + 8 * (wave + 8 * j) * 64), 16,
                                     0, 0);
  };
  auto bpiece = [&](int kt, int buf, int j) {
    unsigned short* S = lds16 + buf * STG;
    __builtin_amdgcn_global_load_lds((const void*)(bsrc[j] + 2 * kt * BK),
                                     (lds_ptr_t)(S + (BM + 8 * (wave + 8 * j)) * 64), 16, 0, 0);
  };
  auto bpieces = [&](int kt, int buf) {
    bpiece(kt, buf, 0);
    bpiece(kt, buf, 1);
    if (b3) bpiece(kt, buf, 2);
  };

  const int rin = lane & 15, hh = lane >> 4;
  const int ck0 = (hh ^ ((rin >> 1) & 7)) * 8, ck1 = ((4 + hh) ^ ((rin >> 1) & 7)) * 8;
  const int aoff = (wave * TM * 16 + rin) * 64, boff = (BM + rin) * 64;
  auto read_a = [&](int buf, h8v (&fa)[TM][2]) {
    const unsigned short* S = lds16 + buf * STG;
#pragma unroll
    for (int a = 0; a < TM; ++a) {
      fa[a][1] = *reinterpret_cast<const h8v*>(S + aoff + a * 16 * 64 + ck1);
      fa[a][0] = *reinterpret_cast<const h8v*>(S + aoff + a * 16 * 64 + ck0);
    }
  };
  auto read_b = [&](int buf, int b, h8v (&fb)[2]) {
    const unsigned short* S = lds16 + buf * STG;
    fb[0] = *reinterpret_cast<const h8v*>(S + boff + b * 16 * 64 + ck0);
    fb[1] = *reinterpret_cast<const h8v*>(S + boff + b * 16 * 64 + ck1);
  };

  accv acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[a][b][r] = 0.0f;

  // the 6 MFMAs of column block b: (l h), (h l), (h h) for a = 0, 1 -- per accumulator tile 48's order
  auto mfma_b = [&](const h8v (&fa)[TM][2], const h8v (&fb)[2], int b) {
#pragma unroll
    for (int a = 0; a < TM; ++a) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[a][1], fb[0], acc[a][b], 0, 0, 0);
#pragma unroll
    for (int a = 0; a < TM; ++a) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[a][0], fb[1], acc[a][b], 0, 0, 0);
#pragma unroll
    for (int a = 0; a < TM; ++a) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[a][0], fb[0], acc[a][b], 0, 0, 0);
  };

  // B blocks read in groups of three, two groups ahead of use (6 slots: g0 / g2 of k-tile t and g1 of k-tile
  // t + 1 in one half, the others in the other half); the reads of group g + 1 go out after the first MFMA block of
  // group g, so the compiler's lgkmcnt waits before each group only find old reads outstanding
  h8v gb[2][3][2];
  auto step4 = [&](int t, const h8v (&fa)[TM][2], h8v (&na)[TM][2], int h) {  // h: half holding groups 0 and 2
    const int cb = t % 3, nbuf = (t + 1) % 3, sb = (t + 2) % 3, sk = kb + min(t + 2, nk - 1);
    // group 0: blocks 0..2 in half h
    mfma_b(fa, gb[h][0], 0);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 3; ++i) read_b(cb, 3 + i, gb[h ^ 1][i]);
    apiece(sk, sb, 0);
    __builtin_amdgcn_sched_barrier(0);
    mfma_b(fa, gb[h][1], 1);
    apiece(sk, sb, 1);
    __builtin_amdgcn_sched_barrier(0);
    mfma_b(fa, gb[h][2], 2);
    apiece(sk, sb, 2);
    __builtin_amdgcn_sched_barrier(0);
    // group 1: blocks 3..5 in half h ^ 1
    mfma_b(fa, gb[h ^ 1][0], 3);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 3; ++i) read_b(cb, 6 + i, gb[h][i]);
    apiece(sk, sb, 3);
    __builtin_amdgcn_sched_barrier(0);
    mfma_b(fa, gb[h ^ 1][1], 4);
    __builtin_amdgcn_sched_barrier(0);
    mfma_b(fa, gb[h ^ 1][2], 5);
    __builtin_amdgcn_sched_barrier(0);
    // group 2: blocks 6..8 in half h; the barrier after block 6 (every read of buffer t % 3 has been waited for)
    mfma_b(fa, gb[h][0], 6);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    read_a(nbuf, na);
#pragma unroll
    for (int i = 0; i < 3; ++i) read_b(nbuf, i, gb[h ^ 1][i]);  // next k-tile's group 0 (its half is h ^ 1)
    bpieces(sk, sb);
    __builtin_amdgcn_sched_barrier(0);
    mfma_b(fa, gb[h][1], 7);
    __builtin_amdgcn_sched_barrier(0);
    mfma_b(fa, gb[h][2], 8);
    __builtin_amdgcn_sched_barrier(0);
  };
  // prologue: k-tiles 0 and 1 in flight, wait for 0, its A fragments and B blocks 0, 1
  h8v fa0[TM][2], fa1[TM][2];
#pragma unroll
  for (int j = 0; j < 4; ++j) apiece(kb, 0, j);
  bpieces(kb, 0);
#pragma unroll
  for (int j = 0; j < 4; ++j) apiece(kb + min(1, nk - 1), 1, j);
  bpieces(kb + min(1, nk - 1), 1);
  if (b3)
    asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  read_a(0, fa0);
#pragma unroll
  for (int i = 0; i < 3; ++i) read_b(0, i, gb[0][i]);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  int t = 0;
  for (; t + 1 < nk; t += 2) {
    step4(t, fa0, fa1, 0);
    step4(t + 1, fa1, fa0, 1);
  }
  if (t < nk) step4(t, fa0, fa1, 0);
  // drain the DMAs still in flight before the workgroup can exit (their LDS must not be reassigned under them)
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");

  // undo the scales: rows of A (2^-e_a), rows of B = columns of C (2^-e_b); 16x16 fragment: row 4 hh + r, col rin
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int col = min(n0 + b * 16 + rin, N - 1);
    const float sbv = G.Bs[(size_t)col * (K / 32)];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = min(m0 + wave * TM * 16 + a * 16 + 4 * hh + r, M - 1);
        const float ia = __uint_as_float((254u << 23) - __float_as_uint(rs[AG ? args.arow[row] : row]));  // 2^-e_a
        acc[a][b][r] *= ia * sbv;
      }
  }
  if (part >= 0) {
    // the chunk's partial in fragment order: element (row 32 wave + 16 a + 4 hh + r, column 16 b + rin) at
    // ((a * TN + b) * 4 + r) * 512 + 64 wave + lane (fixup_stage49 reads it back)
    float* w = args.ws + ((size_t)blockIdx.z * gridDim.x + part) * (size_t)(TM * TN * 4 * 512);
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) w[(size_t)((a * TN + b) * 4 + r) * 512 + tid] = acc[a][b][r];
    return;
  }
  if (EPI != EPI_RESID && !args.crow && m0 + BM <= M && n0 + BN <= N && (args.ldc & 3) == 0 &&
      (args.ldaux & 3) == 0) {
    // full tile: through LDS to a row-wise epilogue (every wave's fragment reads retired first; each wave then
    // writes and reads back only its own 32 rows)
    constexpr int LS = BN + 4;
    __syncthreads();
    float* E = reinterpret_cast<float*>(lds16) + wave * 32 * LS;
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) E[(a * 16 + 4 * hh + r) * LS + b * 16 + rin] = acc[a][b][r];
    epilogue_rows<BN, EPI>(args, G, E, LS, m0 + wave * 32, n0, lane);
    return;
  }
  if (m0 + BM <= M && n0 + BN <= N)
    epilogue<BM, BN, WM, WN, EPI, 16, true>(args, G, acc, m0, n0, wave, 0, rin, hh);
  else
    epilogue<BM, BN, WM, WN, EPI, 16, false>(args, G, acc, m0, n0, wave, 0, rin, hh);
}

template <int EPI, int BM>
static hipError_t launch_h3m_k(const GemmArgs& a, hipStream_t s, dim3 grid, size_t lds, int tail, const float* sc) {
  if (hipError_t e = set_lds_limit((const void*)k_gemm_h3m<EPI, BM>, lds)) return e;
  hipLaunchKernelGGL((k_gemm_h3m<EPI, BM>), grid, dim3(2 * BM), lds, s, a, sc);
  if (tail)  // y: the 4 fragment rows of each wave
    hipLaunchKernelGGL((k_gemm_fixup_sub16<BM, 128, BM / 64, 2, EPI>), dim3(tail, 4, a.ngroups), dim3(2 * BM), 0, s, a);
  return hipGetLastError();
}

template <int EPI, int BM>
static hipError_t launch_h3_k(const GemmArgs& a, hipStream_t s, dim3 grid, size_t lds, int tail, const float* sc) {
  if (hipError_t e = set_lds_limit((const void*)k_gemm_h3<EPI, BM>, lds)) return e;
  hipLaunchKernelGGL((k_gemm_h3<EPI, BM>), grid, dim3(2 * BM), lds, s, a, sc);
  if (tail)
    hipLaunchKernelGGL((k_gemm_fixup_sub<BM, 128, BM / 64, 2, EPI>), dim3(tail, 4, a.ngroups), dim3(2 * BM), 0, s,
                       a);  // y: the 2 x 2 32x32 sub-blocks of each wave
  return hipGetLastError();
}

constexpr size_t kWsFloats = (size_t)1 << 24;      // 64 MB: split-K partials (3 x 144 tiles of 128x128)
constexpr size_t kScaleFloats = (size_t)1 << 19;   // then the A row scales of GEMM_SPLIT16 (groups x M)

// requires fp16 planes for every group's B (registered weights) and a workspace for the A row scales; the
// bf16x6 pipelined kernel otherwise
static bool h3_ready(const GemmArgs& a) {
  bool pre = a.ws && (size_t)a.ngroups * a.M <= kScaleFloats;
  for (int g = 0; g < a.ngroups; ++g) pre = pre && a.g[g].Bh && a.g[g].Bs;
  return pre;
}

// tile 48: the A split pass (k_rowsplit into the caller's plane workspace, GEMM row order) + k_gemm_h4
static bool h4_ready(const GemmArgs& a) {
  if (a.K % 32 || a.K > 4608) return false;
  if (a.apre) return a.ascale != nullptr;
  return a.apl && (size_t)a.ngroups * a.M * 2 * (size_t)a.K <= a.apl_halfs;
}

template <int EPI>
static hipError_t launch_h4_k(const GemmArgs& a, hipStream_t s, dim3 grid, size_t lds, int tail, const float* sc,
                              const unsigned short* planes) {
  if (hipError_t e = set_lds_limit((const void*)k_gemm_h4<EPI>, lds)) return e;
  hipLaunchKernelGGL((k_gemm_h4<EPI>), grid, dim3(512), lds, s, a, sc, planes);
  if (tail && !a.nofix) {  // y: the 4 fragment rows of each wave (4x the workgroups of a per-tile fixup)
    count_launch(CNT_SPLITK_FIXUP);
    hipLaunchKernelGGL((k_gemm_fixup_sub16<256, 128, 4, 2, EPI>), dim3(tail, 4, a.ngroups), dim3(512), 0, s, a);
  }
  return hipGetLastError();
}

template <int EPI, bool AG = false>
static hipError_t launch_h5_k(const GemmArgs& a, hipStream_t s, dim3 grid, size_t lds, const float* sc,
                              const unsigned short* planes) {
  if (hipError_t e = set_lds_limit((const void*)k_gemm_h5<EPI, AG>, lds)) return e;
  hipLaunchKernelGGL((k_gemm_h5<EPI, AG>), grid, dim3(512), lds, s, a, sc, planes);
  return hipGetLastError();
}

// tiles 48 and 49 (t49: 256 x 144 tiles, data-parallel only)
static hipError_t launch_h4(const GemmArgs& a, hipStream_t s, bool t49 = false) {
  if (a.K % 32 || a.ksplit % 32 || !h3_ready(a) || !h4_ready(a)) return hipErrorInvalidValue;
  // tile 49 splits only for gemm_ln (every tile, the fused fixup + LayerNorm sums the partials)
  if (t49 && ((a.tsplit > 1) != (a.nofix != 0) || a.tdp)) return hipErrorInvalidValue;
  float* sc = a.ws + kWsFloats;
  const unsigned short* planes = a.apl;
  bool agather = false;
  if (a.apre) {
    // planes and scales from the producer (physical rows); the kernel gathers plane rows through arow itself
    planes = a.apre;
    const Tuning& TU = a.tune ? *a.tune : kDefaultTuning;
    if (!a.arow) {
      sc = const_cast<float*>(a.ascale);
    } else if (!a.opl && TU.h4_gather && (!t49 || a.epi == EPI_STORE || a.epi == EPI_RESID)) {
      // tiles 48 / 49 read ascale[arow[r]] themselves (no plane epilogue here; tile 49: k_gemm_h5<EPI, true>)
      sc = const_cast<float*>(a.ascale);
      agather = true;
    } else {
      count_launch(CNT_GATHER_SCALES);
      hipLaunchKernelGGL(k_gather_scales, dim3((a.M + 255) / 256, 1, a.ngroups), dim3(256), 0, s, a.ascale, a.arow,
                         sc, a.M);
    }
  } else {
    const dim3 grid((a.M + 3) / 4, 1, a.ngroups);
    const int nv = (a.K + 255) / 256;
    count_launch(CNT_ROWSPLIT);
    switch (nv <= 5 ? 5 : nv <= 9 ? 9 : nv <= 14 ? 14 : 18) {
      case 5: hipLaunchKernelGGL(k_rowsplit<5>, grid, dim3(256), 0, s, a, sc, a.apl); break;
      case 9: hipLaunchKernelGGL(k_rowsplit<9>, grid, dim3(256), 0, s, a, sc, a.apl); break;
      case 14: hipLaunchKernelGGL(k_rowsplit<14>, grid, dim3(256), 0, s, a, sc, a.apl); break;
      default: hipLaunchKernelGGL(k_rowsplit<18>, grid, dim3(256), 0, s, a, sc, a.apl); break;
    }
  }
  GemmArgs b = a;
  b.escale = sc;  // the plane-writing epilogues bound |C| from the row scales the products used
  b.agather = agather ? 1 : 0;
  if (t49) {
    const size_t lds = 3 * (2 * (256 + 144) * 32) * sizeof(unsigned short);
    const dim3 grid(((a.N + 143) / 144) * ((a.M + 255) / 256) * std::max(a.tsplit, 1), 1, a.ngroups);
    switch (a.epi) {
      case EPI_STORE:
        return agather ? launch_h5_k<EPI_STORE, true>(b, s, grid, lds, sc, planes)
                       : launch_h5_k<EPI_STORE>(b, s, grid, lds, sc, planes);
      case EPI_GELU:
        return a.opl ? launch_h5_k<EPI_GELU_PL>(b, s, grid, lds, sc, planes)
                     : launch_h5_k<EPI_GELU>(b, s, grid, lds, sc, planes);
      case EPI_RESID:
        return agather ? launch_h5_k<EPI_RESID, true>(b, s, grid, lds, sc, planes)
                       : launch_h5_k<EPI_RESID>(b, s, grid, lds, sc, planes);
      case EPI_DGELU:
        return a.opl ? launch_h5_k<EPI_DGELU_PL>(b, s, grid, lds, sc, planes)
                     : launch_h5_k<EPI_DGELU>(b, s, grid, lds, sc, planes);
      default: return hipErrorInvalidValue;
    }
  }
  const size_t lds = 3 * (2 * (256 + 128) * 32) * sizeof(unsigned short);
  const int T = ((a.N + 127) / 128) * ((a.M + 255) / 256);
  const int tail = a.tsplit > 1 ? T - a.tdp : 0;
  dim3 grid(tail ? a.tdp + tail * a.tsplit : T, 1, a.ngroups);
  switch (a.epi) {
    case EPI_STORE: return launch_h4_k<EPI_STORE>(b, s, grid, lds, tail, sc, planes);
    case EPI_GELU:
      return a.opl ? launch_h4_k<EPI_GELU_PL>(b, s, grid, lds, tail, sc, planes)
                   : launch_h4_k<EPI_GELU>(b, s, grid, lds, tail, sc, planes);
    case EPI_RESID: return launch_h4_k<EPI_RESID>(b, s, grid, lds, tail, sc, planes);
    case EPI_DGELU:
      return a.opl ? launch_h4_k<EPI_DGELU_PL>(b, s, grid, lds, tail, sc, planes)
                   : launch_h4_k<EPI_DGELU>(b, s, grid, lds, tail, sc, planes);
    default: return hipErrorInvalidValue;
  }
}

template <int BM, int MF = 32>
static hipError_t launch_h3(const GemmArgs& a, hipStream_t s) {
  if (a.K % 32 || a.ksplit % 32) return hipErrorInvalidValue;
  if (!h3_ready(a)) return hipErrorInvalidValue;  // gemm_nt routes such GEMMs to tile 34 before sizing the split
  const float* sc = a.ws + kWsFloats;
  if (a.ascale_phys && !a.arow)
    sc = a.ascale;  // row scales written by the producer of A (LayerNorm), already in GEMM row order
  else if (a.ascale_phys)  // gathered A: the producer's scales permuted into GEMM row order (no pass over A)
    hipLaunchKernelGGL(k_gather_scales, dim3((a.M + 255) / 256, 1, a.ngroups), dim3(256), 0, s, a.ascale, a.arow,
                       const_cast<float*>(sc), a.M);
  else
    launch_rowscale(a, const_cast<float*>(sc), s);
  const size_t lds = 2 * (2 * (BM + 128) * 32) * sizeof(unsigned short);
  const int T = ((a.N + 127) / 128) * ((a.M + BM - 1) / BM);
  const int tail = a.tsplit > 1 ? T - a.tdp : 0;
  dim3 grid(tail ? a.tdp + tail * a.tsplit : T, 1, a.ngroups);
  switch (a.epi) {
    case EPI_STORE: return MF == 16 ? launch_h3m_k<EPI_STORE, BM>(a, s, grid, lds, tail, sc)
                              : launch_h3_k<EPI_STORE, BM>(a, s, grid, lds, tail, sc);
    case EPI_GELU: return MF == 16 ? launch_h3m_k<EPI_GELU, BM>(a, s, grid, lds, tail, sc)
                              : launch_h3_k<EPI_GELU, BM>(a, s, grid, lds, tail, sc);
    case EPI_RESID: return MF == 16 ? launch_h3m_k<EPI_RESID, BM>(a, s, grid, lds, tail, sc)
                              : launch_h3_k<EPI_RESID, BM>(a, s, grid, lds, tail, sc);
    case EPI_DGELU: return MF == 16 ? launch_h3m_k<EPI_DGELU, BM>(a, s, grid, lds, tail, sc)
                              : launch_h3_k<EPI_DGELU, BM>(a, s, grid, lds, tail, sc);
    default: return hipErrorInvalidValue;
  }
}

// the GEMM kernels of the library, by tile hint (vv_gemm's `tile`; gemm_nt rejects every other value):
//   exact f32 MFMA   0: 128x128   2: 64x64   4: 32x64            (GEMM_F32)
//   bf16x6 split    24: 64x64    34: pipelined 128x128           (GEMM_SPLIT, short-K GEMMs of GEMM_SPLIT16)
//   fp16x3 split    36: 128x128, 44: 256x128 (8 waves of 64x64); 46 / 47: the same on 16x16x32 MFMAs
static bool h3_tile(int t) { return t == 36 || t == 44 || t == 46 || t == 47 || t == 48 || t == 49; }
bool gemm_plane_tile(int t) { return t == 48 || t == 49; }
const Tuning kDefaultTuning{};
int* tuning_field(Tuning& t, const char* key) {
  if (!key) return nullptr;
  const std::string k(key);
  if (k == "h3_mink") return &t.h3_mink;
  if (k == "fc_h3_mink") return &t.fc_h3_mink;
  if (k == "h3_big") return &t.h3_big;
  if (k == "h3_mf16") return &t.h3_mf16;
  if (k == "small_split") return &t.small_split;
  if (k == "small_split_minkt") return &t.small_split_minkt;
  if (k == "tail_minkt") return &t.tail_minkt;
  if (k == "ln_scales") return &t.ln_scales;
  if (k == "win_attn") return &t.win_attn;
  if (k == "win_mfma") return &t.win_mfma;
  if (k == "fuse_mlp") return &t.fuse_mlp;
  if (k == "mlp_hc") return &t.mlp_hc;
  if (k == "fuse_attn") return &t.fuse_attn;
  if (k == "attn_mfma") return &t.attn_mfma;
  if (k == "gelu_planes") return &t.gelu_planes;
  if (k == "attn_planes") return &t.attn_planes;
  if (k == "fixup_ln") return &t.fixup_ln;
  if (k == "h4") return &t.h4;
  if (k == "ln_planes") return &t.ln_planes;
  if (k == "gattn") return &t.gattn;
  if (k == "gattn_qf") return &t.gattn_qf;
  if (k == "h4_small") return &t.h4_small;
  if (k == "h4_split_minkt") return &t.h4_split_minkt;
  if (k == "h5") return &t.h5;
  if (k == "h4_gather") return &t.h4_gather;
  if (k == "fixup_ln_rows") return &t.fixup_ln_rows;
  if (k == "fc_conv_mf") return &t.fc_conv_mf;
  if (k == "grid_fused") return &t.grid_fused;
  if (k == "fixup_stage") return &t.fixup_stage;
  if (k == "h5_split") return &t.h5_split;
  if (k == "host_wait") return &t.host_wait;
  if (k == "patch_pers") return &t.patch_pers;
  if (k == "fixup_ln_cross") return &t.fixup_ln_cross;
  if (k == "bs_tile") return &t.bs_tile;
  return nullptr;
}
bool tuning_value_ok(const char* key, int v) {
  const std::string k(key ? key : "");
  if (k == "h3_mink" || k == "fc_h3_mink") return v >= 0;
  if (k == "small_split_minkt" || k == "tail_minkt" || k == "h4_split_minkt") return v >= 1;
  if (k == "mlp_hc") return v == 0 || v == 2 || v == 32 || v == 64;  // vv_tower.hip mlp_run
  if (k == "gattn_qf") return v == 1 || v == 2;
  if (k == "grid_fused") return v >= 0 && v <= 2;
  if (k == "fuse_mlp") return v >= 0 && v <= 3;
  if (k == "fuse_attn") return v >= 0 && v <= 3;
  if (k == "bs_tile") return v >= 24 && v <= 27;
  if (k == "patch_pers") return v == 0 || v == 1 || v == 2 || v == 4;
  return v == 0 || v == 1;  // every other knob is a switch
}

bool valid_tile(int t) { return t == 0 || t == 2 || t == 4 || (t >= 24 && t <= 27) || t == 34 || h3_tile(t); }

static hipError_t launch_variant(int t, const GemmArgs& a, hipStream_t s) {
  switch (t) {
    case 0: return launch_tile<128, 128, 32, 2, 2>(a, s);
    case 2: return launch_tile<64, 64, 32, 2, 2>(a, s);
    case 4: return launch_tile<32, 64, 32, 1, 2>(a, s);
    case 24: return launch_bs<64, 64, 2, 2>(a, s);
    case 25: return launch_bs<128, 64, 2, 2>(a, s);      // bf16x6, 128 x 64 (r05 short-K experiments)
    case 26: return launch_bs<64, 64, 2, 2, 3>(a, s);    // bf16x6, 64 x 64, loads two k-tiles ahead
    case 27: return launch_bs<64, 64, 2, 2, 1>(a, s);    // bf16x6, 64 x 64, one LDS buffer (24 KB: more workgroups per CU)
    case 34: return launch_bs2(a, s);
    case 36: return launch_h3<128>(a, s);
    case 44: return launch_h3<256>(a, s);
    case 46: return launch_h3<128, 16>(a, s);
    case 47: return launch_h3<256, 16>(a, s);
    case 48: return launch_h4(a, s);
    case 49: return launch_h4(a, s, true);
    default: return hipErrorInvalidValue;
  }
}

static long tiles_of(const GemmArgs& a, int bm, int bn) {
  return (long)((a.M + bm - 1) / bm) * ((a.N + bn - 1) / bn) * a.ngroups;
}

// tile choice (measured on MI355X, tools/gemm_bench.py; 4 WGs/CU resident): high-occupancy 64x64 tiles beat
// larger tiles on every decoder shape at M = 2048 / 8192; 32x64 when 64x64 leaves CUs idle


struct SplitArena {
  const float* base;
  size_t n;
  const unsigned short* planes;
};
static std::vector<SplitArena> g_split;   // registered weight arenas (host-side lookup per GEMM launch)

static size_t split16_scale_off(size_t n) { return (10 * n + 255) & ~size_t(255); }  // bytes
size_t split_arena_bytes(size_t n) { return split16_scale_off(n) + (n / 32 + 1) * sizeof(float); }

void register_split_arena(const float* base, size_t n, const unsigned short* planes) {
  unregister_split_arena(base);
  g_split.push_back({base, n, planes});
}
void unregister_split_arena(const float* base) {
  for (size_t i = 0; i < g_split.size(); ++i)
    if (g_split[i].base == base) {
      g_split.erase(g_split.begin() + i);
      return;
    }
}
static const SplitArena* arena_of(const float* B) {
  for (const SplitArena& a : g_split)
    if (B >= a.base && B < a.base + a.n) return &a;
  return nullptr;
}
static const unsigned short* split_planes_exact(const float* A) {
  for (const SplitArena& a : g_split)
    if (A == a.base) return a.planes;
  return nullptr;
}
static const unsigned short* split_planes_of(const float* B) {
  const SplitArena* a = arena_of(B);
  return a ? a->planes + 3 * (size_t)(B - a->base) : nullptr;
}
// fp16 planes and row scales of B (GEMM_SPLIT16); null unless B's offset in its arena is a multiple of 32
static void split16_of(const float* B, int K, const unsigned short*& h, const float*& sc) {
  h = nullptr;
  sc = nullptr;
  const SplitArena* a = arena_of(B);
  if (!a || K % 32) return;
  const size_t o = (size_t)(B - a->base);
  if (o % 32) return;
  h = a->planes + 3 * a->n + 2 * o;
  sc = reinterpret_cast<const float*>(reinterpret_cast<const char*>(a->planes) + split16_scale_off(a->n)) + o / 32;
}

// fp16 split of whole rows (one workgroup per row): e = 141 - exponent(max |x|) puts the row maximum in
// [2^14, 2^15); h = fp16(x 2^e), l = fp16(x 2^e - h) (both round-to-nearest, the residual is exact in fp32);
// row scale 2^-e at sc[r * K / 32]
__global__ __launch_bounds__(256) void k_split16_rows(const float* __restrict__ src, unsigned short* __restrict__ dst,
                                                      float* __restrict__ sc, int K) {
  __shared__ unsigned red[4];
  const int r = blockIdx.x, tid = threadIdx.x;
  const float* x = src + (size_t)r * K;
  unsigned mx = 0;
  for (int k = tid; k < K; k += 256) mx = max(mx, __float_as_uint(fabsf(x[k])));
  mx = lane_max<64>(mx);
  if ((tid & 63) == 0) red[tid >> 6] = mx;
  __syncthreads();
  mx = max(max(red[0], red[1]), max(red[2], red[3]));
  const unsigned E = max(mx >> 23, 15u);
  const float s = __uint_as_float((268u - E) << 23);
  unsigned short* d = dst + (size_t)r * 2 * K;
  for (int k = tid; k < K; k += 256) {
    const float v = x[k] * s;
    const _Float16 h = (_Float16)v;
    const _Float16 l = (_Float16)(v - (float)h);
    d[2 * (k & ~31) + (k & 31)] = __builtin_bit_cast(unsigned short, h);  // chunk-interleaved planes
    d[2 * (k & ~31) + 32 + (k & 31)] = __builtin_bit_cast(unsigned short, l);
  }
  if (tid == 0) sc[(size_t)r * K / 32] = __uint_as_float((E - 14u) << 23);
}

void fp16_planes_of(const float* W, int K, const unsigned short** h, const float** sc) {
  split16_of(W, K, *h, *sc);
}

hipError_t split_registered(const float* W, size_t n, int K, hipStream_t s) {
  if (!n) return hipSuccess;
  if (K <= 0 || n % K) return hipErrorInvalidValue;
  const SplitArena* a = arena_of(W);
  if (!a || W + n > a->base + a->n) return hipErrorInvalidValue;
  hipError_t e = split_planes(W, const_cast<unsigned short*>(a->planes) + 3 * (size_t)(W - a->base), n, K, s);
  if (e != hipSuccess) return e;
  const unsigned short* h;
  const float* sc;
  split16_of(W, K, h, sc);
  if (!h) return hipSuccess;  // K or offset not 32-aligned: no GEMM can use the fp16 planes anyway
  hipLaunchKernelGGL(k_split16_rows, dim3((unsigned)(n / K)), dim3(256), 0, s, W, const_cast<unsigned short*>(h),
                     const_cast<float*>(sc), K);
  return hipGetLastError();
}
size_t gemm_ws_floats() { return kWsFloats + kScaleFloats; }

__global__ __launch_bounds__(256) void k_absmax(const float* __restrict__ x, size_t n, unsigned* __restrict__ out) {
  __shared__ unsigned red[4];
  unsigned mx = 0;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    mx = max(mx, __float_as_uint(fabsf(x[i])));
  mx = lane_max<64>(mx);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) atomicMax(out, max(max(red[0], red[1]), max(red[2], red[3])));  // |x| bits order as floats
}
hipError_t absmax(const float* x, size_t n, float* out, hipStream_t s) {
  if (!x || !out || !n) return hipErrorInvalidValue;
  if (hipError_t e = hipMemsetAsync(out, 0, sizeof(float), s)) return e;
  const unsigned g = (unsigned)std::min<size_t>(512, (n + 4095) / 4096);
  hipLaunchKernelGGL(k_absmax, dim3(g), dim3(256), 0, s, x, n, reinterpret_cast<unsigned*>(out));
  return hipGetLastError();
}

// tile choice (measured on MI355X, tools/gemm_bench.py, tools/gemm_split_check.py)
static int pick_tile(const GemmArgs& a) {
  const Tuning& T = a.tune ? *a.tune : kDefaultTuning;
  if (a.math == GEMM_SPLIT16 || a.math == GEMM_SPLIT) {
    // GEMM_SPLIT16: fp16x3 128x128 for the deep-K GEMMs that give >= 128 tiles; the bf16x6 64x64 kernel for the
    // short-K / few-tile GEMMs of the Swin towers (its pipeline prologue and epilogue dominate there).
    // h3_mink: smallest K sent to the fp16x3 kernel.
    // h3_big: 256x128 tiles where they measured faster than 128x128 (profiles/r02/h3big: 2048 rows x (N 3456,
    // K 1152): 69.0 vs 73.4 us, (1152, 4608): 93.1 vs 98.5, (1152, 3456): 76.1 vs 79.3; slower at N 4608 x K 1152
    // and far slower at 1152 x 1152, where 72 tiles leave most CUs idle).
    // h3_mf16: the 16x16x32-MFMA form of the 256x128 kernel for N 2048..4095 x short K (profiles/r02/mf16:
    // 2048 x 3456 x 1152 at 64.3 vs 69.6 us; slower on the deep-K shapes)
    const int h3_mink = std::max(64, a.h3_mink > 0 ? a.h3_mink : T.h3_mink), h3_big = T.h3_big, h3_mf16 = T.h3_mf16;
    if (a.math == GEMM_SPLIT16 && a.K >= h3_mink && h3_big && tiles_of(a, 256, 128) >= 64 &&
        (a.K >= 3456 || (a.N >= 2048 && a.N < 4096)))
      return h3_mf16 && a.K < 3456 ? 47 : 44;
    if (a.math == GEMM_SPLIT16 && a.K >= h3_mink && tiles_of(a, 128, 128) >= 128) return 36;
    // pipelined 128x128 (64x64 per wave, one barrier per k-tile) for the deep-K GEMMs that fill the chip with
    // 128x128 tiles (LG stage, K >= 1152); 64x64 tiles otherwise (few tiles, or K too short to pipeline: Tuning.bs_tile,
    // one LDS buffer since r06)
    const long t128 = tiles_of(a, 128, 128);
    if (a.K >= 768 && (t128 >= 256 || (t128 >= 128 && a.K <= 1536))) return 34;
    return T.bs_tile;
  }
  // f32 MFMA: high-occupancy 64x64 tiles beat larger tiles on every decoder shape at M = 2048 / 8192;
  // 32x64 when 64x64 leaves CUs idle
  if (tiles_of(a, 64, 64) >= 512) return 2;
  return 4;
}

// tile edge of each variant (for the tail split)
static void variant_tile(int t, int& bm, int& bn, int& bk) {
  bk = 32;
  bm = t == 44 || t == 47 || t == 48 || t == 49 ? 256 : t == 0 || t == 25 || t >= 34 ? 128 : t == 4 ? 32 : 64;
  bn = t == 49 ? 144 : t == 0 || t >= 34 ? 128 : 64;
}

// the routed tile plus the fallbacks gemm_nt applies (no fp16 B planes: bf16x6 34; no A-plane workspace: 47);
// fills the fp16 B plane pointers of `a` (Bh, Bs) as a side effect; -1 for an invalid hint
static int resolve_tile(GemmArgs& a, int tile_hint) {
  int t = tile_hint >= 0 ? tile_hint : pick_tile(a);
  if (!valid_tile(t)) return -1;
  const Tuning& TU = a.tune ? *a.tune : kDefaultTuning;
  // tile 48 wherever the 256x128 fp16x3 tiles run, and for the 128x128-routed ones that still give >= 144 256-row
  // tiles (N 4608 at 2048 rows: fc1 forward, the fc2 input gradient; same-box 2048 x 4608 x 1152: 75.9 us incl. the
  // split pass vs 91.3 / ~90 for tiles 47 / 36); the 72-tile 1152 x 1152 GEMMs stay on 128x128 tiles
  // h4_small: also the 128x128-routed GEMMs with 64..143 256-row tiles (1152 x 1152 at 2048 rows: 72 tiles), which
  // then split along K over the whole chip (tile-48 chunks of >= h4_split_minkt k-tiles, below)
  if (tile_hint < 0 && TU.h4 && a.math == GEMM_SPLIT16 &&
      (t == 44 || t == 47 || (t == 36 && tiles_of(a, 256, 128) >= (TU.h4_small ? 64 : 144))))
    t = 48;
  for (int g = 0; g < a.ngroups; ++g) {
    a.g[g].Bh = nullptr;
    a.g[g].Bs = nullptr;
    if (h3_tile(t) && (!a.ldb || a.ldb == a.K)) split16_of(a.g[g].B, a.K, a.g[g].Bh, a.g[g].Bs);
  }
  // the fp16x3 kernels need every group's fp16 B planes and the scale workspace; without them the GEMM runs the
  // pipelined bf16x6 kernel. Decided BEFORE the tile geometry: the split-K tail sizes its partials from the tile
  // edge of the kernel that actually runs (a 256-row tile count with 128-row fallback tiles overran ws).
  if (h3_tile(t) && !h3_ready(a)) t = 34;
  if ((t == 48 || t == 49) && !h4_ready(a)) t = 47;  // no plane workspace (or too small): the in-loop-split kernel
  // tile 49 (256 x 144) where its tiles fill whole rounds of the chip and tile 48's leave a split-K tail: N 4608 at
  // 2048 rows = 256 tiles (tile 48: 288 = 256 + 32); same operands and per-element products as tile 48
  if (t == 48 && tile_hint < 0 && TU.h5 && a.N % 144 == 0) {
    const long P = device_cus(), t48 = tiles_of(a, 256, 128), t49 = tiles_of(a, 256, 144);
    if (t48 % P != 0 && t49 % P == 0) t = 49;
  }
  return t;
}

int gemm_tile_of(const GemmArgs& a_in, int tile_hint) {
  GemmArgs a = a_in;
  if (!a.ws) a.ws = reinterpret_cast<float*>(1);  // h3_ready only checks that a workspace is passed
  return resolve_tile(a, tile_hint);
}

// validation, tile routing and the split / tile-order plan of one GEMM (gemm_nt, gemm_ln); t = the kernel's tile
static hipError_t gemm_prepare(GemmArgs& a, int tile_hint, float* ws, int& t) {
  if (a.M <= 0 || a.N <= 0 || a.ngroups <= 0 || a.ngroups > kMaxGroups) return hipErrorInvalidValue;
  if (a.K % KALIGN != 0 || a.ksplit % KALIGN != 0 || a.ksplit <= 0 || a.ksplit > a.K) return hipErrorInvalidValue;
  if ((a.lda & 3) || (a.lda2 & 3) || (a.K & 3) || (a.ldb & 3) || (a.ldb && a.ldb < a.K)) return hipErrorInvalidValue;
  if (a.apre && (!a.ascale || a.g[0].A2)) return hipErrorInvalidValue;
  const int num_cu = device_cus();
  a.tdp = 0;
  a.tsplit = 1;
  a.ws = ws;
  a.ascale_phys = 0;
  const Tuning& TU = a.tune ? *a.tune : kDefaultTuning;
  // ln_scales = 0: ignore producer scales, run k_rowscale for every fp16x3 GEMM
  if (a.ascale && TU.ln_scales) {
    bool ok = true;
    for (int g = 0; g < a.ngroups; ++g) ok = ok && !a.g[g].A2;
    a.ascale_phys = ok ? 1 : 0;
  }
  t = resolve_tile(a, tile_hint);
  if (t < 0) return hipErrorInvalidValue;
  // producer planes are only read by tiles 48 / 49; every other kernel reads A itself (which the producer then wrote)
  if (a.apre && !gemm_plane_tile(t)) return hipErrorInvalidValue;
  // plane-writing epilogues: tiles 48 / 49, GELU / DGELU, one group, output rows in GEMM order, N in whole k-tiles
  if (a.opl && (!gemm_plane_tile(t) || (a.epi != EPI_GELU && a.epi != EPI_DGELU) || a.ngroups != 1 || a.crow || a.N % 32 ||
                !a.ors || !a.obw))
    return hipErrorInvalidValue;
  for (int g = 0; g < a.ngroups; ++g) {
    a.g[g].Bp = (t >= 21 && (!a.ldb || a.ldb == a.K)) ? split_planes_of(a.g[g].B) : nullptr;
    // activations are never registered by the engine; a registered A (tests, vv_gemm) must be a matrix's start
    a.g[g].Ap = (t >= 21 && t < 36 && !a.g[g].A2 && !a.g[g].Ap) ? split_planes_exact(a.g[g].A) : a.g[g].Ap;
  }
  {
    // grouped tile order: one XCD runs ~T/8 consecutive logical tiles, a gm x (T/8/gm) block re-reading gm A
    // m-blocks (BM rows) and T/8/gm B n-blocks (BN rows); gm = sqrt(T/8 x BN/BM) minimises those bytes
    // (2048 x 3456 x 1152 on 256 x 128 tiles: 8 -> 4, FETCH 94 -> 73 MB per launch, profiles/r02/tile_group/)
    int bm, bn, bk;
    variant_tile(t, bm, bn, bk);
    const int ntm = (a.M + bm - 1) / bm, ntn = (a.N + bn - 1) / bn;
    const double tx = (double)ntm * ntn / 8.0;
    a.gm = std::max(1, std::min(ntm, (int)std::lround(std::sqrt(tx * bn / bm))));
  }
  if (ws && a.ngroups == 1) {
    int bm, bn, bk;
    variant_tile(t, bm, bn, bk);
    const int T = ((a.N + bn - 1) / bn) * ((a.M + bm - 1) / bm);
    const int P = num_cu, nkt = a.K / bk;
    const int tdp = (T / P) * P, tail = T - tdp;
    if (tdp > 0 && tail > 0 && tail <= P / 2 && t != 49) {
      // chunks of >= 12 k-tiles: below that the fixup launch and partial traffic cost more than the tail
      const int tail_minkt = std::max(1, TU.tail_minkt);  // k-tiles per tail chunk at least
      int S = std::min(P / tail, nkt / tail_minkt);
      const size_t tile_f = (size_t)bm * bn;
      while (S > 1 && (size_t)tail * S * tile_f > kWsFloats) --S;
      if (S > 1) {
        a.tdp = tdp;
        a.tsplit = S;
      }
    } else if (tdp == 0 && h3_tile(t) && t != 49 && TU.small_split) {
      // fewer fp16x3 tiles than CUs (N = 1152 at 2048 tokens: 144 tiles): every tile split along K so that
      // two workgroups share most CUs (the co-resident pair overlaps one's staging with the other's MFMAs)
      // chunks of >= 24 k-tiles (K >= 2304 at S = 3): at K = 1152 the fixup costs more than the split gains
      // k-tiles per chunk at least (tile 48, one workgroup per CU and no co-resident partner: its own floor)
      const int min_kt = std::max(1, t == 48 ? TU.h4_split_minkt : TU.small_split_minkt);
      int S = std::min(((t == 36 || t == 46 ? 2 : 1) * P) / T, nkt / min_kt);  // resident workgroups per CU: 2 / 1
      const size_t tile_f = (size_t)bm * bn;
      while (S > 1 && (size_t)T * S * tile_f > kWsFloats) --S;
      if (S > 1) a.tsplit = S;
    }
  }
  return hipSuccess;
}

hipError_t gemm_nt(const GemmArgs& a_in, hipStream_t s, int tile_hint, float* ws) {
  GemmArgs a = a_in;
  a.nofix = 0;
  a.t49 = 0;
  int t = -1;
  if (hipError_t e = gemm_prepare(a, tile_hint, ws, t)) return e;
  // r06 (h5_split): the plain N = 1152 split-K GEMMs (projection input gradients, Dec_net.proj, ...) on tile 49 split
  // P / T ways as gemm_ln's, their partials summed by k_gemm_fixup49 (tile 48: 72 tiles x 3 = 216 workgroups)
  bool fix49 = false;
  {
    const Tuning& TU = a.tune ? *a.tune : kDefaultTuning;
    const long P = device_cus(), T49 = tiles_of(a, 256, 144);
    if (tile_hint < 0 && TU.h5_split && t == 48 && a.tsplit > 1 && a.tdp == 0 && a.ngroups == 1 && !a.crow &&
        !a.opl && (a.epi == EPI_STORE || a.epi == EPI_RESID) && a.N % 144 == 0 && a.N % 128 == 0 && T49 > 0 &&
        P % T49 == 0 && P / T49 >= 2 && P / T49 <= 4 && (size_t)P * 256 * 144 <= kWsFloats && a.K / 32 >= P / T49) {
      t = 49;
      a.tsplit = (int)(P / T49);
      a.nofix = 1;
      const int ntm = (a.M + 255) / 256, ntn = (a.N + 143) / 144;
      a.gm = std::max(1, std::min(ntm, (int)std::lround(std::sqrt((double)ntm * ntn / 8.0 * 144 / 256))));
      fix49 = true;
    }
  }
  const int ph = prof_begin(s);
  hipError_t e = launch_variant(t, a, s);
  if (e == hipSuccess && fix49) {
    count_launch(CNT_SPLITK_FIXUP);
    const dim3 grid(tiles_of(a, 256, 144), 2, 1);
    if (a.epi == EPI_STORE)
      hipLaunchKernelGGL((k_gemm_fixup49<EPI_STORE>), grid, dim3(512), 0, s, a);
    else
      hipLaunchKernelGGL((k_gemm_fixup49<EPI_RESID>), grid, dim3(512), 0, s, a);
    e = hipGetLastError();
  }
  // algorithmic: 2MNK flops; bytes = A + B + C (+R/aux) once each
  const double G = a.ngroups;
  double bytes = 4.0 * G * ((double)a.M * a.K + (double)a.N * a.K + (double)a.M * a.N);
  if (a.epi == EPI_RESID || a.epi == EPI_GELU || a.epi == EPI_DGELU) bytes += 4.0 * G * (double)a.M * a.N;
  prof_end(ph, s, h3_tile(t) && h3_ready(a) ? PC_GEMM16 : PC_GEMM, 2.0 * G * a.M * a.N * a.K, bytes);
  return e;
}

hipError_t gemm_ln(const GemmArgs& a_in, const GemmLnArgs& l, hipStream_t s, float* ws) {
  GemmArgs a = a_in;
  a.nofix = 0;
  if (a.ngroups != 1 || a.opl || a.N % 4 || a.N > 1280 || !ws || !l.gamma || !l.stats) return hipErrorNotSupported;
  if (!l.bwd && (a.epi != EPI_RESID || !l.beta || !l.pl || !l.rs)) return hipErrorNotSupported;
  if (l.bwd && (a.epi != EPI_STORE || a.g[0].bias || a.crow || !l.x || !l.y || (l.pl && !l.rs)))
    return hipErrorNotSupported;
  int t = -1;
  if (hipError_t e = gemm_prepare(a, -1, ws, t)) return e;
  if (t != 48 || a.tsplit < 2 || a.tsplit > 4 || a.tdp != 0) return hipErrorNotSupported;
  a.nofix = 1;
  a.t49 = 0;
  {
    // r06 (h5_split): tile 49 with every tile split S = P / T ways where that fills the chip exactly (N = 1152 at
    // 2048 rows: 64 tiles x 4 = 256 workgroups; tile 48: 72 x 3 = 216); its partials are staged by the consumer
    // (fixup_stage49), so only where the fused fixup stages (fixup_ln_launch's stg condition)
    const Tuning& TU = a.tune ? *a.tune : kDefaultTuning;
    const long P = device_cus(), T49 = tiles_of(a, 256, 144);
    const bool stg = TU.fixup_stage && (l.bwd || l.ginv || !l.gmap);
    if (TU.h5_split && stg && a.N % 144 == 0 && a.N % 128 == 0 && T49 > 0 && P % T49 == 0 && P / T49 >= 2 &&
        P / T49 <= 4 && (size_t)P * 256 * 144 <= kWsFloats && a.K / 32 >= P / T49) {
      t = 49;
      a.t49 = 1;
      a.tsplit = (int)(P / T49);
      const int ntm = (a.M + 255) / 256, ntn = (a.N + 143) / 144;
      a.gm = std::max(1, std::min(ntm, (int)std::lround(std::sqrt((double)ntm * ntn / 8.0 * 144 / 256))));
    }
  }
  const int ph = prof_begin(s);
  hipError_t e = launch_variant(t, a, s);
  if (e == hipSuccess) e = fixup_ln_launch(a, l, s);
  prof_end(ph, s, PC_GEMM16, 2.0 * a.M * a.N * a.K,
           4.0 * ((double)a.M * a.K + (double)a.N * a.K + 3.0 * (double)a.M * a.N));
  return e;
}

}  // namespace vv

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

namespace vv {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float dgelu_f(float x) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
  const float pdf = 0.39894228040143268f * expf(-0.5f * x * x);
  return cdf + x * pdf;
}

constexpr int BK = 32;
constexpr int LS = BK + 4;  // LDS row stride (floats)

template <int BM, int BN, int WM, int WN, int EPI>
__global__ __launch_bounds__(256) void k_gemm_nt(GemmArgs args) {
  constexpr int TM = BM / WM / 32;
  constexpr int TN = BN / WN / 32;
  constexpr int AI = BM / 32;
  constexpr int BI = BN / 32;
  static_assert(WM * WN == 4, "4 waves");
  extern __shared__ __attribute__((aligned(16))) float smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const GemmGroup G = args.g[blockIdx.z];
  const int M = args.M, N = args.N, K = args.K, ksplit = args.ksplit;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int lr = tid >> 3, lc = (tid & 7) * 4;

  const float* a1p[AI];
  const float* a2p[AI];
  const float* bp[BI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int r = min(m0 + lr + 32 * i, M - 1);
    const int ar = args.arow ? args.arow[r] : r;
    a1p[i] = G.A + (size_t)ar * args.lda + lc;
    a2p[i] = G.A2 ? G.A2 + (size_t)r * args.lda2 + lc - ksplit : a1p[i];
  }
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int n = min(n0 + lr + 32 * i, N - 1);
    bp[i] = G.B + (size_t)n * K + lc;
  }

  f4 ra[AI], rb[BI];
  auto gload = [&](int k0) {
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
  auto sstore = [&](int buf) {
    float* As = smem + buf * (BM + BN) * LS;
    float* Bs = As + BM * LS;
#pragma unroll
    for (int i = 0; i < AI; ++i) *reinterpret_cast<f4*>(As + (lr + 32 * i) * LS + lc) = ra[i];
#pragma unroll
    for (int i = 0; i < BI; ++i) *reinterpret_cast<f4*>(Bs + (lr + 32 * i) * LS + lc) = rb[i];
  };

  const int wm = wave / WN, wn = wave % WN;
  const int rin = lane & 31, hh = lane >> 5;
  f16v acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.0f;

  auto compute = [&](int buf) {
    const float* As = smem + buf * (BM + BN) * LS + (wm * TM * 32 + rin) * LS + hh * 16;
    const float* Bs = smem + buf * (BM + BN) * LS + BM * LS + (wn * TN * 32 + rin) * LS + hh * 16;
#pragma unroll
    for (int kq = 0; kq < 4; ++kq) {
      f4 af[TM], bf[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) af[a] = *reinterpret_cast<const f4*>(As + a * 32 * LS + kq * 4);
#pragma unroll
      for (int b = 0; b < TN; ++b) bf[b] = *reinterpret_cast<const f4*>(Bs + b * 32 * LS + kq * 4);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a][s], bf[b][s], acc[a][b], 0, 0, 0);
    }
  };

  const int nk = K / BK;
  gload(0);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * BK);
    compute(cur);
    if (kt + 1 < nk) sstore(cur ^ 1);
    __syncthreads();
  }

  // epilogue: acc[a][b][r] -> row (r&3) + 8(r>>2) + 4h, col lane&31 of the 32x32 tile
  const float* bias = G.bias;
#pragma unroll
  for (int a = 0; a < TM; ++a) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = m0 + wm * TM * 32 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
      if (row >= M) continue;
      const int o = args.crow ? args.crow[row] : row;
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int col = n0 + wn * TN * 32 + b * 32 + rin;
        if (col >= N) continue;
        float v = acc[a][b][r];
        if (bias) v += bias[col];
        if constexpr (EPI == EPI_GELU) {
          G.aux[(size_t)o * args.ldaux + col] = v;
          v = gelu_f(v);
        } else if constexpr (EPI == EPI_RESID) {
          const int rr = args.rmod > 0 ? o % args.rmod : o;
          v = G.R[(size_t)rr * args.ldr + col] + v;
        } else if constexpr (EPI == EPI_DGELU) {
          v = v * dgelu_f(G.aux[(size_t)o * args.ldaux + col]);
        }
        G.C[(size_t)o * args.ldc + col] = v;
      }
    }
  }
}

template <int BM, int BN, int WM, int WN>
static hipError_t launch_tile(const GemmArgs& a, hipStream_t s) {
  const size_t lds = 2 * (BM + BN) * LS * sizeof(float);
  dim3 grid((a.N + BN - 1) / BN, (a.M + BM - 1) / BM, a.ngroups);
  switch (a.epi) {
#define VV_EPI(E)                                                                                   \
  case E: {                                                                                         \
    static bool init = false;                                                                       \
    if (!init) {                                                                                    \
      hipError_t e = hipFuncSetAttribute((const void*)k_gemm_nt<BM, BN, WM, WN, E>,                 \
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);     \
      if (e != hipSuccess) return e;                                                                \
      init = true;                                                                                  \
    }                                                                                               \
    hipLaunchKernelGGL((k_gemm_nt<BM, BN, WM, WN, E>), grid, dim3(256), lds, s, a);                \
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

static long tiles_of(const GemmArgs& a, int bm, int bn) {
  return (long)((a.M + bm - 1) / bm) * ((a.N + bn - 1) / bn) * a.ngroups;
}

// tile choice: the largest tile that still gives every CU (256 on MI355X) work
static int pick_tile(const GemmArgs& a) {
  if (tiles_of(a, 128, 128) >= 480) return 0;
  if (tiles_of(a, 128, 64) >= 400) return 1;
  return 2;
}

hipError_t gemm_nt(const GemmArgs& a, hipStream_t s, int tile_hint) {
  if (a.M <= 0 || a.N <= 0 || a.ngroups <= 0 || a.ngroups > kMaxGroups) return hipErrorInvalidValue;
  if (a.K % BK != 0 || a.ksplit % BK != 0 || a.ksplit <= 0 || a.ksplit > a.K) return hipErrorInvalidValue;
  if ((a.lda & 3) || (a.lda2 & 3) || (a.K & 3)) return hipErrorInvalidValue;
  const int t = tile_hint >= 0 ? tile_hint : pick_tile(a);
  const int ph = prof_begin(s);
  hipError_t e;
  switch (t) {
    case 0: e = launch_tile<128, 128, 2, 2>(a, s); break;
    case 1: e = launch_tile<128, 64, 2, 2>(a, s); break;
    case 2: e = launch_tile<64, 64, 2, 2>(a, s); break;
    default: return hipErrorInvalidValue;
  }
  // algorithmic: 2MNK flops; bytes = A + B + C (+R/aux) once each
  const double G = a.ngroups;
  double bytes = 4.0 * G * ((double)a.M * a.K + (double)a.N * a.K + (double)a.M * a.N);
  if (a.epi == EPI_RESID || a.epi == EPI_GELU || a.epi == EPI_DGELU) bytes += 4.0 * G * (double)a.M * a.N;
  prof_end(ph, s, PC_GEMM, 2.0 * G * a.M * a.N * a.K, bytes);
  return e;
}

}  // namespace vv

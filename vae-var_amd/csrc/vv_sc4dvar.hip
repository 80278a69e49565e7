// sc4dvar B-matrix transform (da_4dvar.py:878-931) on gfx950: the control variable w (69, 128, 256) is mapped to
// the analysis increment by
//   horizontal   per channel c: isht( sph_scale * sht(w_c) * kernel_c[l, m=0] ) * 11 / len_c^2     (:883-888)
//                (RealSHT / InverseRealSHT of torch_harmonics, grid "equiangular", :614-618; zonal Gaussian
//                correlation kernel of the first hpad latitude rows, :620-628)
//   balance      v = s + reg_coeff . psi  (psi = stream-function levels, :890-897)
//   vertical     surface channels * std_sur, each 13-level block by E_b diag(sqrt(lambda_b))       (:899-906)
//   winds        u = d(sf)/dy - d(vp)/dx, v = -d(sf)/dx - d(vp)/dy on the 128 x 256 grid         (:908-926)
// and its exact adjoint (the gradient of the closure). Layout: fields (C, 128, 256) fp32, one row per (c, lat).
//
// The SHT is linear and separable: a longitude DFT (as an exact-f32 MFMA GEMM with a 256 x 256 real DFT matrix:
// rows 0-127 the cosine / real parts of m = 0..127, rows 128-255 the sine / imaginary parts; the Nyquist order
// m = 128 has no Legendre function below lmax = 128 and drops out), then per order m a 128 x 128 Legendre
// analysis (quadrature weights folded in), the per-(c, l) spectral filter, and the 128 x 128 synthesis — one
// kernel per m that keeps the 16 columns of 8 channels in LDS between the two matrix passes. The five linear
// per-pixel steps (balance, surface scaling, vertical EOFs) are one precomputed 69 x 69 matrix; the finite
// differences are a 3-point stencil. Every table is computed on the host in double (the same recursions as
// torch_harmonics, Clenshaw-Curtis weights in closed form) and stored fp32.
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "vv_kernels.h"

namespace vv {

constexpr int kLat = 128, kLon = 256, kM = 128, kQ = 256;  // latitudes, longitudes, orders kept, spectral rows
constexpr int kCPB = 8;                                    // channels per workgroup of k_sht_filter

struct Sc4dvarB {
  int C = 0, nreg = 0;
  float* arena = nullptr;
  float *WaT, *Wa, *P, *PT;       // [m][k][l] / [m][l][k] Legendre analysis (x quadrature) and synthesis
  float *Df, *DfT, *Di, *DiT;     // [q][j] forward DFT (2 pi / 256 scaled), its transpose, inverse [j][q], transpose
  float* F;                       // [C][l] spectral filter incl. 11 / len^2
  float *A, *AT;                  // [C][C] per-pixel channel map and its transpose
  float* stc;                     // [4][128]: rdx, ylo, ydi, yup
};

namespace {

// stage 1: u[l] = sum_k A1[m][k][l] v[k];  u *= F[c][l];  stage 2: out[k] = sum_l A2[m][l][k] u[l]
// in / out: [q][C*128] (q = m for the real parts, 128 + m for the imaginary parts); one workgroup per (m, 8 channels)
__global__ __launch_bounds__(256) void k_sht_filter(const float* __restrict__ in, float* __restrict__ out,
                                                    const float* __restrict__ A1, const float* __restrict__ A2,
                                                    const float* __restrict__ F, int C) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) float v[2][kCPB][kLat];
  __shared__ __attribute__((aligned(16))) float u[2][kCPB][kLat];
  const int m = blockIdx.x, c0 = blockIdx.y * kCPB, tid = threadIdx.x;
  const int nc = min(kCPB, C - c0);
  const size_t NR = (size_t)C * kLat;
  const int i = tid & 127, ri = tid >> 7;  // i: l (stage 1) / k (stage 2); ri: real / imaginary column
  const float* src = in + (size_t)(ri * kM + m) * NR + (size_t)c0 * kLat;
  for (int ch = 0; ch < kCPB; ++ch) v[ri][ch][i] = ch < nc ? src[(size_t)ch * kLat + i] : 0.f;
  __syncthreads();
  // k / l run in steps of 4: four independent matrix loads, float4 reads of the LDS columns (broadcast)
  const int m4 = m & ~3;
  {
    float acc[kCPB];
#pragma unroll
    for (int ch = 0; ch < kCPB; ++ch) acc[ch] = 0.f;
    const float* a = A1 + (size_t)m * kLat * kLat + i;  // A1[m][k][l = i]
    if (i >= m) {
      for (int k = 0; k < kLat; k += 4) {
        const float w0 = a[(size_t)k * kLat], w1 = a[(size_t)(k + 1) * kLat], w2 = a[(size_t)(k + 2) * kLat],
                    w3 = a[(size_t)(k + 3) * kLat];
#pragma unroll
        for (int ch = 0; ch < kCPB; ++ch) {
          const f4 x = *reinterpret_cast<const f4*>(&v[ri][ch][k]);
          acc[ch] = fmaf(w3, x[3], fmaf(w2, x[2], fmaf(w1, x[1], fmaf(w0, x[0], acc[ch]))));
        }
      }
    }
#pragma unroll
    for (int ch = 0; ch < kCPB; ++ch) u[ri][ch][i] = ch < nc ? acc[ch] * F[(size_t)(c0 + ch) * kLat + i] : 0.f;
  }
  __syncthreads();
  float acc[kCPB];
#pragma unroll
  for (int ch = 0; ch < kCPB; ++ch) acc[ch] = 0.f;
  const float* a = A2 + (size_t)m * kLat * kLat + i;  // A2[m][l][k = i]; rows l < m are zero
  for (int l = m4; l < kLat; l += 4) {
    const float w0 = a[(size_t)l * kLat], w1 = a[(size_t)(l + 1) * kLat], w2 = a[(size_t)(l + 2) * kLat],
                w3 = a[(size_t)(l + 3) * kLat];
#pragma unroll
    for (int ch = 0; ch < kCPB; ++ch) {
      const f4 x = *reinterpret_cast<const f4*>(&u[ri][ch][l]);
      acc[ch] = fmaf(w3, x[3], fmaf(w2, x[2], fmaf(w1, x[1], fmaf(w0, x[0], acc[ch]))));
    }
  }
  float* dst = out + (size_t)(ri * kM + m) * NR + (size_t)c0 * kLat;
  for (int ch = 0; ch < nc; ++ch) dst[(size_t)ch * kLat + i] = acc[ch];
}

// out[i][p] = sum_j A[i][j] in[j][p] over the C channels of one pixel p. 256 threads = 64 pixels x 4 output
// groups; each thread keeps its pixel's column in registers and forms every fourth output from float4 broadcasts of
// A's rows (zero-padded to kMaxC in LDS), four independent partial sums per output
constexpr int kMaxC = 72;
__global__ __launch_bounds__(256) void k_colmix(const float* __restrict__ in, float* __restrict__ out,
                                                const float* __restrict__ A, int C, int HW) {
  __shared__ __attribute__((aligned(16))) float As[kMaxC * kMaxC];
  for (int e = threadIdx.x; e < kMaxC * kMaxC; e += blockDim.x) {
    const int i = e / kMaxC, j = e % kMaxC;
    As[e] = (i < C && j < C) ? A[i * C + j] : 0.f;
  }
  __syncthreads();
  const int p = blockIdx.x * 64 + (threadIdx.x & 63), og = threadIdx.x >> 6;
  if (p >= HW) return;
  float x[kMaxC];
#pragma unroll
  for (int j = 0; j < kMaxC; ++j) x[j] = j < C ? in[(size_t)j * HW + p] : 0.f;
  typedef float f4 __attribute__((ext_vector_type(4)));
  for (int i = og; i < C; i += 4) {
    const f4* a = reinterpret_cast<const f4*>(As + i * kMaxC);
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll
    for (int q = 0; q < kMaxC / 4; ++q) {
      const f4 v = a[q];
      s0 = fmaf(v[0], x[4 * q], s0);
      s1 = fmaf(v[1], x[4 * q + 1], s1);
      s2 = fmaf(v[2], x[4 * q + 2], s2);
      s3 = fmaf(v[3], x[4 * q + 3], s3);
    }
    out[(size_t)i * HW + p] = (s0 + s1) + (s2 + s3);
  }
}

// winds from stream function sf = f[su + r] and velocity potential vp = f[sv + r] (:908-926); every other channel
// is copied. Gx f = (f[j-1] - f[j+1]) * rdx[k] (periodic in longitude), Gy f = ylo f[k-1] + ydi f[k] + yup f[k+1]
__device__ __forceinline__ float gx(const float* f, int k, int j, const float* rdx) {
  return (f[k * kLon + ((j + kLon - 1) & (kLon - 1))] - f[k * kLon + ((j + 1) & (kLon - 1))]) * rdx[k];
}
__device__ __forceinline__ float gy(const float* f, int k, int j, const float* lo, const float* di, const float* up) {
  float s = di[k] * f[k * kLon + j];
  if (k > 0) s = fmaf(lo[k], f[(k - 1) * kLon + j], s);
  if (k < kLat - 1) s = fmaf(up[k], f[(k + 1) * kLon + j], s);
  return s;
}
// adjoints: (Gx^T g)[k][j] = rdx[k] (g[j+1] - g[j-1]); (Gy^T g)[k] = lo[k+1] g[k+1] + di[k] g[k] + up[k-1] g[k-1]
__device__ __forceinline__ float gxt(const float* g, int k, int j, const float* rdx) {
  return (g[k * kLon + ((j + 1) & (kLon - 1))] - g[k * kLon + ((j + kLon - 1) & (kLon - 1))]) * rdx[k];
}
__device__ __forceinline__ float gyt(const float* g, int k, int j, const float* lo, const float* di, const float* up) {
  float s = di[k] * g[k * kLon + j];
  if (k < kLat - 1) s = fmaf(lo[k + 1], g[(k + 1) * kLon + j], s);
  if (k > 0) s = fmaf(up[k - 1], g[(k - 1) * kLon + j], s);
  return s;
}

__global__ __launch_bounds__(256) void k_winds(const float* __restrict__ f, float* __restrict__ out,
                                               const float* __restrict__ stc, int C, int su, int sv, int nl,
                                               int adjoint) {
  const size_t HW = (size_t)kLat * kLon;
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (size_t)C * HW) return;
  const int c = (int)(e / HW), p = (int)(e % HW), k = p / kLon, j = p % kLon;
  const float *rdx = stc, *lo = stc + kLat, *di = stc + 2 * kLat, *up = stc + 3 * kLat;
  float r;
  if (c >= su && c < su + nl) {
    const float* a = f + (size_t)c * HW;              // sf (forward) / g_u (adjoint)
    const float* b = f + (size_t)(c - su + sv) * HW;  // vp (forward) / g_v (adjoint)
    // forward u = Gy sf - Gx vp ; adjoint g_sf = Gy^T g_u - Gx^T g_v
    r = adjoint ? gyt(a, k, j, lo, di, up) - gxt(b, k, j, rdx) : gy(a, k, j, lo, di, up) - gx(b, k, j, rdx);
  } else if (c >= sv && c < sv + nl) {
    const float* a = f + (size_t)(c - sv + su) * HW;  // sf / g_u
    const float* b = f + (size_t)c * HW;              // vp / g_v
    // forward v = -Gx sf - Gy vp ; adjoint g_vp = -Gx^T g_u - Gy^T g_v
    r = adjoint ? -gxt(a, k, j, rdx) - gyt(b, k, j, lo, di, up) : -gx(a, k, j, rdx) - gy(b, k, j, lo, di, up);
  } else {
    r = f[e];
  }
  out[e] = r;
}

// C = A . B^T on the exact-f32 MFMA (+ R: residual epilogue)
hipError_t gemm_f32(const float* A, const float* B, float* C, const float* R, int M, int N, int K, float* ws,
                    hipStream_t s) {
  GemmArgs a;
  memset(&a, 0, sizeof(a));
  a.math = GEMM_F32;
  a.M = M;
  a.N = N;
  a.K = K;
  a.ksplit = K;
  a.lda = K;
  a.ldc = N;
  a.ldr = N;
  a.ldaux = N;
  a.epi = R ? EPI_RESID : EPI_STORE;
  a.ngroups = 1;
  a.g[0].A = A;
  a.g[0].B = B;
  a.g[0].C = C;
  a.g[0].R = R;
  return gemm_nt(a, s, -1, ws);
}

// Clenshaw-Curtis weights on theta_k = pi k / (n - 1) (closed form; torch_harmonics clenshaw_curtiss_weights)
std::vector<double> cc_weights(int n) {
  const int N = n - 1;
  std::vector<double> w(n);
  for (int k = 0; k < n; ++k) {
    const double th = M_PI * k / N;
    double s = 0.0;
    for (int j = 1; j <= N / 2; ++j) s += (2 * j == N ? 1.0 : 2.0) / (4.0 * j * j - 1.0) * std::cos(2.0 * j * th);
    w[k] = (k == 0 || k == N ? 1.0 : 2.0) / N * (1.0 - s);
  }
  return w;
}

// orthonormal associated Legendre functions with the Condon-Shortley phase, P[m][l][k] (m, l < 128) at x_k
// (torch_harmonics legendre.legpoly, norm "ortho")
std::vector<double> legpoly(const std::vector<double>& x) {
  const int n = kLat, K = (int)x.size();
  std::vector<double> v((size_t)n * n * K, 0.0);
  auto V = [&](int m, int l) { return &v[((size_t)m * n + l) * K]; };
  for (int k = 0; k < K; ++k) V(0, 0)[k] = 1.0 / std::sqrt(4 * M_PI);
  for (int l = 1; l < n; ++l)
    for (int k = 0; k < K; ++k) {
      V(l - 1, l)[k] = std::sqrt(2.0 * l + 1) * x[k] * V(l - 1, l - 1)[k];
      V(l, l)[k] = std::sqrt((2.0 * l + 1) * (1 + x[k]) * (1 - x[k]) / 2 / l) * V(l - 1, l - 1)[k];
    }
  for (int l = 2; l < n; ++l)
    for (int m = 0; m < l - 1; ++m) {
      const double a = std::sqrt((2.0 * l - 1) / (l - m) * (2.0 * l + 1) / (l + m));
      const double b = std::sqrt((l + m - 1.0) / (l - m) * (2.0 * l + 1) / (2.0 * l - 3) * (l - m - 1.0) / (l + m));
      for (int k = 0; k < K; ++k) V(m, l)[k] = x[k] * a * V(m, l - 1)[k] - b * V(m, l - 2)[k];
    }
  for (int m = 1; m < n; m += 2)
    for (int l = 0; l < n; ++l)
      for (int k = 0; k < K; ++k) V(m, l)[k] = -V(m, l)[k];
  return v;
}

}  // namespace

int sc4dvar_create(Sc4dvarB** out, int C, const double* len_scale, const double* reg, int nreg,
                   const double* std_sur, const double* eigval, const double* eigvec, double scale_factor, int hpad,
                   std::string& err) {
  const int nl = 13;
  if (C != 4 + 5 * nl) {
    err = "sc4dvar needs the 69-channel ERA5 layout (4 surface + 5 x 13 levels)";
    return -1;
  }
  if (nreg != nl && nreg != 2 * nl) {
    err = "reg_coeff must be (69, 13) or (69, 26)";
    return -1;
  }
  if (hpad < 0 || hpad > kLat) {
    err = "hpad must be in [0, 128]";
    return -1;
  }
  for (int c = 0; c < C; ++c)
    if (!(len_scale[c] * scale_factor > 0)) {
      err = "len_scale * scale_factor must be positive";
      return -1;
    }
  auto* b = new Sc4dvarB();
  b->C = C;
  b->nreg = nreg;
  const size_t L3 = (size_t)kLat * kLat * kLat, Q2 = (size_t)kQ * kLon;
  const size_t total = 4 * L3 + 4 * Q2 + (size_t)C * kLat + 2 * (size_t)C * C + 4 * kLat;
  if (hipMalloc(&b->arena, total * sizeof(float)) != hipSuccess) {
    delete b;
    err = "sc4dvar tables: out of device memory";
    return -2;
  }
  float* p = b->arena;
  b->WaT = p; p += L3;
  b->Wa = p; p += L3;
  b->P = p; p += L3;
  b->PT = p; p += L3;
  b->Df = p; p += Q2;
  b->DfT = p; p += Q2;
  b->Di = p; p += Q2;
  b->DiT = p; p += Q2;
  b->F = p; p += (size_t)C * kLat;
  b->A = p; p += (size_t)C * C;
  b->AT = p; p += (size_t)C * C;
  b->stc = p;

  std::vector<float> h(total);
  float* hp = h.data();
  // Legendre tables at x_k = cos(pi k / 127), quadrature weights folded into the analysis
  const std::vector<double> w = cc_weights(kLat);
  std::vector<double> x(kLat);
  for (int k = 0; k < kLat; ++k) x[k] = std::cos(M_PI * k / (kLat - 1));
  const std::vector<double> Pd = legpoly(x);
  auto Pv = [&](int m, int l, int k) { return Pd[((size_t)m * kLat + l) * kLat + k]; };
  for (int m = 0; m < kM; ++m)
    for (int l = 0; l < kLat; ++l)
      for (int k = 0; k < kLat; ++k) {
        const double pv = Pv(m, l, k), wa = pv * w[k];
        const size_t mlk = ((size_t)m * kLat + l) * kLat + k, mkl = ((size_t)m * kLat + k) * kLat + l;
        hp[mkl] = (float)wa;               // WaT
        hp[L3 + mlk] = (float)wa;          // Wa
        hp[2 * L3 + mlk] = (float)pv;      // P
        hp[3 * L3 + mkl] = (float)pv;      // PT
      }
  // DFTs: X = 2 pi rfft(x, norm="forward") (rows q: Re m, then Im m), x = irfft(X, n=256, norm="forward")
  float* df = hp + 4 * L3;
  for (int q = 0; q < kQ; ++q)
    for (int j = 0; j < kLon; ++j) {
      const int m = q % kM;
      const double ang = 2.0 * M_PI * m * j / kLon, cm = m == 0 ? 1.0 : 2.0;
      const double f = q < kM ? 2.0 * M_PI / kLon * std::cos(ang) : -2.0 * M_PI / kLon * std::sin(ang);
      const double i = q < kM ? cm * std::cos(ang) : -cm * std::sin(ang);
      df[(size_t)q * kLon + j] = (float)f;           // Df[q][j]
      df[Q2 + (size_t)j * kQ + q] = (float)f;        // DfT[j][q]
      df[2 * Q2 + (size_t)j * kQ + q] = (float)i;    // Di[j][q]
      df[3 * Q2 + (size_t)q * kLon + j] = (float)i;  // DiT[q][j]
    }
  // filter: sph_scale[l] * (m = 0 coefficient of the zonal kernel) * 11 / len^2 (:620-628, :885-888)
  float* F = hp + 4 * L3 + 4 * Q2;
  for (int c = 0; c < C; ++c) {
    const double Lc = len_scale[c] * scale_factor;
    for (int l = 0; l < kLat; ++l) {
      double a = 0.0;  // sum_k (2 pi * kernel row k) * w_k P[0][l][k]
      for (int k = 0; k < hpad; ++k) a += 2.0 * M_PI * std::exp(-(double)k * k / (8.0 * Lc * Lc)) * w[k] * Pv(0, l, k);
      const double sph = 2.0 * M_PI * std::sqrt(4.0 * M_PI / (2.0 * l + 1));
      F[(size_t)c * kLat + l] = (float)(sph * a * 11.0 / (Lc * Lc));
    }
  }
  // per-pixel map A = D (I + Reg): Reg[i][psi_j] = reg[i][j] (:890-897); D = diag(std_sur) (+) E_b diag(sqrt l_b)
  std::vector<double> Reg((size_t)C * C, 0.0), D((size_t)C * C, 0.0);
  for (int i = 0; i < C; ++i) {
    Reg[(size_t)i * C + i] = 1.0;
    for (int j = 0; j < nreg; ++j) {
      const int src = nreg == nl ? 4 + 2 * nl + j : (j < nl ? 4 + j : 4 + 2 * nl + (j - nl));
      Reg[(size_t)i * C + src] += reg[(size_t)i * nreg + j];
    }
  }
  for (int i = 0; i < 4; ++i) D[(size_t)i * C + i] = std_sur[i];
  for (int bl = 0; bl < 5; ++bl)
    for (int r = 0; r < nl; ++r)
      for (int q = 0; q < nl; ++q)
        D[(size_t)(4 + bl * nl + r) * C + 4 + bl * nl + q] =
            eigvec[((size_t)bl * nl + r) * nl + q] * std::sqrt(eigval[(size_t)bl * nl + q]);
  float* A = F + (size_t)C * kLat;
  for (int i = 0; i < C; ++i)
    for (int j = 0; j < C; ++j) {
      double s = 0.0;
      for (int q = 0; q < C; ++q) s += D[(size_t)i * C + q] * Reg[(size_t)q * C + j];
      A[(size_t)i * C + j] = (float)s;
      A[(size_t)C * C + (size_t)j * C + i] = (float)s;  // AT
    }
  // stencils (:908-916): partial_x = (f[j-1] - f[j+1]) / (2 * 111195 * 180 / 128 * sin(lat')), lat' the fp32
  // torch.linspace(pi/180, 179 pi/180, 128); partial_y = torch.gradient on the fp32 coordinates
  // k * 111195 * 180 / 127 (edge_order 1: one-sided first differences at the poles)
  float* st = A + 2 * (size_t)C * C;
  std::vector<double> cy(kLat);
  for (int k = 0; k < kLat; ++k) {
    const float a0 = (float)(M_PI / 180.0), a1 = (float)(179.0 * M_PI / 180.0);
    const float step = (a1 - a0) / (float)(kLat - 1);
    const float lat = k < kLat / 2 ? a0 + step * (float)k : a1 - step * (float)(kLat - 1 - k);  // torch.linspace
    st[k] = (float)(1.0 / (2.0 * 111195.0 * 180.0 / kLat * (double)sinf(lat)));
    cy[k] = (double)(float)((float)((long long)k * 111195 * 180) / (float)(kLat - 1));
  }
  float *lo = st + kLat, *di = st + 2 * kLat, *up = st + 3 * kLat;
  for (int k = 0; k < kLat; ++k) {
    if (k == 0) {
      const double h0 = cy[1] - cy[0];
      lo[k] = 0.f, di[k] = (float)(-1.0 / h0), up[k] = (float)(1.0 / h0);
    } else if (k == kLat - 1) {
      const double h1 = cy[k] - cy[k - 1];
      lo[k] = (float)(-1.0 / h1), di[k] = (float)(1.0 / h1), up[k] = 0.f;
    } else {
      const double d1 = cy[k] - cy[k - 1], d2 = cy[k + 1] - cy[k];
      lo[k] = (float)(-d2 / (d1 * (d1 + d2)));
      di[k] = (float)((d2 - d1) / (d1 * d2));
      up[k] = (float)(d1 / (d2 * (d1 + d2)));
    }
  }
  if (hipMemcpy(b->arena, h.data(), total * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(b->arena);
    delete b;
    err = "sc4dvar tables: copy failed";
    return -2;
  }
  *out = b;
  return 0;
}

void sc4dvar_destroy(Sc4dvarB* b) {
  if (!b) return;
  (void)hipFree(b->arena);
  delete b;
}

size_t sc4dvar_field_floats(const Sc4dvarB* b) { return (size_t)b->C * kLat * kLon; }

// recon = transform core of w (da_4dvar.py:883-926, before the interpolation and + xb); t1, t2: field-sized scratch
hipError_t sc4dvar_fwd(const Sc4dvarB* b, const float* w, float* recon, float* t1, float* t2, float* gemm_ws,
                       hipStream_t s) {
  const int C = b->C, NR = C * kLat, HW = kLat * kLon;
  hipError_t e;
  // t1 = X^T [q][(c,k)] = Df . w_rows^T
  if ((e = gemm_f32(b->Df, w, t1, nullptr, kQ, NR, kLon, gemm_ws, s))) return e;
  hipLaunchKernelGGL(k_sht_filter, dim3(kM, (C + kCPB - 1) / kCPB), dim3(256), 0, s, t1, t2, b->WaT, b->P, b->F, C);
  if ((e = transpose2d(t2, t1, kQ, NR, s))) return e;           // t1 = Y [(c,k)][q]
  if ((e = gemm_f32(t1, b->Di, t2, nullptr, NR, kLon, kQ, gemm_ws, s))) return e;  // t2 = inc_static
  hipLaunchKernelGGL(k_colmix, dim3((HW + 63) / 64), dim3(256), 0, s, t2, t1, b->A, C, HW);  // t1 = sfvp
  const size_t n = (size_t)C * HW;
  hipLaunchKernelGGL(k_winds, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, t1, recon, b->stc, C, 4 + 2 * 13,
                     4 + 3 * 13, 13, 0);
  return hipGetLastError();
}

// g_w = (transform core)^T g_recon + add (add may be null); g_recon is preserved; t1, t2: field-sized scratch
hipError_t sc4dvar_adj(const Sc4dvarB* b, const float* g_recon, const float* add, float* g_w, float* t1, float* t2,
                       float* gemm_ws, hipStream_t s) {
  const int C = b->C, NR = C * kLat, HW = kLat * kLon;
  const size_t n = (size_t)C * HW;
  hipError_t e;
  hipLaunchKernelGGL(k_winds, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, g_recon, t1, b->stc, C,
                     4 + 2 * 13, 4 + 3 * 13, 13, 1);                                  // t1 = g_sfvp
  hipLaunchKernelGGL(k_colmix, dim3((HW + 63) / 64), dim3(256), 0, s, t1, t2, b->AT, C, HW);  // t2 = g_static
  if ((e = gemm_f32(b->DiT, t2, t1, nullptr, kQ, NR, kLon, gemm_ws, s))) return e;  // t1 = g_Y^T [q][(c,k)]
  hipLaunchKernelGGL(k_sht_filter, dim3(kM, (C + kCPB - 1) / kCPB), dim3(256), 0, s, t1, t2, b->PT, b->Wa, b->F, C);
  if ((e = transpose2d(t2, t1, kQ, NR, s))) return e;                                  // t1 = g_X [(c,k)][q]
  if ((e = gemm_f32(t1, b->DfT, g_w, add, NR, kLon, kQ, gemm_ws, s))) return e;     // g_w = g_X . Df (+ add)
  return hipGetLastError();
}

}  // namespace vv

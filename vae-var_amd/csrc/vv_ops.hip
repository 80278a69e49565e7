// Non-GEMM kernels of the Swin-U-Net engine and the DA inner loop (fp32, gfx950).
//   LayerNorm fwd/bwd with the window / PatchMerging / PatchExpand gathers folded into addressing
//   window attention fwd/bwd (16-token windows, relative-position bias, quirk-Q1 shift mask)
//   PatchEmbed conv + absolute_pos_embed, ConvTranspose2d with the quirk-Q2 channel reorder
//   misfit J_o and its adjoint, vector primitives of L-BFGS / Adam
#include "vv_kernels.h"
#include "vv_lanes.h"
#include "vv_gelu.h"

#include <algorithm>
#include <atomic>
#include <vector>

namespace vv {

// ============================================================================
// live profiler
// ============================================================================
namespace {
struct ProfRec {
  int cls;
  double flops, bytes;
};
bool g_prof_on = false;
std::vector<hipEvent_t> g_ev;  // pairs
std::vector<ProfRec> g_rec;
size_t g_used = 0;
}  // namespace

bool prof_enabled() { return g_prof_on; }
void prof_enable(bool on) {
  g_prof_on = on;
  g_used = 0;
  g_rec.clear();
}
static std::atomic<long long> g_counters[CNT_N];
void count_launch(int c) { g_counters[c].fetch_add(1, std::memory_order_relaxed); }
long long launch_count(int c) { return g_counters[c].load(std::memory_order_relaxed); }

int prof_begin(hipStream_t s) {
  if (!g_prof_on) return -1;
  if (2 * g_used + 2 > g_ev.size()) {
    for (int i = 0; i < 512; ++i) {
      hipEvent_t e;
      if (hipEventCreate(&e) != hipSuccess) return -1;
      g_ev.push_back(e);
    }
  }
  const int h = (int)g_used++;
  (void)hipEventRecord(g_ev[2 * h], s);
  return h;
}
void prof_end(int h, hipStream_t s, int cls, double flops, double bytes) {
  if (h < 0) return;
  (void)hipEventRecord(g_ev[2 * h + 1], s);
  if ((int)g_rec.size() <= h) g_rec.resize(h + 1);
  g_rec[h] = {cls, flops, bytes};
}
void prof_read(double* ms, double* flops, double* bytes, int* n) {
  for (int c = 0; c < PC_N; ++c) ms[c] = flops[c] = bytes[c] = 0, n[c] = 0;
  if (g_used) (void)hipEventSynchronize(g_ev[2 * (g_used - 1) + 1]);
  for (size_t h = 0; h < g_used && h < g_rec.size(); ++h) {
    float t = 0.f;
    (void)hipEventElapsedTime(&t, g_ev[2 * h], g_ev[2 * h + 1]);
    const int c = g_rec[h].cls;
    ms[c] += t;
    flops[c] += g_rec[h].flops;
    bytes[c] += g_rec[h].bytes;
    n[c] += 1;
  }
}

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float wave_sum(float v) { return lane_sum<64>(v); }
__device__ __forceinline__ double wave_sum_d(double v) { return lane_sum<64>(v); }

// ============================================================================
// LayerNorm  (nn.LayerNorm: biased variance, y = (x-mean)/sqrt(var+eps)*g + b)
// ============================================================================
// One row per L-lane sub-wave, the row held in registers as float4 (NV <= 8 per lane): one HBM read of x,
// one write of y. Gathers (window / merge / expand) keep float4 granularity (segment widths are multiples of 4).
constexpr int LN_NVMAX = 8;

// (r05: vv_lanes.h's lane permutes, the same exchange order as the __shfl_xor loops they replace)
template <int L>
__device__ __forceinline__ float sub_sum(float v) { return lane_sum<L>(v); }
template <int L>
__device__ __forceinline__ unsigned sub_max(unsigned v) { return lane_max<L>(v); }
// the fp16x3 GEMM row scale of a row whose largest |value| has bit pattern mx (k_rowscale's formula, bit-identical)
__device__ __forceinline__ float row_scale_of(unsigned mx) { return __uint_as_float((268u - max(mx >> 23, 15u)) << 23); }
__device__ __forceinline__ unsigned absmax4(unsigned m, const f4& o) {
  return max(max(m, max(__float_as_uint(fabsf(o[0])), __float_as_uint(fabsf(o[1])))),
             max(__float_as_uint(fabsf(o[2])), __float_as_uint(fabsf(o[3]))));
}

// the row (this lane's float4s ov[v] = elements 4 (sl + v L) ..) scaled by sc and split into fp16 planes at p,
// chunk-interleaved per 32 elements ([h(32) | l(32)] ...): h = fp16(x sc), l = fp16(x sc - h) -- k_rowsplit's arithmetic, bit for bit
template <int L, int NV>
__device__ __forceinline__ void store_planes(unsigned short* p, int C, int sl, const bool (&ok)[NV], const f4 (&ov)[NV],
                                             float sc) {
  typedef _Float16 h4t __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    if (!ok[v]) continue;
    const int k = 4 * (sl + v * L);
    h4t hv, lv;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float x = ov[v][e] * sc;
      hv[e] = (_Float16)x;
      lv[e] = (_Float16)(x - (float)hv[e]);
    }
    *reinterpret_cast<h4t*>(p + 2 * (k & ~31) + (k & 31)) = hv;  // chunk-interleaved (k_rowsplit's layout)
    *reinterpret_cast<h4t*>(p + 2 * (k & ~31) + 32 + (k & 31)) = lv;
  }
}

// element offsets (relative to the input base, row stride ld) of this lane's float4s of output row r; float4
// indices past the row end are clamped to its last float4 (always a valid address)
template <int L, int NV>
__device__ __forceinline__ void ln_offsets(const LnArgs& a, int r, int sl, int ld, size_t (&eo)[NV]) {
  const int C = a.C, f4n = C >> 2;
  if (a.mode == LN_ROWMAP) {
    const size_t base = (size_t)(a.map ? a.map[r] : r) * ld;
#pragma unroll
    for (int v = 0; v < NV; ++v) eo[v] = base + 4 * min(sl + v * L, f4n - 1);
  } else if (a.mode == LN_MERGE) {
    const int Hh = a.Hin >> 1, Wh = a.Win >> 1;
    const int b = r / (Hh * Wh);
    const int rem = r - b * Hh * Wh;
    const int h = rem / Wh, w = rem - h * Wh;
    const int Cs = C >> 2;
    size_t tb[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      tb[q] = (size_t)((b * a.Hin + 2 * h + (q & 1)) * a.Win + 2 * w + (q >> 1)) * ld;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int c = 4 * min(sl + v * L, f4n - 1);
      const int q = min(c / Cs, 3);
      eo[v] = tb[q] + (c - q * Cs);
    }
  } else {
    const int Wo = a.Win * 2, Ho = a.Hin * 2;
    const int b = r / (Ho * Wo);
    const int rem = r - b * Ho * Wo;
    const int y = rem / Wo, x = rem - y * Wo;
    const size_t base = (size_t)((b * a.Hin + (y >> 1)) * a.Win + (x >> 1)) * ld + ((y & 1) * 2 + (x & 1)) * C;
#pragma unroll
    for (int v = 0; v < NV; ++v) eo[v] = base + 4 * min(sl + v * L, f4n - 1);
  }
}

// Every global load of a row (x, gamma, beta; dy, res) is issued up front and unconditionally (lanes past the
// row end re-read its last float4 and contribute 0): one memory round trip per row instead of one per pass, and
// no loads under branches (which make the compiler wait for all outstanding memory operations).
template <int L, int NV>
__global__ __launch_bounds__(256) void k_ln_fwd(LnArgs a) {
  constexpr int RPB = 256 / L;
  const int sl = threadIdx.x % L;
  const int r = blockIdx.x * RPB + threadIdx.x / L;
  if (r >= a.rows) return;
  const LnGroup G = a.g[blockIdx.y];
  const int C = a.C, f4n = C >> 2;
  size_t eo[NV];
  ln_offsets<L, NV>(a, r, sl, a.ldx, eo);
  f4 xv[NV], gv[NV], bv[NV];
  bool ok[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int j = sl + v * L;
    ok[v] = j < f4n;
    const int jj = ok[v] ? j : f4n - 1;
    xv[v] = *reinterpret_cast<const f4*>(G.x + eo[v]);
    gv[v] = *reinterpret_cast<const f4*>(G.gamma + 4 * jj);
    bv[v] = *reinterpret_cast<const f4*>(G.beta + 4 * jj);
  }
  // masked operands, not masked sums: the accumulations keep the exact form (and FMA contraction) of the
  // per-element branches they replace, so the results are bit-identical
  float s = 0.f;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const f4 x = ok[v] ? xv[v] : f4{0.f, 0.f, 0.f, 0.f};
    s += (x[0] + x[1]) + (x[2] + x[3]);
  }
  const float mean = sub_sum<L>(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = ok[v] ? xv[v][e] - mean : 0.f;
      q += d * d;
    }
  }
  const float rstd = 1.0f / sqrtf(sub_sum<L>(q) / (float)C + a.eps);
  float* y = G.y ? G.y + (size_t)r * a.ldy : nullptr;
  unsigned mx = 0;
  f4 ov[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int j = sl + v * L;
#pragma unroll
    for (int e = 0; e < 4; ++e) ov[v][e] = (xv[v][e] - mean) * rstd * gv[v][e] + bv[v][e];
    if (ok[v]) {
      if (y) *reinterpret_cast<f4*>(y + 4 * j) = ov[v];
      mx = absmax4(mx, ov[v]);
    }
  }
  if (G.rs) {
    mx = sub_max<L>(mx);
    const float sc = row_scale_of(mx);
    if (sl == 0) G.rs[r] = sc;
    if (G.pl) store_planes<L, NV>(G.pl + (size_t)r * 2 * C, C, sl, ok, ov, sc);
  }
  if (sl == 0 && G.stats) {
    G.stats[2 * r] = mean;
    G.stats[2 * r + 1] = rstd;
  }
}

// dx = rstd * (g*dy - mean(g*dy) - xhat * mean(g*dy*xhat)), written back at the input position (+ res);
// x, dx and res share the input layout (ldx == ldy == ldres, checked on the host). The row (x, dy, gamma, res)
// stays in registers between the two reductions and the write.
template <int L, int NV>
__global__ __launch_bounds__(256) void k_ln_bwd(LnArgs a) {
  constexpr int RPB = 256 / L;
  const int sl = threadIdx.x % L;
  const int r = blockIdx.x * RPB + threadIdx.x / L;
  if (r >= a.rows) return;
  const LnGroup G = a.g[blockIdx.y];
  const int C = a.C, f4n = C >> 2;
  size_t eo[NV];
  ln_offsets<L, NV>(a, r, sl, a.ldx, eo);
  const float mean = G.stats[2 * r], rstd = G.stats[2 * r + 1];
  const float* dy = G.dy + (size_t)r * a.lddy;
  const float* res = G.res ? G.res : G.x;  // dummy source when there is no residual (never added)
  f4 xv[NV], dv[NV], gv[NV], rv[NV];
  bool ok[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int j = sl + v * L;
    ok[v] = j < f4n;
    const int jj = ok[v] ? j : f4n - 1;
    xv[v] = *reinterpret_cast<const f4*>(G.x + eo[v]);
    dv[v] = *reinterpret_cast<const f4*>(dy + 4 * jj);
    gv[v] = *reinterpret_cast<const f4*>(G.gamma + 4 * jj);
    rv[v] = *reinterpret_cast<const f4*>(res + eo[v]);
  }
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const f4 d = ok[v] ? dv[v] : f4{0.f, 0.f, 0.f, 0.f};  // masked operand (see k_ln_fwd): gd = 0 adds nothing
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float gd = gv[v][e] * d[e];
      s1 += gd;
      s2 += gd * ((xv[v][e] - mean) * rstd);
    }
  }
  const float m1 = sub_sum<L>(s1) / (float)C;
  const float m2 = sub_sum<L>(s2) / (float)C;
  unsigned mx = 0;
  f4 ov[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
#pragma unroll
    for (int e = 0; e < 4; ++e) ov[v][e] = rstd * (gv[v][e] * dv[v][e] - m1 - ((xv[v][e] - mean) * rstd) * m2);
    if (G.res) {
#pragma unroll
      for (int e = 0; e < 4; ++e) ov[v][e] += rv[v][e];
    }
    if (ok[v]) {
      *reinterpret_cast<f4*>(G.y + eo[v]) = ov[v];
      mx = absmax4(mx, ov[v]);
    }
  }
  if (G.rs) {  // LN_ROWMAP: the row written is map[r]
    mx = sub_max<L>(mx);
    const float sc = row_scale_of(mx);
    const int pr = a.map ? a.map[r] : r;
    if (sl == 0) G.rs[pr] = sc;
    if (G.pl) store_planes<L, NV>(G.pl + (size_t)pr * 2 * C, C, sl, ok, ov, sc);
  }
}

// gemm_ln's LayerNorm half: the fixup of a tile-48 split-K RESID GEMM (k_gemm_h4 with every tile split, partials
// in ws as written by its part >= 0 path: tile tl, chunk c at ((tl S + c) 16 4 512 + ((a 4 + b) 4 + r) 512 + tid),
// the thread / register of the 256 x 128 tile's 8 waves of 64 x 64 on 16x16 fragments) fused into k_ln_fwd<64, NV>:
// one wave per LayerNorm row j. x = R + ((p0 + p1 + ...) + bias) is exactly k_gemm_fixup_sub16's arithmetic, the
// LayerNorm exactly k_ln_fwd's, so the results are bit-identical to the two launches they replace.
// 8 rows (waves) per workgroup: GEMM rows 8i .. 8i + 7 are fragment rows r = 0..3 of two lane quarters, so each
// 128-B line of a partial (rows r and r + 4 of one 16-column block) is consumed inside one workgroup
constexpr int kFixupLnMaxN = 1280;  // gemm_ln's N limit
// the chunk-order sums of the S-chunk partials of the 8 GEMM rows gr0 .. gr0 + 7 (gr0 % 8 == 0: one 8-row block of a
// 256-row tile, i.e. fixed a, wm and the fragment-row pair hh = 2 hk, 2 hk + 1), read a whole 128-B line per 8 threads
// (the per-row loads take half lines: rows r and r + 4 share each line) into stg[row][ntn 128] (r05 late). The sum of
// every element is the per-row loads' (p0 + p1 + ... in chunk order): identical values.
template <int S>
__device__ __forceinline__ void fixup_stage(const GemmArgs& args, int gr0, float* stg) {
  constexpr int PMAX = 5;  // pieces per thread: ntn 32 lines x 8 / 512 <= 5 for N <= 1280
  const int ntm = (args.M + 255) >> 8, ntn = (args.N + 127) >> 7, LS = ntn * 128, nl = ntn * 256;
  const int mb = gr0 >> 8, rr0 = gr0 & 255, wm = rr0 >> 6, a = (rr0 >> 4) & 3, hk = (rr0 >> 3) & 1;
  const int GM = args.gm > 0 ? args.gm : 8;
  const int g0 = mb / GM, m0 = g0 * GM, gmm = min(GM, ntm - m0);
  f4 pv[PMAX][S];
#pragma unroll
  for (int p = 0; p < PMAX; ++p) {
    const int e = min((int)threadIdx.x + 512 * p, nl - 1);
    const int q = e & 7, L = e >> 3, wn = L & 1, r = (L >> 1) & 3, b = (L >> 3) & 3, nb = L >> 5;
    const int tl = g0 * GM * ntn + nb * gmm + (mb - m0) - args.tdp;
    const size_t off = (size_t)((a * 4 + b) * 4 + r) * 512 + (size_t)((wm * 2 + wn) * 64 + (2 * hk + (q >> 2)) * 16 +
                                                                     (q & 3) * 4);
#pragma unroll
    for (int c = 0; c < S; ++c) pv[p][c] = *reinterpret_cast<const f4*>(args.ws + (size_t)(tl * S + c) * (16 * 4 * 512) + off);
  }
#pragma unroll
  for (int p = 0; p < PMAX; ++p) {
    const int e = threadIdx.x + 512 * p;
    if (e < nl) {
      const int q = e & 7, L = e >> 3, wn = L & 1, r = (L >> 1) & 3, b = (L >> 3) & 3, nb = L >> 5;
      f4 acc = pv[p][0];
#pragma unroll
      for (int c = 1; c < S; ++c) acc += pv[p][c];
      *reinterpret_cast<f4*>(stg + ((q >> 2) * 4 + r) * LS + nb * 128 + wn * 64 + b * 16 + (q & 3) * 4) = acc;
    }
  }
}

// The same for tile 49's partials (r06, Tuning.h5_split: 256 x 144 tiles, every tile split S ways; k_gemm_h5 writes
// element (row 32 w + 16 a + 4 hh + r, column 16 b + rin) of a tile at ((a * 9 + b) * 4 + r) * 512 + 64 w + 16 hh + rin).
// The 8 rows gr0 .. gr0 + 7 are one wave w, one a and the fragment-row pair hh = 2 hk, 2 hk + 1: for each (tile column
// nb, b, r) one 128-B line holds rows 4 (hh & 1) + r of 16 columns. Chunk-order sums, as fixup_stage.
template <int S>
__device__ __forceinline__ void fixup_stage49(const GemmArgs& args, int gr0, float* stg) {
  constexpr int PMAX = 5;  // pieces per thread: ntn 8 x 36 lines x 8 / 512 = 4.5 for N = 1152
  const int ntm = (args.M + 255) >> 8, ntn = args.N / 144, LS = ((args.N + 127) >> 7) * 128, nl = ntn * 36 * 8;
  const int mb = gr0 >> 8, rr0 = gr0 & 255, w = rr0 >> 5, a = (rr0 >> 4) & 1, hk = (rr0 >> 3) & 1;
  const int GM = args.gm > 0 ? args.gm : 8;
  const int g0 = mb / GM, m0 = g0 * GM, gmm = min(GM, ntm - m0);
  f4 pv[PMAX][S];
#pragma unroll
  for (int p = 0; p < PMAX; ++p) {
    const int e = min((int)threadIdx.x + 512 * p, nl - 1);
    const int q = e & 7, L = e >> 3, r = L & 3, b = (L >> 2) % 9, nb = (L >> 2) / 9;
    const int tl = g0 * GM * ntn + nb * gmm + (mb - m0);
    const size_t off = (size_t)((a * 9 + b) * 4 + r) * 512 + (size_t)(w * 64 + (2 * hk + (q >> 2)) * 16 + (q & 3) * 4);
#pragma unroll
    for (int c = 0; c < S; ++c) pv[p][c] = *reinterpret_cast<const f4*>(args.ws + (size_t)(tl * S + c) * (18 * 4 * 512) + off);
  }
#pragma unroll
  for (int p = 0; p < PMAX; ++p) {
    const int e = threadIdx.x + 512 * p;
    if (e < nl) {
      const int q = e & 7, L = e >> 3, r = L & 3, b = (L >> 2) % 9, nb = (L >> 2) / 9;
      f4 acc = pv[p][0];
#pragma unroll
      for (int c = 1; c < S; ++c) acc += pv[p][c];
      *reinterpret_cast<f4*>(stg + ((q >> 2) * 4 + r) * LS + nb * 144 + b * 16 + (q & 3) * 4) = acc;
    }
  }
}

template <int NV, int S, bool STG = false, bool T49 = false>
__global__ __launch_bounds__(512) void k_fixup_ln(GemmArgs args, GemmLnArgs l) {
  // wave = GEMM row gr (ginv) or LN row j: with a gather, walking GEMM rows keeps each 128-B line of a partial
  // (two GEMM rows of one wave quarter) inside one workgroup
  const int w = blockIdx.x * 8 + (threadIdx.x >> 6), sl = threadIdx.x & 63;
  const GemmGroup G = args.g[0];
  const int N = args.N, f4n = N >> 2;
  // the row-invariant vectors (bias, gamma, beta) once per workgroup into LDS (r05: 15 of a wave's 35 global loads
  // re-read them per row; the kernel is bound by vector-memory issue, r04 PMC)
  __shared__ __attribute__((aligned(16))) float lv[3][kFixupLnMaxN];
  extern __shared__ __attribute__((aligned(16))) float stg[];  // STG: the workgroup's 8 rows of chunk sums
  for (int i = threadIdx.x; i < 3 * f4n; i += 512) {
    const int q = i / f4n, c4 = 4 * (i - q * f4n);
    const float* src = q == 0 ? G.bias : q == 1 ? l.gamma : l.beta;
    *reinterpret_cast<f4*>(&lv[q][c4]) = src ? *reinterpret_cast<const f4*>(src + c4) : f4{0.f, 0.f, 0.f, 0.f};
  }
  // (STG: the row's own loads are issued after the staging: issued before it they measured slower, r05ae)
  const int wl = min(w, args.M - 1);  // rows past M (the last workgroup) read row M - 1 and store nothing
  const int j = l.ginv ? l.ginv[wl] : wl;
  const int gr = l.ginv ? wl : l.gmap ? l.gmap[j] : j;
  const int xo = args.crow ? args.crow[gr] : gr;
  const int lo = l.lo_x ? xo : j;
  const int rrow = args.rmod > 0 ? xo % args.rmod : xo;
  f4 pv[S][NV], rv[NV], bv[NV], gv[NV], bb[NV];
  if constexpr (STG && T49) fixup_stage49<S>(args, blockIdx.x * 8, stg);  // GEMM row = w (host: ginv or no gmap)
  else if constexpr (STG) fixup_stage<S>(args, blockIdx.x * 8, stg);
  __syncthreads();
  if (w >= args.M) return;
  const int ntm = (args.M + 255) >> 8, ntn = (N + 127) >> 7;
  const int mb = gr >> 8, rr = gr & 255, wm = rr >> 6, a = (rr >> 4) & 3, hh = (rr >> 2) & 3, r = rr & 3;
  const int GM = args.gm > 0 ? args.gm : 8;  // tile_mn's grouped order (gemm_nt always sets gm)
  const int g0 = mb / GM, m0 = g0 * GM, gmm = min(GM, ntm - m0);
  bool ok[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int jv = sl + v * 64;
    ok[v] = jv < f4n;
    const int c4 = 4 * (ok[v] ? jv : f4n - 1);
    const int nb = c4 >> 7, cc = c4 & 127, wn = cc >> 6, b = (cc >> 4) & 3, rin = cc & 15;
    const int tl = g0 * GM * ntn + nb * gmm + (mb - m0) - args.tdp;
    const size_t off = (size_t)((a * 4 + b) * 4 + r) * 512 + (size_t)((wm * 2 + wn) * 64 + hh * 16 + rin);
    if (STG) {  // the chunk sum, staged in LDS (pv[0] holds it, the sum below adds nothing more)
      pv[0][v] = *reinterpret_cast<const f4*>(stg + (threadIdx.x >> 6) * (((N + 127) >> 7) * 128) + c4);
    } else {
#pragma unroll
      for (int c = 0; c < S; ++c)
        pv[c][v] = *reinterpret_cast<const f4*>(args.ws + (size_t)(tl * S + c) * (16 * 4 * 512) + off);
    }
    rv[v] = *reinterpret_cast<const f4*>(G.R + (size_t)rrow * args.ldr + c4);
  }
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int c4 = 4 * (ok[v] ? sl + v * 64 : f4n - 1);
    bv[v] = *reinterpret_cast<const f4*>(&lv[0][c4]);
    gv[v] = *reinterpret_cast<const f4*>(&lv[1][c4]);
    bb[v] = *reinterpret_cast<const f4*>(&lv[2][c4]);
  }
  // the fixup: chunk partials in chunk order, then + bias, then residual + (k_gemm_fixup_sub16 + epilogue)
  f4 xv[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    f4 acc = pv[0][v];
#pragma unroll
    for (int c = 1; c < (STG ? 1 : S); ++c) acc += pv[c][v];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float t = acc[e] + bv[v][e];
      xv[v][e] = rv[v][e] + t;
    }
    if (ok[v]) *reinterpret_cast<f4*>(G.C + (size_t)xo * args.ldc + 4 * (sl + v * 64)) = xv[v];
  }
  // k_ln_fwd<64, NV> on the row
  constexpr int L = 64;
  const int C = N;
  float s = 0.f;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const f4 x = ok[v] ? xv[v] : f4{0.f, 0.f, 0.f, 0.f};
    s += (x[0] + x[1]) + (x[2] + x[3]);
  }
  const float mean = sub_sum<L>(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = ok[v] ? xv[v][e] - mean : 0.f;
      q += d * d;
    }
  }
  const float rstd = 1.0f / sqrtf(sub_sum<L>(q) / (float)C + l.eps);
  unsigned mx = 0;
  f4 ov[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
#pragma unroll
    for (int e = 0; e < 4; ++e) ov[v][e] = (xv[v][e] - mean) * rstd * gv[v][e] + bb[v][e];
    if (ok[v]) mx = absmax4(mx, ov[v]);
  }
  mx = sub_max<L>(mx);
  const float sc = row_scale_of(mx);
  if (sl == 0) {
    l.rs[lo] = sc;
    l.stats[2 * lo] = mean;
    l.stats[2 * lo + 1] = rstd;
  }
  store_planes<L, NV>(l.pl + (size_t)lo * 2 * C, C, sl, ok, ov, sc);
}

// the backward form: dy = the fixup of a STORE GEMM without bias (chunk-order sum + 0, k_gemm_fixup_sub16's
// value), then k_ln_bwd<64, NV> on the row (x, res, y and the planes at row lmap[j], stats at j)
template <int NV, int S, bool STG = false, bool T49 = false>
__global__ __launch_bounds__(512) void k_fixup_ln_bwd(GemmArgs args, GemmLnArgs l) {
  const int j = blockIdx.x * 8 + (threadIdx.x >> 6), sl = threadIdx.x & 63;
  const int N = args.N, f4n = N >> 2, C = N;
  __shared__ __attribute__((aligned(16))) float lg[kFixupLnMaxN];  // gamma once per workgroup (as k_fixup_ln)
  extern __shared__ __attribute__((aligned(16))) float stg[];        // STG: the 8 rows' chunk sums
  for (int i = threadIdx.x; i < f4n; i += 512)
    *reinterpret_cast<f4*>(&lg[4 * i]) = *reinterpret_cast<const f4*>(l.gamma + 4 * i);
  const int jl = min(j, args.M - 1);  // rows past M read row M - 1 and store nothing
  const int pr = l.lmap ? l.lmap[jl] : jl;
  const float* res = l.res ? l.res : l.x;  // dummy source when there is no residual (never added)
  f4 pv[S][NV], xv[NV], gv[NV], rv[NV];
  if constexpr (STG && T49) fixup_stage49<S>(args, blockIdx.x * 8, stg);  // GEMM row = j
  else if constexpr (STG) fixup_stage<S>(args, blockIdx.x * 8, stg);
  __syncthreads();
  if (j >= args.M) return;
  const int gr = j;
  const int ntm = (args.M + 255) >> 8, ntn = (N + 127) >> 7;
  const int mb = gr >> 8, rr = gr & 255, wm = rr >> 6, a = (rr >> 4) & 3, hh = (rr >> 2) & 3, r = rr & 3;
  const int GM = args.gm > 0 ? args.gm : 8;
  const int g0 = mb / GM, m0 = g0 * GM, gmm = min(GM, ntm - m0);
  const float mean = l.stats[2 * j], rstd = l.stats[2 * j + 1];
  bool ok[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int jv = sl + v * 64;
    ok[v] = jv < f4n;
    const int c4 = 4 * (ok[v] ? jv : f4n - 1);
    const int nb = c4 >> 7, cc = c4 & 127, wn = cc >> 6, b = (cc >> 4) & 3, rin = cc & 15;
    const int tl = g0 * GM * ntn + nb * gmm + (mb - m0) - args.tdp;
    const size_t off = (size_t)((a * 4 + b) * 4 + r) * 512 + (size_t)((wm * 2 + wn) * 64 + hh * 16 + rin);
    if (STG) {
      pv[0][v] = *reinterpret_cast<const f4*>(stg + (threadIdx.x >> 6) * (((N + 127) >> 7) * 128) + c4);
    } else {
#pragma unroll
      for (int c = 0; c < S; ++c)
        pv[c][v] = *reinterpret_cast<const f4*>(args.ws + (size_t)(tl * S + c) * (16 * 4 * 512) + off);
    }
    xv[v] = *reinterpret_cast<const f4*>(l.x + (size_t)pr * N + c4);
    rv[v] = *reinterpret_cast<const f4*>(res + (size_t)pr * N + c4);
  }
#pragma unroll
  for (int v = 0; v < NV; ++v) gv[v] = *reinterpret_cast<const f4*>(&lg[4 * (ok[v] ? sl + v * 64 : f4n - 1)]);
  f4 dv[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    f4 acc = pv[0][v];
#pragma unroll
    for (int c = 1; c < (STG ? 1 : S); ++c) acc += pv[c][v];
#pragma unroll
    for (int e = 0; e < 4; ++e) dv[v][e] = acc[e] + 0.0f;  // the STORE epilogue's v = acc + bias (none)
  }
  // k_ln_bwd<64, NV>
  constexpr int L = 64;
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const f4 d = ok[v] ? dv[v] : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float gd = gv[v][e] * d[e];
      s1 += gd;
      s2 += gd * ((xv[v][e] - mean) * rstd);
    }
  }
  const float m1 = sub_sum<L>(s1) / (float)C;
  const float m2 = sub_sum<L>(s2) / (float)C;
  unsigned mx = 0;
  f4 ov[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
#pragma unroll
    for (int e = 0; e < 4; ++e) ov[v][e] = rstd * (gv[v][e] * dv[v][e] - m1 - ((xv[v][e] - mean) * rstd) * m2);
    if (l.res) {
#pragma unroll
      for (int e = 0; e < 4; ++e) ov[v][e] += rv[v][e];
    }
    if (ok[v]) {
      *reinterpret_cast<f4*>(l.y + (size_t)pr * N + 4 * (sl + v * 64)) = ov[v];
      mx = absmax4(mx, ov[v]);
    }
  }
  if (l.rs) {
    mx = sub_max<L>(mx);
    const float sc = row_scale_of(mx);
    if (sl == 0) l.rs[pr] = sc;
    if (l.pl) store_planes<L, NV>(l.pl + (size_t)pr * 2 * C, C, sl, ok, ov, sc);
  }
}

hipError_t fixup_ln_launch(const GemmArgs& a, const GemmLnArgs& l, hipStream_t s) {
  const int nv = (a.N / 4 + 63) / 64;
  if (nv > 5 || a.N % 4) return hipErrorInvalidValue;
  const dim3 grid((a.M + 7) / 8);
  count_launch(CNT_FIXUP_LN);
  // staged chunk sums (whole-line partial reads, fixup_stage) where the workgroup's 8 waves are 8 consecutive GEMM
  // rows: always in the backward, in the forward when the rows are walked in GEMM order (ginv) or not gathered
  const Tuning& TU = a.tune ? *a.tune : kDefaultTuning;
  const bool stg = TU.fixup_stage && (l.bwd || l.ginv || !l.gmap);
  const size_t sl = stg ? (size_t)8 * ((a.N + 127) / 128) * 128 * sizeof(float) : 0;
  if (a.t49 && !stg) return hipErrorInvalidValue;  // tile 49's partials are read by fixup_stage49 only
  if (a.t49) count_launch(CNT_H5_SPLIT);
#define VV_FIXUP_LN(K, S)                                                        \
  do {                                                                           \
    if (a.t49)                                                                   \
      hipLaunchKernelGGL((K<5, S, true, true>), grid, dim3(512), sl, s, a, l);   \
    else if (stg)                                                                \
      hipLaunchKernelGGL((K<5, S, true>), grid, dim3(512), sl, s, a, l);         \
    else                                                                         \
      hipLaunchKernelGGL((K<5, S, false>), grid, dim3(512), 0, s, a, l);         \
  } while (0)
  if (l.bwd) {
    switch (a.tsplit) {
      case 2: VV_FIXUP_LN(k_fixup_ln_bwd, 2); break;
      case 3: VV_FIXUP_LN(k_fixup_ln_bwd, 3); break;
      case 4: VV_FIXUP_LN(k_fixup_ln_bwd, 4); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  switch (a.tsplit) {
    case 2: VV_FIXUP_LN(k_fixup_ln, 2); break;
    case 3: VV_FIXUP_LN(k_fixup_ln, 3); break;
    case 4: VV_FIXUP_LN(k_fixup_ln, 4); break;
    default: return hipErrorInvalidValue;
  }
#undef VV_FIXUP_LN
  return hipGetLastError();
}

// lanes per row: <= 3 float4 per lane up to C = 384, then a full wave (C = 1152: 4.5 float4 per lane)
static int ln_lanes(int C) {
  const int f4n = C / 4;
  if (f4n <= 24) return 8;
  if (f4n <= 48) return 16;
  if (f4n <= 96) return 32;
  return 64;
}

template <bool FWD>
static hipError_t ln_launch(const LnArgs& a, hipStream_t s) {
  if (a.rows <= 0 || a.ngroups <= 0 || a.ngroups > kMaxGroups) return hipErrorInvalidValue;
  if ((a.C & 3) || a.C / 4 > 64 * LN_NVMAX) return hipErrorInvalidValue;
  if ((a.ldx & 3) || (a.ldy & 3) || (a.lddy & 3) || (a.ldres & 3)) return hipErrorInvalidValue;
  if (a.mode == LN_MERGE && ((a.C / 4) & 3)) return hipErrorInvalidValue;
  if (!FWD && (a.ldy != a.ldx || (a.g[0].res && a.ldres != a.ldx))) return hipErrorInvalidValue;
  for (int g = 0; g < a.ngroups; ++g) {
    if (a.g[g].rs && a.mode != LN_ROWMAP) return hipErrorInvalidValue;
    if (a.g[g].pl && !a.g[g].rs) return hipErrorInvalidValue;
    if (FWD && !a.g[g].y && !a.g[g].pl) return hipErrorInvalidValue;
  }
  const int L = ln_lanes(a.C);
  const int need = (a.C / 4 + L - 1) / L;
  const int NV = need <= 1 ? 1 : need <= 2 ? 2 : need <= 3 ? 3 : need <= 5 ? 5 : 8;
  const int rpb = 256 / L;
  dim3 grid((a.rows + rpb - 1) / rpb, a.ngroups);
  const int key = L * 16 + NV;
  switch (key) {
#define LNL(LL, NN)                                                                               \
  case LL * 16 + NN:                                                                              \
    if (FWD)                                                                                      \
      hipLaunchKernelGGL((k_ln_fwd<LL, NN>), grid, dim3(256), 0, s, a);                           \
    else                                                                                          \
      hipLaunchKernelGGL((k_ln_bwd<LL, NN>), grid, dim3(256), 0, s, a);                           \
    break;
    LNL(8, 1) LNL(8, 2) LNL(8, 3)
    LNL(16, 1) LNL(16, 2) LNL(16, 3)
    LNL(32, 1) LNL(32, 2) LNL(32, 3)
    LNL(64, 1) LNL(64, 2) LNL(64, 3) LNL(64, 5) LNL(64, 8)
#undef LNL
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t layernorm_fwd(const LnArgs& a, hipStream_t s) {
  if (a.rows <= 0 || a.ngroups <= 0 || a.ngroups > kMaxGroups) return hipErrorInvalidValue;
  const int ph = prof_begin(s);
  const hipError_t e = ln_launch<true>(a, s);
  prof_end(ph, s, PC_LN, 8.0 * a.rows * a.C * a.ngroups, 8.0 * a.rows * a.C * a.ngroups);
  return e;
}
hipError_t layernorm_bwd(const LnArgs& a, hipStream_t s) {
  if (a.rows <= 0 || a.ngroups <= 0 || a.ngroups > kMaxGroups) return hipErrorInvalidValue;
  const int ph = prof_begin(s);
  const hipError_t e = ln_launch<false>(a, s);
  prof_end(ph, s, PC_LN, 12.0 * a.rows * a.C * a.ngroups, (a.g[0].res ? 16.0 : 12.0) * a.rows * a.C * a.ngroups);
  return e;
}

// ============================================================================
// Window attention, 4x4 windows (N = 16 tokens), one workgroup per (window, chunk of heads)
// ============================================================================
constexpr int WN_ = 16;

// tb: this block's heads' slices of the relative-position table, staged in LDS as [hl][(2ws-1)^2]
__device__ __forceinline__ float attn_bias_mask(const AttnArgs& a, const float* tb, int win, int hl, int i, int j) {
  const int ws = a.ws;
  const int ri = i / ws, ci = i - ri * ws, rj = j / ws, cj = j - rj * ws;
  float b = tb[hl * (2 * ws - 1) * (2 * ws - 1) + (ri - rj + ws - 1) * (2 * ws - 1) + (ci - cj + ws - 1)];
  if (a.shift > 0) {
    // quirk Q1 (swinblock.py:240-258): labels depend on the (shifted-frame) row only
    const int wr = (win % (a.nWh * a.nWw)) / a.nWw;
    const int yi = wr * ws + ri, yj = wr * ws + rj;
    const int H = a.H;
    const int li = yi < H - ws ? 0 : (yi < H - a.shift ? 1 : 2);
    const int lj = yj < H - ws ? 0 : (yj < H - a.shift ? 1 : 2);
    if (li != lj) b += -100.0f;
  }
  return b;
}

// One workgroup (256 threads) per (window, chunk of HPB heads), HPB * hd <= 192: for the LG stage (hd 192) one
// head per block with the 64 score quads split four ways along d; for the Swin towers (hd 32) all heads of a
// window per block, so every token row is one contiguous HPB*hd-float load of q, k and v. Tokens of a window
// are 16 consecutive rows (window order, made by the LayerNorm gather).
//   scores: entry e = (head hl, row i, column quad jq), DP lanes per entry along d (interleaved 16-B steps),
//           reduced by xor shuffles; softmax over the 4 jq lanes of a row (same wave)
//   outputs: item = (token t, head hl, 4 consecutive d), d fastest -> coalesced row writes
// LDS: rows of HPB*hd + 4 floats (16-B aligned, consecutive rows start 4 banks apart).
#ifndef VV_ATTN_THREADS
#define VV_ATTN_THREADS 256
#endif
constexpr int kAttnThreads = VV_ATTN_THREADS;  // threads per attention workgroup
static_assert(kAttnThreads >= 256 && kAttnThreads % 64 == 0, "attn_rows_all stages 3 float4 per thread (768 per block)");

struct AttnShape {
  int hd, hpb, dp, st;  // head dim, heads per block, lanes per score quad, LDS row stride
};
__device__ __forceinline__ AttnShape attn_shape(const AttnArgs& a) {
  AttnShape s;
  s.hd = a.C / a.heads;
  s.hpb = a.heads / gridDim.y;
  const int e = s.hpb * 64;
  s.dp = e >= kAttnThreads ? 1 : kAttnThreads / e;  // 1, 2 or 4 (e in {64, 128, 192, 256, ...})
  s.st = s.hpb * s.hd + 4;
  return s;
}

// rows [16][n] (n floats from src row t at src + t * ld) -> LDS rows of stride st
__device__ __forceinline__ void attn_rows(const float* __restrict__ src, int ld, float* dst, int st, int n) {
  const int q4 = n >> 2;
  for (int idx = threadIdx.x; idx < WN_ * q4; idx += kAttnThreads) {
    const int t = idx / q4, d = (idx - t * q4) * 4;
    *reinterpret_cast<f4*>(dst + t * st + d) = *reinterpret_cast<const f4*>(src + (size_t)t * ld + d);
  }
}

// NA such [16][n] blocks (n <= 192: at most 3 float4 per thread each), every global load issued before the
// first LDS store so the workgroup waits for one memory round trip instead of one per block
template <int NA>
__device__ __forceinline__ void attn_rows_all(const float* const (&src)[NA], const int (&ld)[NA], float* const (&dst)[NA],
                                              int st, int n) {
  constexpr int IT = 3;
  const int q4 = n >> 2, tot = WN_ * q4;
  f4 r[NA][IT];
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int idx = threadIdx.x + i * kAttnThreads;
      if (idx < tot) {
        const int t = idx / q4, d = (idx - t * q4) * 4;
        r[a][i] = *reinterpret_cast<const f4*>(src[a] + (size_t)t * ld[a] + d);
      }
    }
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int idx = threadIdx.x + i * kAttnThreads;
      if (idx < tot) {
        const int t = idx / q4, d = (idx - t * q4) * 4;
        *reinterpret_cast<f4*>(dst[a] + t * st + d) = r[a][i];
      }
    }
}

// sv[jj] = sum_d x[i][hl*hd + d] y[j0+jj][hl*hd + d] over this lane's d-part, then over the DP lanes
__device__ __forceinline__ void attn_quad(const float* x, const float* y, const AttnShape& S, int hl, int i, int j0,
                                          int dpi, float sv[4]) {
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) sv[jj] = 0.0f;
  const float* xr = x + i * S.st + hl * S.hd;
  const float* yr = y + j0 * S.st + hl * S.hd;
  for (int d = dpi * 4; d < S.hd; d += 4 * S.dp) {
    const f4 xd = *reinterpret_cast<const f4*>(xr + d);
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const f4 yd = *reinterpret_cast<const f4*>(yr + jj * S.st + d);
      sv[jj] += xd[0] * yd[0] + xd[1] * yd[1] + xd[2] * yd[2] + xd[3] * yd[3];
    }
  }
  for (int o = 1; o < S.dp; o <<= 1)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) sv[jj] += __shfl_xor(sv[jj], o);
}

__global__ __launch_bounds__(kAttnThreads) void k_attn_fwd(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const AttnShape S = attn_shape(a);
  const int win = blockIdx.x, h0 = blockIdx.y * S.hpb, tid = threadIdx.x;
  const AttnGroup G = a.g[blockIdx.z];
  const int C = a.C, ldq = 3 * C, W = S.hpb * S.hd;
  float* q = sm;
  float* k = q + WN_ * S.st;
  float* v = k + WN_ * S.st;
  float* p = v + WN_ * S.st;          // [hpb][16][17]
  float* tb = p + S.hpb * WN_ * 17;   // [hpb][49]: the block's relative-position bias (ws = 4)
  const float* base = G.qkv + (size_t)win * WN_ * ldq + h0 * S.hd;
  // the bias slice is loaded with the q/k/v rows (one memory round trip), not inside the score loop
  constexpr int NTB = 49;
  float tv[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = min(tid + i * kAttnThreads, S.hpb * NTB - 1);
    tv[i] = G.table[(idx % NTB) * a.heads + h0 + idx / NTB];
  }
  if (W <= 192) {
    const float* const srcs[3] = {base, base + C, base + 2 * C};
    const int lds_[3] = {ldq, ldq, ldq};
    float* const dsts[3] = {q, k, v};
    attn_rows_all<3>(srcs, lds_, dsts, S.st, W);
  } else {
    attn_rows(base, ldq, q, S.st, W);
    attn_rows(base + C, ldq, k, S.st, W);
    attn_rows(base + 2 * C, ldq, v, S.st, W);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
    if (tid + i * kAttnThreads < S.hpb * NTB) tb[tid + i * kAttnThreads] = tv[i];
  __syncthreads();
  // S = (q k^T) scale + bias + mask -> softmax (swinblock.py:151-168)
  const int dpi = tid % S.dp;
  for (int e = tid / S.dp; e < S.hpb * 64; e += kAttnThreads / S.dp) {
    const int hl = e >> 6, i = (e >> 2) & 15, j0 = (e & 3) * 4, h = h0 + hl;
    float sv[4];
    attn_quad(q, k, S, hl, i, j0, dpi, sv);
    float mx = -INFINITY;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      sv[jj] = sv[jj] * a.scale + attn_bias_mask(a, tb, win, hl, i, j0 + jj);
      mx = fmaxf(mx, sv[jj]);
    }
    mx = fmaxf(mx, __shfl_xor(mx, S.dp));
    mx = fmaxf(mx, __shfl_xor(mx, 2 * S.dp));
    float sum = 0.f;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      sv[jj] = expf(sv[jj] - mx);
      sum += sv[jj];
    }
    sum += __shfl_xor(sum, S.dp);
    sum += __shfl_xor(sum, 2 * S.dp);
    const float inv = 1.0f / sum;
    if (dpi == 0) {
      f4 pv;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        pv[jj] = sv[jj] * inv;
        p[(hl * WN_ + i) * 17 + j0 + jj] = pv[jj];
      }
      *reinterpret_cast<f4*>(G.P + (((size_t)win * a.heads + h) * WN_ + i) * WN_ + j0) = pv;
    }
  }
  __syncthreads();
  // O = P v
  float* ob = G.o + (size_t)win * WN_ * C + h0 * S.hd;
  const int q4 = S.hd >> 2;
  for (int idx = tid; idx < WN_ * S.hpb * q4; idx += kAttnThreads) {
    const int t = idx / (S.hpb * q4), r = idx - t * S.hpb * q4, hl = r / q4, d = hl * S.hd + (r - hl * q4) * 4;
    const float* pr = p + (hl * WN_ + t) * 17;
    f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int jj = 0; jj < WN_; ++jj) {
      const float pj = pr[jj];
      const f4 vv = *reinterpret_cast<const f4*>(v + jj * S.st + d);
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] += pj * vv[c];
    }
    *reinterpret_cast<f4*>(ob + (size_t)t * C + d) = acc;
  }
}

__global__ __launch_bounds__(kAttnThreads) void k_attn_bwd(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const AttnShape S = attn_shape(a);
  const int win = blockIdx.x, h0 = blockIdx.y * S.hpb, tid = threadIdx.x;
  const AttnGroup G = a.g[blockIdx.z];
  const int C = a.C, ldq = 3 * C, W = S.hpb * S.hd;
  float* q = sm;
  float* k = q + WN_ * S.st;
  float* v = k + WN_ * S.st;
  float* dO = v + WN_ * S.st;
  float* p = dO + WN_ * S.st;       // [hpb][16][17]
  float* ds = p + S.hpb * WN_ * 17;  // [hpb][16][17]
  const float* base = G.qkv + (size_t)win * WN_ * ldq + h0 * S.hd;
  const float* dOb = G.dO + (size_t)win * WN_ * C + h0 * S.hd;
  // the block's P (hpb x 16 x 16 <= 3 per thread for hpb <= 3) is loaded with the rows: one round trip
  const float* Pg = G.P + ((size_t)win * a.heads + h0) * WN_ * WN_;
  const int np = S.hpb * WN_ * WN_;
  float pv[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) pv[i] = Pg[min(tid + i * kAttnThreads, np - 1)];
  if (W <= 192) {
    const float* const srcs[4] = {base, base + C, base + 2 * C, dOb};
    const int lds_[4] = {ldq, ldq, ldq, C};
    float* const dsts[4] = {q, k, v, dO};
    attn_rows_all<4>(srcs, lds_, dsts, S.st, W);
  } else {
    attn_rows(base, ldq, q, S.st, W);
    attn_rows(base + C, ldq, k, S.st, W);
    attn_rows(base + 2 * C, ldq, v, S.st, W);
    attn_rows(dOb, C, dO, S.st, W);
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int idx = tid + i * kAttnThreads;
    if (idx < np) p[(idx >> 4) * 17 + (idx & 15)] = pv[i];
  }
  for (int idx = tid + 3 * kAttnThreads; idx < np; idx += kAttnThreads) p[(idx >> 4) * 17 + (idx & 15)] = Pg[idx];
  __syncthreads();
  // dP = dO v^T ; dS = P (dP - rowsum(P dP))
  const int dpi = tid % S.dp;
  for (int e = tid / S.dp; e < S.hpb * 64; e += kAttnThreads / S.dp) {
    const int hl = e >> 6, i = (e >> 2) & 15, j0 = (e & 3) * 4;
    float dp[4];
    attn_quad(dO, v, S, hl, i, j0, dpi, dp);
    const float* pr = p + (hl * WN_ + i) * 17 + j0;
    float rd = 0.f;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) rd += pr[jj] * dp[jj];
    rd += __shfl_xor(rd, S.dp);
    rd += __shfl_xor(rd, 2 * S.dp);
    if (dpi == 0)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) ds[(hl * WN_ + i) * 17 + j0 + jj] = pr[jj] * (dp[jj] - rd);
  }
  __syncthreads();
  // dQ[t] = scale sum_u dS[t][u] k[u] ; dK[t] = scale sum_u dS[u][t] q[u] ; dV[t] = sum_u P[u][t] dO[u]
  float* gb = G.dqkv + (size_t)win * WN_ * ldq + h0 * S.hd;
  const int q4 = S.hd >> 2;
  for (int idx = tid; idx < WN_ * S.hpb * q4; idx += kAttnThreads) {
    const int t = idx / (S.hpb * q4), r = idx - t * S.hpb * q4, hl = r / q4, d = hl * S.hd + (r - hl * q4) * 4;
    const float* dsh = ds + hl * WN_ * 17;
    const float* ph = p + hl * WN_ * 17;
    f4 aq = {0.f, 0.f, 0.f, 0.f}, ak = aq, av = aq;
#pragma unroll
    for (int u = 0; u < WN_; ++u) {
      const float s_tu = dsh[t * 17 + u], s_ut = dsh[u * 17 + t], p_ut = ph[u * 17 + t];
      const f4 kk = *reinterpret_cast<const f4*>(k + u * S.st + d);
      const f4 qq = *reinterpret_cast<const f4*>(q + u * S.st + d);
      const f4 oo = *reinterpret_cast<const f4*>(dO + u * S.st + d);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        aq[c] += s_tu * kk[c];
        ak[c] += s_ut * qq[c];
        av[c] += p_ut * oo[c];
      }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      aq[c] *= a.scale;
      ak[c] *= a.scale;
    }
    float* row = gb + (size_t)t * ldq + d;
    *reinterpret_cast<f4*>(row) = aq;
    *reinterpret_cast<f4*>(row + C) = ak;
    *reinterpret_cast<f4*>(row + 2 * C) = av;
  }
}

// ---------------------------------------------------------------------------------------------------------
// LG-stage window attention on the exact-f32 MFMA (v_mfma_f32_16x16x4f32: fp32 products, fp32 accumulation, as
// torch's fp32 matmul; swinblock.py:151-172 for one head of hd = HD, one workgroup per (window, head)). Same
// inputs, outputs and saved P as k_attn_fwd / k_attn_bwd. The VALU kernels read every FMA operand from LDS
// (~490 KB of LDS reads per (window, head) against 36 KB of rows): their score and P.V phases are LDS-bound and
// serialised behind the loads. Here each operand element is read from LDS once per product.
//   scores (and dP = dO v^T): 16 x 16, K = HD split over the 4 waves (HD / 4 dims each); lane group g of a wave
//     takes a contiguous run of R = HD / 16 dims (the same dim permutation on both operands, so the product is
//     the plain dot product), loaded as float4s straight from global memory into the fragment registers; the four
//     wave partials are summed in wave order through LDS
//   softmax / dS: one thread per (i, j), the row reductions over the 16 lanes of the row
//   products with K = 16 keys (P v, dS k, dS^T q, P^T dO): lane group g takes keys 4g .. 4g + 3 (one per k-step);
//     wave w the output columns [w HD / 4, (w + 1) HD / 4) as HD / 64 tiles of 16 x 16
// Only the operands of the key-indexed products (v; q, k, dO) are staged in LDS, rows of HD + 4 floats (196: rows
// 4 banks apart, so the b32 reads of rows 4g + s x 16 consecutive columns are conflict-free); P and dS rows of 20.
// LDS 18 KB forward / 45 KB backward: all 768 workgroups of the LG stage resident at once.
typedef float f4m __attribute__((ext_vector_type(4)));
constexpr int kAmfP = 20;  // row stride of P / dS in LDS

// this lane's fragment run of a [16][HD] row block at src (row stride ld): row li, the R = HD / 16 dims of lane
// group g inside wave w's HD / 4 (straight from global memory: operands used only in the row-indexed pattern)
template <int HD>
__device__ __forceinline__ void amf_frag(const float* src, int ld, int w, int li, int g, f4 (&fr)[HD / 64]) {
  const float* r = src + (size_t)li * ld + w * (HD / 4) + g * (HD / 16);
#pragma unroll
  for (int s4 = 0; s4 < HD / 64; ++s4) fr[s4] = *reinterpret_cast<const f4*>(r + 4 * s4);
}

// S = X . Y^T partial of wave w over its HD / 4 dims (fragments from amf_frag), stored as part[w][16][17]
template <int HD>
__device__ __forceinline__ void amf_partial(const f4 (&xa)[HD / 64], const f4 (&yb)[HD / 64], float* part, int w,
                                            int li, int g) {
  static_assert(HD % 64 == 0, "HD must be a multiple of 64");
  f4m acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s4 = 0; s4 < HD / 64; ++s4)
#pragma unroll
    for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[s4][e], yb[s4][e], acc, 0, 0, 0);
#pragma unroll
  for (int r = 0; r < 4; ++r) part[(w * 16 + 4 * g + r) * 17 + li] = acc[r];
}

template <int HD>
__global__ __launch_bounds__(256) void k_attn_fwd_mf(AttnArgs a) {
  constexpr int ST = HD + 4, NT = HD / 64;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* v = sm;                     // [16][ST]: the only operand read in the key-indexed pattern
  float* part = v + WN_ * ST;        // [4][16][17]
  float* p = part + 4 * WN_ * 17;    // [16][20]
  float* tb = p + WN_ * kAmfP;       // [49]
  const int win = blockIdx.x, h = blockIdx.y, tid = threadIdx.x;
  const int w = tid >> 6, l = tid & 63, li = l & 15, g = l >> 4;
  const AttnGroup G = a.g[blockIdx.z];
  const int C = a.C, ldq = 3 * C;
  const float* base = G.qkv + (size_t)win * WN_ * ldq + h * HD;
  // every load issued before the first wait: q / k fragments to registers, the bias slice, v rows to LDS
  f4 qf[NT], kf[NT];
  amf_frag<HD>(base, ldq, w, li, g, qf);
  amf_frag<HD>(base + C, ldq, w, li, g, kf);
  const float tv = G.table[min(tid, 48) * a.heads + h];
  {
    const float* const srcs[1] = {base + 2 * C};
    const int lds_[1] = {ldq};
    float* const dsts[1] = {v};
    attn_rows_all<1>(srcs, lds_, dsts, ST, HD);
  }
  if (tid < 49) tb[tid] = tv;
  // plane output: one row scale for the window from the bound on |v| (loaded with the rows)
  float so = 0.f;
  if (a.opl) {
    const float vr = a.vrs[(size_t)win * WN_ + li];  // 2^e_j: max|A_j| < 2^15 / vr
    const float tw = *a.vbw, tbb = *(a.vbb ? a.vbb : a.vbw);
    float ia = __uint_as_float((254u << 23) - __float_as_uint(vr));
    ia = lane_max<16>(ia);
    const unsigned mx = __float_as_uint(2.0f * ((float)C * tw * (32768.0f * ia) + (a.vbb ? tbb : 0.0f)));
    so = __uint_as_float((268u - max(mx >> 23, 15u)) << 23);
    if (h == 0 && tid < WN_) a.ors[(size_t)win * WN_ + tid] = so;
  }
  amf_partial<HD>(qf, kf, part, w, li, g);
  __syncthreads();
  {
    // S = (q k^T) scale + bias + mask -> softmax (swinblock.py:151-168); thread = (row i, column j)
    const int i = tid >> 4, j = tid & 15;
    const float* pp = part + i * 17 + j;
    float s = ((pp[0] + pp[WN_ * 17]) + (pp[2 * WN_ * 17] + pp[3 * WN_ * 17])) * a.scale +
              attn_bias_mask(a, tb, win, 0, i, j);
    float mx = s;
    mx = lane_max16_up(mx);
    const float e = expf(s - mx);
    float sum = e;
    sum = lane_sum16_up(sum);
    const float pv = e * (1.0f / sum);
    p[i * kAmfP + j] = pv;
    G.P[((size_t)win * a.heads + h) * WN_ * WN_ + tid] = pv;
  }
  __syncthreads();
  // O = P v: A = P[i][4g + s], B = v[4g + s][n]
  const f4 pa = *reinterpret_cast<const f4*>(p + li * kAmfP + 4 * g);
  float* ob = G.o + (size_t)win * WN_ * C + h * HD;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int n0 = w * (HD / 4) + 16 * nt;
    f4m acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 4; ++s)
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[s], v[(4 * g + s) * ST + n0 + li], acc, 0, 0, 0);
    if (a.opl) {
      const int c = h * HD + n0 + li;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float x = acc[r] * so;
        const _Float16 hv = (_Float16)x;
        const _Float16 lv = (_Float16)(x - (float)hv);
        unsigned short* pp = a.opl + ((size_t)win * WN_ + 4 * g + r) * 2 * C + 2 * (c & ~31) + (c & 31);
        pp[0] = __builtin_bit_cast(unsigned short, hv);
        pp[32] = __builtin_bit_cast(unsigned short, lv);
      }
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) ob[(size_t)(4 * g + r) * C + n0 + li] = acc[r];
    }
  }
}

template <int HD>
__global__ __launch_bounds__(256) void k_attn_bwd_mf(AttnArgs a) {
  constexpr int ST = HD + 4, NT = HD / 64;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* q = sm;                     // q, k, dO: read in the key-indexed pattern (dK, dQ, dV)
  float* k = q + WN_ * ST;
  float* dO = k + WN_ * ST;
  float* part = dO + WN_ * ST;       // [4][16][17]
  float* p = part + 4 * WN_ * 17;    // [16][20]
  float* ds = p + WN_ * kAmfP;       // [16][20]
  const int win = blockIdx.x, h = blockIdx.y, tid = threadIdx.x;
  const int w = tid >> 6, l = tid & 63, li = l & 15, g = l >> 4;
  const AttnGroup G = a.g[blockIdx.z];
  const int C = a.C, ldq = 3 * C;
  const float* base = G.qkv + (size_t)win * WN_ * ldq + h * HD;
  const float* dOg = G.dO + (size_t)win * WN_ * C + h * HD;
  // every load issued before the first wait: dO / v fragments (dP) to registers, P, the q / k / dO rows to LDS
  f4 of[NT], vf[NT];
  amf_frag<HD>(dOg, C, w, li, g, of);
  amf_frag<HD>(base + 2 * C, ldq, w, li, g, vf);
  const float pij = G.P[((size_t)win * a.heads + h) * WN_ * WN_ + tid];  // thread = (i, j) = (tid >> 4, tid & 15)
  {
    const float* const srcs[3] = {base, base + C, dOg};
    const int lds_[3] = {ldq, ldq, C};
    float* const dsts[3] = {q, k, dO};
    attn_rows_all<3>(srcs, lds_, dsts, ST, HD);
  }
  const int i = tid >> 4, j = tid & 15;
  p[i * kAmfP + j] = pij;
  amf_partial<HD>(of, vf, part, w, li, g);  // dP = dO v^T
  __syncthreads();
  {
    // dS = P (dP - rowsum(P dP))
    const float* pp = part + i * 17 + j;
    const float dp = (pp[0] + pp[WN_ * 17]) + (pp[2 * WN_ * 17] + pp[3 * WN_ * 17]);
    float rd = pij * dp;
    rd = lane_sum16_up(rd);
    ds[i * kAmfP + j] = pij * (dp - rd);
  }
  __syncthreads();
  // dQ = scale dS k ; dK = scale dS^T q ; dV = P^T dO  (k-step s: key 4g + s)
  const f4 dsa = *reinterpret_cast<const f4*>(ds + li * kAmfP + 4 * g);
  float dst[4], pt[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    dst[s] = ds[(4 * g + s) * kAmfP + li];
    pt[s] = p[(4 * g + s) * kAmfP + li];
  }
  float* gb = G.dqkv + (size_t)win * WN_ * ldq + h * HD;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int n0 = w * (HD / 4) + 16 * nt;
    f4m aq = {0.f, 0.f, 0.f, 0.f}, ak = aq, av = aq;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int rr = (4 * g + s) * ST + n0 + li;
      aq = __builtin_amdgcn_mfma_f32_16x16x4f32(dsa[s], k[rr], aq, 0, 0, 0);
      ak = __builtin_amdgcn_mfma_f32_16x16x4f32(dst[s], q[rr], ak, 0, 0, 0);
      av = __builtin_amdgcn_mfma_f32_16x16x4f32(pt[s], dO[rr], av, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float* row = gb + (size_t)(4 * g + r) * ldq + n0 + li;
      row[0] = aq[r] * a.scale;
      row[C] = ak[r] * a.scale;
      row[2 * C] = av[r];
    }
  }
}

// Swin-tower window attention (head dim 32: the dim-96 / dim-192 stages, 3 / 6 heads) on the exact-f32 MFMA, one
// wave per (window, head), four per workgroup, no LDS in the forward. The scores are computed transposed,
// S^T = k q^T (keys on the accumulator rows), so each lane (query li, lane group g) holds P[li][4g + r] in register r:
// exactly the A operand of O = P v for k-step r (key 4g + r). Softmax over a query's 16 keys: 4 registers, then
// lanes li, li + 16, li + 32, li + 48. Row operands (q, k for S^T; v, dO for dP^T) are loaded as float4 fragments
// straight from global memory (lane group g: dims 8g .. 8g + 7); key-indexed operands (v, k, q, dO) as one float
// per lane (16 consecutive columns of row 4g + s). The backward transposes dS through 1 KB of LDS per wave.
__device__ __forceinline__ void awin_frag(const float* src, int ld, int li, int g, f4& a, f4& b) {
  const float* r = src + (size_t)li * ld + 8 * g;
  a = *reinterpret_cast<const f4*>(r);
  b = *reinterpret_cast<const f4*>(r + 4);
}
__device__ __forceinline__ f4m awin_st(const f4& xa, const f4& xb, const f4& ya, const f4& yb) {
  f4m acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[e], ya[e], acc, 0, 0, 0);
#pragma unroll
  for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xb[e], yb[e], acc, 0, 0, 0);
  return acc;
}

__global__ __launch_bounds__(256) void k_attn_fwd_w32(AttnArgs a) {
  constexpr int HD = 32;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, li = l & 15, g = l >> 4;
  const int item = blockIdx.x * 4 + w, win = item / a.heads, h = item - win * a.heads;
  const AttnGroup G = a.g[blockIdx.z];
  const int C = a.C, ldq = 3 * C;
  const float* base = G.qkv + (size_t)win * WN_ * ldq + h * HD;
  f4 qa, qb, ka, kb;
  awin_frag(base, ldq, li, g, qa, qb);
  awin_frag(base + C, ldq, li, g, ka, kb);
  float vv[2][4];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int s = 0; s < 4; ++s) vv[nt][s] = base[2 * C + (size_t)(4 * g + s) * ldq + 16 * nt + li];
  // bias table entries of (query li, key 4g + r): loaded with the rows
  const int ri = li >> 2, ci = li & 3;
  float bias[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int j = 4 * g + r, rj = j >> 2, cj = j & 3;
    bias[r] = G.table[((ri - rj + 3) * 7 + (ci - cj + 3)) * a.heads + h];
  }
  const f4m st = awin_st(ka, kb, qa, qb);  // S^T: row = key 4g + r, column = query li
  float sv[4], mx = -INFINITY;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float b = bias[r];
    if (a.shift > 0) {  // quirk Q1 (swinblock.py:240-258), as attn_bias_mask
      const int wr = (win % (a.nWh * a.nWw)) / a.nWw, j = 4 * g + r;
      const int yi = wr * 4 + ri, yj = wr * 4 + (j >> 2), H = a.H;
      const int lbi = yi < H - 4 ? 0 : (yi < H - a.shift ? 1 : 2);
      const int lbj = yj < H - 4 ? 0 : (yj < H - a.shift ? 1 : 2);
      if (lbi != lbj) b += -100.0f;
    }
    sv[r] = st[r] * a.scale + b;
    mx = fmaxf(mx, sv[r]);
  }
  mx = fmaxf(mx, xshfl<16>(mx));
  mx = fmaxf(mx, xshfl<32>(mx));
  float sum = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    sv[r] = expf(sv[r] - mx);
    sum += sv[r];
  }
  sum += xshfl<16>(sum);
  sum += xshfl<32>(sum);
  const float inv = 1.0f / sum;
  f4 pv;
#pragma unroll
  for (int r = 0; r < 4; ++r) pv[r] = sv[r] * inv;
  *reinterpret_cast<f4*>(G.P + ((size_t)win * a.heads + h) * WN_ * WN_ + li * WN_ + 4 * g) = pv;
  float* ob = G.o + (size_t)win * WN_ * C + h * HD;
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    f4m acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(pv[s], vv[nt][s], acc, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 4; ++r) ob[(size_t)(4 * g + r) * C + 16 * nt + li] = acc[r];
  }
}

__global__ __launch_bounds__(256) void k_attn_bwd_w32(AttnArgs a) {
  constexpr int HD = 32;
  __shared__ float dsm[4][WN_ * 17];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, li = l & 15, g = l >> 4;
  const int item = blockIdx.x * 4 + w, win = item / a.heads, h = item - win * a.heads;
  const AttnGroup G = a.g[blockIdx.z];
  const int C = a.C, ldq = 3 * C;
  const float* base = G.qkv + (size_t)win * WN_ * ldq + h * HD;
  const float* dOg = G.dO + (size_t)win * WN_ * C + h * HD;
  const float* Pg = G.P + ((size_t)win * a.heads + h) * WN_ * WN_;
  f4 va, vb, oa, ob;
  awin_frag(base + 2 * C, ldq, li, g, va, vb);
  awin_frag(dOg, C, li, g, oa, ob);
  const f4 pr = *reinterpret_cast<const f4*>(Pg + li * WN_ + 4 * g);  // P[li][4g + r]
  float pt[4], kc[2][4], qc[2][4], oc[2][4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    pt[s] = Pg[(4 * g + s) * WN_ + li];  // P[4g + s][li]
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const size_t rr = (size_t)(4 * g + s) * ldq + 16 * nt + li;
      qc[nt][s] = base[rr];
      kc[nt][s] = base[C + rr];
      oc[nt][s] = dOg[(size_t)(4 * g + s) * C + 16 * nt + li];
    }
  }
  const f4m dpt = awin_st(va, vb, oa, ob);  // dP^T: row = key 4g + r, column = query li
  float rd = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) rd += pr[r] * dpt[r];
  rd += xshfl<16>(rd);
  rd += xshfl<32>(rd);
  f4 ds;  // dS[li][4g + r]
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    ds[r] = pr[r] * (dpt[r] - rd);
    dsm[w][li * 17 + 4 * g + r] = ds[r];
  }
  __syncthreads();
  float dt[4];  // dS[4g + s][li]
#pragma unroll
  for (int s = 0; s < 4; ++s) dt[s] = dsm[w][(4 * g + s) * 17 + li];
  float* gb = G.dqkv + (size_t)win * WN_ * ldq + h * HD;
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    f4m aq = {0.f, 0.f, 0.f, 0.f}, ak = aq, av = aq;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      aq = __builtin_amdgcn_mfma_f32_16x16x4f32(ds[s], kc[nt][s], aq, 0, 0, 0);
      ak = __builtin_amdgcn_mfma_f32_16x16x4f32(dt[s], qc[nt][s], ak, 0, 0, 0);
      av = __builtin_amdgcn_mfma_f32_16x16x4f32(pt[s], oc[nt][s], av, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float* row = gb + (size_t)(4 * g + r) * ldq + 16 * nt + li;
      row[0] = aq[r] * a.scale;
      row[C] = ak[r] * a.scale;
      row[2 * C] = av[r];
    }
  }
}

static bool attn_w32_ok(const AttnArgs& a) {
  return a.mfma && a.ws == 4 && a.heads > 0 && a.C == 32 * a.heads && (a.nwin * a.heads) % 4 == 0;
}

// the MFMA kernels serve one head of 192 per workgroup (the LG stage, 6 heads of 192) with 4x4 windows
static bool attn_mf_ok(const AttnArgs& a) {
  return a.mfma && a.ws == 4 && a.heads > 0 && a.C == 192 * a.heads;
}

// heads per block: the largest divisor of heads with hpb * hd <= 192
static int attn_hpb(const AttnArgs& a) {
  const int hd = a.C / a.heads;
  int hpb = 1;
  for (int c = 1; c <= a.heads; ++c)
    if (a.heads % c == 0 && c * hd <= 192) hpb = c;
  return hpb;
}
static bool attn_ok(const AttnArgs& a) {
  if (a.ws != 4 || a.heads <= 0 || a.C % a.heads != 0 || a.ngroups <= 0 || a.ngroups > kMaxGroups) return false;
  const int hd = a.C / a.heads;
  return (hd & 3) == 0 && hd <= 256;
}

hipError_t attn_fwd(const AttnArgs& a, hipStream_t s) {
  if (!attn_ok(a)) return hipErrorInvalidValue;
  if (a.opl && (!attn_mf_ok(a) || attn_w32_ok(a) || a.ngroups != 1 || !a.ors || !a.vrs || !a.vbw))
    return hipErrorInvalidValue;
  const int hpb = attn_hpb(a), st = hpb * (a.C / a.heads) + 4;
  if (2 * kAttnThreads < hpb * 49) return hipErrorInvalidValue;  // the staged bias slice (ws = 4)
  const size_t lds = (3 * WN_ * st + hpb * WN_ * 17 + hpb * 49) * sizeof(float);
  const int ph = prof_begin(s);
  if (attn_w32_ok(a)) {
    hipLaunchKernelGGL(k_attn_fwd_w32, dim3(a.nwin * a.heads / 4, 1, a.ngroups), dim3(256), 0, s, a);
  } else if (attn_mf_ok(a)) {
    const size_t lds_mf = (WN_ * 196 + 4 * WN_ * 17 + WN_ * kAmfP + 49) * sizeof(float);
    hipLaunchKernelGGL(k_attn_fwd_mf<192>, dim3(a.nwin, a.heads, a.ngroups), dim3(256), lds_mf, s, a);
  } else
    hipLaunchKernelGGL(k_attn_fwd, dim3(a.nwin, a.heads / hpb, a.ngroups), dim3(kAttnThreads), lds, s, a);
  prof_end(ph, s, PC_ATTN, 4.0 * a.nwin * WN_ * WN_ * a.C * a.ngroups,
           4.0 * a.ngroups * ((double)a.nwin * WN_ * 4 * a.C + (double)a.nwin * a.heads * WN_ * WN_));
  return hipGetLastError();
}
hipError_t attn_bwd(const AttnArgs& a, hipStream_t s) {
  if (!attn_ok(a)) return hipErrorInvalidValue;
  const int hpb = attn_hpb(a), st = hpb * (a.C / a.heads) + 4;
  const size_t lds = (4 * WN_ * st + 2 * hpb * WN_ * 17) * sizeof(float);
  const int ph = prof_begin(s);
  if (attn_w32_ok(a)) {
    hipLaunchKernelGGL(k_attn_bwd_w32, dim3(a.nwin * a.heads / 4, 1, a.ngroups), dim3(256), 0, s, a);
  } else if (attn_mf_ok(a)) {
    const size_t lds_mf = (3 * WN_ * 196 + 4 * WN_ * 17 + 2 * WN_ * kAmfP) * sizeof(float);
    hipLaunchKernelGGL(k_attn_bwd_mf<192>, dim3(a.nwin, a.heads, a.ngroups), dim3(256), lds_mf, s, a);
  } else
    hipLaunchKernelGGL(k_attn_bwd, dim3(a.nwin, a.heads / hpb, a.ngroups), dim3(kAttnThreads), lds, s, a);
  prof_end(ph, s, PC_ATTN, 8.0 * a.nwin * WN_ * WN_ * a.C * a.ngroups,
           4.0 * a.ngroups * ((double)a.nwin * WN_ * 7 * a.C + (double)a.nwin * a.heads * WN_ * WN_));
  return hipGetLastError();
}

// ============================================================================
// PatchEmbed (Conv2d k=s=2) + absolute_pos_embed   (transformer.py:41-49, 392-394)
// ConvTranspose2d(k=s=2) + Dec_net mean/std reorder (transformer.py:593-623, quirk Q2)
// ============================================================================
// PatchEmbed and ConvTranspose2d with k = s = 2 are per-token GEMMs (the im2col of a stride-2 2x2 patch is a plain
// gather of 4 cin pixels): two kernels on the exact-f32 MFMA (v_mfma_f32_16x16x4_f32: fp32 products and sums, as
// torch's fp32 conv; only the summation order differs), one wave per 16 tokens, four waves per workgroup sharing the
// tower's weights in LDS. Fragment layout of 16x16x4: lane l gives A[l % 16][k = l / 16] and B[k][l % 16] and holds
// D[4 (l / 16) + r][l % 16]. A float4 read of 4 consecutive k per lane serves 4 k-steps when the k index of step i
// in lane group g is kappa(i, g) = 16 (i / 4) + 4 g + i % 4 (the same permutation on both operands).
//
// k_p2t_mf (pixels -> token rows: PatchEmbed forward, ConvTranspose backward): D[t][c] = sum_j X[t][j] W[c][j] with
//   X the 2x2xC patches of the 64 tokens staged in LDS by coalesced image-row loads ([t][KP], zero-padded), W[c][j]
//   staged in LDS; lane (c, g) writes D[4 g + r][c]: 16 consecutive channels of a token row per 16 lanes.
//   MODE 0: tok = (D + bias) + pos, x[t][ci 4 + 2 p + q] = img[cin_off + ci][2ho + p][2wo + q]
//   MODE 1: dtok = D, x[t][co 4 + 2 p + q] = dout[ch(co)][2ho + p][2wo + q] (0 at channels >= climit)
// k_t2p_mf (token rows -> pixels: PatchEmbed backward, ConvTranspose forward): D[j][t] = sum_c W[c][j] Y[t][c] with
//   Y's rows read per lane as float4 from global memory and W transposed in LDS; lane (t, g) holds D[4 g + r][t], i.e.
//   outputs j = 4 (4 mt + g) + 2 p + q of token t: two float2 stores (q = 0, 1) of horizontally adjacent pixels,
//   consecutive lanes = consecutive pixels (needs Wo % 16 == 0).
//   MODE 0: dimg = add + D; MODE 1: out[ch(co)] = D + bias[co] (ch < climit)
constexpr int PT = 64;  // tokens per workgroup (4 waves x 16)

__device__ __forceinline__ void tok_coords(int tok, int Ho, int Wo, int& b, int& ho, int& wo) {
  b = tok / (Ho * Wo);
  const int rem = tok - b * Ho * Wo;
  ho = rem / Wo;
  wo = rem - ho * Wo;
}

__device__ __forceinline__ int unembed_ch(const PatchGroup& G, int co) {
  const int half = G.cout / 2;
  return co < half ? G.mean_off + co : G.std_off + co - half;
}

constexpr int kPatchKmax = 112;  // patch taps per token (4 x channels), padded to 16
constexpr int kPatchCmax = 128;  // token channels

template <int MODE, int KPM>
__global__ __launch_bounds__(256) void k_p2t_mf(PatchArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const PatchGroup& G = a.g[blockIdx.y];
  const int Ho = a.Himg / 2, Wo = a.Wimg / 2, ntok = a.B * Ho * Wo;
  const int kc = MODE == 0 ? G.cin * 4 : G.cout * 4, C = a.Ctok;
  const int KP = (kc + 15) / 16 * 16, KS = KP + 4;  // padded K; LDS row stride (floats)
  const int OS = C + 4;                             // row stride of the per-wave output staging (floats)
  float* Xs = sm;             // [64][KS]
  float* Wsm = Xs + PT * KS;  // [C][KS]
  float* Os = sm;             // [4 waves][16][OS]: D + bias, rows = tokens, for whole-row float4 stores; over Xs / Wsm
                              // once every wave's MFMAs are done (r05: separate, it cost the KPM 64 / 112 launches
                              // a resident workgroup per CU -- 1.5 and 3 rounds of 768 workgroups)
  const int t0 = blockIdx.x * PT;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
  const int tb = wave * 16;  // this wave's 16 tokens within the workgroup: one contiguous [16][C] block of rows
  const bool wok = t0 + tb < ntok;
  constexpr int NO = kPatchCmax / 16;  // float4 of the wave's [16][C] block per lane (C / 16 used)
  // every global load of the kernel is issued here, before any LDS store or MFMA: the pixels of the patches, the
  // weights, and (MODE 0) the absolute_pos_embed rows and the bias -- one memory latency per workgroup, not three
  f4 pv[NO];
  if (MODE == 0) {
    const size_t pbase = (size_t)((wok ? t0 + tb : 0) % (Ho * Wo)) * C;
#pragma unroll
    for (int i = 0; i < NO; ++i)
      pv[i] = (i < C / 16 && wok) ? *reinterpret_cast<const f4*>(G.pos + pbase + 4 * (i * 64 + lane))
                                  : f4{0.f, 0.f, 0.f, 0.f};
  }
  constexpr int NTM = kPatchCmax / 16;
  float bv[NTM];
#pragma unroll
  for (int n = 0; n < NTM; ++n) bv[n] = MODE == 0 ? G.bias[min(n * 16 + li, C - 1)] : 0.f;
  constexpr int NR = KPM / 4;  // (ci, p) rows per thread at most (KPM: the padded K this instantiation serves)
  float xv[NR];
  // thread (t, q) of one of two row phases: consecutive threads read consecutive pixels of an image row
  const int xq = threadIdx.x & 1, xt = (threadIdx.x >> 1) & (PT - 1), half = threadIdx.x >> 7;
  {
    const int tok = t0 + xt;
    const bool okt = tok < ntok;
    int b, ho, wo;
    tok_coords(okt ? tok : 0, Ho, Wo, b, ho, wo);
    const size_t plane = (size_t)a.Himg * a.Wimg;
    const float* base = a.img + (size_t)b * a.Cimg * plane + (size_t)(2 * ho) * a.Wimg + 2 * wo + xq;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int rest = half + 2 * r, ci = rest >> 1, pp = rest & 1;  // rest = ci 2 + p (co 2 + p)
      xv[r] = 0.f;
      if (rest < KP / 2 && okt && ci * 4 < kc) {
        const int ch = MODE == 0 ? G.cin_off + ci : unembed_ch(G, ci);
        if (MODE == 0 || ch < a.climit) xv[r] = base[(size_t)ch * plane + pp * a.Wimg];
      }
    }
  }
  // weights (L2-resident: every workgroup of the tower reads them) in batches of 16 loads; the first batch is in
  // flight with the pixels before the first LDS store
  constexpr int NW = kPatchCmax * KPM / 256, NB = NW < 16 ? NW : 16;
#pragma unroll
  for (int h = 0; h < NW; h += NB) {
    float wv[NB];
#pragma unroll
    for (int r = 0; r < NB; ++r) {
      const int i = threadIdx.x + 256 * (h + r), c = i / KP, j = i - c * KP;
      wv[r] = (c < C && j < kc) ? G.w[(size_t)c * kc + j] : 0.f;
    }
    if (h == 0) {
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const int rest = half + 2 * r;
        if (rest < KP / 2) Xs[xt * KS + (rest >> 1) * 4 + (rest & 1) * 2 + xq] = xv[r];
      }
    }
#pragma unroll
    for (int r = 0; r < NB; ++r) {
      const int i = threadIdx.x + 256 * (h + r), c = i / KP, j = i - c * KP;
      if (c < C) Wsm[c * KS + j] = wv[r];
    }
  }
  __syncthreads();
  typedef float fr4 __attribute__((ext_vector_type(4)));
  const int nt = (C + 15) / 16;
  fr4 acc[NTM];
  const float* xr = Xs + (tb + li) * KS + 4 * g;
#pragma unroll
  for (int n = 0; n < NTM; ++n) {
    acc[n] = fr4{0.f, 0.f, 0.f, 0.f};
    if (n < nt) {
      const float* wr = Wsm + min(n * 16 + li, C - 1) * KS + 4 * g;
      for (int s4 = 0; s4 < KP; s4 += 16) {
        const f4 xa = *reinterpret_cast<const f4*>(xr + s4);
        const f4 wb = *reinterpret_cast<const f4*>(wr + s4);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[e], wb[e], acc[n], 0, 0, 0);
      }
    }
  }
  // lane (channel n 16 + li, g) holds tokens 4 g + r: (D + bias) into the wave's staging rows, then read back as the
  // wave's contiguous [16][C] block, float4 per lane, + pos: whole 1-KB row runs per store instruction
  __syncthreads();  // every wave's Xs / Wsm reads are done: the staging rows overlay them
  float* O = Os + wave * 16 * OS;
#pragma unroll
  for (int n = 0; n < NTM; ++n) {
    const int c = n * 16 + li;
    if (n >= nt || c >= C) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) O[(4 * g + r) * OS + c] = MODE == 0 ? acc[n][r] + bv[n] : acc[n][r];
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's staging stores done (no other wave reads them)
  __builtin_amdgcn_wave_barrier();
  if (!wok) return;
  float* out = G.tok + (size_t)(t0 + tb) * C;
#pragma unroll
  for (int i = 0; i < NO; ++i) {
    if (i >= C / 16) break;
    const int e = 4 * (i * 64 + lane), row = e / C, col = e - row * C;
    f4 v = *reinterpret_cast<const f4*>(O + row * OS + col);
    if (MODE == 0) v = v + pv[i];
    *reinterpret_cast<f4*>(out + e) = v;
  }
}

template <int MODE, int KPM>
__global__ __launch_bounds__(256) void k_t2p_mf(PatchArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const PatchGroup& G = a.g[blockIdx.y];
  const int Ho = a.Himg / 2, Wo = a.Wimg / 2, ntok = a.B * Ho * Wo;
  const int kc = MODE == 0 ? G.cin * 4 : G.cout * 4, C = a.Ctok;
  const int CP = (C + 15) / 16 * 16, CS = CP + 4;
  float* Wt = sm;  // [KP][CS]: W[c][j] at Wt[j][c]
  const int KP = (kc + 15) / 16 * 16;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
  const int tok = blockIdx.x * PT + wave * 16 + li;
  const bool ok = tok < ntok;
  constexpr int NMT = KPM / 16;
  const int nmt = KP / 16;
  int b, ho, wo;
  tok_coords(ok ? tok : 0, Ho, Wo, b, ho, wo);
  // every global load first (token rows, the added image / bias, the weights), then the LDS transposition: one
  // memory latency per workgroup
  const float* yr = (MODE == 0 ? G.dtok : G.tok) + (size_t)(ok ? tok : 0) * C + 4 * g;
  f4 y[kPatchCmax / 16];
#pragma unroll
  for (int s = 0; s < kPatchCmax / 16; ++s) {
    f4 v = {0.f, 0.f, 0.f, 0.f};
    if (16 * s + 4 * g < C) v = *reinterpret_cast<const f4*>(yr + 16 * s);
    y[s] = v;
  }
  // rows 4 g + r of output tile mt: channel o = 4 mt + g, p = r / 2, q = r % 2
  size_t off[NMT];
  bool st[NMT];
  float2 ex[NMT][2];
#pragma unroll
  for (int mt = 0; mt < NMT; ++mt) {
    const int o = 4 * mt + g;
    const int oc = min(o, kc / 4 - 1);
    const int ch = MODE == 0 ? G.cin_off + oc : unembed_ch(G, oc);
    st[mt] = ok && mt < nmt && o * 4 < kc && (MODE == 0 || ch < a.climit);
    off[mt] = (((size_t)b * a.Cimg + ch) * a.Himg + 2 * ho) * a.Wimg + 2 * wo;
    if (MODE == 0) {
#pragma unroll
      for (int pp = 0; pp < 2; ++pp)
        ex[mt][pp] = (a.add_img && st[mt]) ? *reinterpret_cast<const float2*>(a.add_img + off[mt] + pp * a.Wimg)
                                          : make_float2(0.f, 0.f);
    } else {
      const float bias = G.bias[oc];
      ex[mt][0] = ex[mt][1] = make_float2(bias, bias);
    }
  }
  {
    // coalesced over W's rows, transposed into LDS, in batches of 16 loads
    constexpr int NW = kPatchCmax * KPM / 256, NB = NW < 16 ? NW : 16;
#pragma unroll
    for (int h = 0; h < NW; h += NB) {
      float v[NB];
#pragma unroll
      for (int r = 0; r < NB; ++r) {
        const int i = threadIdx.x + 256 * (h + r), c = i / KP, j = i - c * KP;
        v[r] = (c < C && j < kc) ? G.w[(size_t)c * kc + j] : 0.f;
      }
#pragma unroll
      for (int r = 0; r < NB; ++r) {
        const int i = threadIdx.x + 256 * (h + r), c = i / KP, j = i - c * KP;
        if (c < CP) Wt[j * CS + c] = v[r];
      }
    }
  }
  __syncthreads();
  typedef float fr4 __attribute__((ext_vector_type(4)));
  fr4 acc[NMT];
#pragma unroll
  for (int mt = 0; mt < NMT; ++mt) {
    acc[mt] = fr4{0.f, 0.f, 0.f, 0.f};
    if (mt < nmt) {
      const float* wr = Wt + (mt * 16 + li) * CS + 4 * g;
#pragma unroll
      for (int s = 0; s < kPatchCmax / 16; ++s) {
        if (16 * s < CP) {
          const f4 wa = *reinterpret_cast<const f4*>(wr + 16 * s);
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[e], y[s][e], acc[mt], 0, 0, 0);
        }
      }
    }
  }
  // two float2 stores per tile: consecutive lanes = consecutive tokens = horizontally adjacent pixel pairs
#pragma unroll
  for (int mt = 0; mt < NMT; ++mt) {
    if (!st[mt]) continue;
#pragma unroll
    for (int pp = 0; pp < 2; ++pp)
      *reinterpret_cast<float2*>(a.img_out + off[mt] + pp * a.Wimg) =
          make_float2(acc[mt][2 * pp] + ex[mt][pp].x, acc[mt][2 * pp + 1] + ex[mt][pp].y);
  }
}

// Persistent forms (r06). The r05 kernels above stage the weights per 64-token workgroup (57 KB from L2 for every 64
// tokens at 112 taps), run their loads, MFMAs and stores in lockstep per workgroup, and chain each accumulator's
// MFMAs back to back (40-cycle dependent latency against a 32-cycle issue). Here a workgroup of 8 waves per CU share
// of a group stages its group's weights once; each wave walks its own 16-token tiles (a contiguous range of the
// group's tiles per workgroup), prefetching the next tile's operands into registers behind the current tile's MFMAs,
// and interleaves its accumulators (k step outer, output tile inner). Per output element the MFMA sequence -- k in
// steps of 4, ascending -- is the r05 kernels', so both forms give bit-identical results.
constexpr int kPmWaves = 8;

// the 16-token tiles [r0, r1) of workgroup j of P over a group's nwt tiles
__device__ __forceinline__ void pm_range(int nwt, int& r0, int& r1) {
  r0 = (int)((long long)blockIdx.x * nwt / gridDim.x);
  r1 = (int)((long long)(blockIdx.x + 1) * nwt / gridDim.x);
}

// CT: the token width at compile time (96 -- the decoder's enc_dim -- and 128 are instantiated; 0 = any width up to
// kPatchCmax, zero-padded to it, with the row loads and stores under a runtime bound). With CT the MFMA tiles are the
// width's own (no zero tiles) and the loads are branch-free (clamped address, then a select), the prefetch
// unconditional (the last tile again past the range): a load or store under a branch leaves the compiler unable to
// count vmcnt, and it then waits for every one of them, this tile's stores included, before the next tile's rows
template <int MODE, int KPM, int CT>
__global__ __launch_bounds__(512) void k_p2t_mp(PatchArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const PatchGroup G = a.g[blockIdx.y];
  const int Ho = a.Himg / 2, Wo = a.Wimg / 2, ntok = a.B * Ho * Wo;
  constexpr int CM = CT ? CT : kPatchCmax;  // channels the MFMA tiles cover
  const int kc = MODE == 0 ? G.cin * 4 : G.cout * 4, C = CT ? CT : a.Ctok;
  // compile-time shapes (zero-padded to KPM taps and CM channels): MFMAs under runtime conditions made the compiler
  // keep every accumulator live across branches (thousands of VGPRs spilled)
  constexpr int KS = KPM + 4;                       // weight row stride (floats)
  constexpr int RS = KS > CM + 4 ? KS : CM + 4;     // the wave's rows: operands, then the staging
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
  float* Wsm = sm;                             // [CM][KS]
  float* R = sm + CM * KS + wave * 16 * RS;   // [16][RS], this wave's only
  int r0, r1;
  pm_range(ntok / 16, r0, r1);
  constexpr int NC = KPM / 4;  // channel rows per lane: lane (pp = lane / 32, col = lane % 32) of the tile's
                               // 32-pixel-wide, 2-row image strip, one channel per load
  constexpr int NO = CM / 16, NTM = CM / 16;
  const int col = lane & 31, pp = lane >> 5;
  const size_t plane = (size_t)a.Himg * a.Wimg;
  float xv[NC];
  f4 pv[NO];
  auto load_tile = [&](int wt) {
    int b, ho, wo;
    tok_coords(wt * 16, Ho, Wo, b, ho, wo);
    const float* base = a.img + (size_t)b * a.Cimg * plane + (size_t)(2 * ho + pp) * a.Wimg + 2 * wo + col;
#pragma unroll
    for (int ci = 0; ci < NC; ++ci) {
      const int ch = MODE == 0 ? G.cin_off + min(ci, kc / 4 - 1) : unembed_ch(G, min(ci, kc / 4 - 1));
      const bool ok = ci * 4 < kc && (MODE == 0 || ch < a.climit);
      const float v = base[(size_t)(ok ? ch : 0) * plane];
      xv[ci] = ok ? v : 0.f;
    }
    if (MODE == 0) {
      const size_t pbase = (size_t)((wt * 16) % (Ho * Wo)) * C;
#pragma unroll
      for (int i = 0; i < NO; ++i) {
        const f4 v = *reinterpret_cast<const f4*>(G.pos + pbase + 4 * ((CT ? i : min(i, C / 16 - 1)) * 64 + lane));
        pv[i] = CT || i < C / 16 ? v : f4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };
  int wt = r0 + wave;
  load_tile(min(wt, r1 - 1));  // (r1 > r0: the grid has at most one workgroup per 8 tiles)
  float bv[NTM];
#pragma unroll
  for (int n = 0; n < NTM; ++n) bv[n] = MODE == 0 ? G.bias[min(n * 16 + li, C - 1)] : 0.f;
  {
    constexpr int NW = CM * KPM / 512, NB = NW < 16 ? NW : 16;
#pragma unroll
    for (int h = 0; h < NW; h += NB) {
      float wv[NB];
#pragma unroll
      for (int r = 0; r < NB; ++r) {
        const int i = threadIdx.x + 512 * (h + r), c = i / KPM, j = i - c * KPM;
        wv[r] = (c < C && j < kc) ? G.w[(size_t)c * kc + j] : 0.f;
      }
#pragma unroll
      for (int r = 0; r < NB; ++r) {
        const int i = threadIdx.x + 512 * (h + r), c = i / KPM, j = i - c * KPM;
        if (h + r < NW) Wsm[c * KS + j] = wv[r];  // NW need not be a multiple of NB (28 at 112 taps)
      }
    }
  }
  __syncthreads();
  typedef float fr4 __attribute__((ext_vector_type(4)));
  for (; wt < r1; wt += kPmWaves) {
    // this tile's operand rows (zeros at the padded taps); the previous tile's staging is read back already
#pragma unroll
    for (int ci = 0; ci < NC; ++ci) R[(col >> 1) * RS + ci * 4 + pp * 2 + (col & 1)] = xv[ci];
    f4 pc[NO];
#pragma unroll
    for (int i = 0; i < NO; ++i) pc[i] = pv[i];
    load_tile(min(wt + kPmWaves, r1 - 1));  // in flight behind this tile's MFMAs
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    fr4 acc[NTM];
#pragma unroll
    for (int n = 0; n < NTM; ++n) acc[n] = fr4{0.f, 0.f, 0.f, 0.f};
    const float* xr = R + li * RS + 4 * g;
#pragma unroll
    for (int s4 = 0; s4 < KPM; s4 += 16) {
      const f4 xa = *reinterpret_cast<const f4*>(xr + s4);
      f4 wb[NTM];
#pragma unroll
      for (int n = 0; n < NTM; ++n) wb[n] = *reinterpret_cast<const f4*>(Wsm + (n * 16 + li) * KS + 4 * g + s4);
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int n = 0; n < NTM; ++n) acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[e], wb[n][e], acc[n], 0, 0, 0);
    }
    // (D + bias) over the operand rows (every lane's reads of them are issued: same-wave LDS order), then whole-row
    // float4 stores of the tile's contiguous [16][C] block (+ pos)
#pragma unroll
    for (int n = 0; n < NTM; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) R[(4 * g + r) * RS + n * 16 + li] = MODE == 0 ? acc[n][r] + bv[n] : acc[n][r];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    float* out = G.tok + (size_t)wt * 16 * C;
#pragma unroll
    for (int i = 0; i < NO; ++i) {
      if (!CT && i >= C / 16) break;
      const int e = 4 * (i * 64 + lane), row = e / C, cc = e - row * C;
      f4 v = *reinterpret_cast<const f4*>(R + row * RS + cc);
      if (MODE == 0) v = v + pc[i];
      *reinterpret_cast<f4*>(out + e) = v;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // staging reads done before the next operand rows overlay them
    __builtin_amdgcn_wave_barrier();
  }
}

// CT, branch-free loads and the unconditional prefetch: as k_p2t_mp
template <int MODE, int KPM, int CT>
__global__ __launch_bounds__(512) void k_t2p_mp(PatchArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const PatchGroup G = a.g[blockIdx.y];
  const int Ho = a.Himg / 2, Wo = a.Wimg / 2, ntok = a.B * Ho * Wo;
  constexpr int CM = CT ? CT : kPatchCmax;
  const int kc = MODE == 0 ? G.cin * 4 : G.cout * 4, C = CT ? CT : a.Ctok;
  constexpr int CS = CM + 4;
  float* Wt = sm;  // [KPM][CS]: W[c][j] at Wt[j][c], zero-padded (compile-time MFMA shapes, as k_p2t_mp)
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
  int r0, r1;
  pm_range(ntok / 16, r0, r1);
  constexpr int NMT = KPM / 16, NS = CM / 16;
  f4 y[NS];
  float2 ex[NMT][2];
  // lane (token li, g): the token row's float4 at 16 s + 4 g, and what its outputs add (the added image, the bias)
  auto load_tile = [&](int wt) {
    const int tok = wt * 16 + li;
    const float* yr = (MODE == 0 ? G.dtok : G.tok) + (size_t)tok * C + 4 * g;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (CT) {
        y[s] = *reinterpret_cast<const f4*>(yr + 16 * s);
      } else {
        y[s] = 16 * s < C ? *reinterpret_cast<const f4*>(yr + 16 * s) : f4{0.f, 0.f, 0.f, 0.f};
      }
    }
    if (MODE == 0 && a.add_img) {
      int b, ho, wo;
      tok_coords(tok, Ho, Wo, b, ho, wo);
#pragma unroll
      for (int mt = 0; mt < NMT; ++mt) {
        const int o = 4 * mt + g;
        const size_t off = (((size_t)b * a.Cimg + G.cin_off + min(o, kc / 4 - 1)) * a.Himg + 2 * ho) * a.Wimg + 2 * wo;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const float2 v = *reinterpret_cast<const float2*>(a.add_img + off + q * a.Wimg);
          ex[mt][q] = o * 4 < kc ? v : make_float2(0.f, 0.f);
        }
      }
    }
  };
  int wt = r0 + wave;
  float bz[NMT];  // MODE 1: the bias of output channel 4 mt + g
#pragma unroll
  for (int mt = 0; mt < NMT; ++mt) {
    bz[mt] = MODE == 1 ? G.bias[min(4 * mt + g, kc / 4 - 1)] : 0.f;
    if (MODE == 1 || !a.add_img) ex[mt][0] = ex[mt][1] = make_float2(0.f, 0.f);
  }
  load_tile(min(wt, r1 - 1));
  {
    constexpr int NW = CM * KPM / 512, NB = NW < 16 ? NW : 16;
#pragma unroll
    for (int h = 0; h < NW; h += NB) {
      float v[NB];
#pragma unroll
      for (int r = 0; r < NB; ++r) {
        const int i = threadIdx.x + 512 * (h + r), c = i / KPM, j = i - c * KPM;
        v[r] = (c < C && j < kc) ? G.w[(size_t)c * kc + j] : 0.f;
      }
#pragma unroll
      for (int r = 0; r < NB; ++r) {
        const int i = threadIdx.x + 512 * (h + r), c = i / KPM, j = i - c * KPM;
        if (h + r < NW) Wt[j * CS + c] = v[r];  // NW need not be a multiple of NB (28 at 112 taps)
      }
    }
  }
  __syncthreads();
  typedef float fr4 __attribute__((ext_vector_type(4)));
  for (; wt < r1; wt += kPmWaves) {
    f4 yc[NS];
    float2 xc[NMT][2];
#pragma unroll
    for (int s = 0; s < NS; ++s) yc[s] = y[s];
#pragma unroll
    for (int mt = 0; mt < NMT; ++mt)
      if (MODE == 0) xc[mt][0] = ex[mt][0], xc[mt][1] = ex[mt][1];
    load_tile(min(wt + kPmWaves, r1 - 1));  // in flight behind this tile's MFMAs
    fr4 acc[NMT];
#pragma unroll
    for (int mt = 0; mt < NMT; ++mt) acc[mt] = fr4{0.f, 0.f, 0.f, 0.f};
    // W^T fragments one k step ahead (double-buffered): left to itself the scheduler hoisted every step's LDS reads
    // and spilled
    const float* wr = Wt + li * CS + 4 * g;
    f4 wa[2][NMT];
#pragma unroll
    for (int mt = 0; mt < NMT; ++mt) wa[0][mt] = *reinterpret_cast<const f4*>(wr + mt * 16 * CS);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (s + 1 < NS)
#pragma unroll
        for (int mt = 0; mt < NMT; ++mt)
          wa[(s + 1) & 1][mt] = *reinterpret_cast<const f4*>(wr + mt * 16 * CS + 16 * (s + 1));
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int mt = 0; mt < NMT; ++mt)
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[s & 1][mt][e], yc[s][e], acc[mt], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    int b, ho, wo;
    tok_coords(wt * 16 + li, Ho, Wo, b, ho, wo);
#pragma unroll
    for (int mt = 0; mt < NMT; ++mt) {
      const int o = 4 * mt + g;
      if (o * 4 >= kc) continue;
      const int ch = MODE == 0 ? G.cin_off + o : unembed_ch(G, o);
      if (MODE == 1 && ch >= a.climit) continue;
      float* dst = a.img_out + (((size_t)b * a.Cimg + ch) * a.Himg + 2 * ho) * a.Wimg + 2 * wo;
#pragma unroll
      for (int q = 0; q < 2; ++q)
        *reinterpret_cast<float2*>(dst + q * a.Wimg) =
            MODE == 0 ? make_float2(acc[mt][2 * q] + xc[mt][q].x, acc[mt][2 * q + 1] + xc[mt][q].y)
                      : make_float2(acc[mt][2 * q] + bz[mt], acc[mt][2 * q + 1] + bz[mt]);
    }
  }
}

// persistent grid: P workgroups per group, `per_cu` resident per CU, at most one per 8 of the group's 16-token tiles
static int pm_grid(const PatchArgs& a, int per_cu) {
  const int nwt = a.B * (a.Himg / 2) * (a.Wimg / 2) / 16;
  return std::max(1, std::min((nwt + kPmWaves - 1) / kPmWaves, device_cus() * per_cu / a.ngroups));
}

template <int MODE, int KPM, int CT>
static hipError_t p2t_mp_launch(const PatchArgs& a, hipStream_t s) {
  constexpr int CM = CT ? CT : kPatchCmax;
  constexpr size_t lds = ((size_t)CM * (KPM + 4) + (size_t)kPmWaves * 16 * std::max(KPM + 4, CM + 4)) * sizeof(float);
  if (hipError_t e = set_lds_limit((const void*)k_p2t_mp<MODE, KPM, CT>, lds)) return e;
  hipLaunchKernelGGL((k_p2t_mp<MODE, KPM, CT>), dim3(pm_grid(a, 1), a.ngroups), dim3(64 * kPmWaves), lds, s, a);
  return hipGetLastError();
}

template <int MODE, int KPM, int CT>
static hipError_t t2p_mp_launch(const PatchArgs& a, hipStream_t s) {
  constexpr size_t lds = (size_t)KPM * ((CT ? CT : kPatchCmax) + 4) * sizeof(float);
  if (lds > 64 * 1024)
    if (hipError_t e = set_lds_limit((const void*)k_t2p_mp<MODE, KPM, CT>, lds)) return e;
  hipLaunchKernelGGL((k_t2p_mp<MODE, KPM, CT>), dim3(pm_grid(a, 1), a.ngroups), dim3(64 * kPmWaves), lds, s, a);
  return hipGetLastError();
}

static int max_k(const PatchArgs& a, bool in) {
  int m = 0;
  for (int g = 0; g < a.ngroups; ++g) m = std::max(m, (in ? a.g[g].cin : a.g[g].cout) * 4);
  return m;
}

template <int MODE, int KPM>
static hipError_t p2t_launch_k(const PatchArgs& a, int kc, hipStream_t s) {
  const int ntok = a.B * (a.Himg / 2) * (a.Wimg / 2);
  if ((a.tune ? a.tune->patch_pers : kDefaultTuning.patch_pers) > 0) {
    return a.Ctok == 96 ? p2t_mp_launch<MODE, KPM, 96>(a, s) : a.Ctok == 128 ? p2t_mp_launch<MODE, KPM, 128>(a, s)
                                                                           : p2t_mp_launch<MODE, KPM, 0>(a, s);
  }
  const int KS = (kc + 15) / 16 * 16 + 4;
  const size_t lds = std::max((size_t)(PT + a.Ctok) * KS, (size_t)PT * (a.Ctok + 4)) * sizeof(float);
  if (lds > 64 * 1024)
    if (hipError_t e = set_lds_limit((const void*)k_p2t_mf<MODE, KPM>,
                                     std::max((size_t)(PT + kPatchCmax) * (KPM + 4), (size_t)PT * (kPatchCmax + 4)) * 4))
      return e;
  hipLaunchKernelGGL((k_p2t_mf<MODE, KPM>), dim3((ntok + PT - 1) / PT, a.ngroups), dim3(256), lds, s, a);
  return hipGetLastError();
}
// the instantiation whose padded K (32, 64 or 112 taps) covers kc: registers scale with it
template <int MODE>
static hipError_t p2t_launch(const PatchArgs& a, int kc, hipStream_t s) {
  return kc <= 32 ? p2t_launch_k<MODE, 32>(a, kc, s) : kc <= 64 ? p2t_launch_k<MODE, 64>(a, kc, s)
                                                                 : p2t_launch_k<MODE, kPatchKmax>(a, kc, s);
}

template <int MODE, int KPM>
static hipError_t t2p_launch_k(const PatchArgs& a, int kc, hipStream_t s) {
  const int ntok = a.B * (a.Himg / 2) * (a.Wimg / 2);
  const size_t lds = (size_t)((kc + 15) / 16 * 16) * ((a.Ctok + 15) / 16 * 16 + 4) * sizeof(float);
  if ((a.tune ? a.tune->patch_pers : kDefaultTuning.patch_pers) > 0) {
    return a.Ctok == 96 ? t2p_mp_launch<MODE, KPM, 96>(a, s) : a.Ctok == 128 ? t2p_mp_launch<MODE, KPM, 128>(a, s)
                                                                           : t2p_mp_launch<MODE, KPM, 0>(a, s);
  }
  hipLaunchKernelGGL((k_t2p_mf<MODE, KPM>), dim3((ntok + PT - 1) / PT, a.ngroups), dim3(256), lds, s, a);
  return hipGetLastError();
}
template <int MODE>
static hipError_t t2p_launch(const PatchArgs& a, int kc, hipStream_t s) {
  return kc <= 32 ? t2p_launch_k<MODE, 32>(a, kc, s) : kc <= 64 ? t2p_launch_k<MODE, 64>(a, kc, s)
                                                                 : t2p_launch_k<MODE, kPatchKmax>(a, kc, s);
}

// preconditions: 2x2 patches, 16 tokens of a wave in one image row (Wo % 16), at most kPatchKmax taps per token and
// kPatchCmax token channels, a multiple of 16 (LDS: <= 64 KB); parse_cfg refuses configs outside them
static hipError_t patch_check(const PatchArgs& a, int kc) {
  if (a.ngroups <= 0 || a.ngroups > kMaxGroups || (a.Himg | a.Wimg) & 1 || (a.Wimg / 2) % 16 || a.Ctok <= 0 ||
      a.Ctok > kPatchCmax || a.Ctok % 16 || kc <= 0 || kc > kPatchKmax)
    return hipErrorInvalidValue;
  return hipSuccess;
}

hipError_t patch_embed_fwd(const PatchArgs& a, hipStream_t s) {
  const int kc = max_k(a, true);
  if (hipError_t e = patch_check(a, kc)) return e;
  const int ph = prof_begin(s);
  const hipError_t e = p2t_launch<0>(a, kc, s);
  prof_end(ph, s, PC_PATCH, 0.0, 0.0);
  return e;
}
hipError_t patch_embed_bwd(const PatchArgs& a, hipStream_t s) {
  const int kc = max_k(a, true);
  if (hipError_t e = patch_check(a, kc)) return e;
  const int ph = prof_begin(s);
  const hipError_t e = t2p_launch<0>(a, kc, s);
  prof_end(ph, s, PC_PATCH, 0.0, 0.0);
  return e;
}
hipError_t patch_unembed_fwd(const PatchArgs& a, hipStream_t s) {
  const int kc = max_k(a, false);
  if (hipError_t e = patch_check(a, kc)) return e;
  const int ph = prof_begin(s);
  const hipError_t e = t2p_launch<1>(a, kc, s);
  prof_end(ph, s, PC_PATCH, 0.0, 0.0);
  return e;
}
hipError_t patch_unembed_bwd(const PatchArgs& a, hipStream_t s) {
  const int kc = max_k(a, false);
  if (hipError_t e = patch_check(a, kc)) return e;
  const int ph = prof_begin(s);
  const hipError_t e = p2t_launch<1>(a, kc, s);
  prof_end(ph, s, PC_PATCH, 0.0, 0.0);
  return e;
}

// ============================================================================
// Misfit  J_o = 1/2 sum H (x - yo)^2 / R   (da_4dvar.py:1207) and its adjoint
// ============================================================================
template <typename T>
__device__ __forceinline__ T block_sum(T v, T* red) {
  v = lane_sum<64>(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[w] = v;
  __syncthreads();
  T t = 0;
  if (threadIdx.x == 0) {
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
  }
  return t;
}

// V4 (r05): same-grid states (no maps) with HW % 4 == 0 and 16-B aligned fields, four consecutive elements per thread
// and float4 accesses (the per-element arithmetic unchanged; the J partial sums its terms in a different order)
template <bool V4>
__global__ __launch_bounds__(256) void k_misfit_fwd(MisfitArgs a) {
  __shared__ double red[4];
  const int HW = a.Hs * a.Ws;
  const int n = a.C * HW;
  const int HWl = a.Hl * a.Wl;
  double acc = 0.0;
  if (V4) {
    for (int id = 4 * (blockIdx.x * 256 + threadIdx.x); id < n; id += gridDim.x * 1024) {
      const int c = id / HW;
      const int p = id - c * HW;
      const f4 nv = *reinterpret_cast<const f4*>(a.net + (size_t)c * HWl + p);
      const float s1 = a.scale[c], s2 = a.scale2 ? a.scale2[c] : 1.f, of = a.offset ? a.offset[c] : 0.f;
      const f4 xb = a.xb ? *reinterpret_cast<const f4*>(a.xb + id) : f4{0.f, 0.f, 0.f, 0.f};
      f4 yo, hm, rr;
      if (a.Hm) {
        yo = *reinterpret_cast<const f4*>(a.yo + id);
        hm = *reinterpret_cast<const f4*>(a.Hm + id);
        rr = *reinterpret_cast<const f4*>(a.R + id);
      }
      f4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float t = nv[e] * s1;
        if (a.scale2) t = t * s2;
        if (a.xb) t = t + xb[e];
        if (a.offset) t = t + of;
        v[e] = t;
      }
      *reinterpret_cast<f4*>(a.x_out + id) = v;
      if (a.flow_in) {
        const float mu = a.mean[c], sd = a.std_[c];
        f4 fi;
#pragma unroll
        for (int e = 0; e < 4; ++e) fi[e] = (v[e] - mu) / sd;
        *reinterpret_cast<f4*>(a.flow_in + id) = fi;
      }
      if (a.Hm) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = v[e] - yo[e];
          acc += (double)((hm[e] * (d * d)) / rr[e]);
        }
      }
    }
    const double t = block_sum(acc, red);
    if (threadIdx.x == 0) a.partial[blockIdx.x] = t;
    return;
  }
  for (int id = blockIdx.x * 256 + threadIdx.x; id < n; id += gridDim.x * 256) {
    const int c = id / HW;
    const int p = id - c * HW;
    int q = p;  // network-grid pixel (decoder_hr / integrate up-sampling, nearest)
    if (a.mi) {
      const int i = p / a.Ws, j = p - i * a.Ws;
      q = a.mi[i] * a.Wl + a.mj[j];
    }
    float v = a.net[(size_t)c * HWl + q] * a.scale[c];
    if (a.scale2) v = v * a.scale2[c];
    if (a.xb) v = v + a.xb[id];
    if (a.offset) v = v + a.offset[c];
    a.x_out[id] = v;
    if (a.flow_in && !a.mi) a.flow_in[id] = (v - a.mean[c]) / a.std_[c];
    if (a.Hm) {
      const float d = v - a.yo[id];
      acc += (double)((a.Hm[id] * (d * d)) / a.R[id]);
    }
  }
  const double t = block_sum(acc, red);
  if (threadIdx.x == 0) a.partial[blockIdx.x] = t;
}

template <bool V4>
__global__ __launch_bounds__(256) void k_misfit_bwd(MisfitBwdArgs a) {
  const int HW = a.Hs * a.Ws;
  const int n = a.C * HW;
  if (V4) {  // as k_misfit_fwd<true>: four consecutive elements per thread, float4 accesses, same arithmetic
    for (int id = 4 * (blockIdx.x * 256 + threadIdx.x); id < n; id += gridDim.x * 1024) {
      const int c = id / HW;
      f4 g;
      if (a.g_obs) {
        g = *reinterpret_cast<const f4*>(a.g_obs + id);
      } else {
        const f4 hm = *reinterpret_cast<const f4*>(a.Hm + id), x = *reinterpret_cast<const f4*>(a.x + id),
                 yo = *reinterpret_cast<const f4*>(a.yo + id), rr = *reinterpret_cast<const f4*>(a.R + id);
#pragma unroll
        for (int e = 0; e < 4; ++e) g[e] = a.coeff * ((hm[e] * (x[e] - yo[e])) / rr[e]);
      }
      if (a.g_carry) {
        const f4 gc = *reinterpret_cast<const f4*>(a.g_carry + id);
#pragma unroll
        for (int e = 0; e < 4; ++e) g[e] += gc[e];
      }
      const float sc = a.scale[c];
#pragma unroll
      for (int e = 0; e < 4; ++e) g[e] = g[e] * sc;
      *reinterpret_cast<f4*>(a.g_net + id) = g;
    }
    return;
  }
  for (int id = blockIdx.x * 256 + threadIdx.x; id < n; id += gridDim.x * 256) {
    const int c = id / HW;
    const int p = id - c * HW;
    float g = a.g_obs ? a.g_obs[id] : a.coeff * ((a.Hm[id] * (a.x[id] - a.yo[id])) / a.R[id]);
    if (a.g_carry) g += a.g_carry[id];
    a.g_net[(size_t)c * HW + p] = g * a.scale[c];
  }
}

// adjoint of the nearest up-sampling for general grids: each network pixel (a,b) sums the state rectangle
// [ri0[a], ri0[a+1]) x [rj0[b], rj0[b+1]) that maps onto it (mi/mj are monotone), deterministic order
__global__ __launch_bounds__(256) void k_misfit_bwd_gather(MisfitBwdArgs a) {
  const int HWl = a.Hl * a.Wl, HW = a.Hs * a.Ws;
  const int n = a.C * HWl;
  for (int id = blockIdx.x * 256 + threadIdx.x; id < n; id += gridDim.x * 256) {
    const int c = id / HWl;
    const int q = id - c * HWl;
    const int ra = q / a.Wl, cb = q - ra * a.Wl;
    float g = 0.f;
    for (int i = a.ri0[ra]; i < a.ri0[ra + 1]; ++i)
      for (int j = a.rj0[cb]; j < a.rj0[cb + 1]; ++j) {
        const size_t e = (size_t)c * HW + (size_t)i * a.Ws + j;
        float v = a.g_obs ? a.g_obs[e] : a.coeff * ((a.Hm[e] * (a.x[e] - a.yo[e])) / a.R[e]);
        if (a.g_carry) v += a.g_carry[e];
        g += v;
      }
    a.g_net[(size_t)c * HWl + q] = g * a.scale[c];
  }
}

// The misfit on an interpolated state grid in ONE pass over the state fields (config 5: 721x1440 state, 128x256
// networks; da_4dvar.py:1184-1207 with decoder_hr's / integrate's nearest up-sampling, nf_model/vae.py:90,
// da_4dvar.py:679). One workgroup per (channel c, network row ra) reads the preimage rows [ri0[ra], ri0[ra+1]) of
// xb / yo / H / R once, as float4 along the row (a thread owns 4 columns for every row of the band), and produces:
//  - x = net[mi[i]][mj[j]] * scale (* scale2) + xb (+ offset), stored only when x_out is set (J-only evaluations);
//  - the J partial of its band (fp64, deterministic: one partial per workgroup);
//  - the observation gradient already reduced onto the network grid (the adjoint of the up-sampling):
//    g_net_obs[c][ra][cb] = sum over the preimage rectangle of coeff * H (x - yo) / R — column sums over the band in
//    registers, then the columns [rj0[cb], rj0[cb+1]) summed from LDS;
//  - the next flow step's input (integrate's down-sampling, da_4dvar.py:671) at the pixels it samples.
// The backward pass then never reads a state field again (k_misfit_net_bwd runs on the network grid).
template <int MR, bool XB>
__global__ __launch_bounds__(384) void k_misfit_grid(MisfitArgs a) {
  extern __shared__ float colsum[];  // [Ws]
  __shared__ double red[6];
  const int c = blockIdx.x / a.Hl, ra = blockIdx.x - c * a.Hl;
  const int r0 = a.ri0[ra], r1 = a.ri0[ra + 1];
  const int W4 = a.Ws >> 2, HWl = a.Hl * a.Wl;
  const float sc = a.scale[c];
  const float sc2 = a.scale2 ? a.scale2[c] : 1.f;
  const float off = a.offset ? a.offset[c] : 0.f;
  const float mean = a.flow_in ? a.mean[c] : 0.f, sd = a.flow_in ? a.std_[c] : 1.f;
  // every row i of the band up-samples from network row ra (mi[i] == ra by the definition of ri0), so the network
  // values of a column are the same for the whole band: one gather per column, no per-row map lookup (a per-row
  // mi[i] load put a dependent wait between the rows' field loads)
  const float* __restrict__ nrow = a.net + (size_t)c * HWl + (size_t)ra * a.Wl;
  // the column ranges of the final reduction, loaded up front (after the barrier they would be one more round trip)
  int cb0[2], cb1[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int cb = min((int)threadIdx.x + u * (int)blockDim.x, a.Wl - 1);
    cb0[u] = a.rj0[cb];
    cb1[u] = a.rj0[cb + 1];
  }
  double acc = 0.0;
  for (int j4 = threadIdx.x; j4 < W4; j4 += blockDim.x) {
    const int j = 4 * j4;
    const int4 q = *reinterpret_cast<const int4*>(a.mj + j);
    // the flow-input sampling maps of this thread's columns (loaded with the others, not under a store)
    const int4 fcv = a.flow_in ? *reinterpret_cast<const int4*>(a.colinv + j) : make_int4(-1, -1, -1, -1);
    const int fcs[4] = {fcv.x, fcv.y, fcv.z, fcv.w};
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    for (int i0 = r0; i0 < r1; i0 += MR) {
      int frs[MR];
#pragma unroll
      for (int k = 0; k < MR; ++k) frs[k] = a.flow_in ? a.rowinv[min(i0 + k, r1 - 1)] : -1;
      // the band's field loads (streamed once: nontemporal), then the column's network values (they wait for mj
      // only, the oldest load)
      f4 xv[MR], yv[MR], hv[MR], rv[MR];
#pragma unroll
      for (int k = 0; k < MR; ++k) {
        const int i = min(i0 + k, r1 - 1);
        const size_t e = ((size_t)c * a.Hs + i) * a.Ws + j;
        if (XB) xv[k] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(a.xb + e));
        yv[k] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(a.yo + e));
        hv[k] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(a.Hm + e));
        rv[k] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(a.R + e));
      }
      const float nn[4] = {nrow[q.x], nrow[q.y], nrow[q.z], nrow[q.w]};
      float base[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float t = nn[u] * sc;
        if (a.scale2) t = t * sc2;
        base[u] = t;
      }
#pragma unroll
      for (int k = 0; k < MR; ++k) {
        const int i = i0 + k;
        if (i >= r1) break;
        float v[4], g[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          // x as k_misfit_fwd forms it (bit-identical x_t); the misfit multiplies by one reciprocal of R where
          // k_misfit_fwd divides twice, so J_o and the gradient agree with the per-element path at fp32 level only
          float t = base[u];
          if (XB) t = t + xv[k][u];
          if (a.offset) t = t + off;
          v[u] = t;
          const float d = t - yv[k][u];
          const float ri = 1.0f / rv[k][u];
          acc += (double)((hv[k][u] * (d * d)) * ri);
          g[u] = a.coeff * ((hv[k][u] * d) * ri);
        }
        s0 += g[0];
        s1 += g[1];
        s2 += g[2];
        s3 += g[3];
        const size_t e = ((size_t)c * a.Hs + i) * a.Ws + j;
        if (a.x_out) *reinterpret_cast<f4*>(a.x_out + e) = f4{v[0], v[1], v[2], v[3]};
        if (frs[k] >= 0) {
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (fcs[u] >= 0) a.flow_in[(size_t)c * HWl + (size_t)frs[k] * a.Wl + fcs[u]] = (v[u] - mean) / sd;
        }
      }
    }
    *reinterpret_cast<f4*>(colsum + j) = f4{s0, s1, s2, s3};
  }
  // J partial of the band
  acc = lane_sum<64>(acc);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[w] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) t += red[k];
    a.partial[blockIdx.x] = t;
  }
  if (!a.g_net_obs) return;
  // the up-sampling adjoint along the row: network column cb sums its preimage columns
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int cb = threadIdx.x + u * blockDim.x;
    if (cb >= a.Wl) break;
    float g = 0.f;
    for (int j = cb0[u]; j < cb1[u]; ++j) g += colsum[j];
    a.g_net_obs[(size_t)c * HWl + (size_t)ra * a.Wl + cb] = g;
  }
}

__global__ __launch_bounds__(256) void k_misfit_net_bwd(MisfitNetBwdArgs a) {
  const int HWl = a.Hl * a.Wl;
  const int n = a.C * HWl;
  for (int id = blockIdx.x * 256 + threadIdx.x; id < n; id += gridDim.x * 256) {
    const int c = id / HWl, q = id - c * HWl;
    float g = a.g_net_obs[id];
    if (a.gfi) {
      // the flow-input adjoint (integrate's down-sampling, k_flow_input_adj's gfi / std) followed by the up-sampling
      // adjoint, composed on the network grid
      const int ra = q / a.Wl, cb = q - ra * a.Wl;
      const float sd = a.std_[c];
      float s = 0.f;
      for (int r = a.cr0[ra]; r < a.cr0[ra + 1]; ++r)
        for (int k = a.cc0[cb]; k < a.cc0[cb + 1]; ++k) s += a.gfi[(size_t)c * HWl + (size_t)r * a.Wl + k] / sd;
      g += s;
    }
    a.g_net[id] = g * a.scale[c];
  }
}

__global__ __launch_bounds__(256) void k_flow_input(const float* x, float* fi, const int* di, const int* dj,
                                                    const float* mean, const float* std_, int C, int Hs, int Ws,
                                                    int Hl, int Wl) {
  const int HWl = Hl * Wl;
  const int n = C * HWl;
  for (int id = blockIdx.x * 256 + threadIdx.x; id < n; id += gridDim.x * 256) {
    const int c = id / HWl, q = id - c * HWl;
    const int ra = q / Wl, cb = q - ra * Wl;
    fi[id] = (x[((size_t)c * Hs + di[ra]) * Ws + dj[cb]] - mean[c]) / std_[c];
  }
}

__global__ __launch_bounds__(256) void k_zero(float* __restrict__ p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) p[i] = 0.f;
}

__global__ __launch_bounds__(256) void k_flow_input_adj(const float* gfi, float* carry, const int* di, const int* dj,
                                                        const float* std_, int C, int Hs, int Ws, int Hl, int Wl) {
  const int HWl = Hl * Wl;
  const int n = C * HWl;
  for (int id = blockIdx.x * 256 + threadIdx.x; id < n; id += gridDim.x * 256) {
    const int c = id / HWl, q = id - c * HWl;
    const int ra = q / Wl, cb = q - ra * Wl;
    // di/dj are injective when down-sampling (Hs >= Hl), so every target is written at most once
    carry[((size_t)c * Hs + di[ra]) * Ws + dj[cb]] = gfi[id] / std_[c];
  }
}

hipError_t flow_input(const float* x, float* fi, const int* di, const int* dj, const float* mean, const float* std_,
                      int C, int Hs, int Ws, int Hl, int Wl, hipStream_t s) {
  const int ph = prof_begin(s);
  hipLaunchKernelGGL(k_flow_input, dim3(1024), dim3(256), 0, s, x, fi, di, dj, mean, std_, C, Hs, Ws, Hl, Wl);
  prof_end(ph, s, PC_MISFIT, 2.0 * C * Hl * Wl, 8.0 * C * Hl * Wl);
  return hipGetLastError();
}

hipError_t flow_input_adjoint(const float* gfi, float* carry, const int* di, const int* dj, const float* std_, int C,
                              int Hs, int Ws, int Hl, int Wl, hipStream_t s) {
  if (Hs < Hl || Ws < Wl) return hipErrorNotSupported;
  // zero the whole carry with a kernel, not hipMemsetAsync: a memset node captured into the closure's hipGraph was
  // not ordered before the scatter below on replay (config 5's wrong gradients in r01)
  const int ph = prof_begin(s);
  const size_t n = (size_t)C * Hs * Ws;
  hipLaunchKernelGGL(k_zero, dim3((unsigned)std::min<size_t>((n + 255) / 256, 4096)), dim3(256), 0, s, carry, n);
  hipLaunchKernelGGL(k_flow_input_adj, dim3(1024), dim3(256), 0, s, gfi, carry, di, dj, std_, C, Hs, Ws, Hl, Wl);
  prof_end(ph, s, PC_MISFIT, 1.0 * C * Hl * Wl, 8.0 * C * Hl * Wl);
  return hipGetLastError();
}

// F.interpolate(mode='nearest') of (BC, Hi, Wi) fields to (Ho, Wo) with the source maps mi[Ho], mj[Wo] (quirk Q3),
// and its adjoint: gin[i][j] = sum of gout over the rows y in [ri0[i], ri0[i+1]) and columns x in [rj0[j], rj0[j+1])
// (the maps are monotone, so every preimage is a contiguous range; a deterministic gather, no atomics)
__global__ __launch_bounds__(256) void k_resample(const float* __restrict__ in, float* __restrict__ out,
                                                  const int* __restrict__ mi, const int* __restrict__ mj, int BC,
                                                  int Hi, int Wi, int Ho, int Wo) {
  const size_t n = (size_t)BC * Ho * Wo;
  for (size_t id = (size_t)blockIdx.x * 256 + threadIdx.x; id < n; id += (size_t)gridDim.x * 256) {
    const size_t c = id / ((size_t)Ho * Wo);
    const int q = (int)(id - c * Ho * Wo), y = q / Wo, x = q - y * Wo;
    out[id] = in[(c * Hi + mi[y]) * Wi + mj[x]];
  }
}
__global__ __launch_bounds__(256) void k_resample_adj(const float* __restrict__ gout, float* __restrict__ gin,
                                                      const int* __restrict__ ri0, const int* __restrict__ rj0, int BC,
                                                      int Hi, int Wi, int Ho, int Wo) {
  const size_t n = (size_t)BC * Hi * Wi;
  for (size_t id = (size_t)blockIdx.x * 256 + threadIdx.x; id < n; id += (size_t)gridDim.x * 256) {
    const size_t c = id / ((size_t)Hi * Wi);
    const int q = (int)(id - c * Hi * Wi), i = q / Wi, j = q - i * Wi;
    float s = 0.f;
    for (int y = ri0[i]; y < ri0[i + 1]; ++y)
      for (int x = rj0[j]; x < rj0[j + 1]; ++x) s += gout[(c * Ho + y) * Wo + x];
    gin[id] = s;
  }
}
hipError_t resample_nearest(const float* in, float* out, const int* maps, int BC, int Hi, int Wi, int Ho, int Wo,
                            bool adjoint, hipStream_t s) {
  const size_t n = (size_t)BC * (adjoint ? (size_t)Hi * Wi : (size_t)Ho * Wo);
  const unsigned g = (unsigned)std::min<size_t>((n + 255) / 256, 8192);
  if (adjoint)
    hipLaunchKernelGGL(k_resample_adj, dim3(g), dim3(256), 0, s, in, out, maps, maps + Hi + 1, BC, Hi, Wi, Ho, Wo);
  else
    hipLaunchKernelGGL(k_resample, dim3(g), dim3(256), 0, s, in, out, maps, maps + Ho, BC, Hi, Wi, Ho, Wo);
  return hipGetLastError();
}

hipError_t misfit_fwd(const MisfitArgs& a, hipStream_t s) {
  if ((a.mi == nullptr) != (a.mj == nullptr)) return hipErrorInvalidValue;
  if (!a.mi && (a.Hs != a.Hl || a.Ws != a.Wl)) return hipErrorInvalidValue;
  const int ph = prof_begin(s);
  bool v4 = !a.mi && (a.Hs * a.Ws) % 4 == 0;
  for (const void* p : {(const void*)a.net, (const void*)a.xb, (const void*)a.yo, (const void*)a.Hm, (const void*)a.R,
                        (const void*)a.x_out, (const void*)a.flow_in})
    v4 = v4 && !(reinterpret_cast<uintptr_t>(p) & 15);
  if (v4) hipLaunchKernelGGL(k_misfit_fwd<true>, dim3(a.nblk), dim3(256), 0, s, a);
  else hipLaunchKernelGGL(k_misfit_fwd<false>, dim3(a.nblk), dim3(256), 0, s, a);
  prof_end(ph, s, PC_MISFIT, 6.0 * a.C * a.Hs * a.Ws, 4.0 * a.C * a.Hs * a.Ws * ((a.xb ? 6 : 5) + (a.flow_in ? 1 : 0)));
  return hipGetLastError();
}
hipError_t misfit_grid_fwd(const MisfitArgs& a, hipStream_t s) {
  // Wl <= 768: two network columns per thread in the final reduction (vv_bind_problem checks the same)
  if (!a.mi || !a.mj || !a.ri0 || !a.rj0 || !a.Hm || !a.yo || !a.R || (a.Ws & 3) || a.nblk != a.C * a.Hl ||
      a.Ws > 16384 || a.Wl > 2 * 384 || (a.flow_in && (!a.rowinv || !a.colinv)))
    return hipErrorInvalidValue;
  for (const void* p : {(const void*)a.xb, (const void*)a.yo, (const void*)a.Hm, (const void*)a.R,
                        (const void*)a.x_out, (const void*)a.mj, (const void*)a.colinv})
    if (reinterpret_cast<uintptr_t>(p) & 15) return hipErrorInvalidValue;
  const int ph = prof_begin(s);
  const size_t n = (size_t)a.C * a.Hs * a.Ws;
  // mr: rows of the band whose loads are in flight together (6: the whole 721 -> 128 band, 152 VGPRs, 3 waves per
  // SIMD; 3: two passes per band, 5 waves per SIMD)
  const dim3 g(a.C * a.Hl), b(384);
  const size_t l = a.Ws * sizeof(float);
  if (a.mr == 3) {
    if (a.xb) hipLaunchKernelGGL((k_misfit_grid<3, true>), g, b, l, s, a);
    else hipLaunchKernelGGL((k_misfit_grid<3, false>), g, b, l, s, a);
  } else {
    if (a.xb) hipLaunchKernelGGL((k_misfit_grid<6, true>), g, b, l, s, a);
    else hipLaunchKernelGGL((k_misfit_grid<6, false>), g, b, l, s, a);
  }
  // algorithmic bytes: the state fields once (xb, yo, H, R; x when stored)
  prof_end(ph, s, PC_MISFIT, 8.0 * n, 4.0 * n * ((a.xb ? 4 : 3) + (a.x_out ? 1 : 0)));
  return hipGetLastError();
}
hipError_t misfit_net_bwd(const MisfitNetBwdArgs& a, hipStream_t s) {
  if (!a.g_net_obs || !a.g_net || !a.scale || (a.gfi && (!a.cr0 || !a.cc0 || !a.std_))) return hipErrorInvalidValue;
  const int ph = prof_begin(s);
  const int n = a.C * a.Hl * a.Wl;
  hipLaunchKernelGGL(k_misfit_net_bwd, dim3(std::min((n + 255) / 256, 2048)), dim3(256), 0, s, a);
  prof_end(ph, s, PC_MISFIT, 2.0 * n, 4.0 * n * (a.gfi ? 3 : 2));
  return hipGetLastError();
}
hipError_t misfit_bwd(const MisfitBwdArgs& a, hipStream_t s) {
  if (!a.ri0 && (a.Hs != a.Hl || a.Ws != a.Wl)) return hipErrorInvalidValue;
  const int ph = prof_begin(s);
  if (a.ri0) {
    hipLaunchKernelGGL(k_misfit_bwd_gather, dim3(1024), dim3(256), 0, s, a);
  } else {
    bool v4 = (a.Hs * a.Ws) % 4 == 0;
    for (const void* p : {(const void*)a.g_obs, (const void*)a.Hm, (const void*)a.x, (const void*)a.yo, (const void*)a.R,
                          (const void*)a.g_carry, (const void*)a.g_net})
      v4 = v4 && !(reinterpret_cast<uintptr_t>(p) & 15);
    if (v4) hipLaunchKernelGGL(k_misfit_bwd<true>, dim3(1024), dim3(256), 0, s, a);
    else hipLaunchKernelGGL(k_misfit_bwd<false>, dim3(1024), dim3(256), 0, s, a);
  }
  prof_end(ph, s, PC_MISFIT, 5.0 * a.C * a.Hs * a.Ws, 4.0 * a.C * a.Hs * a.Ws * (a.g_carry ? 6 : 5));
  return hipGetLastError();
}

// real-observation operator: one thread per pixel holds the pixel's 13-level column of each variable in
// registers; every state and observation channel is read once, coalesced along the pixel axis. J partials in
// fp64 (deterministic block order, as k_misfit_fwd), the gradient formed in the same pass.
__global__ __launch_bounds__(256) void k_obs_misfit(ObsArgs a) {
  __shared__ float Ps[kObsMaxOut * kObsMaxIn];
  __shared__ double red[4];
  const int nin = a.nin, nout = a.nout, HW = a.HW;
  for (int i = threadIdx.x; i < nout * nin; i += 256) Ps[i] = a.P[i];
  __syncthreads();
  double acc = 0.0;
  for (int p = blockIdx.x * 256 + threadIdx.x; p < HW; p += gridDim.x * 256) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const size_t e = (size_t)c * HW + p;
      const float d = a.x[e] - a.yo[e];
      acc += (double)((a.Hm[e] * (d * d)) / a.R[e]);
      a.g_obs[e] = a.coeff * ((a.Hm[e] * d) / a.R[e]);
    }
    for (int v = 0; v < 5; ++v) {
      float xs[kObsMaxIn], gs[kObsMaxIn];
#pragma unroll
      for (int j = 0; j < kObsMaxIn; ++j) {
        xs[j] = j < nin ? a.x[(size_t)(4 + nin * v + j) * HW + p] : 0.0f;
        gs[j] = 0.0f;
      }
      for (int o = 0; o < nout; ++o) {
        const float* pr = Ps + o * nin;
        float y = 0.0f;
#pragma unroll
        for (int j = 0; j < kObsMaxIn; ++j)
          if (j < nin) y += pr[j] * xs[j];
        const size_t e = (size_t)(4 + nout * v + o) * HW + p;
        const float d = y - a.yo[e], h = a.Hm[e], r = a.R[e];
        acc += (double)((h * (d * d)) / r);
        const float g = a.coeff * ((h * d) / r);
#pragma unroll
        for (int j = 0; j < kObsMaxIn; ++j)
          if (j < nin) gs[j] += pr[j] * g;
      }
#pragma unroll
      for (int j = 0; j < kObsMaxIn; ++j)
        if (j < nin) a.g_obs[(size_t)(4 + nin * v + j) * HW + p] = gs[j];
    }
  }
  const double t = block_sum(acc, red);
  if (threadIdx.x == 0) a.partial[blockIdx.x] = t;
}

__global__ __launch_bounds__(256) void k_obs_augment(const float* P, int nin, int nout, const float* x, float* xa,
                                                     int HW) {
  __shared__ float Ps[kObsMaxOut * kObsMaxIn];
  for (int i = threadIdx.x; i < nout * nin; i += 256) Ps[i] = P[i];
  __syncthreads();
  const float* xt = x + (size_t)blockIdx.y * (4 + 5 * nin) * HW;
  float* yt = xa + (size_t)blockIdx.y * (4 + 5 * nout) * HW;
  for (int p = blockIdx.x * 256 + threadIdx.x; p < HW; p += gridDim.x * 256) {
#pragma unroll
    for (int c = 0; c < 4; ++c) yt[(size_t)c * HW + p] = xt[(size_t)c * HW + p];
    for (int v = 0; v < 5; ++v) {
      float xs[kObsMaxIn];
#pragma unroll
      for (int j = 0; j < kObsMaxIn; ++j) xs[j] = j < nin ? xt[(size_t)(4 + nin * v + j) * HW + p] : 0.0f;
      for (int o = 0; o < nout; ++o) {
        float y = 0.0f;
#pragma unroll
        for (int j = 0; j < kObsMaxIn; ++j)
          if (j < nin) y += Ps[o * nin + j] * xs[j];
        yt[(size_t)(4 + nout * v + o) * HW + p] = y;
      }
    }
  }
}

// metrics: grid (nchunk, B*C); rows of a plane split into nchunk contiguous chunks, fp64 block sums
__global__ __launch_bounds__(256) void k_metric_partial(MetricArgs a) {
  __shared__ double red[4], red1[4];
  const int bc = blockIdx.y, c = bc % a.C, HW = a.H * a.W;
  const int r0 = (int)(((long)blockIdx.x * a.H) / a.nchunk), r1 = (int)(((long)(blockIdx.x + 1) * a.H) / a.nchunk);
  const float* p = a.pred + (size_t)bc * HW;
  const float* g = a.gt + (size_t)bc * HW;
  const float m = a.mean[c], sd = a.std_[c];
  double s2 = 0.0, s1 = 0.0;
  for (int i = r0 * a.W + threadIdx.x; i < r1 * a.W; i += 256) {
    const float w = a.wlat[i / a.W];
    const float d = (p[i] - m) / sd - (g[i] - m) / sd;
    s2 += (double)(w * (d * d));
    s1 += (double)(w * d);
  }
  s2 = block_sum(s2, red);
  s1 = block_sum(s1, red1);
  if (threadIdx.x == 0) {
    a.partial[((size_t)bc * a.nchunk + blockIdx.x) * 2] = s2;
    a.partial[((size_t)bc * a.nchunk + blockIdx.x) * 2 + 1] = s1;
  }
}
__global__ __launch_bounds__(64) void k_metric_final(MetricArgs a) {
  const int c = blockIdx.x, lane = threadIdx.x;
  const double n = (double)a.H * a.W;
  double r = 0.0, b = 0.0;
  for (int bb = 0; bb < a.B; ++bb) {
    const double* q = a.partial + (size_t)(bb * a.C + c) * a.nchunk * 2;
    double s2 = 0.0, s1 = 0.0;
    for (int k = lane; k < a.nchunk; k += 64) {
      s2 += q[2 * k];
      s1 += q[2 * k + 1];
    }
    s2 = wave_sum_d(s2);
    s1 = wave_sum_d(s1);
    r += (double)sqrtf((float)(s2 / n));  // torch.sqrt(torch.mean(...)) of an fp32 tensor
    b += (double)(float)(s1 / n);
  }
  if (lane == 0) {
    a.wrmse[c] = (double)(float)(r / a.B) * a.scale[c];
    a.bias[c] = (double)(float)(b / a.B) * a.scale[c];
  }
}
hipError_t metrics(const MetricArgs& a, hipStream_t s) {
  if (a.B < 1 || a.C < 1 || a.H < 1 || a.W < 1 || a.nchunk < 1) return hipErrorInvalidValue;
  const int ph = prof_begin(s);
  hipLaunchKernelGGL(k_metric_partial, dim3(a.nchunk, a.B * a.C), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_metric_final, dim3(a.C), dim3(64), 0, s, a);
  prof_end(ph, s, PC_MISFIT, 8.0 * a.B * a.C * a.H * a.W, 8.0 * a.B * a.C * a.H * a.W);
  return hipGetLastError();
}

hipError_t obs_misfit(const ObsArgs& a, hipStream_t s) {
  if (a.nin < 1 || a.nin > kObsMaxIn || a.nout < 1 || a.nout > kObsMaxOut) return hipErrorInvalidValue;
  const int ph = prof_begin(s);
  hipLaunchKernelGGL(k_obs_misfit, dim3(a.nblk), dim3(256), 0, s, a);
  const double ca = 4.0 + 5.0 * a.nout, cs = 4.0 + 5.0 * a.nin;
  prof_end(ph, s, PC_MISFIT, (4.0 * 5 * a.nin * a.nout + 8.0 * ca) * a.HW, 4.0 * a.HW * (3 * ca + 2 * cs));
  return hipGetLastError();
}
hipError_t obs_augment(const float* P, int nin, int nout, const float* x, float* x_aug, int T, int HW,
                       hipStream_t s) {
  if (nin < 1 || nin > kObsMaxIn || nout < 1 || nout > kObsMaxOut || T < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_obs_augment, dim3(std::min((HW + 255) / 256, 2048), T), dim3(256), 0, s, P, nin, nout, x, x_aug,
                     HW);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_scale_channels(const float* in, float* out, const float* std_, int C, int HW,
                                                        const float* add) {
  const int n = C * HW;
  for (int id = blockIdx.x * 256 + threadIdx.x; id < n; id += gridDim.x * 256) {
    float v = in[id] / std_[id / HW];
    if (add) v += add[id];
    out[id] = v;
  }
}
hipError_t scale_channels(const float* in, float* out, const float* std_, int C, int HW, const float* add,
                          hipStream_t s) {
  hipLaunchKernelGGL(k_scale_channels, dim3(1024), dim3(256), 0, s, in, out, std_, C, HW, add);
  return hipGetLastError();
}

// ============================================================================
// reductions and vector primitives (torch/optim/lbfgs.py two-loop + line search, adam.py)
// ============================================================================
__global__ __launch_bounds__(256) void k_sumsq(const float* x, int64_t n, double* partial) {
  __shared__ double red[4];
  double acc = 0.0;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const double v = x[i];
    acc += v * v;
  }
  const double t = block_sum(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = t;
}
__global__ __launch_bounds__(256) void k_dot(const float* __restrict__ a, const float* __restrict__ b, int64_t n,
                                             double* partial) {
  __shared__ double red[4];
  double acc = 0.0;
#pragma unroll 4
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    acc += (double)a[i] * (double)b[i];
  const double t = block_sum(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = t;
}
__global__ __launch_bounds__(256) void k_abssum(const float* a, int64_t n, double* partial) {
  __shared__ double red[4];
  double acc = 0.0;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) acc += fabs((double)a[i]);
  const double t = block_sum(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = t;
}
__global__ __launch_bounds__(256) void k_absmax(const float* a, int64_t n, float* partial) {
  __shared__ float red[4];
  float m = 0.f;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) m = fmaxf(m, fabsf(a[i]));
  m = lane_max<64>(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}
__global__ __launch_bounds__(256) void k_final_d(const double* partial, int n, double* out) {
  __shared__ double red[4];
  double acc = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) acc += partial[i];
  const double t = block_sum(acc, red);
  if (threadIdx.x == 0) out[0] = t;
}
__global__ __launch_bounds__(256) void k_final_max(const float* partial, int n, float* out) {
  __shared__ float red[4];
  float m = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) m = fmaxf(m, partial[i]);
  m = lane_max<64>(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// k_final_max with the result widened to double (vv_reduce_enqueue's device outputs are all doubles; exact)
__global__ __launch_bounds__(256) void k_final_max_d(const float* partial, int n, double* out) {
  __shared__ float red[4];
  float m = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) m = fmaxf(m, partial[i]);
  m = lane_max<64>(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = (double)fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// vv_reduce_batch / vv_reduce_enqueue in two launches: blockIdx.y = request i runs k_dot / k_abssum / k_absmax's
// loop over the same grid-stride element partition (gridDim.x = their nblk) with the same block reduction, into
// request i's partial area; k_final_multi's block i then finishes it as k_final_d / k_final_max_d, and one more
// block copies the caller's device extras beside the results. Identical values to the per-request kernels, 2
// launches instead of 2 per request (+ a copy).
__global__ __launch_bounds__(256) void k_reduce_multi(ReduceReqs r, int64_t n, double* partial) {
  __shared__ double red[4];
  __shared__ float redf[4];
  const int i = blockIdx.y;
  const int op = r.op[i];
  const float* a = r.a[i];
  double* part = partial + (size_t)i * gridDim.x;
  const int64_t k0 = (int64_t)blockIdx.x * 256 + threadIdx.x, stride = (int64_t)gridDim.x * 256;
  if (op == 2) {
    float m = 0.f;
    for (int64_t k = k0; k < n; k += stride) m = fmaxf(m, fabsf(a[k]));
    m = lane_max<64>(m);
    if ((threadIdx.x & 63) == 0) redf[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0)
      reinterpret_cast<float*>(part)[blockIdx.x] = fmaxf(fmaxf(redf[0], redf[1]), fmaxf(redf[2], redf[3]));
    return;
  }
  double acc = 0.0;
  if (op == 0) {
    const float* b = r.b[i];
#pragma unroll 4
    for (int64_t k = k0; k < n; k += stride) acc += (double)a[k] * (double)b[k];
  } else {
    for (int64_t k = k0; k < n; k += stride) acc += fabs((double)a[k]);
  }
  const double t = block_sum(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}
__global__ __launch_bounds__(256) void k_final_multi(ReduceReqs r, int count, int nblk, const double* partial,
                                                     double* out, const double* extra, int n_extra) {
  __shared__ double red[4];
  __shared__ float redf[4];
  const int i = blockIdx.x;
  if (i == count) {  // the extras block
    for (int j = threadIdx.x; j < n_extra; j += 256) out[count + j] = extra[j];
    return;
  }
  const double* part = partial + (size_t)i * nblk;
  if (r.op[i] == 2) {
    const float* pf = reinterpret_cast<const float*>(part);
    float m = 0.f;
    for (int j = threadIdx.x; j < nblk; j += 256) m = fmaxf(m, pf[j]);
    m = lane_max<64>(m);
    if ((threadIdx.x & 63) == 0) redf[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) out[i] = (double)fmaxf(fmaxf(redf[0], redf[1]), fmaxf(redf[2], redf[3]));
    return;
  }
  double acc = 0.0;
  for (int j = threadIdx.x; j < nblk; j += 256) acc += part[j];
  const double t = block_sum(acc, red);
  if (threadIdx.x == 0) out[i] = t;
}
hipError_t reduce_multi(const ReduceReqs& r, int count, int64_t n, double* partial, int nblk, double* out,
                        const double* extra, int n_extra, hipStream_t s) {
  if (count < 0 || count > ReduceReqs::kMax || n_extra < 0 || (n_extra && !extra)) return hipErrorInvalidValue;
  if (count) hipLaunchKernelGGL(k_reduce_multi, dim3(nblk, count), dim3(256), 0, s, r, n, partial);
  const int blocks = count + (n_extra ? 1 : 0);
  if (blocks)
    hipLaunchKernelGGL(k_final_multi, dim3(blocks), dim3(256), 0, s, r, count, nblk, partial, out, extra, n_extra);
  return hipGetLastError();
}

hipError_t vec_absmax_d(const float* x, int64_t n, float* partial, int nblk, double* out, hipStream_t s) {
  hipLaunchKernelGGL(k_absmax, dim3(nblk), dim3(256), 0, s, x, n, partial);
  hipLaunchKernelGGL(k_final_max_d, dim3(1), dim3(256), 0, s, partial, nblk, out);
  return hipGetLastError();
}

hipError_t reduce_sumsq(const float* x, int64_t n, double* partial, int nblk, hipStream_t s) {
  hipLaunchKernelGGL(k_sumsq, dim3(nblk), dim3(256), 0, s, x, n, partial);
  return hipGetLastError();
}
hipError_t reduce_final(const double* partial, int n, double* out, hipStream_t s) {
  hipLaunchKernelGGL(k_final_d, dim3(1), dim3(256), 0, s, partial, n, out);
  return hipGetLastError();
}
hipError_t vec_dot(const float* a, const float* b, int64_t n, double* partial, int nblk, double* out, hipStream_t s) {
  hipLaunchKernelGGL(k_dot, dim3(nblk), dim3(256), 0, s, a, b, n, partial);
  hipLaunchKernelGGL(k_final_d, dim3(1), dim3(256), 0, s, partial, nblk, out);
  return hipGetLastError();
}
hipError_t vec_abssum(const float* x, int64_t n, double* partial, int nblk, double* out, hipStream_t s) {
  hipLaunchKernelGGL(k_abssum, dim3(nblk), dim3(256), 0, s, x, n, partial);
  hipLaunchKernelGGL(k_final_d, dim3(1), dim3(256), 0, s, partial, nblk, out);
  return hipGetLastError();
}
hipError_t vec_absmax(const float* x, int64_t n, float* partial, int nblk, float* out, hipStream_t s) {
  hipLaunchKernelGGL(k_absmax, dim3(nblk), dim3(256), 0, s, x, n, partial);
  hipLaunchKernelGGL(k_final_max, dim3(1), dim3(256), 0, s, partial, nblk, out);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_axpby(float* out, const float* x, float a, const float* y, float b,
                                               int64_t n) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    out[i] = (y ? b * y[i] : 0.f) + a * x[i];
}
__global__ __launch_bounds__(256) void k_axpy(float* y, const float* x, float a, int64_t n) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) y[i] = y[i] + a * x[i];
}
__global__ __launch_bounds__(256) void k_scale(float* y, float a, int64_t n) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) y[i] = y[i] * a;
}
__global__ __launch_bounds__(256) void k_fill(float* y, float v, int64_t n) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) y[i] = v;
}
static int vgrid(int64_t n) { return (int)std::min<int64_t>((n + 255) / 256, 2048); }
hipError_t vec_axpy(float* y, const float* x, float alpha, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_axpy, dim3(vgrid(n)), dim3(256), 0, s, y, x, alpha, n);
  return hipGetLastError();
}
hipError_t vec_axpby(float* out, const float* x, float a, const float* y, float b, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_axpby, dim3(vgrid(n)), dim3(256), 0, s, out, x, a, y, b, n);
  return hipGetLastError();
}
hipError_t vec_scale(float* y, float alpha, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_scale, dim3(vgrid(n)), dim3(256), 0, s, y, alpha, n);
  return hipGetLastError();
}
// L-BFGS two-loop recursion (torch/optim/lbfgs.py:404-442) with its scalars kept on the device: per history
// pair one kernel whose blocks each finish the pending dot from its partials exactly as k_final_d does and form the
// coefficient in fp32 as torch does on 0-d tensors (no host round trip), apply the axpy, and leave the partials of
// the next pair's dot. First loop (mode 0): al[i] = f32(s_i . q) * ro[i], q += (-al[i]) y_i. Second loop (mode 1):
// be = f32(y_i . r) * ro[i], r += (al[i] - be) s_i.
// the axpy of history pair i fused with the dot of pair i -+ 1 on the updated q: grid = the k_dot grid (nblk blocks,
// the same grid-stride element partition and accumulation order per thread, the same block_sum), so part_out holds
// exactly the partials k_dot would write on the new q; the coefficient comes from part_in as in k_twoloop_axpy
// (the two partial buffers alternate: blocks still reading part_in while others write part_out).
// One launch and one pass over q per history pair instead of two.
__global__ __launch_bounds__(256) void k_twoloop_axpy_dot(float* y, const float* x, const double* part_in, int nblk,
                                                          float ro, float* al, int i, int mode, int64_t n,
                                                          const float* next, double* part_out) {
  __shared__ double red[4], red2[4];
  __shared__ float coef;
  // this thread's first PF elements are loaded before the pending dot is finished (they do not depend on the
  // coefficient): the partials' reduction no longer sits in front of the vector loads (r05). Same elements, same
  // order of the d accumulation as the plain grid-stride loop below.
  constexpr int PF = 4;
  const int64_t k0 = (int64_t)blockIdx.x * 256 + threadIdx.x, stride = (int64_t)gridDim.x * 256;
  float yv[PF], xv[PF], nv[PF];
#pragma unroll
  for (int j = 0; j < PF; ++j) {
    const int64_t k = k0 + j * stride;
    yv[j] = k < n ? y[k] : 0.f;
    xv[j] = k < n ? x[k] : 0.f;
    nv[j] = next && k < n ? next[k] : 0.f;
  }
  double acc = 0.0;
  for (int j = threadIdx.x; j < nblk; j += 256) acc += part_in[j];
  const double t = block_sum(acc, red);
  if (threadIdx.x == 0) {
    const float v = (float)t * ro;
    if (mode == 0) {
      if (blockIdx.x == 0) al[i] = v;
      coef = -v;
    } else {
      coef = al[i] - v;
    }
  }
  __syncthreads();
  const float a = coef;
  double d = 0.0;
#pragma unroll
  for (int j = 0; j < PF; ++j) {
    const int64_t k = k0 + j * stride;
    if (k < n) {
      const float v = yv[j] + a * xv[j];
      y[k] = v;
      if (next) d += (double)nv[j] * (double)v;
    }
  }
  for (int64_t k = k0 + PF * stride; k < n; k += stride) {
    const float v = y[k] + a * x[k];
    y[k] = v;
    if (next) d += (double)next[k] * (double)v;
  }
  if (next) {
    const double u = block_sum(d, red2);
    if (threadIdx.x == 0) part_out[blockIdx.x] = u;
  }
}

// partial: 2 * nblk doubles (the fused kernels alternate between its halves)
hipError_t lbfgs_two_loop(float* q, const float* const* S, const float* const* Y, const float* ro, int m, float H_diag,
                          int64_t n, double* partial, int nblk, float* al, hipStream_t s) {
  double* pb[2] = {partial, partial + nblk};
  int c = 0;
  if (m > 0) hipLaunchKernelGGL(k_dot, dim3(nblk), dim3(256), 0, s, S[m - 1], q, n, pb[c]);
  for (int i = m - 1; i >= 0; --i, c ^= 1)
    hipLaunchKernelGGL(k_twoloop_axpy_dot, dim3(nblk), dim3(256), 0, s, q, Y[i], pb[c], nblk, ro[i], al, i, 0, n,
                       i > 0 ? S[i - 1] : nullptr, pb[c ^ 1]);
  hipLaunchKernelGGL(k_scale, dim3(vgrid(n)), dim3(256), 0, s, q, H_diag, n);
  c = 0;
  if (m > 0) hipLaunchKernelGGL(k_dot, dim3(nblk), dim3(256), 0, s, Y[0], q, n, pb[c]);
  for (int i = 0; i < m; ++i, c ^= 1)
    hipLaunchKernelGGL(k_twoloop_axpy_dot, dim3(nblk), dim3(256), 0, s, q, S[i], pb[c], nblk, ro[i], al, i, 1, n,
                       i + 1 < m ? Y[i + 1] : nullptr, pb[c ^ 1]);
  return hipGetLastError();
}
hipError_t fill(float* p, float v, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_fill, dim3(vgrid(n)), dim3(256), 0, s, p, v, n);
  return hipGetLastError();
}

// Adam (torch/optim/adam.py single-tensor path, no weight decay, no amsgrad):
//   m = b1 m + (1-b1) g ; v = b2 v + (1-b2) g^2 ; p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps)
__global__ __launch_bounds__(256) void k_adam(float* p, const float* g, float* m, float* v, int64_t n, float lr,
                                              float b1, float b2, float eps, float bc1, float bc2_sqrt) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float gi = g[i];
    const float mi = m[i] + (gi - m[i]) * (1.0f - b1);  // torch: exp_avg.lerp_(grad, 1-beta1)
    const float vi = v[i] * b2 + (1.0f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    p[i] = p[i] - (lr / bc1) * (mi / denom);
  }
}
hipError_t adam_step(float* p, const float* g, float* m, float* v, int64_t n, float lr, float b1, float b2, float eps,
                     float bc1, float bc2_sqrt, hipStream_t s) {
  hipLaunchKernelGGL(k_adam, dim3(vgrid(n)), dim3(256), 0, s, p, g, m, v, n, lr, b1, b2, eps, bc1, bc2_sqrt);
  return hipGetLastError();
}

// 32x32 LDS-tiled transpose (weights W [N][K] -> W^T [K][N], once at load time)
__global__ __launch_bounds__(256) void k_transpose(const float* in, float* out, int rows, int cols) {
  __shared__ float t[32][33];
  const int bx = blockIdx.x * 32, by = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int j = ty; j < 32; j += 8) {
    const int r = by + j, c = bx + tx;
    if (r < rows && c < cols) t[j][tx] = in[(size_t)r * cols + c];
  }
  __syncthreads();
  for (int j = ty; j < 32; j += 8) {
    const int r = bx + j, c = by + tx;  // out row = in col
    if (r < cols && c < rows) out[(size_t)r * rows + c] = t[tx][j];
  }
}
hipError_t transpose2d(const float* in, float* out, int rows, int cols, hipStream_t s) {
  hipLaunchKernelGGL(k_transpose, dim3((cols + 31) / 32, (rows + 31) / 32), dim3(256), 0, s, in, out, rows, cols);
  return hipGetLastError();
}

}  // namespace vv

namespace vv {
// the GELU / GELU' device functions every epilogue uses (vv_gelu.h), evaluated as they are compiled there: form 0 the
// one-value forms (gelu_fast / dgelu_fast: the GEMM epilogues), 1 the four-value interleaved forms (gelu4 / dgelu4: the
// fused tower MLP, the tile-49 row epilogue)
__global__ __launch_bounds__(256) void k_gelu_eval(const float* __restrict__ x, float* __restrict__ y,
                                                   float* __restrict__ dy, int64_t n, int form) {
  for (int64_t i = 4 * ((int64_t)blockIdx.x * 256 + threadIdx.x); i < n; i += 4 * (int64_t)gridDim.x * 256) {
    float v[4], g[4], d[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = i + u < n ? x[i + u] : 0.f;
    if (form) {
      gelu4(v, g);
      dgelu4(v, d);
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        g[u] = gelu_fast(v[u]);
        d[u] = dgelu_fast(v[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + u < n) {
        y[i + u] = g[u];
        dy[i + u] = d[u];
      }
  }
}
hipError_t gelu_eval(const float* x, float* y, float* dy, int64_t n, int form, hipStream_t s) {
  const unsigned g = (unsigned)std::min<int64_t>((n + 1023) / 1024, 4096);
  hipLaunchKernelGGL(k_gelu_eval, dim3(std::max(g, 1u)), dim3(256), 0, s, x, y, dy, n, form);
  return hipGetLastError();
}
}  // namespace vv

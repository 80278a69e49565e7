// Fused Swin-tower MLP sub-block (networks_old/utils/swinblock.py:13-29 Mlp, :296-309 the second residual of
// SwinTransformerBlock.forward): x2 = x1 + fc2(GELU(fc1(LN2(x1)))) and its input gradient, one launch each instead
// of LayerNorm + two GEMM launches, with the 4C-wide hidden layer never in HBM except the pre-activation the
// backward needs (quirk Q5: input gradients only, so no weight-gradient GEMM wants the hidden layer either).
//
// One workgroup per 16 NW tokens, one wave per 16 tokens; the hidden layer runs in chunks of HC units:
//   GEMM1^T  S[h][t] = sum_k W1[h][k] Y[t][k]     (Y = LN2(x1) fwd / dx2 bwd, per-token fp16 planes in LDS)
//   epilogue v = S + b1 -> h1 (fwd) ; u = GELU(v)  |  bwd: u = S * GELU'(h1)
//   GEMM2^T  O[n][t] += sum_h W2[n][h] u[t][h]     (u's fp16 planes built in registers straight from the
//                                                   GEMM1 accumulators: they ARE the B operand, in the permuted
//                                                   hidden order the W2 chunk is staged in)
//   epilogue x2 = x1 + (O + b2)  |  bwd: dx1 = dx2 + LayerNorm-backward(O) over the full row in registers.
// Arithmetic: fp16x3 (vv_gemm.hip k_gemm_h3 §): every operand row scaled by a power of two and split into fp16
// h / l planes, products l.h + h.l + h.h on v_mfma_f32_16x16x32_f16, scales applied after the k loop. The hidden
// operand u gets one scale per (token, HC chunk) -- no cross-workgroup row maximum -- and each chunk's partial
// product is rescaled into the fp32 accumulator (exact: powers of two).
#include <hip/hip_runtime.h>

#include <cmath>

#include "vv_gelu.h"
#include "vv_lanes.h"
#include "vv_kernels.h"

namespace vv {
namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef unsigned short u16;
typedef unsigned u4v __attribute__((ext_vector_type(4)));
typedef unsigned u2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

#ifdef VV_TRACE
// Development builds only (make EXTRA=-DVV_TRACE, tools/tower_trace.py): wave 0 of every workgroup records the shader
// clock at fixed points of the tower kernels into vv_trace_buf[region][workgroup][64] (slot 0..2: realtime at entry,
// HW_ID, XCC_ID; the rest s_memtime), vector stores from lane 0; the product build has none of it.
__device__ unsigned long long* vv_trace_buf;
#define VV_TR(region, slot)                                                                                       \
  do {                                                                                                            \
    unsigned long long* tb_ = vv_trace_buf;                                                                       \
    if (tb_ && threadIdx.x == 0) {                                                                                \
      tb_ += ((size_t)(region) * 2048 + blockIdx.x) * 64;                                                         \
      if ((slot) == 3) {                                                                                          \
        tb_[0] = __builtin_amdgcn_s_memrealtime();                                                                \
        tb_[1] = (unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11));                                             \
        tb_[2] = (unsigned)__builtin_amdgcn_s_getreg(20 | (15 << 11));                                            \
      }                                                                                                           \
      tb_[slot] = __builtin_readcyclecounter();                                                                   \
      if ((slot) == 63) tb_[62] = __builtin_amdgcn_s_memrealtime();                                               \
    }                                                                                                             \
  } while (0)
#else
#define VV_TR(region, slot) \
  do {                      \
  } while (0)
#endif

__device__ __forceinline__ float gelu_t(float x) { return gelu_fast(x); }  // vv_gelu.h
__device__ __forceinline__ float dgelu_t(float x) { return dgelu_fast(x); }
// fp16x3 row scale 2^(141 - E) of a row whose largest |value| has bit pattern mx, and its inverse 2^(E - 141)
__device__ __forceinline__ float sc_of(unsigned mx) { return __uint_as_float((268u - max(mx >> 23, 15u)) << 23); }
__device__ __forceinline__ float inv_of(unsigned mx) { return __uint_as_float((max(mx >> 23, 15u) - 14u) << 23); }
__device__ __forceinline__ unsigned amax(unsigned m, float v) { return max(m, __float_as_uint(fabsf(v))); }
// XCD-aware workgroup order (r05): the tower launches are 1-D over ngroups x nb workgroups, numbered tower-major,
// and XCD x (workgroups are dealt round-robin to the 8 XCDs, each with its own 4 MB L2) gets a contiguous range of
// them (vv_gemm.hip xcd_remap's formula), so an XCD streams the weights of at most two towers instead of all six
// (the dim-192 MLP's fp16x3 weight planes are 1.18 MB per tower, 7.1 MB for six)
__device__ __forceinline__ void tower_wg(int nb, int ng, int& blk, int& grp) {
  const int n = nb * ng, bid = blockIdx.x;
  const int q = n >> 3, r = n & 7, x = bid & 7, l = bid >> 3;
  const int w = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + l;
  grp = w / nb;
  blk = w - grp * nb;
}
// [rows][32 halves] plane blocks: 16-B chunk q of row r at q ^ h((r >> 2) & 3), h = {0, 2, 3, 1}, so the four lane
// groups of a 16x16x32 fragment read (rows lane & 15, chunk lane >> 4) hit 16 distinct 16-B slots
__device__ __forceinline__ int hsw(int q) { return (0x78 >> (2 * (q & 3))) & 3; }
__device__ __forceinline__ int frag(int r, int q) { return r * 32 + ((q ^ hsw(r >> 2)) << 3); }
// weight-chunk plane blocks padded by 32 halves (64 B): unpadded, the chunk staging stores hit one bank group six ways
// (dim 192: 68.7 / 68.9 -> 67.6 / 67.7 us, profiles/r04/ab_r04ab)
constexpr int kMlpBlockPad = 32;
// k_ablk_fwd's per-wave v buffer row stride (floats): 32, not 36, so that three dim-96 workgroups fit a CU's LDS (the v
// rows are read as broadcasts, 4 addresses per instruction; only the 6 row stores per wave take a 4-way conflict)
constexpr int kAblkHBS = 32;

// NH = 2 splits the hidden layer between two waves per 16 tokens (wave hh runs hidden units [hh 2C, hh 2C + 2C)):
// twice the waves per CU for the same LDS weight stream, the two partial fc2 sums added through LDS at the end.
template <int C, int NW, int HC, bool FWD, int NH>
__global__ __launch_bounds__(64 * NW * NH, C == 96 ? 3 : 1) void k_mlp(MlpArgs a) {
  constexpr int NT = 64 * NW * NH, KS1 = C / 32, KS2 = HC / 32, NJ = HC / 16, NQ = C / 16, NC = 4 * C / (HC * NH);
  constexpr int HH = 4 * C / NH;             // hidden units per wave half
  constexpr int CQ = C / 4;                  // channels per lane in the row phases (4 lanes per token)
  constexpr int A1W = KS1 * 2 * 16 * 32;     // halves of one wave's Y planes
  // plane blocks of a weight chunk (32 halves per row) padded by 64 B: unpadded they sit a multiple of 64 banks x 4 B
  // apart, and the staging stores of one row (all its blocks at once) hit the same bank group (r04 PMC: ~1.1
  // conflict cycles per LDS instruction); fragment reads stay inside one block (unchanged)
  constexpr int BP = kMlpBlockPad;
  constexpr int BLK1 = HC * 32 + BP, BLK2 = C * 32 + BP;
  constexpr int W1S = KS1 * 2 * BLK1;        // halves of a W1 chunk (HC rows x C)
  constexpr int W2S = KS2 * 2 * BLK2;        // halves of a W2 chunk (C rows x HC)
  static_assert(C % 32 == 0 && HC % 32 == 0 && HH % HC == 0 && CQ % 4 == 0 && (NH == 1 || NH == 2), "shape");
  static_assert(NH == 1 || NW * NQ * 64 * 16 <= 2 * NH * (W1S + W2S), "fc2 partial sums fit the weight buffers");
  extern __shared__ __attribute__((aligned(16))) u16 lds[];
  constexpr int TRR = (C == 96 ? 0 : 4) + (FWD ? 0 : 1);  // trace region (VV_TRACE builds)
  VV_TR(TRR, 3);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 15, g4 = lane >> 4;
  const int tg = wave % NW, hh = wave / NW;  // token group, hidden half
  const int hoff = hh * HH;
  int blk, grp;
  tower_wg(a.M / (16 * NW), a.ngroups, blk, grp);
  const MlpGroup G = a.g[grp];
  u16* A1 = lds + tg * A1W;
  u16* W1 = lds + NW * A1W;
  u16* W2 = W1 + NH * W1S;
  u16* W1w = W1 + hh * W1S;  // this wave's half of the chunk
  u16* W2w = W2 + hh * W2S;
  // per-row tables: W1 row scales / fc1 bias [4C], W2 row scales / fc2 bias [C] (fwd; bwd: no biases)
  float* T1s = reinterpret_cast<float*>(W2 + NH * W2S);
  float* T1b = T1s + 4 * C;
  float* T2s = T1b + 4 * C;
  float* T2b = T2s + C;
  const int t0 = blk * 16 * NW + 16 * tg;  // this wave's first token

  // prologue (r05): the token rows, then chunk 0's weights, then the tables, all in flight together (r04 order:
  // tables, rows, weights -- three memory round trips before the first chunk; tools/tower_trace.py)
  const int tt = lane >> 2, qd = lane & 3;  // token, quarter of the row
  f4 yv[CQ / 4];
  {
    const f4* src = reinterpret_cast<const f4*>((FWD ? G.x : G.dy) + (size_t)(t0 + tt) * C + qd * CQ);
#pragma unroll
    for (int v = 0; v < CQ / 4; ++v) yv[v] = src[v];
  }
  // weight chunks: global -> registers one chunk ahead (every load of a chunk in flight at once, under the
  // previous chunk's MFMAs), registers -> LDS between two barriers
  constexpr int P1 = NH * HC * KS1 * 8 / NT, P2 = NH * C * KS2 * 16 / NT;
  static_assert(P1 * NT == NH * HC * KS1 * 8 && P2 * NT == NH * C * KS2 * 16, "staging split");
  u4v r1[P1];
  u2v r2[P2];
  // W1 chunk: rows c HC + r, the whole K = C; global row = KS1 x [h(32) | l(32)]. W2 chunk: rows n < C, hidden units
  // [c HC, c HC + HC) in the order of the u fragments: position 8 g + e of k-step kk holds hidden
  // 32 kk + (e < 4 ? 4 g + e : 16 + 4 g + e - 4). (Plain unrolled loops, no lambdas: the staging registers must
  // not become a stack array.)
#define VV_MLP_LOAD(c)                                                                                            \
  {                                                                                                               \
    _Pragma("unroll") for (int i = 0; i < P1; ++i) {                                                             \
      const int e = tid + i * NT, r = e / (KS1 * 8), rem = e - r * (KS1 * 8), rh = r / HC, rl = r - rh * HC;     \
      r1[i] = *reinterpret_cast<const u4v*>(G.w1h + (size_t)(rh * HH + (c) * HC + rl) * 2 * C + (rem >> 3) * 64 + \
                                              ((rem >> 2) & 1) * 32 + (rem & 3) * 8);                             \
    }                                                                                                             \
    _Pragma("unroll") for (int i = 0; i < P2; ++i) {                                                             \
      const int e0 = tid + i * NT, eh = e0 / (C * KS2 * 16), e = e0 - eh * (C * KS2 * 16), n = e / (KS2 * 16),   \
                rem = e - n * (KS2 * 16);                                                                         \
      r2[i] = *reinterpret_cast<const u2v*>(G.w2h + (size_t)n * 2 * (4 * C) +                                   \
                                              (eh * (HH / 32) + (c) * KS2 + (rem >> 4)) * 64 +                   \
                                              ((rem >> 3) & 1) * 32 + 4 * ((rem >> 1) & 3) + 16 * (rem & 1));     \
    }                                                                                                             \
  }
  // (the forward loads chunk 0's weights after its row phase: at dim 192 they would spill beside gamma / beta, at dim 96
  // the earlier issue measured 2.7 K cycles slower, tools/tower_trace.py)
  constexpr bool kEarlyW = !FWD;
  if (kEarlyW) VV_MLP_LOAD(0)
  {  // every table load issued before the first LDS store (one memory round trip)
    constexpr int N1 = (4 * C + NT - 1) / NT, N2 = (C + NT - 1) / NT;
    float a1[N1], c1[N1], a2[N2], c2[N2];
#pragma unroll
    for (int i = 0; i < N1; ++i) {
      const int r = min(tid + i * NT, 4 * C - 1);
      a1[i] = G.w1s[(size_t)r * (C / 32)];
      c1[i] = FWD ? G.b1[r] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < N2; ++i) {
      const int r = min(tid + i * NT, C - 1);
      a2[i] = G.w2s[(size_t)r * (4 * C / 32)];
      c2[i] = FWD ? G.b2[r] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < N1; ++i)
      if (tid + i * NT < 4 * C) {
        T1s[tid + i * NT] = a1[i];
        T1b[tid + i * NT] = c1[i];
      }
#pragma unroll
    for (int i = 0; i < N2; ++i)
      if (tid + i * NT < C) {
        T2s[tid + i * NT] = a2[i];
        T2b[tid + i * NT] = c2[i];
      }
  }
  // ---- row phase: Y = LN2(x1) (fwd) or dx2 (bwd), scaled per token and split into planes ----
  float iy_own;                             // 2^-e of token tt's Y row
  {
    if (FWD) {
      f4 gv[CQ / 4], bv[CQ / 4];
#pragma unroll
      for (int v = 0; v < CQ / 4; ++v) {
        gv[v] = reinterpret_cast<const f4*>(G.gamma + qd * CQ)[v];
        bv[v] = reinterpret_cast<const f4*>(G.beta + qd * CQ)[v];
      }
      float s = 0.f;
#pragma unroll
      for (int v = 0; v < CQ / 4; ++v) s += (yv[v][0] + yv[v][1]) + (yv[v][2] + yv[v][3]);
      s += xshfl<1>(s);
      s += xshfl<2>(s);
      const float mean = s / (float)C;
      float q = 0.f;
#pragma unroll
      for (int v = 0; v < CQ / 4; ++v)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = yv[v][e] - mean;
          q += d * d;
        }
      q += xshfl<1>(q);
      q += xshfl<2>(q);
      const float rstd = 1.0f / sqrtf(q / (float)C + a.eps);
#pragma unroll
      for (int v = 0; v < CQ / 4; ++v)
#pragma unroll
        for (int e = 0; e < 4; ++e) yv[v][e] = (yv[v][e] - mean) * rstd * gv[v][e] + bv[v][e];
      if (qd == 0 && hh == 0) *reinterpret_cast<float2*>(G.stats + 2 * (size_t)(t0 + tt)) = make_float2(mean, rstd);
    }
    unsigned mx = 0;
#pragma unroll
    for (int v = 0; v < CQ / 4; ++v)
#pragma unroll
      for (int e = 0; e < 4; ++e) mx = amax(mx, yv[v][e]);
    mx = max(mx, (unsigned)xshfl<1>((int)mx));
    mx = max(mx, (unsigned)xshfl<2>((int)mx));
    const float sy = sc_of(mx);
    iy_own = inv_of(mx);
    typedef _Float16 h4t __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int v = 0; v < CQ / 4; ++v) {
      if (hh != 0) continue;  // the other half's wave only needs the scale
      const int k = qd * CQ + 4 * v, ks = k >> 5, kk = k & 31;
      h4t hv, lv;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float x = yv[v][e] * sy;
        hv[e] = (_Float16)x;
        lv[e] = (_Float16)(x - (float)hv[e]);
      }
      *reinterpret_cast<h4t*>(A1 + frag((ks * 2 + 0) * 16 + tt, kk >> 3) + (kk & 7)) = hv;
      *reinterpret_cast<h4t*>(A1 + frag((ks * 2 + 1) * 16 + tt, kk >> 3) + (kk & 7)) = lv;
    }
  }
  const float iy = __shfl(iy_own, li << 2);  // this lane's token (li) in the fragment layouts
  const size_t trow = (size_t)(t0 + li);

  f4 acc2[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) acc2[q] = f4{0.f, 0.f, 0.f, 0.f};
  if (!kEarlyW) VV_MLP_LOAD(0)
  VV_TR(TRR, 4);

  // two chunks per loop trip for the dim-192 forward (the hidden-split backward spills at 2; dim 96 runs faster
  // without: profiles/r04/ab_r04p)
  constexpr int UNR = (C == 96 || (NH == 2 && !FWD)) ? 1 : 2;  // dim 96: 50.0 / 54.0 vs 53.2 / 55.3 us unrolled
#pragma unroll UNR
  for (int c = 0; c < NC; ++c) {
    // bwd: this chunk's pre-activations, in flight before the next chunk's weight loads (vmcnt is in order)
    f4 ex[NJ];
    if (!FWD) {
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        ex[j] = *reinterpret_cast<const f4*>(G.h1 + trow * (4 * C) + hoff + c * HC + 16 * j + 4 * g4);
    }
    __syncthreads();  // the previous chunk's W1 / W2 fragment reads are done (and, at c = 0, the Y planes written)
#pragma unroll
    for (int i = 0; i < P1; ++i) {
      const int e = tid + i * NT, r = e / (KS1 * 8), rem = e - r * (KS1 * 8), rh = r / HC, rl = r - rh * HC;
      *reinterpret_cast<u4v*>(W1 + rh * W1S + ((rem >> 3) * 2 + ((rem >> 2) & 1)) * BLK1 + frag(rl, rem & 3)) =
          r1[i];
    }
#pragma unroll
    for (int i = 0; i < P2; ++i) {
      const int e0 = tid + i * NT, eh = e0 / (C * KS2 * 16), e = e0 - eh * (C * KS2 * 16), n = e / (KS2 * 16),
                rem = e - n * (KS2 * 16);
      *reinterpret_cast<u2v*>(W2 + eh * W2S + ((rem >> 4) * 2 + ((rem >> 3) & 1)) * BLK2 +
                                frag(n, (rem >> 1) & 3) + 4 * (rem & 1)) = r2[i];
    }
    __syncthreads();
    VV_TR(TRR, 5 + 2 * (c & 15));
    if (c + 1 < NC) VV_MLP_LOAD(c + 1)
    float s1[NJ][4];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = hoff + c * HC + 16 * j + 4 * g4;
      const f4 sv = *reinterpret_cast<const f4*>(T1s + n);
#pragma unroll
      for (int i = 0; i < 4; ++i) s1[j][i] = sv[i];
      if (FWD) ex[j] = *reinterpret_cast<const f4*>(T1b + n);
    }

    // GEMM1^T: rows = hidden units 16 j + 4 g4 + i of the chunk, columns = tokens
    f4 acc1[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc1[j] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks) {
      const h8v yh = *reinterpret_cast<const h8v*>(A1 + frag((ks * 2 + 0) * 16 + li, g4));
      const h8v yl = *reinterpret_cast<const h8v*>(A1 + frag((ks * 2 + 1) * 16 + li, g4));
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const h8v wh = *reinterpret_cast<const h8v*>(W1w + (ks * 2 + 0) * BLK1 + frag(16 * j + li, g4));
        const h8v wl = *reinterpret_cast<const h8v*>(W1w + (ks * 2 + 1) * BLK1 + frag(16 * j + li, g4));
        acc1[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, yh, acc1[j], 0, 0, 0);
        acc1[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, yl, acc1[j], 0, 0, 0);
        acc1[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, yh, acc1[j], 0, 0, 0);
      }
    }
    // epilogue 1
    float u[NJ][4];
    unsigned mx = 0;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = hoff + c * HC + 16 * j + 4 * g4;
      if (FWD) {
        f4 v;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = acc1[j][i] * (iy * s1[j][i]) + ex[j][i];
        *reinterpret_cast<f4*>(G.h1 + trow * (4 * C) + n) = v;
        const float vv[4] = {v[0], v[1], v[2], v[3]};
        gelu4(vv, u[j]);
      } else {
        const float xv[4] = {ex[j][0], ex[j][1], ex[j][2], ex[j][3]};
        float dg[4];
        dgelu4(xv, dg);
#pragma unroll
        for (int i = 0; i < 4; ++i) u[j][i] = acc1[j][i] * (iy * s1[j][i]) * dg[i];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) mx = amax(mx, u[j][i]);
    }
    mx = max(mx, (unsigned)xshfl<16>((int)mx));
    mx = max(mx, (unsigned)xshfl<32>((int)mx));
    const float su = sc_of(mx), iu = inv_of(mx);
    // GEMM2^T: rows = output channels 16 q + 4 g4 + i, columns = tokens; u's planes are the B fragments
    f4 tmp[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) tmp[q] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < KS2; ++kk) {
      h8v bh, bl;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float x = u[2 * kk + (e >> 2)][e & 3] * su;
        bh[e] = (_Float16)x;
        bl[e] = (_Float16)(x - (float)bh[e]);
      }
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const h8v wh = *reinterpret_cast<const h8v*>(W2w + (kk * 2 + 0) * BLK2 + frag(16 * q + li, g4));
        const h8v wl = *reinterpret_cast<const h8v*>(W2w + (kk * 2 + 1) * BLK2 + frag(16 * q + li, g4));
        tmp[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, bh, tmp[q], 0, 0, 0);
        tmp[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, bl, tmp[q], 0, 0, 0);
        tmp[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, bh, tmp[q], 0, 0, 0);
      }
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc2[q][i] += tmp[q][i] * iu;
    VV_TR(TRR, 6 + 2 * (c & 15));
  }
  VV_TR(TRR, 40);
  if (NH == 2) {  // half 1's fc2 partial sums through LDS (over the weight buffers) to half 0, which finishes
    f4* R = reinterpret_cast<f4*>(W1);
    __syncthreads();
    if (hh == 1) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) R[(tg * NQ + q) * 64 + lane] = acc2[q];
    }
    __syncthreads();
    if (hh == 1) return;
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc2[q] += R[(tg * NQ + q) * 64 + lane];
  }

  // ---- epilogue 2 (lane: token li, channels 16 q + 4 g4 + i) ----
  float o[NQ][4];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int n = 16 * q + 4 * g4;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[q][i] = acc2[q][i] * T2s[n + i];
  }
  if (FWD) {
    f4 xv[NQ];  // all residual loads before the first store (see k_ablk_fwd)
#pragma unroll
    for (int q = 0; q < NQ; ++q) xv[q] = *reinterpret_cast<const f4*>(G.x + trow * C + 16 * q + 4 * g4);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int n = 16 * q + 4 * g4;
      const f4 bv = *reinterpret_cast<const f4*>(T2b + n);
      f4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = xv[q][i] + (o[q][i] + bv[i]);
      *reinterpret_cast<f4*>(G.out + trow * C + n) = v;
    }
  } else {
    // LayerNorm backward over the row (this lane's 4 NQ channels + the other three lane groups):
    // dx = rstd (g dy - mean(g dy) - xhat mean(g dy xhat)), then + dx2 (the residual), k_ln_bwd's formula
    const float2 st = *reinterpret_cast<const float2*>(G.stats + 2 * trow);
    const float mean = st.x, rstd = st.y;
    f4 xv[NQ], gv[NQ];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int n = 16 * q + 4 * g4;
      xv[q] = *reinterpret_cast<const f4*>(G.x + trow * C + n);
      gv[q] = *reinterpret_cast<const f4*>(G.gamma + n);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float gd = gv[q][i] * o[q][i];
        s1 += gd;
        s2 += gd * ((xv[q][i] - mean) * rstd);
      }
    }
    s1 += xshfl<16>(s1);
    s1 += xshfl<32>(s1);
    s2 += xshfl<16>(s2);
    s2 += xshfl<32>(s2);
    const float m1 = s1 / (float)C, m2 = s2 / (float)C;
    unsigned omx = 0;
    f4 dv[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) dv[q] = *reinterpret_cast<const f4*>(G.dy + trow * C + 16 * q + 4 * g4);
    // every lane has read its dy before any lane of the workgroup writes (out may alias dy: same rows only)
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      f4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[i] = rstd * (gv[q][i] * o[q][i] - m1 - ((xv[q][i] - mean) * rstd) * m2) + dv[q][i];
        omx = amax(omx, v[i]);
      }
      *reinterpret_cast<f4*>(G.out + trow * C + 16 * q + 4 * g4) = v;
    }
    if (G.rs) {
      omx = max(omx, (unsigned)xshfl<16>((int)omx));
      omx = max(omx, (unsigned)xshfl<32>((int)omx));
      if (g4 == 0) G.rs[trow] = sc_of(omx);
    }
  }
  VV_TR(TRR, 63);
}

#undef VV_MLP_LOAD

template <int C, int NW, int HC, bool FWD, int NH = 1>
hipError_t launch_mlp(const MlpArgs& a, hipStream_t s) {
  constexpr size_t lds = 2 * ((size_t)NW * (C / 32) * 2 * 16 * 32 + (size_t)NH * (C / 32) * 2 * (HC * 32 + kMlpBlockPad) +
                              (size_t)NH * (HC / 32) * 2 * (C * 32 + kMlpBlockPad)) + 4 * (8 * C + 2 * C);
  static_assert(C != 96 || lds <= 53760, "three dim-96 workgroups per CU (k_ablk_fwd launch: LDS granules)");
  static_assert(lds <= 163840, "LDS");
  if (hipError_t e = set_lds_limit((const void*)k_mlp<C, NW, HC, FWD, NH>, lds)) return e;
  hipLaunchKernelGGL((k_mlp<C, NW, HC, FWD, NH>), dim3(a.M / (16 * NW) * a.ngroups), dim3(64 * NW * NH), lds, s, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------------------
// Fused Swin-tower attention sub-block, forward (swinblock.py:265-296 SwinTransformerBlock.forward up to the first
// residual; WindowAttention :133-172): x1 = x + proj(WindowAttention(LN1(x) in window order)) in window-reverse
// order. One wave per 16-token window, four windows per workgroup. Per head h four 8C-half weight chunks go
// through LDS (two chunks ahead in registers): the q, k and v rows of the qkv weight (GEMM^T: 2 tiles x C/32
// k-steps, fp16x3) -- the head's 16 x 32 q / k / v go to HBM (saved for the backward) and to a per-wave LDS buffer,
// scores + bias + mask, softmax and P.V run on the VALU in fp32 as in k_attn_fwd -- then the head's 32 columns of
// the proj weight: the head output, scaled per (token, head) and split in registers, is already the B fragment of
// that k-step (lane = token, 8 consecutive channels), and its partial product is rescaled into the proj
// accumulator (exact). No O buffer, and the scores come from q / k fragments in registers (fp16x3 MFMA): 54 KB of
// LDS, three workgroups per CU.
template <int C>
__global__ __launch_bounds__(256, C == 96 ? 3 : 1) void k_ablk_fwd(AblkArgs a) {
  constexpr int NW = 4, NT = 256, KS = C / 32, H = C / 32, CQ = C / 4, NQ = C / 16;
  constexpr int YW = KS * 2 * 16 * 32;        // halves of one wave's Y planes
  constexpr int WCH = 8 * C * 8;              // halves of a weight chunk (8 C 16-B pieces)
  constexpr int HBS = kAblkHBS;               // fp32 row stride of the per-wave v head buffers
  constexpr int PBS = 16;                     // fp32 row stride of the per-wave P buffer
  constexpr int NSC = 4 * H;                  // chunks: q, k, v rows and proj columns per head
  constexpr int PC = 8 * C / NT;              // 16-B staging pieces per thread and chunk
  static_assert(PC * NT == 8 * C, "staging split");
  extern __shared__ __attribute__((aligned(16))) u16 lds[];
  constexpr int TRR = C == 96 ? 2 : 6;
  VV_TR(TRR, 3);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 15, g4 = lane >> 4;
  int blk, grp;
  tower_wg(a.M / 64, a.ngroups, blk, grp);
  const AblkGroup G = a.g[grp];
  u16* Ypl = lds + wave * YW;
  u16* Wc = lds + NW * YW;
  float* fl = reinterpret_cast<float*>(Wc + WCH);
  float* hb = fl + wave * 16 * HBS;                       // [16][HBS]: v of the head
  float* pb = fl + NW * 16 * HBS + wave * 16 * PBS;       // [16][PBS]: P of the head
  float* tb = fl + NW * (16 * HBS + 16 * PBS);            // [H][49], padded to 16 B
  float* Tqs = tb + ((H * 49 + 3) & ~3);  // qkv row scales [3C]
  float* Tqb = Tqs + 3 * C;      // qkv bias [3C]
  float* Tps = Tqb + 3 * C;      // proj row scales [C]
  float* Tpb = Tps + C;          // proj bias [C]
  const int win = blk * NW + wave;  // this wave's window (over the batch)
  const int r0 = win * 16;                 // its first window-order row

  // prologue (r05): the window's token rows, then chunks 0 and 1, then the tables, all in flight together (r04:
  // tables, weights, rows -- the rows a round trip after the rest; tools/tower_trace.py)
  const int tt = lane >> 2, qd = lane & 3;
  f4 yv[CQ / 4];
  {
    const size_t prow = (size_t)a.map[r0 + tt];
    const f4* src = reinterpret_cast<const f4*>(G.x + prow * C + qd * CQ);
#pragma unroll
    for (int v = 0; v < CQ / 4; ++v) yv[v] = src[v];
  }
  // weight chunk sc = 4 h + part: part < 3 -> rows part C + 32 h + r (r < 32) of the qkv weight, the whole K = C
  // ([ks][plane][32 rows][32]); part 3 -> k-chunk h of every proj row n < C ([plane][C rows][32])
  u4v rw[2][PC];
#define VV_ABLK_LOAD(buf, sc)                                                                                    \
  {                                                                                                              \
    const int h_ = (sc) >> 2, part_ = (sc)&3;                                                                    \
    _Pragma("unroll") for (int i = 0; i < PC; ++i) {                                                            \
      const int e = tid + i * NT;                                                                                \
      if (part_ < 3) {                                                                                           \
        const int r = e / (KS * 8), rem = e - r * (KS * 8);                                                      \
        rw[buf][i] = *reinterpret_cast<const u4v*>(G.wqh + (size_t)(part_ * C + 32 * h_ + r) * 2 * C +            \
                                                   (rem >> 3) * 64 + ((rem >> 2) & 1) * 32 + (rem & 3) * 8);     \
      } else {                                                                                                   \
        const int n = e >> 3, rem = e & 7;                                                                       \
        rw[buf][i] = *reinterpret_cast<const u4v*>(G.wph + (size_t)n * 2 * C + h_ * 64 + (rem >> 2) * 32 +         \
                                                   (rem & 3) * 8);                                               \
      }                                                                                                          \
    }                                                                                                            \
  }
  VV_ABLK_LOAD(0, 0)
  VV_ABLK_LOAD(1, 1)
  {  // every table load issued before the first LDS store (one memory round trip)
    constexpr int NB = (H * 49 + NT - 1) / NT, N1 = (3 * C + NT - 1) / NT, N2 = (C + NT - 1) / NT;
    float tv[NB], a1[N1], c1[N1], a2[N2], c2[N2];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int r = min(tid + i * NT, H * 49 - 1);
      tv[i] = G.table[(r % 49) * a.heads + r / 49];
    }
#pragma unroll
    for (int i = 0; i < N1; ++i) {
      const int r = min(tid + i * NT, 3 * C - 1);
      a1[i] = G.wqs[(size_t)r * (C / 32)];
      c1[i] = G.wqb[r];
    }
#pragma unroll
    for (int i = 0; i < N2; ++i) {
      const int r = min(tid + i * NT, C - 1);
      a2[i] = G.wps[(size_t)r * (C / 32)];
      c2[i] = G.wpb[r];
    }
#pragma unroll
    for (int i = 0; i < NB; ++i)
      if (tid + i * NT < H * 49) tb[tid + i * NT] = tv[i];
#pragma unroll
    for (int i = 0; i < N1; ++i)
      if (tid + i * NT < 3 * C) {
        Tqs[tid + i * NT] = a1[i];
        Tqb[tid + i * NT] = c1[i];
      }
#pragma unroll
    for (int i = 0; i < N2; ++i)
      if (tid + i * NT < C) {
        Tps[tid + i * NT] = a2[i];
        Tpb[tid + i * NT] = c2[i];
      }
  }

  VV_TR(TRR, 4);

  // ---- LN1 of the window's 16 rows (gathered through the window map), planes in LDS ----
  float iy_own;
  {
    f4 gv[CQ / 4], bv[CQ / 4];
#pragma unroll
    for (int v = 0; v < CQ / 4; ++v) {
      gv[v] = reinterpret_cast<const f4*>(G.n1g + qd * CQ)[v];
      bv[v] = reinterpret_cast<const f4*>(G.n1b + qd * CQ)[v];
    }
    float sm = 0.f;
#pragma unroll
    for (int v = 0; v < CQ / 4; ++v) sm += (yv[v][0] + yv[v][1]) + (yv[v][2] + yv[v][3]);
    sm += xshfl<1>(sm);
    sm += xshfl<2>(sm);
    const float mean = sm / (float)C;
    float q = 0.f;
#pragma unroll
    for (int v = 0; v < CQ / 4; ++v)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = yv[v][e] - mean;
        q += d * d;
      }
    q += xshfl<1>(q);
    q += xshfl<2>(q);
    const float rstd = 1.0f / sqrtf(q / (float)C + a.eps);
    unsigned mx = 0;
#pragma unroll
    for (int v = 0; v < CQ / 4; ++v)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        yv[v][e] = (yv[v][e] - mean) * rstd * gv[v][e] + bv[v][e];
        mx = amax(mx, yv[v][e]);
      }
    if (qd == 0) *reinterpret_cast<float2*>(G.stats + 2 * (size_t)(r0 + tt)) = make_float2(mean, rstd);
    mx = max(mx, (unsigned)xshfl<1>((int)mx));
    mx = max(mx, (unsigned)xshfl<2>((int)mx));
    const float sy = sc_of(mx);
    iy_own = inv_of(mx);
    typedef _Float16 h4t __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int v = 0; v < CQ / 4; ++v) {
      const int k = qd * CQ + 4 * v, ks = k >> 5, kk = k & 31;
      h4t hv, lv;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float x = yv[v][e] * sy;
        hv[e] = (_Float16)x;
        lv[e] = (_Float16)(x - (float)hv[e]);
      }
      *reinterpret_cast<h4t*>(Ypl + frag((ks * 2 + 0) * 16 + tt, kk >> 3) + (kk & 7)) = hv;
      *reinterpret_cast<h4t*>(Ypl + frag((ks * 2 + 1) * 16 + tt, kk >> 3) + (kk & 7)) = lv;
    }
  }
  const float iy = __shfl(iy_own, li << 2);
  const size_t trow = (size_t)(r0 + li);         // this lane's token, window order
  const size_t tphys = (size_t)a.map[r0 + li];   // ... physical row
  const int wr = (win % (a.nWh * a.nWw)) / a.nWw;
  auto lab = [&](int rr) {
    const int y = wr * 4 + rr;
    return y < a.H - 4 ? 0 : (y < a.H - a.shift ? 1 : 2);
  };
  const bool masked_row = a.shift > 0 && lab(g4) != lab(li >> 2);

  f4 pacc[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) pacc[q] = f4{0.f, 0.f, 0.f, 0.f};
  h8v oh, ol;  // the current head's output planes (B fragment: token li, channels 8 g4 .. 8 g4 + 7)
  float io = 0.f;
  h8v qh, ql, kh, kl;  // the head's q (A operand) and k (B operand) planes, token li
  float iq = 0.f, ik = 0.f;
  for (int sc = 0; sc < NSC; ++sc) {
    const int h = sc >> 2, part = sc & 3;
    __syncthreads();
    // chunk sc from register set sc & 1 into LDS, then chunk sc + 2 into that set
#define VV_ABLK_STORE(buf)                                                                                       \
  _Pragma("unroll") for (int i = 0; i < PC; ++i) {                                                              \
    const int e = tid + i * NT;                                                                                  \
    if (part < 3) {                                                                                              \
      const int r = e / (KS * 8), rem = e - r * (KS * 8);                                                        \
      *reinterpret_cast<u4v*>(Wc + ((rem >> 3) * 2 + ((rem >> 2) & 1)) * 32 * 32 + frag(r, rem & 3)) = rw[buf][i]; \
    } else {                                                                                                     \
      const int n = e >> 3, rem = e & 7;                                                                         \
      *reinterpret_cast<u4v*>(Wc + (rem >> 2) * C * 32 + frag(n, rem & 3)) = rw[buf][i];                         \
    }                                                                                                            \
  }
    if (sc & 1) {
      VV_ABLK_STORE(1)
    } else {
      VV_ABLK_STORE(0)
    }
    __syncthreads();
    VV_TR(TRR, 5 + 2 * sc);
    if (sc + 2 < NSC) {
      if (sc & 1) {
        VV_ABLK_LOAD(1, sc + 2)
      } else {
        VV_ABLK_LOAD(0, sc + 2)
      }
    }
    if (part < 3) {
      f4 acc[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const h8v yh = *reinterpret_cast<const h8v*>(Ypl + frag((ks * 2 + 0) * 16 + li, g4));
        const h8v yl = *reinterpret_cast<const h8v*>(Ypl + frag((ks * 2 + 1) * 16 + li, g4));
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const h8v wh = *reinterpret_cast<const h8v*>(Wc + (ks * 2 + 0) * 32 * 32 + frag(16 * j + li, g4));
          const h8v wl = *reinterpret_cast<const h8v*>(Wc + (ks * 2 + 1) * 32 * 32 + frag(16 * j + li, g4));
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, yh, acc[j], 0, 0, 0);
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, yl, acc[j], 0, 0, 0);
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, yh, acc[j], 0, 0, 0);
        }
      }
      // q / k / v of head h for token li, channels 16 j + 4 g4 + i of the head
      f4 val[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c = 16 * j + 4 * g4, R = part * C + h * 32 + c;
        const f4 sv = *reinterpret_cast<const f4*>(Tqs + R);
        const f4 bv = *reinterpret_cast<const f4*>(Tqb + R);
#pragma unroll
        for (int i = 0; i < 4; ++i) val[j][i] = acc[j][i] * (iy * sv[i]) + bv[i];
        *reinterpret_cast<f4*>(G.qkv + trow * (3 * C) + R) = val[j];
        if (part == 2) *reinterpret_cast<f4*>(hb + li * HBS + c) = val[j];
      }
      if (part < 2) {
        // q (part 0) / k (part 1) of the head as fp16x3 fragments straight from the accumulators: lane = token,
        // k index e <-> channel 16 (e >> 2) + 4 g4 + (e & 3) (the same permutation for both operands)
        unsigned mx = 0;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i) mx = amax(mx, val[j][i]);
        mx = max(mx, (unsigned)xshfl<16>((int)mx));
        mx = max(mx, (unsigned)xshfl<32>((int)mx));
        const float ss = sc_of(mx);
        h8v fh, fl8;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float x = val[e >> 2][e & 3] * ss;
          fh[e] = (_Float16)x;
          fl8[e] = (_Float16)(x - (float)fh[e]);
        }
        if (part == 0) {
          qh = fh;
          ql = fl8;
          iq = inv_of(mx);
        } else {
          kh = fh;
          kl = fl8;
          ik = inv_of(mx);
        }
      } else {
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's v stores to LDS are done
        __builtin_amdgcn_wave_barrier();
        // S[t1][t2] (t1 = 4 g4 + i, t2 = li) = q[t1].k[t2] (fp16x3 MFMA) scale + bias + mask; softmax over t2
        f4 sacc = {0.f, 0.f, 0.f, 0.f};
        sacc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ql, kh, sacc, 0, 0, 0);
        sacc = __builtin_amdgcn_mfma_f32_16x16x32_f16(qh, kl, sacc, 0, 0, 0);
        sacc = __builtin_amdgcn_mfma_f32_16x16x32_f16(qh, kh, sacc, 0, 0, 0);
        float sv4[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) sv4[i] = sacc[i] * (__shfl(iq, 4 * g4 + i) * ik);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int cj = li & 3, rj = li >> 2;
          float b = tb[h * 49 + (g4 - rj + 3) * 7 + (i - cj + 3)];
          if (masked_row) b += -100.0f;
          float x = sv4[i] * a.scale + b;
          float mx = x;
          mx = fmaxf(mx, xshfl<1>(mx)); mx = fmaxf(mx, xshfl<2>(mx)); mx = fmaxf(mx, xshfl<4>(mx)); mx = fmaxf(mx, xshfl<8>(mx));
          x = expf(x - mx);
          float sum = x;
          sum += xshfl<1>(sum); sum += xshfl<2>(sum); sum += xshfl<4>(sum); sum += xshfl<8>(sum);
          const float pv = x * (1.0f / sum);
          G.P[(((size_t)win * a.heads + h) * 16 + 4 * g4 + i) * 16 + li] = pv;
          pb[(4 * g4 + i) * PBS + li] = pv;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        // O[t][c] (t = li, c = 8 g4 + e of the head) = sum_t2 P[t][t2] v[t2][c]
        float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t2 = 0; t2 < 16; t2 += 4) {
          const f4 p4 = *reinterpret_cast<const f4*>(pb + li * PBS + t2);
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const float* vr = hb + (t2 + u) * HBS + 8 * g4;
            const f4 v0 = *reinterpret_cast<const f4*>(vr), v1 = *reinterpret_cast<const f4*>(vr + 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              o[e] += p4[u] * v0[e];
              o[4 + e] += p4[u] * v1[e];
            }
          }
        }
        unsigned omx = 0;
#pragma unroll
        for (int e = 0; e < 8; ++e) omx = amax(omx, o[e]);
        omx = max(omx, (unsigned)xshfl<16>((int)omx));
        omx = max(omx, (unsigned)xshfl<32>((int)omx));
        const float so = sc_of(omx);
        io = inv_of(omx);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float x = o[e] * so;
          oh[e] = (_Float16)x;
          ol[e] = (_Float16)(x - (float)oh[e]);
        }
      }
    } else {
      // proj^T k-step h: rows n = 16 q + 4 g4 + i, columns = tokens; rescaled by the head output's scale
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const h8v wh = *reinterpret_cast<const h8v*>(Wc + frag(16 * q + li, g4));
        const h8v wl = *reinterpret_cast<const h8v*>(Wc + C * 32 + frag(16 * q + li, g4));
        f4 t = {0.f, 0.f, 0.f, 0.f};
        t = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, oh, t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, ol, t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, oh, t, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 4; ++i) pacc[q][i] += t[i] * io;
      }
    }
    VV_TR(TRR, 6 + 2 * sc);
  }
#undef VV_ABLK_STORE
#undef VV_ABLK_LOAD
  // every residual load issued before the first store (out may alias x as far as the compiler knows: a load
  // after a store would wait for it, one memory round trip per float4)
  f4 xv[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) xv[q] = *reinterpret_cast<const f4*>(G.x + tphys * C + 16 * q + 4 * g4);
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int n = 16 * q + 4 * g4;
    const f4 sv = *reinterpret_cast<const f4*>(Tps + n);
    const f4 bv = *reinterpret_cast<const f4*>(Tpb + n);
    f4 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = xv[q][i] + (pacc[q][i] * sv[i] + bv[i]);
    *reinterpret_cast<f4*>(G.out + tphys * C + n) = v;
  }
  VV_TR(TRR, 63);
}

// Backward of the attention sub-block (the input gradient only, quirk Q5), one wave per window:
//   dO = gx[window rows] W_proj                      (GEMM^T per head: projW^T rows of the head, B = gx planes)
//   dP = dO v^T (fp16x3 MFMA from registers), dS = P (dP - rowsum(P dP)); dq = scale dS k, dk = scale dS^T q,
//   dv = P^T dO on the VALU (fp32, as k_attn_bwd), each already a B fragment of the dY GEMM (8 consecutive
//   channels of the token) scaled per (token, k-step)
//   dY = dqkv W_qkv                                 (qkvW^T k-chunks of q_h, k_h, v_h, rescaled per k-step)
//   gx[window rows] += LN1-backward(dY)             (full rows in registers, k_ln_bwd's formula), in place.
template <int C>
__global__ __launch_bounds__(256, C == 96 ? 2 : 1) void k_ablk_bwd(AblkArgs a) {
  constexpr int NW = 4, NT = 256, KS = C / 32, H = C / 32, CQ = C / 4, NQ = C / 16;
  constexpr int YW = KS * 2 * 16 * 32;        // halves of one wave's gx planes
  constexpr int WCH = 8 * C * 8;              // halves of a weight chunk
  constexpr int BS = 36;                      // fp32 row stride of the per-wave q / k / dO buffers
  constexpr int SS = 17;                      // ... of dS / P
  constexpr int PWAVE = 3 * 16 * BS + 2 * 16 * SS;
  constexpr int NSC = 4 * H;
  constexpr int PC = 8 * C / NT;
  static_assert(PC * NT == 8 * C, "staging split");
  extern __shared__ __attribute__((aligned(16))) u16 lds[];
  constexpr int TRR = C == 96 ? 3 : 7;
  VV_TR(TRR, 3);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 15, g4 = lane >> 4;
  int blk, grp;
  tower_wg(a.M / 64, a.ngroups, blk, grp);
  const AblkGroup G = a.g[grp];
  u16* Dpl = lds + wave * YW;
  u16* Wc = lds + NW * YW;
  float* fl = reinterpret_cast<float*>(Wc + WCH);
  float* qb = fl + wave * PWAVE;   // [16][BS] q of the head
  float* kb = qb + 16 * BS;        // [16][BS] k
  float* ob = kb + 16 * BS;        // [16][BS] dO
  float* sb = ob + 16 * BS;        // [16][SS] dS
  float* pb = sb + 16 * SS;        // [16][SS] P
  float* Tos = fl + NW * PWAVE;    // proj^T row scales [C]
  float* Tqs = Tos + C;            // qkv^T row scales [C]
  const int win = blk * NW + wave;
  const int r0 = win * 16;
  // prologue (r05): the window's gx rows, then chunks 0 and 1, then the tables, all in flight together
  const int tt = lane >> 2, qd = lane & 3;
  f4 yv[CQ / 4];
  {
    const size_t prow = (size_t)a.map[r0 + tt];
    const f4* src = reinterpret_cast<const f4*>(G.out + prow * C + qd * CQ);
#pragma unroll
    for (int v = 0; v < CQ / 4; ++v) yv[v] = src[v];
  }
  const size_t trow = (size_t)(r0 + li);  // this lane's token, window order
  // the saved q, k, v rows and P of a head (HBM), loaded three chunks before the head's dO GEMM needs them (r05:
  // loaded at that chunk, they cost an exposed HBM round trip per head, 40 % of the workgroup's cycles)
  f4 sq[2], sk[2], sv3[2];
  float sp[4];
#define VV_ABWD_SAVED(h_)                                                                                         \
  {                                                                                                               \
    const float* qr_ = G.qkv + trow * (3 * C) + (h_)*32;                                                          \
    _Pragma("unroll") for (int j = 0; j < 2; ++j) {                                                              \
      sq[j] = *reinterpret_cast<const f4*>(qr_ + 16 * j + 4 * g4);                                               \
      sk[j] = *reinterpret_cast<const f4*>(qr_ + C + 16 * j + 4 * g4);                                           \
      sv3[j] = *reinterpret_cast<const f4*>(qr_ + 2 * C + 16 * j + 4 * g4);                                      \
    }                                                                                                             \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) sp[i] =                                                        \
        G.P[(((size_t)win * a.heads + (h_)) * 16 + 4 * g4 + i) * 16 + li];                                       \
  }
  VV_ABWD_SAVED(0)
  // chunk sc = 4 h + part: part 0 -> proj^T rows 32 h + r, the whole K = C ([ks][plane][32][32]); part 1..3 ->
  // k-chunk (part - 1) KS + h of every qkv^T row c < C ([plane][C][32])
  u4v rw[2][PC];
#define VV_ABWD_LOAD(buf, sc)                                                                                    \
  {                                                                                                              \
    const int h_ = (sc) >> 2, part_ = (sc)&3;                                                                    \
    _Pragma("unroll") for (int i = 0; i < PC; ++i) {                                                            \
      const int e = tid + i * NT;                                                                                \
      if (part_ == 0) {                                                                                          \
        const int r = e / (KS * 8), rem = e - r * (KS * 8);                                                      \
        rw[buf][i] = *reinterpret_cast<const u4v*>(G.wpth + (size_t)(32 * h_ + r) * 2 * C + (rem >> 3) * 64 +     \
                                                   ((rem >> 2) & 1) * 32 + (rem & 3) * 8);                       \
      } else {                                                                                                   \
        const int n = e >> 3, rem = e & 7;                                                                       \
        rw[buf][i] = *reinterpret_cast<const u4v*>(G.wqth + (size_t)n * 2 * (3 * C) +                            \
                                                   ((part_ - 1) * KS + h_) * 64 + (rem >> 2) * 32 + (rem & 3) * 8); \
      }                                                                                                          \
    }                                                                                                            \
  }
  VV_ABWD_LOAD(0, 0)
  VV_ABWD_LOAD(1, 1)
  {
    constexpr int N1 = (C + NT - 1) / NT;
    float a1[N1], c1[N1];
#pragma unroll
    for (int i = 0; i < N1; ++i) {
      const int r = min(tid + i * NT, C - 1);
      a1[i] = G.wpts[(size_t)r * (C / 32)];
      c1[i] = G.wqts[(size_t)r * (3 * C / 32)];
    }
#pragma unroll
    for (int i = 0; i < N1; ++i)
      if (tid + i * NT < C) {
        Tos[tid + i * NT] = a1[i];
        Tqs[tid + i * NT] = c1[i];
      }
  }
  VV_TR(TRR, 4);

  // ---- gx rows of the window (gathered), scaled per token and split into planes ----
  float id_own;
  {
    unsigned mx = 0;
#pragma unroll
    for (int v = 0; v < CQ / 4; ++v)
#pragma unroll
      for (int e = 0; e < 4; ++e) mx = amax(mx, yv[v][e]);
    mx = max(mx, (unsigned)xshfl<1>((int)mx));
    mx = max(mx, (unsigned)xshfl<2>((int)mx));
    const float sy = sc_of(mx);
    id_own = inv_of(mx);
    typedef _Float16 h4t __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int v = 0; v < CQ / 4; ++v) {
      const int k = qd * CQ + 4 * v, ks = k >> 5, kk = k & 31;
      h4t hv, lv;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float x = yv[v][e] * sy;
        hv[e] = (_Float16)x;
        lv[e] = (_Float16)(x - (float)hv[e]);
      }
      *reinterpret_cast<h4t*>(Dpl + frag((ks * 2 + 0) * 16 + tt, kk >> 3) + (kk & 7)) = hv;
      *reinterpret_cast<h4t*>(Dpl + frag((ks * 2 + 1) * 16 + tt, kk >> 3) + (kk & 7)) = lv;
    }
  }
  const float idx1 = __shfl(id_own, li << 2);
  const size_t tphys = (size_t)a.map[r0 + li];

  f4 yacc[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) yacc[q] = f4{0.f, 0.f, 0.f, 0.f};
  h8v fh[3], fl8[3];  // dq, dk, dv planes of the head (token li, 8 consecutive channels of the k-step)
  float fi[3] = {0.f, 0.f, 0.f};
  // fully unrolled at dim 96 (r05): as a loop, the two staging register sets were swapped by copies at the back
  // edge, which waited for every load in flight (vmcnt(0)) once per chunk (dim 192 unrolled spills)
  constexpr int ABU = C == 96 ? NSC : 1;
  constexpr bool kEpf = C == 96;  // epilogue operands prefetched inside the (unrolled) loop
  f4 exv[NQ], edv[NQ];
  float2 est = make_float2(0.f, 0.f);
#pragma unroll ABU
  for (int sc = 0; sc < NSC; ++sc) {
    const int h = sc >> 2, part = sc & 3;
    __syncthreads();
#define VV_ABWD_STORE(buf)                                                                                       \
  _Pragma("unroll") for (int i = 0; i < PC; ++i) {                                                              \
    const int e = tid + i * NT;                                                                                  \
    if (part == 0) {                                                                                             \
      const int r = e / (KS * 8), rem = e - r * (KS * 8);                                                        \
      *reinterpret_cast<u4v*>(Wc + ((rem >> 3) * 2 + ((rem >> 2) & 1)) * 32 * 32 + frag(r, rem & 3)) = rw[buf][i]; \
    } else {                                                                                                     \
      const int n = e >> 3, rem = e & 7;                                                                         \
      *reinterpret_cast<u4v*>(Wc + (rem >> 2) * C * 32 + frag(n, rem & 3)) = rw[buf][i];                         \
    }                                                                                                            \
  }
    if (sc & 1) {
      VV_ABWD_STORE(1)
    } else {
      VV_ABWD_STORE(0)
    }
    __syncthreads();
    VV_TR(TRR, 5 + 2 * (sc & 15));
    if (sc + 2 < NSC) {
      if (sc & 1) {
        VV_ABWD_LOAD(1, sc + 2)
      } else {
        VV_ABWD_LOAD(0, sc + 2)
      }
    }
    if (part == 0) {
      // this head's saved q, k, v rows and P (HBM), issued ahead of the dO GEMM
      f4 qv[2], kv[2], vv[2];
      float pv[4];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        qv[j] = sq[j];
        kv[j] = sk[j];
        vv[j] = sv3[j];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) pv[i] = sp[i];
      // dO^T rows c = 32 h + 16 j + 4 g4 + i, columns = tokens
      f4 acc[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const h8v yh = *reinterpret_cast<const h8v*>(Dpl + frag((ks * 2 + 0) * 16 + li, g4));
        const h8v yl = *reinterpret_cast<const h8v*>(Dpl + frag((ks * 2 + 1) * 16 + li, g4));
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const h8v wh = *reinterpret_cast<const h8v*>(Wc + (ks * 2 + 0) * 32 * 32 + frag(16 * j + li, g4));
          const h8v wl = *reinterpret_cast<const h8v*>(Wc + (ks * 2 + 1) * 32 * 32 + frag(16 * j + li, g4));
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, yh, acc[j], 0, 0, 0);
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, yl, acc[j], 0, 0, 0);
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, yh, acc[j], 0, 0, 0);
        }
      }
      f4 dov[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c = 16 * j + 4 * g4;
        const f4 sv = *reinterpret_cast<const f4*>(Tos + h * 32 + c);
#pragma unroll
        for (int i = 0; i < 4; ++i) dov[j][i] = acc[j][i] * (idx1 * sv[i]);
        *reinterpret_cast<f4*>(ob + li * BS + c) = dov[j];
        *reinterpret_cast<f4*>(qb + li * BS + c) = qv[j];
        *reinterpret_cast<f4*>(kb + li * BS + c) = kv[j];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) pb[(4 * g4 + i) * SS + li] = pv[i];
      // dP[t1][t2] = dO[t1] . v[t2]: dO (A, row = token) and v (B, column = token) fragments from registers
      unsigned mo = 0, mv = 0;
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          mo = amax(mo, dov[j][i]);
          mv = amax(mv, vv[j][i]);
        }
      mo = max(mo, (unsigned)xshfl<16>((int)mo));
      mo = max(mo, (unsigned)xshfl<32>((int)mo));
      mv = max(mv, (unsigned)xshfl<16>((int)mv));
      mv = max(mv, (unsigned)xshfl<32>((int)mv));
      const float so = sc_of(mo), svs = sc_of(mv);
      h8v oh, ol, vh, vl;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float x = dov[e >> 2][e & 3] * so, y = vv[e >> 2][e & 3] * svs;
        oh[e] = (_Float16)x;
        ol[e] = (_Float16)(x - (float)oh[e]);
        vh[e] = (_Float16)y;
        vl[e] = (_Float16)(y - (float)vh[e]);
      }
      f4 dp = {0.f, 0.f, 0.f, 0.f};
      dp = __builtin_amdgcn_mfma_f32_16x16x32_f16(ol, vh, dp, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_16x16x32_f16(oh, vl, dp, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_16x16x32_f16(oh, vh, dp, 0, 0, 0);
      const float io_ = inv_of(mo), iv_ = inv_of(mv);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float d = dp[i] * (__shfl(io_, 4 * g4 + i) * iv_);
        float rsum = pv[i] * d;
        rsum += xshfl<1>(rsum); rsum += xshfl<2>(rsum); rsum += xshfl<4>(rsum); rsum += xshfl<8>(rsum);
        sb[(4 * g4 + i) * SS + li] = pv[i] * (d - rsum);
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS stores are done
      __builtin_amdgcn_wave_barrier();
      // dq / dk / dv for token li, channels 8 g4 + e of the head
      float dq[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, dk[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f},
            dv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const float s_tu = sb[li * SS + u], s_ut = sb[u * SS + li], p_ut = pb[u * SS + li];
        const f4 k0 = *reinterpret_cast<const f4*>(kb + u * BS + 8 * g4), k1 = *reinterpret_cast<const f4*>(kb + u * BS + 8 * g4 + 4);
        const f4 q0 = *reinterpret_cast<const f4*>(qb + u * BS + 8 * g4), q1 = *reinterpret_cast<const f4*>(qb + u * BS + 8 * g4 + 4);
        const f4 o0 = *reinterpret_cast<const f4*>(ob + u * BS + 8 * g4), o1 = *reinterpret_cast<const f4*>(ob + u * BS + 8 * g4 + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          dq[e] += s_tu * k0[e];
          dq[4 + e] += s_tu * k1[e];
          dk[e] += s_ut * q0[e];
          dk[4 + e] += s_ut * q1[e];
          dv[e] += p_ut * o0[e];
          dv[4 + e] += p_ut * o1[e];
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        dq[e] *= a.scale;
        dk[e] *= a.scale;
      }
      // per (token, k-step) scales and planes of dq, dk, dv
#pragma unroll
      for (int p3 = 0; p3 < 3; ++p3) {
        const float* src = p3 == 0 ? dq : (p3 == 1 ? dk : dv);
        unsigned m = 0;
#pragma unroll
        for (int e = 0; e < 8; ++e) m = amax(m, src[e]);
        m = max(m, (unsigned)xshfl<16>((int)m));
        m = max(m, (unsigned)xshfl<32>((int)m));
        const float sf = sc_of(m);
        fi[p3] = inv_of(m);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float x = src[e] * sf;
          fh[p3][e] = (_Float16)x;
          fl8[p3][e] = (_Float16)(x - (float)fh[p3][e]);
        }
      }
    } else {
      if (part == 1 && h + 1 < H) VV_ABWD_SAVED(h + 1)
      // dY^T k-step (part - 1, h): rows c = 16 q + 4 g4 + i, columns = tokens
      const int p3 = part - 1;
      const h8v bh = p3 == 0 ? fh[0] : (p3 == 1 ? fh[1] : fh[2]);
      const h8v bl = p3 == 0 ? fl8[0] : (p3 == 1 ? fl8[1] : fl8[2]);
      const float bi = p3 == 0 ? fi[0] : (p3 == 1 ? fi[1] : fi[2]);
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const h8v wh = *reinterpret_cast<const h8v*>(Wc + frag(16 * q + li, g4));
        const h8v wl = *reinterpret_cast<const h8v*>(Wc + C * 32 + frag(16 * q + li, g4));
        f4 t = {0.f, 0.f, 0.f, 0.f};
        t = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, bh, t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, bl, t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, bh, t, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 4; ++i) yacc[q][i] += t[i] * bi;
      }
    }
    VV_TR(TRR, 6 + 2 * (sc & 15));
    if (kEpf && sc == NSC - 4) {
      // the epilogue's row operands, three chunks ahead (r05: loaded after the loop they were an exposed HBM round
      // trip, ~13 K cycles); the last head's attention part is done, so its registers are free
      est = *reinterpret_cast<const float2*>(G.stats + 2 * trow);
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        exv[q] = *reinterpret_cast<const f4*>(G.x + tphys * C + 16 * q + 4 * g4);
        edv[q] = *reinterpret_cast<const f4*>(G.out + tphys * C + 16 * q + 4 * g4);
      }
    }
  }
#undef VV_ABWD_STORE
#undef VV_ABWD_LOAD
#undef VV_ABWD_SAVED
  // ---- LN1 backward over the row (lane: token li, channels 16 q + 4 g4 + i) + the residual gradient ----
  const float2 st = kEpf ? est : *reinterpret_cast<const float2*>(G.stats + 2 * trow);
  const float mean = st.x, rstd = st.y;
  float o[NQ][4];
  f4 xv[NQ], gv[NQ];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int n = 16 * q + 4 * g4;
    const f4 sv = *reinterpret_cast<const f4*>(Tqs + n);
    xv[q] = kEpf ? exv[q] : *reinterpret_cast<const f4*>(G.x + tphys * C + n);
    gv[q] = *reinterpret_cast<const f4*>(G.n1g + n);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      o[q][i] = yacc[q][i] * sv[i];
      const float gd = gv[q][i] * o[q][i];
      s1 += gd;
      s2 += gd * ((xv[q][i] - mean) * rstd);
    }
  }
  s1 += xshfl<16>(s1);
  s1 += xshfl<32>(s1);
  s2 += xshfl<16>(s2);
  s2 += xshfl<32>(s2);
  const float m1 = s1 / (float)C, m2 = s2 / (float)C;
  f4 dv4[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) dv4[q] = kEpf ? edv[q] : *reinterpret_cast<const f4*>(G.out + tphys * C + 16 * q + 4 * g4);
  unsigned omx = 0;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    f4 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] = rstd * (gv[q][i] * o[q][i] - m1 - ((xv[q][i] - mean) * rstd) * m2) + dv4[q][i];
      omx = amax(omx, v[i]);
    }
    *reinterpret_cast<f4*>(G.out + tphys * C + 16 * q + 4 * g4) = v;
  }
  if (G.rs) {
    omx = max(omx, (unsigned)xshfl<16>((int)omx));
    omx = max(omx, (unsigned)xshfl<32>((int)omx));
    if (g4 == 0) G.rs[tphys] = sc_of(omx);
  }
  VV_TR(TRR, 63);
}

template <int C>
hipError_t launch_ablk_bwd(const AblkArgs& a, hipStream_t s) {
  constexpr int NW = 4, KS = C / 32;
  constexpr size_t lds = 2 * ((size_t)NW * KS * 2 * 16 * 32 + 64 * (size_t)C) +
                         4 * ((size_t)NW * (3 * 16 * 36 + 2 * 16 * 17) + 2 * C);
  if (hipError_t e = set_lds_limit((const void*)k_ablk_bwd<C>, lds)) return e;
  hipLaunchKernelGGL(k_ablk_bwd<C>, dim3(a.M / (16 * NW) * a.ngroups), dim3(256), lds, s, a);
  return hipGetLastError();
}

template <int C>
hipError_t launch_ablk_fwd(const AblkArgs& a, hipStream_t s) {
  constexpr int NW = 4, KS = C / 32, H = C / 32;
  constexpr size_t lds = 2 * ((size_t)NW * KS * 2 * 16 * 32 + 64 * (size_t)C) +
                         4 * ((size_t)NW * (16 * kAblkHBS + 16 * 16) + ((H * 49 + 3) & ~3) + 8 * C);
  // three dim-96 workgroups per CU: gfx950 allocates LDS in granules, and 3 x 53,836 B measured 2 per CU
  // (tools/tower_trace.py, r05) while 3 x 53,504 B (k_mlp<96>) gives 3; 53,760 B is the largest size both fit
  static_assert(C != 96 || lds <= 53760, "three dim-96 workgroups per CU");
  if (hipError_t e = set_lds_limit((const void*)k_ablk_fwd<C>, lds)) return e;
  hipLaunchKernelGGL(k_ablk_fwd<C>, dim3(a.M / (16 * NW) * a.ngroups), dim3(256), lds, s, a);
  return hipGetLastError();
}

}  // namespace

bool mlp_supported(int C, int M) { return (C == 96 || C == 192) && M > 0 && M % 64 == 0; }

static hipError_t mlp_run(const MlpArgs& a, hipStream_t s, bool fwd) {
  if (!mlp_supported(a.C, a.M) || a.ngroups <= 0 || a.ngroups > kMaxGroups) return hipErrorInvalidValue;
  if (a.hc != 0 && a.hc != 32 && a.hc != 64 && a.hc != 2) return hipErrorInvalidValue;
  for (int g = 0; g < a.ngroups; ++g) {
    const MlpGroup& G = a.g[g];
    if (!G.x || !G.gamma || !G.stats || !G.w1h || !G.w1s || !G.w2h || !G.w2s || !G.h1 || !G.out)
      return hipErrorInvalidValue;
    if (fwd ? (!G.beta || !G.b1 || !G.b2) : !G.dy) return hipErrorInvalidValue;
  }
  const int ph = prof_begin(s);
  const hipError_t e =
      a.C == 96    ? (fwd ? launch_mlp<96, 4, 32, true>(a, s) : launch_mlp<96, 4, 32, false>(a, s))
      : a.hc == 64 ? (fwd ? launch_mlp<192, 4, 64, true>(a, s) : launch_mlp<192, 4, 64, false>(a, s))
      : a.hc == 2  ? (fwd ? launch_mlp<192, 4, 32, true, 2>(a, s) : launch_mlp<192, 4, 32, false, 2>(a, s))
                   : (fwd ? launch_mlp<192, 4, 32, true>(a, s) : launch_mlp<192, 4, 32, false>(a, s));
  // 2 GEMMs of M x 4C x C per group; bytes: x1 / dx2 (+ out, + x1 bwd) and the 4C-wide pre-activation
  prof_end(ph, s, PC_TOWER, 4.0 * a.ngroups * a.M * 4.0 * a.C * a.C,
           (double)a.ngroups * a.M * 4.0 * (fwd ? 2.0 * a.C + 4.0 * a.C : 3.0 * a.C + 4.0 * a.C));
  return e;
}
hipError_t mlp_fwd(const MlpArgs& a, hipStream_t s) { return mlp_run(a, s, true); }

bool ablk_supported(int C, int heads, int ws, int M) {
  // dim 96 only: the dim-192 form (2048-token towers, 192 workgroups of one wave per SIMD) measured slower than the
  // unfused launches (r04: closure 8.62-8.65 vs 8.51-8.54 ms; r05: +0.4-0.9 %) and was removed in r06
  return C == 96 && heads == 3 && ws == 4 && M > 0 && M % 64 == 0;
}

hipError_t ablk_fwd(const AblkArgs& a, hipStream_t s) {
  if (!ablk_supported(a.C, a.heads, a.ws, a.M) || a.ngroups <= 0 || a.ngroups > kMaxGroups || !a.map)
    return hipErrorInvalidValue;
  for (int g = 0; g < a.ngroups; ++g) {
    const AblkGroup& G = a.g[g];
    if (!G.x || !G.n1g || !G.n1b || !G.stats || !G.wqh || !G.wqs || !G.wqb || !G.table || !G.qkv || !G.P ||
        !G.wph || !G.wps || !G.wpb || !G.out)
      return hipErrorInvalidValue;
  }
  const int ph = prof_begin(s);
  const hipError_t e = launch_ablk_fwd<96>(a, s);
  // qkv + proj GEMMs (2 M 4C C) and the window attention (4 M 16 C); bytes: x in, qkv + P + stats + x1 out
  prof_end(ph, s, PC_TOWER, a.ngroups * (8.0 * a.M * a.C * a.C + 64.0 * a.M * a.C),
           (double)a.ngroups * a.M * 4.0 * (a.C + 3 * a.C + 16 * a.heads + 2 + a.C));
  return e;
}

hipError_t ablk_bwd(const AblkArgs& a, hipStream_t s) {
  if (!ablk_supported(a.C, a.heads, a.ws, a.M) || a.ngroups <= 0 || a.ngroups > kMaxGroups || !a.map)
    return hipErrorInvalidValue;
  for (int g = 0; g < a.ngroups; ++g) {
    const AblkGroup& G = a.g[g];
    if (!G.x || !G.n1g || !G.stats || !G.qkv || !G.P || !G.wpth || !G.wpts || !G.wqth || !G.wqts || !G.out)
      return hipErrorInvalidValue;
  }
  const int ph = prof_begin(s);
  const hipError_t e = launch_ablk_bwd<96>(a, s);
  // proj^T and qkv^T GEMMs (2 M 4C C), the attention backward (8 M 16 C); bytes: gx in / out, qkv, P, x
  prof_end(ph, s, PC_TOWER, a.ngroups * (8.0 * a.M * a.C * a.C + 128.0 * a.M * a.C),
           (double)a.ngroups * a.M * 4.0 * (2 * a.C + 3 * a.C + 16 * a.heads + 2 + a.C));
  return e;
}
hipError_t mlp_bwd(const MlpArgs& a, hipStream_t s) { return mlp_run(a, s, false); }

#ifdef VV_TRACE
// tools/tower_trace.py: point the tower kernels' clock records at buf (8 regions x 2048 workgroups x 64 u64; null: off)
extern "C" __attribute__((visibility("default"))) int vv_debug_tower_trace(void* buf) {
  unsigned long long* p = static_cast<unsigned long long*>(buf);
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(vv_trace_buf), &p, sizeof(p));
}
#endif

}  // namespace vv

// Forecast network networks.LGUnet_all.LGUnet_all_1 (used by integrate(xa, forecast_model, 1),
// da_4dvar.py:1329, and at initialisation, :652): forward-only HIP engine.
//
// Differences from the networks_old engine (vv_engine.hip), all taken from the reference:
//   * Windowattn_block / SD_attn (networks/utils/Blocks.py:143-159, Attention.py:599-664): pre-norm blocks,
//     LayerNorm eps 1e-6 everywhere, 2-D RoPE on q and k over window-local (row, col) instead of a
//     relative-position bias (positional_encodings.py:230-270), shifted-window mask -inf (Attention.py:562),
//     applied only when the last shift > 0 and the window is narrower than the grid (:609-612);
//   * rectangular windows [wh, ww] with shift [wh/2, ww/2] on odd blocks (LGUnet_all.py:202, 288, 523);
//   * LG layer 0 is one window over the whole LG grid (LGUnet_all.py:689, 696) -> attention over Hg*Wg tokens
//     (16,200 at 0.25 degree): k_attn_flash streams keys through LDS with an online softmax (any N);
//   * any number of encoder levels; PatchEmbed conv and ConvTranspose2d with kernel > stride ((3,2)/(2,2)).
// Layout as in vv_engine.hip: tokens NHWC, towers group-major [G][B*H*W][C], every kernel runs all towers in
// one launch. Forward only: each stage keeps ONE activation buffer updated in place (the residual GEMM
// epilogues read and write the same element), and the encoder level buffers double as the decoder skips.
#include "vv_fcst.h"

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <unordered_map>

#include "vv_kernels.h"

namespace vvf {

using namespace vv;

// ============================================================================
// kernels
// ============================================================================
typedef float f4 __attribute__((ext_vector_type(4)));

struct RopeArgs {
  float* qkv[kMaxGroups];
  int rows, C, heads, hd, d1, d2, N;  // N = window tokens (row % N = window-local index)
  const float *c1, *s1, *c2, *s2;     // [N][d1], [N][d1], [N][d2], [N][d2]
  float scale;
};

// rope2 (positional_encodings.py:261-270) on q and k, then q * scale (Attention.py:634-639). Each thread rotates
// one pair (x[j], x[j + hd/2]); the products and sums are rounded separately, as torch evaluates them.
__global__ void k_rope(RopeArgs a) {
  const int half = a.hd / 2;
  const size_t per = (size_t)a.rows * a.heads * half;
  const int g = blockIdx.y;
  float* qkv = a.qkv[g];
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < per; t += (size_t)gridDim.x * blockDim.x) {
    const int j = (int)(t % half);
    const size_t rh = t / half;
    const int h = (int)(rh % a.heads);
    const size_t row = rh / a.heads;
    const int i = (int)(row % a.N);
    float c, s;
    if (j < a.d1) {
      c = a.c1[i * a.d1 + j];
      s = a.s1[i * a.d1 + j];
    } else {
      c = a.c2[i * a.d2 + (j - a.d1)];
      s = a.s2[i * a.d2 + (j - a.d1)];
    }
#pragma unroll
    for (int part = 0; part < 2; ++part) {
      float* base = qkv + row * 3 * a.C + part * a.C + h * a.hd;
      const float x0 = base[j], x1 = base[j + half];
      float r0 = __fsub_rn(__fmul_rn(x0, c), __fmul_rn(x1, s));
      float r1 = __fadd_rn(__fmul_rn(x1, c), __fmul_rn(x0, s));
      if (part == 0) {
        r0 = __fmul_rn(r0, a.scale);
        r1 = __fmul_rn(r1, a.scale);
      }
      base[j] = r0;
      base[j + half] = r1;
    }
  }
}

struct FlashArgs {
  const float* qkv[kMaxGroups];  // [nwin*N][3C], q already rotated and scaled, k rotated
  float* out[kMaxGroups];        // [nwin*N][C]
  int N, C, heads;
  int masked, H, wh, ww, sh, nWh, nWw;  // -inf mask by rolled-frame row label (Attention.py:533-562)
};

__device__ __forceinline__ int row_label(int R, int H, int wh, int sh) {
  return R < H - wh ? 0 : (R < H - sh ? 1 : 2);
}

// softmax(q k^T + mask) v for one (window, head, 32-query block): 8 lanes per query, each holding hd/8 of q and
// of the output accumulator; keys and values stream through LDS in tiles of 32 with an online softmax, so any
// window size works (16-token windows up to the 16,200-token global LG window).
template <int DPL>
__global__ __launch_bounds__(256) void k_attn_flash(FlashArgs a) {
  constexpr int QB = 32, KT = 32, HD = 8 * DPL, LDK = HD + 4;
  __shared__ __attribute__((aligned(16))) float Ks[KT * LDK];
  __shared__ __attribute__((aligned(16))) float Vs[KT * LDK];
  const int g = blockIdx.z, w = blockIdx.x;
  const int h = blockIdx.y % a.heads, qblk = blockIdx.y / a.heads;
  const int N = a.N, C = a.C;
  const size_t ld = 3 * (size_t)C;
  const float* base = a.qkv[g] + (size_t)w * N * ld;
  const int tid = threadIdx.x, lane8 = tid & 7, qi = qblk * QB + (tid >> 3);
  const bool active = qi < N;
  const int wr = (w / a.nWw) % a.nWh;
  const int lab_q = a.masked ? row_label(wr * a.wh + (active ? qi : 0) / a.ww, a.H, a.wh, a.sh) : 0;
  float qv[DPL], acc[DPL];
#pragma unroll
  for (int d = 0; d < DPL; ++d) {
    qv[d] = active ? base[(size_t)qi * ld + h * HD + lane8 * DPL + d] : 0.f;
    acc[d] = 0.f;
  }
  float m = -INFINITY, l = 0.f;
  for (int k0 = 0; k0 < N; k0 += KT) {
    for (int e = tid; e < KT * (HD / 4); e += 256) {
      const int r = e / (HD / 4), c4 = (e % (HD / 4)) * 4;
      const int j = k0 + r;
      f4 kv = {0.f, 0.f, 0.f, 0.f}, vv = {0.f, 0.f, 0.f, 0.f};
      if (j < N) {
        kv = *reinterpret_cast<const f4*>(base + (size_t)j * ld + C + h * HD + c4);
        vv = *reinterpret_cast<const f4*>(base + (size_t)j * ld + 2 * C + h * HD + c4);
      }
      *reinterpret_cast<f4*>(Ks + r * LDK + c4) = kv;
      *reinterpret_cast<f4*>(Vs + r * LDK + c4) = vv;
    }
    __syncthreads();
    float s[KT];
    float tmax = -INFINITY;
#pragma unroll
    for (int j = 0; j < KT; ++j) {
      const float* kr = Ks + j * LDK + lane8 * DPL;
      float part = 0.f;
#pragma unroll
      for (int d = 0; d < DPL; ++d) part = fmaf(qv[d], kr[d], part);
      part += __shfl_xor(part, 1);
      part += __shfl_xor(part, 2);
      part += __shfl_xor(part, 4);
      const int kj = k0 + j;
      bool ok = kj < N;
      if (a.masked && ok) ok = row_label(wr * a.wh + kj / a.ww, a.H, a.wh, a.sh) == lab_q;
      s[j] = ok ? part : -INFINITY;
      tmax = fmaxf(tmax, s[j]);
    }
    const float mn = fmaxf(m, tmax);
    if (mn != -INFINITY) {
      const float corr = (m == -INFINITY) ? 0.f : expf(m - mn);
      l *= corr;
#pragma unroll
      for (int d = 0; d < DPL; ++d) acc[d] *= corr;
#pragma unroll
      for (int j = 0; j < KT; ++j) {
        const float p = s[j] == -INFINITY ? 0.f : expf(s[j] - mn);
        l += p;
        const float* vr = Vs + j * LDK + lane8 * DPL;
#pragma unroll
        for (int d = 0; d < DPL; ++d) acc[d] = fmaf(p, vr[d], acc[d]);
      }
      m = mn;
    }
    __syncthreads();
  }
  if (active) {
    float* o = a.out[g] + ((size_t)w * N + qi) * C + h * HD + lane8 * DPL;
    const float inv = 1.f / l;
#pragma unroll
    for (int d = 0; d < DPL; ++d) o[d] = acc[d] * inv;
  }
}

// Small windows (N <= 96 tokens, hd <= 64; the [6, 12] = 72-token windows of every non-global stage): one
// workgroup per (window, head) holds q, k, v of the window and the N x N scores in LDS. S in 4x4 register blocks
// (8 float4 LDS reads per 64 FMAs), an exact row softmax (one wave per row, max then sum), O = P V in 4-row x
// float4 blocks; each score's exp is evaluated once (the streaming kernel above recomputes every exp on the 8
// lanes of a query and runs its online rescale per 32-key tile).
constexpr int kWinMaxN = 96, kWinMaxHd = 64;  // LDS <= 116 KB
__global__ __launch_bounds__(256) void k_attn_win(FlashArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smw[];
  const int g = blockIdx.z, w = blockIdx.x, h = blockIdx.y, tid = threadIdx.x;
  const int N = a.N, C = a.C, hd = C / a.heads, ld = hd + 4, ls = N + 1, nb = (N + 3) / 4;
  float* q = smw;
  float* k = q + N * ld;
  float* v = k + N * ld;
  float* S = v + N * ld;  // [N][N+1]
  const float* base = a.qkv[g] + (size_t)w * N * 3 * C + h * hd;
  const int q4 = hd / 4;
  for (int e = tid; e < N * q4; e += 256) {
    const int t = e / q4, c = (e - t * q4) * 4;
    const float* src = base + (size_t)t * 3 * C + c;
    *reinterpret_cast<f4*>(q + t * ld + c) = *reinterpret_cast<const f4*>(src);
    *reinterpret_cast<f4*>(k + t * ld + c) = *reinterpret_cast<const f4*>(src + C);
    *reinterpret_cast<f4*>(v + t * ld + c) = *reinterpret_cast<const f4*>(src + 2 * C);
  }
  __syncthreads();
  const int wr = (w / a.nWw) % a.nWh;
  for (int b = tid; b < nb * nb; b += 256) {
    const int i0 = (b / nb) * 4, j0 = (b % nb) * 4;
    float acc[4][4] = {};
    for (int d = 0; d < hd; d += 4) {
      f4 qa[4], ka[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        qa[r] = *reinterpret_cast<const f4*>(q + min(i0 + r, N - 1) * ld + d);
        ka[r] = *reinterpret_cast<const f4*>(k + min(j0 + r, N - 1) * ld + d);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          acc[r][c] += qa[r][0] * ka[c][0] + qa[r][1] * ka[c][1] + qa[r][2] * ka[c][2] + qa[r][3] * ka[c][3];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + r;
      if (i >= N) break;
      const int li = a.masked ? row_label(wr * a.wh + i / a.ww, a.H, a.wh, a.sh) : 0;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int j = j0 + c;
        if (j >= N) break;
        const bool ok = !a.masked || row_label(wr * a.wh + j / a.ww, a.H, a.wh, a.sh) == li;
        S[i * ls + j] = ok ? acc[r][c] : -INFINITY;
      }
    }
  }
  __syncthreads();
  // row softmax (Attention.py:563: softmax over keys; -inf entries give exact zeros)
  const int wave = tid >> 6, lane = tid & 63;
  for (int i = wave; i < N; i += 4) {
    float* row = S + i * ls;
    float mx = -INFINITY;
    for (int j = lane; j < N; j += 64) mx = fmaxf(mx, row[j]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    float sum = 0.f;
    for (int j = lane; j < N; j += 64) {
      const float e = expf(row[j] - mx);
      row[j] = e;
      sum += e;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
    const float inv = 1.f / sum;
    for (int j = lane; j < N; j += 64) row[j] *= inv;
  }
  __syncthreads();
  float* ob = a.out[g] + (size_t)w * N * C + h * hd;
  for (int b = tid; b < nb * q4; b += 256) {
    const int i0 = (b / q4) * 4, c = (b % q4) * 4;
    f4 acc[4] = {};
    for (int j = 0; j < N; ++j) {
      const f4 vv = *reinterpret_cast<const f4*>(v + j * ld + c);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = S[min(i0 + r, N - 1) * ls + j];
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[r][e] += p * vv[e];
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (i0 + r < N) *reinterpret_cast<f4*>(ob + (size_t)(i0 + r) * C + c) = acc[r];
  }
}

// The same window attention on the exact-f32 MFMA (v_mfma_f32_16x16x4_f32: fp32 products, fp32 accumulation, as
// torch's fp32 matmul), with rope2 + the q scale fused into the LDS staging (the same rounded products and sums as
// k_rope, so q and k are bit-identical to the unfused path). One workgroup per (window, head), one wave per
// 16-query tile. Per tile: S^T = K Q^T (keys on the accumulator rows, queries on the lanes; the NT key tiles are
// independent accumulators, so the MFMA chain never waits on itself), the -inf row-label mask from per-lane label
// bitmasks built once per wave, softmax over the keys (registers x the 4 lane groups), then O^T = V^T P^T with
// P^T straight from the score registers: the k index of each 16x16x4 step is the lane group, so the step over
// register r pairs keys 4 g + r with V rows 4 g + r read from LDS. N <= 96 (kWinMaxN), hd a multiple of 16 <= 64.
template <int HD, int NT>
__global__ __launch_bounds__(64 * NT) void k_attn_win_mf(FlashArgs a, RopeArgs ra) {
  typedef float f4m __attribute__((ext_vector_type(4)));
  extern __shared__ __attribute__((aligned(16))) float smf[];
  const int g = blockIdx.z, w = blockIdx.x, h = blockIdx.y, tid = threadIdx.x, nth = blockDim.x;
  const int lane = tid & 63, wave = tid >> 6;
  constexpr int hd = HD, ld = HD + 1, q4 = HD / 4, half = HD / 2;
  constexpr int NP = NT * 16;
  const int N = a.N, C = a.C;
  float* q = smf;
  float* k = q + NP * ld;
  float* v = k + NP * ld;
  int* lab = reinterpret_cast<int*>(v + NP * ld);  // row label per token, -1 past N
  const int wr = (w / a.nWw) % a.nWh, li = lane & 15, gq = lane >> 4;
  for (int t = tid; t < NP; t += nth)
    lab[t] = t >= N ? -1 : (a.masked ? row_label(wr * a.wh + t / a.ww, a.H, a.wh, a.sh) : 0);
  const float* base = a.qkv[g] + (size_t)w * N * 3 * C + h * hd;
  for (int e = tid; e < NP * q4; e += nth) {
    const int t = e / q4, c = (e - t * q4) * 4;
    f4 x = {0.f, 0.f, 0.f, 0.f}, y = x, z = x;
    if (t < N) {
      const float* src = base + (size_t)t * 3 * C + c;
      x = *reinterpret_cast<const f4*>(src);
      y = *reinterpret_cast<const f4*>(src + C);
      z = *reinterpret_cast<const f4*>(src + 2 * C);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      q[t * ld + c + i] = x[i];
      k[t * ld + c + i] = y[i];
      v[t * ld + c + i] = z[i];
    }
  }
  __syncthreads();
  if (ra.c1) {  // rope2 (positional_encodings.py:261-270) on q and k, then q * scale, as k_rope
    for (int e = tid; e < N * half; e += nth) {
      const int t = e / half, j = e - t * half;
      float c, sn;
      if (j < ra.d1) {
        c = ra.c1[t * ra.d1 + j];
        sn = ra.s1[t * ra.d1 + j];
      } else {
        c = ra.c2[t * ra.d2 + (j - ra.d1)];
        sn = ra.s2[t * ra.d2 + (j - ra.d1)];
      }
      float* pq = q + t * ld;
      float* pk = k + t * ld;
      float x0 = pq[j], x1 = pq[j + half];
      pq[j] = __fmul_rn(__fsub_rn(__fmul_rn(x0, c), __fmul_rn(x1, sn)), ra.scale);
      pq[j + half] = __fmul_rn(__fadd_rn(__fmul_rn(x1, c), __fmul_rn(x0, sn)), ra.scale);
      x0 = pk[j];
      x1 = pk[j + half];
      pk[j] = __fsub_rn(__fmul_rn(x0, c), __fmul_rn(x1, sn));
      pk[j + half] = __fadd_rn(__fmul_rn(x1, c), __fmul_rn(x0, sn));
    }
    __syncthreads();
  }
  float* ob = a.out[g] + (size_t)w * N * C + h * hd;
  const int qt = wave;  // one wave per query tile (blockDim = 64 NT)
  const int qi = 16 * qt + li;
  const int lq = lab[min(qi, N - 1)];
  float qf[q4];
#pragma unroll
  for (int s4 = 0; s4 < q4; ++s4)
    qf[s4] = q[qi * ld + 4 * s4 + gq];
  f4m sc[NT];
#pragma unroll
  for (int kt = 0; kt < NT; ++kt) sc[kt] = f4m{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s4 = 0; s4 < q4; ++s4) {
#pragma unroll
    for (int kt = 0; kt < NT; ++kt)
      sc[kt] = __builtin_amdgcn_mfma_f32_16x16x4f32(k[(16 * kt + li) * ld + 4 * s4 + gq], qf[s4], sc[kt], 0, 0, 0);
  }
  float mx = -INFINITY;
#pragma unroll
  for (int kt = 0; kt < NT; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float x = lab[16 * kt + 4 * gq + r] == lq ? sc[kt][r] : -INFINITY;
        sc[kt][r] = x;
        mx = fmaxf(mx, x);
      }
  mx = fmaxf(mx, __shfl_xor(mx, 16));
  mx = fmaxf(mx, __shfl_xor(mx, 32));
  float sum = 0.f;
#pragma unroll
  for (int kt = 0; kt < NT; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float e = expf(sc[kt][r] - mx);
        sc[kt][r] = e;
        sum += e;
      }
  sum += __shfl_xor(sum, 16);
  sum += __shfl_xor(sum, 32);
  const float inv = 1.f / sum;
#pragma unroll
  for (int kt = 0; kt < NT; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) sc[kt][r] *= inv;
  // O^T tiles: rows d = 16 dt + 4 gq + r, columns = queries; the hd/16 tiles are independent accumulators
  constexpr int DT = HD / 16;
  f4m o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt] = f4m{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kt = 0; kt < NT; ++kt) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float* vr = v + (16 * kt + 4 * gq + r) * ld + li;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(vr[16 * dt], sc[kt][r], o[dt], 0, 0, 0);
    }
  }
  if (qi < N)
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
      *reinterpret_cast<f4*>(ob + (size_t)qi * C + 16 * dt + 4 * gq) = f4{o[dt][0], o[dt][1], o[dt][2], o[dt][3]};
}

bool win_mf_ok(int N, int hd, const vv::Tuning& TU) {
  return N <= kWinMaxN && hd <= kWinMaxHd && hd % 16 == 0 && TU.win_attn && TU.win_mfma;
}

struct ConvArgs {
  int B, Cimg, Himg, Wimg;  // image (B, Cimg, Himg, Wimg)
  int Ho, Wo, Ctok, kh, kw, sh, sw;
  int climit, Ctot;         // convT: channel limit, channels of the output image
  const float* img;         // conv input
  float* img_out;           // convT output
  const float* w[kMaxGroups];
  const float* bias[kMaxGroups];
  const float* pos[kMaxGroups];  // conv: absolute_pos_embed [Ho*Wo][Ctok]
  float* tok[kMaxGroups];        // conv out / convT in: [B*Ho*Wo][Ctok]
  int cin_off[kMaxGroups], cin[kMaxGroups];
  int mean_off[kMaxGroups], std_off[kMaxGroups], cout[kMaxGroups];
};

// PatchEmbed (LGUnet_all.py:42-50): Conv2d(k=(kh,kw), stride=(sh,sw)) -> tokens, + absolute_pos_embed
__global__ void k_conv_patch(ConvArgs a) {
  const int g = blockIdx.y;
  const size_t total = (size_t)a.B * a.Ho * a.Wo * a.Ctok;
  const int cin = a.cin[g];
  const float* w = a.w[g];
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < total; t += (size_t)gridDim.x * blockDim.x) {
    const int co = (int)(t % a.Ctok);
    const size_t tok = t / a.Ctok;
    const int pix = (int)(tok % ((size_t)a.Ho * a.Wo));
    const int b = (int)(tok / ((size_t)a.Ho * a.Wo));
    const int oy = pix / a.Wo, ox = pix % a.Wo;
    float acc = 0.f;
    for (int ci = 0; ci < cin; ++ci) {
      const float* im = a.img + (((size_t)b * a.Cimg + a.cin_off[g] + ci) * a.Himg + (size_t)oy * a.sh) * a.Wimg +
                        (size_t)ox * a.sw;
      const float* wk = w + ((size_t)co * cin + ci) * a.kh * a.kw;
      for (int ky = 0; ky < a.kh; ++ky)
        for (int kx = 0; kx < a.kw; ++kx) acc = fmaf(wk[ky * a.kw + kx], im[(size_t)ky * a.Wimg + kx], acc);
    }
    a.tok[g][t] = (acc + a.bias[g][co]) + a.pos[g][(size_t)pix * a.Ctok + co];
  }
}

// ConvTranspose2d(k=(kh,kw), stride=(sh,sw)) + quirk Q2 placement of the mean / std halves (LGUnet_all.py:624-650)
__global__ void k_convT(ConvArgs a) {
  const int g = blockIdx.z, co = blockIdx.y;
  const int cout = a.cout[g];
  if (co >= cout) return;
  const int oc = co < cout / 2 ? a.mean_off[g] + co : a.std_off[g] + (co - cout / 2);
  if (a.climit > 0 && oc >= a.climit) return;
  const size_t npix = (size_t)a.B * a.Himg * a.Wimg;
  const float* w = a.w[g];
  for (size_t p = blockIdx.x * (size_t)blockDim.x + threadIdx.x; p < npix; p += (size_t)gridDim.x * blockDim.x) {
    const int x = (int)(p % a.Wimg);
    const int y = (int)((p / a.Wimg) % a.Himg);
    const int b = (int)(p / ((size_t)a.Himg * a.Wimg));
    float acc = a.bias[g][co];
    for (int ky = 0; ky < a.kh; ++ky) {
      const int yy = y - ky;
      if (yy < 0 || yy % a.sh) continue;
      const int iy = yy / a.sh;
      if (iy >= a.Ho) continue;
      for (int kx = 0; kx < a.kw; ++kx) {
        const int xx = x - kx;
        if (xx < 0 || xx % a.sw) continue;
        const int ix = xx / a.sw;
        if (ix >= a.Wo) continue;
        const float* tr = a.tok[g] + (((size_t)b * a.Ho + iy) * a.Wo + ix) * a.Ctok;
        const float* wk = w + ((size_t)co * a.kh + ky) * a.kw + kx;
        const size_t wstride = (size_t)cout * a.kh * a.kw;
        for (int ci = 0; ci < a.Ctok; ++ci) acc = fmaf(tr[ci], wk[ci * wstride], acc);
      }
    }
    a.img_out[(((size_t)b * a.Ctot + oc) * a.Himg + y) * a.Wimg + x] = acc;
  }
}

// PatchEmbed as a GEMM: im2col rows [pix][k], k = (ci*kh + ky)*kw + kx, zero-padded to Kp (multiple of 32)
__global__ void k_im2col(ConvArgs a, float* col0, int Kp, size_t gstride) {
  const int g = blockIdx.y;
  const int cin = a.cin[g], kk = a.kh * a.kw, K = cin * kk;
  const size_t total = (size_t)a.B * a.Ho * a.Wo * Kp;
  float* col = col0 + g * gstride;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < total; t += (size_t)gridDim.x * blockDim.x) {
    const int k = (int)(t % Kp);
    const size_t pix = t / Kp;
    float v = 0.f;
    if (k < K) {
      const int ci = k / kk, ky = (k % kk) / a.kw, kx = k % a.kw;
      const int b = (int)(pix / ((size_t)a.Ho * a.Wo));
      const int p = (int)(pix % ((size_t)a.Ho * a.Wo));
      const int oy = p / a.Wo, ox = p % a.Wo;
      v = a.img[(((size_t)b * a.Cimg + a.cin_off[g] + ci) * a.Himg + (size_t)oy * a.sh + ky) * a.Wimg +
                (size_t)ox * a.sw + kx];
    }
    col[t] = v;
  }
}

// ConvTranspose2d after the GEMM Y[pix][(co*kh + ky)*kw + kx] = tok[pix] . w[:, co, ky, kx]: col2im gather of
// the (overlapping) taps + bias, quirk Q2 channel placement
__global__ void k_col2im(ConvArgs a, const float* Y0, int ldy, size_t gstride) {
  const int g = blockIdx.z, co = blockIdx.y;
  const int cout = a.cout[g];
  if (co >= cout) return;
  const int oc = co < cout / 2 ? a.mean_off[g] + co : a.std_off[g] + (co - cout / 2);
  if (a.climit > 0 && oc >= a.climit) return;
  const float* Y = Y0 + g * gstride;
  const size_t npix = (size_t)a.B * a.Himg * a.Wimg;
  const float b0 = a.bias[g][co];
  for (size_t p = blockIdx.x * (size_t)blockDim.x + threadIdx.x; p < npix; p += (size_t)gridDim.x * blockDim.x) {
    const int x = (int)(p % a.Wimg);
    const int y = (int)((p / a.Wimg) % a.Himg);
    const int b = (int)(p / ((size_t)a.Himg * a.Wimg));
    float acc = 0.f;
    for (int ky = 0; ky < a.kh; ++ky) {
      const int yy = y - ky;
      if (yy < 0 || yy % a.sh) continue;
      const int iy = yy / a.sh;
      if (iy >= a.Ho) continue;
      for (int kx = 0; kx < a.kw; ++kx) {
        const int xx = x - kx;
        if (xx < 0 || xx % a.sw) continue;
        const int ix = xx / a.sw;
        if (ix >= a.Wo) continue;
        acc += Y[(((size_t)b * a.Ho + iy) * a.Wo + ix) * ldy + (co * a.kh + ky) * a.kw + kx];
      }
    }
    a.img_out[(((size_t)b * a.Ctot + oc) * a.Himg + y) * a.Wimg + x] = acc + b0;
  }
}

// PatchEmbed and ConvTranspose2d of LGUnet_all_1 (patch (kh, 2), stride (2, 2)) on the exact-f32 MFMA
// (v_mfma_f32_16x16x4_f32, fp32 products and sums; only the summation order differs from torch's conv), reading the
// image / writing the pixels directly: no im2col / col2im buffer (the 0.25-degree model's im2col rows were 600 MB).
// Fragment layout and the k permutation of the float4 reads as the decoder's k_p2t_mf / k_t2p_mf (vv_ops.hip).
//
// k_fc_patch_mf: 64 tokens per workgroup (4 waves x 16); their kh x 2 x cin patches staged in LDS ([t][KP],
// k = (ci kh + ky) 2 + kx as the im2col rows), each thread loading the two horizontally adjacent pixels of a patch
// row for its token (all of a thread's loads in flight before its LDS stores); Wp [C0][Kp] staged in LDS;
// tok[t][c] = (sum_k X[t][k] W[c][k] + bias[c]) + pos[t % (Ho Wo)][c].
constexpr int kFcKP = 96;    // patch taps, padded to 16 (cin kh kw <= 96)
// stage n floats f(i) into LDS at d(i) in batches of 16 loads in flight per thread (a load issued behind an LDS store
// of the previous one would expose one memory latency per element)
template <typename F, typename D>
__device__ __forceinline__ void stage_batched(int n, F f, D d) {
  for (int i0 = threadIdx.x; i0 < n; i0 += 256 * 16) {
    float v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = i0 + 256 * r < n ? f(i0 + 256 * r) : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (i0 + 256 * r < n) d(i0 + 256 * r, v[r]);
  }
}

template <int C0>
__global__ __launch_bounds__(256) void k_fc_patch_mf(ConvArgs a, int Kp) {  // a.w[g]: Wp [C0][Kp]
  extern __shared__ __attribute__((aligned(16))) float sm[];
  constexpr int kFcC0 = C0, C = C0;
  const int g = blockIdx.y;
  const int ntok = a.B * a.Ho * a.Wo, K = a.cin[g] * a.kh * 2;
  const int KP = (K + 15) / 16 * 16, KS = KP + 4;
  float* Xs = sm;            // [64][KS]
  float* Wsm = Xs + 64 * KS; // [C][KS]
  const int t0 = blockIdx.x * 64;
  {
    const int q = threadIdx.x & 1, t = (threadIdx.x >> 1) & 63, half = threadIdx.x >> 7;
    const int tok = min(t0 + t, ntok - 1);
    const int b = tok / (a.Ho * a.Wo), rem = tok - b * a.Ho * a.Wo, oy = rem / a.Wo, ox = rem - oy * a.Wo;
    const size_t plane = (size_t)a.Himg * a.Wimg;
    const float* base = a.img + ((size_t)b * a.Cimg + a.cin_off[g]) * plane + (size_t)(oy * a.sh) * a.Wimg + ox * 2 + q;
    constexpr int NR = kFcKP / 4;  // patch rows (ci, ky) per thread at most
    float v[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int rest = half + 2 * r;  // = ci kh + ky
      const int ci = rest / a.kh, ky = rest - ci * a.kh;
      v[r] = (rest * 2 < K && t0 + t < ntok) ? base[(size_t)ci * plane + (size_t)ky * a.Wimg] : 0.f;
    }
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int rest = half + 2 * r;
      if (rest * 2 < KP) Xs[t * KS + rest * 2 + q] = v[r];
    }
  }
  {
    const float* W = a.w[g];
    stage_batched(C * KP, [&](int i) { const int c = i / KP, j = i - c * KP; return j < K ? W[(size_t)c * Kp + j] : 0.f; },
                  [&](int i, float v) { const int c = i / KP, j = i - c * KP; Wsm[c * KS + j] = v; });
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 15, gq = lane >> 4;
  typedef float fr4 __attribute__((ext_vector_type(4)));
  constexpr int NTM = kFcC0 / 16;
  const int nt = (C + 15) / 16;
  fr4 acc[NTM];
  const float* xr = Xs + (wave * 16 + li) * KS + 4 * gq;
#pragma unroll
  for (int n = 0; n < NTM; ++n) {
    acc[n] = fr4{0.f, 0.f, 0.f, 0.f};
    if (n < nt) {
      const float* wr = Wsm + min(n * 16 + li, C - 1) * KS + 4 * gq;
      for (int s4 = 0; s4 < KP; s4 += 16) {
        const f4 xa = *reinterpret_cast<const f4*>(xr + s4);
        const f4 wb = *reinterpret_cast<const f4*>(wr + s4);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[e], wb[e], acc[n], 0, 0, 0);
      }
    }
  }
  const int tk0 = t0 + wave * 16 + 4 * gq;
  float ex[NTM][4];
#pragma unroll
  for (int n = 0; n < NTM; ++n) {  // every epilogue load before the first store
    const int c = min(n * 16 + li, C - 1);
    const float bias = a.bias[g][c];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int tok = min(tk0 + r, ntok - 1);
      ex[n][r] = n < nt ? a.pos[g][(size_t)(tok % (a.Ho * a.Wo)) * C + c] : 0.f;
      acc[n][r] += bias;
    }
  }
#pragma unroll
  for (int n = 0; n < NTM; ++n) {
    const int c = n * 16 + li;
    if (n >= nt || c >= C) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (tk0 + r < ntok) a.tok[g][(size_t)(tk0 + r) * C + c] = ex[n][r] + acc[n][r];
  }
}

// k_fc_convT_mf: ConvTranspose2d (kernel (kh, 2), stride (2, 2)) gathered per OUTPUT pixel row y, so overlapping taps
// (kh = 3: rows 2 iy + 2 = 2 (iy + 1) + 0) sum in registers without atomics: out[oc(co)][y][2 ix + kx] = bias[co] +
// sum over (iy, ky) with y = 2 iy + ky of sum_c tok[iy][ix][c] W2[(co kh + ky) 2 + kx][c]. A workgroup (4 waves of 16
// token columns) covers 8 output rows of one parity with the weights of that parity's taps staged in LDS as
// [tap][j = co 2 + kx][c]; each wave: per row, one MFMA chain per 16 outputs j over the taps' K = C0 each; stores of
// two horizontally adjacent pixels (kx = 0, 1) per lane, consecutive lanes = consecutive pixels.
constexpr int kFcRows = 8;
template <int C0>
__global__ __launch_bounds__(256) void k_fc_convT_mf(ConvArgs a) {  // a.w[g]: W2 [(co kh + ky) kw + kx][C0]
  extern __shared__ __attribute__((aligned(16))) float sm[];
  constexpr int kFcC0 = C0, C = C0, CS = C0 + 4;
  const int g = blockIdx.z, cout = a.cout[g];
  const int par = blockIdx.y & 1, y0 = par + 2 * kFcRows * (blockIdx.y >> 1);
  const int ntap = (a.kh - par + 1) / 2;  // taps ky = par, par + 2, ...
  const int J = 2 * cout, JP = (J + 15) / 16 * 16;
  // stage [tap][j][c] for ky = par + 2 tap: W2 row (co kh + ky) 2 + kx
  const float* W = a.w[g];
  stage_batched(ntap * JP * C,
                [&](int i) {
                  const int c = i % C, jj = (i / C) % JP, tap = i / (C * JP);
                  return jj < J ? W[((size_t)((jj >> 1) * a.kh + par + 2 * tap) * 2 + (jj & 1)) * C + c] : 0.f;
                },
                [&](int i, float v) {
                  const int c = i % C, r = i / C;  // r = tap JP + jj
                  sm[r * CS + c] = v;
                });
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 15, gq = lane >> 4;
  const int ix = (blockIdx.x * 4 + wave) * 16 + li;
  if ((blockIdx.x * 4 + wave) * 16 >= a.Wo) return;
  const bool okx = ix < a.Wo;
  typedef float fr4 __attribute__((ext_vector_type(4)));
  constexpr int NMT = 64 / 16;  // j tiles: 2 cout <= 64
  const int nmt = JP / 16;
  for (int yy = 0; yy < kFcRows; ++yy) {
    const int y = y0 + 2 * yy;
    if (y >= a.Himg) break;
    for (int b = 0; b < a.B; ++b) {
      fr4 acc[NMT];
#pragma unroll
      for (int m = 0; m < NMT; ++m) acc[m] = fr4{0.f, 0.f, 0.f, 0.f};
      for (int tap = 0; tap < ntap; ++tap) {
        const int ky = par + 2 * tap, iy2 = y - ky;
        if (iy2 < 0 || iy2 >= 2 * a.Ho) continue;
        const int iy = iy2 >> 1;
        const float* tr = a.tok[g] + (((size_t)b * a.Ho + iy) * a.Wo + (okx ? ix : 0)) * C + 4 * gq;
        f4 yv[kFcC0 / 16];
#pragma unroll
        for (int s = 0; s < kFcC0 / 16; ++s) {
          f4 v = {0.f, 0.f, 0.f, 0.f};
          if (16 * s < C) v = *reinterpret_cast<const f4*>(tr + 16 * s);
          yv[s] = v;
        }
#pragma unroll
        for (int m = 0; m < NMT; ++m) {
          if (m < nmt) {
            const float* wr = sm + (tap * JP + m * 16 + li) * CS + 4 * gq;
#pragma unroll
            for (int s = 0; s < kFcC0 / 16; ++s) {
              if (16 * s < C) {
                const f4 wa = *reinterpret_cast<const f4*>(wr + 16 * s);
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[e], yv[s][e], acc[m], 0, 0, 0);
              }
            }
          }
        }
      }
      // lane holds j = 16 m + 4 gq + r: co = 8 m + 2 gq + r / 2, kx = r % 2
      float bs[NMT][2];
#pragma unroll
      for (int m = 0; m < NMT; ++m)
#pragma unroll
        for (int h = 0; h < 2; ++h) bs[m][h] = a.bias[g][min(8 * m + 2 * gq + h, cout - 1)];
      if (!okx) continue;
#pragma unroll
      for (int m = 0; m < NMT; ++m) {
        if (m >= nmt) continue;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int co = 8 * m + 2 * gq + h;
          if (co >= cout) continue;
          const int oc = co < cout / 2 ? a.mean_off[g] + co : a.std_off[g] + (co - cout / 2);
          if (a.climit > 0 && oc >= a.climit) continue;
          float* o = a.img_out + (((size_t)b * a.Ctot + oc) * a.Himg + y) * a.Wimg + 2 * ix;
          *reinterpret_cast<float2*>(o) = make_float2(acc[m][2 * h] + bs[m][h], acc[m][2 * h + 1] + bs[m][h]);
        }
      }
    }
  }
}

// Global-window attention as GEMMs (LG layer 0, Hg*Wg tokens): V^T per head, zero-padded to Np columns
__global__ void k_vt(const float* qkv, float* vt, int N, int Np, int C, int heads, int hd) {
  const size_t total = (size_t)heads * hd * Np;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < total; t += (size_t)gridDim.x * blockDim.x) {
    const int j = (int)(t % Np);
    const size_t hdrow = t / Np;
    const int d = (int)(hdrow % hd), h = (int)(hdrow / hd);
    vt[t] = j < N ? qkv[(size_t)j * 3 * C + 2 * C + h * hd + d] : 0.f;
  }
}

// row softmax of S [rows][Np] (first N columns), in place; pad columns set to 0 (they feed the P.V GEMM's K)
// one row held in registers (Np <= 256 * 4 * RV): one read and one write of the row, each exp once
constexpr int kSmRV = 16;
__global__ __launch_bounds__(256) void k_softmax_rows_reg(float* S, int N, int Np) {
  __shared__ float red[8];
  float* row = S + (size_t)blockIdx.x * Np;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  f4 x[kSmRV];
  float mx = -INFINITY;
#pragma unroll
  for (int i = 0; i < kSmRV; ++i) {
    const int j = (tid + 256 * i) * 4;
    x[i] = j < Np ? *reinterpret_cast<const f4*>(row + j) : f4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (j + e >= N) x[i][e] = -INFINITY;  // padding columns [N, Np)
      mx = fmaxf(mx, x[i][e]);
    }
  }
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  if (lane == 0) red[wv] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < kSmRV; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      x[i][e] = expf(x[i][e] - mx);  // exp(-inf) = 0 for the padding
      sum += x[i][e];
    }
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
  if (lane == 0) red[4 + wv] = sum;
  __syncthreads();
  const float inv = 1.f / ((red[4] + red[5]) + (red[6] + red[7]));
#pragma unroll
  for (int i = 0; i < kSmRV; ++i) {
    const int j = (tid + 256 * i) * 4;
    if (j < Np) {
      f4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = x[i][e] * inv;
      *reinterpret_cast<f4*>(row + j) = o;
    }
  }
}

__global__ __launch_bounds__(256) void k_softmax_rows(float* S, int N, int Np) {
  __shared__ float red[8];
  float* row = S + (size_t)blockIdx.x * Np;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  float mx = -INFINITY;
  for (int j = tid; j < N; j += 256) mx = fmaxf(mx, row[j]);
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  if (lane == 0) red[wv] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  float sum = 0.f;
  for (int j = tid; j < N; j += 256) sum += expf(row[j] - mx);
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
  __syncthreads();
  if (lane == 0) red[4 + wv] = sum;
  __syncthreads();
  const float inv = 1.f / ((red[4] + red[5]) + (red[6] + red[7]));
  for (int j = tid; j < Np; j += 256) row[j] = j < N ? expf(row[j] - mx) * inv : 0.f;
}

__global__ void k_norm_resample(const float* x, float* y, const int* di, const int* dj, const float* mean,
                                const float* sd, int C, int Hs, int Ws, int Hl, int Wl) {
  const size_t n = (size_t)C * Hl * Wl;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < n; t += (size_t)gridDim.x * blockDim.x) {
    const int j = (int)(t % Wl);
    const int i = (int)((t / Wl) % Hl);
    const int c = (int)(t / ((size_t)Hl * Wl));
    const int si = di ? di[i] : i, sj = dj ? dj[j] : j;
    y[t] = __fdiv_rn(__fsub_rn(x[((size_t)c * Hs + si) * Ws + sj], mean[c]), sd[c]);
  }
}

__global__ void k_denorm_resample(const float* net, int cstride, float* out, const int* mi, const int* mj,
                                  const float* mean, const float* sd, int C, int Hs, int Ws, int Hl, int Wl) {
  const size_t n = (size_t)C * Hs * Ws;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < n; t += (size_t)gridDim.x * blockDim.x) {
    const int j = (int)(t % Ws);
    const int i = (int)((t / Ws) % Hs);
    const int c = (int)(t / ((size_t)Hs * Ws));
    const int si = mi ? mi[i] : i, sj = mj ? mj[j] : j;
    out[t] = __fadd_rn(__fmul_rn(net[((size_t)c * Hl + si) * Wl + sj], sd[c]), mean[c]);
  }
}

static int grid_for(size_t n) { return (int)std::min<size_t>((n + 255) / 256, 65536); }

hipError_t normalize_resample(const float* x, float* net_in, const int* di, const int* dj, const float* mean,
                              const float* std_, int C, int Hs, int Ws, int Hl, int Wl, hipStream_t st) {
  hipLaunchKernelGGL(k_norm_resample, dim3(grid_for((size_t)C * Hl * Wl)), dim3(256), 0, st, x, net_in, di, dj,
                     mean, std_, C, Hs, Ws, Hl, Wl);
  return hipGetLastError();
}

hipError_t denormalize_resample(const float* net, int net_cstride, float* out, const int* mi, const int* mj,
                                const float* mean, const float* std_, int C, int Hs, int Ws, int Hl, int Wl,
                                hipStream_t st) {
  hipLaunchKernelGGL(k_denorm_resample, dim3(grid_for((size_t)C * Hs * Ws)), dim3(256), 0, st, net, net_cstride,
                     out, mi, mj, mean, std_, C, Hs, Ws, Hl, Wl);
  return hipGetLastError();
}

// ============================================================================
// model
// ============================================================================
namespace {

int ferr(std::string& err, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  err = buf;
  return code;
}

#define FH(expr)                                                                                         \
  do {                                                                                                   \
    hipError_t e_ = (expr);                                                                              \
    if (e_ != hipSuccess) return ferr(err, (int)e_, "%s:%d %s -> %s", __FILE__, __LINE__, #expr,         \
                                      hipGetErrorString(e_));                                            \
  } while (0)

struct FCfg {
  vv_lgunet_config raw;
  int G, L, Himg, Wimg, kh, kw, sh, sw, wh, ww, E, Cin, Cout, Hg, Wg;
  std::vector<int> Cl, Hl, Wl, heads, depth, lg_depth, lg_heads;
};

int parse(const vv_lgunet_config* c, FCfg& o, std::string& err) {
  if (!c) return ferr(err, VV_E_ARG, "null config");
  if (c->arch != VV_ARCH_LGUNET1) return ferr(err, VV_E_ARG, "not an LGUnet_all_1 config");
  o.raw = *c;
  o.G = c->n_groups;
  o.L = c->n_enc_levels;
  if (o.G < 1 || o.G > kMaxGroups) return ferr(err, VV_E_ARG, "n_groups %d out of range", o.G);
  if (o.L < 1 || o.L > 4) return ferr(err, VV_E_ARG, "n_enc_levels %d out of range", o.L);
  if (c->n_lg_layers < 1 || c->n_lg_layers > 8) return ferr(err, VV_E_ARG, "n_lg_layers out of range");
  o.Himg = c->img_size[0];
  o.Wimg = c->img_size[1];
  o.kh = c->patch_size[0];
  o.kw = c->patch_size[1];
  o.sh = c->stride[0];
  o.sw = c->stride[1];
  o.wh = c->window_hw[0];
  o.ww = c->window_hw[1];
  o.E = c->embed_dim;
  if (o.kh < o.sh || o.kw < o.sw || o.sh < 1 || o.sw < 1 || o.wh < 1 || o.ww < 1)
    return ferr(err, VV_E_ARG, "bad patch/stride/window");
  const int H0 = o.Himg / o.sh, W0 = o.Wimg / o.sw;
  // PatchEmbed: conv output size must equal img // stride (LGUnet_all.py:28, 42-48)
  if ((o.Himg - o.kh) / o.sh + 1 != H0 || (o.Wimg - o.kw) / o.sw + 1 != W0)
    return ferr(err, VV_E_ARG, "patch kernel/stride do not give img // stride tokens");
  // ConvTranspose2d must reproduce the image size
  if ((H0 - 1) * o.sh + o.kh != o.Himg || (W0 - 1) * o.sw + o.kw != o.Wimg)
    return ferr(err, VV_E_ARG, "ConvTranspose2d would not restore the image size");
  o.Cin = o.Cout = 0;
  for (int g = 0; g < o.G; ++g) {
    o.Cin += c->inchans[g];
    o.Cout += c->outchans[g];
  }
  for (int l = 0; l < o.L; ++l) {
    o.Cl.push_back(c->enc_dim << l);
    o.Hl.push_back(H0 >> l);
    o.Wl.push_back(W0 >> l);
    o.heads.push_back(c->enc_heads[l]);
    o.depth.push_back(c->enc_depths[l]);
    if (l > 0 && (o.Hl[l - 1] % 2 || o.Wl[l - 1] % 2)) return ferr(err, VV_E_ARG, "odd grid before PatchMerging");
    if (o.Hl[l] % o.wh || o.Wl[l] % o.ww) return ferr(err, VV_E_ARG, "level %d grid not window-aligned", l);
    if (o.Cl[l] % o.heads[l]) return ferr(err, VV_E_ARG, "dim not divisible by heads");
  }
  o.Hg = o.Himg / (o.sh << (o.L - 1));
  o.Wg = o.Wimg / (o.sw << (o.L - 1));
  if (o.Hg != o.Hl.back() || o.Wg != o.Wl.back()) return ferr(err, VV_E_ARG, "LG grid != last encoder grid");
  o.lg_depth.assign(c->lg_depths, c->lg_depths + c->n_lg_layers);
  o.lg_heads.assign(c->lg_heads, c->lg_heads + c->n_lg_layers);
  for (int li = 0; li < c->n_lg_layers; ++li) {
    if (o.E % o.lg_heads[li]) return ferr(err, VV_E_ARG, "embed_dim not divisible by lg heads");
    if (li > 0 && (o.Hg % o.wh || o.Wg % o.ww)) return ferr(err, VV_E_ARG, "LG grid not window-aligned");
  }
  // kernel constraints: GEMM K multiple of 32, head_dim in {8,16,...,256} step 8 for the flash kernel
  if (c->enc_dim % 32 || o.E % 32) return ferr(err, VV_E_ARG, "enc_dim and embed_dim must be multiples of 32");
  auto hd_ok = [](int hd) { return hd % 8 == 0 && hd <= 256 && (hd / 8 <= 8 || hd / 8 == 16 || hd / 8 == 24 || hd / 8 == 32); };
  for (int l = 0; l < o.L; ++l)
    if (!hd_ok(o.Cl[l] / o.heads[l])) return ferr(err, VV_E_ARG, "head_dim %d unsupported", o.Cl[l] / o.heads[l]);
  for (int h : o.lg_heads)
    if (!hd_ok(o.E / h)) return ferr(err, VV_E_ARG, "head_dim %d unsupported", o.E / h);
  return 0;
}

void add_block(std::vector<ParamInfo>& v, const std::string& pre, int64_t C) {
  v.push_back({pre + ".norm.weight", {C}});
  v.push_back({pre + ".norm.bias", {C}});
  v.push_back({pre + ".attn.qkv.weight", {3 * C, C}});
  v.push_back({pre + ".attn.qkv.bias", {3 * C}});
  v.push_back({pre + ".attn.proj.weight", {C, C}});
  v.push_back({pre + ".attn.proj.bias", {C}});
  v.push_back({pre + ".norm2.weight", {C}});
  v.push_back({pre + ".norm2.bias", {C}});
  v.push_back({pre + ".mlp.fc1.weight", {4 * C, C}});
  v.push_back({pre + ".mlp.fc1.bias", {4 * C}});
  v.push_back({pre + ".mlp.fc2.weight", {C, 4 * C}});
  v.push_back({pre + ".mlp.fc2.bias", {C}});
}

std::vector<ParamInfo> enumerate(const FCfg& c) {
  std::vector<ParamInfo> v;
  const int L = c.L;
  const int64_t C0 = c.Cl[0], CL = c.Cl.back(), E = c.E;
  for (int g = 0; g < c.G; ++g) {
    const std::string e = "enc.enc_list." + std::to_string(g);
    v.push_back({e + ".absolute_pos_embed", {1, (int64_t)c.Hl[0] * c.Wl[0], C0}});
    v.push_back({e + ".patch_embed.proj.weight", {C0, c.raw.inchans[g], c.kh, c.kw}});
    v.push_back({e + ".patch_embed.proj.bias", {C0}});
    for (int l = 0; l < L; ++l) {
      const std::string pl = e + ".layers." + std::to_string(l);
      for (int b = 0; b < c.depth[l]; ++b) add_block(v, pl + ".blocks." + std::to_string(b), c.Cl[l]);
      if (l > 0) {
        v.push_back({pl + ".downsample.reduction.weight", {c.Cl[l], 2 * (int64_t)c.Cl[l]}});
        v.push_back({pl + ".downsample.norm.weight", {2 * (int64_t)c.Cl[l]}});
        v.push_back({pl + ".downsample.norm.bias", {2 * (int64_t)c.Cl[l]}});
      }
    }
    v.push_back({e + ".norm.weight", {CL}});
    v.push_back({e + ".norm.bias", {CL}});
  }
  v.push_back({"enc.proj.weight", {E, CL * c.G}});
  v.push_back({"enc.proj.bias", {E}});
  v.push_back({"net.pos_embed", {1, (int64_t)c.Hg * c.Wg, E}});
  for (size_t li = 0; li < c.lg_depth.size(); ++li)
    for (int b = 0; b < c.lg_depth[li]; ++b)
      add_block(v, "net.layers." + std::to_string(li) + ".blocks." + std::to_string(b), E);
  for (int g = 0; g < c.G; ++g) {
    const std::string d = "dec.dec_list." + std::to_string(g);
    for (int i = 0; i < L; ++i) {
      const int lev = L - 1 - i;
      const int64_t Cv = c.Cl[lev];
      const std::string pu = d + ".layers_up." + std::to_string(i);
      for (int b = 0; b < c.depth[lev]; ++b) add_block(v, pu + ".blocks." + std::to_string(b), Cv);
      if (i < L - 1) {
        v.push_back({pu + ".upsample.expand.weight", {2 * Cv, Cv}});
        v.push_back({pu + ".upsample.norm.weight", {Cv / 2}});
        v.push_back({pu + ".upsample.norm.bias", {Cv / 2}});
      }
      v.push_back({d + ".concat_back_dim." + std::to_string(i) + ".weight", {Cv, 2 * Cv}});
      v.push_back({d + ".concat_back_dim." + std::to_string(i) + ".bias", {Cv}});
    }
    v.push_back({d + ".norm_up.weight", {C0}});
    v.push_back({d + ".norm_up.bias", {C0}});
  }
  for (int g = 0; g < c.G; ++g) {
    const std::string f = "dec.final_proj_list." + std::to_string(g);
    v.push_back({f + ".weight", {C0, c.raw.outchans[g], c.kh, c.kw}});
    v.push_back({f + ".bias", {c.raw.outchans[g]}});
  }
  v.push_back({"dec.proj.weight", {CL * c.G, E}});
  v.push_back({"dec.proj.bias", {CL * c.G}});
  return v;
}

int64_t numel(const std::vector<int64_t>& s) {
  int64_t n = 1;
  for (auto x : s) n *= x;
  return n;
}

// window-order position -> token index of the rolled image (torch.roll by (-sh, -sw), window_partition)
std::vector<int> window_map(int B, int H, int W, int wh, int ww, int sh, int sw) {
  std::vector<int> m((size_t)B * H * W);
  size_t p = 0;
  for (int b = 0; b < B; ++b)
    for (int wr = 0; wr < H / wh; ++wr)
      for (int wc = 0; wc < W / ww; ++wc)
        for (int i = 0; i < wh; ++i)
          for (int j = 0; j < ww; ++j) m[p++] = (b * H + (wr * wh + i + sh) % H) * W + (wc * ww + j + sw) % W;
  return m;
}

}  // namespace

// windows of at least this many tokens (the global LG window at 0.25 degree: 16,200) run as two split GEMMs
// (S = Q K^T, O = softmax(S) V) instead of the streaming kernel
constexpr int kGemmAttnMin = 1024;

struct FBlock {
  const float *n1g, *n1b, *qkvW, *qkvb, *projW, *projb, *n2g, *n2b, *fc1W, *fc1b, *fc2W, *fc2b;
};

struct FStage {
  int G = 1, H = 0, W = 0, C = 0, heads = 1, depth = 0, M = 0, wh = 0, ww = 0, hd = 0, d1 = 0, d2 = 0;
  bool global = false;
  std::vector<std::array<FBlock, kMaxGroups>> w;
  const int* idx0 = nullptr;
  const int* idx1 = nullptr;
  const float *c1 = nullptr, *s1 = nullptr, *c2 = nullptr, *s2 = nullptr;
  float* x = nullptr;  // [G][M][C], updated in place block by block
};

struct FModel {
  FCfg c;
  int B = 1;
  std::vector<ParamInfo> params;
  std::vector<float*> pptr;
  std::unordered_map<std::string, float*> W;
  float* warena = nullptr;
  size_t wfloats = 0;
  unsigned short* planes = nullptr;
  std::vector<FStage> enc, dec, lg;
  float *t1 = nullptr, *t2 = nullptr, *qkv = nullptr, *h = nullptr, *aux = nullptr, *xm = nullptr, *ex = nullptr,
        *xe = nullptr, *cat = nullptr, *dp = nullptr, *yn = nullptr, *lgx = nullptr, *ws = nullptr;
  std::vector<void*> owned;
  int64_t bytes = 0;
  bool loaded = false;
  // PatchEmbed / ConvTranspose2d as GEMMs: per tower the conv weight [C0][Kp] (zero-padded K) and the transposed
  // ConvTranspose weight [NT][C0] (rows (co*kh+ky)*kw+kx, zero rows up to the widest tower)
  float* convw = nullptr;
  unsigned short* convp = nullptr;
  size_t conv_floats = 0;
  std::vector<float*> Wp, W2;
  int Kp = 0, NT = 0;
  int math = vv::GEMM_SPLIT16;  // GEMM arithmetic (the owning context's setting)
  const vv::Tuning* tune = nullptr;  // the owning context's dispatch knobs
  // global-window attention through the split GEMM when the window is large: S/P [heads][N][Np], V^T [heads][hd][Np]
  float *att_s = nullptr, *att_vt = nullptr;
  void* gattn_ws = nullptr;  // the flash MFMA kernel's planes and scales (vv::gattn_ws_bytes), when it applies
  unsigned short* apl = nullptr;  // tile-48 A planes (k_rowsplit): the largest fp16x3 A, G x M x 4C of a stage
  size_t apl_halfs = 0;
};

namespace {

int dalloc(FModel& m, size_t floats, float** out, std::string& err) {
  void* p = nullptr;
  if (hipMalloc(&p, std::max<size_t>(floats, 1) * sizeof(float)) != hipSuccess)
    return ferr(err, VV_E_ALLOC, "device allocation of %zu floats failed", floats);
  m.owned.push_back(p);
  m.bytes += (int64_t)floats * 4;
  *out = reinterpret_cast<float*>(p);
  return 0;
}

int upload_map(FModel& m, const std::vector<int>& h, const int** out, std::string& err) {
  void* d = nullptr;
  FH(hipMalloc(&d, h.size() * sizeof(int)));
  m.owned.push_back(d);
  FH(hipMemcpy(d, h.data(), h.size() * sizeof(int), hipMemcpyHostToDevice));
  *out = reinterpret_cast<const int*>(d);
  return 0;
}

// rope2 tables (positional_encodings.py:232-251) in fp32: inv_freq = 10000 ** -(i / d), angle = coord * inv_freq
int rope_tables(FModel& m, FStage& s, std::string& err) {
  const int half = s.hd / 2;
  s.d1 = half / 2;
  s.d2 = half - half / 2;
  const int N = s.wh * s.ww;
  std::vector<float> c1((size_t)N * s.d1), s1v(c1.size()), c2((size_t)N * s.d2), s2v(c2.size());
  for (int i = 0; i < N; ++i) {
    const int r = i / s.ww, cc = i % s.ww;
    for (int k = 0; k < s.d1; ++k) {
      const float f = powf(10000.f, -((float)k / (float)s.d1));
      const float ang = (float)r * f;
      c1[(size_t)i * s.d1 + k] = (float)cos((double)ang);
      s1v[(size_t)i * s.d1 + k] = (float)sin((double)ang);
    }
    for (int k = 0; k < s.d2; ++k) {
      const float f = powf(10000.f, -((float)k / (float)s.d2));
      const float ang = (float)cc * f;
      c2[(size_t)i * s.d2 + k] = (float)cos((double)ang);
      s2v[(size_t)i * s.d2 + k] = (float)sin((double)ang);
    }
  }
  float* d = nullptr;
  int r;
  if ((r = dalloc(m, 2 * (c1.size() + c2.size()), &d, err))) return r;
  FH(hipMemcpy(d, c1.data(), c1.size() * 4, hipMemcpyHostToDevice));
  FH(hipMemcpy(d + c1.size(), s1v.data(), c1.size() * 4, hipMemcpyHostToDevice));
  FH(hipMemcpy(d + 2 * c1.size(), c2.data(), c2.size() * 4, hipMemcpyHostToDevice));
  FH(hipMemcpy(d + 2 * c1.size() + c2.size(), s2v.data(), c2.size() * 4, hipMemcpyHostToDevice));
  s.c1 = d;
  s.s1 = d + c1.size();
  s.c2 = d + 2 * c1.size();
  s.s2 = d + 2 * c1.size() + c2.size();
  return 0;
}

int init_stage(FModel& m, FStage& s, int G, int H, int W, int C, int heads, int depth, bool global, float* x,
               std::string& err) {
  s.G = G;
  s.H = H;
  s.W = W;
  s.C = C;
  s.heads = heads;
  s.depth = depth;
  s.M = m.B * H * W;
  s.global = global;
  s.wh = global ? H : m.c.wh;
  s.ww = global ? W : m.c.ww;
  s.hd = C / heads;
  s.x = x;
  s.w.assign(depth, {});
  int r;
  if ((r = upload_map(m, window_map(m.B, H, W, s.wh, s.ww, 0, 0), &s.idx0, err))) return r;
  if (!global && depth > 1 && s.ww / 2 > 0)
    if ((r = upload_map(m, window_map(m.B, H, W, s.wh, s.ww, s.wh / 2, s.ww / 2), &s.idx1, err))) return r;
  return rope_tables(m, s, err);
}

FBlock blk(FModel& m, const std::string& pre) {
  auto w = [&](const std::string& n) -> const float* { return m.W.at(n); };
  return {w(pre + ".norm.weight"),     w(pre + ".norm.bias"),      w(pre + ".attn.qkv.weight"),
          w(pre + ".attn.qkv.bias"),   w(pre + ".attn.proj.weight"), w(pre + ".attn.proj.bias"),
          w(pre + ".norm2.weight"),    w(pre + ".norm2.bias"),     w(pre + ".mlp.fc1.weight"),
          w(pre + ".mlp.fc1.bias"),    w(pre + ".mlp.fc2.weight"), w(pre + ".mlp.fc2.bias")};
}

GemmArgs gbase(int M, int N, int K, int G, int epi, const FModel& m) {
  GemmArgs a;
  memset(&a, 0, sizeof(a));
  a.math = m.math;
  a.tune = m.tune;
  a.h3_mink = (m.tune ? *m.tune : vv::kDefaultTuning).fc_h3_mink;
  a.apl = m.apl;  // the tile-48 A-plane workspace (k_rowsplit)
  a.apl_halfs = m.apl_halfs;
  a.M = M;
  a.N = N;
  a.K = K;
  a.ksplit = K;
  a.lda = K;
  a.ldc = a.ldr = a.ldaux = N;
  a.epi = epi;
  a.ngroups = G;
  return a;
}

LnArgs lbase(int rows, int C, int G) {
  LnArgs a;
  memset(&a, 0, sizeof(a));
  a.rows = rows;
  a.C = C;
  a.ldx = a.ldy = a.lddy = a.ldres = C;
  a.mode = LN_ROWMAP;
  a.eps = 1e-6f;  // partial(nn.LayerNorm, eps=1e-6) everywhere in LGUnet_all_1
  a.ngroups = G;
  return a;
}

// win_attn: the tuning knob (0: the streaming kernel for small windows too)
hipError_t flash(const FlashArgs& a, int hd, int nwin, int G, hipStream_t st, const vv::Tuning& TU,
                 const RopeArgs* rope) {
  const bool win_attn = TU.win_attn != 0;
  if (rope) {  // rope fused (win_mf_ok)
    const int NT = (a.N + 15) / 16;
    const size_t lds = (3 * (size_t)NT * 16 * (hd + 1) + NT * 16) * sizeof(float);
    const dim3 grid(nwin, a.heads, G), block(64 * NT);
    hipError_t e = hipSuccess;
    switch (hd * 8 + NT) {
#define WM(D, T)                                                                                           \
  case D * 8 + T: {                                                                                        \
    if (lds > 65536) { /* only past 64 KB: the attribute is not needed below */                            \
      e = set_lds_limit((const void*)k_attn_win_mf<D, T>, (3 * kWinMaxN * (kWinMaxHd + 1) + kWinMaxN) * 4); \
      if (e != hipSuccess) return e;                                                                       \
    }                                                                                                      \
    hipLaunchKernelGGL((k_attn_win_mf<D, T>), grid, block, lds, st, a, *rope);                             \
    break;                                                                                                 \
  }
#define WM6(D) WM(D, 1) WM(D, 2) WM(D, 3) WM(D, 4) WM(D, 5) WM(D, 6)
      WM6(16) WM6(32) WM6(48) WM6(64)
#undef WM6
#undef WM
      default:
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  if (a.N <= kWinMaxN && hd <= kWinMaxHd && hd % 4 == 0 && win_attn) {
    const size_t lds = (3 * (size_t)a.N * (hd + 4) + (size_t)a.N * (a.N + 1)) * sizeof(float);
    if (hipError_t e = set_lds_limit((const void*)k_attn_win,
                                     (size_t)(3 * kWinMaxN * (kWinMaxHd + 4) + kWinMaxN * (kWinMaxN + 1)) * 4))
      return e;
    hipLaunchKernelGGL(k_attn_win, dim3(nwin, a.heads, G), dim3(256), lds, st, a);
    return hipGetLastError();
  }
  const int qblocks = (a.N + 31) / 32;
  dim3 grid(nwin, a.heads * qblocks, G);
  switch (hd / 8) {
#define FL(D) \
  case D: hipLaunchKernelGGL((k_attn_flash<D>), grid, dim3(256), 0, st, a); break;
    FL(1) FL(2) FL(3) FL(4) FL(5) FL(6) FL(7) FL(8) FL(16) FL(24) FL(32)
#undef FL
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

int stage_fwd(FModel& m, FStage& S, hipStream_t st, std::string& err) {
  const int G = S.G, M = S.M, C = S.C;
  const size_t MC = (size_t)M * C;
  const int N = S.wh * S.ww, nwin = M / N;
  for (int b = 0; b < S.depth; ++b) {
    const bool shifted = !S.global && (b % 2 == 1) && S.ww / 2 > 0;  // shift [wh//2, ww//2] on odd blocks
    const int sh = shifted ? S.wh / 2 : 0;
    const bool masked = shifted && S.ww != S.W;                          // Attention.py:609-612
    const int* idx = shifted ? S.idx1 : S.idx0;
    // norm -> window order
    LnArgs ln = lbase(M, C, G);
    ln.map = idx;
    for (int g = 0; g < G; ++g)
      ln.g[g] = {S.x + g * MC, S.w[b][g].n1g, S.w[b][g].n1b, m.t1 + g * MC, nullptr, nullptr, nullptr};
    FH(layernorm_fwd(ln, st));
    GemmArgs q = gbase(M, 3 * C, C, G, EPI_STORE, m);
    for (int g = 0; g < G; ++g)
      q.g[g] = {m.t1 + g * MC, nullptr, S.w[b][g].qkvW, S.w[b][g].qkvb, m.qkv + g * MC * 3, nullptr, nullptr};
    FH(gemm_nt(q, st, -1, m.ws));
    RopeArgs ra;
    memset(&ra, 0, sizeof(ra));
    for (int g = 0; g < G; ++g) ra.qkv[g] = m.qkv + g * MC * 3;
    ra.rows = M;
    ra.C = C;
    ra.heads = S.heads;
    ra.hd = S.hd;
    ra.d1 = S.d1;
    ra.d2 = S.d2;
    ra.N = N;
    ra.c1 = S.c1;
    ra.s1 = S.s1;
    ra.c2 = S.c2;
    ra.s2 = S.s2;
    ra.scale = (float)std::pow((double)S.hd, -0.5);
    const vv::Tuning& TU = m.tune ? *m.tune : vv::kDefaultTuning;
    const bool use_gattn = S.global && m.gattn_ws && G == 1 && gattn_supported(C, S.heads) && TU.gattn;
    const bool use_gemm_attn = !use_gattn && S.global && N >= kGemmAttnMin && m.att_s && G == 1;
    const bool rope_fused = !use_gattn && !use_gemm_attn && S.c1 && win_mf_ok(N, S.hd, TU);
    int ph = -1;
    if (!rope_fused) {
      ph = prof_begin(st);
      hipLaunchKernelGGL(k_rope, dim3(grid_for((size_t)M * S.heads * (S.hd / 2)), G), dim3(256), 0, st, ra);
      FH(hipGetLastError());
      prof_end(ph, st, PC_ATTN, 6.0 * G * M * C, 16.0 * G * M * C);
    }
    FlashArgs fa;
    memset(&fa, 0, sizeof(fa));
    for (int g = 0; g < G; ++g) {
      fa.qkv[g] = m.qkv + g * MC * 3;
      fa.out[g] = m.t2 + g * MC;
    }
    fa.N = N;
    fa.C = C;
    fa.heads = S.heads;
    fa.masked = masked ? 1 : 0;
    fa.H = S.H;
    fa.wh = S.wh;
    fa.ww = S.ww;
    fa.sh = sh;
    fa.nWh = S.H / S.wh;
    fa.nWw = S.W / S.ww;
    if (use_gattn) {
      // one window over the whole grid per image: the flash MFMA kernel (vv_gattn.hip), scores never in HBM
      ph = prof_begin(st);
      for (int b0 = 0; b0 < nwin; ++b0)
        FH(gattn(m.qkv + (size_t)b0 * N * 3 * C, m.t2 + (size_t)b0 * N * C, C, N, C, S.heads, m.gattn_ws, st,
                 TU.gattn_qf));
      prof_end(ph, st, PC_ATTN, 4.0 * nwin * (double)N * N * C, 16.0 * nwin * (double)N * C);
    } else if (use_gemm_attn) {
      // S_h = Q_h K_h^T (heads as GEMM groups; q rotated + scaled, k rotated), P = softmax_rows(S), O_h = P V_h
      const int Np = (N + 31) / 32 * 32, hd = S.hd;
      for (int b0 = 0; b0 < nwin; ++b0) {
        const float* qkv = m.qkv + (size_t)b0 * N * 3 * C;
        GemmArgs sq = gbase(N, N, hd, S.heads, EPI_STORE, m);
        sq.lda = 3 * C;
        sq.ldb = 3 * C;
        sq.ldc = Np;
        for (int hh = 0; hh < S.heads; ++hh)
          sq.g[hh] = {qkv + hh * hd, nullptr, qkv + C + hh * hd, nullptr, m.att_s + (size_t)hh * N * Np, nullptr,
                      nullptr};
        FH(gemm_nt(sq, st, -1, nullptr));
        ph = prof_begin(st);
        if (Np % 4 == 0 && Np <= 256 * 4 * kSmRV)
          hipLaunchKernelGGL(k_softmax_rows_reg, dim3(S.heads * N), dim3(256), 0, st, m.att_s, N, Np);
        else
          hipLaunchKernelGGL(k_softmax_rows, dim3(S.heads * N), dim3(256), 0, st, m.att_s, N, Np);
        FH(hipGetLastError());
        hipLaunchKernelGGL(k_vt, dim3(grid_for((size_t)C * Np)), dim3(256), 0, st, qkv, m.att_vt, N, Np, C, S.heads,
                           hd);
        FH(hipGetLastError());
        prof_end(ph, st, PC_ATTN, 4.0 * S.heads * N * (double)Np, 12.0 * S.heads * N * (double)Np);
        GemmArgs pv = gbase(N, hd, Np, S.heads, EPI_STORE, m);
        pv.ldc = C;
        for (int hh = 0; hh < S.heads; ++hh)
          pv.g[hh] = {m.att_s + (size_t)hh * N * Np, nullptr, m.att_vt + (size_t)hh * hd * Np, nullptr,
                      m.t2 + (size_t)b0 * N * C + hh * hd, nullptr, nullptr};
        FH(gemm_nt(pv, st, -1, nullptr));
      }
    } else {
      ph = prof_begin(st);
      FH(flash(fa, S.hd, nwin, G, st, TU, rope_fused ? &ra : nullptr));
      prof_end(ph, st, PC_ATTN, 4.0 * G * (double)M * N * C, 16.0 * G * (double)M * C);
    }
    // proj + window reverse / roll back + residual, in place
    GemmArgs p = gbase(M, C, C, G, EPI_RESID, m);
    p.crow = idx;
    for (int g = 0; g < G; ++g)
      p.g[g] = {m.t2 + g * MC, nullptr, S.w[b][g].projW, S.w[b][g].projb, S.x + g * MC, S.x + g * MC, nullptr};
    FH(gemm_nt(p, st, -1, m.ws));
    LnArgs ln2 = lbase(M, C, G);
    for (int g = 0; g < G; ++g)
      ln2.g[g] = {S.x + g * MC, S.w[b][g].n2g, S.w[b][g].n2b, m.t1 + g * MC, nullptr, nullptr, nullptr};
    FH(layernorm_fwd(ln2, st));
    GemmArgs f1 = gbase(M, 4 * C, C, G, EPI_GELU, m);
    for (int g = 0; g < G; ++g)
      f1.g[g] = {m.t1 + g * MC, nullptr, S.w[b][g].fc1W, S.w[b][g].fc1b, m.h + g * MC * 4, nullptr, nullptr};
    FH(gemm_nt(f1, st, -1, m.ws));
    GemmArgs f2 = gbase(M, C, 4 * C, G, EPI_RESID, m);
    for (int g = 0; g < G; ++g)
      f2.g[g] = {m.h + g * MC * 4, nullptr, S.w[b][g].fc2W, S.w[b][g].fc2b, S.x + g * MC, S.x + g * MC, nullptr};
    FH(gemm_nt(f2, st, -1, m.ws));
  }
  return 0;
}

}  // namespace

int params(const vv_lgunet_config* cfg, std::vector<ParamInfo>& out, std::string& err) {
  FCfg c;
  int r = parse(cfg, c, err);
  if (r) return r;
  out = enumerate(c);
  return 0;
}

void destroy(FModel* m) {
  if (!m) return;
  if (m->warena) unregister_split_arena(m->warena);
  if (m->convw) unregister_split_arena(m->convw);
  for (void* p : m->owned) (void)hipFree(p);
  delete m;
}

int create(const vv_lgunet_config* cfg, int batch, FModel** out, std::string& err) {
  FCfg c;
  int r = parse(cfg, c, err);
  if (r) return r;
  if (batch < 1) return ferr(err, VV_E_ARG, "batch must be >= 1");
  FModel* m = new FModel();
  m->c = c;
  m->B = batch;
  m->params = enumerate(c);
  auto bail = [&](int code) {
    destroy(m);
    return code;
  };
  // weights (fp32, 64-float aligned) + their bf16 split planes for the GEMMs
  size_t off = 0;
  std::vector<size_t> offs;
  for (auto& p : m->params) {
    offs.push_back(off);
    off += (numel(p.shape) + 63) & ~size_t(63);
  }
  m->wfloats = off;
  if ((r = dalloc(*m, off, &m->warena, err))) return bail(r);
  void* pl = nullptr;
  if (hipMalloc(&pl, split_arena_bytes(off)) != hipSuccess)
    return bail(ferr(err, VV_E_ALLOC, "weight split planes"));
  m->owned.push_back(pl);
  m->planes = reinterpret_cast<unsigned short*>(pl);
  register_split_arena(m->warena, off, m->planes);
  for (size_t i = 0; i < m->params.size(); ++i) {
    m->pptr.push_back(m->warena + offs[i]);
    m->W[m->params[i].name] = m->warena + offs[i];
  }
  // activations
  const int G = c.G, L = c.L, B = batch;
  const size_t Mg = (size_t)B * c.Hg * c.Wg;
  size_t smax = Mg * c.E, s2max = 1;
  std::vector<size_t> S(L);
  for (int l = 0; l < L; ++l) {
    S[l] = (size_t)G * B * c.Hl[l] * c.Wl[l] * c.Cl[l];
    smax = std::max(smax, S[l]);
    if (l > 0) s2max = std::max(s2max, 2 * S[l]);
  }
  if ((r = dalloc(*m, smax, &m->t1, err)) || (r = dalloc(*m, smax, &m->t2, err)) ||
      (r = dalloc(*m, 3 * smax, &m->qkv, err)) || (r = dalloc(*m, 4 * smax, &m->h, err)) ||
      (r = dalloc(*m, s2max, &m->xm, err)) ||
      (r = dalloc(*m, s2max, &m->ex, err)) || (r = dalloc(*m, smax, &m->xe, err)) ||
      (r = dalloc(*m, Mg * G * c.Cl.back(), &m->cat, err)) || (r = dalloc(*m, Mg * G * c.Cl.back(), &m->dp, err)) ||
      (r = dalloc(*m, S[0], &m->yn, err)) || (r = dalloc(*m, Mg * c.E, &m->lgx, err)) ||
      (r = dalloc(*m, gemm_ws_floats(), &m->ws, err)))
    return bail(r);
  {
    // tile-48 A planes: the widest A of the stages that reach the fp16x3 kernels (K >= 768: the LG stage's fc2
    // forward, Mg x 4E), two fp16 planes = 4 B per element
    float* p = nullptr;
    if ((r = dalloc(*m, (size_t)Mg * 4 * c.E, &p, err))) return bail(r);
    m->apl = reinterpret_cast<unsigned short*>(p);
    m->apl_halfs = (size_t)Mg * 4 * c.E * 2;
  }
  {
    int kmax = 0, nmax = 0;
    for (int g = 0; g < G; ++g) {
      kmax = std::max(kmax, c.raw.inchans[g] * c.kh * c.kw);
      nmax = std::max(nmax, c.raw.outchans[g] * c.kh * c.kw);
    }
    m->Kp = (kmax + 31) / 32 * 32;
    m->NT = nmax;
    const size_t per = (size_t)c.Cl[0] * m->Kp + (size_t)m->NT * c.Cl[0];
    m->conv_floats = per * G;
    if ((r = dalloc(*m, m->conv_floats, &m->convw, err))) return bail(r);
    void* cp = nullptr;
    if (hipMalloc(&cp, split_arena_bytes(m->conv_floats)) != hipSuccess)
      return bail(ferr(err, VV_E_ALLOC, "conv split planes"));
    m->owned.push_back(cp);
    m->convp = reinterpret_cast<unsigned short*>(cp);
    register_split_arena(m->convw, m->conv_floats, m->convp);
    for (int g = 0; g < G; ++g) {
      m->Wp.push_back(m->convw + g * per);
      m->W2.push_back(m->convw + g * per + (size_t)c.Cl[0] * m->Kp);
    }
    // im2col rows and the ConvTranspose GEMM output live in the MLP scratch (4 x the widest level)
    if ((size_t)B * c.Hl[0] * c.Wl[0] * std::max(m->Kp, m->NT) * G > 4 * smax)
      return bail(ferr(err, VV_E_ARG, "conv GEMM scratch too small"));
  }
  m->enc.resize(L);
  m->dec.resize(L);
  for (int l = 0; l < L; ++l) {
    float *xe_ = nullptr, *xd_ = nullptr;
    if ((r = dalloc(*m, S[l], &xe_, err)) || (r = dalloc(*m, S[l], &xd_, err))) return bail(r);
    if ((r = init_stage(*m, m->enc[l], G, c.Hl[l], c.Wl[l], c.Cl[l], c.heads[l], c.depth[l], false, xe_, err)) ||
        (r = init_stage(*m, m->dec[l], G, c.Hl[l], c.Wl[l], c.Cl[l], c.heads[l], c.depth[l], false, xd_, err)))
      return bail(r);
  }
  m->lg.resize(c.lg_depth.size());
  for (size_t li = 0; li < m->lg.size(); ++li)
    if ((r = init_stage(*m, m->lg[li], 1, c.Hg, c.Wg, c.E, c.lg_heads[li], c.lg_depth[li], li == 0, m->lgx, err)))
      return bail(r);
  {
    const size_t N = (size_t)c.Hg * c.Wg, Np = (N + 31) / 32 * 32;
    const int h0 = c.lg_heads[0];  // LG layer 0 is the global window
    if (gattn_supported(c.E, h0)) {
      void* p = nullptr;
      if (hipMalloc(&p, gattn_ws_bytes((int)N, c.E, h0)) != hipSuccess)
        return bail(ferr(err, VV_E_ALLOC, "global-attention workspace"));
      m->owned.push_back(p);
      m->bytes += (int64_t)gattn_ws_bytes((int)N, c.E, h0);
      m->gattn_ws = p;
    }
    if (N >= (size_t)kGemmAttnMin && !m->gattn_ws) {
      const int hmax = *std::max_element(c.lg_heads.begin(), c.lg_heads.end());
      if ((r = dalloc(*m, (size_t)hmax * N * Np, &m->att_s, err)) || (r = dalloc(*m, (size_t)c.E * Np, &m->att_vt, err)))
        return bail(r);
    }
  }
  *out = m;
  return 0;
}

int load(FModel* m, const void* const* ptrs, int n, std::string& err) {
  if (n != (int)m->params.size()) return ferr(err, VV_E_ARG, "expected %zu params, got %d", m->params.size(), n);
  for (int i = 0; i < n; ++i) {
    if (!ptrs[i]) return ferr(err, VV_E_ARG, "null pointer for %s", m->params[i].name.c_str());
    FH(hipMemcpy(m->pptr[i], ptrs[i], numel(m->params[i].shape) * 4, hipMemcpyDefault));
  }
  for (size_t i = 0; i < m->params.size(); ++i) {
    const auto& p = m->params[i];
    if (p.shape.size() != 2) continue;
    FH(split_registered(m->pptr[i], numel(p.shape), (int)p.shape[1], 0));
  }
  FH(hipDeviceSynchronize());
  const FCfg& c = m->c;
  {
    const int C0 = c.Cl[0], kk = c.kh * c.kw;
    std::vector<float> host;
    for (int g = 0; g < c.G; ++g) {
      // conv: [C0][cin][kh][kw] -> [C0][Kp]
      const int cin = c.raw.inchans[g];
      host.resize((size_t)C0 * cin * kk);
      FH(hipMemcpy(host.data(), m->W.at("enc.enc_list." + std::to_string(g) + ".patch_embed.proj.weight"),
                   host.size() * 4, hipMemcpyDeviceToHost));
      std::vector<float> wp((size_t)C0 * m->Kp, 0.f);
      for (int co = 0; co < C0; ++co)
        for (int k = 0; k < cin * kk; ++k) wp[(size_t)co * m->Kp + k] = host[(size_t)co * cin * kk + k];
      FH(hipMemcpy(m->Wp[g], wp.data(), wp.size() * 4, hipMemcpyHostToDevice));
      // convT: [C0][cout][kh][kw] -> [(co*kh+ky)*kw+kx][C0], zero rows up to NT
      const int cout = c.raw.outchans[g];
      host.resize((size_t)C0 * cout * kk);
      FH(hipMemcpy(host.data(), m->W.at("dec.final_proj_list." + std::to_string(g) + ".weight"), host.size() * 4,
                   hipMemcpyDeviceToHost));
      std::vector<float> w2((size_t)m->NT * C0, 0.f);
      for (int ci = 0; ci < C0; ++ci)
        for (int j = 0; j < cout * kk; ++j) w2[(size_t)j * C0 + ci] = host[(size_t)ci * cout * kk + j];
      FH(hipMemcpy(m->W2[g], w2.data(), w2.size() * 4, hipMemcpyHostToDevice));
      // split planes (rows of K = Kp for Wp, C0 for W2)
      FH(split_registered(m->Wp[g], (size_t)C0 * m->Kp, m->Kp, 0));
      FH(split_registered(m->W2[g], (size_t)m->NT * C0, C0, 0));
    }
    FH(hipDeviceSynchronize());
  }
  for (int g = 0; g < c.G; ++g) {
    const std::string e = "enc.enc_list." + std::to_string(g), d = "dec.dec_list." + std::to_string(g);
    for (int l = 0; l < c.L; ++l) {
      for (int b = 0; b < c.depth[l]; ++b)
        m->enc[l].w[b][g] = blk(*m, e + ".layers." + std::to_string(l) + ".blocks." + std::to_string(b));
      const int i = c.L - 1 - l;
      for (int b = 0; b < c.depth[l]; ++b)
        m->dec[l].w[b][g] = blk(*m, d + ".layers_up." + std::to_string(i) + ".blocks." + std::to_string(b));
    }
  }
  for (size_t li = 0; li < m->lg.size(); ++li)
    for (int b = 0; b < m->lg[li].depth; ++b)
      m->lg[li].w[b][0] = blk(*m, "net.layers." + std::to_string(li) + ".blocks." + std::to_string(b));
  m->loaded = true;
  return 0;
}

int forward(FModel* m, const float* in, float* out, int climit, hipStream_t st, std::string& err) {
  if (!m->loaded) return ferr(err, VV_E_STATE, "weights not loaded");
  const FCfg& c = m->c;
  const int G = c.G, L = c.L, B = m->B;
  auto w = [&](const std::string& n) -> const float* { return m->W.at(n); };
  auto eg = [&](int g) { return "enc.enc_list." + std::to_string(g); };
  auto dg = [&](int g) { return "dec.dec_list." + std::to_string(g); };
  std::vector<int> M(L);
  std::vector<size_t> S(L);
  for (int l = 0; l < L; ++l) {
    M[l] = B * c.Hl[l] * c.Wl[l];
    S[l] = (size_t)M[l] * c.Cl[l];
  }
  const int Mg = B * c.Hg * c.Wg, CL = c.Cl.back();
  int r;
  // ---- Enc_net (LGUnet_all.py:578-592): PatchEmbed + absolute_pos_embed
  ConvArgs pa;
  memset(&pa, 0, sizeof(pa));
  pa.B = B;
  pa.Cimg = c.Cin;
  pa.Himg = c.Himg;
  pa.Wimg = c.Wimg;
  pa.Ho = c.Hl[0];
  pa.Wo = c.Wl[0];
  pa.Ctok = c.Cl[0];
  pa.kh = c.kh;
  pa.kw = c.kw;
  pa.sh = c.sh;
  pa.sw = c.sw;
  pa.img = in;
  for (int g = 0, off = 0; g < G; off += c.raw.inchans[g], ++g) {
    pa.w[g] = w(eg(g) + ".patch_embed.proj.weight");
    pa.bias[g] = w(eg(g) + ".patch_embed.proj.bias");
    pa.pos[g] = w(eg(g) + ".absolute_pos_embed");
    pa.tok[g] = m->enc[0].x + g * S[0];
    pa.cin_off[g] = off;
    pa.cin[g] = c.raw.inchans[g];
  }
  const vv::Tuning& TU = m->tune ? *m->tune : vv::kDefaultTuning;
  // the direct MFMA conv kernels: patch (kh, 2) / stride (2, 2), C0 32 or 96, <= kFcKP taps (LGUnet_all_1's configs)
  const bool conv_mf = TU.fc_conv_mf && c.kw == 2 && c.sw == 2 && c.sh == 2 && c.kh <= 3 && m->Kp <= kFcKP &&
                       (c.Cl[0] == 32 || c.Cl[0] == 96) && 2 * c.Wl[0] == c.Wimg && (c.Himg - c.kh) / 2 + 1 == c.Hl[0];
  int ph = prof_begin(st);
  if (conv_mf) {
    ConvArgs pm = pa;
    for (int g = 0; g < G; ++g) pm.w[g] = m->Wp[g];
    const size_t lds = (size_t)(64 + c.Cl[0]) * (m->Kp + 4) * sizeof(float);
    const dim3 grid((M[0] + 63) / 64, G);
    if (c.Cl[0] == 96) {
      FH(set_lds_limit((const void*)k_fc_patch_mf<96>, (64 + 96) * (kFcKP + 4) * sizeof(float)));
      hipLaunchKernelGGL(k_fc_patch_mf<96>, grid, dim3(256), lds, st, pm, m->Kp);
    } else {
      hipLaunchKernelGGL(k_fc_patch_mf<32>, grid, dim3(256), lds, st, pm, m->Kp);
    }
    FH(hipGetLastError());
    prof_end(ph, st, PC_PATCH, 2.0 * G * M[0] * c.Cl[0] * m->Kp, 4.0 * ((double)B * c.Cin * c.Himg * c.Wimg + 2.0 * G * M[0] * c.Cl[0]));
  } else {
    // PatchEmbed = im2col + GEMM (+bias, +absolute_pos_embed in the epilogue)
    const size_t colg = (size_t)M[0] * m->Kp;
    hipLaunchKernelGGL(k_im2col, dim3(grid_for(colg), G), dim3(256), 0, st, pa, m->h, m->Kp, colg);
    FH(hipGetLastError());
    prof_end(ph, st, PC_PATCH, 0.0, 8.0 * G * colg);
    GemmArgs pe = gbase(M[0], c.Cl[0], m->Kp, G, EPI_RESID, *m);
    pe.rmod = c.Hl[0] * c.Wl[0];
    pe.ldr = c.Cl[0];
    for (int g = 0; g < G; ++g)
      pe.g[g] = {m->h + g * colg, nullptr, m->Wp[g], pa.bias[g], pa.tok[g], pa.pos[g], nullptr};
    FH(gemm_nt(pe, st, -1, m->ws));
  }
  for (int l = 0; l < L; ++l) {
    if (l > 0) {
      // PatchMerging (LGUnet_all.py:77-96): gather + LN(4C) + reduction, BEFORE the blocks (:236-246)
      const int Cp = c.Cl[l - 1];
      LnArgs lm = lbase(M[l], 4 * Cp, G);
      lm.mode = LN_MERGE;
      lm.Hin = c.Hl[l - 1];
      lm.Win = c.Wl[l - 1];
      lm.ldx = Cp;
      const std::string pl = ".layers." + std::to_string(l) + ".downsample";
      for (int g = 0; g < G; ++g)
        lm.g[g] = {m->enc[l - 1].x + g * S[l - 1], w(eg(g) + pl + ".norm.weight"), w(eg(g) + pl + ".norm.bias"),
                   m->xm + (size_t)g * M[l] * 4 * Cp, nullptr, nullptr, nullptr};
      FH(layernorm_fwd(lm, st));
      GemmArgs red = gbase(M[l], c.Cl[l], 4 * Cp, G, EPI_STORE, *m);
      for (int g = 0; g < G; ++g)
        red.g[g] = {m->xm + (size_t)g * M[l] * 4 * Cp, nullptr, w(eg(g) + pl + ".reduction.weight"), nullptr,
                    m->enc[l].x + g * S[l], nullptr, nullptr};
      FH(gemm_nt(red, st, -1, m->ws));
    }
    if ((r = stage_fwd(*m, m->enc[l], st, err))) return r;
  }
  // encoder norm -> concat over towers (LGUnet_all.py:409, 590-591)
  LnArgs le = lbase(Mg, CL, G);
  le.ldy = G * CL;
  for (int g = 0; g < G; ++g)
    le.g[g] = {m->enc[L - 1].x + g * S[L - 1], w(eg(g) + ".norm.weight"), w(eg(g) + ".norm.bias"), m->cat + g * CL,
               nullptr, nullptr, nullptr};
  FH(layernorm_fwd(le, st));
  GemmArgs ep = gbase(Mg, c.E, G * CL, 1, EPI_RESID, *m);
  ep.rmod = c.Hg * c.Wg;  // + LG_net.pos_embed (LGUnet_all.py:727)
  ep.ldr = c.E;
  ep.g[0] = {m->cat, nullptr, w("enc.proj.weight"), w("enc.proj.bias"), m->lgx, w("net.pos_embed"), nullptr};
  FH(gemm_nt(ep, st, -1, m->ws));
  // ---- LG_net (LGUnet_all.py:722-740)
  for (auto& s : m->lg)
    if ((r = stage_fwd(*m, s, st, err))) return r;
  // ---- Dec_net (LGUnet_all.py:624-650)
  GemmArgs dp = gbase(Mg, G * CL, c.E, 1, EPI_STORE, *m);
  dp.g[0] = {m->lgx, nullptr, w("dec.proj.weight"), w("dec.proj.bias"), m->dp, nullptr, nullptr};
  FH(gemm_nt(dp, st, -1, m->ws));
  for (int i = 0; i < L; ++i) {
    const int lev = L - 1 - i, Cv = c.Cl[lev];
    // cat(x, skip) -> concat_back_dim[i] (LGUnet_all.py:473-476)
    GemmArgs cb = gbase(M[lev], Cv, 2 * Cv, G, EPI_STORE, *m);
    cb.ksplit = Cv;
    cb.lda = i == 0 ? G * CL : Cv;
    cb.lda2 = Cv;
    const std::string ci = ".concat_back_dim." + std::to_string(i);
    for (int g = 0; g < G; ++g)
      cb.g[g] = {i == 0 ? m->dp + g * CL : m->xe + g * S[lev], m->enc[lev].x + g * S[lev], w(dg(g) + ci + ".weight"),
                 w(dg(g) + ci + ".bias"), m->dec[lev].x + g * S[lev], nullptr, nullptr};
    FH(gemm_nt(cb, st, -1, m->ws));
    if ((r = stage_fwd(*m, m->dec[lev], st, err))) return r;
    if (i < L - 1) {
      // PatchExpand (LGUnet_all.py:107-118): expand (no bias) + rearrange + LN(C/2)
      const std::string pu = ".layers_up." + std::to_string(i) + ".upsample";
      GemmArgs ex = gbase(M[lev], 2 * Cv, Cv, G, EPI_STORE, *m);
      for (int g = 0; g < G; ++g)
        ex.g[g] = {m->dec[lev].x + g * S[lev], nullptr, w(dg(g) + pu + ".expand.weight"), nullptr,
                   m->ex + (size_t)g * M[lev] * 2 * Cv, nullptr, nullptr};
      FH(gemm_nt(ex, st, -1, m->ws));
      LnArgs lx = lbase(M[lev - 1], Cv / 2, G);
      lx.mode = LN_EXPAND;
      lx.Hin = c.Hl[lev];
      lx.Win = c.Wl[lev];
      lx.ldx = 2 * Cv;
      for (int g = 0; g < G; ++g)
        lx.g[g] = {m->ex + (size_t)g * M[lev] * 2 * Cv, w(dg(g) + pu + ".norm.weight"), w(dg(g) + pu + ".norm.bias"),
                   m->xe + g * S[lev - 1], nullptr, nullptr, nullptr};
      FH(layernorm_fwd(lx, st));
    }
  }
  LnArgs lu = lbase(M[0], c.Cl[0], G);
  for (int g = 0; g < G; ++g)
    lu.g[g] = {m->dec[0].x + g * S[0], w(dg(g) + ".norm_up.weight"), w(dg(g) + ".norm_up.bias"), m->yn + g * S[0],
               nullptr, nullptr, nullptr};
  FH(layernorm_fwd(lu, st));
  // ConvTranspose2d + quirk Q2 (mean halves of all towers, then std halves)
  ConvArgs pu;
  memset(&pu, 0, sizeof(pu));
  pu.B = B;
  pu.Himg = c.Himg;
  pu.Wimg = c.Wimg;
  pu.Ho = c.Hl[0];
  pu.Wo = c.Wl[0];
  pu.Ctok = c.Cl[0];
  pu.kh = c.kh;
  pu.kw = c.kw;
  pu.sh = c.sh;
  pu.sw = c.sw;
  pu.Ctot = c.Cout;
  pu.climit = climit;
  pu.img_out = out;
  int mean_total = 0, maxc = 0;
  for (int g = 0; g < G; ++g) mean_total += c.raw.outchans[g] / 2;
  for (int g = 0, mo = 0, so = mean_total; g < G; ++g) {
    const int co = c.raw.outchans[g];
    pu.w[g] = w("dec.final_proj_list." + std::to_string(g) + ".weight");
    pu.bias[g] = w("dec.final_proj_list." + std::to_string(g) + ".bias");
    pu.tok[g] = m->yn + g * S[0];
    pu.mean_off[g] = mo;
    pu.std_off[g] = so;
    pu.cout[g] = co;
    mo += co / 2;
    so += co - co / 2;
    maxc = std::max(maxc, co);
  }
  if (conv_mf && maxc <= 32) {
    // ConvTranspose2d gathered per output row (overlapping taps summed in registers), no GEMM / col2im buffers
    ConvArgs pm = pu;
    for (int g = 0; g < G; ++g) pm.w[g] = m->W2[g];
    const int JP = (2 * maxc + 15) / 16 * 16, ntap = (c.kh + 1) / 2;
    const size_t lds = (size_t)ntap * JP * (c.Cl[0] + 4) * sizeof(float);
    const dim3 grid((c.Wl[0] + 63) / 64, 2 * ((c.Himg + 2 * kFcRows - 1) / (2 * kFcRows)), G);
    ph = prof_begin(st);
    if (c.Cl[0] == 96) {
      FH(set_lds_limit((const void*)k_fc_convT_mf<96>, (size_t)2 * 64 * (96 + 4) * sizeof(float)));
      hipLaunchKernelGGL(k_fc_convT_mf<96>, grid, dim3(256), lds, st, pm);
    } else {
      hipLaunchKernelGGL(k_fc_convT_mf<32>, grid, dim3(256), lds, st, pm);
    }
    FH(hipGetLastError());
    prof_end(ph, st, PC_PATCH, 2.0 * M[0] * c.Cl[0] * c.kh * c.kw * (double)c.Cout / 2,
             4.0 * ((double)G * M[0] * c.Cl[0] + (double)B * c.Cout * c.Himg * c.Wimg));
    return 0;
  }
  // ConvTranspose2d = GEMM (tokens x transposed weight) + col2im of the overlapping taps
  const size_t yg = (size_t)M[0] * m->NT;
  GemmArgs ct = gbase(M[0], m->NT, c.Cl[0], G, EPI_STORE, *m);
  for (int g = 0; g < G; ++g) ct.g[g] = {pu.tok[g], nullptr, m->W2[g], nullptr, m->h + g * yg, nullptr, nullptr};
  FH(gemm_nt(ct, st, -1, m->ws));
  ph = prof_begin(st);
  hipLaunchKernelGGL(k_col2im, dim3(grid_for((size_t)B * c.Himg * c.Wimg), maxc, G), dim3(256), 0, st, pu, m->h,
                     m->NT, yg);
  FH(hipGetLastError());
  prof_end(ph, st, PC_PATCH, 0.0, 4.0 * G * (yg + (size_t)c.Cout * c.Himg * c.Wimg / G));
  return 0;
}

int64_t workspace_bytes(const FModel* m) { return m->bytes; }
void set_math(FModel* m, int math) { m->math = math; }
void set_tuning(FModel* m, const vv::Tuning* t) { m->tune = t; }
int in_channels(const FModel* m) { return m->c.Cin; }
int out_channels(const FModel* m) { return m->c.Cout; }
int img_h(const FModel* m) { return m->c.Himg; }
int img_w(const FModel* m) { return m->c.Wimg; }

}  // namespace vvf

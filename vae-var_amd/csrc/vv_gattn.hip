// Global-window attention of LGUnet_all_1's LG layer 0 (networks/LGUnet_all.py:689, 696: one window over the whole
// LG grid, 16,200 tokens at 0.25 degree; Attention.py:599-664 SD_attn without mask), softmax(q k^T) v per head, as
// one flash-style MFMA kernel: keys and values stream through LDS, the scores never reach HBM.
//
// Arithmetic: fp32 results from fp16 MFMAs (the fp16x3 form of vv_gemm.hip) for both products.
//   S = q . k   q rows scaled by 2^eq (per token and head, max |q| to [2^14, 2^15)), k by ONE 2^ek per head
//               (a per-head scale keeps the error of every logit below 2^-22 of the largest |q_i . k|, which is
//               what the softmax is sensitive to); q = h + l, k = h + l in fp16, three products (l h, h l, h h)
//   O = P v     P = exp(s - m) <= 1 scaled by 2^14, v by one 2^ev per head; three products again
// Everything else (scales, online softmax with its rescales, the final 1 / sum) is fp32.
//
// Layout (written by k_gattn_prep, read straight by the kernel):
//   Q, K  per head, per 16-token block t and 32-deep d-step s and plane p: one 1 KB "fragment block", lane l holding
//         the 8 fp16 [token 16 t + (l & 15)][d 32 s + 8 (l >> 4) .. + 7] -- exactly the operand of one
//         v_mfma_f32_16x16x32_f16, so every fragment read is one lane-linear ds_read_b128 (no bank conflicts);
//   V^T   per head, per 32-key block and 16-wide d-block and plane: one 1 KB block, lane l (g = l >> 4) holding
//         v[key pi(g, j)][d 16 db + (l & 15)], j = 0..7, pi(g, j) = j < 4 ? 4 g + j : 16 + 4 g + j - 4: the key
//         order in which the score accumulator S^T (keys on the rows of a 16x16 C tile: 4 g + r) already holds
//         P^T, so P^T is the B operand of O^T += V^T P^T with no data movement (k order permuted identically in
//         both operands, cdna_hip_programming.md §3 'An accumulator tile as the next MFMA's operand').
// Tokens past N are zero and their scores are masked to -inf.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "vv_kernels.h"

namespace vv {

namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_t;

constexpr int kQB = 128;         // queries per workgroup: QF 16-query column blocks per wave x 8 / QF waves
constexpr int kKB = 32;          // keys per LDS stage
constexpr int kVmaxBlocks = 64;  // partial-maximum blocks of k_gattn_max

__device__ __forceinline__ unsigned absmax_bits(float x) { return __float_as_uint(fabsf(x)); }
// 2^(141 - e(m)): the scale that puts a maximum m (as bits) into [2^14, 2^15) (k_rowscale's formula)
__device__ __forceinline__ float scale_of(unsigned mx) { return __uint_as_float((268u - max(mx >> 23, 15u)) << 23); }

// per head: max |k| and max |v| over all tokens, as partial maxima of kVmaxBlocks blocks (no atomics, no memset)
__global__ __launch_bounds__(256) void k_gattn_max(GattnArgs a, unsigned* __restrict__ part) {
  const int h = blockIdx.y, hd = a.C / a.heads;
  unsigned mk = 0, mv = 0;
  for (int t = blockIdx.x; t < a.N; t += gridDim.x) {
    const float* row = a.qkv + (size_t)t * 3 * a.C + h * hd;
    for (int d = threadIdx.x; d < hd; d += 256) {
      mk = max(mk, absmax_bits(row[a.C + d]));
      mv = max(mv, absmax_bits(row[2 * a.C + d]));
    }
  }
  for (int o = 32; o; o >>= 1) {
    mk = max(mk, (unsigned)__shfl_xor((int)mk, o));
    mv = max(mv, (unsigned)__shfl_xor((int)mv, o));
  }
  __shared__ unsigned red[2][4];
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = mk;
    red[1][threadIdx.x >> 6] = mv;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    const unsigned m = max(max(red[threadIdx.x][0], red[threadIdx.x][1]), max(red[threadIdx.x][2], red[threadIdx.x][3]));
    part[((size_t)h * 2 + threadIdx.x) * kVmaxBlocks + blockIdx.x] = m;
  }
}

// one workgroup per (32-token block, head): q planes with per-token scales, k and v^T planes with the head's scales
__global__ __launch_bounds__(256) void k_gattn_prep(GattnArgs a, const unsigned* __restrict__ part) {
  const int b = blockIdx.x, h = blockIdx.y, hd = a.C / a.heads, KS = hd / 32, tid = threadIdx.x;
  extern __shared__ float sm[];           // q, k, v of the 32 tokens: [3][32][hd + 1]
  const int ld = hd + 1;
  float* sq = sm;
  float* sk = sm + 32 * ld;
  float* sv = sm + 64 * ld;
  __shared__ float qsc[32];
  __shared__ float hsc[2];
  if (tid < 2) {
    unsigned m = 0;
    for (int i = 0; i < kVmaxBlocks; ++i) m = max(m, part[((size_t)h * 2 + tid) * kVmaxBlocks + i]);
    hsc[tid] = scale_of(m);
  }
  for (int e = tid; e < 32 * hd; e += 256) {
    const int r = e / hd, d = e - r * hd, t = 32 * b + r;
    const float* row = a.qkv + (size_t)t * 3 * a.C + h * hd + d;
    const bool ok = t < a.N;
    sq[r * ld + d] = ok ? row[0] : 0.f;
    sk[r * ld + d] = ok ? row[a.C] : 0.f;
    sv[r * ld + d] = ok ? row[2 * a.C] : 0.f;
  }
  __syncthreads();
  if (tid < 32 * 8) {  // per-token q scale: 8 lanes per token
    const int r = tid >> 3, sl = tid & 7;
    unsigned m = 0;
    for (int d = sl; d < hd; d += 8) m = max(m, absmax_bits(sq[r * ld + d]));
    for (int o = 4; o; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o));
    if (sl == 0) qsc[r] = scale_of(m);
  }
  __syncthreads();
  if (tid < 32) {  // 2^-eq_i 2^-ek of the head: what the kernel multiplies every score of query t by
    const float iq = __uint_as_float((254u << 23) - __float_as_uint(qsc[tid]));
    const float ik = __uint_as_float((254u << 23) - __float_as_uint(hsc[0]));
    a.qs[(size_t)h * a.Np + 32 * b + tid] = iq * ik;
  }
  const float ks = hsc[0], vs = hsc[1];
  // Q / K fragment blocks of this 32-token block: 2 token blocks x KS d-steps x 2 planes, 64 lanes x 8 halfs each
  unsigned short* Qo = a.qp + ((size_t)h * a.Np + 32 * b) * 2 * hd;
  unsigned short* Ko = a.kp + ((size_t)h * a.Np + 32 * b) * 2 * hd;
  unsigned short* Vo = a.vp + ((size_t)h * a.Np + 32 * b) * 2 * hd;
  const int nq = 2 * KS * 64;  // (token block, d-step, lane) items per plane pair
  for (int it = tid; it < nq; it += 256) {
    const int lane = it & 63, s = (it >> 6) % KS, tb = (it >> 6) / KS;
    const int r = 16 * tb + (lane & 15), d0 = 32 * s + 8 * (lane >> 4);
    h8 qh, ql, kh, kl;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float x = sq[r * ld + d0 + j] * qsc[r];
      qh[j] = (_Float16)x;
      ql[j] = (_Float16)(x - (float)qh[j]);
      const float y = sk[r * ld + d0 + j] * ks;
      kh[j] = (_Float16)y;
      kl[j] = (_Float16)(y - (float)kh[j]);
    }
    // block index (tb, s, p): ((tb * KS + s) * 2 + p) KB
    const size_t o = ((size_t)(tb * KS + s) * 2) * 512 + lane * 8;
    *reinterpret_cast<h8*>(Qo + o) = qh;
    *reinterpret_cast<h8*>(Qo + o + 512) = ql;
    *reinterpret_cast<h8*>(Ko + o) = kh;
    *reinterpret_cast<h8*>(Ko + o + 512) = kl;
  }
  // V^T fragment blocks: hd / 16 d-blocks x 2 planes
  const int nv = (hd / 16) * 64;
  for (int it = tid; it < nv; it += 256) {
    const int lane = it & 63, db = it >> 6, g = lane >> 4;
    const int d = 16 * db + (lane & 15);
    h8 vh, vl;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int key = j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4);
      const float x = sv[key * ld + d] * vs;
      vh[j] = (_Float16)x;
      vl[j] = (_Float16)(x - (float)vh[j]);
    }
    const size_t o = ((size_t)db * 2) * 512 + lane * 8;
    *reinterpret_cast<h8*>(Vo + o) = vh;
    *reinterpret_cast<h8*>(Vo + o + 512) = vl;
  }
  if (b == 0 && tid == 0) a.vsc[h] = __uint_as_float((254u << 23) - __float_as_uint(vs)) * (1.0f / 16384.0f);
}

// softmax(q k^T) v for one head and 128 queries (8 waves of 16 or 4 of 32). Per 32-key block (three-stage LDS
// ring filled by LDS-DMA): S^T = K Q^T (36 QF MFMAs per wave), online softmax on S^T in registers (the keys of a
// query live on 4 registers x 4 lane groups x 2 blocks), O^T += V^T P^T (36 QF MFMAs). KS = head_dim / 32.
template <int KS, int QF>
__global__ __launch_bounds__(64 * 8 / QF, 1) void k_gattn(GattnArgs a) {
  constexpr int HD = 32 * KS, DB = HD / 16;
  constexpr int kWaves = 8 / QF, kQW = 16 * QF;  // QF = 2: one wave per SIMD (~300 registers); 1: two per SIMD
  constexpr int KBLK = 2 * KS * 2, VBLK = DB * 2, SKB = KBLK + VBLK;  // 1 KB blocks per stage (48 at hd 192)
  constexpr int PW = SKB / kWaves;                                    // DMA instructions per wave per stage
  static_assert(SKB % kWaves == 0, "stage blocks per wave");
  extern __shared__ __attribute__((aligned(16))) unsigned short lds[];
  const int h = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int q0 = blockIdx.x * kQB + wave * kQW;
  const int N = a.N, nb = (N + kKB - 1) / kKB;
  const unsigned short* Kg = a.kp + (size_t)h * a.Np * 2 * HD;
  const unsigned short* Vg = a.vp + (size_t)h * a.Np * 2 * HD;

  // this wave's Q fragments (B operands of S^T = K Q^T) and score scales, for the whole kernel
  h8 qf[QF][KS][2];
  const unsigned short* Qg = a.qp + ((size_t)h * a.Np + q0) * 2 * HD + lane * 8;
#pragma unroll
  for (int j = 0; j < QF; ++j)
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int p = 0; p < 2; ++p) qf[j][s][p] = *reinterpret_cast<const h8*>(Qg + ((j * KS + s) * 2 + p) * 512);
  float qsc[QF];
#pragma unroll
  for (int j = 0; j < QF; ++j) qsc[j] = a.qs[(size_t)h * a.Np + q0 + 16 * j + (lane & 15)];

  auto stage = [&](int b, int buf) {
    unsigned short* S = lds + buf * SKB * 512;
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int c = wave + kWaves * i;
      const unsigned short* src = c < KBLK ? Kg + ((size_t)b * KBLK + c) * 512 : Vg + ((size_t)b * VBLK + c - KBLK) * 512;
      __builtin_amdgcn_global_load_lds((const void*)(src + lane * 8), (lds_t)(S + c * 512), 16, 0, 0);
    }
  };

  f4v O[DB][QF];
#pragma unroll
  for (int d = 0; d < DB; ++d)
#pragma unroll
    for (int j = 0; j < QF; ++j) O[d][j] = f4v{0.f, 0.f, 0.f, 0.f};
  float m[QF], lsum[QF];
#pragma unroll
  for (int j = 0; j < QF; ++j) m[j] = -INFINITY, lsum[j] = 0.f;

  // S^T(b) = K(b) Q^T: rows = keys 16 kb + 4 g + r, columns = queries 16 j + (lane & 15)
  auto smfma = [&](int b, f4v (&sc)[2][QF]) {
    const unsigned short* S = lds + (b % 3) * SKB * 512 + lane * 8;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int j = 0; j < QF; ++j) sc[kb][j] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        const h8 kh = *reinterpret_cast<const h8*>(S + ((kb * KS + s) * 2) * 512);
        const h8 kl = *reinterpret_cast<const h8*>(S + ((kb * KS + s) * 2 + 1) * 512);
#pragma unroll
        for (int j = 0; j < QF; ++j) {
          sc[kb][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kl, qf[j][s][0], sc[kb][j], 0, 0, 0);
          sc[kb][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kh, qf[j][s][1], sc[kb][j], 0, 0, 0);
          sc[kb][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kh, qf[j][s][0], sc[kb][j], 0, 0, 0);
        }
      }
  };
  // online softmax of block b per query column: P (scaled by 2^14, split into fp16 planes in the B-operand order of
  // the PV product), the rescale alpha of what O holds, the running max and the lane-partial row sums
  auto softmax = [&](int b, f4v (&sc)[2][QF], h8 (&ph)[QF], h8 (&pl)[QF], float (&alpha)[QF]) {
#pragma unroll
    for (int j = 0; j < QF; ++j) {
      float mb = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = b * kKB + 16 * kb + 4 * g + r;
          const float x = key < N ? sc[kb][j][r] * qsc[j] : -INFINITY;
          sc[kb][j][r] = x;
          mb = fmaxf(mb, x);
        }
      mb = fmaxf(mb, __shfl_xor(mb, 16));
      mb = fmaxf(mb, __shfl_xor(mb, 32));
      const float mn = fmaxf(m[j], mb);
      alpha[j] = expf(m[j] - mn);
      m[j] = mn;
      float ps = 0.f;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = expf(sc[kb][j][r] - mn);
          ps += p;
          const float x = p * 16384.0f;
          const _Float16 hv = (_Float16)x;
          ph[j][4 * kb + r] = hv;
          pl[j][4 * kb + r] = (_Float16)(x - (float)hv);
        }
      lsum[j] = lsum[j] * alpha[j] + ps;
    }
  };
  // O^T += V^T(b) P^T(b): rows = d 16 db + 4 g + r, columns = queries
  auto pv = [&](int b, const h8 (&ph)[QF], const h8 (&pl)[QF]) {
    const unsigned short* S = lds + (b % 3) * SKB * 512 + lane * 8;
#pragma unroll
    for (int db = 0; db < DB; ++db) {
      const h8 vh = *reinterpret_cast<const h8*>(S + (KBLK + db * 2) * 512);
      const h8 vl = *reinterpret_cast<const h8*>(S + (KBLK + db * 2 + 1) * 512);
#pragma unroll
      for (int j = 0; j < QF; ++j) {
        O[db][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vh, pl[j], O[db][j], 0, 0, 0);
        O[db][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vl, ph[j], O[db][j], 0, 0, 0);
        O[db][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vh, ph[j], O[db][j], 0, 0, 0);
      }
    }
  };

  // Per key block b: the DMA of block b + 2 (clamped: the last two iterations re-stage the last block into a buffer
  // nobody reads again), S(b), the softmax, O = O alpha + V^T P^T; then wait for my block b + 1 pieces (those of
  // b + 2 may stay in flight) and barrier (everyone's b + 1 landed; everyone's reads of the buffer b + 2
  // overwrites, block b - 1, retired before the previous barrier) -- k_gemm_h4's ring protocol.
  stage(0, 0);
  stage(min(1, nb - 1), 1);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PW) : "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  for (int b = 0; b < nb; ++b) {
    stage(min(b + 2, nb - 1), (b + 2) % 3);
    f4v sc[2][QF];
    smfma(b, sc);
    h8 ph[QF], pl[QF];
    float alpha[QF];
    softmax(b, sc, ph, pl, alpha);
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int j = 0; j < QF; ++j) O[db][j] *= alpha[j];
    pv(b, ph, pl);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PW) : "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // 1 / row sum (the lane partial sums of a query over its 4 lane groups) and the head's V / P scales
  const float vs = a.vsc[h];
#pragma unroll
  for (int j = 0; j < QF; ++j) {
    float l = lsum[j];
    l += __shfl_xor(l, 16);
    l += __shfl_xor(l, 32);
    const int q = q0 + 16 * j + (lane & 15);
    if (q >= N) continue;
    const float f = vs / l;
    float* o = a.out + (size_t)q * a.ldo + h * HD + 4 * g;
#pragma unroll
    for (int db = 0; db < DB; ++db) *reinterpret_cast<f4v*>(o + 16 * db) = O[db][j] * f;
  }
}

}  // namespace

size_t gattn_np(int N) { return (size_t)(N + kQB - 1) / kQB * kQB; }

size_t gattn_ws_bytes(int N, int C, int heads) {
  const size_t Np = gattn_np(N);
  return 3 * Np * C * 2 * sizeof(unsigned short) + (size_t)heads * Np * sizeof(float) +
         (size_t)heads * 2 * kVmaxBlocks * sizeof(unsigned) + (size_t)heads * sizeof(float) + 1024;
}

bool gattn_supported(int C, int heads) {
  const int hd = heads > 0 ? C / heads : 0;
  return heads > 0 && C % heads == 0 && (hd == 64 || hd == 96 || hd == 128 || hd == 192);
}

hipError_t gattn(const float* qkv, float* out, int ldo, int N, int C, int heads, void* ws, hipStream_t st,
                 int qf_per_wave) {
  if (!qkv || !out || !ws || N <= 0 || !gattn_supported(C, heads) || ldo < C || (ldo & 3)) return hipErrorInvalidValue;
  GattnArgs a;
  a.qkv = qkv;
  a.out = out;
  a.ldo = ldo;
  a.N = N;
  a.Np = (int)gattn_np(N);
  a.C = C;
  a.heads = heads;
  char* p = reinterpret_cast<char*>(ws);
  const size_t plane = (size_t)a.Np * C * 2 * sizeof(unsigned short);
  a.qp = reinterpret_cast<unsigned short*>(p);
  a.kp = reinterpret_cast<unsigned short*>(p + plane);
  a.vp = reinterpret_cast<unsigned short*>(p + 2 * plane);
  a.qs = reinterpret_cast<float*>(p + 3 * plane);
  unsigned* part = reinterpret_cast<unsigned*>(a.qs + (size_t)heads * a.Np);
  a.vsc = reinterpret_cast<float*>(part + (size_t)heads * 2 * kVmaxBlocks);
  const int hd = C / heads;
  hipLaunchKernelGGL(k_gattn_max, dim3(kVmaxBlocks, heads), dim3(256), 0, st, a, part);
  const size_t lp = 3 * 32 * (size_t)(hd + 1) * sizeof(float);
  if (lp > 65536)  // head dim 192: 74 KB
    if (hipError_t e = set_lds_limit((const void*)k_gattn_prep, 3 * 32 * (size_t)(192 + 1) * sizeof(float))) return e;
  hipLaunchKernelGGL(k_gattn_prep, dim3(a.Np / 32, heads), dim3(256), lp, st, a, (const unsigned*)part);
  const dim3 grid(a.Np / kQB, heads);
  const int qf = qf_per_wave == 1 ? 1 : 2;
  switch (hd / 32 * 4 + qf) {
#define GA(KS, QF)                                                                                          \
  case KS * 4 + QF: {                                                                                       \
    constexpr size_t lds = 3 * (2 * KS * 2 + KS * 2 * 2) * 1024;                                            \
    if (hipError_t e = set_lds_limit((const void*)k_gattn<KS, QF>, lds)) return e;                         \
    hipLaunchKernelGGL((k_gattn<KS, QF>), grid, dim3(64 * 8 / QF), lds, st, a);                             \
    break;                                                                                                  \
  }
    GA(2, 1) GA(3, 1) GA(4, 1) GA(6, 1) GA(2, 2) GA(3, 2) GA(4, 2) GA(6, 2)
#undef GA
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace vv

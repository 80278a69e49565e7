// Internal kernel interface of libvaevar (not the public C-ABI; see include/vaevar.h).
// All kernels are fp32, gfx950-only, launched on the caller's stream.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <string>

namespace vv {

constexpr int kMaxGroups = 8;

// Per-context tuning knobs (vv_set_tuning / vv_get_tuning): the measured routing choices of the GEMM and
// attention dispatch, kept settable so that A/B runs need no rebuild. The defaults are the shipped choices
// (DESIGN.md §3 / §9 give the measurements behind each one); kernels never read them, only host dispatch does.
struct Tuning {
  int h3_mink = 768;            // smallest K sent to the fp16x3 kernels (profiles/r02/mink)
  int fc_h3_mink = 192;         // ... in the forecast network LGUnet_all_1 (profiles/r03/fcst_mink)
  int h3_big = 1;               // 256x128 fp16x3 tiles where they measured faster (profiles/r02/h3big)
  int h3_mf16 = 1;              // the 16x16x32-MFMA form of the 256x128 tile for N 2048..4095 x short K
  int small_split = 1;          // whole-grid split-K of sub-chip fp16x3 GEMMs
  int small_split_minkt = 24;   // k-tiles per chunk at least, for that split (profiles/r02/smallk)
  int tail_minkt = 12;          // k-tiles per chunk at least, for the split-K tail (profiles/r02/tailk)
  int ln_scales = 1;            // fp16x3 row scales from the LayerNorm producer (0: k_rowscale everywhere)
  int h4 = 1;                   // the split-operand LDS-DMA fp16x3 kernel (tile 48) where the 256x128 tiles run
  int ln_planes = 1;            // LayerNorm writes the fp16x3 planes of the tile-48 GEMM it feeds (no split pass)
  int h4_small = 1;             // tile 48 + whole-chip split-K also for 64..143 256-row tiles (1152 x 1152 at 2048 rows):
                                // neutral while the proj GEMM needed its own split pass (77.5 / 77.4 off vs 77.4 / 76.3 on,
                                // profiles/r03/ab_h4small); with the attention writing its planes (attn_planes) 86.9 / 86.6
                                // on vs 81.0 / 81.8 off, same box (profiles/r03/ab_attn_planes)
  int h4_split_minkt = 12;      // k-tiles per chunk at least, for that split of tile 48
  int h5 = 1;                   // tile 49 (256 x 144, k_gemm_h5) where its tiles fill whole rounds and tile 48's do not
  int fc_conv_mf = 1;           // LGUnet_all_1 PatchEmbed / ConvTranspose2d as direct MFMA kernels (0: im2col / col2im + GEMM)
  int gattn = 1;                // LGUnet_all_1 global window: the flash MFMA kernel (0: split GEMMs / streaming kernel)
  int gattn_qf = 1;             // its 16-query blocks per wave (1: 8 waves, two per SIMD; 2: 4 waves of 32 queries)
  int win_attn = 1;             // LGUnet_all_1: the LDS window-attention kernel for small windows (0: streaming)
  int win_mfma = 1;             // ... on the exact-f32 MFMA (0: the VALU kernel)
  int fuse_mlp = 3;             // the fused Swin-tower MLP sub-block (vv_tower.hip): bit 0 at dim 96, bit 1 at dim 192
  int attn_mfma = 1;            // LG-stage window attention (hd 192) on the exact-f32 MFMA (0: the VALU kernels)
  int attn_planes = 1;          // the LG-stage attention forward writes the fp16x3 planes of a tile-48 proj GEMM
  int fixup_ln = 1;             // the proj GEMM's split-K fixup fused into the LG-stage LN2 (gemm_ln)
  int gelu_planes = 1;          // the LG-stage fc1 (GELU) / fc2-input-gradient (gelu') GEMMs write the fp16x3 planes of
                                // the K = 4C GEMM that follows (bound-derived row scales: no k_rowsplit pass)
  int fixup_ln_rows = 1;        // the fused fixup + LN1 walks GEMM rows in order through the inverse window map
  int h4_gather = 1;            // tiles 48 / 49 read gathered producer row scales through arow themselves (tile 49: the
                                // STORE / RESID epilogues, k_gemm_h5<EPI, true>; 0: k_gather_scales)
  int mlp_hc = 2;               // the fused dim-192 MLP: hidden units per chunk (32 or 64: fewer chunk steps, 151 KB LDS),
                                // or 2: 32-unit chunks, the hidden layer split over two waves per 16 tokens
  int fuse_attn = 3;            // the fused Swin-tower attention sub-block (vv_tower.hip) at dim 96: bit 0 the forward,
                                // bit 1 the backward (r03: neutral; r04: closure 8.56 vs 8.69 ms, same box, profiles/r04/ab_r04j)
  int h5_split = 1;             // gemm_ln: tile 49 with every tile split P / T ways (64 tiles x 4 = 256 workgroups for the
                                // N = 1152 GEMMs at 2048 rows) instead of tile 48's 72 tiles x 3 = 216 (r06: closure 16.62 ->
                                // 16.56 ms same process, profiles/r06/knob_ab_h5_split.jsonl); later in r06 also gemm_nt's
                                // plain N = 1152 split GEMMs (k_gemm_fixup49): 16.649 / 16.671 -> 16.585 / 16.594 ms with
                                // both, profiles/r06/knob_ab_h5_split_r06t.jsonl
  int fixup_stage = 1;          // the fused fixup + LayerNorm sums a workgroup's 8 rows of split-K partials with whole
                                // 128-B line reads into LDS first (0: each row's loads straight from the partials)
  int grid_fused = 1;           // interpolated state grids (config 5): the one-pass misfit k_misfit_grid + the network-grid
                                // adjoint k_misfit_net_bwd (0: k_misfit_fwd / k_misfit_bwd_gather / k_flow_input(_adj));
                                // 1: 3 rows of a band in flight per pass (more waves per SIMD), 2: 6 rows (r05: misfit
                                // class 0.404 vs 0.480 ms / eval at 721x1440, profiles/r05/knob_ab_grid_mr_r05g.jsonl);
                                // read by vv_bind_problem
  int host_wait = 1;            // the host's wait in vv_reduce_batch (vv_engine.hip host_sync): 0 hipStreamSynchronize
                                // (a busy CPU), 1 sleep + hipStreamQuery polls (r06: main thread 1.00 -> 0.04 CPU at
                                // equal throughput, 51.91 / 51.89 vs 51.91 / 52.01 it/s, profiles/r06/host_wait_ab)
  int bs_tile = 27;             // the bf16x6 tile of the short-K tower GEMMs: 27 = 64x64 with one LDS buffer (24 KB: four
                                // workgroups per CU; r06: closure 16.816 / 16.856 -> 16.780 / 16.800 ms, bf16x6 class
                                // 1.206 -> 1.186 ms / eval, bit-identical, profiles/r06/knob_ab_bs_tile.jsonl); 24 the
                                // two-buffer form (r05), 25 128x64, 26 loads two k-tiles ahead (both slower)
  int fixup_ln_cross = 1;       // the fused fixup + LN1 also across consecutive LG stages (the last fc2 of a stage + the
                                // next stage's first LN1; 0: tile-48 split + fixup + a separate LayerNorm there)
  int patch_pers = 1;           // the decoder PatchEmbed / ConvTranspose2d kernels in their persistent form (one workgroup
                                // of 8 waves per CU share, weights staged once, each wave prefetching its next 16-token
                                // tile behind the current one's MFMAs; 0: one 64-token workgroup per tile, bit-identical;
                                // r06: patch class 0.295 -> 0.177 ms / eval, profiles/r06/knob_ab_patch_pers.jsonl)
};
extern const Tuning kDefaultTuning;
// the tuning key names (vv_set_tuning); returns the field or null
int* tuning_field(Tuning& t, const char* key);
// whether `value` is one the dispatch of `key` accepts (vv_set_tuning rejects the others with VV_E_ARG)
bool tuning_value_ok(const char* key, int value);

// ---------------------------------------------------------------------------
// GEMM: C[o(r)][n] = epi( sum_k A(r,k) * B[n][k] )      (B is [N][K] = nn.Linear weight)
//   A(r,k) = k <  ksplit : A [arow ? arow[r] : r][k]          (row stride lda)
//            k >= ksplit : A2[r][k - ksplit]                  (row stride lda2) -- torch.cat on -1
//   o(r)   = crow ? crow[r] : r
// ---------------------------------------------------------------------------
enum Epi : int {
  EPI_STORE = 0,   // C = acc (+bias)
  EPI_GELU = 1,    // aux = acc + bias (unless aux is null) ; C = gelu(acc + bias)   (Mlp fc1 fwd, swinblock.py:23-29)
  EPI_RESID = 2,   // C = R[o % rmod] + acc (+bias)            (residual adds)
  EPI_DGELU = 3,   // C = acc * gelu'(aux[o])                  (fc1 backward)
};

struct GemmGroup {
  const float* A;
  const float* A2;
  const float* B;
  const float* bias;
  float* C;
  const float* R;
  float* aux;
  const unsigned short* Bp;  // filled in by gemm_nt: bf16 split planes of B (registered weight arena) or null
  const unsigned short* Ap;  // bf16 split planes of A, rows [3][lda] (caller-provided or registered), or null
  const unsigned short* Bh;  // filled in by gemm_nt (GEMM_SPLIT16): fp16 planes of B, per row 2K halfs chunk-interleaved
                             // ([h(k 0..31) | l(k 0..31) | h(k 32..63) | ...]), or null
  const float* Bs;           // ... and the row scales: row n of B has 2^-e = Bs[n * K / 32]
};

struct GemmArgs {
  int M, N, K, ksplit;
  int lda, lda2, ldc, ldr, ldaux;
  int ldb;  // row stride of B (0 = K); a registered weight (split planes) is always contiguous
  int rmod;
  const int* arow;
  const int* crow;
  int epi;
  int ngroups;
  // tail split (filled in by gemm_nt): the first tdp tiles run whole; each remaining tile is split into
  // tsplit k-chunks whose fp32 partials go to ws and are summed (in chunk order) by the fixup kernel
  int tdp, tsplit;
  // m-blocks per group of the grouped tile order (filled in by gemm_nt: ~sqrt(tiles per XCD x BN / BM), so the
  // block of tiles one XCD runs re-reads the least A + B through the fabric)
  int gm;
  float* ws;
  int math;  // GemmMath of this GEMM (the context's setting)
  // GEMM_SPLIT16: null, or the row scales of A as its producer wrote them (LayerNorm rs), indexed by the physical A
  // row (arow[r] when gathered), z * M + row; the fp16x3 kernels then skip k_rowscale (no concat A2 allowed)
  const float* ascale;
  int ascale_phys;  // set by gemm_nt: the kernel indexes its row scales by physical row
  int agather;      // set by launch_h4 (tile 48, producer planes, gathered rows): ascale[arow[r]] read in the kernel
  // GEMM_SPLIT16 tile 48: workspace for A's fp16 planes in GEMM row order (groups x M x 2K halfs), or null
  unsigned short* apl;
  size_t apl_halfs;
  // null, or A's planes as its producer wrote them (LayerNorm pl, same layout, indexed by the physical A row like
  // ascale, which must be set); tile 48 then reads them directly (no k_rowsplit pass)
  const unsigned short* apre;
  // tile 48, EPI_GELU / EPI_DGELU only (ngroups 1, no crow): write the result as fp16x3 A planes of the next tile-48
  // GEMM (opl, k_rowsplit's layout, N halfs x 2 per row) and their row scales (ors) instead of fp32 C. The row scale
  // comes from an a-priori bound on |C| (no pass over the output, no cross-tile row maximum):
  //   |C[r][n]| <= f (K max|A_r| max|B| + max|bias|),  f = 1 (GELU: |gelu(x)| <= |x|), 1.25 (DGELU: |gelu'| < 1.13)
  // with max|A_r| < 2^15 2^-e_r from A's own row scale and max|B|, max|bias| device scalars (obw, obb or null).
  unsigned short* opl;
  float* ors;
  const float* obw;
  const float* obb;
  const float* escale;  // set by the tile-48 launch: A's row scales in GEMM row order (what the kernel used)
  int nofix;            // set by gemm_ln: the split-K partials are summed by the consumer (no fixup launch)
  int t49;              // set by gemm_ln: the partials are tile 49's (256 x 144 tiles, fragment order of k_gemm_h5)
  const Tuning* tune;  // host-side dispatch knobs of the owning context (null: kDefaultTuning); never read on the device
  int h3_mink;         // > 0: this GEMM's own smallest K for the fp16x3 kernels (the forecast: Tuning.fc_h3_mink)
  GemmGroup g[kMaxGroups];
};

// Global-window attention (vv_gattn.hip): out[t][h hd + d] = softmax_j(q_t . k_j) v_j per head, for N tokens of a
// qkv buffer [N][3C] (q already scaled / rotated); fp16x3 MFMA products, fp32 softmax. ws: gattn_ws_bytes().
struct GattnArgs {
  const float* qkv;
  float* out;
  int ldo, N, Np, C, heads;
  unsigned short *qp, *kp, *vp;  // fragment-ordered fp16 planes (k_gattn_prep)
  float* qs;                     // [heads][Np] score scale per query: 2^-eq 2^-ek
  float* vsc;                    // [heads] output scale 2^-ev 2^-14
};
// raise a kernel's dynamic-LDS limit to `lds` once per (kernel, device) (hipFuncSetAttribute acts on the current
// device; locked, so concurrent contexts on several devices are safe). The first value set for a kernel stays: callers
// whose LDS varies pass their maximum.
hipError_t set_lds_limit(const void* k, size_t lds);
int device_cus();  // compute units of the current device (cached)
// the split-operand fp16x3 kernels that read producer planes (GemmArgs.apre) and write them (opl): tiles 48, 49
bool gemm_plane_tile(int t);
bool gattn_supported(int C, int heads);
size_t gattn_ws_bytes(int N, int C, int heads);
// qf_per_wave: 16-query blocks per wave (2: 4 waves of 32 queries, one per SIMD; 1: 8 waves of 16, two per SIMD)
hipError_t gattn(const float* qkv, float* out, int ldo, int N, int C, int heads, void* ws, hipStream_t st,
                 int qf_per_wave = 1);

// ws: scratch of at least gemm_ws_floats() floats (may be null: no tail split)
hipError_t gemm_nt(const GemmArgs& a, hipStream_t s, int tile_hint = -1, float* ws = nullptr);

// A residual GEMM whose split-K fixup is fused into the LayerNorm that consumes its output (tile 48 with every tile
// split, EPI_RESID, one group, N <= 1280): one row per wave sums the S chunk partials in chunk order, adds bias and
// residual (the fixup epilogue's arithmetic), stores the row x at its output row, then runs k_ln_fwd's LayerNorm
// on it (the same reductions, so bit-identical to fixup + k_ln_fwd) and writes fp16x3 planes, row scales and stats.
// LN row j reads GEMM row gmap[j] (null: j); its output row is the x row written (lo_x) or j.
struct GemmLnArgs {
  const int* gmap;
  const int* ginv;  // the inverse of gmap (or null): workgroups then walk GEMM rows in order (partial lines stay local)
  int lo_x;
  const float* gamma;
  const float* beta;
  float eps;
  unsigned short* pl;  // planes [row][2N] (k_rowsplit's layout)
  float* rs;           // row scales
  float* stats;        // (mean, rstd) per row (the backward reads them)
  // backward (bwd = 1; the GEMM: EPI_STORE without bias, its output dy = C is not stored): k_ln_bwd on LN row j with
  // dy = GEMM row j, x / res / y (in place allowed) and pl / rs at row lmap[j] (null: j), stats at j; y, x, res row
  // stride N. pl may be null (no planes wanted), rs may be null with it.
  int bwd;
  const int* lmap;
  const float* x;
  const float* res;
  float* y;
};
// VV_E-style: hipErrorNotSupported when the GEMM does not take this form (the caller then runs gemm_nt + LayerNorm)
hipError_t gemm_ln(const GemmArgs& a, const GemmLnArgs& l, hipStream_t s, float* ws);
// the LayerNorm half (vv_ops.hip), launched by gemm_ln with the GEMM's final arguments (tdp, tsplit, gm)
hipError_t fixup_ln_launch(const GemmArgs& a, const GemmLnArgs& l, hipStream_t s);
// the kernel gemm_nt would run for `a` (tile hint -1: the routed choice, incl. the fallbacks), so a producer can
// decide what form to write A in (tile 48: fp16x3 planes)
int gemm_tile_of(const GemmArgs& a, int tile_hint = -1);
size_t gemm_ws_floats();

// GEMM arithmetic:
//   GEMM_F32     v_mfma_f32_32x32x2_f32 (exact f32 fma chain)
//   GEMM_SPLIT   fp32 operands split into three bf16 planes, six v_mfma_f32_32x32x16_bf16 products
//   GEMM_SPLIT16 fp32 operands scaled by a power of two per row (A and B) and split
//                into two fp16 planes, three v_mfma_f32_32x32x16_f16 products (both fp32-level error)
enum GemmMath : int { GEMM_F32 = 0, GEMM_SPLIT = 1, GEMM_SPLIT16 = 2 };
// tile hints gemm_nt accepts (the product kernels; see vv_gemm.hip)
bool valid_tile(int t);
// Weight arenas with precomputed split planes. The planes buffer of an arena of n floats holds, at these
// offsets (split_arena_bytes(n) bytes in all):
//   bf16: [0, 3n) unsigned shorts; row r of the [N][K] operand at float offset o = B - base: 3*(o + r*K) = h[K], m[K], l[K]
//   fp16: [3n, 5n) unsigned shorts; at 3n + 2*(o + r*K): the row scaled by 2^e as h / l fp16 planes, interleaved
//         per 32-element k-chunk (h(32) | l(32) per chunk: one 128-B line per row and k-tile)
//   row scales: floats after that; 2^-e of the row starting at float offset f at index f / 32
size_t split_arena_bytes(size_t n);
void register_split_arena(const float* base, size_t n, const unsigned short* planes);
void unregister_split_arena(const float* base);
// fill the planes of the rows of W[n/K][K], which lies inside a registered arena (W - base and K multiples of 32)
hipError_t split_registered(const float* W, size_t n, int K, hipStream_t s);
// out[0] = max |x[i]| over n floats (one workgroup; load-time bounds of the plane-writing GEMM epilogues)
hipError_t absmax(const float* x, size_t n, float* out, hipStream_t s);
// dst[n/K][3][K] = exact bf16 split of the rows of src[n/K][K] (h = bf16(x), m = bf16(x-h), l = bf16(x-h-m))
hipError_t split_planes(const float* src, unsigned short* dst, size_t n, int K, hipStream_t s);

// ---------------------------------------------------------------------------
// LayerNorm over the last dim, one wave per output row.
// ---------------------------------------------------------------------------
enum LnMode : int {
  LN_ROWMAP = 0,   // in row = map ? map[r] : r
  LN_MERGE = 1,    // PatchMerging gather (transformer.py:86-91): row (b,h,w) of the half grid,
                   // feature q*Cs + c, q = dh + 2*dw, from token (b, 2h+dh, 2w+dw) of (Hin,Win)
  LN_EXPAND = 2,   // PatchExpand rearrange (transformer.py:114): out (b,y,x) <- in row (b,y/2,x/2),
                   // segment (y%2)*2 + x%2 of width C; (Hin,Win) = half grid
};

struct LnGroup {
  const float* x;     // input
  const float* gamma;
  const float* beta;
  float* y;           // output (fwd) / dx destination (bwd)
  float* stats;       // [rows][2] mean, rstd
  const float* dy;    // bwd: gradient wrt LN output
  const float* res;   // bwd: added to dx (may alias y), may be null
  float* rs;          // null, or the fp16x3 GEMM row scale of every row written (k_rowscale's value, indexed by
                      // the physical output row: fwd r, bwd map[r]); LN_ROWMAP only
  unsigned short* pl; // null, or (with rs) the written rows as fp16x3 planes [row][2C], chunk-interleaved, scaled by rs (the
                      // split of k_rowsplit, bit for bit), same row index as rs; fwd: y may then be null
};

struct LnArgs {
  int rows, C;        // output rows and normalised width
  int ldx, ldy, lddy, ldres;
  int mode;
  const int* map;
  int Hin, Win;       // mode geometry (input grid for MERGE, half grid for EXPAND)
  float eps;
  int ngroups;
  LnGroup g[kMaxGroups];
};

hipError_t layernorm_fwd(const LnArgs& a, hipStream_t s);
hipError_t layernorm_bwd(const LnArgs& a, hipStream_t s);

// ---------------------------------------------------------------------------
// Window attention (swinblock.py:133-172) on qkv in window order.
// ---------------------------------------------------------------------------
struct AttnGroup {
  const float* qkv;   // [nwin*N][3C]
  const float* table; // relative_position_bias_table [(2ws-1)^2][nH]
  float* o;           // fwd out [nwin*N][C]
  float* P;           // saved softmax [nwin][nH][N][N]
  const float* dO;    // bwd in
  float* dqkv;        // bwd out [nwin*N][3C]
};

struct AttnArgs {
  int nwin;           // windows over the whole batch
  int nWh, nWw;       // windows per image per axis
  int ws, shift, H;   // H: image rows (mask labels, quirk Q1)
  int C, heads;
  float scale;
  int ngroups;
  int mfma;           // 1: the exact-f32 MFMA kernels where attn_mf_ok (one head of 192 per workgroup)
  // forward, one head of 192 per workgroup, group 0 only: null, or write the output as the fp16x3 A planes of the
  // tile-48 proj GEMM (opl: [row][2C], k_rowsplit's layout) with row scales ors instead of fp32 o. The scale of a
  // window's rows comes from a bound: |o| <= max |v| over the window (P is a convex combination), and
  // |v_j| <= C max|A_j| max|W_qkv| + max|b_qkv| with max|A_j| < 2^15 / vrs[j] (the qkv GEMM's A row scales, window
  // order) and vbw / vbb device scalars (vbb may be null).
  unsigned short* opl;
  float* ors;
  const float* vrs;
  const float* vbw;
  const float* vbb;
  AttnGroup g[kMaxGroups];
};

hipError_t attn_fwd(const AttnArgs& a, hipStream_t s);
hipError_t attn_bwd(const AttnArgs& a, hipStream_t s);

// ---------------------------------------------------------------------------
// PatchEmbed conv (k = stride = 2) + absolute_pos_embed, and ConvTranspose2d (k = stride = 2)
// ---------------------------------------------------------------------------
struct PatchGroup {
  const float* w;     // conv: [Cout][cin][2][2] ; convT: [Cin][cout][2][2]
  const float* bias;
  const float* pos;   // conv: absolute_pos_embed [Ho*Wo][Cout]
  float* tok;         // tokens [B*Ho*Wo][Ctok]
  const float* dtok;  // bwd
  int cin_off, cin;   // conv: channel slice of the image ; convT: mean/std channel placement
  int mean_off, std_off, cout;
};

struct PatchArgs {
  int B, Himg, Wimg, Cimg;   // image tensor (B, Cimg, Himg, Wimg)
  int Ctok;                  // token width (enc_dim)
  int climit;                // convT: only channels < climit are produced / back-propagated
  const float* img;          // conv fwd input / convT bwd input (dimg)
  float* img_out;            // conv bwd output (dz) / convT fwd output
  const float* add_img;      // conv bwd: added to dz (latent regulariser term z), may be null
  int ngroups;
  PatchGroup g[kMaxGroups];
  const Tuning* tune;        // null: kDefaultTuning (host dispatch only)
};

hipError_t patch_embed_fwd(const PatchArgs& a, hipStream_t s);
hipError_t patch_embed_bwd(const PatchArgs& a, hipStream_t s);   // img_out = add_img + d img
hipError_t patch_unembed_fwd(const PatchArgs& a, hipStream_t s); // ConvTranspose2d
hipError_t patch_unembed_bwd(const PatchArgs& a, hipStream_t s); // dtok <- d out

// ---------------------------------------------------------------------------
// DA misfit (da_4dvar.py:1183-1208) and vector primitives
// ---------------------------------------------------------------------------
struct MisfitArgs {
  int C, Hs, Ws;          // state grid
  int Hl, Wl;             // network grid (nearest maps when different)
  const int* mi;          // [Hs] state row -> net row (nearest)  (null: identity)
  const int* mj;          // [Ws]
  const int* ri0;         // adjoint row ranges [Hl+1] (null: identity)
  const int* rj0;         // [Wl+1]
  const float* net;       // network output (C', Hl, Wl) first C channels used
  int net_cstride;        // channels in net tensor
  const float* scale;     // [C] first multiply (stdTr for the decoder, std for the flow)
  const float* scale2;    // null or [C] second multiply (std for the decoder): (net*scale)*scale2
  const float* offset;    // null or [C] per-channel additive (mean, flow step)
  const float* xb;        // null or (C,Hs,Ws) additive field (background, decoder step)
  const float* yo;
  const float* Hm;
  const float* R;
  float* x_out;           // state x_t (C,Hs,Ws)
  float* flow_in;         // null or (C,Hl,Wl) next-step normalised input (x - mean)/std
  const float* mean;      // for flow_in
  const float* std_;
  double* partial;        // per-block partial sums of H(x-yo)^2/R
  int nblk;
  // misfit_grid_fwd only (interpolated grids with Hs >= Hl, Ws >= Wl): the observation gradient reduced onto the
  // network grid in the forward pass, and the next flow input written at the down-sampled pixels
  const int* rowinv;      // [Hs] state row -> the network row that down-samples from it (integrate), or -1
  const int* colinv;      // [Ws]
  float* g_net_obs;       // null or (C,Hl,Wl): coeff * Up^T(H (x-yo)/R)
  float coeff;
  int mr;                 // rows in flight per pass (Tuning.grid_fused: 1 -> 3, 2 -> 6)
};

hipError_t misfit_fwd(const MisfitArgs& a, hipStream_t s);
// one pass over the state fields per time slot (interpolated grids): x (only when x_out is set), the J partials (one
// per (channel, network row): nblk must be C * Hl), g_net_obs, flow_in at the down-sampled pixels
hipError_t misfit_grid_fwd(const MisfitArgs& a, hipStream_t s);
// network-grid adjoint of misfit_grid_fwd: g_net[c][q] = (g_net_obs[c][q] + sum_{q' in S(q)} gfi[c][q'] / std[c])
// * scale[c], S(q) = the network pixels whose down-sampled source pixel up-samples onto q (ranges cr0 / cc0)
struct MisfitNetBwdArgs {
  int C, Hl, Wl;
  const float* g_net_obs; // (C,Hl,Wl)
  const float* gfi;       // null or (C,Hl,Wl): gradient of the next flow step's input
  const int* cr0;         // [Hl+1]
  const int* cc0;         // [Wl+1]
  const float* std_;
  const float* scale;
  float* g_net;           // (C',Hl,Wl) first C channels written
};
hipError_t misfit_net_bwd(const MisfitNetBwdArgs& a, hipStream_t s);
// y = GELU(x), dy = GELU'(x) by the epilogues' device functions (vv_gelu.h); form 0 one-value, 1 four-value forms
hipError_t gelu_eval(const float* x, float* y, float* dy, int64_t n, int form, hipStream_t s);
// g_state = coeff*H*(x-yo)/R + g_carry ; g_net(net grid) = adjoint(g_state) * scale
struct MisfitBwdArgs {
  int C, Hs, Ws, Hl, Wl;
  const int* ri0; const int* rj0; const int* mi; const int* mj;
  const float* x; const float* yo; const float* Hm; const float* R;
  const float* g_carry;   // null or (C,Hs,Ws) gradient arriving from later times
  const float* g_obs;     // null, or (C,Hs,Ws) observation-term gradient already formed (real-obs operator);
                          // then it replaces coeff*H*(x-yo)/R and yo/Hm/R are not read
  float coeff;
  const float* scale;     // [C]
  float* g_net;           // (C', Hl, Wl) first C channels written, the rest zero-filled
  int net_cstride;
  float* g_state;         // scratch (C,Hs,Ws) (needed when maps are not identity)
};
hipError_t misfit_bwd(const MisfitBwdArgs& a, hipStream_t s);
// real-observation operator (da_4dvar.py:62-94 obs_interpolater, loss x_aug :1196-1206): the state (C,HW),
// C = 4 + 5*nin, maps to Ca = 4 + 5*nout observation channels: channels 0..3 directly, and for each of the five
// pressure-level variables i, x_aug[4 + nout*i + o] = sum_j P[o][j] x[4 + nin*i + j] (F.linear over the level axis)
struct ObsArgs {
  int nin, nout, HW;
  const float* P;       // [nout][nin] (obs_interpolater.interp)
  const float* x;       // (C, HW) state
  const float* yo;      // (Ca, HW)
  const float* Hm;
  const float* R;
  float coeff;
  float* g_obs;         // (C, HW): coeff * Op^T (H (Op x - yo) / R)
  double* partial;      // per-block partial sums of H (Op x - yo)^2 / R
  int nblk;
};
constexpr int kObsMaxIn = 16, kObsMaxOut = 64;
hipError_t obs_misfit(const ObsArgs& a, hipStream_t s);
// x_aug (T, Ca, HW) = Op x (T, C, HW) for T fields (also get_R_matrix_from_gt, da_4dvar.py:729-756, on R)
// latitude-weighted WRMSE / Bias of one_step_DA's logging (utils/metrics.py:282-296 weighted_rmse_torch_channels,
// :65-82 type_weighted_bias_torch 'all'; da_4dvar.py:1256-1262), on normalised fields (x - mean)/std, scaled
// back by std: wrmse[c] = mean_b sqrt(mean_hw w_h d^2) * std[c], bias[c] = mean_b mean_hw (w_h d) * std[c]
struct MetricArgs {
  const float* pred;    // (B, C, H, W) physical
  const float* gt;      // (B, C, H, W)
  const float* mean;    // [C]
  const float* std_;    // [C] normalisation (fp32, as model_std_gpu)
  const double* scale;  // [C] final multiply (the reference's float64 model_std)
  const float* wlat;    // [H] latitude weights (fp32, as the reference computes them)
  int B, C, H, W;
  double* partial;      // [B*C][nchunk][2]
  int nchunk;
  double* wrmse;        // [C]
  double* bias;         // [C]
};
hipError_t metrics(const MetricArgs& a, hipStream_t s);
hipError_t obs_augment(const float* P, int nin, int nout, const float* x, float* x_aug, int T, int HW, hipStream_t s);
// general (nearest-interpolated) grids, F.interpolate mode='nearest' (quirk Q3):
//   flow_in[c][a][b] = (x[c][di[a]][dj[b]] - mean[c]) / std[c]          (integrate: down-sample, da_4dvar.py:668-671)
hipError_t flow_input(const float* x, float* flow_in, const int* di, const int* dj, const float* mean,
                      const float* std_, int C, int Hs, int Ws, int Hl, int Wl, hipStream_t s);
//   carry[c][i][j] = sum over (a,b) with (di[a],dj[b]) == (i,j) of gfi[c][a][b] / std[c]   (adjoint of the above)
hipError_t flow_input_adjoint(const float* gfi, float* carry, const int* di, const int* dj, const float* std_, int C,
                              int Hs, int Ws, int Hl, int Wl, hipStream_t s);
// g_x(prev step) = g_flow_in / std (+ nothing else): flow input normalisation adjoint (identity grids)
hipError_t scale_channels(const float* in, float* out, const float* inv_std, int C, int HW, const float* add,
                          hipStream_t s);

// nearest resampling (BC, Hi, Wi) -> (BC, Ho, Wo); maps: mi[Ho], mj[Wo] (forward) or the preimage ranges
// ri0[Hi + 1], rj0[Wi + 1] (adjoint: in = gout (BC, Ho, Wo), out = gin (BC, Hi, Wi))
hipError_t resample_nearest(const float* in, float* out, const int* maps, int BC, int Hi, int Wi, int Ho, int Wo,
                            bool adjoint, hipStream_t s);
hipError_t reduce_sumsq(const float* x, int64_t n, double* partial, int nblk, hipStream_t s);
hipError_t reduce_final(const double* partial, int n, double* out, hipStream_t s);

// L-BFGS / Adam vector primitives (torch/optim/lbfgs.py, torch/optim/adam.py)
hipError_t vec_dot(const float* a, const float* b, int64_t n, double* partial, int nblk, double* out, hipStream_t s);
hipError_t vec_axpy(float* y, const float* x, float alpha, int64_t n, hipStream_t s);       // y += alpha x
hipError_t vec_axpby(float* out, const float* x, float a, const float* y, float b, int64_t n, hipStream_t s);
hipError_t vec_scale(float* y, float alpha, int64_t n, hipStream_t s);
hipError_t vec_absmax(const float* x, int64_t n, float* partial, int nblk, float* out, hipStream_t s);
hipError_t vec_absmax_d(const float* x, int64_t n, float* partial, int nblk, double* out, hipStream_t s);
hipError_t vec_abssum(const float* x, int64_t n, double* partial, int nblk, double* out, hipStream_t s);
// count reductions over equal-length vectors in two launches, request i: op 0 dot(a, b), 1 abssum(a), 2 absmax(a)
// (the values of vec_dot / vec_abssum / vec_absmax_d with the same nblk); out[i] (device- or host-mapped doubles),
// then the n_extra device doubles of `extra` copied to out[count...]. partial: count * nblk doubles.
struct ReduceReqs {
  static constexpr int kMax = 8;
  const float* a[kMax];
  const float* b[kMax];
  int op[kMax];
};
hipError_t reduce_multi(const ReduceReqs& r, int count, int64_t n, double* partial, int nblk, double* out,
                        const double* extra, int n_extra, hipStream_t s);
// q (= -g on entry) -> L-BFGS direction d (two-loop recursion, device scalars); al: >= m device floats;
// partial: 2 * nblk doubles
hipError_t lbfgs_two_loop(float* q, const float* const* S, const float* const* Y, const float* ro, int m, float H_diag,
                          int64_t n, double* partial, int nblk, float* al, hipStream_t s);
hipError_t adam_step(float* p, const float* g, float* m, float* v, int64_t n, float lr, float b1, float b2,
                     float eps, float bc1, float bc2_sqrt, hipStream_t s);
// ---------------------------------------------------------------------------
// live profiler: HIP events around every launch, bucketed by kernel class
// ---------------------------------------------------------------------------
// PC_GEMM16: the GEMMs that ran the fp16x3 kernel (k_rowscale + k_gemm_h3 [+ fixup]); PC_GEMM: every other GEMM
// PC_TOWER: the fused Swin-tower sub-blocks (vv_tower.hip)
enum ProfClass : int { PC_GEMM = 0, PC_ATTN = 1, PC_LN = 2, PC_PATCH = 3, PC_MISFIT = 4, PC_VEC = 5, PC_GEMM16 = 6,
                       PC_TOWER = 7, PC_N = 8 };
int prof_begin(hipStream_t s);                                        // -1 when disabled
void prof_end(int h, hipStream_t s, int cls, double flops, double bytes);
void prof_enable(bool on);
bool prof_enabled();
// sums since enable: ms, flops, bytes, launches per class (synchronises)
void prof_read(double* ms, double* flops, double* bytes, int* n);
// host-side launch counters of the fused-path alternatives (vv_get_counter): tests assert that a fused path really
// ran, since every fused launcher falls back to the unfused launches with equal results when it does not apply
enum Counter : int { CNT_ROWSPLIT = 0, CNT_FIXUP_LN = 1, CNT_SPLITK_FIXUP = 2, CNT_GATHER_SCALES = 3, CNT_H5_SPLIT = 4, CNT_N = 5 };
void count_launch(int c);
long long launch_count(int c);

hipError_t transpose2d(const float* in, float* out, int rows, int cols, hipStream_t s);

// ---------------------------------------------------------------------------
// Fused Swin-tower MLP sub-block (vv_tower.hip): fwd x2 = x1 + fc2(GELU(fc1(LN2(x1)))), writing the LN2 statistics
// and the fc1 pre-activation; bwd dx1 = dx2 + LN2-backward(fc1^T-path(GELU'(h1) * fc2^T-path(dx2))), in place
// allowed (out == dy). Weights as fp16x3 planes + row scales (fp16_planes_of).
// ---------------------------------------------------------------------------
struct MlpGroup {
  const float* x;                    // x1 [M][C]: LN2 input (and the forward residual)
  const float *gamma, *beta;         // LN2 weight / bias (beta: forward only)
  float* stats;                      // [M][2] mean, rstd: written (fwd) / read (bwd)
  const unsigned short* w1h;         // fwd fc1.weight [4C][C], bwd fc2.weight^T [4C][C]: fp16 planes
  const float* w1s;                  //   their row scales (stride K / 32)
  const float* b1;                   // fc1.bias (fwd)
  const unsigned short* w2h;         // fwd fc2.weight [C][4C], bwd fc1.weight^T [C][4C]
  const float* w2s;
  const float* b2;                   // fc2.bias (fwd)
  float* h1;                         // [M][4C] fc1 pre-activation: written (fwd) / read (bwd)
  const float* dy;                   // bwd: dx2 [M][C]
  float* out;                        // fwd x2, bwd dx1 [M][C]
  float* rs;                         // bwd, optional: fp16x3 row scales of dx1 (k_rowscale's formula)
};
struct MlpArgs {
  int M, C, ngroups;
  int hc;  // C = 192: hidden units per chunk (32 or 64; 0 = 32), or 2 (32, hidden layer split over two waves)
  float eps;
  MlpGroup g[kMaxGroups];
};
bool mlp_supported(int C, int M);
// Fused Swin-tower attention sub-block (vv_tower.hip), forward: LN1 (window gather) + qkv + window attention
// (rel-pos bias, quirk-Q1 mask) + proj + residual (window reverse), writing what the backward reads: LN1 stats and
// qkv in window order, the softmax P. ws = 4 (16-token windows), head dim 32.
struct AblkGroup {
  const float* x;                    // stage input rows [M][C] (physical order); the residual
  const float *n1g, *n1b;            // LN1
  float* stats;                      // [M][2] LN1 mean, rstd (window order)
  const unsigned short* wqh;         // qkv.weight [3C][C] fp16 planes
  const float *wqs, *wqb;            //   row scales (stride C / 32), qkv.bias
  const float* table;                // relative_position_bias_table [49][heads]
  float* qkv;                        // [M][3C] window order (saved for the backward)
  float* P;                          // [nwin][heads][16][16] softmax (saved)
  const unsigned short* wph;         // proj.weight [C][C] fp16 planes
  const float *wps, *wpb;            //   row scales, proj.bias
  float* out;                        // x1 [M][C] physical order
  // backward (ablk_bwd): dy = out = the stage gradient (physical rows, in place); qkv, P, stats, x read
  const unsigned short* wpth;        // proj.weight^T [C][C] planes (dO = dx1 W_proj)
  const float* wpts;
  const unsigned short* wqth;        // qkv.weight^T [C][3C] planes (dY = dqkv W_qkv)
  const float* wqts;
  float* rs;                         // optional: fp16x3 row scales of the result (physical rows)
};
struct AblkArgs {
  int M, C, heads, ngroups;
  int nWh, nWw, ws, shift, H;        // window grid per image, window size, shift (mask labels, quirk Q1)
  float scale, eps;
  const int* map;                    // window-order row -> physical row (the cyclic shift + partition)
  AblkGroup g[kMaxGroups];
};
bool ablk_supported(int C, int heads, int ws, int M);
hipError_t ablk_fwd(const AblkArgs& a, hipStream_t s);
// backward of the same sub-block: gx (G.out, physical rows) <- gx + LN1-backward(dqkv W_qkv) with
// dqkv = WindowAttention-backward(gx gathered W_proj), in place
hipError_t ablk_bwd(const AblkArgs& a, hipStream_t s);
hipError_t mlp_fwd(const MlpArgs& a, hipStream_t s);
hipError_t mlp_bwd(const MlpArgs& a, hipStream_t s);
// fp16 planes and row scales of a registered weight W [N][K] (null when it has none: K or offset not 32-aligned)
void fp16_planes_of(const float* W, int K, const unsigned short** h, const float** sc);

// ---------------------------------------------------------------------------
// sc4dvar B-matrix transform (da_4dvar.py:878-931; vv_sc4dvar.hip) on the fixed 128 x 256 grid
// ---------------------------------------------------------------------------
struct Sc4dvarB;
// tables from the B-matrix statistics (init_b_matrix :520-526, float64 as in dataset/bq_info_lr/*.npy):
// len_scale[C], reg[C][nreg] (nreg 13 or 26), std_sur[4], eigval[5][13], eigvec[5][13][13]; 0 or nonzero + err
int sc4dvar_create(Sc4dvarB** out, int C, const double* len_scale, const double* reg, int nreg,
                   const double* std_sur, const double* eigval, const double* eigvec, double scale_factor, int hpad,
                   std::string& err);
void sc4dvar_destroy(Sc4dvarB* b);
size_t sc4dvar_field_floats(const Sc4dvarB* b);  // C * 128 * 256
// recon = transform core of w (before the interpolation and + xb); t1, t2: field-sized scratch
hipError_t sc4dvar_fwd(const Sc4dvarB* b, const float* w, float* recon, float* t1, float* t2, float* gemm_ws,
                       hipStream_t s);
// g_w = core^T g_recon (+ add)
hipError_t sc4dvar_adj(const Sc4dvarB* b, const float* g_recon, const float* add, float* g_w, float* t1, float* t2,
                       float* gemm_ws, hipStream_t s);
hipError_t fill(float* p, float v, int64_t n, hipStream_t s);

}  // namespace vv

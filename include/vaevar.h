/*
 * vaevar.h — C ABI of libvaevar.so, the MI355X-native (gfx950, HIP) VAE-Var 4D-Var inner loop.
 *
 * The reference (xiaoyi018/VAE-Var) has no FFI: its boundary is the PyTorch module + optimiser
 * protocol. Each entry point below replaces one piece of that protocol:
 *
 *   vv_lgunet_param_count/_info   the state_dict key set of networks_old.transformer.LGUnet_all
 *                                 (networks_old/transformer.py:716-745, swinblock.py:189-262), or with
 *                                 arch = VV_ARCH_LGUNET1 of networks.LGUnet_all.LGUnet_all_1 (LGUnet_all.py:742-776)
 *   vv_model_create/load_weights  LGUnet_all(**cfg) + load_state_dict (da_4dvar.py:590-603, 571-588)
 *   vv_model_forward              LGUnet_all.forward (transformer.py:747-752) = VAE_lr.decoder (vae.py:83-85)
 *   vv_model_backward             autograd of the above w.r.t. its input (input gradient only, quirk Q5)
 *   vv_bind_problem               the closure state of one_step_DA 'vae4dvar' (da_4dvar.py:1179-1251)
 *   vv_closure                    closure() -> loss(z); backward (da_4dvar.py:1183-1208, 1242-1246)
 *   vv_decode                     the analysis xa = decoder_hr(z)*stdTr*std + xb (da_4dvar.py:1301-1306)
 *   vv_set_obs_operator/_augment  the real-observation operator obs_interpolater (da_4dvar.py:62-94, :1196-1206)
 *   vv_metrics                    WRMSE / Bias of the DA logging (utils/metrics.py, da_4dvar.py:1256-1262)
 *   vv_integrate                  integrate(x, model, 1) (da_4dvar.py:666-681): the outer-cycle forecast with
 *                                 the 0.25-degree LGUnet_all_1 (da_4dvar.py:1329, :652), forward only
 *   vv_dot/axpy/... , vv_adam     vector arithmetic of torch/optim/lbfgs.py:333-535 and adam.py
 *
 * Conventions: every function returns 0 on success, a non-zero status otherwise (HIP error code or
 * VV_E_*), never throws; vv_last_error() describes the last failure of the calling thread.
 *   vv_nearest_map                F.interpolate(mode='nearest') index maps (nf_model/vae.py:90, da_4dvar.py:671,679)
 * All float pointers passed to compute entry points are DEVICE pointers (fp32, 16-byte aligned)
 * owned by the caller; `stream` is a hipStream_t (NULL = default stream). A context is bound to
 * one device and is not thread-safe. All work is enqueued on the given stream; only functions
 * that return host scalars (vv_closure, vv_dot, ...) synchronise it.
 */
#ifndef VAEVAR_H
#define VAEVAR_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VV_E_ARG 1001     /* invalid argument / unsupported configuration */
#define VV_E_STATE 1002   /* call out of order (e.g. closure before bind_problem) */
#define VV_E_ALLOC 1003   /* device allocation failed */

typedef struct vv_ctx vv_ctx;

#define VV_ARCH_LGUNET 0   /* networks_old.transformer.LGUnet_all (VAE decoder, flow model): fwd + input bwd */
#define VV_ARCH_LGUNET1 1  /* networks.LGUnet_all.LGUnet_all_1 (forecast model): forward only */

/* LGUnet_all keyword arguments (nf_model/parameters0_old.yaml:49-96; for VV_ARCH_LGUNET1
   output/model/model_0.25degree/training_options.yaml:64-119). Zero-initialise, then fill. */
typedef struct vv_lgunet_config {
  int img_size[2];
  int patch_size[2];   /* must equal stride: (2,2) */
  int stride[2];
  int n_groups;        /* len(inchans_list) == len(outchans_list) */
  int inchans[8];
  int outchans[8];
  int enc_dim;
  int embed_dim;
  int window_size;     /* 4 */
  int n_enc_levels;    /* len(enc_depths) == 2 */
  int enc_depths[4];
  int enc_heads[4];
  int n_lg_layers;
  int lg_depths[8];
  int lg_heads[8];
  /* appended for VV_ARCH_LGUNET1 (ignored by VV_ARCH_LGUNET, whose window is window_size x window_size) */
  int arch;            /* VV_ARCH_* */
  int window_hw[2];    /* [wh, ww] (LGUnet_all_1 window_size); patch_size may then exceed stride (3,2)/(2,2) */
} vv_lgunet_config;

int vv_version(void);
int vv_last_error(char* buf, int cap);

/* parameter enumeration (no device needed) */
int vv_lgunet_param_count(const vv_lgunet_config* cfg, int* count);
int vv_lgunet_param_info(const vv_lgunet_config* cfg, int index, char* name, int name_cap, int64_t* shape,
                         int* ndim);

int vv_ctx_create(int device, vv_ctx** out);
int vv_ctx_destroy(vv_ctx* ctx);

/* a network instance: `batch` images per forward, `n_slots` independent saved-activation sets
   (one per forecast step of the 4D-Var window) */
int vv_model_create(vv_ctx* ctx, const vv_lgunet_config* cfg, int batch, int n_slots, int* model_id);
/* free a network instance (its weights, planes, saved activations and workspace; `del model` in the reference): the
   id becomes invalid; a problem bound to it (vv_bind_problem / vv_sc4dvar_bind) is unbound and the context's closure
   graphs are dropped. Synchronises the device. */
int vv_model_destroy(vv_ctx* ctx, int model_id);
/* ptrs[i] points to parameter i in vv_lgunet_param_info order (host or device memory, fp32) */
int vv_load_weights(vv_ctx* ctx, int model_id, const void* const* ptrs, int n);
/* out: (batch, sum(outchans), H, W); only channels < out_limit are written (0 = all) */
int vv_model_forward(vv_ctx* ctx, int model_id, int slot, const float* in, float* out, int out_limit, void* stream);
/* din = add + (d out / d in)^T dout, reading only dout channels < out_limit; add may be NULL */
int vv_model_backward(vv_ctx* ctx, int model_id, int slot, const float* dout, float* din, const float* add,
                      int out_limit, void* stream);
int vv_model_workspace_bytes(vv_ctx* ctx, int model_id, int64_t* bytes);

/* one_step_DA 'vae4dvar' problem: state (C,Hs,Ws), window of T times; flow_model_id < 0 when T == 1.
   When (Hs,Ws) differs from the network grid (e.g. 721x1440 vs 128x256) the decoder output and each forecast are
   nearest-up-sampled to the state grid and the forecast input nearest-down-sampled, as decoder_hr / integrate do.
   B independent analyses (ensemble members / windows) are bound at once when the decoder model (and the flow model)
   were created with batch B: every evaluation then runs ONE decoder launch sequence over the B latents (GEMMs of
   B x 2048 rows) and one flow sequence per forecast step; each analysis keeps its own J.
   xb (B,C,Hs,Ws); yo, Hmask, R (B,T,C,Hs,Ws); mean, std, std_tr (C). Buffers stay owned by the caller. */
int vv_bind_problem(vv_ctx* ctx, int dec_model_id, int flow_model_id, int T, int C, int Hs, int Ws,
                    const float* xb, const float* yo, const float* Hmask, const float* R, const float* mean,
                    const float* std_, const float* std_tr, float obs_coeff);
/* J = J_b + obs_coeff * J_o at latent z (B,32,128,256); grad_z = dJ/dz (B,32,128,256); J_b, J_o: B doubles each
   (host), one per analysis. Synchronises `stream`. */
int vv_closure(vv_ctx* ctx, const float* z, float* grad_z, double* J_b, double* J_o, void* stream);
/* same, leaving {J_b, J_o} per analysis in device memory d_J[2B]; no synchronisation */
int vv_closure_async(vv_ctx* ctx, const float* z, float* grad_z, double* d_J, void* stream);
/* replay the closure from a hipGraph (default on; the Python Context turns it off for VAEVAR_GRAPH=0): the evaluation's
   ~540 kernel launches are captured once per kind (J only / J + gradient) and replayed as one graph launch, with z
   and grad_z copied through problem-owned buffers; results are bit-identical to the eager launches */
int vv_set_closure_graph(vv_ctx* ctx, int enable);
/* state of the closure graph of one kind (0: J only, 1: J + gradient) since the last bind / vv_set_closure_graph:
   info[0] graphs enabled, info[1] graph instantiated, info[2] capture failed (this kind runs eagerly: a silent
   slowdown otherwise, the results are identical), info[3] graph launches */
int vv_get_closure_graph(vv_ctx* ctx, int kind, long long* info);
/* process-wide host-side launch counters (monotonic; eager launches only, a graph replay does not count):
   "rowsplit" (k_rowsplit passes building a GEMM's fp16x3 A planes), "fixup_ln" (split-K fixups fused into a
   LayerNorm), "splitk_fixup" (stand-alone tile-48 split-K fixups), "gather_scales" (k_gather_scales passes of tile 48),
   "h5_split" (fused fixup + LayerNorm launches consuming tile 49's split-K partials, tuning key "h5_split").
   Tests use them to show a fused path ran. */
int vv_get_counter(const char* name, long long* value);
/* analysis states xa (B,C,Hs,Ws) */
int vv_decode(vv_ctx* ctx, const float* z, float* xa, void* stream);
/* out = integrate(x, model, steps) (da_4dvar.py:666-681): z = (x - mean)/std (nearest to the model grid when
   (Hs,Ws) differs, interpolation=True); `steps` times z = model(z)[:, :C]; nearest back to (Hs,Ws); *std + mean.
   x, out (C,Hs,Ws); mean, std (C). The model (either arch, batch 1) must map C channels to >= C. */
int vv_integrate(vv_ctx* ctx, int model_id, const float* x, float* out, int C, int Hs, int Ws, const float* mean,
                 const float* std_, int steps, void* stream);
/* sc4dvar (da_4dvar.py:1064-1177): the B-matrix control-variable transform of the static 3D/4D-Var mode.
   Replaces init_b_matrix (:520-526), get_static_info (:608-628: RealSHT/InverseRealSHT of torch_harmonics on the
   equiangular 128x256 grid, the zonal Gaussian kernel of the first hpad = 112 rows, sph_scale) and binds the
   loss of :1071-1101. B-matrix tables as the reference loads them from dataset/bq_info_lr (one .npy per table, float64, host):
   len_scale[69] (multiplied by scale_factor, :521), reg_coeff[69][n_reg] (n_reg 13 or 26, :890-893),
   std_sur[4], vert_eig_value[5][13], vert_eig_vec[5][13][13]. Problem buffers (device, caller-owned) as in
   vv_bind_problem: xb (69,Hs,Ws), yo/Hmask/R (T, C_obs, Hs, Ws), mean/std (69) for the flow steps; C = 69 and
   (Hs,Ws) >= (128,256). interp: null for observations of the state (C_obs = 69), else the (n_out, 13)
   obs_interpolater.interp of obs_type 'real*' (C_obs = 4 + 5*n_out, host or device, copied). T > 1 needs a
   networks_old LGUnet_all flow model (69 -> >= 69 channels, 128x256, batch 1): x_t = integrate(x_{t-1}) is
   detached in the reference (:1080), so those terms enter J but not dJ/dw. */
int vv_sc4dvar_bind(vv_ctx* ctx, int flow_model_id, int T, int C, int Hs, int Ws, const float* xb, const float* yo,
                    const float* Hmask, const float* R, const float* mean, const float* std_, float obs_coeff,
                    const float* interp, int n_out, const double* len_scale, const double* reg_coeff, int n_reg,
                    const double* std_sur, const double* vert_eig_value, const double* vert_eig_vec,
                    double scale_factor, int hpad);
/* loss(w) = J_b + obs_coeff * J_o (:1099-1101) at w (69,128,256); grad_w (may be null) = its gradient with the
   reference's detach; J_b, J_o to the host. Synchronises `stream`. */
int vv_sc4dvar_closure(vv_ctx* ctx, const float* w, float* grad_w, double* J_b, double* J_o, void* stream);
/* xhat (69,Hs,Ws) = transform(w, xb) (:878-931) */
int vv_sc4dvar_transform(vv_ctx* ctx, const float* w, float* xhat, void* stream);
/* F.interpolate(x, (Ho, Wo)) with the default mode 'nearest' (quirk Q3; nf_model/vae.py:90 decoder_hr,
   da_4dvar.py:671/679/928) on (BC, Hi, Wi) device fields -> out (BC, Ho, Wo); with adjoint != 0 the transposed
   map: in (BC, Ho, Wo) -> out (BC, Hi, Wi), each source pixel the sum over its nearest preimage (deterministic).
   Synchronises `stream`. */
int vv_resample_nearest(vv_ctx* ctx, const float* in, float* out, int BC, int Hi, int Wi, int Ho, int Wo, int adjoint,
                        void* stream);
/* real-observation operator (da_4dvar.py:62-94 obs_interpolater; the loss's x_aug, :1196-1206): after
   vv_bind_problem, the bound yo, Hmask, R become (T, 4 + 5*n_out, Hs, Ws) observation-space fields. Channels 0..3
   are observed directly; for each of the five 13-level variables i (z, q, u, v, t) x_aug[4 + n_out*i + o] =
   sum_j interp[o][j] x[4 + n_in*i + j]. interp: (n_out, n_in) fp32, host or device, copied. Needs C = 4 + 5*n_in,
   n_in <= 16, n_out <= 64; n_out = 0 restores the identity operator (synthetic observations). */
int vv_set_obs_operator(vv_ctx* ctx, int n_out, int n_in, const float* interp);
/* x_aug (T, 4 + 5*n_out, Hs, Ws) = the operator applied to x (T, 4 + 5*n_in, Hs, Ws); interp on the device.
   Also get_R_matrix_from_gt (da_4dvar.py:729-756) when applied to R. */
int vv_obs_augment(vv_ctx* ctx, const float* interp, int n_out, int n_in, const float* x, float* x_aug, int T,
                   int Hs, int Ws, void* stream);
/* latitude-weighted WRMSE and Bias per channel as one_step_DA logs them (da_4dvar.py:1256-1262 with
   utils/metrics.py Metrics.WRMSE / Metrics.Bias, weighted_rmse_torch_channels :282-289, type_weighted_bias_torch
   'all' :65-82): both fields normalised by (x - mean)/std, then scaled by `scale` (the float64 model_std).
   pred, gt (B,C,H,W); mean, std_ (C) fp32; scale (C) fp64; wrmse, bias (C) fp64 device. Synchronises `stream`. */
int vv_metrics(vv_ctx* ctx, const float* pred, const float* gt, const float* mean, const float* std_,
               const double* scale, int B, int C, int H, int W, double* wrmse, double* bias, void* stream);
/* trajectories x_t (B,T,C,Hs,Ws) of the last closure / forward evaluation (device pointer, read-only). On an
   interpolated state grid with the one-pass misfit ("grid_fused", config 5) a gradient closure does not store x_t (the
   state fields are read once and nothing is written at the state grid); a J-only evaluation (cal_loss, vv_closure with
   grad_z = NULL) does, so the per-outer-pass logging of da_4dvar.py:1256-1262 sees the pass's x_t. */
int vv_state_ptr(vv_ctx* ctx, const float** x);

/* vector primitives (n floats). Host-returning ones synchronise `stream`. */
int vv_dot(vv_ctx* ctx, const float* a, const float* b, int64_t n, double* out, void* stream);
int vv_abssum(vv_ctx* ctx, const float* a, int64_t n, double* out, void* stream);
int vv_absmax(vv_ctx* ctx, const float* a, int64_t n, float* out, void* stream);
/* Several of the reductions above in one host round trip: op i = 0 dot(a[i], b[i]), 1 abssum(a[i]), 2 absmax(a[i])
   over n floats each (count <= 8), with the same kernels and partial layouts as vv_dot / vv_abssum / vv_absmax (the
   same values); then n_extra (<= 16) device doubles at dev_extra (e.g. the J of a vv_closure_async) are appended:
   out[count + n_extra], one synchronisation. The L-BFGS mirror (vaevar/lbfgs.py) asks for the scalars of an
   iteration together instead of one synchronising call each (torch/optim/lbfgs.py computes them one by one). */
int vv_reduce_batch(vv_ctx* ctx, int count, const int* ops, const float* const* a, const float* const* b, int64_t n,
                    const double* dev_extra, int n_extra, double* out, void* stream);
/* The same reductions queued without a host round trip: the results stay in the caller's device doubles dev_out[count]
   (absmax widened exactly), to be fetched later as another call's dev_extra. The partial sums live in the context's
   reduction scratch, which vv_reduce_batch and the next vv_reduce_enqueue reuse: every such call of one context must
   go to the same stream (calls on two streams race on that scratch). */
int vv_reduce_enqueue(vv_ctx* ctx, int count, const int* ops, const float* const* a, const float* const* b, int64_t n,
                      double* dev_out, void* stream);
int vv_axpy(vv_ctx* ctx, float* y, const float* x, float alpha, int64_t n, void* stream);
int vv_axpby(vv_ctx* ctx, float* out, const float* x, float a, const float* y, float b, int64_t n, void* stream);
int vv_scale(vv_ctx* ctx, float* y, float alpha, int64_t n, void* stream);
int vv_copy(vv_ctx* ctx, float* dst, const float* src, int64_t n, void* stream);
/* L-BFGS two-loop recursion (torch/optim/lbfgs.py:404-442): q holds -g on entry and the direction d on return;
   S, Y: host arrays of m device vectors (old_stps, old_dirs, oldest first), ro[m] = 1/(y.s) (host, fp32),
   m <= 256. The dot products and coefficients stay on the device (fp32 as torch's 0-d tensors); no sync. */
int vv_lbfgs_two_loop(vv_ctx* ctx, float* q, const float* const* S, const float* const* Y, const float* ro, int m,
                      float H_diag, int64_t n, void* stream);
/* torch.optim.Adam step (no weight decay / amsgrad): step is the 1-based step count */
int vv_adam(vv_ctx* ctx, float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1,
            float beta2, float eps, int step, void* stream);

/* live profiler: HIP events around every kernel launch, summed per kernel class
   (0 GEMM (bf16x6 / f32), 1 window attention, 2 LayerNorm, 3 patch conv/convT, 4 misfit, 5 vector, 6 fp16x3 GEMM,
   7 fused Swin-tower sub-blocks); ncls >= 8.
   ms = summed launch durations, flops/bytes = algorithmic work, launches = count. stop synchronises. */
int vv_profile_start(vv_ctx* ctx);
int vv_profile_stop(vv_ctx* ctx, double* ms, double* flops, double* bytes, int* launches, int ncls);

/* F.interpolate(mode='nearest') source index map for in_size -> out_size (quirk Q3), as used by
   decoder_hr (nf_model/vae.py:90) and integrate (da_4dvar.py:671, 679); map has out_size entries (host) */
int vv_nearest_map(int in_size, int out_size, int* map);

/* GEMM arithmetic for every nn.Linear of the context's models (per context; default VV_GEMM_SPLIT16; the Python
   Context applies VAEVAR_GEMM_MATH=f32|split|split16 through this call, the library reads no environment):
   VV_GEMM_F32     = v_mfma_f32_32x32x2_f32, an exact fp32 fma chain (torch fp32 matmul semantics);
   VV_GEMM_SPLIT   = each fp32 operand split exactly into three bf16 planes (x = h + m + l) and the six
                     products of order >= 2^-16 accumulated in fp32 by v_mfma_f32_32x32x16_bf16;
   VV_GEMM_SPLIT16 = each fp32 operand scaled by a power of two per row (its maximum to [2^14, 2^15)) and
                     split into two fp16 planes (x = h + l, 22 bits), three products (hh, hl, lh) accumulated
                     in fp32 by v_mfma_f32_32x32x16_f16.
   Both split modes have fp32-level error (measured vs fp64, tests/test_gpu_kernels.py). */
#define VV_GEMM_F32 0
#define VV_GEMM_SPLIT 1
#define VV_GEMM_SPLIT16 2
int vv_set_gemm_math(vv_ctx* ctx, int math);
int vv_get_gemm_math(vv_ctx* ctx, int* math);

/* Per-context dispatch knobs, for A/B runs without a rebuild (defaults = the measured choices).
   Keys: "h3_mink" (smallest K on the fp16x3 kernels, 768), "h3_big" (256x128 fp16x3 tiles, 1), "h3_mf16" (their
   16x16x32-MFMA form, 1), "small_split" (whole-grid split-K of sub-chip fp16x3 GEMMs, 1), "small_split_minkt"
   (24), "tail_minkt" (k-tiles per split-K tail chunk, 12), "ln_scales" (row scales from the LayerNorm, 1),
   "win_attn" (LGUnet_all_1 LDS window attention, 1), "win_mfma" (that kernel on the exact-f32 MFMA, 1),
   "fc_h3_mink" (smallest K of the forecast network's fp16x3 GEMMs, 192), "fuse_mlp" (the fused Swin-tower
   LN2 + fc1 + GELU + fc2 + residual sub-block and its backward: bit 0 at dim 96, bit 1 at dim 192, 3), "fuse_attn" (the fused Swin-tower
   LN1 + qkv + window attention + proj + residual sub-block at dim 96: bits 0 / 1 forward / backward, 3), "attn_mfma" (the window attention of
   the LG stage, head dim 192, and of the unfused tower stages, head dim 32, on the exact-f32 MFMA, 1), "gelu_planes" (the LG-stage GELU / gelu' GEMM
   epilogues write the fp16x3 planes of the K = 4C GEMM after them, 1), "attn_planes" (the LG-stage attention
   forward writes the planes of a tile-48 proj GEMM, 1), "fixup_ln" (that GEMM's split-K fixup fused into the LN2
   after it, 1), "h4" (the split-operand LDS-DMA fp16x3 kernel, tile 48, where
   the 256x128 tiles run, 1), "ln_planes" (the LayerNorm writes that kernel's fp16 A planes, 1), "gattn" (the
   LGUnet_all_1 global window on the flash MFMA kernel, vv_attention_global, 1), "gattn_qf" (its 16-query blocks per
   wave: 1 = eight waves, two per SIMD; 2 = four waves of 32 queries, 1), "h4_small" (tile 48 with whole-chip split-K
   also for 64..143 256-row tiles, 1), "h4_split_minkt" (k-tiles per chunk of that split, 12), "h5" (tile 49, 256x144, where its
   tiles fill whole rounds of the chip and tile 48's leave a split-K tail: the N = 4608 GEMMs at 2048 rows, 1), "fc_conv_mf" (LGUnet_all_1's PatchEmbed / ConvTranspose2d as direct
   exact-f32 MFMA kernels instead of im2col / col2im + GEMM, 1), "mlp_hc" (the fused dim-192 MLP: 32 or 64 hidden units
   per chunk step, or 2 = 32-unit chunks with the hidden layer split over two waves per 16 tokens, 2), "h4_gather"
   (tiles 48 and 49 read a gathered A's producer row scales through the row map themselves instead of a
   k_gather_scales launch, 1), "fixup_ln_rows" (the fused fixup + LN1 after fc2 walks the GEMM's rows in order through the
   inverse window map, 1), "h5_split" (the N = 1152 split-K GEMMs -- those whose fixup is fused into a LayerNorm and the
   plain ones, summed by k_gemm_fixup49 -- on tile 49 with every tile split P / T ways, 256 workgroups at 2048 rows,
   instead of tile 48's 216, 1), "fixup_stage" (the fused fixup + LayerNorm reads a workgroup's split-K partials as whole 128-B lines into LDS, 1, or per row, 0), "grid_fused" (interpolated state grids, Hs >= Hl and Ws >= Wl with synthetic observations:
   the misfit reads each state field once per evaluation and its adjoint runs on the network grid, k_misfit_grid /
   k_misfit_net_bwd, 3 rows of a band in flight per pass; 2 = the same with 6 rows; read by vv_bind_problem, 1), "host_wait" (how
   vv_reduce_batch waits for the stream: 0 hipStreamSynchronize, which keeps a host CPU busy; 1 sleeps, then polls
   hipStreamQuery), "patch_pers" (the decoder PatchEmbed / ConvTranspose2d kernels in their persistent form, one
   workgroup of 8 waves per CU share with the weights staged once, bit-identical to 0 = one workgroup per 64-token
   tile, 1), "bs_tile" (the bf16x6 tile of the short-K tower GEMMs: 27 = 64x64 with one LDS buffer, 27; 24 = two buffers, 25 =
   128x64, 26 = two k-tiles ahead: 24..27, bit-identical), "fixup_ln_cross" (the fused fixup + LN1 also between
   consecutive LG stages, 1). Results stay fp32-level for every value; a change drops the
   context's captured closure graphs. Unknown key, or a value the dispatch does not accept (switches 0 / 1; "mlp_hc"
   0, 2, 32, 64; "gattn_qf" 1, 2; "grid_fused" 0..2; "fuse_mlp" and "fuse_attn" 0..3; the k-tile floors >= 1; the
   minimum K >= 0): VV_E_ARG, and the knob keeps its value. */
int vv_set_tuning(vv_ctx* ctx, const char* key, int value);
int vv_get_tuning(vv_ctx* ctx, const char* key, int* value);
/* process-wide debug aid: synchronise after every library launch and report the first failing op (default 0) */
int vv_set_debug_sync(int enable);

/* give a device weight B[N][K] (used as the B operand of vv_gemm) precomputed split planes, as the
   engine does for every model weight at vv_load_weights; B must stay alive and unchanged until
   vv_ctx_destroy (which frees the planes) */
int vv_gemm_register_weight(vv_ctx* ctx, const float* B, int N, int K);

/* global-window attention as LGUnet_all_1's LG layer 0 runs it (networks/LGUnet_all.py:689, 696; SD_attn without
   mask, networks/utils/Attention.py:599-664): out[t][h d_h + d] = sum_j softmax_j(q_t . k_j) v_j[d] per head h, for
   qkv [N][3C] (q already scaled by head_dim^-0.5 and rotated, k rotated, as the kernel after the qkv projection
   sees them) and out [N][C]; the flash MFMA kernel of vv_gattn.hip (fp16x3 products, fp32 softmax). head_dim 64,
   96, 128 or 192, otherwise VV_E_ARG. Kernel tests and tools; the forecast model calls the kernel itself. */
int vv_attention_global(vv_ctx* ctx, const float* qkv, float* out, int N, int C, int heads, void* stream);

/* raw GEMM entry for kernel tests: C[M][N] = A[M][K] . B[N][K]^T (+bias), K a multiple of 32. tile = -1 picks the
   kernel as the engine does; otherwise one of the library kernels: 0 / 2 / 4 exact-f32 MFMA 128x128 / 64x64 /
   32x64, 24 / 34 bf16x6 split 64x64 / pipelined 128x128, 36 / 44 fp16x3 split 128x128 / 256x128 (32x32x16 MFMAs),
   46 / 47 the same on 16x16x32 MFMAs, 48 fp16x3 256x128 on pre-split A planes staged by LDS-DMA (the engine's
   default for the LG GEMMs), 49 the same operands on 256x144 tiles (data-parallel only). Any other tile: VV_E_ARG. An fp16x3 tile whose B has no fp16 planes (not registered)
   runs tile 34. */
int vv_gemm(vv_ctx* ctx, int M, int N, int K, const float* A, const float* B, const float* bias, float* C,
            int tile, void* stream);
/* vv_gemm with the Mlp epilogues of the engine (kernel tests): epi 0 store; 1 GELU: C = gelu(acc + bias) and, when aux
   is not null, aux = acc + bias (the fc1 forward, swinblock.py:23-29); 3 GELU': C = acc * gelu'(aux) (the fc1 input
   gradient). Other epi values: VV_E_ARG. */
int vv_gemm_epi(vv_ctx* ctx, int M, int N, int K, const float* A, const float* B, const float* bias, float* C,
                float* aux, int epi, int tile, void* stream);
/* y = GELU(x), dy = GELU'(x) (nn.GELU(), exact erf form) by the device functions of every GEMM / fused-MLP epilogue
   (vv_gelu.h): form 0 the one-value forms, 1 the four-value interleaved forms (kernel tests). */
int vv_gelu_eval(vv_ctx* ctx, const float* x, float* y, float* dy, int64_t n, int form, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* VAEVAR_H */

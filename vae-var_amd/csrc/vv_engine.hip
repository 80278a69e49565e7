// libvaevar engine: the Swin-U-Net (networks_old.transformer.LGUnet_all) forward and input-gradient
// backward as a fixed schedule of HIP kernels over a library-owned weight/activation arena, and the
// vae4dvar closure (da_4dvar.py:1183-1246) on top of it. C-ABI: include/vaevar.h.
//
// Data layout (HBM): tokens NHWC [B][H][W][C] fp32; encoder/decoder towers (Enc_net.enc_list,
// Dec_net.dec_list, transformer.py:538-594) are stored group-major [G][B*H*W][C] and every kernel
// runs all G towers in one launch (blockIdx.z / .y = tower). Linear weights are kept as given
// ([N][K], forward operand) plus a transposed copy ([K][N], backward operand).
#include <hip/hip_runtime.h>

#include <sys/prctl.h>
#include <time.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/vaevar.h"
#include "vv_fcst.h"
#include "vv_kernels.h"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define VV_HIP(expr)                                                                           \
  do {                                                                                         \
    hipError_t e_ = (expr);                                                                    \
    if (e_ != hipSuccess) return fail((int)e_, "%s:%d %s -> %s", __FILE__, __LINE__, #expr,     \
                                      hipGetErrorString(e_));                                  \
  } while (0)

using namespace vv;

// ----------------------------------------------------------------------------
// configuration
// ----------------------------------------------------------------------------
struct Cfg {
  vv_lgunet_config raw;
  int G, C0, C1, E, ws;
  int Himg, Wimg, H0, W0, H1, W1;
  int d0, d1, h0, h1;
  int Cin, Cout;
  std::vector<int> lg_depth, lg_heads;
};

int parse_cfg(const vv_lgunet_config* c, Cfg& o) {
  if (!c) return fail(VV_E_ARG, "null config");
  o.raw = *c;
  if (c->n_groups < 1 || c->n_groups > kMaxGroups) return fail(VV_E_ARG, "n_groups %d out of range", c->n_groups);
  if (c->patch_size[0] != 2 || c->patch_size[1] != 2 || c->stride[0] != 2 || c->stride[1] != 2)
    return fail(VV_E_ARG, "only patch_size = stride = (2,2) is supported");
  if (c->n_enc_levels != 2) return fail(VV_E_ARG, "only 2 encoder levels (enc_depths of length 2) supported");
  if (c->window_size != 4) return fail(VV_E_ARG, "only window_size 4 supported");
  if (c->n_lg_layers < 0 || c->n_lg_layers > 8) return fail(VV_E_ARG, "n_lg_layers out of range");
  o.G = c->n_groups;
  o.C0 = c->enc_dim;
  o.C1 = 2 * c->enc_dim;
  o.E = c->embed_dim;
  o.ws = c->window_size;
  o.Himg = c->img_size[0];
  o.Wimg = c->img_size[1];
  o.H0 = o.Himg / 2;
  o.W0 = o.Wimg / 2;
  o.H1 = o.H0 / 2;
  o.W1 = o.W0 / 2;
  if (o.H1 % o.ws || o.W1 % o.ws || o.Himg % 4 || o.Wimg % 4) return fail(VV_E_ARG, "image size not window-aligned");
  o.d0 = c->enc_depths[0];
  o.d1 = c->enc_depths[1];
  o.h0 = c->enc_heads[0];
  o.h1 = c->enc_heads[1];
  if (o.C0 % o.h0 || o.C1 % o.h1) return fail(VV_E_ARG, "dims not divisible by heads");
  if (o.C0 % 32 || o.E % 32) return fail(VV_E_ARG, "enc_dim and embed_dim must be multiples of 32");
  o.Cin = o.Cout = 0;
  for (int g = 0; g < o.G; ++g) {
    o.Cin += c->inchans[g];
    o.Cout += c->outchans[g];
  }
  // the PatchEmbed / ConvTranspose2d MFMA kernels (vv_ops.hip k_p2t_mf / k_t2p_mf, patch_check) take 16 tokens of
  // one image row per wave, at most kPatchCmax token channels and kPatchKmax = 4 x 28 taps per token: refused here
  // with a message instead of a failing first closure
  if (o.W0 % 16) return fail(VV_E_ARG, "img_size[1] / 2 = %d must be a multiple of 16 (patch kernels)", o.W0);
  if (o.C0 > 128 || o.C0 % 16)
    return fail(VV_E_ARG, "enc_dim %d must be a multiple of 16 and <= 128 (patch kernels)", o.C0);
  for (int g = 0; g < o.G; ++g)
    if (c->inchans[g] < 1 || c->inchans[g] > 28 || c->outchans[g] < 1 || c->outchans[g] > 28)
      return fail(VV_E_ARG, "group %d: inchans %d / outchans %d outside 1..28 (patch kernels)", g, c->inchans[g],
                  c->outchans[g]);
  o.lg_depth.assign(c->lg_depths, c->lg_depths + c->n_lg_layers);
  o.lg_heads.assign(c->lg_heads, c->lg_heads + c->n_lg_layers);
  for (int l = 0; l < c->n_lg_layers; ++l)
    if (o.E % o.lg_heads[l]) return fail(VV_E_ARG, "embed_dim not divisible by lg heads");
  return 0;
}

// ----------------------------------------------------------------------------
// parameter enumeration: the exact state_dict keys of LGUnet_all (buffers excluded)
// ----------------------------------------------------------------------------
struct PInfo {
  std::string name;
  std::vector<int64_t> shape;
};

void add_block(std::vector<PInfo>& v, const std::string& pre, int C, int nh, int ws) {
  const int64_t T = (int64_t)(2 * ws - 1) * (2 * ws - 1);
  v.push_back({pre + ".norm1.weight", {C}});
  v.push_back({pre + ".norm1.bias", {C}});
  v.push_back({pre + ".attn.relative_position_bias_table", {T, nh}});
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

std::vector<PInfo> enumerate_params(const Cfg& c) {
  std::vector<PInfo> v;
  const int C0 = c.C0, C1 = c.C1, E = c.E, ws = c.ws;
  for (int g = 0; g < c.G; ++g) {
    const std::string e = "enc.enc_list." + std::to_string(g);
    v.push_back({e + ".absolute_pos_embed", {1, (int64_t)c.H0 * c.W0, C0}});
    v.push_back({e + ".patch_embed.proj.weight", {C0, c.raw.inchans[g], 2, 2}});
    v.push_back({e + ".patch_embed.proj.bias", {C0}});
    for (int b = 0; b < c.d0; ++b) add_block(v, e + ".layers.0.blocks." + std::to_string(b), C0, c.h0, ws);
    v.push_back({e + ".layers.1.downsample.reduction.weight", {C1, 4 * C0}});
    v.push_back({e + ".layers.1.downsample.norm.weight", {4 * C0}});
    v.push_back({e + ".layers.1.downsample.norm.bias", {4 * C0}});
    for (int b = 0; b < c.d1; ++b) add_block(v, e + ".layers.1.blocks." + std::to_string(b), C1, c.h1, ws);
    v.push_back({e + ".norm.weight", {C1}});
    v.push_back({e + ".norm.bias", {C1}});
  }
  v.push_back({"enc.proj.weight", {E, (int64_t)C1 * c.G}});
  v.push_back({"enc.proj.bias", {E}});
  v.push_back({"net.pos_embed", {1, (int64_t)c.H1 * c.W1, E}});
  for (size_t l = 0; l < c.lg_depth.size(); ++l)
    for (int b = 0; b < c.lg_depth[l]; ++b)
      add_block(v, "net.layers." + std::to_string(l) + ".blocks." + std::to_string(b), E, c.lg_heads[l], ws);
  for (int g = 0; g < c.G; ++g) {
    const std::string d = "dec.dec_list." + std::to_string(g);
    for (int b = 0; b < c.d1; ++b) add_block(v, d + ".layers_up.0.blocks." + std::to_string(b), C1, c.h1, ws);
    v.push_back({d + ".layers_up.0.upsample.expand.weight", {2 * C1, C1}});
    v.push_back({d + ".layers_up.0.upsample.norm.weight", {C1 / 2}});
    v.push_back({d + ".layers_up.0.upsample.norm.bias", {C1 / 2}});
    for (int b = 0; b < c.d0; ++b) add_block(v, d + ".layers_up.1.blocks." + std::to_string(b), C0, c.h0, ws);
    v.push_back({d + ".concat_back_dim.0.weight", {C1, 2 * C1}});
    v.push_back({d + ".concat_back_dim.0.bias", {C1}});
    v.push_back({d + ".concat_back_dim.1.weight", {C0, 2 * C0}});
    v.push_back({d + ".concat_back_dim.1.bias", {C0}});
    v.push_back({d + ".norm_up.weight", {C0}});
    v.push_back({d + ".norm_up.bias", {C0}});
  }
  for (int g = 0; g < c.G; ++g) {
    const std::string f = "dec.final_proj_list." + std::to_string(g);
    v.push_back({f + ".weight", {C0, c.raw.outchans[g], 2, 2}});
    v.push_back({f + ".bias", {c.raw.outchans[g]}});
  }
  v.push_back({"dec.proj.weight", {(int64_t)C1 * c.G, E}});
  v.push_back({"dec.proj.bias", {(int64_t)C1 * c.G}});
  return v;
}

int64_t numel(const std::vector<int64_t>& s) {
  int64_t n = 1;
  for (auto x : s) n *= x;
  return n;
}

// ----------------------------------------------------------------------------
// device arena
// ----------------------------------------------------------------------------
struct Arena {
  char* base = nullptr;
  size_t cap = 0, used = 0;
  ~Arena() {
    if (base) (void)hipFree(base);
  }
  static size_t up(size_t x) { return (x + 255) & ~size_t(255); }
};

struct Planner {  // two-pass: first count bytes, then hand out pointers
  size_t bytes = 0;
  char* base = nullptr;
  float* f(size_t n) {
    char* p = base ? base + bytes : nullptr;
    bytes += Arena::up(n * sizeof(float));
    return reinterpret_cast<float*>(p);
  }
};

// ----------------------------------------------------------------------------
// model
// ----------------------------------------------------------------------------
struct BlockW {
  const float *n1g, *n1b, *table, *qkvW, *qkvWT, *qkvb, *projW, *projWT, *projb, *n2g, *n2b, *fc1W, *fc1WT, *fc1b,
      *fc2W, *fc2WT, *fc2b;
  const float *fc1Wmax, *fc1bmax, *fc2Wmax, *qkvWmax, *qkvbmax;  // device scalars max |w| (the plane-writing GEMM epilogues' bounds)
};

struct Stage {
  int G, H, W, C, heads, depth, M, nWh, nWw;
  std::vector<std::array<BlockW, kMaxGroups>> w;  // [depth][G]
  const int* idx[2];                              // window maps, shift 0 / ws/2
  const int* idxinv[2];                           // their inverses (fused fixup + LN1 walks GEMM rows in order)
};

struct StageSave {
  std::vector<float*> x, st1, qkv, P, x1, st2, h1;  // x has depth+1 entries
};

struct Scratch {
  float *t1, *t2, *h, *dqkv;
  float* rs;  // fp16x3 row scales of a LayerNorm output / input gradient, consumed by the GEMM that follows
  float* rs2;  // row scales of the planes a GELU / gelu' epilogue writes (into h) for the K = 4C GEMM after it
  float* ws;  // GEMM tail-split partials (vv::gemm_ws_floats())
  int math = vv::GEMM_SPLIT16;  // GEMM arithmetic (the context's vv_set_gemm_math)
  const vv::Tuning* tune = nullptr;  // the context's dispatch knobs (vv_set_tuning)
  unsigned short* apl = nullptr;     // fp16x3 A planes of the tile-48 GEMMs (k_rowsplit or the LayerNorm writes them)
  size_t apl_halfs = 0;
};

struct Save {
  StageSave enc0, enc1, dec1, dec0;
  std::vector<StageSave> lg;
  float *st_m, *st_en, *ex, *st_ex, *st_nu;
};

struct Model {
  Cfg cfg;
  int B = 1, nslots = 1;
  std::vector<PInfo> params;
  std::vector<float*> pptr;  // device pointer per param
  std::unordered_map<std::string, const float*> W;   // name -> weights ; name + "^T" -> transposed
  std::unordered_map<std::string, const float*> Wmax;  // name -> device scalar max |param| (filled at load)
  std::unique_ptr<Arena> warena, aarena;
  std::unique_ptr<Arena> parena;  // bf16 split planes of warena (3 x 2 B per float), GEMM_SPLIT B operands
  std::unique_ptr<Arena> marena;  // one float per param: max |param| (Wmax)
  Stage enc0, enc1, dec1, dec0;
  std::vector<Stage> lg;
  std::vector<Save> saves;
  Scratch sc;
  // model-level scratch / gradient buffers
  float *xm, *cat, *dp, *xe, *yn, *gy, *gd0, *gxe, *gsk0, *gex, *gd1, *gdp, *gsk1, *glg, *gcat, *gxm, *gtok;
  std::vector<int*> maps_owned;
  bool loaded = false;
  int64_t workspace = 0;
  vvf::FModel* fm = nullptr;  // VV_ARCH_LGUNET1: the forward-only forecast engine (vv_fcst.hip)
  ~Model() { vvf::destroy(fm); }
};

struct Problem {
  bool bound = false;
  int dec = -1, flow = -1, B = 1, T = 1, C = 0, Hs = 0, Ws = 0, Hl = 0, Wl = 0;  // B analyses (the decoder's batch)
  bool interp = false;                 // state grid != network grid: nearest maps (quirk Q3)
  int *mi = nullptr, *mj = nullptr;    // state -> net (decoder_hr / integrate up-sampling)
  int *ri0 = nullptr, *rj0 = nullptr;  // net -> first state row/col mapping onto it (adjoint ranges)
  int *di = nullptr, *dj = nullptr;    // net -> state (integrate down-sampling)
  // grid_fused (interpolated grids with Hs >= Hl, Ws >= Wl, synthetic observations): the misfit reads each state
  // field once per evaluation (k_misfit_grid) and its adjoint runs on the network grid (k_misfit_net_bwd)
  bool grid_fused = false;
  int grid_mr = 3;                           // k_misfit_grid rows in flight per pass
  int *rowinv = nullptr, *colinv = nullptr;  // [Hs] / [Ws]: inverse of di / dj, -1 off the sampled rows / columns
  int *cr0 = nullptr, *cc0 = nullptr;        // [Hl+1] / [Wl+1]: ranges of mi[di[.]] / mj[dj[.]]
  float* GON = nullptr;                      // (B,T,C,Hl,Wl): coeff * Up^T(H (x_t - yo_t) / R_t)
  const float *xb, *yo, *Hm, *R, *mean, *std_, *std_tr;
  float obs_coeff = 1.f;
  std::unique_ptr<Arena> arena;
  float *X, *dec_out, *gdec, *prod, *FI, *FO, *GFO, *GFI, *carry;
  float *Z = nullptr, *GZ = nullptr;  // the closure graph's latent input / gradient output
  size_t zn = 0;                      // floats of the latent
  double *partial, *dJ;
  int nblk = 1024;
  // real-observation operator (vv_set_obs_operator): nout = 0 is the identity (synthetic observations)
  int nin = 0, nout = 0;
  std::unique_ptr<Arena> obs_arena;
  float *Pobs = nullptr, *GOBS = nullptr;  // [nout][nin] ; (B,T,C,Hs,Ws) observation-term gradient
  size_t obs_hw() const { return (size_t)(nout ? 4 + 5 * nout : C) * Hs * Ws; }  // floats per time of yo/Hm/R
};

// sc4dvar (da_4dvar.py:1064-1177): control variable w (C, 128, 256), x_0 = transform(w, xb) on the state grid,
// x_t = integrate(x_{t-1}) with the flow model detached (:1080: integrate(..., interpolation=True, detach=True)),
// so the forecasts add to J_o but not to dJ/dw
struct Sc4Problem {
  bool bound = false;
  int flow = -1, T = 1, C = 0, Hs = 0, Ws = 0, Hl = 128, Wl = 256;
  bool interp = false;
  const float *xb = nullptr, *yo = nullptr, *Hm = nullptr, *R = nullptr, *mean = nullptr, *std_ = nullptr;
  float obs_coeff = 1.f;
  int nin = 0, nout = 0;
  vv::Sc4dvarB* bm = nullptr;
  std::unique_ptr<Arena> arena;
  float *t1, *t2, *recon, *grec, *X, *FI, *FO, *ones, *Pobs, *GOBS;
  int *mi, *mj, *ri0, *rj0, *di, *dj;
  double *partial, *dJ;
  int nblk = 1024;
  size_t wn = 0;  // floats of w
  ~Sc4Problem() { vv::sc4dvar_destroy(bm); }
  size_t obs_hw() const { return (size_t)(nout ? 4 + 5 * nout : C) * Hs * Ws; }
};

}  // namespace

struct vv_ctx {
  int device = 0;
  int math = vv::GEMM_SPLIT16;  // GEMM arithmetic of every model of this context (vv_set_gemm_math)
  vv::Tuning tune;              // dispatch knobs of every model of this context (vv_set_tuning)
  unsigned short* apl = nullptr;  // vv_gemm's A-plane workspace (tile 48), grown on demand
  size_t apl_halfs = 0;
  void* gattn_ws = nullptr;       // vv_attention_global's workspace, grown on demand
  size_t gattn_bytes = 0;
  std::vector<std::unique_ptr<Model>> models;
  Problem prob;
  std::unique_ptr<Sc4Problem> sc4;  // vv_sc4dvar_bind
  double* red = nullptr;   // reduction scratch
  float* gemm_ws = nullptr;
  float* redf = nullptr;
  double* dout = nullptr;  // device scalar
  float* doutf = nullptr;
  double* redb = nullptr;   // vv_reduce_batch: kMaxBatch reduction scratch areas
  double* hredb = nullptr;      // vv_reduce_batch's results: coherent host-mapped doubles (kMaxBatch + kMaxExtra)
  double* hredb_dev = nullptr;  // ... the device view the final kernel writes through
  float* twoloop = nullptr;  // L-BFGS two-loop scalars: al[kMaxHistory]
  char* metric_ws = nullptr;  // vv_metrics partial sums + latitude weights
  size_t metric_cap = 0;
  struct SplitW {
    const float* base;
    size_t n;
    unsigned short* planes;
  };
  std::vector<SplitW> split_owned;  // vv_gemm_register_weight planes
  // hipGraph of the closure: the ~540 launches of one evaluation replayed as one graph launch. One graph per kind
  // (J only / J + gradient), captured at the second evaluation of that kind, against the problem-owned latent and
  // gradient buffers (Problem::Z / GZ), so it does not depend on the caller's pointers. VAEVAR_GRAPH=0 disables.
  struct ClosureGraph {
    hipGraphExec_t exec = nullptr;
    int eager_runs = 0;
    bool eager_only = false;  // capture or instantiation failed once: this kind runs eagerly until rebind
    long long launches = 0;   // graph launches since the last rebind / vv_set_closure_graph (vv_get_closure_graph)
  } graphs[2];
  hipStream_t cap_stream = nullptr;
  bool use_graphs = true;  // vv_set_closure_graph / VAEVAR_GRAPH
  double long_wait_us[2] = {0.0, 0.0};  // host_wait: the last two waits of kind 1 longer than 1 ms (host_sync)
};

namespace {
// The host's wait for the stream (the L-BFGS mirror's scalar round trips, vv_reduce_batch). Tuning.host_wait 0:
// hipStreamSynchronize, whose wait keeps a host CPU busy (ROCm's Yield schedule, the default, is a sched_yield loop;
// BlockingSync is a synonym for it: hip_runtime_api.h hipSetDeviceFlags). 1: poll hipStreamQuery at 20-us sleeps;
// for a wait of kind `cls` 1 (the caller expects a queued closure ahead: vv_reduce_batch with device extras, which
// carry its J), first sleep through 0.8 x the shorter of that kind's last two waits if both exceeded 1 ms. A wait
// that the sleep overshot clears that history. Returns what hipStreamSynchronize would: hipSuccess once the
// stream's work is done, or its error.
hipError_t host_sync(vv_ctx* ctx, hipStream_t st, int cls = 0) {
  if (!ctx->tune.host_wait) return hipStreamSynchronize(st);
  static thread_local bool slack = false;
  if (!slack) {
    prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);  // 1-us timer slack for this thread's short sleeps (default 50 us)
    slack = true;
  }
  auto nap = [](double us) {
    timespec ts{(time_t)(us * 1e-6), (long)(std::fmod(us, 1e6) * 1e3)};
    nanosleep(&ts, nullptr);
  };
  const auto t0 = std::chrono::steady_clock::now();
  auto elapsed_us = [&] {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  };
  hipError_t e = hipStreamQuery(st);
  if (e != hipErrorNotReady) return e;
  double* hist = ctx->long_wait_us;
  const double lw = std::min(hist[0], hist[1]);
  const bool slept = cls == 1 && lw > 1000.0;
  if (slept) nap(0.8 * lw);
  bool first = true, over = false;
  while ((e = hipStreamQuery(st)) == hipErrorNotReady) {
    first = false;
    nap(20.0);
  }
  over = slept && first;  // done by the end of the long sleep: it may have overshot
  if (cls == 1) {
    const double us = elapsed_us();
    if (over) {
      hist[0] = hist[1] = 0.0;
    } else if (us > 1000.0) {
      hist[0] = hist[1];
      hist[1] = us;
    }
  }
  return e;
}
}  // namespace

namespace {

constexpr int kRedBlocks = 1024;
constexpr int kMaxBatch = 8, kMaxExtra = 16;  // vv_reduce_batch
static_assert(kMaxBatch <= vv::ReduceReqs::kMax, "vv_reduce_batch requests exceed the multi-reduction kernel");
constexpr int kMaxHistory = 256;  // L-BFGS history pairs accepted by vv_lbfgs_two_loop

int set_dev(vv_ctx* ctx) {
  VV_HIP(hipSetDevice(ctx->device));
  return 0;
}

// torch nearest_idx (aten/src/ATen/native/UpSample.h): identity when equal, >>1 for exact 2x, otherwise
// min(floor(dst * (float)in/out), in-1) in fp32 (quirk Q3; pinned by tests/golden/g4_nearest_maps.npz)
std::vector<int> nearest_map(int in, int out) {
  std::vector<int> m(out);
  const float scale = (float)in / (float)out;
  for (int i = 0; i < out; ++i) {
    if (in == out)
      m[i] = i;
    else if (out == 2 * in)
      m[i] = i >> 1;
    else
      m[i] = std::min((int)floorf((float)i * scale), in - 1);
  }
  return m;
}

std::vector<int> window_map(int B, int H, int W, int ws, int shift) {
  std::vector<int> m((size_t)B * H * W);
  const int nWh = H / ws, nWw = W / ws;
  size_t p = 0;
  for (int b = 0; b < B; ++b)
    for (int wr = 0; wr < nWh; ++wr)
      for (int wc = 0; wc < nWw; ++wc)
        for (int i = 0; i < ws; ++i)
          for (int j = 0; j < ws; ++j) {
            const int r = (wr * ws + i + shift) % H, c = (wc * ws + j + shift) % W;
            m[p++] = (b * H + r) * W + c;
          }
  return m;
}

int upload_map(Model& m, const std::vector<int>& h, const int** out) {
  int* d = nullptr;
  VV_HIP(hipMalloc(&d, h.size() * sizeof(int)));
  VV_HIP(hipMemcpy(d, h.data(), h.size() * sizeof(int), hipMemcpyHostToDevice));
  m.maps_owned.push_back(d);
  *out = d;
  return 0;
}

int init_stage(Model& m, Stage& s, int G, int H, int W, int C, int heads, int depth) {
  s.G = G;
  s.H = H;
  s.W = W;
  s.C = C;
  s.heads = heads;
  s.depth = depth;
  s.M = m.B * H * W;
  s.nWh = H / m.cfg.ws;
  s.nWw = W / m.cfg.ws;
  s.w.assign(depth, {});
  int rc;
  for (int k = 0; k < 2; ++k) {
    const std::vector<int> fwd = window_map(m.B, H, W, m.cfg.ws, k ? m.cfg.ws / 2 : 0);
    std::vector<int> inv(fwd.size(), -1);
    for (size_t j = 0; j < fwd.size(); ++j) {
      if (fwd[j] < 0 || (size_t)fwd[j] >= fwd.size() || inv[fwd[j]] >= 0) return VV_E_STATE;  // not a permutation
      inv[fwd[j]] = (int)j;
    }
    if ((rc = upload_map(m, fwd, &s.idx[k]))) return rc;
    if ((rc = upload_map(m, inv, &s.idxinv[k]))) return rc;
  }
  return 0;
}

void plan_stage_save(Planner& P, const Stage& s, StageSave& sv, float* x0_external) {
  const size_t GMC = (size_t)s.G * s.M * s.C;
  sv.x.assign(s.depth + 1, nullptr);
  sv.st1.assign(s.depth, nullptr);
  sv.qkv = sv.P = sv.x1 = sv.st2 = sv.h1 = sv.st1;
  sv.x[0] = x0_external ? x0_external : P.f(GMC);
  const size_t nwin = (size_t)s.M / 16;
  for (int b = 0; b < s.depth; ++b) {
    sv.st1[b] = P.f((size_t)s.G * s.M * 2);
    sv.qkv[b] = P.f(GMC * 3);
    sv.P[b] = P.f((size_t)s.G * nwin * s.heads * 256);
    sv.x1[b] = P.f(GMC);
    sv.st2[b] = P.f((size_t)s.G * s.M * 2);
    sv.h1[b] = P.f(GMC * 4);
    sv.x[b + 1] = P.f(GMC);
  }
}

int bind_weights(Model& m) {
  const Cfg& c = m.cfg;
  auto w = [&](const std::string& n) -> const float* {
    auto it = m.W.find(n);
    return it == m.W.end() ? nullptr : it->second;
  };
  auto blk = [&](const std::string& pre) {
    BlockW b;
    b.n1g = w(pre + ".norm1.weight");
    b.n1b = w(pre + ".norm1.bias");
    b.table = w(pre + ".attn.relative_position_bias_table");
    b.qkvW = w(pre + ".attn.qkv.weight");
    b.qkvWT = w(pre + ".attn.qkv.weight^T");
    b.qkvb = w(pre + ".attn.qkv.bias");
    b.projW = w(pre + ".attn.proj.weight");
    b.projWT = w(pre + ".attn.proj.weight^T");
    b.projb = w(pre + ".attn.proj.bias");
    b.n2g = w(pre + ".norm2.weight");
    b.n2b = w(pre + ".norm2.bias");
    b.fc1W = w(pre + ".mlp.fc1.weight");
    b.fc1WT = w(pre + ".mlp.fc1.weight^T");
    b.fc1b = w(pre + ".mlp.fc1.bias");
    b.fc2W = w(pre + ".mlp.fc2.weight");
    b.fc2WT = w(pre + ".mlp.fc2.weight^T");
    b.fc2b = w(pre + ".mlp.fc2.bias");
    auto wm = [&](const std::string& n) -> const float* {
      auto it = m.Wmax.find(n);
      return it == m.Wmax.end() ? nullptr : it->second;
    };
    b.fc1Wmax = wm(pre + ".mlp.fc1.weight");
    b.fc1bmax = wm(pre + ".mlp.fc1.bias");
    b.fc2Wmax = wm(pre + ".mlp.fc2.weight");
    b.qkvWmax = wm(pre + ".attn.qkv.weight");
    b.qkvbmax = wm(pre + ".attn.qkv.bias");
    return b;
  };
  for (int g = 0; g < c.G; ++g) {
    const std::string e = "enc.enc_list." + std::to_string(g), d = "dec.dec_list." + std::to_string(g);
    for (int b = 0; b < c.d0; ++b) {
      m.enc0.w[b][g] = blk(e + ".layers.0.blocks." + std::to_string(b));
      m.dec0.w[b][g] = blk(d + ".layers_up.1.blocks." + std::to_string(b));
    }
    for (int b = 0; b < c.d1; ++b) {
      m.enc1.w[b][g] = blk(e + ".layers.1.blocks." + std::to_string(b));
      m.dec1.w[b][g] = blk(d + ".layers_up.0.blocks." + std::to_string(b));
    }
  }
  for (size_t l = 0; l < m.lg.size(); ++l)
    for (int b = 0; b < m.lg[l].depth; ++b)
      m.lg[l].w[b][0] = blk("net.layers." + std::to_string(l) + ".blocks." + std::to_string(b));
  return 0;
}

// ----------------------------------------------------------------------------
// forward / backward of one Swin stage (BasicLayer / BasicLayer_up / Layer: blocks only)
// ----------------------------------------------------------------------------
GemmArgs gemm_base(int M, int N, int K, int G, int epi, int math, const vv::Tuning* tune) {
  GemmArgs a;
  memset(&a, 0, sizeof(a));
  a.math = math;
  a.tune = tune;
  a.M = M;
  a.N = N;
  a.K = K;
  a.ksplit = K;
  a.lda = K;
  a.lda2 = 0;
  a.ldc = N;
  a.ldr = N;
  a.ldaux = N;
  a.epi = epi;
  a.ngroups = G;
  return a;
}

GemmArgs gemm_base(int M, int N, int K, int G, int epi, const Scratch& sc) {
  GemmArgs a = gemm_base(M, N, K, G, epi, sc.math, sc.tune);
  a.apl = sc.apl;
  a.apl_halfs = sc.apl_halfs;
  return a;
}

// the LayerNorm feeding GEMM `a` writes the fp16x3 planes of its output (and no fp32 copy when `fp32_too` is false)
// if the GEMM runs the split-operand kernel (tile 48); returns whether it does
// the GELU / gelu' GEMM p writes the fp16x3 A planes (into its output buffer h, same bytes as the fp32 C) and the
// row scales (rs2) of the K = 4C GEMM c that consumes that output, when both run on tile 48 (GemmArgs.opl: the
// row scale from an a-priori bound, so no k_rowsplit pass over the 2048 x 4608 activation)
bool gelu_feeds_planes(GemmArgs& p, GemmArgs& c, const float* wmax, const float* bmax, const Scratch& sc) {
  const vv::Tuning& T = sc.tune ? *sc.tune : vv::kDefaultTuning;
  if (!T.gelu_planes || !wmax || p.ngroups != 1 || c.ngroups != 1 || !sc.apl || c.g[0].A != p.g[0].C) return false;
  GemmArgs cc = c;
  cc.apre = reinterpret_cast<const unsigned short*>(p.g[0].C);
  cc.ascale = sc.rs2;
  if (!vv::gemm_plane_tile(vv::gemm_tile_of(p)) || !vv::gemm_plane_tile(vv::gemm_tile_of(cc))) return false;
  p.opl = reinterpret_cast<unsigned short*>(p.g[0].C);
  p.ors = sc.rs2;
  p.obw = wmax;
  p.obb = bmax;
  c.apre = cc.apre;
  c.ascale = sc.rs2;
  return true;
}

// the LG-stage attention forward writes the proj GEMM's fp16x3 A planes (into o's buffer) and row scales (rs2)
// when that GEMM runs on tile 48 (AttnArgs.opl); q: the qkv GEMM whose output the attention reads (its A row scales
// bound |v|)
bool attn_feeds_planes(AttnArgs& at, GemmArgs& p, const GemmArgs& q, const BlockW& w, const Scratch& sc) {
  const vv::Tuning& T = sc.tune ? *sc.tune : vv::kDefaultTuning;
  if (!T.attn_planes || !at.mfma || !w.qkvWmax || at.ngroups != 1 || at.ws != 4 || at.C != 192 * at.heads ||
      !q.ascale || !sc.apl || p.ngroups != 1 || p.g[0].A != at.g[0].o)
    return false;
  GemmArgs pp = p;
  pp.apre = reinterpret_cast<const unsigned short*>(at.g[0].o);
  pp.ascale = sc.rs2;
  if (!vv::gemm_plane_tile(vv::gemm_tile_of(pp))) return false;
  at.opl = reinterpret_cast<unsigned short*>(at.g[0].o);
  at.ors = sc.rs2;
  at.vrs = q.ascale;
  at.vbw = w.qkvWmax;
  at.vbb = w.qkvbmax;
  p.apre = pp.apre;
  p.ascale = sc.rs2;
  return true;
}

bool ln_feeds_planes(const GemmArgs& a, const Scratch& sc) {
  const vv::Tuning& T = sc.tune ? *sc.tune : vv::kDefaultTuning;
  return sc.apl && T.ln_planes && T.ln_scales && vv::gemm_plane_tile(vv::gemm_tile_of(a));
}

LnArgs ln_base(int rows, int C, int G, float eps) {
  LnArgs a;
  memset(&a, 0, sizeof(a));
  a.rows = rows;
  a.C = C;
  a.ldx = a.ldy = a.lddy = a.ldres = C;
  a.mode = LN_ROWMAP;
  a.eps = eps;
  a.ngroups = G;
  return a;
}

// vv_set_debug_sync(1): synchronise after every launch and report the first failing op (debug only)
std::atomic<int> g_sync_check{0};
bool sync_check() { return g_sync_check.load(std::memory_order_relaxed) != 0; }

#define CK(expr)                                                                                   \
  do {                                                                                             \
    hipError_t e_ = (expr);                                                                        \
    if (e_ == hipSuccess && sync_check()) {                                                        \
      e_ = hipDeviceSynchronize();                                                                 \
      if (e_ != hipSuccess) fprintf(stderr, "debug sync: %s:%d %s -> %s\n", __FILE__, __LINE__, \
                                    #expr, hipGetErrorString(e_));                                 \
    }                                                                                              \
    if (e_ != hipSuccess) return fail((int)e_, "%s:%d %s -> %s", __FILE__, __LINE__, #expr,         \
                                      hipGetErrorString(e_));                                      \
  } while (0)

// the fused MLP sub-block (vv_tower.hip) for block b of a stage, fwd or bwd (gx: the stage gradient, in place);
// false where it does not apply (fp16x3 math only, dim 96, weights with fp16 planes): the unfused launches run
bool mlp_args(const Stage& S, int b, const StageSave& sv, const Scratch& sc, bool fwd, float* gx, vv::MlpArgs& ma) {
  const vv::Tuning& T = sc.tune ? *sc.tune : vv::kDefaultTuning;
  // fuse_mlp: bit 0 the dim-96 stages, bit 1 the dim-192 stages
  if (!(T.fuse_mlp & (S.C == 96 ? 1 : S.C == 192 ? 2 : 0)) || sc.math != vv::GEMM_SPLIT16 ||
      !vv::mlp_supported(S.C, S.M))
    return false;
  memset(&ma, 0, sizeof(ma));
  const int M = S.M, C = S.C;
  const size_t MC = (size_t)M * C;
  ma.M = M;
  ma.C = C;
  ma.ngroups = S.G;
  ma.eps = 1e-5f;
  ma.hc = T.mlp_hc;
  for (int g = 0; g < S.G; ++g) {
    const auto& w = S.w[b][g];
    vv::MlpGroup& G = ma.g[g];
    G.x = sv.x1[b] + g * MC;
    G.gamma = w.n2g;
    G.stats = sv.st2[b] + (size_t)g * M * 2;
    G.h1 = sv.h1[b] + g * MC * 4;
    if (fwd) {
      G.beta = w.n2b;
      vv::fp16_planes_of(w.fc1W, C, &G.w1h, &G.w1s);
      vv::fp16_planes_of(w.fc2W, 4 * C, &G.w2h, &G.w2s);
      G.b1 = w.fc1b;
      G.b2 = w.fc2b;
      G.out = sv.x[b + 1] + g * MC;
    } else {
      vv::fp16_planes_of(w.fc2WT, C, &G.w1h, &G.w1s);
      vv::fp16_planes_of(w.fc1WT, 4 * C, &G.w2h, &G.w2s);
      G.dy = gx + g * MC;
      G.out = gx + g * MC;
      G.rs = sc.rs + (size_t)g * M;
    }
    if (!G.w1h || !G.w2h) return false;
  }
  return true;
}

// the fused attention sub-block (vv_tower.hip) for block b, forward; false where it does not apply
bool ablk_args(const Stage& S, int b, const StageSave& sv, const Scratch& sc, int ws, int shift, const int* idx,
               vv::AblkArgs& aa, float* gx = nullptr) {
  const vv::Tuning& T = sc.tune ? *sc.tune : vv::kDefaultTuning;
  // fuse_attn: bit 0 the forward, bit 1 the backward (dim 96)
  if (!(T.fuse_attn & (gx ? 2 : 1)) || sc.math != vv::GEMM_SPLIT16 ||
      !vv::ablk_supported(S.C, S.heads, ws, S.M))
    return false;
  memset(&aa, 0, sizeof(aa));
  const int M = S.M, C = S.C;
  const size_t MC = (size_t)M * C;
  aa.M = M;
  aa.C = C;
  aa.heads = S.heads;
  aa.ngroups = S.G;
  aa.nWh = S.nWh;
  aa.nWw = S.nWw;
  aa.ws = ws;
  aa.shift = shift;
  aa.H = S.H;
  aa.scale = (float)std::pow((double)(C / S.heads), -0.5);
  aa.eps = 1e-5f;
  aa.map = idx;
  for (int g = 0; g < S.G; ++g) {
    const auto& w = S.w[b][g];
    vv::AblkGroup& G = aa.g[g];
    G.x = sv.x[b] + g * MC;
    G.n1g = w.n1g;
    G.n1b = w.n1b;
    G.stats = sv.st1[b] + (size_t)g * M * 2;
    vv::fp16_planes_of(w.qkvW, C, &G.wqh, &G.wqs);
    G.wqb = w.qkvb;
    G.table = w.table;
    G.qkv = sv.qkv[b] + g * MC * 3;
    G.P = sv.P[b] + (size_t)g * (M / 16) * S.heads * 256;
    vv::fp16_planes_of(w.projW, C, &G.wph, &G.wps);
    G.wpb = w.projb;
    G.out = sv.x1[b] + g * MC;
    if (!G.wqh || !G.wph || !G.wqb || !G.wpb) return false;
    if (gx) {  // backward: the stage gradient in place, the transposed weights
      G.out = gx + g * MC;
      G.rs = sc.rs + (size_t)g * M;
      vv::fp16_planes_of(w.projWT, C, &G.wpth, &G.wpts);
      vv::fp16_planes_of(w.qkvWT, 3 * C, &G.wqth, &G.wqts);
      if (!G.wpth || !G.wqth) return false;
    }
  }
  return true;
}

// the LG-stage proj GEMM (RESID) with its split-K fixup fused into LN2 (vv::gemm_ln) when LN2 only has to write
// fc1's tile-48 planes; hipErrorNotSupported where that does not apply (the caller runs gemm_nt + LayerNorm)
hipError_t proj_ln2(const Stage& S, int b, const StageSave& sv, const Scratch& sc, const GemmArgs& p, hipStream_t st) {
  const vv::Tuning& T = sc.tune ? *sc.tune : vv::kDefaultTuning;
  if (!T.fixup_ln || S.G != 1) return hipErrorNotSupported;
  vv::MlpArgs ma;
  if (mlp_args(S, b, sv, sc, true, nullptr, ma)) return hipErrorNotSupported;  // the fused MLP does its own LN2
  GemmArgs f1 = gemm_base(S.M, 4 * S.C, S.C, 1, EPI_GELU, sc);
  f1.ascale = sc.rs;
  f1.g[0] = {sc.t1, nullptr, S.w[b][0].fc1W, S.w[b][0].fc1b, sc.h, nullptr, sv.h1[b]};
  if (!ln_feeds_planes(f1, sc)) return hipErrorNotSupported;
  vv::GemmLnArgs l;
  memset(&l, 0, sizeof(l));
  l.gmap = nullptr;
  l.lo_x = 1;  // LN2 rows are the physical rows proj writes (through its crow)
  l.gamma = S.w[b][0].n2g;
  l.beta = S.w[b][0].n2b;
  l.eps = 1e-5f;
  l.pl = sc.apl;
  l.rs = sc.rs;
  l.stats = sv.st2[b];
  return vv::gemm_ln(p, l, st, sc.ws);
}

// the LG-stage fc2 GEMM (RESID) of block b with its split-K fixup fused into the next block's LN1 (window gather:
// LN row j reads GEMM row idx[j]) when that LayerNorm only has to write qkv's tile-48 planes. The next block is
// block b + 1, or for the last block block 0 of the next LG stage NS (r06: same rows and width, its input buffer
// is this stage's output, plan_stage_save), whose stage_fwd then skips that LN1
// a RESID GEMM `f` (one group, output = block nb's input x) with its split-K fixup fused into block nb's LN1 of stage
// TS (the LayerNorm then writes only qkv's tile-48 planes, row scales and stats); hipErrorNotSupported where that
// does not apply
hipError_t gemm_ln1_into(const GemmArgs& f, const Stage& TS, const StageSave& tsv, int nb, const Scratch& sc, int ws,
                         hipStream_t st) {
  const vv::Tuning& T = sc.tune ? *sc.tune : vv::kDefaultTuning;
  if (!T.fixup_ln || TS.G != 1 || f.ngroups != 1 || f.M != TS.M || f.N != TS.C || f.g[0].C != tsv.x[nb])
    return hipErrorNotSupported;
  const int shift = (nb % 2 == 0) ? 0 : ws / 2;
  vv::AblkArgs aa;
  if (ablk_args(TS, nb, tsv, sc, ws, shift, TS.idx[shift ? 1 : 0], aa)) return hipErrorNotSupported;
  GemmArgs q = gemm_base(TS.M, 3 * TS.C, TS.C, 1, EPI_STORE, sc);
  q.ascale = sc.rs;
  q.g[0] = {sc.t1, nullptr, TS.w[nb][0].qkvW, TS.w[nb][0].qkvb, tsv.qkv[nb], nullptr, nullptr};
  if (!ln_feeds_planes(q, sc)) return hipErrorNotSupported;
  vv::GemmLnArgs l;
  memset(&l, 0, sizeof(l));
  l.gmap = TS.idx[shift ? 1 : 0];  // LN1 -> window order
  l.ginv = T.fixup_ln_rows ? TS.idxinv[shift ? 1 : 0] : nullptr;
  l.lo_x = 0;
  l.gamma = TS.w[nb][0].n1g;
  l.beta = TS.w[nb][0].n1b;
  l.eps = 1e-5f;
  l.pl = sc.apl;
  l.rs = sc.rs;
  l.stats = tsv.st1[nb];
  return vv::gemm_ln(f, l, st, sc.ws);
}

hipError_t fc2_ln1(const Stage& S, int b, const StageSave& sv, const Scratch& sc, int ws, const GemmArgs& f2,
                   hipStream_t st, const Stage* NS = nullptr, const StageSave* nsv = nullptr) {
  if (b + 1 < S.depth) return gemm_ln1_into(f2, S, sv, b + 1, sc, ws, st);
  if (!NS || !nsv || NS->depth < 1) return hipErrorNotSupported;
  return gemm_ln1_into(f2, *NS, *nsv, 0, sc, ws, st);
}

// NS / nsv: the LG stage that follows (its block 0's LN1 may be fused into this stage's last fc2 fixup: *ln1_next
// says whether it was); ln1_pre: this stage's block-0 LN1 already ran, fused into the previous stage's last fc2
int stage_fwd(const Stage& S, StageSave& sv, const Scratch& sc, int ws, hipStream_t st, const Stage* NS = nullptr,
              const StageSave* nsv = nullptr, bool ln1_pre = false, bool* ln1_next = nullptr) {
  const int G = S.G, M = S.M, C = S.C;
  const size_t MC = (size_t)M * C;
  const int nwin = M / 16;
  if (ln1_next) *ln1_next = false;
  bool ln1_done = ln1_pre;  // block b's LN1 already ran, fused into the fc2 fixup before it
  for (int b = 0; b < S.depth; ++b) {
    const int shift = (b % 2 == 0) ? 0 : ws / 2;
    const int* idx = S.idx[shift ? 1 : 0];
    bool ln2_done = false;
    const bool ln1_fused = ln1_done;
    ln1_done = false;
    vv::AblkArgs aa;
    if (ablk_args(S, b, sv, sc, ws, shift, idx, aa)) {
      CK(vv::ablk_fwd(aa, st));  // LN1 + qkv + window attention + proj + residual in one launch
    } else {
    // qkv (A's fp16x3 row scales from LN1; with tile 48 also A's planes, and LN1 writes no fp32 copy)
    GemmArgs q = gemm_base(M, 3 * C, C, G, EPI_STORE, sc);
    q.ascale = sc.rs;
    for (int g = 0; g < G; ++g)
      q.g[g] = {sc.t1 + g * MC, nullptr, S.w[b][g].qkvW, S.w[b][g].qkvb, sv.qkv[b] + g * MC * 3, nullptr, nullptr};
    const bool q_pl = ln_feeds_planes(q, sc);
    // LN1 -> window order
    LnArgs ln = ln_base(M, C, G, 1e-5f);
    ln.map = idx;
    for (int g = 0; g < G; ++g)
      ln.g[g] = {sv.x[b] + g * MC, S.w[b][g].n1g, S.w[b][g].n1b, q_pl ? nullptr : sc.t1 + g * MC,
                 sv.st1[b] + (size_t)g * M * 2, nullptr, nullptr, sc.rs + (size_t)g * M,
                 q_pl ? sc.apl + (size_t)g * M * 2 * C : nullptr};
    if (!ln1_fused) CK(layernorm_fwd(ln, st));
    if (q_pl) q.apre = sc.apl;
    CK(gemm_nt(q, st, -1, sc.ws));
    // window attention
    AttnArgs at;
    memset(&at, 0, sizeof(at));
    at.nwin = nwin;
    at.nWh = S.nWh;
    at.nWw = S.nWw;
    at.ws = ws;
    at.shift = shift;
    at.H = S.H;
    at.C = C;
    at.heads = S.heads;
    at.scale = (float)std::pow((double)(C / S.heads), -0.5);
    at.ngroups = G;
    at.mfma = (sc.tune ? *sc.tune : vv::kDefaultTuning).attn_mfma;
    for (int g = 0; g < G; ++g)
      at.g[g] = {sv.qkv[b] + g * MC * 3, S.w[b][g].table, sc.t2 + g * MC,
                 sv.P[b] + (size_t)g * nwin * S.heads * 256, nullptr, nullptr};
    // proj + window reverse + residual
    GemmArgs p = gemm_base(M, C, C, G, EPI_RESID, sc);
    p.crow = idx;
    for (int g = 0; g < G; ++g)
      p.g[g] = {sc.t2 + g * MC, nullptr, S.w[b][g].projW, S.w[b][g].projb, sv.x1[b] + g * MC, sv.x[b] + g * MC,
                nullptr};
    attn_feeds_planes(at, p, q, S.w[b][0], sc);
    CK(attn_fwd(at, st));
    // proj's split-K fixup fused into LN2 where that LayerNorm feeds fc1's planes (gemm_ln)
    const hipError_t pe = proj_ln2(S, b, sv, sc, p, st);
    if (pe == hipSuccess)
      ln2_done = true;
    else if (pe == hipErrorNotSupported)
      CK(gemm_nt(p, st, -1, sc.ws));
    else
      CK(pe);
    }
    vv::MlpArgs ma;
    if (mlp_args(S, b, sv, sc, true, nullptr, ma)) {  // LN2 + fc1 + GELU + fc2 + residual in one launch
      CK(vv::mlp_fwd(ma, st));
      continue;
    }
    // fc1 + GELU (row scales, and with tile 48 the planes, from LN2)
    GemmArgs f1 = gemm_base(M, 4 * C, C, G, EPI_GELU, sc);
    f1.ascale = sc.rs;
    for (int g = 0; g < G; ++g)
      f1.g[g] = {sc.t1 + g * MC, nullptr, S.w[b][g].fc1W, S.w[b][g].fc1b, sc.h + g * MC * 4, nullptr,
                 sv.h1[b] + g * MC * 4};
    const bool f1_pl = ln_feeds_planes(f1, sc);
    // LN2
    LnArgs ln2 = ln_base(M, C, G, 1e-5f);
    for (int g = 0; g < G; ++g)
      ln2.g[g] = {sv.x1[b] + g * MC, S.w[b][g].n2g, S.w[b][g].n2b, f1_pl ? nullptr : sc.t1 + g * MC,
                  sv.st2[b] + (size_t)g * M * 2, nullptr, nullptr, sc.rs + (size_t)g * M,
                  f1_pl ? sc.apl + (size_t)g * M * 2 * C : nullptr};
    if (!ln2_done) CK(layernorm_fwd(ln2, st));
    if (f1_pl) f1.apre = sc.apl;
    // fc2 + residual (with tile 48, fc1's epilogue writes its A planes)
    GemmArgs f2 = gemm_base(M, C, 4 * C, G, EPI_RESID, sc);
    for (int g = 0; g < G; ++g)
      f2.g[g] = {sc.h + g * MC * 4, nullptr, S.w[b][g].fc2W, S.w[b][g].fc2b, sv.x[b + 1] + g * MC, sv.x1[b] + g * MC,
                 nullptr};
    gelu_feeds_planes(f1, f2, S.w[b][0].fc1Wmax, S.w[b][0].fc1bmax, sc);
    CK(gemm_nt(f1, st, -1, sc.ws));
    // fc2's split-K fixup fused into the next block's LN1 where that LayerNorm feeds qkv's planes
    const hipError_t fe = fc2_ln1(S, b, sv, sc, ws, f2, st, ln1_next ? NS : nullptr, nsv);
    if (fe == hipSuccess) {
      ln1_done = true;
      if (b + 1 == S.depth) *ln1_next = true;
    }
    else if (fe == hipErrorNotSupported)
      CK(gemm_nt(f2, st, -1, sc.ws));
    else
      CK(fe);
  }
  return 0;
}

// an input-gradient GEMM g (EPI_STORE into ln's dy) with its split-K fixup fused into the LayerNorm backward ln that
// consumes it (vv::gemm_ln, bwd): dy never goes to HBM; hipErrorNotSupported where that does not apply
hipError_t gemm_ln_bwd(const GemmArgs& g, const LnArgs& ln, const Scratch& sc, hipStream_t st) {
  const vv::Tuning& T = sc.tune ? *sc.tune : vv::kDefaultTuning;
  if (!T.fixup_ln || ln.ngroups != 1 || g.ngroups != 1 || ln.mode != LN_ROWMAP || ln.rows != g.M || ln.C != g.N ||
      ln.ldx != ln.C || ln.ldy != ln.C || ln.lddy != ln.C || ln.ldres != ln.C || ln.g[0].dy != g.g[0].C)
    return hipErrorNotSupported;
  vv::GemmLnArgs l;
  memset(&l, 0, sizeof(l));
  l.bwd = 1;
  l.lmap = ln.map;
  l.x = ln.g[0].x;
  l.res = ln.g[0].res;
  l.y = ln.g[0].y;
  l.gamma = ln.g[0].gamma;
  l.stats = ln.g[0].stats;
  l.rs = ln.g[0].rs;
  l.pl = ln.g[0].pl;
  l.eps = ln.eps;
  return vv::gemm_ln(g, l, st, sc.ws);
}

// gx: [G][M][C] gradient w.r.t. the stage output, overwritten in place with the input gradient. Consecutive LG
// stages (r06, Tuning.fixup_ln_cross): planes_out -- block 0's LN1 backward also writes gx's row scales and fp16x3
// planes for the last fc2 input-gradient GEMM of the stage below; gx_planes_in -- this stage's gx arrives with them
int stage_bwd(const Stage& S, const StageSave& sv, const Scratch& sc, int ws, float* gx, hipStream_t st,
              bool gx_planes_in = false, bool planes_out = false) {
  const int G = S.G, M = S.M, C = S.C;
  const size_t MC = (size_t)M * C;
  const int nwin = M / 16;
  // the fc2 input-gradient GEMM of every block but the last takes gx from the LN1 backward of the block above it
  // (same shapes in every block): with tile 48 that LayerNorm writes gx's planes too
  GemmArgs f2x = gemm_base(M, 4 * C, C, G, EPI_DGELU, sc);
  f2x.ascale = sc.rs;
  for (int g = 0; g < G; ++g) f2x.g[g] = {gx, nullptr, S.w[0][g].fc2WT, nullptr, sc.h, nullptr, sv.h1[0]};
  const bool f2_pl = ln_feeds_planes(f2x, sc);
  for (int b = S.depth - 1; b >= 0; --b) {
    const int shift = (b % 2 == 0) ? 0 : ws / 2;
    const int* idx = S.idx[shift ? 1 : 0];
    GemmArgs p = gemm_base(M, C, C, G, EPI_STORE, sc);
    p.arow = idx;
    p.ascale = sc.rs;  // per physical row of gx (the gather is applied to the scales too)
    for (int g = 0; g < G; ++g)
      p.g[g] = {gx + g * MC, nullptr, S.w[b][g].projWT, nullptr, sc.t2 + g * MC, nullptr, nullptr};
    const bool p_pl = ln_feeds_planes(p, sc);
    vv::MlpArgs ma;
    if (!p_pl && mlp_args(S, b, sv, sc, false, gx, ma)) {
      CK(vv::mlp_bwd(ma, st));  // fc2^T + GELU' + fc1^T + LN2 backward + residual, gx in place (+ its row scales)
    } else {
      GemmArgs f2 = gemm_base(M, 4 * C, C, G, EPI_DGELU, sc);
      if (b < S.depth - 1 || gx_planes_in) {
        f2.ascale = sc.rs;  // gx from the LN1 backward of block b + 1 (below) or of the next stage, with its row scales
        if (f2_pl) f2.apre = sc.apl;
      }
      for (int g = 0; g < G; ++g)
        f2.g[g] = {gx + g * MC, nullptr, S.w[b][g].fc2WT, nullptr, sc.h + g * MC * 4, nullptr, sv.h1[b] + g * MC * 4};
      GemmArgs f1 = gemm_base(M, C, 4 * C, G, EPI_STORE, sc);
      for (int g = 0; g < G; ++g)
        f1.g[g] = {sc.h + g * MC * 4, nullptr, S.w[b][g].fc1WT, nullptr, sc.t1 + g * MC, nullptr, nullptr};
      gelu_feeds_planes(f2, f1, S.w[b][0].fc2Wmax, nullptr, sc);  // max |fc2^T| = max |fc2|
      CK(gemm_nt(f2, st, -1, sc.ws));
      LnArgs ln2 = ln_base(M, C, G, 1e-5f);
      for (int g = 0; g < G; ++g)
        ln2.g[g] = {sv.x1[b] + g * MC, S.w[b][g].n2g, nullptr, gx + g * MC, sv.st2[b] + (size_t)g * M * 2,
                    sc.t1 + g * MC, gx + g * MC, sc.rs + (size_t)g * M, p_pl ? sc.apl + (size_t)g * M * 2 * C : nullptr};
      const hipError_t fe = gemm_ln_bwd(f1, ln2, sc, st);  // fc1^T with its fixup fused into the LN2 backward
      if (fe == hipErrorNotSupported) {
        CK(gemm_nt(f1, st, -1, sc.ws));
        CK(layernorm_bwd(ln2, st));
      } else {
        CK(fe);
      }
    }
    if (p_pl) p.apre = sc.apl;  // planes in physical row order: the kernel gathers them through arow
    vv::AblkArgs ab;
    if (!(f2_pl && (b > 0 || planes_out)) && ablk_args(S, b, sv, sc, ws, shift, idx, ab, gx)) {
      CK(vv::ablk_bwd(ab, st));  // proj^T + window-attention backward + qkv^T + LN1 backward + residual, in place
      continue;
    }
    CK(gemm_nt(p, st, -1, sc.ws));
    AttnArgs at;
    memset(&at, 0, sizeof(at));
    at.nwin = nwin;
    at.nWh = S.nWh;
    at.nWw = S.nWw;
    at.ws = ws;
    at.shift = shift;
    at.H = S.H;
    at.C = C;
    at.heads = S.heads;
    at.scale = (float)std::pow((double)(C / S.heads), -0.5);
    at.ngroups = G;
    at.mfma = (sc.tune ? *sc.tune : vv::kDefaultTuning).attn_mfma;
    for (int g = 0; g < G; ++g)
      at.g[g] = {sv.qkv[b] + g * MC * 3, S.w[b][g].table, nullptr, sv.P[b] + (size_t)g * nwin * S.heads * 256,
                 sc.t2 + g * MC, sc.dqkv + g * MC * 3};
    CK(attn_bwd(at, st));
    GemmArgs q = gemm_base(M, C, 3 * C, G, EPI_STORE, sc);
    for (int g = 0; g < G; ++g)
      q.g[g] = {sc.dqkv + g * MC * 3, nullptr, S.w[b][g].qkvWT, nullptr, sc.t1 + g * MC, nullptr, nullptr};
    LnArgs ln1 = ln_base(M, C, G, 1e-5f);
    ln1.map = idx;
    const bool l1_pl = f2_pl && (b > 0 || planes_out);  // planes for the next fc2 input-gradient GEMM
    for (int g = 0; g < G; ++g)
      ln1.g[g] = {sv.x[b] + g * MC, S.w[b][g].n1g, nullptr, gx + g * MC, sv.st1[b] + (size_t)g * M * 2,
                  sc.t1 + g * MC, gx + g * MC, sc.rs + (size_t)g * M, l1_pl ? sc.apl + (size_t)g * M * 2 * C : nullptr};
    const hipError_t qe = gemm_ln_bwd(q, ln1, sc, st);  // qkv^T with its fixup fused into the LN1 backward
    if (qe == hipErrorNotSupported) {
      CK(gemm_nt(q, st, -1, sc.ws));
      CK(layernorm_bwd(ln1, st));
    } else {
      CK(qe);
    }
  }
  return 0;
}

// ----------------------------------------------------------------------------
// model construction
// ----------------------------------------------------------------------------
int create_model(vv_ctx* ctx, const vv_lgunet_config* rc, int B, int nslots, int* id) {
  auto m = std::make_unique<Model>();
  int r;
  if ((r = parse_cfg(rc, m->cfg))) return r;
  if (B < 1 || nslots < 1) return fail(VV_E_ARG, "batch and n_slots must be >= 1");
  m->B = B;
  m->nslots = nslots;
  const Cfg& c = m->cfg;
  m->params = enumerate_params(c);
  // weights arena: params + transposed copies of 2-D weights
  size_t wbytes = 0;
  for (auto& p : m->params) {
    wbytes += Arena::up(numel(p.shape) * 4);
    if (p.shape.size() == 2 && p.name.size() > 7 && p.name.compare(p.name.size() - 7, 7, ".weight") == 0)
      wbytes += Arena::up(numel(p.shape) * 4);
  }
  m->warena = std::make_unique<Arena>();
  if (hipMalloc(&m->warena->base, wbytes) != hipSuccess) return fail(VV_E_ALLOC, "weights: %zu bytes", wbytes);
  m->warena->cap = wbytes;
  m->parena = std::make_unique<Arena>();
  const size_t pbytes = vv::split_arena_bytes(wbytes / 4);
  if (hipMalloc(&m->parena->base, pbytes) != hipSuccess) return fail(VV_E_ALLOC, "weight split planes: %zu bytes", pbytes);
  m->parena->cap = pbytes;
  vv::register_split_arena(reinterpret_cast<const float*>(m->warena->base), wbytes / 4,
                           reinterpret_cast<const unsigned short*>(m->parena->base));
  m->marena = std::make_unique<Arena>();
  if (hipMalloc(&m->marena->base, m->params.size() * sizeof(float)) != hipSuccess)
    return fail(VV_E_ALLOC, "param maxima");
  m->marena->cap = m->params.size() * sizeof(float);
  for (size_t i = 0; i < m->params.size(); ++i)
    m->Wmax[m->params[i].name] = reinterpret_cast<const float*>(m->marena->base) + i;
  size_t off = 0;
  for (auto& p : m->params) {
    float* d = reinterpret_cast<float*>(m->warena->base + off);
    off += Arena::up(numel(p.shape) * 4);
    m->pptr.push_back(d);
    m->W[p.name] = d;
    if (p.shape.size() == 2 && p.name.size() > 7 && p.name.compare(p.name.size() - 7, 7, ".weight") == 0) {
      float* t = reinterpret_cast<float*>(m->warena->base + off);
      off += Arena::up(numel(p.shape) * 4);
      m->W[p.name + "^T"] = t;
    }
  }
  // stages
  if ((r = init_stage(*m, m->enc0, c.G, c.H0, c.W0, c.C0, c.h0, c.d0))) return r;
  if ((r = init_stage(*m, m->enc1, c.G, c.H1, c.W1, c.C1, c.h1, c.d1))) return r;
  if ((r = init_stage(*m, m->dec1, c.G, c.H1, c.W1, c.C1, c.h1, c.d1))) return r;
  if ((r = init_stage(*m, m->dec0, c.G, c.H0, c.W0, c.C0, c.h0, c.d0))) return r;
  m->lg.resize(c.lg_depth.size());
  for (size_t l = 0; l < m->lg.size(); ++l)
    if ((r = init_stage(*m, m->lg[l], 1, c.H1, c.W1, c.E, c.lg_heads[l], c.lg_depth[l]))) return r;
  bind_weights(*m);
  // activation arena (two passes: size, then carve)
  const size_t M0 = (size_t)B * c.H0 * c.W0, M1 = (size_t)B * c.H1 * c.W1;
  const size_t G = c.G;
  for (int pass = 0; pass < 2; ++pass) {
    Planner P;
    if (pass == 1) P.base = m->aarena->base;
    // scratch sized for the largest stage
    size_t mx = 0;
    auto upd = [&](const Stage& s) { mx = std::max(mx, (size_t)s.G * s.M * s.C); };
    upd(m->enc0);
    upd(m->enc1);
    for (auto& s : m->lg) upd(s);
    m->sc.t1 = P.f(mx);
    m->sc.t2 = P.f(mx);
    m->sc.h = P.f(mx * 4);
    m->sc.dqkv = P.f(mx * 3);
    size_t mrows = 0;
    for (auto* st : {&m->enc0, &m->enc1, &m->dec1, &m->dec0}) mrows = std::max(mrows, (size_t)st->G * st->M);
    for (auto& st : m->lg) mrows = std::max(mrows, (size_t)st.G * st.M);
    m->sc.rs = P.f(mrows);
    m->sc.rs2 = P.f(mrows);
    m->sc.ws = P.f(vv::gemm_ws_floats());
    // tile-48 A planes: the largest A of a stage GEMM (fc2 forward / fc1 input gradient, K = 4C) as two fp16 planes
    m->sc.apl = reinterpret_cast<unsigned short*>(P.f(mx * 4));
    m->sc.apl_halfs = mx * 8;
    m->xm = P.f(G * M1 * 4 * c.C0);
    m->cat = P.f(M1 * G * c.C1);
    m->dp = P.f(M1 * G * c.C1);
    m->xe = P.f(G * M0 * c.C0);
    m->yn = P.f(G * M0 * c.C0);
    m->gy = P.f(G * M0 * c.C0);
    m->gd0 = P.f(G * M0 * c.C0);
    m->gxe = P.f(G * M0 * c.C0);
    m->gsk0 = P.f(G * M0 * c.C0);
    m->gex = P.f(G * M1 * 2 * c.C1);
    m->gd1 = P.f(G * M1 * c.C1);
    m->gdp = P.f(M1 * G * c.C1);
    m->gsk1 = P.f(G * M1 * c.C1);
    m->glg = P.f(M1 * c.E);
    m->gcat = P.f(M1 * G * c.C1);
    m->gxm = P.f(G * M1 * 4 * c.C0);
    m->saves.assign(nslots, Save{});
    for (int s = 0; s < nslots; ++s) {
      Save& sv = m->saves[s];
      plan_stage_save(P, m->enc0, sv.enc0, nullptr);
      sv.st_m = P.f(G * M1 * 2);
      plan_stage_save(P, m->enc1, sv.enc1, nullptr);
      sv.st_en = P.f(G * M1 * 2);
      sv.lg.resize(m->lg.size());
      for (size_t l = 0; l < m->lg.size(); ++l)
        plan_stage_save(P, m->lg[l], sv.lg[l], l == 0 ? nullptr : sv.lg[l - 1].x.back());
      plan_stage_save(P, m->dec1, sv.dec1, nullptr);
      sv.ex = P.f(G * M1 * 2 * c.C1);
      sv.st_ex = P.f(G * M0 * 2);
      plan_stage_save(P, m->dec0, sv.dec0, nullptr);
      sv.st_nu = P.f(G * M0 * 2);
    }
    if (pass == 0) {
      m->aarena = std::make_unique<Arena>();
      if (hipMalloc(&m->aarena->base, P.bytes) != hipSuccess)
        return fail(VV_E_ALLOC, "activations: %zu bytes", P.bytes);
      m->aarena->cap = P.bytes;
      m->workspace = (int64_t)(P.bytes + wbytes);
    }
  }
  *id = (int)ctx->models.size();
  ctx->models.push_back(std::move(m));
  return 0;
}

Model* get_model(vv_ctx* ctx, int id) {
  if (!ctx || id < 0 || id >= (int)ctx->models.size()) return nullptr;
  return ctx->models[id].get();
}

// ----------------------------------------------------------------------------
// whole-network forward / backward   (LGUnet_all.forward, transformer.py:747-752)
// ----------------------------------------------------------------------------
int model_fwd(Model& m, int slot, const float* in, float* out, int climit, hipStream_t st) {
  const Cfg& c = m.cfg;
  Save& sv = m.saves[slot];
  const int G = c.G, B = m.B, C0 = c.C0, C1 = c.C1, E = c.E;
  const int M0 = B * c.H0 * c.W0, M1 = B * c.H1 * c.W1;
  const size_t M0C0 = (size_t)M0 * C0, M1C1 = (size_t)M1 * C1;
  auto w = [&](const std::string& n) { return m.W.at(n); };
  auto eg = [&](int g) { return "enc.enc_list." + std::to_string(g); };
  auto dg = [&](int g) { return "dec.dec_list." + std::to_string(g); };

  // ---- Enc_net: PatchEmbed + absolute_pos_embed (transformer.py:392-394)
  PatchArgs pa;
  memset(&pa, 0, sizeof(pa));
  pa.B = B;
  pa.Himg = c.Himg;
  pa.Wimg = c.Wimg;
  pa.Cimg = c.Cin;
  pa.Ctok = C0;
  pa.img = in;
  pa.ngroups = G;
  pa.tune = m.sc.tune;
  for (int g = 0, off = 0; g < G; off += c.raw.inchans[g], ++g) {
    pa.g[g].w = w(eg(g) + ".patch_embed.proj.weight");
    pa.g[g].bias = w(eg(g) + ".patch_embed.proj.bias");
    pa.g[g].pos = w(eg(g) + ".absolute_pos_embed");
    pa.g[g].tok = sv.enc0.x[0] + g * M0C0;
    pa.g[g].cin_off = off;
    pa.g[g].cin = c.raw.inchans[g];
  }
  CK(patch_embed_fwd(pa, st));
  int r;
  if ((r = stage_fwd(m.enc0, sv.enc0, m.sc, c.ws, st))) return r;
  float* skip0 = sv.enc0.x.back();
  // PatchMerging: gather + LN(4C0, eps 1e-6) + reduction (transformer.py:76-96)
  LnArgs lm = ln_base(M1, 4 * C0, G, 1e-6f);
  lm.mode = LN_MERGE;
  lm.Hin = c.H0;
  lm.Win = c.W0;
  lm.ldx = C0;
  for (int g = 0; g < G; ++g)
    lm.g[g] = {skip0 + g * M0C0, w(eg(g) + ".layers.1.downsample.norm.weight"),
               w(eg(g) + ".layers.1.downsample.norm.bias"), m.xm + (size_t)g * M1 * 4 * C0,
               sv.st_m + (size_t)g * M1 * 2, nullptr, nullptr};
  CK(layernorm_fwd(lm, st));
  GemmArgs red = gemm_base(M1, C1, 4 * C0, G, EPI_STORE, m.sc);
  for (int g = 0; g < G; ++g)
    red.g[g] = {m.xm + (size_t)g * M1 * 4 * C0, nullptr, w(eg(g) + ".layers.1.downsample.reduction.weight"), nullptr,
                sv.enc1.x[0] + g * M1C1, nullptr, nullptr};
  CK(gemm_nt(red, st, -1, m.sc.ws));
  if ((r = stage_fwd(m.enc1, sv.enc1, m.sc, c.ws, st))) return r;
  float* skip1 = sv.enc1.x.back();
  // encoder norm -> concat (transformer.py:402, 567)
  LnArgs le = ln_base(M1, C1, G, 1e-6f);
  le.ldy = G * C1;
  for (int g = 0; g < G; ++g)
    le.g[g] = {skip1 + g * M1C1, w(eg(g) + ".norm.weight"), w(eg(g) + ".norm.bias"), m.cat + g * C1,
               sv.st_en + (size_t)g * M1 * 2, nullptr, nullptr};
  CK(layernorm_fwd(le, st));
  // Enc_net.proj (+ LG_net.pos_embed, transformer.py:704)
  float* lg_in = m.lg.empty() ? sv.dec1.x[0] : sv.lg[0].x[0];
  GemmArgs ep = gemm_base(M1, E, G * C1, 1, EPI_RESID, m.sc);
  ep.rmod = c.H1 * c.W1;
  ep.ldr = E;
  ep.g[0] = {m.cat, nullptr, w("enc.proj.weight"), w("enc.proj.bias"), lg_in, w("net.pos_embed"), nullptr};
  // consecutive LG stages: the last fc2 fixup of one runs the next stage's first LN1, and Enc_net.proj's fixup the
  // first LG stage's (Tuning.fixup_ln_cross)
  const bool cross = (m.sc.tune ? *m.sc.tune : vv::kDefaultTuning).fixup_ln_cross;
  size_t pre = 0;
  {
    const hipError_t e = cross && !m.lg.empty() ? gemm_ln1_into(ep, m.lg[0], sv.lg[0], 0, m.sc, c.ws, st)
                                                : hipErrorNotSupported;
    if (e == hipSuccess)
      pre = 1;
    else if (e == hipErrorNotSupported)
      CK(gemm_nt(ep, st, -1, m.sc.ws));
    else
      CK(e);
  }
  // ---- LG_net layers
  for (size_t l = 0; l < m.lg.size(); ++l) {
    bool nxt = false;
    const bool has_next = cross && l + 1 < m.lg.size();
    if ((r = stage_fwd(m.lg[l], sv.lg[l], m.sc, c.ws, st, has_next ? &m.lg[l + 1] : nullptr,
                       has_next ? &sv.lg[l + 1] : nullptr, pre != 0, &nxt)))
      return r;
    pre = nxt;
  }
  const float* lg_out = m.lg.empty() ? lg_in : sv.lg.back().x.back();
  // ---- Dec_net.proj (transformer.py:600)
  GemmArgs dp = gemm_base(M1, G * C1, E, 1, EPI_STORE, m.sc);
  dp.g[0] = {lg_out, nullptr, w("dec.proj.weight"), w("dec.proj.bias"), m.dp, nullptr, nullptr};
  CK(gemm_nt(dp, st, -1, m.sc.ws));
  // concat_back_dim[0]: cat(x, skip1) (transformer.py:468-469)
  GemmArgs c0 = gemm_base(M1, C1, 2 * C1, G, EPI_STORE, m.sc);
  c0.lda = G * C1;
  c0.ksplit = C1;
  c0.lda2 = C1;
  for (int g = 0; g < G; ++g)
    c0.g[g] = {m.dp + g * C1, skip1 + g * M1C1, w(dg(g) + ".concat_back_dim.0.weight"),
               w(dg(g) + ".concat_back_dim.0.bias"), sv.dec1.x[0] + g * M1C1, nullptr, nullptr};
  CK(gemm_nt(c0, st, -1, m.sc.ws));
  if ((r = stage_fwd(m.dec1, sv.dec1, m.sc, c.ws, st))) return r;
  // PatchExpand: expand (no bias) + rearrange + LN(C0, eps 1e-6) (transformer.py:106-118)
  GemmArgs ex = gemm_base(M1, 2 * C1, C1, G, EPI_STORE, m.sc);
  for (int g = 0; g < G; ++g)
    ex.g[g] = {sv.dec1.x.back() + g * M1C1, nullptr, w(dg(g) + ".layers_up.0.upsample.expand.weight"), nullptr,
               sv.ex + (size_t)g * M1 * 2 * C1, nullptr, nullptr};
  CK(gemm_nt(ex, st, -1, m.sc.ws));
  LnArgs lx = ln_base(M0, C0, G, 1e-6f);
  lx.mode = LN_EXPAND;
  lx.Hin = c.H1;
  lx.Win = c.W1;
  lx.ldx = 2 * C1;
  for (int g = 0; g < G; ++g)
    lx.g[g] = {sv.ex + (size_t)g * M1 * 2 * C1, w(dg(g) + ".layers_up.0.upsample.norm.weight"),
               w(dg(g) + ".layers_up.0.upsample.norm.bias"), m.xe + g * M0C0, sv.st_ex + (size_t)g * M0 * 2, nullptr,
               nullptr};
  CK(layernorm_fwd(lx, st));
  // concat_back_dim[1]: cat(x, skip0)
  GemmArgs c1 = gemm_base(M0, C0, 2 * C0, G, EPI_STORE, m.sc);
  c1.lda = C0;
  c1.ksplit = C0;
  c1.lda2 = C0;
  for (int g = 0; g < G; ++g)
    c1.g[g] = {m.xe + g * M0C0, skip0 + g * M0C0, w(dg(g) + ".concat_back_dim.1.weight"),
               w(dg(g) + ".concat_back_dim.1.bias"), sv.dec0.x[0] + g * M0C0, nullptr, nullptr};
  CK(gemm_nt(c1, st, -1, m.sc.ws));
  if ((r = stage_fwd(m.dec0, sv.dec0, m.sc, c.ws, st))) return r;
  // norm_up (transformer.py:472)
  LnArgs lu = ln_base(M0, C0, G, 1e-6f);
  for (int g = 0; g < G; ++g)
    lu.g[g] = {sv.dec0.x.back() + g * M0C0, w(dg(g) + ".norm_up.weight"), w(dg(g) + ".norm_up.bias"),
               m.yn + g * M0C0, sv.st_nu + (size_t)g * M0 * 2, nullptr, nullptr};
  CK(layernorm_fwd(lu, st));
  // ConvTranspose2d + mean/std reorder (transformer.py:605-623, quirk Q2)
  PatchArgs pu;
  memset(&pu, 0, sizeof(pu));
  pu.B = B;
  pu.Himg = c.Himg;
  pu.Wimg = c.Wimg;
  pu.Cimg = c.Cout;
  pu.Ctok = C0;
  pu.climit = climit > 0 ? std::min(climit, c.Cout) : c.Cout;
  pu.img_out = out;
  pu.ngroups = G;
  pu.tune = m.sc.tune;
  int moff = 0, soff = 0;
  for (int g = 0; g < G; ++g) soff += c.raw.outchans[g] / 2;
  for (int g = 0; g < G; ++g) {
    const std::string f = "dec.final_proj_list." + std::to_string(g);
    pu.g[g].w = w(f + ".weight");
    pu.g[g].bias = w(f + ".bias");
    pu.g[g].tok = m.yn + g * M0C0;
    pu.g[g].cout = c.raw.outchans[g];
    pu.g[g].mean_off = moff;
    pu.g[g].std_off = soff;
    moff += c.raw.outchans[g] / 2;
    soff += c.raw.outchans[g] - c.raw.outchans[g] / 2;
  }
  CK(patch_unembed_fwd(pu, st));
  return 0;
}

int model_bwd(Model& m, int slot, const float* dout, float* din, const float* add, int climit, hipStream_t st) {
  const Cfg& c = m.cfg;
  Save& sv = m.saves[slot];
  const int G = c.G, B = m.B, C0 = c.C0, C1 = c.C1, E = c.E;
  const int M0 = B * c.H0 * c.W0, M1 = B * c.H1 * c.W1;
  const size_t M0C0 = (size_t)M0 * C0, M1C1 = (size_t)M1 * C1;
  auto w = [&](const std::string& n) { return m.W.at(n); };
  auto eg = [&](int g) { return "enc.enc_list." + std::to_string(g); };
  auto dg = [&](int g) { return "dec.dec_list." + std::to_string(g); };
  int r;
  // ConvTranspose2d backward
  PatchArgs pu;
  memset(&pu, 0, sizeof(pu));
  pu.B = B;
  pu.Himg = c.Himg;
  pu.Wimg = c.Wimg;
  pu.Cimg = c.Cout;
  pu.Ctok = C0;
  pu.climit = climit > 0 ? std::min(climit, c.Cout) : c.Cout;
  pu.img = dout;
  pu.ngroups = G;
  pu.tune = m.sc.tune;
  int moff = 0, soff = 0;
  for (int g = 0; g < G; ++g) soff += c.raw.outchans[g] / 2;
  for (int g = 0; g < G; ++g) {
    pu.g[g].w = w("dec.final_proj_list." + std::to_string(g) + ".weight");
    pu.g[g].tok = m.gy + g * M0C0;
    pu.g[g].cout = c.raw.outchans[g];
    pu.g[g].mean_off = moff;
    pu.g[g].std_off = soff;
    moff += c.raw.outchans[g] / 2;
    soff += c.raw.outchans[g] - c.raw.outchans[g] / 2;
  }
  CK(patch_unembed_bwd(pu, st));
  // norm_up backward
  LnArgs lu = ln_base(M0, C0, G, 1e-6f);
  for (int g = 0; g < G; ++g)
    lu.g[g] = {sv.dec0.x.back() + g * M0C0, w(dg(g) + ".norm_up.weight"), nullptr, m.gd0 + g * M0C0,
               sv.st_nu + (size_t)g * M0 * 2, m.gy + g * M0C0, nullptr};
  CK(layernorm_bwd(lu, st));
  if ((r = stage_bwd(m.dec0, sv.dec0, m.sc, c.ws, m.gd0, st))) return r;
  // concat_back_dim[1] backward: left -> PatchExpand output, right -> skip0
  for (int half = 0; half < 2; ++half) {
    GemmArgs cb = gemm_base(M0, C0, C0, G, EPI_STORE, m.sc);
    for (int g = 0; g < G; ++g)
      cb.g[g] = {m.gd0 + g * M0C0, nullptr, w(dg(g) + ".concat_back_dim.1.weight^T") + (size_t)half * C0 * C0,
                 nullptr, (half ? m.gsk0 : m.gxe) + g * M0C0, nullptr, nullptr};
    CK(gemm_nt(cb, st, -1, m.sc.ws));
  }
  // PatchExpand backward: LN (expand mode) then expand^T
  LnArgs lx = ln_base(M0, C0, G, 1e-6f);
  lx.mode = LN_EXPAND;
  lx.Hin = c.H1;
  lx.Win = c.W1;
  lx.ldx = lx.ldy = 2 * C1;
  for (int g = 0; g < G; ++g)
    lx.g[g] = {sv.ex + (size_t)g * M1 * 2 * C1, w(dg(g) + ".layers_up.0.upsample.norm.weight"), nullptr,
               m.gex + (size_t)g * M1 * 2 * C1, sv.st_ex + (size_t)g * M0 * 2, m.gxe + g * M0C0, nullptr};
  CK(layernorm_bwd(lx, st));
  GemmArgs ex = gemm_base(M1, C1, 2 * C1, G, EPI_STORE, m.sc);
  for (int g = 0; g < G; ++g)
    ex.g[g] = {m.gex + (size_t)g * M1 * 2 * C1, nullptr, w(dg(g) + ".layers_up.0.upsample.expand.weight^T"), nullptr,
               m.gd1 + g * M1C1, nullptr, nullptr};
  CK(gemm_nt(ex, st, -1, m.sc.ws));
  if ((r = stage_bwd(m.dec1, sv.dec1, m.sc, c.ws, m.gd1, st))) return r;
  // concat_back_dim[0] backward: left -> Dec_net.proj output slice g, right -> skip1
  for (int half = 0; half < 2; ++half) {
    GemmArgs cb = gemm_base(M1, C1, C1, G, EPI_STORE, m.sc);
    if (!half) cb.ldc = G * C1;
    for (int g = 0; g < G; ++g)
      cb.g[g] = {m.gd1 + g * M1C1, nullptr, w(dg(g) + ".concat_back_dim.0.weight^T") + (size_t)half * C1 * C1,
                 nullptr, half ? m.gsk1 + g * M1C1 : m.gdp + g * C1, nullptr, nullptr};
    CK(gemm_nt(cb, st, -1, m.sc.ws));
  }
  // Dec_net.proj backward
  float* glg = m.glg;
  GemmArgs dp = gemm_base(M1, E, G * C1, 1, EPI_STORE, m.sc);
  dp.g[0] = {m.gdp, nullptr, w("dec.proj.weight^T"), nullptr, glg, nullptr, nullptr};
  CK(gemm_nt(dp, st, -1, m.sc.ws));
  {
    const bool cross = (m.sc.tune ? *m.sc.tune : vv::kDefaultTuning).fixup_ln_cross;
    for (int l = (int)m.lg.size() - 1; l >= 0; --l)
      if ((r = stage_bwd(m.lg[l], sv.lg[l], m.sc, c.ws, glg, st, cross && l + 1 < (int)m.lg.size(), cross && l > 0)))
        return r;
  }
  // pos_embed: identity ; Enc_net.proj backward
  GemmArgs ep = gemm_base(M1, G * C1, E, 1, EPI_STORE, m.sc);
  ep.g[0] = {glg, nullptr, w("enc.proj.weight^T"), nullptr, m.gcat, nullptr, nullptr};
  CK(gemm_nt(ep, st, -1, m.sc.ws));
  // encoder norm backward (+ skip1 gradient), in place on gsk1
  float* skip1 = sv.enc1.x.back();
  LnArgs le = ln_base(M1, C1, G, 1e-6f);
  le.lddy = G * C1;
  for (int g = 0; g < G; ++g)
    le.g[g] = {skip1 + g * M1C1, w(eg(g) + ".norm.weight"), nullptr, m.gsk1 + g * M1C1, sv.st_en + (size_t)g * M1 * 2,
               m.gcat + g * C1, m.gsk1 + g * M1C1};
  CK(layernorm_bwd(le, st));
  if ((r = stage_bwd(m.enc1, sv.enc1, m.sc, c.ws, m.gsk1, st))) return r;
  // PatchMerging backward: reduction^T, then LN (merge mode) scattered onto level-0 tokens (+ skip0 grad)
  GemmArgs red = gemm_base(M1, 4 * C0, C1, G, EPI_STORE, m.sc);
  for (int g = 0; g < G; ++g)
    red.g[g] = {m.gsk1 + g * M1C1, nullptr, w(eg(g) + ".layers.1.downsample.reduction.weight^T"), nullptr,
                m.gxm + (size_t)g * M1 * 4 * C0, nullptr, nullptr};
  CK(gemm_nt(red, st, -1, m.sc.ws));
  float* skip0 = sv.enc0.x.back();
  LnArgs lm = ln_base(M1, 4 * C0, G, 1e-6f);
  lm.mode = LN_MERGE;
  lm.Hin = c.H0;
  lm.Win = c.W0;
  lm.ldx = lm.ldy = lm.ldres = C0;
  for (int g = 0; g < G; ++g)
    lm.g[g] = {skip0 + g * M0C0, w(eg(g) + ".layers.1.downsample.norm.weight"), nullptr, m.gsk0 + g * M0C0,
               sv.st_m + (size_t)g * M1 * 2, m.gxm + (size_t)g * M1 * 4 * C0, m.gsk0 + g * M0C0};
  CK(layernorm_bwd(lm, st));
  if ((r = stage_bwd(m.enc0, sv.enc0, m.sc, c.ws, m.gsk0, st))) return r;
  // PatchEmbed backward (+ add)
  PatchArgs pa;
  memset(&pa, 0, sizeof(pa));
  pa.B = B;
  pa.Himg = c.Himg;
  pa.Wimg = c.Wimg;
  pa.Cimg = c.Cin;
  pa.Ctok = C0;
  pa.img_out = din;
  pa.add_img = add;
  pa.ngroups = G;
  pa.tune = m.sc.tune;
  for (int g = 0, off = 0; g < G; off += c.raw.inchans[g], ++g) {
    pa.g[g].w = w(eg(g) + ".patch_embed.proj.weight");
    pa.g[g].dtok = m.gsk0 + g * M0C0;
    pa.g[g].cin_off = off;
    pa.g[g].cin = c.raw.inchans[g];
  }
  CK(patch_embed_bwd(pa, st));
  return 0;
}

// ----------------------------------------------------------------------------
// closure  (da_4dvar.py:1183-1208 loss(z) + backward)
// ----------------------------------------------------------------------------
// the observation term of time t under the real-observation operator (no-op for the identity operator):
// J partials of slot t and the state-space gradient GOBS[t] (da_4dvar.py:1196-1207)
hipError_t obs_term(const Problem& P, int b, int t, hipStream_t st) {
  if (!P.nout) return hipSuccess;
  const size_t HW = (size_t)P.Hs * P.Ws, OHW = P.obs_hw(), bt = (size_t)b * P.T + t;
  ObsArgs oa;
  oa.nin = P.nin;
  oa.nout = P.nout;
  oa.HW = (int)HW;
  oa.P = P.Pobs;
  oa.x = P.X + bt * P.C * HW;
  oa.yo = P.yo + bt * OHW;
  oa.Hm = P.Hm + bt * OHW;
  oa.R = P.R + bt * OHW;
  oa.coeff = P.obs_coeff;
  oa.g_obs = P.GOBS + bt * P.C * HW;
  oa.partial = P.partial + ((size_t)b * (P.T + 1) + t) * P.nblk;
  oa.nblk = P.nblk;
  return obs_misfit(oa, st);
}

void set_maps(const Problem& P, MisfitArgs& m) {
  m.Hl = P.Hl;
  m.Wl = P.Wl;
  m.mi = P.interp ? P.mi : nullptr;
  m.mj = P.interp ? P.mj : nullptr;
  m.ri0 = P.interp ? P.ri0 : nullptr;
  m.rj0 = P.interp ? P.rj0 : nullptr;
}

// the problem's index maps in one block of ints (offsets): mj and colinv 16-B aligned (k_misfit_grid reads them as
// int4), the rest packed
struct MapLayout {
  size_t mi, mj, ri0, rj0, di, dj, rowinv, colinv, cr0, cc0, n;
};
MapLayout map_layout(int Hs, int Ws, int Hl, int Wl) {
  auto al4 = [](size_t v) { return (v + 3) & ~(size_t)3; };
  MapLayout L;
  L.mi = 0;
  L.mj = al4(L.mi + Hs);
  L.ri0 = L.mj + Ws;
  L.rj0 = L.ri0 + Hl + 1;
  L.di = L.rj0 + Wl + 1;
  L.dj = L.di + Hl;
  L.rowinv = L.dj + Wl;
  L.colinv = al4(L.rowinv + Hs);
  L.cr0 = L.colinv + Ws;
  L.cc0 = L.cr0 + Hl + 1;
  L.n = al4(L.cc0 + Wl + 1);
  return L;
}

// B analyses per evaluation (the decoder's batch): one decoder launch sequence over all B, one flow launch
// sequence per forecast step; the misfit / adjoint kernels run per analysis (each has its own J partials).
// Layouts: X (B, T, C, Hs, Ws); decoder output / gradient (B, Cout, Hl, Wl); flow input FI[t] (B, C, Hl, Wl), flow
// output FO[t] (B, Fcout, Hl, Wl); carry (B, C, Hs, Ws); J partials [b][t + J_b][nblk]; dJ[b] = {J_b, J_o}.
int closure_impl(vv_ctx* ctx, const float* z, float* grad, hipStream_t st) {
  Problem& P = ctx->prob;
  if (!P.bound) return fail(VV_E_STATE, "vv_bind_problem first");
  Model& D = *ctx->models[P.dec];
  Model* F = P.flow >= 0 ? ctx->models[P.flow].get() : nullptr;
  const int C = P.C, HW = P.Hs * P.Ws, HWl = P.Hl * P.Wl, B = P.B, T = P.T;
  const size_t CHW = (size_t)C * HW, CHWl = (size_t)C * HWl, OHW = P.obs_hw();
  const size_t DO = (size_t)D.cfg.Cout * HWl, FO = F ? (size_t)F->cfg.Cout * HWl : 0;
  const size_t zper = (size_t)D.cfg.Cin * D.cfg.Himg * D.cfg.Wimg;
  auto part = [&](int b, int t) { return P.partial + ((size_t)b * (T + 1) + t) * P.nblk; };
  auto X = [&](int b, int t) { return P.X + ((size_t)b * T + t) * CHW; };
  auto FI = [&](int t, int b) { return P.FI + ((size_t)t * B + b) * CHWl; };
  // one pass over the state fields per slot (interpolated grids, synthetic observations): k_misfit_grid
  const bool gf = P.grid_fused && !P.nout;
  auto GON = [&](int b, int t) { return P.GON + ((size_t)b * T + t) * CHWl; };
  int r;
  // forward: x_0 = decoder(z)*stdTr*std + xb
  if ((r = model_fwd(D, 0, z, P.dec_out, C, st))) return r;
  MisfitArgs ma;
  memset(&ma, 0, sizeof(ma));
  ma.C = C;
  ma.Hs = P.Hs;
  ma.Ws = P.Ws;
  set_maps(P, ma);
  ma.scale = P.std_tr;
  ma.scale2 = P.std_;
  ma.mean = P.mean;
  ma.std_ = P.std_;
  ma.nblk = P.nblk;
  if (gf) {
    ma.rowinv = P.rowinv;
    ma.colinv = P.colinv;
    ma.coeff = P.obs_coeff;
    ma.mr = P.grid_mr;
  }
  for (int b = 0; b < B; ++b) {
    MisfitArgs m0 = ma;
    m0.net = P.dec_out + b * DO;
    m0.xb = P.xb + b * CHW;
    m0.yo = P.yo + (size_t)b * T * OHW;
    m0.Hm = P.nout ? nullptr : P.Hm + (size_t)b * T * OHW;  // J from the observation operator when set
    m0.R = P.R + (size_t)b * T * OHW;
    m0.x_out = X(b, 0);
    m0.flow_in = T > 1 ? FI(0, b) : nullptr;
    m0.partial = part(b, 0);
    if (gf) {
      m0.x_out = grad ? nullptr : X(b, 0);  // the state is kept for J-only (logging) evaluations only
      m0.g_net_obs = grad ? GON(b, 0) : nullptr;
      CK(misfit_grid_fwd(m0, st));
      continue;
    }
    CK(misfit_fwd(m0, st));
    CK(obs_term(P, b, 0, st));
    if (T > 1 && P.interp)
      CK(flow_input(X(b, 0), FI(0, b), P.di, P.dj, P.mean, P.std_, C, P.Hs, P.Ws, P.Hl, P.Wl, st));
  }
  for (int t = 1; t < T; ++t) {
    // x_t = integrate(x_{t-1}) = flow((x - mean)/std)[:C]*std + mean   (da_4dvar.py:666-681)
    float* fo = P.FO + (size_t)(t - 1) * B * FO;
    if ((r = model_fwd(*F, t - 1, FI(t - 1, 0), fo, C, st))) return r;
    for (int b = 0; b < B; ++b) {
      MisfitArgs mt = ma;
      mt.net = fo + b * FO;
      mt.scale = P.std_;
      mt.scale2 = nullptr;
      mt.offset = P.mean;
      mt.yo = P.yo + ((size_t)b * T + t) * OHW;
      mt.Hm = P.nout ? nullptr : P.Hm + ((size_t)b * T + t) * OHW;
      mt.R = P.R + ((size_t)b * T + t) * OHW;
      mt.x_out = X(b, t);
      mt.flow_in = t < T - 1 ? FI(t, b) : nullptr;
      mt.partial = part(b, t);
      if (gf) {
        mt.x_out = grad ? nullptr : X(b, t);
        mt.g_net_obs = grad ? GON(b, t) : nullptr;
        CK(misfit_grid_fwd(mt, st));
        continue;
      }
      CK(misfit_fwd(mt, st));
      CK(obs_term(P, b, t, st));
      if (t < T - 1 && P.interp)
        CK(flow_input(X(b, t), FI(t, b), P.di, P.dj, P.mean, P.std_, C, P.Hs, P.Ws, P.Hl, P.Wl, st));
    }
  }
  for (int b = 0; b < B; ++b) {
    CK(reduce_final(part(b, 0), P.nblk * T, P.dJ + 2 * b + 1, st));
    CK(reduce_sumsq(z + b * zper, (int64_t)zper, part(b, T), P.nblk, st));
    CK(reduce_final(part(b, T), P.nblk, P.dJ + 2 * b, st));
  }
  if (!grad) return 0;
  if (gf) {
    // backward on the network grid: g_net = (g_net_obs[t] + the flow-input adjoint of step t + 1) * scale
    MisfitNetBwdArgs nb;
    memset(&nb, 0, sizeof(nb));
    nb.C = C;
    nb.Hl = P.Hl;
    nb.Wl = P.Wl;
    nb.cr0 = P.cr0;
    nb.cc0 = P.cc0;
    nb.std_ = P.std_;
    for (int t = T - 1; t >= 0; --t) {
      for (int b = 0; b < B; ++b) {
        MisfitNetBwdArgs n = nb;
        n.g_net_obs = GON(b, t);
        n.gfi = t < T - 1 ? P.GFI + b * CHWl : nullptr;
        n.scale = t ? P.std_ : P.prod;
        n.g_net = t ? P.GFO + b * FO : P.gdec + b * DO;
        CK(misfit_net_bwd(n, st));
      }
      if (t && (r = model_bwd(*F, t - 1, P.GFO, P.GFI, nullptr, C, st))) return r;
    }
    return model_bwd(D, 0, P.gdec, grad, z, C, st);
  }
  // backward
  MisfitBwdArgs mb0;
  memset(&mb0, 0, sizeof(mb0));
  mb0.C = C;
  mb0.Hs = P.Hs;
  mb0.Ws = P.Ws;
  mb0.Hl = P.Hl;
  mb0.Wl = P.Wl;
  mb0.ri0 = P.interp ? P.ri0 : nullptr;
  mb0.rj0 = P.interp ? P.rj0 : nullptr;
  mb0.coeff = P.obs_coeff;
  bool carry = false;
  for (int t = T - 1; t >= 1; --t) {
    for (int b = 0; b < B; ++b) {
      MisfitBwdArgs mb = mb0;
      mb.x = X(b, t);
      mb.yo = P.yo + ((size_t)b * T + t) * OHW;
      mb.Hm = P.Hm + ((size_t)b * T + t) * OHW;
      mb.R = P.R + ((size_t)b * T + t) * OHW;
      mb.g_obs = P.nout ? P.GOBS + ((size_t)b * T + t) * CHW : nullptr;
      mb.g_carry = carry ? P.carry + b * CHW : nullptr;
      mb.scale = P.std_;
      mb.g_net = P.GFO + b * FO;
      mb.net_cstride = F->cfg.Cout;
      CK(misfit_bwd(mb, st));
    }
    if ((r = model_bwd(*F, t - 1, P.GFO, P.GFI, nullptr, C, st))) return r;
    for (int b = 0; b < B; ++b) {
      if (P.interp)
        CK(flow_input_adjoint(P.GFI + b * CHWl, P.carry + b * CHW, P.di, P.dj, P.std_, C, P.Hs, P.Ws, P.Hl, P.Wl, st));
      else
        CK(scale_channels(P.GFI + b * CHWl, P.carry + b * CHW, P.std_, C, HW, nullptr, st));
    }
    carry = true;
  }
  for (int b = 0; b < B; ++b) {
    MisfitBwdArgs mb = mb0;
    mb.x = X(b, 0);
    mb.yo = P.yo + (size_t)b * T * OHW;
    mb.Hm = P.Hm + (size_t)b * T * OHW;
    mb.R = P.R + (size_t)b * T * OHW;
    mb.g_obs = P.nout ? P.GOBS + (size_t)b * T * CHW : nullptr;
    mb.g_carry = carry ? P.carry + b * CHW : nullptr;
    mb.scale = P.prod;
    mb.g_net = P.gdec + b * DO;
    mb.net_cstride = D.cfg.Cout;
    CK(misfit_bwd(mb, st));
  }
  // grad_z = z + decoder^T(g)   (d/dz of sum(z^2)/2 is z)
  if ((r = model_bwd(D, 0, P.gdec, grad, z, C, st))) return r;
  return 0;
}

// sc4dvar loss(w) (da_4dvar.py:1099-1101) and, with grad, its gradient: J_b = sum(w^2)/2, J_o = sum_t H (x_t - yo_t)^2
// / R / 2 (x_aug of the real-observation operator when set, :1085-1097); dJ/dw = w + obs_coeff * core^T(adjoint of
// the nearest interpolation of H (x_0 - yo_0) / R) — the detached forecasts contribute no gradient
int sc4_closure_impl(vv_ctx* ctx, const float* w, float* grad, hipStream_t st) {
  Sc4Problem& P = *ctx->sc4;
  const int C = P.C, T = P.T;
  const size_t HW = (size_t)P.Hs * P.Ws, CHW = (size_t)C * HW, OHW = P.obs_hw();
  auto part = [&](int t) { return P.partial + (size_t)t * P.nblk; };
  auto X = [&](int t) { return P.X + (size_t)t * CHW; };
  Model* F = P.flow >= 0 ? ctx->models[P.flow].get() : nullptr;
  CK(vv::sc4dvar_fwd(P.bm, w, P.recon, P.t1, P.t2, ctx->gemm_ws, st));
  MisfitArgs ma;
  memset(&ma, 0, sizeof(ma));
  ma.C = C;
  ma.Hs = P.Hs;
  ma.Ws = P.Ws;
  ma.Hl = P.Hl;
  ma.Wl = P.Wl;
  ma.mi = P.interp ? P.mi : nullptr;
  ma.mj = P.interp ? P.mj : nullptr;
  ma.mean = P.mean;
  ma.std_ = P.std_;
  ma.nblk = P.nblk;
  auto obs = [&](int t) -> hipError_t {  // real-observation operator: J partials + (t = 0) the state gradient
    if (!P.nout) return hipSuccess;
    ObsArgs oa;
    oa.nin = P.nin;
    oa.nout = P.nout;
    oa.HW = (int)HW;
    oa.P = P.Pobs;
    oa.x = X(t);
    oa.yo = P.yo + t * OHW;
    oa.Hm = P.Hm + t * OHW;
    oa.R = P.R + t * OHW;
    oa.coeff = P.obs_coeff;
    oa.g_obs = t == 0 ? P.GOBS : P.GOBS + CHW;  // the gradient of t = 0 is kept; later times: scratch
    oa.partial = part(t);
    oa.nblk = P.nblk;
    return obs_misfit(oa, st);
  };
  // x_0 = interpolate(recon) + xb   (:928)
  {
    MisfitArgs m0 = ma;
    m0.net = P.recon;
    m0.net_cstride = C;
    m0.scale = P.ones;
    m0.xb = P.xb;
    m0.yo = P.yo;
    m0.Hm = P.nout ? nullptr : P.Hm;
    m0.R = P.R;
    m0.x_out = X(0);
    m0.flow_in = (T > 1 && !P.interp) ? P.FI : nullptr;
    m0.partial = part(0);
    CK(misfit_fwd(m0, st));
    CK(obs(0));
  }
  for (int t = 1; t < T; ++t) {
    // x_t = integrate(x_{t-1}, flow, 1, True)[:69]   (:1079-1081, detached)
    if (P.interp) CK(flow_input(X(t - 1), P.FI, P.di, P.dj, P.mean, P.std_, C, P.Hs, P.Ws, P.Hl, P.Wl, st));
    int r = model_fwd(*F, 0, P.FI, P.FO, C, st);
    if (r) return r;
    MisfitArgs mt = ma;
    mt.net = P.FO;
    mt.net_cstride = F->cfg.Cout;
    mt.scale = P.std_;
    mt.offset = P.mean;
    mt.yo = P.yo + t * OHW;
    mt.Hm = P.nout ? nullptr : P.Hm + t * OHW;
    mt.R = P.R + t * OHW;
    mt.x_out = X(t);
    mt.flow_in = (t < T - 1 && !P.interp) ? P.FI : nullptr;
    mt.partial = part(t);
    CK(misfit_fwd(mt, st));
    CK(obs(t));
  }
  CK(reduce_final(part(0), P.nblk * T, P.dJ + 1, st));
  CK(reduce_sumsq(w, (int64_t)P.wn, part(T), P.nblk, st));
  CK(reduce_final(part(T), P.nblk, P.dJ, st));
  if (!grad) return 0;
  MisfitBwdArgs mb;
  memset(&mb, 0, sizeof(mb));
  mb.C = C;
  mb.Hs = P.Hs;
  mb.Ws = P.Ws;
  mb.Hl = P.Hl;
  mb.Wl = P.Wl;
  mb.ri0 = P.interp ? P.ri0 : nullptr;
  mb.rj0 = P.interp ? P.rj0 : nullptr;
  mb.coeff = P.obs_coeff;
  mb.x = X(0);
  mb.yo = P.yo;
  mb.Hm = P.Hm;
  mb.R = P.R;
  mb.g_obs = P.nout ? P.GOBS : nullptr;
  mb.scale = P.ones;
  mb.g_net = P.grec;
  mb.net_cstride = C;
  CK(misfit_bwd(mb, st));
  CK(vv::sc4dvar_adj(P.bm, P.grec, w, grad, P.t1, P.t2, ctx->gemm_ws, st));
  return 0;
}

__global__ void k_prod(const float* a, const float* b, float* o, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) o[i] = a[i] * b[i];
}
__global__ void k_half(double* d, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) d[i] *= 0.5;
}

}  // namespace

namespace {
int closure_enqueue(vv_ctx* ctx, const float* z, float* grad_z, double* d_J, hipStream_t st) {
  int r;
  if ((r = closure_impl(ctx, z, grad_z, st))) return r;
  hipLaunchKernelGGL(k_half, dim3(1), dim3(64), 0, st, ctx->prob.dJ, 2 * ctx->prob.B);
  VV_HIP(hipGetLastError());
  if (d_J) VV_HIP(hipMemcpyAsync(d_J, ctx->prob.dJ, 2 * ctx->prob.B * sizeof(double), hipMemcpyDeviceToDevice, st));
  return 0;
}


void drop_graphs(vv_ctx* ctx) {
  for (auto& g : ctx->graphs) {
    if (g.exec) (void)hipGraphExecDestroy(g.exec);
    g = vv_ctx::ClosureGraph{};
  }
}

// the closure through its cached graph: z -> Problem::Z, replay (J and, with grad_z, Problem::GZ), GZ -> grad_z
int closure_graphed(vv_ctx* ctx, const float* z, float* grad_z, double* d_J, hipStream_t st) {
  Problem& P = ctx->prob;
  auto& g = ctx->graphs[grad_z ? 1 : 0];
  float* gz = grad_z ? P.GZ : nullptr;
  VV_HIP(hipMemcpyAsync(P.Z, z, P.zn * sizeof(float), hipMemcpyDeviceToDevice, st));
  if (g.eager_only || (!g.exec && g.eager_runs == 0)) {
    // the first evaluation of each kind runs eagerly (it also performs the one-time kernel attribute set-up)
    g.eager_runs = 1;
    int r = closure_enqueue(ctx, P.Z, gz, nullptr, st);
    if (r) return r;
  } else {
    if (!g.exec) {
      if (!ctx->cap_stream) VV_HIP(hipStreamCreateWithFlags(&ctx->cap_stream, hipStreamNonBlocking));
      hipError_t ec = hipStreamBeginCapture(ctx->cap_stream, hipStreamCaptureModeRelaxed);
      int r = 0;
      hipGraph_t graph = nullptr;
      if (ec == hipSuccess) {
        r = closure_enqueue(ctx, P.Z, gz, nullptr, ctx->cap_stream);
        ec = hipStreamEndCapture(ctx->cap_stream, &graph);
      }
      hipError_t ei = hipSuccess;
      if (!r && ec == hipSuccess) ei = hipGraphInstantiate(&g.exec, graph, nullptr, nullptr, 0);
      if (graph) (void)hipGraphDestroy(graph);
      if (r || ec != hipSuccess || ei != hipSuccess) {
        // one failed capture must not disable the closure: record the error once, run this kind eagerly from now
        // on (nothing of the failed capture executed, so this evaluation is complete after the eager run)
        g.exec = nullptr;
        g.eager_only = true;
        (void)hipGetLastError();
        (void)fail(r ? r : (int)(ec != hipSuccess ? ec : ei), "closure graph capture failed (%s); eager launches",
                   hipGetErrorString(ec != hipSuccess ? ec : ei));
        const int r2 = closure_enqueue(ctx, P.Z, gz, nullptr, st);
        if (r2) return r2;
      }
    }
    if (g.exec) {
      VV_HIP(hipGraphLaunch(g.exec, st));
      ++g.launches;
    }
  }
  if (grad_z) VV_HIP(hipMemcpyAsync(grad_z, P.GZ, P.zn * sizeof(float), hipMemcpyDeviceToDevice, st));
  if (d_J) VV_HIP(hipMemcpyAsync(d_J, P.dJ, 2 * P.B * sizeof(double), hipMemcpyDeviceToDevice, st));
  return 0;
}

}  // namespace

// ============================================================================
// C ABI
// ============================================================================
extern "C" {

int vv_version(void) { return 100; }

int vv_last_error(char* buf, int cap) {
  if (!buf || cap <= 0) return VV_E_ARG;
  snprintf(buf, cap, "%s", g_err.c_str());
  return 0;
}

int vv_lgunet_param_count(const vv_lgunet_config* cfg, int* count) {
  if (cfg && cfg->arch == VV_ARCH_LGUNET1) {
    std::vector<vvf::ParamInfo> v;
    std::string err;
    const int r = vvf::params(cfg, v, err);
    if (r) return fail(r, "%s", err.c_str());
    *count = (int)v.size();
    return 0;
  }
  Cfg c;
  int r = parse_cfg(cfg, c);
  if (r) return r;
  *count = (int)enumerate_params(c).size();
  return 0;
}

int vv_lgunet_param_info(const vv_lgunet_config* cfg, int index, char* name, int name_cap, int64_t* shape,
                         int* ndim) {
  if (cfg && cfg->arch == VV_ARCH_LGUNET1) {
    std::vector<vvf::ParamInfo> v;
    std::string err;
    const int r = vvf::params(cfg, v, err);
    if (r) return fail(r, "%s", err.c_str());
    if (index < 0 || index >= (int)v.size()) return fail(VV_E_ARG, "param index %d out of range", index);
    if (name) snprintf(name, name_cap, "%s", v[index].name.c_str());
    if (ndim) *ndim = (int)v[index].shape.size();
    if (shape)
      for (size_t i = 0; i < v[index].shape.size(); ++i) shape[i] = v[index].shape[i];
    return 0;
  }
  Cfg c;
  int r = parse_cfg(cfg, c);
  if (r) return r;
  auto v = enumerate_params(c);
  if (index < 0 || index >= (int)v.size()) return fail(VV_E_ARG, "param index %d out of range", index);
  if (name) snprintf(name, name_cap, "%s", v[index].name.c_str());
  if (ndim) *ndim = (int)v[index].shape.size();
  if (shape)
    for (size_t i = 0; i < v[index].shape.size(); ++i) shape[i] = v[index].shape[i];
  return 0;
}

// the context's fixed device buffers; on failure the caller destroys the partly built context (nothing leaks)
static int ctx_alloc(vv_ctx* c) {
  VV_HIP(hipSetDevice(c->device));
  VV_HIP(hipMalloc(&c->red, 2 * kRedBlocks * sizeof(double)));  // two halves: lbfgs_two_loop alternates
  VV_HIP(hipMalloc(&c->redf, kRedBlocks * sizeof(float)));
  VV_HIP(hipMalloc(&c->twoloop, kMaxHistory * sizeof(float)));
  VV_HIP(hipMalloc(&c->dout, 4 * sizeof(double)));
  VV_HIP(hipMalloc(&c->doutf, 4 * sizeof(float)));
  VV_HIP(hipMalloc(&c->redb, (size_t)kMaxBatch * kRedBlocks * sizeof(double)));
  VV_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->hredb), (size_t)(kMaxBatch + kMaxExtra) * sizeof(double),
                       hipHostMallocMapped | hipHostMallocCoherent));
  VV_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&c->hredb_dev), c->hredb, 0));
  VV_HIP(hipMalloc(&c->gemm_ws, vv::gemm_ws_floats() * sizeof(float)));
  return 0;
}

int vv_ctx_create(int device, vv_ctx** out) {
  if (!out) return fail(VV_E_ARG, "null out");
  int n = 0;
  VV_HIP(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) return fail(VV_E_ARG, "device %d of %d", device, n);
  auto* c = new vv_ctx();
  c->device = device;
  if (const int r = ctx_alloc(c)) {
    (void)vv_ctx_destroy(c);
    return r;
  }
  *out = c;
  return 0;
}

int vv_ctx_destroy(vv_ctx* ctx) {
  if (!ctx) return 0;
  (void)hipSetDevice(ctx->device);
  (void)hipDeviceSynchronize();
  for (auto& m : ctx->models) {
    if (!m) continue;  // vv_model_destroy'ed
    for (int* p : m->maps_owned) (void)hipFree(p);
    if (m->warena) vv::unregister_split_arena(reinterpret_cast<const float*>(m->warena->base));
  }
  for (auto& w : ctx->split_owned) {
    vv::unregister_split_arena(w.base);
    (void)hipFree(w.planes);
  }

  drop_graphs(ctx);
  if (ctx->cap_stream) (void)hipStreamDestroy(ctx->cap_stream);
  (void)hipFree(ctx->red);
  (void)hipFree(ctx->twoloop);
  if (ctx->metric_ws) (void)hipFree(ctx->metric_ws);
  (void)hipFree(ctx->redf);
  (void)hipFree(ctx->dout);
  (void)hipFree(ctx->doutf);
  (void)hipFree(ctx->redb);
  if (ctx->hredb) (void)hipHostFree(ctx->hredb);
  (void)hipFree(ctx->gemm_ws);
  if (ctx->apl) (void)hipFree(ctx->apl);
  if (ctx->gattn_ws) (void)hipFree(ctx->gattn_ws);
  delete ctx;
  return 0;
}

int vv_model_create(vv_ctx* ctx, const vv_lgunet_config* cfg, int batch, int n_slots, int* model_id) {
  if (!ctx || !model_id || !cfg) return fail(VV_E_ARG, "null argument");
  int r = set_dev(ctx);
  if (r) return r;
  if (cfg->arch == VV_ARCH_LGUNET1) {
    auto m = std::make_unique<Model>();
    std::string err;
    if ((r = vvf::create(cfg, batch, &m->fm, err))) return fail(r, "%s", err.c_str());
    vvf::set_math(m->fm, ctx->math);
    vvf::set_tuning(m->fm, &ctx->tune);
    m->B = batch;
    m->nslots = 1;
    m->workspace = vvf::workspace_bytes(m->fm);
    m->cfg.raw = *cfg;
    m->cfg.Cin = vvf::in_channels(m->fm);
    m->cfg.Cout = vvf::out_channels(m->fm);
    m->cfg.Himg = vvf::img_h(m->fm);
    m->cfg.Wimg = vvf::img_w(m->fm);
    ctx->models.push_back(std::move(m));
    *model_id = (int)ctx->models.size() - 1;
    return 0;
  }
  if (cfg->arch != VV_ARCH_LGUNET) return fail(VV_E_ARG, "unknown arch %d", cfg->arch);
  if ((r = create_model(ctx, cfg, batch, n_slots, model_id))) return r;
  ctx->models[*model_id]->sc.math = ctx->math;
  ctx->models[*model_id]->sc.tune = &ctx->tune;
  return 0;
}

int vv_load_weights(vv_ctx* ctx, int model_id, const void* const* ptrs, int n) {
  Model* m = get_model(ctx, model_id);
  if (!m || !ptrs) return fail(VV_E_ARG, "bad model or ptrs");
  drop_graphs(ctx);
  if (m->fm) {
    int r = set_dev(ctx);
    if (r) return r;
    std::string err;
    if ((r = vvf::load(m->fm, ptrs, n, err))) return fail(r, "%s", err.c_str());
    m->loaded = true;
    return 0;
  }
  if (n != (int)m->params.size()) return fail(VV_E_ARG, "expected %zu params, got %d", m->params.size(), n);
  int r = set_dev(ctx);
  if (r) return r;
  for (int i = 0; i < n; ++i) {
    if (!ptrs[i]) return fail(VV_E_ARG, "null pointer for param %s", m->params[i].name.c_str());
    VV_HIP(hipMemcpy(m->pptr[i], ptrs[i], numel(m->params[i].shape) * 4, hipMemcpyDefault));
  }
  for (auto& p : m->params) {
    auto it = m->W.find(p.name + "^T");
    if (it == m->W.end()) continue;
    VV_HIP(vv::transpose2d(m->W[p.name], const_cast<float*>(it->second), (int)p.shape[0], (int)p.shape[1], 0));
  }
  // max |param| of the tensors whose maxima bound a plane-writing GEMM epilogue (BlockW.fc1Wmax, ...)
  auto ends = [](const std::string& n, const char* suf) {
    const size_t l = strlen(suf);
    return n.size() >= l && n.compare(n.size() - l, l, suf) == 0;
  };
  for (size_t i = 0; i < m->params.size(); ++i) {
    const std::string& nm = m->params[i].name;
    if (ends(nm, ".mlp.fc1.weight") || ends(nm, ".mlp.fc1.bias") || ends(nm, ".mlp.fc2.weight") ||
        ends(nm, ".attn.qkv.weight") || ends(nm, ".attn.qkv.bias"))
      VV_HIP(vv::absmax(m->pptr[i], numel(m->params[i].shape), const_cast<float*>(m->Wmax[nm]), 0));
  }
  // split planes (bf16 and fp16) of every GEMM weight and its transpose (GEMM_SPLIT / GEMM_SPLIT16 B operands)
  for (auto& p : m->params) {
    auto it = m->W.find(p.name + "^T");
    if (it == m->W.end()) continue;
    const size_t n = numel(p.shape);
    VV_HIP(vv::split_registered(m->W[p.name], n, (int)p.shape[1], 0));
    VV_HIP(vv::split_registered(it->second, n, (int)p.shape[0], 0));
  }
  VV_HIP(hipDeviceSynchronize());
  m->loaded = true;
  return 0;
}

int vv_model_destroy(vv_ctx* ctx, int model_id) {
  Model* m = get_model(ctx, model_id);
  if (!m) return fail(VV_E_ARG, "bad model id %d", model_id);
  int r = set_dev(ctx);
  if (r) return r;
  VV_HIP(hipDeviceSynchronize());  // no launch in flight reads its memory
  drop_graphs(ctx);
  if (ctx->prob.bound && (ctx->prob.dec == model_id || ctx->prob.flow == model_id)) ctx->prob = Problem();
  if (ctx->sc4 && ctx->sc4->flow == model_id) ctx->sc4.reset();
  for (int* p : m->maps_owned) (void)hipFree(p);
  if (m->warena) vv::unregister_split_arena(reinterpret_cast<const float*>(m->warena->base));
  ctx->models[model_id].reset();
  return 0;
}

int vv_model_workspace_bytes(vv_ctx* ctx, int model_id, int64_t* bytes) {
  Model* m = get_model(ctx, model_id);
  if (!m || !bytes) return fail(VV_E_ARG, "bad model");
  *bytes = m->workspace;
  return 0;
}

int vv_model_forward(vv_ctx* ctx, int model_id, int slot, const float* in, float* out, int out_limit, void* stream) {
  Model* m = get_model(ctx, model_id);
  if (!m || !in || !out) return fail(VV_E_ARG, "bad model or pointers");
  if (!m->loaded) return fail(VV_E_STATE, "weights not loaded");
  if (slot < 0 || slot >= m->nslots) return fail(VV_E_ARG, "slot %d out of range", slot);
  int r = set_dev(ctx);
  if (r) return r;
  if (m->fm) {
    std::string err;
    if ((r = vvf::forward(m->fm, in, out, out_limit, (hipStream_t)stream, err))) return fail(r, "%s", err.c_str());
    return 0;
  }
  return model_fwd(*m, slot, in, out, out_limit, (hipStream_t)stream);
}

int vv_model_backward(vv_ctx* ctx, int model_id, int slot, const float* dout, float* din, const float* add,
                      int out_limit, void* stream) {
  Model* m = get_model(ctx, model_id);
  if (!m || !dout || !din) return fail(VV_E_ARG, "bad model or pointers");
  if (m->fm) return fail(VV_E_STATE, "LGUnet_all_1 (forecast model) is forward-only");
  if (!m->loaded) return fail(VV_E_STATE, "weights not loaded");
  if (slot < 0 || slot >= m->nslots) return fail(VV_E_ARG, "slot %d out of range", slot);
  int r = set_dev(ctx);
  if (r) return r;
  return model_bwd(*m, slot, dout, din, add, out_limit, (hipStream_t)stream);
}

int vv_bind_problem(vv_ctx* ctx, int dec_model_id, int flow_model_id, int T, int C, int Hs, int Ws, const float* xb,
                    const float* yo, const float* Hmask, const float* R, const float* mean, const float* std_,
                    const float* std_tr, float obs_coeff) {
  Model* D = get_model(ctx, dec_model_id);
  if (!D) return fail(VV_E_ARG, "bad decoder model");
  if (D->fm || (flow_model_id >= 0 && get_model(ctx, flow_model_id) && get_model(ctx, flow_model_id)->fm))
    return fail(VV_E_ARG, "the closure needs differentiable networks_old LGUnet_all models");
  if (T < 1 || C < 1) return fail(VV_E_ARG, "bad T/C");

  if (D->cfg.Cout < C) return fail(VV_E_ARG, "decoder produces %d channels < C=%d", D->cfg.Cout, C);
  if (Hs < D->cfg.Himg || Ws < D->cfg.Wimg)
    return fail(VV_E_ARG, "state grid %dx%d coarser than the network grid %dx%d", Hs, Ws, D->cfg.Himg, D->cfg.Wimg);
  Model* F = nullptr;
  if (T > 1) {
    F = get_model(ctx, flow_model_id);
    if (!F) return fail(VV_E_ARG, "T > 1 needs a flow model");
    if (F->cfg.Cin != C || F->cfg.Cout < C || F->nslots < T - 1 || F->B != D->B)
      return fail(VV_E_ARG, "flow model shape/slots/batch incompatible (Cin %d Cout %d slots %d batch %d vs %d)",
                  F->cfg.Cin, F->cfg.Cout, F->nslots, F->B, D->B);
    if (F->cfg.Himg != D->cfg.Himg || F->cfg.Wimg != D->cfg.Wimg) return fail(VV_E_ARG, "flow grid mismatch");
  }
  if (!xb || !yo || !Hmask || !R || !mean || !std_ || !std_tr) return fail(VV_E_ARG, "null problem buffer");
  int r = set_dev(ctx);
  if (r) return r;
  drop_graphs(ctx);
  Problem& P = ctx->prob;
  P = Problem();
  P.dec = dec_model_id;
  P.flow = T > 1 ? flow_model_id : -1;
  P.B = D->B;
  P.T = T;
  P.C = C;
  P.Hs = Hs;
  P.Ws = Ws;
  P.xb = xb;
  P.yo = yo;
  P.Hm = Hmask;
  P.R = R;
  P.mean = mean;
  P.std_ = std_;
  P.std_tr = std_tr;
  P.obs_coeff = obs_coeff;
  P.Hl = D->cfg.Himg;
  P.Wl = D->cfg.Wimg;
  P.interp = (Hs != P.Hl || Ws != P.Wl);
  {
    bool aligned = true;
    for (const void* p : {(const void*)xb, (const void*)yo, (const void*)Hmask, (const void*)R})
      aligned = aligned && !(reinterpret_cast<uintptr_t>(p) & 15);
    // misfit_grid_fwd's preconditions (vv_ops.hip), so a bound grid_fused problem never fails a closure there
    P.grid_fused = P.interp && ctx->tune.grid_fused && Hs >= P.Hl && Ws >= P.Wl && Ws % 4 == 0 && Ws <= 16384 &&
                   P.Wl <= 768 && aligned;
    if (P.grid_fused) P.nblk = C * P.Hl;  // one J partial per (channel, network row) workgroup of k_misfit_grid
    P.grid_mr = ctx->tune.grid_fused == 2 ? 6 : 3;
  }
  const size_t CHW = (size_t)C * Hs * Ws;
  const size_t HWl = (size_t)P.Hl * P.Wl;
  const size_t CHWl = (size_t)C * HWl;
  const int fcout = F ? F->cfg.Cout : 0;
  const size_t B = (size_t)P.B;
  for (int pass = 0; pass < 2; ++pass) {
    Planner pl;
    if (pass) pl.base = P.arena->base;
    P.X = pl.f(B * CHW * T);
    P.dec_out = pl.f(B * D->cfg.Cout * HWl);
    P.gdec = pl.f(B * D->cfg.Cout * HWl);
    P.prod = pl.f(C);
    P.FI = pl.f(B * CHWl * std::max(T - 1, 1));
    P.FO = pl.f(B * fcout * HWl * std::max(T - 1, 1) + 1);
    P.GFO = pl.f(B * fcout * HWl + 1);
    P.GFI = pl.f(B * CHWl);
    // the per-element backward's flow-input adjoint (T > 1). Kept even when grid_fused is chosen: a later
    // vv_set_obs_operator switches the closure to the per-element path (closure_impl: gf needs nout == 0)
    P.carry = pl.f(T > 1 ? B * CHW : 1);
    P.GON = P.grid_fused ? pl.f(B * CHWl * T) : nullptr;
    P.zn = B * D->cfg.Cin * D->cfg.Himg * D->cfg.Wimg;
    P.Z = pl.f(P.zn);
    P.GZ = pl.f(P.zn);
    float* maps = pl.f(map_layout(Hs, Ws, P.Hl, P.Wl).n);
    double* pd = reinterpret_cast<double*>(pl.f(2 * (B * P.nblk * (T + 1) + 2 * B + 8)));
    if (pass) {
      P.partial = pd;
      P.dJ = pd + B * P.nblk * (T + 1) + 2;
      int* mp = reinterpret_cast<int*>(maps);
      const MapLayout L = map_layout(Hs, Ws, P.Hl, P.Wl);
      P.mi = mp + L.mi;
      P.mj = mp + L.mj;
      P.ri0 = mp + L.ri0;
      P.rj0 = mp + L.rj0;
      P.di = mp + L.di;
      P.dj = mp + L.dj;
      P.rowinv = mp + L.rowinv;
      P.colinv = mp + L.colinv;
      P.cr0 = mp + L.cr0;
      P.cc0 = mp + L.cc0;
    }
    if (!pass) {
      P.arena = std::make_unique<Arena>();
      if (hipMalloc(&P.arena->base, pl.bytes) != hipSuccess) return fail(VV_E_ALLOC, "problem arena");
      P.arena->cap = pl.bytes;
    }
  }
  {
    // nearest maps (F.interpolate mode='nearest', quirk Q3) and the adjoint row/col ranges
    std::vector<int> mi = nearest_map(P.Hl, Hs), mj = nearest_map(P.Wl, Ws);
    std::vector<int> di = nearest_map(Hs, P.Hl), dj = nearest_map(Ws, P.Wl);
    auto ranges = [](const std::vector<int>& m, int n) {
      std::vector<int> r(n + 1, (int)m.size());
      for (int k = (int)m.size() - 1; k >= 0; --k) r[m[k]] = k;
      for (int a = n - 1; a >= 0; --a) r[a] = std::min(r[a], r[a + 1]);
      return r;
    };
    for (size_t k = 1; k < mi.size(); ++k)
      if (mi[k] < mi[k - 1]) return fail(VV_E_ARG, "non-monotone nearest map");
    std::vector<int> ri0 = ranges(mi, P.Hl), rj0 = ranges(mj, P.Wl);
    // grid_fused: the inverse of the (injective, Hs >= Hl) down-sampling maps, and for each network pixel the
    // network pixels whose down-sampled source up-samples back onto it (mi[di[.]], mj[dj[.]] are monotone)
    std::vector<int> rowinv(Hs, -1), colinv(Ws, -1), ci(P.Hl), cj(P.Wl);
    for (int a = 0; a < P.Hl; ++a) {
      rowinv[di[a]] = a;
      ci[a] = mi[di[a]];
    }
    for (int b = 0; b < P.Wl; ++b) {
      colinv[dj[b]] = b;
      cj[b] = mj[dj[b]];
    }
    std::vector<int> cr0 = ranges(ci, P.Hl), cc0 = ranges(cj, P.Wl);
    const MapLayout L = map_layout(Hs, Ws, P.Hl, P.Wl);
    std::vector<int> all(L.n, 0);
    const std::pair<const std::vector<int>*, size_t> parts[] = {
        {&mi, L.mi}, {&mj, L.mj}, {&ri0, L.ri0}, {&rj0, L.rj0}, {&di, L.di}, {&dj, L.dj},
        {&rowinv, L.rowinv}, {&colinv, L.colinv}, {&cr0, L.cr0}, {&cc0, L.cc0}};
    for (const auto& pv : parts) std::copy(pv.first->begin(), pv.first->end(), all.begin() + pv.second);
    VV_HIP(hipMemcpy(P.mi - L.mi, all.data(), all.size() * sizeof(int), hipMemcpyHostToDevice));
  }
  hipLaunchKernelGGL(k_prod, dim3((C + 255) / 256), dim3(256), 0, 0, std_tr, std_, P.prod, C);
  VV_HIP(hipGetLastError());
  VV_HIP(hipDeviceSynchronize());
  P.bound = true;
  return 0;
}

int vv_closure_async(vv_ctx* ctx, const float* z, float* grad_z, double* d_J, void* stream) {
  if (!ctx || !z) return fail(VV_E_ARG, "null argument");
  int r = set_dev(ctx);
  if (r) return r;
  if (!ctx->prob.bound) return fail(VV_E_STATE, "vv_bind_problem first");
  hipStream_t st = (hipStream_t)stream;
  if (!ctx->use_graphs || vv::prof_enabled() || sync_check()) return closure_enqueue(ctx, z, grad_z, d_J, st);
  return closure_graphed(ctx, z, grad_z, d_J, st);
}

int vv_closure(vv_ctx* ctx, const float* z, float* grad_z, double* J_b, double* J_o, void* stream) {
  int r = vv_closure_async(ctx, z, grad_z, nullptr, stream);
  if (r) return r;
  const int B = ctx->prob.B;
  std::vector<double> h(2 * B);
  hipStream_t st = (hipStream_t)stream;
  VV_HIP(hipMemcpyAsync(h.data(), ctx->prob.dJ, h.size() * sizeof(double), hipMemcpyDeviceToHost, st));
  VV_HIP(hipStreamSynchronize(st));
  for (int b = 0; b < B; ++b) {
    if (J_b) J_b[b] = h[2 * b];
    if (J_o) J_o[b] = h[2 * b + 1];
  }
  return 0;
}

int vv_decode(vv_ctx* ctx, const float* z, float* xa, void* stream) {
  if (!ctx || !z || !xa) return fail(VV_E_ARG, "null argument");
  Problem& P = ctx->prob;
  if (!P.bound) return fail(VV_E_STATE, "vv_bind_problem first");
  int r = set_dev(ctx);
  if (r) return r;
  hipStream_t st = (hipStream_t)stream;
  Model& D = *ctx->models[P.dec];
  if ((r = model_fwd(D, 0, z, P.dec_out, P.C, st))) return r;
  MisfitArgs ma;
  memset(&ma, 0, sizeof(ma));
  ma.C = P.C;
  ma.Hs = P.Hs;
  ma.Ws = P.Ws;
  set_maps(P, ma);
  ma.scale = P.std_tr;
  ma.scale2 = P.std_;
  ma.yo = P.yo;
  ma.R = P.R;
  ma.Hm = nullptr;  // the analysis only: no misfit
  ma.partial = P.partial;
  ma.nblk = P.nblk;
  const size_t CHW = (size_t)P.C * P.Hs * P.Ws;
  for (int b = 0; b < P.B; ++b) {
    ma.net = P.dec_out + (size_t)b * D.cfg.Cout * P.Hl * P.Wl;
    ma.xb = P.xb + b * CHW;
    ma.x_out = xa + b * CHW;
    CK(misfit_fwd(ma, st));
  }
  return 0;
}

int vv_set_obs_operator(vv_ctx* ctx, int n_out, int n_in, const float* interp) {
  if (!ctx) return fail(VV_E_ARG, "null context");
  Problem& P = ctx->prob;
  if (!P.bound) return fail(VV_E_STATE, "vv_bind_problem first");
  int r = set_dev(ctx);
  if (r) return r;
  drop_graphs(ctx);
  if (n_out == 0) {
    P.nout = P.nin = 0;
    return 0;
  }
  if (!interp) return fail(VV_E_ARG, "null interp");
  if (n_in < 1 || n_in > vv::kObsMaxIn || n_out < 1 || n_out > vv::kObsMaxOut)
    return fail(VV_E_ARG, "operator %dx%d outside 1..%d x 1..%d", n_out, n_in, vv::kObsMaxOut, vv::kObsMaxIn);
  if (P.C != 4 + 5 * n_in) return fail(VV_E_ARG, "state has %d channels, the operator needs 4 + 5*%d", P.C, n_in);
  const size_t CHW = (size_t)P.C * P.Hs * P.Ws;
  const size_t nP = Arena::up((size_t)n_out * n_in * sizeof(float));
  P.obs_arena = std::make_unique<Arena>();
  P.obs_arena->cap = nP + CHW * P.T * P.B * sizeof(float);
  if (hipMalloc(&P.obs_arena->base, P.obs_arena->cap) != hipSuccess) return fail(VV_E_ALLOC, "observation operator");
  P.Pobs = reinterpret_cast<float*>(P.obs_arena->base);
  P.GOBS = reinterpret_cast<float*>(P.obs_arena->base + nP);
  VV_HIP(hipMemcpy(P.Pobs, interp, (size_t)n_out * n_in * sizeof(float), hipMemcpyDefault));
  P.nin = n_in;
  P.nout = n_out;
  return 0;
}

int vv_metrics(vv_ctx* ctx, const float* pred, const float* gt, const float* mean, const float* std_,
               const double* scale, int B, int C, int H, int W, double* wrmse, double* bias, void* stream) {
  if (!ctx || !pred || !gt || !mean || !std_ || !scale || !wrmse || !bias) return fail(VV_E_ARG, "null argument");
  if (B < 1 || C < 1 || H < 2 || W < 1) return fail(VV_E_ARG, "bad field shape");
  int r = set_dev(ctx);
  if (r) return r;
  // latitude weights as utils/metrics.py:4-9 + :287-289 compute them in fp32:
  // lat = 90 - j*180/(H-1); c = cos(3.1416/180 * lat); w = H * c / sum(c)
  std::vector<float> cw(H);
  float csum = 0.0f;
  for (int j = 0; j < H; ++j) {
    const float lat = 90.0f - ((float)j * 180.0f) / (float)(H - 1);
    cw[j] = cosf((float)(3.1416 / 180.0) * lat);
  }
  // torch.sum of a float32 vector: pairwise; a double sum rounded once differs by < 1 ulp of the total
  double cs = 0.0;
  for (int j = 0; j < H; ++j) cs += cw[j];
  csum = (float)cs;
  for (int j = 0; j < H; ++j) cw[j] = ((float)H * cw[j]) / csum;
  const int nchunk = std::max(1, std::min(64, H / 8));
  const size_t need = (size_t)H * sizeof(float) + (size_t)B * C * nchunk * 2 * sizeof(double);
  if (ctx->metric_cap < need) {
    if (ctx->metric_ws) (void)hipFree(ctx->metric_ws);
    ctx->metric_ws = nullptr;
    ctx->metric_cap = 0;
    if (hipMalloc(&ctx->metric_ws, need) != hipSuccess) return fail(VV_E_ALLOC, "metric workspace");
    ctx->metric_cap = need;
  }
  hipStream_t st = (hipStream_t)stream;
  double* part = reinterpret_cast<double*>(ctx->metric_ws);
  float* wl = reinterpret_cast<float*>(ctx->metric_ws + (size_t)B * C * nchunk * 2 * sizeof(double));
  VV_HIP(hipMemcpyAsync(wl, cw.data(), (size_t)H * sizeof(float), hipMemcpyHostToDevice, st));
  vv::MetricArgs a{pred, gt, mean, std_, scale, wl, B, C, H, W, part, nchunk, wrmse, bias};
  VV_HIP(vv::metrics(a, st));
  // the host weight table must outlive the async copy
  VV_HIP(hipStreamSynchronize(st));
  return 0;
}

int vv_obs_augment(vv_ctx* ctx, const float* interp, int n_out, int n_in, const float* x, float* x_aug, int T,
                   int Hs, int Ws, void* stream) {
  if (!ctx || !interp || !x || !x_aug) return fail(VV_E_ARG, "null argument");
  if (n_in < 1 || n_in > vv::kObsMaxIn || n_out < 1 || n_out > vv::kObsMaxOut || T < 1 || Hs < 1 || Ws < 1)
    return fail(VV_E_ARG, "bad operator / field shape");
  int r = set_dev(ctx);
  if (r) return r;
  VV_HIP(vv::obs_augment(interp, n_in, n_out, x, x_aug, T, Hs * Ws, (hipStream_t)stream));
  return 0;
}

int vv_state_ptr(vv_ctx* ctx, const float** x) {
  if (!ctx || !x || !ctx->prob.bound) return fail(VV_E_STATE, "no problem bound");
  *x = ctx->prob.X;
  return 0;
}

int vv_dot(vv_ctx* ctx, const float* a, const float* b, int64_t n, double* out, void* stream) {
  if (!ctx || !a || !b || !out) return fail(VV_E_ARG, "null argument");
  hipStream_t st = (hipStream_t)stream;
  VV_HIP(vv::vec_dot(a, b, n, ctx->red, kRedBlocks, ctx->dout, st));
  VV_HIP(hipMemcpyAsync(out, ctx->dout, sizeof(double), hipMemcpyDeviceToHost, st));
  VV_HIP(hipStreamSynchronize(st));
  return 0;
}
int vv_abssum(vv_ctx* ctx, const float* a, int64_t n, double* out, void* stream) {
  if (!ctx || !a || !out) return fail(VV_E_ARG, "null argument");
  hipStream_t st = (hipStream_t)stream;
  VV_HIP(vv::vec_abssum(a, n, ctx->red, kRedBlocks, ctx->dout, st));
  VV_HIP(hipMemcpyAsync(out, ctx->dout, sizeof(double), hipMemcpyDeviceToHost, st));
  VV_HIP(hipStreamSynchronize(st));
  return 0;
}
int vv_absmax(vv_ctx* ctx, const float* a, int64_t n, float* out, void* stream) {
  if (!ctx || !a || !out) return fail(VV_E_ARG, "null argument");
  hipStream_t st = (hipStream_t)stream;
  VV_HIP(vv::vec_absmax(a, n, ctx->redf, kRedBlocks, ctx->doutf, st));
  VV_HIP(hipMemcpyAsync(out, ctx->doutf, sizeof(float), hipMemcpyDeviceToHost, st));
  VV_HIP(hipStreamSynchronize(st));
  return 0;
}
int vv_reduce_batch(vv_ctx* ctx, int count, const int* ops, const float* const* a, const float* const* b, int64_t n,
                    const double* dev_extra, int n_extra, double* out, void* stream) {
  if (!ctx || count < 0 || count > kMaxBatch || n_extra < 0 || n_extra > kMaxExtra || (count && (!ops || !a)) ||
      (n_extra && !dev_extra) || !out || n < 0)
    return fail(VV_E_ARG, "reduce_batch: bad arguments");
  for (int i = 0; i < count; ++i)
    if (ops[i] < 0 || ops[i] > 2 || !a[i] || (ops[i] == 0 && (!b || !b[i])))
      return fail(VV_E_ARG, "reduce_batch: bad op %d", i);
  int r = set_dev(ctx);
  if (r) return r;
  hipStream_t st = (hipStream_t)stream;
  // the same grids, element partitions and partial layouts as vv_dot / vv_abssum / vv_absmax (identical values), all
  // requests in one launch and their finals + the extras in a second, written straight into the host-mapped results
  vv::ReduceReqs rq{};
  for (int i = 0; i < count; ++i) {
    rq.op[i] = ops[i];
    rq.a[i] = a[i];
    rq.b[i] = ops[i] == 0 ? b[i] : nullptr;
  }
  VV_HIP(vv::reduce_multi(rq, count, n, ctx->redb, kRedBlocks, ctx->hredb_dev, dev_extra, n_extra, st));
  VV_HIP(host_sync(ctx, st, n_extra > 0 ? 1 : 0));
  for (int i = 0; i < count + n_extra; ++i) out[i] = ctx->hredb[i];  // absmax widened from float: exact
  return 0;
}
int vv_reduce_enqueue(vv_ctx* ctx, int count, const int* ops, const float* const* a, const float* const* b, int64_t n,
                      double* dev_out, void* stream) {
  if (!ctx || count <= 0 || count > kMaxBatch || !ops || !a || !dev_out || n < 0)
    return fail(VV_E_ARG, "reduce_enqueue: bad arguments");
  for (int i = 0; i < count; ++i)
    if (ops[i] < 0 || ops[i] > 2 || !a[i] || (ops[i] == 0 && (!b || !b[i])))
      return fail(VV_E_ARG, "reduce_enqueue: bad op %d", i);
  int r = set_dev(ctx);
  if (r) return r;
  hipStream_t st = (hipStream_t)stream;
  // vv_reduce_batch's kernels and partial layouts (the same values), results left in dev_out (doubles), no sync
  vv::ReduceReqs rq{};
  for (int i = 0; i < count; ++i) {
    rq.op[i] = ops[i];
    rq.a[i] = a[i];
    rq.b[i] = ops[i] == 0 ? b[i] : nullptr;
  }
  VV_HIP(vv::reduce_multi(rq, count, n, ctx->redb, kRedBlocks, dev_out, nullptr, 0, st));
  return 0;
}
int vv_axpy(vv_ctx* ctx, float* y, const float* x, float alpha, int64_t n, void* stream) {
  if (!ctx || !y || !x) return fail(VV_E_ARG, "null argument");
  VV_HIP(vv::vec_axpy(y, x, alpha, n, (hipStream_t)stream));
  return 0;
}
int vv_axpby(vv_ctx* ctx, float* out, const float* x, float a, const float* y, float b, int64_t n, void* stream) {
  if (!ctx || !out || !x) return fail(VV_E_ARG, "null argument");
  VV_HIP(vv::vec_axpby(out, x, a, y, b, n, (hipStream_t)stream));
  return 0;
}
int vv_scale(vv_ctx* ctx, float* y, float alpha, int64_t n, void* stream) {
  if (!ctx || !y) return fail(VV_E_ARG, "null argument");
  VV_HIP(vv::vec_scale(y, alpha, n, (hipStream_t)stream));
  return 0;
}
int vv_lbfgs_two_loop(vv_ctx* ctx, float* q, const float* const* S, const float* const* Y, const float* ro, int m,
                      float H_diag, int64_t n, void* stream) {
  if (!ctx || !q || (m > 0 && (!S || !Y || !ro))) return fail(VV_E_ARG, "null argument");
  if (m < 0 || m > kMaxHistory) return fail(VV_E_ARG, "history size out of range");
  for (int i = 0; i < m; ++i)
    if (!S[i] || !Y[i]) return fail(VV_E_ARG, "null history vector");
  VV_HIP(vv::lbfgs_two_loop(q, S, Y, ro, m, H_diag, n, ctx->red, kRedBlocks, ctx->twoloop,
                            (hipStream_t)stream));
  return 0;
}
int vv_copy(vv_ctx* ctx, float* dst, const float* src, int64_t n, void* stream) {
  if (!ctx || !dst || !src) return fail(VV_E_ARG, "null argument");
  VV_HIP(hipMemcpyAsync(dst, src, n * sizeof(float), hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return 0;
}
int vv_adam(vv_ctx* ctx, float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2,
            float eps, int step, void* stream) {
  if (!ctx || !p || !g || !m || !v || step < 1) return fail(VV_E_ARG, "bad argument");
  const float bc1 = 1.0f - std::pow(beta1, (float)step);
  const float bc2 = 1.0f - std::pow(beta2, (float)step);
  VV_HIP(vv::adam_step(p, g, m, v, n, lr, beta1, beta2, eps, bc1, std::sqrt(bc2), (hipStream_t)stream));
  return 0;
}

int vv_profile_start(vv_ctx* ctx) {
  if (!ctx) return fail(VV_E_ARG, "null ctx");
  vv::prof_enable(true);
  return 0;
}

int vv_profile_stop(vv_ctx* ctx, double* ms, double* flops, double* bytes, int* launches, int ncls) {
  if (!ctx || ncls < vv::PC_N) return fail(VV_E_ARG, "need %d class slots", (int)vv::PC_N);
  vv::prof_read(ms, flops, bytes, launches);
  vv::prof_enable(false);
  return 0;
}

int vv_nearest_map(int in_size, int out_size, int* map) {
  if (in_size <= 0 || out_size <= 0 || !map) return fail(VV_E_ARG, "bad argument");
  auto m = nearest_map(in_size, out_size);
  std::copy(m.begin(), m.end(), map);
  return 0;
}

int vv_set_gemm_math(vv_ctx* ctx, int math) {
  if (!ctx || (math != VV_GEMM_F32 && math != VV_GEMM_SPLIT && math != VV_GEMM_SPLIT16))
    return fail(VV_E_ARG, "bad gemm math %d", math);
  if (math != ctx->math) drop_graphs(ctx);
  ctx->math = math;
  for (auto& m : ctx->models) {
    if (!m) continue;  // vv_model_destroy'ed
    m->sc.math = math;
    if (m->fm) vvf::set_math(m->fm, math);
  }
  return 0;
}

int vv_set_tuning(vv_ctx* ctx, const char* key, int value) {
  if (!ctx) return fail(VV_E_ARG, "null context");
  int* f = vv::tuning_field(ctx->tune, key);
  if (!f) return fail(VV_E_ARG, "unknown tuning key '%s'", key ? key : "(null)");
  if (!vv::tuning_value_ok(key, value)) return fail(VV_E_ARG, "tuning key '%s': value %d not accepted", key, value);
  if (*f != value) drop_graphs(ctx);
  *f = value;
  return 0;
}

int vv_get_tuning(vv_ctx* ctx, const char* key, int* value) {
  if (!ctx || !value) return fail(VV_E_ARG, "null argument");
  int* f = vv::tuning_field(ctx->tune, key);
  if (!f) return fail(VV_E_ARG, "unknown tuning key '%s'", key ? key : "(null)");
  *value = *f;
  return 0;
}

int vv_set_debug_sync(int enable) {
  g_sync_check.store(enable ? 1 : 0, std::memory_order_relaxed);
  return 0;
}

int vv_set_closure_graph(vv_ctx* ctx, int enable) {
  if (!ctx) return fail(VV_E_ARG, "null context");
  int r = set_dev(ctx);
  if (r) return r;
  drop_graphs(ctx);
  ctx->use_graphs = enable != 0;
  return 0;
}

int vv_get_counter(const char* name, long long* value) {
  if (!name || !value) return fail(VV_E_ARG, "null argument");
  static const char* names[vv::CNT_N] = {"rowsplit", "fixup_ln", "splitk_fixup", "gather_scales", "h5_split"};
  for (int c = 0; c < vv::CNT_N; ++c)
    if (!strcmp(name, names[c])) {
      *value = vv::launch_count(c);
      return 0;
    }
  return fail(VV_E_ARG, "unknown counter '%s'", name);
}

int vv_get_closure_graph(vv_ctx* ctx, int kind, long long* info) {
  if (!ctx || !info || kind < 0 || kind > 1) return fail(VV_E_ARG, "null context / info or kind not 0 / 1");
  const auto& g = ctx->graphs[kind];
  info[0] = ctx->use_graphs ? 1 : 0;
  info[1] = g.exec ? 1 : 0;
  info[2] = g.eager_only ? 1 : 0;
  info[3] = g.launches;
  return 0;
}

int vv_get_gemm_math(vv_ctx* ctx, int* math) {
  if (!ctx || !math) return fail(VV_E_ARG, "null argument");
  *math = ctx->math;
  return 0;
}

int vv_integrate(vv_ctx* ctx, int model_id, const float* x, float* out, int C, int Hs, int Ws, const float* mean,
                 const float* std_, int steps, void* stream) {
  Model* m = get_model(ctx, model_id);
  if (!m || !x || !out || !mean || !std_) return fail(VV_E_ARG, "bad model or pointers");
  if (!m->loaded) return fail(VV_E_STATE, "weights not loaded");
  if (steps < 1) return fail(VV_E_ARG, "steps must be >= 1");
  const int Hl = m->cfg.Himg, Wl = m->cfg.Wimg;
  if (m->B != 1 || m->cfg.Cin != C || m->cfg.Cout < C)
    return fail(VV_E_ARG, "model must map C=%d channels to >= C (has %d -> %d, batch %d)", C, m->cfg.Cin,
                m->cfg.Cout, m->B);
  if (C < 1 || Hs < 1 || Ws < 1) return fail(VV_E_ARG, "bad state shape");
  int r = set_dev(ctx);
  if (r) return r;
  hipStream_t st = (hipStream_t)stream;
  // nearest maps (quirk Q3) when the state grid differs from the model grid (integrate(interpolation=True))
  const bool interp = Hs != Hl || Ws != Wl;
  const size_t nin = (size_t)C * Hl * Wl, nout = (size_t)m->cfg.Cout * Hl * Wl;
  std::vector<int> maps;
  if (interp) {
    for (auto& v : {nearest_map(Hs, Hl), nearest_map(Ws, Wl), nearest_map(Hl, Hs), nearest_map(Wl, Ws)})
      maps.insert(maps.end(), v.begin(), v.end());
  }
  float *a = nullptr, *b = nullptr;
  int* dm = nullptr;
  VV_HIP(hipMallocAsync((void**)&a, nin * sizeof(float), st));
  VV_HIP(hipMallocAsync((void**)&b, nout * sizeof(float), st));
  if (interp) {
    VV_HIP(hipMallocAsync((void**)&dm, maps.size() * sizeof(int), st));
    VV_HIP(hipMemcpyAsync(dm, maps.data(), maps.size() * sizeof(int), hipMemcpyHostToDevice, st));
  }
  const int* di = interp ? dm : nullptr;
  const int* dj = interp ? dm + Hl : nullptr;
  const int* mi = interp ? dm + Hl + Wl : nullptr;
  const int* mj = interp ? dm + Hl + Wl + Hs : nullptr;
  // z = (x - mean)/std (-> model grid); z = model(z)[:, :C] `steps` times (da_4dvar.py:667-676)
  VV_HIP(vvf::normalize_resample(x, a, di, dj, mean, std_, C, Hs, Ws, Hl, Wl, st));
  for (int k = 0; k < steps && !r; ++k) {
    if (m->fm) {
      std::string err;
      r = vvf::forward(m->fm, a, b, C, st, err);
      if (r) fail(r, "%s", err.c_str());
    } else {
      r = model_fwd(*m, 0, a, b, C, st);
    }
    if (!r && k + 1 < steps) VV_HIP(hipMemcpyAsync(a, b, nin * sizeof(float), hipMemcpyDeviceToDevice, st));
  }
  // (-> state grid) * std + mean (:678-681)
  if (!r) VV_HIP(vvf::denormalize_resample(b, m->cfg.Cout, out, mi, mj, mean, std_, C, Hs, Ws, Hl, Wl, st));
  (void)hipFreeAsync(a, st);
  (void)hipFreeAsync(b, st);
  if (dm) (void)hipFreeAsync(dm, st);
  return r;
}

int vv_gemm_register_weight(vv_ctx* ctx, const float* B, int N, int K) {
  if (!ctx || !B || N <= 0 || K <= 0) return fail(VV_E_ARG, "bad argument");
  int r = set_dev(ctx);
  if (r) return r;
  unsigned short* planes = nullptr;
  const size_t n = (size_t)N * K;
  // a registration overlapping this range is stale (its weight was freed and the memory reused): drop it
  VV_HIP(hipDeviceSynchronize());
  for (size_t i = 0; i < ctx->split_owned.size();) {
    auto& w = ctx->split_owned[i];
    if (w.base < B + n && B < w.base + w.n) {
      vv::unregister_split_arena(w.base);
      (void)hipFree(w.planes);
      ctx->split_owned.erase(ctx->split_owned.begin() + i);
    } else {
      ++i;
    }
  }
  if (hipMalloc(&planes, vv::split_arena_bytes(n)) != hipSuccess) return fail(VV_E_ALLOC, "planes");
  vv::register_split_arena(B, n, planes);
  const hipError_t se = vv::split_registered(B, n, K, 0);
  if (se != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    vv::unregister_split_arena(B);
    (void)hipFree(planes);
    return fail((int)se, "split planes: %s", hipGetErrorString(se));
  }
  ctx->split_owned.push_back({B, n, planes});
  return 0;
}

static int gemm_entry(vv_ctx* ctx, int M, int N, int K, const float* A, const float* B, const float* bias, float* C,
                      float* aux, int epi, int tile, void* stream) {
  if (!ctx || !A || !B || !C) return fail(VV_E_ARG, "null argument");
  if (tile >= 0 && !vv::valid_tile(tile)) return fail(VV_E_ARG, "tile hint %d is not a library kernel", tile);
  if (M <= 0 || N <= 0 || K <= 0 || K % 32) return fail(VV_E_ARG, "bad GEMM shape %dx%dx%d (K a multiple of 32)", M, N, K);
  if (epi != EPI_STORE && epi != EPI_GELU && epi != EPI_DGELU) return fail(VV_E_ARG, "epilogue %d", epi);
  if (epi == EPI_DGELU && !aux) return fail(VV_E_ARG, "EPI_DGELU reads the pre-activation aux");
  int r = set_dev(ctx);
  if (r) return r;
  GemmArgs a = gemm_base(M, N, K, 1, epi, ctx->math, &ctx->tune);
  a.g[0] = {A, nullptr, B, bias, C, nullptr, aux};
  if (ctx->math == vv::GEMM_SPLIT16) {
    // A-plane workspace of the split-operand kernel (tile 48), grown on demand (vv_gemm is never graph-captured)
    const size_t need = (size_t)M * 2 * K;
    if (need > ctx->apl_halfs) {
      VV_HIP(hipStreamSynchronize((hipStream_t)stream));
      if (ctx->apl) VV_HIP(hipFree(ctx->apl));
      ctx->apl = nullptr;
      ctx->apl_halfs = 0;
      VV_HIP(hipMalloc(&ctx->apl, need * sizeof(unsigned short)));
      ctx->apl_halfs = need;
    }
    a.apl = ctx->apl;
    a.apl_halfs = ctx->apl_halfs;
  }
  VV_HIP(vv::gemm_nt(a, (hipStream_t)stream, tile, ctx->gemm_ws));
  return 0;
}

int vv_gemm(vv_ctx* ctx, int M, int N, int K, const float* A, const float* B, const float* bias, float* C, int tile,
            void* stream) {
  return gemm_entry(ctx, M, N, K, A, B, bias, C, nullptr, EPI_STORE, tile, stream);
}

int vv_gemm_epi(vv_ctx* ctx, int M, int N, int K, const float* A, const float* B, const float* bias, float* C,
                float* aux, int epi, int tile, void* stream) {
  return gemm_entry(ctx, M, N, K, A, B, bias, C, aux, epi, tile, stream);
}

int vv_gelu_eval(vv_ctx* ctx, const float* x, float* y, float* dy, int64_t n, int form, void* stream) {
  if (!ctx || !x || !y || !dy || n < 0 || (form != 0 && form != 1)) return fail(VV_E_ARG, "bad argument");
  int r = set_dev(ctx);
  if (r) return r;
  VV_HIP(vv::gelu_eval(x, y, dy, n, form, (hipStream_t)stream));
  return 0;
}

int vv_attention_global(vv_ctx* ctx, const float* qkv, float* out, int N, int C, int heads, void* stream) {
  if (!ctx || !qkv || !out) return fail(VV_E_ARG, "null argument");
  if (N <= 0 || !vv::gattn_supported(C, heads))
    return fail(VV_E_ARG, "global attention needs N > 0 and head_dim 64, 96, 128 or 192 (N %d, C %d, heads %d)", N, C,
                heads);
  int r = set_dev(ctx);
  if (r) return r;
  const size_t need = vv::gattn_ws_bytes(N, C, heads);
  if (need > ctx->gattn_bytes) {
    VV_HIP(hipStreamSynchronize((hipStream_t)stream));
    if (ctx->gattn_ws) VV_HIP(hipFree(ctx->gattn_ws));
    ctx->gattn_ws = nullptr;
    ctx->gattn_bytes = 0;
    VV_HIP(hipMalloc(&ctx->gattn_ws, need));
    ctx->gattn_bytes = need;
  }
  VV_HIP(vv::gattn(qkv, out, C, N, C, heads, ctx->gattn_ws, (hipStream_t)stream, ctx->tune.gattn_qf));
  return 0;
}

int vv_sc4dvar_bind(vv_ctx* ctx, int flow_model_id, int T, int C, int Hs, int Ws, const float* xb, const float* yo,
                    const float* Hmask, const float* R, const float* mean, const float* std_, float obs_coeff,
                    const float* interp, int n_out, const double* len_scale, const double* reg_coeff, int n_reg,
                    const double* std_sur, const double* vert_eig_value, const double* vert_eig_vec,
                    double scale_factor, int hpad) {
  if (!ctx) return fail(VV_E_ARG, "null context");
  if (T < 1 || C != 69) return fail(VV_E_ARG, "sc4dvar needs T >= 1 and the 69-channel state (C = %d)", C);
  if (Hs < 128 || Ws < 256) return fail(VV_E_ARG, "state grid %dx%d coarser than the 128x256 transform grid", Hs, Ws);
  if (!xb || !yo || !Hmask || !R || !mean || !std_) return fail(VV_E_ARG, "null problem buffer");
  if (!len_scale || !reg_coeff || !std_sur || !vert_eig_value || !vert_eig_vec) return fail(VV_E_ARG, "null B-matrix table");
  if (interp && (n_out < 1 || n_out > kObsMaxOut)) return fail(VV_E_ARG, "n_out %d out of range", n_out);
  Model* F = nullptr;
  if (T > 1) {
    F = get_model(ctx, flow_model_id);
    if (!F || F->fm) return fail(VV_E_ARG, "T > 1 needs a networks_old LGUnet_all flow model");
    if (!F->loaded) return fail(VV_E_STATE, "flow weights not loaded");
    if (F->cfg.Cin != C || F->cfg.Cout < C || F->B != 1 || F->cfg.Himg != 128 || F->cfg.Wimg != 256)
      return fail(VV_E_ARG, "flow model must map 69 channels on the 128x256 grid at batch 1");
  }
  int r = set_dev(ctx);
  if (r) return r;
  auto P = std::make_unique<Sc4Problem>();
  std::string err;
  if ((r = vv::sc4dvar_create(&P->bm, C, len_scale, reg_coeff, n_reg, std_sur, vert_eig_value, vert_eig_vec,
                              scale_factor, hpad, err)))
    return fail(r < 0 ? (r == -2 ? VV_E_ALLOC : VV_E_ARG) : r, "%s", err.c_str());
  P->flow = T > 1 ? flow_model_id : -1;
  P->T = T;
  P->C = C;
  P->Hs = Hs;
  P->Ws = Ws;
  P->interp = Hs != P->Hl || Ws != P->Wl;
  P->xb = xb;
  P->yo = yo;
  P->Hm = Hmask;
  P->R = R;
  P->mean = mean;
  P->std_ = std_;
  P->obs_coeff = obs_coeff;
  P->nin = interp ? 13 : 0;
  P->nout = interp ? n_out : 0;
  const size_t CHW = (size_t)C * Hs * Ws, fld = vv::sc4dvar_field_floats(P->bm), HWl = (size_t)P->Hl * P->Wl;
  P->wn = fld;
  for (int pass = 0; pass < 2; ++pass) {
    Planner pl;
    if (pass) pl.base = P->arena->base;
    P->t1 = pl.f(fld);
    P->t2 = pl.f(fld);
    P->recon = pl.f(fld);
    P->grec = pl.f(fld);
    P->X = pl.f(CHW * T);
    P->FI = pl.f((size_t)C * HWl);
    P->FO = pl.f((F ? (size_t)F->cfg.Cout : 1) * HWl);
    P->ones = pl.f(C);
    P->Pobs = pl.f((size_t)std::max(P->nout, 1) * 13);
    P->GOBS = pl.f(P->nout ? 2 * CHW : 1);
    int* mp = reinterpret_cast<int*>(pl.f((size_t)Hs + Ws + 2 * (P->Hl + 1) + 2 * (P->Wl + 1)));
    double* pd = reinterpret_cast<double*>(pl.f(2 * ((size_t)P->nblk * (T + 1) + 8)));
    if (pass) {
      P->partial = pd;
      P->dJ = pd + (size_t)P->nblk * (T + 1) + 2;
      P->mi = mp;
      P->mj = P->mi + Hs;
      P->ri0 = P->mj + Ws;
      P->rj0 = P->ri0 + P->Hl + 1;
      P->di = P->rj0 + P->Wl + 1;
      P->dj = P->di + P->Hl;
    } else {
      P->arena = std::make_unique<Arena>();
      if (hipMalloc(&P->arena->base, pl.bytes) != hipSuccess) return fail(VV_E_ALLOC, "sc4dvar arena");
      P->arena->cap = pl.bytes;
    }
  }
  {
    // nearest maps (quirk Q3): transform output 128x256 -> state grid (:928), integrate's down/up-sampling
    std::vector<int> mi = nearest_map(P->Hl, Hs), mj = nearest_map(P->Wl, Ws);
    std::vector<int> di = nearest_map(Hs, P->Hl), dj = nearest_map(Ws, P->Wl);
    auto ranges = [](const std::vector<int>& m, int n) {
      std::vector<int> rr(n + 1, (int)m.size());
      for (int k = (int)m.size() - 1; k >= 0; --k) rr[m[k]] = k;
      for (int a = n - 1; a >= 0; --a) rr[a] = std::min(rr[a], rr[a + 1]);
      return rr;
    };
    std::vector<int> ri0 = ranges(mi, P->Hl), rj0 = ranges(mj, P->Wl);
    std::vector<int> all;
    for (auto* v : {&mi, &mj, &ri0, &rj0, &di, &dj}) all.insert(all.end(), v->begin(), v->end());
    VV_HIP(hipMemcpy(P->mi, all.data(), all.size() * sizeof(int), hipMemcpyHostToDevice));
    std::vector<float> ones(C, 1.0f);
    VV_HIP(hipMemcpy(P->ones, ones.data(), C * sizeof(float), hipMemcpyHostToDevice));
    if (interp) VV_HIP(hipMemcpy(P->Pobs, interp, (size_t)n_out * 13 * sizeof(float), hipMemcpyDefault));
  }
  VV_HIP(hipDeviceSynchronize());
  P->bound = true;
  ctx->sc4 = std::move(P);
  return 0;
}

int vv_sc4dvar_closure(vv_ctx* ctx, const float* w, float* grad_w, double* J_b, double* J_o, void* stream) {
  if (!ctx || !w) return fail(VV_E_ARG, "null argument");
  if (!ctx->sc4 || !ctx->sc4->bound) return fail(VV_E_STATE, "vv_sc4dvar_bind first");
  int r = set_dev(ctx);
  if (r) return r;
  hipStream_t st = (hipStream_t)stream;
  if ((r = sc4_closure_impl(ctx, w, grad_w, st))) return r;
  hipLaunchKernelGGL(k_half, dim3(1), dim3(64), 0, st, ctx->sc4->dJ, 2);
  VV_HIP(hipGetLastError());
  double h[2];
  VV_HIP(hipMemcpyAsync(h, ctx->sc4->dJ, sizeof(h), hipMemcpyDeviceToHost, st));
  VV_HIP(hipStreamSynchronize(st));
  if (J_b) *J_b = h[0];
  if (J_o) *J_o = h[1];
  return 0;
}

int vv_sc4dvar_transform(vv_ctx* ctx, const float* w, float* xhat, void* stream) {
  if (!ctx || !w || !xhat) return fail(VV_E_ARG, "null argument");
  if (!ctx->sc4 || !ctx->sc4->bound) return fail(VV_E_STATE, "vv_sc4dvar_bind first");
  int r = set_dev(ctx);
  if (r) return r;
  Sc4Problem& P = *ctx->sc4;
  hipStream_t st = (hipStream_t)stream;
  VV_HIP(vv::sc4dvar_fwd(P.bm, w, P.recon, P.t1, P.t2, ctx->gemm_ws, st));
  MisfitArgs m;
  memset(&m, 0, sizeof(m));
  m.C = P.C;
  m.Hs = P.Hs;
  m.Ws = P.Ws;
  m.Hl = P.Hl;
  m.Wl = P.Wl;
  m.mi = P.interp ? P.mi : nullptr;
  m.mj = P.interp ? P.mj : nullptr;
  m.net = P.recon;
  m.net_cstride = P.C;
  m.scale = P.ones;
  m.xb = P.xb;
  m.x_out = xhat;  // Hm null: no misfit partials
  m.partial = P.partial;
  m.nblk = P.nblk;
  VV_HIP(misfit_fwd(m, st));
  return 0;
}

int vv_resample_nearest(vv_ctx* ctx, const float* in, float* out, int BC, int Hi, int Wi, int Ho, int Wo, int adjoint,
                        void* stream) {
  if (!ctx || !in || !out) return fail(VV_E_ARG, "null argument");
  if (BC < 1 || Hi < 1 || Wi < 1 || Ho < 1 || Wo < 1) return fail(VV_E_ARG, "bad shape");
  int r = set_dev(ctx);
  if (r) return r;
  hipStream_t st = (hipStream_t)stream;
  std::vector<int> maps;
  std::vector<int> mi = nearest_map(Hi, Ho), mj = nearest_map(Wi, Wo);
  if (adjoint) {
    auto ranges = [](const std::vector<int>& m, int n) {
      std::vector<int> rr(n + 1, (int)m.size());
      for (int k = (int)m.size() - 1; k >= 0; --k) rr[m[k]] = k;
      for (int a = n - 1; a >= 0; --a) rr[a] = std::min(rr[a], rr[a + 1]);
      return rr;
    };
    for (size_t k = 1; k < mi.size(); ++k)
      if (mi[k] < mi[k - 1]) return fail(VV_E_ARG, "non-monotone nearest map");
    for (size_t k = 1; k < mj.size(); ++k)
      if (mj[k] < mj[k - 1]) return fail(VV_E_ARG, "non-monotone nearest map");
    for (auto& v : {ranges(mi, Hi), ranges(mj, Wi)}) maps.insert(maps.end(), v.begin(), v.end());
  } else {
    maps = mi;
    maps.insert(maps.end(), mj.begin(), mj.end());
  }
  int* dm = nullptr;
  VV_HIP(hipMallocAsync((void**)&dm, maps.size() * sizeof(int), st));
  VV_HIP(hipMemcpyAsync(dm, maps.data(), maps.size() * sizeof(int), hipMemcpyHostToDevice, st));
  const hipError_t e = vv::resample_nearest(in, out, dm, BC, Hi, Wi, Ho, Wo, adjoint != 0, st);
  // the host vector must outlive the async copy
  VV_HIP(hipStreamSynchronize(st));
  (void)hipFreeAsync(dm, st);
  VV_HIP(e);
  return 0;
}

}  // extern "C"

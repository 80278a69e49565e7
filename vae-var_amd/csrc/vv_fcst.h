// Forecast network networks.LGUnet_all.LGUnet_all_1: forward-only engine.
// Internal interface between vv_engine.hip (C-ABI dispatch) and vv_fcst.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/vaevar.h"
#include "vv_kernels.h"

namespace vvf {

struct FModel;

struct ParamInfo {
  std::string name;
  std::vector<int64_t> shape;
};

// configuration check + the exact state_dict key set of LGUnet_all_1 (LGUnet_all.py:742-776)
int params(const vv_lgunet_config* cfg, std::vector<ParamInfo>& out, std::string& err);
int create(const vv_lgunet_config* cfg, int batch, FModel** out, std::string& err);
void destroy(FModel* m);
int load(FModel* m, const void* const* ptrs, int n, std::string& err);
// out (batch, sum(outchans), H, W), channels < climit (0 = all)
int forward(FModel* m, const float* in, float* out, int climit, hipStream_t st, std::string& err);
int64_t workspace_bytes(const FModel* m);
// GEMM arithmetic (vv::GemmMath) of the model's forward
void set_math(FModel* m, int math);
void set_tuning(FModel* m, const vv::Tuning* t);  // the owning context's knobs (kept by pointer)
int in_channels(const FModel* m);
int out_channels(const FModel* m);
int img_h(const FModel* m);
int img_w(const FModel* m);

// integrate() input / output maps (da_4dvar.py:666-681), fp32 op order of the reference:
//   net_in[c][i][j] = (x[c][di[i]][dj[j]] - mean[c]) / std[c]           (di/dj null: identity)
//   out[c][i][j]    = net[c][mi[i]][mj[j]] * std[c] + mean[c]             (mi/mj null: identity)
hipError_t normalize_resample(const float* x, float* net_in, const int* di, const int* dj, const float* mean,
                              const float* std_, int C, int Hs, int Ws, int Hl, int Wl, hipStream_t st);
hipError_t denormalize_resample(const float* net, int net_cstride, float* out, const int* mi, const int* mj,
                                const float* mean, const float* std_, int C, int Hs, int Ws, int Hl, int Wl,
                                hipStream_t st);

}  // namespace vvf

"""Host-side mirror of the reference's module protocol over libvaevar.

  LGUnet       ~ networks_old.transformer.LGUnet_all (transformer.py:716-752): state_dict-keyed weights,
                 __call__ is a differentiable forward (torch.autograd.Function over the HIP path)
  VAE_lr       ~ nf_model/vae.py:53-90 decoder half: .decoder(z), .decoder_hr(z)
  DAProblem    ~ the closure state of one_step_DA 'vae4dvar' (da_4dvar.py:1179-1251)

torch is plumbing here (device memory, streams); every FLOP runs in libvaevar.so.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import _lib
from ._lib import VVConfig, check, lib


def _ptr(t: torch.Tensor):
    if not t.is_cuda:
        raise ValueError("libvaevar compute entry points take device tensors")
    if t.dtype != torch.float32 or not t.is_contiguous():
        raise ValueError("expected a contiguous float32 tensor")
    return ctypes.c_void_p(t.data_ptr())


def _stream(stream=None):
    # the current stream's raw handle without building a torch.cuda.Stream object (a third of a vector op's host
    # cost on the L-BFGS mirror's launch-bound stretches)
    if stream is not None:
        return ctypes.c_void_p(stream.cuda_stream)
    return ctypes.c_void_p(torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice()))


class Context:
    """One libvaevar context per device (vv_ctx_create)."""

    _by_dev: dict = {}

    # per-context dispatch knobs (vv_set_tuning; defaults = the measured choices). A/B runs set them from the
    # environment as VAEVAR_<KEY> (e.g. VAEVAR_H3_MINK=384); the library itself reads no environment.
    TUNING_KEYS = ("h3_mink", "h3_big", "h3_mf16", "small_split", "small_split_minkt", "tail_minkt", "ln_scales",
                   "win_attn", "h4", "ln_planes", "gattn", "gattn_qf", "h4_small", "h4_split_minkt",
                   "win_mfma", "fc_h3_mink", "fuse_mlp", "fuse_attn", "attn_mfma", "gelu_planes", "attn_planes", "fixup_ln", "h5", "fc_conv_mf",
                   "mlp_hc", "h4_gather", "fixup_ln_rows", "grid_fused", "fixup_stage", "host_wait", "h5_split",
                   "patch_pers", "bs_tile", "fixup_ln_cross")

    def __init__(self, device: int = 0):
        self.device = device
        self.h = ctypes.c_void_p()
        # the environment is parsed and validated before the native context exists (a bad value must not leak it)
        env = os.environ
        math = env.get("VAEVAR_GEMM_MATH") or None
        if math is not None and math not in self.GEMM_MATH:
            raise ValueError(f"VAEVAR_GEMM_MATH={math!r}: expected one of {sorted(self.GEMM_MATH)}")
        tuning = {}
        for k in self.TUNING_KEYS:
            v = env.get("VAEVAR_" + k.upper())
            if v is not None and v != "":
                try:
                    tuning[k] = int(v)
                except ValueError:
                    raise ValueError(f"VAEVAR_{k.upper()}={v!r} is not an integer") from None
        check(lib.vv_ctx_create(device, ctypes.byref(self.h)), "ctx_create")
        try:
            if math is not None:
                self.gemm_math = math
            if env.get("VAEVAR_GRAPH", "1")[:1] == "0":
                self.set_closure_graph(False)
            if env.get("VAEVAR_SYNC_CHECK", "0")[:1] == "1":
                check(lib.vv_set_debug_sync(1), "set_debug_sync")
            for k, v in tuning.items():
                self.set_tuning(k, v)
        except Exception:
            lib.vv_ctx_destroy(self.h)
            self.h = ctypes.c_void_p()
            raise

    def set_tuning(self, key: str, value: int):
        """Set one dispatch knob of this context (keys: TUNING_KEYS; include/vaevar.h vv_set_tuning)."""
        check(lib.vv_set_tuning(self.h, key.encode(), int(value)), f"set_tuning({key})")

    def get_tuning(self, key: str) -> int:
        v = ctypes.c_int()
        check(lib.vv_get_tuning(self.h, key.encode(), ctypes.byref(v)), f"get_tuning({key})")
        return v.value

    @classmethod
    def get(cls, device: int = 0) -> "Context":
        if device not in cls._by_dev:
            cls._by_dev[device] = cls(device)
        return cls._by_dev[device]

    # --- vector primitives (torch/optim/lbfgs.py arithmetic) ---
    def dot(self, a, b) -> float:
        out = ctypes.c_double()
        check(lib.vv_dot(self.h, _ptr(a), _ptr(b), a.numel(), ctypes.byref(out), _stream()), "dot")
        return out.value

    def abssum(self, a) -> float:
        out = ctypes.c_double()
        check(lib.vv_abssum(self.h, _ptr(a), a.numel(), ctypes.byref(out), _stream()), "abssum")
        return out.value

    def absmax(self, a) -> float:
        out = ctypes.c_float()
        check(lib.vv_absmax(self.h, _ptr(a), a.numel(), ctypes.byref(out), _stream()), "absmax")
        return out.value

    def reduce_batch(self, reqs, extra=None) -> list:
        """vv_reduce_batch: reqs = [(op, a, b)] with op 0 dot(a, b), 1 abssum(a), 2 absmax(a) (equal-length vectors,
        <= 8), plus the float64 device tensor `extra` (<= 16 values) appended: one synchronisation for all of them,
        the values of the one-call-each vv_dot / vv_abssum / vv_absmax."""
        k = len(reqs)
        n = reqs[0][1].numel() if k else 0
        for op, a, b in reqs:
            if a.numel() != n or (op == 0 and b.numel() != n):
                raise ValueError("reduce_batch: vectors of different lengths")
        ops = (ctypes.c_int * max(k, 1))(*[int(r[0]) for r in reqs])
        A = (ctypes.c_void_p * max(k, 1))(*[_ptr(r[1]).value for r in reqs])
        B = (ctypes.c_void_p * max(k, 1))(*[(_ptr(r[2]).value if r[0] == 0 else None) for r in reqs])
        ne = extra.numel() if extra is not None else 0
        if extra is not None and (extra.dtype != torch.float64 or not extra.is_cuda or not extra.is_contiguous()):
            raise ValueError("reduce_batch: extra must be a contiguous float64 CUDA tensor")
        out = (ctypes.c_double * max(k + ne, 1))()
        check(lib.vv_reduce_batch(self.h, k, ops, A, B, n, ctypes.c_void_p(extra.data_ptr()) if ne else None, ne, out,
                                  _stream()),
              "reduce_batch")
        return list(out[:k + ne])

    def reduce_enqueue(self, reqs, out: torch.Tensor):
        """vv_reduce_enqueue: reqs as in reduce_batch, queued; the values land in the float64 device tensor `out`
        (len(reqs) entries) without a synchronisation — fetch them later as reduce_batch's `extra`."""
        k = len(reqs)
        n = reqs[0][1].numel()
        for op, a, b in reqs:
            if a.numel() != n or (op == 0 and b.numel() != n):
                raise ValueError("reduce_enqueue: vectors of different lengths")
        if out.dtype != torch.float64 or not out.is_cuda or not out.is_contiguous() or out.numel() < k:
            raise ValueError("reduce_enqueue: out must be a contiguous float64 CUDA tensor of len(reqs) entries")
        ops = (ctypes.c_int * k)(*[int(r[0]) for r in reqs])
        A = (ctypes.c_void_p * k)(*[_ptr(r[1]).value for r in reqs])
        B = (ctypes.c_void_p * k)(*[(_ptr(r[2]).value if r[0] == 0 else None) for r in reqs])
        check(lib.vv_reduce_enqueue(self.h, k, ops, A, B, n, ctypes.c_void_p(out.data_ptr()), _stream()),
              "reduce_enqueue")

    def axpy(self, y, x, alpha: float):
        check(lib.vv_axpy(self.h, _ptr(y), _ptr(x), float(alpha), y.numel(), _stream()), "axpy")

    def axpby(self, out, x, a: float, y, b: float):
        yp = _ptr(y) if y is not None else None
        check(lib.vv_axpby(self.h, _ptr(out), _ptr(x), float(a), yp, float(b), out.numel(), _stream()), "axpby")

    def scale(self, y, alpha: float):
        check(lib.vv_scale(self.h, _ptr(y), float(alpha), y.numel(), _stream()), "scale")

    def copy(self, dst, src):
        check(lib.vv_copy(self.h, _ptr(dst), _ptr(src), dst.numel(), _stream()), "copy")

    def lbfgs_two_loop(self, q, stps, dirs, ro, H_diag: float):
        """q = -g in, the L-BFGS direction out (lbfgs.py:404-442), dot products and coefficients on the device."""
        m = len(stps)
        S = (ctypes.c_void_p * max(m, 1))(*[_ptr(v).value for v in stps])
        Y = (ctypes.c_void_p * max(m, 1))(*[_ptr(v).value for v in dirs])
        r = (ctypes.c_float * max(m, 1))(*[float(x) for x in ro])
        check(lib.vv_lbfgs_two_loop(self.h, _ptr(q), S, Y, r, m, float(H_diag), q.numel(), _stream()), "two_loop")

    def adam(self, p, g, m, v, lr, beta1, beta2, eps, step):
        check(lib.vv_adam(self.h, _ptr(p), _ptr(g), _ptr(m), _ptr(v), p.numel(), lr, beta1, beta2, eps, step,
                          _stream()), "adam")

    PROF_CLASSES = ("gemm", "attention", "layernorm", "patch", "misfit", "vector", "gemm16", "tower")

    def profile_start(self):
        check(lib.vv_profile_start(self.h), "profile_start")

    def profile_stop(self) -> dict:
        """{class: dict(ms, flops, bytes, launches)} of every launch since profile_start (HIP events)."""
        n = len(self.PROF_CLASSES)
        ms, fl, by = (ctypes.c_double * n)(), (ctypes.c_double * n)(), (ctypes.c_double * n)()
        cnt = (ctypes.c_int * n)()
        check(lib.vv_profile_stop(self.h, ms, fl, by, cnt, n), "profile_stop")
        return {c: {"ms": ms[i], "flops": fl[i], "bytes": by[i], "launches": cnt[i]}
                for i, c in enumerate(self.PROF_CLASSES)}

    GEMM_MATH = {"f32": 0, "split": 1, "split16": 2}

    @property
    def gemm_math(self) -> str:
        """'split16' (fp16x3 scaled split, default), 'split' (bf16x6 split) or 'f32' (exact f32 MFMA); per context
        (VAEVAR_GEMM_MATH sets it at construction).

        Both split modes carry fp32-level error (measured against fp64 in tests/test_gpu_kernels.py)."""
        v = ctypes.c_int()
        check(lib.vv_get_gemm_math(self.h, ctypes.byref(v)), "get_gemm_math")
        return {0: "f32", 1: "split", 2: "split16"}[v.value]

    @gemm_math.setter
    def gemm_math(self, name: str):
        check(lib.vv_set_gemm_math(self.h, self.GEMM_MATH[name]), "set_gemm_math")

    def set_closure_graph(self, enable: bool):
        """Replay the closure from a captured hipGraph (default) or launch its kernels eagerly."""
        check(lib.vv_set_closure_graph(self.h, 1 if enable else 0), "set_closure_graph")

    @staticmethod
    def counter(name: str) -> int:
        """vv_get_counter: process-wide eager launch count of a fused-path alternative ("rowsplit", "fixup_ln",
        "splitk_fixup", "gather_scales", "h5_split")."""
        v = ctypes.c_longlong()
        check(lib.vv_get_counter(name.encode(), ctypes.byref(v)), "get_counter")
        return v.value

    def closure_graph_state(self, kind: int = 1) -> dict:
        """vv_get_closure_graph: whether the closure of this kind (0: J only, 1: J + gradient) runs from its graph."""
        info = (ctypes.c_longlong * 4)()
        check(lib.vv_get_closure_graph(self.h, kind, info), "get_closure_graph")
        return {"enabled": bool(info[0]), "instantiated": bool(info[1]), "eager_only": bool(info[2]),
                "launches": int(info[3])}

    def attention_global(self, qkv, heads: int):
        """softmax(q k^T) v per head over all N tokens of qkv [N, 3C] (vv_attention_global); returns out [N, C]."""
        if not (qkv.is_cuda and qkv.dtype == torch.float32 and qkv.dim() == 2 and qkv.is_contiguous()):
            raise ValueError("qkv must be a contiguous 2-D float32 CUDA tensor [N, 3C] (row stride 3C)")
        N, C3 = qkv.shape
        if C3 % 3 or (C3 // 3) % heads:
            raise ValueError(f"qkv width {C3} is not 3C with C divisible by heads={heads}")
        out = torch.empty(N, C3 // 3, device=qkv.device, dtype=torch.float32)
        check(lib.vv_attention_global(self.h, _ptr(qkv), _ptr(out), N, C3 // 3, heads, _stream()), "attention_global")
        return out

    def gemm_register_weight(self, B):
        """Precompute B's split planes (bf16 and fp16; B must outlive the context and stay unchanged)."""
        check(lib.vv_gemm_register_weight(self.h, _ptr(B), B.shape[0], B.shape[1]), "gemm_register_weight")

    def gemm(self, A, B, bias=None, tile=-1):
        M, K = A.shape
        N = B.shape[0]
        C = torch.empty(M, N, device=A.device, dtype=torch.float32)
        bp = _ptr(bias) if bias is not None else None
        check(lib.vv_gemm(self.h, M, N, K, _ptr(A), _ptr(B), bp, _ptr(C), tile, _stream()), "gemm")
        return C

    EPI = {"store": 0, "gelu": 1, "dgelu": 3}

    def gemm_epi(self, A, B, epi, aux=None, bias=None, tile=-1):
        """vv_gemm_epi: C = gelu(A B^T + bias) (aux, if given, receives A B^T + bias) or C = (A B^T) * gelu'(aux)."""
        M, K = A.shape
        N = B.shape[0]
        C = torch.empty(M, N, device=A.device, dtype=torch.float32)
        bp = _ptr(bias) if bias is not None else None
        ap = _ptr(aux) if aux is not None else None
        check(lib.vv_gemm_epi(self.h, M, N, K, _ptr(A), _ptr(B), bp, _ptr(C), ap, self.EPI[epi], tile, _stream()),
              "gemm_epi")
        return C

    def gelu_eval(self, x, form=0):
        """(GELU(x), GELU'(x)) by the epilogues' device functions (vv_gelu_eval; form 1: the four-value forms)."""
        y, dy = torch.empty_like(x), torch.empty_like(x)
        check(lib.vv_gelu_eval(self.h, _ptr(x), _ptr(y), _ptr(dy), x.numel(), form, _stream()), "gelu_eval")
        return y, dy


class _NetFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, net, slot, out_limit):
        out = net.forward_raw(x, slot, out_limit)
        ctx.net, ctx.slot, ctx.out_limit, ctx.shape = net, slot, out_limit, x.shape
        return out

    @staticmethod
    def backward(ctx, g):
        dx = torch.empty(ctx.shape, device=g.device, dtype=torch.float32)
        ctx.net.backward_raw(g.contiguous(), dx, ctx.slot, ctx.out_limit)
        return dx, None, None, None


class LGUnet:
    """networks_old.transformer.LGUnet_all on the HIP engine, or with cfg["arch"] == "lgunet1" the
    forecast network networks.LGUnet_all.LGUnet_all_1 (forward only, LGUnet_all.py:742-776).

    Weights are the reference's state_dict entries (module./max_logvar filtering as in
    da_4dvar.py:594-601 is applied by `load_state_dict`). Input gradients only (quirk Q5).
    """

    def __init__(self, cfg: dict, batch: int = 1, n_slots: int = 1, device: int = 0):
        self.cfg = dict(cfg)
        self.ctx = Context.get(device)
        self.device = torch.device("cuda", device)
        self.batch, self.n_slots = batch, n_slots
        self._c = VVConfig.from_dict(cfg)
        mid = ctypes.c_int()
        check(lib.vv_model_create(self.ctx.h, ctypes.byref(self._c), batch, n_slots, ctypes.byref(mid)),
              "model_create")
        self.id = mid.value
        self.params = _lib.param_list(cfg)
        self.in_ch = int(sum(cfg["inchans_list"]))
        self.out_ch = int(sum(cfg["outchans_list"]))
        self.H, self.W = cfg["img_size"]

    def __del__(self):
        # vv_model_destroy: the network's device memory goes with the object (a DAProblem keeps its networks alive;
        # the bound problem of a destroyed network is unbound by the library). Skipped at interpreter shutdown.
        mid = getattr(self, "id", None)
        if mid is not None and lib is not None and getattr(self.ctx, "h", None):
            try:
                lib.vv_model_destroy(self.ctx.h, mid)
            except Exception:
                pass
        self.id = None

    def workspace_bytes(self) -> int:
        b = ctypes.c_int64()
        check(lib.vv_model_workspace_bytes(self.ctx.h, self.id, ctypes.byref(b)), "workspace_bytes")
        return b.value

    def load_state_dict(self, sd: dict, prefix: str = ""):
        clean = {}
        for k, v in sd.items():
            name = k[7:] if k.startswith("module.") else k
            if name in ("max_logvar", "min_logvar"):
                continue
            clean[name] = v
        keep = []
        ptrs = (ctypes.c_void_p * len(self.params))()
        for i, (name, shape) in enumerate(self.params):
            key = prefix + name
            if key not in clean:
                raise KeyError(f"missing parameter {key}")
            v = clean[key]
            if isinstance(v, np.ndarray):
                v = torch.from_numpy(np.ascontiguousarray(v, dtype=np.float32))
            v = v.detach().to(torch.float32).contiguous()
            if tuple(v.shape) != tuple(shape):
                raise ValueError(f"{key}: shape {tuple(v.shape)} != {shape}")
            keep.append(v)
            ptrs[i] = v.data_ptr()
        check(lib.vv_load_weights(self.ctx.h, self.id, ptrs, len(self.params)), "load_weights")
        return self

    def load_synthetic(self, base_seed: int = 20250620, prefix: str = ""):
        from .synth import param_value

        sd = {prefix + n: param_value(prefix + n, s, base_seed) for n, s in self.params}
        return self.load_state_dict(sd, prefix)

    # raw device entry points (no autograd)
    def forward_raw(self, x: torch.Tensor, slot: int = 0, out_limit: int = 0, out=None):
        if tuple(x.shape) != (self.batch, self.in_ch, self.H, self.W):
            raise ValueError(f"input shape {tuple(x.shape)} != {(self.batch, self.in_ch, self.H, self.W)}")
        x = x.contiguous()
        if out is None:
            out = torch.empty(self.batch, self.out_ch, self.H, self.W, device=x.device, dtype=torch.float32)
        check(lib.vv_model_forward(self.ctx.h, self.id, slot, _ptr(x), _ptr(out), out_limit, _stream()), "forward")
        return out

    def backward_raw(self, g: torch.Tensor, dx: torch.Tensor, slot: int = 0, out_limit: int = 0, add=None):
        ap = _ptr(add) if add is not None else None
        check(lib.vv_model_backward(self.ctx.h, self.id, slot, _ptr(g), _ptr(dx), ap, out_limit, _stream()),
              "backward")
        return dx

    def __call__(self, x: torch.Tensor, slot: int = 0, out_limit: int = 0):
        """Differentiable forward (input gradient). One pending backward per slot."""
        return _NetFn.apply(x, self, slot, out_limit)


def integrate(model: LGUnet, x: torch.Tensor, mean: torch.Tensor, std: torch.Tensor, steps: int = 1,
              out: torch.Tensor = None) -> torch.Tensor:
    """`cyclic_4dvar.integrate(x, model, steps)` (da_4dvar.py:666-681) on libvaevar (vv_integrate): the
    outer-cycle forecast x_b = integrate(x_a, forecast_model, 1) (:1329). x: (C, Hs, Ws) on the device; a
    state grid other than the model grid is nearest-resampled both ways (interpolation=True)."""
    C, Hs, Ws = x.shape
    x = x.contiguous()
    mean = mean.to(x.device, torch.float32).contiguous()
    std = std.to(x.device, torch.float32).contiguous()
    if out is None:
        out = torch.empty_like(x)
    check(lib.vv_integrate(model.ctx.h, model.id, _ptr(x), _ptr(out), C, Hs, Ws, _ptr(mean), _ptr(std), steps,
                           _stream()), "integrate")
    return out


class VAE_lr:
    """Decoder half of nf_model/vae.py:53-90 (VAE_lr.dec is networks_old LGUnet_all)."""

    def __init__(self, dec_cfg: dict, device: int = 0, state_grid=None):
        self.dec = LGUnet(dec_cfg, 1, 1, device)
        self.state_grid = tuple(state_grid) if state_grid else tuple(dec_cfg["img_size"])

    def decoder(self, z):
        return self.dec(z)

    def decoder_hr(self, z):
        x = self.dec(z)
        if self.state_grid != tuple(x.shape[-2:]):
            # nearest interpolation to the state grid (vae.py:90) on the GPU (vv_resample_nearest), differentiable
            x = resample_nearest(self.dec.ctx, x, self.state_grid)
        return x


class _Resample(torch.autograd.Function):
    @staticmethod
    def forward(actx, x, ctx, size):
        B, C, Hi, Wi = x.shape
        out = torch.empty(B, C, size[0], size[1], device=x.device, dtype=torch.float32)
        check(lib.vv_resample_nearest(ctx.h, _ptr(x.contiguous()), _ptr(out), B * C, Hi, Wi, size[0], size[1], 0,
                                      _stream()), "resample_nearest")
        actx.ctx, actx.shape = ctx, x.shape
        return out

    @staticmethod
    def backward(actx, g):
        B, C, Hi, Wi = actx.shape
        gin = torch.empty(actx.shape, device=g.device, dtype=torch.float32)
        check(lib.vv_resample_nearest(actx.ctx.h, _ptr(g.contiguous()), _ptr(gin), B * C, Hi, Wi, g.shape[2],
                                      g.shape[3], 1, _stream()), "resample_nearest")
        return gin, None, None


def resample_nearest(ctx: Context, x: torch.Tensor, size) -> torch.Tensor:
    """F.interpolate(x, size) (mode 'nearest', quirk Q3) of a (B, C, H, W) device tensor on libvaevar, with its
    adjoint as the backward."""
    return _Resample.apply(x, ctx, tuple(int(v) for v in size))


class LazyLoss:
    """A queued closure's loss: `dev` holds (J_b, J_o) on the device; `resolve(values)` turns the fetched pair into
    the loss. `float()` fetches it on its own (one synchronisation)."""

    def __init__(self, dev: torch.Tensor, finish, discard=None):
        self.dev, self.finish, self._discard = dev, finish, discard

    def resolve(self, values) -> float:
        return self.finish(values)

    def discard(self):
        """The evaluation is dropped (the mirror speculated past an exit the reference takes before it): uncount it."""
        if self._discard is not None:
            self._discard()

    def __float__(self) -> float:
        v = self.dev.cpu().tolist()
        return float(self.finish(v))


class DAProblem:
    """The vae4dvar closure (da_4dvar.py:1183-1208) bound to device buffers; evaluated by libvaevar.

    With a decoder (and flow model) of batch B > 1 the problem holds B independent analyses: xb (B,C,Hs,Ws) and
    yo, H, R (B,T,C,Hs,Ws) — or pass a list of B single-analysis problem dicts — and one evaluation runs all B
    (closure_batch: J per analysis)."""

    def __init__(self, dec: LGUnet, prob, flow: LGUnet | None = None, obs_coeff: float = 1.0, device: int = 0,
                 obs_interp=None):
        """obs_interp: None (synthetic observations of the state) or the (n_out, n_in) obs_interpolater.interp of
        obs_type 'real*' (da_4dvar.py:1196-1206); `prob["interp"]` is used when present. yo, H, R then hold
        4 + 5*n_out observation channels."""
        dev = torch.device("cuda", device)
        self.B = dec.batch
        if isinstance(prob, (list, tuple)):
            if len(prob) != self.B:
                raise ValueError(f"{len(prob)} problems for a decoder of batch {self.B}")
            stacked = {k: np.stack([np.asarray(p[k], np.float32) for p in prob]) for k in ("xb", "yo", "H", "R")}
            prob = dict(prob[0], **stacked)
        elif self.B > 1 and np.ndim(prob["xb"]) != 4:
            raise ValueError("a batched problem needs xb (B,C,Hs,Ws) and yo/H/R (B,T,C,Hs,Ws)")

        def t(a):
            if isinstance(a, torch.Tensor):
                return a.to(device=dev, dtype=torch.float32).contiguous()
            return torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float32).to(dev)

        self.xb, self.yo, self.H, self.R = t(prob["xb"]), t(prob["yo"]), t(prob["H"]), t(prob["R"])
        self.mean, self.std, self.std_tr = t(prob["mean"]), t(prob["std"]), t(prob["std_tr"])
        if self.B > 1:
            if self.xb.shape[0] != self.B or self.yo.shape[0] != self.B:
                raise ValueError(f"leading dimension of xb/yo must be the batch {self.B}")
            self.T, self.C = self.yo.shape[1], self.xb.shape[1]
        else:
            self.T, self.C = self.yo.shape[0], self.xb.shape[0]
        self.Hs, self.Ws = self.xb.shape[-2:]
        self.dec, self.flow, self.obs_coeff = dec, flow, float(obs_coeff)
        self.ctx = dec.ctx
        self.latent_shape = (self.B, dec.in_ch, dec.H, dec.W)
        if obs_interp is None:
            obs_interp = prob.get("interp")
        self.interp = None if obs_interp is None else t(obs_interp)
        ych = self.yo.shape[-3]
        if self.interp is not None:
            n_out, n_in = self.interp.shape
            if ych != 4 + 5 * n_out:
                raise ValueError(f"yo has {ych} channels, the operator gives {4 + 5 * n_out}")
        elif ych != self.C:
            raise ValueError("yo/H/R channels differ from the state's: pass the observation operator (obs_interp)")
        fid = flow.id if flow is not None else -1
        check(lib.vv_bind_problem(self.ctx.h, dec.id, fid, self.T, self.C, self.Hs, self.Ws, _ptr(self.xb),
                                  _ptr(self.yo), _ptr(self.H), _ptr(self.R), _ptr(self.mean), _ptr(self.std),
                                  _ptr(self.std_tr), self.obs_coeff), "bind_problem")
        if self.interp is not None:
            check(lib.vv_set_obs_operator(self.ctx.h, n_out, n_in, _ptr(self.interp)), "set_obs_operator")
        self.n_evals = 0
        # evaluations the speculative L-BFGS mirror ran and discarded (vaevar/lbfgs.py: the line search's first
        # evaluation started before gtd is known, where the reference stops on gtd > -tolerance_change); their time is
        # inside one_step_da's seconds and the bench's timed region
        self.n_discarded = 0

    def closure_batch(self, z: torch.Tensor, grad: torch.Tensor | None):
        """One evaluation of all B analyses: (J_b[B], J_o[B]) as float64 arrays; grad <- dJ/dz (B,...) if given."""
        jb, jo = (ctypes.c_double * self.B)(), (ctypes.c_double * self.B)()
        gp = _ptr(grad) if grad is not None else None
        check(lib.vv_closure(self.ctx.h, _ptr(z), gp, jb, jo, _stream()), "closure")
        self.n_evals += 1
        return np.array(jb[:], np.float64), np.array(jo[:], np.float64)

    def closure_lazy(self, z: torch.Tensor, grad: torch.Tensor | None) -> "LazyLoss":
        """The closure queued without a host round trip (vv_closure_async): J_b, J_o stay in a device buffer until
        the L-BFGS mirror fetches them together with its reductions (vaevar.lbfgs, vv_reduce_batch). Single
        analysis (B = 1); the loss is loss_f32 of the fetched pair."""
        if self.B != 1:
            raise ValueError("batched problem: use closure_batch")
        if getattr(self, "_dJ", None) is None:
            self._dJ = torch.empty(2, device=self.xb.device, dtype=torch.float64)
        gp = _ptr(grad) if grad is not None else None
        check(lib.vv_closure_async(self.ctx.h, _ptr(z), gp, ctypes.c_void_p(self._dJ.data_ptr()), _stream()),
              "closure_async")
        self.n_evals += 1

        def uncount():  # a speculative evaluation the reference would not have made (counted, not hidden)
            self.n_evals -= 1
            self.n_discarded += 1

        return LazyLoss(self._dJ, lambda v: self.loss_f32(v[0], v[1]), uncount)

    def closure(self, z: torch.Tensor, grad: torch.Tensor | None):
        """Returns (J_b, J_o) as Python floats (double sums); grad <- dJ/dz if given. Single analysis (B = 1)."""
        if self.B != 1:
            raise ValueError("batched problem: use closure_batch")
        jb, jo = self.closure_batch(z, grad)
        return float(jb[0]), float(jo[0])

    def loss_f32(self, jb: float, jo: float) -> float:
        """loss_reg + obs_coeff * loss_obs with the reference's fp32 scalar arithmetic (quirk Q7)."""
        return float(np.float32(jb) + np.float32(np.float32(self.obs_coeff) * np.float32(jo)))

    def analysis(self, z: torch.Tensor) -> torch.Tensor:
        """xa (C,Hs,Ws), or (B,C,Hs,Ws) for a batched problem."""
        shape = (self.C, self.Hs, self.Ws) if self.B == 1 else (self.B, self.C, self.Hs, self.Ws)
        xa = torch.empty(shape, device=z.device, dtype=torch.float32)
        check(lib.vv_decode(self.ctx.h, _ptr(z.contiguous()), _ptr(xa), _stream()), "decode")
        return xa

    def trajectory(self) -> torch.Tensor:
        """x_t (T,C,Hs,Ws) of the last closure (a copy); (B,T,C,Hs,Ws) for a batched problem."""
        p = ctypes.c_void_p()
        check(lib.vv_state_ptr(self.ctx.h, ctypes.byref(p)), "state_ptr")
        n = self.B * self.T * self.C * self.Hs * self.Ws
        out = torch.empty(n, device=self.xb.device, dtype=torch.float32)
        check(lib.vv_copy(self.ctx.h, _ptr(out), p, n, _stream()), "copy")
        shape = (self.T, self.C, self.Hs, self.Ws) if self.B == 1 else (self.B, self.T, self.C, self.Hs, self.Ws)
        return out.view(shape)


class _ClosureFn(torch.autograd.Function):
    """J(z) as a differentiable scalar, so torch.optim.LBFGS can drive the HIP closure unchanged."""

    @staticmethod
    def forward(ctx, z, prob):
        g = torch.empty_like(z)
        jb, jo = prob.closure(z.detach().contiguous(), g)
        ctx.save_for_backward(g)
        return torch.tensor(prob.loss_f32(jb, jo), device=z.device, dtype=torch.float32)

    @staticmethod
    def backward(ctx, gout):
        (g,) = ctx.saved_tensors
        return g * gout, None


def loss(prob: DAProblem, z: torch.Tensor) -> torch.Tensor:
    """Drop-in for the reference's `loss(z)` (da_4dvar.py:1183-1208)."""
    return _ClosureFn.apply(z, prob)


def obs_augment(ctx: Context, interp: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """x_aug (da_4dvar.py:1196-1206) of (T, 4 + 5*n_in, H, W) device fields on the GPU; applied to R it is
    get_R_matrix_from_gt (da_4dvar.py:729-756)."""
    n_out, n_in = interp.shape
    T, C, Hs, Ws = x.shape
    if C != 4 + 5 * n_in:
        raise ValueError(f"{C} channels, the operator expects {4 + 5 * n_in}")
    interp = interp.to(device=x.device, dtype=torch.float32).contiguous()
    x = x.contiguous()
    out = torch.empty(T, 4 + 5 * n_out, Hs, Ws, device=x.device, dtype=torch.float32)
    check(lib.vv_obs_augment(ctx.h, _ptr(interp), n_out, n_in, _ptr(x), _ptr(out), T, Hs, Ws, _stream()),
          "obs_augment")
    return out

"""Training-mode render path: `RayCaster.render_rays` with stratified
sampling (`perturb`), density noise (`raw_noise_std`), stochastic importance sampling and
gradients to the networks AND to the skeleton transforms (A-NeRF's pose optimisation).

Mirrors `core/raycasters.py:361-474` (training branch of `RayCaster.forward`, :349-359) and the
loss of `Trainer._compute_nerf_loss` (`core/trainer.py:350-381`).  The per-sample stages run as
HIP kernels through the C ABI (include/anerf.h, `anerf_train_*`): sample placement, the skeleton-
relative encoding and its backward (dL/dskts), raw2outputs and its backward, importance sampling.
The MLP between them is one autograd Function on the hand-written split-bf16 GEMMs of
`anerf_gemm.hip` (`mlp.py`; default `mlp="mixed"`: bf16x6 forward, bf16x3 gradients; `mlp="fp32"`
keeps torch's fp32 GEMMs), with the reference's concatenations (`cat([x, h])` at the skip,
`cat([feature, views(, code)])` at the view layer) replaced by operand segments / split weight
blocks, so no concatenated activation is ever materialised.

Random numbers: torch's generator on the device by default; pass `rand={"t_rand": (N,S),
"noise0": (N,S), "u": (N,I), "noise1": (N,S+I)}` (standard-uniform / standard-normal draws; with
ray_noise_std also "pts_noise0": (N,S,3), "pts_noise1": (N,I,3)) to reproduce a given draw — the
parity tests feed the reference's.
"""
import contextlib

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from .config import RenderConfig, feature_scales
from .model import DeviceModel


def _stream(dev):
    return _lib.stream_handle(dev)


# (round 6) the fine pass of a training step on a stream of its own: the coarse and fine networks' backward passes
# are independent (the fine samples come from the detached coarse weights, raycasters.py:456-466), and autograd runs
# each node on the stream its forward ran on, so the two backward passes overlap on the GPU -- each pass's GEMMs
# are latency-bound (≈40 % of the MFMA rate) and could fill each other's gaps.  Measured 1.5 %
# SLOWER (profiles/r06s_train_fine_stream_ab.txt: the fused backward passes hold a CU each with 152 KB of LDS, so
# the other pass's kernels cannot share it, and the two passes' activations compete for the caches), so off: an
# A/B switch for tools/train_bench.py (bit-identical results either way, tests/test_gpu_train.py), never read from
# the environment.
FINE_STREAM = False
_FINE = {}


def _fine_stream(dev):
    key = torch.device(dev).index
    if key not in _FINE:
        _FINE[key] = torch.cuda.Stream(device=dev)
    return _FINE[key]


# ----------------------------------------------------------------------------- autograd stages
class _Encode(torch.autograd.Function):
    """encode_inputs of every sample (raycasters.py:476-555): features [N*S, F]; backward -> dL/dskts."""

    @staticmethod
    def forward(ctx, skts, model, rb, z, ray_pose, pts_noise=None):
        n, ns = z.shape
        cfg = model.cfg
        # (the view-window layout: the view part is the NJ windows, anerf.h ANERF_ENC_VIEW_WINDOWS)
        F_ = cfg.input_ch + cfg.input_ch_bones + cfg.n_joints if model.view_windows else cfg.feature_dim
        feat = torch.empty(n * ns, F_, device=z.device, dtype=torch.float32)
        n_poses = skts.shape[0]
        _lib.check(_lib.load().anerf_train_encode(model.handle, _lib.ptr(rb), rb.shape[1], n, _lib.ptr(z), ns,
                                                  _lib.ptr(skts), n_poses, _lib.ptr(ray_pose), _lib.ptr(pts_noise),
                                                  _lib.ptr(feat), _stream(z.device)), "anerf_train_encode")
        ctx.model = model
        e = torch.empty(0)
        ctx.save_for_backward(skts, rb, z, ray_pose if ray_pose is not None else e,
                              pts_noise if pts_noise is not None else e)
        ctx.has_pose = ray_pose is not None
        ctx.has_noise = pts_noise is not None
        return feat

    @staticmethod
    def backward(ctx, g_feat):
        skts, rb, z, ray_pose, pts_noise = ctx.saved_tensors
        if not ctx.needs_input_grad[0]:
            return None, None, None, None, None, None
        n, ns = z.shape
        g = torch.zeros_like(skts)
        gf = g_feat.contiguous()
        _lib.check(_lib.load().anerf_train_encode_backward(
            ctx.model.handle, _lib.ptr(rb), rb.shape[1], n, _lib.ptr(z), ns, _lib.ptr(skts), skts.shape[0],
            _lib.ptr(ray_pose if ctx.has_pose else None), _lib.ptr(pts_noise if ctx.has_noise else None),
            _lib.ptr(gf), _lib.ptr(g), _stream(z.device)), "anerf_train_encode_backward")
        return g, None, None, None, None, None


class _Composite(torch.autograd.Function):
    """NeRF.raw2outputs (nerf.py:150-205) with noise: rgb, disp, acc, weights, alpha."""

    @staticmethod
    def forward(ctx, raw, model, z, rb, noise):
        n, ns = z.shape
        dev = z.device
        f32 = dict(device=dev, dtype=torch.float32)
        rgb, disp, acc = torch.empty(n, 3, **f32), torch.empty(n, **f32), torch.empty(n, **f32)
        w, a, tr = torch.empty(n, ns, **f32), torch.empty(n, ns, **f32), torch.empty(n, ns, **f32)
        raw = raw.contiguous()
        _lib.check(_lib.load().anerf_train_composite(model.handle, _lib.ptr(raw), _lib.ptr(z), _lib.ptr(rb),
                                                     rb.shape[1], n, ns, _lib.ptr(noise), _lib.ptr(rgb),
                                                     _lib.ptr(disp), _lib.ptr(acc), _lib.ptr(w), _lib.ptr(a),
                                                     _lib.ptr(tr), _stream(dev)), "anerf_train_composite")
        ctx.model = model
        ctx.has_noise = noise is not None
        ctx.save_for_backward(raw, z, rb, noise if noise is not None else torch.empty(0), w, a, tr)
        return rgb, disp, acc, w, a

    @staticmethod
    def backward(ctx, g_rgb, g_disp, g_acc, g_w, g_a):
        raw, z, rb, noise, w, a, tr = ctx.saved_tensors
        n, ns = z.shape
        g_raw = torch.empty_like(raw)
        c = lambda t: None if t is None else t.contiguous()  # noqa: E731
        _lib.check(_lib.load().anerf_train_composite_backward(
            ctx.model.handle, _lib.ptr(raw), _lib.ptr(z), _lib.ptr(rb), rb.shape[1], n, ns,
            _lib.ptr(noise if ctx.has_noise else None), _lib.ptr(w), _lib.ptr(a), _lib.ptr(tr), _lib.ptr(c(g_rgb)),
            _lib.ptr(c(g_disp)), _lib.ptr(c(g_acc)), _lib.ptr(c(g_w)), _lib.ptr(c(g_a)), _lib.ptr(g_raw),
            _stream(z.device)), "anerf_train_composite_backward")
        return g_raw, None, None, None, None


# ----------------------------------------------------------------------------- networks
def _splitk_wgrad(gy, x):
    """gy^T x for the weight gradient of a linear layer over M = rays x samples rows: M is in the
    hundred-thousands and out x in is at most 256 x 1080, so one GEMM has too few output tiles to
    fill 256 CUs; split M into c slabs (a batched GEMM) and sum the c partial products."""
    m = gy.shape[0]
    c = 1
    while c < 64 and m % (2 * c) == 0 and m // (2 * c) >= 1024:
        c *= 2
    if c == 1:
        return gy.t().mm(x)
    return torch.bmm(gy.reshape(c, m // c, -1).transpose(1, 2), x.reshape(c, m // c, -1)).sum(0)


class _Linear(torch.autograd.Function):
    """F.linear whose weight gradient is a split-M batched GEMM (_splitk_wgrad)."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        return F.linear(x, w, b)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gx = gy.mm(w) if ctx.needs_input_grad[0] else None
        gw = _splitk_wgrad(gy, x) if ctx.needs_input_grad[1] else None
        gb = gy.sum(0) if ctx.has_b and ctx.needs_input_grad[2] else None
        return gx, gw, gb


def _lin(x, w, b=None):
    return _Linear.apply(x, w, b)


class _LinearReLU(torch.autograd.Function):
    """relu(F.linear(x, w, b)) with bias and relu in the GEMM's epilogue (torch._addmm_activation),
    so the forward launches no separate relu; backward masks by the saved output as relu does."""

    @staticmethod
    def forward(ctx, x, w, b):
        out = torch._addmm_activation(b, x, w.t(), use_gelu=False)
        ctx.save_for_backward(x, w, out)
        return out

    @staticmethod
    def backward(ctx, gy):
        x, w, out = ctx.saved_tensors
        gp = torch.ops.aten.threshold_backward(gy, out, 0.0)
        need = ctx.needs_input_grad
        gx = gp.mm(w) if need[0] else None
        gw = _splitk_wgrad(gp, x) if need[1] else None
        gb = gp.sum(0) if need[2] else None
        return gx, gw, gb


class _Linear2(torch.autograd.Function):
    """a @ wa.T + b @ wb.T + bias (the skip layer's cat([x, h]) and the view layer's cat([feature,
    views]) with the weight split by columns): the second product accumulates into the first
    GEMM's output (beta = 1), so neither direction launches a separate add."""

    @staticmethod
    def forward(ctx, a, wa, b, wb, bias, relu=False):
        ctx.has_bias = bias is not None
        ctx.relu = relu
        out = F.linear(b, wb, bias).addmm_(a, wa.t())
        if relu:
            out.relu_()
        ctx.save_for_backward(a, wa, b, wb, out if relu else None)
        return out

    @staticmethod
    def backward(ctx, g):
        a, wa, b, wb, out = ctx.saved_tensors
        if ctx.relu:
            g = torch.ops.aten.threshold_backward(g, out, 0.0)
        need = ctx.needs_input_grad
        ga = g.mm(wa) if need[0] else None
        gwa = _splitk_wgrad(g, a) if need[1] else None
        gb = g.mm(wb) if need[2] else None
        gwb = _splitk_wgrad(g, b) if need[3] else None
        gbias = g.sum(0) if ctx.has_bias and need[4] else None
        return ga, gwa, gb, gwb, gbias, None


class _SplitCols(torch.autograd.Function):
    """(x, x, views) = (feat[:, :d] twice, feat[:, d:]): x feeds layer 0 and the skip layer through
    separate outputs, so the backward writes dL/dfeat once — the two x gradients summed straight
    into its first columns, the views gradient into the rest — instead of autograd's sum of the x
    gradients plus two zero-filled full-width slice gradients and their sum."""

    @staticmethod
    def forward(ctx, feat, d):
        ctx.shape = feat.shape
        ctx.d = d
        return feat[:, :d], feat[:, :d], feat[:, d:]

    @staticmethod
    def backward(ctx, gx0, gx1, gv):
        m, f = ctx.shape
        d = ctx.d
        g = None
        for t in (gx0, gx1, gv):
            if t is not None:
                g = torch.empty(m, f, device=t.device, dtype=t.dtype)
                break
        if g is None:
            return None, None
        if gx0 is not None and gx1 is not None:
            torch.add(gx0, gx1, out=g[:, :d])
        elif gx0 is not None or gx1 is not None:
            g[:, :d] = gx0 if gx0 is not None else gx1
        else:
            g[:, :d] = 0
        if gv is not None:
            g[:, d:] = gv
        else:
            g[:, d:] = 0
        return g, None


class _Heads(torch.autograd.Function):
    """alpha_linear and feature_linear on the same h: the gradient of h is one GEMM plus a rank-1
    update accumulated into it (no separate add of two [M, W] gradients)."""

    @staticmethod
    def forward(ctx, h, wa, ba, wf, bf):
        ctx.save_for_backward(h, wa, wf)
        return F.linear(h, wa, ba), F.linear(h, wf, bf)

    @staticmethod
    def backward(ctx, g_alpha, g_feat):
        h, wa, wf = ctx.saved_tensors
        need = ctx.needs_input_grad
        if g_alpha is None:
            g_alpha = torch.zeros(h.shape[0], wa.shape[0], device=h.device, dtype=h.dtype)
        if g_feat is None:
            g_feat = torch.zeros(h.shape[0], wf.shape[0], device=h.device, dtype=h.dtype)
        gh = g_feat.mm(wf).addmm_(g_alpha, wa) if need[0] else None
        gwa = _splitk_wgrad(g_alpha, h) if need[1] else None
        gba = g_alpha.sum(0) if need[2] else None
        gwf = _splitk_wgrad(g_feat, h) if need[3] else None
        gbf = g_feat.sum(0) if need[4] else None
        return gh, gwa, gba, gwf, gbf

class Optcodes(nn.Module):
    """core/networks/embedding.py:6-46 (training: codes(idx); eval with all idx < 0: the mean code)."""

    def __init__(self, n_codes, code_ch):
        super().__init__()
        self.codes = nn.Embedding(n_codes, code_ch)

    def forward(self, idx):
        idx = idx.reshape(-1)
        if not self.training and bool((idx.max() < 0).item()):
            return self.codes.weight.mean(0, keepdim=True).expand(len(idx), -1)
        return self.codes(idx.long())


class NeRF(nn.Module):
    """Parameters with the names of core/networks/nerf.py:57-88 (state_dict-compatible); forward
    on the split feature buffer [x | views] of the encoder."""

    def __init__(self, cfg):
        super().__init__()
        W, D = cfg.netwidth, cfg.netdepth
        self.cfg = cfg
        self.skips = tuple(cfg.skips)
        self.dnet = cfg.input_ch + cfg.input_ch_bones
        self.pts_linears = nn.ModuleList(
            [nn.Linear(self.dnet, W)] + [nn.Linear(W + self.dnet if i in self.skips else W, W) for i in range(D - 1)])
        self.alpha_linear = nn.Linear(W, 1)
        self.feature_linear = nn.Linear(W, W)
        self.views_linears = nn.ModuleList([nn.Linear(W + cfg.input_ch_views + cfg.framecode_ch, W // 2)])
        self.rgb_linear = nn.Linear(W // 2, 3)
        if cfg.opt_framecode:
            self.framecodes = Optcodes(cfg.n_framecodes, cfg.framecode_size)

    # "mixed" / "bf16x6" / "bf16x3": the hand-written split-bf16 GEMMs (mlp.py / anerf_gemm.hip); "fp32":
    # torch GEMMs
    mlp = "mixed"

    def forward(self, feat, cams=None, G=None):
        """feat [M, F] = [v | r | views] -> raw [M, 4] (rgb, alpha): forward_density + forward_view.  G [rays, NJ,
        W/2] (view_factor): feat is in the view-window layout [v | r | w] (the NJ view windows) and the view
        layer's view part is sum_j w_j G_j."""
        if self.mlp in ("mixed", "mixed16", "bf16x6", "bf16x3"):
            from . import mlp as _mlp
            codes = self.framecodes(cams) if self.cfg.opt_framecode else None
            return _mlp.nerf_forward(self, feat, codes, G)
        if self.mlp != "fp32":
            raise ValueError(f"mlp={self.mlp!r}: 'mixed', 'mixed16', 'bf16x6', 'bf16x3' or 'fp32'")
        x, x_skip, views = _SplitCols.apply(feat, self.dnet)
        h = x
        for i, lin in enumerate(self.pts_linears):
            if i > 0 and (i - 1) in self.skips:  # cat([input_pts, h]) @ W.T = x @ Wx.T + h @ Wh.T
                h = _Linear2.apply(x_skip, lin.weight[:, :self.dnet], h, lin.weight[:, self.dnet:], lin.bias, True)
            else:
                h = _LinearReLU.apply(h, lin.weight, lin.bias)
        alpha, feature = _Heads.apply(h, self.alpha_linear.weight, self.alpha_linear.bias,
                                      self.feature_linear.weight, self.feature_linear.bias)
        W = feature.shape[1]
        vl = self.views_linears[0]
        nv = self.cfg.input_ch_views
        if G is not None:
            n = G.shape[0]
            g = _lin(feature, vl.weight[:, :W], vl.bias) + torch.bmm(views.reshape(n, -1, G.shape[1]), G).reshape(-1, W // 2)
            if self.cfg.opt_framecode:
                g = g + _lin(self.framecodes(cams), vl.weight[:, W + nv:])
            g = F.relu(g)
        elif self.cfg.opt_framecode:
            g = _Linear2.apply(feature, vl.weight[:, :W], views, vl.weight[:, W:W + nv], vl.bias)
            g = F.relu(g + _lin(self.framecodes(cams), vl.weight[:, W + nv:]))
        else:
            g = _Linear2.apply(feature, vl.weight[:, :W], views, vl.weight[:, W:W + nv], vl.bias, True)
        rgb = _lin(g, self.rgb_linear.weight, self.rgb_linear.bias)
        return torch.cat([rgb, alpha], -1)


class _Embed(nn.Module):
    """CutoffEmbedder state (cutoff_embedder.py:60-95): cutoff_dist (not trained), tau buffer, and
    its tau schedule (update_threshold / update_tau / get_tau, :101-102, 176-183)."""

    init_tau = 20.0

    def __init__(self, n_joints, cutoff_dist, init_alpha=None):
        """init_alpha: --freq_schedule's --init_freq (a `sched_alpha` buffer, :97-99), None without."""
        super().__init__()
        self.cutoff_dist = nn.Parameter(torch.full((n_joints,), float(cutoff_dist)), requires_grad=False)
        self.register_buffer("tau", torch.tensor(self.init_tau))
        self.freq_schedule = init_alpha is not None
        if self.freq_schedule:
            self.init_alpha = float(init_alpha)
            self.register_buffer("sched_alpha", torch.tensor(self.init_alpha))
        self._hc = {}  # host copies of the scalar buffers: name -> ((data_ptr, version), value)

    def host(self, name):
        """The float value of scalar buffer `name`.  The schedule updates below write the host copy
        with the buffer, so a training step reads nothing back from the device; a write they did
        not make (load_state_dict, .to(), a caller's in-place edit) changes the buffer's identity or
        version, and the value is read from the device once."""
        t = getattr(self, name)
        key = (t.data_ptr(), t._version)
        c = self._hc.get(name)
        if c is None or c[0] != key:
            c = (key, float(t))
            self._hc[name] = c
        return c[1]

    def _set(self, name, value):
        """buffer `name` <- value (a 0-d float32 CPU tensor), host copy included.  fill_ with the
        Python float (exact: a float32 value) launches a fill kernel and never waits on the stream, where
        a host-to-device copy_ of a pageable 0-d tensor would."""
        t = getattr(self, name)
        v = float(value)
        with torch.no_grad():
            t.fill_(v)
        self._hc[name] = ((t.data_ptr(), t._version), v)

    def get_tau(self):
        return self.host("tau")

    def update_threshold(self, global_step, tau_step, tau_rate, alpha_step=None, alpha_target=None):
        self.update_tau(global_step, tau_step, tau_rate)
        self.update_alpha(global_step, alpha_step, alpha_target)

    def update_alpha(self, global_step, step, target=None):
        """sched_alpha = init + (target - init) * global_step / (step * 1000) (cutoff_embedder.py:185-190;
        the reference's target is multires - 1 for every embedder, raycasters.py:737), in place."""
        if not self.freq_schedule:
            return
        self._set("sched_alpha", torch.tensor(self.init_alpha + (target - self.init_alpha) * global_step
                                              / float(step * 1000)))

    def update_tau(self, global_step, step, rate):
        """tau = (20 * rate ** (global_step / (step * 1000))).clamp(max=2000), the reference's own
        expression and dtype flow (cutoff_embedder.py:181-183: float32 tensor times a Python float,
        the same float32 arithmetic on the host as on the device), written into the buffer in place."""
        new = (self.init_tau * torch.ones((), dtype=self.tau.dtype) * rate ** (global_step / float(step * 1000))).clamp(
            max=2000.)
        self._set("tau", new)


def view_mix_lds_ok(n_joints, width):
    """The per-ray factors G [NJ][width] and a chunk of 32 samples' windows fit anerf_train_view_mix's and its
    backward's LDS plans (anerf.h: 64 KB) and the backward's dL/dG registers (NJ width <= 9216); width 128 -> NJ <= 72."""
    nj4 = (n_joints + 3) // 4 * 4
    fwd = 4 * (n_joints * width + 32 * n_joints)
    bwd = 4 * (nj4 * (width + 4) + 32 * (width + 4) + 32 * n_joints)
    return width % 4 == 0 and max(fwd, bwd) <= 64 * 1024 and n_joints * width <= 9216


def view_windows_ok(cfg):
    """The view-window layout (anerf.h ANERF_ENC_VIEW_WINDOWS) holds for this configuration: every view feature is
    a window times a function of the ray (a windowed view embedder -- cutoff_viewdir with use_cutoff,
    RenderConfig.view_window -- and cutoff_inputs, relray / world directions), and the per-ray factors G fit
    anerf_train_view_mix's LDS plan (view_mix_lds_ok).  Rows whose kp + bone block or width are not multiples of 4
    (NJ % 4 != 0) run on a zero-padded copy (mlp._pad_to_segments)."""
    return (cfg.view_window and cfg.cutoff_inputs and not cfg.view_angle and not cfg.staged
            and cfg.netwidth // 2 <= 128 and view_mix_lds_ok(cfg.n_joints, cfg.netwidth // 2))


class _ViewFactor(torch.autograd.Function):
    """G [rays, NJ, W/2]: the per-ray view factors of the view-window layout (anerf_train_view_factor; anerf.h
    ANERF_ENC_VIEW_WINDOWS) -- joint j's view features without their window times the view layer's view columns
    (times the --freq_schedule weights fs [input_ch_views] or None); backward -> dL/dskts, dL/d(views_linears.0.weight)."""

    @staticmethod
    def forward(ctx, skts, weight, model, rb, fs):
        n = rb.shape[0]
        cfg = model.cfg
        W = cfg.netwidth
        G = torch.empty(n, cfg.n_joints, W // 2, device=rb.device, dtype=torch.float32)
        _lib.check(_lib.load().anerf_train_view_factor(model.handle, _lib.ptr(rb), rb.shape[1], n, _lib.ptr(skts),
                                                       skts.shape[0], None, weight.data_ptr() + 4 * W,
                                                       weight.stride(0), W // 2, _lib.ptr(fs), _lib.ptr(G),
                                                       _stream(rb.device)), "anerf_train_view_factor")
        ctx.model = model
        ctx.save_for_backward(skts, weight, rb, fs if fs is not None else torch.empty(0))
        ctx.has_fs = fs is not None
        return G

    @staticmethod
    def backward(ctx, gG):
        skts, weight, rb, fs = ctx.saved_tensors
        W = ctx.model.cfg.netwidth
        gs, gw = torch.zeros_like(skts), torch.zeros_like(weight)
        cfg = ctx.model.cfg
        lib = _lib.load()
        need = lib.anerf_train_view_factor_workspace(rb.shape[0], cfg.n_joints, cfg.multires_views, W // 2)
        ws = torch.empty(max(need, 16), device=rb.device, dtype=torch.uint8)
        _lib.check(lib.anerf_train_view_factor_backward(
            ctx.model.handle, _lib.ptr(rb), rb.shape[1], rb.shape[0], _lib.ptr(skts), skts.shape[0], None,
            weight.data_ptr() + 4 * W, weight.stride(0), W // 2, _lib.ptr(fs if ctx.has_fs else None),
            _lib.ptr(gG.contiguous()), _lib.ptr(gs), gw.data_ptr() + 4 * W, _lib.ptr(ws), ws.numel(),
            _stream(rb.device)),
            "anerf_train_view_factor_backward")
        return (gs if ctx.needs_input_grad[0] else None), (gw if ctx.needs_input_grad[1] else None), None, None, None


class TrainRayCaster(nn.Module):
    """Trainable RayCaster (core/raycasters.py:326-474): nn.Module with the reference's
    state_dict layout (network_fn.*, network_fine.*, embed_fn.*, embeddirs_fn.*).  In training
    mode `forward`/`render_rays` run the stochastic, differentiable render path; in eval mode
    they delegate to the fused HIP render kernel (weights repacked when they changed)."""

    def __init__(self, cfg, ckpt=None, device=None, mlp="mixed"):
        """mlp: arithmetic of the training MLP — "mixed" (hand-written split-bf16 GEMMs on the MFMA pipe,
        mlp.py: an fp32-accurate bf16x6 forward, a bf16x3 backward), "bf16x6" (fp32-accurate both
        ways), "bf16x3" (~16-bit operands both ways) or "fp32" (torch GEMMs); the eval delegate
        uses cfg.precision."""
        super().__init__()
        self.cfg = cfg.validate()
        if not (1 <= cfg.multires <= 10 and 0 <= cfg.multires_views <= 4):
            # (the render kernel's zero-padded instances; the encoder backward has tuned instances for
            # multires 7 / 10 x multires_views 0 / 4 and a generic one for the rest)
            raise NotImplementedError("training: multires 1-10 and multires_views 0-4")
        if mlp not in ("mixed", "mixed16", "bf16x6", "bf16x3", "fp32"):
            raise ValueError(f"mlp={mlp!r}: 'mixed', 'mixed16', 'bf16x6', 'bf16x3' or 'fp32'")
        if isinstance(device, (str, torch.device)):
            dev = torch.device(device)  # (a CPU device holds the parameters only: checkpoints, no rendering)
        else:
            dev = torch.device(f"cuda:{torch.cuda.current_device() if device is None else int(device)}")
        self.network_fn = NeRF(cfg)
        # single_net: network_fine IS network_fn (core/raycasters.py:98-104); the module is registered
        # under both names, so state_dict() has both keys, as the reference's does
        if cfg.N_importance > 0:
            self.network_fine = self.network_fn if cfg.single_net else NeRF(cfg)
        else:
            self.network_fine = None
        # fresh models: cutoff_mm (default 500, run_nerf.py:416) x ext_scale (raycasters.py:33), tau 20
        cut = float(cfg.extra.get("cutoff_mm", 500.0)) * cfg.ext_scale
        alpha0 = cfg.init_freq if cfg.freq_schedule else None
        self.embed_fn = _Embed(3 if cfg.kp_query else cfg.n_joints, cut, alpha0)  # (querypts: cutoff_dim 3)
        self.embeddirs_fn = _Embed(cfg.n_joints, cut, alpha0)
        # --cutoff_bones: the bone embedder is a CutoffEmbedder too (raycasters.py:52-64), with its own
        # tau schedule (update_embed_fns, :745-747); otherwise it has no state
        self.embedbones_fn = _Embed(cfg.n_joints, cut, alpha0) if cfg.bone_window else None
        for net in (self.network_fn, self.network_fine):
            if net is not None:
                net.mlp = mlp
        if ckpt is not None:
            self.load_checkpoint(ckpt)
        self.to(dev)
        self._dev = dev
        self._consts = None  # DeviceModel holding the encoder / density constants (cutoffs, tau, B)
        self._consts_embed = None
        self._eval = None
        self._eval_version = None
        self._eval_embed = None
        self._fs_cache = None  # (sched_alpha values, device feature scales)

    @property
    def module(self):
        """The reference's Trainer reaches the caster through nn.DataParallel's `.module`
        (core/trainer.py:263-270); here the caster is its own module."""
        return self

    def update_embed_fns(self, global_step, args):
        """core/raycasters.py:731-748: the tau schedule of both embedders (args.cutoff_step,
        args.cutoff_rate) and, with --freq_schedule, their sched_alpha (args.freq_schedule_step,
        target multires - 1); the kernels pick the new tau up at the next launch, the new schedule
        weights at the next feature product."""
        for e in self._embedders():
            e.update_threshold(global_step, args.cutoff_step, args.cutoff_rate,
                               getattr(args, "freq_schedule_step", 5), getattr(args, "multires", 7) - 1)

    def _embedders(self):
        return (self.embed_fn, self.embeddirs_fn) + ((self.embedbones_fn,) if self.embedbones_fn is not None else ())

    # -- checkpoints in the reference's key layout (raycasters.py:752-788)
    def load_checkpoint(self, ck):
        def t(v):
            return torch.as_tensor(v).float()
        self.network_fn.load_state_dict({k: t(v) for k, v in ck["network_fn_state_dict"].items()})
        # (single_net: the same module again; the fine keys load last and win, as in raycasters.py:768-788)
        if self.network_fine is not None and "network_fine_state_dict" in ck:
            self.network_fine.load_state_dict({k: t(v) for k, v in ck["network_fine_state_dict"].items()})
        mods = [(self.embed_fn, "embed_state_dict"), (self.embeddirs_fn, "embeddirs_state_dict")]
        if self.embedbones_fn is not None:
            mods.append((self.embedbones_fn, "embedbones_state_dict"))
        for mod, key in mods:
            mod.load_state_dict({k: t(v) for k, v in ck[key].items()})
        self._consts = None
        self._eval = None

    def checkpoint(self):
        """The reference's checkpoint layout (raycasters.py:752-766) with CPU tensors: torch.save of it
        loads with torch.load(weights_only=True) and nn.Module.load_state_dict on either side."""
        def sd(m):
            return {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
        ck = {"network_fn_state_dict": sd(self.network_fn), "embed_state_dict": sd(self.embed_fn),
              "embedbones_state_dict": sd(self.embedbones_fn) if self.embedbones_fn is not None else {},
              "embeddirs_state_dict": sd(self.embeddirs_fn)}
        if self.network_fine is not None:
            ck["network_fine_state_dict"] = sd(self.network_fine)
        return ck

    def _version(self):
        """Identity + version of every network tensor (a tensor replaced by assignment changes the
        identity, an in-place update the version) and of the schedule buffers (folded into the eval
        caster's packed weights)."""
        nets = [self.network_fn] + ([self.network_fine] if self.network_fine is not None else [])
        sched = [e.sched_alpha for e in (self.embed_fn, self.embeddirs_fn) if e.freq_schedule]
        return tuple((p.data_ptr(), p._version) for n in nets for p in n.parameters()) + tuple(
            (t.data_ptr(), t._version) for t in sched)

    def _feature_scale(self):
        """--freq_schedule: the per-column schedule weights of the MLP input (config.feature_scales at
        the current sched_alpha), on the device; None without a schedule."""
        if not self.cfg.freq_schedule:
            return None
        eb = self.embedbones_fn
        a = (self.embed_fn.host("sched_alpha"), self.embeddirs_fn.host("sched_alpha"),
             eb.host("sched_alpha") if eb is not None and eb.freq_schedule else None)
        if self._fs_cache is None or self._fs_cache[0] != a or self._fs_cache[1].device != self._dev:
            self._fs_cache = (a, torch.from_numpy(feature_scales(self.cfg, *a)).to(self._dev))
        return self._fs_cache[1]

    def _embed_version(self):
        """(tau versions, cutoff_dist versions) of both embedders: the tau schedule moves the first
        every step, the second only changes on a load or a caller's edit."""
        es = self._embedders()
        return (tuple((e.tau.data_ptr(), e.tau._version) for e in es),
                tuple((e.cutoff_dist.data_ptr(), e.cutoff_dist._version) for e in es))

    def _embed_state(self):
        """(embed_fn, embeddirs_fn, embedbones_fn or None) states for DeviceModel.set_embed."""
        return tuple(None if e is None else {"tau": e.host("tau"), "cutoff_dist": e.cutoff_dist}
                     for e in (self.embed_fn, self.embeddirs_fn, self.embedbones_fn))

    def _sync_embed(self, model, seen):
        """New tau / cutoff_dist into a DeviceModel without a repack; a tau-only change (the schedule,
        every step) is a host-side field write, no device synchronisation or copy."""
        v = self._embed_version()
        if v != seen:
            e, ev, eb = self._embed_state()
            model.set_embed(e, ev, cutoffs=v[1] != seen[1], embedbones_sd=eb)
        return v

    # the training stages' view-window layout where the configuration allows it (view_windows_ok): the encoder
    # writes NJ windows instead of 3 NJ (1 + 2 multires_views) view features, the view layer reads them through the
    # per-ray factors G (view_factor); False: the full view columns
    _view_windows = True

    @property
    def view_windows(self):
        return self._view_windows

    @view_windows.setter
    def view_windows(self, on):
        """ the layout lives in the DeviceModel of the encoder constants: a change drops it, so the next
        pass builds it in the new layout (a plain class attribute was read once and later changes were ignored)."""
        on = bool(on)
        if on != self._view_windows:
            self._consts = None
            self._consts_embed = None
        self._view_windows = on

    def _constants(self):
        if self._consts is None:
            self._consts = DeviceModel(self.cfg, self.checkpoint(), device=self._dev.index,
                                       view_windows=self.view_windows and view_windows_ok(self.cfg))
            self._consts_embed = self._embed_version()
        else:
            self._consts_embed = self._sync_embed(self._consts, self._consts_embed)
        return self._consts

    @property
    def model(self):
        """The DeviceModel holding the encoder / compositing constants (device index for `render`)."""
        return self._constants()

    def weights_changed(self):
        """Force the next eval render to repack the weights: for updates the version counters do not show (an
        optimizer that writes the parameters in place without advancing them, e.g. torch's fused Adam)."""
        self._eval_version = None

    def eval_caster(self):
        """The fused eval RayCaster over the current weights (repacked only after they changed; a new
        tau / cutoff reaches it without a repack); for a staged encoder (cfg.staged) the training stages
        run deterministically instead (StagedCaster)."""
        if self.cfg.staged:
            return StagedCaster(self)
        from .raycaster import RayCaster
        v = self._version()
        if self._eval is None or v != self._eval_version:
            self._eval = RayCaster(self.cfg, self.checkpoint(), device=self._dev.index)
            self._eval_version = v
            self._eval_embed = self._embed_version()
        else:
            self._eval_embed = self._sync_embed(self._eval.model, self._eval_embed)
        return self._eval

    def forward(self, *args, fwd_type="", **kwargs):
        if fwd_type in ("density", "mesh", "density_color"):  # (core/raycasters.py:349-359)
            return self.eval_caster()(*args, fwd_type=fwd_type, **kwargs)
        if not self.training:
            with torch.no_grad():
                return self.eval_caster().render_rays(*args, **kwargs)
        return self.render_rays(*args, **kwargs)

    # -- the training render path
    def render_rays(self, ray_batch, N_samples, kp_batch=None, skts=None, cyls=None, bones=None, cams=None,
                    subject_idxs=None, retraw=False, lindisp=False, perturb=0., N_importance=0, network_fine=None,
                    raw_noise_std=0., ray_noise_std=0., verbose=False, ext_scale=0.001, pytest=False,
                    preproc_kwargs=None, nerf_type="nerf", rand=None, chunk=None):
        """core/raycasters.py:361-474 with autograd: gradients reach the networks' parameters and
        `skts` (when it requires grad).  `rand` overrides the random draws (module docstring)."""
        if subject_idxs is not None:  # (as the reference's NeRF.forward split, core/networks/nerf.py:135-137)
            raise RuntimeError("subject_idxs: the NeRF input has one column more than "
                               "input_ch + input_ch_bones + input_ch_views + cam_ch (core/networks/nerf.py:135)")
        if skts is None or cyls is None:
            raise ValueError("skts and cyls are required")
        cfg = self.cfg
        B = cfg.density_scale
        if preproc_kwargs and preproc_kwargs.get("density_scale", B) != B:
            raise ValueError("density_scale differs from the model's configuration")
        dev = self._dev
        rand = rand or {}
        model = self._constants()
        rb = ray_batch.to(dev, torch.float32).detach().contiguous()
        n = rb.shape[0]
        S, I = int(N_samples), int(N_importance)
        nj = cfg.n_joints
        if I > 0 and self.network_fine is None:
            raise ValueError("N_importance > 0 needs a fine network")
        # skeletons: one per ray (the reference's layout, gradients flow back through any expand)
        sk = skts.to(dev, torch.float32)
        if sk.dim() == 3:
            sk = sk.unsqueeze(0)
        sk = sk.expand(n, nj, 4, 4).contiguous() if sk.shape[0] != n else sk.contiguous()
        cyl = cyls.to(dev, torch.float32).detach()
        cyl = cyl.expand(n, 5).contiguous() if cyl.dim() == 1 or cyl.shape[0] != n else cyl.contiguous()
        pose = torch.arange(n, device=dev, dtype=torch.int32)
        # near / far in the bounding cylinder (+ the chunk NaN fill)
        nearv = torch.empty(n, device=dev, dtype=torch.float32)
        farv = torch.empty(n, device=dev, dtype=torch.float32)
        ws, need = model.workspace(n, S, 0)
        _lib.check(_lib.load().anerf_near_far(_lib.ptr(rb), rb.shape[1], n, _lib.ptr(cyl), n, _lib.ptr(pose),
                                              int(chunk or max(n, 1)), _lib.ptr(nearv), _lib.ptr(farv),
                                              _lib.ptr(ws), need, _stream(dev)), "anerf_near_far")
        stochastic = perturb > 0
        t_rand = rand.get("t_rand")
        if stochastic and t_rand is None:
            t_rand = torch.rand(n, S, device=dev)
        t_rand = t_rand.to(dev, torch.float32).contiguous() if stochastic else None
        z = torch.empty(n, S, device=dev, dtype=torch.float32)
        _lib.check(_lib.load().anerf_train_samples(_lib.ptr(nearv), _lib.ptr(farv), n, S, _lib.ptr(t_rand),
                                                   _lib.ANERF_FLAG_LINDISP if lindisp else 0, _lib.ptr(z),
                                                   _stream(dev)), "anerf_train_samples")
        cam_t = None
        if cfg.opt_framecode:
            if cams is None:
                raise ValueError("this model uses framecodes: cams are required")
            cam_t = cams.to(dev).reshape(n)

        def noise_for(key, ns):
            if raw_noise_std <= 0:
                return None
            g = rand.get(key)
            g = torch.randn(n, ns, device=dev) if g is None else g.to(dev, torch.float32)
            return (g * raw_noise_std * B).contiguous()

        def pts_noise_for(key, ns):
            """sample_pts / sample_pts_is' `randn_like(pts) * ray_noise_std` (raycasters.py:660-661, 673-674)."""
            if ray_noise_std <= 0:
                return None
            g = rand.get(key)
            g = torch.randn(n, ns, 3, device=dev) if g is None else g.to(dev, torch.float32)
            return (g * ray_noise_std).contiguous()

        fscale = self._feature_scale()
        fs_view = None
        if model.view_windows and fscale is not None:  # (the view columns' schedule weights go into G)
            dnet = cfg.input_ch + cfg.input_ch_bones
            fs_view = fscale[dnet:].contiguous()
            fscale = torch.cat([fscale[:dnet], fscale.new_ones(nj)])

        def raw_of(net, zz, pn=None):
            ns = zz.shape[1]
            feat = _Encode.apply(sk, model, rb, zz, None, pn)
            if fscale is not None:  # (embedded * get_schedule_w(), cutoff_embedder.py:150; autograd scales dL/dfeat)
                feat = feat * fscale
            G = _ViewFactor.apply(sk, net.views_linears[0].weight, model, rb, fs_view) if model.view_windows else None
            return net(feat, None if cam_t is None else cam_t.repeat_interleave(ns), G).reshape(n, ns, 4)

        def composite(raw, zz, noise):
            return _Composite.apply(raw, model, zz, rb, noise)

        pn0 = pts_noise_for("pts_noise0", S)
        raw0 = raw_of(self.network_fn, z, pn0)
        rgb, disp, acc, w, a = composite(raw0, z, noise_for("noise0", S))
        out = {"rgb_map": rgb, "disp_map": disp, "acc_map": acc, "alpha": a}
        if I > 0:
            u = rand.get("u")
            if stochastic and u is None:
                u = torch.rand(n, I, device=dev)
            u = u.to(dev, torch.float32).contiguous() if stochastic else None
            z_all = torch.empty(n, S + I, device=dev, dtype=torch.float32)
            want_idx = cfg.single_net or pn0 is not None
            sidx = torch.empty(n, S + I, device=dev, dtype=torch.int32) if want_idx else None
            wd = w.detach().contiguous()
            _lib.check(_lib.load().anerf_train_importance(_lib.ptr(z), _lib.ptr(wd), n, S, I, _lib.ptr(u),
                                                          int(cfg.single_net), _lib.ptr(z_all), _lib.ptr(sidx),
                                                          _stream(dev)), "anerf_train_importance")
            # the new samples' points get their own ray noise; the merged coarse samples keep theirs
            # (the reference merges the coarse encodings, raycasters.py:456-466)
            pn_is = pts_noise_for("pts_noise1", I)
            if cfg.single_net:
                # raycasters.py:462-468: the one network on the I new samples only, then
                # raw = cat([raw, raw_is])[sorted_idx] (gradients reach both through the gather)
                si = sidx.long()
                z_is = torch.empty_like(z_all).scatter_(1, si, z_all)[:, S:].contiguous()
                raw_cat = torch.cat([raw0, raw_of(self.network_fn, z_is, pn_is)], 1)
                raw1 = torch.gather(raw_cat, 1, si[..., None].expand(-1, -1, 4))
            else:
                pn1 = None
                if pn0 is not None:
                    pn1 = torch.gather(torch.cat([pn0, pn_is], 1), 1,
                                       sidx.long()[..., None].expand(-1, -1, 3)).contiguous()
                noise1 = noise_for("noise1", S + I)
                if FINE_STREAM and torch.is_grad_enabled():
                    main = torch.cuda.current_stream(dev)
                    fine = _fine_stream(dev)
                    fine.wait_stream(main)
                    for t in (rb, sk, z_all, pn1, noise1, cam_t, fscale, fs_view):  # (made on main, read on fine)
                        if t is not None:
                            t.record_stream(fine)
                    with torch.cuda.stream(fine):
                        raw1 = raw_of(self.network_fine, z_all, pn1)
                        rgb1, disp1, acc1, w1, a1 = composite(raw1, z_all, noise1)
                    main.wait_stream(fine)
                    for t in (rgb1, disp1, acc1, w1, a1):  # (made on fine, read on main)
                        t.record_stream(main)
                else:
                    raw1 = raw_of(self.network_fine, z_all, pn1)
                    rgb1, disp1, acc1, w1, a1 = composite(raw1, z_all, noise1)
            if cfg.single_net:
                rgb1, disp1, acc1, w1, a1 = composite(raw1, z_all, noise_for("noise1", S + I))
            out = {"rgb_map": rgb1, "disp_map": disp1, "acc_map": acc1, "alpha": a1,
                   "rgb0": rgb, "disp0": disp, "acc0": acc, "alpha0": a}
        return out


class StagedCaster:
    """Eval renders of a staged-encoder model (RenderConfig.staged: --multires_bones > 0, --kp_dist_type
    relpos | querypts, --view_type rayangle; include/anerf.h) on the training stages: TrainRayCaster.render_rays with
    perturb 0 and no noise -- the reference's eval path (core/raycasters.py:361-474, deterministic
    sample_pdf) -- under no_grad, the MLP on the trainable networks' GEMMs (mlp.py; the default "mixed"
    forward is the fp32-accurate bf16x6).  Density queries (fwd_type 'density' / 'mesh',
    raycasters.py:579-648) encode the points the same way and read alpha_linear."""

    def __init__(self, trainable):
        self._t = trainable

    @contextlib.contextmanager
    def _eval_mode(self):
        """The trainable in eval mode for the call, its mode restored afterwards: called from a
        TrainRayCaster still in training mode (forward(fwd_type='density'), an eval render with cams = -1) the
        framecodes must take the eval-mode mean code (FrameCodes, gated on `training`), as the fused caster does."""
        was = self._t.training
        self._t.eval()
        try:
            yield
        finally:
            self._t.train(was)

    @property
    def model(self):
        return self._t.model

    @property
    def cfg(self):
        return self._t.cfg

    def __call__(self, *args, fwd_type="", **kwargs):
        if fwd_type == "density":
            return self.render_pts_density(*args, **kwargs)
        if fwd_type == "mesh":
            return self.render_mesh_density(*args, **kwargs)
        if fwd_type == "density_color":
            raise AssertionError("need to have texture layer!")
        return self.render_rays(*args, **kwargs)

    @torch.no_grad()
    def render_rays(self, ray_batch, N_samples, kp_batch=None, skts=None, cyls=None, bones=None, cams=None,
                    subject_idxs=None, retraw=False, lindisp=False, perturb=0., N_importance=0, network_fine=None,
                    raw_noise_std=0., ray_noise_std=0., verbose=False, ext_scale=0.001, pytest=False,
                    preproc_kwargs=None, nerf_type="nerf", chunk=None, ret_alpha=True, **unused):
        if perturb or raw_noise_std or ray_noise_std:
            raise NotImplementedError("the eval caster renders deterministically; train() for stochastic renders")
        with self._eval_mode():
            out = self._t.render_rays(ray_batch, N_samples, kp_batch=kp_batch, skts=skts, cyls=cyls, bones=bones,
                                      cams=cams, subject_idxs=subject_idxs, lindisp=lindisp, perturb=0.,
                                      N_importance=N_importance, preproc_kwargs=preproc_kwargs, chunk=chunk)
        out = {k: v.detach() for k, v in out.items()}
        if not ret_alpha:
            out.pop("alpha", None)
            out.pop("alpha0", None)
        return out

    @torch.no_grad()
    def render_pts_density(self, pts, kps, skts, bones, render_kwargs=None, subject_idxs=None, netchunk=1024 * 64,
                           network=None, color=False, v=None):
        """alpha_linear at points (raycasters.py:597-648): the points as zero-length rays through the
        training encoder (the view part, which the density does not read, from a fixed direction)."""
        if color:
            raise NotImplementedError("color=True needs texture layers the NeRF model does not have")
        if v is not None:
            raise NotImplementedError("precomputed kp inputs (v) are not supported")
        t = self._t
        dev = t._dev
        nj = self.cfg.n_joints
        p = torch.as_tensor(pts).to(dev, torch.float32)
        shape = p.shape[:-1]
        p = p.reshape(-1, 3)
        n = p.shape[0]
        sk = torch.as_tensor(skts).to(dev, torch.float32).reshape(-1, nj, 4, 4)[:1].contiguous()
        if network in (None, -1):
            net = t.network_fine if t.network_fine is not None else t.network_fn
        elif network in ("coarse", 0):
            net = t.network_fn
        elif network in ("fine", 1):
            if t.network_fine is None:
                raise ValueError("this model has no fine network")
            net = t.network_fine
        else:
            raise ValueError(f"network must be None, 'coarse' or 'fine', got {network!r}")
        rb = torch.zeros(n, 11, device=dev, dtype=torch.float32)
        rb[:, :3] = p
        rb[:, 5] = 1.0
        z = torch.zeros(n, 1, device=dev, dtype=torch.float32)
        feat = _Encode.apply(sk, t._constants(), rb, z, torch.zeros(n, device=dev, dtype=torch.int32), None)
        fs = t._feature_scale()
        if fs is not None:
            feat = feat * fs
        cams = torch.zeros(n, device=dev, dtype=torch.long) if self.cfg.opt_framecode else None
        with self._eval_mode():
            return net(feat, cams)[:, 3:4].reshape(*shape, 1)

    @torch.no_grad()
    def render_mesh_density(self, kps, skts, bones, subject_idxs=None, radius=1.0, res=64, render_kwargs=None,
                            netchunk=1024 * 64, v=None, network=None):
        """raycasters.py:579-595: np.meshgrid of linspace(-radius, radius, res + 1) around kps[0, 0]."""
        t = np.linspace(-radius, radius, int(res) + 1)
        grid = np.stack(np.meshgrid(t, t, t), axis=-1).astype(np.float32)
        kp0 = torch.as_tensor(kps).to(torch.float32).reshape(-1, 3)[0].cpu()
        pts = torch.from_numpy(grid.reshape(-1, 3)) + kp0
        raw = self.render_pts_density(pts, kps, skts, bones, network=network, v=v)
        return raw.reshape(*grid.shape[:-1])


def _img_loss(name, x, y, reduction="mean", beta=0.1):
    """get_loss_fn / get_reg_fn (core/trainer.py:10-58, 147-170): MSE (img2mse), L1 (img2l1),
    Huber (F.smooth_l1_loss with beta), BCE (acc2bce, eps 1e-8; reduction 'off' = the mean over
    y < 1)."""
    if name == "MSE":
        d = (x - y) ** 2
    elif name == "L1":
        d = (x - y).abs()
    elif name == "Huber":
        return F.smooth_l1_loss(x, y, reduction=reduction, beta=beta)
    elif name == "BCE":
        d = -(y * torch.log(x + 1e-8) + (1.0 - y) * torch.log(1 - x + 1e-8))
        if reduction == "off":
            return torch.mean(d[y < 1.0])
    else:
        raise NotImplementedError(f"loss {name!r}")
    if reduction == "mean":
        return torch.mean(d)
    if reduction == "sum":
        return torch.sum(d)
    return d


def nerf_loss(preds, target, bgs=None, use_background=False, coarse_weight=1.0, loss_fn="MSE", loss_beta=0.1,
              reg_fn=None, reg_coef=0.1, fgs=None, return_dict=False):
    """Trainer._compute_nerf_loss (core/trainer.py:350-381) for the fine and the coarse outputs, summed
    as Trainer.compute_loss sums them (:325-345): the rgb loss (`loss_fn` MSE / L1 / Huber with
    `loss_beta`) of the prediction composited over the background with (1 - acc) when
    use_background, the coarse one times `coarse_weight`; with `reg_fn` (BCE / L1 / MSE) the
    regulariser reg_fn(acc, fgs[..., 0], reduction='off') * reg_coef per pass (not coarse-weighted).
    Returns the total, or (total, {name: loss}) with return_dict (the reference's loss_dict keys)."""
    if reg_fn is not None and fgs is None:
        raise ValueError("reg_fn needs the batch's fgs")

    def one(rgb, acc, coarse, out):
        if use_background:
            rgb = rgb + (1.0 - acc)[..., None] * (1.0 if bgs is None else bgs)
        loss = _img_loss(loss_fn, rgb, target, "mean", loss_beta)
        if coarse:
            loss = loss * coarse_weight
        out["rgb_loss0" if coarse else "rgb_loss"] = loss
        if reg_fn is not None:
            out["reg_loss0" if coarse else "reg_loss"] = _img_loss(reg_fn, acc, fgs[..., 0], "off") * reg_coef

    parts = {}
    one(preds["rgb_map"], preds["acc_map"], False, parts)
    if "rgb0" in preds:
        one(preds["rgb0"], preds["acc0"], True, parts)
    total = 0.0
    for v in parts.values():
        total = total + v
    return (total, parts) if return_dict else total


__all__ = ["TrainRayCaster", "NeRF", "nerf_loss", "RenderConfig"]

"""Device model: the reference checkpoint's weights packed once into HBM.

Replaces the weight side of `create_raycaster` / `RayCaster.load_state_dict`
(`core/raycasters.py:17-184, 768-788`): it takes the same state-dict keys
(`network_fn_state_dict`, `network_fine_state_dict`, `embed_state_dict`,
`embeddirs_state_dict`, `core/raycasters.py:752-766`) and hands host copies to
`anerf_model_create`, which permutes them into the MFMA operand order and uploads them
once (the reference's DataParallel re-broadcasts every weight on every forward).
"""
import ctypes

import numpy as np
import torch

from . import _lib
from .config import feature_scales


def _np(x):
    if isinstance(x, torch.Tensor):
        x = x.detach().cpu().numpy()
    return np.ascontiguousarray(np.asarray(x, dtype=np.float32))


class DeviceModel:
    """Owns one `anerf_model*` on one GPU."""

    def __init__(self, cfg, ckpt, device=None, view_windows=False):
        """view_windows: the training stages' view-window layout (anerf.h ANERF_ENC_VIEW_WINDOWS; the trainable
        TrainRayCaster's own model)."""
        cfg.validate()
        self.cfg = cfg
        lib = _lib.load()
        if device is None:
            device = torch.cuda.current_device()
        self.device = int(device)
        self._keep = []
        d = _lib.ModelDesc()
        d.n_joints, d.net_depth, d.net_width = cfg.n_joints, cfg.netdepth, cfg.netwidth
        d.skip = cfg.skips[0]
        d.multires, d.multires_views = cfg.multires, cfg.multires_views
        # (cutoff_viewdir as the reference builds it: a windowed view embedder only under use_cutoff too,
        # RenderConfig.view_window; anerf_model_create applies the same rule to a raw descriptor)
        d.use_cutoff, d.cutoff_inputs, d.cutoff_viewdir = int(cfg.use_cutoff), int(cfg.cutoff_inputs), int(
            cfg.view_window)
        d.framecode_ch = cfg.framecode_ch
        d.n_framecodes = cfg.n_framecodes if cfg.opt_framecode else 0
        d.density_softplus = int(cfg.density_type == "softplus")
        d.softplus_shift, d.density_scale = cfg.softplus_shift, cfg.density_scale
        fine_sd = ckpt.get("network_fine_state_dict")
        coarse_sd = ckpt["network_fn_state_dict"]
        if cfg.single_net:
            # network_fine IS network_fn (core/raycasters.py:101-104); RayCaster.load_state_dict loads
            # network_fn_state_dict, then network_fine_state_dict into the same module (:768-788), so
            # the latter wins when a checkpoint has both
            if fine_sd is not None:
                coarse_sd = fine_sd
            fine_sd = None
        d.single_net = int(cfg.single_net)
        d.encoder_flags = ((_lib.ANERF_ENC_CUT_TO_DIST if cfg.cut_to_dist else 0) |
                           (_lib.ANERF_ENC_CUTOFF_SHIFT if cfg.cutoff_shift else 0) |
                           (_lib.ANERF_ENC_CUTOFF_BONES if cfg.bone_window else 0) |
                           (_lib.ANERF_ENC_VIEW_RAW if cfg.extra.get("view_type", "relray") == "world" else 0) |
                           (_lib.ANERF_ENC_KP_RELPOS if cfg.kp_relpos else 0) |
                           (_lib.ANERF_ENC_VIEW_ANGLE if cfg.view_angle else 0) |
                           (_lib.ANERF_ENC_KP_QUERYPTS if cfg.kp_query else 0) |
                           (_lib.ANERF_ENC_VIEW_WINDOWS if view_windows else 0))
        self.view_windows = bool(view_windows)
        d.multires_bones = cfg.multires_bones
        # (the C side windows the bare bone directions under the reference's condition, cutoff_inputs too:
        # anerf.h, ANERF_ENC_CUTOFF_BONES)
        self.staged = cfg.staged  # (no packed weights: the training stages serve the model, anerf.h)
        d.has_fine = int(fine_sd is not None and cfg.N_importance > 0)
        self.has_fine = bool(d.has_fine)
        e, ev = ckpt["embed_state_dict"], ckpt["embeddirs_state_dict"]
        # --freq_schedule: the embedders' per-frequency weights are folded into the weight columns
        # that consume those features (layer 0, the skip layer's x part, the view layer's direction
        # part) -- the same products up to one rounding of w * s (config.feature_scales)
        self._fs = None
        if cfg.freq_schedule and not cfg.staged:
            if "sched_alpha" not in e or "sched_alpha" not in ev:
                raise ValueError("freq_schedule: the checkpoint's embed state has no sched_alpha buffer")
            self._fs = feature_scales(cfg, float(_np(e["sched_alpha"]).reshape(-1)[0]),
                                      float(_np(ev["sched_alpha"]).reshape(-1)[0]))
        coarse = self._net(coarse_sd) if not cfg.staged else None
        fine = self._net(fine_sd) if d.has_fine and not cfg.staged else None
        emb = _lib.EmbedParams()
        emb.cutoff_dist, emb.tau = self._p(e["cutoff_dist"]), float(_np(e["tau"]).reshape(-1)[0])
        emb.cutoff_dist_v, emb.tau_v = self._p(ev["cutoff_dist"]), float(_np(ev["tau"]).reshape(-1)[0])
        if cfg.bone_window:  # --cutoff_bones: the bone CutoffEmbedder's state (embedbones_state_dict)
            eb = ckpt.get("embedbones_state_dict") or {}
            if "cutoff_dist" not in eb or "tau" not in eb:
                raise ValueError("cutoff_bones: the checkpoint's embedbones_state_dict has no cutoff_dist / tau")
            emb.cutoff_dist_b, emb.tau_b = self._p(eb["cutoff_dist"]), float(_np(eb["tau"]).reshape(-1)[0])
        h = ctypes.c_void_p()
        rc = lib.anerf_model_create(ctypes.byref(d), ctypes.byref(coarse) if coarse else None,
                                    ctypes.byref(fine) if fine else None,
                                    ctypes.byref(emb), self.device, ctypes.byref(h))
        _lib.check(rc, "anerf_model_create")
        self.handle = h
        self._keep = []  # host copies are no longer needed once packed
        self._ws = None

    def _p(self, a):
        a = _np(a)
        self._keep.append(a)
        return a.ctypes.data_as(_lib.c_f)

    def _net(self, sd):
        cfg = self.cfg
        fs = self._fs
        dnet = cfg.input_ch + cfg.input_ch_bones
        w = _lib.NetWeights()
        for i in range(cfg.netdepth):
            wi = sd[f"pts_linears.{i}.weight"]
            if fs is not None and (i == 0 or i == cfg.skips[0] + 1):  # (inputs [x] / [x | h])
                wi = _np(wi).copy()
                wi[:, :dnet] *= fs[None, :dnet]
            w.pts_w[i] = self._p(wi)
            w.pts_b[i] = self._p(sd[f"pts_linears.{i}.bias"])
        w.alpha_w, w.alpha_b = self._p(sd["alpha_linear.weight"]), self._p(sd["alpha_linear.bias"])
        w.feature_w, w.feature_b = self._p(sd["feature_linear.weight"]), self._p(sd["feature_linear.bias"])
        wv = sd["views_linears.0.weight"]
        if fs is not None:  # (inputs [feature | views | framecode])
            wv = _np(wv).copy()
            wv[:, cfg.netwidth:cfg.netwidth + cfg.input_ch_views] *= fs[None, dnet:]
        w.views_w, w.views_b = self._p(wv), self._p(sd["views_linears.0.bias"])
        w.rgb_w, w.rgb_b = self._p(sd["rgb_linear.weight"]), self._p(sd["rgb_linear.bias"])
        w.codes = self._p(sd["framecodes.codes.weight"]) if cfg.opt_framecode else None
        return w

    def set_embed(self, embed_sd, embeddirs_sd, cutoffs=True, embedbones_sd=None):
        """New tau (and cutoff_dist) of the embedders (the bone one with --cutoff_bones) without
        repacking the weights (anerf_model_set_embed): the training tau schedule."""
        emb = _lib.EmbedParams()
        keep = []
        def scalar(v):  # (a host float passes as is: no device read)
            return v if isinstance(v, float) else float(_np(v).reshape(-1)[0])
        emb.tau = scalar(embed_sd["tau"])
        emb.tau_v = scalar(embeddirs_sd["tau"])
        if cutoffs:
            a, b = _np(embed_sd["cutoff_dist"]), _np(embeddirs_sd["cutoff_dist"])
            keep += [a, b]
            emb.cutoff_dist, emb.cutoff_dist_v = a.ctypes.data_as(_lib.c_f), b.ctypes.data_as(_lib.c_f)
        if embedbones_sd is not None:
            emb.tau_b = scalar(embedbones_sd["tau"])
            if cutoffs:
                c = _np(embedbones_sd["cutoff_dist"])
                keep.append(c)
                emb.cutoff_dist_b = c.ctypes.data_as(_lib.c_f)
        _lib.check(_lib.load().anerf_model_set_embed(self.handle, ctypes.byref(emb)), "anerf_model_set_embed")

    @property
    def nbytes(self):
        return int(_lib.load().anerf_model_bytes(self.handle))

    def workspace(self, n_rays, S, I):
        """Cached device workspace, grown on demand (allocation happens outside any launch)."""
        need = int(_lib.load().anerf_workspace_size(self.handle, int(n_rays), int(S), int(I)))
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(max(need, 256), dtype=torch.uint8, device=f"cuda:{self.device}")
        return self._ws, need

    def close(self):
        if getattr(self, "handle", None):
            _lib.load().anerf_model_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

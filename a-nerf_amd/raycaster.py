"""Drop-in `RayCaster` for the eval render path, backed by the HIP kernels.

Mirrors `core/raycasters.py:326-474` (`RayCaster.forward` / `render_rays` and the output
dict of `_collect_outputs`, :711-724) and the model factory `create_raycaster`
(:17-184).  `render_rays` keeps the reference signature; what the reference does in a
dozen ATen ops per stage happens in one fused launch (`anerf_render_rays`).

Staged encoders (`--multires_bones > 0`, `--kp_dist_type relpos | querypts`, `--view_type rayangle`; anerf.h)
render on the training stages instead (`train.StagedCaster`, deterministic).

Supported: eval-mode rendering (`perturb=0`, `raw_noise_std=0`, `ray_noise_std=0`; `lindisp`
either way), any per-ray poses (`skts`/`cyls` may be expanded views of one pose —
detected without copying — or genuinely per-ray), framecodes via `cams`; density-only
queries `fwd_type='density'` / `'mesh'` (`render_pts_density` / `render_mesh_density`,
:579-648).  Anything else raises `NotImplementedError`; nothing silently falls back to the CPU.
"""
import ctypes
import glob
import os

import numpy as np
import torch

from . import _lib
from .config import RenderConfig
from .model import DeviceModel


def _pose_table(x, n, per_ray_shape):
    """(table, ray_pose) from a per-ray tensor that is often an expand() of one pose."""
    x = x.to(dtype=torch.float32)
    if x.dim() == len(per_ray_shape):
        x = x.unsqueeze(0)
    if x.shape[0] == 1 or x.stride(0) == 0:
        return x[:1].contiguous(), None
    if x.shape[0] != n:
        raise ValueError(f"per-ray tensor has {x.shape[0]} rows for {n} rays")
    flat = x.reshape(n, -1)
    table, inverse = torch.unique(flat, dim=0, return_inverse=True)
    return table.reshape(-1, *per_ray_shape).contiguous(), inverse.to(torch.int32).contiguous()



def _check_subject_idxs(subject_idxs):
    """The density paths take `subject_idxs` as the reference does (an integer index per query; it
    selects joint_coords rows that no encoder reads)."""
    if subject_idxs is None:
        return
    t = torch.as_tensor(subject_idxs)
    if t.is_floating_point() or t.is_complex():
        raise IndexError("subject_idxs: tensors used as indices must be long, int, byte or bool tensors")

class RayCaster:
    """Eval-mode RayCaster over a DeviceModel (the reference class is an nn.Module; this one holds
    no torch parameters: its weights live packed in HBM)."""

    def __init__(self, cfg, ckpt, device=None):
        self.cfg = cfg.validate()
        self._staged = None
        if cfg.staged:
            # (bone frequencies / relpos / ray angles: the training stages render the model deterministically,
            # include/anerf.h "staged encoders", train.StagedCaster)
            from .train import TrainRayCaster
            self._staged = TrainRayCaster(cfg, ckpt, device=device).eval()
            self.model = self._staged.model
        else:
            self.model = DeviceModel(cfg, ckpt, device=device)
        self.training = False
        self.last_debug = None

    # nn.Module-like surface used by the reference's callers
    def eval(self):
        self.training = False
        return self

    def train(self, mode=True):
        if mode:
            raise NotImplementedError("training (backward) is not implemented; use eval()")
        return self

    def load_state_dict(self, ckpt, strict=True):
        if self._staged is not None:
            self._staged.load_checkpoint(ckpt)
            self.model = self._staged.model
            return
        self.model.close()
        self.model = DeviceModel(self.cfg, ckpt, device=self.model.device)

    def __call__(self, *args, fwd_type="", **kwargs):
        return self.forward(*args, fwd_type=fwd_type, **kwargs)

    def forward(self, *args, fwd_type="", **kwargs):
        """core/raycasters.py:349-359."""
        if self._staged is not None:
            return self._staged.eval_caster()(*args, fwd_type=fwd_type, **kwargs)
        if fwd_type == "density":
            return self.render_pts_density(*args, **kwargs)
        if fwd_type == "mesh":
            return self.render_mesh_density(*args, **kwargs)
        if fwd_type == "density_color":
            # (the reference asserts the network has texture layers, _get_density_fwd_fn :623-624; its
            # NeRF has none, so the call fails the same way there)
            raise AssertionError("need to have texture layer!")
        return self.render_rays(*args, **kwargs)  # (any other fwd_type renders rays, as :357-359)

    # ------------------------------------------------------------------ density-only queries
    def _net_index(self, network):
        if network is None or network == -1:
            return -1  # fine if the model has one (raycasters.py:616-620)
        if network in ("coarse", 0):
            return 0
        if network in ("fine", 1):
            if not self.model.has_fine and not self.cfg.single_net:  # (single_net: fine IS coarse)
                raise ValueError("this model has no fine network")
            return 1
        raise ValueError(f"network must be None, 'coarse' or 'fine', got {network!r}")

    def _one_pose(self, skts, dev):
        sk = torch.as_tensor(skts).to(dev, torch.float32)
        nj = self.cfg.n_joints
        sk = sk.reshape(-1, nj, 4, 4)
        if sk.shape[0] != 1 and not (sk.stride(0) == 0):
            raise NotImplementedError("density queries take one pose (skts of shape (1, NJ, 4, 4))")
        return sk[:1].contiguous()

    @torch.no_grad()
    def render_pts_density(self, pts, kps, skts, bones, render_kwargs=None, subject_idxs=None, netchunk=1024 * 64,
                           network=None, color=False, v=None):
        """Raw density (alpha_linear, before the density activation) at points, shape
        pts.shape[:-1] + (1,)  (core/raycasters.py:597-648; `netchunk` is only a batching hint there).

        `subject_idxs` selects the reference's per-subject `joint_coords` rows (raycasters.py:601,
        726-729), which only reach the bone encoder's unused `coords` argument (no encoder in
        core/encoders.py reads them): the density does not depend on them, here as there."""
        if color:
            raise NotImplementedError("color=True needs texture layers the NeRF model does not have")
        _check_subject_idxs(subject_idxs)
        if self._staged is not None:
            return self._staged.eval_caster().render_pts_density(pts, kps, skts, bones, network=network, v=v)
        if v is not None:
            raise NotImplementedError("precomputed kp inputs (v) are not supported")
        dev = torch.device(f"cuda:{self.model.device}")
        p = torch.as_tensor(pts).to(dev, torch.float32)
        shape = p.shape[:-1]
        p = p.reshape(-1, 3).contiguous()
        sk = self._one_pose(skts, dev)
        out = torch.empty(p.shape[0], device=dev, dtype=torch.float32)
        _lib.check(_lib.load().anerf_density_points(self.model.handle, _lib.ptr(p), p.shape[0], _lib.ptr(sk),
                                                    self._net_index(network), _lib.PRECISIONS[self.cfg.precision],
                                                    _lib.ptr(out), _lib.stream_handle(dev)), "anerf_density_points")
        return out.reshape(*shape, 1)

    @torch.no_grad()
    def render_mesh_density(self, kps, skts, bones, subject_idxs=None, radius=1.0, res=64, render_kwargs=None,
                            netchunk=1024 * 64, v=None, network=None):
        """Raw density on the (res+1)^3 grid around kps[0, 0] (core/raycasters.py:579-595), generated
        on the device; same grid and element order as the reference's meshgrid (`subject_idxs`: as
        in render_pts_density)."""
        _check_subject_idxs(subject_idxs)
        if self._staged is not None:
            return self._staged.eval_caster().render_mesh_density(kps, skts, bones, radius=radius, res=res, v=v,
                                                                  network=network)
        if v is not None:
            raise NotImplementedError("precomputed kp inputs (v) are not supported")
        dev = torch.device(f"cuda:{self.model.device}")
        res1 = int(res) + 1
        axis = torch.from_numpy(np.linspace(-radius, radius, res1).astype(np.float32)).to(dev)
        kp0 = torch.as_tensor(kps).to(dev, torch.float32).reshape(-1, 3)[0].contiguous()
        sk = self._one_pose(skts, dev)
        out = torch.empty((res1, res1, res1), device=dev, dtype=torch.float32)
        _lib.check(_lib.load().anerf_density_grid(self.model.handle, _lib.ptr(axis), res1, _lib.ptr(kp0),
                                                  _lib.ptr(sk), self._net_index(network),
                                                  _lib.PRECISIONS[self.cfg.precision], _lib.ptr(out),
                                                  _lib.stream_handle(dev)), "anerf_density_grid")
        return out

    def render_rays(self, ray_batch, N_samples, kp_batch=None, skts=None, cyls=None, bones=None, cams=None,
                    subject_idxs=None, retraw=False, lindisp=False, perturb=0., N_importance=0, network_fine=None,
                    raw_noise_std=0., ray_noise_std=0., verbose=False, ext_scale=0.001, pytest=False,
                    preproc_kwargs=None, nerf_type="nerf", chunk=None, debug=False, ret_alpha=True,
                    count_mfma=False, near_far_given=False):
        """Same arguments and output dict as core/raycasters.py:361-474.

        `chunk` (extension): NaN-fill granularity; the reference fills per render_rays call,
        i.e. per batchify chunk, so the default is the whole batch.
        `near_far_given` (extension): ray_batch[:, 6:8] already hold the rays' near / far after the
        cylinder intersection and the chunk NaN fill (near_far() over the chunks that contain them),
        so any sub-range of a chunked ray list renders as in the whole list (ANERF_FLAG_NEAR_FAR)."""
        if perturb or raw_noise_std or ray_noise_std:
            raise NotImplementedError("stochastic sampling / noise (training mode) is not implemented")
        if self._staged is not None:
            if debug or count_mfma or near_far_given:
                raise NotImplementedError("debug / count_mfma / near_far_given: fused-kernel options (staged encoder)")
            return self._staged.eval_caster().render_rays(
                ray_batch, N_samples, skts=skts, cyls=cyls, cams=cams, subject_idxs=subject_idxs, lindisp=lindisp,
                N_importance=N_importance, preproc_kwargs=preproc_kwargs, chunk=chunk, ret_alpha=ret_alpha)
        if subject_idxs is not None:
            # the reference appends the indices to the view encoding (raycasters.py:545-548) and its
            # NeRF.forward then cannot split [pts | views | cam] (nerf.py:135-137): the same error
            raise RuntimeError("subject_idxs: the NeRF input has one column more than "
                               "input_ch + input_ch_bones + input_ch_views + cam_ch (core/networks/nerf.py:135)")
        if preproc_kwargs:
            B = preproc_kwargs.get("density_scale", self.cfg.density_scale)
            if B != self.cfg.density_scale:
                raise ValueError("density_scale differs from the model's configuration")
        if skts is None or cyls is None:
            raise ValueError("skts and cyls are required")
        dev = torch.device(f"cuda:{self.model.device}")
        rb = ray_batch.to(dev, torch.float32)
        if rb.stride(-1) != 1 or rb.stride(0) != rb.shape[1]:
            rb = rb.contiguous()
        n = rb.shape[0]
        S, I = int(N_samples), int(N_importance)
        T = S + I
        nj = self.cfg.n_joints
        skt_tab, pose = _pose_table(skts.to(dev), n, (nj, 4, 4))
        cyl_tab, cpose = _pose_table(cyls.to(dev), n, (5,))
        if (pose is None) != (cpose is None) or (pose is not None and not torch.equal(pose, cpose)):
            if pose is None:
                skt_tab = skt_tab.expand(n, nj, 4, 4).contiguous()
            if cpose is None:
                cyl_tab = cyl_tab.expand(n, 5).contiguous()
            if pose is not None:
                skt_tab = skt_tab[pose.long()].contiguous()
            if cpose is not None:
                cyl_tab = cyl_tab[cpose.long()].contiguous()
            pose = torch.arange(n, device=dev, dtype=torch.int32)
        cam_t = None
        if self.cfg.opt_framecode:
            if cams is None:
                raise ValueError("this model uses framecodes: cams are required")
            cam_t = cams.to(dev, torch.float32).reshape(n).contiguous()
        f32 = dict(device=dev, dtype=torch.float32)
        out = {"rgb_map": torch.empty(n, 3, **f32), "disp_map": torch.empty(n, **f32),
               "acc_map": torch.empty(n, **f32)}
        out["alpha"] = torch.empty(n, T if I > 0 else S, **f32) if ret_alpha else None
        if I > 0:
            out.update(rgb0=torch.empty(n, 3, **f32), disp0=torch.empty(n, **f32), acc0=torch.empty(n, **f32),
                       alpha0=torch.empty(n, S, **f32) if ret_alpha else None)
        dbg = None
        if debug or count_mfma:
            dbg = _lib.Debug()
        if count_mfma:
            self.last_mfma = torch.zeros(2, device=dev, dtype=torch.int64)  # [f32 MFMAs, bf16 MFMAs]
            dbg.mfma_count = ctypes.cast(self.last_mfma.data_ptr(), ctypes.POINTER(ctypes.c_uint64))
        if debug:
            dd = {"near": torch.empty(n, **f32), "far": torch.empty(n, **f32), "z_coarse": torch.empty(n, S, **f32),
                  "raw_coarse": torch.empty(n, S, 4, **f32)}
            if I > 0:
                dd.update(weights0=torch.empty(n, S, **f32), z_fine=torch.empty(n, T, **f32),
                          raw_fine=torch.empty(n, T, 4, **f32))
            for k, v in dd.items():
                setattr(dbg, k, ctypes.cast(v.data_ptr(), _lib.c_f))
            self.last_debug = dd
        ws, need = self.model.workspace(n, S, I)
        rc = _lib.load().anerf_render_rays(
            self.model.handle, _lib.ptr(rb), rb.shape[1], n, _lib.ptr(skt_tab), _lib.ptr(cyl_tab),
            skt_tab.shape[0], _lib.ptr(pose), _lib.ptr(cam_t), S, I, int(chunk or max(n, 1)),
            _lib.PRECISIONS[self.cfg.precision] | (_lib.ANERF_FLAG_LINDISP if lindisp else 0)
            | (_lib.ANERF_FLAG_NEAR_FAR if near_far_given else 0),
            _lib.ptr(out["rgb_map"]), _lib.ptr(out["disp_map"]), _lib.ptr(out["acc_map"]),
            _lib.ptr(out.get("rgb0")), _lib.ptr(out.get("disp0")), _lib.ptr(out.get("acc0")),
            _lib.ptr(out["alpha"]), _lib.ptr(out.get("alpha0")), ctypes.byref(dbg) if dbg else None,
            _lib.ptr(ws), need, _lib.stream_handle(dev))
        _lib.check(rc, "anerf_render_rays")
        if not ret_alpha:
            out.pop("alpha")
            out.pop("alpha0", None)
        return out


def near_far(ray_batch, cyls, chunk=None, out=None):
    """get_near_far_in_cylinder + the chunk NaN fill (core/utils/ray_utils.py:292-344) of a ray list on
    the device (anerf_near_far): near / far [n] of every ray, the fill over consecutive `chunk`-ray
    chunks (default: the whole list).  cyls: [5], [1, 5] (one pose) or [n, 5] per ray.  `out` =
    (near, far) tensors to fill, e.g. strided views of a ray batch's columns 6 and 7."""
    rb = ray_batch
    dev = rb.device
    if rb.dtype != torch.float32 or rb.stride(-1) != 1 or rb.stride(0) != rb.shape[1]:
        rb = rb.to(torch.float32).contiguous()
    n = rb.shape[0]
    cyl_tab, pose = _pose_table(cyls.to(dev), n, (5,))
    nearv = torch.empty(n, device=dev, dtype=torch.float32)
    farv = torch.empty(n, device=dev, dtype=torch.float32)
    if n:
        ws = torch.empty(13 * n + 1024, device=dev, dtype=torch.uint8)  # (ws_near_far_bytes, anerf_render.hip)
        _lib.check(_lib.load().anerf_near_far(_lib.ptr(rb), rb.shape[1], n, _lib.ptr(cyl_tab), cyl_tab.shape[0],
                                              _lib.ptr(pose), int(chunk or max(n, 1)), _lib.ptr(nearv),
                                              _lib.ptr(farv), _lib.ptr(ws), ws.numel(), _lib.stream_handle(dev)),
                   "anerf_near_far")
    if out is not None:
        out[0].copy_(nearv)
        out[1].copy_(farv)
    return nearv, farv


def load_checkpoint(path):
    """torch.load with weights_only=True (never unpickles code) -> dict of state dicts."""
    ck = torch.load(path, map_location="cpu", weights_only=True)
    return ck


class _EvalView:
    """render_kwargs_test's ray caster over a TrainRayCaster: always the fused eval kernel on the
    CURRENT weights (the reference shares one module between its train and test kwargs)."""

    def __init__(self, trainable):
        self._t = trainable

    @property
    def model(self):
        return self._t.eval_caster().model

    def __call__(self, *args, **kwargs):
        return self._t.eval_caster()(*args, **kwargs)

    def __getattr__(self, name):
        return getattr(self._t.eval_caster(), name)


def create_raycaster(args, data_attrs, device=None, ckpt=None):
    """Mirror of core/raycasters.py:17-184.

    Returns (render_kwargs_train, render_kwargs_test, start, grad_vars, optimizer, ckpt) like the
    reference: the train kwargs hold a `train.TrainRayCaster` (the reference's perturb /
    raw_noise_std flags), the test kwargs a view that renders the same weights with the fused eval
    kernel; `optimizer` is Adam(lr=args.lrate, betas=(0.9, 0.999)) over the trainable parameters,
    restored from the checkpoint unless `finetune` (load_ckpt_from_path,
    core/utils/run_nerf_helpers.py:6-17).  Without a checkpoint (or with no_reload) the networks
    start from torch's default initialisation, as in the reference."""
    from .train import TrainRayCaster
    skel = data_attrs["skel_type"]
    nj = len(skel.joint_names) if hasattr(skel, "joint_names") else int(skel)
    cfg = RenderConfig.from_args(args, nj)
    start = 0
    if ckpt is None:
        ft = getattr(args, "ft_path", None)
        if ft is not None and ft != "None":
            paths = [ft]
        else:
            paths = sorted(p for p in glob.glob(os.path.join(args.basedir, args.expname, "*")) if "tar" in
                           os.path.basename(p) and "pose" not in os.path.basename(p))
        if paths and not getattr(args, "no_reload", False):
            ckpt = load_checkpoint(paths[-1])
            start = 0 if getattr(args, "finetune", False) else int(ckpt.get("global_step", 0))
    caster = TrainRayCaster(cfg, ckpt, device=device)
    grad_vars = [p for p in caster.parameters() if p.requires_grad]
    # (the reference's Adam.  The fused implementation measured +0.5 % per step, profiles/r05zm_adam_ab.txt, but
    # its step writes the parameters without advancing their version counters (p._version, by which the eval
    # caster notices new weights): tests/test_host.py::test_fused_adam_leaves_version_counters checks exactly
    # that, and TrainRayCaster.weights_changed() is the hook for such optimizers)
    optimizer = torch.optim.Adam(params=grad_vars, lr=getattr(args, "lrate", 5e-4), betas=(0.9, 0.999))
    if ckpt is not None and "optimizer_state_dict" in ckpt and not getattr(args, "finetune", False):
        optimizer.load_state_dict(ckpt["optimizer_state_dict"])
    common = {"N_importance": cfg.N_importance, "N_samples": cfg.N_samples, "use_viewdirs": cfg.use_viewdirs,
              "ext_scale": cfg.ext_scale, "preproc_kwargs": {"density_scale": cfg.density_scale},
              "lindisp": cfg.lindisp, "nerf_type": getattr(args, "nerf_type", "nerf")}
    render_kwargs_train = {"ray_caster": caster, "perturb": getattr(args, "perturb", 1.0),
                           "raw_noise_std": getattr(args, "raw_noise_std", 0.0),
                           "ray_noise_std": getattr(args, "ray_noise_std", 0.0), **common}
    render_kwargs_test = {"ray_caster": _EvalView(caster), "perturb": False, "raw_noise_std": 0.,
                          "ray_noise_std": 0., **common}
    return render_kwargs_train, render_kwargs_test, start, grad_vars, optimizer, ckpt

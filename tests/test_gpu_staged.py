"""GPU parity of the staged encoders (include/anerf.h, ABI 15: --multires_bones > 0, --kp_dist_type relpos,
--view_type rayangle) against the reference's own outputs (tests/golden/sg*.npz, made by make_golden.py with
those flags; the training-mode fixture t12 is in test_gpu_train.py).

The fused render kernel does not stream these inputs; `RayCaster` renders such a model on the training stages
(train.StagedCaster: anerf_train_samples / _encode / _composite / _importance, the MLP on the fp32-accurate
split-bf16 GEMMs) with perturb 0 and no noise.  Tolerances as test_gpu_parity.py: rgb / disp / acc 1e-4
absolute, per-sample alpha 2e-3 (hazard H11), raw density 1e-4.
"""
import importlib

import numpy as np
import pytest
import torch

from _golden import STAGED, Golden

pytestmark = pytest.mark.gpu

anerf = importlib.import_module("a-nerf_amd")
train = importlib.import_module("a-nerf_amd.train")
_lib = importlib.import_module("a-nerf_amd._lib")

TOL = 1e-4
TOL_ALPHA = 2e-3


@pytest.fixture(scope="module", autouse=True)
def _cuda():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _maxdiff(a, b):
    return float(np.nanmax(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64))))


def _render(rc, g, **kw):
    rb = torch.from_numpy(g.ray_batch()).cuda()
    n = rb.shape[0]
    skts = torch.from_numpy(g["skts"][0:1]).cuda().expand(n, -1, -1, -1)
    cyls = torch.from_numpy(g["cyls"][0:1]).cuda().expand(n, -1)
    out = rc.render_rays(rb, g.cfg.N_samples, skts=skts, cyls=cyls, N_importance=g.cfg.N_importance, chunk=4096,
                         lindisp=g.cfg.lindisp, **kw)
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in out.items() if v is not None}


@pytest.mark.parametrize("name", STAGED)
def test_staged_render_matches_reference_golden(name):
    g = Golden(name)
    assert g.cfg.staged
    rc = anerf.RayCaster(g.cfg, g.ckpt)
    out = _render(rc, g)
    for k in ("rgb_map", "disp_map", "acc_map", "rgb0", "disp0", "acc0"):
        if g.has("out_" + k):
            assert out[k].shape == g["out_" + k].shape
            d = _maxdiff(out[k], g["out_" + k])
            assert d <= TOL, f"{name} {k}: max |gpu - reference| = {d:.3e}"
    for k in ("alpha", "alpha0"):
        if g.has("out_" + k):
            d = _maxdiff(out[k], g["out_" + k])
            assert d <= TOL_ALPHA, f"{name} {k}: {d:.3e}"


def test_staged_density_matches_reference():
    """fwd_type 'density' / 'mesh' of a staged model (relpos kp inputs, windowed bone frequencies)."""
    g = Golden("sgd1_relpos_mrb2_density")
    rc = anerf.RayCaster(g.cfg, g.ckpt)
    pts = torch.from_numpy(g["pts"]).reshape(-1, 1, 3)
    out = rc(pts, torch.from_numpy(g["kps"]), torch.from_numpy(g["skts"]), torch.from_numpy(g["bones"]),
             render_kwargs={}, fwd_type="density")
    torch.cuda.synchronize()
    assert tuple(out.shape) == g["pts_density"].shape
    assert _maxdiff(out.cpu().numpy(), g["pts_density"]) <= TOL
    grid = rc(kps=torch.from_numpy(g["kps"]), skts=torch.from_numpy(g["skts"]), bones=torch.from_numpy(g["bones"]),
              radius=g.meta["radius"], res=g.meta["res"], render_kwargs={}, netchunk=1024, fwd_type="mesh")
    torch.cuda.synchronize()
    assert tuple(grid.shape) == g["grid_density"].shape
    assert _maxdiff(grid.cpu().numpy(), g["grid_density"]) <= TOL


def test_fused_entries_reject_a_staged_model():
    """anerf_render_rays / anerf_density_points refuse a staged model with ANERF_EINVAL (no silent wrong
    layout); the training stages take it."""
    g = Golden(STAGED[0])
    m = importlib.import_module("a-nerf_amd.model").DeviceModel(g.cfg, g.ckpt)
    lib = _lib.load()
    dev = torch.device("cuda:0")
    rb = torch.from_numpy(g.ray_batch()).to(dev)
    n = rb.shape[0]
    sk = torch.from_numpy(g["skts"][0:1]).to(dev).contiguous()
    cy = torch.from_numpy(g["cyls"][0:1]).to(dev).contiguous()
    o = torch.empty(n, 3, device=dev)
    o1 = torch.empty(n, device=dev)
    ws, need = m.workspace(n, 32, 16)
    rc = lib.anerf_render_rays(m.handle, _lib.ptr(rb), rb.shape[1], n, _lib.ptr(sk), _lib.ptr(cy), 1, None, None, 32,
                               16, 4096, 0, _lib.ptr(o), _lib.ptr(o1), _lib.ptr(o1), None, None, None, None, None,
                               None, _lib.ptr(ws), need, _lib.stream_handle(dev))
    assert rc == -1 and b"staged encoder" in lib.anerf_last_error()
    p = torch.zeros(4, 3, device=dev)
    rc = lib.anerf_density_points(m.handle, _lib.ptr(p), 4, _lib.ptr(sk), -1, 0, _lib.ptr(o1), _lib.stream_handle(dev))
    assert rc == -1 and b"staged encoder" in lib.anerf_last_error()
    m.close()


def test_staged_caster_rejects_fused_kernel_options():
    g = Golden(STAGED[0])
    rc = anerf.RayCaster(g.cfg, g.ckpt)
    with pytest.raises(NotImplementedError):
        _render(rc, g, debug=True)
    with pytest.raises(NotImplementedError):
        _render(rc, g, perturb=1.0)


def test_staged_eval_caster_equals_training_path_without_noise():
    """TrainRayCaster.eval() on a staged model renders through StagedCaster: the same numbers as the
    training path run with perturb 0 and no noise (one code path, no fused fallback)."""
    g = Golden("sg2_rayangle_mrb2_cb_s32i16_d8w128")
    tr = train.TrainRayCaster(g.cfg, g.ckpt)
    assert isinstance(tr.eval_caster(), train.StagedCaster)
    rb = torch.from_numpy(g.ray_batch()).cuda()
    n = rb.shape[0]
    skts = torch.from_numpy(g["skts"][0:1]).cuda().expand(n, -1, -1, -1)
    cyls = torch.from_numpy(g["cyls"][0:1]).cuda().expand(n, -1)
    tr.eval()
    a = tr(rb, g.cfg.N_samples, skts=skts, cyls=cyls, N_importance=g.cfg.N_importance)
    tr.train()
    with torch.no_grad():
        b = tr.render_rays(rb, g.cfg.N_samples, skts=skts, cyls=cyls, N_importance=g.cfg.N_importance)
    for k in ("rgb_map", "disp_map", "acc_map"):
        assert torch.equal(a[k], b[k]), k


def test_staged_render_path_frame_matches_reference():
    """render_path (the caller of render_rays, run_nerf.py:27-145) over a staged model: a 64 x 64 frame with
    relpos kp inputs and ray angles, pixel set exact and images within 1e-4 of the reference's own frame."""
    g = Golden("sgf1_frame_relpos_rayangle_d4w128")
    rc = anerf.RayCaster(g.cfg, g.ckpt)
    kw = {"ray_caster": rc, "N_samples": g.cfg.N_samples, "N_importance": g.cfg.N_importance, "perturb": False,
          "raw_noise_std": 0., "ray_noise_std": 0., "use_viewdirs": True, "preproc_kwargs": {"density_scale": 1.0},
          "lindisp": False}
    H = g.meta["H"]
    rgbs, disps, accs, vids, bbs = anerf.render_path(
        torch.from_numpy(g["c2ws"]), (H, H, g.meta["focal"]), 4096, kw, kp=torch.from_numpy(g["kps"]),
        skts=torch.from_numpy(g["skts"]), ret_acc=True, ext_scale=0.001)
    np.testing.assert_array_equal(vids[0].numpy(), g["valid_idx"])
    assert rgbs.shape == g["frame_rgb"].shape
    assert _maxdiff(rgbs, g["frame_rgb"]) <= TOL
    assert _maxdiff(disps, g["frame_disp"]) <= TOL
    assert _maxdiff(accs, g["frame_acc"]) <= TOL

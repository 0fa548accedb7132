"""CPU: the oracle (oracle/anerf_oracle.c) pinned against the reference's golden outputs.

The fixtures come from running the reference's own Python render path (tests/golden/make_golden.py).
Stage by stage:
  ray generation, near/far (incl. the chunk NaN fill), coarse z  -> bit-exact
  encodings                                                       -> bit-exact (same fma chains as torch)
  MLP raw outputs                                                 -> 1e-5 relative (MKL sgemm order differs)
  compositing weights; sample_pdf on the reference's own weights  -> bit-exact / 1e-6
  final rgb / disp / acc                                          -> 1e-4 absolute
"""
import ctypes
import importlib
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))

import oracle  # noqa: E402
from _golden import FRAMES, Golden, NAMES, assert_near_far_z, sqrt_tie_rays  # noqa: E402

STAGED = [n for n in NAMES if n.startswith(("c2", "c3", "c4", "fc", "v", "s1", "t2000", "fs", "cd1", "cs1", "cb1", "mx1",
                                            "su1", "mr"))]


def importance_weights(w, single_net):
    """isample_from_lineseg's weights (ray_utils.py:265-277): w[1:-1], or with is_only (single_net)
    0.5 (max(w_l, w_k) + max(w_k, w_u)) + 0.01 in float32 (numpy scalars stay float32, NEP 50)."""
    w = np.asarray(w, np.float32)
    if not single_net:
        return w[..., 1:-1]
    return 0.5 * (np.maximum(w[..., :-2], w[..., 1:-1]) + np.maximum(w[..., 1:-1], w[..., 2:])) + np.float32(0.01)


def _om(g):
    return oracle.OracleModel(g.cfg, g.ckpt)


def test_linspace_matches_torch():
    for n in list(range(1, 300)) + [512, 1000]:
        np.testing.assert_array_equal(oracle.linspace(n), torch.linspace(0., 1., n).numpy())


def test_torch_sum_emulation_is_bit_exact():
    L = oracle.lib()
    rng = np.random.default_rng(7)
    for n in list(range(1, 260)) + [1000, 4096]:
        x = (rng.random(n) ** 2 * 10 ** rng.uniform(-5, 2, size=n)).astype(np.float32)
        got = np.float32(L.oracle_torch_sum(x.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), ctypes.c_int64(n)))
        assert got == np.float32(torch.from_numpy(x).sum().item()), n
        X = np.ascontiguousarray(rng.random((1, n, 3)).astype(np.float32))
        t = torch.from_numpy(X).sum(-2).numpy()[0]
        for c in range(3):
            p = ctypes.cast(X.ctypes.data + 4 * c, ctypes.POINTER(ctypes.c_float))
            assert np.float32(L.oracle_torch_sum_strided(p, ctypes.c_int64(3), ctypes.c_int64(n))) == t[c]


@pytest.mark.parametrize("name", NAMES)
def test_ray_generation_matches_reference(name):
    g = Golden(name)
    idx = g["valid_idx"][g["sel"]]
    rb = oracle.gen_rays(g["c2ws"][0], g.meta["H"], g.meta["H"], g.meta["focal"], idx)
    np.testing.assert_array_equal(rb[:, 0:3], g["rays_o"])
    np.testing.assert_array_equal(rb[:, 3:6], g["rays_d"])


@pytest.mark.parametrize("name", STAGED)
def test_near_far_and_z_bit_exact(name):
    g = Golden(name)
    om = _om(g)
    rb = g.ray_batch()[:4]
    near, far, _, _ = om.near_far(rb, g["cyls"][0:1], chunk=4096)
    out = om.render_rays(rb, g["skts"][0], g["cyls"][0:1], cams=g["cams"][:4] if g.has("cams") else None,
                         N_importance=0, with_z=True)
    # bit-exact, but for a ray whose cylinder Q is a float32 rounding near-tie (hazard H13)
    assert_near_far_z(near, far, out["z"], g, rb, name)


def test_nan_fill_chunk_is_exercised():
    """hazard H1: the h1 fixture's chunk holds rays that miss the cylinder."""
    g = Golden("h1_nanfill_s32i16_d4w128")
    near, far, q, filled = _om(g).near_far(g.ray_batch(), g["cyls"][0:1], chunk=4096)
    assert filled > 0 and filled == int(np.isnan(q).sum())
    assert not np.isnan(near).any() and not np.isnan(far).any()


@pytest.mark.parametrize("name", STAGED)
def test_encoding_matches_reference(name):
    g = Golden(name)
    om = _om(g)
    rb = g.ray_batch()[:4]
    z = g["stage_z"][:, :4]
    pts = (rb[:, None, 0:3] + rb[:, None, 3:6] * z[..., None]).reshape(-1, 3).astype(np.float32)
    dirs = np.repeat(rb[:, 3:6], 4, axis=0)
    ref = g["stage_feat"].reshape(16, -1)
    F = om.feature_dim()
    got = om.encode(g["skts"][0], pts, dirs)
    np.testing.assert_allclose(got, ref[:, :F], rtol=0, atol=1e-6)


@pytest.mark.parametrize("name", STAGED)
def test_network_matches_reference(name):
    g = Golden(name)
    om = _om(g)
    rb = g.ray_batch()[:4]
    z = g["stage_z"]
    S = z.shape[1]
    pts = (rb[:, None, 0:3] + rb[:, None, 3:6] * z[..., None]).reshape(-1, 3).astype(np.float32)
    dirs = np.repeat(rb[:, 3:6], S, axis=0)
    feat = om.encode(g["skts"][0], pts, dirs)
    code = None
    if g.cfg.opt_framecode:
        codes = g.ckpt["network_fn_state_dict"]["framecodes.codes.weight"]
        code = np.repeat(codes[g["cams"][:4].astype(np.int64)], S, axis=0)
    raw = om.network(feat, code=code).reshape(4, S, 4)
    ref = g["stage_raw"]
    np.testing.assert_allclose(raw, ref, rtol=0, atol=1e-5 * max(1.0, float(np.abs(ref).max())))


@pytest.mark.parametrize("name", STAGED)
def test_compositing_and_sample_pdf_match_reference(name):
    g = Golden(name)
    om = _om(g)
    rb = g.ray_batch()[:4]
    r = om.raw2outputs(g["stage_raw"], g["stage_z"], rb[:, 3:6])
    # (<= 2 ulp of a weight near 1: at 96 samples torch's cumprod rounds one product differently)
    np.testing.assert_allclose(r["weights"], g["stage_weights"], rtol=0, atol=2e-7)
    if g.cfg.N_importance > 0:
        z = g["stage_z"]
        mids = 0.5 * (z[:, 1:] + z[:, :-1])
        wts = importance_weights(g["stage_weights"], g.cfg.single_net)
        zis = om.sample_pdf(mids.astype(np.float32), wts, g.cfg.N_importance)
        np.testing.assert_array_equal(zis, g["stage_z_is"])  # same inputs -> same branch -> bit-exact
        np.testing.assert_array_equal(np.sort(np.concatenate([z, zis], -1), -1), g["stage_z_all"])


@pytest.mark.parametrize("name", NAMES)
def test_render_rays_matches_reference(name):
    g = Golden(name)
    om = _om(g)
    out = om.render_rays(g.ray_batch(), g["skts"][0], g["cyls"][0:1], cams=g["cams"] if g.has("cams") else None,
                         chunk=4096)
    for k in ("rgb_map", "disp_map", "acc_map", "rgb0", "disp0", "acc0"):
        if g.has("out_" + k):
            np.testing.assert_allclose(out[k], g["out_" + k], rtol=0, atol=1e-4, err_msg=k)
    for k in ("alpha", "alpha0"):
        if g.has("out_" + k):
            np.testing.assert_allclose(out[k], g["out_" + k], rtol=0, atol=2e-3, err_msg=k)
    if g.has("cams_neg"):
        neg = om.render_rays(g.ray_batch(), g["skts"][0], g["cyls"][0:1], cams=g["cams_neg"], chunk=4096)
        np.testing.assert_allclose(neg["rgb_map"], g["outneg_rgb_map"], rtol=0, atol=1e-4)


@pytest.mark.parametrize("name", FRAMES)
def test_render_path_frame_matches_reference(name):
    """render_path frames end to end on CPU: host pixel sets + oracle rays + render + the background
    compose of run_nerf.py:100-131 (0, white_bkgd's 1, or bg_imgs[bg_indices[i]] resized by bilinear
    F.interpolate) == the reference's frames."""
    import torch.nn.functional as F
    rays = importlib.import_module("a-nerf_amd.rays")
    g = Golden(name)
    H, f = g.meta["H"], g.meta["focal"]
    idxs, cyls, boxes = rays.valid_pixels(g["c2ws"], H, H, f, kps=g["kps"], ext_scale=0.001)
    np.testing.assert_array_equal(idxs[0], g["valid_idx"])
    np.testing.assert_array_equal(cyls, g["cyls"])
    om = _om(g)
    for fi in range(g["c2ws"].shape[0]):
        if g.has(f"frame_valid_idx_{fi}"):
            np.testing.assert_array_equal(idxs[fi], g[f"frame_valid_idx_{fi}"])
        rb = oracle.gen_rays(g["c2ws"][fi], H, H, f, idxs[fi])
        out = om.render_rays(rb, g["skts"][fi], cyls[fi:fi + 1], chunk=4096)
        if g.has("bg_imgs"):
            b = torch.from_numpy(g["bg_imgs"][g["bg_indices"][fi]]).permute(2, 0, 1)[None]
            img = F.interpolate(b, size=(H, H), mode="bilinear", align_corners=False)[0].permute(1, 2, 0).reshape(
                H * H, 3).numpy().copy()
        else:
            img = np.full((H * H, 3), 1.0 if g.meta.get("white_bkgd") else 0.0, np.float32)
        disp = np.zeros(H * H, np.float32)
        acc = np.zeros(H * H, np.float32)
        img[idxs[fi]] = out["rgb_map"] + (1.0 - out["acc_map"][:, None]) * img[idxs[fi]]
        disp[idxs[fi]] = out["disp_map"]
        acc[idxs[fi]] = out["acc_map"]
        np.testing.assert_allclose(img.reshape(H, H, 3), g["frame_rgb"][fi], rtol=0, atol=1e-4)
        np.testing.assert_allclose(disp.reshape(H, H, 1), g["frame_disp"][fi], rtol=0, atol=1e-4)
        np.testing.assert_allclose(acc.reshape(H, H, 1), g["frame_acc"][fi], rtol=0, atol=1e-4)


@pytest.mark.parametrize("name", ["dm_fine_d8w256", "dm_coarse_d4w128"])
def test_density_matches_reference(name):
    """fwd_type='density' / 'mesh' (core/raycasters.py:579-648): the oracle's trunk + alpha_linear on
    the reference's scattered points and on its mesh grid (rebuilt with the reference's meshgrid)."""
    g = Golden(name)
    om = _om(g)
    fine = g.cfg.N_importance > 0
    ref = g["pts_density"].reshape(-1)
    got = om.density(g["skts"][0], g["pts"], fine=fine)
    assert np.abs(got - ref).max() <= 1e-5 * max(1.0, np.abs(ref).max())
    gp = oracle.mesh_grid_points(g.meta["radius"], g.meta["res"], g["kps"][0, 0])
    refg = g["grid_density"].reshape(-1)
    assert gp.shape[0] == refg.shape[0]
    assert np.abs(om.density(g["skts"][0], gp, fine=fine) - refg).max() <= 1e-5 * max(1.0, np.abs(refg).max())


def test_near_empty_rays_h12_reference_vs_oracle():
    """Hazard H12 on the reference's own outputs (tests/golden/h12_nearempty_c5.npz: BASELINE config 5's
    frame, every ray with 0 < acc < 2^-20 (all hit the cylinder; 169 of 853,182), plus 64 ordinary rays,
    rendered by core.raycasters.render_rays): the oracle regenerates the fixture's rays bit for bit
    and matches every output of every ray at 1e-4 -- on the near-empty rays too, where disp =
    1 / max(1e-10, depth / acc) is a ratio of a few 2^-24 alpha quanta (max 6.2e-5 although the two
    MLPs sum in different orders: MKL sgemm vs sequential fma)."""
    import ast
    z = np.load(os.path.join(HERE, "golden", "h12_nearempty_c5.npz"))
    meta = ast.literal_eval(str(z["meta"]))
    syn = importlib.import_module("a-nerf_amd.synthetic")
    anerf = importlib.import_module("a-nerf_amd")
    sc = syn.make_scene(n_joints=24, H=meta["H"], W=meta["H"], seed=meta["seed"])
    ck = syn.make_checkpoint(meta["seed"], n_joints=24, D=8, W=256, fine=True, tau=meta["tau"])
    assert syn.checkpoint_sha256(ck) == meta["sha256"]
    cfg = anerf.RenderConfig(N_samples=64, N_importance=128).validate()
    idx, cyls, _ = anerf.rays.valid_pixels(sc["c2ws"], meta["H"], meta["H"], sc["focal"], kps=sc["kps"],
                                           ext_scale=0.001)
    rb = oracle.gen_rays(sc["c2ws"][0], meta["H"], meta["H"], sc["focal"], idx[0][z["sel"]])
    np.testing.assert_array_equal(rb[:, 0:3], z["rays_o"])
    np.testing.assert_array_equal(rb[:, 3:6], z["rays_d"])
    om = oracle.OracleModel(cfg, ck)
    out = om.render_rays(rb, sc["skts"][0], cyls[0:1], chunk=4096, near=z["near"], far=z["far"])
    ne = z["near_empty"]
    assert ne.sum() >= 1 and (~ne).sum() >= 1
    for k in ("rgb_map", "acc_map", "rgb0", "disp0", "acc0"):
        d = np.abs(out[k].astype(np.float64) - z["out_" + k]).reshape(len(ne), -1).max(-1)
        assert d.max() <= 1e-4, (k, float(d.max()))
    dd = np.abs(out["disp_map"].astype(np.float64) - z["out_disp_map"])
    assert dd[~ne].max() <= 1e-4
    assert dd[ne].max() <= 1e-4, float(dd[ne].max())
    print(f"H12: {int(ne.sum())} near-empty rays, |oracle - reference| disp max {dd[ne].max():.3e}, "
          f"{int((dd[ne] > 1e-4).sum())} above 1e-4; ordinary rays max {dd[~ne].max():.3e}")



def test_sqrt_tie_hazard_is_what_moves_near():
    """Hazard H13: on the mr9 fixture's third staged ray the cylinder's Q = sqrt(c) has its exact value
    0.502 / 0.498 ulp from the two nearest floats; the reference's torch CPU sqrt returned the farther
    one (one ulp below the correctly rounded sqrtf the oracle and the GPU use), so near differs by one
    ulp.  Every other staged ray of every fixture is bit-exact (test_near_far_and_z_bit_exact)."""
    g = Golden("mr9_mrv3_s32i16_d8w128")
    rb = g.ray_batch()[:4]
    tie = sqrt_tie_rays(rb, g["cyls"][0])
    assert tie.tolist() == [False, False, True, False]
    near, _, _, _ = _om(g).near_far(rb, g["cyls"][0:1], chunk=4096)
    assert near[2] != g["stage_near"][2, 0]
    assert abs(int(near[2:3].view(np.int32)[0]) - int(g["stage_near"][2:3, 0].view(np.int32)[0])) == 1

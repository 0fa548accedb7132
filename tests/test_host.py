"""CPU: host-side logic of the drop-in (integer pixel sets, configuration, synthetic inputs)."""
import dataclasses
import importlib
import os
import types

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
rays = importlib.import_module("a-nerf_amd.rays")
config = importlib.import_module("a-nerf_amd.config")
syn = importlib.import_module("a-nerf_amd.synthetic")


BOXES = np.load(os.path.join(HERE, "golden", "bboxes.npz"))


@pytest.mark.parametrize("name", ["c2", "c3", "c4", "c5", "c3_f3"])
def test_bounding_boxes_bit_exact_vs_reference(name):
    """kp_to_valid_rays' integer boxes at every config's full size (hazard H2), 3 camera yaws."""
    H, NJ, seed = (int(x) for x in BOXES[name + "_meta"])
    sc = syn.make_scene(n_joints=NJ, H=H, W=H, seed=seed, n_frames=3, yaw_step=0.4)
    idxs, cyls, boxes = rays.valid_pixels(sc["c2ws"], H, H, sc["focal"], kps=sc["kps"], ext_scale=0.001)
    np.testing.assert_array_equal(cyls, BOXES[name + "_cyls"])
    np.testing.assert_array_equal(np.stack([b[0] for b in boxes]), BOXES[name + "_tl"])
    np.testing.assert_array_equal(np.stack([b[1] for b in boxes]), BOXES[name + "_br"])
    np.testing.assert_array_equal([len(i) for i in idxs], BOXES[name + "_n"])
    for i, (tl, br) in enumerate(boxes):
        # exclusive upper bound, clipped to W-1/H-1: the last row/column is never traced
        assert idxs[i].max() < (H - 1) * H + (H - 1)
        assert np.all(np.diff(idxs[i]) > 0)


def test_box_pixels_row_major_exclusive():
    idx = rays.box_pixels(np.array([2, 1]), np.array([4, 3]), W=10)
    np.testing.assert_array_equal(idx, [12, 13, 22, 23])
    assert rays.box_pixels(np.array([3, 3]), np.array([3, 5]), W=10).size == 0


def test_config_rejects_unsupported_flags():
    cfg = config.RenderConfig
    with pytest.raises(NotImplementedError):
        cfg(use_viewdirs=False).validate()
    with pytest.raises(NotImplementedError):  # (bone frequencies 1-10: staged encoders, round 5)
        cfg(multires_bones=11).validate()
    assert cfg(multires_bones=2, cutoff_bones=True).validate().staged
    assert cfg(cutoff_bones=True).validate().bone_window
    assert not cfg(cutoff_bones=True, use_cutoff=False).validate().bone_window
    with pytest.raises(NotImplementedError):  # (the reference's bone embedder fails on this pair)
        cfg(extra={"kp_dist_type": "querypts"}, cutoff_bones=True).validate()
    with pytest.raises(NotImplementedError):
        cfg(extra={"kp_dist_type": "knn"}).validate()
    assert cfg(extra={"kp_dist_type": "querypts"}).validate().staged
    assert cfg(extra={"kp_dist_type": "relpos"}).validate().staged
    assert cfg(extra={"view_type": "rayangle"}).validate().staged
    assert not cfg(extra={"view_type": "world"}).validate().staged
    with pytest.raises(NotImplementedError):
        cfg(density_type="exp").validate()
    cfg().validate()


def test_freq_schedule_weights_and_columns():
    """--freq_schedule (core/cutoff_embedder.py:150, 185-197): frequency k's sin and cos weighted by
    0.5 (1 - cos(pi clamp(alpha - k, 0, 1))); the MLP input columns they land on (pts: f * NJ + j,
    views: dnet + f * 3 NJ + 3 j + c, f = 1 + 2k / 2 + 2k), everything else 1."""
    import torch
    w = config.schedule_weights(2.3, 7)
    fk = torch.log2(2.0 ** torch.linspace(0.0, 6, steps=7))
    ref = (0.5 * (1.0 - torch.cos(np.pi * torch.clamp(torch.tensor(2.3) - fk, 0, 1)))).numpy()
    np.testing.assert_array_equal(w, ref)
    assert w[0] == w[1] == 1.0 and 0.2 < w[2] < 0.21 and not w[3:].any()
    cfg = config.RenderConfig(freq_schedule=True, init_freq=2.3).validate()
    s = config.feature_scales(cfg, 2.3, 1.5)
    nj, dnet = cfg.n_joints, cfg.input_ch + cfg.input_ch_bones
    assert s.shape == (dnet + cfg.input_ch_views,)
    assert (s[:nj] == 1).all() and (s[cfg.input_ch:dnet] == 1).all()  # distance input, bone directions
    for k in range(7):
        assert (s[(1 + 2 * k) * nj:(3 + 2 * k) * nj] == w[k]).all()
    wv = config.schedule_weights(1.5, 4)
    assert (s[dnet:dnet + 3 * nj] == 1).all()
    for k in range(4):
        assert (s[dnet + (1 + 2 * k) * 3 * nj:dnet + (3 + 2 * k) * 3 * nj] == wv[k]).all()
    assert config.feature_scales(config.RenderConfig().validate(), 2.3, 2.3) is None


def test_freq_schedule_update_follows_update_alpha():
    """update_embed_fns moves sched_alpha as CutoffEmbedder.update_alpha does (cutoff_embedder.py:185-190,
    target multires - 1 for both embedders, raycasters.py:737-744); checkpoints carry the buffer."""
    import argparse
    import torch
    train = importlib.import_module("a-nerf_amd.train")
    cfg = config.RenderConfig(freq_schedule=True, init_freq=0.5, N_importance=0).validate()
    tr = train.TrainRayCaster(cfg, device="cpu")
    args = argparse.Namespace(cutoff_step=250, cutoff_rate=10.0, freq_schedule=True, freq_schedule_step=5, multires=7)
    for step in (0, 1234, 5000, 9999):
        tr.update_embed_fns(step, args)
        want = torch.tensor(0.5 + (6 - 0.5) * step / float(5 * 1000))
        assert tr.embed_fn.sched_alpha.item() == want.item() == tr.embeddirs_fn.sched_alpha.item()
    ck = tr.checkpoint()
    assert "sched_alpha" in ck["embed_state_dict"] and "sched_alpha" in ck["embeddirs_state_dict"]


def test_no_viewdirs_refusal_matches_the_reference():
    """use_viewdirs=False is refused up front; the reference itself cannot run it either: its
    render_rays raises TypeError at encode_inputs' call of embeddirs_fn = None (recorded from the
    reference by tests/golden/probe_reference_flags.py)."""
    import json
    with open(os.path.join(os.path.dirname(__file__), "golden", "reference_flags.json")) as f:
        rec = json.load(f)["use_viewdirs=False"]
    assert rec["raises"] == "TypeError" and "core/raycasters.py:538" in rec["reference_frames"]
    with pytest.raises(NotImplementedError, match="raycasters.py:67, 538"):
        config.RenderConfig(use_viewdirs=False).validate()


def test_encoder_selectors_follow_the_reference():
    """The non-default encoder selectors (core/raycasters.py:251-305) as the reference behaves on them
    (reference_flags.json, recorded by tests/golden/probe_reference_flags.py): kp_dist_type 'cat' and
    bone_type 'axisang' raise TypeError there and here; view_type 'world' runs there and renders here
    (fixture vw1_viewworld_s32i16_d8w128); relpos and rayangle run there and render here on the training
    stages (staged encoders, fixtures sg*), querypts too (not with --cutoff_bones, which fails there)."""
    import json
    with open(os.path.join(os.path.dirname(__file__), "golden", "reference_flags.json")) as f:
        rec = json.load(f)
    cfg = config.RenderConfig
    for key, val in (("kp_dist_type", "cat"), ("bone_type", "axisang")):
        assert rec[f"{key}={val}"]["raises"] == "TypeError"
        with pytest.raises(TypeError):
            cfg(extra={key: val}).validate()
    assert rec["view_type=world"]["raises"] is None
    assert cfg(extra={"view_type": "world"}).validate().extra["view_type"] == "world"
    for key, val in (("kp_dist_type", "relpos"), ("kp_dist_type", "querypts"), ("view_type", "rayangle")):
        assert rec[f"{key}={val}"]["raises"] is None
        assert cfg(extra={key: val}).validate().staged


def test_config_lindisp_from_args():
    args = types.SimpleNamespace(lindisp=True, N_samples=32)
    assert config.RenderConfig.from_args(args, 24).lindisp
    assert not config.RenderConfig.from_args(types.SimpleNamespace(), 24).lindisp


def test_precision_modes_plumbing():
    """Every precision mode the C header declares is selectable from Python (RenderConfig, the
    `anerf_precision` attribute of a run_nerf namespace) and maps to the header's enum value."""
    import re
    lib = importlib.import_module("a-nerf_amd._lib")
    hdr = open(os.path.join(os.path.dirname(HERE), "include", "anerf.h")).read()
    enum = dict((k.lower(), int(v)) for k, v in re.findall(r"ANERF_PREC_(\w+) = (\d+)", hdr))
    assert enum == {"fp32": 0, "bf16x3": 1, "bf16x6": 2, "fp16x3": 3, "fp16x4": 4}
    assert lib.PRECISIONS == enum
    for p in enum:
        assert config.RenderConfig(precision=p).validate().precision == p
        assert config.RenderConfig.from_args(types.SimpleNamespace(anerf_precision=p), 24).precision == p
    assert config.RenderConfig.from_args(types.SimpleNamespace(), 24).precision == "fp16x4"
    with pytest.raises(ValueError, match="precision"):
        config.RenderConfig(precision="fp16x5").validate()


def test_drop_in_renders_in_the_benched_precision():
    """create_raycaster(args) on a run_nerf namespace WITHOUT the non-reference `anerf_precision`
    attribute builds the precision bench.py's headline measures: the number in
    the bench line is what the untouched drop-in does.  The eval view of the test kwargs renders
    through the same config."""
    import ast
    anerf = importlib.import_module("a-nerf_amd")
    src = open(os.path.join(os.path.dirname(HERE), "bench.py")).read()
    tree = ast.parse(src)
    bench_default = None
    for node in ast.walk(tree):
        if (isinstance(node, ast.Call) and getattr(node.func, "attr", "") == "add_argument" and node.args
                and isinstance(node.args[0], ast.Constant) and node.args[0].value == "--precision"):
            bench_default = next(k.value.value for k in node.keywords if k.arg == "default")
    assert bench_default == "fp16x4"
    args = types.SimpleNamespace(netdepth=4, netwidth=64, N_samples=8, N_importance=0, lrate=5e-4,
                                 basedir="/nonexistent", expname="x", no_reload=True, ft_path=None)
    assert not hasattr(args, "anerf_precision")
    rk_train, rk_test, *_ = anerf.create_raycaster(args, {"skel_type": 24}, device="cpu")
    assert rk_train["ray_caster"].cfg.precision == bench_default
    assert config.RenderConfig().precision == bench_default


def test_config_from_args_matches_surreal_config():
    args = types.SimpleNamespace(netdepth=8, netwidth=256, multires=7, multires_views=4, use_cutoff=True,
                                 cutoff_inputs=True, cutoff_viewdir=True, use_viewdirs=True, N_samples=64,
                                 N_importance=16, chunk=4096, ext_scale=0.001, kp_dist_type="reldist",
                                 bone_type="reldir", view_type="relray", pts_tr_type="local", density_type="relu",
                                 opt_framecode=False, framecode_size=16, n_framecodes=None, single_net=False)
    cfg = config.RenderConfig.from_args(args, 24)
    assert cfg.feature_dim == 360 + 72 + 648
    assert config.flops_per_sample(cfg) == 1_723_648
    cfg.N_importance = 128
    assert config.flops_per_sample(cfg) * config.samples_per_ray(cfg) == 441_253_888


def test_flops_match_survey_table():
    assert config.flops_per_sample(config.RenderConfig(netdepth=4, netwidth=128)) == 341_632
    assert config.flops_per_sample(config.RenderConfig(n_joints=65)) == 2_762_752


def test_synthetic_weights_are_reproducible():
    a = syn.make_checkpoint(5, n_joints=24, D=4, W=128)
    b = syn.make_checkpoint(5, n_joints=24, D=4, W=128)
    assert syn.checkpoint_sha256(a) == syn.checkpoint_sha256(b)
    assert a["network_fn_state_dict"]["pts_linears.0.weight"].shape == (128, 432)
    assert a["network_fn_state_dict"]["views_linears.0.weight"].shape == (64, 128 + 648)


def test_synthetic_skeleton_chain_is_rigid():
    sc = syn.make_scene(n_joints=24, H=64, W=64, seed=3)
    l2w = np.linalg.inv(sc["skts"][0].astype(np.float64))
    np.testing.assert_allclose(l2w[:, :3, 3], sc["kps"][0], atol=1e-5)
    for j in range(1, 24):  # bone lengths preserved
        p = syn.SMPL_PARENTS[j]
        a = np.linalg.norm(sc["kps"][0][j] - sc["kps"][0][p])
        b = np.linalg.norm(syn.REST_POSE_24[j] - syn.REST_POSE_24[p])
        assert abs(a - b) < 1e-5


RANDOM_BOXES = np.load(os.path.join(HERE, "golden", "boxes_random.npz"))


def _random_frame(z, i):
    H, W = (int(v) for v in z["hw"][i])
    f = z["focal"][i]
    focal = float(f[0]) if f[0] == f[1] else f.copy()
    centers = z["center"][i:i + 1] if z["has_center"][i] else None
    return H, W, focal, centers


def test_random_boxes_bit_exact_vs_reference():
    """400 random poses / cameras / focals / principal points / image sizes: the host restatement
    gives the reference's get_kp_bounding_cylinder + cylinder_to_box_2d integers exactly."""
    z = RANDOM_BOXES
    for i in range(z["kps"].shape[0]):
        H, W, focal, centers = _random_frame(z, i)
        _, cyls, boxes = rays.valid_pixels(z["c2w"][i:i + 1], H, W, focal if isinstance(focal, float) else [focal],
                                           kps=z["kps"][i:i + 1], ext_scale=0.001, centers=centers)
        np.testing.assert_array_equal(cyls[0], z["cyl"][i])
        np.testing.assert_array_equal(boxes[0][0], z["tl"][i])
        np.testing.assert_array_equal(boxes[0][1], z["br"][i])


def test_normalize_cutoff_is_a_noop_like_the_reference():
    """--normalize_cutoff never reaches CutoffEmbedder.normalize in the reference (the kwarg is named
    normalize_cutoff, core/raycasters.py:32 vs core/cutoff_embedder.py:64); recorded from the reference
    by tests/golden/probe_reference_flags.py.  Accepted here with the same (absent) effect."""
    import json
    with open(os.path.join(HERE, "golden", "reference_flags.json")) as f:
        rec = json.load(f)["normalize_cutoff"]
    assert rec["raises"] is None
    assert not rec["embedder_attributes"]["embed_fn.normalize"]
    assert not rec["embedder_attributes"]["embeddirs_fn.normalize"]
    args = types.SimpleNamespace(normalize_cutoff=True, cut_to_dist=True, cutoff_shift=True)
    cfg = config.RenderConfig.from_args(args, 24)
    assert cfg.normalize_cutoff and cfg.cut_to_dist and cfg.cutoff_shift
    assert config.RenderConfig.from_args(types.SimpleNamespace(cutoff_bones=True), 24).cutoff_bones
    # (bone frequencies: a staged encoder since round 5, include/anerf.h)
    assert config.RenderConfig.from_args(types.SimpleNamespace(cutoff_bones=True, multires_bones=4), 24).staged


def test_forward_dispatch_matches_the_reference():
    """RayCaster.forward's fwd_type dispatch (core/raycasters.py:349-359): 'density' / 'mesh' to the
    density queries, 'density_color' fails the reference's texture-layer assertion (:623-624, NeRF
    has no texture_linears), anything else renders rays."""
    rc_mod = importlib.import_module("a-nerf_amd.raycaster")
    rc = object.__new__(rc_mod.RayCaster)  # (dispatch only: no device model)
    rc._staged = None
    rc.render_pts_density = lambda *a, **k: "density"
    rc.render_mesh_density = lambda *a, **k: "mesh"
    rc.render_rays = lambda *a, **k: "rays"
    assert rc(fwd_type="density") == "density" and rc(fwd_type="mesh") == "mesh"
    assert rc() == "rays" and rc(fwd_type="something") == "rays"
    with pytest.raises(AssertionError, match="texture layer"):
        rc(fwd_type="density_color")


def test_staged_encoder_configs_match_reference_checkpoints():
    """Round 5: --multires_bones > 0, --kp_dist_type relpos and --view_type rayangle build (staged encoders,
    include/anerf.h) with the reference's input widths: the fixtures' checkpoints, made by the reference's
    create_raycaster with those flags (tests/golden/make_golden.py), have exactly these layer shapes."""
    from _golden import STAGED, Golden
    for name in STAGED + ["sgd1_relpos_mrb2_density"]:
        g = Golden(name)
        cfg = g.cfg
        assert cfg.staged
        sd = g.ckpt["network_fn_state_dict"]
        dnet = cfg.input_ch + cfg.input_ch_bones
        assert sd["pts_linears.0.weight"].shape == (cfg.netwidth, dnet), name
        assert sd["views_linears.0.weight"].shape[1] == cfg.netwidth + cfg.input_ch_views + cfg.framecode_ch, name
        if cfg.netdepth > 5:
            assert sd[f"pts_linears.{cfg.skips[0] + 1}.weight"].shape == (cfg.netwidth, cfg.netwidth + dnet), name
    g = Golden("sg3_all_fs_s32i16_d8w256")
    assert (g.cfg.kp_relpos, g.cfg.view_angle, g.cfg.multires_bones) == (True, True, 3)
    with pytest.raises(NotImplementedError):
        dataclasses.replace(g.cfg, multires_bones=11).validate()
    with pytest.raises(NotImplementedError):  # (querypts with --cutoff_bones fails in the reference)
        dataclasses.replace(g.cfg, extra={"kp_dist_type": "querypts"}).validate()
    assert Golden("sg4_querypts_shift_s32i16_d8w128").cfg.input_ch == 3 * (1 + 2 * 7)
    assert Golden("sg4_querypts_shift_s32i16_d8w128").ckpt["embed_state_dict"]["cutoff_dist"].shape == (3,)


def test_feature_scales_follow_the_staged_layout():
    """--freq_schedule weights per frequency block of each part: relpos 3 NJ columns per slot, windowed bone
    frequencies 3 NJ (their own sched_alpha), ray angles NJ."""
    from _golden import Golden
    cfg = Golden("sg3_all_fs_s32i16_d8w256").cfg
    nj = cfg.n_joints
    s = config.feature_scales(cfg, 2.3, 1.6, 0.4)
    assert s.shape == (cfg.feature_dim,)
    wp, wv, wb = (config.schedule_weights(a, n) for a, n in ((2.3, cfg.multires), (1.6, cfg.multires_views),
                                                              (0.4, cfg.multires_bones)))
    assert np.all(s[:3 * nj] == 1.0)
    for k in range(cfg.multires):
        assert np.all(s[(1 + 2 * k) * 3 * nj:(3 + 2 * k) * 3 * nj] == wp[k])
    ob = cfg.input_ch
    assert np.all(s[ob:ob + 3 * nj] == 1.0)
    for k in range(cfg.multires_bones):
        assert np.all(s[ob + (1 + 2 * k) * 3 * nj:ob + (3 + 2 * k) * 3 * nj] == wb[k])
    ov = cfg.input_ch + cfg.input_ch_bones
    assert np.all(s[ov:ov + nj] == 1.0)
    for k in range(cfg.multires_views):
        assert np.all(s[ov + (1 + 2 * k) * nj:ov + (3 + 2 * k) * nj] == wv[k])


def test_fused_adam_leaves_version_counters():
    """ADVICE r5 (raycaster.py's note on torch's fused Adam): the fused step updates a parameter in place without
    advancing p._version, while the foreach step advances it -- the cause of the eval caster missing fused updates
    (its repack check reads the version counters; TrainRayCaster.weights_changed() forces the repack instead)."""
    import torch
    for fused, advances in ((True, False), (False, True)):
        p = torch.nn.Parameter(torch.ones(8))
        opt = torch.optim.Adam([p], lr=0.1, **({"fused": True} if fused else {"foreach": True}))
        p.grad = torch.ones(8)
        v0 = p._version
        opt.step()
        assert float(p.detach()[0]) < 1.0  # (the step did update the values)
        assert (p._version != v0) == advances, (fused, v0, p._version)

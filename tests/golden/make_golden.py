"""Generate the golden fixtures under tests/golden/ by running the REFERENCE render path.

Runs ONLY in the survey/build container, where /root/reference exists; it is never
needed on the GPU box (the fixtures it writes are committed).  It imports the
reference's own Python modules (run_nerf.render_path, core.trainer.render,
core.raycasters.create_raycaster / RayCaster stages) with empty stubs for the
third-party modules that never touch the render arithmetic (SURVEY.md §8c,
Appendix B), feeds them our deterministic synthetic scenes and seeded weights
(a-nerf_amd/synthetic.py), and stores inputs + outputs as small .npz files.

Weights are not stored: the fixture records (seed, sha256) and the tests
regenerate them with a-nerf_amd/synthetic.py and check the hash.

Usage:  python tests/golden/make_golden.py  [--only NAME]
"""
import argparse
import importlib
import importlib.abc
import importlib.machinery
import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

sys.path.insert(0, REPO)
anerf_syn = importlib.import_module("a-nerf_amd.synthetic")

_STUBS = ["cv2", "pytorch3d", "imageio", "deepdish", "h5py", "smplx", "pytorch_msssim",
          "tensorboard", "mcubes", "trimesh", "plotly", "skimage", "lpips"]


class _StubFinder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    """Empty modules for imports the render arithmetic never uses."""

    def find_spec(self, name, path, target=None):
        if name.split(".")[0] in _STUBS or name.startswith("torch.utils.tensorboard"):
            return importlib.machinery.ModuleSpec(name, self, is_package=True)
        return None

    def create_module(self, spec):
        m = types.ModuleType(spec.name)
        m.__path__ = []
        def _attr(attr):
            if attr.startswith("__"):
                raise AttributeError(attr)
            if attr[:1].isupper():
                return type(attr, (), {"__init__": lambda self, *a, **k: None})
            return lambda *a, **k: None
        m.__getattr__ = _attr
        return m

    def exec_module(self, module):
        pass


def import_reference():
    sys.dont_write_bytecode = True
    sys.meta_path.insert(0, _StubFinder())
    cap = types.ModuleType("configargparse")

    class _AP(argparse.ArgumentParser):
        def add_argument(self, *a, **k):
            k.pop("is_config_file", None)
            return super().add_argument(*a, **k)

    cap.ArgumentParser = _AP
    sys.modules["configargparse"] = cap
    sys.path.insert(0, REF)
    import torch  # noqa: F401
    run_nerf = importlib.import_module("run_nerf")
    trainer = importlib.import_module("core.trainer")
    raycasters = importlib.import_module("core.raycasters")
    ray_utils = importlib.import_module("core.utils.ray_utils")
    sk = importlib.import_module("core.utils.skeleton_utils")
    return run_nerf, trainer, raycasters, ray_utils, sk


# name -> config (BASELINE.json configs 1-4, plus small edge cases)
CONFIGS = {
    "c1_64_s32_d4w128": dict(H=64, NJ=24, S=32, I=0, D=4, W=128, tau=20.0, kind="frame", seed=11),
    "c2_256_s64_d8w256": dict(H=256, NJ=24, S=64, I=0, D=8, W=256, tau=20.0, kind="rays", n_rays=512, seed=12),
    "c3_512_s64i128_d8w256": dict(H=512, NJ=24, S=64, I=128, D=8, W=256, tau=79.6, kind="rays", n_rays=256, seed=13),
    "c4_512_s64i128_j65": dict(H=512, NJ=65, S=64, I=128, D=8, W=256, tau=20.0, kind="rays", n_rays=128, seed=14),
    # chunk-coupled NaN fill of near/far (hazard H1): a chunk that contains rays missing the cylinder
    "h1_nanfill_s32i16_d4w128": dict(H=128, NJ=24, S=32, I=16, D=4, W=128, tau=20.0, kind="nanfill", seed=15),
    # per-frame code (opt_framecode, mixamo configs) with cam index >= 0 and the eval-mode mean code (< 0)
    "fc_64_s32i32_d4w128": dict(H=64, NJ=24, S=32, I=32, D=4, W=128, tau=20.0, kind="framecode", n_rays=192, seed=16),
    # density-only queries (RayCaster.forward fwd_type='mesh' / 'density', core/raycasters.py:579-648):
    # the fine net of the config-3 model, and the coarse-only D=4 model
    "dm_fine_d8w256": dict(H=64, NJ=24, S=64, I=128, D=8, W=256, tau=79.6, kind="density", seed=13, res=16,
                           radius=1.8, n_pts=1000),
    "dm_coarse_d4w128": dict(H=64, NJ=24, S=32, I=0, D=4, W=128, tau=20.0, kind="density", seed=11, res=12,
                             radius=1.8, n_pts=600),
    # flag variants of the render path (kernel template / branch coverage)
    "v1_mr10_w64_d4": dict(H=128, NJ=24, S=32, I=16, D=4, W=64, tau=20.0, kind="rays", n_rays=128, seed=21, mr=10),
    "v2_softplus_nocutview": dict(H=128, NJ=24, S=32, I=16, D=4, W=128, tau=20.0, kind="rays", n_rays=128, seed=22,
                                  flags=["--density_type", "softplus", "--softplus_shift", "1.0"],
                                  drop=["--cutoff_viewdir"]),
    "v3_nocutinputs": dict(H=128, NJ=24, S=32, I=16, D=4, W=128, tau=20.0, kind="rays", n_rays=128, seed=23,
                           drop=["--cutoff_inputs"]),
    "v4_nocutoff": dict(H=128, NJ=24, S=32, I=16, D=4, W=128, tau=20.0, kind="rays", n_rays=128, seed=24,
                        drop=["--use_cutoff", "--cutoff_inputs", "--cutoff_viewdir"]),
    # configs/surreal/surreal_single.txt: single_net (one network, fine pass on the I new samples only,
    # max-filtered importance weights), multires_views 0, 96 + 48 samples; the checkpoint carries two
    # different network state dicts (load_state_dict loads network_fine's last into the shared module)
    "s1_single_s96i48_mrv0": dict(H=256, NJ=24, S=96, I=48, D=8, W=256, tau=20.0, kind="rays", n_rays=192, seed=31,
                                  mrv=0, single=True),
    # the tau schedule's ceiling (CutoffEmbedder.update_tau clamps at 2000): the sharpest window
    "t2000_512_s64i128": dict(H=512, NJ=24, S=64, I=128, D=8, W=256, tau=2000.0, kind="rays", n_rays=256, seed=32),
    # --lindisp: samples linear in inverse depth (sample_from_lineseg, ray_utils.py:223-226)
    "l1_lindisp_s32i16_d4w128": dict(H=128, NJ=24, S=32, I=16, D=4, W=128, tau=20.0, kind="rays", n_rays=128,
                                     seed=25, flags=["--lindisp"]),
    # --freq_schedule at sched_alpha 2.3 (frequencies 0-1 full, 2 at 0.206, 3+ off) in both cutoff
    # embedders (core/cutoff_embedder.py:150, 192-197); D = 8 so the skip layer's x part is covered
    "fs1_freqsched_s32i16_d8w128": dict(H=128, NJ=24, S=32, I=16, D=8, W=128, tau=20.0, kind="rays", n_rays=128,
                                        seed=26, flags=["--freq_schedule", "--init_freq", "2.3"], sched=2.3),
    # --cut_to_dist (the kp encoding of c_j - dist) and --cutoff_shift (frequencies of dist * 2 / c_j - 1),
    # core/cutoff_embedder.py:125-134
    "cd1_cuttodist_s32i16_d8w128": dict(H=128, NJ=24, S=32, I=16, D=8, W=128, tau=20.0, kind="rays", n_rays=128,
                                        seed=27, flags=["--cut_to_dist"]),
    "cs1_cutoffshift_s32i16_d4w128": dict(H=128, NJ=24, S=32, I=16, D=4, W=128, tau=20.0, kind="rays",
                                          n_rays=128, seed=25, flags=["--cutoff_shift"]),
    # --view_type world: IdentityExpandEncoder of the joint-frame ray directions (not normalised)
    "vw1_viewworld_s32i16_d8w128": dict(H=128, NJ=24, S=32, I=16, D=8, W=128, tau=20.0, kind="rays", n_rays=128,
                                        seed=29, flags=["--view_type", "world"]),
    # --cutoff_bones (the bone embedder a CutoffEmbedder with its own tau / cutoff_dist: bone directions
    # times w_b, core/raycasters.py:52-64, cutoff_embedder.py:108-166); D = 8 for the skip layer's x part
    "cb1_cutoffbones_s32i16_d8w128": dict(H=128, NJ=24, S=32, I=16, D=8, W=128, tau=20.0, kind="rays", n_rays=128,
                                          seed=28, flags=["--cutoff_bones"], cb=True, tau_b=35.0),
    # (round 5) staged encoders (include/anerf.h, rendered on the training stages): --kp_dist_type relpos;
    # --view_type rayangle with --multires_bones 2 and --cutoff_bones; all three at 8 x 256 (the skip layer's
    # [x | h]) with --multires_bones 3 and --freq_schedule
    "sgd1_relpos_mrb2_density": dict(H=64, NJ=24, S=32, I=16, D=8, W=128, tau=20.0, kind="density", seed=54, res=10,
                                     radius=1.0, n_pts=300, cb=True, tau_b=35.0,
                                     flags=["--kp_dist_type", "relpos", "--multires_bones", "2", "--cutoff_bones"]),
    # --kp_dist_type querypts (the world point as the kp input, windowed per coordinate) with --cutoff_shift
    "sg4_querypts_shift_s32i16_d8w128": dict(H=128, NJ=24, S=32, I=16, D=8, W=128, tau=20.0, kind="rays", n_rays=128,
                                             seed=55, flags=["--kp_dist_type", "querypts", "--cutoff_shift"]),
    # a render_path frame (64 x 64) of a staged model: relpos + rayangle, 32 + 16 samples
    "sgf1_frame_relpos_rayangle_d4w128": dict(H=64, NJ=24, S=32, I=16, D=4, W=128, tau=20.0, kind="frame", seed=56,
                                              flags=["--kp_dist_type", "relpos", "--view_type", "rayangle"]),
    "sg1_relpos_s32i16_d4w128": dict(H=128, NJ=24, S=32, I=16, D=4, W=128, tau=20.0, kind="rays", n_rays=128,
                                     seed=51, flags=["--kp_dist_type", "relpos"]),
    "sg2_rayangle_mrb2_cb_s32i16_d8w128": dict(H=128, NJ=24, S=32, I=16, D=8, W=128, tau=20.0, kind="rays",
                                               n_rays=128, seed=52, cb=True, tau_b=35.0,
                                               flags=["--view_type", "rayangle", "--multires_bones", "2",
                                                      "--cutoff_bones"]),
    "sg3_all_fs_s32i16_d8w256": dict(H=128, NJ=24, S=32, I=16, D=8, W=256, tau=20.0, kind="rays", n_rays=96,
                                     seed=53, sched=2.3, cb=True, tau_b=35.0,
                                     flags=["--kp_dist_type", "relpos", "--view_type", "rayangle",
                                            "--multires_bones", "3", "--cutoff_bones", "--freq_schedule",
                                            "--init_freq", "2.3"]),
    # the shipped configs' render shape (configs/{mixamo,h36m,perfcap}/*.txt: 8x256, multires 7 / 4,
    # N_samples 64, N_importance 16, opt_framecode; configs/surreal/surreal.txt the same without
    # framecodes): the view layer's framecode column at W = 256 and the 64 + 16 importance pass
    "mx1_mixamo_s64i16_d8w256_fc": dict(H=256, NJ=24, S=64, I=16, D=8, W=256, tau=200.0, kind="framecode",
                                        n_rays=160, seed=41),
    "su1_surreal_s64i16_d8w256": dict(H=512, NJ=24, S=64, I=16, D=8, W=256, tau=20.0, kind="rays", n_rays=192,
                                      seed=42),
    # --multires / --multires_views other than the shipped 7 / 4 and the default 10 (run_nerf.py:275-280):
    # the kernels' instances for 7 / 10 and 0 / 4 run them with the missing frequencies' weights zero
    # (anerf_pack.hpp layout_multires); bf16x6 windowed part at W = 256 and 128, the f32 one at W = 64
    "mr5_mrv2_s32i16_d8w256": dict(H=128, NJ=24, S=32, I=16, D=8, W=256, tau=20.0, kind="rays", n_rays=128, seed=51,
                                   mr=5, mrv=2),
    "mr9_mrv3_s32i16_d8w128": dict(H=128, NJ=24, S=32, I=16, D=8, W=128, tau=20.0, kind="rays", n_rays=128, seed=52,
                                   mr=9, mrv=3),
    "mr3_mrv1_s32i16_d4w64": dict(H=128, NJ=24, S=32, I=16, D=4, W=64, tau=20.0, kind="rays", n_rays=128, seed=53,
                                  mr=3, mrv=1),
    # render_path's background compose (run_nerf.py:100-131): white_bkgd (bg = 1), and bg_imgs resized
    # with F.interpolate(bilinear, align_corners=False) and picked per frame by bg_indices; two frames
    # (reuse_input of the pose tensors, run_nerf.py:63-74)
    "pw_64_white_d4w128": dict(H=64, NJ=24, S=32, I=16, D=4, W=128, tau=20.0, kind="frame", seed=43, n_frames=2,
                               white_bkgd=True),
    "pb_64_bgimg_d4w128": dict(H=64, NJ=24, S=32, I=16, D=4, W=128, tau=20.0, kind="frame", seed=44, n_frames=2,
                               bg_imgs=(3, 48, 40), bg_indices=[2, 0]),
}


def staged_dims(flags):
    """make_checkpoint's input-shape arguments for the staged encoders' flags (--multires_bones,
    --kp_dist_type relpos, --view_type rayangle)."""
    def val(k, d):
        return flags[flags.index(k) + 1] if k in flags else d
    return dict(multires_bones=int(val("--multires_bones", 0)), kp_dims=3 if val("--kp_dist_type", "") == "relpos" else 1,
                view_dims=1 if val("--view_type", "") == "rayangle" else 3,
                kp_query=val("--kp_dist_type", "") == "querypts")


def build_reference(mods, cfg, tmp):
    run_nerf, trainer, raycasters, ray_utils, sk = mods
    import torch
    NJ = cfg["NJ"]
    use_fc = cfg["kind"] == "framecode"
    argv = ["--N_samples", str(cfg["S"]), "--N_importance", str(cfg["I"]),
            "--netdepth", str(cfg["D"]), "--netwidth", str(cfg["W"]),
            "--multires", str(cfg.get("mr", 7)), "--multires_views", str(cfg.get("mrv", 4)),
            "--use_cutoff", "--cutoff_viewdir", "--cutoff_inputs", "--use_viewdirs",
            "--ext_scale", "0.001", "--chunk", "4096", "--no_reload",
            "--basedir", tmp, "--expname", "x"]
    argv = [a for a in argv if a not in cfg.get("drop", [])] + cfg.get("flags", [])
    if use_fc:
        argv += ["--opt_framecode", "--n_framecodes", "5"]
    if cfg.get("single"):
        argv += ["--single_net"]
    args = run_nerf.config_parser().parse_args(argv)
    os.makedirs(os.path.join(tmp, "x"), exist_ok=True)
    parents, rest = anerf_syn.skeleton(NJ)
    if NJ == 24:
        skel = sk.SMPLSkeleton
    else:
        skel = sk.Skeleton(joint_names=[f"j{i}" for i in range(NJ)], joint_trees=parents, root_id=0,
                           nonroot_id=list(range(1, NJ)), cutoffs={}, end_effectors=[])
    data_attrs = {"skel_type": skel, "near": 0.0, "far": 1.0, "n_views": 5,
                  "joint_coords": np.zeros((NJ, 3, 3), np.float32)}
    _, render_kwargs, _, _, _, _ = raycasters.create_raycaster(args, data_attrs)
    ck = anerf_syn.make_checkpoint(cfg["seed"], n_joints=NJ, D=cfg["D"], W=cfg["W"], fine=cfg["I"] > 0,
                                   tau=cfg["tau"], use_framecode=use_fc, n_framecodes=5, multires=cfg.get("mr", 7),
                                   multires_views=cfg.get("mrv", 4), sched_alpha=cfg.get("sched"),
                                   cutoff_bones=cfg.get("cb", False), tau_bones=cfg.get("tau_b"),
                                   **staged_dims(cfg.get("flags", [])))
    ck_t = {k: {n: torch.from_numpy(np.array(v)) for n, v in d.items()} for k, d in ck.items()}
    rc = render_kwargs["ray_caster"]
    rc.load_state_dict(ck_t, strict=True)
    rc.eval()
    return args, render_kwargs, ck


def scene_for(cfg):
    if cfg.get("n_frames", 1) > 1:
        return anerf_syn.make_scene(n_joints=cfg["NJ"], H=cfg["H"], W=cfg["H"], seed=cfg["seed"],
                                    n_frames=cfg["n_frames"], yaw_step=0.7)
    return anerf_syn.make_scene(n_joints=cfg["NJ"], H=cfg["H"], W=cfg["H"], seed=cfg["seed"])


def bg_for(cfg):
    """(bg_imgs float32 [B, h, w, 3] in [0, 1], bg_indices) of a background-compose fixture, or Nones."""
    if "bg_imgs" not in cfg:
        return None, None
    bg = np.random.default_rng(cfg["seed"] + 300).random(cfg["bg_imgs"] + (3,)).astype(np.float32)
    return bg, np.asarray(cfg["bg_indices"], np.int64)


def rays_for(mods, sc):
    """reference kp_to_valid_rays on frame 0."""
    import torch
    _, _, _, ray_utils, _ = mods
    c2w = torch.from_numpy(sc["c2ws"])
    kp = torch.from_numpy(sc["kps"])
    rays, valid_idxs, cyls, bboxes = ray_utils.kp_to_valid_rays(c2w, sc["H"], sc["W"], sc["focal"], kps=kp,
                                                                ext_scale=0.001)
    return rays[0], valid_idxs[0].numpy(), cyls.numpy(), bboxes[0]


def render_subset(mods, render_kwargs, o, d, sc, cams=None):
    import torch
    _, trainer, _, _, _ = mods
    n = o.shape[0]
    kp = torch.from_numpy(sc["kps"][0:1]).expand(n, -1, -1)
    skts = torch.from_numpy(sc["skts"][0:1]).expand(n, -1, -1, -1)
    bones = torch.from_numpy(sc["bones"][0:1]).expand(n, -1, -1)
    cyl = torch.from_numpy(sc["cyls"][0:1]).expand(n, -1)
    cam_t = None if cams is None else torch.from_numpy(cams)
    with torch.no_grad():
        ret = trainer.render(sc["H"], sc["W"], sc["focal"], chunk=4096, rays=(o, d),
                             c2w=torch.from_numpy(sc["c2ws"][0][:3, :4]),
                             kp_batch=kp, skts=skts, cyls=cyl, bones=bones, cams=cam_t, subject_idxs=None,
                             **render_kwargs)
    return {k: v.numpy() for k, v in ret.items()}


def stage_dump(mods, render_kwargs, o, d, sc, n_stage, cams=None):
    """Per-stage tensors of render_rays (core/raycasters.py:411-474) for a few rays."""
    import torch
    _, _, raycasters, ray_utils, _ = mods
    rc = render_kwargs["ray_caster"]
    pk = render_kwargs["preproc_kwargs"]
    S, I = render_kwargs["N_samples"], render_kwargs["N_importance"]
    o, d = o[:n_stage], d[:n_stage]
    n = o.shape[0]
    kp = torch.from_numpy(sc["kps"][0:1]).expand(n, -1, -1)
    skts = torch.from_numpy(sc["skts"][0:1]).expand(n, -1, -1, -1)
    bones = torch.from_numpy(sc["bones"][0:1]).expand(n, -1, -1)
    cyl = torch.from_numpy(sc["cyls"][0:1]).expand(n, -1)
    cam_t = None if cams is None else torch.from_numpy(cams[:n_stage])
    out = {}
    with torch.no_grad():
        near, far = ray_utils.get_near_far_in_cylinder(o, d, cyl, near=torch.zeros(n, 1), far=torch.ones(n, 1))
        pts, z = rc.sample_pts(o, d, near, far, n, S, 0.0, bool(render_kwargs.get("lindisp", False)))
        jc = rc.get_subject_joint_coords(None, pts.device)
        enc = rc.encode_inputs(pts, [o[:, None, :], d[:, None, :]], kp, skts, bones, cam_idxs=cam_t,
                               subject_idxs=None, joint_coords=jc, network=rc.network, **pk)
        feat = torch.cat([enc["v"], enc["r"], enc["d"]], dim=-1)  # (+ cam column when cams given)
        raw = rc.run_network(enc, rc.network)
        ret = rc.network.raw2outputs(raw, z, d, 0.0, encoded=enc, B=pk["density_scale"], act_fn=pk["density_fn"])
        out.update(near=near.numpy(), far=far.numpy(), z=z.numpy(), feat=feat[:, :4].numpy(),
                   raw=raw.numpy(), weights=ret["weights"].numpy())
        if I > 0:
            single = bool(rc.single_net)
            pts_is, z_all, z_is, sidx = rc.sample_pts_is(o, d, z, ret["weights"], I, det=True, is_only=single)
            enc_is = rc.encode_inputs(pts_is, [o[:, None, :], d[:, None, :]], kp, skts, bones, cam_idxs=cam_t,
                                      subject_idxs=None, joint_coords=jc, network=rc.network_fine, **pk)
            if single:  # raycasters.py:462-468
                raw_is = rc.run_network(enc_is, rc.network_fine)
                raw_f = rc._merge_encodings({"raw": raw}, {"raw": raw_is}, sidx, n, S + I)["raw"]
            else:
                merged = rc._merge_encodings(enc, enc_is, sidx, n, S + I)
                raw_f = rc.run_network(merged, rc.network_fine)
            out.update(z_is=z_is.numpy(), z_all=z_all.numpy(), raw_f=raw_f.numpy())
    return {"stage_" + k: v for k, v in out.items()}


def make_density(name, cfg, mods, tmp):
    """fwd_type='mesh' on a small grid and fwd_type='density' on scattered points (frame 0 pose)."""
    import torch
    args, render_kwargs, ck = build_reference(mods, cfg, os.path.join(tmp, name))
    sc = scene_for(cfg)
    rc = render_kwargs["ray_caster"]
    pk = render_kwargs["preproc_kwargs"]
    kps = torch.from_numpy(sc["kps"][0:1])
    skts = torch.from_numpy(sc["skts"][0:1])
    bones = torch.from_numpy(sc["bones"][0:1])
    rng = np.random.default_rng(cfg["seed"] + 100)
    pts = (sc["kps"][0][rng.integers(0, cfg["NJ"], cfg["n_pts"])] +
           rng.normal(0.0, 0.15, (cfg["n_pts"], 3))).astype(np.float32)
    with torch.no_grad():
        grid = rc(kps=kps, skts=skts, bones=bones, radius=cfg["radius"], render_kwargs=pk, res=cfg["res"],
                  netchunk=1024, fwd_type="mesh")
        dens = rc(torch.from_numpy(pts).reshape(-1, 1, 3), kps, skts, bones, render_kwargs=pk, netchunk=1024,
                  fwd_type="density")
    meta = dict(seed=cfg["seed"], sha256=anerf_syn.checkpoint_sha256(ck), NJ=cfg["NJ"], S=cfg["S"], I=cfg["I"],
                D=cfg["D"], W=cfg["W"], tau=cfg["tau"], H=sc["H"], focal=sc["focal"], ext_scale=0.001, chunk=4096,
                framecode=0, res=cfg["res"], radius=cfg["radius"], flags=cfg.get("flags", []),
                cb=bool(cfg.get("cb", False)), tau_b=cfg.get("tau_b"))
    data = {"kps": sc["kps"][0:1], "skts": sc["skts"][0:1], "bones": sc["bones"][0:1], "pts": pts,
            "grid_density": grid.numpy(), "pts_density": dens.numpy()}
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, meta=np.array(repr(meta)), **data)
    print(f"wrote {path}  grid={grid.shape}  pts={dens.shape}  ({os.path.getsize(path) / 1024:.0f} KiB)")


def make(name, cfg, mods, tmp):
    import torch
    if cfg["kind"] == "density":
        return make_density(name, cfg, mods, tmp)
    run_nerf = mods[0]
    args, render_kwargs, ck = build_reference(mods, cfg, os.path.join(tmp, name))
    sc = scene_for(cfg)
    sha = anerf_syn.checkpoint_sha256(ck)
    meta = dict(seed=cfg["seed"], sha256=sha, NJ=cfg["NJ"], S=cfg["S"], I=cfg["I"], D=cfg["D"], W=cfg["W"],
                tau=cfg["tau"], H=sc["H"], focal=sc["focal"], ext_scale=0.001, chunk=4096,
                framecode=int(cfg["kind"] == "framecode"), mr=cfg.get("mr", 7), flags=cfg.get("flags", []),
                drop=cfg.get("drop", []), mrv=cfg.get("mrv", 4), single=bool(cfg.get("single", False)),
                sched=cfg.get("sched"), white_bkgd=bool(cfg.get("white_bkgd", False)),
                n_frames=int(cfg.get("n_frames", 1)), cb=bool(cfg.get("cb", False)), tau_b=cfg.get("tau_b"))
    data = {"c2ws": sc["c2ws"], "kps": sc["kps"], "skts": sc["skts"], "bones": sc["bones"]}
    (o, d), vidx, cyls, (tl, br) = rays_for(mods, sc)
    sc["cyls"] = cyls
    data.update(cyls=cyls, valid_idx=vidx, tl=np.asarray(tl), br=np.asarray(br))
    if cfg["kind"] == "frame":
        bg_imgs, bg_indices = bg_for(cfg)
        with torch.no_grad():
            rgbs, disps, accs, vids, bbs = run_nerf.render_path(
                torch.from_numpy(sc["c2ws"]), (sc["H"], sc["W"], sc["focal"]), 4096, render_kwargs,
                kp=torch.from_numpy(sc["kps"]), skts=torch.from_numpy(sc["skts"]),
                bones=torch.from_numpy(sc["bones"]), ret_acc=True, ext_scale=0.001,
                white_bkgd=bool(cfg.get("white_bkgd", False)), bg_imgs=bg_imgs, bg_indices=bg_indices)
        data.update(frame_rgb=rgbs, frame_disp=disps, frame_acc=accs)
        if bg_imgs is not None:
            data.update(bg_imgs=bg_imgs, bg_indices=bg_indices)
        data.update(**{f"frame_valid_idx_{f}": v.numpy() for f, v in enumerate(vids)})
        sel = np.arange(min(64, len(vidx)))
    elif cfg["kind"] == "nanfill":
        # contiguous 4096-ray chunk starting at the top of the box: its corner rays miss the cylinder
        sel = np.arange(0, min(4096, len(vidx)))
    else:
        # a contiguous run from the middle of the box (one NaN-fill chunk)
        start = len(vidx) // 2 - cfg["n_rays"] // 2
        sel = np.arange(start, start + cfg["n_rays"])
    o_s, d_s = o[sel], d[sel]
    cams = None
    if cfg["kind"] == "framecode":
        cams = np.where(np.arange(len(sel)) % 3 == 0, 2.0, 4.0).astype(np.float32)
    ret = render_subset(mods, render_kwargs, o_s, d_s, sc, cams=cams)
    data.update(sel=sel, rays_o=o_s.numpy(), rays_d=d_s.numpy(),
                **{"out_" + k: v for k, v in ret.items()})
    if cams is not None:
        data["cams"] = cams
        # eval-mode mean code: every cam index < 0 (core/networks/embedding.py:23-24)
        cams_neg = np.full(len(sel), -1.0, np.float32)
        ret_neg = render_subset(mods, render_kwargs, o_s, d_s, sc, cams=cams_neg)
        data["cams_neg"] = cams_neg
        data.update(**{"outneg_" + k: v for k, v in ret_neg.items()})
    if cfg["kind"] in ("rays", "framecode"):
        data.update(stage_dump(mods, render_kwargs, o_s, d_s, sc, n_stage=4, cams=cams))
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, meta=np.array(repr(meta)), **data)
    print(f"wrote {path}  rays={len(sel)}  ({os.path.getsize(path) / 1024:.0f} KiB)")


def bbox_table(mods):
    """Integer boxes / pixel counts of the full-size frames of every config (hazard H2)."""
    import torch
    _, _, _, ray_utils, _ = mods
    rows = {}
    for name, (H, NJ, seed) in {"c2": (256, 24, 12), "c3": (512, 24, 13), "c4": (512, 65, 14),
                                "c5": (1024, 24, 13), "c3_f3": (512, 24, 40)}.items():
        sc = anerf_syn.make_scene(n_joints=NJ, H=H, W=H, seed=seed, n_frames=3, yaw_step=0.4)
        rays, vids, cyls, bbs = ray_utils.kp_to_valid_rays(torch.from_numpy(sc["c2ws"]), H, H, sc["focal"],
                                                           kps=torch.from_numpy(sc["kps"]), ext_scale=0.001)
        rows[name + "_tl"] = np.stack([np.asarray(b[0]) for b in bbs])
        rows[name + "_br"] = np.stack([np.asarray(b[1]) for b in bbs])
        rows[name + "_n"] = np.array([len(v) for v in vids])
        rows[name + "_cyls"] = cyls.numpy()
        rows[name + "_rays_d_first"] = np.stack([r[1][:8].numpy() for r in rays])
        rows[name + "_rays_d_last"] = np.stack([r[1][-8:].numpy() for r in rays])
        rows[name + "_rays_o"] = np.stack([r[0][0].numpy() for r in rays])
        rows[name + "_meta"] = np.array([H, NJ, seed])
    path = os.path.join(HERE, "bboxes.npz")
    np.savez_compressed(path, **rows)
    print(f"wrote {path}")


def random_boxes_table(mods, n=400):
    """Cylinders and integer boxes of n random frames straight from the reference's
    get_kp_bounding_cylinder + cylinder_to_box_2d (the calls kp_to_valid_rays makes,
    ray_utils.py:89-123): random poses, camera distances / yaws / pitches, focals (scalar or
    (fx, fy)), principal points and image sizes, incl. boxes clipped at the image border."""
    sk = mods[4]
    rs = np.random.RandomState(777)
    parents, rest = anerf_syn.skeleton(24)
    rows = {k: [] for k in ("kps", "c2w", "focal", "center", "has_center", "hw", "cyl", "tl", "br")}
    for _ in range(n):
        bones = rs.normal(scale=0.3, size=(24, 3))
        bones[0] = [np.pi, 0.0, 0.0] + rs.normal(scale=0.3, size=3)
        l2ws = anerf_syn.pose_l2ws(bones, rest * rs.uniform(0.5, 1.5), parents)
        kps = (l2ws[:, :3, 3] + rs.normal(scale=0.3, size=3)).astype(np.float32)
        c2w = anerf_syn.camera_c2w(distance=rs.uniform(2.5, 9.0), yaw=rs.uniform(-np.pi, np.pi))
        pitch = rs.uniform(-0.3, 0.3)
        rx = np.array([[1, 0, 0, 0], [0, np.cos(pitch), -np.sin(pitch), 0], [0, np.sin(pitch), np.cos(pitch), 0],
                       [0, 0, 0, 1]])
        c2w = (rx @ c2w).astype(np.float32)
        H, W = int(rs.choice([64, 200, 512, 1000])), int(rs.choice([64, 256, 512, 777]))
        f = np.array([rs.uniform(0.8, 2.0) * H, rs.uniform(0.8, 2.0) * H]) if rs.rand() < 0.3 else \
            np.array([rs.uniform(0.8, 2.0) * H] * 2)
        has_c = rs.rand() < 0.3
        center = np.array([rs.uniform(0.3, 0.7) * W, rs.uniform(0.3, 0.7) * H]) if has_c else np.zeros(2)
        ext = 0.001
        cyl = sk.get_kp_bounding_cylinder(kps[None], skel_type=sk.SMPLSkeleton, ext_scale=ext, extend_mm=250,
                                          top_expand_ratio=1.6, bot_expand_ratio=1.1, head="-y")[0]
        cyl = np.asarray(cyl, dtype=np.float32)   # torch.FloatTensor(cylinder_params) in kp_to_valid_rays
        w2c = sk.nerf_c2w_to_extrinsic(c2w)
        focal = float(f[0]) if f[0] == f[1] else f
        tl, br, _ = sk.cylinder_to_box_2d(cyl, [H, W, focal], w2c, center=center if has_c else None)
        for k, v in (("kps", kps), ("c2w", c2w), ("focal", f), ("center", center), ("has_center", has_c),
                     ("hw", (H, W)), ("cyl", cyl), ("tl", tl), ("br", br)):
            rows[k].append(np.asarray(v))
    path = os.path.join(HERE, "boxes_random.npz")
    np.savez_compressed(path, **{k: np.stack(v) for k, v in rows.items()})
    print(f"wrote {path}")


def kinematics_table(mods):
    """Pose -> skeleton transforms from the reference's own functions:
    * PoseOptLayer.calculate_kinematic (core/pose_opt.py:372-445, unrolled chain :482-521) with the
      6-D rotation parameters (rot6d_to_rotmat, skeleton_utils.py:420-436, is plain torch; the
      axis-angle branch needs pytorch3d, which is absent here, so it is not run);
    * get_kinematic_chain_T (pose_opt.py:448-479) on 6-D rotations;
    * get_smpl_l2ws (skeleton_utils.py:334-376, numpy float64 + scipy Rotation) on axis-angle bones
      for SMPL-24 and the 65-joint stress skeleton, incl. zero and tiny rotation vectors."""
    import torch
    po = importlib.import_module("core.pose_opt")
    sk = mods[4]
    rs = np.random.RandomState(1234)
    rows = {}
    F = 6
    parents, rest24 = anerf_syn.skeleton(24)
    rest = (rest24 * 0.7).astype(np.float32)[None]
    bones6 = rs.normal(size=(F, 24, 6)).astype(np.float32)
    pelvis = rs.normal(scale=0.5, size=(F, 3)).astype(np.float32)
    L = po.PoseOptLayer.__new__(po.PoseOptLayer)   # __init__ would call pytorch3d's axis_angle_to_matrix
    torch.nn.Module.__init__(L)
    L.skel_type, L.use_cache, L.unroll_kinematic_chain, L.use_rot6d = sk.SMPLSkeleton, False, True, True
    L.rest_pose_idxs, L.kp_map, L.kp_uidxs, L.root_id, L.N_kps = None, None, None, 0, F
    L.register_buffer("rest_pose", torch.tensor(rest))
    L.register_parameter("pelvis", torch.nn.Parameter(torch.tensor(pelvis)))
    L.register_parameter("bones", torch.nn.Parameter(torch.tensor(bones6)))
    idxs = np.array([3, 0, 5, 3, 1], dtype=np.int64)
    with torch.no_grad():
        kp, bone, skts, l2ws, rots = L.calculate_kinematic(idxs)
    rows.update(ck_bones6=bones6, ck_pelvis=pelvis, ck_rest=rest, ck_idxs=idxs, ck_kp=kp.numpy(),
                ck_bone=bone.numpy(), ck_skts=skts.numpy(), ck_l2ws=l2ws.numpy(), ck_rots=rots.numpy())
    with torch.no_grad():
        kpsT, _, sktsT, l2wsT, rotsT = po.get_kinematic_chain_T(torch.tensor(rest), torch.tensor(bones6[:4]))
    rows.update(ct_kps=kpsT.numpy(), ct_skts=sktsT.numpy(), ct_l2ws=l2wsT.numpy(), ct_rots=rotsT.numpy())
    # get_smpl_l2ws: float64 numpy/scipy, SMPL-24 and 65 joints
    for tag, nj in (("s24", 24), ("s65", 65)):
        par, rst = anerf_syn.skeleton(nj)
        skel = sk.SMPLSkeleton if nj == 24 else sk.Skeleton(
            joint_names=[f"j{i}" for i in range(nj)], joint_trees=par, root_id=0,
            nonroot_id=list(range(1, nj)), cutoffs={}, end_effectors=[])
        bones = rs.normal(scale=0.4, size=(4, nj, 3)).astype(np.float32)
        bones[0, 1] = 0.0
        bones[0, 2] = [1e-5, -2e-5, 0.5e-5]
        bones[1, 3] = [2e-4, 0.0, 0.0]
        bones[2, 0] = [np.pi, 0.0, 0.0]
        scale = 0.8
        l2 = np.stack([sk.get_smpl_l2ws(b.astype(np.float64), rst.astype(np.float64), scale, skel_type=skel)
                       for b in bones])
        rows[f"gl_{tag}_bones"] = bones
        rows[f"gl_{tag}_rest"] = rst
        rows[f"gl_{tag}_parents"] = par.astype(np.int32)
        rows[f"gl_{tag}_scale"] = np.array(scale)
        rows[f"gl_{tag}_l2ws"] = l2
        rows[f"gl_{tag}_skts"] = np.linalg.inv(l2)
    path = os.path.join(HERE, "kinematics.npz")
    np.savez_compressed(path, **rows)
    print(f"wrote {path}")


def kinematics_grad_table(mods):
    """Pose-optimisation gradients from the reference's own autograd:
    PoseOptLayer.calculate_kinematic on 6-D rotations (the axis-angle branch needs pytorch3d, absent
    here) with repeated indices, loss = sum of seeded weights times kp, skts (all 16 entries, the
    gradient torch.inverse propagates), l2ws and rots; stores d loss / d bones (6-D) and / d pelvis."""
    import torch
    po = importlib.import_module("core.pose_opt")
    sk = mods[4]
    rs = np.random.RandomState(4321)
    F = 6
    parents, rest24 = anerf_syn.skeleton(24)
    rest = (rest24 * 0.7).astype(np.float32)[None]
    bones6 = rs.normal(size=(F, 24, 6)).astype(np.float32)
    pelvis = rs.normal(scale=0.5, size=(F, 3)).astype(np.float32)
    L = po.PoseOptLayer.__new__(po.PoseOptLayer)   # __init__ would call pytorch3d's axis_angle_to_matrix
    torch.nn.Module.__init__(L)
    L.skel_type, L.use_cache, L.unroll_kinematic_chain, L.use_rot6d = sk.SMPLSkeleton, False, True, True
    L.rest_pose_idxs, L.kp_map, L.kp_uidxs, L.root_id, L.N_kps = None, None, None, 0, F
    L.register_buffer("rest_pose", torch.tensor(rest))
    L.register_parameter("pelvis", torch.nn.Parameter(torch.tensor(pelvis)))
    L.register_parameter("bones", torch.nn.Parameter(torch.tensor(bones6)))
    idxs = np.array([3, 0, 5, 3, 1], dtype=np.int64)
    kp, bone, skts, l2ws, rots = L.calculate_kinematic(idxs)
    n = len(idxs)
    w = {"kp": rs.normal(size=(n, 24, 3)), "skts": rs.normal(size=(n, 24, 4, 4)),
         "l2ws": rs.normal(size=(n, 24, 4, 4)), "rots": rs.normal(size=(n, 24, 3, 3))}
    w = {k: v.astype(np.float32) for k, v in w.items()}
    loss = ((kp * torch.tensor(w["kp"])).sum() + (skts * torch.tensor(w["skts"])).sum() +
            (l2ws * torch.tensor(w["l2ws"])).sum() + (rots * torch.tensor(w["rots"])).sum())
    loss.backward()
    rows = dict(bones6=bones6, pelvis=pelvis, rest=rest, idxs=idxs, loss=np.float64(loss.item()),
                g_bones6=L.bones.grad.numpy(), g_pelvis=L.pelvis.grad.numpy(),
                **{"w_" + k: v for k, v in w.items()})
    path = os.path.join(HERE, "kinematics_grad.npz")
    np.savez_compressed(path, **rows)
    print(f"wrote {path}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    import torch
    torch.set_num_threads(8)
    mods = import_reference()
    with tempfile.TemporaryDirectory() as tmp:
        for name, cfg in CONFIGS.items():
            if a.only and a.only != name:
                continue
            make(name, cfg, mods, tmp)
    if not a.only or a.only == "bboxes":
        bbox_table(mods)
    if not a.only or a.only == "kinematics":
        kinematics_table(mods)
    if not a.only or a.only == "kinematics_grad":
        kinematics_grad_table(mods)
    if not a.only or a.only == "boxes_random":
        random_boxes_table(mods)


if __name__ == "__main__":
    main()

"""Golden fixtures for the TRAINING render path, made by running the
reference's own `RayCaster.render_rays` in training mode (core/raycasters.py:361-474: perturb=1,
raw_noise_std=1, stochastic importance sampling) and autograd on CPU.

The reference draws its randomness with torch.rand / torch.randn (ray_utils.py:240, 168;
nerf.py:176); here those two functions are replaced, for the duration of the call, by a queue of
pre-drawn tensors that are stored in the fixture, so the build's training path can be fed the
same draws.  Each fixture holds the inputs (per-ray rays, skeletons, cylinders, targets), the
draws, the outputs, the loss, the gradient w.r.t. the per-ray skeleton transforms (pose
optimisation) and the gradients of every network parameter (in full for small tensors, else a
fixed strided sample of entries plus the norm).

Runs ONLY in the build container (/root/reference).  Usage: python tests/golden/make_train_golden.py
"""
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402

CONFIGS = {
    "t1_s32i16_d4w128": dict(H=128, NJ=24, S=32, I=16, D=4, W=128, tau=20.0, kind="rays", seed=31, n_rays=96,
                             n_poses=3),
    "t2_s64i16_d8w256": dict(H=256, NJ=24, S=64, I=16, D=8, W=256, tau=79.6, kind="rays", seed=32, n_rays=48,
                             n_poses=2),
    "t3_softplus_fc": dict(H=128, NJ=24, S=32, I=16, D=4, W=128, tau=20.0, kind="framecode", seed=33, n_rays=64,
                           n_poses=2, flags=["--density_type", "softplus", "--softplus_shift", "1.0"]),
    # the tau schedule: RayCaster.update_embed_fns at global step 250,000 (cutoff_step 250, rate 10:
    # tau = 20 * 10 ** 1 = 200) before the step, from a checkpoint at tau 20
    "t4_tau200": dict(H=128, NJ=24, S=32, I=16, D=4, W=128, tau=20.0, kind="rays", seed=34, n_rays=64, n_poses=2,
                      global_step=250000, cutoff_step=250, cutoff_rate=10.0),
    # single_net + multires_views 0 (configs/surreal/surreal_single.txt's flags, smaller net)
    "t5_single_mrv0": dict(H=128, NJ=24, S=48, I=24, D=4, W=128, tau=20.0, kind="rays", seed=35, n_rays=64,
                           n_poses=2, mrv=0, single=True),
    # --lindisp and --ray_noise_std (sample_pts / sample_pts_is add randn_like(pts) * std,
    # raycasters.py:660-661, 673-674): two more recorded draws of shape (N, S, 3) and (N, I, 3)
    "t6_lindisp_raynoise": dict(H=128, NJ=24, S=32, I=16, D=4, W=128, tau=20.0, kind="rays", seed=36, n_rays=64,
                                n_poses=2, lindisp=True, ray_noise_std=0.01),
    "t7_single_raynoise": dict(H=128, NJ=24, S=32, I=16, D=4, W=128, tau=20.0, kind="rays", seed=37, n_rays=64,
                               n_poses=2, single=True, ray_noise_std=0.02),
    # --freq_schedule: checkpoint at sched_alpha 1.0 (--init_freq 1), update_embed_fns at step 1,700
    # (freq_schedule_step 5: alpha = 1 + 5 * 1700 / 5000 = 2.7; tau 20 -> 20.3) before the step; D = 8
    "t8_freqsched": dict(H=128, NJ=24, S=32, I=16, D=8, W=128, tau=20.0, kind="rays", seed=38, n_rays=64,
                         n_poses=2, flags=["--freq_schedule", "--init_freq", "1.0"], sched=1.0,
                         global_step=1700, cutoff_step=250, cutoff_rate=10.0),
    # --cut_to_dist with --cutoff_shift: the training encoder and its gradient to the poses
    "t9_cutto_shift": dict(H=128, NJ=24, S=32, I=16, D=4, W=128, tau=20.0, kind="rays", seed=39, n_rays=64,
                           n_poses=2, flags=["--cut_to_dist", "--cutoff_shift"]),
    # --cutoff_bones: bone directions windowed by the bone embedder's own tau (35) / cutoffs; D = 8
    # (the skip layer's x part), the gradient through w_b to the poses.  (Seed 40 gave a coarse view-layer
    # unit whose views_linears.0.bias gradient differed from the reference by 1.25e-5 = 2.3e-3 of its max
    # identically in all three MLP modes (so decided before the arithmetic modes differ: consistent
    # with a pre-activation within the reference's float32 rounding of 0, not isolated further),
    # with every output, the loss and dL/dskts within their bounds.)
    "t10_cutoffbones": dict(H=128, NJ=24, S=32, I=16, D=8, W=128, tau=20.0, kind="rays", seed=44, n_rays=64,
                            n_poses=2, flags=["--cutoff_bones"], cb=True, tau_b=35.0),
    # (round 5) multires 5 / multires_views 2 (the training encoder backward's generic instance) with
    # --view_type world (un-normalised joint-frame ray directions: the identity's gradient to the poses)
    "t11_mr5_mrv2_world": dict(H=128, NJ=24, S=32, I=16, D=4, W=128, tau=20.0, kind="rays", seed=45, n_rays=64,
                               n_poses=2, mr=5, mrv=2, flags=["--view_type", "world"]),
    # (round 5) the staged encoders (include/anerf.h): relpos kp inputs, ray angles, bone frequencies windowed
    # by --cutoff_bones; D = 8 (the skip layer's [x | h])
    "t12_staged_relpos_rayangle_mrb2": dict(H=128, NJ=24, S=32, I=16, D=8, W=128, tau=20.0, kind="rays", seed=46,
                                            n_rays=64, n_poses=2, cb=True, tau_b=35.0,
                                            flags=["--kp_dist_type", "relpos", "--view_type", "rayangle",
                                                   "--multires_bones", "2", "--cutoff_bones"]),
    # --kp_dist_type querypts (no gradient to the poses through the kp part) with --cutoff_shift
    "t13_querypts_shift": dict(H=128, NJ=24, S=32, I=16, D=4, W=128, tau=20.0, kind="rays", seed=47, n_rays=64,
                               n_poses=2, flags=["--kp_dist_type", "querypts", "--cutoff_shift"]),
    # (round 6) BASELINE config 4's 65-joint skeleton at 8 x 256 (the LDS-pressure case): the view-window layout
    # with zero-padded rows (1170 kp + bone columns -> 1172, then the 65 windows; G 65 x 128 in anerf_train_view_mix's
    # LDS) and the full view columns both run against it; the fused hidden-layer backward at W 256
    "t14_nj65_d8w256": dict(H=256, NJ=65, S=32, I=16, D=8, W=256, tau=20.0, kind="rays", seed=48, n_rays=32,
                            n_poses=2),
}
FULL_LIMIT = 20000   # parameters with more entries are sampled
SAMPLE = 4096


def sample_idx(numel):
    step = max(1, numel // SAMPLE)
    return np.arange(0, numel, step)[:SAMPLE]


def make(name, cfg, mods, tmp):
    import torch
    import torch.nn.functional as F
    _, _, raycasters, ray_utils, _ = mods
    args, render_kwargs, ck = mg.build_reference(mods, cfg, os.path.join(tmp, name))
    rc = render_kwargs["ray_caster"]
    pk = render_kwargs["preproc_kwargs"]
    S, I, NJ, P = cfg["S"], cfg["I"], cfg["NJ"], cfg["n_poses"]
    sc = mg.anerf_syn.make_scene(n_joints=NJ, H=cfg["H"], W=cfg["H"], seed=cfg["seed"], n_frames=P, yaw_step=0.5)
    rng = np.random.default_rng(cfg["seed"] + 1000)
    per = cfg["n_rays"] // P
    o_l, d_l, pose_l, cyl_l = [], [], [], []
    for f in range(P):
        rays, vids, cyls, _ = ray_utils.kp_to_valid_rays(torch.from_numpy(sc["c2ws"][f:f + 1]), sc["H"], sc["W"],
                                                         sc["focal"], kps=torch.from_numpy(sc["kps"][f:f + 1]),
                                                         ext_scale=0.001)
        sel = np.sort(rng.choice(len(vids[0]), per, replace=False))
        o_l.append(rays[0][0][sel].numpy())
        d_l.append(rays[0][1][sel].numpy())
        pose_l.append(np.full(per, f))
        cyl_l.append(np.repeat(cyls.numpy()[0:1], per, 0))
    o = np.concatenate(o_l).astype(np.float32)
    d = np.concatenate(d_l).astype(np.float32)
    pose = np.concatenate(pose_l).astype(np.int64)
    cyl = np.concatenate(cyl_l).astype(np.float32)
    n = len(o)
    T = S + I
    draws = {"t_rand": rng.random((n, S), dtype=np.float32),
             "noise0": rng.standard_normal((n, S), dtype=np.float32),
             "u": rng.random((n, I), dtype=np.float32),
             "noise1": rng.standard_normal((n, T), dtype=np.float32)}
    rns = float(cfg.get("ray_noise_std", 0.0))
    if rns > 0:
        draws["pts_noise0"] = rng.standard_normal((n, S, 3), dtype=np.float32)
        draws["pts_noise1"] = rng.standard_normal((n, I, 3), dtype=np.float32)
    target = rng.random((n, 3), dtype=np.float32)
    bg = rng.random((n, 3), dtype=np.float32)
    cams = None
    if cfg["kind"] == "framecode":
        cams = (np.arange(n) % 5).astype(np.float32)

    # the reference's draw order: t_rand (sample_from_lineseg), [points noise (sample_pts)], raw noise
    # (raw2outputs), u (sample_pdf), [points noise of the new samples (sample_pts_is)], raw noise
    queue = [("rand", draws["t_rand"])] + ([("randn_like", draws["pts_noise0"])] if rns > 0 else []) + \
            [("randn", draws["noise0"]), ("rand", draws["u"])] + \
            ([("randn_like", draws["pts_noise1"])] if rns > 0 else []) + [("randn", draws["noise1"])]
    real_rand, real_randn, real_randn_like = torch.rand, torch.randn, torch.randn_like

    def fake(kind):
        def fn(*shape, **kw):
            k, arr = queue.pop(0)
            if kind == "randn_like":
                shape = (tuple(shape[0].shape),)
            shp = tuple(shape[0]) if len(shape) == 1 and not isinstance(shape[0], int) else tuple(shape)
            assert k == kind and shp == arr.shape, (kind, shp, k, arr.shape)
            return torch.from_numpy(arr.copy())
        return fn

    rb = np.concatenate([o, d, np.zeros((n, 1)), np.ones((n, 1)), d / np.linalg.norm(d, axis=-1, keepdims=True)],
                        -1).astype(np.float32)
    skts_t = torch.from_numpy(sc["skts"][pose]).requires_grad_(True)
    kp_t = torch.from_numpy(sc["kps"][pose])
    bones_t = torch.from_numpy(sc["bones"][pose])
    rc.train()
    if "global_step" in cfg:
        args.cutoff_step, args.cutoff_rate = cfg["cutoff_step"], cfg["cutoff_rate"]
        rc.update_embed_fns(cfg["global_step"], args)
    taus = (float(rc.embed_fn.get_tau()), float(rc.embeddirs_fn.get_tau()))
    torch.rand, torch.randn, torch.randn_like = fake("rand"), fake("randn"), fake("randn_like")
    try:
        ret = rc(torch.from_numpy(rb), S, kp_batch=kp_t, skts=skts_t, cyls=torch.from_numpy(cyl), bones=bones_t,
                 cams=None if cams is None else torch.from_numpy(cams), perturb=1.0, N_importance=I,
                 raw_noise_std=1.0, lindisp=bool(cfg.get("lindisp", False)), ray_noise_std=rns, preproc_kwargs=pk)
    finally:
        torch.rand, torch.randn, torch.randn_like = real_rand, real_randn, real_randn_like
    assert not queue, "the reference drew fewer random tensors than expected"
    tgt, bgt = torch.from_numpy(target), torch.from_numpy(bg)
    # Trainer._compute_nerf_loss (MSE, use_background) on fine and coarse outputs
    loss = (F.mse_loss(ret["rgb_map"] + (1 - ret["acc_map"])[:, None] * bgt, tgt) +
            F.mse_loss(ret["rgb0"] + (1 - ret["acc0"])[:, None] * bgt, tgt))
    loss.backward()
    meta = dict(seed=cfg["seed"], sha256=mg.anerf_syn.checkpoint_sha256(ck), NJ=NJ, S=S, I=I, D=cfg["D"],
                W=cfg["W"], tau=cfg["tau"], H=sc["H"], focal=sc["focal"], ext_scale=0.001, chunk=4096,
                framecode=int(cfg["kind"] == "framecode"), mr=cfg.get("mr", 7), flags=cfg.get("flags", []), drop=[],
                raw_noise_std=1.0, n_poses=P, mrv=cfg.get("mrv", 4), single=bool(cfg.get("single", False)),
                global_step=cfg.get("global_step"), cutoff_step=cfg.get("cutoff_step"),
                cutoff_rate=cfg.get("cutoff_rate"), tau_step=taus, lindisp=bool(cfg.get("lindisp", False)),
                ray_noise_std=rns, sched=cfg.get("sched"), cb=bool(cfg.get("cb", False)), tau_b=cfg.get("tau_b"),
                sched_step=(float(rc.embed_fn.sched_alpha), float(rc.embeddirs_fn.sched_alpha))
                if cfg.get("sched") is not None else None)
    data = dict(rays=rb, pose=pose, skts=sc["skts"][pose], kps=sc["kps"][pose], bones=sc["bones"][pose], cyls=cyl,
                target=target, bg=bg, loss=np.float32(loss.item()), grad_skts=skts_t.grad.numpy(),
                **{"rand_" + k: v for k, v in draws.items()},
                **{"out_" + k: v.detach().numpy() for k, v in ret.items()})
    if cams is not None:
        data["cams"] = cams
    for net_name, net in (("fn", rc.network), ("fine", rc.network_fine)):
        for pname, p in net.named_parameters():
            if p.grad is None:
                continue
            g = p.grad.numpy().reshape(-1)
            key = f"grad_{net_name}__{pname}"
            if g.size <= FULL_LIMIT:
                data[key] = g
            else:
                data[key + "__idx"] = sample_idx(g.size)
                data[key] = g[data[key + "__idx"]]
                data[key + "__norm"] = np.float64(np.linalg.norm(g.astype(np.float64)))
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, meta=np.array(repr(meta)), **data)
    print(f"wrote {path}  rays={n}  loss={loss.item():.6f}  ({os.path.getsize(path) / 1024:.0f} KiB)")


def main():
    mods = mg.import_reference()
    only = sys.argv[1:]
    with tempfile.TemporaryDirectory() as tmp:
        for name, cfg in CONFIGS.items():
            if only and name not in only:
                continue
            make(name, cfg, mods, tmp)


if __name__ == "__main__":
    main()

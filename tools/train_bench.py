"""Training-step benchmark at the reference's training configuration
(configs/surreal/surreal.txt: N_rand 2048 rays, N_samples 64, N_importance 16, 8x256 nets,
raw_noise_std 1, perturb 1, rays drawn from N_sample_images 128 images, i.e. 128 skeletons with pose
optimisation on): one step = render_rays forward + the MSE/background loss + backward (networks and
the per-image skeleton deltas) + Adam.  Synthetic scene and seeded weights.

Prints one JSON line: training rays/s, steps/s, the MLP's GEMM FLOPs (3 x forward: the input
gradient is needed for the pose gradient) and their rate against the peak of the MFMA pipe the
GEMMs run on: BF16 dense for the split-bf16 modes ("mixed": bf16x6 forward, bf16x3 backward), FP32
matrix for "fp32".
Usage: python tools/train_bench.py [--steps K] [--warmup W] [--rays N]
"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _ablib  # noqa: E402,F401  (ANERF_LIB_PATH: an experiment build, A/B tooling only)
FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md, FP32 matrix
BF16_MFMA_PEAK_TFLOPS = 2516.6  # MI355X_MICROARCH.md, BF16 dense


def parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rays", type=int, default=2048)
    ap.add_argument("--images", type=int, default=128)
    ap.add_argument("--joints", type=int, default=24,
                    help="skeleton joints: 24 (SMPL) or more (synthetic skeleton, e.g. 65 = BASELINE config 4's "
                         "LDS-pressure case)")
    ap.add_argument("--samples", type=int, default=64)
    ap.add_argument("--importance", type=int, default=16)
    ap.add_argument("--mlp", default="mixed", choices=["mixed", "mixed16", "bf16x6", "bf16x3", "fp32"],
                    help="training MLP arithmetic (train.TrainRayCaster mlp=)")
    ap.add_argument("--no-wgrad-overlap", action="store_true",
                    help="ablation: the weight gradients on the caller's stream (mlp.WGRAD_OVERLAP off)")
    ap.add_argument("--no-fused-backward", action="store_true",
                    help="ablation: the hidden layers' backward as the two GEMMs (mlp.FUSED_BACKWARD off)")
    ap.add_argument("--full-view", action="store_true",
                    help="ablation: the full view columns instead of the view-window layout (TrainRayCaster.view_windows)")
    ap.add_argument("--adam", default="foreach", choices=["fused", "foreach"],
                    help="torch.optim.Adam's implementation (foreach: the drop-in's, create_raycaster; fused: one "
                         "kernel per step, +0.5 %%, but it does not advance the version counters the eval caster "
                         "reads)")
    ap.add_argument("--host-index", action="store_true",
                    help="hand PoseOptLayer the host image indices (np.unique per step) instead of the device batch")
    ap.add_argument("--pose", default="kinematic", choices=["kinematic", "delta"],
                    help="pose optimisation: kinematic (default; Trainer.train_batch with --opt_pose --opt_rot6d, "
                         "core/trainer.py:230-273, 382-403, 451-481): a kinematics.PoseOptLayer over the images runs "
                         "calculate_kinematic for every ray's image each step (anerf_pose_kinematics and its backward), "
                         "the rot6d anchor loss (opt_pose_tol 0.01, opt_pose_coef 2.0, configs/h36m/h36m_prot2.txt) "
                         "joins the loss and a second Adam (opt_pose_lrate 5e-4) steps the poses every step; delta "
                         "(rounds 1-5): a skts + delta leaf per image")
    ap.add_argument("--no-fused-skip", action="store_true",
                    help="ablation: the skip layer's backward as two GEMMs and its x part apart from layer 0's")
    ap.add_argument("--fine-stream", action="store_true",
                    help="experiment: the fine pass on a stream of its own (train.FINE_STREAM; off in the product: "
                         "-1.5 to -2 %, profiles/r06st/ab.txt)")
    ap.add_argument("--no-fine-stream", action="store_true", help="(the default; kept for older scripts)")
    ap.add_argument("--no-fused-head", action="store_true",
                    help="ablation: the heads' backward as two GEMMs")
    ap.add_argument("--no-defer-sync", action="store_true",
                    help="ablation: the caller's stream waits for the weight-gradient side stream at the end of the "
                         "MLP's backward (not at the end of the whole backward)")
    ap.add_argument("--no-forward-persistent", action="store_true",
                    help="ablation: the hidden layers' forward on anerf_mlp_gemm instead of anerf_mlp_forward_hidden")
    ap.add_argument("--split-single", action="store_true",
                    help="ablation: one split launch per weight instead of the batched split")
    ap.add_argument("--probe", default="", choices=["", "no-hidden-reduce", "no-wgrad", "no-wgrad-no-reduce"],
                    help="TIMING ONLY (wrong gradients): skip the fused backward's slab reduce and/or the other "
                         "layers' weight gradients, to bound what speeding them up could give")
    return ap


def measure(a, dev=None):
    """One training-step measurement (the dict main() prints); also bench.py's `training` leg."""
    anerf = importlib.import_module("a-nerf_amd")
    syn = importlib.import_module("a-nerf_amd.synthetic")
    train = importlib.import_module("a-nerf_amd.train")
    dev = dev or torch.device("cuda:0")
    if getattr(a, "split_single", False):
        mlp = importlib.import_module("a-nerf_amd.mlp")
        mlp.split_weights = lambda jobs, prec: [mlp.split_weight(j[0], j[1], j[2] if len(j) > 2 else prec)
                                                   for j in jobs]
    S, I, n = a.samples, a.importance, a.rays
    nj = getattr(a, "joints", 24)
    cfg = anerf.RenderConfig(n_joints=nj, N_samples=S, N_importance=I).validate()
    ck = syn.make_checkpoint(13, n_joints=nj, D=8, W=256, fine=True, tau=20.0)
    sc = syn.make_scene(n_joints=nj, H=512, W=512, seed=13, n_frames=a.images, yaw_step=2 * np.pi / a.images)
    idx, cyls, _ = anerf.rays.valid_pixels(sc["c2ws"], 512, 512, sc["focal"], kps=sc["kps"], ext_scale=0.001)
    rng = np.random.default_rng(0)
    probe = getattr(a, "probe", "")
    if probe:
        lib = importlib.import_module("a-nerf_amd._lib").load()
        if "reduce" in probe:
            lib.anerf_mlp_backward_hidden_reduce = lambda *args: 0
        if "wgrad" in probe:
            lib.anerf_mlp_wgrad = lambda *args: 0
    if getattr(a, "no_wgrad_overlap", False):
        importlib.import_module("a-nerf_amd.mlp").WGRAD_OVERLAP = False
    importlib.import_module("a-nerf_amd.mlp").FUSED_BACKWARD = not getattr(a, "no_fused_backward", False)
    importlib.import_module("a-nerf_amd.mlp").FUSED_SKIP = not getattr(a, "no_fused_skip", False)
    importlib.import_module("a-nerf_amd.mlp").FUSED_HEAD = not getattr(a, "no_fused_head", False)
    importlib.import_module("a-nerf_amd.mlp").FORWARD_PERSISTENT = not getattr(a, "no_forward_persistent", False)
    importlib.import_module("a-nerf_amd.mlp").DEFER_WGRAD_SYNC = not getattr(a, "no_defer_sync", False)
    train.FINE_STREAM = bool(getattr(a, "fine_stream", False))  # (the product default: off)
    tr = train.TrainRayCaster(cfg, ck, device=dev, mlp=a.mlp).train()
    tr.view_windows = not getattr(a, "full_view", False)
    adam_kw = {"fused": True} if getattr(a, "adam", "foreach") == "fused" else {"foreach": True}
    kinematic = getattr(a, "pose", "kinematic") == "kinematic"
    if kinematic:  # the reference's PoseOptLayer (core/pose_opt.py:240-445) on 6-D rotations (--opt_rot6d)
        kin = importlib.import_module("a-nerf_amd.kinematics")
        # (rest pose relative to the root, the pelvis parameter = the root keypoint: the chain then reproduces
        # the scene's skeletons, pose_opt.py:398-431 adds the pelvis to every joint)
        skel = kin.SMPLSkeleton if nj == 24 else kin.Skeleton(
            [f"j{i}" for i in range(nj)], np.asarray(sc["parents"]), 0, list(range(1, nj)), {}, None)
        popt = kin.PoseOptLayer(sc["kps"], sc["bones"], sc["rest"][None] - sc["rest"][None, :1], skel,
                                use_rot6d=True, device=dev)
        with torch.no_grad():  # popt_anchors["rots"] (core/pose_opt.py:60-72): the initial poses
            anchor = popt.calculate_kinematic(np.arange(a.images))[4][..., :3, :2].flatten(start_dim=-2).clone()
        opt = torch.optim.Adam(list(tr.parameters()), lr=5e-4, **adam_kw)
        popt_opt = torch.optim.Adam(list(popt.parameters()), lr=5e-4, **adam_kw)
    else:
        skts = torch.from_numpy(sc["skts"]).to(dev)
        delta = torch.zeros_like(skts, requires_grad=True)  # pose optimisation variable per image
        opt = torch.optim.Adam(list(tr.parameters()) + [delta], lr=5e-4, **adam_kw)

    def batch():
        img = rng.integers(0, a.images, n)
        rays = np.empty((n, 11), np.float32)
        for f in np.unique(img):
            sel = np.nonzero(img == f)[0]
            pix = rng.choice(idx[f], len(sel))
            y, x = pix // 512, pix % 512
            c2w = sc["c2ws"][f].astype(np.float64)
            d = np.stack([(x - 256.0) / sc["focal"], -(y - 256.0) / sc["focal"], -np.ones(len(sel))], -1) @ c2w[:3, :3].T
            rays[sel, 0:3] = c2w[:3, 3]
            rays[sel, 3:6] = d
            rays[sel, 8:11] = d / np.linalg.norm(d, axis=-1, keepdims=True)
        rays[:, 6], rays[:, 7] = 0.0, 1.0
        return (torch.from_numpy(rays).to(dev), img, torch.from_numpy(img).to(dev),
                torch.from_numpy(cyls[img]).to(dev), torch.rand(n, 3, device=dev))

    batches = [batch() for _ in range(4)]

    def step(b):
        rb, img_np, img, cy, tgt = b
        opt.zero_grad(set_to_none=True)
        if kinematic:
            # Trainer.get_kp_args (core/trainer.py:285-312): the layer's kinematics for every ray's image
            popt_opt.zero_grad(set_to_none=True)
            kp, bone, sk, _, rots = popt(img_np if a.host_index else img)
            out = tr.render_rays(rb, S, kp_batch=kp, skts=sk, cyls=cy, bones=bone, perturb=1.0, N_importance=I,
                                 raw_noise_std=1.0)
            # Trainer._compute_kp_loss (core/trainer.py:382-403) with --opt_rot6d, tol 0.01, coef 2.0
            kl = (anchor[img] - rots[..., :3, :2].flatten(start_dim=-2)).pow(2.0)[:, 1:]
            kl = torch.lerp(torch.zeros_like(kl), kl - 0.01, (kl > 0.01).float()).sum(-1).mean() * 2.0
            loss = train.nerf_loss(out, tgt, bgs=1.0, use_background=True) + kl
        else:
            out = tr.render_rays(rb, S, skts=(skts + delta)[img], cyls=cy, perturb=1.0, N_importance=I,
                                 raw_noise_std=1.0)
            loss = train.nerf_loss(out, tgt, bgs=1.0, use_background=True)
        loss.backward()
        opt.step()
        if kinematic:  # Trainer.optimize (core/trainer.py:451-481) with opt_pose_step 1
            popt_opt.step()
        return loss

    for i in range(a.warmup):
        step(batches[i % 4])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        step(batches[i % 4])
    t_issue = time.perf_counter() - t0  # (the host's issue time: ~dt when the host, not the GPU, bounds the step)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    flop = 3 * anerf.flops_per_sample(cfg) * n * anerf.samples_per_ray(cfg)
    return {
        "metric": ("training rays/s (Trainer.train_batch: PoseOptLayer kinematics for every ray + render_rays fwd + "
                   "loss (rgb + rot6d pose anchor) + bwd through the nets and the kinematic chain + Adam on both; "
                   "N_rand 2048, 64+16 samples, 8x256, 128 images)" if kinematic else
                   "training rays/s (render_rays fwd + loss + bwd + Adam; N_rand 2048, 64+16 samples, 8x256, "
                   "128 images with a skts + delta pose leaf)"),
        "pose": ("PoseOptLayer: anerf_pose_kinematics + its backward every step, "
                 + ("host indices (np.unique)" if a.host_index else "device indices (all frames + gather)")
                 if kinematic
                 else "skts + delta leaf"),
        "value": round(n / dt, 1), "unit": "rays/s", "ms_per_step": round(1e3 * dt, 3), "steps": a.steps,
        "host_issue_ms_per_step": round(1e3 * t_issue / a.steps, 3),
        **({"probe": probe + " (timing only: wrong gradients)"} if probe else {}),
        "dtype": "fp32" if a.mlp == "fp32" else f"fp32 in/out, MLP GEMMs as split bf16 ({a.mlp})", "mlp": a.mlp,
        "mlp_gemm_flop_per_step": flop, "mlp_tflops": round(flop / dt / 1e12, 2),
        "peak_tflops": FP32_MFMA_PEAK_TFLOPS if a.mlp == "fp32" else BF16_MFMA_PEAK_TFLOPS,
        "frac_of_pipe_peak": round(flop / dt / 1e12 / (FP32_MFMA_PEAK_TFLOPS if a.mlp == "fp32"
                                                       else BF16_MFMA_PEAK_TFLOPS), 4),
        "pipe": "FP32 matrix" if a.mlp == "fp32" else "BF16 dense (the split-bf16 GEMMs' v_mfma_f32_32x32x16_bf16)",
        "precision_note": {"mixed": "forward bf16x6 (fp32-accurate), gradients bf16x3 (~16-bit operands, relative "
                                    "error ~1e-5; pinned at 2e-3 of max |ref| per gradient tensor)",
                           "mixed16": "as mixed, the forward's hidden-to-hidden layers and head as fp16x4 (row-scaled "
                                      "two-way fp16 split, the bf16x6 error bound)",
                           "bf16x6": "fp32-accurate forward and gradients", "bf16x3": "~16-bit operands",
                           "fp32": "torch fp32 GEMMs"}[a.mlp],
        "adam": getattr(a, "adam", "foreach"),
        "hidden_backward": ("fused (anerf_mlp_backward_hidden: input + weight gradients from one read of dY and H)"
                            + ("; the skip layer's h part fused too, its x part merged with layer 0's products"
                               if importlib.import_module("a-nerf_amd.mlp").FUSED_SKIP else "")
                            + ("; the heads (feature_linear + alpha_linear's rank-1 term) fused"
                               if importlib.import_module("a-nerf_amd.mlp").FUSED_HEAD else "")
                            if importlib.import_module("a-nerf_amd.mlp").FUSED_BACKWARD and a.mlp in ("mixed", "bf16x3",
                                                                                                    "mixed16")
                            else "two GEMMs (anerf_mlp_gemm + anerf_mlp_wgrad)"),
        "hidden_forward": (("persistent (anerf_mlp_forward_layer: every trunk layer and feature_linear + alpha; the feature gradient "
                            "on anerf_mlp_gemm_persistent; layer 0's weight-gradient wait deferred to the end of the "
                            "backward)") if importlib.import_module("a-nerf_amd.mlp")
                           .FORWARD_PERSISTENT and a.mlp in ("mixed", "bf16x6", "bf16x3") else "anerf_mlp_gemm"),
        "fine_stream": bool(train.FINE_STREAM),
        "joints": nj,
        "view_layout": (f"view windows (anerf.h ANERF_ENC_VIEW_WINDOWS: {nj} windows per sample + per-ray factors)"
                        if tr.model.view_windows else f"full view columns ({cfg.input_ch_views} per sample)"),
        "data": "synthetic (seeded SMPL-24 poses, 128 cameras on a circle, seeded weights)"}


def main():
    print(json.dumps(measure(parser().parse_args())), flush=True)


if __name__ == "__main__":
    main()

"""Diagnostic (round 5): eval-render throughput of the staged encoders (include/anerf.h) on the training stages,
at config 3's network and sampling (8x256, 64 + 128 samples, tau 79.6) over 32,768 rays of its frame, next to
the fused kernel on the same rays.  Prints one JSON line per encoder setting."""
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
anerf = importlib.import_module("a-nerf_amd")
syn = importlib.import_module("a-nerf_amd.synthetic")


def main():
    sc = syn.make_scene(n_joints=24, H=512, W=512, seed=13)
    idx, cyls, _ = anerf.rays.valid_pixels(sc["c2ws"], 512, 512, sc["focal"], kps=sc["kps"], ext_scale=0.001)
    pix = idx[0][:32768]
    y, x = pix // 512, pix % 512
    c2w = sc["c2ws"][0].astype(np.float64)
    d = np.stack([(x - 256.0) / sc["focal"], -(y - 256.0) / sc["focal"], -np.ones(len(pix))], -1) @ c2w[:3, :3].T
    n = len(pix)
    rb = torch.from_numpy(np.concatenate([np.broadcast_to(c2w[:3, 3], d.shape), d, np.zeros((n, 1)), np.ones((n, 1)),
                                          d / np.linalg.norm(d, axis=-1, keepdims=True)], -1).astype(np.float32)).cuda()
    sk = torch.from_numpy(sc["skts"][0:1]).cuda().expand(n, -1, -1, -1)
    cy = torch.from_numpy(cyls[0:1]).cuda().expand(n, -1)
    cases = [("fused fp16x4 (reference encoders)", {}, 0, "fp16x4"),
             ("staged: kp relpos", {"kp_dist_type": "relpos"}, 0, "fp16x4"),
             ("staged: view rayangle", {"view_type": "rayangle"}, 0, "fp16x4"),
             ("staged: multires_bones 2", {}, 2, "fp16x4")]
    for name, extra, mrb, prec in cases:
        cfg = anerf.RenderConfig(N_samples=64, N_importance=128, precision=prec, extra=extra,
                                 multires_bones=mrb).validate()
        dims = dict(multires_bones=mrb, kp_dims=3 if cfg.kp_relpos else 1, view_dims=1 if cfg.view_angle else 3)
        ck = syn.make_checkpoint(13, n_joints=24, D=8, W=256, fine=True, tau=79.6, **dims)
        rc = anerf.RayCaster(cfg, ck)
        ts = []
        for it in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rc.render_rays(rb, 64, skts=sk, cyls=cy, N_importance=128, chunk=4096, ret_alpha=False)
            torch.cuda.synchronize()
            if it:
                ts.append(time.perf_counter() - t0)
        dt = float(np.mean(ts))
        print(json.dumps({"case": name, "rays": n, "ms": round(dt * 1e3, 2), "rays_per_s": round(n / dt, 1)}))


if __name__ == "__main__":
    main()

"""Diagnostic (round 5): the render kernel's HBM writes per launch.  Renders config 3's
frame (512^2, 64+128 samples, 8x256, fp16x4) a few times, with importance sampling (coarse launch writes
the T-float z hand-off, the fine launch reads it) and without (one launch, no hand-off), with no MFMA
tally or debug dumps, so that rocprofv3 --pmc WRITE_SIZE / TCC_EA0_WRREQ* can be read per dispatch.
Usage: rocprofv3 --pmc WRITE_SIZE --kernel-trace ... -- python3 tools/write_probe.py [precision]"""
import importlib
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _ablib  # noqa: E402,F401  (ANERF_LIB_PATH: an experiment build, A/B tooling only)
anerf = importlib.import_module("a-nerf_amd")
syn = importlib.import_module("a-nerf_amd.synthetic")


def main():
    prec = sys.argv[1] if len(sys.argv) > 1 else "fp16x4"
    ck = syn.make_checkpoint(13, n_joints=24, D=8, W=256, fine=True, tau=79.6)
    sc = syn.make_scene(n_joints=24, H=512, W=512, seed=13)
    idx, cyls, _ = anerf.rays.valid_pixels(sc["c2ws"], 512, 512, sc["focal"], kps=sc["kps"], ext_scale=0.001)
    pix = idx[0]
    y, x = pix // 512, pix % 512
    c2w = sc["c2ws"][0].astype(np.float64)
    d = np.stack([(x - 256.0) / sc["focal"], -(y - 256.0) / sc["focal"], -np.ones(len(pix))], -1) @ c2w[:3, :3].T
    n = len(pix)
    rb = torch.from_numpy(np.concatenate([np.broadcast_to(c2w[:3, 3], d.shape), d, np.zeros((n, 1)),
                                          np.ones((n, 1)), d / np.linalg.norm(d, axis=-1, keepdims=True)],
                                         -1).astype(np.float32)).cuda()
    sk = torch.from_numpy(sc["skts"][0:1]).cuda().expand(n, -1, -1, -1)
    cy = torch.from_numpy(cyls[0:1]).cuda().expand(n, -1)
    for I in (128, 0):
        cfg = anerf.RenderConfig(N_samples=64, N_importance=I, precision=prec).validate()
        rc = anerf.RayCaster(cfg, ck)
        for _ in range(3):
            rc.render_rays(rb, 64, skts=sk, cyls=cy, N_importance=I, ret_alpha=False)
            torch.cuda.synchronize()
    print(f"rays {n}: z hand-off {n * 192 * 4 / 1e6:.1f} MB per call (I = 128), outputs "
          f"{n * 10 * 4 / 1e6:.1f} MB (rgb, disp, acc + coarse copies)")


if __name__ == "__main__":
    main()

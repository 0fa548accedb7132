"""Render the config-3 frame (bench.py's workload, tau 79.6 and 20) with the library that
ANERF_LIB_PATH names and save the outputs, for bit-identity checks between two builds on one box.
Usage: python tools/ab_outputs.py OUT.npz [precision ...]"""
import importlib
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _ablib  # noqa: E402,F401  (ANERF_LIB_PATH: an experiment build, A/B tooling only)


def main():
    out = sys.argv[1]
    precs = sys.argv[2:] or ["bf16x6", "fp16x3", "fp32"]
    anerf = importlib.import_module("a-nerf_amd")
    syn = importlib.import_module("a-nerf_amd.synthetic")
    sc = syn.make_scene(n_joints=24, H=512, W=512, seed=13)
    idx, cyls, _ = anerf.rays.valid_pixels(sc["c2ws"], 512, 512, sc["focal"], kps=sc["kps"], ext_scale=0.001)
    _lib = importlib.import_module("a-nerf_amd._lib")
    dev = torch.device("cuda:0")
    pix = torch.from_numpy(np.asarray(idx[0], np.int64)).to(dev)
    c2w = torch.from_numpy(np.ascontiguousarray(sc["c2ws"][0][:3, :4], np.float32)).to(dev)
    rb = torch.empty(pix.shape[0], 11, device=dev)
    _lib.check(_lib.load().anerf_gen_rays(_lib.ptr(c2w), 512, 512, sc["focal"], sc["focal"], 0.0, 0.0, 0,
                                          _lib.ptr(pix), pix.shape[0], 0.0, 1.0, _lib.ptr(rb),
                                          _lib.stream_handle(dev)), "gen_rays")
    sk = torch.from_numpy(sc["skts"][0:1]).to(dev)
    cy = torch.from_numpy(cyls[0:1]).to(dev)
    n = rb.shape[0]
    res = {}
    for tau in (79.6, 20.0):
        ck = syn.make_checkpoint(13, n_joints=24, D=8, W=256, fine=True, tau=tau)
        for p in precs:
            cfg = anerf.RenderConfig(n_joints=24, N_samples=64, N_importance=128, precision=p).validate()
            rc = anerf.RayCaster(cfg, ck)
            o = rc.render_rays(rb, 64, skts=sk.expand(n, -1, -1, -1), cyls=cy.expand(n, -1), N_importance=128,
                               chunk=4096, ret_alpha=False)
            torch.cuda.synchronize()
            for k in ("rgb_map", "disp_map", "acc_map", "rgb0", "disp0", "acc0"):
                res[f"{p}_{tau}_{k}"] = o[k].cpu().numpy()
            del rc
    np.savez_compressed(out, **res)
    print(f"{out}: {len(res)} arrays, {n} rays")


if __name__ == "__main__":
    main()

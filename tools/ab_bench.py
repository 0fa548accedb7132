"""A/B of env-selected variants in ONE process on one device (MI355X_MICROARCH.md 'DVFS give-back';
cdna_hip_programming.md rule 24): interleaved rounds of config-3 frames, median ms per variant.
Usage: python tools/ab_bench.py ENV_VAR val_a val_b [rounds] [precision]"""
import importlib
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _ablib  # noqa: E402,F401  (ANERF_LIB_PATH: an experiment build, A/B tooling only)


def main():
    var, va, vb = sys.argv[1:4]
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 6
    prec = sys.argv[5] if len(sys.argv) > 5 else "bf16x6"
    anerf = importlib.import_module("a-nerf_amd")
    syn = importlib.import_module("a-nerf_amd.synthetic")
    cfg = anerf.RenderConfig(N_samples=64, N_importance=128, precision=prec).validate()
    ck = syn.make_checkpoint(13, n_joints=24, D=8, W=256, fine=True, tau=79.6)
    sc = syn.make_scene(n_joints=24, H=512, W=512, seed=13)
    casters = {}
    for v in (va, vb):  # the flag is read at model creation
        os.environ[var] = v
        casters[v] = anerf.RayCaster(cfg, ck)
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
    times = {va: [], vb: []}
    outs = {}
    for r in range(rounds + 1):
        for v in (va, vb):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            outs[v] = casters[v].render_rays(rb, 64, skts=sk, cyls=cy, N_importance=128, ret_alpha=False)
            e1.record()
            torch.cuda.synchronize()
            if r:
                times[v].append(e0.elapsed_time(e1))
    diff = float((outs[va]["rgb_map"] - outs[vb]["rgb_map"]).abs().max())
    print(json.dumps({"var": var, "precision": prec, "rays": n,
                      **{f"{var}={v}_ms_median": round(float(np.median(t)), 3) for v, t in times.items()},
                      **{f"{var}={v}_ms_min": round(float(np.min(t)), 3) for v, t in times.items()},
                      "max_abs_rgb_diff": diff}))


if __name__ == "__main__":
    main()

"""Throughput of the density-only path (fwd_type='mesh', run_render.render_mesh's defaults:
res=255 -> 256^3 grid, radius 1.8) on the config-3 model (fine net, 8x256, 24 joints).

Prints one JSON line: points/s, kernel ms (HIP events on the launch stream), and the
algorithmic dense-trunk FLOP rate against the FP32 MFMA peak."""
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
anerf = importlib.import_module("a-nerf_amd")
syn = importlib.import_module("a-nerf_amd.synthetic")


def trunk_flops(cfg):
    nj, W, D = cfg.n_joints, cfg.netwidth, cfg.netdepth
    cin = nj * (1 + 2 * cfg.multires) + 3 * nj
    macs = cin * W + W  # layer 0 + alpha_linear
    for i in range(1, D):
        macs += (cin + W if i == cfg.skips[0] + 1 else W) * W
    return 2 * macs


def main():
    res = int(sys.argv[1]) if len(sys.argv) > 1 else 255
    prec = sys.argv[2] if len(sys.argv) > 2 else "fp32"
    cfg = anerf.RenderConfig(N_samples=64, N_importance=128, precision=prec).validate()
    ck = syn.make_checkpoint(13, n_joints=24, D=8, W=256, fine=True, tau=79.6)
    sc = syn.make_scene(n_joints=24, H=512, W=512, seed=13)
    rc = anerf.RayCaster(cfg, ck)
    kps, skts = torch.from_numpy(sc["kps"][0:1]), torch.from_numpy(sc["skts"][0:1])
    rc.render_mesh_density(kps, skts, None, radius=1.8, res=res)  # warm-up
    torch.cuda.synchronize()
    times = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = rc.render_mesh_density(kps, skts, None, radius=1.8, res=res)
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
    ms = float(np.median(times))
    n = (res + 1) ** 3
    fl = trunk_flops(cfg)
    print(json.dumps({"metric": "density grid points/s (fwd_type='mesh', res=%d, config3 fine net)" % res,
                      "value": round(n / (ms * 1e-3), 1), "unit": "points/s", "precision": prec, "points": n, "ms": round(ms, 3),
                      "dense_trunk_flop_per_point": fl,
                      "dense_equivalent_tflops": round(fl * n / (ms * 1e-3) / 1e12, 2),
                      "frac_of_fp32_mfma_peak": round(fl * n / (ms * 1e-3) / 1e12 / 157.3, 4),
                      "finite": bool(torch.isfinite(out).all().item())}), flush=True)


if __name__ == "__main__":
    main()

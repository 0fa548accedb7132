"""Config-5 fp32 disp_map outlier diagnosis (GPU box): renders the 1024^2 frame with debug stages,
finds the rays where |gpu - oracle| disp exceeds 1e-5 among an evenly spaced sample, and reports
for each whether the fine samples (z_fine) differ from the oracle's (hazard H11: a u within an ulp
of a cdf edge takes the other sample_pdf branch when the coarse weights differ by ulps), together
with the coarse pass's disp difference.  Test infrastructure: imports the oracle as the checker."""
import argparse
import importlib
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _ablib  # noqa: E402,F401  (ANERF_LIB_PATH: an experiment build, A/B tooling only)
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))

anerf = importlib.import_module("a-nerf_amd")
import oracle  # noqa: E402
from test_gpu_frames import _frame  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--rays", type=int, default=20000)
    a = ap.parse_args()
    sc, ck, cyls, rb = _frame(a.res, 24, 13, 79.6)
    cfg = anerf.RenderConfig(n_joints=24, N_samples=64, N_importance=128, precision=a.precision).validate()
    rc = anerf.RayCaster(cfg, ck)
    n = rb.shape[0]
    sk = torch.from_numpy(sc["skts"][0:1]).cuda().expand(n, -1, -1, -1)
    cy = torch.from_numpy(cyls[0:1]).cuda().expand(n, -1)
    out = rc.render_rays(rb, 64, skts=sk, cyls=cy, N_importance=128, chunk=4096, ret_alpha=False, debug=True)
    torch.cuda.synchronize()
    om = oracle.OracleModel(cfg, ck)
    rb_h = rb.cpu().numpy()
    near, far, _, _ = om.near_far(rb_h, cyls[0:1], chunk=4096)
    sel = np.linspace(0, n - 1, a.rays).astype(np.int64)
    ref = om.render_rays(rb_h[sel], sc["skts"][0], cyls[0:1], chunk=4096, near=near[sel], far=far[sel], with_z=True)
    zf = rc.last_debug["z_fine"].cpu().numpy()[sel]
    d0 = np.abs(out["disp0"].cpu().numpy()[sel].astype(np.float64) - ref["disp0"])
    for k in ("rgb_map", "disp_map", "acc_map"):
        d = np.abs(out[k].cpu().numpy()[sel].astype(np.float64) - ref[k])
        print(f"{k}: max {d.max():.3e}  rays > 1e-5: {int((d.reshape(len(sel), -1).max(-1) > 1e-5).sum())}")
    dd = np.abs(out["disp_map"].cpu().numpy()[sel].astype(np.float64) - ref["disp_map"])
    same_z = np.all(zf == ref["z"], axis=-1)
    print(f"rays with identical fine z: {int(same_z.sum())} / {len(sel)}")
    if (~same_z).any():
        print(f"max disp err where z identical: {dd[same_z].max():.3e}; where z differs: {dd[~same_z].max():.3e}")
    for r in np.argsort(-dd)[:5]:
        nz = int((zf[r] != ref["z"][r]).sum())
        print(f"ray {sel[r]}: disp gpu {out['disp_map'][sel[r]].item():.6f} oracle {ref['disp_map'][r]:.6f} "
              f"acc {ref['acc_map'][r]:.3e} fine z differing {nz}/192 (max |dz| "
              f"{float(np.abs(zf[r] - ref['z'][r]).max()):.3e}) coarse disp0 diff {d0[r]:.3e}")


if __name__ == "__main__":
    main()

"""H12 diagnosis (GPU box): render the rays of tests/golden/h12_nearempty_c5.npz with the debug stages
(near / far, coarse z / raw / weights, fine z / raw) in the given precisions and save them with the
outputs to gpurun_out/h12_diag_<precision>.npz, for the host-side comparison with the reference's
outputs and the oracle (tools/diag_h12_host.py).  Diagnostic only; never used by tests or bench."""
import ast
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
    z = np.load(os.path.join(REPO, "tests", "golden", "h12_nearempty_c5.npz"))
    meta = ast.literal_eval(str(z["meta"]))
    ck = syn.make_checkpoint(meta["seed"], n_joints=24, D=8, W=256, fine=True, tau=meta["tau"])
    sc = syn.make_scene(n_joints=24, H=meta["H"], W=meta["H"], seed=meta["seed"])
    n = z["sel"].shape[0]
    rb = np.zeros((n, 11), np.float32)
    rb[:, 0:3], rb[:, 3:6], rb[:, 6], rb[:, 7] = z["rays_o"], z["rays_d"], z["near"], z["far"]
    rb[:, 8:11] = z["rays_d"] / np.linalg.norm(z["rays_d"], axis=-1, keepdims=True)
    cy = torch.from_numpy(z["cyls"]).cuda()
    sk = torch.from_numpy(sc["skts"][0:1]).cuda()
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    for prec in sys.argv[1:] or ["fp32"]:
        cfg = anerf.RenderConfig(N_samples=64, N_importance=128, precision=prec).validate()
        rc = anerf.RayCaster(cfg, ck)
        out = rc.render_rays(torch.from_numpy(rb).cuda(), 64, skts=sk.expand(n, -1, -1, -1), cyls=cy.expand(n, -1),
                             N_importance=128, ret_alpha=True, near_far_given=True, debug=True)
        torch.cuda.synchronize()
        save = {k: v.cpu().numpy() for k, v in out.items() if v is not None}
        save.update({"dbg_" + k: v.cpu().numpy() for k, v in rc.last_debug.items()})
        np.savez_compressed(os.path.join(REPO, "gpurun_out", f"h12_diag_{prec}.npz"), **save)
        dd = np.abs(save["disp_map"].astype(np.float64) - z["out_disp_map"])
        worst = np.argsort(-dd)[:6]
        sp = np.load(os.path.join(REPO, "tests", "golden", "h12_spread_c5.npz"))
        nei = np.flatnonzero(sp["near_empty"])
        for i in worst:
            print(f"{prec} ray {int(z['sel'][i])} (#{i}): disp gpu {save['disp_map'][i]:.6f} ref {z['out_disp_map'][i]:.6f} "
                  f"ref-f64 {sp['f64_disp_map'][i]:.6f} oracle {z['oracle_disp_map'][i]:.6f}; acc gpu {save['acc_map'][i]:.3e} "
                  f"ref {z['out_acc_map'][i]:.3e} ref-f64 {sp['f64_acc_map'][i]:.3e}")
            if i in nei:  # per-sample: alpha in 2^-24 quanta, raw sigma, z (GPU fine pass vs the reference's)
                k = int(np.flatnonzero(nei == i)[0])
                ga = save["alpha"][i].astype(np.float64)
                gs = save["dbg_raw_fine"][i][..., 3] if "dbg_raw_fine" in save else None
                gz = save["dbg_z_fine"][i] if "dbg_z_fine" in save else None
                live = np.flatnonzero((ga > 0) | (sp["t8_alpha"][k] > 0) | (sp["f64_alpha"][k] > 2.0 ** -26))
                for s in live[:12]:
                    print(f"    sample {s}: alpha quanta gpu {ga[s] * 2**24:.3f} ref {sp['t8_alpha'][k][s] * 2**24:.3f} "
                          f"f64 {sp['f64_alpha'][k][s] * 2**24:.3f}; sigma gpu {gs[s] if gs is not None else float('nan'):.9g} "
                          f"ref {sp['t8_sigma'][k][s]:.9g} f64 {sp['f64_sigma'][k][s]:.9g}; z gpu "
                          f"{gz[s] if gz is not None else float('nan'):.9g} ref {sp['t8_z'][k][s]:.9g}")


if __name__ == "__main__":
    main()

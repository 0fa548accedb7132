"""Diagnostic: per-phase shader-cycle shares of render_kernel (stamps build, tools/libanerf_hip_stamps.so).

Never used by tests or bench; the stamp values go to a buffer of their own."""
import ctypes
import importlib
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _ablib  # noqa: E402,F401  (ANERF_LIB_PATH: an experiment build, A/B tooling only)
_lib = importlib.import_module("a-nerf_amd._lib")
_lib.LIB_PATH = os.path.join(REPO, "tools", os.environ.get("ANERF_STAMPS_LIB", "ab/libanerf_hip_stamps.so"))
anerf = importlib.import_module("a-nerf_amd")
syn = importlib.import_module("a-nerf_amd.synthetic")
NAMES = {0: "prologue", 1: "view factor G (G + bias column)", 7: "  view factor: bias staging + trig table", 2: "MLP coarse", 3: "composite+importance", 4: "MLP fine",
         5: "composite fine", 6: "barrier wait after MLP", 8: "  L0 u-part", 9: "  L0 v-part",
         10: "  bias/relu boundaries", 11: "  hidden h-parts", 12: "  skip u+v", 13: "  heads (alpha/feat/view/rgb)",
         14: "  L0 u-part prologue", 15: "  v-part prologues (L0 + skip)",
         16: "  heads: view layer (+ alpha)", 17: "  heads: view-direction part", 13: "  heads: rgb head + stores",
         18: "  barrier wait before hidden layers (bf16x6)"}


def main():
    lib = _lib.load()
    lib.anerf_diag_set_stamps.argtypes = [ctypes.c_void_p]
    H = 512
    tau = float(sys.argv[1]) if len(sys.argv) > 1 else 79.6
    prec = os.environ.get("ANERF_PRECISION", "fp32")
    cfg = anerf.RenderConfig(N_samples=64, N_importance=128, precision=prec).validate()
    ck = syn.make_checkpoint(13, n_joints=24, D=8, W=256, fine=True, tau=tau)
    sc = syn.make_scene(n_joints=24, H=H, W=H, seed=13)
    rc = anerf.RayCaster(cfg, ck)
    kw = {"ray_caster": rc, "N_samples": 64, "N_importance": 128, "use_viewdirs": True,
          "preproc_kwargs": {"density_scale": 1.0}}
    st = torch.zeros(24, dtype=torch.int64, device="cuda")
    anerf.render_frames(torch.from_numpy(sc["c2ws"]), (H, H, sc["focal"]), 4096, kw, kp=torch.from_numpy(sc["kps"]),
                        skts=torch.from_numpy(sc["skts"]), ext_scale=0.001, to_host=False)
    lib.anerf_diag_set_stamps(ctypes.c_void_p(st.data_ptr()))
    anerf.render_frames(torch.from_numpy(sc["c2ws"]), (H, H, sc["focal"]), 4096, kw, kp=torch.from_numpy(sc["kps"]),
                        skts=torch.from_numpy(sc["skts"]), ext_scale=0.001, to_host=False)
    torch.cuda.synchronize()
    v = st.cpu().numpy().astype(np.float64)
    tot = v[0:24].sum()  # top-level phases + the MLP sub-phases (stamped separately)
    print(f"tau={tau} precision={prec}: total wave-cycles {tot:.3e}")
    for i, nm in NAMES.items():
        print(f"{nm:34s} {100 * v[i] / tot:6.2f} %")


if __name__ == "__main__":
    main()

"""Microbenchmark of the training MLP's forward at the training step's shapes (8x256, 24 joints,
M = 163840 fine / 131072 coarse rows): the fused kernel (anerf_mlp_forward) vs the layer-by-layer
bf16x6 GEMMs, interleaved in one process.  Prints ms per forward for each."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _ablib  # noqa: E402,F401  (ANERF_LIB_PATH: an experiment build, A/B tooling only)
anerf = importlib.import_module("a-nerf_amd")
syn = importlib.import_module("a-nerf_amd.synthetic")
train = importlib.import_module("a-nerf_amd.train")
mlp = importlib.import_module("a-nerf_amd.mlp")


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 163840
    cfg = anerf.RenderConfig(n_joints=24, netdepth=8, netwidth=256).validate()
    ck = syn.make_checkpoint(3, n_joints=24, D=8, W=256, fine=False)
    tr = train.TrainRayCaster(cfg, ck, mlp="bf16x6").train()
    feat = (torch.rand(M, cfg.feature_dim, device="cuda") * 2 - 1).requires_grad_(True)
    res = {True: [], False: []}
    for rnd in range(4):
        for fused in (True, False):
            mlp.FUSED_FORWARD = fused
            for _ in range(2):
                tr.network_fn(feat)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(5):
                tr.network_fn(feat)
            b.record()
            torch.cuda.synchronize()
            res[fused].append(a.elapsed_time(b) / 5)
    for k, v in res.items():
        print(f"{'fused' if k else 'gemm '} forward: {min(v):.3f} ms (rounds {', '.join(f'{x:.3f}' for x in v)})")


if __name__ == "__main__":
    main()

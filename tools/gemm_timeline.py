"""Diagnostic timeline of one training-GEMM launch (ANERF_GEMM_STAMPS=1 builds the s_memtime
buffer): prints per-point average cycles since kernel entry over the first 64 workgroups.
Usage: ANERF_GEMM_STAMPS=1 python tools/gemm_timeline.py"""
import ctypes
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mlp = importlib.import_module("a-nerf_amd.mlp")


def main():
    dev = torch.device("cuda:0")
    M, W = 163840, 256
    x = torch.randn(M, W, device=dev)
    w = torch.randn(W, W, device=dev) / 16
    b = torch.randn(W, device=dev)
    out = torch.empty(M, W, device=dev)
    ws = mlp.split_weight(w, False, 6)
    for _ in range(3):
        mlp.gemm(M, W, W, [mlp._seg(x, W)], ws, b, True, [(out, W, W, 0, None, False)], dev, 6)
    torch.cuda.synchronize()
    lib = mlp._lib.load()
    buf = (ctypes.c_ulonglong * (64 * 4 * 64))()
    fn = lib.anerf_mlp_diag_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    assert fn(ctypes.cast(buf, ctypes.c_void_p), 64 * 4 * 64) == 0
    t = np.frombuffer(buf, dtype=np.uint64).reshape(64, 4, 64).astype(np.int64)
    base = t[:, :, 0:1]
    rel = np.where(t > 0, t - base, -1)
    for i in range(64):
        v = rel[:, :, i]
        v = v[v >= 0]
        if v.size:
            print(f"point {i:2d}: mean {v.mean():9.0f}  min {v.min():9.0f}  max {v.max():9.0f}  (n={v.size})")


if __name__ == "__main__":
    main()

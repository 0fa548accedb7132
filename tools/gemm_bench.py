"""Microbenchmark of the training MLP GEMMs (anerf_gemm.hip) at the training step's shapes:
forward (NT, bias + relu), input gradient (NT, relu' mask), weight gradient (TN + slab reduce).
Prints one JSON line per case: microseconds per call and the HBM GB/s of its algorithmic bytes.
Usage: python tools/gemm_bench.py [--prec 6|3] [--reps N]"""
import argparse
import importlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _ablib  # noqa: E402,F401  (ANERF_LIB_PATH: an experiment build, A/B tooling only)
mlp = importlib.import_module("a-nerf_amd.mlp")


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prec", type=int, default=6)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--m", type=int, default=163840)
    ap.add_argument("--k", type=int, default=256, help="k of the forward / input-gradient cases (n = 256)")
    ap.add_argument("--cases", default="forward,input_grad,weight_grad,torch_fp32_mm,copy")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    M, W, K = a.m, 256, a.k
    x = torch.randn(M, W, device=dev)
    xk = torch.randn(M, K, device=dev)
    wk = torch.randn(W, K, device=dev) / 16
    wk_f = mlp.split_weight(wk, False, a.prec)
    h = torch.relu(torch.randn(M, W, device=dev))
    w = torch.randn(W, W, device=dev) / 16
    b = torch.randn(W, device=dev)
    out = torch.empty(M, W, device=dev)
    ws_f = mlp.split_weight(w, False, a.prec)
    ws_t = mlp.split_weight(w, True, a.prec)
    lib = mlp._lib.load()
    wsp = torch.empty(lib.anerf_mlp_wgrad_workspace(M, W, W), device=dev, dtype=torch.uint8)
    dw, db = torch.empty(W, W, device=dev), torch.empty(W, device=dev)
    cases = {
        "forward": (lambda: mlp.gemm(M, W, K, [mlp._seg(xk, K)], wk_f, b, True, [(out, W, W, 0, None, False)], dev,
                                     a.prec), M * (K + W) * 4),
        "forward_persistent": (lambda: mlp.forward_hidden(M, x, ws_f, a.prec, b, out, dev), 2 * M * W * 4),
        "forward_256": (lambda: mlp.gemm(M, W, W, [mlp._seg(x, W)], ws_f, b, True, [(out, W, W, 0, None, False)], dev,
                                         a.prec), 2 * M * W * 4),
        "input_grad": (lambda: mlp.gemm(M, W, W, [mlp._seg(x, W)], ws_t, None, False, [(out, W, W, 0, h, False)], dev,
                                        a.prec), 3 * M * W * 4),
        "weight_grad": (lambda: mlp.wgrad(M, W, W, x, [mlp._seg(h, W)], dw, db, wsp, dev, a.prec), 2 * M * W * 4),
        "torch_fp32_mm": (lambda: torch.mm(x, w.t(), out=out), 2 * M * W * 4),
        "copy": (lambda: out.copy_(x), 2 * M * W * 4),
    }
    for name in a.cases.split(","):
        fn, by = cases[name]
        us = timeit(fn, a.reps)
        k = K if name == "forward" else W  # (forward_persistent, forward_256: K = 256)
        print(json.dumps({"case": name, "M": M, "N": W, "K": k, "prec": a.prec, "us": round(us, 1),
                          "GBps": round(by / us / 1e3, 1),
                          "TFLOPs_ref": round(2 * M * W * k / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()

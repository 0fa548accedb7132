"""Microbenchmark of one 256 x 256 hidden layer's backward at the training step's fine-pass rows (M = 163,840):
the fused anerf_mlp_backward_hidden (dX, dW, db from one pass) against the two bf16x3 GEMMs it replaces
(anerf_mlp_gemm with the relu' mask + anerf_mlp_wgrad), sequential and on two streams as mlp.py ran them.
Prints one JSON line: microseconds per layer of each.  Usage: python tools/dgw_bench.py [--m M] [--reps N]"""
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
    ap.add_argument("--m", type=int, default=163840)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--cases", default="fused,two_seq,two_streams")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    M = a.m
    lib = mlp._lib.load()
    P = mlp._lib.ptr
    torch.manual_seed(0)
    dy = torch.randn(M, 256, device=dev)
    x = torch.relu(torch.randn(M, 256, device=dev))
    w = torch.randn(256, 256, device=dev) / 16
    wt = mlp.split_weight(w, True, 3)
    dx = torch.empty(M, 256, device=dev)
    dw, db = torch.empty(256, 256, device=dev), torch.empty(256, device=dev)
    fws = torch.empty(lib.anerf_mlp_backward_hidden_workspace(M, 256), device=dev, dtype=torch.uint8)
    ws = torch.empty(lib.anerf_mlp_wgrad_workspace(M, 256, 256), device=dev, dtype=torch.uint8)
    side = torch.cuda.Stream(device=dev)
    st = mlp._stream(dev)

    def fused():
        mlp._lib.check(lib.anerf_mlp_backward_hidden(M, 256, P(dy), 256, P(x), 256, P(wt), 3, P(dx), 256, P(dw), 256,
                                                     P(db), P(fws), fws.numel(), st), "backward_hidden")

    def dgrad():
        mlp.gemm(M, 256, 256, [mlp._seg(dy, 256)], wt, None, False, [(dx, 256, 256, 0, x, False)], dev, 3)

    def wgrad():
        mlp.wgrad(M, 256, 256, dy, [mlp._seg(x, 256)], dw, db, ws, dev, 3)

    def two_seq():
        wgrad()
        dgrad()

    def two_streams():
        main = torch.cuda.current_stream(dev)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            wgrad()
        dgrad()
        main.wait_stream(side)

    res = {"m": M}
    for c in a.cases.split(","):
        res[c + "_us"] = round(timeit({"fused": fused, "two_seq": two_seq, "two_streams": two_streams}[c], a.reps), 1)
    res["lib"] = mlp._lib.LIB_PATH
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

"""Forward GEMM timings at the training shape (M = 163,840 rows, 256 x 256, bias + relu): bf16x6, bf16x3,
fp16x4 with and without the row-max epilogue, and the split (+ exponent) launch.  Prints one line per
variant: mean µs over 50 launches (torch events on the current stream, which the GEMMs use)."""
import importlib
import os
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _ablib  # noqa: E402,F401  (ANERF_LIB_PATH: an experiment build, A/B tooling only)
mlp = importlib.import_module("a-nerf_amd.mlp")


def timeit(fn, n=50):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return 1e3 * e0.elapsed_time(e1) / n


def main():
    dev = torch.device("cuda:0")
    M, N, K = 163840, 256, 256
    torch.manual_seed(0)
    a = torch.relu(torch.randn(M, K, device=dev))
    w = torch.randn(N, K, device=dev) / 16
    b = torch.randn(N, device=dev) * 0.1
    out = torch.empty(M, N, device=dev)
    rin = a.abs().amax(1).contiguous().view(torch.int32)
    rout = torch.zeros(M, device=dev, dtype=torch.int32)
    sp = {p: mlp.split_weights([(w, False, p)], p)[0] for p in (3, 4, 6)}
    o = [(out, N, N, 0, None, False)]
    seg = [mlp._seg(a, K)]
    res = {
        "bf16x6": timeit(lambda: mlp.gemm(M, N, K, seg, sp[6], b, True, o, dev, 6)),
        "bf16x6+rout": timeit(lambda: mlp.gemm(M, N, K, seg, sp[6], b, True, o, dev, 6, rout=rout)),
        "bf16x3": timeit(lambda: mlp.gemm(M, N, K, seg, sp[3], b, True, o, dev, 3)),
        "fp16x4": timeit(lambda: mlp.gemm(M, N, K, seg, sp[4], b, True, o, dev, 4, rin=rin)),
        "fp16x4+rout": timeit(lambda: mlp.gemm(M, N, K, seg, sp[4], b, True, o, dev, 4, rin=rin, rout=rout)),
        "split7_bf16x6": timeit(lambda: mlp.split_weights([(w, False, 6)] * 7, 6)),
        "split7_fp16x4": timeit(lambda: mlp.split_weights([(w, False, 4)] * 7, 4)),
    }
    for k, v in res.items():
        print(f"{k:16s} {v:8.1f} us", flush=True)


if __name__ == "__main__":
    main()

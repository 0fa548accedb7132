"""Kernel times of the view-window layout's stages at the training bench's shape (2048 rays, 24 joints, W 256; 64
and 80 samples): anerf_train_view_factor (+ _backward) and anerf_train_view_mix (+ _backward), HIP events over 20
calls each.  ANERF_LIB_PATH selects an experiment build."""
import importlib
import json
import os
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _ablib  # noqa: E402,F401  (ANERF_LIB_PATH: an experiment build, A/B tooling only)
anerf = importlib.import_module("a-nerf_amd")
train = importlib.import_module("a-nerf_amd.train")
_lib = importlib.import_module("a-nerf_amd._lib")
dev = torch.device("cuda:0")
cfg = anerf.RenderConfig().validate()
tr = train.TrainRayCaster(cfg, device=dev)
model = tr.model
nj, W, nv = cfg.n_joints, cfg.netwidth, cfg.input_ch_views
n = 2048
sk = torch.randn(n, nj, 4, 4, device=dev)
rb = torch.randn(n, 11, device=dev)
weight = torch.randn(W // 2, W + nv, device=dev) * 0.1
lib = _lib.load()
st = torch.cuda.current_stream().cuda_stream
G = torch.empty(n, nj, W // 2, device=dev)
gG = torch.randn_like(G)
gs, gw = torch.zeros_like(sk), torch.zeros_like(weight)


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) / reps * 1000, 1)


out = {}
wp = weight.data_ptr() + 4 * W
out["view_factor_us"] = timed(lambda: lib.anerf_train_view_factor(model.handle, _lib.ptr(rb), 11, n, _lib.ptr(sk), n,
                                                                  None, wp, weight.stride(0), W // 2, None,
                                                                  _lib.ptr(G), st))
ws = torch.empty(lib.anerf_train_view_factor_workspace(n, nj, cfg.multires_views, W // 2), device=dev, dtype=torch.uint8)
out["view_factor_backward_us"] = timed(lambda: lib.anerf_train_view_factor_backward(
    model.handle, _lib.ptr(rb), 11, n, _lib.ptr(sk), n, None, wp, weight.stride(0), W // 2, None, _lib.ptr(gG),
    _lib.ptr(gs), gw.data_ptr() + 4 * W, _lib.ptr(ws), ws.numel(), st))
for ns in (64, 80):
    M = n * ns
    feat = torch.rand(M, 456, device=dev)
    o = torch.empty(M, W // 2, device=dev)
    gz = torch.randn(M, W // 2, device=dev)
    gf = torch.empty(M, 456, device=dev)
    gGm = torch.empty(n, nj, W // 2, device=dev)
    fp = feat.data_ptr() + 4 * 432
    out[f"view_mix_{ns}_us"] = timed(lambda: lib.anerf_train_view_mix(n, ns, nj, W // 2, fp, 456, _lib.ptr(G),
                                                                      _lib.ptr(o), st))
    out[f"view_mix_backward_{ns}_us"] = timed(lambda: lib.anerf_train_view_mix_backward(
        n, ns, nj, W // 2, fp, 456, _lib.ptr(G), _lib.ptr(gz), gf.data_ptr() + 4 * 432, 456, _lib.ptr(gGm), st))
print(json.dumps(out), flush=True)

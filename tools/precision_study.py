"""Precision study: max-abs error of the render outputs when every MLP GEMM runs as
  * bf16x3: x = x_hi + x_lo, W = W_hi + W_lo (bf16, round-to-nearest-even), y = x_hi W_hi + x_hi W_lo + x_lo W_hi
    with exact products accumulated in fp32 (what v_mfma_f32_32x32x16_bf16 computes);
  * bf16: y = bf16(x) bf16(W), fp32 accumulate;
against the fp32 golden outputs of the reference (tests/golden/*.npz), on the reference's own render
path (F.linear patched).  Runs only in the build container (imports /root/reference).

Usage: python tools/precision_study.py [names...]
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import make_golden as mg  # noqa: E402

_lin = F.linear


def _split(x):
    hi = x.to(torch.bfloat16).float()
    lo = (x - hi).to(torch.bfloat16).float()
    return hi, lo


def lin_bf16x3(x, w, b=None):
    xh, xl = _split(x)
    wh, wl = _split(w)
    y = _lin(xh.double(), wh.double()).float()  # exact products; fp32-accumulate order is immaterial here
    y = y + _lin(xh.double(), wl.double()).float() + _lin(xl.double(), wh.double()).float()
    return y if b is None else y + b


def _split3(x):
    p0 = x.to(torch.bfloat16).float()
    r = x - p0
    p1 = r.to(torch.bfloat16).float()
    p2 = (r - p1).to(torch.bfloat16).float()
    return p0, p1, p2


def lin_bf16x6(x, w, b=None):
    xs, ws = _split3(x), _split3(w)
    y = None
    for i in range(3):
        for j in range(3 - i):
            t = _lin(xs[i].double(), ws[j].double())
            y = t if y is None else y + t
    y = y.float()
    return y if b is None else y + b


def _pow2_scale(a, dim=None):
    """Power-of-2 factor putting max|a| (per row when dim is given) into [2^10, 2^11), as the kernel."""
    m = a.abs().amax(dim=dim, keepdim=True) if dim is not None else a.abs().max()
    e = torch.floor(torch.log2(torch.where(m > 0, m, torch.ones_like(m))))
    return torch.exp2(10.0 - e)


def _ftz16(h):
    """fp16 with subnormals flushed to zero (ANERF_FTZ16=1: what an MFMA that flushes f16 inputs sees)."""
    if os.environ.get("ANERF_FTZ16") == "1":
        h = torch.where(h.abs() < 2.0 ** -14, torch.zeros_like(h), h)
    return h


def _split16(x):
    hi = _ftz16(x.half()).float()
    lo = _ftz16((x - hi).half()).float()
    return hi, lo


def lin_fp16x3(x, w, b=None):
    """x = x0 + x1, W = W0 + W1 in fp16 after power-of-2 scaling (per sample row for x, per tensor for W),
    y = (x0 W0 + x0 W1 + x1 W0) / scales: three fp16 MFMA products with fp32 accumulation."""
    sx, sw = _pow2_scale(x, dim=-1), _pow2_scale(w)
    x0, x1 = _split16(x * sx)
    w0, w1 = _split16(w * sw)
    y = (_lin(x0.double(), w0.double()) + _lin(x0.double(), w1.double()) + _lin(x1.double(), w0.double()))
    y = (y / (sx.double() * sw.double())).float()
    return y if b is None else y + b


def lin_fp16x4(x, w, b=None):
    sx, sw = _pow2_scale(x, dim=-1), _pow2_scale(w)
    x0, x1 = _split16(x * sx)
    w0, w1 = _split16(w * sw)
    y = (_lin(x0.double(), w0.double()) + _lin(x0.double(), w1.double()) + _lin(x1.double(), w0.double()) +
         _lin(x1.double(), w1.double()))
    y = (y / (sx.double() * sw.double())).float()
    return y if b is None else y + b


def lin_bf16(x, w, b=None):
    y = _lin(x.to(torch.bfloat16).double(), w.to(torch.bfloat16).double()).float()
    return y if b is None else y + b


def run(name, mode, mods, tmp):
    cfg = mg.CONFIGS[name]
    z = np.load(os.path.join(REPO, "tests", "golden", name + ".npz"), allow_pickle=False)
    args, kw, ck = mg.build_reference(mods, cfg, os.path.join(tmp, name + mode))
    sc = mg.scene_for(cfg)
    sc["cyls"] = z["cyls"]
    o, d = torch.from_numpy(z["rays_o"]), torch.from_numpy(z["rays_d"])
    cams = z["cams"] if "cams" in z.files else None
    F.linear = {"bf16x6": lin_bf16x6, "bf16x3": lin_bf16x3, "bf16": lin_bf16, "fp32": _lin, "fp16x3": lin_fp16x3,
                "fp16x4": lin_fp16x4}[mode]
    torch.nn.modules.linear.F.linear = F.linear
    try:
        ret = mg.render_subset(mods, kw, o, d, sc, cams=cams)
    finally:
        F.linear = _lin
        torch.nn.modules.linear.F.linear = _lin
    errs = {k: float(np.abs(ret[k] - z["out_" + k]).max()) for k in ("rgb_map", "disp_map", "acc_map", "rgb0")
            if k in ret and "out_" + k in z.files}
    return errs


def main():
    import tempfile
    names = sys.argv[1:] or ["c2_256_s64_d8w256", "c3_512_s64i128_d8w256", "c4_512_s64i128_j65",
                             "v1_mr10_w64_d4", "fc_64_s32i32_d4w128"]
    torch.set_num_threads(8)
    mods = mg.import_reference()
    with tempfile.TemporaryDirectory() as tmp:
        for n in names:
            for mode in os.environ.get("MODES", "fp32,bf16x6,fp16x4,fp16x3,bf16x3,bf16").split(","):
                print(n, mode, run(n, mode, mods, tmp), flush=True)


if __name__ == "__main__":
    main()

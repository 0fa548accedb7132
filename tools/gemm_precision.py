"""Per-product accuracy of the MLP arithmetic modes on the render path's own activations (CPU).

For every layer of the config-3 fine net (8x256, seeded synthetic checkpoint; the hidden layers and
the fused view layer, i.e. the contractions the split modes replace) it feeds fp32 inputs x taken
from a float64 forward pass of real encoder features (the oracle's encoding of config-3 rays) and
measures each mode's output against the exact product sum of the same fp32 operands, normalised by
sum_k |x_k w_k| (the scale every fp32 error bound of a dot product is stated in):

  fp32-sgemm   torch float32 matmul (the reference's addmm arithmetic on this CPU: rounding of
               the accumulation only)
  fp32-chain   one fp32 FMA chain per output in k order (what v_mfma_f32_32x32x2_f32 computes)
  bf16x6       x split by truncation into 3 bf16 parts, w by RNE into 3, the six products i + j <= 2
               summed exactly (the kernel's MFMAs accumulate in fp32 like the modes above)
  fp16x4       power-of-two scaled, x and w split by RNE into 2 fp16 parts, all four products
  fp16x3       the same split, x1 w1 dropped
  bf16x3       2 bf16 parts (RNE), x1 w1 dropped

The split modes' products are summed exactly here (float64), so their columns show what the
operand representation and the dropped products cost; the fp32 columns show the accumulation
rounding every mode also pays.  Test infrastructure (imports the oracle for the features).

Usage: python tools/gemm_precision.py [n_samples]
"""
import importlib
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _ablib  # noqa: E402,F401  (ANERF_LIB_PATH: an experiment build, A/B tooling only)
sys.path.insert(0, os.path.join(REPO, "oracle"))
anerf = importlib.import_module("a-nerf_amd")
syn = importlib.import_module("a-nerf_amd.synthetic")


def f32(a):
    return a.astype(np.float32)


def trunc_bf16(x):
    return (x.view(np.uint32) & np.uint32(0xffff0000)).view(np.float32)


def rne_bf16(x):
    return torch.from_numpy(x).to(torch.bfloat16).float().numpy()


def rne_f16(x):
    return x.astype(np.float16).astype(np.float32)


def split_bf16x3_trunc(x):
    x0 = trunc_bf16(x)
    r = f32(x - x0)
    x1 = trunc_bf16(r)
    return [x0, x1, f32(r - x1)]


def split_bf16x3_rne(w):
    parts, r = [], w.copy()
    for _ in range(3):
        p = rne_bf16(r)
        parts.append(p)
        r = f32(r - p)
    return parts


def pow2_scale(a, axis=None):
    m = np.abs(a).max(axis=axis, keepdims=axis is not None)
    m = np.where(m > 0, m, 1.0)
    return np.exp2(10.0 - np.floor(np.log2(m))).astype(np.float32)


def split_f16(x, low_rtz):
    """kernel's split2_pair: high = x rounded (half away) to 11 bits, low = remainder -> fp16."""
    u = x.view(np.uint32)
    hi = ((u + np.uint32(0x1000)) & np.uint32(0xffffe000)).view(np.float32)
    r = f32(x - hi)
    if low_rtz:  # v_cvt_pkrtz
        lo = (np.sign(r) * rtz_f16(np.abs(r))).astype(np.float32)
    else:
        lo = rne_f16(r)
    return [rne_f16(hi), lo]


def rtz_f16(a):
    h = a.astype(np.float16).astype(np.float32)
    return np.where(h > a, np.nextafter(h.astype(np.float16), np.float16(0)).astype(np.float32), h)


def products(xs, ws, pairs):
    y = 0.0
    for i, j in pairs:
        y = y + xs[i].astype(np.float64) @ ws[j].astype(np.float64).T
    return y


def modes(x, w):
    """x [M, K] fp32, w [N, K] fp32 -> {mode: y [M, N] (float64 of what the mode computes)}."""
    out = {}
    out["fp32-sgemm"] = (torch.from_numpy(x) @ torch.from_numpy(w).T).numpy().astype(np.float64)
    acc = np.zeros((x.shape[0], w.shape[0]), np.float32)
    for k in range(x.shape[1]):
        acc = f32(acc + f32(x[:, k:k + 1] * w[None, :, k]))  # (fma rounding ~ product rounding here)
    out["fp32-chain"] = acc.astype(np.float64)
    xs, ws = split_bf16x3_trunc(x), split_bf16x3_rne(w)
    out["bf16x6"] = products(xs, ws, [(i, j) for i in range(3) for j in range(3 - i)])
    sx, sw = pow2_scale(x, axis=1), pow2_scale(w)
    for name, pairs, rtz in (("fp16x4", [(0, 0), (0, 1), (1, 0), (1, 1)], False),
                             ("fp16x3", [(0, 0), (0, 1), (1, 0)], False)):
        xs = split_f16(f32(x * sx), rtz)
        ws = [rne_f16(f32(w * sw))]
        ws.append(rne_f16(f32(w * sw - ws[0])))
        out[name] = products(xs, ws, pairs) / (sx.astype(np.float64) * sw.astype(np.float64))
    x0 = rne_bf16(x)
    w0 = rne_bf16(w)
    out["bf16x3"] = products([x0, rne_bf16(f32(x - x0))], [w0, rne_bf16(f32(w - w0))], [(0, 0), (0, 1), (1, 0)])
    return out


def main():
    import oracle
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    cfg = anerf.RenderConfig(N_samples=64, N_importance=128).validate()
    ck = syn.make_checkpoint(13, n_joints=24, D=8, W=256, fine=True, tau=79.6)
    sc = syn.make_scene(n_joints=24, H=512, W=512, seed=13)
    idx, cyls, _ = anerf.rays.valid_pixels(sc["c2ws"], 512, 512, sc["focal"], kps=sc["kps"], ext_scale=0.001)
    sel = idx[0][np.linspace(0, len(idx[0]) - 1, n // 64).astype(np.int64)]
    rb = oracle.gen_rays(sc["c2ws"][0], 512, 512, sc["focal"], sel)
    om = oracle.OracleModel(cfg, ck)
    near, far, _, _ = om.near_far(rb, cyls[0:1])
    t = np.linspace(0, 1, 64, dtype=np.float32)
    z = near[:, None] * (1 - t) + far[:, None] * t
    pts = f32(rb[:, None, 0:3] + rb[:, None, 3:6] * z[..., None]).reshape(-1, 3)
    dirs = np.repeat(rb[:, 3:6], 64, 0)
    feat = om.encode(sc["skts"][0], pts, dirs)
    sd = ck["network_fine_state_dict"]
    D, W = 8, 256
    dnet = cfg.input_ch + cfg.input_ch_bones
    xin = feat[:, :dnet].astype(np.float64)
    h = xin
    stats = {}

    def record(tag, x, w):
        y = modes(x, w)
        exact = x.astype(np.float64) @ w.astype(np.float64).T
        scale = np.abs(x).astype(np.float64) @ np.abs(w).astype(np.float64).T
        scale = np.where(scale > 0, scale, 1.0)
        stats[tag] = {m: {"max": float(np.max(np.abs(v - exact) / scale)),
                          "rms": float(np.sqrt(np.mean((np.abs(v - exact) / scale) ** 2)))} for m, v in y.items()}
        return exact
    for i in range(D):
        w = f32(np.asarray(sd[f"pts_linears.{i}.weight"]))
        b = np.asarray(sd[f"pts_linears.{i}.bias"], np.float64)
        x = f32(np.concatenate([xin, h], 1) if i == 5 else h)
        if i >= 1:  # the hidden layers (the skip layer's h part: its x part is a bone/window stream)
            xh = f32(h)
            wh = w[:, dnet:] if i == 5 else w
            record(f"pts_linears.{i}" + (" (h part)" if i == 5 else ""), xh, wh)
        h = np.maximum(x.astype(np.float64) @ w.astype(np.float64).T + b, 0.0)
    wf = np.asarray(sd["feature_linear.weight"], np.float64)
    wv = np.asarray(sd["views_linears.0.weight"], np.float64)
    fused = f32(wv[:, :W] @ wf)  # the kernel's fused view layer (feature_linear folded, nerf.py:110-112)
    record("views_linears.0 (feature_linear fused)", f32(h), fused)
    print(json.dumps({"samples": int(xin.shape[0]), "metric": "|y - exact| / sum_k |x_k w_k|", "layers": stats},
                     indent=1))
    worst = {m: max(s[m]["max"] for s in stats.values()) for m in next(iter(stats.values()))}
    print("worst max over layers:", json.dumps({m: float(f"{v:.3e}") for m, v in worst.items()}))


if __name__ == "__main__":
    main()

"""GPU numerics of the training MLP's split-bf16 GEMMs (a-nerf_amd/csrc/anerf_gemm.hip) against
plain torch fp64 products of the same operands, and of the whole network (mlp.nerf_forward,
forward + autograd) against the torch fp32 path of the same module.

Bound for one product: bf16x3 keeps ~16 significant bits per operand (x = x0 + x1, bf16 RNE each;
dropped x1 w1), so |C - C_ref| <= 2^-15 * (|A| |B|^T) + fp32 accumulation slack — the tests use
4e-5 (|A| |B|^T) + 1e-6; bf16x6 (three planes, six products) is fp32-accurate: 2e-6 (|A| |B|^T) + 1e-6
(fp32 accumulation of up to ~1000 terms).
"""
import importlib

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

mlp = importlib.import_module("a-nerf_amd.mlp")
train = importlib.import_module("a-nerf_amd.train")
anerf = importlib.import_module("a-nerf_amd")
syn = importlib.import_module("a-nerf_amd.synthetic")

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _cuda():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


REL = {3: 4e-5, 6: 2e-6}


def _bound(a, b, prec=3):
    return REL[prec] * (a.double().abs() @ b.double().abs().t()) + 1e-6


@pytest.mark.parametrize("prec", [3, 6])
def test_split_weights_batch_matches_single(prec):
    """anerf_mlp_split_weights_batch writes byte-identical planes to one anerf_mlp_split_weights per job
    (ragged shapes, strided rows, both orientations, more than one 32-job launch)."""
    torch.manual_seed(prec)
    shapes = [(256, 432), (3, 128), (257, 256), (1, 1), (128, 904), (33, 17)] * 6
    jobs = []
    for i, (n, k) in enumerate(shapes):
        w = torch.randn(n, k + 3, device=DEV)[:, :k]  # ldw = k + 3
        jobs.append((w, bool(i % 2)))
    outs = mlp.split_weights(jobs, prec)
    assert len(outs) == len(jobs)
    for (w, t), o in zip(jobs, outs):
        assert torch.equal(o, mlp.split_weight(w, t, prec))


@pytest.mark.parametrize("prec", [3, 6])
@pytest.mark.parametrize("m,n,ks", [(1000, 257, (256, 648, 16)), (4096, 256, (432, 256)), (77, 3, (128,)),
                                    (130, 128, (904,)), (0, 64, (32,)), (20011, 920, (128,)),
                                    (163857, 256, (256,)), (9000, 432, (256,)), (33, 200, (12, 20))])
def test_gemm_forward_segments_bias_relu(m, n, ks, prec):
    torch.manual_seed(m + n)
    k = sum(ks)
    parts = [torch.randn(m, c + 4, device=DEV)[:, :c] for c in ks]  # strided rows (ld = c + 4)
    a = torch.cat(parts, 1) if m else torch.empty(0, k, device=DEV)
    w = torch.randn(n, k, device=DEV) / k ** 0.5
    b = torch.randn(n, device=DEV)
    out = torch.full((m, n + 5), 7.0, device=DEV)
    if m:
        mlp.gemm(m, n, k, [mlp._seg(p, p.shape[1]) for p in parts], mlp.split_weight(w, False, prec), b, True,
                 [(out, n + 5, n, 0, None, False)], torch.device(DEV), prec)
    ref = torch.relu(a.double() @ w.double().t() + b.double())
    assert torch.all(out[:, n:] == 7.0)  # nothing written past the segment
    err = (out[:, :n].double() - ref).abs()
    assert torch.all(err <= _bound(a, w, prec)), float(err.max())


@pytest.mark.parametrize("m,n,k", [(1000, 128, 256), (163857, 128, 256), (77, 130, 264), (33, 3, 12)])
def test_gemm_preactivation_accumulate(m, n, k):
    """accumulate == 2 (anerf.h anerf_oseg): the old output joins the pre-activation, relu(A W^T + b + old) -- the
    view layer of the view-window layout (old = sum_j w_j G_j); ragged columns take the per-element path."""
    torch.manual_seed(m + n)
    a = torch.randn(m, k, device=DEV)
    w = torch.randn(n, k, device=DEV) / k ** 0.5
    b = torch.randn(n, device=DEV)
    old = torch.randn(m, n, device=DEV)
    out = old.clone()
    mlp.gemm(m, n, k, [mlp._seg(a, k)], mlp.split_weight(w, False, 6), b, True, [(out, n, n, 0, None, 2)],
             torch.device(DEV), 6)
    ref = torch.relu(a.double() @ w.double().t() + b.double() + old.double())
    err = (out.double() - ref).abs()
    assert torch.all(err <= _bound(a, w, 6) + 1e-6 * old.double().abs()), float(err.max())


def _rowmax_bits(t):
    """int32 [m]: the bit pattern of each row's largest |value| (what the GEMM epilogue's rout holds)."""
    return t.abs().amax(1).contiguous().view(torch.int32) if t.shape[1] else torch.zeros(t.shape[0], dtype=torch.int32)


@pytest.mark.parametrize("m,n,k", [(1000, 256, 256), (163857, 256, 256), (77, 257, 256), (4096, 128, 128),
                                   (3001, 3, 128), (9000, 256, 432)])
def test_gemm_fp16x4_row_scaled(m, n, k):
    """fp16x4 (anerf_mlp_gemm_rows, precision 4): each A row scaled by a power of two from its row
    maximum, the weights by one from their maximum, both split into two fp16 planes, four products.
    Rows spanning 2^-40 .. 2^40 (and all-zero rows) keep the bf16x6 error bound 2e-6 (|a| |w|) per
    element, and rout holds the exact row maxima of the relu output."""
    torch.manual_seed(m + k)
    a = torch.relu(torch.randn(m, k, device=DEV))
    a *= torch.pow(2.0, torch.randint(-40, 41, (m, 1), device=DEV).float())
    a[::97] = 0.0
    # rows at the ends of the exponent range the row shift covers (advisor r4: the shift was clamped to
    # +-100, so rows past ~2^110 overflowed fp16): ~2^115 and ~2^-118
    a[1::131] = torch.relu(torch.randn_like(a[1::131])) * 2.0 ** 115
    a[2::131] = torch.relu(torch.randn_like(a[2::131])) * 2.0 ** -118
    w = torch.randn(n, k, device=DEV) / k ** 0.5 * 1e-3
    b = torch.randn(n, device=DEV) * 1e-3
    out = torch.full((m, n), 7.0, device=DEV)
    rin = _rowmax_bits(a)
    rout = torch.zeros(m, device=DEV, dtype=torch.int32) if n % 128 == 0 else None
    sp = mlp.split_weights([(w, False, 4)], 6)[0]
    mlp.gemm(m, n, k, [mlp._seg(a, k)], sp, b, True, [(out, n, n, 0, None, False)], torch.device(DEV), 4,
             rin=rin, rout=rout)
    ref = torch.relu(a.double() @ w.double().t() + b.double())
    err = (out.double() - ref).abs()
    bound = 2e-6 * (a.double().abs() @ w.double().abs().t()) + 1e-6 * b.double().abs().max() + 1e-30
    assert torch.all(err <= bound), float((err / bound).max())
    if rout is not None:
        assert torch.equal(rout, _rowmax_bits(out))


def test_gemm_fp16x4_rejects_bad_arguments():
    x = torch.rand(64, 128, device=DEV)
    w = torch.randn(128, 128, device=DEV)
    sp4 = mlp.split_weights([(w, False, 4)], 6)[0]
    o = [(torch.empty(64, 128, device=DEV), 128, 128, 0, None, False)]
    with pytest.raises(mlp._lib.AnerfError, match="row maxima"):
        mlp.gemm(64, 128, 128, [mlp._seg(x, 128)], sp4, None, False, o, torch.device(DEV), 4)
    with pytest.raises(mlp._lib.AnerfError, match="row maxima"):
        mlp.gemm(64, 128, 128, [mlp._seg(x, 64), mlp._seg(x, 64, 64)], sp4, None, False, o, torch.device(DEV), 4,
                 rin=_rowmax_bits(x))
    with pytest.raises(mlp._lib.AnerfError, match="row maxima are fp16x4"):
        mlp.gemm(64, 128, 128, [mlp._seg(x, 128)], mlp.split_weight(w), None, False, o, torch.device(DEV), 6,
                 rin=_rowmax_bits(x))
    for oseg in ([(torch.empty(64, 128, device=DEV), 128, 128, 0, torch.ones(64, 128, device=DEV), False)],
                 [(torch.zeros(64, 128, device=DEV), 128, 128, 0, None, True)],
                 [(torch.empty(64, 64, device=DEV), 64, 64, 0, None, False)] * 2):
        with pytest.raises(mlp._lib.AnerfError, match="one 16-byte aligned output segment"):
            mlp.gemm(64, 128, 128, [mlp._seg(x, 128)], sp4, None, False, oseg, torch.device(DEV), 4,
                     rin=_rowmax_bits(x), rout=torch.zeros(64, device=DEV, dtype=torch.int32))
    with pytest.raises(mlp._lib.AnerfError, match="n % 128"):
        mlp.gemm(64, 64, 128, [mlp._seg(x, 128)], mlp.split_weight(w[:64].contiguous()), None, False,
                 [(torch.empty(64, 64, device=DEV), 64, 64, 0, None, False)], torch.device(DEV), 6,
                 rout=torch.zeros(64, device=DEV, dtype=torch.int32))


def test_gemm_rejects_misaligned_segments():
    x = torch.randn(64, 35, device=DEV)
    w = torch.randn(16, 34, device=DEV)
    with pytest.raises(mlp._lib.AnerfError, match="16-byte aligned"):
        mlp.gemm(64, 16, 34, [mlp._seg(x, 2), mlp._seg(x, 32, 2)], mlp.split_weight(w), None, False,
                 [(torch.empty(64, 16, device=DEV), 16, 16, 0, None, False)], torch.device(DEV))
    with pytest.raises(mlp._lib.AnerfError, match="ld < cols"):  # the last segment is read to a multiple of 4
        z = torch.randn(64, 3, device=DEV)
        mlp.gemm(64, 16, 3, [mlp._seg(z, 3)], mlp.split_weight(w[:, :3].contiguous()), None, False,
                 [(torch.empty(64, 16, device=DEV), 16, 16, 0, None, False)], torch.device(DEV))


@pytest.mark.parametrize("prec", [3, 6])
def test_gemm_input_gradient_mask_accumulate_discard(prec):
    torch.manual_seed(1)
    m, k, n = 2000, 256, 688  # the skip layer's input gradient: [x (432) | h (256)]
    gz = torch.randn(m, k, device=DEV)
    w = torch.randn(k, n, device=DEV) / k ** 0.5  # the layer's weight [out = k][in = n]
    h = torch.relu(torch.randn(m, 256, device=DEV))
    gx = torch.randn(m, 432, device=DEV)
    gx0 = gx.clone()
    gh = torch.empty(m, 256, device=DEV)
    mlp.gemm(m, n, k, [mlp._seg(gz, k)], mlp.split_weight(w, True, prec), None, False,
             [(gx, 432, 432, 0, None, True), (gh, 256, 256, 0, h, False)], torch.device(DEV), prec)
    full = gz.double() @ w.double()
    bound = _bound(gz, w.t(), prec)
    assert torch.all((gx.double() - (gx0.double() + full[:, :432])).abs() <= bound[:, :432] + 1e-6)
    ref_h = torch.where(h > 0, full[:, 432:], torch.zeros_like(full[:, 432:]))
    assert torch.all((gh.double() - ref_h).abs() <= bound[:, 432:])
    # a discarded segment writes nothing
    keep = gx.clone()
    mlp.gemm(m, n, k, [mlp._seg(gz, k)], mlp.split_weight(w, True, prec), None, False,
             [(None, 432, 432, 0, None, False), (gh, 256, 256, 0, h, False)], torch.device(DEV), prec)
    assert torch.equal(gx, keep)


@pytest.mark.parametrize("prec", [3, 6])
@pytest.mark.parametrize("m,n,ks", [(131072, 256, (256,)), (5000, 257, (256,)), (3001, 3, (128,)),
                                    (777, 128, (256, 648, 16)), (40, 256, (432, 256))])
def test_wgrad_and_bias_gradient(m, n, ks, prec):
    torch.manual_seed(m)
    k = sum(ks)
    # dY rows padded past round_up(n, 4), the padding holding values that must reach no output
    dy = torch.randn(m, (n + 3) // 4 * 4 + 4, device=DEV)[:, :n]
    parts = [torch.randn(m, c, device=DEV) for c in ks]
    x = torch.cat(parts, 1)
    lib = mlp._lib.load()
    ws = torch.empty(lib.anerf_mlp_wgrad_workspace(m, n, k), device=DEV, dtype=torch.uint8)
    dw = torch.empty(n, k, device=DEV)
    db = torch.empty(n, device=DEV)
    mlp.wgrad(m, n, k, dy, [mlp._seg(p, p.shape[1]) for p in parts], dw, db, ws, torch.device(DEV), prec)
    ref = dy.double().t() @ x.double()
    bound = 2 * REL[prec] * (dy.double().abs().t() @ x.double().abs()) + 1e-5
    assert torch.all((dw.double() - ref).abs() <= bound), float((dw.double() - ref).abs().max())
    ref_b = dy.double().sum(0)
    assert torch.all((db.double() - ref_b).abs() <= 1e-5 * dy.double().abs().sum(0) + 1e-5)


def test_wgrad_rejects_unaligned_dy():
    m, n, k = 64, 5, 16
    lib = mlp._lib.load()
    x = torch.randn(m, k, device=DEV)
    ws = torch.empty(lib.anerf_mlp_wgrad_workspace(m, n, k), device=DEV, dtype=torch.uint8)
    dw, db = torch.empty(n, k, device=DEV), torch.empty(n, device=DEV)
    for dy in (torch.randn(m, n, device=DEV), torch.randn(m, 9, device=DEV)[:, :n],
               torch.randn(m * 8 + 1, device=DEV)[1:].view(m, 8)[:, :n]):
        with pytest.raises(mlp._lib.AnerfError, match="dy must be"):
            mlp.wgrad(m, n, k, dy, [mlp._seg(x, k)], dw, db, ws, torch.device(DEV))


def test_wgrad_is_deterministic():
    torch.manual_seed(3)
    m, n, k = 50000, 256, 256
    dy, x = torch.randn(m, n, device=DEV), torch.randn(m, k, device=DEV)
    lib = mlp._lib.load()
    ws = torch.empty(lib.anerf_mlp_wgrad_workspace(m, n, k), device=DEV, dtype=torch.uint8)
    outs = []
    for _ in range(2):
        dw, db = torch.empty(n, k, device=DEV), torch.empty(n, device=DEV)
        mlp.wgrad(m, n, k, dy, [mlp._seg(x, k)], dw, db, ws, torch.device(DEV))
        outs.append((dw, db))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("impl", ["bf16x6", "mixed", "mixed16", "bf16x3"])
@pytest.mark.parametrize("D,W,fc,nj", [(8, 256, False, 24), (4, 128, True, 24),
                                       # joint counts whose feature blocks are not multiples of 4 columns
                                       # (mlp._pad_to_segments): 17 (odd), 26 (even, not % 4), 65 (config 4)
                                       (8, 256, False, 17), (4, 128, True, 26), (8, 128, False, 65)])
def test_nerf_forward_backward_matches_fp32_module(D, W, fc, nj, impl):
    """The whole network (skip layer, heads, view layer, framecodes) and its autograd vs the same
    module on torch's fp32 GEMMs."""
    cfg = anerf.RenderConfig(n_joints=nj, netdepth=D, netwidth=W, opt_framecode=fc,
                             n_framecodes=5 if fc else 0).validate()
    ck = syn.make_checkpoint(5, n_joints=nj, D=D, W=W, fine=False, use_framecode=fc, n_framecodes=5)
    torch.manual_seed(0)
    M = 3000
    feat = (torch.rand(M, cfg.feature_dim, device=DEV) * 2 - 1)
    cams = torch.randint(0, 5, (M,), device=DEV) if fc else None
    gout = torch.randn(M, 4, device=DEV)
    res = {}
    for mode in (impl, "fp32"):
        tr = train.TrainRayCaster(cfg, ck, mlp=mode).train()
        net = tr.network_fn
        f = feat.clone().requires_grad_(True)
        raw = net(f, cams)
        (raw * gout).sum().backward()
        res[mode] = (raw.detach(), f.grad, {k: p.grad for k, p in net.named_parameters()})
    raw_b, gf_b, gp_b = res[impl]
    raw_f, gf_f, gp_f = res["fp32"]
    assert float((raw_b - raw_f).abs().max()) <= 1e-4 * max(1.0, float(raw_f.abs().max()))
    # gradients: relative Frobenius error (a pre-activation within rounding of 0 may take the other
    # relu branch in either implementation; elementwise maxima are pinned by the reference goldens
    # in test_gpu_train.py)
    def rel(a, b):
        return float((a.double() - b.double()).norm() / max(b.double().norm(), 1e-30))
    row = ((gf_b.double() - gf_f.double()).norm(dim=1) / gf_f.double().norm(dim=1).clamp_min(1e-30))
    q99 = float(torch.quantile(row.float(), 0.99))
    print(f"{impl} feature gradient: rel {rel(gf_b, gf_f):.2e}, per-row 99% {q99:.2e}, max {float(row.max()):.2e}")
    assert q99 <= 1e-3 and rel(gf_b, gf_f) <= 5e-3, (q99, rel(gf_b, gf_f))
    for k in gp_f:
        assert rel(gp_b[k], gp_f[k]) <= 5e-3, (k, rel(gp_b[k], gp_f[k]))


@pytest.mark.parametrize("switch", ["FUSED_SKIP", "FUSED_HEAD"])
@pytest.mark.parametrize("D,fc,nj,need_feat", [(8, False, 24, True), (8, True, 17, True), (8, False, 65, True),
                                                (8, False, 24, False), (6, False, 24, True)])
def test_fused_skip_and_head_backward_match_two_gemms(D, fc, nj, need_feat, switch, monkeypatch):
    """mlp.FUSED_SKIP (round 6): the skip layer's h part on anerf_mlp_backward_hidden and its x part merged into
    layer 0's products ([dY_0 | dY_s] against [W_0 ; W_s,x]); mlp.FUSED_HEAD (ABI 18): feature_linear +
    alpha_linear on anerf_mlp_backward_head.  Each == the same layers as two GEMMs: FUSED_SKIP the same bf16x3
    products summed in another order, every gradient within 1e-5 (relative Frobenius); FUSED_HEAD computes alpha's
    terms in fp32 where the GEMMs take them as bf16x3 products (relative error ~4e-5 each, REL[3]), so within 1e-4.
    17 / 65 joints: zero-padded kp + bone blocks; D 6: the skip layer is the last (no merge); no feature gradient."""
    mlp = importlib.import_module("a-nerf_amd.mlp")
    cfg = anerf.RenderConfig(n_joints=nj, netdepth=D, netwidth=256, opt_framecode=fc,
                             n_framecodes=5 if fc else 0).validate()
    ck = syn.make_checkpoint(7, n_joints=nj, D=D, W=256, fine=False, use_framecode=fc, n_framecodes=5)
    torch.manual_seed(1)
    M = 4000
    feat = (torch.rand(M, cfg.feature_dim, device=DEV) * 2 - 1)
    cams = torch.randint(0, 5, (M,), device=DEV) if fc else None
    gout = torch.randn(M, 4, device=DEV)
    res = {}
    for on in (True, False):
        monkeypatch.setattr(mlp, switch, on)
        tr = train.TrainRayCaster(cfg, ck, mlp="mixed").train()
        net = tr.network_fn
        f = feat.clone().requires_grad_(need_feat)
        (net(f, cams) * gout).sum().backward()
        res[on] = (f.grad, {k: p.grad.clone() for k, p in net.named_parameters()})

    def rel(a, b):
        return float((a.double() - b.double()).norm() / max(b.double().norm(), 1e-30))
    tol = 1e-5 if switch == "FUSED_SKIP" else 1e-4
    if need_feat:
        assert rel(res[True][0], res[False][0]) <= tol
    else:
        assert res[True][0] is None
    for k in res[False][1]:
        assert res[True][1][k].shape == res[False][1][k].shape
        assert rel(res[True][1][k], res[False][1][k]) <= tol, (k, rel(res[True][1][k], res[False][1][k]))


@pytest.mark.parametrize("D,W,fc,nj,M", [(8, 256, False, 24, 5000), (4, 128, True, 24, 3001), (8, 256, True, 17, 77),
                                         (8, 128, False, 65, 1000), (2, 256, False, 24, 40)])
def test_fused_forward_matches_layer_by_layer_gemms(D, W, fc, nj, M, monkeypatch):
    """anerf_mlp_forward (one kernel, bf16x6) against the layer-by-layer bf16x6 GEMMs on the same
    weights and features: raw and every saved activation (h_i, feature, view hidden) within fp32
    accuracy (2e-6 of each tensor's max |.| + 1e-6: both are fp32-accurate, in other summation
    orders); ragged M (77, 3001) and framecodes included."""
    cfg = anerf.RenderConfig(n_joints=nj, netdepth=D, netwidth=W, opt_framecode=fc,
                             n_framecodes=5 if fc else 0).validate()
    ck = syn.make_checkpoint(7, n_joints=nj, D=D, W=W, fine=False, use_framecode=fc, n_framecodes=5)
    torch.manual_seed(1)
    feat = torch.rand(M, cfg.feature_dim, device=DEV) * 2 - 1
    cams = torch.randint(0, 5, (M,), device=DEV) if fc else None
    saved = {}
    for fused in (True, False):
        monkeypatch.setattr(mlp, "FUSED_FORWARD", fused)
        tr = train.TrainRayCaster(cfg, ck, mlp="bf16x6").train()
        f = feat.clone().requires_grad_(True)
        raw = tr.network_fn(f, cams)
        node = raw.grad_fn
        saved[fused] = (raw.detach(), [t.detach().clone() for t in node.saved_tensors])
    (ra, sa), (rb, sb) = saved[True], saved[False]
    assert torch.all(torch.isfinite(ra))

    def close(a, b, what):
        d = float((a.double() - b.double()).abs().max()) if a.numel() else 0.0
        scale = float(b.abs().max()) if b.numel() else 0.0
        assert d <= 2e-6 * scale + 1e-6, f"{what}: max diff {d:.3e} (max |ref| {scale:.3e})"
    close(ra, rb, "raw")
    assert len(sa) == len(sb)
    for i, (a, b) in enumerate(zip(sa, sb)):  # feat, codes, hf, g, whead, h_0 .. h_{D-1}, params
        assert a.shape == b.shape
        close(a, b, f"saved tensor {i}")


def _forward_hidden(m, x, w_split, prec, b, ldy=256):
    y = torch.full((m, ldy), float("nan"), device=DEV)
    mlp.forward_hidden(m, x, w_split, prec, b, y, torch.device(DEV))
    return y


@pytest.mark.parametrize("prec", [6, 3])
@pytest.mark.parametrize("m", [163840, 131072, 5000, 777, 65, 64, 63, 1, 300001])
def test_forward_hidden_is_bit_identical_to_the_gemm(m, prec):
    """Round 6, ABI 19: the persistent hidden-layer forward (anerf_mlp_forward_hidden) computes relu(x W^T + b) with
    anerf_mlp_gemm's split, products and order, so every output bit matches the GEMM's: ragged m (not a multiple of
    the 64-row chunk, fewer rows than workgroups, more chunks per workgroup than the training step's), strided
    input and output rows (the output's padding column is never written), inputs spanning 2^-60 .. 2^60 with zeros,
    and the fp64 bound of the arithmetic as a second check."""
    torch.manual_seed(m % 997 + prec)
    x = torch.relu(torch.randn(m, 260, device=DEV))[:, :256]  # (ld 260; half the entries exactly 0)
    if m > 10:
        x[::7] *= 2.0 ** 60
        x[3::11] *= 2.0 ** -60
    w = torch.randn(256, 256, device=DEV) / 16
    b = torch.randn(256, device=DEV)
    ws = mlp.split_weight(w, False, prec)
    y = _forward_hidden(m, x, ws, prec, b, ldy=260)
    ref = torch.full((m, 260), float("nan"), device=DEV)
    mlp.gemm(m, 256, 256, [mlp._seg(x, 256)], ws, b, True, [(ref, 260, 256, 0, None, False)], torch.device(DEV), prec)
    assert torch.isnan(y[:, 256:]).all()
    assert torch.equal(y[:, :256], ref[:, :256]), float((y[:, :256] - ref[:, :256]).abs().max())
    full = torch.relu(x.double() @ w.double().t() + b.double())
    bound = _bound(x, w, prec) + 1e-6 * b.double().abs()
    assert torch.all((y[:, :256].double() - full).abs() <= bound)


def test_forward_hidden_edge_cases_and_bad_arguments():
    lib = mlp._lib.load()
    dev = torch.device(DEV)
    w = torch.randn(256, 256, device=DEV)
    ws = mlp.split_weight(w, False, 6)
    b = torch.zeros(256, device=DEV)
    x = torch.randn(64, 256, device=DEV)
    y = torch.empty(64, 256, device=DEV)
    st = mlp._stream(dev)
    P = mlp._lib.ptr
    assert lib.anerf_mlp_forward_hidden(0, 256, P(x), 256, P(ws), 6, P(b), P(y), 256, st) == 0  # (empty: nothing)
    bad = [dict(width=128), dict(prec=4), dict(ldx=255), dict(ldy=258), dict(xoff=1), dict(ldx=1 << 22),
           dict(overlap=True), dict(bias=False)]
    for case in bad:
        xp = x.data_ptr() + 4 * case.get("xoff", 0)
        yp = x.data_ptr() + 4 * 128 if case.get("overlap") else y.data_ptr()
        rc = lib.anerf_mlp_forward_hidden(64, case.get("width", 256), xp, case.get("ldx", 256), P(ws),
                                          case.get("prec", 6), P(b) if case.get("bias", True) else None, yp,
                                          case.get("ldy", 256), st)
        assert rc != 0, case


@pytest.mark.parametrize("prec", [6, 3])
@pytest.mark.parametrize("m", [163840, 4097, 65, 1])
@pytest.mark.parametrize("shape", ["layer0", "skip", "k132"])
def test_forward_layer_segments_are_bit_identical_to_the_gemm(m, prec, shape):
    """anerf_mlp_forward_layer on the trunk's other inputs: layer 0 on the encoder rows' first 432 columns (ld 456),
    the skip layer on [x (432 of ld 456) | h (256)] as two segments (a 128-column unit straddles them), and k = 132
    (the last unit 4 columns wide): every output bit as anerf_mlp_gemm's on the same segments."""
    torch.manual_seed(m % 991 + prec)
    feat = torch.rand(m, 456, device=DEV) * 2 - 1
    h = torch.relu(torch.randn(m, 256, device=DEV))
    if shape == "layer0":
        segs, k = [mlp._seg(feat, 432)], 432
    elif shape == "skip":
        segs, k = [mlp._seg(feat, 432), mlp._seg(h, 256)], 688
    else:
        segs, k = [mlp._seg(feat, 132)], 132
    w = torch.randn(256, k, device=DEV) / 16
    b = torch.randn(256, device=DEV)
    ws = mlp.split_weight(w, False, prec)
    y = torch.full((m, 260), float("nan"), device=DEV)
    mlp.forward_layer(m, k, segs, ws, prec, b, True, y, torch.device(DEV))
    ref = torch.full((m, 260), float("nan"), device=DEV)
    mlp.gemm(m, 256, k, segs, ws, b, True, [(ref, 260, 256, 0, None, False)], torch.device(DEV), prec)
    assert torch.isnan(y[:, 256:]).all()
    assert torch.equal(y[:, :256], ref[:, :256]), float((y[:, :256] - ref[:, :256]).abs().max())


@pytest.mark.parametrize("prec", [3, 6])
@pytest.mark.parametrize("m", [163840, 777, 1])
@pytest.mark.parametrize("n", [432, 176, 256, 4])
def test_gemm_persistent_is_bit_identical_to_the_gemm(m, n, prec):
    """anerf_mlp_gemm_persistent (one launch per 256 output columns) as the training backward's feature gradient:
    dX = [dY_0 | dY_s] W^T with W [512][n] split transposed, no bias, no relu, written into the first n columns of
    rows with ld 460 (the rest of each row untouched), every bit as anerf_mlp_gemm's; with a bias and relu too."""
    torch.manual_seed(m % 89 + n + prec)
    dy = torch.randn(m, 512, device=DEV)
    w = torch.randn(512, n, device=DEV) / 16
    wt = mlp.split_weight(w, True, prec)
    for bias, relu in ((None, False), (torch.randn(n, device=DEV), True)):
        y = torch.full((m, 460), float("nan"), device=DEV)
        mlp.gemm_persistent(m, n, 512, [mlp._seg(dy, 512)], wt, prec, bias, relu, y, torch.device(DEV))
        ref = torch.full((m, 460), float("nan"), device=DEV)
        mlp.gemm(m, n, 512, [mlp._seg(dy, 512)], wt, bias, relu, [(ref, 460, n, 0, None, False)], torch.device(DEV),
                 prec)
        assert torch.isnan(y[:, n:]).all()
        assert torch.equal(y[:, :n], ref[:, :n]), float((y[:, :n] - ref[:, :n]).abs().max())


@pytest.mark.parametrize("m", [163840, 777, 1])
def test_forward_layer_head_with_alpha(m):
    """feature_linear (no relu) with alpha_linear beside it: the 256 outputs bit-identical to the GEMM's, alpha (fp32
    dot products of the staged rows) within fp32 accumulation error of fp64, written to its strided column only."""
    torch.manual_seed(m % 101)
    x = torch.relu(torch.randn(m, 256, device=DEV))
    wf = torch.randn(256, 256, device=DEV) / 16
    bf = torch.randn(256, device=DEV)
    wa = torch.randn(1, 256, device=DEV) / 16
    ba = torch.randn(1, device=DEV)
    ws = mlp.split_weight(wf, False, 6)
    hf = torch.empty(m, 256, device=DEV)
    raw = torch.full((m, 4), float("nan"), device=DEV)
    mlp.forward_layer(m, 256, [mlp._seg(x, 256)], ws, 6, bf, False, hf, torch.device(DEV), alpha=(wa, ba, raw[:, 3]))
    ref = torch.empty(m, 256, device=DEV)
    mlp.gemm(m, 256, 256, [mlp._seg(x, 256)], ws, bf, False, [(ref, 256, 256, 0, None, False)], torch.device(DEV), 6)
    assert torch.equal(hf, ref)
    assert (hf < 0).any()  # (no relu)
    assert torch.isnan(raw[:, :3]).all()
    full = x.double() @ wa.double().t()[:, 0] + ba.double()
    bound = 4e-6 * (x.double().abs() @ wa.double().abs().t()[:, 0] + ba.double().abs()) + 1e-7
    assert torch.all((raw[:, 3].double() - full).abs() <= bound), float((raw[:, 3].double() - full).abs().max())


def test_forward_layer_rejects_bad_arguments():
    lib = mlp._lib.load()
    dev = torch.device(DEV)
    x = torch.randn(64, 512, device=DEV)
    y = torch.empty(64, 256, device=DEV)
    b = torch.zeros(256, device=DEV)
    ws = mlp.split_weight(torch.randn(256, 512, device=DEV), False, 6)
    P = mlp._lib.ptr

    def call(segs, k, prec=6, bias=b, alpha=None):
        sa, na = mlp._segs(segs)
        wa, ba, out = alpha if alpha else (None, None, None)
        return lib.anerf_mlp_forward_layer(64, k, sa, na, P(ws), prec, P(bias), 1, P(y), 256, P(wa), P(ba), P(out), 4,
                                           mlp._stream(dev))
    assert call([mlp._seg(x, 256)], 256) == 0
    assert call([mlp._seg(x, 128)], 128) != 0                        # (k <= 128)
    assert call([mlp._seg(x, 130)], 130) != 0                        # (cols % 4)
    assert call([mlp._seg(x, 128), mlp._seg(x, 128, 128), mlp._seg(x, 128, 256)], 384) != 0  # (3 segments)
    assert call([mlp._seg(x, 256)], 260) != 0                        # (segments do not add up to k)
    assert call([mlp._seg(x, 256)], 256, prec=4) != 0
    assert call([mlp._seg(x, 256)], 256, bias=None) != 0
    assert call([mlp._seg(x, 256)], 256, alpha=(b, None, y)) != 0    # (alpha: all or none)
    sa, na = mlp._segs([mlp._seg(x, 256)])
    assert lib.anerf_mlp_gemm_persistent(64, 254, 256, sa, na, P(ws), 6, None, 0, P(y), 256, mlp._stream(dev)) != 0
    assert lib.anerf_mlp_gemm_persistent(64, 260, 256, sa, na, P(ws), 6, None, 0, P(y), 256, mlp._stream(dev)) != 0


@pytest.mark.parametrize("prec", ["bf16x6", "mixed", "bf16x3"])
def test_network_forward_with_the_persistent_layers(prec, monkeypatch):
    """The training network with every trunk layer and feature_linear on anerf_mlp_forward_layer against the same
    network on anerf_mlp_gemm: the saved activations (h_i, feature, view hidden) and rgb bit-identical, alpha (fp32
    beside the head instead of a 257th split-arithmetic output) to fp32 rounding, the gradients to what that
    difference propagates."""
    cfg = anerf.RenderConfig(n_joints=24, netdepth=8, netwidth=256).validate()
    ck = syn.make_checkpoint(3, n_joints=24, D=8, W=256, fine=False)
    torch.manual_seed(2)
    feat = torch.rand(20000, cfg.feature_dim, device=DEV) * 2 - 1
    out = {}
    for pers in (True, False):
        monkeypatch.setattr(mlp, "FORWARD_PERSISTENT", pers)
        tr = train.TrainRayCaster(cfg, ck, mlp=prec).train()
        f = feat.clone().requires_grad_(True)
        raw = tr.network_fn(f, None)
        saved = [t.detach().clone() for t in raw.grad_fn.saved_tensors]
        raw.square().sum().backward()
        grads = [f.grad.clone()] + [p.grad.clone() for p in tr.parameters() if p.grad is not None]
        out[pers] = (raw.detach(), saved, grads)
    (ra, sa, ga), (rb, sb, gb) = out[True], out[False]
    assert torch.equal(ra[:, :3], rb[:, :3])
    tol = 4e-5 if prec == "bf16x3" else 2e-6  # (the GEMM's alpha column carries its mode's split error)
    assert float((ra[:, 3] - rb[:, 3]).abs().max()) <= tol * float(rb[:, 3].abs().max()) + 1e-7
    assert len(sa) == len(sb) and all(torch.equal(a, b) for a, b in zip(sa, sb))
    assert len(ga) == len(gb)
    for a, b in zip(ga, gb):
        assert float((a - b).abs().max()) <= 10 * tol * float(b.abs().max()) + 1e-9


@pytest.mark.parametrize("accumulate", [False, True])
def test_deferred_side_stream_sync_gives_the_same_gradients(accumulate, monkeypatch):
    """mlp.DEFER_WGRAD_SYNC: layer 0's side-stream weight gradient is waited for at the end of the whole backward
    (an engine callback) instead of inside the MLP's.  The gradients read right after backward() -- including a
    second backward accumulating into existing .grad tensors, where the MLP waits at once -- are bit-identical to
    the immediate wait's, and so are the feature gradient and the encoder rows behind it."""
    cfg = anerf.RenderConfig(n_joints=24, netdepth=8, netwidth=256).validate()
    ck = syn.make_checkpoint(5, n_joints=24, D=8, W=256, fine=False)
    torch.manual_seed(4)
    feat = torch.rand(30000, cfg.feature_dim, device=DEV) * 2 - 1
    out = {}
    for defer in (True, False):
        monkeypatch.setattr(mlp, "DEFER_WGRAD_SYNC", defer)
        tr = train.TrainRayCaster(cfg, ck, mlp="mixed").train()
        f = feat.clone().requires_grad_(True)
        (tr.network_fn(f, None).square().sum() * 1e3).backward()
        if accumulate:
            (tr.network_fn(f, None).sum()).backward()
        out[defer] = [f.grad.clone()] + [p.grad.clone() for p in tr.parameters() if p.grad is not None]
    assert len(out[True]) == len(out[False]) > 10
    for a, b in zip(out[True], out[False]):
        assert torch.equal(a, b)


def _backward_hidden(m, dy, x, w, lddx=None):
    """anerf_mlp_backward_hidden on dy [m][256] and x [m][256] (strided views allowed) with W [256][256]."""
    lib = mlp._lib.load()
    dev = torch.device(DEV)
    wt = mlp.split_weight(w, True, 3)
    dx = torch.full((m, lddx or 256), float("nan"), device=DEV)
    dw, db = torch.empty(256, 256, device=DEV), torch.empty(256, device=DEV)
    ws = torch.empty(lib.anerf_mlp_backward_hidden_workspace(m, 256), device=DEV, dtype=torch.uint8)
    mlp._lib.check(lib.anerf_mlp_backward_hidden(m, 256, mlp._lib.ptr(dy), dy.stride(0), mlp._lib.ptr(x), x.stride(0),
                                                 mlp._lib.ptr(wt), 3, mlp._lib.ptr(dx), dx.stride(0), mlp._lib.ptr(dw),
                                                 256, mlp._lib.ptr(db), mlp._lib.ptr(ws), ws.numel(),
                                                 mlp._stream(dev)), "anerf_mlp_backward_hidden")
    return dx, dw, db


@pytest.mark.parametrize("m", [163840, 131072, 5000, 777, 33, 1, 300001])
def test_backward_hidden_matches_fp64(m):
    """Round 6: the fused hidden-layer backward (one pass over dY and X) against fp64 torch of the same sums, at
    the bf16x3 bounds of the two GEMMs it replaces: dX = (dY W) masked by X > 0 (test_gemm_input_gradient_*),
    dW = dY^T X and db = sum dY (test_wgrad_and_bias_gradient); ragged m (not a multiple of the 32-row chunk,
    fewer rows than workgroups, more chunks per workgroup than the training step's) and strided rows."""
    torch.manual_seed(m % 1000)
    dy = torch.randn(m, 260, device=DEV)[:, :256]        # (ld 260)
    x = torch.relu(torch.randn(m, 264, device=DEV))[:, :256]  # (ld 264; half the entries exactly 0)
    w = torch.randn(256, 256, device=DEV) / 16
    dx, dw, db = _backward_hidden(m, dy, x, w, lddx=257)
    full = dy.double() @ w.double()
    ref_dx = torch.where(x > 0, full, torch.zeros_like(full))
    bound = _bound(dy, w.t(), 3)
    assert not torch.isnan(dx[:, :256]).any()
    assert torch.all((dx[:, :256].double() - ref_dx).abs() <= bound), float((dx[:, :256].double() - ref_dx).abs().max())
    assert torch.isnan(dx[:, 256]).all()  # (the padding column of the output rows is never written)
    ref_w = dy.double().t() @ x.double()
    bw = 2 * REL[3] * (dy.double().abs().t() @ x.double().abs()) + 1e-5
    assert torch.all((dw.double() - ref_w).abs() <= bw), float((dw.double() - ref_w).abs().max())
    ref_b = dy.double().sum(0)
    assert torch.all((db.double() - ref_b).abs() <= 1e-5 * dy.double().abs().sum(0) + 1e-5)


def test_backward_hidden_matches_the_two_gemms():
    """The fused pass and the two kernels it replaces (anerf_mlp_gemm with the relu' mask + anerf_mlp_wgrad, bf16x3)
    compute the same bf16x3 products: dX agrees to fp32 summation-order noise and the relu' mask exactly; dW, db to
    fp32 summation order over 163,840 rows.  Deterministic: a second call is bit-identical."""
    torch.manual_seed(5)
    m = 163840
    dy = torch.randn(m, 256, device=DEV)
    x = torch.relu(torch.randn(m, 256, device=DEV))
    w = torch.randn(256, 256, device=DEV) / 16
    dx, dw, db = _backward_hidden(m, dy, x, w)
    dx2, dw2, db2 = _backward_hidden(m, dy, x, w)
    assert torch.equal(dx, dx2) and torch.equal(dw, dw2) and torch.equal(db, db2)
    lib = mlp._lib.load()
    ref_dx = torch.empty(m, 256, device=DEV)
    mlp.gemm(m, 256, 256, [mlp._seg(dy, 256)], mlp.split_weight(w, True, 3), None, False,
             [(ref_dx, 256, 256, 0, x, False)], torch.device(DEV), 3)
    ws = torch.empty(lib.anerf_mlp_wgrad_workspace(m, 256, 256), device=DEV, dtype=torch.uint8)
    ref_dw, ref_db = torch.empty(256, 256, device=DEV), torch.empty(256, device=DEV)
    mlp.wgrad(m, 256, 256, dy, [mlp._seg(x, 256)], ref_dw, ref_db, ws, torch.device(DEV), 3)
    assert torch.equal(dx == 0, ref_dx == 0)
    scale = float(ref_dx.abs().max())
    assert float((dx - ref_dx).abs().max()) <= 1e-6 * scale
    assert float((dw - ref_dw).abs().max()) <= 2e-6 * float(ref_dw.abs().max())
    assert float((db - ref_db).abs().max()) <= 2e-6 * float(ref_db.abs().max())


def test_backward_hidden_rejects_bad_arguments():
    lib = mlp._lib.load()
    m = 64
    dy, x = torch.randn(m, 256, device=DEV), torch.randn(m, 256, device=DEV)
    out = torch.empty(m, 256, device=DEV)
    dw, db = torch.empty(256, 256, device=DEV), torch.empty(256, device=DEV)
    ws = torch.empty(lib.anerf_mlp_backward_hidden_workspace(m, 256), device=DEV, dtype=torch.uint8)
    wt = mlp.split_weight(torch.randn(256, 256, device=DEV), True, 3)
    P = mlp._lib.ptr
    st = mlp._stream(torch.device(DEV))
    assert lib.anerf_mlp_backward_hidden_workspace(m, 128) == 0
    assert lib.anerf_mlp_backward_hidden(m, 128, P(dy), 256, P(x), 256, P(wt), 3, P(out), 256, P(dw), 256, P(db),
                                         P(ws), ws.numel(), st) == -1
    assert lib.anerf_mlp_backward_hidden(m, 256, P(dy), 256, P(x), 256, P(wt), 6, P(out), 256, P(dw), 256, P(db),
                                         P(ws), ws.numel(), st) == -1
    bad = torch.randn(m * 256 + 1, device=DEV)[1:].view(m, 256)  # (rows not 16 B aligned)
    assert lib.anerf_mlp_backward_hidden(m, 256, P(bad), 256, P(x), 256, P(wt), 3, P(out), 256, P(dw), 256, P(db),
                                         P(ws), ws.numel(), st) == -1
    assert lib.anerf_mlp_backward_hidden(m, 256, P(dy), 256, P(x), 256, P(wt), 3, P(out), 256, P(dw), 256, P(db),
                                         P(ws), 16, st) == -3  # (ANERF_EWORKSPACE)


def test_backward_hidden_deferred_reduce_is_identical():
    """dw = db = NULL leaves the slabs in the workspace; anerf_mlp_backward_hidden_reduce (on another stream, as
    mlp.py runs it beside the next layer) gives the same bits as the in-call reduce.  m = 0: zeros."""
    lib = mlp._lib.load()
    P = mlp._lib.ptr
    dev = torch.device(DEV)
    for m in (20000, 0):
        torch.manual_seed(7)
        dy = torch.randn(max(m, 1), 256, device=DEV)
        x = torch.relu(torch.randn(max(m, 1), 256, device=DEV))
        wt = mlp.split_weight(torch.randn(256, 256, device=DEV) / 16, True, 3)
        dx = torch.empty(max(m, 1), 256, device=DEV)
        ws = torch.empty(lib.anerf_mlp_backward_hidden_workspace(m, 256), device=DEV, dtype=torch.uint8)
        dw0, db0 = torch.full((256, 256), 7.0, device=DEV), torch.full((256,), 7.0, device=DEV)
        mlp._lib.check(lib.anerf_mlp_backward_hidden(m, 256, P(dy), 256, P(x), 256, P(wt), 3, P(dx), 256, P(dw0), 256,
                                                     P(db0), P(ws), ws.numel(), mlp._stream(dev)), "direct")
        mlp._lib.check(lib.anerf_mlp_backward_hidden(m, 256, P(dy), 256, P(x), 256, P(wt), 3, P(dx), 256, None, 256,
                                                     None, P(ws), ws.numel(), mlp._stream(dev)), "deferred")
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        dw1, db1 = torch.full((256, 256), 3.0, device=DEV), torch.full((256,), 3.0, device=DEV)
        with torch.cuda.stream(side):
            mlp._lib.check(lib.anerf_mlp_backward_hidden_reduce(m, 256, P(ws), ws.numel(), P(dw1), 256, P(db1),
                                                                mlp._stream(dev)), "reduce")
        torch.cuda.synchronize()
        assert torch.equal(dw0, dw1) and torch.equal(db0, db1)
        if m == 0:
            assert not dw1.any() and not db1.any()


def _backward_head(m, dy, x, wf, wa, lddx=None, defer=False):
    """anerf_mlp_backward_head on dy [m][>= 257] (feature gradients, then alpha's at column 256) and x [m][256]."""
    lib = mlp._lib.load()
    dev = torch.device(DEV)
    P = mlp._lib.ptr
    wt = mlp.split_weight(wf, True, 3)
    dx = torch.full((m, lddx or 256), float("nan"), device=DEV)
    dw, db = torch.full((257, 256), 7.0, device=DEV), torch.full((257,), 7.0, device=DEV)
    ws = torch.empty(lib.anerf_mlp_backward_head_workspace(m, 256), device=DEV, dtype=torch.uint8)
    mlp._lib.check(lib.anerf_mlp_backward_head(m, 256, P(dy), dy.stride(0), P(x), x.stride(0), P(wt), P(wa), 3, P(dx),
                                               dx.stride(0), None if defer else P(dw), 256, None if defer else P(db),
                                               P(ws), ws.numel(), mlp._stream(dev)), "anerf_mlp_backward_head")
    if defer:
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            mlp._lib.check(lib.anerf_mlp_backward_head_reduce(m, 256, P(ws), ws.numel(), P(dw), 256, P(db),
                                                              mlp._stream(dev)), "anerf_mlp_backward_head_reduce")
        torch.cuda.synchronize()
    return dx, dw, db


@pytest.mark.parametrize("m", [163840, 5000, 777, 33, 1, 300001])
def test_backward_head_matches_fp64(m):
    """Round 6 (ABI 18): feature_linear + alpha_linear's backward in one pass, against fp64 torch: dX = (dY_f Wf +
    g_a w_a^T) masked by X > 0 at the bf16x3 bound of the feature part (alpha's rank-1 term in fp32), dW [257][256]
    (row 256 = g_a^T X, fp32 sums), db [257]; ragged m, strided rows (dy ld 260 as the training backward's [g_feature
    | g_alpha | pad] buffer, the pad columns holding garbage that must not reach any output)."""
    torch.manual_seed(m % 997)
    dy = torch.randn(m, 260, device=DEV)
    dy[:, 257:] = float("nan")  # (never read)
    x = torch.relu(torch.randn(m, 264, device=DEV))[:, :256]
    wf = torch.randn(256, 256, device=DEV) / 16
    wa = torch.randn(1, 256, device=DEV) / 16
    dx, dw, db = _backward_head(m, dy, x, wf, wa, lddx=257)
    dyf, ga = dy[:, :256].double(), dy[:, 256].double()
    full = dyf @ wf.double() + ga[:, None] * wa.double()
    ref_dx = torch.where(x > 0, full, torch.zeros_like(full))
    bound = _bound(dy[:, :256], wf.t(), 3) + 1e-6 * (ga.abs()[:, None] * wa.double().abs())
    assert not torch.isnan(dx[:, :256]).any()
    assert torch.all((dx[:, :256].double() - ref_dx).abs() <= bound), float((dx[:, :256].double() - ref_dx).abs().max())
    assert torch.isnan(dx[:, 256]).all()
    ref_w = dy[:, :257].double().t() @ x.double()
    bw = 2 * REL[3] * (dy[:, :257].double().abs().t() @ x.double().abs()) + 1e-5
    bw[256] = 1e-5 * (ga.abs() @ x.double().abs()) + 1e-5  # (alpha's row: fp32 sums)
    assert torch.all((dw.double() - ref_w).abs() <= bw), float((dw.double() - ref_w).abs().max())
    ref_b = dy[:, :257].double().sum(0)
    assert torch.all((db.double() - ref_b).abs() <= 1e-5 * dy[:, :257].double().abs().sum(0) + 1e-5)


def test_backward_head_deferred_and_deterministic():
    """The deferred reduce (another stream) gives the in-call reduce's bits, a second call is bit-identical, and the
    feature part equals anerf_mlp_backward_hidden's on the same dY columns when alpha's gradient is zero."""
    torch.manual_seed(11)
    m = 20000
    dy = torch.randn(m, 260, device=DEV)
    x = torch.relu(torch.randn(m, 256, device=DEV))
    wf, wa = torch.randn(256, 256, device=DEV) / 16, torch.randn(1, 256, device=DEV) / 16
    a = _backward_head(m, dy, x, wf, wa)
    b = _backward_head(m, dy, x, wf, wa, defer=True)
    c = _backward_head(m, dy, x, wf, wa)
    for u, v, w in zip(a, b, c):
        assert torch.equal(u, v) and torch.equal(u, w)
    dy0 = dy.clone()
    dy0[:, 256] = 0.0
    dxh, dwh, dbh = _backward_head(m, dy0, x, wf, wa)
    dx1, dw1, db1 = _backward_hidden(m, dy0[:, :256], x, wf)
    assert torch.equal(dxh, dx1) and torch.equal(dwh[:256], dw1) and torch.equal(dbh[:256], db1)
    assert not dwh[256].any() and float(dbh[256]) == 0.0


def test_backward_head_rejects_bad_arguments():
    lib = mlp._lib.load()
    m = 64
    P = mlp._lib.ptr
    st = mlp._stream(torch.device(DEV))
    dy, x = torch.randn(m, 260, device=DEV), torch.randn(m, 256, device=DEV)
    out = torch.empty(m, 256, device=DEV)
    dw, db = torch.empty(257, 256, device=DEV), torch.empty(257, device=DEV)
    wa = torch.randn(256, device=DEV)
    ws = torch.empty(lib.anerf_mlp_backward_head_workspace(m, 256), device=DEV, dtype=torch.uint8)
    wt = mlp.split_weight(torch.randn(256, 256, device=DEV), True, 3)
    assert lib.anerf_mlp_backward_head_workspace(m, 128) == 0
    assert lib.anerf_mlp_backward_head_workspace(m, 256) > lib.anerf_mlp_backward_hidden_workspace(m, 256)
    ok = (m, 256, P(dy), 260, P(x), 256, P(wt), P(wa), 3, P(out), 256, P(dw), 256, P(db), P(ws), ws.numel(), st)
    assert lib.anerf_mlp_backward_head(*ok) == 0
    bad_ld = list(ok)
    bad_ld[3] = 256  # (no room for alpha's column)
    assert lib.anerf_mlp_backward_head(*bad_ld) == -1
    no_wa = list(ok)
    no_wa[7] = None
    assert lib.anerf_mlp_backward_head(*no_wa) == -1
    small = list(ok)
    small[15] = lib.anerf_mlp_backward_hidden_workspace(m, 256)  # (the hidden pass's size is too small here)
    assert lib.anerf_mlp_backward_head(*small) == -3
    torch.cuda.synchronize()

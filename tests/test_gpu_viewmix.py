"""GPU: anerf_train_view_mix (+ _backward), the view-window layout's view part (anerf.h ANERF_ENC_VIEW_WINDOWS),
against fp64 torch on the same inputs: out = sum_j w_j G_j per sample, dL/dw and dL/dG.  Ragged sample counts
(chunks of 32 in the backward), row strides wider than NJ, joint counts off the powers of two up to the LDS plan's
72 at width 128 (the 65-joint training rows: 1170 kp + bone columns padded to 1172, then the windows; dL/dG in 4 or
9 float4 registers per lane), widths 4-128.
Tolerance 1e-5 relative to the largest |value| (fp32 sums of at most 128 terms)."""
import importlib

import pytest
import torch

pytestmark = pytest.mark.gpu
_lib = importlib.import_module("a-nerf_amd._lib")


@pytest.fixture(scope="module", autouse=True)
def _cuda():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _close(a, ref):
    d = float((a.double() - ref).abs().max())
    assert d <= 1e-5 * float(ref.abs().max()) + 1e-12, d


@pytest.mark.parametrize("n,ns,nj,wh,ld", [(3, 64, 24, 128, 456), (5, 80, 24, 128, 24), (7, 33, 17, 64, 21),
                                           (2, 1, 1, 4, 1), (4, 100, 32, 128, 40), (6, 16, 65, 32, 70),
                                           (5, 80, 65, 128, 1236), (3, 47, 72, 128, 72), (2, 40, 100, 64, 101)])
def test_view_mix_matches_torch(n, ns, nj, wh, ld):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(n * 1000 + ns)
    rows = torch.rand(n * ns, ld, device=dev, generator=g)
    w = rows[:, ld - nj:]  # (the windows at a column offset of a wider row)
    G = torch.randn(n, nj, wh, device=dev, generator=g)
    gz = torch.randn(n * ns, wh, device=dev, generator=g)
    lib = _lib.load()
    st = torch.cuda.current_stream().cuda_stream
    out = torch.empty(n * ns, wh, device=dev)
    _lib.check(lib.anerf_train_view_mix(n, ns, nj, wh, w.data_ptr(), ld, G.data_ptr(), out.data_ptr(), st), "mix")
    gw = torch.full((n * ns, nj + 2), 7.0, device=dev)  # (the window columns 1..NJ of a wider row)
    gG = torch.empty_like(G)
    _lib.check(lib.anerf_train_view_mix_backward(n, ns, nj, wh, w.data_ptr(), ld, G.data_ptr(), gz.data_ptr(),
                                                 gw[:, 1:].data_ptr(), nj + 2, gG.data_ptr(), st), "mix backward")
    torch.cuda.synchronize()
    w3, G3, gz3 = w.double().reshape(n, ns, nj), G.double(), gz.double().reshape(n, ns, wh)
    _close(out.reshape(n, ns, wh), torch.bmm(w3, G3))
    _close(gw[:, 1:nj + 1].reshape(n, ns, nj), torch.bmm(gz3, G3.transpose(1, 2)))
    assert bool((gw[:, nj + 1:] == 7.0).all()) and bool((gw[:, 0] == 7.0).all())  # (only the window columns)
    _close(gG, torch.bmm(w3.transpose(1, 2), gz3))



@pytest.mark.parametrize("mrv,world,sched", [(4, False, False), (4, False, True), (0, False, False), (2, True, True)])
def test_view_factor_matches_torch(mrv, world, sched):
    """anerf_train_view_factor (+ _backward) through train._ViewFactor against the torch restatement
    (tests/_view_ref.py) in fp64 on the host: G, dL/dskts, dL/d(views_linears.0.weight) for a random dL/dG; 300 rays (ragged
    workgroups), relray / world directions, multires_views 4 / 2 / 0, with and without schedule weights.
    Tolerance: G 1e-5, gradients 1e-4 of the largest |value| (fp32 sums over the rays, atomics)."""
    import dataclasses
    from _view_ref import fs_view_of, view_factor, view_terms
    anerf = importlib.import_module("a-nerf_amd")
    train = importlib.import_module("a-nerf_amd.train")
    dev = torch.device("cuda:0")
    cfg = anerf.RenderConfig(multires_views=mrv, extra={"view_type": "world" if world else "relray"}).validate()
    tr = train.TrainRayCaster(cfg, device=dev)
    model = tr.model
    nj, W, nv = cfg.n_joints, cfg.netwidth, cfg.input_ch_views
    g = torch.Generator(device=dev).manual_seed(mrv * 10 + int(world))
    n = 300
    sk = torch.randn(n, nj, 4, 4, device=dev, generator=g)
    rb = torch.randn(n, 11, device=dev, generator=g)
    weight = torch.randn(W // 2, W + nv, device=dev, generator=g) * 0.1
    fs = torch.rand(nv, device=dev, generator=g) + 0.5 if sched else None
    gG = torch.randn(n, nj, W // 2, device=dev, generator=g)
    sk1, w1 = sk.clone().requires_grad_(True), weight.clone().requires_grad_(True)
    G = train._ViewFactor.apply(sk1, w1, model, rb, fs)
    G.backward(gG)
    # (the fp64 restatement on the host: no device BLAS in the checker)
    sk2, w2 = sk.double().cpu().requires_grad_(True), weight.double().cpu().requires_grad_(True)
    fsv = None if fs is None else fs_view_of(fs.double().cpu(), nj)
    Gr = view_factor(w2, cfg, view_terms(cfg, sk2, rb[:, 3:6].double().cpu(), fsv))
    Gr.backward(gG.double().cpu())
    torch.cuda.synchronize()

    def close(a, ref, tol):
        d = float((a.detach().double().cpu() - ref.detach()).abs().max())
        assert d <= tol * float(ref.abs().max()) + 1e-12, d
    close(G, Gr.detach(), 1e-5)
    close(sk1.grad, sk2.grad, 1e-4)
    assert bool((sk1.grad[:, :, 3, :] == 0).all()) and bool((sk1.grad[:, :, :, 3] == 0).all())
    close(w1.grad, w2.grad, 1e-4)
    assert bool((w1.grad[:, :W] == 0).all())  # (only the view columns)

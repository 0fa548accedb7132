"""GPU parity of the training render path against the reference's own
training-mode render_rays + autograd (tests/golden/t*.npz, made by make_train_golden.py with the
reference's torch.rand / torch.randn draws recorded and fed back here).

Tolerances:
  * rgb_map / disp_map / acc_map (+ coarse): 1e-4 absolute (north star); per-sample alpha 2e-3
    (hazard H11, see test_gpu_parity.py); loss 1e-5 relative
  * gradients (per-ray skeleton transforms, every network parameter): |g - g_ref| <= 2e-3 max|g_ref|
    per tensor and the norm of sampled tensors within 1e-3 relative — fp32 sums of thousands of
    sample terms in a different order (GEMM reductions, atomics over samples)
"""
import importlib

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from _golden import Golden

pytestmark = pytest.mark.gpu

anerf = importlib.import_module("a-nerf_amd")
train = importlib.import_module("a-nerf_amd.train")

TRAIN = ["t1_s32i16_d4w128", "t2_s64i16_d8w256", "t3_softplus_fc", "t4_tau200", "t5_single_mrv0",
         "t6_lindisp_raynoise", "t7_single_raynoise", "t8_freqsched", "t9_cutto_shift", "t10_cutoffbones",
         "t11_mr5_mrv2_world", "t12_staged_relpos_rayangle_mrb2", "t13_querypts_shift", "t14_nj65_d8w256"]
TOL = 1e-4
TOL_ALPHA = 2e-3
GRAD_REL = 2e-3


@pytest.fixture(scope="module", autouse=True)
def _cuda():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _loss(out, tgt, bg):
    return (F.mse_loss(out["rgb_map"] + (1 - out["acc_map"])[:, None] * bg, tgt) +
            F.mse_loss(out["rgb0"] + (1 - out["acc0"])[:, None] * bg, tgt))


def _run(name, mlp="mixed", view_windows=True):
    g = Golden(name)
    m = g.meta
    tr = train.TrainRayCaster(g.cfg, g.ckpt, mlp=mlp).train()
    tr.view_windows = view_windows  # (the view-window layout where the configuration allows it, anerf.h)
    dev = torch.device("cuda:0")
    if m.get("global_step") is not None:
        # Trainer.train_batch's call (core/trainer.py:263-265), through the DataParallel-style alias
        import argparse
        tr.module.update_embed_fns(m["global_step"], argparse.Namespace(
            cutoff_step=m["cutoff_step"], cutoff_rate=m["cutoff_rate"], freq_schedule_step=5, multires=7))
        assert (tr.module.embed_fn.get_tau(), tr.module.embeddirs_fn.get_tau()) == tuple(m["tau_step"])
        if m.get("sched_step") is not None:  # --freq_schedule: sched_alpha moved as update_alpha moves it
            assert (float(tr.embed_fn.sched_alpha), float(tr.embeddirs_fn.sched_alpha)) == tuple(m["sched_step"])
    c = lambda k: torch.from_numpy(g[k]).to(dev)  # noqa: E731
    sk = c("skts").clone().requires_grad_(True)
    rand = {k: c("rand_" + k) for k in ("t_rand", "noise0", "u", "noise1", "pts_noise0", "pts_noise1")
            if g.has("rand_" + k)}
    out = tr.render_rays(c("rays"), m["S"], skts=sk, cyls=c("cyls"), cams=c("cams") if g.has("cams") else None,
                         perturb=1.0, N_importance=m["I"], raw_noise_std=m["raw_noise_std"], rand=rand,
                         lindisp=m.get("lindisp", False), ray_noise_std=m.get("ray_noise_std", 0.0))
    loss = _loss(out, c("target"), c("bg"))
    loss.backward()
    torch.cuda.synchronize()
    assert tr.model.view_windows == (view_windows and train.view_windows_ok(g.cfg))
    return g, tr, sk, out, loss


# the training MLP on the hand-written split-bf16 GEMMs (mixed — the default —, mixed16 and bf16x6) and on
# torch's fp32 GEMMs; the view-window layout (the default where it applies) and the full view columns
@pytest.fixture(scope="module", params=[(n, mlp, vw) for n in TRAIN for mlp in ("mixed", "mixed16", "bf16x6", "fp32")
                                        for vw in (True, False) if vw or mlp in ("mixed", "fp32")],
                ids=lambda p: f"{p[0]}-{p[1]}" + ("" if p[2] else "-fullview"))
def run(request):
    return _run(*request.param)


def test_train_outputs_match_reference(run):
    g, tr, sk, out, loss = run
    for k in ("rgb_map", "disp_map", "acc_map", "rgb0", "disp0", "acc0"):
        d = float(np.abs(out[k].detach().cpu().numpy() - g["out_" + k]).max())
        assert d <= TOL, f"{g.name} {k}: max |gpu - reference| = {d:.3e}"
    for k in ("alpha", "alpha0"):
        d = float(np.abs(out[k].detach().cpu().numpy() - g["out_" + k]).max())
        assert d <= TOL_ALPHA, f"{g.name} {k}: {d:.3e}"
    assert abs(loss.item() - float(g["loss"])) <= 1e-5 * abs(float(g["loss"])), (loss.item(), float(g["loss"]))


def _close(a, ref, what):
    scale = float(np.abs(ref).max())
    d = float(np.abs(a - ref).max())
    assert d <= GRAD_REL * scale + 1e-12, f"{what}: max |grad - ref| {d:.3e} vs max |ref| {scale:.3e}"


def test_train_pose_gradient_matches_reference(run):
    g, tr, sk, out, loss = run
    gs = sk.grad.detach().cpu().numpy()
    _close(gs, g["grad_skts"], f"{g.name} dL/dskts")
    assert np.all(gs[:, :, 3, :] == 0.0)


def test_train_parameter_gradients_match_reference(run):
    g, tr, sk, out, loss = run
    nets = {"fn": tr.network_fn, "fine": tr.network_fine}
    n_checked = 0
    for key in g.d:
        if not key.startswith("grad_") or key == "grad_skts" or key.endswith("__idx") or key.endswith("__norm"):
            continue
        net, pname = key[len("grad_"):].split("__", 1)
        p = dict(nets[net].named_parameters())[pname]
        gp = p.grad.detach().cpu().numpy().reshape(-1)
        if g.has(key + "__idx"):
            norm_ref = float(g[key + "__norm"])
            assert abs(np.linalg.norm(gp.astype(np.float64)) - norm_ref) <= 1e-3 * norm_ref + 1e-12, key
            gp = gp[g[key + "__idx"]]
        _close(gp, g[key], f"{g.name} {key}")
        n_checked += 1
    assert n_checked >= 10


@pytest.mark.parametrize("name", ["t2_s64i16_d8w256", "t14_nj65_d8w256"])
def test_fine_stream_is_bit_identical(name, monkeypatch):
    """train.FINE_STREAM (round 6, measured slower and off by default): the fine pass on its own stream, so that the
    coarse and fine backward passes overlap, gives the single-stream step's outputs, pose gradient and parameter
    gradients bit for bit (the same kernels on the same inputs; the streams only reorder independent work), over a
    step of Adam and a second forward."""
    if name not in TRAIN:
        pytest.skip(f"{name}: no golden")
    res = {}
    for on in (True, False):
        monkeypatch.setattr(train, "FINE_STREAM", on)
        g, tr, sk, out, loss = _run(name)
        opt = torch.optim.Adam(tr.parameters(), lr=1e-3)
        opt.step()
        out2 = _run_again(g, tr)
        torch.cuda.synchronize()
        res[on] = ({k: v.detach().clone() for k, v in out.items()}, sk.grad.clone(),
                   {k: p.detach().clone() for k, p in tr.named_parameters()}, out2)
    (o1, s1, p1, q1), (o0, s0, p0, q0) = res[True], res[False]
    for k in o0:
        assert torch.equal(o1[k], o0[k]), k
    assert torch.equal(s1, s0)
    for k in p0:
        assert torch.equal(p1[k], p0[k]), k
    for k in q0:
        assert torch.equal(q1[k], q0[k]), k


def _run_again(g, tr):
    """A second forward of the stepped model on the golden's rays (its outputs, detached)."""
    m = g.meta
    dev = torch.device("cuda:0")
    c = lambda k: torch.from_numpy(g[k]).to(dev)  # noqa: E731
    rand = {k: c("rand_" + k) for k in ("t_rand", "noise0", "u", "noise1", "pts_noise0", "pts_noise1")
            if g.has("rand_" + k)}
    out = tr.render_rays(c("rays"), m["S"], skts=c("skts"), cyls=c("cyls"), cams=c("cams") if g.has("cams") else None,
                         perturb=1.0, N_importance=m["I"], raw_noise_std=m["raw_noise_std"], rand=rand,
                         lindisp=m.get("lindisp", False), ray_noise_std=m.get("ray_noise_std", 0.0))
    return {k: v.detach().clone() for k, v in out.items()}


def test_eval_mode_delegates_to_fused_kernel():
    g = Golden("t1_s32i16_d4w128")
    m = g.meta
    tr = train.TrainRayCaster(g.cfg, g.ckpt).eval()
    dev = torch.device("cuda:0")
    rb = torch.from_numpy(g["rays"]).to(dev)
    sk = torch.from_numpy(g["skts"]).to(dev)
    cy = torch.from_numpy(g["cyls"]).to(dev)
    out = tr(rb, m["S"], skts=sk, cyls=cy, N_importance=m["I"])
    ref = anerf.RayCaster(g.cfg, g.ckpt).render_rays(rb, m["S"], skts=sk, cyls=cy, N_importance=m["I"])
    for k in ("rgb_map", "disp_map", "acc_map", "rgb0"):
        assert torch.equal(out[k], ref[k]), k
    # after a parameter update the eval delegate is repacked
    with torch.no_grad():
        tr.network_fine.rgb_linear.bias.add_(0.5)
    out2 = tr(rb, m["S"], skts=sk, cyls=cy, N_importance=m["I"])
    assert not torch.equal(out2["rgb_map"], out["rgb_map"])


def test_deterministic_training_path_matches_eval_kernel():
    """perturb=0, raw_noise_std=0: the training stages reproduce the fused eval kernel (1e-4)."""
    g = Golden("t2_s64i16_d8w256")
    m = g.meta
    tr = train.TrainRayCaster(g.cfg, g.ckpt).train()
    dev = torch.device("cuda:0")
    rb = torch.from_numpy(g["rays"]).to(dev)
    sk = torch.from_numpy(g["skts"]).to(dev)
    cy = torch.from_numpy(g["cyls"]).to(dev)
    with torch.no_grad():
        out = tr.render_rays(rb, m["S"], skts=sk, cyls=cy, N_importance=m["I"])
    ref = anerf.RayCaster(g.cfg, g.ckpt).render_rays(rb, m["S"], skts=sk, cyls=cy, N_importance=m["I"])
    for k in ("rgb_map", "disp_map", "acc_map", "rgb0", "disp0", "acc0"):
        d = float((out[k] - ref[k]).abs().max())
        assert d <= TOL, f"{k}: {d:.3e}"


def test_adam_steps_reduce_loss_and_move_pose():
    g = Golden("t1_s32i16_d4w128")
    m = g.meta
    tr = train.TrainRayCaster(g.cfg, g.ckpt).train()
    dev = torch.device("cuda:0")
    c = lambda k: torch.from_numpy(g[k]).to(dev)  # noqa: E731
    sk0 = c("skts")
    delta = torch.zeros_like(sk0, requires_grad=True)
    opt = torch.optim.Adam(list(tr.parameters()) + [delta], lr=5e-4)
    losses = []
    torch.manual_seed(0)
    for _ in range(30):
        opt.zero_grad()
        out = tr.render_rays(c("rays"), m["S"], skts=sk0 + delta, cyls=c("cyls"), perturb=1.0,
                             N_importance=m["I"], raw_noise_std=1.0)
        loss = _loss(out, c("target"), c("bg"))
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert np.mean(losses[-5:]) < 0.8 * np.mean(losses[:5]), losses
    assert float(delta.detach().abs().max()) > 0.0


def test_create_raycaster_training_drop_in(tmp_path):
    """create_raycaster (core/raycasters.py:17-184) returns train kwargs with the trainable caster,
    grad_vars and Adam; one core.trainer.render-style step through anerf.render trains it, and the
    test kwargs render the updated weights with the fused kernel."""
    import argparse
    kin = importlib.import_module("a-nerf_amd.kinematics")
    g = Golden("t1_s32i16_d4w128")
    m = g.meta
    args = argparse.Namespace(netdepth=4, netwidth=128, N_samples=m["S"], N_importance=m["I"], use_cutoff=True,
                              cutoff_inputs=True, cutoff_viewdir=True, use_viewdirs=True, perturb=1.0,
                              raw_noise_std=1.0, lrate=5e-4, basedir=str(tmp_path), expname="x", no_reload=False,
                              ft_path=None, ext_scale=0.001, chunk=4096)
    os_ = importlib.import_module("os")
    os_.makedirs(tmp_path / "x", exist_ok=True)
    tr_kw, te_kw, start, grad_vars, opt, ck = anerf.create_raycaster(args, {"skel_type": kin.SMPLSkeleton},
                                                                     device=0, ckpt=g.ckpt)
    assert start == 0
    assert len(grad_vars) == len([p for p in tr_kw["ray_caster"].parameters() if p.requires_grad])
    dev = torch.device("cuda:0")
    rays = torch.from_numpy(g["rays"]).to(dev)
    sk = torch.from_numpy(g["skts"]).to(dev)
    cy = torch.from_numpy(g["cyls"]).to(dev)
    te0 = anerf.render(None, None, None, chunk=4096, rays=(rays[:, :3], rays[:, 3:6]), skts=sk, cyls=cy, **te_kw)
    # (the drop-in renders in the default precision, fp16x4: the same kernel as a RayCaster in that mode)
    import dataclasses
    assert tr_kw["ray_caster"].cfg.precision == "fp16x4"
    ref = anerf.RayCaster(dataclasses.replace(g.cfg, precision="fp16x4"), g.ckpt).render_rays(
        rays, m["S"], skts=sk, cyls=cy, N_importance=m["I"])
    assert torch.equal(te0["rgb_map"], ref["rgb_map"])
    out = anerf.render(None, None, None, chunk=4096, rays=(rays[:, :3], rays[:, 3:6]), skts=sk, cyls=cy, **tr_kw)
    loss = train.nerf_loss(out, torch.from_numpy(g["target"]).to(dev))
    loss.backward()
    opt.step()
    te1 = anerf.render(None, None, None, chunk=4096, rays=(rays[:, :3], rays[:, 3:6]), skts=sk, cyls=cy, **te_kw)
    assert not torch.equal(te1["rgb_map"], te0["rgb_map"])
    # no checkpoint: torch's default initialisation, as the reference
    tr_kw2, *_ = anerf.create_raycaster(args, {"skel_type": kin.SMPLSkeleton}, device=0)
    assert isinstance(tr_kw2["ray_caster"], train.TrainRayCaster)
    assert torch.allclose(tr_kw2["ray_caster"].embed_fn.cutoff_dist, torch.full((24,), 0.5, device=dev))


def test_tau_schedule_reaches_eval_kernel_without_repack():
    """update_embed_fns changes tau for the training stages AND the fused eval delegate; the eval
    model is updated in place (anerf_model_set_embed), and matches a RayCaster built at that tau."""
    import argparse
    g = Golden("t4_tau200")
    m = g.meta
    tr = train.TrainRayCaster(g.cfg, g.ckpt).eval()
    dev = torch.device("cuda:0")
    rb, sk, cy = (torch.from_numpy(g[k]).to(dev) for k in ("rays", "skts", "cyls"))
    out20 = tr(rb, m["S"], skts=sk, cyls=cy, N_importance=m["I"])
    handle = tr.eval_caster().model.handle.value
    tr.module.update_embed_fns(m["global_step"], argparse.Namespace(cutoff_step=m["cutoff_step"],
                                                                    cutoff_rate=m["cutoff_rate"]))
    out200 = tr(rb, m["S"], skts=sk, cyls=cy, N_importance=m["I"])
    assert tr.eval_caster().model.handle.value == handle          # no repack
    assert not torch.equal(out200["rgb_map"], out20["rgb_map"])
    ck = {k: dict(v) for k, v in g.ckpt.items()}
    for e in ("embed_state_dict", "embeddirs_state_dict"):
        ck[e]["tau"] = np.array(200.0, np.float32)
    ref = anerf.RayCaster(g.cfg, ck).render_rays(rb, m["S"], skts=sk, cyls=cy, N_importance=m["I"])
    for k in ("rgb_map", "disp_map", "acc_map", "rgb0"):
        assert torch.equal(out200[k], ref[k]), k


def test_checkpoint_round_trip_through_torch_save(tmp_path):
    """checkpoint() -> torch.save -> load_checkpoint (weights_only) -> TrainRayCaster renders the same."""
    g = Golden("t1_s32i16_d4w128")
    m = g.meta
    tr = train.TrainRayCaster(g.cfg, g.ckpt).eval()
    with torch.no_grad():
        tr.network_fine.rgb_linear.bias.add_(0.25)
    path = tmp_path / "000100.tar"
    torch.save(tr.checkpoint(), path)
    tr2 = train.TrainRayCaster(g.cfg, anerf.raycaster.load_checkpoint(str(path))).eval()
    dev = torch.device("cuda:0")
    rb, sk, cy = (torch.from_numpy(g[k]).to(dev) for k in ("rays", "skts", "cyls"))
    a = tr(rb, m["S"], skts=sk, cyls=cy, N_importance=m["I"])
    b = tr2(rb, m["S"], skts=sk, cyls=cy, N_importance=m["I"])
    for k in ("rgb_map", "disp_map", "acc_map", "rgb0"):
        assert torch.equal(a[k], b[k]), k


def test_weights_changed_forces_the_eval_repack():
    """TrainRayCaster.weights_changed(): after an update the version counters may not show (torch's fused Adam),
    the next eval render repacks and renders the new weights."""
    g = Golden("t1_s32i16_d4w128")
    m = g.meta
    tr = train.TrainRayCaster(g.cfg, g.ckpt).eval()
    dev = torch.device("cuda:0")
    rays, sk, cy = (torch.from_numpy(g[k]).to(dev) for k in ("rays", "skts", "cyls"))
    r0 = tr.eval_caster().render_rays(rays, m["S"], skts=sk, cyls=cy, N_importance=m["I"])["rgb_map"].clone()
    with torch.no_grad():
        for p in tr.network_fn.parameters():
            p.data.mul_(1.01)  # (through .data: the version counter does not move)
    tr.weights_changed()
    r1 = tr.eval_caster().render_rays(rays, m["S"], skts=sk, cyls=cy, N_importance=m["I"])["rgb_map"]
    assert not torch.equal(r0, r1)

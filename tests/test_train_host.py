"""CPU checks of the training path's host side: the torch NeRF module (split skip / view weights
instead of the reference's concatenations) against a direct transcription of
core/networks/nerf.py:94-148, and state-dict key compatibility with the reference fixtures."""
import importlib

import numpy as np
import torch
import torch.nn.functional as F

from _golden import Golden
from _view_ref import fs_view_of, view_factor, view_terms

train = importlib.import_module("a-nerf_amd.train")


def _ref_forward(sd, cfg, feat, codes=None):
    """nerf.py forward_density + forward_view with torch.cat, as the reference writes it."""
    dnet = cfg.input_ch + cfg.input_ch_bones
    x, views = feat[:, :dnet], feat[:, dnet:]
    h = x
    for i in range(cfg.netdepth):
        h = F.relu(F.linear(h, sd[f"pts_linears.{i}.weight"], sd[f"pts_linears.{i}.bias"]))
        if i in cfg.skips:
            h = torch.cat([x, h], -1)
    alpha = F.linear(h, sd["alpha_linear.weight"], sd["alpha_linear.bias"])
    feature = F.linear(h, sd["feature_linear.weight"], sd["feature_linear.bias"])
    if codes is not None:
        views = torch.cat([views, codes], -1)
    g = F.relu(F.linear(torch.cat([feature, views], -1), sd["views_linears.0.weight"], sd["views_linears.0.bias"]))
    return torch.cat([F.linear(g, sd["rgb_linear.weight"], sd["rgb_linear.bias"]), alpha], -1)


def test_split_weight_nerf_matches_concatenating_reference():
    for name in ("t2_s64i16_d8w256", "t3_softplus_fc"):
        g = Golden(name)
        cfg = g.cfg
        net = train.NeRF(cfg).double()
        net.mlp = "fp32"  # the torch form (the split-bf16 GEMMs are GPU-only: test_gpu_mlp.py)
        sd = {k: torch.from_numpy(np.asarray(v, np.float64)) for k, v in g.ckpt["network_fn_state_dict"].items()}
        net.load_state_dict(sd)
        feat = torch.from_numpy(np.random.default_rng(0).normal(size=(37, cfg.feature_dim)))
        cams = None
        codes = None
        if cfg.opt_framecode:
            cams = torch.arange(37) % 5
            codes = sd["framecodes.codes.weight"][cams]
        out = net(feat, cams)
        ref = _ref_forward(sd, cfg, feat, codes)
        assert torch.allclose(out, ref, rtol=1e-12, atol=1e-12)


def test_parameter_names_match_reference_gradients():
    g = Golden("t2_s64i16_d8w256")
    names = set(dict(train.NeRF(g.cfg).named_parameters()))
    ref = {k[len("grad_fn__"):] for k in g.d if k.startswith("grad_fn__") and not k.endswith("__idx")
           and not k.endswith("__norm")}
    assert ref and ref == names


def test_tau_schedule_follows_update_tau():
    """update_embed_fns -> CutoffEmbedder.update_tau (core/cutoff_embedder.py:181-183):
    20 * rate ** (step / (cutoff_step * 1000)) clamped at 2000, float32, in both embedders."""
    import argparse
    g = Golden("t1_s32i16_d4w128")
    tr = train.TrainRayCaster(g.cfg, g.ckpt, device="cpu")
    args = argparse.Namespace(cutoff_step=250, cutoff_rate=10.0, freq_schedule_step=5, multires=7)
    for step, want in ((0, 20.0), (250000, 200.0), (500000, 2000.0), (10 ** 7, 2000.0), (123457, None)):
        tr.module.update_embed_fns(step, args)
        with np.errstate(over="ignore"):
            exp = np.float32(np.float32(20.0) * np.float32(10.0 ** (step / 250000.0)))
        exp = min(exp, np.float32(2000.0))
        assert tr.embed_fn.get_tau() == tr.embeddirs_fn.get_tau() == float(exp)
        if want is not None:
            assert abs(tr.embed_fn.get_tau() - want) <= 1e-3 * want
    assert tr.module is tr


def test_schedule_host_copies_and_tau_only_embed_updates():
    """The tau / sched_alpha schedule keeps host copies (no device read per step), a write it did not
    make is picked up (load_state_dict, in-place edits), and a tau-only change reaches a DeviceModel
    as set_embed(cutoffs=False): no device synchronisation or copy."""
    import argparse
    g = Golden("t1_s32i16_d4w128")
    tr = train.TrainRayCaster(g.cfg, g.ckpt, device="cpu")
    args = argparse.Namespace(cutoff_step=250, cutoff_rate=10.0, freq_schedule_step=5, multires=7)
    tr.update_embed_fns(123457, args)
    assert tr.embed_fn.host("tau") == float(tr.embed_fn.tau)  # the host copy is the buffer's value
    # the device expression of the reference (ones_like on the buffer) gives the same float32
    ref = (20.0 * torch.ones_like(tr.embed_fn.tau) * 10.0 ** (123457 / 250000.0)).clamp(max=2000.)
    assert float(ref) == tr.embed_fn.get_tau()
    with torch.no_grad():
        tr.embed_fn.tau.fill_(77.0)  # a write the schedule did not make
    assert tr.embed_fn.get_tau() == 77.0
    sd = tr.embeddirs_fn.state_dict()
    sd["tau"] = torch.tensor(33.0)
    tr.embeddirs_fn.load_state_dict(sd)
    assert tr.embeddirs_fn.get_tau() == 33.0

    class Rec:
        def __init__(self):
            self.calls = []

        def set_embed(self, e, ev, cutoffs=True, embedbones_sd=None):
            self.calls.append((e["tau"], ev["tau"], cutoffs))
    m = Rec()
    seen = tr._embed_version()
    assert tr._sync_embed(m, seen) == seen and m.calls == []  # nothing changed
    tr.update_embed_fns(250000, args)
    seen = tr._sync_embed(m, seen)
    assert len(m.calls) == 1 and m.calls[-1][2] is False  # tau only
    assert m.calls[-1][:2] == (tr.embed_fn.get_tau(), tr.embeddirs_fn.get_tau())
    assert isinstance(m.calls[-1][0], float)
    with torch.no_grad():
        tr.embed_fn.cutoff_dist.mul_(1.5)
    seen = tr._sync_embed(m, seen)
    assert m.calls[-1][2] is True and len(m.calls) == 2


def test_checkpoint_is_tensors_and_round_trips(tmp_path):
    """checkpoint() holds CPU tensors in the reference's layout: torch.save -> torch.load(weights_only)
    -> nn.Module.load_state_dict on a fresh module (the reference's loader) and back."""
    g = Golden("t3_softplus_fc")
    tr = train.TrainRayCaster(g.cfg, g.ckpt, device="cpu")
    ck = tr.checkpoint()
    for top in ("network_fn_state_dict", "network_fine_state_dict", "embed_state_dict", "embeddirs_state_dict"):
        assert all(isinstance(v, torch.Tensor) and v.device.type == "cpu" for v in ck[top].values()), top
    path = tmp_path / "ck.tar"
    torch.save(ck, path)
    ld = torch.load(path, weights_only=True)
    fresh = train.NeRF(g.cfg)
    fresh.load_state_dict(ld["network_fine_state_dict"])
    for k, v in fresh.state_dict().items():
        assert torch.equal(v, ck["network_fine_state_dict"][k]), k
    tr2 = train.TrainRayCaster(g.cfg, ld, device="cpu")
    for (k, a), (_, b) in zip(tr.state_dict().items(), tr2.state_dict().items()):
        assert torch.equal(a, b), k


def test_single_net_shares_one_module_and_fine_keys_win():
    """single_net: network_fine IS network_fn (raycasters.py:98-104), both keys in the state dict;
    a checkpoint with two different nets loads network_fine's last (RayCaster.load_state_dict)."""
    g = Golden("t5_single_mrv0")
    tr = train.TrainRayCaster(g.cfg, g.ckpt, device="cpu")
    assert tr.network_fine is tr.network_fn
    ck = tr.checkpoint()
    assert set(ck["network_fn_state_dict"]) == set(ck["network_fine_state_dict"])
    for k, v in ck["network_fn_state_dict"].items():
        assert torch.equal(v, torch.as_tensor(g.ckpt["network_fine_state_dict"][k])), k


def test_nerf_loss_functions_follow_trainer():
    """loss_fn MSE / L1 / Huber (the shipped h36m / mixamo / perfcap configs use L1) and the BCE
    regulariser, restated from core/trainer.py:10-58 (img2mse, img2l1, acc2bce, img2huber) and
    _compute_nerf_loss / compute_loss (:325-381): background composite, coarse weight on the rgb
    term only, reg over fgs < 1, everything summed."""
    g = torch.Generator().manual_seed(0)
    n = 257
    preds = {"rgb_map": torch.rand(n, 3, generator=g), "acc_map": torch.rand(n, generator=g) * 0.98 + 0.01,
             "rgb0": torch.rand(n, 3, generator=g), "acc0": torch.rand(n, generator=g) * 0.98 + 0.01}
    tgt = torch.rand(n, 3, generator=g)
    fgs = (torch.rand(n, 1, generator=g) > 0.5).float()
    bgs = torch.rand(n, 3, generator=g)
    for fn, ref in (("MSE", lambda x, y: ((x - y) ** 2).mean()), ("L1", lambda x, y: (x - y).abs().mean()),
                    ("Huber", lambda x, y: F.smooth_l1_loss(x, y, beta=0.05))):
        total, parts = train.nerf_loss(preds, tgt, bgs=bgs, use_background=True, coarse_weight=0.5, loss_fn=fn,
                                       loss_beta=0.05, reg_fn="BCE", reg_coef=0.3, fgs=fgs, return_dict=True)
        want = {}
        for c, (rk, ak) in enumerate((("rgb_map", "acc_map"), ("rgb0", "acc0"))):
            rgb = preds[rk] + (1.0 - preds[ak])[..., None] * bgs
            acc, y = preds[ak], fgs[..., 0]
            bce = -(y * torch.log(acc + 1e-8) + (1.0 - y) * torch.log(1 - acc + 1e-8))
            want["rgb_loss" + ("0" if c else "")] = ref(rgb, tgt) * (0.5 if c else 1.0)
            want["reg_loss" + ("0" if c else "")] = bce[y < 1.0].mean() * 0.3
        assert set(parts) == set(want)
        for k in want:
            assert torch.allclose(parts[k], want[k], rtol=1e-6, atol=0), (fn, k)
        assert torch.allclose(total, sum(want.values()), rtol=1e-6)
    # the default stays the round-1 MSE form
    plain = train.nerf_loss(preds, tgt)
    assert torch.allclose(plain, ((preds["rgb_map"] - tgt) ** 2).mean() + ((preds["rgb0"] - tgt) ** 2).mean())


def test_segment_padding_is_exact_for_any_joint_count():
    """mlp._pad_to_segments (joint counts whose feature blocks are not multiples of 4 columns):
    the padded layer-0, skip and view products equal the unpadded ones (zeros added), and
    autograd through the pads gives the unpadded gradients."""
    mlp = importlib.import_module("a-nerf_amd.mlp")
    anerf = importlib.import_module("a-nerf_amd")
    for nj, fc in ((17, False), (26, True), (65, False)):
        cfg = anerf.RenderConfig(n_joints=nj, netdepth=8, netwidth=64, opt_framecode=fc,
                                 n_framecodes=5 if fc else 0).validate()
        net = train.NeRF(cfg).double()
        D, W, skip, dnet, nv = 8, 64, cfg.skips[0], net.dnet, cfg.input_ch_views
        params = []
        for lin in net.pts_linears:
            params += [lin.weight, lin.bias]
        params += [net.alpha_linear.weight, net.alpha_linear.bias, net.feature_linear.weight,
                   net.feature_linear.bias, net.views_linears[0].weight, net.views_linears[0].bias,
                   net.rgb_linear.weight, net.rgb_linear.bias]
        feat = torch.randn(9, cfg.feature_dim, dtype=torch.float64, requires_grad=True)
        fp, pp, d4, v4 = mlp._pad_to_segments(feat, params, W, D, skip, dnet, nv)
        assert d4 % 4 == 0 and v4 % 4 == 0 and fp.shape[1] == d4 + v4
        h = torch.randn(9, W, dtype=torch.float64)
        code = torch.randn(9, cfg.framecode_ch, dtype=torch.float64)
        ref = (feat[:, :dnet] @ params[0].t(), torch.cat([feat[:, :dnet], h], 1) @ params[2 * (skip + 1)].t(),
               torch.cat([h, feat[:, dnet:dnet + nv], code], 1) @ params[2 * D + 4].t())
        got = (fp[:, :d4] @ pp[0].t(), torch.cat([fp[:, :d4], h], 1) @ pp[2 * (skip + 1)].t(),
               torch.cat([h, fp[:, d4:d4 + v4], code], 1) @ pp[2 * D + 4].t())
        for r, g in zip(ref, got):  # (BLAS blocks a longer k differently: equal up to double rounding)
            assert torch.allclose(r, g, rtol=1e-12, atol=1e-12)
        sum(g.sum() for g in got).backward()
        gf = feat.grad.clone()
        feat.grad = None
        sum(r.sum() for r in ref).backward()
        assert torch.allclose(gf, feat.grad, rtol=1e-12, atol=1e-12)


def test_training_caster_takes_generic_multires_and_world_views():
    """Round 5: the training encoder backward has a generic instance (multires 1-10, multires_views 0-4)
    and takes --view_type world; the GPU parity is tests/test_gpu_train.py's t11 fixture."""
    import dataclasses

    import pytest
    g = Golden("t11_mr5_mrv2_world")
    cfg = g.cfg
    assert (cfg.multires, cfg.multires_views, cfg.extra.get("view_type")) == (5, 2, "world")
    tr = train.TrainRayCaster(cfg, g.ckpt, device="cpu")  # (CPU: the parameters only)
    assert tr.network_fn.pts_linears[0].weight.shape[1] == cfg.input_ch + cfg.input_ch_bones
    with pytest.raises(NotImplementedError, match="multires"):
        train.TrainRayCaster(dataclasses.replace(cfg, multires=11), device="cpu")


def test_view_window_layout_matches_full_view_columns():
    """anerf.h ANERF_ENC_VIEW_WINDOWS: the view layer on [x | NJ windows] with G = view_factor(view_terms(...))
    (tests/_view_ref.py, the checker of anerf_train_view_factor) equals
    the reference forward on the full view columns w_j T_f(e_j)_c (column f 3 NJ + 3 j + c; encode_joint's view part,
    transcribed here per element), with a --freq_schedule weight per view column; relray and world directions,
    multires_views 4 and 0."""
    import dataclasses
    base = Golden("t2_s64i16_d8w256")
    rng = np.random.default_rng(3)
    for mrv, world in ((4, False), (0, False), (4, True)):
        cfg = dataclasses.replace(base.cfg, multires_views=mrv,
                                  extra=dict(base.cfg.extra, view_type="world" if world else "relray"))
        assert train.view_windows_ok(cfg)
        nj, W, dnet, nv = cfg.n_joints, cfg.netwidth, cfg.input_ch + cfg.input_ch_bones, cfg.input_ch_views
        nf = 1 + 2 * mrv
        net = train.NeRF(cfg).double()
        net.mlp = "fp32"
        for p in net.parameters():
            p.data.normal_(0.0, 0.1, generator=torch.Generator().manual_seed(int(rng.integers(1 << 30))))
        n, ns = 5, 7
        sk = rng.normal(size=(n, nj, 4, 4))
        d = rng.normal(size=(n, 3))
        w = rng.uniform(size=(n, ns, nj))
        x = rng.normal(size=(n * ns, dnet))
        fsv = rng.uniform(0.5, 1.5, size=nv)
        full = np.zeros((n, ns, nv))
        for r in range(n):
            for j in range(nj):
                e = sk[r, j, :3, :3] @ d[r]
                if not world:
                    e = e / max(np.linalg.norm(e), 1e-12)
                for f in range(nf):
                    t = e if f == 0 else (np.sin if f % 2 else np.cos)(e * 2.0 ** ((f - 1) // 2))
                    for c in range(3):
                        col = f * 3 * nj + 3 * j + c
                        full[r, :, col] = w[r, :, j] * t[c] * fsv[col]
        feat_full = torch.from_numpy(np.concatenate([x, full.reshape(n * ns, nv)], 1))
        ref = net(feat_full)
        T = view_terms(cfg, torch.from_numpy(sk), torch.from_numpy(d), fs_view_of(torch.from_numpy(fsv), nj))
        G = view_factor(net.views_linears[0].weight, cfg, T)
        assert G.shape == (n, nj, W // 2)
        got = net(torch.from_numpy(np.concatenate([x, w.reshape(n * ns, nj)], 1)), None, G)
        np.testing.assert_allclose(got.detach().numpy(), ref.detach().numpy(), rtol=1e-10, atol=1e-10)


def test_view_window_layout_conditions():
    """view_windows_ok: every view feature windowed (cutoff_viewdir and cutoff_inputs), no ray-angle views, no staged
    encoder, the per-ray factors within anerf_train_view_mix's LDS plan (anerf.h: width 128 -> NJ <= 72; other NJ % 4
    run on zero-padded rows)."""
    import dataclasses
    cfg = Golden("t2_s64i16_d8w256").cfg
    assert train.view_windows_ok(cfg)
    assert not train.view_windows_ok(dataclasses.replace(cfg, cutoff_viewdir=False))
    assert not train.view_windows_ok(dataclasses.replace(cfg, cutoff_inputs=False))
    #  --cutoff_viewdir without --use_cutoff: the reference's view embedder is a plain Embedder
    # (core/raycasters.py:31, 68-71 -> cutoff_embedder.py:216-220), no window to factor and none to schedule
    nocut = dataclasses.replace(cfg, use_cutoff=False)
    assert nocut.cutoff_viewdir and not nocut.view_window
    assert not train.view_windows_ok(nocut)
    fs = importlib.import_module("a-nerf_amd.config").feature_scales(dataclasses.replace(nocut, freq_schedule=True), 1.5, 1.5)
    assert (fs == 1).all()  # (neither the pts nor the view embedder is a CutoffEmbedder: no schedule weights)
    assert train.view_windows_ok(dataclasses.replace(cfg, n_joints=17))
    assert train.view_windows_ok(dataclasses.replace(cfg, n_joints=65))
    assert not train.view_windows_ok(dataclasses.replace(cfg, n_joints=80))
    assert train.view_mix_lds_ok(72, 128) and not train.view_mix_lds_ok(73, 128)
    assert train.view_mix_lds_ok(140, 64) and not train.view_mix_lds_ok(141, 64)

"""CPU checks of the training path's host side: the torch NeRF module (split skip / view weights
instead of the reference's concatenations) against a direct transcription of
core/networks/nerf.py:94-148, and state-dict key compatibility with the reference fixtures."""
import importlib

import numpy as np
import torch
import torch.nn.functional as F

from _golden import Golden

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

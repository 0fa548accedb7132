"""Torch restatement of the view-window layout's per-ray view factors (anerf.h ANERF_ENC_VIEW_WINDOWS): the checker
for anerf_train_view_factor (+ _backward) and, on the CPU, of the layout's algebra against the full view columns.
Test infrastructure only (autograd gives its gradients)."""
import torch


def view_terms(cfg, sk, d, fs_view=None):
    """T [rays, NJ, 3 (1 + 2 multires_views)]: joint j's view features of a ray without their window -- e = R_j d /
    max(|R_j d|, 1e-12) (R_j d itself for --view_type world) and its sin / cos at 2^k, slot f component c at 3 f + c
    (the train encoder's view part; core/encoders.py:172-193, cutoff_embedder.py:111-166), times the --freq_schedule
    weights fs_view [NJ, 3 (1 + 2 multires_views)].  sk [rays, NJ, 4, 4], d [rays, 3]."""
    e = (sk[:, :, :3, :3] * d[:, None, None, :]).sum(-1)
    if cfg.extra.get("view_type", "relray") != "world":
        e = e / e.norm(dim=-1, keepdim=True).clamp_min(1e-12)
    n, nj = e.shape[:2]
    parts = [e[:, :, None, :]]
    if cfg.multires_views > 0:
        fr = 2.0 ** torch.arange(cfg.multires_views, device=e.device, dtype=e.dtype)
        a = e[:, :, None, :] * fr[:, None]
        parts.append(torch.stack([torch.sin(a), torch.cos(a)], 3).reshape(n, nj, 2 * cfg.multires_views, 3))
    T = torch.cat(parts, 2).reshape(n, nj, -1)
    return T if fs_view is None else T * fs_view


def view_factor(weight, cfg, T):
    """G [rays, NJ, W/2] = per joint, views_linears.0's view columns (column f 3 NJ + 3 j + c of its view part) times
    T (view_terms)."""
    W, nj = cfg.netwidth, T.shape[1]
    nv = cfg.input_ch_views
    wv = weight[:, W:W + nv].reshape(W // 2, -1, nj, 3).permute(2, 1, 3, 0).reshape(nj, -1, W // 2)
    return torch.bmm(T.transpose(0, 1), wv).transpose(0, 1)


def fs_view_of(fs_cols, nj):
    """The view columns' schedule weights [input_ch_views] (column f 3 NJ + 3 j + c) as view_terms' [NJ, 3 NF]."""
    return fs_cols.reshape(-1, nj, 3).transpose(0, 1).reshape(nj, -1)

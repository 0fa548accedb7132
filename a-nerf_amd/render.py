"""Drop-in `render`, `batchify_rays` and `render_path` over the HIP render path.

Signatures and return values mirror the reference:
  * `batchify_rays(rays_flat, chunk, ray_caster, **kwargs)` — core/trainer.py:64-79
  * `render(H, W, focal, chunk, rays, c2w, near, far, center, use_viewdirs, c2w_staticcam, **kw)`
    — core/trainer.py:82-145
  * `render_path(render_poses, hwf, chunk, render_kwargs, ...)` — run_nerf.py:27-145
The reference loops over 4096-ray chunks in Python and launches dozens of ATen ops per
chunk; here one `anerf_render_rays` launch covers every ray of a frame and `chunk` only sets
the NaN-fill granularity of get_near_far_in_cylinder (ray_utils.py:328-342), which keeps the
results identical to the chunked reference.
"""
import numpy as np
import torch
import torch.nn.functional as F

from . import _lib
from . import rays as host_rays


def batchify_rays(rays_flat, chunk=1024 * 32, ray_caster=None, **kwargs):
    """core/trainer.py:64-79: render in chunk-sized groups (one fused launch, chunked NaN fill)."""
    return ray_caster(rays_flat, chunk=chunk, **kwargs)


def _ray_batch(rays_o, rays_d, near, far, use_viewdirs):
    sh = rays_d.shape
    rays_o = rays_o.reshape(-1, 3).float()
    rays_d = rays_d.reshape(-1, 3).float()
    n = rays_d.shape[0]
    near_t = near * torch.ones(n, 1, device=rays_d.device) if not torch.is_tensor(near) else near.reshape(n, 1).float()
    far_t = far * torch.ones(n, 1, device=rays_d.device) if not torch.is_tensor(far) else far.reshape(n, 1).float()
    cols = [rays_o.to(rays_d.device), rays_d, near_t, far_t]
    if use_viewdirs:
        cols.append(rays_d / torch.norm(rays_d, dim=-1, keepdim=True))
    return torch.cat(cols, -1).contiguous(), sh


def render(H, W, focal, chunk=1024 * 32, rays=None, c2w=None, near=0., far=1., center=None, use_viewdirs=False,
           c2w_staticcam=None, **kwargs):
    """core/trainer.py:82-145 (the `rays` form; the full-image c2w form is served by render_path)."""
    if rays is None:
        raise NotImplementedError("render() without an explicit ray batch: use render_path")
    if c2w_staticcam is not None:
        raise NotImplementedError("c2w_staticcam is not implemented")
    rays_o, rays_d = rays
    dev = kwargs["ray_caster"].model.device
    rays_o = torch.as_tensor(rays_o).to(f"cuda:{dev}")
    rays_d = torch.as_tensor(rays_d).to(f"cuda:{dev}")
    rb, sh = _ray_batch(rays_o, rays_d, near, far, use_viewdirs)
    all_ret = batchify_rays(rb, chunk, **kwargs)
    for k in list(all_ret):
        if all_ret[k] is None or all_ret[k].dim() >= 4:
            continue
        all_ret[k] = torch.reshape(all_ret[k], list(sh[:-1]) + list(all_ret[k].shape[1:]))
    return all_ret


def _to_np(x):
    if x is None:
        return None
    if torch.is_tensor(x):
        return x.detach().cpu().numpy()
    return np.asarray(x)


def _frame_rows(x, i):
    """reuse_input of run_nerf.py:63-74: frame i uses row i % len(x)."""
    if x is None:
        return None
    x = torch.as_tensor(x)
    return x[i % x.shape[0]: i % x.shape[0] + 1]


@torch.no_grad()
def render_frames(render_poses, hwf, chunk, render_kwargs, centers=None, kp=None, skts=None, cyls=None, bones=None,
                  bg_imgs=None, bg_indices=None, cams=None, subject_idxs=None, render_factor=0, white_bkgd=False,
                  ret_acc=False, ext_scale=0.00035, frame_ids=None, to_host=True):
    """Core of render_path; frame_ids restricts the work to some frames (used by the multi-GPU path).
    Returns per-frame lists (device tensors when to_host=False)."""
    H, W, focal = hwf
    if render_factor != 0:
        H, W = H // render_factor, W // render_factor
        if isinstance(focal, float):
            focal = focal / render_factor
            centers = None if centers is None else np.asarray(centers) / render_factor
        else:
            focal = np.array(focal, copy=True) / render_factor
            centers = None if centers is None else np.array(centers, copy=True) / render_factor
    if subject_idxs is not None:  # (render_rays raises for them, as the reference's NeRF does)
        raise RuntimeError("subject_idxs: the NeRF input has one column more than "
                           "input_ch + input_ch_bones + input_ch_views + cam_ch (core/networks/nerf.py:135)")
    rc = render_kwargs["ray_caster"]
    dev = torch.device(f"cuda:{rc.model.device}")
    poses_np = _to_np(render_poses).astype(np.float32)
    n_frames = poses_np.shape[0]
    if kp is None and cyls is None:
        raise NotImplementedError("full-image rendering without a skeleton bounding cylinder is not implemented")
    on_dev = any(torch.is_tensor(x) and x.is_cuda for x in (kp, cyls)) and isinstance(H, int) and isinstance(W, int)
    if on_dev:
        # skeleton already on the device (e.g. kinematics.PoseOptLayer): cylinder and box there too
        cyl_params, bboxes = host_rays.device_boxes(poses_np, H, W, focal, kps=kp, cylinders=cyls,
                                                    ext_scale=ext_scale,
                                                    centers=None if centers is None else _to_np(centers), device=dev)
        valid_idxs = [host_rays.box_pixels(tl, br, W) for tl, br in bboxes]
    else:
        valid_idxs, cyl_params, bboxes = host_rays.valid_pixels(
            poses_np, H, W, focal, kps=_to_np(kp), cylinders=_to_np(cyls), ext_scale=ext_scale,
            centers=None if centers is None else _to_np(centers))
        cyl_params = torch.from_numpy(np.ascontiguousarray(cyl_params))
    lib = _lib.load()
    st = _lib.stream_handle(dev)
    frames = range(n_frames) if frame_ids is None else frame_ids
    out = []
    kw = {k: v for k, v in render_kwargs.items() if k not in ("ray_caster", "use_viewdirs")}
    for i in frames:
        h = H if isinstance(H, int) else int(H[i])
        w = W if isinstance(W, int) else int(W[i])
        fa = np.asarray(focal if isinstance(focal, float) else focal[i], dtype=np.float64).reshape(-1)
        fx = float(fa[0])
        fy = float(fa[1]) if fa.size >= 2 else fx
        # the pixel set is the box [tl, br) (valid_idxs[i] is its row-major enumeration): rays are
        # generated on the device from the box, nothing per pixel crosses PCIe
        (x0, y0), (x1, y1) = (int(v) for v in bboxes[i][0]), (int(v) for v in bboxes[i][1])
        n = max(x1 - x0, 0) * max(y1 - y0, 0)
        assert n == len(valid_idxs[i])
        c2w = torch.from_numpy(np.ascontiguousarray(poses_np[i][:3, :4])).to(dev)
        rb = torch.empty(n, 11, device=dev, dtype=torch.float32)
        has_c = centers is not None
        cx, cy = (float(centers[i][0]), float(centers[i][1])) if has_c else (0.0, 0.0)
        _lib.check(lib.anerf_gen_rays_box(_lib.ptr(c2w), h, w, fx, fy, cx, cy, int(has_c), x0, y0, x1, y1, 0.0, 1.0,
                                          _lib.ptr(rb), st), "anerf_gen_rays_box")
        if n > 0:
            cam_i = _frame_rows(cams, i)
            ret = rc.render_rays(rb, kw.get("N_samples"), kp_batch=None, skts=_frame_rows(skts, i).to(dev),
                                 cyls=_frame_rows(cyl_params, i).to(dev),
                                 cams=None if cam_i is None else cam_i.to(dev).float().expand(n),
                                 N_importance=kw.get("N_importance", 0), perturb=kw.get("perturb", 0.),
                                 raw_noise_std=kw.get("raw_noise_std", 0.), ray_noise_std=kw.get("ray_noise_std", 0.),
                                 lindisp=kw.get("lindisp", False), preproc_kwargs=kw.get("preproc_kwargs"),
                                 chunk=chunk, ret_alpha=False)
            rgb, disp, acc = ret["rgb_map"], ret["disp_map"], ret["acc_map"]
        else:
            rgb = disp = acc = None
        bg = None
        if bg_imgs is not None and not white_bkgd:
            b = bg_imgs[bg_indices[i]] if bg_indices is not None else bg_imgs[0]
            b = torch.as_tensor(np.asarray(b)).permute(2, 0, 1)[None].float().to(dev)
            bg = F.interpolate(b, size=(h, w), mode="bilinear", align_corners=False)[0].permute(1, 2, 0).reshape(
                h * w, 3).contiguous()
        img = torch.empty(h * w, 3, device=dev)
        dimg = torch.empty(h * w, device=dev)
        aimg = torch.empty(h * w, device=dev)
        _lib.check(lib.anerf_compose_box(_lib.ptr(rgb), _lib.ptr(disp), _lib.ptr(acc), x0, y0, x1, y1, _lib.ptr(bg),
                                         int(bool(white_bkgd)), h, w, _lib.ptr(img), _lib.ptr(dimg), _lib.ptr(aimg),
                                         st), "anerf_compose_box")
        fr = (img.view(h, w, 3), dimg.view(h, w, 1), aimg.view(h, w, 1))
        if to_host:
            fr = tuple(t.cpu().numpy() for t in fr)
        out.append(fr)
    return out, [torch.from_numpy(v) for v in valid_idxs], bboxes


@torch.no_grad()
def render_path(render_poses, hwf, chunk, render_kwargs, centers=None, kp=None, skts=None, cyls=None, bones=None,
                gt_imgs=None, bg_imgs=None, bg_indices=None, cams=None, subject_idxs=None, render_factor=0,
                white_bkgd=False, ret_acc=False, ext_scale=0.00035, base_bg=1.0):
    """run_nerf.py:27-145 -> (rgbs (F,H,W,3), disps (F,H,W,1), accs, valid_idxs, bboxes) as numpy."""
    frames, valid_idxs, bboxes = render_frames(render_poses, hwf, chunk, render_kwargs, centers=centers, kp=kp,
                                               skts=skts, cyls=cyls, bones=bones, bg_imgs=bg_imgs,
                                               bg_indices=bg_indices, cams=cams, subject_idxs=subject_idxs,
                                               render_factor=render_factor, white_bkgd=white_bkgd,
                                               ret_acc=ret_acc, ext_scale=ext_scale)
    rgbs = np.stack([f[0] for f in frames], 0)
    disps = np.stack([f[1] for f in frames], 0)
    accs = np.stack([f[2] for f in frames], 0) if ret_acc else []
    return rgbs, disps, accs, valid_idxs, bboxes

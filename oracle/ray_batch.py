"""CPU restatement of the image dataset's ray batch.  TEST INFRASTRUCTURE ONLY.

Only tests/ import this module (the product path is anerf_ray_batch in libanerf_hip.so, driven by
a-nerf_amd/dataset.py).  Pinned by tests/golden/raybatch.npz, produced by running the reference's
own BaseH5Dataset.__getitem__ over in-memory arrays (tests/golden/make_dataset_golden.py).

float32 numpy arithmetic in the reference's order:
* get_rays (core/dataset.py:346-364): dirs = (x - W/2, -(y - H/2), -1) precomputed
  (core/dataset.py:146-163; with per-image centers the offsets are 0 and dirs[:2] -= (cx, -cy)),
  dirs[:2] /= focal, rays_d = sum(dirs * c2w[:3, :3], -1) unless np.isclose(I, c2w[:3, :3]).all(),
  rays_o = c2w[:3, 3];
* get_img_data (core/dataset.py:259-275): img / 255., fg = mask, bg = bkgds[bkgd_idxs[idx]] / 255.,
  img * fg + (1 - fg) * bg when mask_img.
"""
import numpy as np


def image_rays(c2w, focal, pixel_idxs, H, W, center=None):
    i = (pixel_idxs % W).astype(np.float32)
    j = (pixel_idxs // W).astype(np.float32)
    if center is None:
        ox, oy = np.float32(W * 0.5), np.float32(H * 0.5)
    else:
        ox = oy = np.float32(0.0)
    dirs = np.stack([i - ox, -(j - oy), -np.ones_like(i)], axis=-1).astype(np.float32)
    if center is not None:
        c = np.asarray(center, np.float32).copy()
        c[1] *= -1
        dirs[:, :2] -= c
    dirs[:, :2] /= np.float32(focal)
    c2w = np.asarray(c2w, np.float32)
    if np.isclose(np.eye(3), c2w[:3, :3]).all():
        rays_d = dirs
    else:
        rays_d = np.sum(dirs[:, None, :] * c2w[:3, :3], -1, dtype=np.float32)
    rays_o = np.broadcast_to(c2w[:3, 3], rays_d.shape)
    return rays_o.copy(), rays_d.copy()


def image_data(img, mask, pixel_idxs, bg=None, mask_img=False):
    fg = mask[pixel_idxs].astype(np.float32).reshape(-1, 1)
    rgb = img[pixel_idxs].astype(np.float32) / np.float32(255.0)
    b = None
    if bg is not None:
        b = bg[pixel_idxs].astype(np.float32) / np.float32(255.0)
        if mask_img:
            rgb = rgb * fg + (np.float32(1.0) - fg) * b
    return rgb, fg, b


def ray_batch(data, rows, pixels, mask_img=False):
    """Flattened batch of several images: dict rays_o, rays_d, target_s, fgs, bgs."""
    H, W = int(data["img_shape"][1]), int(data["img_shape"][2])
    imgs = np.asarray(data["imgs"]).reshape(-1, H * W, 3)
    masks = np.asarray(data["masks"]).reshape(-1, H * W)
    has_bg = "bkgds" in data
    out = {k: [] for k in ("rays_o", "rays_d", "target_s", "fgs", "bgs")}
    for r, pix in zip(rows, pixels):
        center = data["centers"][r] if "centers" in data else None
        o, d = image_rays(data["c2ws"][r], data["focals"][r], pix, H, W, center)
        bg = np.asarray(data["bkgds"]).reshape(-1, H * W, 3)[data["bkgd_idxs"][r]] if has_bg else None
        rgb, fg, b = image_data(imgs[r], masks[r], pix, bg, mask_img and has_bg)
        for k, v in zip(out, (o, d, rgb, fg, b)):
            out[k].append(v)
    return {k: (np.concatenate(v) if v and v[0] is not None else None) for k, v in out.items()}

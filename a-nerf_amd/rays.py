"""Host-side per-frame ray selection (integer pixel sets), bit-exact with the reference.

Restates, in numpy with the same dtype flow, the host half of the render path:

* bounding cylinder of a skeleton  — `get_kp_bounding_cylinder`
  (`core/utils/skeleton_utils.py:542-592`), called by `kp_to_valid_rays` with
  extend_mm=250, top_expand_ratio=1.6, bot_expand_ratio=1.1, head='-y'
  (`core/utils/ray_utils.py:88-104`);
* projection of the cylinder's two caps to a 2-D box — `cylinder_to_box_2d`
  (`skeleton_utils.py:607-694`) with `nerf_c2w_to_extrinsic` / `swap_mat` /
  `focal_to_intrinsic_np` (`skeleton_utils.py:442-443, 1308-1327`);
* the row-major pixel list `idx = y*W + x`, y in [tl_y, br_y), x in [tl_x, br_x)
  (`ray_utils.py:127-130`; exclusive upper bound, box clipped to W-1/H-1, so the
  last row/column is never traced — parity hazard H2).

The float math is float64 numpy exactly as in the reference (float32 cylinder,
float64 cap points, float32 extrinsic/intrinsic), so floor/ceil land on the same
integers.  Ray origins/directions are generated on the GPU from these indices
(`anerf_gen_rays` in the C-ABI).
"""
import numpy as np


def bounding_cylinder(kps, ext_scale, extend_mm=250, top_expand_ratio=1.6,
                      bot_expand_ratio=1.1, head="-y", root_id=0):
    """kps (F,NJ,3) float32 -> cylinders (F,5) float32 = (cx, cz, r, top, bot)."""
    if head.endswith("z"):
        g_axes, h_axis = [0, 1], 2
    elif head.endswith("y"):
        g_axes, h_axis = [0, 2], 1
    else:
        raise NotImplementedError(f"head orientation {head}")
    flip = -1 if head.startswith("-") else 1
    kps = np.asarray(kps)
    if kps.ndim != 3:
        raise ValueError("kps must be (F, NJ, 3)")
    root = kps[..., root_id, :]
    dist = np.linalg.norm(kps[..., g_axes] - root[:, None, g_axes], axis=-1)
    max_dist = dist.max(-1)
    heights = flip * kps[..., h_axis]
    max_h = heights.max(-1)
    min_h = heights.min(-1)
    ext = extend_mm * ext_scale
    radius = max_dist + ext
    top = flip * (max_h + ext * top_expand_ratio)
    bot = flip * (min_h - ext * bot_expand_ratio)
    return np.stack([root[..., g_axes[0]], root[..., g_axes[1]], radius, top, bot], axis=-1)


def _extrinsic_from_c2w(c2w):
    c2w = np.asarray(c2w)
    swapped = np.concatenate([c2w[..., 0:1], -c2w[..., 1:2], -c2w[..., 2:3], c2w[..., 3:]], axis=-1)
    return np.linalg.inv(swapped)


def _intrinsic(focal):
    if isinstance(focal, float) or np.asarray(focal).size < 2:
        fx = fy = focal
    else:
        fx, fy = focal
    return np.array([[fx, 0, 0, 0], [0, fy, 0, 0], [0, 0, 1, 0]], dtype=np.float32)


def cylinder_box(cyl, H, W, focal, c2w, center=None, scale=1.0):
    """2-D integer box (tl, br) of one cylinder (5,) seen by camera c2w (4,4); `scale` grows it about
    its centre as cylinder_to_box_2d(..., scale) does (skeleton_utils.py:672-682)."""
    cyl = np.asarray(cyl)
    root, radius = cyl[..., :2][None], cyl[..., 2:3][None]
    top, bot = cyl[..., 3:4][None], cyl[..., 4:5][None]
    angles = np.linspace(0.0, 2 * np.pi, 50)
    x = root[..., 0:1] + np.cos(angles)[None] * radius
    z = root[..., 1:2] + np.sin(angles)[None] * radius
    ones = np.ones_like(x)
    caps = np.concatenate([np.stack([x, top * ones, z, ones], axis=-1),
                           np.stack([x, bot * ones, z, ones], axis=-1)], axis=-2).reshape(-1, 4)
    w2c = _extrinsic_from_c2w(c2w)
    caps = caps @ w2c.T
    caps = caps @ _intrinsic(focal).T
    caps = caps.reshape(1, -1, 3)
    p2 = caps[..., :2] / caps[..., 2:3]
    max_x = np.ceil(p2[..., 0].max(-1)).astype(np.int32)
    min_x = np.floor(p2[..., 0].min(-1)).astype(np.int32)
    max_y = np.ceil(p2[..., 1].max(-1)).astype(np.int32)
    min_y = np.floor(p2[..., 1].min(-1)).astype(np.int32)
    tl = np.stack([min_x, min_y], axis=-1)
    br = np.stack([max_x, max_y], axis=-1)
    if center is None:
        ox, oy = int(W * .5), int(H * .5)
    else:
        ox, oy = int(center[0]), int(center[1])
    tl[:, 0] += ox
    tl[:, 1] += oy
    br[:, 0] += ox
    br[:, 1] += oy
    if scale != 1.0:
        # float64 half-extents and centre, stored back into the int32 boxes (truncation)
        half_w = (max_x - min_x) * 0.5 * scale
        half_h = (max_y - min_y) * 0.5 * scale
        cx = (br[:, 0] + tl[:, 0]).copy() * 0.5
        cy = (br[:, 1] + tl[:, 1]).copy() * 0.5
        tl[:, 0] = cx - half_w
        br[:, 0] = cx + half_w
        tl[:, 1] = cy - half_h
        br[:, 1] = cy + half_h
    tl[:, 0] = np.clip(tl[:, 0], 0, W - 1)
    br[:, 0] = np.clip(br[:, 0], 0, W - 1)
    tl[:, 1] = np.clip(tl[:, 1], 0, H - 1)
    br[:, 1] = np.clip(br[:, 1], 0, H - 1)
    return tl[0], br[0]


def box_pixels(tl, br, W):
    """Row-major int64 pixel indices of the half-open box [tl, br)."""
    ys = np.arange(int(tl[1]), int(br[1]), dtype=np.int64)
    xs = np.arange(int(tl[0]), int(br[0]), dtype=np.int64)
    return (ys[:, None] * W + xs[None, :]).reshape(-1)


def valid_pixels(c2ws, H, W, focal, kps=None, cylinders=None, ext_scale=0.00035, centers=None):
    """Per-frame pixel sets, like kp_to_valid_rays (ray_utils.py:83-136) minus the ray tensors.

    Returns (valid_idxs list[int64 array], cylinders (F,5) float32, bboxes list[(tl, br)])."""
    if cylinders is None:
        if kps is None:
            raise ValueError("need kps or cylinders")
        cylinders = bounding_cylinder(np.asarray(kps, dtype=np.float32), ext_scale)
    cylinders = np.asarray(cylinders, dtype=np.float32)
    n_pose = cylinders.shape[0]
    idxs, boxes = [], []
    for i, c2w in enumerate(c2ws):
        f = focal if isinstance(focal, float) else focal[i]
        h = H if isinstance(H, int) else int(H[i])
        w = W if isinstance(W, int) else int(W[i])
        center = None if centers is None else centers[i]
        tl, br = cylinder_box(cylinders[i % n_pose], h, w, f, np.asarray(c2w, dtype=np.float32), center)
        idxs.append(box_pixels(tl, br, w))
        boxes.append((tl, br))
    return idxs, cylinders, boxes


# float64 (cos, sin) of the 50 cap angles exactly as numpy computes them (cylinder_to_box_2d)
_CAP_ANGLES = np.linspace(0.0, 2 * np.pi, 50)
CAP_DIRS = np.ascontiguousarray(np.stack([np.cos(_CAP_ANGLES), np.sin(_CAP_ANGLES)], axis=-1))
_cap_dev = {}


def device_boxes(c2ws, H, W, focal, kps=None, cylinders=None, ext_scale=0.00035, centers=None, device=None):
    """valid_pixels with the cylinder and box computed on the GPU (anerf_kp_boxes).

    kps (P, NJ, 3) / cylinders (P, 5) may be device tensors (e.g. from kinematics.PoseOptLayer): they
    never leave the device; only the (F, 4) integer boxes come back.  The extrinsics
    inv(swap_mat(c2w)) are computed on the host with numpy, as the reference does (4x4 per camera).
    Returns (cylinders (P, 5) float32 device tensor, bboxes list[(tl, br)] int32 like valid_pixels)."""
    import torch
    from . import _lib
    if not isinstance(H, int) or not isinstance(W, int):
        raise NotImplementedError("device_boxes: one image size for all frames")
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    c2ws = np.asarray(c2ws, dtype=np.float32)
    F = c2ws.shape[0]
    w2cs = np.stack([_extrinsic_from_c2w(c) for c in c2ws]).astype(np.float32)
    fo = []
    for i in range(F):
        f = np.asarray(focal if isinstance(focal, float) else focal[i], dtype=np.float32).reshape(-1)
        fo.append((f[0], f[1] if f.size >= 2 else f[0]))
    focals = np.asarray(fo, dtype=np.float32)
    src = kps if kps is not None else cylinders
    if src is None:
        raise ValueError("need kps or cylinders")
    src = torch.as_tensor(src).to(device=dev, dtype=torch.float32).contiguous()
    n_kp = int(src.shape[0])
    nj = int(src.shape[1]) if kps is not None else 0
    if dev not in _cap_dev:
        _cap_dev[dev] = torch.from_numpy(CAP_DIRS).to(dev)
    cyl = torch.empty(n_kp, 5, device=dev, dtype=torch.float32)
    boxes = torch.empty(F, 4, device=dev, dtype=torch.int32)
    w2c_d = torch.from_numpy(w2cs).to(dev)
    foc_d = torch.from_numpy(focals).to(dev)
    cen_d = None
    if centers is not None:   # int(center[0]), int(center[1]) on the host, as cylinder_to_box_2d does
        offs = np.array([[int(c[0]), int(c[1])] for c in centers], dtype=np.int32)
        cen_d = torch.from_numpy(offs).to(dev)
    lib = _lib.load()
    with torch.cuda.device(dev):
        rc = lib.anerf_kp_boxes(_lib.ptr(src) if kps is not None else None, None if kps is not None else _lib.ptr(src),
                                n_kp, nj, 0, float(ext_scale), _lib.ptr(w2c_d), _lib.ptr(foc_d), _lib.ptr(cen_d), F,
                                H, W, _lib.ptr(_cap_dev[dev]), _lib.ptr(cyl), _lib.ptr(boxes), _lib.stream_handle(dev))
    _lib.check(rc, "anerf_kp_boxes")
    b = boxes.cpu().numpy()
    bboxes = [(b[i, :2].copy(), b[i, 2:].copy()) for i in range(F)]
    return cyl, bboxes

"""Training ray sampler of the image dataset on the device.

Mirrors core/dataset.py's BaseH5Dataset (:20-405), RandIntGenerator / RayImageSampler (:728-794)
and ray_collate_fn (:796-802) for the case the MI355X has room for: the whole dataset (uint8
images, foreground and sampling masks, backgrounds, cameras, poses) uploaded once and kept in HBM
(a 10 k-image 512x512 set is ~8 GB of the 288 GB).  Per batch the host draws the pixel indices
exactly as the reference does (same numpy calls in the same order, so a seeded run selects the same
pixels), and one launch of anerf_ray_batch builds every image's rays, target colours,
foreground and background values in ray_collate_fn's flattened layout.

Not mirrored: the subject / split / multiview sub-datasets (`_idx_map`, `_get_subset_idxs`,
`_load_multiview_pose`), the temporal-validity wrapper and h5 streaming (the arrays are read whole).
"""
import math

import numpy as np
import torch

from . import _lib
from .rays import cylinder_box


def _arr(data, key):
    return np.asarray(data[key][:])


class RayImageDataset:
    """BaseH5Dataset over HBM-resident arrays.

    data: the .h5 file's arrays (any mapping with the reference's keys: imgs (N, H*W, 3) uint8,
    masks and sampling_masks (N, H*W, 1), c2ws (N, 4, 4), focals (N,), kp3d, bones, skts, cyls,
    img_shape (4,), optional centers (N, 2), bkgds (B, H, W, 3) uint8 with bkgd_idxs (N,)); an
    open h5py.File works.  N_samples, patch_size, N_nms and mask_img mean what they mean in the
    reference (core/dataset.py:22-55).  nms_rng is the generator factory of _sample_in_box2d
    (the reference uses an unseeded np.random.default_rng(); a seeded factory makes it repeatable).
    """

    def __init__(self, data, N_samples=96, patch_size=1, N_nms=0, mask_img=False, device=None,
                 nms_rng=np.random.default_rng):
        self.device = torch.device("cuda", 0) if device is None else torch.device(device)
        self.N_samples = int(N_samples)
        self.patch_size = int(patch_size)
        self.N_nms = int(math.floor(N_nms)) if N_nms >= 1.0 else float(N_nms)
        self.mask_img = bool(mask_img)
        self.nms_rng = nms_rng
        keys = list(data.keys())
        self.has_bg = "bkgds" in keys
        img_shape = _arr(data, "img_shape")
        self._N_total_img = int(img_shape[0])
        self.HW = (int(img_shape[1]), int(img_shape[2]))
        H, W = self.HW
        self._pixel_idxs = np.arange(H * W).reshape(H, W)
        self.centers = _arr(data, "centers").astype(np.float32) if "centers" in keys else None
        self.kp3d, self.bones = _arr(data, "kp3d"), _arr(data, "bones")
        self.skts, self.cyls = _arr(data, "skts"), _arr(data, "cyls")
        self.focals = _arr(data, "focals")
        self.c2ws = _arr(data, "c2ws")
        self.sampling_masks = _arr(data, "sampling_masks").reshape(-1, H * W)
        imgs = _arr(data, "imgs")
        self.data_len = len(imgs)
        dev = self.device

        def up(x, dtype):
            return torch.as_tensor(np.ascontiguousarray(x, dtype=dtype)).to(dev)

        if imgs.dtype != np.uint8:
            raise ValueError("imgs must be uint8 (the .h5 layout)")
        self._imgs = up(imgs.reshape(-1, H * W, 3), np.uint8)
        self._masks = up(_arr(data, "masks").reshape(-1, H * W), np.uint8)
        self._c2ws = up(self.c2ws.reshape(-1, 16), np.float32)
        self._focals = up(self.focals.reshape(-1), np.float32)
        self._centers = None if self.centers is None else up(self.centers.reshape(-1, 2), np.float32)
        self._bgs = self._bg_idxs = None
        if self.has_bg:
            self._bgs = up(_arr(data, "bkgds").reshape(-1, H * W, 3), np.uint8)
            self.bg_idxs = _arr(data, "bkgd_idxs").astype(np.int64)
            self._bg_idxs = up(self.bg_idxs, np.int64)
        self._pose = {k: up(v, np.float32) for k, v in
                      (("kp3d", self.kp3d), ("bones", self.bones), ("skts", self.skts), ("cyls", self.cyls))}
        self._bad = torch.zeros(1, dtype=torch.int32, device=dev)
        self.box2d = None
        if self.N_nms > 0.0:
            self.init_box2d()

    def __len__(self):
        return self.data_len

    # ---- host side: which pixels (numpy RNG, as the reference draws them) ----

    def init_box2d(self):
        """Per-image 2-D box of the cylinder, scale 1.3 (core/dataset.py:207-236)."""
        H, W = self.HW
        boxes = []
        for i in range(self.data_len):
            center = None if self.centers is None else self.centers[i]
            tl, br = cylinder_box(self.cyls[i].astype(np.float32), H, W, self.focals[i],
                                  self.c2ws[i].astype(np.float32), center=center, scale=1.3)
            boxes.append((tl, br))
        self.box2d = np.array(boxes)

    def sample_pixels(self, idx, q_idx):
        """Sorted pixel indices of one image (core/dataset.py:277-323)."""
        p = self.patch_size
        N_rand = self.N_samples // int(p ** 2)
        sampling_mask = self.sampling_masks[idx]
        valid_idxs, = np.where(sampling_mask > 0)
        sampled_idxs = np.random.choice(valid_idxs, N_rand, replace=False)
        if p > 1:
            H, W = self.HW
            hs = np.clip(sampled_idxs // W, 0, H - p)
            ws = np.clip(sampled_idxs % W, 0, W - p)
            sampled_idxs = np.stack([self._pixel_idxs[h:h + p, w:w + p].reshape(-1)
                                     for h, w in zip(hs, ws)]).reshape(-1)
        if isinstance(self.N_nms, int):
            N_nms = self.N_nms
        else:
            N_nms = int(self.N_nms > np.random.random())
        if N_nms > 0:
            nms_idxs = self._sample_in_box2d(idx, q_idx, sampling_mask, N_nms)
            sampled_idxs = np.sort(sampled_idxs)
            sampled_idxs[np.random.choice(len(sampled_idxs), size=(N_nms,), replace=False)] = nms_idxs
        return np.sort(sampled_idxs)

    def _sample_in_box2d(self, idx, q_idx, fg, N_samples):
        """Out-of-mask pixels inside the image's box (core/dataset.py:325-344)."""
        H, W = self.HW
        tl, br = self.box2d[idx].copy()
        cropped = fg.reshape(H, W)[tl[1]:br[1], tl[0]:br[0]]
        vy, vx = np.where(cropped < 1)
        idxs = (vy + tl[1]) * W + (vx + tl[0])
        return self.nms_rng().choice(idxs, size=(N_samples,), replace=False)

    # ---- device side: the batch ----

    def __getitem__(self, q_idx):
        """One image's rays (core/dataset.py:57-105), as device tensors."""
        return self.get_batch([q_idx])

    def get_batch(self, q_idxs):
        """The rays of several images in ray_collate_fn's flattened layout (core/dataset.py:796-802):
        rays_o, rays_d, target_s, fgs, bgs (n, ...), rays (2, n, 3), kp_idx, cam_idxs (n,) int64 and
        the per-ray kp3d, bones, skts, cyls of each image, n = len(q_idxs) * pixels per image."""
        q = np.asarray(q_idxs, dtype=np.int64).reshape(-1)
        if q.size and (q.min() < 0 or q.max() >= self.data_len):
            raise IndexError("dataset index out of range")
        pix = np.stack([self.sample_pixels(int(i), int(i)) for i in q]) if q.size else np.zeros((0, 0), np.int64)
        return self.gather(q, pix)

    def gather(self, rows, pixels):
        """anerf_ray_batch for given rows (n_img,) and sorted pixel indices (n_img, n_per)."""
        rows = np.asarray(rows, dtype=np.int64).reshape(-1)
        pixels = np.ascontiguousarray(pixels, dtype=np.int64)
        if pixels.ndim != 2 or pixels.shape[0] != len(rows):
            raise ValueError("pixels must be (n_img, n_per), one row per image")
        n_img, n_per = pixels.shape
        n = n_img * n_per
        dev = self.device
        if dev.type != "cuda":
            raise RuntimeError("RayImageDataset.gather runs anerf_ray_batch on a GPU device (no CPU path)")
        rows_d = torch.as_tensor(rows).to(dev)
        pix_d = torch.as_tensor(pixels).to(dev)
        rays = torch.empty(2, n, 3, dtype=torch.float32, device=dev)
        target = torch.empty(n, 3, dtype=torch.float32, device=dev)
        fg = torch.empty(n, 1, dtype=torch.float32, device=dev)
        bg = torch.empty(n, 3, dtype=torch.float32, device=dev) if self.has_bg else None
        self._bad.zero_()
        H, W = self.HW
        lib = _lib.load()
        with torch.cuda.device(dev):
            rc = lib.anerf_ray_batch(_lib.ptr(self._imgs), _lib.ptr(self._masks), _lib.ptr(self._bgs),
                                     _lib.ptr(self._bg_idxs), _lib.ptr(self._c2ws), _lib.ptr(self._focals),
                                     _lib.ptr(self._centers), self.data_len,
                                     0 if self._bgs is None else int(self._bgs.shape[0]), H, W,
                                     _lib.ptr(rows_d), n_img, _lib.ptr(pix_d), n_per,
                                     int(self.mask_img and self.has_bg), _lib.ptr(rays), _lib.ptr(target),
                                     _lib.ptr(fg), _lib.ptr(bg), _lib.ptr(self._bad), _lib.stream_handle(dev))
        _lib.check(rc, "anerf_ray_batch")
        if int(self._bad.item()):
            raise IndexError("anerf_ray_batch: pixel, row or background index out of range")
        rep = rows_d.repeat_interleave(n_per)
        out = {"rays_o": rays[0], "rays_d": rays[1], "target_s": target, "fgs": fg, "bgs": bg,
               "kp_idx": rep, "cam_idxs": rep.clone(), "rays": rays}
        # every ray carries its image's pose rows (core/dataset.py:96-104): one anerf_gather_rows each
        with torch.cuda.device(dev):
            for k, v in self._pose.items():
                dst = torch.empty((n,) + tuple(v.shape[1:]), dtype=torch.float32, device=dev)
                width = int(v[0].numel()) if v.shape[0] else 0
                rc = lib.anerf_gather_rows(_lib.ptr(v), width, int(v.shape[0]), _lib.ptr(rows_d), n_img, n_per,
                                           _lib.ptr(dst), None, _lib.stream_handle(dev))
                _lib.check(rc, "anerf_gather_rows")
                out[k] = dst
        return out


class RandIntGenerator:
    """Every index once per n draws: torch.randperm epochs (core/dataset.py:728-752)."""

    def __init__(self, n, generator=None):
        self._n = n
        self.generator = generator

    def __iter__(self):
        generator = self.generator
        if generator is None:
            generator = torch.Generator(device=torch.tensor(0.).device)
            generator.manual_seed(int(torch.empty((), dtype=torch.int64).random_().item()))
        yield from torch.randperm(self._n, generator=generator)

    def __len__(self):
        return self._n


class RayImageSampler:
    """Batches of N_images sorted image indices (core/dataset.py:754-794); feed each batch to
    RayImageDataset.get_batch."""

    def __init__(self, data_source, N_images=1024, N_iter=None, generator=None):
        self.data_source = data_source
        self.N_images = N_images
        self._N_iter = len(data_source) if N_iter is None else N_iter
        self.generator = generator
        self.sampler = RandIntGenerator(n=len(data_source))

    def __iter__(self):
        it = iter(self.sampler)
        for _ in range(self._N_iter):
            batch = []
            while len(batch) < self.N_images:
                try:
                    idx = next(it)
                except StopIteration:
                    it = iter(self.sampler)
                    idx = next(it)
                batch.append(idx.item())
            yield np.sort(batch)

    def __len__(self):
        return self._N_iter

"""Time the image dataset's ray batch (anerf_ray_batch via RayImageDataset.gather) on the device
against the reference's host-side arithmetic (the numpy restatement in oracle/ray_batch.py, the
same float32 numpy calls as core/dataset.py:259-275, 346-364).  Prints one JSON line."""
import importlib
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _ablib  # noqa: E402,F401  (ANERF_LIB_PATH: an experiment build, A/B tooling only)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import ray_batch as odata  # noqa: E402

dmod = importlib.import_module("a-nerf_amd.dataset")


def main():
    rs = np.random.RandomState(0)
    n, H, W, n_img, n_per = 256, 512, 512, 128, 3072
    c2w = np.tile(np.eye(4, dtype=np.float32), (n, 1, 1))
    c2w[:, :3, 3] = rs.normal(size=(n, 3))
    c2w[:, 0, 2] = 0.3
    data = dict(imgs=rs.randint(0, 256, (n, H * W, 3)).astype(np.uint8),
                masks=(rs.uniform(size=(n, H * W, 1)) < 0.5).astype(np.uint8),
                sampling_masks=np.ones((n, H * W, 1), np.uint8), c2ws=c2w,
                focals=np.full(n, 700.0, np.float32), bkgds=rs.randint(0, 256, (8, H, W, 3)).astype(np.uint8),
                bkgd_idxs=rs.randint(0, 8, n), kp3d=np.zeros((n, 24, 3), np.float32),
                bones=np.zeros((n, 24, 3), np.float32), skts=np.zeros((n, 24, 4, 4), np.float32),
                cyls=np.zeros((n, 5), np.float32), img_shape=np.array([n, H, W, 3]))
    ds = dmod.RayImageDataset(data, N_samples=n_per, mask_img=True)
    rows = np.sort(rs.choice(n, n_img, replace=False))
    pix = np.sort(np.stack([rs.choice(H * W, n_per, replace=False) for _ in rows]), axis=1)
    for _ in range(5):
        ds.gather(rows, pix)
    torch.cuda.synchronize()
    K = 50
    t0 = time.perf_counter()
    for _ in range(K):
        ds.gather(rows, pix)
    torch.cuda.synchronize()
    dev_ms = (time.perf_counter() - t0) / K * 1e3
    t0 = time.perf_counter()
    odata.ray_batch(data, rows, pix, mask_img=True)
    cpu_ms = (time.perf_counter() - t0) * 1e3
    rays = n_img * n_per
    print(json.dumps({"what": "RayImageDataset.gather (anerf_ray_batch + pose gathers, host call incl.)",
                      "images": n_img, "rays": rays, "device_ms": round(dev_ms, 3),
                      "device_rays_per_s": round(rays / dev_ms * 1e3), "cpu_numpy_ms_1thread": round(cpu_ms, 1),
                      "cpu_rays_per_s": round(rays / cpu_ms * 1e3)}))


if __name__ == "__main__":
    main()

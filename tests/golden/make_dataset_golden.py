"""Generate tests/golden/raybatch.npz by running the REFERENCE's image dataset (core/dataset.py).

Runs ONLY in the build container, where /root/reference exists.  core.dataset.BaseH5Dataset reads
an .h5 file through h5py (absent here, stubbed by make_golden.import_reference); this script hands
it an in-memory stand-in for h5py.File holding a small synthetic dataset, so the reference's own
init_meta / init_box2d / sample_pixels / get_rays / get_img_data / __getitem__ run unchanged.
Stored per case: the dataset arrays (inputs), the numpy seed, the images queried, every
__getitem__ output, and the pixel indices (sample_pixels re-run under the same seed; the
reference does not return them).

Usage:  python tests/golden/make_dataset_golden.py
"""
import importlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden  # noqa: E402

syn = make_golden.anerf_syn
rays = importlib.import_module("a-nerf_amd.rays")


class _H5(dict):
    """What BaseH5Dataset uses of an h5py.File: keys(), [key][...], `in`, close, context manager."""

    def close(self):
        pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def synthetic_data(seed, H, W, n_img, centers, bg, near_identity):
    rs = np.random.RandomState(seed)
    sc = syn.make_scene(n_joints=24, H=H, W=W, seed=seed, n_frames=n_img, yaw_step=0.5)
    c2ws = sc["c2ws"].astype(np.float32)
    if near_identity:
        # camera 0: rotation within np.isclose of I (the reference skips the rotation), camera 1: exact I
        # (isclose: |a - b| <= 1e-8 + 1e-5 |b|, so 3e-6 on the diagonal, 5e-9 off it)
        eps = np.where(np.eye(3) > 0, 3e-6, 5e-9) * rs.uniform(-1, 1, (3, 3))
        c2ws[0, :3, :3] = (np.eye(3) + eps).astype(np.float32)
        c2ws[1, :3, :3] = np.eye(3, dtype=np.float32)
    cyls = rays.bounding_cylinder(sc["kps"], 0.001).astype(np.float32)
    fg = (rs.uniform(size=(n_img, H * W, 1)) < 0.6).astype(np.uint8)
    samp = (rs.uniform(size=(n_img, H * W, 1)) < 0.7).astype(np.uint8)
    d = _H5(imgs=rs.randint(0, 256, size=(n_img, H * W, 3)).astype(np.uint8), masks=fg, sampling_masks=samp,
            c2ws=c2ws, focals=(1.5 * H + rs.uniform(-3, 3, n_img)).astype(np.float32),
            kp3d=sc["kps"].astype(np.float32), bones=sc["bones"].astype(np.float32),
            skts=sc["skts"].astype(np.float32), cyls=cyls, img_shape=np.array([n_img, H, W, 3]))
    if centers:
        d["centers"] = np.stack([W * 0.5 + rs.uniform(-4, 4, n_img), H * 0.5 + rs.uniform(-4, 4, n_img)],
                                axis=-1).astype(np.float32)
    if bg:
        d["bkgds"] = rs.randint(0, 256, size=(3, H, W, 3)).astype(np.uint8)
        d["bkgd_idxs"] = rs.randint(0, 3, size=n_img).astype(np.int64)
    return d


CASES = {
    # name: (data kwargs, dataset kwargs, queried images)
    "plain": (dict(seed=1, H=24, W=32, n_img=5, centers=False, bg=False, near_identity=True),
              dict(N_samples=40), [3, 0, 4, 1]),
    "centers_bg_maskimg": (dict(seed=2, H=20, W=28, n_img=4, centers=True, bg=True, near_identity=False),
                           dict(N_samples=36, mask_img=True), [2, 3, 0]),
    "patch2_bg": (dict(seed=3, H=24, W=24, n_img=4, centers=False, bg=True, near_identity=False),
                  dict(N_samples=32, patch_size=2), [1, 2]),
    "nms3": (dict(seed=4, H=32, W=32, n_img=4, centers=True, bg=True, near_identity=False),
             dict(N_samples=48, N_nms=3), [0, 2, 3]),
}
NMS_SEED = 77


def main():
    mods = make_golden.import_reference()  # noqa: F841  (stubs + sys.path)
    h5py = sys.modules["h5py"]
    ds_mod = importlib.import_module("core.dataset")
    rows = {}
    for name, (dk, kw, queries) in CASES.items():
        data = synthetic_data(**dk)
        h5py.File = lambda *a, **k: data
        ds = ds_mod.BaseH5Dataset("synthetic.h5", **kw)
        # _sample_in_box2d draws from an unseeded np.random.default_rng(); seed it for the fixture
        real_default_rng = np.random.default_rng
        np.random.default_rng = lambda *a: real_default_rng(NMS_SEED)
        try:
            np.random.seed(1000 + dk["seed"])
            outs = [ds[q] for q in queries]
            np.random.seed(1000 + dk["seed"])
            pix = [ds.sample_pixels(q, q) for q in queries]
        finally:
            np.random.default_rng = real_default_rng
        for k, v in data.items():
            rows[f"{name}/in/{k}"] = v
        rows[f"{name}/queries"] = np.array(queries)
        rows[f"{name}/kwargs"] = np.array(repr(kw))
        rows[f"{name}/np_seed"] = np.array(1000 + dk["seed"])
        rows[f"{name}/pixels"] = np.stack(pix)
        if ds.box2d is not None:
            rows[f"{name}/box2d"] = np.asarray(ds.box2d)
        for k in ("rays_o", "rays_d", "target_s", "fgs", "bgs", "kp_idx", "kp3d", "cam_idxs"):
            if outs[0][k] is not None:
                rows[f"{name}/out/{k}"] = np.concatenate([o[k] for o in outs])
    path = os.path.join(HERE, "raybatch.npz")
    np.savez_compressed(path, **rows)
    print(f"wrote {path}: {len(rows)} arrays")


if __name__ == "__main__":
    main()

"""GPU: anerf_ray_batch (the image dataset's ray sampler) through
a-nerf_amd/dataset.py, against the oracle (bit-exact) and the reference's own outputs
(tests/golden/raybatch.npz)."""
import ast
import importlib
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import ray_batch as odata  # noqa: E402

pytestmark = pytest.mark.gpu
dmod = importlib.import_module("a-nerf_amd.dataset")
G = np.load(os.path.join(HERE, "golden", "raybatch.npz"))
CASES = sorted({k.split("/")[0] for k in G.files})


def case(name):
    data = {k.split("/", 2)[2]: G[k] for k in G.files if k.startswith(name + "/in/")}
    return data, ast.literal_eval(str(G[name + "/kwargs"])), G[name + "/queries"], G[name + "/pixels"]


def _np(t):
    return None if t is None else t.detach().cpu().numpy()


@pytest.mark.parametrize("name", CASES)
def test_ray_batch_vs_reference(name):
    data, kw, q, pix = case(name)
    ds = dmod.RayImageDataset(data, nms_rng=lambda: np.random.default_rng(77), **kw)
    np.random.seed(int(G[name + "/np_seed"]))
    out = ds.get_batch(q)
    ref = odata.ray_batch(data, q, pix, mask_img=kw.get("mask_img", False))
    for k in ("rays_o", "rays_d", "target_s", "fgs", "bgs"):
        if ref[k] is None:
            assert out[k] is None
            continue
        np.testing.assert_array_equal(_np(out[k]), ref[k], err_msg=k)        # bit-exact vs the oracle
        g = G[f"{name}/out/{k}"]
        np.testing.assert_allclose(_np(out[k]), g, rtol=0, atol=2.5e-7, err_msg=k)  # the reference
    for k in ("kp_idx", "cam_idxs", "kp3d"):
        np.testing.assert_array_equal(_np(out[k]), G[f"{name}/out/{k}"], err_msg=k)
    np.testing.assert_array_equal(_np(out["rays"][0]), _np(out["rays_o"]))
    assert out["skts"].shape == (len(q) * pix.shape[1], 24, 4, 4)
    rep = np.repeat(np.asarray(q), pix.shape[1])
    for k in ("kp3d", "bones", "skts", "cyls"):  # anerf_gather_rows: each ray carries its image's rows
        np.testing.assert_array_equal(_np(out[k]), np.asarray(data[k], np.float32)[rep], err_msg=k)


def test_ray_batch_full_size_vs_oracle():
    """64 images of 512x512, 3072 pixels each (a training batch of the SURREAL configs), with
    per-image centers, backgrounds and mask_img: bit-exact against the oracle."""
    rs = np.random.RandomState(5)
    n, H, W = 64, 512, 512
    c2w = np.tile(np.eye(4, dtype=np.float32), (n, 1, 1))
    for i in range(n):
        a = 0.1 * i
        c2w[i, :3, :3] = [[np.cos(a), 0, np.sin(a)], [0, 1, 0], [-np.sin(a), 0, np.cos(a)]]
        c2w[i, :3, 3] = rs.normal(size=3)
    data = dict(imgs=rs.randint(0, 256, (n, H * W, 3)).astype(np.uint8),
                masks=(rs.uniform(size=(n, H * W, 1)) < 0.5).astype(np.uint8),
                sampling_masks=np.ones((n, H * W, 1), np.uint8), c2ws=c2w,
                focals=rs.uniform(500, 900, n).astype(np.float32),
                centers=rs.uniform(200, 300, (n, 2)).astype(np.float32),
                bkgds=rs.randint(0, 256, (4, H, W, 3)).astype(np.uint8), bkgd_idxs=rs.randint(0, 4, n),
                kp3d=rs.normal(size=(n, 24, 3)).astype(np.float32), bones=np.zeros((n, 24, 3), np.float32),
                skts=np.tile(np.eye(4, dtype=np.float32), (n, 24, 1, 1)), cyls=np.zeros((n, 5), np.float32),
                img_shape=np.array([n, H, W, 3]))
    ds = dmod.RayImageDataset(data, N_samples=3072, mask_img=True)
    np.random.seed(9)
    q = np.sort(rs.choice(n, 48, replace=False))
    out = ds.get_batch(q)
    np.random.seed(9)
    pix = np.stack([ds.sample_pixels(int(i), int(i)) for i in q])
    ref = odata.ray_batch(data, q, pix, mask_img=True)
    for k in ("rays_o", "rays_d", "target_s", "fgs", "bgs"):
        np.testing.assert_array_equal(_np(out[k]), ref[k], err_msg=k)
    rep = np.repeat(q, 3072)
    for k in ("kp3d", "bones", "skts", "cyls"):  # float4 rows (kp3d, bones, skts) and 5-float rows (cyls)
        np.testing.assert_array_equal(_np(out[k]), data[k][rep], err_msg=k)


def test_ray_batch_rejects_out_of_range():
    data, kw, q, pix = case("plain")
    ds = dmod.RayImageDataset(data, **kw)
    bad = pix.copy()
    bad[0, 0] = 24 * 32
    with pytest.raises(IndexError):
        ds.gather(q, bad)
    with pytest.raises(IndexError):
        ds.gather(np.array([0, 7, 1, 2]), pix)
    with pytest.raises(IndexError):
        ds.get_batch([5])
    ok = ds.gather(q, pix)           # the flag is reset per call
    assert torch.isfinite(ok["rays_d"]).all()


def test_ray_batch_empty():
    data, kw, q, pix = case("plain")
    ds = dmod.RayImageDataset(data, **kw)
    out = ds.get_batch([])
    assert out["rays_o"].shape == (0, 3) and out["target_s"].shape == (0, 3)


def test_gather_rows_out_of_range_rows_are_nan_and_flagged():
    lib = importlib.import_module("a-nerf_amd._lib")
    L = lib.load()
    src = torch.arange(3 * 8, dtype=torch.float32, device="cuda").reshape(3, 8)
    for width, s in ((8, src), (5, src[:, :5].contiguous())):
        rows = torch.tensor([2, 3, 0], dtype=torch.int64, device="cuda")
        dst = torch.empty(6, width, device="cuda")
        bad = torch.zeros(1, dtype=torch.int32, device="cuda")
        rc = L.anerf_gather_rows(lib.ptr(s), width, 3, lib.ptr(rows), 3, 2, lib.ptr(dst), lib.ptr(bad),
                                 lib.stream_handle(torch.device("cuda", 0)))
        lib.check(rc, "anerf_gather_rows")
        torch.cuda.synchronize()
        assert int(bad.item()) == 1
        assert torch.isnan(dst[2:4]).all()
        torch.testing.assert_close(dst[0:2], s[2].expand(2, -1), rtol=0, atol=0)
        torch.testing.assert_close(dst[4:6], s[0].expand(2, -1), rtol=0, atol=0)

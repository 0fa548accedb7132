"""Full-size frames on the GPU against the CPU oracle.

* Configs 3 and 4 (512^2, 64 + 128 samples, 24 / 65 joints, 8x256): a whole frame rendered in
  4096-ray chunks; >= 8,192 evenly spaced rays of it compared with the oracle at 1e-4 (the oracle
  gets the frame's own near / far, i.e. the chunk NaN fill of the whole frame, hazard H1).
* Config 5 (1024^2): the north star's multi-GPU split — the ray list cut into
  distributed.chunk_ranges(n, 4096, 8) shards rendered separately and concatenated — is bit-identical
  to the whole-frame render in the bf16x6, fp16x4, fp16x3 and fp32 precisions (and so is bench.py's
  N > 1 split, 256-ray tiles dealt round-robin with near / far from the whole frame), and 20,000 evenly spaced rays
  (the bench's parity sample) match the oracle at 1e-4 (near-empty rays' disparity, H12: counted and
  bounded, see _oracle_check).  (The RCCL all-gather itself is covered by tests/test_distributed.py over gloo.)
The oracle is pinned to the reference's golden fixtures (tests/test_oracle_golden.py).
"""
import importlib
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))

pytestmark = pytest.mark.gpu

anerf = importlib.import_module("a-nerf_amd")
syn = importlib.import_module("a-nerf_amd.synthetic")
dmod = importlib.import_module("a-nerf_amd.distributed")
_lib = importlib.import_module("a-nerf_amd._lib")

TOL = 1e-4


@pytest.fixture(scope="module", autouse=True)
def _cuda():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _frame(H, nj, seed, tau):
    sc = syn.make_scene(n_joints=nj, H=H, W=H, seed=seed)
    ck = syn.make_checkpoint(seed, n_joints=nj, D=8, W=256, fine=True, tau=tau)
    idx, cyls, boxes = anerf.rays.valid_pixels(sc["c2ws"], H, H, sc["focal"], kps=sc["kps"], ext_scale=0.001)
    (x0, y0), (x1, y1) = (int(v) for v in boxes[0][0]), (int(v) for v in boxes[0][1])
    n = (x1 - x0) * (y1 - y0)
    assert n == len(idx[0])
    c2w = torch.from_numpy(np.ascontiguousarray(sc["c2ws"][0][:3, :4])).cuda()
    rb = torch.empty(n, 11, device="cuda")
    _lib.check(_lib.load().anerf_gen_rays_box(_lib.ptr(c2w), H, H, sc["focal"], sc["focal"], 0.0, 0.0, 0, x0, y0, x1,
                                              y1, 0.0, 1.0, _lib.ptr(rb), _lib.stream_handle()), "gen_rays_box")
    torch.cuda.synchronize()
    return sc, ck, cyls, rb


def _render(rc, rb, sc, cyls):
    n = rb.shape[0]
    sk = torch.from_numpy(sc["skts"][0:1]).cuda().expand(n, -1, -1, -1)
    cy = torch.from_numpy(cyls[0:1]).cuda().expand(n, -1)
    return rc.render_rays(rb, 64, skts=sk, cyls=cy, N_importance=128, chunk=4096, ret_alpha=False)


def _oracle_check(cfg, ck, sc, cyls, rb, out, n_sample):
    """n_sample evenly spaced rays of the frame against the oracle at 1e-4, every output of every ray
    except the disparity of near-empty rays (0 < acc < 2^-20, hazard H12): those are held to 1e-4 plus
    the reference's own measured spread on such rays (oracle.h12_spread: the reference's float32 disp vs
    its float64 disp on config 5's 169 near-empty rays, 1.92e-4), and reported;
    test_near_empty_rays_against_the_reference pins all 169 against the reference itself, ray by ray."""
    import oracle
    ne_tol = TOL + oracle.h12_spread()["float64"]
    om = oracle.OracleModel(cfg, ck)
    rb_h = rb.cpu().numpy()
    near, far, _, _ = om.near_far(rb_h, cyls[0:1], chunk=4096)
    sel = np.linspace(0, rb_h.shape[0] - 1, n_sample).astype(np.int64)
    ref = om.render_rays(rb_h[sel], sc["skts"][0], cyls[0:1], chunk=4096, near=near[sel], far=far[sel])
    report = {}
    for k in ("rgb_map", "disp_map", "acc_map", "rgb0", "disp0", "acc0"):
        got = out[k].cpu().numpy()[sel]
        d = np.abs(got.astype(np.float64) - ref[k]).reshape(n_sample, -1).max(-1)
        acc_k = ref["acc_map" if k in ("rgb_map", "disp_map", "acc_map") else "acc0"]
        empty = (acc_k > 0) & (acc_k < 2.0 ** -20) if k.startswith("disp") else np.zeros(n_sample, bool)
        strict = float(d[~empty].max())
        assert strict <= TOL, f"{k}: max |gpu - oracle| = {strict:.3e} over {n_sample} rays"
        if empty.any():
            ne = float(d[empty].max())
            report[k] = (int(empty.sum()), ne)
            assert ne <= ne_tol, (k, int(empty.sum()), ne, ne_tol)
    print(f"near-empty rays (count, max disp error): {report}")


@pytest.mark.parametrize("nj,precision", [(24, "bf16x6"), (24, "fp16x4"), (24, "fp16x3"), (24, "fp32"), (65, "fp16x3"),
                                          (65, "bf16x6"), (65, "fp16x4")])
def test_full_frame_matches_oracle_on_8192_rays(nj, precision):
    seed = 13 if nj == 24 else 14
    sc, ck, cyls, rb = _frame(512, nj, seed, 79.6 if nj == 24 else 20.0)
    cfg = anerf.RenderConfig(n_joints=nj, N_samples=64, N_importance=128, precision=precision).validate()
    rc = anerf.RayCaster(cfg, ck)
    out = _render(rc, rb, sc, cyls)
    torch.cuda.synchronize()
    _oracle_check(cfg, ck, sc, cyls, rb, out, 8192)


@pytest.mark.parametrize("W,precision", [(256, "bf16x6"), (128, "bf16x6"), (256, "fp16x4"), (256, "fp16x3"), (128, "fp16x3")])
def test_multires10_split_modes_match_oracle(W, precision):
    """--multires 10 at widths 128 / 256 in the split modes: the windowed k-streams run as bf16x6 with
    two k16-steps per joint (10 sin / cos terms + the distance input per lane half; v_part_x6), and
    at W = 128 four groups per joint (three sincos terms per group).  The reference's fixture with
    multires 10 (v1_mr10_w64_d4) is at width 64, which stays on f32 MFMAs; this pins the split path
    against the oracle (itself pinned to v1) on 2,048 rays of a 512^2 frame at tau 20."""
    seed = 17
    sc = syn.make_scene(n_joints=24, H=512, W=512, seed=seed)
    ck = syn.make_checkpoint(seed, n_joints=24, D=8, W=W, fine=True, tau=20.0, multires=10)
    idx, cyls, boxes = anerf.rays.valid_pixels(sc["c2ws"], 512, 512, sc["focal"], kps=sc["kps"], ext_scale=0.001)
    (x0, y0), (x1, y1) = (int(v) for v in boxes[0][0]), (int(v) for v in boxes[0][1])
    n = (x1 - x0) * (y1 - y0)
    c2w = torch.from_numpy(np.ascontiguousarray(sc["c2ws"][0][:3, :4])).cuda()
    rb = torch.empty(n, 11, device="cuda")
    _lib.check(_lib.load().anerf_gen_rays_box(_lib.ptr(c2w), 512, 512, sc["focal"], sc["focal"], 0.0, 0.0, 0, x0, y0,
                                              x1, y1, 0.0, 1.0, _lib.ptr(rb), _lib.stream_handle()), "gen_rays_box")
    cfg = anerf.RenderConfig(n_joints=24, netwidth=W, multires=10, N_samples=64, N_importance=128,
                             precision=precision).validate()
    out = _render(anerf.RayCaster(cfg, ck), rb, sc, cyls)
    torch.cuda.synchronize()
    _oracle_check(cfg, ck, sc, cyls, rb, out, 2048)


@pytest.mark.parametrize("precision", ["bf16x6", "fp16x4", "fp16x3", "fp32"])
def test_config5_pixel_shards_are_bit_identical(precision):
    sc, ck, cyls, rb = _frame(1024, 24, 13, 79.6)
    n = rb.shape[0]
    assert n > 700_000
    cfg = anerf.RenderConfig(N_samples=64, N_importance=128, precision=precision).validate()
    rc = anerf.RayCaster(cfg, ck)
    whole = _render(rc, rb, sc, cyls)
    parts = [_render(rc, rb[s0:s1], sc, cyls) for s0, s1 in dmod.chunk_ranges(n, 4096, 8)]
    torch.cuda.synchronize()
    for k in ("rgb_map", "disp_map", "acc_map", "rgb0", "disp0", "acc0"):
        assert torch.equal(torch.cat([p[k] for p in parts], 0), whole[k]), k
    _oracle_check(cfg, ck, sc, cyls, rb, whole, 20000)


def test_config5_ray_balanced_shards_are_bit_identical():
    """Ray-balanced pixel sharding (distributed.ray_ranges, what bench.py runs at N > 1): each of 8
    ranks fills near / far over the whole chunks covering its equal share (raycaster.near_far) and
    renders its rays with them (ANERF_FLAG_NEAR_FAR); the concatenation equals the whole frame."""
    near_far = importlib.import_module("a-nerf_amd.raycaster").near_far
    sc, ck, cyls, rb = _frame(1024, 24, 13, 79.6)
    n = rb.shape[0]
    cfg = anerf.RenderConfig(N_samples=64, N_importance=128, precision="bf16x6").validate()
    rc = anerf.RayCaster(cfg, ck)
    whole = _render(rc, rb, sc, cyls)
    cy = torch.from_numpy(cyls[0:1]).cuda()
    sk = torch.from_numpy(sc["skts"][0:1]).cuda()
    parts = []
    for s0, s1 in dmod.ray_ranges(n, 8):
        c0, c1 = dmod.chunk_cover(s0, s1, 4096, n)
        cover = rb[c0:c1].clone()
        near_far(cover, cy, chunk=4096, out=(cover[:, 6], cover[:, 7]))
        mine = cover[s0 - c0:s1 - c0]
        m = mine.shape[0]
        parts.append(rc.render_rays(mine, 64, skts=sk.expand(m, -1, -1, -1), cyls=cy.expand(m, -1), N_importance=128,
                                    chunk=4096, ret_alpha=False, near_far_given=True))
    torch.cuda.synchronize()
    assert max(s1 - s0 for s0, s1 in dmod.ray_ranges(n, 8)) - min(s1 - s0 for s0, s1 in dmod.ray_ranges(n, 8)) <= 1
    for k in ("rgb_map", "disp_map", "acc_map", "rgb0", "disp0", "acc0"):
        assert torch.equal(torch.cat([p[k] for p in parts], 0), whole[k]), k


@pytest.mark.parametrize("precision", ["fp16x4", "bf16x6"])
def test_config5_tile_shards_are_bit_identical(precision):
    """The split bench.py runs at N > 1 (distributed.tile_rows: 256-ray tiles dealt round-robin over 8
    ranks, near / far from the whole frame's 4096-ray chunks, ANERF_FLAG_NEAR_FAR): every rank's rays
    rendered on their own and put back in frame order equal the whole-frame render bit for bit."""
    near_far = importlib.import_module("a-nerf_amd.raycaster").near_far
    sc, ck, cyls, rb = _frame(1024, 24, 13, 79.6)
    n = rb.shape[0]
    cfg = anerf.RenderConfig(N_samples=64, N_importance=128, precision=precision).validate()
    rc = anerf.RayCaster(cfg, ck)
    whole = _render(rc, rb, sc, cyls)
    cy = torch.from_numpy(cyls[0:1]).cuda()
    sk = torch.from_numpy(sc["skts"][0:1]).cuda()
    rbn = rb.clone()
    near_far(rbn, cy, chunk=4096, out=(rbn[:, 6], rbn[:, 7]))
    got = {k: torch.full_like(v, float("nan")) for k, v in whole.items()}
    seen = torch.zeros(n, dtype=torch.int32)
    for r in range(8):
        rows = dmod.tile_rows(n, 8, r, 256)
        seen[rows] += 1
        mine = rbn[rows.cuda()]
        m = mine.shape[0]
        out = rc.render_rays(mine, 64, skts=sk.expand(m, -1, -1, -1), cyls=cy.expand(m, -1), N_importance=128,
                             chunk=4096, ret_alpha=False, near_far_given=True)
        for k in got:
            got[k][rows.cuda()] = out[k]
    torch.cuda.synchronize()
    assert bool((seen == 1).all())
    for k in ("rgb_map", "disp_map", "acc_map", "rgb0", "disp0", "acc0"):
        assert torch.equal(got[k].nan_to_num(7.0), whole[k].nan_to_num(7.0)), k


@pytest.mark.parametrize("precision", ["fp32", "bf16x6", "fp16x4", "fp16x3"])
def test_near_empty_rays_against_the_reference(precision):
    """Hazard H12 against the REFERENCE (tests/golden/h12_nearempty_c5.npz: config 5's near-empty rays,
    0 < acc < 2^-20, and 64 ordinary rays, rendered by core.raycasters.render_rays with the frame's
    own near / far): every output of the ordinary rays and rgb / acc / the coarse outputs of the
    near-empty rays within 1e-4.  Their disp = (acc + 1e-10) / depth is a ratio of a few 2^-24 alpha
    quanta.  tests/golden/h12_spread_c5.npz holds the reference's own spread on these rays:
    its disp does not move with the thread count, but its float64 run differs from its float32 one by
    up to 1.92e-4 (2 rays above 1e-4) -- every quantum is rounded from a sigma * delta that the
    float32 MLP only knows to ~1e-6 relative, and torch's CPU exp rounds exp(-x) for tiny x up from
    k + 29/64 quanta, where alpha_of rounds to nearest.  Asserted per ray: the GPU is within 1e-4 of the
    reference's float64 value widened by the reference's own distance from it,
    |gpu - f64| <= 1e-4 + |ref - f64|; and within 1e-4 + the largest such spread of the reference."""
    import ast
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "h12_nearempty_c5.npz"))
    meta = ast.literal_eval(str(z["meta"]))
    ck = syn.make_checkpoint(meta["seed"], n_joints=24, D=8, W=256, fine=True, tau=meta["tau"])
    assert syn.checkpoint_sha256(ck) == meta["sha256"]
    sc = syn.make_scene(n_joints=24, H=meta["H"], W=meta["H"], seed=meta["seed"])
    cfg = anerf.RenderConfig(N_samples=64, N_importance=128, precision=precision).validate()
    rc = anerf.RayCaster(cfg, ck)
    n = z["sel"].shape[0]
    rb = np.zeros((n, 11), np.float32)
    rb[:, 0:3], rb[:, 3:6], rb[:, 6], rb[:, 7] = z["rays_o"], z["rays_d"], z["near"], z["far"]
    rb[:, 8:11] = z["rays_d"] / np.linalg.norm(z["rays_d"], axis=-1, keepdims=True)
    cy = torch.from_numpy(z["cyls"]).cuda()
    sk = torch.from_numpy(sc["skts"][0:1]).cuda()
    out = rc.render_rays(torch.from_numpy(rb).cuda(), 64, skts=sk.expand(n, -1, -1, -1), cyls=cy.expand(n, -1),
                         N_importance=128, ret_alpha=False, near_far_given=True)
    torch.cuda.synchronize()
    ne = z["near_empty"]
    for k in ("rgb_map", "acc_map", "rgb0", "disp0", "acc0"):
        d = np.abs(out[k].cpu().numpy().astype(np.float64) - z["out_" + k]).reshape(n, -1).max(-1)
        assert d.max() <= TOL, (k, float(d.max()))
    got = out["disp_map"].cpu().numpy().astype(np.float64)
    dd = np.abs(got - z["out_disp_map"])
    assert dd[~ne].max() <= TOL, float(dd[~ne].max())
    sp = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "h12_spread_c5.npz"))
    assert np.array_equal(sp["sel"], z["sel"]) and np.array_equal(sp["t8_disp_map"], z["out_disp_map"])
    f64 = sp["f64_disp_map"]
    own = np.abs(z["out_disp_map"].astype(np.float64) - f64)  # the reference's distance from its float64 value
    margin = np.abs(got - f64) - (TOL + own)
    print(f"{precision} H12: {int(ne.sum())} near-empty rays, |gpu - reference| disp max {dd[ne].max():.3e} "
          f"({int((dd[ne] > TOL).sum())} above 1e-4); |gpu - f64| - |ref - f64| max {(margin[ne] + TOL).max():.3e}; "
          f"reference spread max {own[ne].max():.3e}")
    assert margin[ne].max() <= 0.0, (int(np.argmax(np.where(ne, margin, -1))), float(margin[ne].max()))
    assert dd[ne].max() <= TOL + own[ne].max()



@pytest.mark.parametrize("precision", ["fp16x4", "fp16x3", "bf16x6", "fp32"])
def test_power_of_two_rescaled_hidden_layers_render_identically(precision):
    """relu is positively homogeneous, so scaling hidden layer i's outputs by s_i (its weights' h columns
    by s_i / s_(i-1), the skip layer's x columns and every bias by s_i, the heads by 1 / s_7) leaves the
    network's function unchanged; with powers of two (2^-14 .. 2^15 here) every fp32 product and sum is
    the same up to the exponent.  The fp16 modes scale each sample's activations into [2^10, 2^11) and
    each layer's weights by a power of two, so they must absorb the factors exactly too: all modes render
    the rescaled checkpoint bit-identically to the original (this pins the fp16 range handling at
    activations far outside fp16's own range)."""
    sc, ck, cyls, rb = _frame(512, 24, 13, 79.6)
    rb = rb[::97].contiguous()
    s = [1.0, 2.0 ** 12, 2.0 ** -9, 2.0 ** 15, 2.0 ** -14, 2.0 ** 10, 2.0 ** -6, 2.0 ** 13]
    skip = 4
    ck2 = {k: (dict(v) if isinstance(v, dict) else v) for k, v in ck.items()}
    for net in ("network_fn_state_dict", "network_fine_state_dict"):
        sd = {k: np.array(v, copy=True) for k, v in ck[net].items()}
        for i in range(1, 8):
            w, b = sd[f"pts_linears.{i}.weight"], sd[f"pts_linears.{i}.bias"]
            if i == skip + 1:  # [x | h] input (core/networks/nerf.py: cat([input_pts, h]))
                nx = w.shape[1] - 256
                w[:, :nx] *= np.float32(s[i])
                w[:, nx:] *= np.float32(s[i] / s[i - 1])
            else:
                w *= np.float32(s[i] / s[i - 1])
            b *= np.float32(s[i])
        for k in ("alpha_linear.weight", "feature_linear.weight"):
            sd[k] *= np.float32(1.0 / s[7])
        ck2[net] = {k: torch.from_numpy(v) if isinstance(ck[net][k], torch.Tensor) else v for k, v in sd.items()}
    cfg = anerf.RenderConfig(N_samples=64, N_importance=128, precision=precision).validate()
    a = _render(anerf.RayCaster(cfg, ck), rb, sc, cyls)
    b2 = _render(anerf.RayCaster(cfg, ck2), rb, sc, cyls)
    torch.cuda.synchronize()
    for k in ("rgb_map", "disp_map", "acc_map", "rgb0", "disp0", "acc0"):
        assert torch.equal(a[k].nan_to_num(7.0), b2[k].nan_to_num(7.0)), (k, float((a[k] - b2[k]).abs().max()))

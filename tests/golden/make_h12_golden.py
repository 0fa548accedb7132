"""Fixture for hazard H12 (near-empty rays' disparity) from the REFERENCE render path.

Build container only (imports /root/reference like make_golden.py; the fixture it writes is
committed, the GPU box never runs this).  Two stages:

1. scan: the C oracle (test infrastructure) renders every ray of BASELINE config 5's 1024^2 frame
   (synthetic scene / checkpoint seed 13, tau 79.6: the frame tests/test_gpu_frames.py and the
   bench's pixel-shard leg render) with near / far from the whole frame's 4096-ray chunks, and
   lists the rays with 0 < acc < 2^-20 -- the rays whose disp = 1 / max(1e-10, depth / acc)
   (core/networks/nerf.py:195-199) is a ratio of a few 2^-24 alpha quanta.  Saved to
   /tmp/h12_scan.npz (not committed; ~15 min on 8 cores).
2. fixture: the reference's own render_rays (core.trainer.render -> RayCaster.render_rays,
   core/raycasters.py:361-474) on those rays that hit the bounding cylinder (their near / far do not
   depend on the chunk: the NaN fill of ray_utils.py:328-342 only touches rays that miss it) plus
   evenly spaced ordinary rays of the same frame, written to tests/golden/h12_nearempty_c5.npz
   with the rays' indices in the frame's ray list, the reference's rays (get_rays,
   ray_utils.py:6-28), its outputs, and the oracle's outputs on the same rays.

Usage:  python tests/golden/make_h12_golden.py scan|fixture
"""
import importlib
import os
import sys
import tempfile
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(REPO, "oracle"))

anerf = importlib.import_module("a-nerf_amd")
syn = importlib.import_module("a-nerf_amd.synthetic")

SCAN = "/tmp/h12_scan.npz"
H, NJ, SEED, TAU = 1024, 24, 13, 79.6
N_ORDINARY = 64
MAX_EMPTY = 256


def frame():
    sc = syn.make_scene(n_joints=NJ, H=H, W=H, seed=SEED)
    ck = syn.make_checkpoint(SEED, n_joints=NJ, D=8, W=256, fine=True, tau=TAU)
    idx, cyls, boxes = anerf.rays.valid_pixels(sc["c2ws"], H, H, sc["focal"], kps=sc["kps"], ext_scale=0.001)
    cfg = anerf.RenderConfig(n_joints=NJ, N_samples=64, N_importance=128, precision="fp32").validate()
    return sc, ck, cfg, np.asarray(idx[0], np.int64), cyls


def scan():
    import oracle
    sc, ck, cfg, idx, cyls = frame()
    rb = oracle.gen_rays(sc["c2ws"][0], H, H, sc["focal"], idx)
    om = oracle.OracleModel(cfg, ck)
    near, far, q, _ = om.near_far(rb, cyls[0:1], chunk=4096)
    n = rb.shape[0]
    acc = np.empty(n, np.float32)
    disp = np.empty(n, np.float32)
    t0 = time.time()
    step = 65536
    for s in range(0, n, step):
        e = min(n, s + step)
        out = om.render_rays(rb[s:e], sc["skts"][0], cyls[0:1], chunk=4096, nthreads=8, near=near[s:e], far=far[s:e])
        acc[s:e], disp[s:e] = out["acc_map"], out["disp_map"]
        print(f"{e}/{n} rays  {time.time() - t0:.0f} s", flush=True)
    np.savez(SCAN, acc=acc, disp=disp, near=near, far=far, miss=np.isnan(q), n=n)
    empty = (acc > 0) & (acc < 2.0 ** -20)
    print(f"near-empty rays: {int(empty.sum())} of {n}; of them missing the cylinder: {int((empty & np.isnan(q)).sum())}")


def fixture():
    import torch
    import make_golden as mg
    import oracle
    torch.set_num_threads(8)
    sc, ck, cfg, idx, cyls = frame()
    s = np.load(SCAN)
    n = int(s["n"])
    empty = np.flatnonzero((s["acc"] > 0) & (s["acc"] < 2.0 ** -20) & ~s["miss"])
    if len(empty) > MAX_EMPTY:  # evenly spaced over the frame
        empty = empty[np.linspace(0, len(empty) - 1, MAX_EMPTY).astype(np.int64)]
    hit = np.flatnonzero(~s["miss"] & (s["acc"] >= 2.0 ** -20))
    ordinary = hit[np.linspace(0, len(hit) - 1, N_ORDINARY).astype(np.int64)]
    sel = np.sort(np.concatenate([empty, ordinary]))
    mods = mg.import_reference()
    gcfg = dict(H=H, NJ=NJ, S=64, I=128, D=8, W=256, tau=TAU, kind="rays", seed=SEED)
    with tempfile.TemporaryDirectory() as tmp:
        args, render_kwargs, ck_ref = mg.build_reference(mods, gcfg, tmp)
        assert syn.checkpoint_sha256(ck_ref) == syn.checkpoint_sha256(ck)
        (o, d), vidx, rcyls, _ = mg.rays_for(mods, sc)
        assert np.array_equal(vidx, idx), "host pixel list differs from the reference's kp_to_valid_rays"
        sc["cyls"] = rcyls
        ret = mg.render_subset(mods, render_kwargs, o[sel], d[sel], sc)
    rb = oracle.gen_rays(sc["c2ws"][0], H, H, sc["focal"], idx[sel])
    assert np.array_equal(rb[:, 0:3], o[sel].numpy()) and np.array_equal(rb[:, 3:6], d[sel].numpy())
    orc = oracle.OracleModel(cfg, ck).render_rays(rb, sc["skts"][0], cyls[0:1], chunk=4096, nthreads=8,
                                                   near=s["near"][sel], far=s["far"][sel])
    meta = dict(seed=SEED, sha256=syn.checkpoint_sha256(ck), NJ=NJ, S=64, I=128, D=8, W=256, tau=TAU, H=H,
                focal=sc["focal"], ext_scale=0.001, chunk=4096, n_frame_rays=n,
                n_near_empty_frame=int(((s["acc"] > 0) & (s["acc"] < 2.0 ** -20)).sum()),
                near_empty="0 < acc < 2^-20 by the oracle over the whole frame")
    data = dict(sel=sel, near_empty=np.isin(sel, empty), rays_o=o[sel].numpy(), rays_d=d[sel].numpy(),
                near=s["near"][sel], far=s["far"][sel], cyls=rcyls[0:1],
                **{"out_" + k: v for k, v in ret.items() if not k.startswith("alpha")},
                **{"oracle_" + k: orc[k] for k in ("rgb_map", "disp_map", "acc_map", "rgb0", "disp0", "acc0")})
    path = os.path.join(HERE, "h12_nearempty_c5.npz")
    np.savez_compressed(path, meta=np.array(repr(meta)), **data)
    ne = data["near_empty"]
    dd = np.abs(data["out_disp_map"].astype(np.float64) - orc["disp_map"])
    print(f"wrote {path}: {len(sel)} rays ({int(ne.sum())} near-empty); |reference - oracle| disp: "
          f"near-empty max {dd[ne].max():.3e} ({int((dd[ne] > 1e-4).sum())} > 1e-4), ordinary max {dd[~ne].max():.3e}")


def _reference_runs(mods, render_kwargs, sc, o, d):
    """The reference's render_rays on rays (o, d) three ways: torch.set_num_threads(8) (the fixture's
    own setting), (1), and with the networks, embedders and every input in float64
    (torch.set_default_dtype(float64): linspace, the 1e10 / ones constants of raw2outputs follow).  The
    fine pass's raw sigma, alpha, weights and z are captured by wrapping network_fine.raw2outputs."""
    import torch
    _, trainer, _, _, _ = mods
    rc = render_kwargs["ray_caster"]
    net = rc.network_fine
    orig = net.raw2outputs
    cap = {}

    def hook(raw, z_vals, rays_d, *a, **k):
        ret = orig(raw, z_vals, rays_d, *a, **k)
        cap.setdefault("sigma", []).append(raw[..., 3].detach().to(torch.float64).numpy())
        cap.setdefault("alpha", []).append(ret["alpha"].detach().to(torch.float64).numpy())
        cap.setdefault("weights", []).append(ret["weights"].detach().to(torch.float64).numpy())
        cap.setdefault("z", []).append(z_vals.detach().to(torch.float64).numpy())
        return ret

    net.raw2outputs = hook
    runs = {}
    try:
        for name, threads, f64 in (("t8", 8, False), ("t1", 1, False), ("f64", 8, True)):
            cap.clear()
            torch.set_num_threads(threads)
            dt = torch.float64 if f64 else torch.float32
            torch.set_default_dtype(dt)
            rc.to(dt)
            n = o.shape[0]
            oo, dd = torch.as_tensor(o).to(dt), torch.as_tensor(d).to(dt)
            vd = dd / torch.norm(dd, dim=-1, keepdim=True)
            rays = torch.cat([oo, dd, torch.zeros(n, 1, dtype=dt), torch.ones(n, 1, dtype=dt), vd], -1)
            kw = {k: v for k, v in render_kwargs.items() if k not in ("use_viewdirs", "near", "far", "center", "c2w_staticcam")}
            with torch.no_grad():
                ret = trainer.batchify_rays(rays, 4096, kp_batch=torch.from_numpy(sc["kps"][0:1]).to(dt).expand(n, -1, -1),
                                            skts=torch.from_numpy(sc["skts"][0:1]).to(dt).expand(n, -1, -1, -1),
                                            cyls=torch.from_numpy(sc["cyls"][0:1]).to(dt).expand(n, -1),
                                            bones=torch.from_numpy(sc["bones"][0:1]).to(dt).expand(n, -1, -1),
                                            cams=None, subject_idxs=None, **kw)
            runs[name] = {k: v.to(torch.float64).numpy() for k, v in ret.items() if not k.startswith("alpha")}
            runs[name].update({k: np.concatenate(v, 0) for k, v in cap.items()})
            print(f"reference run {name}: {n} rays", flush=True)
    finally:
        net.raw2outputs = orig
        torch.set_default_dtype(torch.float32)
        rc.to(torch.float32)
        torch.set_num_threads(8)
    return runs


def spread():
    """H12 evidence: how far the REFERENCE's own disp moves on the fixture's rays
    when only its summation order (thread count) or its precision (float64) changes.  Writes
    tests/golden/h12_spread_c5.npz: per ray and run disp / acc / rgb, and for the near-empty rays the
    fine pass's per-sample raw sigma, alpha, weights and z of every run."""
    import make_golden as mg
    z = np.load(os.path.join(HERE, "h12_nearempty_c5.npz"))
    sc, ck, cfg, idx, cyls = frame()
    sel, ne = z["sel"], z["near_empty"]
    mods = mg.import_reference()
    gcfg = dict(H=H, NJ=NJ, S=64, I=128, D=8, W=256, tau=TAU, kind="rays", seed=SEED)
    with tempfile.TemporaryDirectory() as tmp:
        args, render_kwargs, ck_ref = mg.build_reference(mods, gcfg, tmp)
        assert syn.checkpoint_sha256(ck_ref) == syn.checkpoint_sha256(ck)
        (o, d), vidx, rcyls, _ = mg.rays_for(mods, sc)
        sc["cyls"] = rcyls
        runs = _reference_runs(mods, render_kwargs, sc, o[sel], d[sel])
    assert np.array_equal(runs["t8"]["disp_map"].astype(np.float32), z["out_disp_map"]), "t8 run != the fixture"
    data = {"sel": sel, "near_empty": ne}
    for name, r in runs.items():
        for k in ("rgb_map", "disp_map", "acc_map"):
            data[f"{name}_{k}"] = r[k].astype(np.float64 if name == "f64" else np.float32)
        for k in ("sigma", "alpha", "weights", "z"):
            data[f"{name}_{k}"] = r[k][ne].astype(np.float64 if name == "f64" else np.float32)
    path = os.path.join(HERE, "h12_spread_c5.npz")
    np.savez_compressed(path, meta=np.array(repr(dict(seed=SEED, tau=TAU, H=H, runs="t8: 8 threads (= the fixture), "
                                                              "t1: 1 thread, f64: float64 networks/inputs"))), **data)
    d81 = np.abs(data["t8_disp_map"].astype(np.float64) - data["t1_disp_map"])
    d8f = np.abs(data["t8_disp_map"].astype(np.float64) - data["f64_disp_map"])
    print(f"wrote {path}")
    print(f"near-empty ({int(ne.sum())}): |t8 - t1| disp max {d81[ne].max():.3e} ({int((d81[ne] > 1e-4).sum())} > 1e-4); "
          f"|t8 - f64| disp max {d8f[ne].max():.3e} ({int((d8f[ne] > 1e-4).sum())} > 1e-4)")
    print(f"ordinary ({int((~ne).sum())}): |t8 - t1| disp max {d81[~ne].max():.3e}; |t8 - f64| disp max {d8f[~ne].max():.3e}")


if __name__ == "__main__":
    {"scan": scan, "fixture": fixture, "spread": spread}[sys.argv[1]]()

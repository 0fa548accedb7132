"""ctypes front-end of the C oracle (oracle/anerf_oracle.c).  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
MAXL = 16

_f = ctypes.POINTER(ctypes.c_float)
_i32 = ctypes.POINTER(ctypes.c_int32)


class _Net(ctypes.Structure):
    _fields_ = [("w", _f * MAXL), ("b", _f * MAXL), ("wa", _f), ("ba", _f), ("wf", _f), ("bf", _f),
                ("wv", _f), ("bv", _f), ("wrgb", _f), ("brgb", _f), ("codes", _f)]


class _Model(ctypes.Structure):
    _fields_ = [("nj", ctypes.c_int), ("D", ctypes.c_int), ("W", ctypes.c_int), ("skip", ctypes.c_int),
                ("multires", ctypes.c_int), ("multires_views", ctypes.c_int),
                ("use_cutoff", ctypes.c_int), ("cutoff_inputs", ctypes.c_int), ("cutoff_viewdir", ctypes.c_int),
                ("framecode_ch", ctypes.c_int), ("n_framecodes", ctypes.c_int),
                ("density_softplus", ctypes.c_int), ("softplus_shift", ctypes.c_float),
                ("density_scale", ctypes.c_float), ("tau", ctypes.c_float), ("tau_v", ctypes.c_float),
                ("cutoff", _f), ("cutoff_v", _f), ("has_fine", ctypes.c_int), ("single_net", ctypes.c_int),
                ("lindisp", ctypes.c_int), ("sched_w", _f), ("sched_wv", _f), ("cut_to", ctypes.c_int),
                ("shift_in", ctypes.c_int),
                ("coarse", _Net), ("fine", _Net),
                ("bone_cut", ctypes.c_int), ("tau_b", ctypes.c_float), ("cutoff_b", _f), ("view_raw", ctypes.c_int)]


def build():
    subprocess.run(["make", "-C", HERE, "-s"], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_render_rays.restype = ctypes.c_int
        L.oracle_near_far.restype = ctypes.c_int64
        L.oracle_feature_dim.restype = ctypes.c_int
        L.oracle_torch_sum.restype = ctypes.c_float
        L.oracle_torch_sum_strided.restype = ctypes.c_float
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(_f) if a is not None else None


def _f32(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def schedule_w(alpha, n_freqs):
    """CutoffEmbedder.get_schedule_w (core/cutoff_embedder.py:192-197) in float32: frequency k's
    weight 0.5 (1 - cos(pi clamp(alpha - k, 0, 1))) (freq_k = log2(freq_bands) = k exactly)."""
    diff = np.clip(np.float32(np.asarray(alpha, np.float32).reshape(-1)[0]) - np.arange(n_freqs, dtype=np.float32),
                   np.float32(0), np.float32(1))
    return (np.float32(0.5) * (np.float32(1.0) - np.cos(np.float32(np.pi) * diff))).astype(np.float32)


class OracleModel:
    """Holds contiguous (transposed where the C side wants [in][out]) weight copies."""

    def __init__(self, cfg, ckpt):
        self.cfg = cfg
        self._keep = []
        m = _Model()
        m.nj, m.D, m.W, m.skip = cfg.n_joints, cfg.netdepth, cfg.netwidth, cfg.skips[0]
        m.multires, m.multires_views = cfg.multires, cfg.multires_views
        m.use_cutoff, m.cutoff_inputs = int(cfg.use_cutoff), int(cfg.cutoff_inputs)
        # (the view embedder is windowed only under use_cutoff too: core/raycasters.py:31, 68-71)
        m.cutoff_viewdir = int(cfg.cutoff_viewdir and cfg.use_cutoff)
        m.framecode_ch, m.n_framecodes = cfg.framecode_ch, (cfg.n_framecodes if cfg.opt_framecode else 0)
        m.density_softplus = int(cfg.density_type == "softplus")
        m.softplus_shift, m.density_scale = cfg.softplus_shift, cfg.density_scale
        e, ev = ckpt["embed_state_dict"], ckpt["embeddirs_state_dict"]
        m.tau, m.tau_v = float(np.asarray(e["tau"])), float(np.asarray(ev["tau"]))
        m.cutoff, m.cutoff_v = self._k(e["cutoff_dist"]), self._k(ev["cutoff_dist"])
        fine = ckpt.get("network_fine_state_dict")
        coarse = ckpt["network_fn_state_dict"]
        if cfg.single_net:  # network_fine IS network_fn; load_state_dict loads the fine keys last
            coarse, fine = (fine if fine is not None else coarse), None
        m.single_net = int(cfg.single_net)
        m.lindisp = int(cfg.lindisp)
        m.cut_to, m.shift_in = int(getattr(cfg, "cut_to_dist", False)), int(getattr(cfg, "cutoff_shift", False))
        m.view_raw = int(getattr(cfg, "extra", {}).get("view_type", "relray") == "world")
        if getattr(cfg, "cutoff_bones", False) and cfg.use_cutoff and cfg.cutoff_inputs:
            eb = ckpt["embedbones_state_dict"]
            m.bone_cut, m.tau_b, m.cutoff_b = 1, float(np.asarray(eb["tau"])), self._k(eb["cutoff_dist"])
        if getattr(cfg, "freq_schedule", False):
            m.sched_w = self._k(schedule_w(e["sched_alpha"], cfg.multires))
            m.sched_wv = self._k(schedule_w(ev["sched_alpha"], cfg.multires_views))
        self._net(m.coarse, coarse)
        m.has_fine = int(fine is not None)
        if fine is not None:
            self._net(m.fine, fine)
        self.m = m

    def _k(self, a, transpose=False):
        a = _f32(a)
        if transpose:
            a = np.ascontiguousarray(a.T)
        self._keep.append(a)
        return _p(a)

    def _net(self, net, sd):
        for i in range(self.cfg.netdepth):
            net.w[i] = self._k(sd[f"pts_linears.{i}.weight"], transpose=True)
            net.b[i] = self._k(sd[f"pts_linears.{i}.bias"])
        net.wa, net.ba = self._k(sd["alpha_linear.weight"]), self._k(sd["alpha_linear.bias"])
        net.wf, net.bf = self._k(sd["feature_linear.weight"], True), self._k(sd["feature_linear.bias"])
        net.wv, net.bv = self._k(sd["views_linears.0.weight"], True), self._k(sd["views_linears.0.bias"])
        net.wrgb, net.brgb = self._k(sd["rgb_linear.weight"]), self._k(sd["rgb_linear.bias"])
        net.codes = self._k(sd["framecodes.codes.weight"]) if self.cfg.opt_framecode else None

    @property
    def ref(self):
        return ctypes.byref(self.m)

    # ------------------------------------------------------------------ stages
    def feature_dim(self):
        return lib().oracle_feature_dim(self.ref)

    def near_far(self, ray_batch, cyls, ray_pose=None, chunk=4096):
        rb = _f32(ray_batch)
        n, stride = rb.shape
        near = np.empty(n, np.float32)
        far = np.empty(n, np.float32)
        q = np.empty(n, np.float32)
        cy = _f32(cyls)
        rp = None if ray_pose is None else np.ascontiguousarray(ray_pose, dtype=np.int32)
        filled = lib().oracle_near_far(_p(rb), stride, ctypes.c_int64(n), _p(cy),
                                       rp.ctypes.data_as(_i32) if rp is not None else None, chunk,
                                       _p(near), _p(far), _p(q))
        return near, far, q, int(filled)

    def encode(self, skts, pts, dirs):
        pts, dirs, sk = _f32(pts), _f32(dirs), _f32(skts)
        M = pts.shape[0]
        out = np.empty((M, self.feature_dim()), np.float32)
        lib().oracle_encode(self.ref, _p(sk), _p(pts), _p(dirs), ctypes.c_int64(M), _p(out))
        return out

    def density(self, skts, pts, fine=False):
        """Raw density (alpha_linear output) of the density trunk at points (N, 3): the path of
        RayCaster.render_pts_density / _get_density_fwd_fn (core/raycasters.py:597-648) -- the
        trunk reads only the point part of the encoding, so the view directions are arbitrary."""
        pts = _f32(pts).reshape(-1, 3)
        feat = self.encode(skts, pts, np.ones_like(pts))
        return self.network(feat, fine=fine)[:, 3].copy()

    def network(self, feat, fine=False, code=None):
        feat = _f32(feat)
        M = feat.shape[0]
        raw = np.empty((M, 4), np.float32)
        c = None if code is None else _f32(code)
        lib().oracle_network(self.ref, int(fine), _p(feat), ctypes.c_int64(M), _p(c), _p(raw))
        return raw

    def raw2outputs(self, raw, z, dirs):
        raw, z, dirs = _f32(raw), _f32(z), _f32(dirs)
        n, ns = z.shape
        rgb = np.empty((n, 3), np.float32)
        disp, acc = np.empty(n, np.float32), np.empty(n, np.float32)
        w, a = np.empty((n, ns), np.float32), np.empty((n, ns), np.float32)
        lib().oracle_raw2outputs(self.ref, _p(raw), _p(z), _p(dirs), ctypes.c_int64(n), ns, _p(rgb), _p(disp),
                                 _p(acc), _p(w), _p(a))
        return dict(rgb_map=rgb, disp_map=disp, acc_map=acc, weights=w, alpha=a)

    def sample_pdf(self, bins, weights, n_samples):
        bins, weights = _f32(bins), _f32(weights)
        n, nb = bins.shape
        out = np.empty((n, n_samples), np.float32)
        lib().oracle_sample_pdf(_p(bins), _p(weights), ctypes.c_int64(n), nb, n_samples, _p(out))
        return out

    def render_rays(self, ray_batch, skts, cyls, ray_pose=None, cams=None, N_samples=None, N_importance=None,
                    chunk=4096, nthreads=0, with_z=False, near=None, far=None):
        """render_rays over a whole ray list (chunked NaN fill), returns the reference's output dict.
        near / far: the rays' filled near / far (e.g. from near_far() of the whole frame when ray_batch
        is a sample of its rays), instead of the fill over this list's chunks."""
        cfg = self.cfg
        S = cfg.N_samples if N_samples is None else N_samples
        I = cfg.N_importance if N_importance is None else N_importance
        rb = _f32(ray_batch)
        n, stride = rb.shape
        T = S + I
        rgb, disp, acc = np.empty((n, 3), np.float32), np.empty(n, np.float32), np.empty(n, np.float32)
        alpha = np.empty((n, T if I > 0 else S), np.float32)
        out = dict(rgb_map=rgb, disp_map=disp, acc_map=acc, alpha=alpha)
        extra = [None] * 4
        if I > 0:
            out.update(rgb0=np.empty((n, 3), np.float32), disp0=np.empty(n, np.float32),
                       acc0=np.empty(n, np.float32), alpha0=np.empty((n, S), np.float32))
            extra = [out["rgb0"], out["disp0"], out["acc0"], out["alpha0"]]
        z = np.empty((n, T if I > 0 else S), np.float32) if with_z else None
        rp = None if ray_pose is None else np.ascontiguousarray(ray_pose, dtype=np.int32)
        cm = None if cams is None else _f32(cams)
        rc = lib().oracle_render_rays(self.ref, _p(rb), stride, ctypes.c_int64(n), _p(_f32(skts)), _p(_f32(cyls)),
                                      rp.ctypes.data_as(_i32) if rp is not None else None, _p(cm), S, I, chunk,
                                      nthreads, _p(rgb), _p(disp), _p(acc), _p(extra[0]), _p(extra[1]),
                                      _p(extra[2]), _p(alpha), _p(extra[3]), _p(z),
                                      _p(None if near is None else _f32(near)), _p(None if far is None else _f32(far)))
        if rc != 0:
            raise RuntimeError(f"oracle_render_rays failed ({rc})")
        if with_z:
            out["z"] = z
        return out


def gen_rays(c2w, H, W, focal, idx, center=None, near=0.0, far=1.0):
    """Ray batch [n][11] for pixel indices (oracle_gen_rays)."""
    c2w = _f32(np.asarray(c2w)[:3, :4])
    idx = np.ascontiguousarray(idx, dtype=np.int64)
    out = np.empty((idx.shape[0], 11), np.float32)
    fa = np.asarray(focal, dtype=np.float64).reshape(-1)
    fx = float(fa[0])
    fy = float(fa[1]) if fa.size > 1 else fx
    cx, cy = (float(W * 0.5), float(H * 0.5)) if center is None else (float(center[0]), float(center[1]))
    lib().oracle_gen_rays(_p(c2w), H, W, ctypes.c_float(fx), ctypes.c_float(fy), ctypes.c_float(cx),
                          ctypes.c_float(cy), idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                          ctypes.c_int64(idx.shape[0]), ctypes.c_float(near), ctypes.c_float(far), _p(out))
    return out


def mesh_grid_points(radius, res, kp0):
    """Grid of render_mesh_density (core/raycasters.py:583-588): float64 linspace, 'xy' meshgrid,
    cast to float32, then + kps[0, 0] in float32.  Returns ((res+1)^3, 3)."""
    t = np.linspace(-radius, radius, res + 1)
    g = np.stack(np.meshgrid(t, t, t), axis=-1).astype(np.float32).reshape(-1, 3)
    return (g + np.asarray(kp0, np.float32)).astype(np.float32)


def linspace(n):
    out = np.empty(n, np.float32)
    lib().oracle_linspace(n, _p(out))
    return out



H12_SPREAD = os.path.join(os.path.dirname(HERE), "tests", "golden", "h12_spread_c5.npz")


def h12_spread(path=H12_SPREAD):
    """The reference's own disparity spread on near-empty rays (hazard H12), measured by
    tests/golden/make_h12_golden.py spread: the reference's render_rays on config 5's 169 near-empty
    rays (0 < acc < 2^-20) rendered with 8 threads (= the fixture), 1 thread, and in float64.  Returns
    dict(threads=max |t8 - t1|, float64=max |t8 - f64|, per_ray=|t8 - f64| [169]) over those rays:
    a near-empty ray's disp = (acc + 1e-10) / depth is a ratio of a few 2^-24 alpha quanta, and the
    reference's float32 value sits up to that far from its own exact value."""
    z = np.load(path)
    ne = z["near_empty"]
    t8 = z["t8_disp_map"].astype(np.float64)
    d81 = np.abs(t8 - z["t1_disp_map"])[ne]
    d8f = np.abs(t8 - z["f64_disp_map"])[ne]
    return {"threads": float(d81.max()), "float64": float(d8f.max()), "per_ray": d8f}

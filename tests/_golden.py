"""Loading helpers for the committed golden fixtures (tests/golden/*.npz)."""
import ast
import importlib
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")

anerf = importlib.import_module("a-nerf_amd")
syn = importlib.import_module("a-nerf_amd.synthetic")
config = importlib.import_module("a-nerf_amd.config")

NAMES = ["c1_64_s32_d4w128", "c2_256_s64_d8w256", "c3_512_s64i128_d8w256", "c4_512_s64i128_j65",
         "h1_nanfill_s32i16_d4w128", "fc_64_s32i32_d4w128",
         # flag variants: multires 10 + width 64; softplus density without view cutoff; unwindowed
         # distance input; no cutoff window at all
         "v1_mr10_w64_d4", "v2_softplus_nocutview", "v3_nocutinputs", "v4_nocutoff",
         # configs/surreal/surreal_single.txt (single_net, multires_views 0, 96 + 48); tau at its ceiling
         "s1_single_s96i48_mrv0", "t2000_512_s64i128",
         # --lindisp (inverse-depth samples); --freq_schedule at sched_alpha 2.3 (D = 8: skip layer)
         "l1_lindisp_s32i16_d4w128", "fs1_freqsched_s32i16_d8w128",
         # --cut_to_dist, --cutoff_shift (the kp cutoff embedder's input transforms)
         "cd1_cuttodist_s32i16_d8w128", "cs1_cutoffshift_s32i16_d4w128",
         # --cutoff_bones (bone directions windowed by the bone embedder's own tau / cutoffs)
         "cb1_cutoffbones_s32i16_d8w128",
         # the shipped configs' shape: mixamo / h36m / perfcap (8x256, 64 + 16, framecodes incl. the eval-mode
         # mean code), surreal (8x256, 64 + 16)
         "mx1_mixamo_s64i16_d8w256_fc", "su1_surreal_s64i16_d8w256",
         # render_path frames with white_bkgd / resized background images (two frames each)
         "pw_64_white_d4w128", "pb_64_bgimg_d4w128",
         # multires / multires_views other than 7 / 4 and 10 (zero-padded on the 7 / 10, 4 instances) at
         # widths 256 (bf16x6 windowed part), 128 and 64 (f32 windowed part)
         "mr5_mrv2_s32i16_d8w256", "mr9_mrv3_s32i16_d8w128", "mr3_mrv1_s32i16_d4w64",
         # --view_type world (un-normalised joint-frame ray directions into the view embedder)
         "vw1_viewworld_s32i16_d8w128"]
# (round 5) staged encoders (include/anerf.h): rendered by train.StagedCaster on the training stages; GPU parity
# in tests/test_gpu_staged.py
STAGED = ["sg1_relpos_s32i16_d4w128", "sg2_rayangle_mrb2_cb_s32i16_d8w128", "sg3_all_fs_s32i16_d8w256",
          "sg4_querypts_shift_s32i16_d8w128"]
FRAMES = ["c1_64_s32_d4w128", "pw_64_white_d4w128", "pb_64_bgimg_d4w128"]


class Golden:
    def __init__(self, name):
        self.name = name
        z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
        self.d = {k: z[k] for k in z.files}
        self.meta = ast.literal_eval(str(self.d["meta"]))
        m = self.meta
        fc = bool(m.get("framecode", 0))
        drop, flags = m.get("drop", []), m.get("flags", [])
        kw = {}
        if "--density_type" in flags:
            kw["density_type"] = flags[flags.index("--density_type") + 1]
        val = lambda k, d=None: flags[flags.index(k) + 1] if k in flags else d  # noqa: E731
        extra = {k[2:]: val(k) for k in ("--view_type", "--kp_dist_type") if k in flags}
        if extra:
            kw["extra"] = extra
        # (round 5) the staged encoders' input shapes (tests/golden/make_golden.py staged_dims)
        dims = dict(multires_bones=int(val("--multires_bones", 0)), kp_dims=3 if val("--kp_dist_type") == "relpos" else 1,
                    view_dims=1 if val("--view_type") == "rayangle" else 3, kp_query=val("--kp_dist_type") == "querypts")
        if "--softplus_shift" in flags:
            kw["softplus_shift"] = float(flags[flags.index("--softplus_shift") + 1])
        self.cfg = config.RenderConfig(n_joints=m["NJ"], netdepth=m["D"], netwidth=m["W"], N_samples=m["S"],
                                       N_importance=m["I"], opt_framecode=fc, n_framecodes=5 if fc else 0,
                                       chunk=m["chunk"], ext_scale=m["ext_scale"], multires=m.get("mr", 7),
                                       use_cutoff="--use_cutoff" not in drop,
                                       cutoff_inputs="--cutoff_inputs" not in drop,
                                       cutoff_viewdir="--cutoff_viewdir" not in drop,
                                       multires_views=m.get("mrv", 4), single_net=m.get("single", False),
                                       lindisp="--lindisp" in flags or bool(m.get("lindisp", False)),
                                       freq_schedule="--freq_schedule" in flags,
                                       cut_to_dist="--cut_to_dist" in flags, cutoff_shift="--cutoff_shift" in flags,
                                       cutoff_bones="--cutoff_bones" in flags,
                                       init_freq=float(flags[flags.index("--init_freq") + 1])
                                       if "--init_freq" in flags else 0.0,
                                       multires_bones=dims["multires_bones"], precision="fp32", **kw).validate()
        self.ckpt = syn.make_checkpoint(m["seed"], n_joints=m["NJ"], D=m["D"], W=m["W"], fine=m["I"] > 0,
                                        tau=m["tau"], use_framecode=fc, n_framecodes=5, multires=m.get("mr", 7),
                                        multires_views=m.get("mrv", 4), sched_alpha=m.get("sched"),
                                        cutoff_bones=bool(m.get("cb", False)), tau_bones=m.get("tau_b"), **dims)
        assert syn.checkpoint_sha256(self.ckpt) == m["sha256"], "synthetic weights drifted from the fixture"

    def __getitem__(self, k):
        return self.d[k]

    def has(self, k):
        return k in self.d

    def ray_batch(self):
        o, d = self.d["rays_o"], self.d["rays_d"]
        n = o.shape[0]
        vd = d / np.linalg.norm(d, axis=-1, keepdims=True)
        return np.concatenate([o, d, np.zeros((n, 1), np.float32), np.ones((n, 1), np.float32), vd],
                              axis=-1).astype(np.float32)


def sqrt_tie_rays(rb, cyl, tol_ulp=0.02):
    """Rays whose get_near_far_in_cylinder Q = (r^2 - dist^2)^0.5 (core/utils/ray_utils.py:318) is a
    near-tie for float32 rounding: the exact square root of the float32 argument lies within tol_ulp of
    the midpoint between two floats (hazard H13).  torch's CPU sqrt / pow(0.5) is faithful,
    not correctly rounded (MKL VML), and can round such a Q the other way from the correctly rounded
    sqrtf of the oracle and the GPU: near / far then differ by one float32 ulp.  The argument is
    recomputed in the oracle's float32 operation order (oracle/anerf_oracle.c oracle_near_far)."""
    f = np.float32
    rb = np.asarray(rb, np.float32)
    cy = np.asarray(cyl, np.float32).reshape(-1)
    out = np.zeros(rb.shape[0], bool)
    for i, r in enumerate(rb):
        near, far = r[6], r[7]
        rn0, rn1 = f(r[0] + f(r[3] * near)), f(r[2] + f(r[5] * near))
        rf0, rf1 = f(r[0] + f(r[3] * far)), f(r[2] + f(r[5] * far))
        nc0, nc1 = f(cy[0] - rn0), f(cy[1] - rn1)
        nf0, nf1 = f(rf0 - rn0), f(rf1 - rn1)
        nfn = f(np.sqrt(np.float32(np.float64(nf1) * nf1 + np.float64(f(nf0 * nf0)))))
        dist = f(abs(f(f(nc0 * nf1) - f(nc1 * nf0))) / nfn)
        c = f(f(cy[2] * cy[2]) - f(dist * dist))
        if not c > 0:
            continue
        e = float(np.sqrt(np.float64(c)))
        lo = np.float32(e)
        lo = lo if float(lo) <= e else np.nextafter(lo, f(0))
        ulp = float(np.nextafter(lo, f(np.inf))) - float(lo)
        out[i] = abs((e - float(lo)) / ulp - 0.5) < tol_ulp
    return out


def assert_near_far_z(near, far, z, g, rb, what=""):
    """near / far / coarse z against the reference's stage dumps: bit-exact, except on rays with a
    sqrt near-tie (sqrt_tie_rays, hazard H13), where near / far may differ by one float32 ulp and z by
    what that moves (1e-6 relative)."""
    tie = sqrt_tie_rays(rb, g["cyls"][0])
    for got, ref in ((near, g["stage_near"][:, 0]), (far, g["stage_far"][:, 0])):
        np.testing.assert_array_equal(got[~tie], ref[~tie], err_msg=what)
        if tie.any():
            ulps = np.abs(got[tie].view(np.int32).astype(np.int64) - ref[tie].view(np.int32).astype(np.int64))
            assert ulps.max() <= 1, (what, ulps)
    np.testing.assert_array_equal(z[~tie], g["stage_z"][~tie], err_msg=what)
    if tie.any():
        zr = g["stage_z"][tie]
        assert np.abs(z[tie] - zr).max() <= 1e-6 * np.abs(zr).max(), what
    return int(tie.sum())

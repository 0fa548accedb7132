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
         "pw_64_white_d4w128", "pb_64_bgimg_d4w128"]
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
                                       **kw).validate()
        self.ckpt = syn.make_checkpoint(m["seed"], n_joints=m["NJ"], D=m["D"], W=m["W"], fine=m["I"] > 0,
                                        tau=m["tau"], use_framecode=fc, n_framecodes=5, multires=m.get("mr", 7),
                                        multires_views=m.get("mrv", 4), sched_alpha=m.get("sched"),
                                        cutoff_bones=bool(m.get("cb", False)), tau_bones=m.get("tau_b"))
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

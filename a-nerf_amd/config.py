"""Render-path configuration: the subset of run_nerf.py's flags that shape the kernel.

Mirrors the arguments `create_raycaster` reads (`core/raycasters.py:17-184`) and the
flags listed in SURVEY.md §8b.  Flags whose code paths are not implemented raise
`NotImplementedError` up front (the reference raises `NotImplementedError` for unknown
encoder types too, `core/raycasters.py:238,247,267,283,302`) — never a silent fallback.
"""
from dataclasses import dataclass, field


@dataclass
class RenderConfig:
    n_joints: int = 24
    netdepth: int = 8
    netwidth: int = 256
    skips: tuple = (4,)
    multires: int = 7
    multires_views: int = 4
    multires_bones: int = 0
    use_cutoff: bool = True
    cutoff_inputs: bool = True
    cutoff_viewdir: bool = True
    use_viewdirs: bool = True
    opt_framecode: bool = False
    framecode_size: int = 16
    n_framecodes: int = 0
    density_type: str = "relu"
    softplus_shift: float = 1.0
    density_scale: float = 1.0
    N_samples: int = 64
    N_importance: int = 0
    single_net: bool = False
    lindisp: bool = False  # --lindisp: sample in inverse depth (render_kwargs['lindisp'], ray_utils.py:223-226)
    # --freq_schedule: the cutoff embedders weight frequency k's sin/cos by 0.5 (1 - cos(pi clamp(alpha - k,
    # 0, 1))), alpha = the checkpoint's sched_alpha buffer, moved by update_embed_fns from --init_freq
    # over --freq_schedule_step k-steps (core/cutoff_embedder.py:89-99, 185-197; raycasters.py:731-748)
    freq_schedule: bool = False
    init_freq: float = 0.0
    freq_schedule_step: int = 5
    # --cut_to_dist / --cutoff_shift: the kp cutoff embedder encodes c_j - dist (raw input and
    # frequencies) / feeds (input * 2 / c_j - 1) to the frequencies (core/cutoff_embedder.py:125-134)
    cut_to_dist: bool = False
    cutoff_shift: bool = False
    # --normalize_cutoff reaches CutoffEmbedder only as an unused keyword ("normalize_cutoff", not
    # "normalize": core/raycasters.py:32 vs cutoff_embedder.py:64): a no-op in the reference, and here
    normalize_cutoff: bool = False
    # --cutoff_bones: the bone embedder is a CutoffEmbedder with its own tau / cutoff_dist
    # (core/raycasters.py:52-64, embedbones_state_dict); with multires_bones 0 it multiplies each
    # bone direction by w_b = 1 - sigmoid(tau_b (dist - c_b)) when use_cutoff and cutoff_inputs
    # (cutoff_embedder.py:156-166) and passes it through otherwise
    cutoff_bones: bool = False
    chunk: int = 4096
    ext_scale: float = 0.001
    # MLP arithmetic (include/anerf.h), fp32 accumulation in all: "fp16x4" (the default and bench.py's
    # headline: power-of-two scaled two-way fp16 splits, all four products on the fp16 MFMA pipe,
    # fp32-accurate to bf16x6's error bound), "fp32" (fp32 MFMA everywhere), "bf16x6"
    # (three-way split-bf16, six products, fp32-accurate), "fp16x3" (fp16x4 without x1 w1, 22-bit
    # operands) or "bf16x3" (two-way split-bf16, ~16-bit operands)
    precision: str = "fp16x4"
    extra: dict = field(default_factory=dict)

    def validate(self):
        if not self.use_viewdirs:
            # (the reference itself cannot run this: create_raycaster leaves embeddirs_fn = None
            # (core/raycasters.py:66-67) and encode_inputs calls it (:538) -> TypeError; recorded by
            # tests/golden/probe_reference_flags.py in reference_flags.json)
            raise NotImplementedError("use_viewdirs=False: the reference raises TypeError on this path "
                                      "(core/raycasters.py:67, 538); not implemented")
        if not 0 <= self.multires_bones <= 10:
            raise NotImplementedError(f"multires_bones={self.multires_bones} outside [0, 10]")
        if len(self.skips) != 1 or self.skips[0] < 0:
            # a skip index >= netdepth-1 is never reached (D=4 configs): no skip layer
            raise NotImplementedError(f"skips={self.skips}: exactly one skip index is supported")
        if self.netwidth % 64 != 0 or self.netwidth > 256:
            raise NotImplementedError(f"netwidth={self.netwidth}: multiples of 64 up to 256 are supported")
        if self.netdepth < 2 or self.netdepth > 16:
            raise NotImplementedError(f"netdepth={self.netdepth} outside [2, 16]")
        if not 1 <= self.multires <= 10 or not 0 <= self.multires_views <= 4:
            # (kernel instances for multires 7 / 10 and multires_views 0 / 4; smaller counts run on them with
            # the missing frequencies' weights zero, anerf_pack.hpp layout_multires)
            raise NotImplementedError("multires must be in [1, 10] and multires_views in [0, 4]")
        if self.density_type not in ("relu", "softplus"):
            raise NotImplementedError(f"density activation {self.density_type} is undefined")
        if self.opt_framecode and self.n_framecodes <= 0:
            raise ValueError("opt_framecode needs n_framecodes > 0")
        if self.precision not in ("fp32", "bf16x6", "bf16x3", "fp16x3", "fp16x4"):
            raise ValueError(f"precision={self.precision!r}: 'fp32', 'bf16x6', 'fp16x4', 'fp16x3' or 'bf16x3'")
        if self.n_joints < 1 or self.n_joints > 128:
            raise NotImplementedError(f"n_joints={self.n_joints} outside [1, 128]")
        # encoder selectors (core/raycasters.py:251-305).  The reference itself raises TypeError for
        # kp_dist_type 'cat' (KPCatEncoder's expand, encoders.py:168) and bone_type 'axisang'
        # (IdentityExpandEncoder called without refs, raycasters.py:521), recorded by
        # tests/golden/probe_reference_flags.py in reference_flags.json: the same error here
        if self.extra.get("kp_dist_type") == "cat":
            raise TypeError("--kp_dist_type cat: the reference's KPCatEncoder raises TypeError in expand() "
                            "(core/encoders.py:168)")
        if self.extra.get("bone_type") == "axisang":
            raise TypeError("--bone_type axisang: IdentityExpandEncoder.forward() missing 1 required positional "
                            "argument: 'refs' (core/raycasters.py:521)")
        if self.kp_query and self.bone_window:
            # (the reference's bone CutoffEmbedder gets querypts' cutoff_dim 3 for its 3 NJ inputs and fails in
            # _embed's window broadcast, core/cutoff_embedder.py:139-141)
            raise NotImplementedError("--kp_dist_type querypts with --cutoff_bones fails in the reference's bone "
                                      "embedder (cutoff_dim 3 for 3 NJ inputs)")
        for k, allowed in (("kp_dist_type", ("reldist", "relpos", "querypts")), ("bone_type", ("reldir",)),
                           ("view_type", ("relray", "world", "rayangle")), ("pts_tr_type", ("local",))):
            v = self.extra.get(k, allowed[0])
            if v not in allowed:
                raise NotImplementedError(f"--{k}={v}: only {' / '.join(allowed)} implemented")
        return self

    @property
    def bone_window(self):
        """--cutoff_bones makes the bone embedder a CutoffEmbedder (its state is in the checkpoint)."""
        return bool(self.cutoff_bones and self.use_cutoff)

    @property
    def view_window(self):
        """The view embedder is a CutoffEmbedder (its features windowed by w'_j): --cutoff_viewdir AND --use_cutoff.
        create_raycaster copies cutoff_kwargs, whose "cutoff" is args.use_cutoff, for the view embedder
        (core/raycasters.py:31, 68-71), and get_embedder builds a plain Embedder unless it is set
        (core/cutoff_embedder.py:216-220): without --use_cutoff the view features carry no window."""
        return bool(self.use_viewdirs and self.cutoff_viewdir and self.use_cutoff)

    @property
    def kp_relpos(self):
        """--kp_dist_type relpos (core/encoders.py:124-142): three local coordinates per joint."""
        return self.extra.get("kp_dist_type", "reldist") == "relpos"

    @property
    def kp_query(self):
        """--kp_dist_type querypts (core/raycasters.py:263-265): the world point itself, 3 values."""
        return self.extra.get("kp_dist_type", "reldist") == "querypts"

    @property
    def view_angle(self):
        """--view_type rayangle (core/encoders.py:195-212): one ray angle per joint."""
        return self.extra.get("view_type", "relray") == "rayangle"

    @property
    def staged(self):
        """An encoder the fused render kernel does not stream (bone frequencies, relpos, ray angles,
        include/anerf.h "staged encoders"): the training stages render it (train.TrainRayCaster)."""
        return self.multires_bones > 0 or self.kp_relpos or self.kp_query or self.view_angle

    @property
    def framecode_ch(self):
        return self.framecode_size if self.opt_framecode else 0

    @property
    def input_ch(self):
        if self.kp_query:
            return 3 * (1 + 2 * self.multires)
        return self.n_joints * (3 if self.kp_relpos else 1) * (1 + 2 * self.multires)

    @property
    def input_ch_bones(self):
        return 3 * self.n_joints * (1 + 2 * self.multires_bones)

    @property
    def input_ch_views(self):
        return self.n_joints * (1 if self.view_angle else 3) * (1 + 2 * self.multires_views)

    @property
    def feature_dim(self):
        return self.input_ch + self.input_ch_bones + self.input_ch_views

    @classmethod
    def from_args(cls, args, n_joints):
        """Build from a run_nerf.config_parser() namespace (or anything with those attributes)."""
        g = lambda k, d=None: getattr(args, k, d)  # noqa: E731
        extra = {k: g(k) for k in ("kp_dist_type", "bone_type", "view_type", "pts_tr_type",
                                   "cutoff_mm") if g(k) is not None}
        cfg = cls(n_joints=n_joints, netdepth=g("netdepth", 8), netwidth=g("netwidth", 256),
                  multires=g("multires", 7), multires_views=g("multires_views", 4),
                  multires_bones=g("multires_bones", 0), use_cutoff=bool(g("use_cutoff", True)),
                  cutoff_inputs=bool(g("cutoff_inputs", True)), cutoff_viewdir=bool(g("cutoff_viewdir", True)),
                  use_viewdirs=bool(g("use_viewdirs", True)), opt_framecode=bool(g("opt_framecode", False)),
                  framecode_size=g("framecode_size", 16), n_framecodes=g("n_framecodes", 0) or 0,
                  density_type=g("density_type", "relu"), softplus_shift=g("softplus_shift", 1.0),
                  density_scale=g("density_scale", 1.0), N_samples=g("N_samples", 64),
                  N_importance=g("N_importance", 0), single_net=bool(g("single_net", False)),
                  lindisp=bool(g("lindisp", False)), freq_schedule=bool(g("freq_schedule", False)),
                  init_freq=float(g("init_freq", 0.0) or 0.0), freq_schedule_step=int(g("freq_schedule_step", 5) or 5),
                  cut_to_dist=bool(g("cut_to_dist", False)), cutoff_shift=bool(g("cutoff_shift", False)),
                  normalize_cutoff=bool(g("normalize_cutoff", False)), cutoff_bones=bool(g("cutoff_bones", False)),
                  chunk=g("chunk", 4096), ext_scale=g("ext_scale", 0.001), extra=extra,
                  # (not a reference flag: the drop-in renders in the default precision unless the caller sets it)
                  precision=g("anerf_precision", None) or cls.precision)
        return cfg.validate()


def schedule_weights(alpha, n_freqs):
    """CutoffEmbedder.get_schedule_w (core/cutoff_embedder.py:192-197) in float32: the weight of
    frequency k (its sin and its cos), 0.5 (1 - cos(pi clamp(alpha - k, 0, 1)))."""
    import numpy as np
    import torch
    freq_k = torch.log2(2.0 ** torch.linspace(0.0, n_freqs - 1, steps=n_freqs))
    diff = torch.clamp(torch.as_tensor(np.float32(alpha)) - freq_k, 0, 1)
    return (0.5 * (1.0 - torch.cos(np.pi * diff))).numpy().astype(np.float32)


def feature_scales(cfg, alpha_pts, alpha_views, alpha_bones=None):
    """Per-column factor of the MLP input [x (input_ch) | bones | views] under --freq_schedule: the
    schedule weight of the column's frequency for the windowed sin/cos features of the cutoff
    embedders (a part's frequency slot f = 1 + 2k / 2 + 2k, the sin / cos of frequency k, is the column
    block [f B, (f + 1) B) of the part, B its columns per slot: pts NJ (relpos 3 NJ, querypts 3), bones 3 NJ (a
    CutoffEmbedder with --cutoff_bones, `alpha_bones`), views 3 NJ (rayangle NJ)), 1 elsewhere; None
    without a schedule."""
    import numpy as np
    if not cfg.freq_schedule:
        return None
    nj = cfg.n_joints
    dnet = cfg.input_ch + cfg.input_ch_bones
    s = np.ones(dnet + cfg.input_ch_views, np.float32)

    def part(o, b, n_freq, alpha):
        w = schedule_weights(alpha, n_freq)
        for k in range(n_freq):
            for f in (1 + 2 * k, 2 + 2 * k):
                s[o + f * b:o + (f + 1) * b] = w[k]

    if cfg.use_cutoff:  # (the pts embedder is a CutoffEmbedder only then)
        part(0, 3 if cfg.kp_query else nj * (3 if cfg.kp_relpos else 1), cfg.multires, alpha_pts)
    if cfg.bone_window and cfg.multires_bones > 0:
        if alpha_bones is None:
            raise ValueError("freq_schedule with a windowed bone embedder: its sched_alpha is needed")
        part(cfg.input_ch, 3 * nj, cfg.multires_bones, alpha_bones)
    if cfg.view_window and cfg.multires_views > 0:
        part(dnet, nj * (1 if cfg.view_angle else 3), cfg.multires_views, alpha_views)
    return s


def flops_per_sample(cfg):
    """Reference MLP FLOPs per sample point (2 x MACs of core/networks/nerf.py:133-148)."""
    W, D = cfg.netwidth, cfg.netdepth
    dnet = cfg.input_ch + cfg.input_ch_bones
    macs = dnet * W
    for i in range(D - 1):
        macs += (W + dnet if i in cfg.skips else W) * W
    macs += W * 1 + W * W + (W + cfg.input_ch_views + cfg.framecode_ch) * (W // 2) + (W // 2) * 3
    return 2 * macs


def samples_per_ray(cfg):
    """MLP evaluations per ray: coarse S plus, with importance sampling, all S+I merged samples
    through the fine net (core/raycasters.py:456-461)."""
    S, I = cfg.N_samples, cfg.N_importance
    return S + (S + I if I > 0 else 0)

"""ctypes binding of libanerf_hip.so (the C ABI declared in include/anerf.h).

The library is built in-tree (see build.py).  Importing torch first makes the library's
libamdhip64.so.7 dependency resolve to the HIP runtime torch already loaded, so device
pointers and streams are shared with PyTorch.  There is no fallback: if the library is
missing this module raises.
"""
import ctypes
import os

import torch  # noqa: F401  (must be loaded before the HIP library, see module docstring)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libanerf_hip.so")  # (the in-tree build; the package reads no environment)

MAXL = 16
c_f = ctypes.POINTER(ctypes.c_float)
c_i32p = ctypes.POINTER(ctypes.c_int32)
c_i64p = ctypes.POINTER(ctypes.c_int64)

ANERF_PREC_FP32 = 0
ANERF_PREC_BF16X3 = 1
ANERF_PREC_BF16X6 = 2
ANERF_PREC_FP16X3 = 3
ANERF_PREC_FP16X4 = 4
ANERF_FLAG_LINDISP = 0x100  # OR-ed into the precision argument (include/anerf.h)
ANERF_FLAG_NEAR_FAR = 0x200  # ray_batch columns 6, 7 hold the filled near / far (anerf_render_rays)
MLP_PRECISIONS = {"bf16x3": 3, "fp16x4": 4, "bf16x6": 6}  # ANERF_MLP_* (training MLP GEMMs; fp16x4: forward only)
PRECISIONS = {"fp32": ANERF_PREC_FP32, "bf16x3": ANERF_PREC_BF16X3, "bf16x6": ANERF_PREC_BF16X6,
              "fp16x3": ANERF_PREC_FP16X3, "fp16x4": ANERF_PREC_FP16X4}


ANERF_ENC_CUT_TO_DIST, ANERF_ENC_CUTOFF_SHIFT, ANERF_ENC_CUTOFF_BONES = 1, 2, 4  # anerf_model_desc.encoder_flags
ANERF_ENC_VIEW_RAW = 8  # --view_type world
ANERF_ENC_KP_RELPOS, ANERF_ENC_VIEW_ANGLE = 16, 32  # --kp_dist_type relpos, --view_type rayangle (staged, ABI 15)
ANERF_ENC_KP_QUERYPTS = 64  # --kp_dist_type querypts (staged, ABI 15)
ANERF_ENC_VIEW_WINDOWS = 128  # training layout: the view part as the NJ view windows (ABI 16)
ABI_VERSION = 19  # include/anerf.h ANERF_ABI_VERSION: the structs below


class ModelDesc(ctypes.Structure):
    _fields_ = [("n_joints", ctypes.c_int32), ("net_depth", ctypes.c_int32), ("net_width", ctypes.c_int32),
                ("skip", ctypes.c_int32), ("multires", ctypes.c_int32), ("multires_views", ctypes.c_int32),
                ("use_cutoff", ctypes.c_int32), ("cutoff_inputs", ctypes.c_int32),
                ("cutoff_viewdir", ctypes.c_int32), ("framecode_ch", ctypes.c_int32),
                ("n_framecodes", ctypes.c_int32), ("density_softplus", ctypes.c_int32),
                ("softplus_shift", ctypes.c_float), ("density_scale", ctypes.c_float),
                ("has_fine", ctypes.c_int32), ("single_net", ctypes.c_int32), ("encoder_flags", ctypes.c_int32),
                ("multires_bones", ctypes.c_int32)]


class NetWeights(ctypes.Structure):
    _fields_ = [("pts_w", c_f * MAXL), ("pts_b", c_f * MAXL), ("alpha_w", c_f), ("alpha_b", c_f),
                ("feature_w", c_f), ("feature_b", c_f), ("views_w", c_f), ("views_b", c_f),
                ("rgb_w", c_f), ("rgb_b", c_f), ("codes", c_f)]


class EmbedParams(ctypes.Structure):
    _fields_ = [("cutoff_dist", c_f), ("tau", ctypes.c_float), ("cutoff_dist_v", c_f), ("tau_v", ctypes.c_float),
                ("cutoff_dist_b", c_f), ("tau_b", ctypes.c_float)]


class Debug(ctypes.Structure):
    _fields_ = [("near", c_f), ("far", c_f), ("z_coarse", c_f), ("raw_coarse", c_f), ("weights0", c_f),
                ("z_fine", c_f), ("raw_fine", c_f), ("mfma_count", ctypes.POINTER(ctypes.c_uint64))]


class Seg(ctypes.Structure):
    """anerf_seg: a column segment of a GEMM operand."""
    _fields_ = [("p", ctypes.c_void_p), ("ld", ctypes.c_int64), ("cols", ctypes.c_int32)]


class SplitJob(ctypes.Structure):
    """anerf_split_job: one weight of anerf_mlp_split_weights_batch."""
    _fields_ = [("w", ctypes.c_void_p), ("n", ctypes.c_int32), ("k", ctypes.c_int32), ("ldw", ctypes.c_int64),
                ("transpose", ctypes.c_int32), ("precision", ctypes.c_int32), ("out", ctypes.c_void_p)]


class MlpShape(ctypes.Structure):
    """anerf_mlp_shape (the fused training forward)."""
    _fields_ = [("depth", ctypes.c_int32), ("width", ctypes.c_int32), ("skip", ctypes.c_int32),
                ("dnet", ctypes.c_int32), ("nv", ctypes.c_int32), ("cfc", ctypes.c_int32)]


class MlpFwdWeights(ctypes.Structure):
    """anerf_mlp_fwd_weights."""
    _fields_ = [("pts_w", ctypes.c_void_p * 16), ("pts_ld", ctypes.c_int64 * 16), ("feature_w", ctypes.c_void_p),
                ("views_w", ctypes.c_void_p), ("views_ld", ctypes.c_int64)]


class MlpFwdIO(ctypes.Structure):
    """anerf_mlp_fwd_io."""
    _fields_ = [("m", ctypes.c_int64), ("feat", ctypes.c_void_p), ("ld_feat", ctypes.c_int64),
                ("codes", ctypes.c_void_p), ("ld_codes", ctypes.c_int64), ("pts_b", ctypes.c_void_p * 16),
                ("feature_b", ctypes.c_void_p), ("alpha_w", ctypes.c_void_p), ("alpha_b", ctypes.c_void_p),
                ("views_b", ctypes.c_void_p), ("rgb_w", ctypes.c_void_p), ("rgb_b", ctypes.c_void_p),
                ("h", ctypes.c_void_p * 16), ("hf", ctypes.c_void_p), ("g", ctypes.c_void_p), ("raw", ctypes.c_void_p)]


class OSeg(ctypes.Structure):
    """anerf_oseg: a column segment of a GEMM output (+ relu' mask, accumulate)."""
    _fields_ = [("p", ctypes.c_void_p), ("ld", ctypes.c_int64), ("cols", ctypes.c_int32), ("mask", ctypes.c_void_p),
                ("ldm", ctypes.c_int64), ("accumulate", ctypes.c_int32)]


# name -> (restype, argtypes); must cover every entry point of include/anerf.h
SIGNATURES = {
    "anerf_abi_version": (ctypes.c_int, []),
    "anerf_last_error": (ctypes.c_char_p, []),
    "anerf_model_create": (ctypes.c_int, [ctypes.POINTER(ModelDesc), ctypes.POINTER(NetWeights),
                                          ctypes.POINTER(NetWeights), ctypes.POINTER(EmbedParams), ctypes.c_int,
                                          ctypes.POINTER(ctypes.c_void_p)]),
    "anerf_model_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "anerf_model_set_embed": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(EmbedParams)]),
    "anerf_model_bytes": (ctypes.c_size_t, [ctypes.c_void_p]),
    "anerf_workspace_size": (ctypes.c_size_t, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32]),
    "anerf_render_rays": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                         ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.POINTER(Debug), ctypes.c_void_p, ctypes.c_size_t,
                                         ctypes.c_void_p]),
    "anerf_gen_rays": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_float,
                                      ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_int32,
                                      ctypes.c_void_p, ctypes.c_int64, ctypes.c_float, ctypes.c_float,
                                      ctypes.c_void_p, ctypes.c_void_p]),
    "anerf_near_far": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p,
                                      ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "anerf_encode_points": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]),
    "anerf_gen_rays_box": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_float,
                                          ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_int32,
                                          ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                          ctypes.c_float, ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p]),
    "anerf_compose_box": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32,
                                         ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                         ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "anerf_density_points": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                             ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]),
    "anerf_density_grid": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                           ctypes.c_void_p]),
    "anerf_compose": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "anerf_pose_kinematics": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_int64, ctypes.c_void_p, ctypes.c_float, c_i32p,
                                             ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "anerf_pose_kinematics_backward": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                                      ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_float,
                                                      c_i32p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64,
                                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                      ctypes.c_void_p]),
    "anerf_kp_boxes": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                      ctypes.c_int32, ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "anerf_ray_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                       ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                       ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_void_p]),
    "anerf_gather_rows": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                                         ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p]),
    "anerf_train_samples": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                           ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]),
    "anerf_train_encode": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64,
                                          ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "anerf_train_encode_backward": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64,
                                                   ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32,
                                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                   ctypes.c_void_p, ctypes.c_void_p]),
    "anerf_train_composite": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_int32, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "anerf_train_composite_backward": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                      ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32,
                                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                      ctypes.c_void_p, ctypes.c_void_p]),
    "anerf_train_importance": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                              ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_void_p]),
    "anerf_train_view_factor": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64,
                                               ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_void_p]),
    "anerf_train_view_factor_workspace": (ctypes.c_size_t, [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                                            ctypes.c_int32]),
    "anerf_train_view_factor_backward": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32,
                                                        ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32,
                                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                                        ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                        ctypes.c_size_t, ctypes.c_void_p]),
    "anerf_train_view_mix": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                            ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p]),
    "anerf_train_view_mix_backward": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                                     ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                                     ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                                     ctypes.c_void_p]),
    "anerf_mlp_split_bytes": (ctypes.c_size_t, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]),
    "anerf_mlp_forward_pack_bytes": (ctypes.c_size_t, [ctypes.POINTER(MlpShape)]),
    "anerf_mlp_forward_pack": (ctypes.c_int, [ctypes.POINTER(MlpShape), ctypes.POINTER(MlpFwdWeights),
                                              ctypes.c_void_p, ctypes.c_void_p]),
    "anerf_mlp_forward": (ctypes.c_int, [ctypes.POINTER(MlpShape), ctypes.POINTER(MlpFwdIO), ctypes.c_void_p,
                                         ctypes.c_void_p]),
    "anerf_mlp_split_weights": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64,
                                               ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]),
    "anerf_mlp_split_weights_batch": (ctypes.c_int, [ctypes.POINTER(SplitJob), ctypes.c_int32, ctypes.c_void_p]),
    "anerf_mlp_gemm": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(Seg),
                                      ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                      ctypes.c_int32, ctypes.POINTER(OSeg), ctypes.c_int32, ctypes.c_void_p]),
    "anerf_mlp_gemm_rows": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(Seg),
                                           ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                           ctypes.c_int32, ctypes.POINTER(OSeg), ctypes.c_int32, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_void_p]),
    "anerf_mlp_wgrad_workspace": (ctypes.c_size_t, [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32]),
    "anerf_mlp_backward_hidden_workspace": (ctypes.c_size_t, [ctypes.c_int64, ctypes.c_int32]),
    "anerf_mlp_backward_hidden_reduce": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p, ctypes.c_size_t,
                                                        ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                                        ctypes.c_void_p]),
    "anerf_mlp_backward_hidden": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64,
                                                 ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32,
                                                 ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "anerf_mlp_gemm_persistent": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(Seg),
                                                 ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                                 ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]),
    "anerf_mlp_forward_layer": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int32, ctypes.POINTER(Seg), ctypes.c_int32,
                                               ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32,
                                               ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]),
    "anerf_mlp_forward_hidden": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64,
                                                ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                                ctypes.c_int64, ctypes.c_void_p]),
    "anerf_mlp_backward_head_workspace": (ctypes.c_size_t, [ctypes.c_int64, ctypes.c_int32]),
    "anerf_mlp_backward_head_reduce": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p, ctypes.c_size_t,
                                                      ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                                      ctypes.c_void_p]),
    "anerf_mlp_backward_head": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64,
                                               ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                               ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                               ctypes.c_void_p]),
    "anerf_mlp_wgrad": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                       ctypes.c_int64, ctypes.POINTER(Seg), ctypes.c_int32, ctypes.c_int32,
                                       ctypes.c_void_p,
                                       ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                       ctypes.c_size_t, ctypes.c_void_p]),
}

_lib = None


class AnerfError(RuntimeError):
    pass


def use_library(path):
    """A/B tooling only (tools/_ablib.py, bench.py --lib): load an experiment build of the library instead of
    the in-tree one.  Must run before the first load(); the ABI check below applies to it as to the default."""
    global LIB_PATH
    if _lib is not None and os.path.abspath(path) != os.path.abspath(LIB_PATH):
        raise AnerfError(f"use_library({path!r}) after {LIB_PATH} was loaded")
    LIB_PATH = os.path.abspath(path)


def load():
    """Load libanerf_hip.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise AnerfError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                         "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    cdll = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(cdll, name)
        fn.restype = res
        fn.argtypes = args
    lib = _Checked(cdll)
    if lib.anerf_abi_version() != ABI_VERSION:  # (a stale build would read these structs with another layout)
        raise AnerfError(f"{LIB_PATH} has ABI {lib.anerf_abi_version()}, this binding {ABI_VERSION}: rebuild it")
    _lib = lib
    return lib


class _Checked:
    """The library with every entry point's argument count enforced: ctypes passes surplus arguments of a
    function with argtypes through unchecked (a call with one argument too many shifts the stream handle into
    another slot), so each call is checked against SIGNATURES first."""

    def __init__(self, cdll):
        self._cdll = cdll
        for name, (_, args) in SIGNATURES.items():
            setattr(self, name, self._wrap(getattr(cdll, name), name, len(args)))

    @staticmethod
    def _wrap(fn, name, n):
        def call(*a):
            if len(a) != n:
                raise TypeError(f"{name} takes {n} arguments, got {len(a)}")
            return fn(*a)
        call.__name__ = name
        return call

    def __getattr__(self, name):  # (symbols outside SIGNATURES: the raw ctypes function)
        return getattr(self._cdll, name)


def check(rc, what):
    if rc != 0:
        msg = load().anerf_last_error().decode(errors="replace")
        raise AnerfError(f"{what} failed ({rc}): {msg}")


def ptr(t):
    """Device (or host) pointer of a tensor / None."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def stream_handle(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)

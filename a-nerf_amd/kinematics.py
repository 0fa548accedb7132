"""Pose -> skeleton transforms on the GPU, mirroring the reference's
`PoseOptLayer` forward path (core/pose_opt.py:240-445), `get_kinematic_chain_T`
(core/pose_opt.py:448-479) and `get_smpl_l2ws` (core/utils/skeleton_utils.py:334-376).

All of them reduce to one C-ABI call, `anerf_pose_kinematics` (include/anerf.h): a batched
kinematic chain + inverse that produces the `skts` / `kps` the render path consumes, on the
device, for any number of frames.  It is differentiable: `anerf_pose_kinematics_backward`
(the reference's autograd through the chain and torch.inverse) takes the gradients of
kps / skts / l2ws / rots back to the rotation parameters and the pelvis, so PoseOptLayer is an
nn.Module whose `bones` / `pelvis` (/ `root_bones`) are trained by A-NeRF's pose optimisation
together with the training render path (a-nerf_amd/train.py).

Differences from the reference, by design:
* any tree skeleton up to 128 joints with any root (the reference's PoseOptLayer accepts only
  SMPLSkeleton and `get_smpl_l2ws` assumes root 0 and parents < child);
* float64 arithmetic inside the kernel, float32 outputs (the reference's PoseOptLayer runs in
  float32 torch, get_smpl_l2ws in float64 numpy; both agree with this to float32 rounding);
* `get_smpl_l2ws` needs an explicit rest pose (the SMPL template is not shipped here).
"""
from collections import namedtuple

import numpy as np
import torch

from . import _lib
from .synthetic import SMPL_PARENTS

Skeleton = namedtuple("Skeleton", ["joint_names", "joint_trees", "root_id", "nonroot_id", "cutoffs",
                                   "end_effectors"])

# skeleton_utils.py:83-105 (topology only)
SMPLSkeleton = Skeleton(
    joint_names=["pelvis", "left_hip", "right_hip", "spine1", "left_knee", "right_knee", "spine2", "left_ankle",
                 "right_ankle", "spine3", "left_foot", "right_foot", "neck", "left_collar", "right_collar",
                 "head", "left_shoulder", "right_shoulder", "left_elbow", "right_elbow", "left_wrist",
                 "right_wrist", "left_hand", "right_hand"],
    joint_trees=SMPL_PARENTS.copy(), root_id=0, nonroot_id=list(range(1, 24)), cutoffs={},
    end_effectors=[10, 11, 15, 22, 23])

# skeleton_utils.py:61-81: root 14, parents not ordered by index
CanonicalSkeleton = Skeleton(
    joint_names=["head_top", "neck", "right_shoulder", "right_elbow", "right_wrist", "left_shoulder",
                 "left_elbow", "left_wrist", "right_hip", "right_knee", "right_ankle", "left_hip", "left_knee",
                 "left_ankle", "pelvis", "spine", "head"],
    joint_trees=np.array([1, 15, 1, 2, 3, 1, 5, 6, 14, 8, 9, 14, 11, 12, 14, 14, 1]), root_id=14,
    nonroot_id=[i for i in range(17) if i != 14], cutoffs={}, end_effectors=None)


def _dev_f32(x, device):
    if isinstance(x, torch.Tensor):
        return x.detach().to(device=device, dtype=torch.float32).contiguous()
    return torch.as_tensor(np.ascontiguousarray(x, dtype=np.float32), device=device)


class _Kinematics(torch.autograd.Function):
    """anerf_pose_kinematics with its backward (gradients to bones and pelvis)."""

    @staticmethod
    def forward(ctx, b, pel, rest, ridx, parents, root_id, scale, device, outputs):
        lib = _lib.load()
        F, nj = int(b.shape[0]), int(b.shape[1])
        shapes = {"kps": (F, nj, 3), "skts": (F, nj, 4, 4), "l2ws": (F, nj, 4, 4), "rots": (F, nj, 3, 3)}
        out = {k: torch.empty(shapes[k], dtype=torch.float32, device=device) for k in outputs}
        with torch.cuda.device(device):
            rc = lib.anerf_pose_kinematics(_lib.ptr(b), b.shape[-1], _lib.ptr(rest), _lib.ptr(ridx), rest.shape[0],
                                           _lib.ptr(pel), float(scale), parents.ctypes.data_as(_lib.c_i32p), nj,
                                           int(root_id), F, _lib.ptr(out.get("kps")), _lib.ptr(out.get("skts")),
                                           _lib.ptr(out.get("l2ws")), _lib.ptr(out.get("rots")),
                                           _lib.stream_handle(device))
        _lib.check(rc, "anerf_pose_kinematics")
        ctx.save_for_backward(b, pel if pel is not None else torch.empty(0), rest,
                              ridx if ridx is not None else torch.empty(0))
        ctx.meta = (pel is not None, ridx is not None, parents, root_id, scale, device, tuple(outputs))
        return tuple(out[k] for k in outputs)

    @staticmethod
    def backward(ctx, *grads):
        b, pel, rest, ridx = ctx.saved_tensors
        has_pel, has_ridx, parents, root_id, scale, device, outputs = ctx.meta
        g = {k: (None if gk is None else gk.contiguous()) for k, gk in zip(outputs, grads)}
        gb = torch.empty_like(b)
        gp = torch.empty(b.shape[0], 3, dtype=torch.float32, device=device) if has_pel else None
        lib = _lib.load()
        with torch.cuda.device(device):
            rc = lib.anerf_pose_kinematics_backward(
                _lib.ptr(b), b.shape[-1], _lib.ptr(rest), _lib.ptr(ridx if has_ridx else None), rest.shape[0],
                _lib.ptr(pel if has_pel else None), float(scale), parents.ctypes.data_as(_lib.c_i32p), int(b.shape[1]),
                int(root_id), int(b.shape[0]), _lib.ptr(g.get("kps")), _lib.ptr(g.get("skts")),
                _lib.ptr(g.get("l2ws")), _lib.ptr(g.get("rots")), _lib.ptr(gb), _lib.ptr(gp),
                _lib.stream_handle(device))
        _lib.check(rc, "anerf_pose_kinematics_backward")
        return gb, gp, None, None, None, None, None, None, None


def _dev_index(idx, device):
    """Indices (host array or tensor) -> a device int64 tensor; a device tensor passes through."""
    if isinstance(idx, torch.Tensor):
        return idx.to(device=device, dtype=torch.long).view(-1)
    return torch.as_tensor(np.ascontiguousarray(np.asarray(idx), dtype=np.int64).reshape(-1), device=device)


# PoseOptLayer.calculate_kinematic on DEVICE indices: with at most this many frames every frame's chain runs once
# and the requested rows are gathered on the device -- the same values and, through the gather's backward, the
# same gradients as the reference's np.unique + inverse (pose_opt.py:380-381, 436-442), without taking the indices
# to the host (np.unique) and back (two copies that each wait for the stream to drain, every training step)
ALL_FRAMES_MAX = 8192


def _dev_f32_grad(x, device):
    """float32 contiguous device tensor that keeps the autograd graph of a tensor input."""
    if isinstance(x, torch.Tensor):
        return x.to(device=device, dtype=torch.float32).contiguous()
    return torch.as_tensor(np.ascontiguousarray(x, dtype=np.float32), device=device)


def pose_kinematics(bones, rest_pose, skel_type=SMPLSkeleton, pelvis=None, scale=1.0, rest_idx=None,
                    device=None, outputs=("kps", "skts", "l2ws", "rots")):
    """Batched kinematic chain: bones (F, NJ, 3|6|9) -> dict of float32 device tensors
    kps (F, NJ, 3), skts (F, NJ, 4, 4), l2ws (F, NJ, 4, 4), rots (F, NJ, 3, 3).

    rest_pose (NJ, 3) or (R, NJ, 3) with rest_idx (F,) selecting one per frame; pelvis (F, 3)
    is added to every joint's translation; rest offsets are scaled by `scale`.  Differentiable
    w.r.t. `bones` and `pelvis` when they are tensors that require grad."""
    if device is None:
        device = bones.device if isinstance(bones, torch.Tensor) and bones.is_cuda else torch.device("cuda", 0)
    b = _dev_f32_grad(bones, device)
    if b.dim() != 3 or b.shape[-1] not in (3, 6, 9):
        raise ValueError("bones must be (F, NJ, 3 | 6 | 9)")
    F, nj = int(b.shape[0]), int(b.shape[1])
    rest = _dev_f32(rest_pose, device).reshape(-1, nj, 3)
    ridx = None
    if rest_idx is not None:
        if isinstance(rest_idx, torch.Tensor):
            ridx = rest_idx.to(device=device, dtype=torch.int32).reshape(-1).contiguous()
        else:
            ridx = torch.as_tensor(np.asarray(rest_idx), dtype=torch.int32).to(device).contiguous()
        if ridx.numel() != F:
            raise ValueError("rest_idx must have one entry per frame")
    elif rest.shape[0] != 1:
        if rest.shape[0] != F:
            raise ValueError("rest_pose (R, NJ, 3) needs rest_idx unless R == F")
        ridx = torch.arange(F, dtype=torch.int32, device=device)
    pel = None if pelvis is None else _dev_f32_grad(pelvis, device).reshape(F, 3)
    parents = np.ascontiguousarray(np.asarray(skel_type.joint_trees), dtype=np.int32)
    if parents.shape[0] != nj:
        raise ValueError(f"skeleton has {parents.shape[0]} joints, bones have {nj}")
    outs = _Kinematics.apply(b, pel, rest, ridx, parents, int(skel_type.root_id), float(scale), device,
                             tuple(outputs))
    return dict(zip(outputs, outs))


def get_kinematic_chain_T(rest_pose, bones, skel_type=SMPLSkeleton):
    """pose_opt.py:448-479 -> (kps, bones, skts, l2ws, rots)."""
    o = pose_kinematics(bones, rest_pose, skel_type)
    return o["kps"], bones, o["skts"], o["l2ws"], o["rots"]


def get_smpl_l2ws(pose, rest_pose=None, scale=1.0, skel_type=SMPLSkeleton):
    """skeleton_utils.py:334-376 for one pose (NJ, 3) or a batch (F, NJ, 3): local-to-world 4x4s
    (float32 device tensor, float64 arithmetic)."""
    if rest_pose is None:
        raise ValueError("get_smpl_l2ws: pass rest_pose explicitly (the SMPL template is not shipped)")
    p = pose if isinstance(pose, torch.Tensor) else torch.as_tensor(np.asarray(pose, dtype=np.float32))
    single = p.dim() == 2
    o = pose_kinematics(p[None] if single else p, rest_pose, skel_type, scale=scale, outputs=("l2ws",))
    return o["l2ws"][0] if single else o["l2ws"]


class PoseOptLayer(torch.nn.Module):
    """The reference's PoseOptLayer (core/pose_opt.py:240-445) on the device, trainable: `pelvis`
    (N, 3) and `bones` (N, NJ, 3|6) — with kp_map, `root_bones` (N, 3|6) and the shared per-view
    `bones` (U, NJ-1, 3|6) — are nn.Parameters (pose_opt.py:276-295); calculate_kinematic runs the
    batched chain + inverse with its backward (anerf_pose_kinematics[_backward]).

    kps (N, NJ, 3), bones (N, NJ, 3) axis-angle, rest_pose (1 | R, NJ, 3).  use_rot6d stores the
    6-D parameters (pose_opt.py:284-289)."""

    def __init__(self, kps, bones, rest_pose, skel_type=SMPLSkeleton, kp_map=None, kp_uidxs=None, use_cache=False,
                 use_rot6d=False, beta=None, rest_pose_idxs=None, device=None):
        super().__init__()
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.skel_type = skel_type
        self.root_id = skel_type.root_id
        self.use_cache = use_cache
        self.use_rot6d = use_rot6d
        self.rest_pose_idxs = None if rest_pose_idxs is None else np.asarray(rest_pose_idxs)
        self.beta = beta
        self.register_buffer("rest_pose",
                             _dev_f32(rest_pose, self.device).reshape(-1, len(skel_type.joint_trees), 3))
        kps = _dev_f32(kps, self.device)
        bones = _dev_f32(bones, self.device)
        self.pelvis = torch.nn.Parameter(kps[:, self.root_id].contiguous())
        if use_rot6d:
            nj = bones.shape[1]
            with torch.no_grad():
                rots = pose_kinematics(bones, self.rest_pose[:1], skel_type, outputs=("rots",))["rots"]
            bones = rots[..., :3, :2].reshape(-1, nj, 6).contiguous()
        if kp_map is None:
            self.kp_map = self.kp_uidxs = None
            self.bones = torch.nn.Parameter(bones)
        else:
            self.register_buffer("kp_map", torch.as_tensor(np.asarray(kp_map), dtype=torch.long, device=self.device))
            self.register_buffer("kp_uidxs",
                                 torch.as_tensor(np.asarray(kp_uidxs), dtype=torch.long, device=self.device))
            self.root_bones = torch.nn.Parameter(bones[:, self.root_id].contiguous())
            self.bones = torch.nn.Parameter(bones[self.kp_uidxs, self.root_id + 1:].contiguous())
        self.N_kps = self.pelvis.shape[0]
        if use_cache:
            self.update_cache()

    def idx_to_params(self, idx):
        idx = _dev_index(idx, self.device)
        pelvis = self.pelvis[idx]
        if self.kp_map is None:
            return pelvis, self.bones[idx]
        root = self.root_bones[idx, None, :]
        return pelvis, torch.cat([root, self.bones[self.kp_map[idx]]], dim=1)

    def get_pelvis(self, idx=None):
        return self.idx_to_params(np.arange(self.N_kps) if idx is None else idx)[0]

    def get_rest_pose(self, kp_idxs=None, rest_pose_idxs=None):
        if len(self.rest_pose) == 1:
            return self.rest_pose
        if rest_pose_idxs is not None:
            return self.rest_pose[torch.as_tensor(np.asarray(rest_pose_idxs), device=self.device)]
        return self.rest_pose[torch.as_tensor(self.rest_pose_idxs[np.asarray(kp_idxs)], device=self.device)]

    def calculate_kinematic(self, idxs, rest_pose_idxs=None):
        """-> kp (N, NJ, 3), bone (N, NJ, 3|6), skts (N, NJ, 4, 4), l2ws (N, NJ, 4, 4), rots (N, NJ, 3, 3).
        idxs: a host array (the reference's kp_idx) or a device tensor (a batch already on the device)."""
        if (isinstance(idxs, torch.Tensor) and idxs.device.type != "cpu" and rest_pose_idxs is None
                and self.N_kps <= ALL_FRAMES_MAX):
            g = idxs.to(device=self.device, dtype=torch.long).reshape(-1)
            if self.kp_map is None:
                pelvis, bone = self.pelvis, self.bones
            else:
                pelvis = self.pelvis
                bone = torch.cat([self.root_bones[:, None, :], self.bones[self.kp_map]], dim=1)
            if len(self.rest_pose) == 1 or self.rest_pose_idxs is None:
                ridx = None
            else:
                if getattr(self, "_ridx_all", None) is None or self._ridx_all.device != self.device:
                    self._ridx_all = torch.as_tensor(np.asarray(self.rest_pose_idxs), dtype=torch.int32,
                                                     device=self.device)
                ridx = self._ridx_all
            o = pose_kinematics(bone, self.rest_pose, self.skel_type, pelvis=pelvis, rest_idx=ridx,
                                device=self.device)
            return o["kps"][g], bone[g], o["skts"][g], o["l2ws"][g], o["rots"][g]
        if isinstance(idxs, torch.Tensor):
            idxs = idxs.detach().cpu().numpy()
        if idxs is None:
            idxs = np.arange(self.N_kps)
        idxs = np.atleast_1d(np.asarray(idxs))
        # (as the reference, pose_opt.py:380-381, 436-442: the chain runs once per distinct index -- a training
        # batch names each ray's image -- and the outputs are gathered back in the requested order)
        uniq, inv = np.unique(idxs, return_inverse=True)
        pelvis, bone = self.idx_to_params(uniq)
        if len(self.rest_pose) == 1:
            rest, ridx = self.rest_pose, None
        elif rest_pose_idxs is not None:
            rest, ridx = self.rest_pose, np.asarray(rest_pose_idxs)[np.unique(idxs, return_index=True)[1]]
        else:
            rest, ridx = self.rest_pose, self.rest_pose_idxs[uniq]
        o = pose_kinematics(bone, rest, self.skel_type, pelvis=pelvis, rest_idx=ridx, device=self.device)
        if len(uniq) == len(idxs) and np.array_equal(uniq, idxs):
            return o["kps"], bone, o["skts"], o["l2ws"], o["rots"]
        g = _dev_index(inv, self.device)
        return o["kps"][g], bone[g], o["skts"][g], o["l2ws"][g], o["rots"][g]

    @torch.no_grad()
    def update_cache(self):
        self.cache_kps, self.cache_bones, self.cache_skts, self.cache_l2ws, self.cache_rots = \
            self.calculate_kinematic(np.arange(self.N_kps))

    def forward(self, idxs, rest_pose_idxs=None):
        if not self.use_cache:
            return self.calculate_kinematic(idxs, rest_pose_idxs)
        i = _dev_index(idxs, self.device)
        return self.cache_kps[i], self.cache_bones[i], self.cache_skts[i], self.cache_l2ws[i], self.cache_rots[i]

    def get_bones(self, idx=None):
        if self.use_rot6d:
            raise NotImplementedError("get_bones with use_rot6d needs matrix_to_axis_angle (not on this path)")
        return self.idx_to_params(np.arange(self.N_kps) if idx is None else idx)[1]

"""Deterministic synthetic scenes and seeded NeRF weights for the render path.

The reference renders poses produced by `run_render.load_render_data`
(`/root/reference/run_render.py:116`) from `.h5` datasets and trained `.tar`
checkpoints that are not available offline.  This module produces the same
*kinds* of inputs:

* a SMPL-24-topology skeleton (parent table of `SMPLSkeleton.joint_trees`,
  `core/utils/skeleton_utils.py:98-104`), posed with seeded axis-angle bones and
  chained exactly as `get_smpl_l2ws` does (`skeleton_utils.py:334-376`:
  l2w_root = [R_0 | rest_0], l2w_j = l2w_parent @ [R_j | rest_j - rest_parent]);
* skts = inv(l2ws), kps = l2ws[:, :3, 3] (`skeleton_utils.py:323-332`);
* a SURREAL-style camera (head towards -y, `ray_utils.py:104`);
* NeRF weights with the key layout of `NeRF.state_dict()`
  (`core/networks/nerf.py:57-88`) and the embedder buffers of
  `CutoffEmbedder` (`core/cutoff_embedder.py:91-95`), drawn from
  `numpy.random.default_rng(seed)` so tests regenerate them bit-identically.

The rest pose below is an approximate adult humanoid written for this repo (not
the SMPL template); it only has to look like a person to the bounding cylinder.
"""
import hashlib
import math

import numpy as np

# parent of each joint, SMPL-24 topology (root is its own parent)
SMPL_PARENTS = np.array([0, 0, 0, 0, 1, 2, 3, 4, 5, 6, 7, 8,
                         9, 9, 9, 12, 13, 14, 16, 17, 18, 19, 20, 21], dtype=np.int64)

# approximate humanoid rest joints in metres, y up, x to the subject's left
_REST_M = np.array([
    [0.00, 0.00, 0.00],    # pelvis
    [0.09, -0.09, -0.01],  # left hip
    [-0.09, -0.09, -0.01],  # right hip
    [0.00, 0.11, -0.02],   # spine1
    [0.10, -0.47, -0.01],  # left knee
    [-0.10, -0.47, -0.01],  # right knee
    [0.00, 0.25, -0.02],   # spine2
    [0.09, -0.87, -0.05],  # left ankle
    [-0.09, -0.87, -0.05],  # right ankle
    [0.00, 0.30, 0.01],    # spine3
    [0.11, -0.93, 0.07],   # left foot
    [-0.11, -0.93, 0.07],  # right foot
    [0.00, 0.52, -0.04],   # neck
    [0.08, 0.43, -0.03],   # left collar
    [-0.08, 0.43, -0.03],  # right collar
    [0.00, 0.60, 0.01],    # head
    [0.18, 0.46, -0.03],   # left shoulder
    [-0.18, 0.46, -0.04],  # right shoulder
    [0.44, 0.45, -0.06],   # left elbow
    [-0.44, 0.45, -0.06],  # right elbow
    [0.69, 0.46, -0.06],   # left wrist
    [-0.69, 0.46, -0.06],  # right wrist
    [0.77, 0.45, -0.07],   # left hand
    [-0.77, 0.45, -0.07],  # right hand
], dtype=np.float64)

# scene units: ~2.5 units tall, like the survey's scaled SURREAL rest pose
REST_SCALE = 1.6
REST_POSE_24 = (_REST_M * REST_SCALE).astype(np.float32)


def skeleton(n_joints=24, seed=0):
    """Return (parents, rest_pose) for a 24-joint or extended skeleton.

    Extra joints (n_joints > 24) hang off random earlier joints with N(0, 0.1^2)
    rest offsets (the survey's 65-joint stress skeleton, §8d)."""
    if n_joints == 24:
        return SMPL_PARENTS.copy(), REST_POSE_24.copy()
    if n_joints < 24:
        raise ValueError("n_joints must be >= 24")
    rs = np.random.RandomState(seed)
    parents = list(SMPL_PARENTS)
    rest = [r for r in REST_POSE_24.astype(np.float64)]
    for i in range(n_joints - 24):
        p = int(rs.randint(0, 24 + i))
        parents.append(p)
        rest.append(rest[p] + rs.normal(0.0, 0.1, size=3))
    return np.array(parents, dtype=np.int64), np.array(rest, dtype=np.float32)


def rotvec_to_matrix(rv):
    """Rodrigues formula (what scipy Rotation.from_rotvec().as_matrix() computes)."""
    rv = np.asarray(rv, dtype=np.float64)
    theta = float(np.linalg.norm(rv))
    if theta < 1e-12:
        return np.eye(3)
    k = rv / theta
    K = np.array([[0.0, -k[2], k[1]], [k[2], 0.0, -k[0]], [-k[1], k[0], 0.0]])
    return np.eye(3) + math.sin(theta) * K + (1.0 - math.cos(theta)) * (K @ K)


def pose_l2ws(bones, rest, parents):
    """Local-to-world 4x4 per joint, chained like get_smpl_l2ws (skeleton_utils.py:334-376)."""
    nj = rest.shape[0]
    rest = rest.astype(np.float64)
    l2ws = np.zeros((nj, 4, 4), dtype=np.float64)
    for j in range(nj):
        local = np.eye(4)
        local[:3, :3] = rotvec_to_matrix(bones[j])
        if j == 0:
            local[:3, 3] = rest[0]
            l2ws[0] = local
        else:
            p = int(parents[j])
            local[:3, 3] = rest[j] - rest[p]
            l2ws[j] = l2ws[p] @ local
    return l2ws


def camera_c2w(distance=6.0, yaw=0.0):
    """SURREAL-style camera: at distance along -z looking at the origin, image-up = world -y."""
    base = np.diag([1.0, -1.0, -1.0, 1.0])
    t = np.eye(4)
    t[2, 3] = distance
    c2w = base @ t
    if yaw != 0.0:
        c, s = math.cos(yaw), math.sin(yaw)
        ry = np.array([[c, 0, s, 0], [0, 1, 0, 0], [-s, 0, c, 0], [0, 0, 0, 1.0]])
        c2w = ry @ c2w
    return c2w.astype(np.float32)


def make_scene(n_joints=24, H=512, W=512, seed=0, n_frames=1, yaw_step=0.0,
               bone_std=0.15):
    """Synthetic frames: dict of float32 arrays c2ws (F,4,4), kps (F,NJ,3), skts (F,NJ,4,4),
    bones (F,NJ,3) plus H, W, focal (=1.5 H)."""
    parents, rest = skeleton(n_joints, seed=0)
    c2ws, kps, skts, bones_all = [], [], [], []
    for f in range(n_frames):
        rs = np.random.RandomState(seed + f)
        bones = rs.normal(0.0, bone_std, size=(n_joints, 3))
        bones[0] = [math.pi, 0.0, 0.0]  # head towards -y (SPIN/SURREAL convention)
        l2ws = pose_l2ws(bones, rest, parents)
        kps.append(l2ws[:, :3, 3].astype(np.float32))
        skts.append(np.linalg.inv(l2ws).astype(np.float32))
        bones_all.append(bones.astype(np.float32))
        c2ws.append(camera_c2w(yaw=f * yaw_step))
    return {
        "c2ws": np.stack(c2ws), "kps": np.stack(kps), "skts": np.stack(skts),
        "bones": np.stack(bones_all), "H": int(H), "W": int(W), "focal": 1.5 * H,
        "parents": parents, "rest": rest,
    }


def _linear(rng, n_out, n_in):
    bound = 1.0 / math.sqrt(n_in)
    w = rng.uniform(-bound, bound, size=(n_out, n_in)).astype(np.float32)
    b = rng.uniform(-bound, bound, size=(n_out,)).astype(np.float32)
    return w, b


def nerf_input_dims(n_joints, multires=7, multires_views=4, multires_bones=0, kp_dims=1, view_dims=3, kp_query=False):
    """(input_ch, input_ch_bones, input_ch_views) as create_raycaster derives them
    (core/raycasters.py:24-79, core/cutoff_embedder.py:15-40); kp_dims 3 for --kp_dist_type relpos,
    view_dims 1 for --view_type rayangle."""
    input_ch = (3 if kp_query else n_joints * kp_dims) * (1 + 2 * multires)  # (querypts: the world point)
    input_ch_bones = 3 * n_joints * (1 + 2 * multires_bones)
    input_ch_views = view_dims * n_joints * (1 + 2 * multires_views)
    return input_ch, input_ch_bones, input_ch_views


def make_nerf_state(seed, n_joints=24, D=8, W=256, multires=7, multires_views=4,
                    skips=(4,), use_framecode=False, framecode_ch=16, n_framecodes=0,
                    alpha_bias=2.0, alpha_gain=1.0, rgb_gain=1.0, multires_bones=0, kp_dims=1, view_dims=3,
                    kp_query=False):
    """Seeded NeRF state dict with the key layout of core/networks/nerf.py:57-88."""
    rng = np.random.default_rng(seed)
    input_ch, input_ch_bones, input_ch_views = nerf_input_dims(n_joints, multires, multires_views, multires_bones,
                                                               kp_dims, view_dims, kp_query)
    dnet = input_ch + input_ch_bones
    sd = {}
    w, b = _linear(rng, W, dnet)
    sd["pts_linears.0.weight"], sd["pts_linears.0.bias"] = w, b
    for i in range(D - 1):
        n_in = W + dnet if i in skips else W
        w, b = _linear(rng, W, n_in)
        sd[f"pts_linears.{i + 1}.weight"], sd[f"pts_linears.{i + 1}.bias"] = w, b
    w, b = _linear(rng, 1, W)
    sd["alpha_linear.weight"] = (w * np.float32(alpha_gain)).astype(np.float32)
    sd["alpha_linear.bias"] = np.full((1,), alpha_bias, np.float32)
    vin = input_ch_views + (framecode_ch if use_framecode else 0) + W
    w, b = _linear(rng, W // 2, vin)
    sd["views_linears.0.weight"], sd["views_linears.0.bias"] = w, b
    w, b = _linear(rng, W, W)
    sd["feature_linear.weight"], sd["feature_linear.bias"] = w, b
    w, b = _linear(rng, 3, W // 2)
    sd["rgb_linear.weight"], sd["rgb_linear.bias"] = (w * np.float32(rgb_gain)).astype(np.float32), b
    if use_framecode:
        sd["framecodes.codes.weight"] = rng.normal(0.0, 0.3, size=(n_framecodes, framecode_ch)).astype(np.float32)
    return sd


def make_embed_state(n_joints, cutoff=0.5, tau=20.0, jitter=0.0, seed=0):
    """CutoffEmbedder state: cutoff_dist (NJ,) parameter + tau () buffer."""
    cd = np.full((n_joints,), cutoff, np.float32)
    if jitter:
        cd = (cd + np.random.default_rng(seed).uniform(-jitter, jitter, n_joints)).astype(np.float32)
    return {"cutoff_dist": cd, "tau": np.array(tau, dtype=np.float32)}


def make_checkpoint(seed, n_joints=24, D=8, W=256, fine=True, tau=20.0, tau_views=None,
                    cutoff_jitter=0.05, alpha_bias=0.5, alpha_gain=30.0, rgb_gain=8.0,
                    use_framecode=False, n_framecodes=0, multires=7, multires_views=4, sched_alpha=None,
                    cutoff_bones=False, tau_bones=None, multires_bones=0, kp_dims=1, view_dims=3, kp_query=False):
    """A full RayCaster checkpoint dict with the key layout of RayCaster.state_dict()
    (core/raycasters.py:752-766); sched_alpha: the --freq_schedule buffer of the cutoff embedders
    (core/cutoff_embedder.py:97-99), absent when None; cutoff_bones: the bone embedder is a
    CutoffEmbedder (--cutoff_bones, raycasters.py:52-64) with its own state."""
    ck = {
        "network_fn_state_dict": make_nerf_state(seed, n_joints, D, W, multires, multires_views,
                                                 use_framecode=use_framecode,
                                                 n_framecodes=n_framecodes, alpha_bias=alpha_bias,
                                                 alpha_gain=alpha_gain, rgb_gain=rgb_gain, multires_bones=multires_bones,
                                                 kp_dims=kp_dims, view_dims=view_dims, kp_query=kp_query),
        # (querypts: the kp embedder's cutoff_dim is 3, core/raycasters.py:263-265)
        "embed_state_dict": make_embed_state(3 if kp_query else n_joints, tau=tau, jitter=cutoff_jitter, seed=seed + 101),
        "embedbones_state_dict": {},
        "embeddirs_state_dict": make_embed_state(n_joints, tau=tau if tau_views is None else tau_views,
                                                 jitter=cutoff_jitter, seed=seed + 202),
    }
    if cutoff_bones:
        ck["embedbones_state_dict"] = make_embed_state(n_joints, tau=tau if tau_bones is None else tau_bones,
                                                       jitter=cutoff_jitter, seed=seed + 303)
    if sched_alpha is not None:
        for k in ("embed_state_dict", "embeddirs_state_dict") + (("embedbones_state_dict",) if cutoff_bones else ()):
            ck[k]["sched_alpha"] = np.array(sched_alpha, dtype=np.float32)
    if fine:
        ck["network_fine_state_dict"] = make_nerf_state(seed + 1, n_joints, D, W, multires, multires_views,
                                                        use_framecode=use_framecode,
                                                        n_framecodes=n_framecodes, alpha_bias=alpha_bias,
                                                        alpha_gain=alpha_gain, rgb_gain=rgb_gain,
                                                        multires_bones=multires_bones, kp_dims=kp_dims,
                                                        view_dims=view_dims, kp_query=kp_query)
    return ck


def checkpoint_sha256(ck):
    h = hashlib.sha256()
    for top in sorted(ck):
        for k in sorted(ck[top]):
            h.update(top.encode())
            h.update(k.encode())
            h.update(np.ascontiguousarray(ck[top][k]).tobytes())
    return h.hexdigest()

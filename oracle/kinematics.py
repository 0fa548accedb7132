"""CPU restatement of the reference's pose -> skeleton transforms.  TEST INFRASTRUCTURE ONLY.

Only tests/ import this module (the product path is anerf_pose_kinematics in libanerf_hip.so).
Pinned by tests/golden/kinematics.npz, produced by running the reference's own functions
(tests/golden/make_golden.py:kinematics_table).

Everything is float64 numpy; the device kernel also computes in float64 and rounds the outputs
to float32.

* rotations
  - axis-angle: pytorch3d.transforms.axis_angle_to_matrix as the reference pins it
    (README.md:23, wheel tag pyt190, pytorch3d 0.6 era; skeleton_utils.py:411-412 calls it):
    quaternion (cos(a/2), v sin(a/2)/a) with the small-angle series 0.5 - a^2/48 for |a| < 1e-6,
    then quaternion_to_matrix with two_s = 2/|q|^2.  pytorch3d is absent here, so this branch
    is checked against get_smpl_l2ws (scipy Rotation.from_rotvec, same rotation) instead.
  - 6-D: rot6d_to_rotmat (skeleton_utils.py:420-436): Gram-Schmidt of the two columns of the
    row-major (3,2) parameter, third column = cross product.
  - 3x3 matrices passed through.
* chain: l2w_root = [R_root | s * rest_root];  l2w_j = l2w_parent @ [R_j | s * (rest_j - rest_parent)]
  (get_smpl_l2ws skeleton_utils.py:334-376, calculate_kinematic pose_opt.py:372-445 and its
  unrolled form :482-521 — the same products in the same order), then the pelvis is added to
  every joint's translation (pose_opt.py:426-436); skts = inverse(l2ws) (pose_opt.py:439,
  skeleton_utils.py:330); kps = l2ws[..., :3, 3].
"""
import numpy as np


def axisang_to_rot(v):
    v = np.asarray(v, dtype=np.float64)
    a = np.linalg.norm(v, axis=-1, keepdims=True)
    half = 0.5 * a
    small = np.abs(a) < 1e-6
    with np.errstate(invalid="ignore", divide="ignore"):
        sho = np.where(small, 0.5 - a * a / 48.0, np.sin(half) / np.where(small, 1.0, a))
    q = np.concatenate([np.cos(half), v * sho], axis=-1)
    r, i, j, k = q[..., 0], q[..., 1], q[..., 2], q[..., 3]
    two_s = 2.0 / (q * q).sum(-1)
    o = np.stack([1 - two_s * (j * j + k * k), two_s * (i * j - k * r), two_s * (i * k + j * r),
                  two_s * (i * j + k * r), 1 - two_s * (i * i + k * k), two_s * (j * k - i * r),
                  two_s * (i * k - j * r), two_s * (j * k + i * r), 1 - two_s * (i * i + j * j)], -1)
    return o.reshape(v.shape[:-1] + (3, 3))


def rot6d_to_rot(x):
    x = np.asarray(x, dtype=np.float64).reshape(-1, 3, 2)
    a1, a2 = x[:, :, 0], x[:, :, 1]
    b1 = a1 / np.maximum(np.linalg.norm(a1, axis=-1, keepdims=True), 1e-12)
    c = a2 - (b1 * a2).sum(-1, keepdims=True) * b1
    b2 = c / np.maximum(np.linalg.norm(c, axis=-1, keepdims=True), 1e-12)
    b3 = np.cross(b1, b2)
    return np.stack([b1, b2, b3], axis=-1)


def bones_to_rot(bones):
    bones = np.asarray(bones, dtype=np.float64)
    d = bones.shape[-1]
    lead = bones.shape[:-1] if d != 9 else bones.shape[:-1]
    if d == 3:
        return axisang_to_rot(bones)
    if d == 6:
        return rot6d_to_rot(bones.reshape(-1, 6)).reshape(lead + (3, 3))
    if d == 9:
        return bones.reshape(lead + (3, 3))
    raise ValueError("rotation parameters must have 3, 6 or 9 components")


def kinematic_chain(bones, rest, parents, root_id=0, pelvis=None, scale=1.0):
    """bones (F, NJ, 3|6|9), rest (NJ, 3) or (F, NJ, 3), parents (NJ,) -> kps, skts, l2ws, rots (float64)."""
    rots = bones_to_rot(bones)
    F, nj = rots.shape[:2]
    rest = np.broadcast_to(np.asarray(rest, dtype=np.float64) * scale, (F, nj, 3))
    order = topo_order(parents, root_id)
    l2ws = np.zeros((F, nj, 4, 4))
    for j in order:
        loc = np.zeros((F, 4, 4))
        loc[:, :3, :3] = rots[:, j]
        loc[:, 3, 3] = 1.0
        if j == root_id:
            loc[:, :3, 3] = rest[:, j]
            l2ws[:, j] = loc
        else:
            p = int(parents[j])
            loc[:, :3, 3] = rest[:, j] - rest[:, p]
            l2ws[:, j] = l2ws[:, p] @ loc
    if pelvis is not None:
        l2ws[:, :, :3, 3] += np.asarray(pelvis, dtype=np.float64)[:, None]
    skts = np.linalg.inv(l2ws)
    return l2ws[..., :3, 3].copy(), skts, l2ws, rots


def topo_order(parents, root_id):
    nj = len(parents)
    children = [[] for _ in range(nj)]
    for j in range(nj):
        if j != root_id:
            children[int(parents[j])].append(j)
    order, stack = [], [root_id]
    while stack:
        j = stack.pop(0)
        order.append(j)
        stack.extend(children[j])
    if len(order) != nj:
        raise ValueError("parents do not form a tree rooted at root_id")
    return order

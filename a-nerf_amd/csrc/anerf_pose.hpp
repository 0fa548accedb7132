// anerf_pose.hpp — pose -> skeleton transforms for gfx950.
//
// Restates, for a batch of frames:
//   PoseOptLayer.calculate_kinematic   core/pose_opt.py:372-445 (unrolled chain :482-521)
//   get_kinematic_chain_T              core/pose_opt.py:448-479
//   get_smpl_l2ws (+ inv, pelvis)      core/utils/skeleton_utils.py:296-376
// rotations: axis-angle (pytorch3d axis_angle_to_matrix, via the quaternion, skeleton_utils.py:411),
// 6-D (rot6d_to_rotmat, skeleton_utils.py:420-436) or 3x3 matrices.
//   l2w_root = [R_root | s rest_root],  l2w_j = l2w_parent @ [R_j | s (rest_j - rest_parent)],
//   translation += pelvis,  skts = inverse(l2ws),  kps = l2ws[:3, 3].
//
// One wave per frame; lane j (and j + 64) owns joint j: its rotation, local transform and the
// inverse are computed in parallel, the chain runs level by level of the tree (SMPL-24: 9 levels)
// through a per-wave LDS table of 3x4 transforms.  Arithmetic in float64 (the reference's
// get_smpl_l2ws is float64; the float32 torch path agrees to its own rounding), outputs float32.
#pragma once

namespace anerf {

constexpr int KIN_MAX_JOINTS = 128;
constexpr int KIN_WAVES = 4;

struct KinArgs {
    const float* bones;      // [F][NJ][rot_dim]
    const float* rest;       // [n_rest][NJ][3]
    const int32_t* rest_idx; // [F] or null (rest 0)
    const float* pelvis;     // [F][3] or null
    float* kps;              // [F][NJ][3]   (each output optional)
    float* skts;             // [F][NJ][4][4]
    float* l2ws;             // [F][NJ][4][4]
    float* rots;             // [F][NJ][3][3]
    int64_t n_frames;
    int64_t n_rest;
    float scale;
    int32_t rot_dim;
    int32_t nj;
    int32_t root;
    int32_t max_depth;
    int8_t parent[KIN_MAX_JOINTS];
    uint8_t depth[KIN_MAX_JOINTS];
};

__device__ inline void kin_rotation(const float* p, int rot_dim, double R[9]) {
    if (rot_dim == 3) {
        // axis_angle_to_quaternion + quaternion_to_matrix (pytorch3d)
        const double vx = p[0], vy = p[1], vz = p[2];
        const double a = sqrt(vx * vx + vy * vy + vz * vz);
        const double half = 0.5 * a;
        const double sho = (a < 1e-6) ? 0.5 - a * a / 48.0 : sin(half) / a;
        const double r = cos(half), i = vx * sho, j = vy * sho, k = vz * sho;
        const double two_s = 2.0 / (r * r + i * i + j * j + k * k);
        R[0] = 1.0 - two_s * (j * j + k * k); R[1] = two_s * (i * j - k * r); R[2] = two_s * (i * k + j * r);
        R[3] = two_s * (i * j + k * r); R[4] = 1.0 - two_s * (i * i + k * k); R[5] = two_s * (j * k - i * r);
        R[6] = two_s * (i * k - j * r); R[7] = two_s * (j * k + i * r); R[8] = 1.0 - two_s * (i * i + j * j);
    } else if (rot_dim == 6) {
        // columns a1 = (p0, p2, p4), a2 = (p1, p3, p5) of the row-major (3, 2) parameter
        const double a1x = p[0], a1y = p[2], a1z = p[4], a2x = p[1], a2y = p[3], a2z = p[5];
        const double n1 = fmax(sqrt(a1x * a1x + a1y * a1y + a1z * a1z), 1e-12);
        const double b1x = a1x / n1, b1y = a1y / n1, b1z = a1z / n1;
        const double d = b1x * a2x + b1y * a2y + b1z * a2z;
        const double cx = a2x - d * b1x, cy = a2y - d * b1y, cz = a2z - d * b1z;
        const double n2 = fmax(sqrt(cx * cx + cy * cy + cz * cz), 1e-12);
        const double b2x = cx / n2, b2y = cy / n2, b2z = cz / n2;
        const double b3x = b1y * b2z - b1z * b2y, b3y = b1z * b2x - b1x * b2z, b3z = b1x * b2y - b1y * b2x;
        R[0] = b1x; R[1] = b2x; R[2] = b3x;
        R[3] = b1y; R[4] = b2y; R[5] = b3y;
        R[6] = b1z; R[7] = b2z; R[8] = b3z;
    } else {
#pragma unroll
        for (int e = 0; e < 9; ++e) R[e] = p[e];
    }
}

__global__ __launch_bounds__(64 * KIN_WAVES) void pose_kinematics_kernel(KinArgs a) {
    extern __shared__ double kin_lds[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t f = (int64_t)blockIdx.x * KIN_WAVES + wave;
    if (f >= a.n_frames) return;  // the whole wave leaves; waves never wait for each other
    const int nj = a.nj;
    double* T = kin_lds + (size_t)wave * nj * 12;  // 3x4 transforms, row-major
    int64_t ri = a.rest_idx ? (int64_t)a.rest_idx[f] : 0;
    const bool bad = ri < 0 || ri >= a.n_rest;
    if (bad) ri = 0;
    const float* rest = a.rest + ri * nj * 3;
    const double s = a.scale;

    double R[2][9], t[2][3];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int j = lane + 64 * h;
        if (j < nj) {
            kin_rotation(a.bones + (f * nj + j) * a.rot_dim, a.rot_dim, R[h]);
            const int p = a.parent[j];
#pragma unroll
            for (int c = 0; c < 3; ++c)
                t[h][c] = (j == a.root) ? s * (double)rest[3 * j + c]
                                        : s * (double)rest[3 * j + c] - s * (double)rest[3 * p + c];
        }
    }
    for (int d = 0; d <= a.max_depth; ++d) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int j = lane + 64 * h;
            if (j < nj && a.depth[j] == d) {
                double* o = T + j * 12;
                if (d == 0) {
#pragma unroll
                    for (int r = 0; r < 3; ++r) {
                        o[4 * r + 0] = R[h][3 * r + 0];
                        o[4 * r + 1] = R[h][3 * r + 1];
                        o[4 * r + 2] = R[h][3 * r + 2];
                        o[4 * r + 3] = t[h][r];
                    }
                } else {
                    const double* P = T + a.parent[j] * 12;
#pragma unroll
                    for (int r = 0; r < 3; ++r) {
                        const double p0 = P[4 * r], p1 = P[4 * r + 1], p2 = P[4 * r + 2], p3 = P[4 * r + 3];
#pragma unroll
                        for (int c = 0; c < 3; ++c) o[4 * r + c] = p0 * R[h][c] + p1 * R[h][3 + c] + p2 * R[h][6 + c];
                        o[4 * r + 3] = p0 * t[h][0] + p1 * t[h][1] + p2 * t[h][2] + p3;
                    }
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    const double nanv = __builtin_nan("");
    double pel[3] = {0.0, 0.0, 0.0};
    if (a.pelvis)
#pragma unroll
        for (int c = 0; c < 3; ++c) pel[c] = a.pelvis[f * 3 + c];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int j = lane + 64 * h;
        if (j >= nj) continue;
        double M[12];
#pragma unroll
        for (int e = 0; e < 12; ++e) M[e] = bad ? nanv : T[j * 12 + e];
        M[3] += pel[0];
        M[7] += pel[1];
        M[11] += pel[2];
        const int64_t fj = f * nj + j;
        if (a.l2ws) {
            float* o = a.l2ws + fj * 16;
#pragma unroll
            for (int e = 0; e < 12; ++e) o[e] = (float)M[e];
            o[12] = 0.0f; o[13] = 0.0f; o[14] = 0.0f; o[15] = 1.0f;
        }
        if (a.kps) {
            a.kps[fj * 3 + 0] = (float)M[3];
            a.kps[fj * 3 + 1] = (float)M[7];
            a.kps[fj * 3 + 2] = (float)M[11];
        }
        if (a.rots) {
#pragma unroll
            for (int e = 0; e < 9; ++e) a.rots[fj * 9 + e] = bad ? __builtin_nanf("") : (float)R[h][e];
        }
        if (a.skts) {
            // inverse of [A t; 0 1] = [A^-1, -A^-1 t; 0 1], A^-1 = adj(A) / det(A)
            const double a00 = M[0], a01 = M[1], a02 = M[2], a10 = M[4], a11 = M[5], a12 = M[6];
            const double a20 = M[8], a21 = M[9], a22 = M[10];
            const double c00 = a11 * a22 - a12 * a21, c01 = a02 * a21 - a01 * a22, c02 = a01 * a12 - a02 * a11;
            const double c10 = a12 * a20 - a10 * a22, c11 = a00 * a22 - a02 * a20, c12 = a02 * a10 - a00 * a12;
            const double c20 = a10 * a21 - a11 * a20, c21 = a01 * a20 - a00 * a21, c22 = a00 * a11 - a01 * a10;
            const double inv = 1.0 / (a00 * c00 + a01 * c10 + a02 * c20);
            const double I[9] = {c00 * inv, c01 * inv, c02 * inv, c10 * inv, c11 * inv, c12 * inv,
                                 c20 * inv, c21 * inv, c22 * inv};
            float* o = a.skts + fj * 16;
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                o[4 * r + 0] = (float)I[3 * r + 0];
                o[4 * r + 1] = (float)I[3 * r + 1];
                o[4 * r + 2] = (float)I[3 * r + 2];
                o[4 * r + 3] = (float)(-(I[3 * r] * M[3] + I[3 * r + 1] * M[7] + I[3 * r + 2] * M[11]));
            }
            o[12] = 0.0f; o[13] = 0.0f; o[14] = 0.0f; o[15] = 1.0f;
        }
    }
}

}  // namespace anerf

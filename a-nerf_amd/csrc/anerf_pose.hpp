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

__device__ __forceinline__ void kin_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

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

// Rotations, local offsets and the chain of frame f into T (3x4 per joint, this wave's LDS slice):
// lane j (and j + 64) owns joint j; the chain runs level by level of the tree.
__device__ inline void kin_chain(const KinArgs& a, int64_t f, int lane, double* T, double (&R)[2][9],
                                 double (&t)[2][3], bool& bad) {
    const int nj = a.nj;
    int64_t ri = a.rest_idx ? (int64_t)a.rest_idx[f] : 0;
    bad = ri < 0 || ri >= a.n_rest;
    if (bad) ri = 0;
    const float* rest = a.rest + ri * nj * 3;
    const double s = a.scale;
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
        kin_wave_sync();
    }
}

__global__ __launch_bounds__(64 * KIN_WAVES) void pose_kinematics_kernel(KinArgs a) {
    extern __shared__ double kin_lds[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t f = (int64_t)blockIdx.x * KIN_WAVES + wave;
    if (f >= a.n_frames) return;  // the whole wave leaves; waves never wait for each other
    const int nj = a.nj;
    double* T = kin_lds + (size_t)wave * nj * 12;  // 3x4 transforms, row-major
    double R[2][9], t[2][3];
    bool bad;
    kin_chain(a, f, lane, T, R, t, bad);
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


// ======================================================================= backward
// Gradient of the rotation parametrisations: dL/dp (rot_dim values) from dL/dR (row-major 3x3),
// the reverse of kin_rotation (pytorch3d's axis-angle -> quaternion -> matrix with two_s = 2/|q|^2,
// rot6d_to_rotmat's Gram-Schmidt with F.normalize's eps, identity for matrices).
__device__ inline void kin_rotation_grad(const float* p, int rot_dim, const double gR[9], double* gp) {
    if (rot_dim == 3) {
        const double vx = p[0], vy = p[1], vz = p[2];
        const double a = sqrt(vx * vx + vy * vy + vz * vz);
        const double h = 0.5 * a;
        const bool small = a < 1e-6;
        const double sho = small ? 0.5 - a * a / 48.0 : sin(h) / a;
        const double r = cos(h), i = vx * sho, j = vy * sho, k = vz * sho;
        const double s = 2.0 / (r * r + i * i + j * j + k * k);
        const double gs = -gR[0] * (j * j + k * k) + gR[1] * (i * j - k * r) + gR[2] * (i * k + j * r) +
                          gR[3] * (i * j + k * r) - gR[4] * (i * i + k * k) + gR[5] * (j * k - i * r) +
                          gR[6] * (i * k - j * r) + gR[7] * (j * k + i * r) - gR[8] * (i * i + j * j);
        double gr = s * (-gR[1] * k + gR[2] * j + gR[3] * k - gR[5] * i - gR[6] * j + gR[7] * i);
        double gi = s * (gR[1] * j + gR[2] * k + gR[3] * j - 2.0 * gR[4] * i - gR[5] * r + gR[6] * k + gR[7] * r -
                         2.0 * gR[8] * i);
        double gj = s * (-2.0 * gR[0] * j + gR[1] * i + gR[2] * r + gR[3] * i + gR[5] * k - gR[6] * r + gR[7] * k -
                         2.0 * gR[8] * j);
        double gk = s * (-2.0 * gR[0] * k - gR[1] * r + gR[2] * i + gR[3] * r - 2.0 * gR[4] * k + gR[5] * j +
                         gR[6] * i + gR[7] * j);
        const double cs = -gs * s * s;  // s = 2 / |q|^2: ds/dq = -s^2 q
        gr += cs * r;
        gi += cs * i;
        gj += cs * j;
        gk += cs * k;
        double ga = -0.5 * sin(h) * gr;  // r = cos(a / 2)
        const double dsho = small ? -a / 24.0 : (0.5 * cos(h) * a - sin(h)) / (a * a);
        ga += (gi * vx + gj * vy + gk * vz) * dsho;
        gp[0] = gi * sho;
        gp[1] = gj * sho;
        gp[2] = gk * sho;
        if (a > 0.0) {
            gp[0] += ga * vx / a;
            gp[1] += ga * vy / a;
            gp[2] += ga * vz / a;
        }
    } else if (rot_dim == 6) {
        const double a1[3] = {p[0], p[2], p[4]}, a2[3] = {p[1], p[3], p[5]};
        const double n1r = sqrt(a1[0] * a1[0] + a1[1] * a1[1] + a1[2] * a1[2]);
        const double n1 = fmax(n1r, 1e-12);
        const double b1[3] = {a1[0] / n1, a1[1] / n1, a1[2] / n1};
        const double d = b1[0] * a2[0] + b1[1] * a2[1] + b1[2] * a2[2];
        const double c[3] = {a2[0] - d * b1[0], a2[1] - d * b1[1], a2[2] - d * b1[2]};
        const double n2r = sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
        const double n2 = fmax(n2r, 1e-12);
        const double b2[3] = {c[0] / n2, c[1] / n2, c[2] / n2};
        double gb1[3] = {gR[0], gR[3], gR[6]}, gb2[3] = {gR[1], gR[4], gR[7]};
        const double gb3[3] = {gR[2], gR[5], gR[8]};
        // b3 = b1 x b2: dL/db1 += b2 x g3, dL/db2 += g3 x b1
        gb1[0] += b2[1] * gb3[2] - b2[2] * gb3[1];
        gb1[1] += b2[2] * gb3[0] - b2[0] * gb3[2];
        gb1[2] += b2[0] * gb3[1] - b2[1] * gb3[0];
        gb2[0] += gb3[1] * b1[2] - gb3[2] * b1[1];
        gb2[1] += gb3[2] * b1[0] - gb3[0] * b1[2];
        gb2[2] += gb3[0] * b1[1] - gb3[1] * b1[0];
        double gc[3];
        if (n2r > 1e-12) {
            const double dot = b2[0] * gb2[0] + b2[1] * gb2[1] + b2[2] * gb2[2];
            for (int e = 0; e < 3; ++e) gc[e] = (gb2[e] - b2[e] * dot) / n2r;
        } else {
            for (int e = 0; e < 3; ++e) gc[e] = gb2[e] / 1e-12;
        }
        double ga2[3] = {gc[0], gc[1], gc[2]};
        const double gd = -(gc[0] * b1[0] + gc[1] * b1[1] + gc[2] * b1[2]);
        for (int e = 0; e < 3; ++e) {
            gb1[e] += -d * gc[e] + gd * a2[e];
            ga2[e] += gd * b1[e];
        }
        double ga1[3];
        if (n1r > 1e-12) {
            const double dot = b1[0] * gb1[0] + b1[1] * gb1[1] + b1[2] * gb1[2];
            for (int e = 0; e < 3; ++e) ga1[e] = (gb1[e] - b1[e] * dot) / n1r;
        } else {
            for (int e = 0; e < 3; ++e) ga1[e] = gb1[e] / 1e-12;
        }
        gp[0] = ga1[0]; gp[2] = ga1[1]; gp[4] = ga1[2];
        gp[1] = ga2[0]; gp[3] = ga2[1]; gp[5] = ga2[2];
    } else {
#pragma unroll
        for (int e = 0; e < 9; ++e) gp[e] = gR[e];
    }
}

struct KinGradArgs {
    const float* g_kps;   // [F][NJ][3]      (each optional)
    const float* g_skts;  // [F][NJ][4][4]
    const float* g_l2ws;  // [F][NJ][4][4]
    const float* g_rots;  // [F][NJ][3][3]
    float* g_bones;       // [F][NJ][rot_dim]
    float* g_pelvis;      // [F][3] or null
};

constexpr int KINB_WAVES = 2;

// Reverse of pose_kinematics_kernel for one frame per wave: the chain is recomputed (kin_chain),
// each joint's world transform M gets dL/dM from its outputs (skts = inverse(M): dL/dM =
// -S^T G S^T, torch.inverse's gradient; kps = M[:3, 3]; l2ws = M), the pelvis collects every
// joint's translation gradient, and the chain is walked back deepest level first:
//   M_j = M_p L_j  =>  dL/dA_p += dL/dA_j R_j^T + dL/db_j t_j^T,  dL/db_p += dL/db_j,
//                      dL/dR_j = A_p^T dL/dA_j;   root: dL/dR = dL/dA.
// Per-child contributions go through LDS and each parent sums its children (no atomics).
__global__ __launch_bounds__(64 * KINB_WAVES) void pose_kinematics_backward_kernel(KinArgs a, KinGradArgs g) {
    extern __shared__ double kin_lds[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t f = (int64_t)blockIdx.x * KINB_WAVES + wave;
    if (f >= a.n_frames) return;
    const int nj = a.nj;
    double* T = kin_lds + (size_t)wave * nj * 36;  // forward 3x4 | gradient 3x4 | child contribution 3x4
    double* Gm = T + nj * 12;
    double* C = T + nj * 24;
    double R[2][9], t[2][3];
    bool bad;
    kin_chain(a, f, lane, T, R, t, bad);
    double pel[3] = {0.0, 0.0, 0.0};
    if (a.pelvis)
        for (int c = 0; c < 3; ++c) pel[c] = a.pelvis[f * 3 + c];
    double gpel[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int j = lane + 64 * h;
        if (j >= nj) continue;
        const int64_t fj = f * nj + j;
        double gM[12];
        for (int e = 0; e < 12; ++e) gM[e] = g.g_l2ws ? (double)g.g_l2ws[fj * 16 + e] : 0.0;
        if (g.g_kps)
            for (int r = 0; r < 3; ++r) gM[4 * r + 3] += g.g_kps[fj * 3 + r];
        if (g.g_skts) {
            double M[12];
            for (int e = 0; e < 12; ++e) M[e] = T[j * 12 + e];
            M[3] += pel[0];
            M[7] += pel[1];
            M[11] += pel[2];
            const double a00 = M[0], a01 = M[1], a02 = M[2], a10 = M[4], a11 = M[5], a12 = M[6];
            const double a20 = M[8], a21 = M[9], a22 = M[10];
            const double c00 = a11 * a22 - a12 * a21, c01 = a02 * a21 - a01 * a22, c02 = a01 * a12 - a02 * a11;
            const double c10 = a12 * a20 - a10 * a22, c11 = a00 * a22 - a02 * a20, c12 = a02 * a10 - a00 * a12;
            const double c20 = a10 * a21 - a11 * a20, c21 = a01 * a20 - a00 * a21, c22 = a00 * a11 - a01 * a10;
            const double inv = 1.0 / (a00 * c00 + a01 * c10 + a02 * c20);
            double S[16];  // inverse(M), 4x4
            const double I[9] = {c00 * inv, c01 * inv, c02 * inv, c10 * inv, c11 * inv, c12 * inv,
                                 c20 * inv, c21 * inv, c22 * inv};
            for (int r = 0; r < 3; ++r) {
                S[4 * r + 0] = I[3 * r + 0];
                S[4 * r + 1] = I[3 * r + 1];
                S[4 * r + 2] = I[3 * r + 2];
                S[4 * r + 3] = -(I[3 * r] * M[3] + I[3 * r + 1] * M[7] + I[3 * r + 2] * M[11]);
            }
            S[12] = 0.0; S[13] = 0.0; S[14] = 0.0; S[15] = 1.0;
            const float* Gs = g.g_skts + fj * 16;
            double X[16];  // G S^T
            for (int r = 0; r < 4; ++r)
                for (int c = 0; c < 4; ++c) {
                    double v = 0.0;
                    for (int k = 0; k < 4; ++k) v += (double)Gs[4 * r + k] * S[4 * c + k];
                    X[4 * r + c] = v;
                }
            for (int r = 0; r < 3; ++r)  // -(S^T X), rows 0..2
                for (int c = 0; c < 4; ++c) {
                    double v = 0.0;
                    for (int k = 0; k < 4; ++k) v += S[4 * k + r] * X[4 * k + c];
                    gM[4 * r + c] -= v;
                }
        }
        for (int e = 0; e < 12; ++e) Gm[j * 12 + e] = gM[e];
        gpel[0] += gM[3];
        gpel[1] += gM[7];
        gpel[2] += gM[11];
    }
    kin_wave_sync();
    double gR[2][9];
    for (int h = 0; h < 2; ++h)
        for (int e = 0; e < 9; ++e) gR[h][e] = 0.0;
    for (int d = a.max_depth; d >= 0; --d) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int j = lane + 64 * h;
            if (j >= nj || a.depth[j] != d) continue;
            const double* G = Gm + j * 12;  // complete: all children were added at level d + 1
            if (d == 0) {
                for (int r = 0; r < 3; ++r)
                    for (int c = 0; c < 3; ++c) gR[h][3 * r + c] = G[4 * r + c];
                continue;
            }
            const double* P = T + a.parent[j] * 12;
            for (int r = 0; r < 3; ++r)  // dL/dR_j = A_p^T dL/dA_j
                for (int c = 0; c < 3; ++c)
                    gR[h][3 * r + c] = P[r] * G[c] + P[4 + r] * G[4 + c] + P[8 + r] * G[8 + c];
            double* Cj = C + j * 12;
            for (int r = 0; r < 3; ++r) {
                for (int c = 0; c < 3; ++c)  // dL/dA_j R_j^T + dL/db_j t_j^T
                    Cj[4 * r + c] = G[4 * r] * R[h][3 * c] + G[4 * r + 1] * R[h][3 * c + 1] +
                                    G[4 * r + 2] * R[h][3 * c + 2] + G[4 * r + 3] * t[h][c];
                Cj[4 * r + 3] = G[4 * r + 3];
            }
        }
        kin_wave_sync();
        if (d > 0) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int p = lane + 64 * h;
                if (p >= nj || a.depth[p] != d - 1) continue;
                for (int c = 0; c < nj; ++c) {
                    if (c == a.root || a.parent[c] != p || a.depth[c] != d) continue;
                    for (int e = 0; e < 12; ++e) Gm[p * 12 + e] += C[c * 12 + e];
                }
            }
            kin_wave_sync();
        }
    }
    const double nanv = __builtin_nan("");
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int j = lane + 64 * h;
        if (j >= nj) continue;
        const int64_t fj = f * nj + j;
        if (g.g_rots)
            for (int e = 0; e < 9; ++e) gR[h][e] += g.g_rots[fj * 9 + e];
        double gp[9];
        kin_rotation_grad(a.bones + fj * a.rot_dim, a.rot_dim, gR[h], gp);
        for (int e = 0; e < a.rot_dim; ++e) g.g_bones[fj * a.rot_dim + e] = bad ? (float)nanv : (float)gp[e];
    }
    if (g.g_pelvis) {
        for (int c = 0; c < 3; ++c) {
            double v = gpel[c];
            for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
            if (lane == 0) g.g_pelvis[f * 3 + c] = bad ? (float)nanv : (float)v;
        }
    }
}

}  // namespace anerf

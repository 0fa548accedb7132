// anerf_train.hpp — training-mode stages of RayCaster.render_rays: stratified
// samples, the encoder forward and backward (gradient to the skeleton transforms, i.e. to the pose
// optimisation), raw2outputs forward and backward, and stochastic importance sampling.  The MLP
// between them runs on the hand-written split-bf16 GEMMs of anerf_gemm.hip (a-nerf_amd/mlp.py).
// Random numbers are inputs (t_rand, noise, u), so a caller can feed the reference's draws.
// Part of the single translation unit anerf_render.hip (included there, in order).
#pragma once

// sample_from_lineseg with perturb > 0 (core/utils/ray_utils.py:204-251): z = linspace between
// near and far, then lower + (upper - lower) * t_rand inside the mid-point intervals.  t_rand NULL:
// the deterministic samples (perturb = 0).  One thread per sample.
__global__ void train_z_kernel(const float* __restrict__ nearp, const float* __restrict__ farp, int64_t n, int S,
                               const float* __restrict__ t_rand, int lindisp, float* __restrict__ z) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= n * S) return;
    const int64_t i = idx / S;
    const int s = (int)(idx % S);
    const float nr = nearp[i], fr = farp[i];
    auto zl = [&](int k) {
        return lineseg_z(nr, fr, torch_linspace01(k, S), lindisp != 0);
    };
    const float zs = zl(s);
    float zv = zs;
    if (t_rand) {
        const float upper = s + 1 < S ? 0.5f * (zl(s + 1) + zs) : zs;
        const float lower = s > 0 ? 0.5f * (zs + zl(s - 1)) : zs;
        zv = lower + (upper - lower) * t_rand[idx];
    }
    z[idx] = zv;
}

// Feature-row layout of a model (anerf.h, "staged encoders"): per-joint kp dims (1 reldist / 3 relpos), per-joint
// view dims (3 relray / world, 1 rayangle), the bone and view parts' first columns and the row width.  Column of
// feature (frequency slot f, joint j, component c) in a part: part + (f NJ + j) dims + c.
struct FeatLayout {
    int nkp, nvw, cb, cv, F;
};
__host__ __device__ inline FeatLayout feat_layout(const ModelDev& M) {
    FeatLayout L;
    L.nkp = M.kp_relpos ? 3 : 1;
    L.nvw = M.view_angle ? 1 : 3;
    L.cb = (M.kp_query ? 3 : M.nj * L.nkp) * (1 + 2 * M.mr);  // (querypts: the point's 3 coordinates)
    L.cv = L.cb + 3 * M.nj * (1 + 2 * M.mrb);
    L.F = L.cv + (M.view_win ? M.nj : M.nj * L.nvw * (1 + 2 * M.mrv));  // (ANERF_ENC_VIEW_WINDOWS: the windows)
    return L;
}

// RayAngEncoder's input (core/encoders.py:195-212 -> skeleton_utils.py:594-605): the angle between the local point
// q and the local ray direction e, acos(clamp(q.e / (|q| |e|), -1 + 1e-6, 1 - 1e-6)) - pi / 2; also the cosine
__device__ __forceinline__ float ray_angle(float qx, float qy, float qz, float ex, float ey, float ez, float& cs) {
    const float dot = qx * ex + qy * ey + qz * ez;  // ((a * b).sum(-1): elementwise products, then the sum)
    cs = dot / (norm3(qx, qy, qz) * norm3(ex, ey, ez));
    const float cl = fminf(fmaxf(cs, -1.0f + 1e-6f), 1.0f - 1e-6f);
    return acosf(cl) - 1.5707963267948966f;
}

// encode_inputs over a ray batch: sample s of ray i at p = o + d z (sample_pts,
// raycasters.py:650-663), pose ray_pose[i] (or i when per_ray), feature row [v | r | d] of
// encode_row.  One thread per (sample, joint): consecutive lanes are consecutive joints, so every
// feature k (layout k NJ + j) is written by contiguous lanes.  Staged encoders (anerf.h): relpos kp
// inputs, bone frequencies and ray angles in the same row layout (feat_layout).
__device__ __forceinline__ void encode_joint(const ModelDev& M, const float* __restrict__ S, int j, float px,
                                             float py, float pz, float dx, float dy, float dz, float* __restrict__ f) {
    const int nj = M.nj;
    const FeatLayout L = feat_layout(M);
    float qx, qy, qz;
    joint_local(S, px, py, pz, qx, qy, qz);
    const float dist = norm3(qx, qy, qz);
    const float dn = fmaxf(dist, 1e-12f);
    const float w = M.use_cutoff ? cutoff_w(M.tau, dist, M.cutoff[j]) : 1.0f;
    if (M.kp_query) {  // querypts: joint-threads 0..2 write world coordinate c = j, windowed by itself
        if (j < 3) {
            const float x = j == 0 ? px : (j == 1 ? py : pz);
            const float wq = M.use_cutoff ? cutoff_w(M.tau, x, M.cutoff[j]) : 1.0f;
            float u, uf;
            kp_inputs(M.cut_to, M.shift_in, x, M.cutoff[j], u, uf);
            f[j] = (M.use_cutoff && M.cutoff_inputs) ? u * wq : u;
            for (int fi = 0; fi < M.mr; ++fi) {
                float s, c;
                sincos_rr(uf * (float)(1 << fi), s, c);
                f[3 * (1 + 2 * fi) + j] = s * wq;
                f[3 * (2 + 2 * fi) + j] = c * wq;
            }
        }
    } else if (!M.kp_relpos) {
        float u, uf;
        kp_inputs(M.cut_to, M.shift_in, dist, M.cutoff[j], u, uf);
        f[j] = (M.use_cutoff && M.cutoff_inputs) ? u * w : u;
        for (int fi = 0; fi < M.mr; ++fi) {
            float s, c;
            sincos_rr(uf * (float)(1 << fi), s, c);
            f[(1 + 2 * fi) * nj + j] = s * w;
            f[(2 + 2 * fi) * nj + j] = c * w;
        }
    } else {  // relpos: q itself, the window of all three from the joint distance (dist_inputs)
        const float q[3] = {qx, qy, qz};
        for (int c = 0; c < 3; ++c) {
            f[3 * j + c] = (M.use_cutoff && M.cutoff_inputs) ? q[c] * w : q[c];
            for (int fi = 0; fi < M.mr; ++fi) {
                float s, co;
                sincos_rr(q[c] * (float)(1 << fi), s, co);
                f[3 * ((1 + 2 * fi) * nj + j) + c] = s * w;
                f[3 * ((2 + 2 * fi) * nj + j) + c] = co * w;
            }
        }
    }
    // bone directions, times w_b under --cutoff_bones (bone CutoffEmbedder); with bone frequencies the
    // sin / cos of each direction component, windowed by w_b when the bone embedder is a CutoffEmbedder
    if (M.mrb == 0) {
        const float wb = M.bone_cut ? cutoff_w(M.tau_b, dist, M.cutoff_b[j]) : 1.0f;
        f[L.cb + 3 * j + 0] = M.bone_cut ? (qx / dn) * wb : qx / dn;
        f[L.cb + 3 * j + 1] = M.bone_cut ? (qy / dn) * wb : qy / dn;
        f[L.cb + 3 * j + 2] = M.bone_cut ? (qz / dn) * wb : qz / dn;
    } else {
        const float wb = M.bone_win ? cutoff_w(M.tau_b, dist, M.cutoff_b[j]) : 1.0f;
        const float ub[3] = {qx / dn, qy / dn, qz / dn};
        for (int c = 0; c < 3; ++c) {
            f[L.cb + 3 * j + c] = M.bone_cut ? ub[c] * wb : ub[c];
            for (int fi = 0; fi < M.mrb; ++fi) {
                float s, co;
                sincos_rr(ub[c] * (float)(1 << fi), s, co);
                f[L.cb + 3 * ((1 + 2 * fi) * nj + j) + c] = s * wb;
                f[L.cb + 3 * ((2 + 2 * fi) * nj + j) + c] = co * wb;
            }
        }
    }
    const float wv = M.cutoff_viewdir ? cutoff_w(M.tau_v, dist, M.cutoff_v[j]) : 1.0f;
    if (M.view_win) {  // (the caller contracts the direction terms per ray, anerf.h ANERF_ENC_VIEW_WINDOWS)
        f[L.cv + j] = wv;
        return;
    }
    float ex, ey, ez;
    joint_rot(S, dx, dy, dz, ex, ey, ez);
    if (M.view_angle) {
        float cs;
        const float a = ray_angle(qx, qy, qz, ex, ey, ez, cs);
        f[L.cv + j] = (M.cutoff_viewdir && M.cutoff_inputs) ? a * wv : a;
        for (int fi = 0; fi < M.mrv; ++fi) {
            float s, co;
            sincos_rr(a * (float)(1 << fi), s, co);
            f[L.cv + (1 + 2 * fi) * nj + j] = s * wv;
            f[L.cv + (2 + 2 * fi) * nj + j] = co * wv;
        }
        return;
    }
    const float en = M.view_raw ? 1.0f : fmaxf(norm3(ex, ey, ez), 1e-12f);  // (--view_type world: R_j d itself)
    const float e[3] = {ex / en, ey / en, ez / en};
    const int cx = L.cv;
    for (int c = 0; c < 3; ++c) {
        f[cx + 3 * j + c] = (M.cutoff_viewdir && M.cutoff_inputs) ? e[c] * wv : e[c];
        for (int fi = 0; fi < M.mrv; ++fi) {
            float s, co;
            sincos_rr(e[c] * (float)(1 << fi), s, co);
            f[cx + (1 + 2 * fi) * 3 * nj + 3 * j + c] = s * wv;
            f[cx + (2 + 2 * fi) * 3 * nj + 3 * j + c] = co * wv;
        }
    }
}

__global__ void train_encode_kernel(ModelDev M, const float* __restrict__ rb, int stride, int64_t n,
                                    const float* __restrict__ z, int ns, const float* __restrict__ skts,
                                    const int32_t* __restrict__ ray_pose, int n_poses,
                                    const float* __restrict__ pts_noise, float* __restrict__ feat) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int nj = M.nj;
    if (t >= n * ns * nj) return;
    const int64_t idx = t / nj;
    const int j = (int)(t % nj);
    const int64_t i = idx / ns;
    const int64_t pose = ray_pose ? ray_pose[i] : i;
    const float* ray = rb + i * stride;
    const float zz = z[idx];
    float px = ray[0] + ray[3] * zz, py = ray[1] + ray[4] * zz, pz = ray[2] + ray[5] * zz;
    if (pts_noise) {  // sample_pts' ray_noise_std (raycasters.py:660-661): pts + randn * std
        px += pts_noise[3 * idx], py += pts_noise[3 * idx + 1], pz += pts_noise[3 * idx + 2];
    }
    const int F = feat_layout(M).F;
    f32x4 r0, r1, r2;
    if (pose >= 0 && pose < n_poses) {
        const f32x4* sp = reinterpret_cast<const f32x4*>(skts + (pose * nj + j) * 16);
        r0 = sp[0], r1 = sp[1], r2 = sp[2];
    } else {  // out-of-range pose index: NaN features, no out-of-bounds read
        const float q = __int_as_float(0x7fc00000);
        r0 = r1 = r2 = f32x4{q, q, q, q};
    }
    const float S[12] = {r0[0], r0[1], r0[2], r0[3], r1[0], r1[1], r1[2], r1[3], r2[0], r2[1], r2[2], r2[3]};
    encode_joint(M, S, j, px, py, pz, ray[3], ray[4], ray[5], feat + idx * F);
}

// d feature / d inputs of encode_row for one (sample, joint): accumulates dL/dS[0:3, 0:4] (12
// values, row-major) of joint j given the feature gradients g (one row).  Same flags and forms as
// encode_row (cutoff windows w = 1 - sigmoid(tau (dist - c)), dw/ddist = -tau w (1 - w);
// F.normalize x / max(|x|, 1e-12); torch.norm's gradient 0 at 0).
// MR / MRV: the frequencies (compile-time, so every feature gradient of the joint is loaded up front
// and the loads overlap instead of waiting one loop iteration each); -1: the model's counts at run time
// (multires up to 10, multires_views up to 4: the other configurations' generic instance).  MRV -2: the
// ANERF_ENC_VIEW_WINDOWS layout (the view part is the NJ windows; their gradient reaches skts through dist).
template <int MR, int MRV>
__device__ __forceinline__ void encode_row_grad_joint(const ModelDev& M, const float* __restrict__ S, int j,
                                                      float px, float py, float pz, float dx, float dy, float dz,
                                                      const float* __restrict__ g, float (&gS)[12]) {
    constexpr bool VW = MRV == -2;
    constexpr int MRX = MR >= 0 ? MR : 10, MVX = MRV >= 0 ? MRV : (VW ? 0 : 4);  // (loop bounds; runtime counts below)
    const int mr = MR >= 0 ? MR : M.mr, mrv = MRV >= 0 ? MRV : (VW ? 0 : M.mrv);
    const int nj = M.nj, nv = 1 + 2 * mr;
    const int cx = nj * nv + 3 * nj;
    constexpr int MV = MVX > 0 ? MVX : 1;
    float gs_[MRX > 0 ? MRX : 1], gc_[MRX > 0 ? MRX : 1], gu_[3], gv0_[3], gvs_[3][MV], gvc_[3][MV];
    const float g0 = g[j];
    const float g_win = VW ? g[cx + j] : 0.0f;
#pragma unroll
    for (int fi = 0; fi < MRX; ++fi) {
        gs_[fi] = fi < mr ? g[(1 + 2 * fi) * nj + j] : 0.0f;
        gc_[fi] = fi < mr ? g[(2 + 2 * fi) * nj + j] : 0.0f;
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        gu_[c] = g[nj * nv + 3 * j + c];
        gv0_[c] = VW ? 0.0f : g[cx + 3 * j + c];
#pragma unroll
        for (int fi = 0; fi < MVX; ++fi) {
            gvs_[c][fi] = fi < mrv ? g[cx + (1 + 2 * fi) * 3 * nj + 3 * j + c] : 0.0f;
            gvc_[c][fi] = fi < mrv ? g[cx + (2 + 2 * fi) * 3 * nj + 3 * j + c] : 0.0f;
        }
    }
    float qx, qy, qz;
    joint_local(S, px, py, pz, qx, qy, qz);
    const float dist = norm3(qx, qy, qz);
    // ---- distance block
    const bool cut = M.use_cutoff != 0, cut_in = M.use_cutoff && M.cutoff_inputs;
    const float w = cut ? cutoff_w(M.tau, dist, M.cutoff[j]) : 1.0f;
    // the encoder's inputs u (raw) and uf (frequencies) and their slopes in dist (kp_inputs)
    float u, uf;
    kp_inputs(M.cut_to, M.shift_in, dist, M.cutoff[j], u, uf);
    const float du = M.cut_to ? -1.0f : 1.0f;
    const float duf = M.shift_in ? du * (2.0f / M.cutoff[j]) : du;
    float g_dist = 0.0f, g_w = 0.0f;
    if (cut_in) {
        g_dist += g0 * w * du;
        g_w += g0 * u;
    } else {
        g_dist += g0 * du;
    }
#pragma unroll
    for (int fi = 0; fi < MRX; ++fi) {
        if (fi >= mr) break;
        const float fr = (float)(1 << fi);
        float s, c;
        sincos_rr(uf * fr, s, c);
        const float gs = gs_[fi], gc = gc_[fi];
        g_w += gs * s + gc * c;
        g_dist += (gs * c - gc * s) * w * fr * duf;
    }
    if (cut) g_dist += g_w * (-M.tau * w * (1.0f - w));
    // ---- bone direction u = q / max(|q|, eps) (times w_b under --cutoff_bones)
    float gqx, gqy, gqz;
    {
        float gux = gu_[0], guy = gu_[1], guz = gu_[2];
        if (M.bone_cut) {  // f = u w_b: dL/du = g w_b, dL/dw_b = g . u
            const float wb = cutoff_w(M.tau_b, dist, M.cutoff_b[j]);
            const float dn = fmaxf(dist, 1e-12f);
            const float g_wb = gux * (qx / dn) + guy * (qy / dn) + guz * (qz / dn);
            g_dist += g_wb * (-M.tau_b * wb * (1.0f - wb));
            gux *= wb;
            guy *= wb;
            guz *= wb;
        }
        if (dist > 1e-12f) {
            const float ux = qx / dist, uy = qy / dist, uz = qz / dist;
            const float dot = ux * gux + uy * guy + uz * guz;
            gqx = (gux - ux * dot) / dist;
            gqy = (guy - uy * dot) / dist;
            gqz = (guz - uz * dot) / dist;
        } else {
            gqx = gux / 1e-12f;
            gqy = guy / 1e-12f;
            gqz = guz / 1e-12f;
        }
    }
    // ---- view direction e = R d / max(|R d|, eps), window on dist
    float gex = 0.0f, gey = 0.0f, gez = 0.0f;
    if constexpr (VW) {
        const float wv = cutoff_w(M.tau_v, dist, M.cutoff_v[j]);  // (the flag implies cutoff_viewdir)
        g_dist += g_win * (-M.tau_v * wv * (1.0f - wv));
    } else {
        float ex, ey, ez;
        joint_rot(S, dx, dy, dz, ex, ey, ez);
        const float enr = norm3(ex, ey, ez);
        const float en = M.view_raw ? 1.0f : fmaxf(enr, 1e-12f);  // (--view_type world: no normalisation)
        const float e[3] = {ex / en, ey / en, ez / en};
        const bool cutv = M.cutoff_viewdir != 0;
        const float wv = cutv ? cutoff_w(M.tau_v, dist, M.cutoff_v[j]) : 1.0f;
        float ge[3] = {0.0f, 0.0f, 0.0f}, g_wv = 0.0f;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float gv0 = gv0_[c];
            if (cutv && M.cutoff_inputs) {
                ge[c] += gv0 * wv;
                g_wv += gv0 * e[c];
            } else {
                ge[c] += gv0;
            }
#pragma unroll
            for (int fi = 0; fi < MVX; ++fi) {
                if (fi >= mrv) break;
                const float fr = (float)(1 << fi);
                float s, co;
                sincos_rr(e[c] * fr, s, co);
                const float gs = gvs_[c][fi], gc = gvc_[c][fi];
                g_wv += gs * s + gc * co;
                ge[c] += (gs * co - gc * s) * wv * fr;
            }
        }
        if (cutv) g_dist += g_wv * (-M.tau_v * wv * (1.0f - wv));
        if (M.view_raw) {  // e = R_j d itself
            gex = ge[0];
            gey = ge[1];
            gez = ge[2];
        } else if (enr > 1e-12f) {
            const float dot = e[0] * ge[0] + e[1] * ge[1] + e[2] * ge[2];
            gex = (ge[0] - e[0] * dot) / enr;
            gey = (ge[1] - e[1] * dot) / enr;
            gez = (ge[2] - e[2] * dot) / enr;
        } else {
            gex = ge[0] / 1e-12f;
            gey = ge[1] / 1e-12f;
            gez = ge[2] / 1e-12f;
        }
    }
    // ---- dist = |q|
    if (dist > 0.0f) {
        gqx += g_dist * qx / dist;
        gqy += g_dist * qy / dist;
        gqz += g_dist * qz / dist;
    }
    // q = A p + t, e_raw = A d
    const float gq[3] = {gqx, gqy, gqz}, gr[3] = {gex, gey, gez};
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        gS[4 * r + 0] += gq[r] * px + gr[r] * dx;
        gS[4 * r + 1] += gq[r] * py + gr[r] * dy;
        gS[4 * r + 2] += gq[r] * pz + gr[r] * dz;
        gS[4 * r + 3] += gq[r];
    }
}

// d feature / d inputs for the staged encoders (anerf.h, ABI 15), run-time frequency counts: relpos kp inputs,
// bone frequencies, ray angles, with every option of encode_joint.  With relpos the reference's window distance
// is |p - kp_j| (raycasters.py:530-533), not a function of the poses: no window gradient reaches skts then.
__device__ __noinline__ void encode_row_grad_joint_staged(const ModelDev& M, const float* __restrict__ S, int j,
                                                          float px, float py, float pz, float dx, float dy, float dz,
                                                          const float* __restrict__ g, float (&gS)[12]) {
    const int nj = M.nj;
    const FeatLayout L = feat_layout(M);
    const bool dg = !M.kp_relpos && !M.kp_query;  // (the windows' distance carries a gradient)
    float qx, qy, qz;
    joint_local(S, px, py, pz, qx, qy, qz);
    const float dist = norm3(qx, qy, qz);
    const float q[3] = {qx, qy, qz};
    float gq[3] = {0.0f, 0.0f, 0.0f};
    float g_dist = 0.0f;
    // ---- kp part
    const bool cut = M.use_cutoff != 0, cut_in = M.use_cutoff && M.cutoff_inputs;
    const float w = cut ? cutoff_w(M.tau, dist, M.cutoff[j]) : 1.0f;
    float g_w = 0.0f;
    if (M.kp_query) {
        // querypts: the kp features depend on the world point only -- nothing for skts
    } else if (!M.kp_relpos) {
        float u, uf;
        kp_inputs(M.cut_to, M.shift_in, dist, M.cutoff[j], u, uf);
        const float du = M.cut_to ? -1.0f : 1.0f;
        const float duf = M.shift_in ? du * (2.0f / M.cutoff[j]) : du;
        const float g0 = g[j];
        if (cut_in) {
            g_dist += g0 * w * du;
            g_w += g0 * u;
        } else {
            g_dist += g0 * du;
        }
        for (int fi = 0; fi < M.mr; ++fi) {
            const float fr = (float)(1 << fi);
            float sn, cs;
            sincos_rr(uf * fr, sn, cs);
            const float gs = g[(1 + 2 * fi) * nj + j], gc = g[(2 + 2 * fi) * nj + j];
            g_w += gs * sn + gc * cs;
            g_dist += (gs * cs - gc * sn) * w * fr * duf;
        }
    } else {
        for (int c = 0; c < 3; ++c) {
            const float g0 = g[3 * j + c];
            gq[c] += cut_in ? g0 * w : g0;
            if (cut_in) g_w += g0 * q[c];
            for (int fi = 0; fi < M.mr; ++fi) {
                const float fr = (float)(1 << fi);
                float sn, cs;
                sincos_rr(q[c] * fr, sn, cs);
                const float gs = g[3 * ((1 + 2 * fi) * nj + j) + c], gc = g[3 * ((2 + 2 * fi) * nj + j) + c];
                g_w += gs * sn + gc * cs;
                gq[c] += (gs * cs - gc * sn) * w * fr;
            }
        }
    }
    if (cut && dg) g_dist += g_w * (-M.tau * w * (1.0f - w));
    // ---- bone part: u = q / max(|q|, eps), its frequencies, the bone window
    {
        const float dn = fmaxf(dist, 1e-12f);
        const float ub[3] = {qx / dn, qy / dn, qz / dn};
        const bool win = M.mrb > 0 ? M.bone_win != 0 : M.bone_cut != 0;
        const float wb = win ? cutoff_w(M.tau_b, dist, M.cutoff_b[j]) : 1.0f;
        float gu[3], g_wb = 0.0f;
        for (int c = 0; c < 3; ++c) {
            const float g0 = g[L.cb + 3 * j + c];
            gu[c] = M.bone_cut ? g0 * wb : g0;
            if (M.bone_cut) g_wb += g0 * ub[c];
            for (int fi = 0; fi < M.mrb; ++fi) {
                const float fr = (float)(1 << fi);
                float sn, cs;
                sincos_rr(ub[c] * fr, sn, cs);
                const float gs = g[L.cb + 3 * ((1 + 2 * fi) * nj + j) + c], gc = g[L.cb + 3 * ((2 + 2 * fi) * nj + j) + c];
                g_wb += gs * sn + gc * cs;
                gu[c] += (gs * cs - gc * sn) * wb * fr;
            }
        }
        if (win && dg) g_dist += g_wb * (-M.tau_b * wb * (1.0f - wb));
        if (dist > 1e-12f) {
            const float dot = ub[0] * gu[0] + ub[1] * gu[1] + ub[2] * gu[2];
            for (int c = 0; c < 3; ++c) gq[c] += (gu[c] - ub[c] * dot) / dist;
        } else {
            for (int c = 0; c < 3; ++c) gq[c] += gu[c] / 1e-12f;
        }
    }
    // ---- view part
    float ex, ey, ez;
    joint_rot(S, dx, dy, dz, ex, ey, ez);
    const bool cutv = M.cutoff_viewdir != 0;
    const float wv = cutv ? cutoff_w(M.tau_v, dist, M.cutoff_v[j]) : 1.0f;
    float gr[3] = {0.0f, 0.0f, 0.0f}, g_wv = 0.0f;
    if (M.view_angle) {
        float cs;
        const float a = ray_angle(qx, qy, qz, ex, ey, ez, cs);
        const float g0 = g[L.cv + j];
        float ga = (cutv && M.cutoff_inputs) ? g0 * wv : g0;
        if (cutv && M.cutoff_inputs) g_wv += g0 * a;
        for (int fi = 0; fi < M.mrv; ++fi) {
            const float fr = (float)(1 << fi);
            float sn, co;
            sincos_rr(a * fr, sn, co);
            const float gs = g[L.cv + (1 + 2 * fi) * nj + j], gc = g[L.cv + (2 + 2 * fi) * nj + j];
            g_wv += gs * sn + gc * co;
            ga += (gs * co - gc * sn) * wv * fr;
        }
        // acos' slope inside the clamp (torch.clamp passes the gradient on [min, max]), then the cosine's
        const bool inside = cs >= -1.0f + 1e-6f && cs <= 1.0f - 1e-6f;
        const float gcs = inside ? -ga / sqrtf(fmaxf(1.0f - cs * cs, 1e-30f)) : 0.0f;
        const float nq = dist, ne = norm3(ex, ey, ez);
        const float e[3] = {ex, ey, ez};
        if (nq > 0.0f && ne > 0.0f) {
            const float inv = 1.0f / (nq * ne);
            for (int c = 0; c < 3; ++c) {
                gq[c] += gcs * (e[c] * inv - cs * q[c] / (nq * nq));
                gr[c] += gcs * (q[c] * inv - cs * e[c] / (ne * ne));
            }
        }
    } else {
        const float enr = norm3(ex, ey, ez);
        const float en = M.view_raw ? 1.0f : fmaxf(enr, 1e-12f);
        const float e[3] = {ex / en, ey / en, ez / en};
        float ge[3] = {0.0f, 0.0f, 0.0f};
        for (int c = 0; c < 3; ++c) {
            const float gv0 = g[L.cv + 3 * j + c];
            if (cutv && M.cutoff_inputs) {
                ge[c] += gv0 * wv;
                g_wv += gv0 * e[c];
            } else {
                ge[c] += gv0;
            }
            for (int fi = 0; fi < M.mrv; ++fi) {
                const float fr = (float)(1 << fi);
                float sn, co;
                sincos_rr(e[c] * fr, sn, co);
                const float gs = g[L.cv + (1 + 2 * fi) * 3 * nj + 3 * j + c], gc = g[L.cv + (2 + 2 * fi) * 3 * nj + 3 * j + c];
                g_wv += gs * sn + gc * co;
                ge[c] += (gs * co - gc * sn) * wv * fr;
            }
        }
        if (M.view_raw) {
            for (int c = 0; c < 3; ++c) gr[c] = ge[c];
        } else if (enr > 1e-12f) {
            const float dot = e[0] * ge[0] + e[1] * ge[1] + e[2] * ge[2];
            for (int c = 0; c < 3; ++c) gr[c] = (ge[c] - e[c] * dot) / enr;
        } else {
            for (int c = 0; c < 3; ++c) gr[c] = ge[c] / 1e-12f;
        }
    }
    if (cutv && dg) g_dist += g_wv * (-M.tau_v * wv * (1.0f - wv));
    if (dist > 0.0f)
        for (int c = 0; c < 3; ++c) gq[c] += g_dist * q[c] / dist;
    for (int r = 0; r < 3; ++r) {  // q = A p + t, e_raw = A d
        gS[4 * r + 0] += gq[r] * px + gr[r] * dx;
        gS[4 * r + 1] += gq[r] * py + gr[r] * dy;
        gS[4 * r + 2] += gq[r] * pz + gr[r] * dz;
        gS[4 * r + 3] += gq[r];
    }
}

// Encoder backward: dL/dskts from dL/dfeat.  Block = one ray, thread = (sample slot, joint) with the
// joint fastest (spb sample slots x nj joints, spb = 256 / nj), so each thread keeps one joint's 12
// sums over the samples s = slot, slot + spb, ... and the lanes of a wave read each feature of a
// sample as one nj-float run (the feature rows are joint-minor): every 4.3 KB feature row is read
// once, by one wave, in whole runs.  The slots' sums are added through LDS in slot order
// (deterministic within the ray) and accumulated into grad_skts[pose] (atomic: rays may share a
// pose).  Rows 3 (the [0 0 0 1] row) get no gradient, as in the reference.
template <int MR, int MRV>
__global__ __launch_bounds__(256) void train_encode_backward_kernel(ModelDev M, const float* __restrict__ rb,
                                                                    int stride, int64_t n, const float* __restrict__ z,
                                                                    int ns, const float* __restrict__ skts,
                                                                    const int32_t* __restrict__ ray_pose, int n_poses,
                                                                    const float* __restrict__ pts_noise,
                                                                    const float* __restrict__ gfeat,
                                                                    float* __restrict__ gskts, int spb) {
    extern __shared__ float red[];  // [spb][nj][12]
    const int nj = M.nj;
    const int64_t i = blockIdx.x;
    const int t = threadIdx.x, slot = t / nj, j = t % nj;
    // (an out-of-range pose index contributes no gradient and is never dereferenced)
    const int64_t pose = ray_pose ? ray_pose[i] : i;
    const bool pose_ok = pose >= 0 && pose < n_poses;
    float gS[12] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    if (pose_ok && slot < spb) {
        const float* ray = rb + i * stride;
        const int F = feat_layout(M).F;
        const f32x4* sp = reinterpret_cast<const f32x4*>(skts + (pose * nj + j) * 16);
        const f32x4 r0 = sp[0], r1 = sp[1], r2 = sp[2];
        const float S[12] = {r0[0], r0[1], r0[2], r0[3], r1[0], r1[1], r1[2], r1[3], r2[0], r2[1], r2[2], r2[3]};
        for (int s = slot; s < ns; s += spb) {
            const float zz = z[i * ns + s];
            float px = ray[0] + ray[3] * zz, py = ray[1] + ray[4] * zz, pz = ray[2] + ray[5] * zz;
            if (pts_noise) {
                const float* q = pts_noise + 3 * (i * ns + s);
                px += q[0], py += q[1], pz += q[2];
            }
            if (MR < 0 && M.staged)  // (the generic instance serves the staged encoders too)
                encode_row_grad_joint_staged(M, S, j, px, py, pz, ray[3], ray[4], ray[5], gfeat + (i * ns + s) * F, gS);
            else
                encode_row_grad_joint<MR, MRV>(M, S, j, px, py, pz, ray[3], ray[4], ray[5], gfeat + (i * ns + s) * F, gS);
        }
        float* const rr = red + (slot * nj + j) * 12;
#pragma unroll
        for (int k = 0; k < 12; ++k) rr[k] = gS[k];
    }
    __syncthreads();
    if (!pose_ok) return;
    for (int q = t; q < nj * 12; q += blockDim.x) {
        float v = red[q];
        for (int sl = 1; sl < spb; ++sl) v += red[sl * nj * 12 + q];
        const int jq = q / 12, k = q % 12;
        if (v != 0.0f) atomicAdd(gskts + (pose * nj + jq) * 16 + k, v);
    }
}

// raw2outputs (core/networks/nerf.py:150-205) with the training noise: sigma = act(raw/B + noise),
// alpha = 1 - exp(-sigma delta), weights = alpha * exclusive cumprod(1 - alpha + 1e-10) (torch's CPU
// cumprod accumulates in double), rgb / depth / acc sums, disp with the isclose(acc, 0) zeroing.
// Also writes the transmittance (the exclusive cumprod) for the backward.  One thread per ray.
__device__ __forceinline__ float density_act_grad(const ModelDev& M, float x) {
    if (!M.softplus) return x > 0.0f ? 1.0f : 0.0f;  // relu: grad * (result > 0)
    const float y = x - M.shift;                     // softplus(beta 1, threshold 20)
    if (y > 20.0f) return 1.0f;
    const float e = expf(y);
    return e / (e + 1.0f);
}

// One wave per ray: the per-sample alpha / colour terms in parallel into LDS, the transmittance
// product (double, torch's CPU cumprod) and the sums in sample order by lane 0, then the per-sample
// outputs in parallel -- the same operations in the same order as a thread-per-ray loop.
__global__ __launch_bounds__(64) void train_composite_kernel(ModelDev M, const float* __restrict__ raw,
                                                             const float* __restrict__ z, const float* __restrict__ rb,
                                                             int stride, int64_t n, int ns,
                                                             const float* __restrict__ noise, float* __restrict__ rgb,
                                                             float* __restrict__ disp, float* __restrict__ acc,
                                                             float* __restrict__ wts, float* __restrict__ alpha,
                                                             float* __restrict__ trans) {
    extern __shared__ float cl[];  // [7][ns]: alpha, rgb terms (3), z, transmittance, weight
    const int64_t i = blockIdx.x;
    if (i >= n) return;
    const int lane = threadIdx.x;
    float *la = cl, *lc0 = cl + ns, *lc1 = cl + 2 * ns, *lc2 = cl + 3 * ns, *lz = cl + 4 * ns, *lt = cl + 5 * ns,
          *lw = cl + 6 * ns;
    const float* ray = rb + i * stride;
    const float dn = norm3(ray[3], ray[4], ray[5]);
    const float* zr = z + i * ns;
    const float* rr = raw + i * ns * 4;
    for (int s = lane; s < ns; s += 64) {
        float dist = (s + 1 < ns) ? (zr[s + 1] - zr[s]) : 1e10f;
        dist = dist * dn;
        const float x = rr[4 * s + 3] / M.B + (noise ? noise[i * ns + s] : 0.0f);
        la[s] = alpha_of(density_act(M, x) * dist);
        lz[s] = zr[s];
        lc0[s] = sigmoid(rr[4 * s + 0]) * 1.002f - 0.001f;
        lc1[s] = sigmoid(rr[4 * s + 1]) * 1.002f - 0.001f;
        lc2[s] = sigmoid(rr[4 * s + 2]) * 1.002f - 0.001f;
    }
    __syncthreads();
    if (lane == 0) {
        double T = 1.0;
        float sa = 0.0f, sd = 0.0f, sr = 0.0f, sg = 0.0f, sb = 0.0f;
        for (int s = 0; s < ns; ++s) {
            const float a = la[s];
            const float t = (float)T;
            T *= (double)((1.0f - a) + 1e-10f);
            const float w = a * t;
            lt[s] = t;
            lw[s] = w;
            sa += w;
            sd += w * lz[s];
            sr += w * lc0[s];
            sg += w * lc1[s];
            sb += w * lc2[s];
        }
        const float ratio = sd / (sa + 1e-10f);
        float dsp = 1.0f / fmaxf(ratio, 1e-10f);
        if (ratio != ratio) dsp = ratio;
        if (fabsf(sa) <= 1e-8f) dsp = 0.0f;
        rgb[3 * i] = sr;
        rgb[3 * i + 1] = sg;
        rgb[3 * i + 2] = sb;
        disp[i] = dsp;
        acc[i] = sa < 1.0f ? sa : 1.0f;
    }
    __syncthreads();
    for (int s = lane; s < ns; s += 64) {
        alpha[i * ns + s] = la[s];
        trans[i * ns + s] = lt[s];
        wts[i * ns + s] = lw[s];
    }
}

// Backward of train_composite_kernel: dL/draw (N x ns x 4) from dL/d{rgb, disp, acc, weights, alpha}
// (any may be NULL = zero).  With G_s = dL/dw_s, the transmittance factors f_s = 1 - alpha_s + 1e-10
// and P_s their exclusive product: dL/dalpha_s = G_s P_s + galpha_s - P_s R_s, where
// R_s = sum_{k>s} G_k alpha_k prod_{s<m<k} f_m runs backwards as R_{s-1} = G_s alpha_s + f_s R_s
// (no division by f_s); then dalpha/dsigma = exp(-sigma delta) delta, the activation's gradient, 1/B;
// rgb: w_s g_rgb 1.002 sigmoid'(raw).  One wave per ray: the per-sample terms in parallel, the sums
// and the R recurrence (double) in sample order by lane 0 -- the thread-per-ray loop's operations in
// its order.
__global__ __launch_bounds__(64) void train_composite_backward_kernel(
    ModelDev M, const float* __restrict__ raw, const float* __restrict__ z, const float* __restrict__ rb, int stride,
    int64_t n, int ns, const float* __restrict__ noise, const float* __restrict__ wts, const float* __restrict__ alpha,
    const float* __restrict__ trans, const float* __restrict__ g_rgb, const float* __restrict__ g_disp,
    const float* __restrict__ g_acc, const float* __restrict__ g_w, const float* __restrict__ g_alpha,
    float* __restrict__ g_raw) {
    extern __shared__ float cl[];  // [8][ns]: w, z, alpha, P, sigmoid(rgb) (3), G, then P R
    __shared__ float sc[4];        // r, gd_r, den, ga
    const int64_t i = blockIdx.x;
    if (i >= n) return;
    const int lane = threadIdx.x;
    float *lw = cl, *lz = cl + ns, *la = cl + 2 * ns, *lP = cl + 3 * ns, *lc0 = cl + 4 * ns, *lc1 = cl + 5 * ns,
          *lc2 = cl + 6 * ns, *lG = cl + 7 * ns, *lPR = cl + 8 * ns;
    const float* ray = rb + i * stride;
    const float dn = norm3(ray[3], ray[4], ray[5]);
    const float* zr = z + i * ns;
    const float* rr = raw + i * ns * 4;
    for (int s = lane; s < ns; s += 64) {
        lw[s] = wts[i * ns + s];
        lz[s] = zr[s];
        la[s] = alpha[i * ns + s];
        lP[s] = trans[i * ns + s];
        lc0[s] = sigmoid(rr[4 * s + 0]);
        lc1[s] = sigmoid(rr[4 * s + 1]);
        lc2[s] = sigmoid(rr[4 * s + 2]);
    }
    const float gr = g_rgb ? g_rgb[3 * i] : 0.0f, gg = g_rgb ? g_rgb[3 * i + 1] : 0.0f,
                gb = g_rgb ? g_rgb[3 * i + 2] : 0.0f;
    __syncthreads();
    if (lane == 0) {  // the sums in sample order
        float sa = 0.0f, sd = 0.0f;
        for (int s = 0; s < ns; ++s) {
            sa += lw[s];
            sd += lw[s] * lz[s];
        }
        const float ga = (g_acc && sa < 1.0f) ? g_acc[i] : 0.0f;  // torch.minimum(sum w, 1)
        // disp = mask / max(1e-10, depth / (W + 1e-10)):  d disp / d w_s = -mask / r^2 (z_s - r) / (W + 1e-10)
        float gd_r = 0.0f, r = 0.0f;
        const float den = sa + 1e-10f;
        if (g_disp) {
            r = sd / den;
            if (r > 1e-10f && !(fabsf(sa) <= 1e-8f)) gd_r = -g_disp[i] / (r * r);
        }
        sc[0] = r, sc[1] = gd_r, sc[2] = den, sc[3] = ga;
    }
    __syncthreads();
    const float r = sc[0], gd_r = sc[1], den = sc[2], ga = sc[3];
    for (int s = lane; s < ns; s += 64) {  // G_s = dL/dw_s
        float G = gr * (lc0[s] * 1.002f - 0.001f) + gg * (lc1[s] * 1.002f - 0.001f) + gb * (lc2[s] * 1.002f - 0.001f) +
                  ga;
        if (gd_r != 0.0f) G += gd_r * (lz[s] - r) / den;
        if (g_w) G += g_w[i * ns + s];
        lG[s] = G;
    }
    __syncthreads();
    if (lane == 0) {  // R_s backwards (double), P_s R_s for each sample
        double R = 0.0;
        for (int s = ns - 1; s >= 0; --s) {
            lPR[s] = (float)((double)lP[s] * R);
            R = (double)lG[s] * (double)la[s] + (double)((1.0f - la[s]) + 1e-10f) * R;
        }
    }
    __syncthreads();
    for (int s = lane; s < ns; s += 64) {
        const float G = lG[s], a = la[s], P = lP[s], w = lw[s];
        const float c0 = lc0[s], c1 = lc1[s], c2 = lc2[s];
        (void)a;
        const float gal = G * P + (g_alpha ? g_alpha[i * ns + s] : 0.0f) - lPR[s];
        float dist = (s + 1 < ns) ? (lz[s + 1] - lz[s]) : 1e10f;
        dist = dist * dn;
        const float x = rr[4 * s + 3] / M.B + (noise ? noise[i * ns + s] : 0.0f);
        const float sig = density_act(M, x);
        const float gsig = gal * expf(-sig * dist) * dist;
        float* go = g_raw + (i * ns + s) * 4;
        go[3] = gsig * density_act_grad(M, x) / M.B;
        go[0] = w * gr * 1.002f * c0 * (1.0f - c0);
        go[1] = w * gg * 1.002f * c1 * (1.0f - c1);
        go[2] = w * gb * 1.002f * c2 * (1.0f - c2);
    }
}

// isample_from_lineseg + sample_pdf (det=False: u from torch.rand) + sort, training form of the
// render kernel's importance(): one wave per ray, LDS scratch.  z_all (N x (S+I)) sorted.
__global__ __launch_bounds__(64) void train_importance_kernel(const float* __restrict__ z,
                                                              const float* __restrict__ wts, int64_t n, int S, int I,
                                                              const float* __restrict__ u, int is_only,
                                                              float* __restrict__ z_all,
                                                              int32_t* __restrict__ sorted_idx) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int64_t i = blockIdx.x;
    if (i >= n) return;
    const int lane = threadIdx.x, T = S + I;
    const int zs = pad32(T);
    float* zc = lds;
    float* w = lds + zs;
    float* zf = lds + 2 * zs;
    float* scr2 = lds + 3 * zs;
    for (int s = lane; s < S; s += 64) {
        zc[s] = z[i * S + s];
        w[s] = wts[i * S + s];
    }
    wave_sync();
    int* src = reinterpret_cast<int*>(scr2 + 3 * S + T + 32);  // (after importance()'s scratch)
    importance(zc, w, S, I, zf, scr2, true, lane, u ? u + i * I : nullptr, is_only != 0, sorted_idx ? src : nullptr);
    for (int s = lane; s < T; s += 64) {
        z_all[i * T + s] = zf[s];
        if (sorted_idx) sorted_idx[i * T + s] = src[s];
    }
}

// ---- view-window layout (anerf.h ANERF_ENC_VIEW_WINDOWS): the view layer's view part sum_j w_j G_j per sample.
// One workgroup per ray; G[ray] [NJ][WH] (4 (NJ WH + VM_SC NJ) bytes <= 64 KB) and VM_SC samples' windows in LDS,
// lanes over (sample, 4 columns).  HBM: the windows (NJ floats per sample), G once per ray, the [WH] output row
// per sample.
constexpr int VM_SC = 32;  // (samples per LDS chunk)
// float4 dL/dG accumulators per thread of the backward: 4 for NJ W <= 4096 (24 joints at W 128), 9 up to 9216
// (65-72 joints at W 128)
constexpr int VM_K_SMALL = 4, VM_K_LARGE = 9;
__global__ __launch_bounds__(256) void train_view_mix_kernel(const float* __restrict__ win, int64_t ldw, int ns, int nj,
                                                             const float* __restrict__ G, int wh,
                                                             float* __restrict__ out) {
    extern __shared__ float sh[];
    float* sG = sh;            // [nj][wh]
    float* sW = sG + nj * wh;  // [VM_SC][nj]
    const int64_t r = blockIdx.x;
    const int tid = threadIdx.x, h4n = wh / 4;
    const f32x4* g4 = reinterpret_cast<const f32x4*>(G + r * nj * wh);
    for (int q = tid; q < nj * h4n; q += blockDim.x) reinterpret_cast<f32x4*>(sG)[q] = g4[q];
    for (int s0 = 0; s0 < ns; s0 += VM_SC) {
        const int sc = min(VM_SC, ns - s0);
        __syncthreads();  // (the previous chunk's readers are done)
        for (int q = tid; q < sc * nj; q += blockDim.x) {
            const int s = q / nj, j = q - s * nj;
            sW[q] = win[(r * ns + s0 + s) * ldw + j];
        }
        __syncthreads();
        for (int t = tid; t < sc * h4n; t += blockDim.x) {
            const int s = t / h4n, h4 = t - s * h4n;
            f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
            for (int j = 0; j < nj; ++j) {
                const float wj = sW[s * nj + j];  // (the lanes of one sample read one address)
                const f32x4 gv = reinterpret_cast<const f32x4*>(sG)[j * h4n + h4];
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[e] = fmaf(wj, gv[e], acc[e]);
            }
            reinterpret_cast<f32x4*>(out + (r * ns + s0 + s) * wh)[h4] = acc;
        }
    }
}

// Its gradients: dL/dw_j(s) = sum_h gz[s][h] G[j][h] (into the window columns of g_feat) and dL/dG[j][h] =
// sum_s w_j(s) gz[s][h], per ray; samples in chunks of VM_SC through LDS.  dL/dw: lanes over samples (gz rows
// padded by 4 floats), 4 joints per lane (G rows zero-padded to a multiple of 4 joints); dL/dG: VM_K float4
// column groups per lane (NJ W <= 1024 VM_K), in registers across the chunks.
template <int VM_K>
__global__ __launch_bounds__(256) void train_view_mix_backward_kernel(const float* __restrict__ win, int64_t ldw,
                                                                      int ns, int nj, const float* __restrict__ G,
                                                                      int wh, const float* __restrict__ gz,
                                                                      float* __restrict__ gwin, int64_t ldg,
                                                                      float* __restrict__ gG) {
    extern __shared__ float sh[];
    const int wp = wh + 4;  // (padded row)
    const int nj4 = (nj + 3) / 4;
    float* sG = sh;                   // [4 nj4][wp]
    float* sZ = sG + 4 * nj4 * wp;    // [VM_SC][wp]
    float* sW = sZ + VM_SC * wp;      // [VM_SC][nj]
    const int64_t r = blockIdx.x;
    const int tid = threadIdx.x, h4n = wh / 4;
    for (int q = tid; q < 4 * nj4 * h4n; q += blockDim.x) {
        const int j = q / h4n, h4 = q - j * h4n;
        const f32x4 z4 = {0.0f, 0.0f, 0.0f, 0.0f};
        *reinterpret_cast<f32x4*>(sG + j * wp + 4 * h4) =
            j < nj ? reinterpret_cast<const f32x4*>(G + (r * nj + j) * wh)[h4] : z4;
    }
    f32x4 acc[VM_K];
#pragma unroll
    for (int k = 0; k < VM_K; ++k) acc[k] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    for (int s0 = 0; s0 < ns; s0 += VM_SC) {
        const int sc = min(VM_SC, ns - s0);
        __syncthreads();  // (the previous chunk's readers are done; G is in place on the first pass)
        for (int q = tid; q < sc * h4n; q += blockDim.x) {
            const int s = q / h4n, h4 = q - s * h4n;
            *reinterpret_cast<f32x4*>(sZ + s * wp + 4 * h4) =
                reinterpret_cast<const f32x4*>(gz + (r * ns + s0 + s) * wh)[h4];
        }
        for (int q = tid; q < sc * nj; q += blockDim.x) {
            const int s = q / nj, j = q - s * nj;
            sW[q] = win[(r * ns + s0 + s) * ldw + j];
        }
        __syncthreads();
        for (int q = tid; q < VM_SC * nj4; q += blockDim.x) {
            const int s = q % VM_SC, jg = q / VM_SC;
            if (s >= sc) continue;
            f32x4 d[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) d[u] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
            for (int h = 0; h < wh; h += 4) {
                const f32x4 a = *reinterpret_cast<const f32x4*>(sZ + s * wp + h);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const f32x4 b = *reinterpret_cast<const f32x4*>(sG + (4 * jg + u) * wp + h);
#pragma unroll
                    for (int e = 0; e < 4; ++e) d[u][e] = fmaf(a[e], b[e], d[u][e]);
                }
            }
            float* gw = gwin + (r * ns + s0 + s) * ldg + 4 * jg;
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (4 * jg + u < nj) gw[u] = (d[u][0] + d[u][1]) + (d[u][2] + d[u][3]);
        }
#pragma unroll
        for (int k = 0; k < VM_K; ++k) {
            const int q = tid + 256 * k;  // (float4 group: joint q / h4n, columns 4 (q % h4n) ..)
            if (q >= nj * h4n) break;
            const int j = q / h4n, h = 4 * (q - j * h4n);
            f32x4 a = acc[k];
            for (int s = 0; s < sc; ++s) {
                const float wj = sW[s * nj + j];
                const f32x4 z = *reinterpret_cast<const f32x4*>(sZ + s * wp + h);
#pragma unroll
                for (int e = 0; e < 4; ++e) a[e] = fmaf(wj, z[e], a[e]);
            }
            acc[k] = a;
        }
    }
#pragma unroll
    for (int k = 0; k < VM_K; ++k) {
        const int q = tid + 256 * k;
        if (q >= nj * h4n) break;
        reinterpret_cast<f32x4*>(gG + r * nj * wh)[q] = acc[k];
    }
}

// ---- the per-ray view factors of the view-window layout: G[r][j][h] = sum_k T_k(e_rj) Wv'[j][k][h], e_rj = R_j d_r
// normalised (raw under --view_type world), T = [e, sin 2^m e, cos 2^m e ...] (slot f component c at k = 3 f + c),
// Wv' the view layer's view columns (column f 3 NJ + 3 j + c) times the --freq_schedule weights.  One joint per
// workgroup (its Wv' slice staged in LDS).
#ifndef ANERF_VF_RAYS_B
#define ANERF_VF_RAYS_B 128
#endif
constexpr int VF_RC = 64, VF_RAYS_B = ANERF_VF_RAYS_B, VF_KG = 4;  // (rays per chunk / per backward workgroup; float4
                                                                   // dL/dWv groups per thread)
__device__ __forceinline__ bool view_terms(const ModelDev& M, const float* __restrict__ rb, int stride, int64_t r,
                                           const float* __restrict__ skts, const int32_t* __restrict__ ray_pose,
                                           int n_poses, int j, float (&T)[27], float (&e)[3], float& enr,
                                           int64_t& pose) {
    pose = ray_pose ? ray_pose[r] : r;
    if (pose < 0 || pose >= n_poses) return false;
    const float* S = skts + (pose * M.nj + j) * 16;
    const float* ray = rb + r * stride;
    float ex, ey, ez;
    joint_rot(S, ray[3], ray[4], ray[5], ex, ey, ez);
    enr = norm3(ex, ey, ez);
    const float en = M.view_raw ? 1.0f : fmaxf(enr, 1e-12f);
    e[0] = ex / en, e[1] = ey / en, e[2] = ez / en;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        T[c] = e[c];
#pragma unroll
        for (int fi = 0; fi < 4; ++fi) {
            float s = 0.0f, co = 0.0f;
            if (fi < M.mrv) sincos_rr(e[c] * (float)(1 << fi), s, co);
            T[3 * (1 + 2 * fi) + c] = s;
            T[3 * (2 + 2 * fi) + c] = co;
        }
    }
    return true;
}

__device__ __forceinline__ void stage_view_cols(const ModelDev& M, int j, const float* __restrict__ wv, int64_t ldv,
                                                int wh, const float* __restrict__ fs, float* __restrict__ sw) {
    const int nk = 3 * (1 + 2 * M.mrv);
    for (int q = threadIdx.x; q < nk * wh; q += blockDim.x) {
        const int k = q / wh, h = q - k * wh;
        const int col = (k / 3) * 3 * M.nj + 3 * j + k % 3;
        sw[q] = wv[h * ldv + col] * (fs ? fs[col] : 1.0f);
    }
}

// Rays in chunks of VF_RC: one thread per ray forms T (LDS, padded rows of 28), the workgroup then forms the
// chunk's [VF_RC][WH] outputs with lanes over (ray, 4 columns).
__global__ __launch_bounds__(256) void train_view_factor_kernel(ModelDev M, const float* __restrict__ rb, int stride,
                                                                int64_t n, const float* __restrict__ skts,
                                                                const int32_t* __restrict__ ray_pose, int n_poses,
                                                                const float* __restrict__ wv, int64_t ldv, int wh,
                                                                const float* __restrict__ fs, float* __restrict__ G) {
    extern __shared__ float sh[];
    const int j = blockIdx.y, nj = M.nj, nk = 3 * (1 + 2 * M.mrv);
    float* sw = sh;            // [nk][wh]
    float* sT = sw + nk * wh;  // [VF_RC][28] (column 27: 0, or NaN for a bad pose index)
    stage_view_cols(M, j, wv, ldv, wh, fs, sw);
    const int tid = threadIdx.x, h4n = wh / 4;
    const int64_t r0 = (int64_t)blockIdx.x * VF_RC;
    if (tid < VF_RC && r0 + tid < n) {
        float T[27], e[3], enr;
        int64_t pose;
        const bool ok = view_terms(M, rb, stride, r0 + tid, skts, ray_pose, n_poses, j, T, e, enr, pose);
#pragma unroll
        for (int k = 0; k < 27; ++k) sT[tid * 28 + k] = ok ? T[k] : 0.0f;
        sT[tid * 28 + 27] = ok ? 0.0f : __int_as_float(0x7fc00000);
    }
    __syncthreads();
    for (int q = tid; q < VF_RC * h4n; q += blockDim.x) {
        const int rr = q / h4n, h4 = q - rr * h4n;
        const int64_t r = r0 + rr;
        if (r >= n) break;
        const float bad = sT[rr * 28 + 27];
        f32x4 acc = {bad, bad, bad, bad};
        for (int k = 0; k < nk; ++k) {
            const float t = sT[rr * 28 + k];
            const f32x4 w4 = reinterpret_cast<const f32x4*>(sw)[k * h4n + h4];
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[e] = fmaf(t, w4[e], acc[e]);
        }
        reinterpret_cast<f32x4*>(G + (r * nj + j) * wh)[h4] = acc;
    }
}

// Its gradients: dL/dskts (the rotation block of joint j, atomically added: R_j d's gradient through the
// normalisation and the sin / cos) and dL/dWv (the view columns, atomically added once per workgroup).  Per chunk
// of VF_RC rays: dL/dG rows and T in LDS; dL/dT (lanes over rays, 28-float rows) and the dL/dWv partial sums (float4
// column groups per lane, in registers across the chunks); then one thread per ray maps dL/dT to dL/dR_j.
__global__ __launch_bounds__(256) void train_view_factor_backward_kernel(
    ModelDev M, const float* __restrict__ rb, int stride, int64_t n, const float* __restrict__ skts,
    const int32_t* __restrict__ ray_pose, int n_poses, const float* __restrict__ wv, int64_t ldv, int wh,
    const float* __restrict__ fs, const float* __restrict__ gG, float* __restrict__ gskts, float* __restrict__ part) {
    extern __shared__ float sh[];
    const int j = blockIdx.y, nj = M.nj, nk = 3 * (1 + 2 * M.mrv);
    const int wp = wh + 4, h4n = wh / 4, tid = threadIdx.x;
    float* sw = sh;               // [nk][wh]: Wv' (scaled)
    float* sZ = sw + nk * wh;     // [VF_RC][wp]: dL/dG rows of the chunk
    float* sT = sZ + VF_RC * wp;  // [VF_RC][28]: T
    float* sg = sT + VF_RC * 28;  // [VF_RC][28]: dL/dT
    stage_view_cols(M, j, wv, ldv, wh, fs, sw);
    f32x4 acc[VF_KG];
#pragma unroll
    for (int i = 0; i < VF_KG; ++i) acc[i] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    for (int c0 = 0; c0 < VF_RAYS_B; c0 += VF_RC) {
        const int64_t r0 = (int64_t)blockIdx.x * VF_RAYS_B + c0;
        if (r0 >= n) break;
        const int rc = (int)min<int64_t>(VF_RC, n - r0);
        __syncthreads();  // (the previous chunk's readers are done)
        float T[27], e[3], enr = 0.0f;
        int64_t pose = 0;
        bool ok = false;
        if (tid < rc) {
            ok = view_terms(M, rb, stride, r0 + tid, skts, ray_pose, n_poses, j, T, e, enr, pose);
#pragma unroll
            for (int k = 0; k < 27; ++k) sT[tid * 28 + k] = ok ? T[k] : 0.0f;  // (no gradient for a bad pose)
        }
        for (int q = tid; q < rc * h4n; q += blockDim.x) {
            const int rr = q / h4n, h4 = q - rr * h4n;
            *reinterpret_cast<f32x4*>(sZ + rr * wp + 4 * h4) =
                reinterpret_cast<const f32x4*>(gG + ((r0 + rr) * nj + j) * wh)[h4];
        }
        __syncthreads();
        // dL/dT[rr][k] = sum_h gG[rr][h] Wv'[k][h]: lanes over the rays, Wv' rows broadcast
        for (int q = tid; q < VF_RC * nk; q += blockDim.x) {
            const int rr = q % VF_RC, k = q / VF_RC;
            if (rr >= rc) continue;
            f32x4 d = {0.0f, 0.0f, 0.0f, 0.0f};
            for (int h = 0; h < wh; h += 4) {
                const f32x4 a = *reinterpret_cast<const f32x4*>(sZ + rr * wp + h);
                const f32x4 b = *reinterpret_cast<const f32x4*>(sw + k * wh + h);
#pragma unroll
                for (int u = 0; u < 4; ++u) d[u] = fmaf(a[u], b[u], d[u]);
            }
            sg[rr * 28 + k] = (d[0] + d[1]) + (d[2] + d[3]);
        }
        // dL/dWv'[k][h] += sum_rr T[rr][k] gG[rr][h]
#pragma unroll
        for (int i = 0; i < VF_KG; ++i) {
            const int g = tid + 256 * i;
            if (g < nk * h4n) {
                const int k = g / h4n, h4 = g - k * h4n;
                f32x4 a = acc[i];
                for (int rr = 0; rr < rc; ++rr) {
                    const float t = sT[rr * 28 + k];
                    const f32x4 z = *reinterpret_cast<const f32x4*>(sZ + rr * wp + 4 * h4);
#pragma unroll
                    for (int u = 0; u < 4; ++u) a[u] = fmaf(t, z[u], a[u]);
                }
                acc[i] = a;
            }
        }
        __syncthreads();
        if (tid < rc && ok) {  // dT/de (f = 0 the identity, sin / cos of 2^m e), the normalisation, x = R_j d
            float gT[27];
#pragma unroll
            for (int k = 0; k < 27; ++k) gT[k] = k < nk ? sg[tid * 28 + k] : 0.0f;
            float ge[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                ge[c] = gT[c];
#pragma unroll
                for (int fi = 0; fi < 4; ++fi) {
                    const float fr = (float)(1 << fi);
                    const float s = T[3 * (1 + 2 * fi) + c], co = T[3 * (2 + 2 * fi) + c];
                    if (fi < M.mrv) ge[c] += (gT[3 * (1 + 2 * fi) + c] * co - gT[3 * (2 + 2 * fi) + c] * s) * fr;
                }
            }
            float gx[3];
            if (M.view_raw) {
                gx[0] = ge[0], gx[1] = ge[1], gx[2] = ge[2];
            } else if (enr > 1e-12f) {
                const float dot = e[0] * ge[0] + e[1] * ge[1] + e[2] * ge[2];
#pragma unroll
                for (int c = 0; c < 3; ++c) gx[c] = (ge[c] - e[c] * dot) / enr;
            } else {
#pragma unroll
                for (int c = 0; c < 3; ++c) gx[c] = ge[c] / 1e-12f;
            }
            const float* ray = rb + (r0 + tid) * stride;
            float* gs = gskts + (pose * nj + j) * 16;
#pragma unroll
            for (int c = 0; c < 3; ++c)
#pragma unroll
                for (int b = 0; b < 3; ++b) atomicAdd(gs + 4 * c + b, gx[c] * ray[3 + b]);
        }
    }
    // the workgroup's dL/dWv' partial sums, part[blockIdx.x][j][k][h] (summed by train_view_factor_reduce_kernel)
    f32x4* pp = reinterpret_cast<f32x4*>(part + ((int64_t)blockIdx.x * nj + j) * nk * wh);
#pragma unroll
    for (int i = 0; i < VF_KG; ++i) {
        const int g = tid + 256 * i;
        if (g < nk * h4n) pp[g] = acc[i];
    }
}

// dL/dWv[h][col(k, j)] += fs[col] sum_b part[b][j][k][h]: one thread per (j, k, h), the nb partial sums in order
__global__ __launch_bounds__(256) void train_view_factor_reduce_kernel(const float* __restrict__ part, int nb, int nj,
                                                                       int nk, int wh, const float* __restrict__ fs,
                                                                       float* __restrict__ gwv, int64_t ldv) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t per = (int64_t)nj * nk * wh;
    if (q >= per) return;
    const int j = (int)(q / (nk * wh)), k = (int)(q / wh % nk), h = (int)(q % wh);
    float v = 0.0f;
    for (int b = 0; b < nb; ++b) v += part[b * per + q];
    const int col = (k / 3) * 3 * nj + 3 * j + k % 3;
    gwv[h * ldv + col] += v * (fs ? fs[col] : 1.0f);  // (one thread per element)
}

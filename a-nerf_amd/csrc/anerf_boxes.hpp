// anerf_boxes.hpp — per-frame bounding cylinder and 2-D pixel box on the device.
//
// Restates kp_to_valid_rays' host half (core/utils/ray_utils.py:83-136):
//   get_kp_bounding_cylinder (skeleton_utils.py:542-592) with extend_mm=250, top_expand_ratio=1.6,
//     bot_expand_ratio=1.1, head='-y' (ray_utils.py:89-104)                       float32, numpy's ops
//   cylinder_to_box_2d (skeleton_utils.py:607-694): 2 x 50 cap points, @ w2c^T, @ K^T, x/z, y/z,
//     floor/ceil, + int(W/2), int(H/2) (or int(center)), clip to [0, W-1] x [0, H-1]   float64
// (min/max skip NaN cap points, where numpy's would propagate them).
// with numpy's dtype flow so the integer boxes are the reference's: the cylinder is float32 (numpy
// float32 arrays with Python-float constants rounded to float32 first, NEP 50), the cap points are
// float64 (float64 cos/sin table of linspace(0, 2 pi, 50) — the host passes numpy's own values),
// the extrinsic w2c = inv(swap_mat(c2w)) and the intrinsic are float32 promoted to float64; the
// 4-term products are fma chains in k order (the BLAS dgemm micro-kernel's order).
#pragma once

namespace anerf {

constexpr int BOX_CAP_N = 50;

struct BoxArgs {
    const float* kps;       // [n_kp][NJ][3] or null (then cyls_in)
    const float* cyls_in;   // [n_kp][5]
    const float* w2cs;      // [F][4][4]
    const float* focals;    // [F][2] (fx, fy) as float32, like focal_to_intrinsic_np
    const int32_t* offsets; // [F][2] int(center) or null (int(W/2), int(H/2))
    const double* cap_dirs; // [50][2] cos, sin or null (device math)
    float* cyls_out;        // [n_kp][5] or null
    int32_t* boxes_out;     // [F][4]: x0, y0, x1, y1 (pixels y in [y0, y1), x in [x0, x1))
    int64_t n_kp, n_frames;
    int32_t nj, root, H, W;
    float ext, ext_top, ext_bot;  // float32(250 ext_scale), float32(ext * 1.6), float32(ext * 1.1)
};

__device__ inline void box_cylinder(const BoxArgs& a, int64_t k, int lane, float cyl[5]) {
    if (!a.kps) {
#pragma unroll
        for (int e = 0; e < 5; ++e) cyl[e] = a.cyls_in[k * 5 + e];
        return;
    }
    const float* kp = a.kps + k * a.nj * 3;
    const float rx = kp[a.root * 3 + 0], rz = kp[a.root * 3 + 2];
    float md = -INFINITY, mh = -INFINITY, nh = INFINITY;
    for (int j = lane; j < a.nj; j += 64) {
        const float dx = kp[j * 3 + 0] - rx, dz = kp[j * 3 + 2] - rz;
        md = fmaxf(md, sqrtf(dx * dx + dz * dz));
        const float h = -kp[j * 3 + 1];
        mh = fmaxf(mh, h);
        nh = fminf(nh, h);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        md = fmaxf(md, __shfl_xor(md, o));
        mh = fmaxf(mh, __shfl_xor(mh, o));
        nh = fminf(nh, __shfl_xor(nh, o));
    }
    cyl[0] = rx;
    cyl[1] = rz;
    cyl[2] = md + a.ext;
    cyl[3] = -(mh + a.ext_top);
    cyl[4] = -(nh - a.ext_bot);
}

// one wave per frame (and per kp set for the cylinder output)
__global__ __launch_bounds__(256) void kp_boxes_kernel(BoxArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= a.n_frames && i >= a.n_kp) return;
    if (i < a.n_kp && a.cyls_out) {
        float c[5];
        box_cylinder(a, i, lane, c);
        if (lane == 0)
#pragma unroll
            for (int e = 0; e < 5; ++e) a.cyls_out[i * 5 + e] = c[e];
    }
    if (i >= a.n_frames) return;
    float cyl[5];
    box_cylinder(a, i % a.n_kp, lane, cyl);
    const float* w = a.w2cs + i * 16;
    const double fx = a.focals[i * 2], fy = a.focals[i * 2 + 1];
    double xmax = -INFINITY, xmin = INFINITY, ymax = -INFINITY, ymin = INFINITY;
    if (lane < BOX_CAP_N) {
        double cs, sn;
        if (a.cap_dirs) {
            cs = a.cap_dirs[2 * lane];
            sn = a.cap_dirs[2 * lane + 1];
        } else {
            const double ang = (double)lane * (2.0 * M_PI / (BOX_CAP_N - 1));
            cs = cos(ang);
            sn = sin(ang);
        }
        const double r = cyl[2];
        const double px = (double)cyl[0] + cs * r, pz = (double)cyl[1] + sn * r;
#pragma unroll
        for (int cap = 0; cap < 2; ++cap) {
            const double py = cap == 0 ? (double)cyl[3] : (double)cyl[4];
            double c[3];
#pragma unroll
            for (int row = 0; row < 3; ++row) {
                double s = px * (double)w[4 * row + 0];
                s = fma(py, (double)w[4 * row + 1], s);
                s = fma(pz, (double)w[4 * row + 2], s);
                s = fma(1.0, (double)w[4 * row + 3], s);
                c[row] = s;
            }
            // @ K^T with K = [[fx,0,0,0],[0,fy,0,0],[0,0,1,0]]: the zero terms add nothing
            const double qx = (c[0] * fx) / c[2], qy = (c[1] * fy) / c[2];
            xmax = fmax(xmax, qx);
            xmin = fmin(xmin, qx);
            ymax = fmax(ymax, qy);
            ymin = fmin(ymin, qy);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        xmax = fmax(xmax, __shfl_xor(xmax, o));
        xmin = fmin(xmin, __shfl_xor(xmin, o));
        ymax = fmax(ymax, __shfl_xor(ymax, o));
        ymin = fmin(ymin, __shfl_xor(ymin, o));
    }
    if (lane == 0) {
        const int ox = a.offsets ? a.offsets[i * 2] : (int)(a.W * 0.5);
        const int oy = a.offsets ? a.offsets[i * 2 + 1] : (int)(a.H * 0.5);
        const int x0 = (int)floor(xmin) + ox, x1 = (int)ceil(xmax) + ox;
        const int y0 = (int)floor(ymin) + oy, y1 = (int)ceil(ymax) + oy;
        a.boxes_out[i * 4 + 0] = min(max(x0, 0), a.W - 1);
        a.boxes_out[i * 4 + 1] = min(max(y0, 0), a.H - 1);
        a.boxes_out[i * 4 + 2] = min(max(x1, 0), a.W - 1);
        a.boxes_out[i * 4 + 3] = min(max(y1, 0), a.H - 1);
    }
}

}  // namespace anerf

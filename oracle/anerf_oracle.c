/*
 * anerf_oracle.c — CPU restatement of the A-NeRF render path.  TEST INFRASTRUCTURE ONLY.
 *
 * This file is the parity oracle (and the "port" CPU baseline timed by bench.py).  It is
 * never linked into, called by, or shipped with the product path in a-nerf_amd/; only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it.
 *
 * Pinned against the reference's own outputs: the .npz fixtures in tests/golden/ come from
 * tests/golden/make_golden.py, which runs /root/reference's Python render path
 * (run_nerf.render_path, core.trainer.render, RayCaster stages) on synthetic inputs.
 *
 * Each function cites the reference code it restates (paths relative to /root/reference):
 *   linspace              torch.linspace (float32) as used by ray_utils.py:218, 166
 *   near/far + NaN fill   core/utils/ray_utils.py:292-344 (np.nanmean = numpy pairwise f32 sum)
 *   sample_from_lineseg   core/utils/ray_utils.py:204-251 (det, no lindisp)
 *   encode                core/raycasters.py:476-555, core/encoders.py:8-37,101-122,172-193,
 *                         core/cutoff_embedder.py:111-174
 *   NeRF MLP              core/networks/nerf.py:90-148
 *   raw2outputs           core/networks/nerf.py:150-205 (torch CPU cumprod accumulates in double)
 *   sample_pdf / isample  core/utils/ray_utils.py:157-201, 255-289 (cumsum in double)
 *   render_rays           core/raycasters.py:361-474 (fine net on all S+I merged samples)
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define MAXL 16

typedef struct {
    const float* w[MAXL]; /* pts_linears[i].weight TRANSPOSED: [in][out] */
    const float* b[MAXL];
    const float *wa, *ba;     /* alpha_linear   [1][W]                        */
    const float *wf, *bf;     /* feature_linear, transposed [W][W]            */
    const float *wv, *bv;     /* views_linears.0, transposed [W + Cv (+ Cfc)][W/2] */
    const float *wrgb, *brgb; /* rgb_linear, torch layout [3][W/2]            */
    const float* codes;       /* framecodes.codes.weight [n_codes][Cfc] / NULL */
} oracle_net;

typedef struct {
    int nj, D, W, skip;          /* skip: layer index i in `skips` (4): layer i+1 takes [x, h] */
    int multires, multires_views;
    int use_cutoff, cutoff_inputs, cutoff_viewdir;
    int framecode_ch, n_framecodes; /* 0 when opt_framecode is off */
    int density_softplus;
    float softplus_shift, density_scale;
    float tau, tau_v;
    const float* cutoff;   /* embed_fn.cutoff_dist (NJ)     */
    const float* cutoff_v; /* embeddirs_fn.cutoff_dist (NJ) */
    int has_fine;
    int single_net; /* network_fine IS network_fn; fine pass on the I new samples only (raycasters.py:462-468) */
    int lindisp;    /* sample_from_lineseg in inverse depth (ray_utils.py:223-226) */
    /* --freq_schedule: weight of frequency k (its sin and cos) in the pts / view cutoff embedders,
     * CutoffEmbedder.get_schedule_w (cutoff_embedder.py:192-197), applied before the cutoff window
     * as `embedded * get_schedule_w()` then `* w` (:150-154); NULL = no schedule */
    const float* sched_w;
    const float* sched_wv;
    /* --cut_to_dist / --cutoff_shift (kp CutoffEmbedder only, cutoff_embedder.py:125-134): the raw
     * input is c_j - dist, the frequencies take (input * (2 / c_j) - 1); the window keeps dist */
    int cut_to, shift_in;
    oracle_net coarse, fine;
    /* --cutoff_bones (raycasters.py:52-64): the bone embedder is a CutoffEmbedder(dist_inputs=True);
     * with multires_bones 0 and cutoff_inputs its output is the bone direction times
     * w_b = 1 - sigmoid(tau_b (dist - c_b)) (cutoff_embedder.py:108-121, 143-158) */
    int bone_cut;
    float tau_b;
    const float* cutoff_b; /* embedbones_fn.cutoff_dist (NJ) */
    /* --view_type world (raycasters.py:279-280): IdentityExpandEncoder of the joint-frame ray
     * directions, i.e. R_j d without the VecNorm normalisation (encoders.py:71-79) */
    int view_raw;
} oracle_model;

/* ---------------------------------------------------------------- small helpers */

/* torch.linspace(0, 1, n) for float32 on CPU: step rounded to float, values in double. */
void oracle_linspace(int n, float* out) {
    if (n == 1) { out[0] = 0.0f; return; }
    float step = 1.0f / (float)(n - 1);
    int half = n / 2;
    for (int i = 0; i < n; ++i)
        out[i] = (i < half) ? (float)((double)step * i) : (float)(1.0 - (double)step * (n - 1 - i));
}

static float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

/* numpy pairwise summation of float32 (numpy/_core/src/umath/loops_utils.h.src) */
static float pairwise_sum_f32(const float* a, int64_t n) {
    if (n < 8) {
        float res = 0.0f;
        for (int64_t i = 0; i < n; ++i) res += a[i];
        return res;
    } else if (n <= 128) {
        float r[8];
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        int64_t i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] += a[i + j];
        float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    } else {
        int64_t n2 = n / 2;
        n2 -= n2 % 8;
        return pairwise_sum_f32(a, n2) + pairwise_sum_f32(a + n2, n - n2);
    }
}

/* ---- torch CPU float32 sum (aten SumKernel cascade_sum), verified bit-exact against
 * torch.sum on this image for n <= 5000: contiguous rows of n >= 8 use 8-wide vector
 * accumulators, shorter / strided rows the scalar 4-way ILP path; both with the
 * multi-level cascade of multi_row_sum. */
static int ceil_log2_(int64_t x) {
    int r = 0;
    while (((int64_t)1 << r) < x) ++r;
    return r;
}

/* multi_row_sum<nrows=4> over `size` rows of 4 elements, each element `w` lanes wide.
 * elem(r, k, l) = x[(4 * r + k) * w * xs + l * xs]; result part[4][w]. */
static void multi_row_sum_(const float* x, int64_t xs, int w, int64_t size, float part[4][8]) {
    const int num_levels = 4;
    int lp = ceil_log2_(size) / num_levels;
    if (lp < 4) lp = 4;
    const int64_t step = (int64_t)1 << lp, mask = step - 1;
    float acc[4][4][8];
    memset(acc, 0, sizeof(acc));
    int64_t i = 0;
    while (i + step <= size) {
        for (int64_t j = 0; j < step; ++j, ++i)
            for (int k = 0; k < 4; ++k)
                for (int l = 0; l < w; ++l) acc[0][k][l] += x[((4 * i + k) * w + l) * xs];
        for (int j = 1; j < num_levels; ++j) {
            for (int k = 0; k < 4; ++k)
                for (int l = 0; l < w; ++l) {
                    acc[j][k][l] += acc[j - 1][k][l];
                    acc[j - 1][k][l] = 0.0f;
                }
            if ((i & (mask << (j * lp))) != 0) break;
        }
    }
    for (; i < size; ++i)
        for (int k = 0; k < 4; ++k)
            for (int l = 0; l < w; ++l) acc[0][k][l] += x[((4 * i + k) * w + l) * xs];
    for (int j = 1; j < num_levels; ++j)
        for (int k = 0; k < 4; ++k)
            for (int l = 0; l < w; ++l) acc[0][k][l] += acc[j][k][l];
    for (int k = 0; k < 4; ++k)
        for (int l = 0; l < w; ++l) part[k][l] = acc[0][k][l];
}

/* row_sum<ilp=4> over n elements of width w (stride xs between scalars) -> out[w] */
static void row_sum_(const float* x, int64_t xs, int w, int64_t n, float* out) {
    float part[4][8];
    int64_t n_ilp = n / 4;
    multi_row_sum_(x, xs, w, n_ilp, part);
    for (int64_t i = n_ilp * 4; i < n; ++i)
        for (int l = 0; l < w; ++l) part[0][l] += x[(i * w + l) * xs];
    for (int k = 1; k < 4; ++k)
        for (int l = 0; l < w; ++l) part[0][l] += part[k][l];
    for (int l = 0; l < w; ++l) out[l] = part[0][l];
}

/* torch.sum(x[0:n]) for a contiguous float32 row */
static float torch_sum_f32(const float* x, int64_t n) {
    float r[8];
    if (n >= 8) {
        int64_t nv = n / 8;
        row_sum_(x, 1, 8, nv, r);
        float fin = 0.0f;
        for (int64_t k = nv * 8; k < n; ++k) fin += x[k];
        for (int l = 0; l < 8; ++l) fin += r[l];
        return fin;
    }
    row_sum_(x, 1, 1, n, r);
    return r[0];
}

/* torch.sum over a strided (non-inner) dim, e.g. (N,S,3).sum(-2): scalar row_sum */
static float torch_sum_strided_f32(const float* x, int64_t stride, int64_t n) {
    float r[1];
    row_sum_(x, stride, 1, n, r);
    return r[0];
}

float oracle_torch_sum(const float* x, int64_t n) { return torch_sum_f32(x, n); }
float oracle_torch_sum_strided(const float* x, int64_t stride, int64_t n) { return torch_sum_strided_f32(x, stride, n); }

/* torch.norm(v, dim=-1) on CPU is an fma chain: sqrt(fma(x2,x2,fma(x1,x1,x0*x0))) */
static float norm3_(float a, float b, float c) { return sqrtf(fmaf(c, c, fmaf(b, b, a * a))); }
static float norm2_(float a, float b) { return sqrtf(fmaf(b, b, a * a)); }

/* float32(np.nanmean(x)) ; NaN if every entry is NaN */
static float nanmean_f32(const float* x, int64_t n, float* scratch) {
    int64_t cnt = 0;
    for (int64_t i = 0; i < n; ++i) {
        int nan = isnan(x[i]);
        scratch[i] = nan ? 0.0f : x[i];
        cnt += !nan;
    }
    if (cnt == 0) return NAN;
    float tot = pairwise_sum_f32(scratch, n);
    return (float)((double)tot / (double)cnt);
}

/* ---------------------------------------------------------------- near / far */

/* get_near_far_in_cylinder (ray_utils.py:292-344) for rays [0,n), NaN-filled per chunk of
 * `chunk` rays (the batchify_rays chunk of core/trainer.py:64-79). Returns #filled rays. */
int64_t oracle_near_far(const float* rb, int stride, int64_t n, const float* cyls, const int32_t* ray_pose,
                        int chunk, float* near_out, float* far_out, float* q_out) {
    int64_t filled = 0;
    float* scratch = (float*)malloc(sizeof(float) * (size_t)(chunk > 0 ? chunk : 1));
    for (int64_t c0 = 0; c0 < n; c0 += chunk) {
        int64_t c1 = c0 + chunk < n ? c0 + chunk : n;
        int any_nan = 0;
        for (int64_t i = c0; i < c1; ++i) {
            const float* r = rb + i * stride;
            const float* cy = cyls + 5 * (ray_pose ? ray_pose[i] : 0);
            float near = r[6], far = r[7];
            /* g_axes = [0, -1] -> x, z */
            float o0 = r[0], o2 = r[2], d0 = r[3], d2 = r[5];
            float rn0 = o0 + d0 * near, rn1 = o2 + d2 * near;
            float rf0 = o0 + d0 * far, rf1 = o2 + d2 * far;
            float nc0 = cy[0] - rn0, nc1 = cy[1] - rn1;
            float nf0 = rf0 - rn0, nf1 = rf1 - rn1;
            float nfn = norm2_(nf0, nf1);
            float scale = norm2_(d0, d2);
            float cross = nc0 * nf1 - nc1 * nf0;
            float dist = fabsf(cross) / nfn;
            float rad = cy[2];
            float Q = sqrtf(rad * rad - dist * dist);
            float K = (nc0 * nf0 + nc1 * nf1) / nfn;
            float mask = (Q < K) ? 1.0f : 0.0f;
            float nn = near + (mask * (K - Q)) / scale;
            float nf = near + (K + Q) / scale;
            near_out[i] = nn;
            far_out[i] = nf;
            if (q_out) q_out[i] = Q;
            if (isnan(nn)) any_nan = 1;
        }
        if (any_nan) {
            float mn = nanmean_f32(near_out + c0, c1 - c0, scratch);
            float mf = nanmean_f32(far_out + c0, c1 - c0, scratch);
            for (int64_t i = c0; i < c1; ++i) {
                const float* r = rb + i * stride;
                const float* cy = cyls + 5 * (ray_pose ? ray_pose[i] : 0);
                /* recompute Q's NaN-ness (the fill keys on isnan(Q), ray_utils.py:331) */
                float d0 = r[3], d2 = r[5], o0 = r[0], o2 = r[2], near = r[6], far = r[7];
                float rn0 = o0 + d0 * near, rn1 = o2 + d2 * near;
                float rf0 = o0 + d0 * far, rf1 = o2 + d2 * far;
                float nc0 = cy[0] - rn0, nc1 = cy[1] - rn1;
                float nf0 = rf0 - rn0, nf1 = rf1 - rn1;
                float nfn = norm2_(nf0, nf1);
                float dist = fabsf(nc0 * nf1 - nc1 * nf0) / nfn;
                float Q = sqrtf(cy[2] * cy[2] - dist * dist);
                if (isnan(Q)) {
                    near_out[i] = isnan(mn) ? near : mn;
                    far_out[i] = isnan(mf) ? far : mf;
                    ++filled;
                }
            }
        }
    }
    free(scratch);
    return filled;
}

/* ---------------------------------------------------------------- encoding */

static int feat_dims(const oracle_model* m, int* cx, int* cv) {
    int nj = m->nj;
    int cin = nj * (1 + 2 * m->multires) + 3 * nj; /* v + r */
    int cvw = 3 * nj * (1 + 2 * m->multires_views);
    if (cx) *cx = cin;
    if (cv) *cv = cvw;
    return cin + cvw;
}

int oracle_feature_dim(const oracle_model* m) { return feat_dims(m, NULL, NULL); }

/* Features of one sample point p on a ray with direction d, in MLP input order
 * [v (k*NJ+j), r (3j+c), dv (k*3NJ+3j+c)]  (raycasters.py:560-569). */
static void encode_point(const oracle_model* m, const float* skts, const float p[3], const float d[3],
                         float* feat) {
    const int nj = m->nj, nfk = m->multires, nfv = m->multires_views;
    int cx, cv;
    feat_dims(m, &cx, &cv);
    float* fv = feat;
    float* fr = feat + nj * (1 + 2 * nfk);
    float* fd = feat + cx;
    for (int j = 0; j < nj; ++j) {
        const float* S = skts + 16 * j;
        /* transform_batch_pts: skt @ [p; 1] (encoders.py:8-23) */
        float q[3];
        for (int r = 0; r < 3; ++r)
            q[r] = fmaf(S[4 * r + 3], 1.0f, fmaf(S[4 * r + 2], p[2], fmaf(S[4 * r + 1], p[1], S[4 * r + 0] * p[0])));
        float dist = norm3_(q[0], q[1], q[2]); /* RelDistEncoder */
        float dn = dist > 1e-12f ? dist : 1e-12f;                    /* F.normalize eps */
        fr[3 * j + 0] = q[0] / dn;
        fr[3 * j + 1] = q[1] / dn;
        fr[3 * j + 2] = q[2] / dn;
        if (m->bone_cut) { /* cat([inputs], embedded) * w, w on the dist expanded per coordinate */
            const float wb = 1.0f - sigmoidf_(m->tau_b * (dist - m->cutoff_b[j]));
            for (int c = 0; c < 3; ++c) fr[3 * j + c] *= wb;
        }
        /* kp block: CutoffEmbedder(dist_inputs=False) (cutoff_embedder.py:125-158) */
        float w = 1.0f;
        if (m->use_cutoff) w = 1.0f - sigmoidf_(m->tau * (dist - m->cutoff[j]));
        float u = dist, uf = dist;
        if (m->use_cutoff && m->cut_to) u = m->cutoff[j] - dist; /* inputs = cutoff - inputs */
        uf = u;
        if (m->use_cutoff && m->shift_in) {                       /* shifted = inputs * (2 / c) - 1 */
            const float k2 = 2.0f / m->cutoff[j];
            uf = u * k2 - 1.0f;
        }
        fv[j] = (m->use_cutoff && m->cutoff_inputs) ? u * w : u;
        for (int f = 0; f < nfk; ++f) {
            float a = uf * (float)(1 << f);
            if (m->sched_w && m->use_cutoff) {
                fv[(1 + 2 * f) * nj + j] = (sinf(a) * m->sched_w[f]) * w;
                fv[(2 + 2 * f) * nj + j] = (cosf(a) * m->sched_w[f]) * w;
            } else {
                fv[(1 + 2 * f) * nj + j] = sinf(a) * w;
                fv[(2 + 2 * f) * nj + j] = cosf(a) * w;
            }
        }
        /* view block: rays rotated into the joint frame, normalised (encoders.py:25-37, 181-193) */
        float e[3];
        for (int r = 0; r < 3; ++r) e[r] = fmaf(S[4 * r + 2], d[2], fmaf(S[4 * r + 1], d[1], S[4 * r + 0] * d[0]));
        float en = norm3_(e[0], e[1], e[2]);
        en = en > 1e-12f ? en : 1e-12f;
        if (m->view_raw) en = 1.0f; /* (x = e[c] / 1 = e[c]) */
        float wv = 1.0f;
        if (m->cutoff_viewdir) wv = 1.0f - sigmoidf_(m->tau_v * (dist - m->cutoff_v[j]));
        for (int c = 0; c < 3; ++c) {
            float x = e[c] / en;
            fd[3 * j + c] = (m->cutoff_viewdir && m->cutoff_inputs) ? x * wv : x;
            for (int f = 0; f < nfv; ++f) {
                float a = x * (float)(1 << f);
                if (m->sched_wv && m->cutoff_viewdir) {
                    fd[(1 + 2 * f) * 3 * nj + 3 * j + c] = (sinf(a) * m->sched_wv[f]) * wv;
                    fd[(2 + 2 * f) * 3 * nj + 3 * j + c] = (cosf(a) * m->sched_wv[f]) * wv;
                } else {
                    fd[(1 + 2 * f) * 3 * nj + 3 * j + c] = sinf(a) * wv;
                    fd[(2 + 2 * f) * 3 * nj + 3 * j + c] = cosf(a) * wv;
                }
            }
        }
    }
}

/* Stage entry: features for M points (pts M×3, dirs M×3: each point's ray direction). */
void oracle_encode(const oracle_model* m, const float* skts, const float* pts, const float* dirs, int64_t M,
                   float* feat) {
    int F = oracle_feature_dim(m);
    for (int64_t i = 0; i < M; ++i) encode_point(m, skts, pts + 3 * i, dirs + 3 * i, feat + i * F);
}

/* ---------------------------------------------------------------- MLP */

/* out[M][n_out] (row stride ldo) (+)= X[M][K] (row stride ldx) @ Wt[w0 : w0+K][n_out] (+ b).
 * Wt is the TRANSPOSED torch weight ([in][out]) so the inner loop runs over outputs and
 * vectorises without reassociating any sum: every output accumulates in k order. */
static void linear(const float* X, int ldx, int M, int K, const float* Wt, int w0, const float* b, int n_out,
                   float* out, int ldo, int accumulate) {
    int m = 0;
    for (; m + 4 <= M; m += 4) {
        float* o0 = out + (size_t)(m + 0) * ldo;
        float* o1 = out + (size_t)(m + 1) * ldo;
        float* o2 = out + (size_t)(m + 2) * ldo;
        float* o3 = out + (size_t)(m + 3) * ldo;
        if (!accumulate)
            for (int n = 0; n < n_out; ++n) o0[n] = o1[n] = o2[n] = o3[n] = 0.0f;
        const float* x0 = X + (size_t)(m + 0) * ldx;
        const float* x1 = X + (size_t)(m + 1) * ldx;
        const float* x2 = X + (size_t)(m + 2) * ldx;
        const float* x3 = X + (size_t)(m + 3) * ldx;
        for (int k = 0; k < K; ++k) {
            const float* w = Wt + (size_t)(w0 + k) * n_out;
            float a0 = x0[k], a1 = x1[k], a2 = x2[k], a3 = x3[k];
            for (int n = 0; n < n_out; ++n) {
                float wn = w[n];
                o0[n] += a0 * wn;
                o1[n] += a1 * wn;
                o2[n] += a2 * wn;
                o3[n] += a3 * wn;
            }
        }
        if (!accumulate && b)
            for (int n = 0; n < n_out; ++n) { o0[n] += b[n]; o1[n] += b[n]; o2[n] += b[n]; o3[n] += b[n]; }
    }
    for (; m < M; ++m) {
        float* o = out + (size_t)m * ldo;
        const float* x = X + (size_t)m * ldx;
        if (!accumulate)
            for (int n = 0; n < n_out; ++n) o[n] = 0.0f;
        for (int k = 0; k < K; ++k) {
            const float* w = Wt + (size_t)(w0 + k) * n_out;
            float a = x[k];
            for (int n = 0; n < n_out; ++n) o[n] += a * w[n];
        }
        if (!accumulate && b)
            for (int n = 0; n < n_out; ++n) o[n] += b[n];
    }
}

static void relu_(float* x, size_t n) {
    for (size_t i = 0; i < n; ++i) x[i] = x[i] > 0.0f ? x[i] : 0.0f;
}

/* NeRF.forward (nerf.py:133-148) for M feature rows; code: per-row framecode (M×Cfc) or NULL */
static void network_forward(const oracle_model* m, const oracle_net* net, const float* feat, int M,
                            const float* code, float* raw, float* buf) {
    const int W = m->W, D = m->D, Wh = W / 2;
    int cx, cv;
    int F = feat_dims(m, &cx, &cv);
    const int cfc = m->framecode_ch;
    float* h0 = buf;
    float* h1 = buf + (size_t)M * W;
    float* g = buf + (size_t)2 * M * W;
    /* layer 0 */
    linear(feat, F, M, cx, net->w[0], 0, net->b[0], W, h0, W, 0);
    relu_(h0, (size_t)M * W);
    float* hin = h0;
    float* hout = h1;
    for (int i = 1; i < D; ++i) {
        if (i == m->skip + 1) {
            /* input = cat([x, h]) (nerf.py:100-101): x part first */
            linear(feat, F, M, cx, net->w[i], 0, net->b[i], W, hout, W, 0);
            linear(hin, W, M, W, net->w[i], cx, NULL, W, hout, W, 1);
        } else {
            linear(hin, W, M, W, net->w[i], 0, net->b[i], W, hout, W, 0);
        }
        relu_(hout, (size_t)M * W);
        float* t = hin;
        hin = hout;
        hout = t;
    }
    /* alpha, feature (no activation), view layer, rgb (nerf.py:114-131, 140-144) */
    float* feat_lin = hout;
    linear(hin, W, M, W, net->wf, 0, net->bf, W, feat_lin, W, 0);
    linear(feat_lin, W, M, W, net->wv, 0, net->bv, Wh, g, Wh, 0);
    linear(feat + cx, F, M, cv, net->wv, W, NULL, Wh, g, Wh, 1);
    if (cfc) linear(code, cfc, M, cfc, net->wv, W + cv, NULL, Wh, g, Wh, 1);
    relu_(g, (size_t)M * Wh);
    for (int s = 0; s < M; ++s) {
        float a = 0.0f;
        for (int k = 0; k < W; ++k) a += hin[(size_t)s * W + k] * net->wa[k];
        raw[4 * s + 3] = a + net->ba[0];
        for (int c = 0; c < 3; ++c) {
            float acc = 0.0f;
            for (int k = 0; k < Wh; ++k) acc += g[(size_t)s * Wh + k] * net->wrgb[c * Wh + k];
            raw[4 * s + c] = acc + net->brgb[c];
        }
    }
}

static size_t net_buf_floats(const oracle_model* m, int M) { return (size_t)M * (2 * m->W + m->W / 2); }

/* Stage entry: raw (M×4) of `fine`'s network for M feature rows (code rows optional). */
void oracle_network(const oracle_model* m, int fine, const float* feat, int64_t M, const float* code,
                    float* raw) {
    const oracle_net* net = fine ? &m->fine : &m->coarse;
    const int B = 256;
    int cfc = m->framecode_ch;
    float* buf = (float*)malloc(sizeof(float) * net_buf_floats(m, B));
    for (int64_t s0 = 0; s0 < M; s0 += B) {
        int n = (int)((M - s0) < B ? (M - s0) : B);
        network_forward(m, net, feat + (size_t)s0 * oracle_feature_dim(m), n, code ? code + s0 * cfc : NULL,
                        raw + 4 * s0, buf);
    }
    free(buf);
}

/* ---------------------------------------------------------------- compositing */

static float density_act(const oracle_model* m, float x) {
    if (!m->density_softplus) return x > 0.0f ? x : 0.0f;
    float y = x - m->softplus_shift; /* F.softplus(beta=1, threshold=20) */
    return y > 20.0f ? y : log1pf(expf(y));
}

/* raw2outputs (nerf.py:150-205) for one ray of n samples (n <= 4096).
 * weights/alpha outputs have length n; scratch holds 4*n floats. */
static void raw2outputs(const oracle_model* m, const float* raw, const float* z, int n, const float* d,
                        float* rgb, float* disp, float* acc, float* weights, float* alpha, float* scratch) {
    float dn = norm3_(d[0], d[1], d[2]);
    float* wz = scratch;
    float* wc = scratch + n; /* (n,3) */
    double T = 1.0;          /* torch CPU cumprod accumulates in double */
    for (int i = 0; i < n; ++i) {
        float dist = (i + 1 < n) ? (z[i + 1] - z[i]) : 1e10f;
        dist = dist * dn;
        float a = 1.0f - expf(-density_act(m, raw[4 * i + 3] / m->density_scale) * dist);
        float w = a * (float)T;
        T *= (double)((1.0f - a) + 1e-10f);
        alpha[i] = a;
        weights[i] = w;
        for (int c = 0; c < 3; ++c) wc[3 * i + c] = w * (sigmoidf_(raw[4 * i + c]) * 1.002f - 0.001f);
        wz[i] = w * z[i];
    }
    for (int c = 0; c < 3; ++c) rgb[c] = torch_sum_strided_f32(wc + c, 3, n);
    float accf = torch_sum_f32(weights, n), depth = torch_sum_f32(wz, n);
    float ratio = depth / (accf + 1e-10f);
    float dsp = 1.0f / (ratio > 1e-10f ? ratio : 1e-10f);
    if (fabsf(accf) <= 1e-8f) dsp = 0.0f; /* torch.isclose(acc, 0): |acc| <= atol */
    *disp = dsp;
    *acc = accf < 1.0f ? accf : 1.0f;
}

/* sample_pdf(det=True) (ray_utils.py:157-201) over bins (nb) and weights (nb-1).
 * scratch: 2*nb floats. */
static void sample_pdf(const float* bins, const float* wts, int nb, int n_samples, const float* u,
                       float* out, float* scratch) {
    int nw = nb - 1;
    float* wp = scratch;
    float* cdf = scratch + nb;
    for (int i = 0; i < nw; ++i) wp[i] = wts[i] + 1e-5f;
    float sum = torch_sum_f32(wp, nw);
    double c = 0;
    cdf[0] = 0.0f;
    for (int i = 0; i < nw; ++i) {
        c += (double)(wp[i] / sum); /* torch CPU cumsum accumulates in double */
        cdf[i + 1] = (float)c;
    }
    for (int k = 0; k < n_samples; ++k) {
        /* searchsorted(right=True): number of cdf entries <= u */
        int lo = 0, hi = nb;
        while (lo < hi) {
            int mid = (lo + hi) >> 1;
            if (cdf[mid] <= u[k]) lo = mid + 1; else hi = mid;
        }
        int ind = lo;
        int below = ind - 1 > 0 ? ind - 1 : 0;
        int above = ind < nb - 1 ? ind : nb - 1;
        float cb = cdf[below], ca = cdf[above];
        float bb = bins[below], ba = bins[above];
        float denom = ca - cb;
        if (denom < 1e-5f) denom = 1.0f;
        float t = (u[k] - cb) / denom;
        out[k] = bb + t * (ba - bb);
    }
}

static int cmp_float(const void* a, const void* b) {
    float x = *(const float*)a, y = *(const float*)b;
    if (isnan(x)) return isnan(y) ? 0 : 1;
    if (isnan(y)) return -1;
    return (x > y) - (x < y);
}

/* ---------------------------------------------------------------- render_rays */

static void ray_code(const oracle_model* m, const oracle_net* net, const float* cams, int64_t i, float* code) {
    int cfc = m->framecode_ch;
    if (!cfc) return;
    float cam = cams ? cams[i] : -1.0f;
    if (cam < 0.0f) { /* eval-mode mean code (embedding.py:23-24) */
        for (int c = 0; c < cfc; ++c) {
            double s = 0;
            for (int k = 0; k < m->n_framecodes; ++k) s += net->codes[k * cfc + c];
            code[c] = (float)(s / m->n_framecodes);
        }
    } else {
        int64_t idx = (int64_t)cam;
        for (int c = 0; c < cfc; ++c) code[c] = net->codes[idx * cfc + c];
    }
}

/* encode + MLP over n samples z of one ray: raw [n][4] */
static void ray_raw(const oracle_model* m, const oracle_net* net, const float* o, const float* d,
                    const float* skts, const float* code, const float* z, int n, float* feat, float* raw,
                    float* codes_rows, float* buf) {
    int F = oracle_feature_dim(m);
    int cfc = m->framecode_ch;
    for (int s = 0; s < n; ++s) {
        float p[3];
        for (int c = 0; c < 3; ++c) p[c] = o[c] + d[c] * z[s]; /* sample_pts (raycasters.py:658) */
        encode_point(m, skts, p, d, feat + (size_t)s * F);
        if (cfc) memcpy(codes_rows + (size_t)s * cfc, code, sizeof(float) * cfc);
    }
    const int B = 64;
    for (int s0 = 0; s0 < n; s0 += B) {
        int nb = n - s0 < B ? n - s0 : B;
        network_forward(m, net, feat + (size_t)s0 * F, nb, cfc ? codes_rows + (size_t)s0 * cfc : NULL,
                        raw + 4 * s0, buf);
    }
}

/* One pass (encode + MLP + composite) over n samples z of ray i */
static void ray_pass(const oracle_model* m, const oracle_net* net, const float* o, const float* d,
                     const float* skts, const float* code, const float* z, int n, float* feat, float* raw,
                     float* codes_rows, float* buf, float* rgb, float* disp, float* acc, float* weights,
                     float* alpha) {
    ray_raw(m, net, o, d, skts, code, z, n, feat, raw, codes_rows, buf);
    raw2outputs(m, raw, z, n, d, rgb, disp, acc, weights, alpha, buf);
}

/* torch.maximum: NaN if either operand is NaN */
static float torch_maximum_(float a, float b) { return (isnan(a) || a > b) ? a : b; }

/* argsort of z[0..n) by value (NaN last), ties by index: torch.sort's values (hazard H9) */
static _Thread_local const float* g_sort_keys;  /* per OpenMP thread */
static int cmp_idx(const void* a, const void* b) {
    int i = *(const int*)a, j = *(const int*)b;
    int c = cmp_float(g_sort_keys + i, g_sort_keys + j);
    return c ? c : (i > j) - (i < j);
}

/* near_in / far_in (optional, both or neither): the rays' near / far after the chunk NaN fill,
 * e.g. of the whole frame when rb is a sample of its rays (the fill couples a chunk's rays). */
int oracle_render_rays(const oracle_model* m, const float* rb, int stride, int64_t n, const float* skts,
                       const float* cyls, const int32_t* ray_pose, const float* cams, int S, int I, int chunk,
                       int nthreads, float* rgb, float* disp, float* acc, float* rgb0, float* disp0,
                       float* acc0, float* alpha, float* alpha0, float* z_out, const float* near_in,
                       const float* far_in) {
    if (n <= 0) return 0;
    if (I > 0 && !m->has_fine && !m->single_net) return -1;
    float* near = (float*)malloc(sizeof(float) * n);
    float* far = (float*)malloc(sizeof(float) * n);
    if (near_in && far_in) {
        memcpy(near, near_in, sizeof(float) * n);
        memcpy(far, far_in, sizeof(float) * n);
    } else {
        oracle_near_far(rb, stride, n, cyls, ray_pose, chunk, near, far, NULL);
    }
    const int T = S + I;
    const int F = oracle_feature_dim(m);
    const int cfc = m->framecode_ch;
    float* tv = (float*)malloc(sizeof(float) * S);
    float* uv = (float*)malloc(sizeof(float) * (I > 0 ? I : 1));
    oracle_linspace(S, tv);
    if (I > 0) oracle_linspace(I, uv);
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel
    {
        float* feat = (float*)malloc(sizeof(float) * (size_t)T * F);
        float* raw = (float*)malloc(sizeof(float) * 4 * T);
        size_t nbuf = net_buf_floats(m, 64);
        if (nbuf < (size_t)4 * T) nbuf = (size_t)4 * T;
        float* buf = (float*)malloc(sizeof(float) * nbuf);
        float* codes_rows = (float*)malloc(sizeof(float) * (size_t)T * (cfc ? cfc : 1));
        float* z = (float*)malloc(sizeof(float) * T);
        float* w = (float*)malloc(sizeof(float) * T);
        float* al = (float*)malloc(sizeof(float) * T);
        float* mids = (float*)malloc(sizeof(float) * S);
        float* cdf = (float*)malloc(sizeof(float) * 2 * S);
        float* zm = (float*)malloc(sizeof(float) * T);
        float* rawm = (float*)malloc(sizeof(float) * 4 * T);
        int* order = (int*)malloc(sizeof(int) * T);
        float code[64];
#pragma omp for schedule(dynamic, 4)
        for (int64_t i = 0; i < n; ++i) {
            const float* r = rb + i * stride;
            const float* o = r;
            const float* d = r + 3;
            const float* sk = skts + (size_t)16 * m->nj * (ray_pose ? ray_pose[i] : 0);
            /* sample_from_lineseg (ray_utils.py:218-229) */
            for (int s = 0; s < S; ++s)
                z[s] = m->lindisp ? 1.0f / ((1.0f / near[i]) * (1.0f - tv[s]) + (1.0f / far[i]) * tv[s])
                                  : near[i] * (1.0f - tv[s]) + far[i] * tv[s];
            ray_code(m, &m->coarse, cams, i, code);
            float c_rgb[3], c_disp, c_acc;
            ray_pass(m, &m->coarse, o, d, sk, code, z, S, feat, raw, codes_rows, buf, c_rgb, &c_disp, &c_acc, w,
                     al);
            if (I == 0) {
                for (int c = 0; c < 3; ++c) rgb[3 * i + c] = c_rgb[c];
                disp[i] = c_disp;
                acc[i] = c_acc;
                if (alpha) memcpy(alpha + (size_t)i * S, al, sizeof(float) * S);
                if (z_out) memcpy(z_out + (size_t)i * S, z, sizeof(float) * S);
                continue;
            }
            if (rgb0) for (int c = 0; c < 3; ++c) rgb0[3 * i + c] = c_rgb[c];
            if (disp0) disp0[i] = c_disp;
            if (acc0) acc0[i] = c_acc;
            if (alpha0) memcpy(alpha0 + (size_t)i * S, al, sizeof(float) * S);
            /* isample_from_lineseg (ray_utils.py:255-289) */
            for (int s = 0; s + 1 < S; ++s) mids[s] = 0.5f * (z[s + 1] + z[s]);
            if (m->single_net) {
                /* is_only weights (ray_utils.py:270-277), written over w[0..S-2) (read left to right) */
                for (int k = 0; k + 2 < S; ++k)
                    w[k] = 0.5f * (torch_maximum_(w[k], w[k + 1]) + torch_maximum_(w[k + 1], w[k + 2])) + 0.01f;
                sample_pdf(mids, w, S - 1, I, uv, z + S, cdf);
                /* the same net on the I new samples only, raws after the coarse ones (cat order),
                 * then both merged by sorted_idx (raycasters.py:462-468) */
                ray_raw(m, &m->coarse, o, d, sk, code, z + S, I, feat, raw + 4 * S, codes_rows, buf);
                for (int k = 0; k < T; ++k) order[k] = k;
                g_sort_keys = z;
                qsort(order, (size_t)T, sizeof(int), cmp_idx);
                for (int k = 0; k < T; ++k) {
                    zm[k] = z[order[k]];
                    memcpy(rawm + 4 * k, raw + 4 * order[k], 4 * sizeof(float));
                }
                memcpy(z, zm, sizeof(float) * T);
                float f_rgb[3], f_disp, f_acc;
                raw2outputs(m, rawm, z, T, d, f_rgb, &f_disp, &f_acc, w, al, buf);
                for (int c = 0; c < 3; ++c) rgb[3 * i + c] = f_rgb[c];
                disp[i] = f_disp;
                acc[i] = f_acc;
                if (alpha) memcpy(alpha + (size_t)i * T, al, sizeof(float) * T);
                if (z_out) memcpy(z_out + (size_t)i * T, z, sizeof(float) * T);
                continue;
            }
            sample_pdf(mids, w + 1, S - 1, I, uv, z + S, cdf);
            qsort(z, (size_t)T, sizeof(float), cmp_float);
            ray_code(m, &m->fine, cams, i, code);
            float f_rgb[3], f_disp, f_acc;
            ray_pass(m, &m->fine, o, d, sk, code, z, T, feat, raw, codes_rows, buf, f_rgb, &f_disp, &f_acc, w, al);
            for (int c = 0; c < 3; ++c) rgb[3 * i + c] = f_rgb[c];
            disp[i] = f_disp;
            acc[i] = f_acc;
            if (alpha) memcpy(alpha + (size_t)i * T, al, sizeof(float) * T);
            if (z_out) memcpy(z_out + (size_t)i * T, z, sizeof(float) * T);
        }
        free(feat); free(raw); free(buf); free(codes_rows); free(z); free(w); free(al); free(mids); free(cdf);
        free(zm); free(rawm); free(order);
    }
    free(near); free(far); free(tv); free(uv);
    return 0;
}

/* Stage entry: sample_pdf on explicit bins/weights for n rays (bins nb, weights nb-1 each). */
void oracle_sample_pdf(const float* bins, const float* wts, int64_t n, int nb, int n_samples, float* out) {
    float* u = (float*)malloc(sizeof(float) * n_samples);
    float* cdf = (float*)malloc(sizeof(float) * 2 * nb);
    oracle_linspace(n_samples, u);
    for (int64_t i = 0; i < n; ++i)
        sample_pdf(bins + i * nb, wts + i * (nb - 1), nb, n_samples, u, out + i * n_samples, cdf);
    free(u);
    free(cdf);
}

/* Stage entry: raw2outputs for n rays of ns samples. */
void oracle_raw2outputs(const oracle_model* m, const float* raw, const float* z, const float* dirs, int64_t n,
                        int ns, float* rgb, float* disp, float* acc, float* weights, float* alpha) {
    float* scratch = (float*)malloc(sizeof(float) * 4 * ns);
    for (int64_t i = 0; i < n; ++i)
        raw2outputs(m, raw + i * ns * 4, z + i * ns, ns, dirs + 3 * i, rgb + 3 * i, disp + i, acc + i,
                    weights + i * ns, alpha + i * ns, scratch);
    free(scratch);
}

/* Stage entry: get_rays (ray_utils.py:6-28) gathered at pixel indices, as render() packs them
 * (core/trainer.py:116-135): out [n][11] = o, d, near, far, d/|d|. */
void oracle_gen_rays(const float* c2w /*3x4*/, int H, int W, float fx, float fy, float cx, float cy,
                     const int64_t* idx, int64_t n, float nearv, float farv, float* out) {
    (void)H;
    for (int64_t t = 0; t < n; ++t) {
        const float x = (float)(idx[t] % W), y = (float)(idx[t] / W);
        const float d0 = (x - cx) / fx, d1 = -(y - cy) / fy, d2 = -1.0f;
        float* o = out + t * 11;
        for (int r = 0; r < 3; ++r) {
            o[r] = c2w[4 * r + 3];
            o[3 + r] = (d0 * c2w[4 * r + 0] + d1 * c2w[4 * r + 1]) + d2 * c2w[4 * r + 2];
        }
        o[6] = nearv;
        o[7] = farv;
        const float nn = norm3_(o[3], o[4], o[5]);
        o[8] = o[3] / nn;
        o[9] = o[4] / nn;
        o[10] = o[5] / nn;
    }
}

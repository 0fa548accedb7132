// anerf_render.hip — MI355X (gfx950) render path of A-NeRF behind the C ABI in include/anerf.h.
//
// One fused kernel renders a group of R rays per 256-thread workgroup (4 waves, one per SIMD):
//   coarse z (linspace) -> per-sample skeleton-relative encoding generated IN REGISTERS as the
//   MFMA B operand -> 8x256 MLP on v_mfma_f32_32x32x2_f32 with activations resident in the
//   accumulator/VGPR file across layers (the transposed product out^T = W^T in^T keeps each
//   layer's accumulator layout directly usable as the next layer's B operand; weights are
//   packed on the host in that permuted k order) -> alpha / rgb heads on the VALU ->
//   compositing + sample_pdf + merge-sort per ray in LDS -> fine pass over all S+I samples.
// The view layer is factorised: its per-sample direction input dv = T_k(e_jc) * w'_j is
// split into a per-ray matrix G[j][n] (computed once per ray in LDS) and the per-sample cutoff
// weights w'_j, so the per-sample K of the view layer is W + NJ + 1 instead of W + 27 NJ.
//
// Source layout (one translation unit, included in this order):
//   anerf_device.hpp   numerics helpers (torch/numpy-faithful sums, linspace, sincos, relu)
//   anerf_types.hpp    device model / launch structs, LDS plan, diagnostic stamps
//   anerf_mlp.hpp      MFMA building blocks: weight ring, dense layer, encoder streams, trunk
//   anerf_stages.hpp   per-ray stages: view factor G, compositing, importance sampling
//   anerf_kernels.hpp  __global__ kernels (render, density, near/far, rays, compose, encode)
//   anerf_pose.hpp     pose -> skeleton transforms (kinematic chain, inverse)
//   anerf_boxes.hpp    bounding cylinder + 2-D pixel box per frame (kp_to_valid_rays)
//   anerf_pack.hpp     host weight packing / model binding
//   this file          the C ABI (include/anerf.h)
//
// Reference behaviour restated (paths relative to danielajisafe/A-NeRF):
//   core/raycasters.py:361-474 render_rays, 476-555 encode_inputs, 557-577 run_network
//   core/encoders.py:8-37, 101-122, 172-193; core/cutoff_embedder.py:111-174
//   core/networks/nerf.py:90-205; core/utils/ray_utils.py:6-28, 157-251, 255-344
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/anerf.h"
#include "anerf_device.hpp"

using namespace anerf;

#include "anerf_types.hpp"
#include "anerf_mlp.hpp"
#include "anerf_stages.hpp"
#include "anerf_kernels.hpp"
#include "anerf_train.hpp"
#include "anerf_trainfwd.hpp"
#include "anerf_pose.hpp"
#include "anerf_boxes.hpp"
#include "anerf_batch.hpp"
#include "anerf_pack.hpp"

// Experiment switches are compile-time only (tools/build_ab.sh -D...): the shipped library reads no
// environment variable that could change its numerics or schedule.
#ifndef ANERF_UX6
#define ANERF_UX6 1  // split-precision bone-direction parts; 0: f32 MFMA (A/B builds only)
#endif

int anerf_internal_fail(int code, const char* msg) { return fail(code, msg); }  // for anerf_gemm.hip

#ifdef ANERF_STAMPS
static unsigned long long* g_stamps = nullptr;
extern "C" void anerf_diag_set_stamps(unsigned long long* p) { g_stamps = p; }  // diagnostic build only
#endif

// ---- the training MLP's fused forward (anerf_trainfwd.hpp)
namespace {
struct TfLayout {  // offsets (floats) of the packed parts, and the total
    size_t wx0, wl[MAXL], wskipx, wf, wvf, wvv, wvc, total;
};
size_t tf_regs_floats(int n_out, int n_in) { return (size_t)2 * (n_out / 32) * (n_in / 32) * 768; }
size_t tf_mem_floats(int n_out, int K) { return (size_t)tf_xsteps(K) * (n_out / 32) * 768; }
int tf_check(const anerf_mlp_shape* s) {
    if (!s) return fail(ANERF_EINVAL, "anerf_mlp_forward: NULL shape");
    if (s->width != 128 && s->width != 256)
        return fail(ANERF_EINVAL, "anerf_mlp_forward: width 128 or 256");
    if (s->depth < 1 || s->depth > MAXL) return fail(ANERF_EINVAL, "anerf_mlp_forward: depth 1..16");
    if (s->dnet < 1 || s->dnet % 4 || s->nv < 1 || s->nv % 4 || s->cfc < 0 || s->cfc % 4)
        return fail(ANERF_EINVAL, "anerf_mlp_forward: dnet, nv, cfc must be multiples of 4");
    return ANERF_OK;
}
TfLayout tf_layout(const anerf_mlp_shape* s) {
    const int W = s->width, D = s->depth;
    TfLayout L = {};
    size_t o = 0;
    L.wx0 = o; o += tf_mem_floats(W, s->dnet);
    for (int i = 1; i < D; ++i) { L.wl[i] = o; o += tf_regs_floats(W, W); }
    const bool has_skip = s->skip >= 0 && s->skip + 1 < D;
    L.wskipx = o; if (has_skip) o += tf_mem_floats(W, s->dnet);
    L.wf = o; o += tf_regs_floats(W, W);
    L.wvf = o; o += tf_regs_floats(W / 2, W);
    L.wvv = o; o += tf_mem_floats(W / 2, s->nv);
    L.wvc = o; if (s->cfc > 0) o += tf_mem_floats(W / 2, s->cfc);
    L.total = o;
    return L;
}
template <int W>
hipError_t tf_launch(const TfArgs& a, long long m, hipStream_t st) {
    constexpr int RB = W / 32;
    const size_t lds = sizeof(float) * ((size_t)(a.D + 1) * W + W / 2 + 2 * RB * 16 + 3 * 2 * (RB / 2) * 16 +
                                        (size_t)4 * 32 * (W + 4));
    // (per call: the attribute belongs to the current device, and a cached failure would stick)
    const hipError_t attr = hipFuncSetAttribute((const void*)train_mlp_fwd_kernel<W>,
                                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (attr != hipSuccess) return attr;
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const long long nblk = (m + 31) / 32;
    const long long want = (nblk + 3) / 4;
    const unsigned grid = (unsigned)(want < ncu ? want : ncu);
    hipLaunchKernelGGL(train_mlp_fwd_kernel<W>, dim3(grid), dim3(256), lds, st, a);
    return hipGetLastError();
}
}  // namespace

extern "C" {

int anerf_abi_version(void) { return ANERF_ABI_VERSION; }

const char* anerf_last_error(void) { return g_err.c_str(); }

int anerf_model_create(const anerf_model_desc* desc, const anerf_net_weights* coarse, const anerf_net_weights* fine,
                       const anerf_embed_params* embed, int device, anerf_model** out) {
    if (!out) return fail(ANERF_EINVAL, "out is NULL");
    *out = nullptr;
    int rc = validate_desc(desc);
    if (rc) return rc;
    if (!embed) return fail(ANERF_EINVAL, "embed params are NULL");
    const bool staged = desc_staged(desc);  // (the training stages only: no packed weights, anerf.h)
    if (!staged && !coarse) return fail(ANERF_EINVAL, "coarse weights are NULL");
    if (!staged && desc->has_fine && !fine) return fail(ANERF_EINVAL, "has_fine but fine weights are NULL");
    if (!embed->cutoff_dist || !embed->cutoff_dist_v) return fail(ANERF_EINVAL, "cutoff_dist is NULL");
    // --cutoff_bones windows the bone directions only through a CutoffEmbedder that weights its input
    // (use_cutoff, cutoff_inputs; multires_bones 0), as in core/cutoff_embedder.py:156-166; with bone
    // frequencies (staged) the CutoffEmbedder windows their sin / cos whatever cutoff_inputs says
    const bool bone_win = (desc->encoder_flags & ANERF_ENC_CUTOFF_BONES) && desc->use_cutoff;
    const bool bone_cut = bone_win && desc->cutoff_inputs;
    if ((bone_cut || (bone_win && desc->multires_bones > 0)) && !embed->cutoff_dist_b)
        return fail(ANERF_EINVAL, "ANERF_ENC_CUTOFF_BONES: embed->cutoff_dist_b (embedbones_fn.cutoff_dist) is NULL");
    const bool bone_tab = bone_cut || (bone_win && desc->multires_bones > 0);
    const int nj = desc->n_joints;
    const int njh2 = (((nj + 1) / 2) + 1) & ~1;  // joint pairs of the u part, even
    const int ngh = std::max(2 * njh2, nj + 2) / 2;  // G columns / 2: joint p + h*NJH2 at k-step p, bias at NJ
    Packer pk;
    std::vector<size_t> oc, of;
    if (!staged) {
        rc = pack_net(desc, njh2, coarse, pk, oc);
        if (rc) return rc;
        if (desc->has_fine) {
            rc = pack_net(desc, njh2, fine, pk, of);
            if (rc) return rc;
        }
    }
    // (querypts: the kp embedder's cutoff_dim is 3, its cutoff_dist 3 values; padded to NJ)
    const int nkc = (desc->encoder_flags & ANERF_ENC_KP_QUERYPTS) ? 3 : nj;
    std::vector<float> kc(embed->cutoff_dist, embed->cutoff_dist + nkc);
    kc.resize(nj, 0.0f);
    const size_t off_cut = pk.add(kc);
    const size_t off_cutv = pk.add(std::vector<float>(embed->cutoff_dist_v, embed->cutoff_dist_v + nj));
    const size_t off_cutb = pk.add(bone_tab ? std::vector<float>(embed->cutoff_dist_b, embed->cutoff_dist_b + nj)
                                            : std::vector<float>(nj, 0.0f));

    int prev = 0;
    HIP_TRY(hipGetDevice(&prev));
    HIP_TRY(hipSetDevice(device));
    float* dbuf = nullptr;
    const size_t bytes = pk.buf.size() * sizeof(float);
    hipError_t e = hipMalloc(&dbuf, bytes);
    if (e == hipSuccess) e = hipMemcpy(dbuf, pk.buf.data(), bytes, hipMemcpyHostToDevice);
    (void)hipSetDevice(prev);  // restoring the caller's device; the upload's own error is the one reported
    if (e != hipSuccess) {
        if (dbuf) (void)hipFree(dbuf);
        return fail(ANERF_EHIP, std::string("weight upload: ") + hipGetErrorString(e));
    }
    anerf_model* m = new anerf_model();
    m->desc = *desc;
    m->device = device;
    m->njh2 = njh2;
    m->ngh = ngh;
    m->dev_buf = dbuf;
    m->dev_bytes = bytes;
    ModelDev& md = m->md;
    std::memset(&md, 0, sizeof(md));
    md.nj = nj;
    md.njh2 = njh2;
    md.sparse = desc->use_cutoff && desc->cutoff_inputs;
    md.ngh = ngh;
    md.D = desc->net_depth;
    md.skip = desc->skip;
    md.mr = desc->multires;
    md.mrv = desc->multires_views;
    md.use_cutoff = desc->use_cutoff;
    md.cutoff_inputs = desc->cutoff_inputs;
    // (the view embedder is a CutoffEmbedder only under use_cutoff too: create_raycaster copies cutoff_kwargs, whose
    // "cutoff" is use_cutoff, core/raycasters.py:31, 68-71; cutoff_embedder.py:216-220)
    md.cutoff_viewdir = desc->cutoff_viewdir && desc->use_cutoff;
    md.cfc = desc->framecode_ch;
    md.n_codes = desc->n_framecodes;
    md.softplus = desc->density_softplus;
    md.ux6 = ANERF_UX6;  // split bone-direction parts (u_part_x6); 0 only in experiment builds (tools/build_ab.sh)
    md.single_net = desc->single_net ? 1 : 0;
    // (both transforms live in the CutoffEmbedder: without use_cutoff the kp embedder is plain)
    md.cut_to = desc->use_cutoff && (desc->encoder_flags & ANERF_ENC_CUT_TO_DIST) ? 1 : 0;
    md.shift_in = desc->use_cutoff && (desc->encoder_flags & ANERF_ENC_CUTOFF_SHIFT) ? 1 : 0;
    md.h3_top = 127 + h3_target();
    md.shift = desc->softplus_shift;
    md.B = desc->density_scale;
    md.bone_cut = bone_cut ? 1 : 0;
    md.view_raw = (desc->encoder_flags & ANERF_ENC_VIEW_RAW) ? 1 : 0;
    md.mrb = desc->multires_bones;
    md.kp_relpos = (desc->encoder_flags & ANERF_ENC_KP_RELPOS) ? 1 : 0;
    md.view_angle = (desc->encoder_flags & ANERF_ENC_VIEW_ANGLE) ? 1 : 0;
    md.kp_query = (desc->encoder_flags & ANERF_ENC_KP_QUERYPTS) ? 1 : 0;
    md.view_win = (desc->encoder_flags & ANERF_ENC_VIEW_WINDOWS) ? 1 : 0;
    md.bone_win = bone_win ? 1 : 0;
    md.staged = staged ? 1 : 0;
    md.tau = embed->tau;
    md.tau_v = embed->tau_v;
    md.tau_b = bone_tab ? embed->tau_b : 0.0f;
    md.cutoff = dbuf + off_cut;
    md.cutoff_v = dbuf + off_cutv;
    md.cutoff_b = dbuf + off_cutb;
    if (!staged) {
        bind_net(desc, dbuf, oc, coarse->alpha_b[0], md.net[0]);
        if (desc->has_fine) bind_net(desc, dbuf, of, fine->alpha_b[0], md.net[1]);
        else md.net[1] = md.net[0];
    }
    m->cut_host.assign(kc.begin(), kc.end());
    if (!staged) enc16_units(m);
    *out = m;
    return ANERF_OK;
}

int anerf_model_destroy(anerf_model* m) {
    if (!m) return ANERF_OK;
    const hipError_t e = m->dev_buf ? hipFree(m->dev_buf) : hipSuccess;
    delete m;
    if (e != hipSuccess) return fail(ANERF_EHIP, std::string("anerf_model_destroy: ") + hipGetErrorString(e));
    return ANERF_OK;
}

size_t anerf_model_bytes(const anerf_model* m) { return m ? m->dev_bytes : 0; }

int anerf_model_set_embed(anerf_model* m, const anerf_embed_params* embed) {
    if (!m || !embed) return fail(ANERF_EINVAL, "anerf_model_set_embed: NULL argument");
    const bool btab = m->md.bone_cut || (m->md.bone_win && m->md.mrb > 0);  // (the bone window is read)
    const bool cb = btab && embed->cutoff_dist_b;
    if (embed->cutoff_dist || embed->cutoff_dist_v || cb) {
        const size_t nb = sizeof(float) * (size_t)m->desc.n_joints;
        int prev = 0;
        HIP_TRY(hipGetDevice(&prev));
        HIP_TRY(hipSetDevice(m->device));
        hipError_t e = hipDeviceSynchronize();
        if (e == hipSuccess && embed->cutoff_dist)  // (querypts: 3 kp cutoffs, the rest of the table stays 0)
            e = hipMemcpy(const_cast<float*>(m->md.cutoff), embed->cutoff_dist,
                          m->md.kp_query ? 3 * sizeof(float) : nb, hipMemcpyHostToDevice);
        if (e == hipSuccess && embed->cutoff_dist_v)
            e = hipMemcpy(const_cast<float*>(m->md.cutoff_v), embed->cutoff_dist_v, nb, hipMemcpyHostToDevice);
        if (e == hipSuccess && cb)
            e = hipMemcpy(const_cast<float*>(m->md.cutoff_b), embed->cutoff_dist_b, nb, hipMemcpyHostToDevice);
        (void)hipSetDevice(prev);
        if (e != hipSuccess) return fail(ANERF_EHIP, std::string("anerf_model_set_embed: ") + hipGetErrorString(e));
    }
    m->md.tau = embed->tau;
    m->md.tau_v = embed->tau_v;
    if (btab) m->md.tau_b = embed->tau_b;
    if (embed->cutoff_dist && !m->md.kp_query) m->cut_host.assign(embed->cutoff_dist, embed->cutoff_dist + m->desc.n_joints);
    if (!m->md.staged) enc16_units(m);  // (the windowed features' bound moves with tau and the cutoffs)
    return ANERF_OK;
}

static size_t ws_near_far_bytes(int64_t n) {
    // near, far, fill scratch (floats) + qnan flags, each 256-byte aligned
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    return 3 * al(sizeof(float) * (size_t)n) + al((size_t)n);
}

// the coarse -> fine hand-off of the two-launch schedule (anerf_render_rays): n x T floats
static size_t ws_zf_bytes(int64_t n, int32_t n_samples, int32_t n_importance) {
    return n_importance > 0 ? (((size_t)n * (size_t)(n_samples + n_importance) * 4 + 255) & ~(size_t)255) : 0;
}

size_t anerf_workspace_size(const anerf_model* m, int64_t n_rays, int32_t n_samples, int32_t n_importance) {
    (void)m;
    const int64_t n = n_rays > 0 ? n_rays : 1;
    return ws_near_far_bytes(n) + ws_zf_bytes(n, n_samples, n_importance) + 256;  // (+ 2 x 8 queue counters)
}

static int launch_near_far(const float* rb, int stride, int64_t n, const float* cyls, const int32_t* ray_pose,
                           int n_poses, int chunk, char* ws, float** near_o, float** far_o, hipStream_t st) {
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    float* nearp = reinterpret_cast<float*>(ws);
    float* farp = reinterpret_cast<float*>(ws + al(sizeof(float) * n));
    float* scratch = reinterpret_cast<float*>(ws + 2 * al(sizeof(float) * n));
    uint8_t* qnan = reinterpret_cast<uint8_t*>(ws + 3 * al(sizeof(float) * n));
    const int bs = 256;
    hipLaunchKernelGGL(near_far_kernel, dim3((unsigned)((n + bs - 1) / bs)), dim3(bs), 0, st, rb, stride, n, cyls,
                       ray_pose, n_poses, nearp, farp, qnan);
    const int64_t nchunks = (n + chunk - 1) / chunk;
    hipLaunchKernelGGL(nan_fill_kernel, dim3((unsigned)nchunks), dim3(256), 0, st, rb, stride, n, chunk, nearp, farp,
                       qnan, scratch);
    HIP_TRY(hipGetLastError());
    *near_o = nearp;
    *far_o = farp;
    return ANERF_OK;
}

int anerf_near_far(const float* ray_batch, int32_t ray_stride, int64_t n_rays, const float* cyls, int32_t n_poses,
                   const int32_t* ray_pose, int32_t chunk, float* near_out, float* far_out, void* workspace,
                   size_t workspace_bytes, void* stream) {
    if (n_rays <= 0) return ANERF_OK;
    if (!ray_batch || !cyls || !near_out || !far_out || ray_stride < 8 || chunk <= 0 || n_poses < 1)
        return fail(ANERF_EINVAL, "anerf_near_far: bad arguments");
    if (!workspace || workspace_bytes < ws_near_far_bytes(n_rays)) return fail(ANERF_EWORKSPACE, "workspace too small");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    float *np_, *fp_;
    int rc = launch_near_far(ray_batch, ray_stride, n_rays, cyls, ray_pose, n_poses, chunk,
                             (char*)workspace, &np_, &fp_, st);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(near_out, np_, sizeof(float) * n_rays, hipMemcpyDeviceToDevice, st));
    HIP_TRY(hipMemcpyAsync(far_out, fp_, sizeof(float) * n_rays, hipMemcpyDeviceToDevice, st));
    return ANERF_OK;
}

// -DANERF_FUSED_PASSES=1 (experiment builds of tools/build_ab.sh only): both passes in one launch, the
// round-1 schedule kept for A/B measurements
#ifndef ANERF_FUSED_PASSES
#define ANERF_FUSED_PASSES 0
#endif
static constexpr bool fused_passes() { return ANERF_FUSED_PASSES != 0; }

int anerf_render_rays(const anerf_model* m, const float* ray_batch, int32_t ray_stride, int64_t n_rays,
                      const float* skts, const float* cyls, int32_t n_poses, const int32_t* ray_pose,
                      const float* cams, int32_t n_samples, int32_t n_importance, int32_t chunk, int32_t precision,
                      float* rgb, float* disp, float* acc, float* rgb0, float* disp0, float* acc0, float* alpha,
                      float* alpha0, const anerf_debug* debug, void* workspace, size_t workspace_bytes,
                      void* stream) {
    if (!m) return fail(ANERF_EINVAL, "model is NULL");
    if (m->md.staged) return fail(ANERF_EINVAL, "anerf_render_rays: staged encoder (multires_bones > 0, relpos or rayangle kp / view inputs): the training stages serve this model, anerf.h");
    if (n_rays < 0) return fail(ANERF_EINVAL, "n_rays < 0");
    if (n_rays == 0) return ANERF_OK;
    const int flags = precision & ~0xff;  // ANERF_FLAG_* bits above the precision mode
    precision &= 0xff;
    if (flags & ~(ANERF_FLAG_LINDISP | ANERF_FLAG_NEAR_FAR))
        return fail(ANERF_EINVAL, "unknown flags in the precision argument");
    if (precision < ANERF_PREC_FP32 || precision > ANERF_PREC_FP16X4) return fail(ANERF_EINVAL, "unsupported precision");
    if (!ray_batch || ray_stride < 8 || !skts || !cyls || n_poses < 1 || !rgb || !disp || !acc)
        return fail(ANERF_EINVAL, "anerf_render_rays: bad arguments");
    if (n_samples < 2 || n_samples > 1024 || n_importance < 0 || n_importance > 2048)
        return fail(ANERF_EINVAL, "n_samples must be in [2, 1024], n_importance in [0, 2048]");
    if (n_importance > 0 && !m->desc.has_fine && !m->desc.single_net)
        return fail(ANERF_EINVAL, "n_importance > 0 needs a fine network (or a single_net model)");
    if (n_importance > 0 && n_samples < 3) return fail(ANERF_EINVAL, "importance sampling needs n_samples >= 3");
    if (m->desc.framecode_ch > 0 && !cams) return fail(ANERF_EINVAL, "model uses framecodes: cams required");
    if (chunk <= 0) return fail(ANERF_EINVAL, "chunk must be > 0");
    if (!workspace || workspace_bytes < anerf_workspace_size(m, n_rays, n_samples, n_importance))
        return fail(ANERF_EWORKSPACE, "workspace too small");
    int dev = -1;
    HIP_TRY(hipGetDevice(&dev));
    if (dev != m->device) return fail(ANERF_EINVAL, "current device differs from the model's device");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);

    float *nearp, *farp;
    if (flags & ANERF_FLAG_NEAR_FAR) {  // near / far given in columns 6, 7: into the workspace as they are
        auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
        nearp = reinterpret_cast<float*>(workspace);
        farp = reinterpret_cast<float*>((char*)workspace + al(sizeof(float) * n_rays));
        hipLaunchKernelGGL(near_far_given_kernel, dim3((unsigned)((n_rays + 255) / 256)), dim3(256), 0, st, ray_batch,
                           ray_stride, n_rays, nearp, farp);
        HIP_TRY(hipGetLastError());
    } else {
        int rc = launch_near_far(ray_batch, ray_stride, n_rays, cyls, ray_pose, n_poses, chunk, (char*)workspace,
                                 &nearp, &farp, st);
        if (rc) return rc;
    }
    if (debug && debug->near) HIP_TRY(hipMemcpyAsync(debug->near, nearp, 4 * n_rays, hipMemcpyDeviceToDevice, st));
    if (debug && debug->far) HIP_TRY(hipMemcpyAsync(debug->far, farp, 4 * n_rays, hipMemcpyDeviceToDevice, st));

    const int S = n_samples, I = n_importance, T = S + I;
    // rays per workgroup: >= 8 coarse 32-sample blocks (2 per wave) and >= 4 rays, so the per-ray
    // stages (view factor, compositing: one wave per ray) use all 4 waves
    const int nbc = (S + 31) / 32;
    int R = std::max(4, 8 / nbc);
    R = std::min(R, 8);
    const int W = m->desc.net_width;
    const int nj = m->desc.n_joints, mrv = layout_multires_views(m->desc.multires_views), D = m->desc.net_depth;
    LdsPlan P = make_plan(R, nj, W, S, T, mrv, m->ngh, D, m->njh2, true, m->md.bone_cut != 0);
    if (P.total * 4 > 160 * 1024) P = make_plan(R, nj, W, S, T, mrv, m->ngh, D, m->njh2, false, m->md.bone_cut != 0);
    while (R > 1 && P.total * 4 > 160 * 1024) {
        R /= 2;
        P = make_plan(R, nj, W, S, T, mrv, m->ngh, D, m->njh2, false, m->md.bone_cut != 0);
    }
    if (P.total * 4 > 160 * 1024) return fail(ANERF_EINVAL, "configuration exceeds the 160 KiB LDS budget");

    RenderArgs a;
    std::memset(&a, 0, sizeof(a));
    a.rb = ray_batch;
    a.n = n_rays;
    a.stride = ray_stride;
    a.S = S;
    a.I = I;
    a.R = R;
    a.skts = skts;
    a.n_poses = n_poses;
    a.ray_pose = ray_pose;
    a.cams = cams;
    a.near = nearp;
    a.far = farp;
    a.rgb = rgb;
    a.disp = disp;
    a.acc = acc;
    a.rgb0 = rgb0;
    a.disp0 = disp0;
    a.acc0 = acc0;
    a.alpha = alpha;
    a.alpha0 = alpha0;
    a.lindisp = (flags & ANERF_FLAG_LINDISP) ? 1 : 0;
    if (debug) {
        a.dbg_z0 = debug->z_coarse;
        a.dbg_raw0 = debug->raw_coarse;
        a.dbg_w0 = debug->weights0;
        a.dbg_z1 = debug->z_fine;
        a.dbg_raw1 = debug->raw_fine;
        a.mfma_count = debug->mfma_count;
    }
#ifdef ANERF_STAMPS
    a.stamps = g_stamps;
#endif
    // With importance sampling the coarse and the fine pass run as two launches: every CU then
    // streams one network's weights at a time, which fit an XCD's 4 MB L2 (both together do not);
    // the fine z lists (T floats per ray) go through the workspace.
    // (single_net: one network, so one launch; the fine pass reuses the coarse raws, biases and G in LDS)
    const int pstep = (I > 0 && !fused_passes() && !m->desc.single_net) ? 1 : 2;
    a.zf_ws = I > 0 ? reinterpret_cast<float*>((char*)workspace + ws_near_far_bytes(n_rays)) : nullptr;
    unsigned grid = (unsigned)((n_rays + R - 1) / R);
    unsigned* queues = reinterpret_cast<unsigned*>((char*)workspace + ws_near_far_bytes(n_rays) +
                                                   ws_zf_bytes(n_rays, S, I));
    int ncu = 256;  // ANERF_PERSIST: as many workgroups as fit on the chip at once, items from the band queues
    if (ANERF_PERSIST) {
        int dev = 0;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
        HIP_TRY(hipMemsetAsync(queues, 0, 2 * 8 * sizeof(unsigned), st));
    }
    const size_t lds_bytes = (size_t)P.total * 4;
    const int mr = layout_multires(m->desc.multires);  // (the instance; smaller counts zero-padded, anerf_pack.hpp)
#define ANERF_LAUNCH(WW, MM)                                                                         \
    do {                                                                                            \
        auto kfn = precision == ANERF_PREC_BF16X3 ? render_kernel<WW, MM, 1>                       \
                 : precision == ANERF_PREC_BF16X6 ? render_kernel<WW, MM, 2>                       \
                 : precision == ANERF_PREC_FP16X3 ? render_kernel<WW, MM, 3>                       \
                 : precision == ANERF_PREC_FP16X4 ? render_kernel<WW, MM, 4> : render_kernel<WW, MM, 0>; \
        HIP_TRY(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize,  \
                                    (int)lds_bytes));                                               \
        unsigned g = grid;                                                                          \
        if (ANERF_PERSIST) {                                                                        \
            int nb = 1;                                                                             \
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kfn, 256, lds_bytes) != hipSuccess || nb < 1) \
                nb = 1;                                                                             \
            g = std::min<unsigned>(grid, (unsigned)(ncu * nb));                                     \
        }                                                                                           \
        for (int p0 = 0; p0 < 2; p0 += pstep) {                                                     \
            a.pass0 = p0;                                                                           \
            a.pass1 = p0 + pstep;                                                                   \
            a.queue = queues + 8 * p0;                                                              \
            hipLaunchKernelGGL(kfn, dim3(g), dim3(256), lds_bytes, st, m->md, a, P);               \
        }                                                                                           \
    } while (0)
    if (W == 256 && mr == 7) ANERF_LAUNCH(256, 7);
#ifndef ANERF_AB_FAST  // (tools/build_ab.sh: experiment builds with the config-3 instance only)
    else if (W == 128 && mr == 7) ANERF_LAUNCH(128, 7);
    else if (W == 64 && mr == 7) ANERF_LAUNCH(64, 7);
    else if (W == 256 && mr == 10) ANERF_LAUNCH(256, 10);
    else if (W == 128 && mr == 10) ANERF_LAUNCH(128, 10);
    else if (W == 64 && mr == 10) ANERF_LAUNCH(64, 10);
#endif
    else return fail(ANERF_EINVAL, "no kernel instance for this width / multires");
#undef ANERF_LAUNCH
    HIP_TRY(hipGetLastError());
    return ANERF_OK;
}

int anerf_gen_rays(const float* c2w, int32_t H, int32_t W, float focal_x, float focal_y, float center_x,
                   float center_y, int32_t has_center, const int64_t* idx, int64_t n, float nearv, float farv,
                   float* ray_batch_out, void* stream) {
    if (n == 0) return ANERF_OK;
    if (!c2w || !idx || !ray_batch_out || H <= 0 || W <= 0 || n < 0) return fail(ANERF_EINVAL, "anerf_gen_rays: bad arguments");
    const float cx = has_center ? center_x : (float)(W * 0.5);
    const float cy = has_center ? center_y : (float)(H * 0.5);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(gen_rays_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, c2w, H, W, focal_x,
                       focal_y, cx, cy, PixelSet{idx, 0, 0, 1}, n, nearv, farv, ray_batch_out);
    HIP_TRY(hipGetLastError());
    return ANERF_OK;
}

int anerf_gen_rays_box(const float* c2w, int32_t H, int32_t W, float focal_x, float focal_y, float center_x,
                       float center_y, int32_t has_center, int32_t x0, int32_t y0, int32_t x1, int32_t y1, float nearv,
                       float farv, float* ray_batch_out, void* stream) {
    if (!c2w || !ray_batch_out || H <= 0 || W <= 0 || x0 < 0 || y0 < 0 || x1 > W || y1 > H)
        return fail(ANERF_EINVAL, "anerf_gen_rays_box: bad arguments");
    if (x1 <= x0 || y1 <= y0) return ANERF_OK;
    const int64_t n = (int64_t)(x1 - x0) * (y1 - y0);
    const float cx = has_center ? center_x : (float)(W * 0.5);
    const float cy = has_center ? center_y : (float)(H * 0.5);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(gen_rays_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, c2w, H, W, focal_x,
                       focal_y, cx, cy, PixelSet{nullptr, x0, y0, x1 - x0}, n, nearv, farv, ray_batch_out);
    HIP_TRY(hipGetLastError());
    return ANERF_OK;
}

int anerf_compose(const float* rgb, const float* disp, const float* acc, const int64_t* idx, int64_t n,
                  const float* bg, int32_t white_bkgd, int64_t hw, float* out_rgb, float* out_disp, float* out_acc,
                  void* stream) {
    if (hw <= 0 || !out_rgb || !out_disp || n < 0 || (n > 0 && (!rgb || !disp || !acc || !idx)))
        return fail(ANERF_EINVAL, "anerf_compose: bad arguments");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(compose_fill_kernel, dim3((unsigned)((hw + 255) / 256)), dim3(256), 0, st, bg, white_bkgd, hw,
                       out_rgb, out_disp, out_acc);
    if (n > 0)
        hipLaunchKernelGGL(compose_scatter_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, rgb, disp, acc,
                           PixelSet{idx, 0, 0, 1}, 1, n, out_rgb, out_disp, out_acc);
    HIP_TRY(hipGetLastError());
    return ANERF_OK;
}

int anerf_compose_box(const float* rgb, const float* disp, const float* acc, int32_t x0, int32_t y0, int32_t x1,
                      int32_t y1, const float* bg, int32_t white_bkgd, int32_t H, int32_t W, float* out_rgb,
                      float* out_disp, float* out_acc, void* stream) {
    const bool empty = x1 <= x0 || y1 <= y0;
    if (H <= 0 || W <= 0 || !out_rgb || !out_disp || x0 < 0 || y0 < 0 || x1 > W || y1 > H ||
        (!empty && (!rgb || !disp || !acc)))
        return fail(ANERF_EINVAL, "anerf_compose_box: bad arguments");
    const int64_t hw = (int64_t)H * W;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(compose_fill_kernel, dim3((unsigned)((hw + 255) / 256)), dim3(256), 0, st, bg, white_bkgd, hw,
                       out_rgb, out_disp, out_acc);
    if (!empty) {
        const int64_t n = (int64_t)(x1 - x0) * (y1 - y0);
        hipLaunchKernelGGL(compose_scatter_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, rgb, disp, acc,
                           PixelSet{nullptr, x0, y0, x1 - x0}, W, n, out_rgb, out_disp, out_acc);
    }
    HIP_TRY(hipGetLastError());
    return ANERF_OK;
}

int anerf_encode_points(const anerf_model* m, const float* skts, const float* pts, const float* dirs, int64_t n_points,
                        float* feat_out, void* stream) {
    if (!m || !skts || !pts || !dirs || !feat_out || n_points < 0) return fail(ANERF_EINVAL, "anerf_encode_points: bad arguments");
    if (m->md.staged) return fail(ANERF_EINVAL, "anerf_encode_points: staged encoder (multires_bones > 0, relpos or rayangle kp / view inputs): the training stages serve this model, anerf.h");
    if (n_points == 0) return ANERF_OK;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(encode_points_kernel, dim3((unsigned)((n_points + 127) / 128)), dim3(128), 0, st, m->md, skts,
                       pts, dirs, n_points, feat_out);
    HIP_TRY(hipGetLastError());
    return ANERF_OK;
}

// ======================================================================= training stages
// (driven by a-nerf_amd/train.py, the MLP between them is torch autograd)
static inline unsigned blocks_of(int64_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

int anerf_train_samples(const float* near_in, const float* far_in, int64_t n_rays, int32_t n_samples,
                        const float* t_rand, int32_t flags, float* z_out, void* stream) {
    if (flags & ~ANERF_FLAG_LINDISP) return fail(ANERF_EINVAL, "anerf_train_samples: unknown flags");
    if (n_rays < 0 || n_samples < 2 || !near_in || !far_in || !z_out)
        return fail(ANERF_EINVAL, "anerf_train_samples: bad arguments");
    if (n_rays == 0) return ANERF_OK;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(train_z_kernel, dim3(blocks_of(n_rays * n_samples, 256)), dim3(256), 0, st, near_in, far_in,
                       n_rays, n_samples, t_rand, (flags & ANERF_FLAG_LINDISP) ? 1 : 0, z_out);
    HIP_TRY(hipGetLastError());
    return ANERF_OK;
}

static int check_train_rays(const anerf_model* m, const float* ray_batch, int32_t ray_stride, int64_t n_rays,
                            const float* z, int32_t n_samples, const float* skts, int32_t n_poses,
                            const int32_t* ray_pose) {
    if (!m || !ray_batch || ray_stride < 6 || n_rays < 0 || !z || n_samples < 1 || !skts)
        return fail(ANERF_EINVAL, "bad arguments");
    if (!ray_pose && n_poses != n_rays) return fail(ANERF_EINVAL, "per-ray skeletons need n_poses == n_rays");
    if (ray_pose && n_poses < 1) return fail(ANERF_EINVAL, "n_poses < 1");
    return ANERF_OK;
}

int anerf_train_encode(const anerf_model* m, const float* ray_batch, int32_t ray_stride, int64_t n_rays,
                       const float* z, int32_t n_samples, const float* skts, int32_t n_poses, const int32_t* ray_pose,
                       const float* pts_noise, float* feat_out, void* stream) {
    int rc = check_train_rays(m, ray_batch, ray_stride, n_rays, z, n_samples, skts, n_poses, ray_pose);
    if (rc) return rc;
    if (!feat_out) return fail(ANERF_EINVAL, "anerf_train_encode: feat_out is NULL");
    if (n_rays == 0) return ANERF_OK;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(train_encode_kernel, dim3(blocks_of(n_rays * n_samples * m->desc.n_joints, 256)), dim3(256), 0,
                       st, m->md,
                       ray_batch, ray_stride, n_rays, z, n_samples, skts, ray_pose, n_poses, pts_noise, feat_out);
    HIP_TRY(hipGetLastError());
    return ANERF_OK;
}

int anerf_train_encode_backward(const anerf_model* m, const float* ray_batch, int32_t ray_stride, int64_t n_rays,
                                const float* z, int32_t n_samples, const float* skts, int32_t n_poses,
                                const int32_t* ray_pose, const float* pts_noise, const float* grad_feat,
                                float* grad_skts, void* stream) {
    int rc = check_train_rays(m, ray_batch, ray_stride, n_rays, z, n_samples, skts, n_poses, ray_pose);
    if (rc) return rc;
    if (!grad_feat || !grad_skts) return fail(ANERF_EINVAL, "anerf_train_encode_backward: NULL gradient");
    if (n_rays == 0) return ANERF_OK;
    if (n_rays > 0x7fffffff) return fail(ANERF_EINVAL, "too many rays for one launch");
    const int nj = m->desc.n_joints;
    if (nj > 256) return fail(ANERF_EINVAL, "anerf_train_encode_backward: more than 256 joints");
    const int spb = 256 / nj;                      // sample slots per block
    const int threads = (spb * nj + 63) / 64 * 64;  // (whole waves)
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int mr = m->md.mr, mrv = m->md.mrv;
    auto launch = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3((unsigned)n_rays), dim3(threads), (size_t)spb * nj * 12 * sizeof(float), st,
                           m->md, ray_batch, ray_stride, n_rays, z, n_samples, skts, ray_pose, n_poses, pts_noise,
                           grad_feat, grad_skts, spb);
    };
    if (m->md.staged) launch(train_encode_backward_kernel<-1, -1>);  // (the staged encoders: run-time layout)
    else if (m->md.view_win && mr == 7) launch(train_encode_backward_kernel<7, -2>);  // (ANERF_ENC_VIEW_WINDOWS)
    else if (m->md.view_win && mr == 10) launch(train_encode_backward_kernel<10, -2>);
    else if (m->md.view_win && mr >= 0 && mr <= 10) launch(train_encode_backward_kernel<-1, -2>);
    else if (mr == 7 && mrv == 4) launch(train_encode_backward_kernel<7, 4>);
    else if (mr == 7 && mrv == 0) launch(train_encode_backward_kernel<7, 0>);
    else if (mr == 10 && mrv == 4) launch(train_encode_backward_kernel<10, 4>);
    else if (mr == 10 && mrv == 0) launch(train_encode_backward_kernel<10, 0>);
    else if (mr >= 0 && mr <= 10 && mrv >= 0 && mrv <= 4) launch(train_encode_backward_kernel<-1, -1>);  // (generic)
    else return fail(ANERF_EINVAL, "anerf_train_encode_backward: multires 0-10 and multires_views 0-4");
    HIP_TRY(hipGetLastError());
    return ANERF_OK;
}

int anerf_train_composite(const anerf_model* m, const float* raw, const float* z, const float* ray_batch,
                          int32_t ray_stride, int64_t n_rays, int32_t n_samples, const float* noise, float* rgb,
                          float* disp, float* acc, float* weights, float* alpha, float* trans, void* stream) {
    if (!m || !raw || !z || !ray_batch || ray_stride < 6 || n_rays < 0 || n_samples < 1 || !rgb || !disp || !acc ||
        !weights || !alpha || !trans)
        return fail(ANERF_EINVAL, "anerf_train_composite: bad arguments");
    if (n_rays == 0) return ANERF_OK;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (n_rays > 0x7fffffff || n_samples > 1024) return fail(ANERF_EINVAL, "anerf_train_composite: more than 1024 samples per ray");
    hipLaunchKernelGGL(train_composite_kernel, dim3((unsigned)n_rays), dim3(64), (size_t)7 * n_samples * sizeof(float),
                       st, m->md, raw, z, ray_batch, ray_stride, n_rays, n_samples, noise, rgb, disp, acc, weights,
                       alpha, trans);
    HIP_TRY(hipGetLastError());
    return ANERF_OK;
}

int anerf_train_composite_backward(const anerf_model* m, const float* raw, const float* z, const float* ray_batch,
                                   int32_t ray_stride, int64_t n_rays, int32_t n_samples, const float* noise,
                                   const float* weights, const float* alpha, const float* trans, const float* g_rgb,
                                   const float* g_disp, const float* g_acc, const float* g_weights,
                                   const float* g_alpha, float* g_raw, void* stream) {
    if (!m || !raw || !z || !ray_batch || ray_stride < 6 || n_rays < 0 || n_samples < 1 || !weights || !alpha ||
        !trans || !g_raw)
        return fail(ANERF_EINVAL, "anerf_train_composite_backward: bad arguments");
    if (n_rays == 0) return ANERF_OK;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (n_rays > 0x7fffffff || n_samples > 1024)
        return fail(ANERF_EINVAL, "anerf_train_composite_backward: more than 1024 samples per ray");
    hipLaunchKernelGGL(train_composite_backward_kernel, dim3((unsigned)n_rays), dim3(64),
                       (size_t)9 * n_samples * sizeof(float), st, m->md, raw, z, ray_batch, ray_stride, n_rays,
                       n_samples, noise, weights, alpha, trans, g_rgb, g_disp, g_acc, g_weights, g_alpha, g_raw);
    HIP_TRY(hipGetLastError());
    return ANERF_OK;
}

int anerf_train_importance(const float* z, const float* weights, int64_t n_rays, int32_t n_samples,
                           int32_t n_importance, const float* u, int32_t single_net, float* z_all,
                           int32_t* sorted_idx, void* stream) {
    if (!z || !weights || !z_all || n_rays < 0 || n_samples < 3 || n_importance < 1 || n_samples > 1024 ||
        n_importance > 2048)
        return fail(ANERF_EINVAL, "anerf_train_importance: bad arguments");
    if (n_rays == 0) return ANERF_OK;
    if (n_rays > 0x7fffffff) return fail(ANERF_EINVAL, "too many rays for one launch");
    const int T = n_samples + n_importance;
    const size_t lds = (size_t)(3 * pad32(T) + 3 * n_samples + 2 * T + 32) * 4;
    if (lds > 160 * 1024) return fail(ANERF_EINVAL, "n_samples + n_importance too large");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    HIP_TRY(hipFuncSetAttribute((const void*)train_importance_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds));
    hipLaunchKernelGGL(train_importance_kernel, dim3((unsigned)n_rays), dim3(64), lds, st, z, weights, n_rays,
                       n_samples, n_importance, u, single_net, z_all, sorted_idx);
    HIP_TRY(hipGetLastError());
    return ANERF_OK;
}

static int check_view_factor(const char* fn, const anerf_model* m, const float* ray_batch, int32_t ray_stride,
                             int64_t n_rays, const float* skts, int32_t n_poses, const int32_t* ray_pose,
                             const float* weight, int64_t ld_weight, int32_t width) {
    if (!m || !ray_batch || ray_stride < 6 || n_rays < 0 || !skts || !weight || width < 4 || width > 128 || (width & 3))
        return fail(ANERF_EINVAL, std::string(fn) + ": bad arguments (width 4-128, a multiple of 4)");
    if (m->md.view_angle) return fail(ANERF_EINVAL, std::string(fn) + ": ray-angle views have no per-ray factor");
    if (ld_weight < 3LL * m->desc.n_joints * (1 + 2 * m->desc.multires_views))
        return fail(ANERF_EINVAL, std::string(fn) + ": ld_weight shorter than the view columns");
    if (!ray_pose && n_poses != n_rays) return fail(ANERF_EINVAL, "per-ray skeletons need n_poses == n_rays");
    if (ray_pose && n_poses < 1) return fail(ANERF_EINVAL, "n_poses < 1");
    if ((n_rays + VF_RC - 1) / VF_RC > 0x7fffffff) return fail(ANERF_EINVAL, "too many rays for one launch");
    return ANERF_OK;
}

int anerf_train_view_factor(const anerf_model* m, const float* ray_batch, int32_t ray_stride, int64_t n_rays,
                            const float* skts, int32_t n_poses, const int32_t* ray_pose, const float* weight,
                            int64_t ld_weight, int32_t width, const float* col_scale, float* G, void* stream) {
    int rc = check_view_factor("anerf_train_view_factor", m, ray_batch, ray_stride, n_rays, skts, n_poses, ray_pose,
                               weight, ld_weight, width);
    if (rc) return rc;
    if (!G || (reinterpret_cast<uintptr_t>(G) & 15)) return fail(ANERF_EINVAL, "anerf_train_view_factor: G NULL or unaligned");
    if (n_rays == 0) return ANERF_OK;
    const int nk = 3 * (1 + 2 * m->md.mrv);
    hipLaunchKernelGGL(train_view_factor_kernel, dim3((unsigned)((n_rays + VF_RC - 1) / VF_RC), m->desc.n_joints),
                       dim3(256), (size_t)(nk * width + VF_RC * 28) * 4, reinterpret_cast<hipStream_t>(stream), m->md, ray_batch,
                       ray_stride, n_rays, skts, ray_pose, n_poses, weight, ld_weight, width, col_scale, G);
    HIP_TRY(hipGetLastError());
    return ANERF_OK;
}

size_t anerf_train_view_factor_workspace(int64_t n_rays, int32_t n_joints, int32_t multires_views, int32_t width) {
    if (n_rays <= 0 || n_joints < 1 || multires_views < 0 || multires_views > 4 || width < 1) return 0;
    return (size_t)((n_rays + VF_RAYS_B - 1) / VF_RAYS_B) * n_joints * 3 * (1 + 2 * multires_views) * width * 4;
}

int anerf_train_view_factor_backward(const anerf_model* m, const float* ray_batch, int32_t ray_stride, int64_t n_rays,
                                     const float* skts, int32_t n_poses, const int32_t* ray_pose, const float* weight,
                                     int64_t ld_weight, int32_t width, const float* col_scale, const float* grad_G,
                                     float* grad_skts, float* grad_weight, void* workspace, size_t workspace_bytes,
                                     void* stream) {
    int rc = check_view_factor("anerf_train_view_factor_backward", m, ray_batch, ray_stride, n_rays, skts, n_poses,
                               ray_pose, weight, ld_weight, width);
    if (rc) return rc;
    if (!grad_G || !grad_skts || !grad_weight || (reinterpret_cast<uintptr_t>(grad_G) & 15))
        return fail(ANERF_EINVAL, "anerf_train_view_factor_backward: NULL or unaligned gradient");
    if (n_rays == 0) return ANERF_OK;
    const size_t need = anerf_train_view_factor_workspace(n_rays, m->desc.n_joints, m->desc.multires_views, width);
    if (!workspace || workspace_bytes < need || (reinterpret_cast<uintptr_t>(workspace) & 15))
        return fail(ANERF_EINVAL, "anerf_train_view_factor_backward: workspace NULL, unaligned or smaller than "
                                  "anerf_train_view_factor_workspace()");
    const int nk = 3 * (1 + 2 * m->md.mrv), nj = m->desc.n_joints;
    const unsigned nb = (unsigned)((n_rays + VF_RAYS_B - 1) / VF_RAYS_B);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    float* part = static_cast<float*>(workspace);
    hipLaunchKernelGGL(train_view_factor_backward_kernel, dim3(nb, nj), dim3(256),
                       (size_t)(nk * width + VF_RC * (width + 4) + 2 * VF_RC * 28) * 4, st, m->md, ray_batch, ray_stride,
                       n_rays, skts, ray_pose, n_poses, weight, ld_weight, width, col_scale, grad_G, grad_skts, part);
    HIP_TRY(hipGetLastError());
    const int64_t per = (int64_t)nj * nk * width;
    hipLaunchKernelGGL(train_view_factor_reduce_kernel, dim3((unsigned)((per + 255) / 256)), dim3(256), 0, st, part,
                       (int)nb, nj, nk, width, col_scale, grad_weight, ld_weight);
    HIP_TRY(hipGetLastError());
    return ANERF_OK;
}

static int check_view_mix(const char* fn, int64_t n_rays, int32_t n_samples, int32_t n_joints, int32_t width,
                          const float* windows, int64_t ld, const float* G) {
    if (!windows || !G || n_rays < 0 || n_samples < 1 || n_joints < 1 || width < 4 || (width & 3) || width > 4096 ||
        ld < n_joints || (reinterpret_cast<uintptr_t>(G) & 15))
        return fail(ANERF_EINVAL, std::string(fn) + ": bad arguments (width % 4 == 0, ld >= n_joints, G 16-byte "
                                                     "aligned)");
    if (n_rays > 0x7fffffff) return fail(ANERF_EINVAL, "too many rays for one launch");
    return ANERF_OK;
}

int anerf_train_view_mix(int64_t n_rays, int32_t n_samples, int32_t n_joints, int32_t width, const float* windows,
                         int64_t ld_windows, const float* G, float* out, void* stream) {
    int rc = check_view_mix("anerf_train_view_mix", n_rays, n_samples, n_joints, width, windows, ld_windows, G);
    if (rc) return rc;
    if (!out || (reinterpret_cast<uintptr_t>(out) & 15)) return fail(ANERF_EINVAL, "anerf_train_view_mix: out NULL or unaligned");
    if (n_rays == 0) return ANERF_OK;
    if ((size_t)(n_joints * width + VM_SC * n_joints) * 4 > 64 * 1024)
        return fail(ANERF_EINVAL, "anerf_train_view_mix: n_joints too large for the LDS plan");
    hipLaunchKernelGGL(train_view_mix_kernel, dim3((unsigned)n_rays), dim3(256),
                       (size_t)(n_joints * width + VM_SC * n_joints) * 4, reinterpret_cast<hipStream_t>(stream),
                       windows, ld_windows, n_samples, n_joints, G, width, out);
    HIP_TRY(hipGetLastError());
    return ANERF_OK;
}

int anerf_train_view_mix_backward(int64_t n_rays, int32_t n_samples, int32_t n_joints, int32_t width,
                                  const float* windows, int64_t ld_windows, const float* G, const float* grad_out,
                                  float* grad_windows, int64_t ld_grad_windows, float* grad_G, void* stream) {
    int rc = check_view_mix("anerf_train_view_mix_backward", n_rays, n_samples, n_joints, width, windows, ld_windows, G);
    if (rc) return rc;
    if (!grad_out || !grad_windows || !grad_G || ld_grad_windows < n_joints || (reinterpret_cast<uintptr_t>(grad_out) & 15))
        return fail(ANERF_EINVAL, "anerf_train_view_mix_backward: bad gradient arguments");
    if (n_rays == 0) return ANERF_OK;
    const size_t lds = (size_t)(4 * ((n_joints + 3) / 4) * (width + 4) + VM_SC * (width + 4) + VM_SC * n_joints) * 4;
    if (lds > 64 * 1024 || (int64_t)n_joints * width > 1024LL * VM_K_LARGE)
        return fail(ANERF_EINVAL, "anerf_train_view_mix_backward: n_joints too large for the LDS / register plan");
    if ((int64_t)n_joints * width <= 1024LL * VM_K_SMALL)
        hipLaunchKernelGGL(train_view_mix_backward_kernel<VM_K_SMALL>, dim3((unsigned)n_rays), dim3(256), lds,
                           reinterpret_cast<hipStream_t>(stream), windows, ld_windows, n_samples, n_joints, G, width,
                           grad_out, grad_windows, ld_grad_windows, grad_G);
    else
        hipLaunchKernelGGL(train_view_mix_backward_kernel<VM_K_LARGE>, dim3((unsigned)n_rays), dim3(256), lds,
                           reinterpret_cast<hipStream_t>(stream), windows, ld_windows, n_samples, n_joints, G, width,
                           grad_out, grad_windows, ld_grad_windows, grad_G);
    HIP_TRY(hipGetLastError());
    return ANERF_OK;
}

static int launch_density(const anerf_model* m, DensityArgs a, int32_t precision, void* stream) {
    if (precision < ANERF_PREC_FP32 || precision > ANERF_PREC_FP16X4) return fail(ANERF_EINVAL, "unsupported precision");
    if (a.n == 0) return ANERF_OK;
    int dev = -1;
    HIP_TRY(hipGetDevice(&dev));
    if (dev != m->device) return fail(ANERF_EINVAL, "current device differs from the model's device");
    if (a.net < 0) a.net = m->desc.has_fine ? 1 : 0;  // the reference's default network (raycasters.py:616-620)
    if (a.net == 1 && m->desc.single_net) a.net = 0;  // network_fine is network_fn
    if (a.net > 1 || (a.net == 1 && !m->desc.has_fine)) return fail(ANERF_EINVAL, "no such network");
    const int W = m->desc.net_width, mr = layout_multires(m->desc.multires);
    const LdsPlan P = make_density_plan(m->desc.n_joints, W, m->desc.net_depth, m->njh2, m->md.bone_cut != 0);
    if (P.total * 4 > 160 * 1024) return fail(ANERF_EINVAL, "configuration exceeds the 160 KiB LDS budget");
    const int64_t nb = (a.n + 31) / 32;
    const unsigned grid = (unsigned)std::min<int64_t>((nb + 3) / 4, 256 * 32);
    const size_t lds_bytes = (size_t)P.total * 4;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define ANERF_LAUNCH(WW, MM)                                                                         \
    do {                                                                                            \
        auto kfn = precision == ANERF_PREC_BF16X3 ? density_kernel<WW, MM, 1>                      \
                 : precision == ANERF_PREC_BF16X6 ? density_kernel<WW, MM, 2>                      \
                 : precision == ANERF_PREC_FP16X3 ? density_kernel<WW, MM, 3>                      \
                 : precision == ANERF_PREC_FP16X4 ? density_kernel<WW, MM, 4> : density_kernel<WW, MM, 0>; \
        HIP_TRY(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize,  \
                                    (int)lds_bytes));                                               \
        hipLaunchKernelGGL(kfn, dim3(grid), dim3(256), lds_bytes, st, m->md, a, P);                \
    } while (0)
    if (W == 256 && mr == 7) ANERF_LAUNCH(256, 7);
#ifndef ANERF_AB_FAST
    else if (W == 128 && mr == 7) ANERF_LAUNCH(128, 7);
    else if (W == 64 && mr == 7) ANERF_LAUNCH(64, 7);
    else if (W == 256 && mr == 10) ANERF_LAUNCH(256, 10);
    else if (W == 128 && mr == 10) ANERF_LAUNCH(128, 10);
    else if (W == 64 && mr == 10) ANERF_LAUNCH(64, 10);
#endif
    else return fail(ANERF_EINVAL, "no kernel instance for this width / multires");
#undef ANERF_LAUNCH
    HIP_TRY(hipGetLastError());
    return ANERF_OK;
}

int anerf_density_points(const anerf_model* m, const float* pts, int64_t n_points, const float* skts, int32_t net,
                         int32_t precision, float* raw_out, void* stream) {
    if (!m || n_points < 0) return fail(ANERF_EINVAL, "anerf_density_points: bad arguments");
    if (m->md.staged) return fail(ANERF_EINVAL, "anerf_density_points: staged encoder (multires_bones > 0, relpos or rayangle kp / view inputs): the training stages serve this model, anerf.h");
    if (n_points == 0) return ANERF_OK;
    if (!pts || !skts || !raw_out) return fail(ANERF_EINVAL, "anerf_density_points: bad arguments");
    DensityArgs a;
    std::memset(&a, 0, sizeof(a));
    a.pts = pts;
    a.n = n_points;
    a.skts = skts;
    a.net = net;
    a.out = raw_out;
    return launch_density(m, a, precision, stream);
}

int anerf_density_grid(const anerf_model* m, const float* axis, int32_t res1, const float* kp0, const float* skts,
                       int32_t net, int32_t precision, float* raw_out, void* stream) {
    if (!m || !axis || !kp0 || !skts || !raw_out || res1 < 1) return fail(ANERF_EINVAL, "anerf_density_grid: bad arguments");
    if (m->md.staged) return fail(ANERF_EINVAL, "anerf_density_grid: staged encoder (multires_bones > 0, relpos or rayangle kp / view inputs): the training stages serve this model, anerf.h");
    DensityArgs a;
    std::memset(&a, 0, sizeof(a));
    a.t = axis;
    a.kp0 = kp0;
    a.res1 = res1;
    a.n = (int64_t)res1 * res1 * res1;
    a.skts = skts;
    a.net = net;
    a.out = raw_out;
    return launch_density(m, a, precision, stream);
}

// skeleton tables of KinArgs: parents must form a tree rooted at root_id (any index order)
static int kin_setup(KinArgs& a, int32_t rot_dim, const int32_t* parents, int32_t n_joints, int32_t root_id,
                     const char* who) {
    if (n_joints < 1 || n_joints > KIN_MAX_JOINTS || root_id < 0 || root_id >= n_joints || !parents)
        return fail(ANERF_EINVAL, std::string(who) + ": bad skeleton arguments");
    if (rot_dim != 3 && rot_dim != 6 && rot_dim != 9)
        return fail(ANERF_EINVAL, std::string(who) + ": rot_dim must be 3 (axis-angle), 6 (6-D) or 9 (matrix)");
    int depth[KIN_MAX_JOINTS];
    for (int j = 0; j < n_joints; ++j) {
        if (j != root_id && (parents[j] < 0 || parents[j] >= n_joints || parents[j] == j))
            return fail(ANERF_EINVAL, std::string(who) + ": parent index out of range");
        depth[j] = -1;
    }
    depth[root_id] = 0;
    int max_depth = 0;
    for (int j = 0; j < n_joints; ++j) {
        int k = j, steps = 0;
        while (depth[k] < 0 && steps <= n_joints) { k = parents[k]; ++steps; }
        if (depth[k] < 0) return fail(ANERF_EINVAL, std::string(who) + ": parents contain a cycle");
        int d = depth[k] + steps;  // assign depths along the path j -> k
        for (int u = j; depth[u] < 0; u = parents[u]) depth[u] = d--;
    }
    for (int j = 0; j < n_joints; ++j) {
        a.parent[j] = (int8_t)(j == root_id ? 0 : parents[j]);
        a.depth[j] = (uint8_t)depth[j];
        max_depth = std::max(max_depth, depth[j]);
    }
    a.rot_dim = rot_dim;
    a.nj = n_joints;
    a.root = root_id;
    a.max_depth = max_depth;
    return ANERF_OK;
}

int anerf_pose_kinematics(const float* bones, int32_t rot_dim, const float* rest, const int32_t* rest_idx,
                          int64_t n_rest, const float* pelvis, float scale, const int32_t* parents, int32_t n_joints,
                          int32_t root_id, int64_t n_frames, float* kps, float* skts, float* l2ws, float* rots,
                          void* stream) {
    if (n_frames < 0) return fail(ANERF_EINVAL, "anerf_pose_kinematics: n_frames < 0");
    KinArgs a{};
    int rc = kin_setup(a, rot_dim, parents, n_joints, root_id, "anerf_pose_kinematics");
    if (rc) return rc;
    if (n_frames == 0) return ANERF_OK;
    if (!bones || !rest || n_rest < 1 || (!kps && !skts && !l2ws && !rots))
        return fail(ANERF_EINVAL, "anerf_pose_kinematics: bad buffers");
    a.bones = bones; a.rest = rest; a.rest_idx = rest_idx; a.pelvis = pelvis;
    a.kps = kps; a.skts = skts; a.l2ws = l2ws; a.rots = rots;
    a.n_frames = n_frames; a.n_rest = n_rest; a.scale = scale;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const size_t lds = sizeof(double) * 12 * n_joints * KIN_WAVES;
    hipLaunchKernelGGL(pose_kinematics_kernel, dim3((unsigned)((n_frames + KIN_WAVES - 1) / KIN_WAVES)),
                       dim3(64 * KIN_WAVES), lds, st, a);
    HIP_TRY(hipGetLastError());
    return ANERF_OK;
}

int anerf_pose_kinematics_backward(const float* bones, int32_t rot_dim, const float* rest, const int32_t* rest_idx,
                                   int64_t n_rest, const float* pelvis, float scale, const int32_t* parents,
                                   int32_t n_joints, int32_t root_id, int64_t n_frames, const float* g_kps,
                                   const float* g_skts, const float* g_l2ws, const float* g_rots, float* g_bones,
                                   float* g_pelvis, void* stream) {
    if (n_frames < 0) return fail(ANERF_EINVAL, "anerf_pose_kinematics_backward: n_frames < 0");
    KinArgs a{};
    int rc = kin_setup(a, rot_dim, parents, n_joints, root_id, "anerf_pose_kinematics_backward");
    if (rc) return rc;
    if (n_frames == 0) return ANERF_OK;
    if (!bones || !rest || n_rest < 1 || !g_bones) return fail(ANERF_EINVAL, "anerf_pose_kinematics_backward: bad buffers");
    a.bones = bones; a.rest = rest; a.rest_idx = rest_idx; a.pelvis = pelvis;
    a.n_frames = n_frames; a.n_rest = n_rest; a.scale = scale;
    KinGradArgs g{g_kps, g_skts, g_l2ws, g_rots, g_bones, g_pelvis};
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const size_t lds = sizeof(double) * 36 * n_joints * KINB_WAVES;
    HIP_TRY(hipFuncSetAttribute((const void*)pose_kinematics_backward_kernel,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(pose_kinematics_backward_kernel, dim3((unsigned)((n_frames + KINB_WAVES - 1) / KINB_WAVES)),
                       dim3(64 * KINB_WAVES), lds, st, a, g);
    HIP_TRY(hipGetLastError());
    return ANERF_OK;
}

int anerf_kp_boxes(const float* kps, const float* cyls_in, int64_t n_kp, int32_t n_joints, int32_t root_id,
                   double ext_scale, const float* w2cs, const float* focals, const int32_t* offsets, int64_t n_frames,
                   int32_t H, int32_t W, const double* cap_dirs, float* cyls_out, int32_t* boxes_out, void* stream) {
    if (n_kp < 1 || n_frames < 0 || H <= 0 || W <= 0 || (!kps && !cyls_in))
        return fail(ANERF_EINVAL, "anerf_kp_boxes: bad arguments");
    if (kps && (n_joints < 1 || root_id < 0 || root_id >= n_joints))
        return fail(ANERF_EINVAL, "anerf_kp_boxes: bad skeleton arguments");
    if (n_frames > 0 && (!w2cs || !focals || !boxes_out)) return fail(ANERF_EINVAL, "anerf_kp_boxes: bad buffers");
    BoxArgs a{};
    a.kps = kps; a.cyls_in = cyls_in; a.w2cs = w2cs; a.focals = focals; a.offsets = offsets;
    a.cap_dirs = cap_dirs; a.cyls_out = cyls_out; a.boxes_out = boxes_out;
    a.n_kp = n_kp; a.n_frames = n_frames; a.nj = n_joints; a.root = root_id; a.H = H; a.W = W;
    // Python floats meeting float32 arrays: rounded to float32 first (numpy NEP 50)
    const double ext = 250.0 * ext_scale;
    a.ext = (float)ext;
    a.ext_top = (float)(ext * 1.6);
    a.ext_bot = (float)(ext * 1.1);
    const int64_t waves = std::max(n_frames, cyls_out ? n_kp : (int64_t)0);
    if (waves == 0) return ANERF_OK;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(kp_boxes_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, a);
    HIP_TRY(hipGetLastError());
    return ANERF_OK;
}

int anerf_ray_batch(const uint8_t* imgs, const uint8_t* masks, const uint8_t* bgs, const int64_t* bg_idx,
                    const float* c2ws, const float* focals, const float* centers, int64_t n_rows, int64_t n_bg,
                    int32_t H, int32_t W, const int64_t* rows, int64_t n_img, const int64_t* pixels, int64_t n_per,
                    int32_t mask_img, float* rays_out, float* target_out, float* fg_out, float* bg_out,
                    int32_t* bad_out, void* stream) {
    if (n_img < 0 || n_per < 0 || H <= 0 || W <= 0 || n_rows < 1)
        return fail(ANERF_EINVAL, "anerf_ray_batch: bad sizes");
    if (n_img == 0 || n_per == 0) return ANERF_OK;
    if (!imgs || !c2ws || !focals || !rows || !pixels || !rays_out || !target_out)
        return fail(ANERF_EINVAL, "anerf_ray_batch: missing buffer");
    if (bgs && (!bg_idx || n_bg < 1)) return fail(ANERF_EINVAL, "anerf_ray_batch: backgrounds need bg_idx and n_bg");
    if (mask_img && !(bgs && masks)) return fail(ANERF_EINVAL, "anerf_ray_batch: mask_img needs masks and backgrounds");
    if (bg_out && !bgs) return fail(ANERF_EINVAL, "anerf_ray_batch: bg_out without backgrounds");
    if (fg_out && !masks) return fail(ANERF_EINVAL, "anerf_ray_batch: fg_out without masks");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    RayBatchArgs a{};
    a.imgs = imgs; a.masks = masks; a.bgs = bgs; a.bg_idx = bg_idx; a.c2ws = c2ws; a.focals = focals;
    a.centers = centers; a.rows = rows; a.pix = pixels; a.n_rows = n_rows; a.n_bg = bgs ? n_bg : 1;
    a.n_img = n_img; a.n_per = n_per; a.H = H; a.W = W; a.mask_img = mask_img;
    a.rays = rays_out; a.target = target_out; a.fg = fg_out; a.bg = bg_out; a.bad = bad_out;
    const int64_t n = n_img * n_per;
    hipLaunchKernelGGL(ray_batch_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a);
    HIP_TRY(hipGetLastError());
    return ANERF_OK;
}


int anerf_gather_rows(const float* src, int64_t width, int64_t n_rows, const int64_t* rows, int64_t n_img,
                      int64_t n_per, float* dst, int32_t* bad_out, void* stream) {
    if (width < 0 || n_rows < 1 || n_img < 0 || n_per < 0) return fail(ANERF_EINVAL, "anerf_gather_rows: bad sizes");
    const int64_t n = n_img * n_per;
    if (n == 0 || width == 0) return ANERF_OK;
    if (!src || !rows || !dst) return fail(ANERF_EINVAL, "anerf_gather_rows: missing buffer");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const bool v4 = width % 4 == 0 && reinterpret_cast<uintptr_t>(src) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(dst) % 16 == 0;
    const int64_t items = n * (v4 ? width / 4 : width);
    const dim3 grid((unsigned)((items + 255) / 256));
    if (v4)
        hipLaunchKernelGGL(gather_rows_kernel<4>, grid, dim3(256), 0, st, src, width, n_rows, rows, n_per, n, dst, bad_out);
    else
        hipLaunchKernelGGL(gather_rows_kernel<1>, grid, dim3(256), 0, st, src, width, n_rows, rows, n_per, n, dst, bad_out);
    HIP_TRY(hipGetLastError());
    return ANERF_OK;
}

size_t anerf_mlp_forward_pack_bytes(const anerf_mlp_shape* s) {
    if (tf_check(s)) return 0;
    return tf_layout(s).total * sizeof(float);
}

int anerf_mlp_forward_pack(const anerf_mlp_shape* s, const anerf_mlp_fwd_weights* w, void* packed, void* stream) {
    int rc = tf_check(s);
    if (rc) return rc;
    if (!w || !packed) return fail(ANERF_EINVAL, "anerf_mlp_forward_pack: NULL argument");
    const int W = s->width, D = s->depth;
    const TfLayout L = tf_layout(s);
    float* out = static_cast<float*>(packed);
    TfPackBatch b = {};
    long long dw = 0;
    auto job = [&](const float* wp, int64_t ld, int n_out, int col_off, int n_in, int kind, size_t off) {
        TfPackJob& J = b.j[b.n++];
        J.w = wp;
        J.out = out + off;
        J.ld = (int)ld;
        J.n_out = n_out;
        J.col_off = col_off;
        J.n_in = n_in;
        J.kind = kind;
        J.ngroups = kind == 0 ? 2 * (n_out / 32) * (n_in / 32) : tf_xsteps(n_in) * (n_out / 32);
        J.dw0 = dw;
        dw += (long long)J.ngroups * 768;
    };
    for (int i = 0; i < D; ++i)
        if (!w->pts_w[i]) return fail(ANERF_EINVAL, "anerf_mlp_forward_pack: NULL pts_w");
    if (!w->feature_w || !w->views_w) return fail(ANERF_EINVAL, "anerf_mlp_forward_pack: NULL head weights");
    const bool has_skip = s->skip >= 0 && s->skip + 1 < D;
    job(w->pts_w[0], w->pts_ld[0], W, 0, s->dnet, 1, L.wx0);
    for (int i = 1; i < D; ++i) {
        const bool sk = has_skip && i == s->skip + 1;  // [x | h]: the h part from column dnet
        job(w->pts_w[i], w->pts_ld[i], W, sk ? s->dnet : 0, W, 0, L.wl[i]);
        if (sk) job(w->pts_w[i], w->pts_ld[i], W, 0, s->dnet, 1, L.wskipx);
    }
    job(w->feature_w, W, W, 0, W, 0, L.wf);
    job(w->views_w, w->views_ld, W / 2, 0, W, 0, L.wvf);
    job(w->views_w, w->views_ld, W / 2, W, s->nv, 1, L.wvv);
    if (s->cfc > 0) job(w->views_w, w->views_ld, W / 2, W + s->nv, s->cfc, 1, L.wvc);
    hipLaunchKernelGGL(tf_pack_kernel, dim3((unsigned)((dw + 255) / 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), b);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? ANERF_OK : fail(ANERF_EHIP, std::string("anerf_mlp_forward_pack: ") + hipGetErrorString(e));
}

int anerf_mlp_forward(const anerf_mlp_shape* s, const anerf_mlp_fwd_io* io, const void* packed, void* stream) {
    int rc = tf_check(s);
    if (rc) return rc;
    if (!io || !packed || !io->feat || !io->hf || !io->g || !io->raw || !io->feature_b || !io->alpha_w ||
        !io->alpha_b || !io->views_b || !io->rgb_w || !io->rgb_b)
        return fail(ANERF_EINVAL, "anerf_mlp_forward: NULL argument");
    if (io->m <= 0) return ANERF_OK;
    const int W = s->width, D = s->depth;
    if (io->ld_feat < s->dnet + s->nv || io->ld_feat % 4 || (reinterpret_cast<uintptr_t>(io->feat) & 15))
        return fail(ANERF_EINVAL, "anerf_mlp_forward: feat rows must be 16 B aligned with ld % 4 == 0");
    if (s->cfc > 0 && (!io->codes || io->ld_codes < s->cfc || io->ld_codes % 4 ||
                       (reinterpret_cast<uintptr_t>(io->codes) & 15)))
        return fail(ANERF_EINVAL, "anerf_mlp_forward: framecode rows must be 16 B aligned with ld % 4 == 0");
    if ((long long)32 * io->ld_feat * 4 >= (1ll << 31) || (s->cfc > 0 && (long long)32 * io->ld_codes * 4 >= (1ll << 31)))
        return fail(ANERF_EINVAL, "anerf_mlp_forward: row stride too large");
    const TfLayout L = tf_layout(s);
    const float* pk = static_cast<const float*>(packed);
    TfArgs a = {};
    a.D = D;
    a.skip = (s->skip >= 0 && s->skip + 1 < D) ? s->skip : -2;
    a.dnet = s->dnet;
    a.nv = s->nv;
    a.cfc = s->cfc;
    a.M = io->m;
    a.feat = io->feat;
    a.ldf = io->ld_feat;
    a.codes = io->codes;
    a.ldc = s->cfc > 0 ? io->ld_codes : 0;
    a.wx0 = pk + L.wx0;
    for (int i = 1; i < D; ++i) a.wl[i] = pk + L.wl[i];
    a.wskipx = pk + L.wskipx;
    a.wf = pk + L.wf;
    a.wvf = pk + L.wvf;
    a.wvv = pk + L.wvv;
    a.wvc = pk + L.wvc;
    for (int i = 0; i < D; ++i) {
        if (!io->pts_b[i] || !io->h[i]) return fail(ANERF_EINVAL, "anerf_mlp_forward: NULL pts_b / h");
        a.b[i] = io->pts_b[i];
        a.h[i] = io->h[i];
    }
    a.bf = io->feature_b;
    a.wa = io->alpha_w;
    a.ba = io->alpha_b;
    a.bv = io->views_b;
    a.wrgb = io->rgb_w;
    a.brgb = io->rgb_b;
    a.hf = io->hf;
    a.g = io->g;
    a.raw = io->raw;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const hipError_t e = W == 256 ? tf_launch<256>(a, io->m, st) : tf_launch<128>(a, io->m, st);
    return e == hipSuccess ? ANERF_OK : fail(ANERF_EHIP, std::string("anerf_mlp_forward: ") + hipGetErrorString(e));
}

}  // extern "C"

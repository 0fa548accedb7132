/*
 * anerf.h — C ABI of the MI355X-native A-NeRF render path (libanerf_hip.so).
 *
 * Plain pointers and sizes only: every float/int pointer passed to a render or stage entry is
 * a DEVICE pointer (HBM) on the model's device; model creation takes HOST pointers to the
 * reference's weights in their torch layout.  Every entry returns 0 on success or a negative
 * ANERF_E* code; anerf_last_error() returns a thread-local message.  Launch entries never
 * allocate, never synchronise and are safe to capture in a hipGraph; their scratch is the
 * caller's workspace (size from anerf_workspace_size).
 *
 * Reference interfaces replaced (paths relative to danielajisafe/A-NeRF):
 *   anerf_model_create      create_raycaster + RayCaster.load_state_dict      core/raycasters.py:17-184, 768-788
 *   anerf_render_rays       RayCaster.render_rays (eval, perturb=0, no noise)   core/raycasters.py:361-474
 *                           incl. get_near_far_in_cylinder + chunk NaN fill     core/utils/ray_utils.py:292-344
 *                           batchify_rays chunking (NaN-fill granularity)       core/trainer.py:64-79
 *   anerf_gen_rays          get_rays gathered at kp_to_valid_rays' pixel list  core/utils/ray_utils.py:6-28, 127-132
 *   anerf_encode_points     encode_inputs + embedders (stage / debug)          core/raycasters.py:476-555
 *   anerf_near_far          get_near_far_in_cylinder (stage)                   core/utils/ray_utils.py:292-344
 *   anerf_compose           render_path's image composition + NaN disp -> 0    run_nerf.py:100-141
 *   anerf_gen_rays_box,     the same over kp_to_valid_rays' box, the pixel     core/utils/ray_utils.py:127-132
 *   anerf_compose_box       list generated on the device (no index upload)
 *   anerf_density_points    RayCaster.render_pts_density (fwd_type='density')  core/raycasters.py:597-648
 *   anerf_density_grid      RayCaster.render_mesh_density (fwd_type='mesh')    core/raycasters.py:579-595
 *                           (called by run_render.render_mesh)                 run_render.py:970-986
 *   anerf_pose_kinematics   PoseOptLayer.calculate_kinematic, get_smpl_l2ws    core/pose_opt.py:372-521,
 *   anerf_pose_kinematics_backward   its autograd (pose optimisation)
 *                                                                              core/utils/skeleton_utils.py:296-376
 *   anerf_kp_boxes          kp_to_valid_rays' cylinder + pixel box             core/utils/ray_utils.py:83-136
 *   anerf_ray_batch         BaseH5Dataset.__getitem__ + ray_collate_fn (the    core/dataset.py:57-105, 259-275,
 *                           training ray sampler) over HBM-resident images     346-364, 796-802
 *   anerf_gather_rows       ray_collate_fn's per-ray pose rows                 core/dataset.py:96-104, 796-802
 * Training stages of render_rays (perturb, raw noise, stochastic importance sampling, gradients):
 *   anerf_train_samples     sample_from_lineseg (perturb > 0)                  core/utils/ray_utils.py:204-251
 *   anerf_train_encode      sample_pts + encode_inputs (+ embedders)           core/raycasters.py:476-555, 650-663
 *   anerf_train_encode_backward   autograd of the same to skts (pose opt.)     core/encoders.py:8-37, 101-193,
 *                                                                              core/cutoff_embedder.py:111-174
 *   anerf_train_composite   NeRF.raw2outputs with raw_noise_std                core/networks/nerf.py:150-205
 *   anerf_train_composite_backward   its autograd
 *   anerf_train_importance  isample_from_lineseg + sample_pdf(det=False) + sort core/utils/ray_utils.py:157-201, 255-289
 *   anerf_train_view_factor (+ _backward)   per-ray view factors of the view-window layout
 *   anerf_train_view_mix (+ _backward)   the view layer's view part in the view-window layout
 *                           (ANERF_ENC_VIEW_WINDOWS; views_linears.0 on the view columns, core/networks/nerf.py:141-148)
 * The training MLP's linears (NeRF.forward / autograd, core/networks/nerf.py:94-148; the reference runs
 * them as torch addmm over cat()-ed inputs, core/raycasters.py:557-577):
 *   anerf_mlp_split_weights a weight (or its transpose) as bf16 hi / lo planes, once per step
 *   anerf_mlp_split_weights_batch   the same for up to 32 weights in one launch
 *   anerf_mlp_gemm          forward (bias, relu) and input-gradient (relu' mask, accumulate) products
 *   anerf_mlp_wgrad         weight + bias gradients
 *   anerf_mlp_backward_hidden  both of a 256 x 256 hidden layer's backward products in one pass (round 6)
 *   anerf_mlp_backward_head    the same for feature_linear with alpha_linear's rank-1 term (round 6, ABI 18)
 *   anerf_mlp_forward_hidden   a 256 x 256 hidden layer's forward, persistent (round 6, ABI 19)
 *   anerf_mlp_forward_layer    the same for any 256-output layer: layer 0, the skip layer, the heads (ABI 19)
 *   anerf_mlp_gemm_persistent  the same kernel as a product of any width (the feature gradient, ABI 19)
 *   anerf_mlp_forward(_pack)  the whole forward in one kernel (opt-in alternative to the GEMMs)
 */
#ifndef ANERF_H
#define ANERF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ANERF_ABI_VERSION 19

enum {
    ANERF_OK = 0,
    ANERF_EINVAL = -1,      /* bad argument / unsupported configuration */
    ANERF_EHIP = -2,        /* HIP runtime error */
    ANERF_EWORKSPACE = -3,  /* workspace too small */
    ANERF_ENOMEM = -4
};

/* arithmetic used for the MLP contractions:
 *   ANERF_PREC_FP32   every contraction on v_mfma_f32_32x32x2_f32 (exact fp32 products);
 *   ANERF_PREC_BF16X3 the dense hidden layers split as x = x_hi + x_lo (bf16, round to nearest even)
 *                     and computed as x_hi w_hi + x_hi w_lo + x_lo w_hi on v_mfma_f32_32x32x16_bf16
 *                     with fp32 accumulation (~16-bit operands, products exact): outputs within
 *                     1e-5 of the fp32 path on the reference fixtures; encoder and view parts fp32;
 *   ANERF_PREC_BF16X6 the dense hidden layers and the fused view layer split three ways: activations
 *                     x = x0 + x1 + x2 exactly (truncation: 8 + 8 + 8 significant bits), weights
 *                     w = w0 + w1 + w2 (bf16 RNE of the running remainder), computed as the six products
 *                     with i + j <= 2 of x_i w_j on v_mfma_f32_32x32x16_bf16, fp32 accumulation: the
 *                     dropped terms are below 2^-23 of each product (fp32 rounds a product to 2^-24),
 *                     so the contraction is fp32-accurate; layer 0's and the skip layer's bone-direction
 *                     parts the same way, and their windowed (per-joint sin/cos) parts too at widths
 *                     128 / 256 (fp32 at width 64); encoder and heads fp32;
 *   ANERF_PREC_FP16X3 the dense hidden layers and the fused view layer in fp16 after exact power-of-two
 *                     scaling (weights per layer, activations per sample, both to a maximum in
 *                     [2^10, 2^11)): x = x0 + x1, w = w0 + w1 (22 significant bits each), computed as
 *                     x0 w0 + x0 w1 + x1 w0 on v_mfma_f32_32x32x16_f16 (exact products, fp32 accumulation,
 *                     the dropped x1 w1 ~2^-22 of |x w|): half of bf16x6's MFMAs, 22-bit instead of
 *                     24-bit operands;
 *                     bone-direction parts and (widths 128 / 256) the windowed parts of layer 0 and the
 *                     skip layer as in bf16x6 (fp32 at width 64); encoder and heads fp32;
 *   ANERF_PREC_FP16X4 fp16x3 plus the fourth product x1 w1: the contraction is then (x - r_x)(w - r_w)
 *                     with the split remainders |r_x| <= 2^-23 |x|, |r_w| <= 2^-23 |w|, within ~2^-22 of
 *                     |x w| per product — the bound of bf16x6's dropped terms (x1 w2 + x2 w1 + x2 w2 and
 *                     the weights' third remainder, ~2^-22.2), so fp32-accurate like bf16x6, with four
 *                     MFMAs per 16 k instead of six and two weight planes (4 B per weight) instead of
 *                     three; everything else as fp16x3. */
enum { ANERF_PREC_FP32 = 0, ANERF_PREC_BF16X3 = 1, ANERF_PREC_BF16X6 = 2, ANERF_PREC_FP16X3 = 3, ANERF_PREC_FP16X4 = 4 };
/* Flags OR-ed into anerf_render_rays' precision argument (and anerf_train_samples' flags):
 *   ANERF_FLAG_LINDISP  sample linearly in inverse depth, z = 1 / (1/near (1 - t) + 1/far t)
 *                       (render_rays(lindisp=True), core/utils/ray_utils.py:223-226)
 *   ANERF_FLAG_NEAR_FAR (anerf_render_rays only) ray_batch columns 6 and 7 already hold every ray's
 *                       near / far AFTER get_near_far_in_cylinder and its chunk NaN fill
 *                       (core/utils/ray_utils.py:292-344), e.g. anerf_near_far's outputs over the
 *                       whole chunks that contain the rays: the kernel uses them as they are (cyls
 *                       and chunk are then not read).  Lets a rank render any sub-range of a chunked
 *                       ray list with the single-GPU NaN fill (ray-balanced sharding). */
enum { ANERF_FLAG_LINDISP = 0x100, ANERF_FLAG_NEAR_FAR = 0x200 };

typedef struct anerf_model anerf_model;

/* Shape of the path: the subset of run_nerf.py flags that shapes the kernel. */
typedef struct {
    int32_t n_joints;        /* NJ (24 SMPL, 65 Mixamo-like) */
    int32_t net_depth;       /* netdepth D */
    int32_t net_width;       /* netwidth W: 64, 128 or 256 */
    int32_t skip;            /* skips=[skip]; layer skip+1 consumes [x, h]; >= D-1 means none */
    int32_t multires;        /* kp positional-encoding frequencies (7) */
    int32_t multires_views;  /* view-direction frequencies: 4 (default) or 0 (surreal_single.txt) */
    int32_t use_cutoff;      /* --use_cutoff */
    int32_t cutoff_inputs;   /* --cutoff_inputs */
    int32_t cutoff_viewdir;  /* --cutoff_viewdir (windows the view features only together with use_cutoff, as the
                                reference's create_raycaster builds the view embedder, core/raycasters.py:31, 68-71) */
    int32_t framecode_ch;    /* 0, or --framecode_size when --opt_framecode */
    int32_t n_framecodes;
    int32_t density_softplus;/* 0: relu, 1: softplus(x - softplus_shift) */
    float softplus_shift;
    float density_scale;     /* B in raw2outputs */
    int32_t has_fine;        /* a separate network_fine exists (N_importance > 0, !single_net) */
    int32_t single_net;      /* --single_net: network_fine IS network_fn (raycasters.py:101-104); the fine
                                pass evaluates only the I new samples and merges raws (:462-468), the
                                importance weights are 0.5 (max(w_l,w_k) + max(w_k,w_u)) + 0.01
                                (ray_utils.py:270-277); requires has_fine == 0 */
    int32_t encoder_flags;   /* ANERF_ENC_* (kp embedder options of the cutoff embedder; 0 = none) */
    int32_t multires_bones;  /* --multires_bones (ABI 15): bone-direction frequencies, 0-10 (0: the bare
                                directions, the default); > 0 is a staged encoder (below) */
} anerf_model_desc;

/* Staged encoders (ABI 15): --multires_bones > 0, ANERF_ENC_KP_RELPOS / _KP_QUERYPTS and ANERF_ENC_VIEW_ANGLE change the
 * MLP's input layout beyond what the fused render kernel streams (its layer-0 parts and the per-ray view
 * factor G assume one distance per joint, bare bone directions and per-ray view directions).  A model with
 * any of them ("staged") is served by the training stages -- anerf_train_samples / _encode (+ _backward) /
 * _composite (+ _backward) / _importance with the MLP on anerf_mlp_gemm -- which the Python RayCaster runs
 * deterministically (perturb 0, no noise) for eval renders; anerf_render_rays, anerf_density_points /
 * _grid and anerf_encode_points reject it (ANERF_EINVAL), and anerf_model_create takes no weights for it
 * (the anerf_net_weights pointers may be NULL).  The feature row of a sample is
 *   [kp part | bone part | view part], with
 *   kp part   reldist: NJ (1 + 2 multires) columns, column f NJ + j (f = 0 the input, 2k + 1 / 2k + 2 the sin /
 *             cos of frequency 2^k);  relpos: 3 NJ (1 + 2 multires), column 3 f NJ + 3 j + c;  querypts:
 *             3 (1 + 2 multires), column 3 f + c;
 *   bone part 3 NJ (1 + 2 multires_bones), column 3 f NJ + 3 j + c;
 *   view part relray / world: 3 NJ (1 + 2 multires_views), column 3 f NJ + 3 j + c;
 *             rayangle: NJ (1 + 2 multires_views), column f NJ + j. */

/* anerf_model_desc.encoder_flags: the kp (distance) CutoffEmbedder's input transforms
 * (core/cutoff_embedder.py:125-134, only with use_cutoff): CUT_TO_DIST (--cut_to_dist) feeds
 * c_j - dist to the encoding (the raw input and the frequencies); CUTOFF_SHIFT (--cutoff_shift)
 * feeds (input * (2 / c_j) - 1) to the frequencies only.  The cutoff window keeps the distance. */
#define ANERF_ENC_CUT_TO_DIST 1
#define ANERF_ENC_CUTOFF_SHIFT 2
/* --cutoff_bones (core/raycasters.py:52-64): the bone embedder is a CutoffEmbedder (dist_inputs, its
 * own tau and cutoff_dist: anerf_embed_params tau_b / cutoff_dist_b); with --multires_bones 0 its
 * output is the bone direction times w_b = 1 - sigmoid(tau_b (dist - c_b)) when use_cutoff and
 * cutoff_inputs (core/cutoff_embedder.py:111-166), the bare direction otherwise.  With --multires_bones 0
 * the flag is ignored (and tau_b / cutoff_dist_b unused) unless desc->use_cutoff and desc->cutoff_inputs are
 * both set; with --multires_bones > 0 (staged) it needs use_cutoff only: the sin / cos features are windowed
 * by w_b either way, the bare directions with cutoff_inputs. */
#define ANERF_ENC_CUTOFF_BONES 4
/* --view_type world (core/raycasters.py:279-280, ABI 14): the view input of joint j is R_j d itself
 * (IdentityExpandEncoder of transform_batch_rays, encoders.py:25-37, 71-79), not the normalised
 * R_j d / |R_j d| of the default relray (VecNormEncoder, encoders.py:172-193).  Rendering, and (round 5)
 * anerf_train_encode / _encode_backward (the identity's gradient in place of the normalisation's). */
#define ANERF_ENC_VIEW_RAW 8
/* --kp_dist_type relpos (core/encoders.py:124-142, raycasters.py:261-262; staged, ABI 15): the kp input of joint
 * j is its local point q_j (3 values) instead of |q_j|; the kp CutoffEmbedder then has dist_inputs (the window
 * of all three from the joint distance, no cut_to_dist / cutoff_shift transform, cutoff_embedder.py:115-121)
 * and the reference's window distance |p - kp_j| is not a function of the poses (raycasters.py:530-533): its
 * gradient to skts is 0, for every windowed embedder of such a model. */
#define ANERF_ENC_KP_RELPOS 16
/* --view_type rayangle (core/encoders.py:195-212, skeleton_utils.py:594-605; staged, ABI 15): the view input
 * of joint j is one angle, acos(clamp(q_j . R_j d / (|q_j| |R_j d|), -1 + 1e-6, 1 - 1e-6)) - pi / 2. */
#define ANERF_ENC_VIEW_ANGLE 32
/* --kp_dist_type querypts (core/raycasters.py:263-265, IdentityEncoder(1, 3); staged, ABI 15): the kp input is the
 * world point p itself (3 values, not per joint); the kp CutoffEmbedder then has cutoff_dim 3 (embed->cutoff_dist
 * holds 3 values, not NJ) and windows each coordinate by itself, w_c = 1 - sigmoid(tau (p_c - c_c))
 * (cutoff_embedder.py:122-144: dists = inputs; --cut_to_dist / --cutoff_shift apply to the encoded values).  No
 * gradient reaches skts through it.  Not with ANERF_ENC_CUTOFF_BONES (the reference's bone CutoffEmbedder then
 * gets cutoff_dim 3 for 3 NJ inputs and fails). */
#define ANERF_ENC_KP_QUERYPTS 64
/* Training layout of the view part (ABI 16; anerf_train_encode / _encode_backward only, the other entry points
 * ignore the flag): the view part of a feature row is the NJ view windows w_j = 1 - sigmoid(tau_v (dist_j - c_v,j))
 * (column cv + j, cv = the view part's first column) instead of the 3 NJ (1 + 2 multires_views) windowed
 * direction features.  Every one of those features is w_j times a function of the ray alone (R_j d), so the
 * view layer's product with them is sum_j w_j G_j(ray) with G_j = Wv_j T_j(R_j d) per ray: the caller forms
 * T, G and that sum (the view direction's gradient to skts included) and the encoder handles the windows
 * (their gradient in _encode_backward's g_feat column cv + j).  Needs cutoff_viewdir, use_cutoff and cutoff_inputs
 * (every direction feature windowed); not with ANERF_ENC_VIEW_ANGLE or a staged encoder. */
#define ANERF_ENC_VIEW_WINDOWS 128

/* HOST pointers to one NeRF's weights, torch nn.Linear layout [out][in] (core/networks/nerf.py:57-88). */
typedef struct {
    const float* pts_w[16];  /* pts_linears[i].weight, i < net_depth */
    const float* pts_b[16];
    const float* alpha_w;    /* alpha_linear  [1][W]   */
    const float* alpha_b;    /* [1] */
    const float* feature_w;  /* feature_linear [W][W] */
    const float* feature_b;
    const float* views_w;    /* views_linears.0 [W/2][W + 3NJ(1+2*multires_views) + framecode_ch] */
    const float* views_b;
    const float* rgb_w;      /* rgb_linear [3][W/2] */
    const float* rgb_b;
    const float* codes;      /* framecodes.codes.weight [n_framecodes][framecode_ch] or NULL */
} anerf_net_weights;

/* HOST pointers to the embedders' state (core/cutoff_embedder.py:91-95). */
typedef struct {
    const float* cutoff_dist;    /* embed_fn.cutoff_dist [NJ]     */
    float tau;                   /* embed_fn.tau                  */
    const float* cutoff_dist_v;  /* embeddirs_fn.cutoff_dist [NJ] */
    float tau_v;                 /* embeddirs_fn.tau              */
    const float* cutoff_dist_b;  /* embedbones_fn.cutoff_dist [NJ] (ANERF_ENC_CUTOFF_BONES), else NULL */
    float tau_b;                 /* embedbones_fn.tau             */
} anerf_embed_params;

/* Optional per-stage outputs of anerf_render_rays (any member may be NULL). */
typedef struct {
    float* near;      /* [N]   after the chunk NaN fill */
    float* far;       /* [N]   */
    float* z_coarse;  /* [N][S] */
    float* raw_coarse;/* [N][S][4] (rgb, sigma) */
    float* weights0;  /* [N][S] */
    float* z_fine;    /* [N][S+I] sorted merged samples */
    float* raw_fine;  /* [N][S+I][4] */
    unsigned long long* mfma_count; /* [2] += MFMA instructions issued, a kernel-side tally of the
                                       work (agrees with PMC SQ_INSTS_MFMA): [0] v_mfma_f32_32x32x2_f32,
                                       [1] the 16-bit MFMAs, v_mfma_f32_32x32x16_bf16 (bf16x3 / bf16x6
                                       modes, and the bf16x6 bone-direction parts of fp16x3) and
                                       v_mfma_f32_32x32x16_f16 (fp16x3), the same FLOPs and cycles each */
} anerf_debug;

int anerf_abi_version(void);
const char* anerf_last_error(void);

/* Pack (on the host) and upload one model to `device`. fine may be NULL when !has_fine. */
int anerf_model_create(const anerf_model_desc* desc, const anerf_net_weights* coarse,
                       const anerf_net_weights* fine, const anerf_embed_params* embed, int device,
                       anerf_model** out);
int anerf_model_destroy(anerf_model* m);
/* Replace the embedders' state of a model without repacking its weights: tau / tau_v / tau_b always,
 * cutoff_dist / cutoff_dist_v / cutoff_dist_b when not NULL (then synchronously, after the device has
 * drained).
 * Launches issued afterwards use the new values: the tau schedule of training
 * (RayCaster.update_embed_fns -> CutoffEmbedder.update_tau, core/raycasters.py:731-748,
 * core/cutoff_embedder.py:176-183).  Not thread-safe against concurrent launches on the model. */
int anerf_model_set_embed(anerf_model* m, const anerf_embed_params* embed);
/* bytes of packed device weights held by the model */
size_t anerf_model_bytes(const anerf_model* m);

/* Scratch bytes anerf_render_rays needs for n_rays rays. */
size_t anerf_workspace_size(const anerf_model* m, int64_t n_rays, int32_t n_samples, int32_t n_importance);

/*
 * Render n_rays rays (RayCaster.render_rays in eval mode).
 *   ray_batch  [n_rays][ray_stride] float: o(3), d(3), near, far (, viewdirs...) — ray_stride >= 8
 *   skts       [n_poses][NJ][4][4]  world->joint transforms
 *   cyls       [n_poses][5]         bounding cylinder (cx, cz, r, top, bot)
 *   ray_pose   [n_rays] int32 pose index per ray, or NULL (all rays use pose 0)
 *   cams       [n_rays] float framecode index per ray (float, truncated like .long()), or NULL;
 *              a negative index selects the eval-mode mean code (core/networks/embedding.py:23-24)
 *   chunk      NaN-fill granularity in rays (the caller's batchify chunk, 4096 in the configs)
 *   outputs: rgb [n][3], disp [n], acc [n]; rgb0/disp0/acc0 (coarse, only when n_importance>0),
 *            alpha [n][S+I or S], alpha0 [n][S] — any optional output may be NULL
 */
int anerf_render_rays(const anerf_model* m, const float* ray_batch, int32_t ray_stride, int64_t n_rays,
                      const float* skts, const float* cyls, int32_t n_poses, const int32_t* ray_pose,
                      const float* cams, int32_t n_samples, int32_t n_importance, int32_t chunk,
                      int32_t precision, float* rgb, float* disp, float* acc, float* rgb0, float* disp0,
                      float* acc0, float* alpha, float* alpha0, const anerf_debug* debug, void* workspace,
                      size_t workspace_bytes, void* stream);

/* Ray batch [n][11] (o, d, near, far, viewdir) for pixel indices idx (y*W + x) of one camera
 * (get_rays at ray_utils.py:6-28 + the gather at :132 + render's batch at core/trainer.py:116-135). */
int anerf_gen_rays(const float* c2w /*3x4 row-major, device*/, int32_t H, int32_t W, float focal_x,
                   float focal_y, float center_x, float center_y, int32_t has_center, const int64_t* idx,
                   int64_t n, float near, float far, float* ray_batch_out, void* stream);

/* Frame compose of render_path (run_nerf.py:100-141): pixels outside idx get the background
 * (bg [hw][3] if given, else 1 when white_bkgd, else 0), disp 0, acc 0; pixels idx[i] get
 * rgb + (1 - acc) * background, disp (NaN -> 0) and acc.  out_acc may be NULL. */
int anerf_compose(const float* rgb, const float* disp, const float* acc, const int64_t* idx, int64_t n,
                  const float* bg, int32_t white_bkgd, int64_t hw, float* out_rgb, float* out_disp, float* out_acc,
                  void* stream);

/* anerf_gen_rays over the pixels of kp_to_valid_rays' box, y in [y0, y1), x in [x0, x1), row-major
 * (the valid_idx order; ray_utils.py:127-130): n = (x1 - x0)(y1 - y0) rays, no index list. */
int anerf_gen_rays_box(const float* c2w, int32_t H, int32_t W, float focal_x, float focal_y, float center_x,
                       float center_y, int32_t has_center, int32_t x0, int32_t y0, int32_t x1, int32_t y1, float near,
                       float far, float* ray_batch_out, void* stream);

/* anerf_compose for rays produced by anerf_gen_rays_box (same box, same order). */
int anerf_compose_box(const float* rgb, const float* disp, const float* acc, int32_t x0, int32_t y0, int32_t x1,
                      int32_t y1, const float* bg, int32_t white_bkgd, int32_t H, int32_t W, float* out_rgb,
                      float* out_disp, float* out_acc, void* stream);

/* Stage: near/far of get_near_far_in_cylinder with the per-chunk NaN fill; cyls [n_poses][5], ray_pose
 * [n_rays] or NULL (pose 0); a ray whose pose index is outside [0, n_poses) is treated as a miss. */
int anerf_near_far(const float* ray_batch, int32_t ray_stride, int64_t n_rays, const float* cyls, int32_t n_poses,
                   const int32_t* ray_pose, int32_t chunk, float* near_out, float* far_out, void* workspace,
                   size_t workspace_bytes, void* stream);

/* Stage: MLP input features [M][F] of points pts [M][3] on rays with directions dirs [M][3],
 * joint transforms skts [NJ][4][4]; F = NJ(1+2 multires) + 3NJ + 3NJ(1+2 multires_views). */
int anerf_encode_points(const anerf_model* m, const float* skts, const float* pts, const float* dirs,
                        int64_t n_points, float* feat_out, void* stream);

/* Raw density (alpha_linear output, before the density activation) of the trunk of one network at
 * points pts [n][3] in world space, one pose skts [NJ][4][4]: _get_density_fwd_fn's fwd_fn.
 * net: 0 coarse, 1 fine, -1 the reference's default (fine if the model has one); precision ANERF_PREC_*. */
int anerf_density_points(const anerf_model* m, const float* pts, int64_t n_points, const float* skts, int32_t net,
                         int32_t precision, float* raw_out, void* stream);

/* The same on render_mesh_density's grid, generated on the device: raw_out [res1][res1][res1],
 * element (a, b, c) at (axis[b], axis[a], axis[c]) + kp0 (numpy 'xy' meshgrid order), where
 * axis [res1] = float32(linspace(-radius, radius, res1)) and kp0 [3] = kps[0, 0]. */
int anerf_density_grid(const anerf_model* m, const float* axis, int32_t res1, const float* kp0, const float* skts,
                       int32_t net, int32_t precision, float* raw_out, void* stream);

/* Pose -> skeleton transforms for n_frames frames, replacing
 *   PoseOptLayer.calculate_kinematic  core/pose_opt.py:372-445 (+ unrolled_kinematic_chain :482-521),
 *   get_kinematic_chain_T              core/pose_opt.py:448-479,
 *   get_smpl_l2ws + inv                core/utils/skeleton_utils.py:296-376.
 * bones [F][NJ][rot_dim]: rot_dim 3 axis-angle (pytorch3d axis_angle_to_matrix, skeleton_utils.py:411),
 * 6 the 6-D parameters (rot6d_to_rotmat, :420), 9 row-major 3x3 matrices; rest [n_rest][NJ][3],
 * rest_idx [F] (NULL: rest 0; out-of-range index -> NaN outputs for that frame); pelvis [F][3] or NULL,
 * added to every joint's translation; rest offsets are multiplied by scale.  parents [NJ] (HOST
 * memory, the skeleton's joint_trees; the root's entry is ignored) must form a tree rooted at root_id,
 * in any index order; NJ <= 128.  Outputs (any may be NULL): kps [F][NJ][3], skts = inverse(l2ws)
 * [F][NJ][4][4], l2ws [F][NJ][4][4], rots [F][NJ][3][3].  Computed in float64, stored as float32. */
int anerf_pose_kinematics(const float* bones, int32_t rot_dim, const float* rest, const int32_t* rest_idx,
                          int64_t n_rest, const float* pelvis, float scale, const int32_t* parents, int32_t n_joints,
                          int32_t root_id, int64_t n_frames, float* kps, float* skts, float* l2ws, float* rots,
                          void* stream);

/* Backward of anerf_pose_kinematics (the pose-optimisation gradient: PoseOptLayer's autograd,
 * core/pose_opt.py:372-445 + torch.inverse): with the same inputs and the gradients of its outputs
 * (g_kps [F][NJ][3], g_skts / g_l2ws [F][NJ][4][4], g_rots [F][NJ][3][3]; any may be NULL = zero),
 * writes g_bones [F][NJ][rot_dim] and, when not NULL, g_pelvis [F][3] (overwritten, not accumulated).
 * The chain is recomputed in float64. */
int anerf_pose_kinematics_backward(const float* bones, int32_t rot_dim, const float* rest, const int32_t* rest_idx,
                                   int64_t n_rest, const float* pelvis, float scale, const int32_t* parents,
                                   int32_t n_joints, int32_t root_id, int64_t n_frames, const float* g_kps,
                                   const float* g_skts, const float* g_l2ws, const float* g_rots, float* g_bones,
                                   float* g_pelvis, void* stream);

/* Bounding cylinder and 2-D pixel box of every frame on the device, the host
 * half of kp_to_valid_rays (core/utils/ray_utils.py:83-136): get_kp_bounding_cylinder
 * (skeleton_utils.py:542-592; extend_mm 250, top/bot expand 1.6/1.1, head '-y') of kps [n_kp][NJ][3]
 * (or the given cylinders cyls_in [n_kp][5] when kps is NULL), then cylinder_to_box_2d
 * (skeleton_utils.py:607-694) for frame i with cylinder i % n_kp, extrinsic w2cs [F][4][4] =
 * float32 inv(swap_mat(c2w)) (nerf_c2w_to_extrinsic, computed by the caller as the reference does),
 * focals [F][2] float32 (fx, fy), offsets [F][2] = int(center) or NULL (int(W/2), int(H/2)), cap_dirs [50][2] =
 * float64 (cos, sin) of linspace(0, 2 pi, 50) as numpy computes them (NULL: device cos/sin).
 * Outputs cyls_out [n_kp][5] float32 (optional) and boxes_out [F][4] int32 = (x0, y0, x1, y1):
 * pixels y in [y0, y1), x in [x0, x1) — the integers the reference computes. */
int anerf_kp_boxes(const float* kps, const float* cyls_in, int64_t n_kp, int32_t n_joints, int32_t root_id,
                   double ext_scale, const float* w2cs, const float* focals, const int32_t* offsets, int64_t n_frames,
                   int32_t H, int32_t W, const double* cap_dirs, float* cyls_out, int32_t* boxes_out, void* stream);

/* Training ray batch of the image dataset (the `.h5` ray sampler):
 * BaseH5Dataset.__getitem__ (core/dataset.py:57-105) for n_img images at once in ray_collate_fn's
 * flattened layout (core/dataset.py:796-802), from uint8 images resident on the device.  Inputs (the
 * .h5 arrays): imgs [n_rows][H*W][3], masks [n_rows][H*W] (NULL: fg = 1), bgs [n_bg][H*W][3] with
 * bg_idx [n_rows] (NULL: no backgrounds), c2ws [n_rows][4][4] float32, focals [n_rows] float32,
 * centers [n_rows][2] float32 (NULL: image centre); rows [n_img] = dataset row of each batch image,
 * pixels [n_img][n_per] = its sampled pixel indices y*W + x (drawn by the caller: the reference's
 * numpy RNG, sample_pixels core/dataset.py:277-323).  Outputs: rays_out [2][n][3] (rays_o, rays_d of
 * get_rays :346-364, including its isclose(c2w, I) shortcut), target_out [n][3] (get_img_data
 * :259-275; img * fg + (1 - fg) * bg when mask_img and bgs), fg_out [n] and bg_out [n][3] (optional),
 * n = n_img * n_per.  An out-of-range row, pixel or bg_idx makes that ray's outputs NaN and sets
 * *bad_out = 1 (device int32, may be NULL; the check guards the reads either way). */
int anerf_ray_batch(const uint8_t* imgs, const uint8_t* masks, const uint8_t* bgs, const int64_t* bg_idx,
                    const float* c2ws, const float* focals, const float* centers, int64_t n_rows, int64_t n_bg,
                    int32_t H, int32_t W, const int64_t* rows, int64_t n_img, const int64_t* pixels, int64_t n_per,
                    int32_t mask_img, float* rays_out, float* target_out, float* fg_out, float* bg_out,
                    int32_t* bad_out, void* stream);

/* Per-ray copies of per-image rows (ray_collate_fn's kp3d / bones / skts / cyls, core/dataset.py:
 * 96-104, 796-802: every ray of batch image i carries image i's pose rows): dst [n_img * n_per][width]
 * = src [rows[t / n_per]][width] float32, one launch per array (ABI 12; before, torch index_select).
 * A row outside [0, n_rows) gives NaN rows and sets *bad_out = 1 (device int32, may be NULL). */
int anerf_gather_rows(const float* src, int64_t width, int64_t n_rows, const int64_t* rows, int64_t n_img,
                      int64_t n_per, float* dst, int32_t* bad_out, void* stream);

/* ---- Training stages.  All pointers are device pointers; random numbers are
 * inputs (torch.rand / torch.randn draws of the caller), so a run can reproduce the reference's. */

/* z [N][S] of sample_from_lineseg: linspace(near, far) (torch.linspace's float32 values), then with
 * t_rand [N][S] (NULL: perturb = 0) lower + (upper - lower) t_rand inside the mid-point intervals. */
int anerf_train_samples(const float* near_in, const float* far_in, int64_t n_rays, int32_t n_samples,
                        const float* t_rand, int32_t flags /* ANERF_FLAG_LINDISP or 0 */, float* z_out,
                        void* stream);

/* Features feat_out [N][S][F] (the layout of anerf_encode_points) of the points o + d z of the rays
 * ray_batch [N][ray_stride] (o = cols 0-2, d = cols 3-5) at z [N][S]; the rays' skeletons are
 * skts [n_poses][NJ][4][4] with ray_pose [N] (NULL: one skeleton per ray, n_poses == N).  A ray
 * whose ray_pose is outside [0, n_poses) gets NaN features (and no gradient in the backward); the
 * index is never dereferenced.  pts_noise [N][S][3] (NULL: none) is added to the points, sample_pts'
 * `pts + randn_like(pts) * ray_noise_std` (core/raycasters.py:660-661): pass randn * ray_noise_std. */
int anerf_train_encode(const anerf_model* m, const float* ray_batch, int32_t ray_stride, int64_t n_rays,
                       const float* z, int32_t n_samples, const float* skts, int32_t n_poses, const int32_t* ray_pose,
                       const float* pts_noise, float* feat_out, void* stream);

/* dL/dskts of anerf_train_encode (same z and pts_noise) given dL/dfeat [N][S][F], ACCUMULATED into grad_skts
 * [n_poses][NJ][4][4] (row 3 of every transform untouched; the caller zeroes the buffer). */
int anerf_train_encode_backward(const anerf_model* m, const float* ray_batch, int32_t ray_stride, int64_t n_rays,
                                const float* z, int32_t n_samples, const float* skts, int32_t n_poses,
                                const int32_t* ray_pose, const float* pts_noise, const float* grad_feat,
                                float* grad_skts, void* stream);

/* raw2outputs of raw [N][S][4] at z [N][S] with noise [N][S] (= randn * raw_noise_std * B, added to
 * raw_sigma / B; NULL: none): rgb [N][3], disp [N], acc [N], weights, alpha and the exclusive
 * transmittance trans [N][S] (kept for the backward).  S <= 1024 (one wave per ray, LDS-staged). */
int anerf_train_composite(const anerf_model* m, const float* raw, const float* z, const float* ray_batch,
                          int32_t ray_stride, int64_t n_rays, int32_t n_samples, const float* noise, float* rgb,
                          float* disp, float* acc, float* weights, float* alpha, float* trans, void* stream);

/* g_raw [N][S][4] from the gradients of the outputs of anerf_train_composite (g_rgb [N][3], g_disp,
 * g_acc [N], g_weights, g_alpha [N][S]; any may be NULL = zero) and its saved weights/alpha/trans;
 * S <= 1024. */
int anerf_train_composite_backward(const anerf_model* m, const float* raw, const float* z, const float* ray_batch,
                                   int32_t ray_stride, int64_t n_rays, int32_t n_samples, const float* noise,
                                   const float* weights, const float* alpha, const float* trans, const float* g_rgb,
                                   const float* g_disp, const float* g_acc, const float* g_weights,
                                   const float* g_alpha, float* g_raw, void* stream);

/* z_all [N][S+I] (sorted) of isample_from_lineseg: sample_pdf over the mid-points with the coarse
 * weights [N][S] at u [N][I] (NULL: det=True, torch.linspace), merged with z [N][S].  single_net != 0
 * uses is_only's weights 0.5 (max(w_l, w_k) + max(w_k, w_u)) + 0.01 (ray_utils.py:270-277).
 * sorted_idx [N][S+I] (optional): torch.sort's indices into cat([z, z_samples]) (ties: values equal). */
int anerf_train_importance(const float* z, const float* weights, int64_t n_rays, int32_t n_samples,
                           int32_t n_importance, const float* u, int32_t single_net, float* z_all,
                           int32_t* sorted_idx, void* stream);

/* The view-window layout's per-ray view factors (ABI 16, ANERF_ENC_VIEW_WINDOWS): G [N][NJ][width] with
 * G[r][j][h] = sum_{f, c} T_fc(e_rj) weight[h ld_weight + f 3 NJ + 3 j + c] col_scale[f 3 NJ + 3 j + c], e_rj = R_j d_r
 * normalised (R_j d_r itself under ANERF_ENC_VIEW_RAW), T_0c = e_c, T_{2m+1,c} / T_{2m+2,c} = sin / cos (2^m e_c),
 * m < multires_views: joint j's view features without their window (encode_inputs' view part,
 * core/raycasters.py:476-555, core/encoders.py:172-193).  weight points at the view layer's first view column
 * (views_linears.0.weight + W, row stride ld_weight); col_scale (the --freq_schedule weights of the view columns) may
 * be NULL.  Skeletons as anerf_train_encode (ray_pose NULL: one per ray).  width <= 128; not for ray-angle views. */
int anerf_train_view_factor(const anerf_model* m, const float* ray_batch, int32_t ray_stride, int64_t n_rays,
                            const float* skts, int32_t n_poses, const int32_t* ray_pose, const float* weight,
                            int64_t ld_weight, int32_t width, const float* col_scale, float* G, void* stream);
/* Its gradients from grad_G: ADDED into grad_skts [n_poses][NJ][4][4] (the rotation blocks, atomically) and into
 * grad_weight (the view columns, the same layout as weight; no other writer on the stream meanwhile).  workspace:
 * device scratch of anerf_train_view_factor_workspace() bytes (16-byte aligned; the per-workgroup partial sums of the
 * weight gradient, reduced in order by a second launch). */
size_t anerf_train_view_factor_workspace(int64_t n_rays, int32_t n_joints, int32_t multires_views, int32_t width);
int anerf_train_view_factor_backward(const anerf_model* m, const float* ray_batch, int32_t ray_stride, int64_t n_rays,
                                     const float* skts, int32_t n_poses, const int32_t* ray_pose, const float* weight,
                                     int64_t ld_weight, int32_t width, const float* col_scale, const float* grad_G,
                                     float* grad_skts, float* grad_weight, void* workspace, size_t workspace_bytes,
                                     void* stream);

/* The view-window layout's view part (ABI 16, ANERF_ENC_VIEW_WINDOWS): out [N S][width] = sum_j w_j G_j, the NJ
 * windows w of sample s of ray r at windows + (r S + s) ld_windows (the window columns of an anerf_train_encode
 * row) and G [N][NJ][width] the ray's view factors (the view layer's view columns times the ray's direction
 * terms, per joint).  width % 4 == 0, G and out 16-byte aligned; G and a chunk of windows are staged in LDS:
 * 4 (NJ width + 32 NJ) bytes <= 64 KB here, 4 (4 ceil(NJ / 4) (width + 4) + 32 (width + 4) + 32 NJ) bytes in
 * the backward, which also keeps dL/dG in registers: NJ width <= 9216 (width 128: NJ <= 72; ANERF_EINVAL
 * beyond).  In the reference this is
 * part of views_linears.0's product with the view features (core/networks/nerf.py:141-148). */
int anerf_train_view_mix(int64_t n_rays, int32_t n_samples, int32_t n_joints, int32_t width, const float* windows,
                         int64_t ld_windows, const float* G, float* out, void* stream);
/* Its gradients from grad_out [N S][width]: grad_windows (r S + s) ld_grad_windows + j = sum_h grad_out G_j (written),
 * grad_G [N][NJ][width] = sum_s w_j grad_out (written). */
int anerf_train_view_mix_backward(int64_t n_rays, int32_t n_samples, int32_t n_joints, int32_t width,
                                  const float* windows, int64_t ld_windows, const float* G, const float* grad_out,
                                  float* grad_windows, int64_t ld_grad_windows, float* grad_G, void* stream);

/* ---- training MLP linears on the bf16 MFMA pipe, fp32 in / out with split-bf16 operands:
 *   ANERF_MLP_BF16X6  x = x0 + x1 + x2, w likewise, the six products with i + j <= 2 (fp32-accurate:
 *                     the dropped terms are below 2^-23 of |x w|), fp32 accumulation
 *   ANERF_MLP_BF16X3  x = x0 + x1, three products (~16 significant bits per operand)
 *   ANERF_MLP_FP16X4  forward products only (anerf_mlp_gemm_rows): each A row scaled by a power of two
 *                     from its largest |value| (row maxima given), the weights by one from theirs
 *                     (computed on the device by the split), x = x0 + x1 and w = w0 + w1 in fp16, all
 *                     four products on v_mfma_f32_32x32x16_f16: within ~2^-22 of |x w| per product, the
 *                     bound of ANERF_MLP_BF16X6 (the render path's fp16x4) */
enum { ANERF_MLP_BF16X3 = 3, ANERF_MLP_FP16X4 = 4, ANERF_MLP_BF16X6 = 6 };
/*
 * An operand is up to 3 column segments (the reference's torch.cat along features, never
 * materialised here): segment i holds columns [sum of earlier cols, + cols) at p[row * ld + c]. */
typedef struct {
    const float* p;
    int64_t ld;    /* row stride in floats (>= cols) */
    int32_t cols;
} anerf_seg;

/* An output column segment: out[row * ld + c] = v, v *= (mask[row * ldm + c] > 0) when mask is set
 * (relu backward by the saved activation), v += out[...] when accumulate == 1 (after the relu and mask);
 * accumulate == 2 (ABI 16) adds out[...] to the pre-activation instead (product + bias + out, then the relu: the
 * view-window layout's view part, anerf_train_view_mix); p NULL discards it. */
typedef struct {
    float* p;
    int64_t ld;
    int32_t cols;
    const float* mask;
    int64_t ldm;
    int32_t accumulate;
} anerf_oseg;

/* The training MLP's forward as ONE fused kernel (mlp.py with ANERF_TRAIN_FWD=fused, widths 128 /
 * 256, bf16x6 forward; measured equal to the layer GEMMs): NeRF.forward
 * (core/networks/nerf.py:94-148) over M rows of encoder features, every layer's output written once
 * for the backward.  feat [m][ld_feat]: x = columns [0, dnet),
 * views = [dnet, dnet + nv); codes [m][ld_codes] (cfc columns) or NULL.  Outputs: h[i] [m][W] =
 * relu(pts_linears[i](.)), hf [m][W] = feature_linear(h[D-1]), g [m][W/2] = relu(views_linears.0(
 * [hf | views | codes])), raw [m][4] = [rgb_linear(g), alpha_linear(h[D-1])].  Arithmetic as
 * ANERF_MLP_BF16X6.  The weights are packed once per step (anerf_mlp_forward_pack, one launch). */
typedef struct {
    int32_t depth, width;  /* width 128 or 256 */
    int32_t skip;          /* pts_linears[skip + 1] takes [x | h]; -1 (or >= depth - 1): none */
    int32_t dnet, nv, cfc; /* multiples of 4; cfc 0: no framecodes */
} anerf_mlp_shape;
typedef struct {
    const float* pts_w[16]; /* pts_linears[i].weight [W][in] */
    int64_t pts_ld[16];
    const float* feature_w; /* [W][W] */
    const float* views_w;   /* views_linears.0.weight [W/2][W + nv + cfc] */
    int64_t views_ld;
} anerf_mlp_fwd_weights;
typedef struct {
    int64_t m;
    const float* feat;
    int64_t ld_feat;
    const float* codes;
    int64_t ld_codes;
    const float* pts_b[16];
    const float* feature_b;
    const float* alpha_w; /* [W] */
    const float* alpha_b; /* [1] (device) */
    const float* views_b; /* [W/2] */
    const float* rgb_w;   /* [3][W/2] */
    const float* rgb_b;   /* [3] */
    float* h[16];
    float* hf;
    float* g;
    float* raw;
} anerf_mlp_fwd_io;
size_t anerf_mlp_forward_pack_bytes(const anerf_mlp_shape* s);
int anerf_mlp_forward_pack(const anerf_mlp_shape* s, const anerf_mlp_fwd_weights* w, void* packed, void* stream);
int anerf_mlp_forward(const anerf_mlp_shape* s, const anerf_mlp_fwd_io* io, const void* packed, void* stream);

/* Bytes of one split operand of `rows` x `cols` (anerf_mlp_split_weights' output). */
size_t anerf_mlp_split_bytes(int32_t rows, int32_t cols, int32_t precision);
/* w [n][k] (row stride ldw) -> bf16 planes (hi, then lo), zero padded; transpose != 0 splits w^T
 * ([k][n], the B operand of an input gradient).  out: anerf_mlp_split_bytes(rows, cols) bytes. */
int anerf_mlp_split_weights(const float* w, int32_t n, int32_t k, int64_t ldw, int32_t transpose,
                            int32_t precision, void* out, void* stream);
/* One anerf_mlp_split_weights call of a batch. */
typedef struct {
    const float* w;
    int32_t n, k;
    int64_t ldw;
    int32_t transpose, precision;
    void* out;
} anerf_split_job;
/* Up to 32 anerf_mlp_split_weights in one launch (a network's layers: forward or transposed). */
int anerf_mlp_split_weights_batch(const anerf_split_job* jobs, int32_t n_jobs, void* stream);
/* C[m][n] = act(sum_k A[m][k] B[n][k] + bias[n]); A: n_a segments adding up to k columns; B: split
 * [n][k] (the forward's weight, or the transposed weight of an input gradient); bias NULL or [n];
 * relu != 0 applies max(., 0); C: n_c segments adding up to n columns. */
int anerf_mlp_gemm(int64_t m, int32_t n, int32_t k, const anerf_seg* a, int32_t n_a, const void* b_split,
                   int32_t precision, const float* bias, int32_t relu, const anerf_oseg* c, int32_t n_c,
                   void* stream);
/* anerf_mlp_gemm with row maxima: rowmax_in [m] (ANERF_MLP_FP16X4 only, required there; one A segment):
 * the bit patterns of max_k |A[row][k]| (as written by rowmax_out); rowmax_out [m] (NULL or any
 * precision, n % 128 == 0, zeroed by the caller): atomically max'd with the bit patterns of
 * max_j |C[row][j]| after bias and relu (the next layer's rowmax_in).  The split weights of
 * ANERF_MLP_FP16X4 carry their exponent (anerf_mlp_split_bytes includes it). */
int anerf_mlp_gemm_rows(int64_t m, int32_t n, int32_t k, const anerf_seg* a, int32_t n_a, const void* b_split,
                        int32_t precision, const float* bias, int32_t relu, const anerf_oseg* c, int32_t n_c,
                        const int32_t* rowmax_in, int32_t* rowmax_out, void* stream);
/* Workspace bytes of anerf_mlp_wgrad for these sizes. */
size_t anerf_mlp_wgrad_workspace(int64_t m, int32_t n, int32_t k);
/* dW[n][k] (+)= sum_m dY[m][n] X[m][k] and db[n] (+)= sum_m dY[m][n] (db may be NULL); X: n_x
 * segments adding up to k columns.  Summed over row slabs in a fixed order (deterministic).  dY is
 * read in 4-column groups: 16 B aligned, lddy % 4 == 0, lddy >= round_up(n, 4) (columns n.. of the
 * last group are read but reach no output). */
int anerf_mlp_wgrad(int64_t m, int32_t n, int32_t k, const float* dy, int64_t lddy, const anerf_seg* x, int32_t n_x,
                    int32_t precision, float* dw, int64_t lddw, float* db, int32_t accumulate, void* workspace,
                    size_t workspace_bytes, void* stream);

/* Workspace bytes of anerf_mlp_backward_hidden (0 for an unsupported width). */
size_t anerf_mlp_backward_hidden_workspace(int64_t m, int32_t width);
/* The backward of one hidden layer y = relu(x W^T + b) of width 256 (pts_linears[i], i not after the skip,
 * core/networks/nerf.py:133-139; its autograd in the reference), from its pre-activation gradient dy [m][256]
 * and its input x [m][256] (the previous layer's relu output), in ONE pass over both:
 *   dx[m][i] = (sum_o dy[m][o] W[o][i]) if x[m][i] > 0 else 0    (the input gradient, relu' masked by x)
 *   dw[o][i] = sum_m dy[m][o] x[m][i],  db[o] = sum_m dy[m][o]    (written, not accumulated)
 * wt_split: W's transposed planes from anerf_mlp_split_weights(W, 256, 256, ld, transpose 1, precision).
 * precision: ANERF_MLP_BF16X3 (the "mixed" mode's backward arithmetic, as anerf_mlp_gemm / _wgrad).  The
 * same sums as anerf_mlp_gemm (input gradient with the relu' mask) + anerf_mlp_wgrad in another summation order;
 * deterministic (per-workgroup slabs summed in order).  dy, x: 16 B aligned, ld % 4 == 0, 256 <= ld < 2^22.
 * dw = db = NULL: the weight and bias gradients stay as slabs in the workspace for a later
 * anerf_mlp_backward_hidden_reduce (on another stream, beside the next layer's pass). */
int anerf_mlp_backward_hidden(int64_t m, int32_t width, const float* dy, int64_t lddy, const float* x, int64_t ldx,
                              const void* wt_split, int32_t precision, float* dx, int64_t lddx, float* dw, int64_t lddw,
                              float* db, void* workspace, size_t workspace_bytes, void* stream);
/* dw, db of an anerf_mlp_backward_hidden call made with dw = db = NULL, from its workspace (same m, width). */
int anerf_mlp_backward_hidden_reduce(int64_t m, int32_t width, const void* workspace, size_t workspace_bytes, float* dw,
                                     int64_t lddw, float* db, void* stream);

/* Workspace bytes of anerf_mlp_backward_head (0 for an unsupported width). */
size_t anerf_mlp_backward_head_workspace(int64_t m, int32_t width);
/* ABI 18: the backward of the heads on the last hidden layer's output x [m][256] -- feature_linear (256 x 256) and
 * alpha_linear (1 x 256), core/networks/nerf.py:141-145 (the reference runs them as two nn.Linear; here, as in the
 * forward, one [257][256] weight, feature rows then alpha's) -- in ONE pass over dy and x, as
 * anerf_mlp_backward_hidden:
 *   dx[m][i] = (sum_o dy[m][o] Wf[o][i] + dy[m][256] w_alpha[i]) if x[m][i] > 0 else 0
 *   dw[o][i] = sum_m dy[m][o] x[m][i] for o < 257 (row 256: alpha's), db[o] = sum_m dy[m][o] (257 entries)
 * dy rows hold the 256 feature gradients then alpha's at column 256 (lddy >= 257, % 4 == 0); wt_split: Wf's
 * transposed bf16x3 planes (anerf_mlp_split_weights(Wf, 256, 256, ld, 1, ANERF_MLP_BF16X3)); w_alpha [256] fp32.
 * Feature part in bf16x3 (as anerf_mlp_backward_hidden), alpha's terms in fp32.  dw [257][lddw], db [257], or
 * both NULL for a later anerf_mlp_backward_head_reduce. */
int anerf_mlp_backward_head(int64_t m, int32_t width, const float* dy, int64_t lddy, const float* x, int64_t ldx,
                            const void* wt_split, const float* w_alpha, int32_t precision, float* dx, int64_t lddx,
                            float* dw, int64_t lddw, float* db, void* workspace, size_t workspace_bytes, void* stream);
/* dw [257][lddw], db [257] of an anerf_mlp_backward_head call made with dw = db = NULL (same m, width). */
int anerf_mlp_backward_head_reduce(int64_t m, int32_t width, const void* workspace, size_t workspace_bytes, float* dw,
                                   int64_t lddw, float* db, void* stream);

/* ABI 19: the forward of one hidden layer of width 256 (pts_linears[i], core/networks/nerf.py:133-139),
 *   y[m][o] = relu(sum_i x[m][i] W[o][i] + b[o]),
 * bit-identical to anerf_mlp_gemm(m, 256, 256, {x}, w_split, precision, b, relu 1, {y}) -- the same split, the same
 * products in the same order -- on one persistent workgroup per CU whose stager waves stream x from HBM and the
 * output tile back while its compute waves run the MFMAs (anerf_gemm.hip, mlp_fwd_kernel).  w_split:
 * anerf_mlp_split_weights(W, 256, 256, ld, transpose 0, precision); precision ANERF_MLP_BF16X6 or _BF16X3.
 * x, y: 16 B aligned rows, ld % 4 == 0, 256 <= ld < 2^22; y must not overlap x. */
int anerf_mlp_forward_hidden(int64_t m, int32_t width, const float* x, int64_t ldx, const void* w_split,
                             int32_t precision, const float* bias, float* y, int64_t ldy, void* stream);
/* ABI 19: the same persistent kernel for any layer with 256 outputs on k > 128 input columns (k % 4 == 0) given as
 * one or two operand segments (layer 0 on the encoder features, the skip layer on [x | h]; each segment 16 B aligned,
 * cols % 4 == 0, cols <= ld < 2^22, ld % 4 == 0):  y[m][o] = act(sum_i a[m][i] W[o][i] + b[o]), act = relu if
 * relu != 0 -- bit-identical to anerf_mlp_gemm on the same segments.  With w_alpha [k], b_alpha [1] and alpha (all or
 * none) the kernel also writes alpha[m * ld_alpha] = sum_i a[m][i] w_alpha[i] + b_alpha in fp32 from the rows it
 * stages: feature_linear with alpha_linear beside it (core/networks/nerf.py:141-145; anerf_mlp_gemm computes the alpha
 * column as a 257th output in the layer's split arithmetic instead, so alpha agrees to fp32 rounding, not bit for
 * bit).  w_split: anerf_mlp_split_weights(W, 256, k, ld, 0, precision). */
int anerf_mlp_forward_layer(int64_t m, int32_t k, const anerf_seg* a, int32_t n_a, const void* w_split,
                            int32_t precision, const float* bias, int32_t relu, float* y, int64_t ldy,
                            const float* w_alpha, const float* b_alpha, float* alpha, int64_t ld_alpha, void* stream);
/* ABI 19: the persistent kernel as a plain product of any width, one launch per 256 output columns:
 *   c[m][o] = act(sum_i a[m][i] B[o][i] (+ bias[o])), o < n (n % 4 == 0; bias may be NULL),
 * bit-identical to anerf_mlp_gemm with one output segment {c, ldc, n} (no mask, no accumulation).  b_split:
 * anerf_mlp_split_weights(B, n, k, ld, transpose, precision) -- e.g. an input gradient dX = dY W with b_split the
 * transposed split of W, as the training backward's feature gradient [dY_0 | dY_skip] [W_0 ; W_skip,x] (k 512,
 * n = the encoder columns). */
int anerf_mlp_gemm_persistent(int64_t m, int32_t n, int32_t k, const anerf_seg* a, int32_t n_a, const void* b_split,
                              int32_t precision, const float* bias, int32_t relu, float* c, int64_t ldc, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* ANERF_H */

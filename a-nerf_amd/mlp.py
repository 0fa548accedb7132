"""The training MLP (NeRF.forward of core/networks/nerf.py:94-148 and its autograd) on the
hand-written split-bf16 GEMMs of anerf_gemm.hip (`anerf_mlp_*` in include/anerf.h).

One autograd Function runs the whole network: forward_density (pts_linears with the skip
layer's cat([x, h])), alpha_linear and feature_linear (one GEMM with N = W + 1, the alpha row
appended), views_linears[0] on cat([feature, views(, framecode)]) and rgb_linear — the
concatenations are operand segments, never built.  Bias and relu run in the GEMM epilogue; the
backward masks each input gradient by the saved relu output in the epilogue of the GEMM that
produces it (so every gradient that flows is already the pre-activation gradient the weight
gradient needs), writes the encoder-feature gradient in place (the skip layer's x part, then layer
0 accumulating into it; the view columns from the view layer) and sums weight and bias gradients
over the rows in one pass per layer.  Saved for the backward: the relu outputs of every layer.

Precision (`train.NeRF.mlp`): "bf16x6" splits both operands three ways into bf16 and sums the six
products with i + j <= 2 (fp32-accurate, as the render kernel's bf16x6 mode); "bf16x3" two ways,
three products (~16 significant bits per operand); "mixed" (the default) runs the forward in
bf16x6 and the backward in bf16x3; fp32 accumulation in all (`anerf_gemm.hip`).  There is no CPU path: the library must be
built and a GPU present.
"""
import ctypes

import torch

from . import _lib

# FUSED_FORWARD (an A/B switch for tools/fwd_bench.py and tests/test_gpu_mlp.py, never read from the
# environment): the whole bf16x6 forward (width 128 / 256) in one kernel (anerf_mlp_forward) instead of
# the layer-by-layer GEMMs.  Measured equal on MI355X (1.96 vs 1.95 ms at M = 163840): its
# 1.6 GB of saved activations cost as much as the GEMMs' re-reads, so the GEMMs stay the default
FUSED_FORWARD = False
ANERF_MLP_FP16X4 = _lib.MLP_PRECISIONS["fp16x4"]


def _stream(dev):
    return _lib.stream_handle(dev)


# The weight gradients of the backward run on a second stream, beside the input gradients on the
# caller's: a hidden layer's two products read the same dY and the same saved activation, so running
# them together lets the second read of each hit the caches (and the two kernels fill each other's
# tails).  The caller's stream waits for the side stream before the backward returns.
WGRAD_OVERLAP = True
_SIDE = {}

# (round 6) the backward of every 256 x 256 hidden layer (input not the skip layer's [x | h]) as ONE kernel,
# anerf_mlp_backward_hidden: dY and the saved activation are read once for the input gradient (relu' masked)
# and the weight + bias gradients, instead of the input-gradient GEMM on this stream and the weight-gradient
# GEMM on the side stream each reading both.  bf16x3 backward arithmetic only (the "mixed" default); an A/B
# switch for tools/train_bench.py, never read from the environment
FUSED_BACKWARD = True
# (round 6, with FUSED_BACKWARD) the skip layer's h part as one more fused pass and its x part merged into layer
# 0's two products (the backward's comment below); an A/B switch for tools/train_bench.py
FUSED_SKIP = True
# (round 6, ABI 18, with FUSED_BACKWARD) the heads' backward (feature_linear + alpha_linear's rank-1 term) as one
# fused pass, anerf_mlp_backward_head; an A/B switch for tools/train_bench.py
FUSED_HEAD = True
# (round 6) the caller's stream waits for the weight-gradient side stream at the end of the whole backward (an
# autograd engine callback) instead of at the end of the MLP's backward, when no parameter already holds a .grad to
# accumulate into: layer 0's weight gradient then overlaps the encoder's and the poses' backward; an A/B switch for
# tools/train_bench.py, never read from the environment
DEFER_WGRAD_SYNC = True
# (round 6, ABI 19) the forward of every trunk layer (layer 0 on the encoder features, the hidden layers, the skip
# layer on [x | h]) and of feature_linear on the persistent kernel anerf_mlp_forward_layer instead of anerf_mlp_gemm:
# bit-identical outputs (another schedule: stager waves stream the rows from HBM and the outputs back while the compute
# waves run the MFMAs), alpha_linear beside feature_linear in fp32 (the GEMM computed it as a 257th output in the split
# arithmetic: equal to fp32 rounding), and the backward's feature gradient [dY_0 | dY_s] [W_0 ; W_s,x] on the same
# kernel (anerf_mlp_gemm_persistent); bf16x6 / bf16x3 only; an A/B switch for tools/train_bench.py, never read from
# the environment
FORWARD_PERSISTENT = True


def _side_stream(dev):
    """The side stream of the caller's current stream (one per (device, stream): the training step runs the fine
    pass on a stream of its own, train.FINE_STREAM, and the two passes' weight gradients must not queue behind
    each other's)."""
    key = (torch.device(dev).index, torch.cuda.current_stream(dev).stream_id)
    if key not in _SIDE:
        _SIDE[key] = torch.cuda.Stream(device=dev)
    return _SIDE[key]


def _seg(t, cols, off=0):
    """anerf_seg over columns [off, off + cols) of a row-major 2-D tensor."""
    return (t.data_ptr() + 4 * off, t.stride(0), cols)


def _segs(lst):
    arr = (_lib.Seg * len(lst))()
    for i, (p, ld, c) in enumerate(lst):
        arr[i].p, arr[i].ld, arr[i].cols = p, ld, c
    return arr, len(lst)


def _osegs(lst):
    """[(tensor or None, ld, cols, col offset, mask tensor or None, accumulate)]"""
    arr = (_lib.OSeg * len(lst))()
    for i, (t, ld, cols, off, mask, acc) in enumerate(lst):
        arr[i].p = None if t is None else t.data_ptr() + 4 * off
        arr[i].ld, arr[i].cols = ld, cols
        arr[i].mask = None if mask is None else mask.data_ptr()
        arr[i].ldm = 0 if mask is None else mask.stride(0)
        arr[i].accumulate = int(acc)
    return arr, len(lst)


def split_weight(w, transpose=False, prec=6):
    """w [n, k] fp32 (contiguous rows) -> the bf16 planes of w (or w^T) as a uint8 buffer
    (prec: 6 = ANERF_MLP_BF16X6, three planes; 3 = ANERF_MLP_BF16X3, two)."""
    n, k = w.shape
    rows, cols = (k, n) if transpose else (n, k)
    lib = _lib.load()
    out = torch.empty(lib.anerf_mlp_split_bytes(rows, cols, prec), device=w.device, dtype=torch.uint8)
    _lib.check(lib.anerf_mlp_split_weights(_lib.ptr(w), n, k, w.stride(0), int(transpose), prec, _lib.ptr(out),
                                           _stream(w.device)), "anerf_mlp_split_weights")
    return out


def split_weights(jobs, prec):
    """[(w [n, k], transpose[, precision])] -> their split planes (as split_weight), in one launch per
    32 weights (anerf_mlp_split_weights_batch); a job's own precision overrides `prec`."""
    lib = _lib.load()
    outs = []
    for c0 in range(0, len(jobs), 32):
        chunk = jobs[c0:c0 + 32]
        arr = (_lib.SplitJob * len(chunk))()
        for i, job in enumerate(chunk):
            w, transpose = job[0], job[1]
            p = job[2] if len(job) > 2 else prec
            n, k = w.shape
            rows, cols = (k, n) if transpose else (n, k)
            out = torch.empty(lib.anerf_mlp_split_bytes(rows, cols, p), device=w.device, dtype=torch.uint8)
            arr[i].w, arr[i].n, arr[i].k, arr[i].ldw = w.data_ptr(), n, k, w.stride(0)
            arr[i].transpose, arr[i].precision, arr[i].out = int(transpose), p, out.data_ptr()
            outs.append(out)
        _lib.check(lib.anerf_mlp_split_weights_batch(arr, len(chunk), _stream(chunk[0][0].device)),
                   "anerf_mlp_split_weights_batch")
    return outs


def gemm(m, n, k, a, b_split, bias, relu, outs, dev, prec=6, rin=None, rout=None):
    """anerf_mlp_gemm_rows: rin / rout int32 [m] row maxima (fp16x4 input; any precision's output)."""
    sa, na = _segs(a)
    so, no = _osegs(outs)
    _lib.check(_lib.load().anerf_mlp_gemm_rows(m, n, k, sa, na, _lib.ptr(b_split), prec, _lib.ptr(bias), int(relu),
                                               so, no, _lib.ptr(rin), _lib.ptr(rout), _stream(dev)), "anerf_mlp_gemm")


def forward_layer(m, k, a, w_split, prec, bias, relu, y, dev, alpha=None):
    """y [m, 256] = act(a W^T + b) on the persistent kernel (anerf_mlp_forward_layer): a = 1 or 2 operand segments
    adding up to k > 128 columns; alpha = (w_alpha [k], b_alpha [1], out tensor column view [m]) or None."""
    sa, na = _segs(a)
    wa, ba, out = alpha if alpha is not None else (None, None, None)
    _lib.check(_lib.load().anerf_mlp_forward_layer(m, k, sa, na, _lib.ptr(w_split), prec, _lib.ptr(bias), int(relu),
                                                   _lib.ptr(y), y.stride(0), _lib.ptr(wa), _lib.ptr(ba),
                                                   None if out is None else ctypes.c_void_p(out.data_ptr()),
                                                   0 if out is None else out.stride(0), _stream(dev)),
               "anerf_mlp_forward_layer")


def gemm_persistent(m, n, k, a, b_split, prec, bias, relu, c, dev):
    """c[:, :n] = act(a B^T (+ b)) on the persistent kernel (anerf_mlp_gemm_persistent): one output segment, no mask,
    no accumulation; a = 1 or 2 operand segments adding up to k > 128 columns."""
    sa, na = _segs(a)
    _lib.check(_lib.load().anerf_mlp_gemm_persistent(m, n, k, sa, na, _lib.ptr(b_split), prec, _lib.ptr(bias),
                                                     int(relu), _lib.ptr(c), c.stride(0), _stream(dev)),
               "anerf_mlp_gemm_persistent")


def forward_hidden(m, x, w_split, prec, bias, y, dev):
    """y = relu(x W^T + b) of a 256 x 256 hidden layer (anerf_mlp_forward_hidden); w_split from split_weight(W)."""
    _lib.check(_lib.load().anerf_mlp_forward_hidden(m, 256, _lib.ptr(x), x.stride(0), _lib.ptr(w_split), prec,
                                                    _lib.ptr(bias), _lib.ptr(y), y.stride(0), _stream(dev)),
               "anerf_mlp_forward_hidden")


def wgrad(m, n, k, dy, x, dw, db, ws, dev, prec=6):
    sx, nx = _segs(x)
    _lib.check(_lib.load().anerf_mlp_wgrad(m, n, k, _lib.ptr(dy), dy.stride(0), sx, nx, prec, _lib.ptr(dw),
                                           dw.stride(0), _lib.ptr(db), 0, _lib.ptr(ws), ws.numel(), _stream(dev)),
               "anerf_mlp_wgrad")


def _view_mix(feat, dnet, nwin, G):
    """sum_j w_j(sample) G_j(ray) [M, W/2]: the view part of the view layer's pre-activation in the view-window
    layout (anerf.h ANERF_ENC_VIEW_WINDOWS; feat columns dnet.. are the NJ windows, G [rays, NJ, W/2] contiguous),
    anerf_train_view_mix."""
    n, _, wh = G.shape
    M = feat.shape[0]
    out = torch.empty(M, wh, device=feat.device, dtype=torch.float32)
    _lib.check(_lib.load().anerf_train_view_mix(n, M // n, nwin, wh, feat.data_ptr() + 4 * dnet, feat.stride(0),
                                                _lib.ptr(G), _lib.ptr(out), _stream(feat.device)),
               "anerf_train_view_mix")
    return out


class _MLP(torch.autograd.Function):
    """raw [M, 4] = NeRF(feat [M, F] (, codes [M, C])); params = the module's tensors in the order of
    `NeRF.mlp_params()`.  G [rays, NJ, W/2] (view-window layout, shape's nwin = NJ): the view layer's view
    part is sum_j w_j G_j (_view_mix) instead of a product with view columns (nv = 0 then)."""

    @staticmethod
    def forward(ctx, shape, feat, codes, G, *params):
        W, D, skip, dnet, nv, prec, _, nwin = shape
        dev = feat.device
        M, F = feat.shape
        nl = D

        def mm(*a):
            gemm(*a, prec=prec)
        pw, pb = params[0:2 * nl:2], params[1:2 * nl:2]
        wa, ba, wf, bf, wv, bv, wr, br = params[2 * nl:2 * nl + 8]
        whead = torch.cat([wf, wa]).contiguous()
        cfc = 0 if codes is None else codes.shape[1]
        f32 = dict(device=dev, dtype=torch.float32)
        if FUSED_FORWARD and prec == 6 and W in (128, 256) and dnet % 4 == 0 and nv % 4 == 0 and cfc % 4 == 0 and not nwin:
            H, hf, g, raw = _fused_forward(feat, codes, pw, pb, wa, ba, wf, bf, wv, bv, wr, br, W, D, skip, dnet, nv,
                                           cfc, dev)
            ctx.shape = shape
            ctx.has_codes = codes is not None
            ctx.save_for_backward(feat, codes if codes is not None else torch.empty(0), torch.empty(0), hf, g, whead,
                                  *H, *params)
            return raw
        # fp16x4 forward (prec 4): the GEMMs whose input is one hidden layer's output run as fp16x4
        # with that layer's row maxima (written by its GEMM's epilogue); layer 0, the skip layer's
        # [x | h] and the view / rgb layers (encoder columns in their input) stay bf16x6
        f16 = prec == ANERF_MLP_FP16X4 and W % 128 == 0  # (the row-max epilogue's tile width)
        prec = 6 if prec == ANERF_MLP_FP16X4 and not f16 else prec
        lp = [(ANERF_MLP_FP16X4 if (i >= 1 and i - 1 != skip) else 6) if f16 else prec for i in range(D)]
        hp, op_ = (ANERF_MLP_FP16X4, 6) if f16 else (prec, prec)
        # every layer's planes in one launch: [trunk..., head, views, rgb]
        sp = split_weights([(w, False, lp[i]) for i, w in enumerate(pw)] + [(whead, False, hp), (wv, False, op_),
                                                                            (wr, False, op_)], prec)
        rm = torch.zeros(D, M, device=dev, dtype=torch.int32) if f16 else [None] * D
        segx = _seg(feat, dnet)
        H = []
        for i in range(D):
            if i == 0:
                a, k = [segx], dnet
            elif i - 1 == skip:
                a, k = [segx, _seg(H[-1], W)], dnet + W
            else:
                a, k = [_seg(H[-1], W)], W
            h = torch.empty(M, W, **f32)
            if FORWARD_PERSISTENT and W == 256 and k > 128 and lp[i] in (3, 6) and not f16:
                forward_layer(M, k, a, sp[i], lp[i], pb[i], True, h, dev)
            else:
                gemm(M, W, k, a, sp[i], pb[i], True, [(h, W, W, 0, None, False)], dev, lp[i],
                     rin=rm[i - 1] if lp[i] == ANERF_MLP_FP16X4 else None, rout=rm[i] if f16 else None)
            H.append(h)
        # feature_linear + alpha_linear as one GEMM (alpha in raw[:, 3]); no activation
        raw = torch.empty(M, 4, **f32)
        hf = torch.empty(M, W, **f32)
        if FORWARD_PERSISTENT and W == 256 and hp in (3, 6) and not f16:  # (the split rows of whead's first 256 = wf's)
            forward_layer(M, W, [_seg(H[-1], W)], sp[D], hp, bf, False, hf, dev, alpha=(wa, ba, raw[:, 3]))
        else:
            bhead = torch.cat([bf, ba]).contiguous()
            gemm(M, W + 1, W, [_seg(H[-1], W)], sp[D], bhead, False,
                 [(hf, W, W, 0, None, False), (raw, 4, 1, 3, None, False)], dev, hp,
                 rin=rm[D - 1] if hp == ANERF_MLP_FP16X4 else None)
        prec = op_  # (the view and rgb layers)
        # views_linears[0] on cat([feature, views(, framecode)]), relu; view windows: sum_j w_j G_j joins the
        # GEMM's pre-activation (accumulate mode 2: product + bias + sum, then the relu)
        av = [_seg(hf, W)] + ([_seg(feat, nv, dnet)] if nv else []) + ([_seg(codes, cfc)] if cfc else [])
        if nwin:
            G = G.contiguous()
        g = _view_mix(feat, dnet, nwin, G) if nwin else torch.empty(M, W // 2, **f32)
        mm(M, W // 2, W + nv + cfc, av, sp[D + 1], bv, True, [(g, W // 2, W // 2, 0, None, 2 if nwin else 0)], dev)
        # rgb_linear into raw[:, :3]
        mm(M, 3, W // 2, [_seg(g, W // 2)], sp[D + 2], br, False, [(raw, 4, 3, 0, None, False)], dev)
        ctx.shape = shape
        ctx.has_codes = codes is not None
        ctx.save_for_backward(feat, codes if codes is not None else torch.empty(0), G if nwin else torch.empty(0), hf,
                              g, whead, *H, *params)
        return raw

    @staticmethod
    def backward(ctx, g_raw):
        W, D, skip, dnet, nv, _, prec, nwin = ctx.shape  # (the backward's own arithmetic)

        def mm(*a):
            gemm(*a, prec=prec)
        saved = ctx.saved_tensors
        feat, codes, G, hf, g, whead = saved[:6]
        H = saved[6:6 + D]
        params = saved[6 + D:]
        codes = codes if ctx.has_codes else None
        nl = D
        pw = params[0:2 * nl:2]
        wa, ba, wf, bf, wv, bv, wr, br = params[2 * nl:2 * nl + 8]
        dev = feat.device
        M, F = feat.shape
        cfc = 0 if codes is None else codes.shape[1]
        need_feat = ctx.needs_input_grad[1]
        need_codes = ctx.has_codes and ctx.needs_input_grad[2]
        fused = FUSED_BACKWARD and prec == 3 and W == 256
        # (round 6) with the fused kernel the skip layer's h part is one more 256 x 256 pass, and its x part joins
        # layer 0's products: both multiply the encoder features x, so [dY_0 | dY_s] (one [M, 2W] buffer the two
        # passes write) gives gfeat = [dY_0 | dY_s] [W_0 ; W_s,x] in one GEMM (K = 2W) and [dW_0 ; dW_s,x] =
        # [dY_0 | dY_s]^T x in one weight gradient: x, and the feature gradient, are read and written once
        s1 = skip + 1
        merge = fused and FUSED_SKIP and skip >= 0 and s1 < D - 1
        tw = list(pw)
        if merge:
            tw[s1] = pw[s1][:, dnet:]
            tw[0] = torch.cat([pw[0], pw[s1][:, :dnet]]) if need_feat else None
        # (round 6, ABI 18) the heads' backward on the fused pass too: feature_linear is a 256 x 256 layer on the last
        # hidden layer's output, alpha_linear's rank-1 term joins its input gradient (anerf_mlp_backward_head)
        fused_head = fused and FUSED_HEAD
        # every transposed plane in one launch: [trunk (layer 0 only for the feature gradient)..., head, views, rgb]
        st = split_weights([(w, True) for w in tw[0 if need_feat else 1:]]
                           + [(whead[:W] if fused_head else whead, True), (wv, True), (wr, True)], prec)
        st = ([None] if not need_feat else []) + st
        f32 = dict(device=dev, dtype=torch.float32)
        g_raw = g_raw.contiguous()
        lib = _lib.load()
        ws = [torch.empty(0, device=dev, dtype=torch.uint8)]  # grown to the largest layer's need
        grads = [None] * len(params)

        main = torch.cuda.current_stream(dev)
        side = _side_stream(dev) if WGRAD_OVERLAP else None

        def wg(n, k, dy, x, xt=()):
            """dW, db of one layer (x: its input segments over the tensors xt), on the side stream."""
            need = lib.anerf_mlp_wgrad_workspace(M, n, k)
            if ws[0].numel() < need:
                ws[0] = torch.empty(need, device=dev, dtype=torch.uint8)
            dw = torch.empty(n, k, **f32)
            db = torch.empty(n, **f32)
            if side is None:
                wgrad(M, n, k, dy, x, dw, db, ws[0], dev, prec)
                return dw, db
            side.wait_stream(main)  # (dy and the allocations above are the caller stream's work)
            with torch.cuda.stream(side):
                wgrad(M, n, k, dy, x, dw, db, ws[0], dev, prec)
            for t in (dy, dw, db, ws[0], *xt):  # (their memory is not reused before the side stream is done)
                t.record_stream(side)
            return dw, db

        # rgb_linear: input gradient masked by relu(view layer) > 0
        gzv = torch.empty(M, W // 2, **f32)
        mm(M, W // 2, 3, [_seg(g_raw, 3)], st[D + 2], None, False,
             [(gzv, W // 2, W // 2, 0, g, False)], dev)
        grads[2 * nl + 6], grads[2 * nl + 7] = wg(3, W // 2, g_raw, [_seg(g, W // 2)], (g,))
        # views_linears[0]: gradients of feature (into gha[:, :W]), view columns of feat, framecodes
        gha = torch.empty(M, W + 4, **f32)  # [g_feature | g_alpha] (ld padded to 16 B)
        gha[:, W].copy_(g_raw[:, 3])
        gha[:, W + 1:].zero_()  # (read as the ragged last 4-column group; the B planes are zero there)
        gfeat = torch.empty(M, F, **f32) if need_feat else None
        gcodes = torch.empty(M, cfc, **f32) if need_codes else None
        outs = [(gha, W + 4, W, 0, None, False)]
        if need_feat or need_codes:  # (the output columns in order [feature | views | framecode])
            if nv:
                outs.append((gfeat, F, nv, dnet, None, False))
            if cfc:
                outs.append((gcodes, cfc, cfc, 0, None, False))
        nvo = W + sum(o[2] for o in outs[1:])
        mm(M, nvo, W // 2, [_seg(gzv, W // 2)], st[D + 1], None, False, outs, dev)
        av = [_seg(hf, W)] + ([_seg(feat, nv, dnet)] if nv else []) + ([_seg(codes, cfc)] if cfc else [])
        grads[2 * nl + 4], grads[2 * nl + 5] = wg(W // 2, W + nv + cfc, gzv, av,
                                                  (hf, feat) + ((codes,) if cfc else ()))
        gG = None
        if nwin:  # the windows' gradient sum_h gzv G_j (into gfeat's window columns), and G's sum_s w_j gzv
            n = G.shape[0]
            gG = torch.empty_like(G)
            gw, off = (gfeat, dnet) if need_feat else (torch.empty(M, nwin, **f32), 0)
            _lib.check(lib.anerf_train_view_mix_backward(n, M // n, nwin, W // 2, feat.data_ptr() + 4 * dnet,
                                                         feat.stride(0), _lib.ptr(G), _lib.ptr(gzv),
                                                         gw.data_ptr() + 4 * off, gw.stride(0), _lib.ptr(gG),
                                                         _stream(dev)), "anerf_train_view_mix_backward")
        # feature_linear + alpha_linear: one input gradient, masked by relu(last hidden) > 0
        gz = torch.empty(M, W, **f32)
        if fused_head:
            hws = torch.empty(lib.anerf_mlp_backward_head_workspace(M, W), device=dev, dtype=torch.uint8)
            dwh, dbh = torch.empty(W + 1, W, **f32), torch.empty(W + 1, **f32)
            defer = side is not None
            _lib.check(lib.anerf_mlp_backward_head(M, W, _lib.ptr(gha), gha.stride(0), _lib.ptr(H[-1]), H[-1].stride(0),
                                                   _lib.ptr(st[D]), _lib.ptr(wa.contiguous()), prec, _lib.ptr(gz),
                                                   gz.stride(0), None if defer else _lib.ptr(dwh), dwh.stride(0),
                                                   None if defer else _lib.ptr(dbh), _lib.ptr(hws), hws.numel(),
                                                   _stream(dev)), "anerf_mlp_backward_head")
            if defer:  # (the slabs' reduce beside the trunk's first passes)
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    _lib.check(lib.anerf_mlp_backward_head_reduce(M, W, _lib.ptr(hws), hws.numel(), _lib.ptr(dwh),
                                                                  dwh.stride(0), _lib.ptr(dbh), _stream(dev)),
                               "anerf_mlp_backward_head_reduce")
                for t in (dwh, dbh, hws):
                    t.record_stream(side)
        else:
            mm(M, W, W + 1, [_seg(gha, W + 1)], st[D], None, False,
                 [(gz, W, W, 0, H[-1], False)], dev)
            dwh, dbh = wg(W + 1, W, gha, [_seg(H[-1], W)], (H[-1],))
        grads[2 * nl + 2], grads[2 * nl + 3] = dwh[:W], dbh[:W]  # feature_linear
        grads[2 * nl + 0], grads[2 * nl + 1] = dwh[W:], dbh[W:]  # alpha_linear
        # the trunk, last layer first
        segx = _seg(feat, dnet)
        wrote_x = False
        fws, fev, nfused = [None, None], [None, None], 0
        gzx = torch.empty(M, 2 * W, **f32) if merge else None  # [dY_0 | dY_s1]
        dwx = None
        for i in range(D - 1, -1, -1):
            if fused and i >= 1 and (i - 1 != skip or merge):  # one pass: gprev, dW, db (anerf_mlp_backward_hidden)
                # two workspaces in turn: layer i's slabs are summed on the side stream (its reduce beside the next
                # layer's pass) while layer i - 1 writes the other; a workspace is reused once its reduce is done
                slot = nfused & 1
                nfused += 1
                if fws[slot] is None:
                    fws[slot] = torch.empty(lib.anerf_mlp_backward_hidden_workspace(M, W), device=dev,
                                            dtype=torch.uint8)
                if fev[slot] is not None:
                    main.wait_event(fev[slot])
                ws_l = fws[slot]
                if merge and i in (1, s1 + 1):  # (dY_0, dY_s1: halves of gzx)
                    gprev = gzx[:, :W] if i == 1 else gzx[:, W:]
                else:
                    gprev = torch.empty(M, W, **f32)
                if merge and i == s1:  # (the h columns of the skip layer's weight gradient; x columns below)
                    dwf = torch.empty(W, dnet + W, **f32)
                    dw = dwf[:, dnet:]
                else:
                    dwf = dw = torch.empty(W, W, **f32)
                db = torch.empty(W, **f32)
                defer = side is not None
                _lib.check(lib.anerf_mlp_backward_hidden(M, W, _lib.ptr(gz), gz.stride(0), _lib.ptr(H[i - 1]),
                                                         H[i - 1].stride(0), _lib.ptr(st[i]), prec, _lib.ptr(gprev),
                                                         gprev.stride(0), None if defer else _lib.ptr(dw), dw.stride(0),
                                                         None if defer else _lib.ptr(db), _lib.ptr(ws_l),
                                                         ws_l.numel(), _stream(dev)), "anerf_mlp_backward_hidden")
                if defer:
                    side.wait_stream(main)
                    with torch.cuda.stream(side):
                        _lib.check(lib.anerf_mlp_backward_hidden_reduce(M, W, _lib.ptr(ws_l), ws_l.numel(),
                                                                        _lib.ptr(dw), dw.stride(0), _lib.ptr(db),
                                                                        _stream(dev)), "anerf_mlp_backward_hidden_reduce")
                        fev[slot] = torch.cuda.Event()
                        fev[slot].record(side)
                    for t in (dw, db, ws_l):
                        t.record_stream(side)
                grads[2 * i], grads[2 * i + 1] = dwf, db
                gz = gprev
                continue
            if i == 0 and merge:
                # (the feature gradient first: it is on the path to the encoder's and the poses' backward, and the
                # weight gradient's side-stream launch then waits for it instead of taking CUs from it)
                if need_feat:
                    # (one launch per 256 output columns, each reading all of [dY_0 | dY_s]: kept to <= 2 launches)
                    if FORWARD_PERSISTENT and prec in (3, 6) and dnet % 4 == 0 and F % 4 == 0 and dnet <= 2 * W:
                        gemm_persistent(M, dnet, 2 * W, [_seg(gzx, 2 * W)], st[0], prec, None, False, gfeat, dev)
                    else:
                        mm(M, dnet, 2 * W, [_seg(gzx, 2 * W)], st[0], None, False, [(gfeat, F, dnet, 0, None, False)],
                           dev)
                if side is not None:  # (every side-stream gradient before layer 0's: what the end of the MLP's
                    ev_pre = torch.cuda.Event()  # backward waits for when layer 0's own is deferred)
                    ev_pre.record(side)
                dwx, dbx = wg(2 * W, dnet, gzx, [segx], (feat, gzx))
                grads[0], grads[1] = dwx[:W], dbx[:W]
                break
            if i == 0:
                a, k = [segx], dnet
            elif i - 1 == skip:
                a, k = [segx, _seg(H[i - 1], W)], dnet + W
            else:
                a, k = [_seg(H[i - 1], W)], W
            grads[2 * i], grads[2 * i + 1] = wg(W, k, gz, a, (feat,) + ((H[i - 1],) if i > 0 else ()))
            if i == 0:
                if need_feat:
                    mm(M, dnet, W, [_seg(gz, W)], st[0], None, False,
                         [(gfeat, F, dnet, 0, None, wrote_x)], dev)
                break
            gprev = torch.empty(M, W, **f32)
            if i - 1 == skip:  # [x | h] input: the x part into the feature gradient, the h part masked
                mm(M, k, W, [_seg(gz, W)], st[i], None, False,
                     [(gfeat if need_feat else None, F, dnet, 0, None, False), (gprev, W, W, 0, H[i - 1], False)],
                     dev)
                wrote_x = need_feat
            else:
                mm(M, W, W, [_seg(gz, W)], st[i], None, False,
                     [(gprev, W, W, 0, H[i - 1], False)], dev)
            gz = gprev
        if side is not None:
            if dwx is not None:  # (the skip layer's x columns, after its side-stream weight gradient)
                with torch.cuda.stream(side):
                    grads[2 * s1][:, :dnet].copy_(dwx[W:])
                for t in (dwx, grads[2 * s1]):
                    t.record_stream(side)
            late = (params[0], params[1], params[2 * s1]) if dwx is not None else ()
            if DEFER_WGRAD_SYNC and late and all(p.is_leaf and p.grad is None for p in late):
                # layer 0's weight gradient (and the skip layer's x columns after it) are the last side-stream work:
                # the caller's stream waits for everything before them now, and for them once the whole backward has
                # been queued (the encoder's and the poses' backward run on meanwhile).  Their parameters are leaves
                # without a .grad, so the engine hands the tensors over uncopied and no kernel reads them before that
                # wait
                main.wait_event(ev_pre)
                ev = torch.cuda.Event()
                ev.record(side)
                torch.autograd.Variable._execution_engine.queue_callback(lambda: main.wait_event(ev))
            else:
                main.wait_stream(side)
        elif dwx is not None:
            grads[2 * s1][:, :dnet].copy_(dwx[W:])
        return (None, gfeat, gcodes, gG if ctx.needs_input_grad[3] else None, *grads)


def _fused_forward(feat, codes, pw, pb, wa, ba, wf, bf, wv, bv, wr, br, W, D, skip, dnet, nv, cfc, dev):
    """The whole forward in one kernel (anerf_mlp_forward, bf16x6): h_0..h_{D-1}, hf, g, raw."""
    lib = _lib.load()
    M = feat.shape[0]
    st = _stream(dev)
    shp = _lib.MlpShape(D, W, skip if skip >= 0 else -1, dnet, nv, cfc)
    wts = _lib.MlpFwdWeights()
    for i in range(D):
        wts.pts_w[i], wts.pts_ld[i] = pw[i].data_ptr(), pw[i].stride(0)
    wts.feature_w, wts.views_w, wts.views_ld = wf.data_ptr(), wv.data_ptr(), wv.stride(0)
    packed = torch.empty(lib.anerf_mlp_forward_pack_bytes(ctypes.byref(shp)), device=dev, dtype=torch.uint8)
    _lib.check(lib.anerf_mlp_forward_pack(ctypes.byref(shp), ctypes.byref(wts), _lib.ptr(packed), st),
               "anerf_mlp_forward_pack")
    f32 = dict(device=dev, dtype=torch.float32)
    H = [torch.empty(M, W, **f32) for _ in range(D)]
    hf = torch.empty(M, W, **f32)
    g = torch.empty(M, W // 2, **f32)
    raw = torch.empty(M, 4, **f32)
    io = _lib.MlpFwdIO()
    io.m, io.feat, io.ld_feat = M, feat.data_ptr(), feat.stride(0)
    if cfc:
        io.codes, io.ld_codes = codes.data_ptr(), codes.stride(0)
    for i in range(D):
        io.pts_b[i], io.h[i] = pb[i].data_ptr(), H[i].data_ptr()
    io.feature_b, io.alpha_w, io.alpha_b = bf.data_ptr(), wa.data_ptr(), ba.data_ptr()
    io.views_b, io.rgb_w, io.rgb_b = bv.data_ptr(), wr.data_ptr(), br.data_ptr()
    io.hf, io.g, io.raw = hf.data_ptr(), g.data_ptr(), raw.data_ptr()
    _lib.check(lib.anerf_mlp_forward(ctypes.byref(shp), ctypes.byref(io), _lib.ptr(packed), st), "anerf_mlp_forward")
    return H, hf, g, raw


# mode -> (forward, backward) arithmetic (ANERF_MLP_BF16X6 = 6, _BF16X3 = 3, _FP16X4 = 4).  "mixed": the
# forward fp32-accurate (every relu decision as in fp32), the gradients with ~16-bit operands (relative
# error ~1e-5, no branch decisions downstream of them); "mixed16": the forward's hidden-to-hidden
# products as fp16x4 (the same error bound as bf16x6, four products instead of six), else as "mixed"
MODES = {"bf16x6": (6, 6), "bf16x3": (3, 3), "mixed": (6, 3), "mixed16": (4, 3)}


def nerf_forward(net, feat, codes=None, G=None):
    """raw [M, 4] of `train.NeRF` on the split-bf16 GEMMs (same parameters, autograd included;
    precision net.mlp: "bf16x6" or "bf16x3").  G: the view-window layout's per-ray view factors (_MLP)."""
    cfg = net.cfg
    if feat.dtype != torch.float32 or not feat.is_contiguous():
        feat = feat.float().contiguous()
    if codes is not None:
        codes = codes.float().contiguous()
    W, D = cfg.netwidth, cfg.netdepth
    skip = cfg.skips[0] if cfg.skips[0] < D - 1 else -1
    fwd, bwd = MODES[net.mlp]
    dnet, nv = net.dnet, cfg.input_ch_views
    params = []
    for lin in net.pts_linears:
        params += [lin.weight, lin.bias]
    params += [net.alpha_linear.weight, net.alpha_linear.bias, net.feature_linear.weight, net.feature_linear.bias,
               net.views_linears[0].weight, net.views_linears[0].bias, net.rgb_linear.weight, net.rgb_linear.bias]
    nwin = 0
    if G is not None:  # (the view columns of views_linears.0 entered G: the GEMM's weight is [feature | framecode])
        nwin = G.shape[1]
        wv = params[2 * D + 4]
        params[2 * D + 4] = torch.cat([wv[:, :W], wv[:, W + nv:]], 1)
        nv = 0
        if dnet % 4 or feat.shape[1] % 4:  # (the NJ windows play the view block's part: [x | pad | w | pad])
            feat, params, dnet, _ = _pad_to_segments(feat, params, W, D, skip, dnet, nwin, pad_view_weight=False)
    elif dnet % 4 or nv % 4 or feat.shape[1] % 4:
        feat, params, dnet, nv = _pad_to_segments(feat, params, W, D, skip, dnet, nv)
    shape = (W, D, skip, dnet, nv, fwd, bwd, nwin)
    return _MLP.apply(shape, feat, codes, G, *params)


def _ceil4(x):
    return (x + 3) // 4 * 4


def _pad_to_segments(feat, params, W, D, skip, dnet, nv, pad_view_weight=True):
    """The GEMMs read operand segments as 16-byte float4 groups (anerf_gemm.hip set_segs): every
    segment starts 16-byte aligned, rows have ld % 4 == 0 and a segment followed by another has
    cols % 4 == 0.  The encoder's rows [x (18 NJ) | views (27 NJ)] meet that only for NJ % 4 == 0, so
    other joint counts (17, 65, ...) run on a copy whose x and view blocks are zero-padded to
    multiples of 4 columns, with zero weight columns inserted where the padding enters (layer 0, the
    skip layer's x part, the view layer's view part).  The padded products are the same sums plus
    exact zeros; torch autograd carries the gradients back through the pads to feat and the
    unpadded parameters.  The view-window layout's rows [x | w (NJ windows)] pad the same way, nv = NJ; their
    view layer has no view columns (pad_view_weight False)."""
    d4, v4 = _ceil4(dnet), _ceil4(nv)
    M = feat.shape[0]
    z = lambda c: feat.new_zeros(M, c)  # noqa: E731
    featp = torch.cat([feat[:, :dnet], z(d4 - dnet), feat[:, dnet:dnet + nv], z(v4 - nv)], 1).contiguous()

    def pad_cols(w, at, n):
        return torch.cat([w[:, :at], w.new_zeros(w.shape[0], n), w[:, at:]], 1).contiguous() if n else w
    params = list(params)
    params[0] = pad_cols(params[0], dnet, d4 - dnet)  # layer 0: [W][dnet]
    if skip >= 0:
        params[2 * (skip + 1)] = pad_cols(params[2 * (skip + 1)], dnet, d4 - dnet)  # [x | h]
    if pad_view_weight:
        iv = 2 * D + 4  # views_linears.0: [feature (W) | views (nv) | framecode]
        params[iv] = pad_cols(params[iv], W + nv, v4 - nv)
    return featp, params, d4, v4


__all__ = ["nerf_forward", "split_weight", "split_weights", "gemm", "wgrad"]

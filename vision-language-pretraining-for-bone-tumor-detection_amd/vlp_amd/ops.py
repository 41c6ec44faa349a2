"""Tensor-level wrappers over the C ABI (libvlp_hip.so).

PyTorch provides only device memory (caching allocator), the current stream,
and zero-fills; every arithmetic operation below is a hand-written HIP kernel.
All functions enqueue on torch's current stream and never synchronise.
"""
from __future__ import annotations

import torch

from . import ktimer
from ._lib import BF16, F32, lib, ptr, stream_of


def dcode(t: torch.Tensor) -> int:
    if t.dtype == torch.bfloat16:
        return BF16
    if t.dtype == torch.float32:
        return F32
    raise TypeError(f"unsupported storage dtype {t.dtype}")


def _s():
    return stream_of()


def conv_out_hw(H, W, KH, KW, S, P):
    return (H + 2 * P - KH) // S + 1, (W + 2 * P - KW) // S + 1


# kernel-family keys mirror the tile dispatch in csrc (one key = one kernel name)
def _tile_auto(n):
    return "/narrow" if n <= 64 else "/wide"


def _tile_wgrad(m):
    return "/short" if m <= 64 else "/wide"


def _tile_lin(m, n):
    return "/narrow" if n <= 64 else ("/64x256" if m <= 1024 else "/wide")


# ---------------- convolutions ----------------
def conv_fwd(x, wp, Co, KH, KW, S, P, in_scale=None, in_shift=None, stat_sum=None, stat_sumsq=None,
             out=None, stat_rep=1):
    N, H, W, C = x.shape
    Ho, Wo = conv_out_hw(H, W, KH, KW, S, P)
    y = out if out is not None else torch.empty((N, Ho, Wo, Co), dtype=x.dtype, device=x.device)
    if stat_sum is None:
        stat_sum = torch.zeros(Co, dtype=torch.float64, device=x.device)
        stat_sumsq = torch.zeros(Co, dtype=torch.float64, device=x.device)
    tk = ktimer.begin(f"conv_fwd[{'xf' if in_scale is not None else 'raw'}]{_tile_auto(Co)}",
                      2.0 * N * Ho * Wo * Co * C * KH * KW)
    lib().vlp_conv_fwd(dcode(x), ptr(x), ptr(wp), ptr(y), N, H, W, C, Co, KH, KW, S, P,
                       ptr(in_scale), ptr(in_shift), ptr(stat_sum), ptr(stat_sumsq), int(stat_rep), _s())
    ktimer.end(tk)
    return y


def conv_fwd_act_ok(x, Co, KH, KW, S, P):
    N, H, W, C = x.shape
    return bool(lib()._dll.vlp_conv_fwd_act_ok(dcode(x), N, H, W, C, Co, KH, KW, S, P))


def conv_fwd_act(x, wp, Co, KH, KW, S, P, in_scale, in_shift, x_act, stat_sum, stat_sumsq, stat_rep=1, out=None):
    """conv(relu(in_scale*x + in_shift)) with that activation also written to x_act
    (vlp_conv_fwd_act: BN-apply + ReLU fused into the layer-1 rows kernel's ring)."""
    N, H, W, C = x.shape
    Ho, Wo = conv_out_hw(H, W, KH, KW, S, P)
    y = out if out is not None else torch.empty((N, Ho, Wo, Co), dtype=x.dtype, device=x.device)
    tk = ktimer.begin("conv_fwd[act]/" + ("narrow" if C == 64 else "wide"), 2.0 * N * Ho * Wo * Co * C * KH * KW)
    lib().vlp_conv_fwd_act(dcode(x), ptr(x), ptr(wp), ptr(y), ptr(x_act), N, H, W, C, Co, KH, KW, S, P,
                           ptr(in_scale), ptr(in_shift), ptr(stat_sum), ptr(stat_sumsq), int(stat_rep), _s())
    ktimer.end(tk)
    return y


def conv_dgrad(dy, wt, H, W, C, KH, KW, S, P, addend=None, y_bn=None, bn=None, stat1=None,
               stat2=None, out=None, stat_rep=1):
    """bn = (scale, shift, mean, invstd) of the BN+ReLU producing the conv input."""
    N, Ho, Wo, Co = dy.shape
    dx = out if out is not None else torch.empty((N, H, W, C), dtype=dy.dtype, device=dy.device)
    sc = sh = mu = ist = None
    if y_bn is not None:
        sc, sh, mu, ist = bn
    tk = ktimer.begin(f"conv_dgrad[{'bn' if y_bn is not None else 'add'}]{_tile_auto(C)}",
                      2.0 * N * Ho * Wo * Co * C * KH * KW)
    lib().vlp_conv_dgrad(dcode(dy), ptr(dy), ptr(wt), ptr(dx), N, H, W, C, Co, KH, KW, S, P,
                         ptr(addend), ptr(y_bn), ptr(sc), ptr(sh), ptr(mu), ptr(ist), ptr(stat1),
                         ptr(stat2), int(stat_rep), _s())
    ktimer.end(tk)
    return dx


def conv_dgrad_relu(dy, wt, H, W, C, KH, KW, S, P, relu_out, y, mean, invstd, stat1, stat2,
                    addend=None, stat_rep=1, out=None):
    """g = (dgrad(dy) + addend) * (relu_out > 0), plus the BN backward sums of g
    against y (the next block's bn2 input).  relu_out may be the activation or
    its uint8 sign-bit mask (bn_add_relu / maxpool_fwd relu_mask)."""
    N, Ho, Wo, Co = dy.shape
    g = out if out is not None else torch.empty((N, H, W, C), dtype=dy.dtype, device=dy.device)
    bits = relu_out.dtype == torch.uint8
    tk = ktimer.begin(f"conv_dgrad[relu]{_tile_auto(C)}", 2.0 * N * Ho * Wo * Co * C * KH * KW)
    lib().vlp_conv_dgrad_relu(dcode(dy), ptr(dy), ptr(wt), ptr(g), N, H, W, C, Co, KH, KW, S, P,
                              ptr(addend), None if bits else ptr(relu_out), ptr(relu_out) if bits else None,
                              ptr(y), ptr(mean), ptr(invstd), ptr(stat1), ptr(stat2), int(stat_rep), _s())
    ktimer.end(tk)
    return g


def conv_dgrad_act_ok(dy, C, KH, KW, S, P):
    N, H, W, Co = dy.shape
    return bool(lib()._dll.vlp_conv_dgrad_act_ok(dcode(dy), N, H, W, C, Co, KH, KW, S, P))


def bn_bwd_coef(M, gamma, istd, mean, sum_g, sum_gx, coef):
    """coef[3][C] = (k, b, c) of the folded BN backward dy = k*g + b*y + c."""
    lib().vlp_bn_bwd_coef(int(M), gamma.numel(), ptr(gamma), ptr(istd), ptr(mean), ptr(sum_g), ptr(sum_gx),
                          ptr(coef), _s())


def conv_dgrad_bn_act(g_in, y_in, in_coef, dy_out, wt, H, W, C, KH, KW, S, P, y_bn, bn, stat1, stat2,
                      stat_rep=1, out=None):
    """conv_dgrad(dy, y_bn=..., bn=...) with dy = k*g_in + b*y_in + c formed in the
    layer-1 rows kernel's ring from in_coef (bn_bwd_coef) and written to dy_out
    (vlp_conv_dgrad_bn_act: the bn_bwd_apply pass fused)."""
    N, Ho, Wo, Co = g_in.shape
    dx = out if out is not None else torch.empty((N, H, W, C), dtype=g_in.dtype, device=g_in.device)
    sc, sh, mu, ist = bn
    tk = ktimer.begin("conv_dgrad[bn,act]/narrow", 2.0 * N * Ho * Wo * Co * C * KH * KW)
    lib().vlp_conv_dgrad_bn_act(dcode(g_in), ptr(g_in), ptr(y_in), ptr(in_coef), ptr(dy_out), ptr(wt), ptr(dx),
                                N, H, W, C, Co, KH, KW, S, P, ptr(y_bn), ptr(sc), ptr(sh), ptr(mu), ptr(ist),
                                ptr(stat1), ptr(stat2), int(stat_rep), _s())
    ktimer.end(tk)
    return dx


def conv_dgrad_relu_act(g_in, y_in, in_coef, dy_out, wt, H, W, C, KH, KW, S, P, relu_out, y, mean, invstd,
                        stat1, stat2, addend=None, stat_rep=1, out=None):
    """conv_dgrad_relu with its input dy = k*g_in + b*y_in + c formed in the rows
    kernel's ring and written to dy_out (vlp_conv_dgrad_relu_act)."""
    N, Ho, Wo, Co = g_in.shape
    g = out if out is not None else torch.empty((N, H, W, C), dtype=g_in.dtype, device=g_in.device)
    bits = relu_out.dtype == torch.uint8
    tk = ktimer.begin("conv_dgrad[relu,act]/narrow", 2.0 * N * Ho * Wo * Co * C * KH * KW)
    lib().vlp_conv_dgrad_relu_act(dcode(g_in), ptr(g_in), ptr(y_in), ptr(in_coef), ptr(dy_out), ptr(wt), ptr(g),
                                  N, H, W, C, Co, KH, KW, S, P, ptr(addend), None if bits else ptr(relu_out),
                                  ptr(relu_out) if bits else None, ptr(y), ptr(mean), ptr(invstd), ptr(stat1),
                                  ptr(stat2), int(stat_rep), _s())
    ktimer.end(tk)
    return g


def conv_dgrad_relu_ds(dy, dyd, wt, wtd, H, W, C, KH, KW, S, P, relu_out, y, mean, invstd, stat1, stat2,
                       stat_rep=1, out=None):
    """conv_dgrad_relu of a stride-2 conv with the 1x1/2 downsample's data gradient
    (dyd against wtd) folded into parity class (0, 0) in the same GEMMs
    (vlp_conv_dgrad_relu_ds).  dyd must follow dy and wtd follow wt in memory."""
    N, Ho, Wo, Co = dy.shape
    g = out if out is not None else torch.empty((N, H, W, C), dtype=dy.dtype, device=dy.device)
    bits = relu_out.dtype == torch.uint8
    flops = 2.0 * N * Ho * Wo * Co * C * (KH * KW + 1)
    tk = ktimer.begin(f"conv_dgrad[relu,ds]{_tile_auto(C)}", flops)
    lib().vlp_conv_dgrad_relu_ds(dcode(dy), ptr(dy), ptr(dyd), ptr(wt), ptr(wtd), ptr(g), N, H, W, C, Co, KH, KW, S,
                                 P, None if bits else ptr(relu_out), ptr(relu_out) if bits else None, ptr(y),
                                 ptr(mean), ptr(invstd), ptr(stat1), ptr(stat2), int(stat_rep), _s())
    ktimer.end(tk)
    return g


def conv_dgrad_relu2(dy, wt, H, W, C, KH, KW, S, P, relu_mask, y, mean, invstd, yd, meand, invstdd,
                     stat1, stat2, stat3, addend=None, stat_rep=1, out=None):
    """g = (dgrad(dy) + addend) * relu bits, with the three BN backward sums of a
    block whose output feeds its bn2 (y, mean, invstd) and its downsample BN (yd,
    meand, invstdd): sum g, sum g*xhat, sum g*xhatd (vlp_conv_dgrad_relu2)."""
    N, Ho, Wo, Co = dy.shape
    g = out if out is not None else torch.empty((N, H, W, C), dtype=dy.dtype, device=dy.device)
    tk = ktimer.begin(f"conv_dgrad[relu2]{_tile_auto(C)}", 2.0 * N * Ho * Wo * Co * C * KH * KW)
    lib().vlp_conv_dgrad_relu2(dcode(dy), ptr(dy), ptr(wt), ptr(g), N, H, W, C, Co, KH, KW, S, P, ptr(addend),
                               ptr(relu_mask), ptr(y), ptr(mean), ptr(invstd), ptr(yd), ptr(meand), ptr(invstdd),
                               ptr(stat1), ptr(stat2), ptr(stat3), int(stat_rep), _s())
    ktimer.end(tk)
    return g


def conv_wgrad(dy, x, KH, KW, S, P, dw_ws, in_scale=None, in_shift=None):
    N, H, W, C = x.shape
    Co = dy.shape[-1]
    Ho, Wo = dy.shape[1], dy.shape[2]
    tk = ktimer.begin(f"conv_wgrad[{'xf' if in_scale is not None else 'raw'}]{_tile_wgrad(Co)}",
                      2.0 * N * Ho * Wo * Co * C * KH * KW)
    lib().vlp_conv_wgrad(dcode(dy), ptr(dy), ptr(x), ptr(dw_ws), N, H, W, C, Co, KH, KW, S, P,
                         ptr(in_scale), ptr(in_shift), _s())
    ktimer.end(tk)
    return dw_ws


WGRAD_WS_FLOATS = 32 << 20   # 128 MB of split-K slabs (the largest conv needs ~17M floats at bs=256)
# Split-K slab workspaces, one per (device, stream).  A workspace is only ever
# written and folded by launches on ONE stream, so the stream order is its
# only synchronisation: the text tower's backward (its own stream), the image
# tower's weight-gradient side stream and the main stream each get their own
# buffer.  Allocated while that stream is current, so the caching allocator
# also ties the block (and a replaced, smaller block) to that stream.
_WS_CACHE = {}


def _stream_ws(kind, device, elems):
    import torch as _t
    st = _t.cuda.current_stream(device) if device.type == "cuda" else None
    key = (kind, str(device), st.cuda_stream if st is not None else 0)
    buf = _WS_CACHE.get(key)
    if buf is None or buf.numel() < elems:
        buf = torch.empty(elems, dtype=torch.float32, device=device)
        _WS_CACHE[key] = buf
    return buf


def wgrad_ws(device):
    return _stream_ws("wgrad", device, WGRAD_WS_FLOATS)


def conv_wgrad_into(dy, x, KH, KW, S, P, grad):
    """grad[Co][C][KH][KW] = sum over pixels dy x_patch, overwriting grad (the
    parameter's own gradient layout).  The GEMM's K-splits write fp32 slabs of
    a cached workspace; one fold pass sums and transposes them."""
    import ctypes
    N, H, W, C = x.shape
    Co, Ho, Wo = dy.shape[-1], dy.shape[1], dy.shape[2]
    ws = wgrad_ws(dy.device)
    ns = ctypes.c_int(0)
    tk = ktimer.begin(f"conv_wgrad[raw]{_tile_wgrad(Co)}", 2.0 * N * Ho * Wo * Co * C * KH * KW)
    lib().vlp_conv_wgrad_ws(dcode(dy), ptr(dy), ptr(x), ptr(ws), ws.numel(), ctypes.addressof(ns), N, H, W, C,
                            Co, KH, KW, S, P, _s())
    ktimer.end(tk)
    lib().vlp_conv_wgrad_fold(Co, C, KH, KW, ns.value, ptr(ws), ptr(grad), _s())
    return grad


def stem_wgrad_into(dy, xp, N, H, W, grad):
    """grad[64][3][7][7] = stem weight gradient (overwrites), via per-split
    fp32 slabs of the shared weight-gradient workspace and one fold pass."""
    import ctypes
    ws = wgrad_ws(dy.device)
    ns = ctypes.c_int(0)
    tk = ktimer.begin("stem_wgrad", 2.0 * dy.numel() * 147)
    lib().vlp_stem_wgrad_ws(dcode(dy), ptr(dy), ptr(xp), ptr(ws), ws.numel(), ctypes.addressof(ns), N, H, W, _s())
    ktimer.end(tk)
    lib().vlp_stem_wgrad_fold(ns.value, ptr(ws), ptr(grad), _s())
    return grad


def stem_geom(H, W):
    import ctypes
    a, b, c, d = (ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int())
    lib()._dll.vlp_stem_geom(H, W, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c),
                             ctypes.byref(d))
    return a.value, b.value, c.value, d.value


def stem1_geom(H, W):
    """(Ho, Wo, Hp, Wp1) of the single-channel stem, or None when it does not apply
    (Wo % 4 != 0: the caller takes the 3-channel path)."""
    import ctypes
    a, b, c, d = (ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int())
    r = lib()._dll.vlp_stem1_geom(H, W, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c), ctypes.byref(d))
    return None if r else (a.value, b.value, c.value, d.value)


def stem1_prep_u8(x_u8, xs, mean, std):
    N, H, W = x_u8.shape[0], x_u8.shape[-2], x_u8.shape[-1]
    lib().vlp_stem1_prep_u8(dcode(xs), ptr(x_u8), ptr(xs), N, H, W, float(mean), float(std), _s())


def pack_stem1(w, wp1):
    lib().vlp_pack_stem1(dcode(wp1), ptr(w), ptr(wp1), _s())


def stem1_fwd(xs, wp1, N, H, W, y, stat_sum, stat_sumsq, stat_rep=1):
    tk = ktimer.begin("stem_fwd", 2.0 * y.numel() * 147)
    lib().vlp_stem1_fwd(dcode(xs), ptr(xs), ptr(wp1), ptr(y), N, H, W, ptr(stat_sum), ptr(stat_sumsq),
                        int(stat_rep), _s())
    ktimer.end(tk)


def stem1_wgrad_into(dy, xs, N, H, W, grad):
    """grad[64][3][7][7] = stem weight gradient of the single-channel path (overwrites)."""
    import ctypes
    ws = wgrad_ws(dy.device)
    ns = ctypes.c_int(0)
    tk = ktimer.begin("stem_wgrad", 2.0 * dy.numel() * 147)
    lib().vlp_stem1_wgrad_ws(dcode(dy), ptr(dy), ptr(xs), ptr(ws), ws.numel(), ctypes.addressof(ns), N, H, W, _s())
    ktimer.end(tk)
    lib().vlp_stem1_wgrad_fold(ns.value, ptr(ws), ptr(grad), _s())
    return grad


def stem1_fused_ok(H, W):
    return bool(lib()._dll.vlp_stem1_fused_ok(int(H), int(W)))


def stem1_pool_fwd(xs, wp1, gamma, yarg, idx, N, H, W, stat_sum=None, stat_sumsq=None, stat_rep=1):
    """Fused stem conv + BN sums + 3x3/2 max-pool of sign(gamma)*y0 (bf16); y0 is never stored."""
    tk = ktimer.begin("stem_fwd", 2.0 * N * (H // 2) * (W // 2) * 64 * 147)
    lib().vlp_stem1_pool_fwd(ptr(xs), ptr(wp1), ptr(gamma), ptr(yarg), ptr(idx), N, H, W, ptr(stat_sum),
                             ptr(stat_sumsq), int(stat_rep), _s())
    ktimer.end(tk)


def stem1_route_bwd(xs, wp1, dp, idx, sc, sh, mean, istd, gamma, sum_g, sum_gx, dy, N, H, W):
    lib().vlp_stem1_route_bwd(ptr(xs), ptr(wp1), ptr(dp), ptr(idx), ptr(sc), ptr(sh), ptr(mean), ptr(istd),
                              ptr(gamma), ptr(sum_g), ptr(sum_gx), ptr(dy), N, H, W, _s())


def stem1_bwd_fused_into(xs, wp1, dp, idx, mean, istd, gamma, sum_g, sum_gx, N, H, W, grad):
    """grad[64][3][7][7] = the stem weight gradient from the pooled gradient dp
    (ReLU-masked): routing, BN backward and the weight gradient in one pass
    through the batch sums R = sum g P^T, G = sum P P^T, S = sum P (y0 and dy
    never formed); per-workgroup slabs folded in a fixed order."""
    import ctypes
    n = ctypes.c_longlong(0)
    lib().vlp_stem1_bwd_fused_ws_floats(N, H, W, ctypes.byref(n))
    ws = _stream_ws("wgrad", dp.device, max(n.value, WGRAD_WS_FLOATS))
    tk = ktimer.begin("stem_bwd_fused", 6.0 * N * (H // 2) * (W // 2) * 64 * 64)
    lib().vlp_stem1_bwd_fused(ptr(xs), ptr(wp1), ptr(dp), ptr(idx), ptr(mean), ptr(istd), ptr(gamma), ptr(sum_g),
                              ptr(sum_gx), ptr(ws), ws.numel(), ptr(grad), N, H, W, _s())
    ktimer.end(tk)
    return grad


def stem_prep(x_nchw, xp):
    N, _, H, W = x_nchw.shape
    lib().vlp_stem_prep(dcode(xp), ptr(x_nchw), ptr(xp), N, H, W, _s())


def stem_prep_u8(x_u8, xp, mean, std):
    N, H, W = x_u8.shape[0], x_u8.shape[-2], x_u8.shape[-1]
    lib().vlp_stem_prep_u8(dcode(xp), ptr(x_u8), ptr(xp), N, H, W, float(mean), float(std), _s())


def stem_fwd(xp, wp, N, H, W, y, stat_sum, stat_sumsq, stat_rep=1):
    tk = ktimer.begin("stem_fwd", 2.0 * y.numel() * 147)
    lib().vlp_stem_fwd(dcode(xp), ptr(xp), ptr(wp), ptr(y), N, H, W, ptr(stat_sum),
                       ptr(stat_sumsq), int(stat_rep), _s())
    ktimer.end(tk)


def stem_wgrad(dy, xp, N, H, W, dw_ws):
    tk = ktimer.begin("stem_wgrad", 2.0 * dy.numel() * 147)
    lib().vlp_stem_wgrad(dcode(dy), ptr(dy), ptr(xp), ptr(dw_ws), N, H, W, _s())
    ktimer.end(tk)


# ---------------- BN / pooling ----------------
def stat_reduce(rep, C, a, b=None, c=None):
    lib().vlp_stat_reduce(int(rep), int(C), ptr(a), ptr(b), ptr(c), _s())


def bn_finalize_rep(rep, count, s, ss, gamma, beta, eps, momentum, running_mean, running_var, scale, shift,
                    mean, invstd):
    """Fold the [rep][C] replicated sums and finalize in one launch."""
    lib().vlp_bn_finalize_rep(int(rep), gamma.numel(), float(count), ptr(s), ptr(ss), ptr(gamma), ptr(beta),
                              float(eps), float(momentum), ptr(running_mean), ptr(running_var),
                              ptr(scale), ptr(shift), ptr(mean), ptr(invstd), _s())


def bn_grad_rep(rep, C, sum_g, sum_gx, dgamma, dbeta, sum_gxd=None, dgamma_d=None, dbeta_d=None):
    lib().vlp_bn_grad_rep(int(rep), int(C), ptr(sum_g), ptr(sum_gx), ptr(sum_gxd), ptr(dgamma), ptr(dbeta),
                          ptr(dgamma_d), ptr(dbeta_d), _s())


def bn_finalize(count, s, ss, gamma, beta, eps, momentum, running_mean, running_var, scale, shift,
                mean, invstd):
    lib().vlp_bn_finalize(gamma.numel(), float(count), ptr(s), ptr(ss), ptr(gamma), ptr(beta),
                          float(eps), float(momentum), ptr(running_mean), ptr(running_var),
                          ptr(scale), ptr(shift), ptr(mean), ptr(invstd), _s())


def bn_eval_coeffs(gamma, beta, rm, rv, eps, scale, shift):
    lib().vlp_bn_eval_coeffs(gamma.numel(), ptr(gamma), ptr(beta), ptr(rm), ptr(rv), float(eps),
                             ptr(scale), ptr(shift), _s())


def bn_add_relu(y, sc, sh, idt, scd, shd, out, relu_mask=None):
    C = y.shape[-1]
    M = y.numel() // C
    lib().vlp_bn_add_relu(dcode(y), M, C, ptr(y), ptr(sc), ptr(sh), ptr(idt), ptr(scd), ptr(shd),
                          ptr(out), ptr(relu_mask), _s())


def bn_bwd_reduce(M, C, dout, dbc, HW, mask, ya, mean_a, istd_a, yb, mean_b, istd_b, sum_g, sum_ga,
                  sum_gb, dtype_ref, stat_rep=1):
    lib().vlp_bn_bwd_reduce(dcode(dtype_ref), M, C, ptr(dout), ptr(dbc), HW, ptr(mask), ptr(ya),
                            ptr(mean_a), ptr(istd_a), ptr(yb), ptr(mean_b), ptr(istd_b), ptr(sum_g),
                            ptr(sum_ga), ptr(sum_gb), int(stat_rep), _s())


def bn_bwd_apply(M, C, dout, dbc, HW, mask, A, B, g_out, dtype_ref):
    """A/B = (y, mean, istd, gamma, sum_g, sum_gx, dy_out) or None."""
    a = A if A is not None else (None,) * 7
    b = B if B is not None else (None,) * 7
    lib().vlp_bn_bwd_apply(dcode(dtype_ref), M, C, ptr(dout), ptr(dbc), HW, ptr(mask),
                           *[ptr(t) for t in a], *[ptr(t) for t in b], ptr(g_out), _s())


def bn_param_grad(sum_g, sum_gx, dgamma, dbeta):
    lib().vlp_bn_param_grad(dgamma.numel(), ptr(sum_g), ptr(sum_gx), ptr(dgamma), ptr(dbeta), _s())


def maxpool_fwd(y, sc, sh, out, idx, yarg=None, relu_mask=None):
    N, H, W, C = y.shape
    lib().vlp_maxpool_fwd(dcode(y), N, H, W, C, ptr(y), ptr(sc), ptr(sh), ptr(out), ptr(idx), ptr(yarg),
                          ptr(relu_mask), _s())


def maxpool_bwd(dp, idx, y, sc, sh, mean, istd, sum_g, sum_gx, stat_rep=1):
    """BN backward sums of the routed, ReLU-masked stem gradient (nothing stored)."""
    N, H, W, C = y.shape
    lib().vlp_maxpool_bwd(dcode(y), N, H, W, C, ptr(dp), ptr(idx), ptr(y), ptr(sc), ptr(sh),
                          ptr(mean), ptr(istd), ptr(sum_g), ptr(sum_gx), int(stat_rep), _s())


def maxpool_bwd_apply(dp, idx, y, sc, sh, mean, istd, gamma, sum_g, sum_gx, dy):
    """dy = BN1'(relu-masked routed gradient), recomputing the routing."""
    N, H, W, C = y.shape
    lib().vlp_maxpool_bwd_apply(dcode(y), N, H, W, C, ptr(dp), ptr(idx), ptr(y), ptr(sc), ptr(sh),
                                ptr(mean), ptr(istd), ptr(gamma), ptr(sum_g), ptr(sum_gx), ptr(dy), _s())


def avgpool_fwd(x, feat):
    N, H, W, C = x.shape
    lib().vlp_avgpool_fwd(dcode(x), N, H * W, C, ptr(x), ptr(feat), _s())


# ---------------- text tower ----------------
def linear_fwd(x, w, bias, y, M, N, K, ldx=None, ldy=None, mode=0, aux=None, res=None, ldr=None,
               p=0.0, seed=0):
    tk = ktimer.begin(f"linear_fwd{_tile_lin(M, N)}", 2.0 * M * N * K)
    lib().vlp_linear_fwd(dcode(x), M, N, K, ptr(x), ldx or K, ptr(w), ptr(bias), ptr(y), ldy or N,
                         mode, ptr(aux), ptr(res), ldr or N, float(p), int(seed), _s())
    ktimer.end(tk)


def linear_fwd_rs(x, w, bias, y, res, rscale, rps, M, N, K):
    """y = res + rscale[row // rps] * (x W^T + bias)  (residual branch under DropPath)."""
    tk = ktimer.begin(f"linear_fwd{_tile_lin(M, N)}", 2.0 * M * N * K)
    lib().vlp_linear_fwd_rs(dcode(x), M, N, K, ptr(x), K, ptr(w), ptr(bias), ptr(y), N, ptr(res), N, ptr(rscale),
                            int(rps), _s())
    ktimer.end(tk)


def linear_dgrad(dy, w, dx, M, Kin, Nout, lddy=None, lddx=None, mode=0, aux=None, ldaux=None,
                 addend=None, ldad=None):
    tk = ktimer.begin(f"linear_dgrad{_tile_lin(M, Kin)}", 2.0 * M * Kin * Nout)
    lib().vlp_linear_dgrad(dcode(dy), M, Kin, Nout, ptr(dy), lddy or Nout, ptr(w), ptr(dx),
                           lddx or Kin, mode, ptr(aux), ldaux or Kin, ptr(addend), ldad or Kin, _s())
    ktimer.end(tk)


def _linw_ws(device, elems):
    """Split-K slabs of the linear weight gradients: per (device, stream), so the
    text tower's backward on its own stream and NesT's on the main stream never
    share (or free under each other) a workspace."""
    return _stream_ws("linw", device, elems)


def linear_wgrad(dy, x, dw, M, Nout, Kin, lddy=None, ldx=None):
    """dw[Nout][Kin] += dy^T x.  bf16: split-K partial slabs in a cached fp32
    workspace folded by one reduction pass; fp32: atomic split-K."""
    tk = ktimer.begin("linear_wgrad/wide", 2.0 * M * Nout * Kin)
    if dy.dtype == torch.bfloat16 and Kin % 4 == 0:
        import ctypes
        n = ctypes.c_longlong(0)
        lib().vlp_linear_wgrad_ws_floats(M, Nout, Kin, ctypes.byref(n))
        ws = _linw_ws(dy.device, max(n.value, 16 * Nout * Kin))
        lib().vlp_linear_wgrad_ws(dcode(dy), M, Nout, Kin, ptr(dy), lddy or Nout, ptr(x), ldx or Kin,
                                  ptr(dw), ptr(ws), ws.numel(), _s())
    else:
        lib().vlp_linear_wgrad(dcode(dy), M, Nout, Kin, ptr(dy), lddy or Nout, ptr(x), ldx or Kin,
                               ptr(dw), _s())
    ktimer.end(tk)


def colsum(x, out, M, N, ld=None):
    lib().vlp_colsum(dcode(x), M, N, ptr(x), ld or N, ptr(out), _s())


def layernorm_fwd(x, gamma, beta, eps, y, mean, rstd, M, D, p=0.0, seed=0):
    lib().vlp_layernorm_fwd(dcode(x), M, D, ptr(x), ptr(gamma), ptr(beta), float(eps), ptr(y),
                            ptr(mean), ptr(rstd), float(p), int(seed), _s())


def layernorm_bwd(dy, x, mean, rstd, gamma, dx, dxd, dgamma, dbeta, M, D, p_out=0.0, seed_out=0,
                  p_in=0.0, seed_in=0):
    lib().vlp_layernorm_bwd(dcode(dy), M, D, ptr(dy), float(p_out), int(seed_out), ptr(x),
                            ptr(mean), ptr(rstd), ptr(gamma), ptr(dx), ptr(dxd), float(p_in),
                            int(seed_in), ptr(dgamma), ptr(dbeta), _s())


def attn_fwd(qkv, amask, ctx, P, B, T, H, dh, scale, p=0.0, seed=0):
    lib().vlp_attn_fwd(dcode(qkv), B, T, H, dh, ptr(qkv), ptr(amask), ptr(ctx), ptr(P),
                       float(scale), float(p), int(seed), _s())


def attn_bwd(qkv, P, dctx, dqkv, B, T, H, dh, scale, p=0.0, seed=0):
    lib().vlp_attn_bwd(dcode(qkv), B, T, H, dh, ptr(qkv), ptr(P), ptr(dctx), ptr(dqkv),
                       float(scale), float(p), int(seed), _s())


def embed_fwd(ids, tt, wemb, pemb, temb, e_out, M, T, D):
    lib().vlp_embed_fwd(dcode(e_out), M, T, D, ptr(ids), ptr(tt), ptr(wemb), ptr(pemb), ptr(temb),
                        ptr(e_out), _s())


def embed_bwd(ids, tt, de, dwemb, dpemb, dtemb, M, T, D):
    lib().vlp_embed_bwd(dcode(de), M, T, D, ptr(ids), ptr(tt), ptr(de), ptr(dwemb), ptr(dpemb),
                        ptr(dtemb), _s())


def scatter_rows(src, dst, R, D, ldi, ldo):
    lib().vlp_scatter_rows(dcode(src), R, D, ptr(src), ldi, ptr(dst), ldo, _s())


# ---------------- head ----------------
def l2norm_fwd(x, y, norm):
    R, E = x.shape
    lib().vlp_l2norm_fwd(R, E, ptr(x), ptr(y), ptr(norm), _s())


def l2norm_bwd(y, norm, dy, dx=None, dx_t=None, gscale=None):
    R, E = y.shape
    code = dcode(dx_t) if dx_t is not None else F32
    lib().vlp_l2norm_bwd(code, R, E, ptr(y), ptr(norm), ptr(dy), ptr(gscale), ptr(dx), ptr(dx_t),
                         _s())


def scale(x, s, y, accumulate=False):
    lib().vlp_scale(x.numel(), ptr(x), ptr(s), ptr(y), int(accumulate), _s())


def clip_loss_finish(parts, N, out):
    lib().vlp_clip_loss_finish(ptr(parts), int(N), ptr(out), _s())


def clip_loss_fused(B, N, E, offset, img_all, txt_all, logit_scale, g_img_all, g_txt_all, d_ls,
                    loss_parts, lse_out=None, role_w=None):
    """Global-batch symmetric InfoNCE + gradients (three launches, split over key
    chunks; the scratch is a per-(device, stream) cached workspace)."""
    import ctypes
    n = ctypes.c_longlong(0)
    lib().vlp_clip_loss_ws_floats(B, N, E, ctypes.addressof(n))
    ws = _stream_ws("clip", img_all.device, n.value)
    lib().vlp_clip_loss_fused(B, N, E, offset, ptr(img_all), ptr(txt_all), ptr(logit_scale),
                              ptr(g_img_all), ptr(g_txt_all), ptr(d_ls), ptr(loss_parts),
                              ptr(lse_out), ptr(role_w), ptr(ws), ws.numel(), _s())


def ce_sym(logits, out, dlogits=None, role_w=None):
    lib().vlp_ce_sym(logits.shape[0], ptr(logits), ptr(out), ptr(dlogits), ptr(role_w), _s())


def matmul(A, B, C, M, N, K, lda, a_kc, ldb, b_kc, ldc, alpha=1.0, accumulate=False, dtype_ref=None):
    ref = dtype_ref if dtype_ref is not None else A
    out_f32 = 1 if C.dtype == torch.float32 else 0
    lib().vlp_matmul(dcode(ref), M, N, K, ptr(A), lda, int(a_kc), ptr(B), ldb, int(b_kc), ptr(C),
                     ldc, out_f32, float(alpha), int(accumulate), _s())


def cast(x, y):
    lib().vlp_cast(dcode(y), x.numel(), ptr(x), ptr(y), _s())


# ---------------- optimizer / packing ----------------
def adamw(p, g, m, v, lr, beta1, beta2, eps, wd, step):
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    lib().vlp_adamw(p.numel(), ptr(p), ptr(g), ptr(m), ptr(v), float(lr), float(beta1),
                    float(beta2), float(eps), float(wd), float(lr / bc1), float(bc2 ** 0.5), _s())


def pack_conv(w, wp, wt):
    Co, C, KH, KW = w.shape
    ref = wp if wp is not None else wt
    lib().vlp_pack_conv(dcode(ref), Co, C, KH, KW, ptr(w), ptr(wp), ptr(wt), _s())


def pack_conv_batch(dtype_ref, entries):
    """entries: [(w fp32 [Co][C][KH][KW], wp, wt)] packed in one launch.
    Returns the ctypes descriptor table (reusable with pack_conv_batch_run)."""
    import ctypes
    rows = []
    for w, wp, wt in entries:
        Co, C, KH, KW = w.shape
        rows += [w.data_ptr(), wp.data_ptr() if wp is not None else 0, wt.data_ptr() if wt is not None else 0,
                 Co, C, KH * KW]
    table = (ctypes.c_longlong * len(rows))(*rows)
    return (dcode(dtype_ref), len(entries), table)


def pack_conv_batch_run(desc):
    import ctypes
    code, n, table = desc
    lib().vlp_pack_conv_batch(code, n, ctypes.addressof(table), _s())


def pack_stem(w, wp):
    lib().vlp_pack_stem(dcode(wp), ptr(w), ptr(wp), _s())


def unpack_conv_grad(ws, g):
    Co, C, KH, KW = g.shape
    lib().vlp_unpack_conv_grad(Co, C, KH, KW, ptr(ws), ptr(g), _s())


def unpack_stem_grad(ws, g):
    lib().vlp_unpack_stem_grad(ptr(ws), ptr(g), _s())


# ---------------- retrieval metrics ----------------
SIM_CHUNK_BYTES = 256 << 20


def sim_topk(q, keys, K):
    """Top-K (values, indices) of q @ keys^T per row, descending (ties to the
    lower index), without materialising the full similarity matrix: query
    chunks of <= 256 MB of fp32 similarities, each an fp32 GEMM
    (vlp_linear_fwd) reduced by vlp_row_topk.  q [Q, E], keys [N, E] fp32."""
    q = q.float().contiguous()
    keys = keys.float().contiguous()
    if q.shape[1] % 4:   # 16-B operand rows: zero columns leave every dot product unchanged
        pad = 4 - q.shape[1] % 4
        q = torch.nn.functional.pad(q, (0, pad))
        keys = torch.nn.functional.pad(keys, (0, pad))
    Q, E = q.shape
    N = keys.shape[0]
    Np = (N + 3) // 4 * 4   # 16-B rows for the GEMM epilogue
    vals = torch.empty(Q, K, device=q.device)
    idx = torch.empty(Q, K, dtype=torch.int32, device=q.device)
    rows = max(1, min(Q, SIM_CHUNK_BYTES // (4 * Np)))
    tile = torch.empty(rows, Np, device=q.device)
    for r0 in range(0, Q, rows):
        r = min(rows, Q - r0)
        linear_fwd(q[r0:r0 + r], keys, None, tile, r, N, E, ldy=Np)
        lib().vlp_row_topk(r, N, ptr(tile), Np, K, ptr(vals[r0:r0 + r]), ptr(idx[r0:r0 + r]), _s())
    return vals, idx.long()


# ---------------- NesT image encoder ----------------
def nest_attn_fwd(qkv, out, lse, BT, H, N, scale):
    tk = ktimer.begin("nest_attn_fwd", 4.0 * BT * H * N * N * 32)
    lib().vlp_nest_attn_fwd(dcode(qkv), BT, H, N, 32, ptr(qkv), ptr(out), ptr(lse), float(scale), _s())
    ktimer.end(tk)


def nest_attn_bwd(qkv, out, dout, lse, delta, dqkv, BT, H, N, scale):
    tk = ktimer.begin("nest_attn_bwd", 10.0 * BT * H * N * N * 32)
    lib().vlp_nest_attn_bwd(dcode(qkv), BT, H, N, 32, ptr(qkv), ptr(out), ptr(dout), ptr(lse), ptr(delta),
                            ptr(dqkv), float(scale), _s())
    ktimer.end(tk)


def nest_blockify(x, y, B, Hg, Wg, bs, C, pos=None, inverse=False):
    lib().vlp_nest_blockify(dcode(x), B, Hg, Wg, bs, C, ptr(x), ptr(pos), ptr(y), int(inverse), _s())


def nest_pos_grad(dy, dpos, B, TN, C):
    lib().vlp_nest_pos_grad(dcode(dy), B, TN, C, ptr(dy), ptr(dpos), _s())


def nest_maxpool_fwd(x, y, idx):
    B, H, W, C = x.shape
    lib().vlp_nest_maxpool_fwd(dcode(x), B, H, W, C, ptr(x), ptr(y), ptr(idx), _s())


def nest_maxpool_bwd(dy, idx, dx):
    B, H, W, C = dx.shape
    lib().vlp_nest_maxpool_bwd(dcode(dy), B, H, W, C, ptr(dy), ptr(idx), ptr(dx), _s())


def nest_patch_prep(out, B, H, W, bs, x=None, x_u8=None, mean=0.0, std=1.0):
    lib().vlp_nest_patch_prep(dcode(out), B, H, W, bs, ptr(x), ptr(x_u8), float(mean), float(std), ptr(out), _s())


def nest_add_bias(y, bias, M, N):
    lib().vlp_nest_add_bias(dcode(y), M, N, ptr(y), ptr(bias), _s())


def nest_permute_cols(src, dst, Nr, H, Dh):
    lib().vlp_nest_permute_cols(dcode(dst), Nr, H, Dh, ptr(src), ptr(dst), _s())


def nest_unpermute_cols(src, dst, Nr, H, Dh):
    lib().vlp_nest_unpermute_cols(Nr, H, Dh, ptr(src), ptr(dst), _s())


def nest_rowscale(x, y, s, M, N, rows, mode):
    lib().vlp_nest_rowscale(dcode(x), M, N, rows, ptr(s), ptr(x), ptr(y), int(mode), _s())


def nest_bcast(dfeat, dy, B, HW, C, inv):
    lib().vlp_nest_bcast(dcode(dy), B, HW, C, ptr(dfeat), float(inv), ptr(dy), _s())


def layernorm_bwd_add(dy, x, mean, rstd, gamma, addend, dx, dgamma, dbeta, M, D, dxs=None, rscale=None, rps=1):
    """dx = LN backward + addend; with rscale also dxs = rscale[row // rps] * dx."""
    if rscale is None:
        lib().vlp_layernorm_bwd_add(dcode(dy), M, D, ptr(dy), ptr(x), ptr(mean), ptr(rstd), ptr(gamma),
                                    ptr(addend), ptr(dx), ptr(dgamma), ptr(dbeta), _s())
    else:
        lib().vlp_layernorm_bwd_add_rs(dcode(dy), M, D, ptr(dy), ptr(x), ptr(mean), ptr(rstd), ptr(gamma),
                                       ptr(addend), ptr(dx), ptr(dxs), ptr(rscale), int(rps), ptr(dgamma),
                                       ptr(dbeta), _s())


# ---------------- radiograph preprocessing / augmentation (csrc/prep_ops.hip) ----------------
PREP_WORK_BYTES_PER_IMAGE = (64 * 2 + 256 + 2) * 4


def prep_images(src, src_u8, off, hw, n, size, mean, std, channels, out, work):
    """src: packed pixels (device, uint8 or fp32); off [n] int64 / hw [n, 2] int32 (device)."""
    lib().vlp_prep_images(n, ptr(src), int(bool(src_u8)), ptr(off), ptr(hw), int(size), float(mean), float(std),
                          int(channels), ptr(out), ptr(work), _s())


def aug_warp(x, out, maps, noise_std, seed, mean=0.0, std=1.0):
    """x: fp32 [B, Cin, H, W] or uint8 [B, 1, H, W]; out fp32 [B, C, H, W]; maps [B, 6] fp32."""
    B, Cin, H, W = x.shape
    C = out.shape[1]
    lib().vlp_aug_warp(B, Cin, C, H, W, ptr(x), int(x.dtype == torch.uint8), float(mean), float(std), ptr(maps),
                       ptr(noise_std), int(seed) & ((1 << 64) - 1), ptr(out), _s())

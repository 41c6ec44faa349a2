"""NesT kernels (csrc/nest_ops.hip) against plain torch references of the timm
nest.py operations they replace (timm==1.0.15, not installed: the references
below restate them; the same restatement is oracle/nest.py).

  attention  vlp_nest_attn_fwd / _bwd vs softmax(q k^T * d^-1/2) v per image
             block and head (timm Attention, fused_attn = F.sdpa), fp64 autograd
  blockify   vlp_nest_blockify (+ pos) / inverse vs timm blockify / deblockify
  maxpool    vlp_nest_maxpool_fwd / _bwd vs F.max_pool2d(3, 2, 1) (ConvPool)
  patch      vlp_nest_patch_prep + GEMM vs the 4x4/4 patch-embedding conv
  misc       column permutation of the proj weight, DropPath row scale, avg-pool
             backward broadcast
Tolerances: fp32 storage rel-L2 <= 1e-5 (attention backward 2e-5); bf16 storage
vs fp32 math on the same bf16-rounded inputs <= 2e-2; index work bit-exact.
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DT = [torch.float32, torch.bfloat16]


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


@pytest.fixture(scope="module")
def ops():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vlp_amd import ops as o
    return o


def ref_attention(qkv, BT, N, H):
    """timm nest Attention on qkv rows [BT*N][3C]; output head-major [BT*N][C]."""
    C = qkv.shape[1] // 3
    q, k, v = qkv.view(BT, N, 3, H, 32).permute(2, 0, 3, 1, 4)           # [BT, H, N, 32]
    p = torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(32), dim=-1)
    o = (p @ v).permute(0, 2, 1, 3).reshape(BT * N, C)
    return o


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("BT,H,N,amp", [(3, 2, 64, 1.0), (2, 3, 200, 1.0), (2, 3, 1024, 1.0), (1, 1, 16, 1.0),
                                         (2, 2, 36, 1.0), (2, 2, 130, 1.0), (2, 1, 300, 3.0)])
def test_attention_fwd_bwd(ops, dt, BT, H, N, amp):
    """amp scales q and k: amp 3 makes peaked rows whose running maximum moves
    between key tiles (the online-softmax rescale path)."""
    g = torch.Generator().manual_seed(N + H)
    C = 32 * H
    qkv = torch.randn(BT * N, 3 * C, generator=g)
    qkv[:, :2 * C] *= amp
    qkv = qkv.to(dt).float()
    do = torch.randn(BT * N, C, generator=g).to(dt).float()
    x = qkv.double().requires_grad_()
    o_ref = ref_attention(x, BT, N, H)
    o_ref.backward(do.double())
    qd = qkv.to(dt).cuda()
    out = torch.empty(BT * N, C, dtype=dt, device="cuda")
    lse = torch.empty(BT * H * N, device="cuda")
    ops.nest_attn_fwd(qd, out, lse, BT, H, N, 1 / math.sqrt(32))
    dqkv = torch.full_like(qd, float("nan"))
    delta = torch.empty(BT * H * N, device="cuda")
    ops.nest_attn_bwd(qd, out, do.to(dt).cuda(), lse, delta, dqkv, BT, H, N, 1 / math.sqrt(32))
    torch.cuda.synchronize()
    tol = 1e-5 if dt == torch.float32 else 2e-2
    assert rel(out.float(), o_ref) < tol, rel(out.float(), o_ref)
    # the saved log2-sum-exp of the scaled scores
    q, k, _ = qkv.double().view(BT, N, 3, H, 32).permute(2, 0, 3, 1, 4)
    lse_ref = torch.logsumexp(q @ k.transpose(-1, -2) / math.sqrt(32), -1) / math.log(2)
    assert (lse.cpu().double().view(BT, H, N) - lse_ref).abs().max().item() < (1e-4 if dt == torch.float32 else 5e-2)
    assert torch.isfinite(dqkv.float()).all()
    assert rel(dqkv.float(), x.grad) < (2e-5 if dt == torch.float32 else 2e-2), rel(dqkv.float(), x.grad)


def test_attention_rejects_bad_head_dim(ops):
    from vlp_amd._lib import lib
    t = torch.zeros(64 * 3 * 48, device="cuda")
    with pytest.raises(RuntimeError):
        lib().vlp_nest_attn_fwd(0, 1, 1, 64, 48, t.data_ptr(), t.data_ptr(), t.data_ptr(), 0.1, None)


def timm_blockify(x, bs):
    B, H, W, C = x.shape
    x = x.reshape(B, H // bs, bs, W // bs, bs, C).transpose(2, 3).reshape(B, (H // bs) * (W // bs), -1, C)
    return x


@pytest.mark.parametrize("dt", DT)
def test_blockify_pos_and_inverse(ops, dt):
    g = torch.Generator().manual_seed(0)
    B, Hg, Wg, bs, C = 2, 2, 3, 4, 16
    x = torch.randn(B, Hg * bs, Wg * bs, C, generator=g).to(dt)
    pos = torch.randn(Hg * Wg, bs * bs, C, generator=g)
    ref = timm_blockify(x.float(), bs) + pos
    y = torch.empty(B, Hg * Wg, bs * bs, C, dtype=dt, device="cuda")
    ops.nest_blockify(x.cuda(), y, B, Hg, Wg, bs, C, pos=pos.cuda())
    back = torch.empty_like(x.cuda())
    ops.nest_blockify(y, back, B, Hg, Wg, bs, C, inverse=True)
    dpos = torch.empty(Hg * Wg * bs * bs, C, device="cuda")
    ops.nest_pos_grad(y, dpos, B, Hg * Wg * bs * bs, C)
    torch.cuda.synchronize()
    assert rel(y.float(), ref) < (1e-6 if dt == torch.float32 else 1e-2)
    # deblockify is the exact inverse permutation (of the stored values)
    assert torch.equal(timm_blockify(back.cpu().float(), bs), y.cpu().float())
    assert rel(dpos.view(Hg * Wg, bs * bs, C), y.float().sum(0).cpu()) < 1e-5


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("H,W", [(8, 8), (7, 10)])
def test_maxpool_3x3s2(ops, dt, H, W):
    g = torch.Generator().manual_seed(H * W)
    B, C = 2, 24
    x = torch.randn(B, H, W, C, generator=g).to(dt)
    xr = x.float().permute(0, 3, 1, 2).contiguous().requires_grad_()
    yr = F.max_pool2d(xr, 3, 2, 1)
    dy = torch.randn(yr.shape, generator=g).to(dt).float()
    yr.backward(dy)
    Ho, Wo = yr.shape[-2:]
    y = torch.empty(B, Ho, Wo, C, dtype=dt, device="cuda")
    idx = torch.empty(B, Ho, Wo, C, dtype=torch.uint8, device="cuda")
    ops.nest_maxpool_fwd(x.cuda(), y, idx)
    dx = torch.empty(B, H, W, C, dtype=dt, device="cuda")
    ops.nest_maxpool_bwd(dy.permute(0, 2, 3, 1).contiguous().to(dt).cuda(), idx, dx)
    torch.cuda.synchronize()
    assert torch.equal(y.cpu().float(), yr.detach().permute(0, 2, 3, 1))
    assert rel(dx.float(), xr.grad.permute(0, 2, 3, 1)) < (1e-6 if dt == torch.float32 else 1e-2)


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("u8", [False, True])
def test_patch_embed(ops, dt, u8):
    g = torch.Generator().manual_seed(7)
    B, Hi, bs, Co = 2, 64, 4, 96                # 16 x 16 patches, 4 x 4 blocks of 4 x 4 tokens
    if u8:
        xu = torch.randint(0, 256, (B, 1, Hi, Hi), generator=g, dtype=torch.uint8)
        x = ((xu.float() - 127.5) / 73.9).expand(B, 3, Hi, Hi).contiguous()
    else:
        x = torch.randn(B, 3, Hi, Hi, generator=g)
    w = torch.randn(Co, 3, 4, 4, generator=g) * 0.1
    bias = torch.randn(Co, generator=g) * 0.1
    ref = F.conv2d(x.to(dt).float(), w.to(dt).float(), bias, stride=4).permute(0, 2, 3, 1)   # [B, 16, 16, Co]
    ref = timm_blockify(ref, bs).reshape(-1, Co)
    M = B * (Hi // 4) ** 2
    pm = torch.empty(M, 48, dtype=dt, device="cuda")
    if u8:
        ops.nest_patch_prep(pm, B, Hi, Hi, bs, x_u8=xu.cuda(), mean=127.5, std=73.9)
    else:
        ops.nest_patch_prep(pm, B, Hi, Hi, bs, x=x.cuda())
    y = torch.empty(M, Co, dtype=dt, device="cuda")
    ops.linear_fwd(pm, w.reshape(Co, 48).to(dt).cuda(), bias.cuda(), y, M, Co, 48)
    torch.cuda.synchronize()
    assert rel(y.float(), ref) < (1e-5 if dt == torch.float32 else 2e-2), rel(y.float(), ref)


def test_permute_rowscale_bcast(ops):
    g = torch.Generator().manual_seed(3)
    Nr, H, Dh = 40, 3, 32
    w = torch.randn(Nr, H * Dh, generator=g)
    wp = torch.empty(Nr, H * Dh, device="cuda")
    ops.nest_permute_cols(w.cuda(), wp, Nr, H, Dh)
    back = torch.empty_like(wp)
    ops.nest_unpermute_cols(wp, back, Nr, H, Dh)
    # proj(o_timm) with o_timm[d*H + h] == (permuted proj)(o_headmajor[h*Dh + d])
    o = torch.randn(5, H, Dh, generator=g)
    o_timm = o.permute(0, 2, 1).reshape(5, H * Dh)
    o_hm = o.reshape(5, H * Dh)
    torch.cuda.synchronize()
    assert torch.allclose(o_timm @ w.T, o_hm @ wp.cpu().T, atol=1e-5)
    assert torch.equal(back.cpu(), w)
    M, N, rows = 12, 16, 4
    x = torch.randn(M, N, generator=g).cuda()
    y = torch.randn(M, N, generator=g).cuda()
    s = torch.tensor([0.0, 2.0, 1.0], device="cuda")
    ref = x + s.repeat_interleave(rows)[:, None] * y
    x2 = x.clone()
    ops.nest_rowscale(x2, y, s, M, N, rows, 0)
    y2 = torch.empty_like(y)
    ops.nest_rowscale(x, y2, s, M, N, rows, 1)
    dfeat = torch.randn(2, 8, generator=g).cuda()
    dy = torch.empty(2 * 5, 8, device="cuda")
    ops.nest_bcast(dfeat, dy, 2, 5, 8, 0.2)
    torch.cuda.synchronize()
    assert torch.allclose(x2, ref, atol=1e-6)
    assert torch.allclose(y2, s.repeat_interleave(rows)[:, None] * x, atol=1e-6)
    assert torch.allclose(dy.view(2, 5, 8), (dfeat * 0.2)[:, None, :].expand(2, 5, 8), atol=1e-7)


@pytest.mark.parametrize("dt", DT)
def test_linear_fwd_rowscale(ops, dt):
    """vlp_linear_fwd_rs: res + s[row // rps] * (x W^T + b) (DropPath residual)."""
    g = torch.Generator().manual_seed(7)
    B, rps, N, K = 3, 40, 96, 192
    M = B * rps
    x = torch.randn(M, K, generator=g).to(dt).float()
    w = torch.randn(N, K, generator=g).mul(0.1).to(dt).float()
    b = torch.randn(N, generator=g)
    res = torch.randn(M, N, generator=g).to(dt).float()
    s = torch.tensor([0.0, 2.0, 1.25])
    ref = res.double() + s.double().repeat_interleave(rps)[:, None] * (x.double() @ w.double().T + b.double())
    y = torch.empty(M, N, dtype=dt, device="cuda")
    ops.linear_fwd_rs(x.to(dt).cuda(), w.to(dt).cuda(), b.cuda(), y, res.to(dt).cuda(), s.cuda(), rps, M, N, K)
    torch.cuda.synchronize()
    assert rel(y.float(), ref) < (1e-5 if dt == torch.float32 else 1e-2)


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("D", [96, 192, 384, 312])
def test_layernorm_fwd_bwd_add_rowscale(ops, dt, D):
    """Vectorized LayerNorm forward (eps 1e-6) and the pre-norm backward with
    addend and the DropPath-scaled second output, vs torch autograd (fp64)."""
    g = torch.Generator().manual_seed(D)
    B, rps = 2, 37
    M = B * rps
    x = torch.randn(M, D, generator=g).mul(2).add(0.5).to(dt).float()
    gam = torch.randn(D, generator=g)
    bet = torch.randn(D, generator=g)
    dy = torch.randn(M, D, generator=g).to(dt).float()
    add = torch.randn(M, D, generator=g).to(dt).float()
    s = torch.tensor([2.0, 0.0])
    xd = x.double().requires_grad_()
    gd, bd = gam.double().requires_grad_(), bet.double().requires_grad_()
    yref = F.layer_norm(xd, (D,), gd, bd, 1e-6)
    yref.backward(dy.double())
    dxref = xd.grad + add.double()
    y = torch.empty(M, D, dtype=dt, device="cuda")
    mu, rs = torch.empty(M, device="cuda"), torch.empty(M, device="cuda")
    xc = x.to(dt).cuda()
    ops.layernorm_fwd(xc, gam.cuda(), bet.cuda(), 1e-6, y, mu, rs, M, D)
    dx = torch.empty(M, D, dtype=dt, device="cuda")
    dxs = torch.empty(M, D, dtype=dt, device="cuda")
    dg, db = torch.zeros(D, device="cuda"), torch.zeros(D, device="cuda")
    ops.layernorm_bwd_add(dy.to(dt).cuda(), xc, mu, rs, gam.cuda(), add.to(dt).cuda(), dx, dg, db, M, D,
                          dxs=dxs, rscale=s.cuda(), rps=rps)
    torch.cuda.synchronize()
    tol = 1e-5 if dt == torch.float32 else 1e-2
    assert rel(y.float(), yref.detach()) < tol
    assert rel(dx.float(), dxref) < tol
    assert rel(dxs.float(), s.double().repeat_interleave(rps)[:, None] * dxref) < tol
    assert rel(dg, gd.grad) < 1e-5 and rel(db, bd.grad) < 1e-5


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("BT,H,N,amp", [(2, 3, 1024, 1.0), (3, 2, 200, 3.0), (4, 12, 256, 1.0), (2, 1, 70, 1.0)])
def test_attention_asm_loads_match_compiler_loads(ops, dt, BT, H, N, amp):
    """the attention kernels issue their tile loads as inline asm and
    wait for them by hand (csrc/nest_ops.hip, VLP_ATTN_ASMLOAD), which is only
    correct while the compiler never copies an in-flight register before the
    wait.  The build refuses scratch in those kernels (csrc/Makefile); here the
    product library must be BIT-IDENTICAL to libvlp_nest_plainload.so, the same
    source built with compiler-placed loads, for fwd, dQ and dK/dV."""
    import ctypes
    import os
    from vlp_amd import _lib
    path = os.path.join(os.path.dirname(_lib.__file__), "libvlp_nest_plainload.so")
    plain = ctypes.CDLL(path)
    protos = _lib.parse_header()
    fns = {}
    for name in ("vlp_nest_attn_fwd", "vlp_nest_attn_bwd"):
        f = getattr(plain, name)
        f.argtypes = [ctypes.c_void_p if t == "ptr" else _lib._CTYPE[t] for t, _ in protos[name]["args"]]
        f.restype = ctypes.c_int
        fns[name] = f
    g = torch.Generator().manual_seed(7 * N + H)
    C = 32 * H
    qkv = torch.randn(BT * N, 3 * C, generator=g)
    qkv[:, :2 * C] *= amp
    qd = qkv.to(dt).cuda()
    do = torch.randn(BT * N, C, generator=g).to(dt).cuda()
    sc = 1 / math.sqrt(32)
    code = _lib.BF16 if dt == torch.bfloat16 else _lib.F32
    st = torch.cuda.current_stream().cuda_stream
    res = []
    for use_plain in (False, True):
        out = torch.full((BT * N, C), float("nan"), dtype=dt, device="cuda")
        lse = torch.full((BT * H * N,), float("nan"), device="cuda")
        dqkv = torch.full_like(qd, float("nan"))
        delta = torch.empty(BT * H * N, device="cuda")
        if use_plain:
            assert fns["vlp_nest_attn_fwd"](code, BT, H, N, 32, qd.data_ptr(), out.data_ptr(), lse.data_ptr(),
                                            sc, st) == 0
            assert fns["vlp_nest_attn_bwd"](code, BT, H, N, 32, qd.data_ptr(), out.data_ptr(), do.data_ptr(),
                                            lse.data_ptr(), delta.data_ptr(), dqkv.data_ptr(), sc, st) == 0
        else:
            ops.nest_attn_fwd(qd, out, lse, BT, H, N, sc)
            ops.nest_attn_bwd(qd, out, do, lse, delta, dqkv, BT, H, N, sc)
        torch.cuda.synchronize()
        res.append((out, lse, dqkv))
    (o0, l0, d0), (o1, l1, d1) = res
    assert torch.isfinite(o0.float()).all() and torch.isfinite(d0.float()).all()
    assert torch.equal(o0, o1) and torch.equal(l0, l1)
    assert torch.equal(d0[:, :C], d1[:, :C]), "dQ differs"
    assert torch.equal(d0[:, C:], d1[:, C:]), "dK/dV differs"

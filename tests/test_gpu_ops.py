"""Op-level parity of the HIP kernels against the CPU fp32 oracle ops.

fp32 storage mode must match torch fp32 to ~1e-5 relative; bf16 mode is
compared against fp32 math on the SAME bf16-rounded inputs, tolerance 2e-2
relative (bf16 output rounding + fp32 accumulation order).
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DT = [torch.float32, torch.bfloat16]


def rel(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def tol(dt):
    return 2e-5 if dt == torch.float32 else 1.5e-2


@pytest.fixture(scope="module")
def ops():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vlp_amd import ops as o
    return o


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("akc,bkc", [(1, 1), (1, 0), (0, 1), (0, 0)])
def test_matmul_layouts(ops, dt, akc, bkc):
    torch.manual_seed(0)
    M, N, K = 208, 136, 328
    A = torch.randn(M, K).to(dt).float()
    B = torch.randn(N, K).to(dt).float()
    ref = A @ B.T
    Ad = (A if akc else A.T.contiguous()).to(dt).cuda()
    Bd = (B if bkc else B.T.contiguous()).to(dt).cuda()
    C = torch.empty(M, N, device="cuda", dtype=torch.float32)
    ops.matmul(Ad, Bd, C, M, N, K, K if akc else M, akc, K if bkc else N, bkc, N)
    torch.cuda.synchronize()
    assert rel(C, ref) < tol(dt) / 4


CONV_CASES = [
    # N, H, W, C, Co, KH, KW, S, P
    (2, 12, 12, 64, 64, 3, 3, 1, 1),
    (2, 12, 12, 64, 128, 3, 3, 2, 1),
    (2, 12, 12, 64, 128, 1, 1, 2, 0),
    (3, 7, 9, 128, 64, 3, 3, 1, 1),
    (3, 5, 128, 64, 64, 3, 3, 1, 1),    # layer-1 width: row-streaming kernel (bf16)
    (2, 12, 12, 256, 256, 3, 3, 1, 1),  # M, N >= 256: 256x256 large-tile kernel (bf16)
    (4, 7, 7, 512, 512, 3, 3, 1, 1),    # layer 4 at 224 px, B = 4
    (4, 14, 14, 256, 512, 3, 3, 2, 1),  # layer-4 stride-2 block at 224 px
    (2, 16, 16, 96, 192, 3, 3, 1, 1),   # NesT ConvPool (C = 96: K-steps straddle filter taps)
    (2, 8, 8, 192, 384, 3, 3, 1, 1),    # NesT ConvPool, level 2
    # ping-pong kernel (gemm_pp_kernel, bf16 M, N >= 256): K = 2880 is an odd number of
    # 64-deep steps (the half-tile ring starts on slot 2); N = 320 / M = 297 end in partial tiles
    (4, 8, 8, 320, 256, 3, 3, 1, 1),
    (2, 12, 12, 128, 128, 3, 3, 1, 1),  # Co = 128 weight gradient: 128x384 ping-pong tiles
    (3, 9, 11, 256, 320, 3, 3, 1, 1),
    # LDS-window kernel (bf16 3x3 stride 1, W in {16, 32, 64}, C and the GEMM N multiples of 128):
    # one window per 256-pixel tile of whole rows, several N tiles, NC = 2 / 4 / 8 channel chunks
    (2, 8, 64, 128, 128, 3, 3, 1, 1),
    (3, 4, 64, 256, 128, 3, 3, 1, 1),
    (2, 8, 64, 128, 256, 3, 3, 1, 1),
    (2, 16, 32, 256, 256, 3, 3, 1, 1),
    (2, 16, 16, 512, 512, 3, 3, 1, 1),
]


def nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def nchw(t):
    return t.permute(0, 3, 1, 2).contiguous()


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("case", CONV_CASES)
@pytest.mark.parametrize("xform", [False, True])
def test_conv_fwd(ops, dt, case, xform):
    N, H, W, C, Co, KH, KW, S, P = case
    torch.manual_seed(1)
    x = torch.randn(N, C, H, W).to(dt).float()
    w = (torch.randn(Co, C, KH, KW) * (C * KH * KW) ** -0.5).to(dt).float()
    sc = torch.rand(C) + 0.5
    sh = torch.randn(C) * 0.3
    xin = torch.relu(x * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1)) if xform else x
    if xform and dt == torch.bfloat16:
        xin = xin.to(dt).float()
    ref = F.conv2d(xin, w, stride=S, padding=P)
    wp = torch.empty(Co, KH, KW, C, dtype=dt, device="cuda")
    ops.pack_conv(w.cuda(), wp, None)
    s1 = torch.zeros(Co, dtype=torch.float64, device="cuda")
    s2 = torch.zeros_like(s1)
    y = ops.conv_fwd(nhwc(x).to(dt).cuda(), wp, Co, KH, KW, S, P,
                     sc.cuda() if xform else None, sh.cuda() if xform else None, s1, s2)
    torch.cuda.synchronize()
    assert rel(nchw(y.float().cpu()), ref) < tol(dt)
    assert rel(s1.cpu(), ref.sum((0, 2, 3))) < 1e-4
    assert rel(s2.cpu(), (ref * ref).sum((0, 2, 3))) < 1e-4


@pytest.mark.parametrize("N,H,W,C,Co", [(32, 64, 64, 128, 128), (128, 16, 16, 512, 512)])
def test_conv_fwd_window_many_tiles(ops, N, H, W, C, Co):
    """The LDS-window forward at >= 2 tiles per CU against torch fp32 on the GPU, with
    the BN sums; every tile's output checked."""
    torch.manual_seed(21)
    dev = torch.device("cuda")
    x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    w = (torch.randn(Co, C, 3, 3, device=dev) * (9 * C) ** -0.5).to(torch.bfloat16)
    wp = torch.empty(Co, 3, 3, C, dtype=torch.bfloat16, device=dev)
    ops.pack_conv(w.float(), wp, None)
    s1 = torch.zeros(4 * Co, dtype=torch.float64, device=dev)
    s2 = torch.zeros_like(s1)
    y = ops.conv_fwd(x, wp, Co, 3, 3, 1, 1, stat_sum=s1, stat_sumsq=s2, stat_rep=4)
    ref = F.conv2d(x.permute(0, 3, 1, 2).float(), w.float(), padding=1).permute(0, 2, 3, 1)
    torch.cuda.synchronize()
    err = (y.float() - ref).reshape(-1, 256, Co).norm(dim=(1, 2)) / ref.reshape(-1, 256, Co).norm(dim=(1, 2))
    assert err.max().item() < 1e-2, f"worst tile rel-L2 {err.max().item():.3e} at tile {err.argmax().item()}"
    assert rel(s1.view(4, Co).sum(0).cpu(), ref.sum((0, 1, 2)).double().cpu()) < 1e-4
    assert rel(s2.view(4, Co).sum(0).cpu(), (ref.double() ** 2).sum((0, 1, 2)).cpu()) < 1e-4


@pytest.mark.parametrize("N,H,W,C", [(3, 5, 128, 64), (2, 128, 128, 64), (300, 4, 128, 64)])
def test_conv_fwd_act_matches_pass_then_conv(ops, N, H, W, C):
    """vlp_conv_fwd_act (bn1 + ReLU applied once per input row in the layer-1 rows
    kernel's ring, W = 128) against the separate bn_add_relu pass + conv_fwd: a1 and
    y bit-identical, BN sums equal up to fp64 atomic order; N = 300 > CUs puts two
    images on some workgroups.  Layers 2-4 are refused (the r6 in-window transform
    measured slower than the pass and was removed)."""
    torch.manual_seed(11)
    dev = torch.device("cuda")
    y1 = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    sc = (torch.rand(C, device=dev) + 0.5) * torch.where(torch.arange(C, device=dev) % 5 == 0, -1.0, 1.0)
    sh = torch.randn(C, device=dev) * 0.3
    w = (torch.randn(C, C, 3, 3) * (9 * C) ** -0.5).to(torch.bfloat16).float()
    wp = torch.empty(C, 3, 3, C, dtype=torch.bfloat16, device=dev)
    ops.pack_conv(w.cuda(), wp, None)
    assert ops.conv_fwd_act_ok(y1, C, 3, 3, 1, 1)
    for (w2, c2) in ((64, 128), (32, 256), (16, 512)):
        assert not ops.conv_fwd_act_ok(torch.empty(2, 16, w2, c2, dtype=torch.bfloat16, device=dev), c2, 3, 3, 1, 1)
    a_ref = torch.empty_like(y1)
    ops.bn_add_relu(y1, sc, sh, None, None, None, a_ref)
    r1, r2 = (torch.zeros(4 * C, dtype=torch.float64, device=dev) for _ in range(2))
    y_ref = ops.conv_fwd(a_ref, wp, C, 3, 3, 1, 1, stat_sum=r1, stat_sumsq=r2, stat_rep=4)
    a = torch.full_like(y1, float("nan"))
    t1, t2 = (torch.zeros(4 * C, dtype=torch.float64, device=dev) for _ in range(2))
    y = ops.conv_fwd_act(y1, wp, C, 3, 3, 1, 1, sc, sh, a, t1, t2, stat_rep=4)
    torch.cuda.synchronize()
    assert torch.equal(a, a_ref)
    assert torch.equal(y, y_ref)
    assert torch.allclose(t1.view(4, C).sum(0), r1.view(4, C).sum(0), rtol=1e-9, atol=1e-9)
    assert torch.allclose(t2.view(4, C).sum(0), r2.view(4, C).sum(0), rtol=1e-9, atol=1e-9)
    # against torch: conv2d(relu(bn(y1))) in fp32 on the bf16 activation
    xin = nchw(a_ref.float().cpu())
    ref = F.conv2d(xin, w, padding=1)
    assert rel(nchw(y.float().cpu()), ref) < tol(torch.bfloat16)
    # other shapes are refused, not silently rerouted
    assert not ops.conv_fwd_act_ok(y1[:, :, :W - 8].contiguous(), C, 3, 3, 1, 1)
    with pytest.raises(RuntimeError):
        ops.conv_fwd_act(y1[:, :, :W - 8].contiguous(), wp, C, 3, 3, 1, 1, sc, sh, a[:, :, :W - 8].contiguous(),
                         t1, t2, stat_rep=4)


@pytest.mark.parametrize("N,H", [(3, 5), (2, 128), (300, 4)])
@pytest.mark.parametrize("epi", ["bn", "relu_bits", "relu_act"])
def test_conv_dgrad_act_matches_pass_then_dgrad(ops, N, H, epi):
    """vlp_conv_dgrad_bn_act / vlp_conv_dgrad_relu_act (the BN backward apply of
    the input formed in the layer-1 rows kernel's ring) against the separate
    bn_bwd_apply pass + conv_dgrad / conv_dgrad_relu: dy and the output
    bit-identical, BN sums equal up to fp64 atomic order; N = 300 > CUs puts two
    images on some workgroups, H = 5 / 4 exercise the first-row and tail paths."""
    torch.manual_seed(12)
    C, W = 64, 128
    dev = torch.device("cuda")
    M = N * H * W
    bf = torch.bfloat16
    g_in = torch.randn(N, H, W, C, device=dev).to(bf)
    y_in = (torch.randn(N, H, W, C, device=dev) * 2 + 0.3).to(bf)
    mean = torch.randn(C, device=dev) * 0.2
    istd = torch.rand(C, device=dev) + 0.5
    gamma = torch.randn(C, device=dev)
    sg = (torch.randn(C, device=dev) * M * 0.01).double()
    sgx = (torch.randn(C, device=dev) * M * 0.01).double()
    w = (torch.randn(C, C, 3, 3) * (9 * C) ** -0.5).to(bf).float()
    wt = torch.empty(C, 3, 3, C, dtype=bf, device=dev)
    ops.pack_conv(w.cuda(), None, wt)
    assert ops.conv_dgrad_act_ok(g_in, C, 3, 3, 1, 1)
    dy_ref = torch.empty_like(g_in)
    ops.bn_bwd_apply(M, C, g_in, None, 1, None, (y_in, mean, istd, gamma, sg, sgx, dy_ref), None, None, g_in)
    coef = torch.empty(3 * C, device=dev)
    ops.bn_bwd_coef(M, gamma, istd, mean, sg, sgx, coef)
    r1, r2, t1, t2 = (torch.zeros(4 * C, dtype=torch.float64, device=dev) for _ in range(4))
    dy = torch.full_like(g_in, float("nan"))
    ye = torch.randn(N, H, W, C, device=dev).to(bf)             # epilogue operand (BN input of the output)
    mu_e, is_e = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5
    if epi == "bn":
        sc_e, sh_e = torch.randn(C, device=dev), torch.randn(C, device=dev) * 0.3
        out_ref = ops.conv_dgrad(dy_ref, wt, H, W, C, 3, 3, 1, 1, y_bn=ye, bn=(sc_e, sh_e, mu_e, is_e),
                                 stat1=r1, stat2=r2, stat_rep=4)
        out = ops.conv_dgrad_bn_act(g_in, y_in, coef, dy, wt, H, W, C, 3, 3, 1, 1, ye, (sc_e, sh_e, mu_e, is_e),
                                    t1, t2, stat_rep=4)
    else:
        act = torch.randn(N, H, W, C, device=dev).to(bf)
        if epi == "relu_bits":
            rm = torch.empty(M * C // 8, dtype=torch.uint8, device=dev)
            ops.bn_add_relu(act, torch.ones(C, device=dev), torch.zeros(C, device=dev), None, None, None,
                            torch.empty_like(act), relu_mask=rm)
            relu = rm
        else:
            relu = act
        addend = torch.randn(N, H, W, C, device=dev).to(bf)
        out_ref = ops.conv_dgrad_relu(dy_ref, wt, H, W, C, 3, 3, 1, 1, relu, ye, mu_e, is_e, r1, r2,
                                      addend=addend, stat_rep=4)
        out = ops.conv_dgrad_relu_act(g_in, y_in, coef, dy, wt, H, W, C, 3, 3, 1, 1, relu, ye, mu_e, is_e, t1, t2,
                                      addend=addend, stat_rep=4)
    torch.cuda.synchronize()
    assert torch.equal(dy, dy_ref)
    assert torch.equal(out, out_ref)
    assert torch.allclose(t1.view(4, C).sum(0), r1.view(4, C).sum(0), rtol=1e-9, atol=1e-9)
    assert torch.allclose(t2.view(4, C).sum(0), r2.view(4, C).sum(0), rtol=1e-9, atol=1e-9)
    # dy against the BN backward restated in torch (fp32 on the bf16 operands)
    k = gamma * istd
    mg, mgx = (sg / M).float(), (sgx / M).float()
    ref = k * (g_in.float() - mg - (y_in.float() - mean) * istd * mgx)
    assert rel(dy.float().cpu(), ref.cpu()) < 1e-2
    assert not ops.conv_dgrad_act_ok(g_in[:, :, :64].contiguous(), C, 3, 3, 1, 1)


@pytest.mark.parametrize("N,H,C", [(2, 64, 128), (4, 32, 256), (8, 16, 512), (3, 13, 128)])
def test_conv_dgrad_relu2_three_sums(ops, N, H, C):
    """vlp_conv_dgrad_relu2 (the block after a downsample): g = (dgrad + addend)
    masked by the previous block's output-ReLU bits, with three BN backward sums
    (against y2 and yd) in the epilogue, against conv_dgrad(addend) + the separate
    mask / bn_bwd_reduce pass: g bit-identical, sums equal up to summation order.
    The 128x128 (C = 128) and 256x256 ping-pong (C >= 256) tiles, an odd size."""
    torch.manual_seed(23)
    bf = torch.bfloat16
    dev = torch.device("cuda")
    M = N * H * H
    dy = torch.randn(N, H, H, C, device=dev).to(bf)
    w = (torch.randn(C, C, 3, 3) * (9 * C) ** -0.5).to(bf).float()
    wt = torch.empty(C, 3, 3, C, dtype=bf, device=dev)
    ops.pack_conv(w.cuda(), None, wt)
    addend = torch.randn(N, H, H, C, device=dev).to(bf)
    act = torch.randn(N, H, H, C, device=dev).to(bf)
    out_act = torch.empty_like(act)
    bits = torch.empty(M * C // 8, dtype=torch.uint8, device=dev)
    ops.bn_add_relu(act, torch.ones(C, device=dev), torch.zeros(C, device=dev), None, None, None, out_act,
                    relu_mask=bits)
    y2, yd = (torch.randn(N, H, H, C, device=dev) * 1.5 + 0.2).to(bf), torch.randn(N, H, H, C, device=dev).to(bf)
    mu2, is2 = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5
    mud, isd = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5
    t1, t2, t3 = (torch.zeros(4 * C, dtype=torch.float64, device=dev) for _ in range(3))
    g = ops.conv_dgrad_relu2(dy, wt, H, H, C, 3, 3, 1, 1, bits, y2, mu2, is2, yd, mud, isd, t1, t2, t3,
                             addend=addend, stat_rep=4)
    dx = ops.conv_dgrad(dy, wt, H, H, C, 3, 3, 1, 1, addend=addend)
    r1, r2, r3 = (torch.zeros(4 * C, dtype=torch.float64, device=dev) for _ in range(3))
    ops.bn_bwd_reduce(M, C, dx, None, 1, out_act, y2, mu2, is2, yd, mud, isd, r1, r2, r3, dx, stat_rep=4)
    torch.cuda.synchronize()
    g_ref = torch.where(out_act > 0, dx, torch.zeros_like(dx))
    assert torch.equal(g, g_ref)
    # the epilogue sums g in fp32 before its bf16 rounding, the pass sums the rounded
    # bf16 g: per channel a random walk of M rounding errors (~2^-9 |g| each)
    for t, r in ((t1, r1), (t2, r2), (t3, r3)):
        a, b = t.view(4, C).sum(0), r.view(4, C).sum(0)
        assert torch.allclose(a, b, rtol=0, atol=4e-3 * b.abs().max().item()), (a - b).abs().max()
    with pytest.raises(RuntimeError):   # C = 64 takes no row-chunk kernel: refused
        ops.conv_dgrad_relu2(dy[..., :64].contiguous(), wt, H, H, 64, 3, 3, 1, 1, bits, y2, mu2, is2, yd, mud, isd,
                             t1, t2, t3)


@pytest.mark.parametrize("N,Hi,C,Co", [(2, 64, 64, 128), (4, 32, 128, 256), (8, 16, 256, 512), (3, 14, 64, 128)])
def test_conv_dgrad_relu_ds_fold(ops, N, Hi, C, Co):
    """vlp_conv_dgrad_relu_ds: conv1 (3x3/2) data gradient with the downsample's
    1x1/2 data gradient folded into parity class (0, 0), against torch autograd of
    conv1(x) + downsample(x) in fp32 on the same bf16 operands, and against the
    unfused HIP path (downsample dgrad as the addend): the fold sums the two in
    fp32 inside one GEMM where the unfused path rounds the addend to bf16 first.
    Shapes: the 256x64 (C = 64), 128x128 (C = 128) and ping-pong 256x256
    (C = 256) class GEMMs, and an odd spatial size (14 -> 7)."""
    torch.manual_seed(21)
    bf = torch.bfloat16
    dev = torch.device("cuda")
    Ho = (Hi + 1) // 2
    x = torch.randn(N, C, Hi, Hi).to(bf).float().requires_grad_()
    w1 = (torch.randn(Co, C, 3, 3) * (9 * C) ** -0.5).to(bf).float()
    wd = (torch.randn(Co, C, 1, 1) * C ** -0.5).to(bf).float()
    y1 = F.conv2d(x, w1, stride=2, padding=1)
    yd = F.conv2d(x, wd, stride=2)
    dy = torch.randn_like(y1).to(bf).float()
    dyd = torch.randn_like(yd).to(bf).float()
    (y1 * dy + yd * dyd).sum().backward()
    buf = torch.empty(C * 9 * Co + C * Co, dtype=bf, device=dev)
    wt, wtd = buf[:C * 9 * Co].view(C, 3, 3, Co), buf[C * 9 * Co:].view(C, 1, 1, Co)
    ops.pack_conv(w1.cuda(), None, wt)
    ops.pack_conv(wd.cuda(), None, wtd)
    pair = torch.empty(2, N, Ho, Ho, Co, dtype=bf, device=dev)
    pair[0].copy_(nhwc(dy).to(bf))
    pair[1].copy_(nhwc(dyd).to(bf))
    act = torch.randn(N, Hi, Hi, C, device=dev).to(bf)            # block input (ReLU output stand-in)
    ye = torch.randn(N, Hi, Hi, C, device=dev).to(bf)
    mu, ist = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5
    s1, s2, r1, r2 = (torch.zeros(4 * C, dtype=torch.float64, device=dev) for _ in range(4))
    g = ops.conv_dgrad_relu_ds(pair[0], pair[1], wt, wtd, Hi, Hi, C, 3, 3, 2, 1, act, ye, mu, ist, s1, s2, stat_rep=4)
    add = ops.conv_dgrad(pair[1], wtd, Hi, Hi, C, 1, 1, 2, 0)
    g_ref = ops.conv_dgrad_relu(pair[0], wt, Hi, Hi, C, 3, 3, 2, 1, act, ye, mu, ist, r1, r2, addend=add, stat_rep=4)
    torch.cuda.synchronize()
    mask = (nchw(act.float().cpu()) > 0).float()
    ref = x.grad * mask
    got = nchw(g.float().cpu())
    assert rel(got, ref) < tol(bf), rel(got, ref)
    assert rel(got, nchw(g_ref.float().cpu())) < tol(bf)
    # BN backward sums of g against ye: both paths, and torch on the HIP output
    xh = (nchw(ye.float().cpu()) - mu.cpu()[None, :, None, None]) * ist.cpu()[None, :, None, None]
    assert rel(s1.view(4, C).sum(0).cpu(), got.sum((0, 2, 3)).double()) < 1e-4
    assert rel(s2.view(4, C).sum(0).cpu(), (got * xh).sum((0, 2, 3)).double()) < 1e-4
    # non-adjacent operands are refused
    with pytest.raises(RuntimeError):
        ops.conv_dgrad_relu_ds(pair[0], pair[0], wt, wtd, Hi, Hi, C, 3, 3, 2, 1, act, ye, mu, ist, s1, s2)


@pytest.mark.parametrize("N,H,C,epi", [(128, 32, 256, "bn"), (139, 31, 256, "relu"), (256, 16, 512, "bn"),
                                        (256, 16, 512, "relu")])
def test_conv_dgrad_bench_shapes(ops, N, H, C, epi):
    """Data gradients with a BN / ReLU epilogue at bench-sized layer-3/4 shapes
    (>= 2 rounds of the chip; the model tests' batches stay below that), one with a
    partial last tile (139 x 31 x 31). Against torch fp32 on the same bf16
    operands; three launches bit-identical."""
    torch.manual_seed(31)
    bf = torch.bfloat16
    dev = torch.device("cuda")
    dy = torch.randn(N, H, H, C, device=dev).to(bf)
    w = (torch.randn(C, C, 3, 3, device=dev) * (9 * C) ** -0.5).to(bf).float()
    wt = torch.empty(C, 3, 3, C, dtype=bf, device=dev)
    ops.pack_conv(w, None, wt)
    y = torch.randn(N, H, H, C, device=dev).to(bf)
    mu, ist = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5
    sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.2
    act = torch.relu(torch.randn(N, H, H, C, device=dev)).to(bf)
    add = torch.randn(N, H, H, C, device=dev).to(bf)
    ref = torch.nn.grad.conv2d_input((N, C, H, H), w, dy.permute(0, 3, 1, 2).float(), padding=1)
    ref = ref.permute(0, 2, 3, 1)
    if epi == "bn":
        mask = (y.float() * sc + sh) > 0
    else:
        ref = ref + add.float()
        mask = act > 0
    gref = torch.where(mask, ref.to(bf).float(), torch.zeros_like(ref))
    outs = []
    for _ in range(3):
        s1 = torch.zeros(C, dtype=torch.float64, device=dev)
        s2 = torch.zeros_like(s1)
        if epi == "bn":
            g = ops.conv_dgrad(dy, wt, H, H, C, 3, 3, 1, 1, y_bn=y, bn=(sc, sh, mu, ist), stat1=s1, stat2=s2)
        else:
            g = ops.conv_dgrad_relu(dy, wt, H, H, C, 3, 3, 1, 1, act, y, mu, ist, s1, s2, addend=add)
        outs.append((g.clone(), s1, s2))
    torch.cuda.synchronize()
    g0 = outs[0][0]
    assert rel(g0.float(), gref) < tol(bf), rel(g0.float(), gref)
    for o in outs[1:]:
        assert torch.equal(o[0], g0)
    xh = (y.float() - mu) * ist
    assert rel(outs[0][1], gref.sum((0, 1, 2))) < tol(bf)
    assert rel(outs[0][2], (gref * xh).sum((0, 1, 2))) < tol(bf)


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_dgrad_wgrad(ops, dt, case):
    N, H, W, C, Co, KH, KW, S, P = case
    torch.manual_seed(2)
    x = torch.randn(N, C, H, W).to(dt).float().requires_grad_()
    w = (torch.randn(Co, C, KH, KW) * (C * KH * KW) ** -0.5).to(dt).float().requires_grad_()
    y = F.conv2d(x, w, stride=S, padding=P)
    dy = torch.randn_like(y).to(dt).float()
    y.backward(dy)
    wt = torch.empty(C, KH, KW, Co, dtype=dt, device="cuda")
    ops.pack_conv(w.detach().cuda(), None, wt)
    add = torch.randn(N, C, H, W).to(dt).float()
    dx = ops.conv_dgrad(nhwc(dy).to(dt).cuda(), wt, H, W, C, KH, KW, S, P,
                        addend=nhwc(add).to(dt).cuda())
    ws = torch.zeros(Co, KH, KW, C, device="cuda")
    ops.conv_wgrad(nhwc(dy).to(dt).cuda(), nhwc(x.detach()).to(dt).cuda(), KH, KW, S, P, ws)
    g = torch.empty(Co, C, KH, KW, device="cuda")
    ops.unpack_conv_grad(ws, g)
    torch.cuda.synchronize()
    assert rel(nchw(dx.float().cpu()), x.grad + add) < tol(dt)
    assert rel(g.cpu(), w.grad) < tol(dt) / 2
    # split-K slabs + fold straight into the parameter layout (training path)
    g3 = torch.full((Co, C, KH, KW), float("nan"), device="cuda")
    ops.conv_wgrad_into(nhwc(dy).to(dt).cuda(), nhwc(x.detach()).to(dt).cuda(), KH, KW, S, P, g3)
    torch.cuda.synchronize()
    assert rel(g3.cpu(), w.grad) < tol(dt) / 2
    assert rel(g3.cpu(), g.cpu()) < 1e-5


@pytest.mark.parametrize("case", [(4, 64, 64, 64, 64, 3, 3, 1, 1), (8, 32, 32, 128, 128, 3, 3, 1, 1),
                                  (32, 32, 32, 64, 128, 1, 1, 2, 0), (32, 16, 16, 256, 256, 3, 3, 1, 1)])
@pytest.mark.parametrize("ws_floats", [None, "tight"])
def test_conv_wgrad_split_slabs(ops, case, ws_floats):
    """Deep pixel reductions (many K-splits, each its own fp32 slab) against
    torch's fp32 weight gradient; "tight" gives the workspace room for only 3
    slabs, so the split count must shrink to fit."""
    import ctypes
    from vlp_amd._lib import lib
    N, H, W, C, Co, KH, KW, S, P = case
    dt = torch.bfloat16
    torch.manual_seed(5)
    x = torch.randn(N, C, H, W).to(dt).float().requires_grad_()
    w = (torch.randn(Co, C, KH, KW) * (C * KH * KW) ** -0.5).requires_grad_()
    y = F.conv2d(x, w, stride=S, padding=P)
    dy = torch.randn_like(y).to(dt).float()
    y.backward(dy)
    slab = Co * C * KH * KW
    nws = 3 * slab if ws_floats == "tight" else 64 * slab
    ws = torch.full((nws + 64,), float("nan"), device="cuda")
    g = torch.full((Co, C, KH, KW), float("nan"), device="cuda")
    ns = ctypes.c_int(0)
    dyd, xd = nhwc(dy).to(dt).cuda(), nhwc(x.detach()).to(dt).cuda()
    lib().vlp_conv_wgrad_ws(1, dyd.data_ptr(), xd.data_ptr(), ws.data_ptr(), nws, ctypes.addressof(ns),
                            N, H, W, C, Co, KH, KW, S, P, torch.cuda.current_stream().cuda_stream)
    assert 1 <= ns.value <= nws // slab
    if ws_floats is None:
        assert ns.value > 1, "deep reduction expected to split"
    lib().vlp_conv_wgrad_fold(Co, C, KH, KW, ns.value, ws.data_ptr(), g.data_ptr(),
                              torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.isnan(ws[nws:]).all().item(), "slab writes past the workspace"
    assert rel(g.cpu(), w.grad) < 2e-3


@pytest.mark.parametrize("N,H,slabs", [(3, 5, None), (2, 1, None), (5, 9, 2), (4, 32, None), (1, 128, None)])
def test_conv_wgrad_rows_layer1(ops, N, H, slabs):
    """Layer-1 weight gradient (3x3, 64 -> 64, W = 128) on the row-streaming
    kernel: one fp32 slab per workgroup (a workgroup loops over several images
    when the workspace holds fewer slabs than images), folded into the parameter
    layout.  Against torch's fp32 weight gradient of the same bf16 operands, and
    bit-identical from run to run (fixed slab order)."""
    import ctypes
    from vlp_amd._lib import lib
    W, C = 128, 64
    dt = torch.bfloat16
    torch.manual_seed(11)
    x = torch.randn(N, C, H, W).to(dt).float().requires_grad_()
    w = (torch.randn(C, C, 3, 3) * (9 * C) ** -0.5).requires_grad_()
    y = F.conv2d(x, w, padding=1)
    dy = torch.randn_like(y).to(dt).float()
    y.backward(dy)
    slab = C * C * 9
    nws = (slabs or 64) * slab
    ws = torch.full((nws + 64,), float("nan"), device="cuda")
    dyd, xd = nhwc(dy).to(dt).cuda(), nhwc(x.detach()).to(dt).cuda()
    st = torch.cuda.current_stream().cuda_stream
    outs = []
    # the product gate takes the row-streaming form from 3/4 of the CU count in
    # images up (bs 256); force it for these small batches
    prev = ctypes.c_int(0)
    lib().vlp_set_wgrad_rows_min_images(1, ctypes.addressof(prev))
    try:
        for _ in range(2):
            g = torch.full((C, C, 3, 3), float("nan"), device="cuda")
            ns = ctypes.c_int(0)
            assert lib().vlp_conv_wgrad_ws(1, dyd.data_ptr(), xd.data_ptr(), ws.data_ptr(), nws,
                                           ctypes.addressof(ns), N, H, W, C, C, 3, 3, 1, 1, st) == 0
            assert ns.value == min(N, slabs or N), ns.value   # one slab per workgroup
            lib().vlp_conv_wgrad_fold(C, C, 3, 3, ns.value, ws.data_ptr(), g.data_ptr(), st)
            outs.append(g)
    finally:
        lib().vlp_set_wgrad_rows_min_images(prev.value, None)
    torch.cuda.synchronize()
    assert torch.isnan(ws[nws:]).all().item(), "slab writes past the workspace"
    assert torch.equal(outs[0], outs[1])
    err = (outs[0].cpu() - w.grad).abs().max().item() / w.grad.abs().max().item()
    assert err < 1e-5, err   # fp32 sums of exact bf16 products: only the summation order differs


def test_conv_wgrad_rows_gate_vs_gemm(ops):
    """The default gate: a batch of at least 3/4 of the CU count in images takes the
    row-streaming kernel (one slab per workgroup), a forced minimum above the batch
    takes the im2col GEMM; both fold to the same fp32 weight gradient."""
    import ctypes
    from vlp_amd._lib import lib
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    N, H, W, C = max(1, (3 * cus) // 4) + 3, 3, 128, 64
    torch.manual_seed(12)
    dyd = torch.randn(N, H, W, C, device="cuda").to(torch.bfloat16)
    xd = torch.randn(N, H, W, C, device="cuda").to(torch.bfloat16)
    slab = C * C * 9
    nws = 4 * N * slab
    ws = torch.empty(nws, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    res = {}
    for name, mn in (("rows", -1), ("gemm", 1 << 30)):
        prev = ctypes.c_int(0)
        lib().vlp_set_wgrad_rows_min_images(mn, ctypes.addressof(prev))
        try:
            g = torch.full((C, C, 3, 3), float("nan"), device="cuda")
            ns = ctypes.c_int(0)
            lib().vlp_conv_wgrad_ws(1, dyd.data_ptr(), xd.data_ptr(), ws.data_ptr(), nws, ctypes.addressof(ns),
                                    N, H, W, C, C, 3, 3, 1, 1, st)
            lib().vlp_conv_wgrad_fold(C, C, 3, 3, ns.value, ws.data_ptr(), g.data_ptr(), st)
            torch.cuda.synchronize()
            res[name] = (g.clone(), ns.value)
        finally:
            lib().vlp_set_wgrad_rows_min_images(prev.value, None)
    assert res["rows"][1] == min(N, cus), res["rows"][1]   # one slab per image workgroup
    a, b = res["rows"][0], res["gemm"][0]
    assert torch.isfinite(a).all() and torch.isfinite(b).all()
    assert (a - b).abs().max().item() <= 1e-5 * b.abs().max().item()


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("N,H,W,C", [(2, 10, 10, 64), (2, 4, 128, 64), (4, 7, 7, 512), (2, 14, 14, 256),
                                     (2, 8, 64, 128), (2, 16, 16, 512)])
def test_conv_dgrad_bn_epilogue(ops, dt, N, H, W, C):
    Co, KH, KW, S, P = C, 3, 3, 1, 1
    torch.manual_seed(3)
    dy = torch.randn(N, Co, H, W).to(dt).float()
    w = (torch.randn(Co, C, KH, KW) * 0.05).to(dt).float()
    ybn = torch.randn(N, C, H, W).to(dt).float()
    sc, sh = torch.rand(C) + 0.5, torch.randn(C) * 0.2
    mu, ist = torch.randn(C) * 0.1, torch.rand(C) + 0.5
    dxr = torch.nn.grad.conv2d_input(ybn.shape, w, dy, stride=S, padding=P)
    if dt == torch.bfloat16:
        dxr = dxr.to(dt).float()
    mask = (ybn * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1)) > 0
    gref = dxr * mask
    xh = (ybn - mu.view(1, -1, 1, 1)) * ist.view(1, -1, 1, 1)
    wt = torch.empty(C, KH, KW, Co, dtype=dt, device="cuda")
    ops.pack_conv(w.cuda(), None, wt)
    s1 = torch.zeros(C, dtype=torch.float64, device="cuda")
    s2 = torch.zeros_like(s1)
    g = ops.conv_dgrad(nhwc(dy).to(dt).cuda(), wt, H, W, C, KH, KW, S, P, y_bn=nhwc(ybn).to(dt).cuda(),
                       bn=(sc.cuda(), sh.cuda(), mu.cuda(), ist.cuda()), stat1=s1, stat2=s2)
    torch.cuda.synchronize()
    assert rel(nchw(g.float().cpu()), gref) < tol(dt)
    assert rel(s1.cpu(), gref.sum((0, 2, 3))) < tol(dt)
    assert rel(s2.cpu(), (gref * xh).sum((0, 2, 3))) < tol(dt)


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("case", [(2, 10, 10, 64, 64, 1), (2, 4, 128, 64, 64, 1), (2, 12, 12, 64, 128, 2),
                                  (4, 7, 7, 512, 512, 1), (4, 14, 14, 256, 512, 2), (2, 8, 64, 128, 128, 1),
                                  (2, 16, 32, 256, 256, 1)])
@pytest.mark.parametrize("with_add", [False, True])
@pytest.mark.parametrize("bits", [False, True])
def test_conv_dgrad_relu_epilogue(ops, dt, case, with_add, bits):
    """g = (dgrad + addend) * (relu_out > 0) and the next block's bn2 sums
    (vlp_conv_dgrad_relu, the fused replacement of the bn_bwd_reduce pass);
    bits: the ReLU sign as the uint8 bit mask vlp_bn_add_relu writes."""
    if bits and dt != torch.bfloat16:
        pytest.skip("bit masks are written by the bf16 producers only")
    N, H, W, C, Co, S = case
    torch.manual_seed(5)
    Ho, Wo = (H - 1) // S + 1, (W - 1) // S + 1
    dy = torch.randn(N, Co, Ho, Wo).to(dt).float()
    w = (torch.randn(Co, C, 3, 3) * 0.05).to(dt).float()
    relu_out = torch.relu(torch.randn(N, C, H, W)).to(dt).float()
    rarg = nhwc(relu_out).to(dt).cuda()
    if bits:
        # the producer: relu(1*x + 0) with its sign bits, bit e&7 of byte e>>3
        pre = nhwc(torch.randn(N, C, H, W)).to(dt).cuda()
        act = torch.empty_like(pre)
        rarg = torch.empty(pre.numel() // 8, dtype=torch.uint8, device="cuda")
        ops.bn_add_relu(pre, torch.ones(C, device="cuda"), torch.zeros(C, device="cuda"), None, None, None, act,
                        relu_mask=rarg)
        torch.cuda.synchronize()
        relu_out = nchw(act.float().cpu())
        bitref = ((act.view(-1, 8) > 0).to(torch.int32) << torch.arange(8, device="cuda")).sum(1)
        assert torch.equal(rarg.to(torch.int32), bitref)
    y2 = torch.randn(N, C, H, W).to(dt).float()
    add = torch.randn(N, C, H, W).to(dt).float() if with_add else None
    mu, ist = torch.randn(C) * 0.1, torch.rand(C) + 0.5
    dxr = torch.nn.grad.conv2d_input((N, C, H, W), w, dy, stride=S, padding=1)
    if add is not None:
        dxr = dxr + add
    if dt == torch.bfloat16:
        dxr = dxr.to(dt).float()
    gref = dxr * (relu_out > 0)
    xh = (y2 - mu.view(1, -1, 1, 1)) * ist.view(1, -1, 1, 1)
    wt = torch.empty(C, 3, 3, Co, dtype=dt, device="cuda")
    ops.pack_conv(w.cuda(), None, wt)
    s1 = torch.zeros(C, dtype=torch.float64, device="cuda")
    s2 = torch.zeros_like(s1)
    g = ops.conv_dgrad_relu(nhwc(dy).to(dt).cuda(), wt, H, W, C, 3, 3, S, 1, rarg,
                            nhwc(y2).to(dt).cuda(), mu.cuda(), ist.cuda(), s1, s2,
                            addend=None if add is None else nhwc(add).to(dt).cuda())
    torch.cuda.synchronize()
    assert rel(nchw(g.float().cpu()), gref) < tol(dt)
    assert rel(s1.cpu(), gref.sum((0, 2, 3))) < tol(dt)
    assert rel(s2.cpu(), (gref * xh).sum((0, 2, 3))) < tol(dt)


@pytest.mark.parametrize("dt", DT)
def test_stem_fwd_wgrad(ops, dt):
    N, H, W = 2, 32, 30
    torch.manual_seed(4)
    x = torch.randn(N, 3, H, W).to(dt).float()
    w = (torch.randn(64, 3, 7, 7) * 0.1).to(dt).float().requires_grad_()
    y = F.conv2d(x, w, stride=2, padding=3)
    dy = torch.randn_like(y).to(dt).float()
    y.backward(dy)
    Ho, Wo, Hp, Wp = ops.stem_geom(H, W)
    assert (Ho, Wo) == tuple(y.shape[2:])
    xp = torch.zeros(N, Hp, Wp, 4, dtype=dt, device="cuda")
    ops.stem_prep(x.cuda(), xp)
    wp = torch.empty(64, 256, dtype=dt, device="cuda")
    ops.pack_stem(w.detach().cuda(), wp)
    yd = torch.empty(N, Ho, Wo, 64, dtype=dt, device="cuda")
    s1 = torch.zeros(64, dtype=torch.float64, device="cuda")
    s2 = torch.zeros_like(s1)
    ops.stem_fwd(xp, wp, N, H, W, yd, s1, s2)
    ws = torch.zeros(64, 256, device="cuda")
    ops.stem_wgrad(nhwc(dy).to(dt).cuda(), xp, N, H, W, ws)
    g = torch.empty(64, 3, 7, 7, device="cuda")
    ops.unpack_stem_grad(ws, g)
    torch.cuda.synchronize()
    assert rel(nchw(yd.float().cpu()), y.detach()) < tol(dt)
    assert rel(g.cpu(), w.grad) < tol(dt) / 2
    g3 = torch.full((64, 3, 7, 7), float("nan"), device="cuda")   # split slabs + fold (training path)
    ops.stem_wgrad_into(nhwc(dy).to(dt).cuda(), xp, N, H, W, g3)
    torch.cuda.synchronize()
    assert rel(g3.cpu(), w.grad) < tol(dt) / 2


@pytest.mark.parametrize("has_b", [False, True])
@pytest.mark.parametrize("bcast", [False, True])
@pytest.mark.parametrize("C", [64, 128])
def test_bn_bwd_apply_formula(ops, has_b, bcast, C):
    """vlp_bn_bwd_apply against the BN backward in torch fp32:
    dy_s = gamma_s istd_s (g - sum_g / M - xhat_s sum_gx_s / M), g = dout masked by
    mask > 0 (or the broadcast pooled gradient dbc / HW), g_out = g."""
    torch.manual_seed(11)
    N, HW = 3, 40
    M = N * HW
    dt = torch.bfloat16
    dev = "cuda"
    dout = torch.randn(M, C, device=dev).to(dt)
    dbc = torch.randn(N, C, device=dev) if bcast else None
    mask = torch.randn(M, C, device=dev).to(dt)
    def side(seed):
        g = torch.Generator(device="cpu").manual_seed(seed)
        y = torch.randn(M, C, generator=g).to(dt).to(dev)
        mean = torch.randn(C, generator=g).to(dev) * 0.1
        istd = (torch.rand(C, generator=g) + 0.5).to(dev)
        gamma = torch.randn(C, generator=g).to(dev)
        sg = (torch.randn(C, generator=g) * M).double().to(dev)
        sgx = (torch.randn(C, generator=g) * M).double().to(dev)
        return [y, mean, istd, gamma, sg, sgx]
    A = side(1)
    B = side(2) if has_b else None
    dya = torch.empty(M, C, device=dev, dtype=dt)
    dyb = torch.empty(M, C, device=dev, dtype=dt) if has_b else None
    gout = torch.empty(M, C, device=dev, dtype=dt)
    ops.bn_bwd_apply(M, C, None if bcast else dout, dbc, HW, mask, A + [dya],
                     (B + [dyb]) if has_b else None, gout, dout)
    torch.cuda.synchronize()
    g = (dbc / HW).repeat_interleave(HW, 0) if bcast else dout.float()
    g = torch.where(mask.float() > 0, g, torch.zeros_like(g))
    assert rel(gout.float(), g.to(dt).float()) < 1e-6
    for sd, dy in ((A, dya), (B, dyb)):
        if sd is None:
            continue
        y, mean, istd, gamma, sg, sgx = sd
        xh = (y.float() - mean) * istd
        ref = gamma * istd * (g - sg.float() / M - xh * sgx.float() / M)
        assert rel(dy.float(), ref) < tol(dt), rel(dy.float(), ref)


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("shape", [(640, 936, 312), (300, 312, 1200), (1100, 312, 312),
                                   (16384, 384, 1152)])   # deep token reduction: ping-pong kernel (bf16)
def test_linear_wgrad(ops, dt, shape):
    """dW += dy^T x (TinyBERT weight gradients): fp32 atomic split-K and the bf16
    split-K workspace path (vlp_linear_wgrad_ws) against fp32 math."""
    M, Nout, Kin = shape
    torch.manual_seed(6)
    dy = torch.randn(M, Nout).to(dt).float()
    x = torch.randn(M, Kin).to(dt).float()
    ref = dy.t() @ x + 0.5
    dw = torch.full((Nout, Kin), 0.5, device="cuda")
    ops.linear_wgrad(dy.to(dt).cuda(), x.to(dt).cuda(), dw, M, Nout, Kin)
    torch.cuda.synchronize()
    assert rel(dw, ref) < tol(dt) / 4


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("M,N,K", [(512, 1152, 384), (300, 384, 1536)])
def test_linear_fwd_dgrad_large(ops, dt, M, N, K):
    """y = x W^T + b and dx = dy W at NesT level-2 sizes (M, N, K >= 256: the 256x256
    ping-pong kernel in bf16; M = 300 ends in a partial tile) against fp32 math."""
    torch.manual_seed(8)
    x = torch.randn(M, K).to(dt).float()
    w = (torch.randn(N, K) * K ** -0.5).to(dt).float()
    b = torch.randn(N)
    y = torch.empty(M, N, device="cuda", dtype=dt)
    ops.linear_fwd(x.to(dt).cuda(), w.to(dt).cuda(), b.cuda(), y, M, N, K)
    dy = torch.randn(M, N).to(dt).float()
    dx = torch.empty(M, K, device="cuda", dtype=dt)
    ops.linear_dgrad(dy.to(dt).cuda(), w.to(dt).cuda(), dx, M, K, N)
    torch.cuda.synchronize()
    assert rel(y.float().cpu(), x @ w.t() + b) < tol(dt) / 2
    assert rel(dx.float().cpu(), dy @ w) < tol(dt) / 2


@pytest.mark.parametrize("M,N,ld,off", [(10240, 312, 312, 0), (10240, 1200, 1200, 0), (777, 936, 944, 8),
                                        (300, 312, 320, 4), (5, 64, 64, 0)])
def test_colsum(ops, M, N, ld, off):
    """Bias-gradient column sums (fp32 atomics onto a pre-filled output):
    16-B vector path for aligned bf16 rows, scalar path otherwise (off=4)."""
    torch.manual_seed(9)
    buf = torch.randn(M * ld + off + 8).to(torch.bfloat16).cuda()
    x = buf[off:off + M * ld].view(M, ld)
    out = torch.full((N,), 0.5, device="cuda")
    ops.colsum(x, out, M, N, ld)
    torch.cuda.synchronize()
    ref = x[:, :N].float().sum(0) + 0.5
    assert (out - ref).abs().max().item() < 1e-3 * (1 + ref.abs().max().item())


@pytest.mark.parametrize("dt", DT)
def test_pack_conv_batch(ops, dt):
    """One-launch packing of many convs == per-conv vlp_pack_conv (bit-exact): the
    64 x 64 LDS-tile path (bf16, aligned, Co and C multiples of 64) and the
    element-per-thread path (fp32, an unaligned view, C = 96) in one call."""
    torch.manual_seed(10)
    shapes = [(64, 64, 3, 3), (128, 64, 1, 1), (256, 128, 3, 3), (512, 512, 3, 3), (128, 64, 3, 3)]
    entries, refs = [], []
    for Co, C, KH, KW in shapes:
        w = torch.randn(Co, C, KH, KW, device="cuda")
        wp = torch.empty(Co, KH, KW, C, dtype=dt, device="cuda")
        wt = torch.empty(C, KH, KW, Co, dtype=dt, device="cuda")
        rp, rt = torch.empty_like(wp), torch.empty_like(wt)
        ops.pack_conv(w, rp, rt)
        entries.append((w, wp, wt))
        refs.append((rp, rt))
    entries[1] = (entries[1][0], entries[1][1], None)   # wt optional
    # not 16-B aligned (a view at an odd float offset) and C % 64 != 0: the
    # element-per-thread path beside the 64 x 64 LDS-tile path in the same launch
    flat = torch.randn(1 + 128 * 64 * 9, device="cuda")
    wu = flat[1:].view(128, 64, 3, 3)
    w96 = torch.randn(64, 96, 3, 3, device="cuda")
    for w in (wu, w96):
        Co, C, KH, KW = w.shape
        wp = torch.empty(Co, KH, KW, C, dtype=dt, device="cuda")
        wt = torch.empty(C, KH, KW, Co, dtype=dt, device="cuda")
        rp, rt = torch.empty_like(wp), torch.empty_like(wt)
        ops.pack_conv(w, rp, rt)
        entries.append((w, wp, wt))
        refs.append((rp, rt))
    ops.pack_conv_batch_run(ops.pack_conv_batch(entries[0][1], entries))
    torch.cuda.synchronize()
    for i, ((w, wp, wt), (rp, rt)) in enumerate(zip(entries, refs)):
        assert torch.equal(wp, rp), i
        if wt is not None:
            assert torch.equal(wt, rt), i


@pytest.mark.parametrize("dt", DT)
def test_maxpool_fwd_argmax_value(ops, dt):
    """maxpool 3x3/2 over relu(sc*y+sh): pooled values, argmax taps and the
    pre-BN y at the argmax (yarg) against torch."""
    torch.manual_seed(11)
    N, H, W, C = 2, 15, 16, 64
    y = torch.randn(N, H, W, C).to(dt)
    sc, sh = torch.randn(C), torch.randn(C) * 0.5
    z = torch.relu(y.float() * sc + sh)
    ref, ridx = F.max_pool2d(nchw(z), 3, 2, 1, return_indices=True)
    Ho, Wo = ref.shape[2], ref.shape[3]
    out = torch.empty(N, Ho, Wo, C, dtype=dt, device="cuda")
    idx = torch.empty(N, Ho, Wo, C, dtype=torch.uint8, device="cuda")
    yarg = torch.empty_like(out)
    ops.maxpool_fwd(y.cuda(), sc.cuda(), sh.cuda(), out, idx, yarg)
    torch.cuda.synchronize()
    # (the kernel rounds sc*y+sh as one fma: compare within an ulp-scale tolerance)
    assert torch.allclose(nchw(out.float().cpu()), ref.to(dt).float(), rtol=1e-2 if dt == torch.bfloat16 else 1e-5,
                          atol=1e-6)
    # value of y at the recorded tap
    t = idx.long().cpu()
    ho = torch.arange(Ho).view(1, Ho, 1, 1) * 2 - 1 + t // 3
    wo = torch.arange(Wo).view(1, 1, Wo, 1) * 2 - 1 + t % 3
    n = torch.arange(N).view(N, 1, 1, 1).expand_as(t)
    c = torch.arange(C).view(1, 1, 1, C).expand_as(t)
    ok = (ho >= 0) & (ho < H) & (wo >= 0) & (wo < W)
    g = y[n, ho.clamp(0, H - 1), wo.clamp(0, W - 1), c]
    assert ok.all()
    assert torch.equal(yarg.cpu(), g)
    # the recorded tap holds the window maximum
    assert torch.allclose(z[n, ho, wo, c].to(dt).float(), out.float().cpu(),
                          rtol=1e-2 if dt == torch.bfloat16 else 1e-5, atol=1e-6)


@pytest.mark.parametrize("N,K", [(3000, 16), (37, 16), (1000, 1), (5, 16)])
def test_row_topk_vs_torch(ops, N, K):
    """vlp_row_topk (via ops.sim_topk's chunked fp32 similarity) against
    torch.topk of the full similarity matrix: values within fp32 rounding,
    indices exact (random data has no ties); rows shorter than K pad with -1."""
    torch.manual_seed(12)
    q = torch.nn.functional.normalize(torch.randn(257, 128, device="cuda"))
    k = torch.nn.functional.normalize(torch.randn(N, 128, device="cuda"))
    vals, idx = ops.sim_topk(q, k, K)
    kk = min(K, N)
    ref = (q @ k.T).topk(kk, dim=1)
    assert torch.equal(idx[:, :kk].cpu(), ref.indices.cpu())
    assert (vals[:, :kk] - ref.values).abs().max().item() < 1e-5
    if K > N:
        assert (idx[:, N:] == -1).all()


def test_retrieval_metrics_vs_oracle(ops):
    """Module precision@k / recall@k on the GPU path against the CPU oracle
    restatement (:364-439) and the reference-generated known answers."""
    import os
    from oracle.clip import precision_at_k, recall_at_k
    from src.models.pretrain.VisionLanguageModule import VisionLanguageModule
    ka = torch.load(os.path.join(os.path.dirname(__file__), "golden", "known_answers.pt"), weights_only=True)
    m = VisionLanguageModule.__new__(VisionLanguageModule)
    ks = [3, 5, 10, 15]
    p = VisionLanguageModule.precision_at_k_on_image_embeddings(m, ka["retr_img"].cuda(), ka["retr_lab"].cuda(), ks)
    r = VisionLanguageModule.recall_at_k_on_image_text_retreival(m, ka["retr_img"].cuda(), ka["retr_txt"].cuda(), ks)
    assert [p[k] for k in ks] == pytest.approx(ka["prec"].tolist(), abs=1e-7)
    assert [r[k] for k in ks] == pytest.approx(ka["recall"].tolist(), abs=1e-7)
    e = torch.tensor([[1, 1], [1, 1.1], [2, 1], [3, 1]], dtype=torch.float32).cuda()   # notebook cell 27
    assert VisionLanguageModule.precision_at_k_on_image_embeddings(m, e, torch.tensor([0, 0, 1, 1]).cuda(), [1]) == {1: 1.0}
    assert VisionLanguageModule.recall_at_k_on_image_text_retreival(m, e, e, [1, 2]) == {1: 1.0, 2: 1.0}
    torch.manual_seed(13)
    img, txt = torch.randn(4096, 128), torch.randn(4096, 128)
    txt = img + 3.0 * txt   # recall between 0 and 1
    lab = torch.randint(0, 7, (4096,))
    p = VisionLanguageModule.precision_at_k_on_image_embeddings(m, img.cuda(), lab.cuda(), ks)
    r = VisionLanguageModule.recall_at_k_on_image_text_retreival(m, img.cuda(), txt.cuda(), ks)
    po, ro = precision_at_k(img, lab, ks), recall_at_k(img, txt, ks)
    assert [p[k] for k in ks] == pytest.approx([po[k] for k in ks], abs=1e-6)
    assert [r[k] for k in ks] == pytest.approx([ro[k] for k in ks], abs=1e-6)
    assert 0.05 < r[3] < 0.95


def test_stem_wgrad_many_splits(ops):
    """Stem weight gradient over 32768 output pixels (16 K-splits of slabs)
    against torch's fp32 weight gradient."""
    N, H, W = 8, 128, 128
    torch.manual_seed(14)
    x = torch.randn(N, 3, H, W).to(torch.bfloat16).float()
    w = (torch.randn(64, 3, 7, 7) * 0.1).requires_grad_()
    y = F.conv2d(x, w, stride=2, padding=3)
    dy = torch.randn_like(y).to(torch.bfloat16).float()
    y.backward(dy)
    Ho, Wo, Hp, Wp = ops.stem_geom(H, W)
    xp = torch.zeros(N, Hp, Wp, 4, dtype=torch.bfloat16, device="cuda")
    ops.stem_prep(x.cuda(), xp)
    g = torch.full((64, 3, 7, 7), float("nan"), device="cuda")
    ops.stem_wgrad_into(nhwc(dy).to(torch.bfloat16).cuda(), xp, N, H, W, g)
    torch.cuda.synchronize()
    assert rel(g.cpu(), w.grad) < 2e-3


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("H,W", [(16, 32), (15, 16), (18, 18)])
def test_maxpool_bwd_sums_and_apply(ops, dt, H, W):
    """Stem backward: the pooled gradient routed to each window's recorded argmax,
    masked by the stem ReLU, its BN sums (sum g, sum g*xhat) and the folded BN
    backward dy = k*g + b*y + c, against torch.  Even H, W take the 2x2-block
    kernel, odd ones the per-pixel kernel."""
    torch.manual_seed(5)
    N, C = 3, 64
    y = torch.randn(N, H, W, C).to(dt)
    sc, sh = torch.rand(C) + 0.5, torch.randn(C) * 0.3
    mu, ist, gam = torch.randn(C) * 0.1, torch.rand(C) + 0.5, torch.rand(C) + 0.5
    z = torch.relu(y.float() * sc + sh)
    _, ridx = F.max_pool2d(nchw(z), 3, 2, 1, return_indices=True)
    Ho, Wo = ridx.shape[2], ridx.shape[3]
    out = torch.empty(N, Ho, Wo, C, dtype=dt, device="cuda")
    idx = torch.empty(N, Ho, Wo, C, dtype=torch.uint8, device="cuda")
    ops.maxpool_fwd(y.cuda(), sc.cuda(), sh.cuda(), out, idx)
    dp = torch.randn(N, Ho, Wo, C).to(dt)
    # torch routing from the kernel's own argmax taps
    t = idx.long().cpu()
    hh = torch.arange(Ho).view(1, Ho, 1, 1) * 2 - 1 + t // 3
    ww = torch.arange(Wo).view(1, 1, Wo, 1) * 2 - 1 + t % 3
    g = torch.zeros(N, H, W, C, dtype=torch.float64)
    n = torch.arange(N).view(N, 1, 1, 1).expand_as(t)
    c = torch.arange(C).view(1, 1, 1, C).expand_as(t)
    g.index_put_((n, hh, ww, c), dp.double(), accumulate=True)
    g = torch.where((y.float() * sc + sh) > 0, g, torch.zeros_like(g))
    xhat = (y.double() - mu.double()) * ist.double()
    rg, rgx = g.sum((0, 1, 2)), (g * xhat).sum((0, 1, 2))
    s1 = torch.zeros(C, dtype=torch.float64, device="cuda")
    s2 = torch.zeros_like(s1)
    ops.maxpool_bwd(dp.cuda(), idx, y.cuda(), sc.cuda(), sh.cuda(), mu.cuda(), ist.cuda(), s1, s2)
    torch.cuda.synchronize()
    assert torch.allclose(s1.cpu(), rg, rtol=1e-4, atol=1e-3)
    assert torch.allclose(s2.cpu(), rgx, rtol=1e-4, atol=1e-3)
    dy = torch.empty(N, H, W, C, dtype=dt, device="cuda")
    ops.maxpool_bwd_apply(dp.cuda(), idx, y.cuda(), sc.cuda(), sh.cuda(), mu.cuda(), ist.cuda(), gam.cuda(),
                          s1, s2, dy)
    torch.cuda.synchronize()
    cnt = N * H * W
    k = gam.double() * ist.double()
    ref = k * g - k * ist.double() * (rgx / cnt) * y.double() + (-k * rg / cnt + k * ist.double() * (rgx / cnt)
                                                                 * mu.double())
    tol = 2e-2 if dt == torch.bfloat16 else 1e-4
    assert torch.allclose(dy.double().cpu(), ref, rtol=tol, atol=tol * ref.abs().max().item())


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("N,H,W", [(2, 32, 32), (3, 48, 64), (8, 128, 128), (2, 224, 224)])
def test_stem1_single_channel_fwd_wgrad(ops, dt, N, H, W):
    """The single-channel stem of the uint8 upload (K = 64, channel-summed weights,
    4 shifted image copies) equals torch's 3-channel conv on the replicated
    normalised image, forward (+ BN sums) and the [64][3][7][7] weight gradient
    through the split slabs (N = 8, 128^2: 32768 output pixels, many splits)."""
    g = torch.Generator().manual_seed(H + N)
    mean, std = 127.5, 73.9
    x8 = torch.randint(0, 256, (N, 1, H, W), generator=g, dtype=torch.uint8)
    x = ((x8.float() - mean) / std).to(dt).float().repeat(1, 3, 1, 1)
    w = (torch.randn(64, 3, 7, 7, generator=g) * 0.1).requires_grad_()
    y = F.conv2d(x, w, stride=2, padding=3)
    dy = torch.randn(y.shape, generator=g).to(dt).float()
    y.backward(dy)
    Ho, Wo, Hp, Wp1 = ops.stem1_geom(H, W)
    assert (Ho, Wo) == tuple(y.shape[2:])
    xs = torch.full((4, N, Hp, Wp1), float("nan"), device="cuda").to(dt)   # the prep writes every element
    ops.stem1_prep_u8(x8.cuda(), xs, mean, std)
    wp1 = torch.empty(64, 64, dtype=dt, device="cuda")
    ops.pack_stem1(w.detach().cuda(), wp1)
    yd = torch.empty(N, Ho, Wo, 64, dtype=dt, device="cuda")
    s1 = torch.zeros(64, dtype=torch.float64, device="cuda")
    s2 = torch.zeros_like(s1)
    ops.stem1_fwd(xs, wp1, N, H, W, yd, s1, s2)
    gw = torch.full((64, 3, 7, 7), float("nan"), device="cuda")
    ops.stem1_wgrad_into(nhwc(dy).to(dt).cuda(), xs, N, H, W, gw)
    torch.cuda.synchronize()
    assert not torch.isnan(xs.float()).any()
    assert rel(nchw(yd.float().cpu()), y.detach()) < tol(dt)
    assert rel(s1.cpu(), y.detach().sum((0, 2, 3))) < tol(dt)
    assert rel(s2.cpu(), (y.detach() ** 2).sum((0, 2, 3))) < tol(dt)
    assert rel(gw.cpu(), w.grad) < tol(dt) / 2, rel(gw.cpu(), w.grad)
    assert torch.equal(gw[:, 0], gw[:, 1]) and torch.equal(gw[:, 0], gw[:, 2])


def test_stem1_geom_rejects_unaligned(ops):
    assert ops.stem1_geom(100, 100) is None        # Wo = 50: the 3-channel path takes it
    assert ops.stem1_geom(512, 512) == (256, 256, 518, 520)


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("N,H,C", [(256, 16, 512), (3, 7, 512), (2, 5, 64), (2, 4, 100)])
def test_avgpool_fwd_vs_torch(ops, dt, N, H, C):
    """vlp_avgpool_fwd (timm's global average pool before the head): the 16-B-row
    kernel (C % 8 == 0, one image per block, fixed-order partial sums) and the
    scalar fallback (C = 100), against torch fp32 on the same operands."""
    torch.manual_seed(41)
    x = torch.randn(N, H, H, C, device="cuda").to(dt)
    feat = torch.empty(N, C, dtype=dt, device="cuda")
    ops.avgpool_fwd(x, feat)
    torch.cuda.synchronize()
    ref = x.float().mean((1, 2))
    assert rel(feat.float(), ref.to(dt).float()) < (1e-6 if dt == torch.float32 else 8e-3)
    feat2 = torch.empty_like(feat)
    ops.avgpool_fwd(x, feat2)
    torch.cuda.synchronize()
    assert torch.equal(feat, feat2)


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("N,H,W", [(2, 32, 32), (3, 48, 64), (2, 224, 224), (1, 512, 512)])
def test_stem1_prep_u8_exact(ops, dt, N, H, W):
    """vlp_stem1_prep_u8 element by element: Xs[s][n][hp][j] = (x[n][hp-3][j+2s-3] - mean)
    * (1/std) rounded to the dtype, zero outside the image, for all four shifted copies
    (including the 512 x 512 bench image)."""
    g = torch.Generator().manual_seed(7 * H + N)
    mean, std = 127.5, 73.9
    x8 = torch.randint(0, 256, (N, 1, H, W), generator=g, dtype=torch.uint8)
    Ho, Wo, Hp, Wp1 = ops.stem1_geom(H, W)
    xs = torch.full((4, N, Hp, Wp1), float("nan"), device="cuda").to(dt)
    ops.stem1_prep_u8(x8.cuda(), xs, mean, std)
    torch.cuda.synchronize()
    inv = torch.tensor(1.0, dtype=torch.float32) / torch.tensor(std, dtype=torch.float32)   # the host's 1.f / std
    xn = (x8[:, 0].float() - mean) * inv
    ref = torch.zeros(4, N, Hp, Wp1)
    for s in range(4):
        j0 = 3 - 2 * s                                  # column j reads image column j + 2s - 3
        lo, hi = max(0, j0), min(Wp1, W + j0)
        hr = min(Hp - 3, H)
        ref[s, :, 3:3 + hr, lo:hi] = xn[:, :hr, lo - j0:hi - j0]
    assert torch.equal(xs.cpu(), ref.to(dt))

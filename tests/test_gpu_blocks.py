"""bf16 BasicBlock ranges at the bench's shapes (bs = 256, 512 x 512 input) against
torch fp64.

Reference: timm resnet34 BasicBlock behind src/models/pretrain/VisionLanguageModule.py:30-32,
trained by training_step (:634-645).  Each case runs a range of consecutive blocks
through the HIP tower (ResNet34Tower.run_block_range_forward / _backward: the same
kernels, tile choices and fusions the whole-tower step takes at these shapes) on a
ReLU-output input with a dense random upstream gradient, every BatchNorm live
(gamma ~ U(0.3, 1), beta ~ U(-0.1, 0.1)):

  layer1  blocks layer1.0-1.2: the W = 128 rows kernels -- bn1 + ReLU applied in
          conv2's ring (vlp_conv_fwd_act), both BN backward applies in the data-
          gradient rings (vlp_conv_dgrad_bn_act / _relu_act), ReLU-bit epilogues
  layer2  layer1.2, layer2.0-2.3: the stride-2 entry block with the downsample's data
          gradient folded into conv1's parity class (vlp_conv_dgrad_relu_ds), the
          block after it with the three-sum epilogue (vlp_conv_dgrad_relu2), the
          128-channel tiles
  layer3  layer2.3, layer3.0-3.2: the 256 x 256 ping-pong GEMMs
  layer4  layer3.5, layer4.0-4.2

Two checks per range, every number printed.

1. Stage by stage (the sharp gate).  Every tensor the HIP range stores --
   forward y1, relu(bn1(y1)), y2, yd, out; backward the gradient reaching each
   block (masked by the epilogue that produced it), dy2, dyd, g1, dy1, the input
   gradient, and every conv-weight and BN-parameter gradient -- is recomputed in
   float64 from HIP's OWN stored inputs of that stage (torch autograd ops / the BN
   backward formula; convolutions through torch's im2col + GEMM path, as MIOpen has
   no fp64 kernels) and rounded to bf16 where HIP stores bf16 -- including the data-
   gradient epilogues' order: the GEMM tile staged as bf16, then the residual added,
   masked and summed for the block below in fp32, then stored.  So each line judges
   one kernel in its real place in the fused chain, at the bench's tile and split
   choices.  Gate: rel-L2 <= 2e-3 for stored bf16 tensors (bf16 is 2^-9 relative;
   an fp32 sum landing next to a rounding tie flips one ulp; measured <= 2e-4),
   <= 1e-3 for the fp32 parameter gradients (measured <= 2e-5).  A wrong mask,
   epilogue, fold or split fails by orders of magnitude.

2. End to end.  The range's output, input gradient and parameter gradients
   against plain fp64 autograd, next to an exact bf16-storage emulation (fp64 with
   a bf16 rounding at each tensor HIP stores).  Through a chain of ReLUs a bf16
   rounding of a pre-activation next to zero flips its mask, and the gradient error
   grows like the square root of the flip rate: two exact bf16 implementations that
   differ only in fp32 summation order land ~10 % apart in gradient (stage-wise each
   is exact, check 1).  Gate: rel-L2(HIP, fp64) <= 1.25 x rel-L2(emul, fp64) +
   1e-2, i.e. HIP is as accurate as exact bf16 storage (and <= 2e-2, the VERDICT's
   bar, wherever the emulation itself is within 1.5e-2); every gradient non-zero,
   finite and cos(HIP, fp64) >= 0.95.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

BS = 256
# (lo, hi) block indices of ResNet34Tower._blocks and the input [H, W, C]
RANGES = {
    "layer1": (0, 3, (128, 128, 64)),
    "layer2": (2, 7, (128, 128, 64)),
    "layer3": (6, 10, (64, 64, 128)),
    "layer4": (12, 16, (32, 32, 256)),
}
F64 = torch.float64


class _Rb(torch.autograd.Function):
    """bf16 storage point: round the value forward and the gradient backward."""

    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).to(g.dtype)


def rb(t):
    return t.to(torch.bfloat16).to(F64)


def rel(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def cos(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return (a @ b / (a.norm() * b.norm() + 1e-30)).item()


def nchw(t):
    return t.permute(0, 3, 1, 2).to(F64)


def block_torch(x, P, pre, stride, has_ds, emul):
    r = _Rb.apply if emul else (lambda t: t)

    def bn(t, k):
        return F.batch_norm(t, None, None, P[k + ".weight"], P[k + ".bias"], True, 0.1, 1e-5)

    y1 = r(F.conv2d(x, P[pre + ".conv1.weight"], stride=stride, padding=1))
    a1 = r(F.relu(bn(y1, pre + ".bn1")))
    y2 = r(F.conv2d(a1, P[pre + ".conv2.weight"], padding=1))
    z = bn(y2, pre + ".bn2")
    if has_ds:
        sc = bn(r(F.conv2d(x, P[pre + ".downsample.0.weight"], stride=stride)), pre + ".downsample.1")
    else:
        sc = x
    return r(F.relu(z + sc))


def run_torch(x, dout, params, blocks, emul):
    P = {k: v.clone().requires_grad_() for k, v in params.items()}
    xi = x.clone().requires_grad_()
    h = xi
    for pre, stride, has_ds in blocks:
        h = block_torch(h, P, pre, stride, has_ds, emul)
    h.backward(dout)
    out = {"out": h.detach().float(), "dx": xi.grad.float()}
    out.update({k: P[k].grad.float() for k in P})
    return out


def bn_fwd(y, gamma, beta):
    """(xhat, istd, out) of train-mode BN over (N, H, W) of an NCHW fp64 tensor."""
    mu = y.mean((0, 2, 3), keepdim=True)
    var = y.var((0, 2, 3), unbiased=False, keepdim=True)
    istd = (var + 1e-5).rsqrt()
    xh = (y - mu) * istd
    return xh, istd, xh * gamma.view(1, -1, 1, 1) + beta.view(1, -1, 1, 1)


def bn_bwd(g, xh, istd, gamma):
    """(dy, dgamma, dbeta) of train-mode BN for the output gradient g."""
    M = g.numel() // g.shape[1]
    db = g.sum((0, 2, 3))
    dg = (g * xh).sum((0, 2, 3))
    dy = gamma.view(1, -1, 1, 1) * istd * (g - db.view(1, -1, 1, 1) / M - xh * dg.view(1, -1, 1, 1) / M)
    return dy, dg, db


def stagewise(tower, saved, dbg, dx_hip, dout, P, blocks, lo):
    """[(stage name, rel-L2, gate)] for every stored tensor and gradient of the range,
    each recomputed in fp64 from HIP's own stored inputs of that stage.

    The data-gradient epilogues stage the fp32 GEMM tile in LDS as bf16 and then
    add the residual addend, apply the ReLU mask and take the BatchNorm sums of the
    block below in fp32 before the final bf16 store: the references follow that
    order (rb(rb(dgrad) + addend) stored, the sums over rb(dgrad) + addend)."""
    rows = []
    dev = dx_hip.device
    Pd = {k: v.to(dev, F64) for k, v in P.items()}
    blk = saved["blocks"]

    def add(name, got, ref, gate):
        rows.append((name, rel(got, ref), gate))

    g_pre = None   # fp64 gradient of the current block's output as the epilogue above summed it
    for i in range(len(blocks) - 1, -1, -1):
        pre, stride, has_ds = blocks[i]
        B = blk[lo + i]
        xin = nchw(B["x"])
        y1, a1, y2, out = nchw(B["y1"]), nchw(B["a1"]), nchw(B["y2"]), nchw(B["out"])
        w1, w2 = Pd[pre + ".conv1.weight"], Pd[pre + ".conv2.weight"]
        g1w, b1w = Pd[pre + ".bn1.weight"], Pd[pre + ".bn1.bias"]
        g2w, b2w = Pd[pre + ".bn2.weight"], Pd[pre + ".bn2.bias"]
        # forward
        add(f"{pre} y1", y1, rb(F.conv2d(xin, w1, stride=stride, padding=1)), 2e-3)
        xh1, is1, z1 = bn_fwd(y1, g1w, b1w)
        add(f"{pre} a1", a1, rb(F.relu(z1)), 2e-3)
        add(f"{pre} y2", y2, rb(F.conv2d(a1, w2, padding=1)), 2e-3)
        xh2, is2, z2 = bn_fwd(y2, g2w, b2w)
        if has_ds:
            wd = Pd[pre + ".downsample.0.weight"]
            yd = nchw(B["yd"])
            add(f"{pre} yd", yd, rb(F.conv2d(xin, wd, stride=stride)), 2e-3)
            xhd, isd, zd = bn_fwd(yd, Pd[pre + ".downsample.1.weight"], Pd[pre + ".downsample.1.bias"])
            sc = zd
        else:
            sc = xin
        add(f"{pre} out", out, rb(F.relu(z2 + sc)), 2e-3)
        # backward: g = the stored (bf16) gradient of this block's output after its
        # ReLU; gs = what the BN sums were taken over
        d, masked = dbg[pre]
        g = nchw(d) if masked else torch.where(out > 0, nchw(d), torch.zeros_like(out))
        gs = g_pre if g_pre is not None else g

        def bn_b(xh, istd, gamma):
            M = g.numel() // g.shape[1]
            db, dg = gs.sum((0, 2, 3)), (gs * xh).sum((0, 2, 3))
            dy = gamma.view(1, -1, 1, 1) * istd * (g - db.view(1, -1, 1, 1) / M - xh * dg.view(1, -1, 1, 1) / M)
            return dy, dg, db

        dy2_ref, dg2, db2 = bn_b(xh2, is2, g2w)
        dy2 = nchw(dbg[pre + "/dy2"][0])
        add(f"{pre} dy2", dy2, rb(dy2_ref), 2e-3)
        add(f"{pre} d bn2.weight", tower.arena.gview(pre + ".bn2.weight"), dg2, 1e-3)
        add(f"{pre} d bn2.bias", tower.arena.gview(pre + ".bn2.bias"), db2, 1e-3)
        if has_ds:
            dyd_ref, dgd, dbd = bn_b(xhd, isd, Pd[pre + ".downsample.1.weight"])
            dyd = nchw(dbg[pre + "/dyd"][0])
            add(f"{pre} dyd", dyd, rb(dyd_ref), 2e-3)
            add(f"{pre} d downsample.1.weight", tower.arena.gview(pre + ".downsample.1.weight"), dgd, 1e-3)
            add(f"{pre} d downsample.1.bias", tower.arena.gview(pre + ".downsample.1.bias"), dbd, 1e-3)
            add(f"{pre} d downsample.0.weight", tower.arena.gview(pre + ".downsample.0.weight"),
                torch.nn.grad.conv2d_weight(xin, wd.shape, dyd, stride=stride), 1e-3)
        g1_ref = torch.nn.grad.conv2d_input(a1.shape, w2, dy2, padding=1)
        g1_ref = torch.where(a1 > 0, g1_ref, torch.zeros_like(g1_ref))
        g1 = nchw(dbg[pre + "/g1"][0])
        add(f"{pre} g1", g1, rb(g1_ref), 2e-3)
        add(f"{pre} d conv2.weight", tower.arena.gview(pre + ".conv2.weight"),
            torch.nn.grad.conv2d_weight(a1, w2.shape, dy2, padding=1), 1e-3)
        dy1_ref, dg1, db1 = bn_bwd(g1, xh1, is1, g1w)   # BN1 sums: the conv2 epilogue's own (exact) g1
        dy1 = nchw(dbg[pre + "/dy1"][0])
        add(f"{pre} dy1", dy1, rb(dy1_ref), 2e-3)
        add(f"{pre} d bn1.weight", tower.arena.gview(pre + ".bn1.weight"), dg1, 1e-3)
        add(f"{pre} d bn1.bias", tower.arena.gview(pre + ".bn1.bias"), db1, 1e-3)
        add(f"{pre} d conv1.weight", tower.arena.gview(pre + ".conv1.weight"),
            torch.nn.grad.conv2d_weight(xin, w1.shape, dy1, stride=stride, padding=1), 1e-3)
        # input gradient as the epilogue forms it
        dg = torch.nn.grad.conv2d_input(xin.shape, w1, dy1, stride=stride, padding=1)
        if has_ds and i > 0:     # downsample folded into conv1's class GEMM (vlp_conv_dgrad_relu_ds)
            v = rb(dg + torch.nn.grad.conv2d_input(xin.shape, wd, dyd, stride=stride))
        elif has_ds:             # separate downsample data gradient, stored bf16, as the addend
            v = rb(dg) + rb(torch.nn.grad.conv2d_input(xin.shape, wd, dyd, stride=stride))
        else:                    # identity branch: the stored g is the addend
            v = rb(dg) + g
        if i > 0:   # the block below receives it through this epilogue (its ReLU, its BN sums)
            dlow, mlow = dbg[blocks[i - 1][0]]
            g_pre = torch.where(xin > 0, v, torch.zeros_like(v)) if mlow else None
            add(f"{pre} dx", nchw(dlow), rb(g_pre if mlow else v), 2e-3)
        else:
            add(f"{pre} dx (range input)", nchw(dx_hip), rb(v), 2e-3)
    return rows


@pytest.fixture(scope="module")
def tower():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vlp_amd.resnet34 import ResNet34Tower
    return ResNet34Tower(compute_dtype="bf16", device="cuda")


@pytest.mark.parametrize("name", list(RANGES))
def test_block_range_bf16_vs_torch_fp64(tower, name):
    lo, hi, (H, W, C) = RANGES[name]
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(500 + lo)
    blocks = []
    params = {}
    for bi in range(lo, hi):
        pre, has_ds = tower._blocks[bi]
        c1 = tower._convs[pre + ".conv1"]
        blocks.append((pre, c1.S, has_ds))
        for k in [pre + ".conv1", pre + ".conv2"] + ([pre + ".downsample.0"] if has_ds else []):
            c = tower._convs[k]
            std = (2.0 / (c.Co * c.KH * c.KW)) ** 0.5   # kaiming fan_out
            params[k + ".weight"] = (torch.randn(c.Co, c.C, c.KH, c.KW, generator=g) * std).to(torch.bfloat16).float()
        for k in [pre + ".bn1", pre + ".bn2"] + ([pre + ".downsample.1"] if has_ds else []):
            Cb = tower._bns[k].C
            params[k + ".weight"] = torch.empty(Cb).uniform_(0.3, 1.0, generator=g)
            params[k + ".bias"] = torch.empty(Cb).uniform_(-0.1, 0.1, generator=g)
    with torch.no_grad():
        for k, v in params.items():
            tower.arena.view(k).copy_(v)
    x = torch.relu(torch.randn(BS, C, H, W, generator=g)).to(torch.bfloat16)

    # HIP bf16 range, every stored tensor and backward intermediate kept
    out_h, saved = tower.run_block_range_forward(x.permute(0, 2, 3, 1).contiguous().to(dev), lo, hi)
    Ho, Wo, Co = out_h.shape[1:]
    dout = torch.randn(BS, Co, Ho, Wo, generator=g).to(torch.bfloat16)
    tower.arena.grad.fill_(float("nan"))   # every gradient of the range must be written
    tower._dbg = {}
    try:
        dx_h = tower.run_block_range_backward(saved, dout.permute(0, 2, 3, 1).contiguous().to(dev))
        torch.cuda.synchronize()
        dbg = tower._dbg
    finally:
        tower._dbg = None
    hip = {"out": out_h.permute(0, 3, 1, 2).float(), "dx": dx_h.permute(0, 3, 1, 2).float()}
    for k in params:
        hip[k] = tower.arena.gview(k).clone()

    fails = []
    # 1. stage by stage from HIP's own stored inputs
    rows = stagewise(tower, saved, dbg, dx_h, dout, params, blocks, lo)
    print(f"\n{name} blocks {lo}..{hi - 1} bs={BS}, stage-wise vs fp64 from HIP's stored inputs (rel-L2):")
    for k, r, gate in rows:
        print(f"  {k:40s} {r:.2e}{'   <-- over ' + format(gate, '.0e') if r > gate else ''}")
        if not r <= gate:
            fails.append((k, r, gate))
    del saved, dbg, out_h, dx_h
    torch.cuda.empty_cache()

    # 2. end to end against fp64, next to the exact bf16-storage emulation
    def refs(dt, emul):
        pd = {k: v.to(dev, dt) for k, v in params.items()}
        return run_torch(x.to(dev, dt), dout.to(dev, dt), pd, blocks, emul=emul)

    ref = refs(F64, False)
    emu = refs(F64, True)
    torch.cuda.synchronize()
    print(f"{name} end to end: tensor  rel(hip,fp64)  rel(emul,fp64)  cos(hip,fp64)  bar")
    for k in ["out", "dx"] + list(params):
        h, e, f = hip[k], emu[k], ref[k]
        r_hf, r_ef, c_hf = rel(h, f), rel(e, f), cos(h, f)
        bar = 2e-2 if r_ef <= 1.5e-2 else 1.25 * r_ef + 1e-2
        print(f"  {k:34s} {r_hf:.2e}  {r_ef:.2e}  {c_hf:.5f}  {bar:.2e}")
        if not torch.isfinite(h).all():
            fails.append((k, "non-finite"))
            continue
        if k != "out" and h.norm() == 0:
            fails.append((k, "zero gradient"))
        if r_hf > bar or c_hf < 0.95:
            fails.append((k, "end to end", r_hf, bar, c_hf))
    assert not fails, fails

"""TinyBERT text-tower kernels vs the HF BertModel sub-modules they replace
(transformers BertModel with the TinyBERT-4L-312D config, the reference's text
encoder: VisionLanguageModule.py:45, :57-60), at the reference's caption length
T = 40 with padding masks (PretrainDataModule.py:210-215), plus T = 12 and
T = 64 (the kernel's two token-tile sizes).

  attention  vlp_attn_fwd / vlp_attn_bwd (one wave per (sequence, head), QK^T,
             softmax and PV on MFMA) vs HF BertSelfAttention's context (captured
             from a 1-layer BertModel, extended mask finfo.min) and torch autograd
  LayerNorm  vlp_layernorm_fwd / _bwd vs nn.LayerNorm(312, eps=1e-12)
  embeddings vlp_embed_fwd (+ LayerNorm) / vlp_embed_bwd vs HF BertEmbeddings

Tolerances: fp32 storage rel-L2 <= 2e-5 (attention backward 5e-5); bf16
storage vs fp32 math on the same bf16-rounded inputs <= 2e-2.
"""
import math

import pytest
import torch

DT = [torch.float32, torch.bfloat16]
H, DH, D = 12, 26, 312


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def tol(dt, fp32=2e-5):
    return fp32 if dt == torch.float32 else 2e-2


@pytest.fixture(scope="module")
def ops():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vlp_amd import ops as o
    return o


def masks(B, T, g):
    """attention_mask rows with 1 + L ~ U{8..T-2} + 1 valid tokens (CLS ... SEP)."""
    am = torch.zeros(B, T, dtype=torch.long)
    for b in range(B):
        L = int(torch.randint(min(8, T - 2), T - 1, (1,), generator=g))
        am[b, :L + 2] = 1
    am[0, :] = 1   # one full-length caption
    return am


def ref_attention(qkv, am, T, scale):
    """HF eager BertSelfAttention math on projected q|k|v rows [B*T, 3*D]."""
    B = qkv.shape[0] // T
    q, k, v = qkv.view(B, T, 3, H, DH).permute(2, 0, 3, 1, 4)       # [B, H, T, dh] each
    s = q @ k.transpose(-1, -2) * scale
    s = s + (1.0 - am[:, None, None, :].to(s.dtype)) * torch.finfo(s.dtype).min
    p = torch.softmax(s, dim=-1)
    ctx = (p @ v).permute(0, 2, 1, 3).reshape(B * T, D)
    return ctx, p


def test_reference_attention_is_hf_self_attention():
    """CPU: the torch restatement above equals HF BertSelfAttention's output (a
    1-layer BertModel, forward hooks on embeddings and attention.self)."""
    import oracle.clip as oc
    cfg = oc.tinybert_config(0.0)
    cfg.num_hidden_layers = 1
    from transformers import BertModel
    torch.manual_seed(0)
    m = BertModel(cfg, add_pooling_layer=False).eval()
    B, T = 4, 40
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(1000, 30000, (B, T), generator=g)
    am = masks(B, T, g)
    cap = {}
    m.embeddings.register_forward_hook(lambda mod, i, o: cap.__setitem__("h", o))
    m.encoder.layer[0].attention.self.register_forward_hook(
        lambda mod, i, o: cap.__setitem__("ctx", o[0] if isinstance(o, tuple) else o))
    with torch.no_grad():
        m(input_ids=ids, attention_mask=am)
    sa = m.encoder.layer[0].attention.self
    h = cap["h"].reshape(B * T, D)
    qkv = torch.cat([h @ sa.query.weight.T + sa.query.bias, h @ sa.key.weight.T + sa.key.bias,
                     h @ sa.value.weight.T + sa.value.bias], 1)
    ctx, _ = ref_attention(qkv, am, T, 1 / math.sqrt(DH))
    assert rel(ctx, cap["ctx"].reshape(B * T, D)) < 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("B,T", [(6, 40), (3, 12), (2, 64)])
def test_attention_fwd_bwd(ops, dt, B, T):
    g = torch.Generator().manual_seed(T)
    am = masks(B, T, g)
    qkv = torch.randn(B * T, 3 * D, generator=g).to(dt).float()
    dctx = torch.randn(B * T, D, generator=g).to(dt).float()
    scale = 1 / math.sqrt(DH)
    x = qkv.clone().double().requires_grad_()
    ctx_ref, p_ref = ref_attention(x, am, T, scale)
    ctx_ref.backward(dctx.double())
    qd, amd = qkv.to(dt).cuda(), am.cuda()
    ctx = torch.empty(B * T, D, dtype=dt, device="cuda")
    P = torch.empty(B, H, T, T, device="cuda")
    ops.attn_fwd(qd, amd, ctx, P, B, T, H, DH, scale)
    dq = torch.empty_like(qd)
    ops.attn_bwd(qd, P, dctx.to(dt).cuda(), dq, B, T, H, DH, scale)
    torch.cuda.synchronize()
    assert rel(P, p_ref) < 2e-5 if dt == torch.float32 else rel(P, p_ref) < 2e-2
    assert rel(ctx.float(), ctx_ref) < tol(dt)
    # padded (masked) keys get exactly zero probability
    pm = P.cpu()[am[:, None, None, :].expand(B, H, T, T) == 0]
    assert pm.abs().max().item() < 1e-30 if pm.numel() else True
    assert rel(dq.float(), x.grad) < tol(dt, 5e-5), rel(dq.float(), x.grad)


@pytest.mark.gpu
def test_attention_rejects_oversize(ops):
    from vlp_amd._lib import lib
    qkv = torch.zeros(65 * 3 * D, device="cuda")
    with pytest.raises(RuntimeError):
        ops.attn_fwd(qkv, None, torch.empty(65 * D, device="cuda"), torch.empty(H * 65 * 65, device="cuda"),
                     1, 65, H, DH, 0.2)
    assert lib() is not None


@pytest.mark.gpu
@pytest.mark.parametrize("dt", DT)
def test_layernorm_fwd_bwd(ops, dt):
    M = 6 * 40
    g = torch.Generator().manual_seed(3)
    x = (torch.randn(M, D, generator=g) * 3 + 1).to(dt).float()
    dy = torch.randn(M, D, generator=g).to(dt).float()
    ln = torch.nn.LayerNorm(D, eps=1e-12)           # BertSelfOutput / BertOutput / BertEmbeddings LayerNorm
    with torch.no_grad():
        ln.weight.copy_(torch.rand(D, generator=g) + 0.5)
        ln.bias.copy_(torch.randn(D, generator=g) * 0.1)
    xr = x.clone().requires_grad_()
    y_ref = ln(xr)
    y_ref.backward(dy)
    xd = x.to(dt).cuda()
    y = torch.empty_like(xd)
    mu, rs = torch.empty(M, device="cuda"), torch.empty(M, device="cuda")
    w, b = ln.weight.detach().cuda(), ln.bias.detach().cuda()
    ops.layernorm_fwd(xd, w, b, 1e-12, y, mu, rs, M, D)
    dx = torch.empty_like(xd)
    dgam, dbet = torch.zeros(D, device="cuda"), torch.zeros(D, device="cuda")
    ops.layernorm_bwd(dy.to(dt).cuda(), xd, mu, rs, w, dx, None, dgam, dbet, M, D)
    torch.cuda.synchronize()
    assert rel(y.float(), y_ref) < tol(dt)
    assert rel(dx.float(), xr.grad) < tol(dt)
    assert rel(dgam, ln.weight.grad) < tol(dt) and rel(dbet, ln.bias.grad) < tol(dt)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", DT)
def test_embeddings_fwd_bwd(ops, dt):
    """word + position + token-type rows -> LayerNorm (HF BertEmbeddings, dropout 0)."""
    import oracle.clip as oc
    from transformers.models.bert.modeling_bert import BertEmbeddings
    cfg = oc.tinybert_config(0.0)
    torch.manual_seed(0)
    emb = BertEmbeddings(cfg).eval()
    B, T = 6, 40
    g = torch.Generator().manual_seed(4)
    ids = torch.randint(0, cfg.vocab_size, (B, T), generator=g)
    ids[:, 5] = ids[:, 9]                     # repeated tokens: scatter-add collisions
    ids[:, -3:] = 0                           # padding id: nn.Embedding(padding_idx=0) gets no gradient
    tt = torch.zeros(B, T, dtype=torch.long)
    tt[:, T // 2:] = 1
    out_ref = emb(input_ids=ids, token_type_ids=tt)
    gout = torch.randn(B, T, D, generator=g).to(dt).float()
    out_ref.backward(gout)
    M = B * T
    W_, P_, T_ = (emb.word_embeddings.weight.detach().cuda(), emb.position_embeddings.weight.detach().cuda(),
                  emb.token_type_embeddings.weight.detach().cuda())
    lw, lb = emb.LayerNorm.weight.detach().cuda(), emb.LayerNorm.bias.detach().cuda()
    e = torch.empty(M, D, dtype=dt, device="cuda")
    idc, ttc = ids.cuda().reshape(-1).contiguous(), tt.cuda().reshape(-1).contiguous()
    ops.embed_fwd(idc, ttc, W_, P_, T_, e, M, T, D)
    h = torch.empty_like(e)
    mu, rs = torch.empty(M, device="cuda"), torch.empty(M, device="cuda")
    ops.layernorm_fwd(e, lw, lb, cfg.layer_norm_eps, h, mu, rs, M, D)
    de = torch.empty_like(e)
    dlw, dlb = torch.zeros(D, device="cuda"), torch.zeros(D, device="cuda")
    ops.layernorm_bwd(gout.reshape(M, D).to(dt).cuda(), e, mu, rs, lw, de, None, dlw, dlb, M, D)
    dW, dP, dT = torch.zeros_like(W_), torch.zeros_like(P_), torch.zeros_like(T_)
    ops.embed_bwd(idc, ttc, de, dW, dP, dT, M, T, D)
    torch.cuda.synchronize()
    assert rel(h.float(), out_ref.reshape(M, D)) < tol(dt)
    rows = torch.unique(ids)
    assert rel(dW.cpu()[rows], emb.word_embeddings.weight.grad[rows]) < tol(dt, 5e-5)
    assert dW.cpu().abs().sum().item() == pytest.approx(dW.cpu()[rows].abs().sum().item())   # untouched rows stay 0
    assert rel(dP.cpu()[:T], emb.position_embeddings.weight.grad[:T]) < tol(dt, 5e-5)
    assert rel(dT, emb.token_type_embeddings.weight.grad) < tol(dt, 5e-5)
    assert rel(dlw, emb.LayerNorm.weight.grad) < tol(dt) and rel(dlb, emb.LayerNorm.bias.grad) < tol(dt)

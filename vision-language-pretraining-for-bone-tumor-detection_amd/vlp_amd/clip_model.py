"""CLIP-style model assembled from the HIP towers and the fused contrastive head.

Mirrors VisionLanguageModule's compute (src/models/pretrain/VisionLanguageModule.py):
  __init__ :98-111   image/text projections ~ N(0, dim^-1/2), logit_scale = ln(1/0.07)
  forward  :441-461  normalize(f @ P), s = min(exp(logit_scale), 100), logits = s * img @ txt^T
  _compute_loss :532-554  symmetric cross-entropy over the batch

Two entry points:
  * `ClipStepFn` — the training hot path: image tower + text tower + projections
    + L2-norm + (data-parallel all-gather) + fused loss/gradient kernel as ONE
    autograd node, so `loss.backward()` runs the explicit HIP backward of the
    whole model and hands autograd views of the flat gradient arenas.
  * `embeddings()/logits()` — the API path used by `forward(batch)`: returns
    logits/embeddings with autograd support through `EmbedFn`/`LogitsFn`.
"""
from __future__ import annotations

import math

import os

import torch
import torch.nn as nn

from . import dist as vdist
from . import ops
from .arena import ArenaModule


# the fused loss kernels (csrc/head_ops.hip) keep a query's embedding in registers
# and a 32-key slab in LDS: 4 <= E <= 256, E % 4 == 0 (the reference configs use
# 32 and 128, configs/experiment/pretrain/*.yaml)
MAX_EMBEDDING_DIM = 256


class ClipHead(ArenaModule):
    def __init__(self, image_dim=512, text_dim=312, embedding_dim=256, compute_dtype="bf16",
                 device=None):
        super().__init__()
        if embedding_dim % 4 or not 4 <= embedding_dim <= MAX_EMBEDDING_DIM:
            raise ValueError(f"embedding_dim={embedding_dim}: the HIP contrastive head supports multiples of 4 "
                             f"up to {MAX_EMBEDDING_DIM} (vlp_clip_loss_fused)")
        if compute_dtype == "bf16" and embedding_dim % 8:
            # the bf16 projection matmuls (vlp_matmul) take E as a contiguous extent,
            # which must be a multiple of 8 bf16 elements (16-B rows)
            raise ValueError(f"embedding_dim={embedding_dim}: compute_dtype='bf16' needs a multiple of 8 "
                             "(16-byte rows in the bf16 projection matmuls)")
        self.image_dim, self.text_dim, self.embedding_dim = image_dim, text_dim, embedding_dim
        self.compute_dtype = compute_dtype
        self._init_arena([("image_projection", (image_dim, embedding_dim)),
                          ("text_projection", (text_dim, embedding_dim)),
                          ("logit_scale", (1,))], device=device)
        self._ws = {}
        self.reset_parameters()

    @torch.no_grad()
    def reset_parameters(self):
        nn.init.normal_(self.arena.view("image_projection"), std=self.image_dim ** -0.5)   # :105
        nn.init.normal_(self.arena.view("text_projection"), std=self.text_dim ** -0.5)     # :109
        self.arena.view("logit_scale").fill_(math.log(1 / 0.07))                           # :111

    def _after_apply(self):
        self._ws = {}

    @property
    def tdtype(self):
        return torch.bfloat16 if self.compute_dtype == "bf16" else torch.float32

    def wcopy(self):
        if self.compute_dtype == "fp32":
            return self.arena.data
        buf = self._ws.get("wT")
        if buf is None:
            buf = torch.empty(self.arena.numel, dtype=self.tdtype, device=self.arena.data.device)
            self._ws["wT"] = buf
        ops.cast(self.arena.data, buf)
        return buf


def _project_normalize(head, wT, feat, ld, dim, proj_name, E):
    """emb = normalize(feat @ P) (fp32 out); feat rows with leading dim `ld`."""
    B = feat.shape[0] if ld == dim else feat.numel() // ld
    raw = torch.empty(B, E, dtype=torch.float32, device=feat.device)
    P = head.arena.view(proj_name, wT)
    # C[b][e] = sum_i feat[b][i] P[i][e]: A = feat (K-contig), B(n=e, k=i) = P[i][e] (MN-contig)
    ops.matmul(feat, P, raw, B, E, dim, ld, 1, E, 0, E, dtype_ref=feat)
    emb = torch.empty_like(raw)
    norm = torch.empty(B, dtype=torch.float32, device=feat.device)
    ops.l2norm_fwd(raw, emb, norm)
    return emb, norm


def _project_backward(head, wT, feat, ld, dim, proj_name, E, emb, norm, g_emb, gscale):
    """Returns d feat [B, dim] (compute dtype); writes d P into the head grad arena."""
    B = emb.shape[0]
    T = head.tdtype
    draw = torch.empty(B, E, dtype=torch.float32, device=emb.device)
    draw_t = draw if T == torch.float32 else torch.empty(B, E, dtype=T, device=emb.device)
    ops.l2norm_bwd(emb, norm, g_emb, draw, None if T == torch.float32 else draw_t, gscale=gscale)
    P = head.arena.view(proj_name, wT)
    # dP[i][e] = sum_b feat[b][i] draw[b][e]: A(m=i,k=b) = feat[b][i] (MN), B(n=e,k=b) = draw[b][e] (MN)
    ops.matmul(feat, draw_t, head.arena.gview(proj_name), dim, E, B, ld, 0, E, 0, E, dtype_ref=feat)
    # dfeat[b][i] = sum_e draw[b][e] P[i][e]: A = draw (K-contig), B(n=i,k=e) = P[i][e] (K-contig)
    dfeat = torch.empty(B, dim, dtype=T, device=emb.device)
    ops.matmul(draw_t, P, dfeat, B, dim, E, E, 1, E, 1, dim, dtype_ref=draw_t)
    return dfeat


_TEXT_STREAMS = {}
_USE_TEXT_STREAM = os.environ.get("VLP_TEXT_STREAM", "1") != "0"
# (r6, measured and not adopted, profiles/r6_text_stream_ab.txt: the text forward
# on the main stream ahead of the image tower, and a high-priority text stream;
# the rocprofv3 timeline shows the main stream waiting ≈1 ms at the join before
# the head, but both alternatives cost more than that wait)


def _text_stream(dev):
    """Second HIP stream for the text tower: its small, latency-bound kernels run
    beside the image tower's instead of after them (the towers only meet in
    the head).  None when disabled (VLP_TEXT_STREAM=0) or not on a GPU."""
    if not _USE_TEXT_STREAM or dev.type != "cuda":
        return None
    s = _TEXT_STREAMS.get(dev)
    if s is None:
        s = torch.cuda.Stream(device=dev)
        _TEXT_STREAMS[dev] = s
    return s


def role_weights(gl, gi, gt, device):
    """Per-direction weights w of sum_r w_r * CE_r / 2 whose gradient is that of
    gl*loss + gi*image_loss + gt*text_loss (loss = (image_loss + text_loss) / 2,
    reference :550-552): w_r = gl + 2 g_r (None = 0).  A device tensor [2]."""
    z = torch.zeros((), dtype=torch.float32, device=device)
    a = gl.reshape(()).float() if gl is not None else z
    wi = a + 2 * gi.reshape(()).float() if gi is not None else a
    wt = a + 2 * gt.reshape(()).float() if gt is not None else a
    return torch.stack([wi, wt]).contiguous()


class ClipStepFn(torch.autograd.Function):
    """loss, image_loss, text_loss, img_emb, txt_emb = f(batch; all parameters)."""

    @staticmethod
    def forward(ctx, model, x, x_u8, input_ids, attention_mask, token_type_ids, *params):
        img_t, txt_t, head = model.image_tower, model.text_tower, model.head
        training = model.training
        u8n = getattr(model, "u8_norm", (127.5, 73.9))
        main = torch.cuda.current_stream(input_ids.device) if input_ids.is_cuda else None
        s_txt = _text_stream(input_ids.device)
        if s_txt is not None:
            # fork: the text tower on its own stream (inputs are ready on main)
            s_txt.wait_stream(main)
            with torch.cuda.stream(s_txt):
                # only the CLS token's last hidden state is used (TextEncoder, :57-60)
                h_last, sv_txt = txt_t.run_forward(input_ids, attention_mask, token_type_ids, training,
                                                   cls_only=True)
            feat_img, sv_img = img_t.run_forward(x, training, x_u8=x_u8, u8_norm=u8n)
            main.wait_stream(s_txt)   # join before the head
        else:
            feat_img, sv_img = img_t.run_forward(x, training, x_u8=x_u8, u8_norm=u8n)
            h_last, sv_txt = txt_t.run_forward(input_ids, attention_mask, token_type_ids, training, cls_only=True)
        B, Tn = input_ids.shape
        D, E = txt_t.cfg.hidden, head.embedding_dim
        wT = head.wcopy()
        Di = head.image_dim
        ie, inorm = _project_normalize(head, wT, feat_img, Di, Di, "image_projection", E)
        te, tnorm = _project_normalize(head, wT, h_last, D, D, "text_projection", E)
        rank, world = vdist.world()
        ie_all = vdist.all_gather_rows(ie)
        te_all = vdist.all_gather_rows(te)
        N = B * world
        dev = ie.device
        g_img_all = torch.zeros(N, E, dtype=torch.float32, device=dev)
        g_txt_all = torch.zeros(N, E, dtype=torch.float32, device=dev)
        small = torch.zeros(4, dtype=torch.float32, device=dev)   # parts[2], d_logit_scale
        ls = head.arena.view("logit_scale")
        ops.clip_loss_fused(B, N, E, rank * B, ie_all, te_all, ls, g_img_all, g_txt_all, small[2:3],
                            small[0:2])
        vdist.all_reduce_sum_(small[0:2])  # global loss terms (the gradient needs no collective)
        out = torch.empty(3, dtype=torch.float32, device=dev)
        ops.clip_loss_finish(small[0:2], N, out)
        ctx.model = model
        ctx.state = (sv_img, sv_txt, wT, feat_img, h_last, ie, inorm, te, tnorm, g_img_all, g_txt_all,
                     small, B, Tn, D, E, (ie_all, te_all, N, rank))
        ctx.mark_non_differentiable(ie, te)
        ctx.set_materialize_grads(False)   # an unused image_loss / text_loss costs nothing
        return out[0], out[1], out[2], ie, te

    @staticmethod
    def backward(ctx, dloss, dli, dlt, die, dte):
        model = ctx.model
        img_t, txt_t, head = model.image_tower, model.text_tower, model.head
        (sv_img, sv_txt, wT, feat_img, h_last, ie, inorm, te, tnorm, g_img_all, g_txt_all, small,
         B, Tn, D, E, (ie_all, te_all, N, rank)) = ctx.state
        ctx.state = None
        for t in (head, img_t, txt_t):
            t.begin_backward()
        if dli is None and dlt is None:
            # the training step's loss alone: the forward's fused kernel already
            # formed d loss / d embeddings, scaled by dloss below
            gs = (dloss.reshape(1).float().contiguous() if dloss is not None
                  else torch.zeros(1, dtype=torch.float32, device=ie.device))
        else:
            # gradients of image_loss / text_loss (reference :550-552 returns them as
            # autograd tensors): rerun the head with per-direction weights
            w = role_weights(dloss, dli, dlt, ie.device)
            scratch = torch.zeros(2, dtype=torch.float32, device=ie.device)
            ops.clip_loss_fused(B, N, E, rank * B, ie_all, te_all, head.arena.view("logit_scale"), g_img_all,
                                g_txt_all, small[2:3], scratch, role_w=w)
            gs = torch.ones(1, dtype=torch.float32, device=ie.device)
        g_img = vdist.reduce_scatter_rows(g_img_all)
        g_txt = vdist.reduce_scatter_rows(g_txt_all)
        head.arena.grad.zero_()
        ops.scale(small[2:3], gs, head.arena.gview("logit_scale"))
        Di = head.image_dim
        dfeat_img = _project_backward(head, wT, feat_img, Di, Di, "image_projection", E, ie, inorm,
                                      g_img, gs)
        dcls = _project_backward(head, wT, h_last, D, D, "text_projection", E, te, tnorm,
                                 g_txt, gs)
        # data parallel: SUM all-reduce of the flat gradient arenas, the head and
        # text tower's launched while the (much longer) image backward runs, the
        # image tower's per stage (layer4 first) as the backward leaves each stage.
        # With the text stream the text backward and its collective also run
        # beside the image backward; every tensor crossing streams stays
        # referenced until the join below.
        reducer = vdist.GradReducer()
        on_stage = None
        if vdist.active():
            def on_stage(off, n):
                reducer.reduce_span(img_t.arena, off, n)
        s_txt = _text_stream(dcls.device)
        if s_txt is not None:
            main = torch.cuda.current_stream(dcls.device)
            s_txt.wait_stream(main)
            with torch.cuda.stream(s_txt):
                txt_t.run_backward(sv_txt, dcls)
                reducer.reduce([txt_t.arena])
            reducer.reduce([head.arena])
            img_t.run_backward(sv_img, dfeat_img, on_stage_done=on_stage)
            main.wait_stream(s_txt)
        else:
            txt_t.run_backward(sv_txt, dcls)
            reducer.reduce([head.arena, txt_t.arena])
            img_t.run_backward(sv_img, dfeat_img, on_stage_done=on_stage)
        reducer.wait()
        grads = (head.grads_for_autograd() + img_t.grads_for_autograd() + txt_t.grads_for_autograd())
        return (None, None, None, None, None, None, *grads)


def model_params(model):
    return (model.head.params_in_arena_order() + model.image_tower.params_in_arena_order()
            + model.text_tower.params_in_arena_order())

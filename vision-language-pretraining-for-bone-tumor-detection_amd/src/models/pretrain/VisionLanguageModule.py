"""Drop-in replacement for the reference's
src/models/pretrain/VisionLanguageModule.py on MI355X.

Same import path (`_target_: src.models.pretrain.VisionLanguageModule.VisionLanguageModule`,
configs/model/vision_language.yaml:1), same classes (ImageEncoder :27-35,
TextEncoder :38-60, VisionLanguageModule :63-705), same constructor kwargs
(including the misspelt `image_encoder_droupout`, :83), same hooks and
state-dict keys (image_encoder.model.<timm>, text_encoder.model.<HF Bert>,
image_projection, text_projection, logit_scale).  All arithmetic runs in the
HIP kernels of libvlp_hip.so (vlp_amd); there is no CPU fallback.

Additions (keyword-only, defaults keep reference behaviour where possible):
  compute_dtype  "fp32" (the reference's arithmetic, default) | "bf16" (throughput mode,
                 the _mi355x experiments; src/train.py also derives it from trainer.precision)
  text_dropout   TinyBERT hidden/attention dropout (reference: 0.1 from the hub config)
  fused_optimizer  build vlp_amd.FusedAdamW when the configured optimizer is
                   torch.optim.AdamW (same hyper-parameters / param groups)
  device         where the parameter arenas live (default: cuda)
"""
from __future__ import annotations

import functools
import logging
import math
import os
import sys
import types
from itertools import chain
from typing import Tuple

import torch
import torch.nn as nn

_PKG = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", ".."))
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

from vlp_amd import ops  # noqa: E402
from vlp_amd.clip_model import ClipHead, ClipStepFn, _project_normalize, role_weights  # noqa: E402
from vlp_amd.optim import FusedAdamW  # noqa: E402
from vlp_amd.nest import NEST_CFGS, NestTower  # noqa: E402
from vlp_amd.resnet34 import ResNet34Tower  # noqa: E402
from vlp_amd.tinybert import TinyBertConfig, TinyBertTower  # noqa: E402

logger = logging.getLogger("project")

try:  # Lightning is optional: the module works as a plain nn.Module without it
    import lightning as L  # type: ignore

    _Base = L.LightningModule
    _HAVE_LIGHTNING = True
except Exception:  # pragma: no cover - lightning absent in this image
    _HAVE_LIGHTNING = False

    class _AttributeDict(dict):
        def __getattr__(self, k):
            try:
                return self[k]
            except KeyError as e:
                raise AttributeError(k) from e

        def __setattr__(self, k, v):
            self[k] = v

    class _Base(nn.Module):
        """The subset of LightningModule the reference module uses."""
        trainer = None

        def save_hyperparameters(self, hp: dict, logger: bool = True):
            object.__setattr__(self, "_hparams", _AttributeDict(hp))

        @property
        def hparams(self):
            return self._hparams

        def log(self, name, value, **kw):
            self.__dict__.setdefault("logged", {})[name] = value


def _default_device(device):
    if device is not None:
        return torch.device(device)
    if not torch.cuda.is_available():
        raise RuntimeError("VisionLanguageModule (MI355X build) needs a ROCm GPU: there is no CPU path")
    return torch.device("cuda", torch.cuda.current_device())


class ImageEncoder(nn.Module):
    """:27-35 — `timm.create_model(model, pretrained=False, num_classes=0,
    global_pool="avg", **kwargs)`; here the MI355X ResNet34 tower."""

    def __init__(self, model, compute_dtype="fp32", device=None, **kwargs):
        super().__init__()
        if model == "resnet34":
            self.model = ResNet34Tower(drop_rate=kwargs.get("drop_rate", 0.0), compute_dtype=compute_dtype,
                                       device=device)
        elif model in NEST_CFGS:
            # timm nest defaults: img_size 224, drop_path_rate 0.5 (SURVEY §8(f) row 2:
            # 512 x 512 inputs need img_size=512, passed through the module's image_size)
            self.model = NestTower(model, img_size=kwargs.get("img_size", 224),
                                   drop_rate=kwargs.get("drop_rate", 0.0),
                                   drop_path_rate=kwargs.get("drop_path_rate", 0.5), compute_dtype=compute_dtype,
                                   device=device)
        else:
            raise ValueError(f"ImageEncoder: model {model} is not built for MI355X "
                             f"(supported: resnet34, {', '.join(NEST_CFGS)})")

    def forward(self, x):
        return self.model(x)


class TextEncoder(nn.Module):
    """:38-60 — TinyBERT; returns the CLS token's last hidden state."""

    def __init__(self, text_encoder_model, compute_dtype="fp32", device=None, dropout=0.1):
        super().__init__()
        if text_encoder_model == "distilbert":
            raise NotImplementedError("TextEncoder: distilbert is outside the MI355X hot path (use tinybert)")
        if text_encoder_model != "tinybert":
            raise ValueError(
                f"VisionLanguageModule: Text encoder model {text_encoder_model} is not supported. "
                f"Supported models are: distilbert, tinybert.")
        self.model = TinyBertTower(TinyBertConfig(dropout, dropout), compute_dtype=compute_dtype,
                                   device=device)
        self.target_token_idx = 0
        self.model.train()

    def forward(self, **kwargs):
        h = self.model(**kwargs)
        return h[:, self.target_token_idx, :]


class _EmbedFn(torch.autograd.Function):
    """normalize(features @ P) for the API forward path (HIP GEMM + L2 norm)."""

    @staticmethod
    def forward(ctx, head, feat, proj_name, P):
        T = head.tdtype
        f = feat.to(T).contiguous()
        wT = head.wcopy()
        emb, norm = _project_normalize(head, wT, f, f.shape[1], f.shape[1], proj_name, head.embedding_dim)
        ctx.head, ctx.f, ctx.wT, ctx.emb, ctx.norm, ctx.name = head, f, wT, emb, norm, proj_name
        return emb

    @staticmethod
    def backward(ctx, g):
        from vlp_amd.clip_model import _project_backward
        head, f = ctx.head, ctx.f
        E = head.embedding_dim
        gP_before = head.arena.gview(ctx.name).clone()
        dfeat = _project_backward(head, ctx.wT, f, f.shape[1], f.shape[1], ctx.name, E, ctx.emb,
                                  ctx.norm, g.float().contiguous(), None)
        dP = head.arena.gview(ctx.name).clone()
        head.arena.gview(ctx.name).copy_(gP_before)
        return None, dfeat.float(), None, dP


def _pad_rows4(t):
    """Zero rows up to a multiple of 4 (vlp_matmul moves 16-B chunks along every
    contiguous extent; zero rows add nothing to the products)."""
    r = (-t.shape[0]) % 4
    t = t.float().contiguous()
    return t if r == 0 else torch.cat([t, t.new_zeros((r,) + tuple(t.shape[1:]))])


class _LogitsFn(torch.autograd.Function):
    """logits = clamp(exp(logit_scale), max=100) * img @ txt^T (:456-459)."""

    @staticmethod
    def forward(ctx, ie, te, ls):
        B, E = ie.shape
        Nt = te.shape[0]
        s = torch.clamp(ls.detach().exp(), max=100).float()
        iep, tep = _pad_rows4(ie), _pad_rows4(te)
        Bp, Np = iep.shape[0], tep.shape[0]
        cos = torch.empty(Bp, Np, dtype=torch.float32, device=ie.device)
        ops.matmul(iep, tep, cos, Bp, Np, E, E, 1, E, 1, Np)
        logits = torch.empty_like(cos)
        ops.scale(cos, s, logits)
        ctx.save_for_backward(iep, tep, ls, cos, s)
        ctx.shape = (B, Nt)
        return logits[:B, :Nt]

    @staticmethod
    def backward(ctx, g):
        iep, tep, ls, cos, s = ctx.saved_tensors
        B, Nt = ctx.shape
        Bp, Np = cos.shape
        E = iep.shape[1]
        gp = torch.zeros(Bp, Np, dtype=torch.float32, device=g.device)
        gp[:B, :Nt] = g
        gs = torch.empty_like(gp)
        ops.scale(gp, s, gs)
        die = torch.empty_like(iep)
        ops.matmul(gs, tep, die, Bp, E, Np, Np, 1, E, 0, E)       # gs @ te
        dte = torch.empty_like(tep)
        ops.matmul(gs, iep, dte, Np, E, Bp, Np, 0, E, 0, E)       # gs^T @ ie
        # d logit_scale = sum(g * cos) * s  (zero when clamped)
        dls = (gp * cos).sum().reshape(1) * s * (ls.detach().exp() <= 100).float()
        return die[:B], dte[:Nt], dls.to(ls.dtype)


class _SymCEFn(torch.autograd.Function):
    """(CE(logits, arange) + CE(logits^T, arange)) / 2, image, text (:550-552).
    All three outputs are differentiable, as the reference's autograd tensors are."""

    @staticmethod
    def forward(ctx, logits):
        lg = logits.float().contiguous()
        out = torch.zeros(3, dtype=torch.float32, device=lg.device)
        dl = torch.zeros_like(lg)
        ops.ce_sym(lg, out, dl)
        ctx.save_for_backward(dl, lg)
        ctx.set_materialize_grads(False)
        return out[0], out[1], out[2]

    @staticmethod
    def backward(ctx, gl, gi, gt):
        dl, lg = ctx.saved_tensors
        if gi is None and gt is None:
            if gl is None:
                return None
            out = torch.empty_like(dl)
            ops.scale(dl, gl.reshape(1).float().contiguous(), out)
            return out
        # gl*loss + gi*image_loss + gt*text_loss = sum_r (gl + 2 g_r) * CE_r / 2
        w = role_weights(gl, gi, gt, lg.device)
        out = torch.zeros_like(lg)
        ops.ce_sym(lg, torch.zeros(3, dtype=torch.float32, device=lg.device), out, role_w=w)
        return out


def _logit_scale_fp64(module, state_dict, prefix, local_metadata):
    """The reference's logit_scale is float64 (torch.tensor([np.log(1/0.07)]), :111);
    the HIP head keeps it in its fp32 arena, the checkpoint carries the reference
    dtype (loading casts back)."""
    k = prefix + "logit_scale"
    if k in state_dict:
        state_dict[k] = state_dict[k].double()


class VisionLanguageModule(_Base):
    # the fused step all-gathers embeddings and all-reduces the gradient arenas
    # itself (vlp_amd.clip_model.ClipStepFn); trainers must not reduce again
    handles_dp_collectives = True

    def __init__(
        self,
        image_model,
        text_encoder_model,
        optimizer: torch.optim.Optimizer,
        deduplicate: bool,
        masked_loss: bool,
        image_embedding_dim: int = 512,
        text_embedding_dim: int = 768,
        embedding_dim: int = 256,
        label_weights: tuple = (1.0, 1.0),
        scheduler: torch.optim.lr_scheduler = None,
        downstream_datamodule=None,
        text_encoder_lr: float = None,
        image_encoder_lr: float = None,
        projections_lr: float = None,
        image_encoder_droupout: float = 0.0,
        compute_dtype: str = "fp32",
        text_dropout: float = 0.1,
        fused_optimizer: bool = True,
        device=None,
        **kwargs,
    ):
        super().__init__()
        if deduplicate:
            if masked_loss:
                logger.warning("Deduplication and masked loss are mutually exclusive. Deduplication will be used.")
            masked_loss = False                                                     # :87-92
        hp = dict(image_model=image_model, text_encoder_model=text_encoder_model, optimizer=optimizer,
                  deduplicate=deduplicate, masked_loss=masked_loss,
                  image_embedding_dim=image_embedding_dim, text_embedding_dim=text_embedding_dim,
                  embedding_dim=embedding_dim, label_weights=label_weights, scheduler=scheduler,
                  downstream_datamodule=downstream_datamodule, text_encoder_lr=text_encoder_lr,
                  image_encoder_lr=image_encoder_lr, projections_lr=projections_lr,
                  image_encoder_droupout=image_encoder_droupout, compute_dtype=compute_dtype,
                  text_dropout=text_dropout, fused_optimizer=fused_optimizer, **kwargs)
        if _HAVE_LIGHTNING:  # pragma: no cover
            self.save_hyperparameters(logger=False)
        else:
            self.save_hyperparameters(hp, logger=False)
        dev = _default_device(device)
        enc_kw = {"drop_rate": image_encoder_droupout}                                # :98
        if "image_size" in kwargs:          # timm img_size (NesT needs it for 512 x 512 inputs)
            enc_kw["img_size"] = kwargs["image_size"]
        if "drop_path_rate" in kwargs:
            enc_kw["drop_path_rate"] = kwargs["drop_path_rate"]
        self.image_encoder = ImageEncoder(image_model, compute_dtype=compute_dtype, device=dev, **enc_kw)
        feat_dim = self.image_encoder.model.num_features if image_model != "resnet34" else 512
        if image_embedding_dim != feat_dim or text_embedding_dim != 312:
            raise ValueError(f"MI355X build: {image_model} ({feat_dim}) + tinybert (312) feature dims, got "
                             f"image_embedding_dim={image_embedding_dim}, text_embedding_dim={text_embedding_dim}")
        self.text_encoder = TextEncoder(text_encoder_model, compute_dtype=compute_dtype, device=dev,
                                        dropout=text_dropout)                        # :99
        # projections + logit scale (:102-111) live in one arena; registered here so
        # the state-dict keys are the reference's top-level names
        head = ClipHead(image_embedding_dim, text_embedding_dim, embedding_dim, compute_dtype, device=dev)
        object.__setattr__(self, "_head", head)
        for name in ("image_projection", "text_projection", "logit_scale"):
            self.register_parameter(name, nn.Parameter(head.arena.view(name)))
            head._param_slots.append((self, name, name))
        self.k_for_precision_at_k = [3, 5, 10, 15]
        self.k_for_image_text_retreival = [3, 5, 10, 15]
        self._val_loss_sum = None
        self._val_loss_n = 0
        self.downstream_datamodule = downstream_datamodule
        if self.downstream_datamodule is not None:
            dm, _ = next(self.downstream_datamodule.get_cv_splits())                 # :120-124
            self.downstream_train_dataloader = dm.train_dataloader()
            self.downstream_val_dataloaders = dm.val_dataloader()
        self.train_image_embeddings_and_labels_cached = {}
        self.val_image_embeddings_and_labels_cached = {}
        self._register_state_dict_hook(_logit_scale_fp64)
        logger.info("VisionLanguageModule (MI355X): initialized, compute_dtype=%s", compute_dtype)

    # ---------------- device moves keep arenas aliased ----------------
    def _apply(self, fn, recurse=True):
        for child in self.children():
            child._apply(fn)
        head = self._head
        head.arena.data = fn(head.arena.data)
        head.arena.grad = fn(head.arena.grad)
        for name in ("image_projection", "text_projection", "logit_scale"):
            self._parameters[name].data = head.arena.view(name)
            self._parameters[name].grad = None
        head._ws = {}
        return self

    @property
    def device(self):
        return self._head.arena.data.device

    def _towers(self):
        m = types.SimpleNamespace(image_tower=self.image_encoder.model, text_tower=self.text_encoder.model,
                                  head=self._head, training=self.training)
        return m

    def _all_params(self):
        return (self._head.params_in_arena_order() + self.image_encoder.model.params_in_arena_order()
                + self.text_encoder.model.params_in_arena_order())

    # ---------------- optimizer (:130-297) ----------------
    def configure_optimizers(self):
        param_groups = self._configure_optimizer_parameters()
        opt_factory = self.hparams.optimizer
        func = getattr(opt_factory, "func", opt_factory)
        if self.hparams.get("fused_optimizer", True) and func is torch.optim.AdamW:
            kw = dict(getattr(opt_factory, "keywords", {}) or {})
            optimizer = FusedAdamW(param_groups, arenas=[self._head, self.image_encoder.model,
                                                         self.text_encoder.model], **kw)
        else:
            optimizer = opt_factory(params=param_groups)
        for group in optimizer.param_groups:
            logger.info("Parameter group '%s': %d params, lr=%s", group.get("name", "unnamed"),
                        sum(p.numel() for p in group["params"]), group.get("lr", "default"))
        num = sum(p.numel() for g in optimizer.param_groups for p in g["params"])
        self.hparams["num_optimized_params"] = num
        if self.hparams.scheduler is not None:
            scheduler = self.hparams.scheduler(optimizer=optimizer)
            return {"optimizer": optimizer,
                    "lr_scheduler": {"scheduler": scheduler, "interval": "epoch", "frequency": 1}}
        return {"optimizer": optimizer}

    def _configure_optimizer_parameters(self):
        image_encoder_params = list(self.image_encoder.parameters())
        text_encoder_params = list(self.text_encoder.parameters())
        proj = [self.image_projection, self.text_projection, self.logit_scale]
        assigned = set(image_encoder_params + text_encoder_params + proj)
        remaining = [p for p in self.parameters() if p not in assigned]
        if remaining:
            logger.warning("VisionLanguageModule: %d parameters are not assigned to any group", len(remaining))
        groups = [{"params": remaining, "name": "remaining_params"}]
        for params, name, lr in ((proj, "projection_and_logitscale", self.hparams.projections_lr),
                                 (image_encoder_params, "image_encoder", self.hparams.image_encoder_lr),
                                 (text_encoder_params, "text_encoder", self.hparams.text_encoder_lr)):
            g = self._get_param_group(params, name, lr)
            if g is not None:
                groups.append(g)
        return groups

    def _get_param_group(self, params, name: str, lr):
        group = {"params": params, "name": name}
        if lr is not None:
            group["lr"] = lr
            if lr == 0:
                for p in params:
                    p.requires_grad = False
                return None
            if lr < 0:
                raise ValueError(f"VisionLanguageModule: {name} scale learning rate must be a non-negative value.")
        return group

    # ---------------- forward / loss ----------------
    def forward(self, batch):
        """:441-461 — returns (logits, image_embeddings, text_embeddings)."""
        x = batch["x-ray"] if "x-ray" in batch else batch["x-ray-u8"]   # u8: on-device normalise
        self.image_encoder.model.u8_norm = tuple(batch.get("x-ray-u8-norm", (127.5, 73.9)))
        image_features = self.image_encoder(x.to(self.device, non_blocking=True))
        text_features = self.text_encoder(**{k: v.to(self.device, non_blocking=True)
                                             for k, v in batch["caption_tokenized"].items()})
        ie = _EmbedFn.apply(self._head, image_features, "image_projection", self.image_projection)
        te = _EmbedFn.apply(self._head, text_features, "text_projection", self.text_projection)
        logits = _LogitsFn.apply(ie, te, self.logit_scale)
        return logits, ie, te

    def _compute_loss(self, logits, deduplicate: bool = True, masked: bool = False, captions=None):
        if deduplicate:                                                              # :535-545
            raise DeprecationWarning(
                "Deduplication loss was made obsolete by generating diverse captions and the custom batch sampler")
        if masked:
            raise DeprecationWarning(
                "Masked loss was made obsolete by generating diverse captions and the custom batch sampler")
        return _SymCEFn.apply(logits)

    def training_step_outputs(self, batch):
        """Fused hot path: loss, image_loss, text_loss, img_emb, txt_emb (global batch under DP)."""
        dev = self.device
        x = batch.get("x-ray")
        x_u8 = batch.get("x-ray-u8")
        if x_u8 is not None:
            x = None
            x_u8 = x_u8.to(dev, non_blocking=True)
        else:
            x = x.to(dev, non_blocking=True)
        ct = batch["caption_tokenized"]
        ids = ct["input_ids"].to(dev, non_blocking=True)
        am = ct.get("attention_mask")
        tt = ct.get("token_type_ids")
        am = am.to(dev, non_blocking=True) if am is not None else None
        tt = tt.to(dev, non_blocking=True) if tt is not None else None
        if self.hparams["deduplicate"] or self.hparams["masked_loss"]:
            raise DeprecationWarning("deduplicate / masked loss were removed by the reference (:535-545)")
        towers = self._towers()
        towers.u8_norm = tuple(batch.get("x-ray-u8-norm", (127.5, 73.9)))   # the collator's normalisation
        return ClipStepFn.apply(towers, x, x_u8, ids, am, tt, *self._all_params())

    def training_step(self, batch, batch_idx=None):
        """:634-645 (fused: the logits matrix is never materialised)."""
        loss, li, lt, ie, te = self.training_step_outputs(batch)
        self._cache_embeddings_and_labels(ie, te, batch["label"], mode="train")
        bs = batch["caption_tokenized"]["input_ids"].shape[0]
        self.log("train/loss", loss, on_step=True, on_epoch=True, batch_size=bs)
        self.log("logit_scale", self.logit_scale.detach().exp(), on_step=True, on_epoch=True, batch_size=bs)
        return loss

    # ---------------- caching / retrieval metrics (:556-628, :364-439) ----------------
    def _cache_embeddings_and_labels(self, image_embeddings, text_embeddings, labels, mode):
        assert mode in ["train", "val"], f"Invalid mode: {mode}"
        cache = (self.train_image_embeddings_and_labels_cached if mode == "train"
                 else self.val_image_embeddings_and_labels_cached)
        # list append, concatenated once at epoch end (the reference's per-step
        # torch.cat is O(steps^2) in copies; the result is identical)
        cache.setdefault("image_embedding", []).append(image_embeddings.detach())
        cache.setdefault("text_embedding", []).append(text_embeddings.detach())
        cache.setdefault("label", []).append(labels.to(image_embeddings.device))

    def _get_cached_embeddings_and_labels(self, mode):
        assert mode in ["train", "val"], f"Invalid mode: {mode}"
        cache = (self.train_image_embeddings_and_labels_cached if mode == "train"
                 else self.val_image_embeddings_and_labels_cached)
        if "image_embedding" not in cache or "label" not in cache:
            raise ValueError(f"No cached embeddings and labels for mode: {mode}")
        return (torch.cat(cache["image_embedding"]), torch.cat(cache["text_embedding"]),
                torch.cat(cache["label"]))

    def precision_at_k_on_image_embeddings(self, image_embeddings, labels, ks: list) -> dict:
        """:364-400.  On the GPU the top-(k+1) lists come from chunked fp32
        similarity GEMMs + vlp_row_topk (no N x N matrix); the first entry (the
        query itself) is dropped as in the reference."""
        assert all(k + 1 <= image_embeddings.shape[0] for k in ks), "k+1 must be less than or equal to the batch size"
        e = torch.nn.functional.normalize(image_embeddings.float())
        labels = labels.to(e.device)
        out = {}
        if e.is_cuda and max(ks) + 1 <= 16:
            _, top_all = ops.sim_topk(e, e, max(ks) + 1)
            for k in ks:
                correct = (labels.unsqueeze(1) == labels[top_all[:, 1:k + 1]]).sum(dim=1)
                out[k] = (correct.float() / k).mean().item()
            return out
        sim = e @ e.T
        for k in ks:
            top = sim.topk(k=k + 1, dim=1).indices[:, 1:]
            correct = (labels.unsqueeze(1) == labels[top]).sum(dim=1)
            out[k] = (correct.float() / k).mean().item()
        return out

    def recall_at_k_on_image_text_retreival(self, image_embeddings, text_embeddings, ks: list) -> dict:
        """:402-439 (GPU: chunked similarity + vlp_row_topk, as above)."""
        i = torch.nn.functional.normalize(image_embeddings.float())
        t = torch.nn.functional.normalize(text_embeddings.float())
        out = {}
        tgt = torch.arange(i.shape[0], device=i.device)
        if i.is_cuda and max(ks) <= 16:
            _, top_all = ops.sim_topk(i, t, max(ks))
            for k in ks:
                out[k] = (top_all[:, :k] == tgt.unsqueeze(1)).any(dim=1).sum().item() / i.shape[0]
            return out
        sim = i @ t.T
        for k in ks:
            top = sim.topk(k=k, dim=1).indices
            out[k] = (top == tgt.unsqueeze(1)).any(dim=1).sum().item() / i.shape[0]
        return out

    def evaluate_downstream_precision_at_k(self, mode="entire") -> Tuple[dict, dict]:
        emb, labs = [], []
        self.eval()
        with torch.no_grad():
            if mode == "entire":
                all_batches = chain(self.downstream_train_dataloader, *self.downstream_val_dataloaders)
            elif mode == "validation":
                all_batches = chain(*self.downstream_val_dataloaders)
            else:
                raise ValueError(f"Invalid mode: {mode}. Supported modes are: 'entire', 'validation'.")
            for batch in all_batches:
                labels = batch["tumor"].to(device=self.device, dtype=torch.int64)
                x = batch["x-ray"] if "x-ray" in batch else batch["x-ray-u8"]   # u8: on-device normalise
                self.image_encoder.model.u8_norm = tuple(batch.get("x-ray-u8-norm", (127.5, 73.9)))
                f = self.image_encoder(x.to(self.device))
                e = _EmbedFn.apply(self._head, f, "image_projection", self.image_projection)
                emb.append(e)
                labs.append(labels)
        self.train()
        return self.precision_at_k_on_image_embeddings(torch.cat(emb), torch.cat(labs), ks=self.k_for_precision_at_k)

    # ---------------- epoch hooks (:631-705) ----------------
    def on_train_epoch_start(self):
        self.train_image_embeddings_and_labels_cached = {}

    def on_train_epoch_end(self):
        ie, te, labels = self._get_cached_embeddings_and_labels(mode="train")
        for k, v in self.precision_at_k_on_image_embeddings(ie, labels, ks=self.k_for_precision_at_k).items():
            self.log(f"train/label_precision_at_{k}", v, on_step=False, on_epoch=True, batch_size=ie.shape[0])
        for k, v in self.recall_at_k_on_image_text_retreival(ie, te, ks=self.k_for_image_text_retreival).items():
            self.log(f"train/image_text_recall_at_{k}", v, on_step=False, on_epoch=True, batch_size=ie.shape[0])

    def on_validation_epoch_start(self):
        self._val_loss_sum, self._val_loss_n = None, 0
        self.val_image_embeddings_and_labels_cached = {}

    def validation_step(self, batch, batch_idx, dataloader_idx=0):
        logits, ie, te = self(batch)
        self._cache_embeddings_and_labels(ie, te, batch["label"], mode="val")
        loss, _, _ = self._compute_loss(logits, self.hparams["deduplicate"], self.hparams["masked_loss"],
                                        batch.get("caption"))
        if dataloader_idx == 0:
            log_path_str = "val/lera"
        elif dataloader_idx == 1:
            log_path_str = "val/mura"
        else:
            raise ValueError(
                f"VisionLanguageModule: Validation dataloader index {dataloader_idx} is not supported. "
                f"Supported indices are: 0, 1. We are assuming that the first dataloader is for the LERA "
                f"dataset and the second dataloader for the MURA dataset")
        bs = logits.shape[0]
        self.log(f"{log_path_str}/loss", loss, on_step=False, on_epoch=True, batch_size=bs,
                 add_dataloader_idx=False)
        self._val_loss_sum = loss.detach() * bs if self._val_loss_sum is None else self._val_loss_sum + loss.detach() * bs
        self._val_loss_n += bs
        return loss

    def on_validation_epoch_end(self):
        # the reference's MeanMetric syncs across ranks: sum and count over every rank.  The
        # collective runs on every rank, also one that saw no validation batch (zeros)
        dev = self._val_loss_sum.device if self._val_loss_sum is not None else self.device
        tot = torch.stack([self._val_loss_sum.double().reshape(()) if self._val_loss_sum is not None
                           else torch.zeros((), dtype=torch.float64, device=dev),
                           torch.tensor(float(self._val_loss_n), dtype=torch.float64, device=dev)])
        d = torch.distributed
        if d.is_available() and d.is_initialized() and d.get_world_size() > 1:
            cdev = tot.device if d.get_backend() == "nccl" else torch.device("cpu")
            tot = tot.to(cdev)
            d.all_reduce(tot)
        if tot[1].item() > 0:
            self.log("val/combined/loss", (tot[0] / tot[1]).float(), prog_bar=True)
        ie, te, labels = self._get_cached_embeddings_and_labels(mode="val")
        for k, v in self.precision_at_k_on_image_embeddings(ie, labels, ks=self.k_for_precision_at_k).items():
            self.log(f"val/combined/label_precision_at_{k}", v, batch_size=ie.shape[0])
        for k, v in self.recall_at_k_on_image_text_retreival(ie, te, ks=self.k_for_image_text_retreival).items():
            self.log(f"val/combined/image_text_recall_at_{k}", v, batch_size=ie.shape[0])
        trainer = getattr(self, "trainer", None)
        if trainer is not None and getattr(trainer, "sanity_checking", False):
            return
        if self.downstream_datamodule is not None:
            for k, v in self.evaluate_downstream_precision_at_k(mode="validation").items():
                self.log(f"downstream_validation/label_precision_at_{k}", v, on_step=False, on_epoch=True)

    # ---------------- checkpoints ----------------
    @classmethod
    def load_from_checkpoint(cls, checkpoint_path, map_location=None, strict=True, **kwargs):
        """Lightning-format checkpoint ({"state_dict", "hyper_parameters"}); loaded
        with weights_only=True (hyper-parameters holding objects must be passed
        again as kwargs, as src/train.py:198 does for the datamodule)."""
        from src.utils.config import instantiate
        ckpt = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
        hp = dict(ckpt.get("hyper_parameters", {}))
        # factories saved as {_target_, _partial_} nodes (src/utils/trainer.serializable_hparams)
        hp = {k: instantiate(v) if isinstance(v, dict) and "_target_" in v else v for k, v in hp.items()}
        hp.pop("num_optimized_params", None)
        hp.update(kwargs)
        model = cls(**hp)
        model.load_state_dict(ckpt["state_dict"], strict=strict)
        return model

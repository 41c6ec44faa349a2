"""ORACLE (test infrastructure): CPU fp32 restatement of the reference's
contrastive head, loss, retrieval metrics and model assembly.

Every function cites the reference line it restates
(src/models/pretrain/VisionLanguageModule.py unless stated).
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from .resnet34 import ResNet34


def tinybert_config(dropout: float = 0.1):
    """huawei-noah/TinyBERT_General_4L_312D config (VisionLanguageModule.py:45)."""
    from transformers import BertConfig
    return BertConfig(vocab_size=30522, hidden_size=312, num_hidden_layers=4,
                      num_attention_heads=12, intermediate_size=1200, hidden_act="gelu",
                      hidden_dropout_prob=dropout, attention_probs_dropout_prob=dropout,
                      max_position_embeddings=512, type_vocab_size=2, layer_norm_eps=1e-12,
                      initializer_range=0.02)


def make_bert(dropout: float = 0.1):
    """The text tower IS the third-party reference (transformers.BertModel); the
    reference pins transformers=4.44.1 (environment.yaml:234), this container has
    5.x whose BertModel arithmetic for this config is the same."""
    from transformers import BertModel
    return BertModel(tinybert_config(dropout), add_pooling_layer=True)


def clip_forward(image_features, text_features, image_projection, text_projection, logit_scale):
    """VisionLanguageModule.forward :441-461."""
    image_embeddings = image_features @ image_projection                    # :448
    text_embeddings = text_features @ text_projection                       # :449
    image_embeddings = F.normalize(image_embeddings)                        # :452
    text_embeddings = F.normalize(text_embeddings)                          # :453
    s = torch.clamp(logit_scale.exp(), max=100)                             # :456-457
    logits = (image_embeddings @ text_embeddings.T) * s                     # :459
    return logits, image_embeddings, text_embeddings


def compute_loss(logits):
    """_compute_loss :532-554 (deduplicate/masked branches raise in the reference)."""
    labels = torch.arange(len(logits), device=logits.device)               # :533
    image_loss = F.cross_entropy(logits, labels, reduction="mean")          # :550
    text_loss = F.cross_entropy(logits.T, labels, reduction="mean")         # :551
    return (image_loss + text_loss) / 2, image_loss, text_loss              # :552-554


def precision_at_k(image_embeddings, labels, ks):
    """precision_at_k_on_image_embeddings :364-400."""
    assert all(k + 1 <= image_embeddings.shape[0] for k in ks)
    e = F.normalize(image_embeddings)
    sim = e @ e.T
    out = {}
    for k in ks:
        top = sim.topk(k=k + 1, dim=1).indices[:, 1:]
        correct = (labels.unsqueeze(1) == labels[top]).sum(dim=1)
        out[k] = (correct.float() / k).mean().item()
    return out


def recall_at_k(image_embeddings, text_embeddings, ks):
    """recall_at_k_on_image_text_retreival :402-439."""
    i = F.normalize(image_embeddings)
    t = F.normalize(text_embeddings)
    sim = i @ t.T
    out = {}
    for k in ks:
        top = sim.topk(k=k, dim=1).indices
        tgt = torch.arange(i.shape[0])
        out[k] = (top == tgt.unsqueeze(1)).any(dim=1).sum().item() / i.shape[0]
    return out


class _ImageEncoder(nn.Module):           # :27-35
    def __init__(self, drop_rate=0.0, model="resnet34", img_size=224):
        super().__init__()
        if model == "resnet34":
            self.model = ResNet34(drop_rate=drop_rate)
        else:                                 # timm nest_small restated (oracle/nest.py)
            from oracle.nest import nest_small
            assert model == "nest_small", model
            self.model = nest_small(img_size=img_size, drop_rate=drop_rate)

    def forward(self, x):
        return self.model(x)


class _TextEncoder(nn.Module):            # :38-60
    def __init__(self, dropout=0.1):
        super().__init__()
        self.model = make_bert(dropout)
        self.target_token_idx = 0

    def forward(self, **kw):
        return self.model(**kw).last_hidden_state[:, self.target_token_idx, :]


class OracleVLP(nn.Module):
    """Same state-dict layout as the reference VisionLanguageModule
    (image_encoder.model.*, text_encoder.model.*, image_projection,
    text_projection, logit_scale; :98-111)."""

    def __init__(self, embedding_dim=128, text_dropout=0.1, image_dropout=0.0, image_model="resnet34",
                 img_size=224):
        super().__init__()
        self.image_encoder = _ImageEncoder(image_dropout, image_model, img_size)
        self.text_encoder = _TextEncoder(text_dropout)
        di = self.image_encoder.model.num_features
        self.image_projection = nn.Parameter(torch.empty(di, embedding_dim))
        nn.init.normal_(self.image_projection, std=di ** -0.5)
        self.text_projection = nn.Parameter(torch.empty(312, embedding_dim))
        nn.init.normal_(self.text_projection, std=312 ** -0.5)
        # float64, as in the reference: torch.tensor([np.log(1/0.07)]) (:111) is fp64, which
        # promotes logits and the loss to fp64 there (the HIP path computes them in fp32)
        self.logit_scale = nn.Parameter(torch.tensor([math.log(1 / 0.07)], dtype=torch.float64))

    def features(self, batch):
        f_img = self.image_encoder(batch["x-ray"])
        f_txt = self.text_encoder(**batch["caption_tokenized"])
        return f_img, f_txt

    def forward(self, batch):
        f_img, f_txt = self.features(batch)
        return clip_forward(f_img, f_txt, self.image_projection, self.text_projection,
                            self.logit_scale)

    def param_groups(self, projections_lr=None, image_encoder_lr=None, text_encoder_lr=None):
        """_configure_optimizer_parameters :186-243 / _get_param_group :245-297."""
        img = list(self.image_encoder.parameters())
        txt = list(self.text_encoder.parameters())
        proj = [self.image_projection, self.text_projection, self.logit_scale]
        assigned = set(img + txt + proj)
        groups = [{"params": [p for p in self.parameters() if p not in assigned],
                   "name": "remaining_params"}]
        for params, name, lr in ((proj, "projection_and_logitscale", projections_lr),
                                 (img, "image_encoder", image_encoder_lr),
                                 (txt, "text_encoder", text_encoder_lr)):
            g = {"params": params, "name": name}
            if lr is not None:
                if lr < 0:
                    raise ValueError(f"VisionLanguageModule: {name} scale learning rate must be a non-negative value.")
                if lr == 0:
                    for p in params:
                        p.requires_grad = False
                    continue
                g["lr"] = lr
            groups.append(g)
        return groups


def global_batch_loss(logits_rows_fn, img_emb_all, txt_emb_all, logit_scale):
    """Definition of the data-parallel loss: embeddings of all
    ranks concatenated (each rank's BN over its own shard), then the reference
    _compute_loss over the N x N logits."""
    s = torch.clamp(logit_scale.exp(), max=100)
    logits = (img_emb_all @ txt_emb_all.T) * s
    return compute_loss(logits)

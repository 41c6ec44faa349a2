"""Generate golden vectors by running the REFERENCE's own hot-path code.

Run in the build container (where /root/reference exists):
    python tests/golden/make_golden.py
The reference never travels to the GPU box; only the small .pt fixtures written
here do (loaded with torch.load(weights_only=True)).

The reference module src/models/pretrain/VisionLanguageModule.py is imported
unmodified.  Third-party packages absent from this image are replaced by
minimal stand-ins that carry no hot-path arithmetic:
  lightning.LightningModule -> nn.Module + save_hyperparameters/log/device
  torchmetrics.MeanMetric   -> running mean
  timm.create_model         -> oracle.resnet34.create_model (architecture restatement)
  src.data.DownstreamDataModule -> empty class (downstream data is out of scope)
  transformers.AutoModel.from_pretrained -> local BertModel(TinyBERT config)
    (hub weights unavailable offline; deterministic recipe weights instead)
The reference's forward (:441-461), _compute_loss (:532-554), training_step
(:634-645), configure_optimizers/_configure_optimizer_parameters (:130-243),
precision@k (:364-400) and recall@k (:402-439) then run as written.
"""
import functools
import inspect
import math
import os
import sys
import types

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("VLP_REFERENCE", "/root/reference")
sys.path.insert(0, ROOT)

from oracle import weights as W  # noqa: E402
from oracle.clip import make_bert  # noqa: E402
from tests.golden.synth import synth_batch  # noqa: E402

TEXT_DROPOUT = 0.0  # parity runs: dropout off (train-mode BN stays on)


def _install_stubs():
    import transformers  # must be imported before the timm stand-in exists

    class AttributeDict(dict):
        def __getattr__(self, k):
            try:
                return self[k]
            except KeyError as e:
                raise AttributeError(k) from e

        def __setattr__(self, k, v):
            self[k] = v

    class LightningModule(torch.nn.Module):
        def save_hyperparameters(self, logger=True):
            fr = inspect.currentframe().f_back
            loc = dict(fr.f_locals)
            hp = AttributeDict()
            for k, v in loc.items():
                if k in ("self", "__class__"):
                    continue
                if k == "kwargs":
                    hp.update(v)
                else:
                    hp[k] = v
            object.__setattr__(self, "_hp", hp)

        @property
        def hparams(self):
            return self._hp

        @property
        def device(self):
            return next(self.parameters()).device

        def log(self, *a, **k):
            pass

    L = types.ModuleType("lightning")
    L.LightningModule = LightningModule
    sys.modules["lightning"] = L

    class MeanMetric:
        def __init__(self):
            self.reset()

        def reset(self):
            self.s, self.n = 0.0, 0.0

        def update(self, v, w=1.0):
            self.s += float(v) * w
            self.n += w

        def compute(self):
            return self.s / max(self.n, 1e-12)

    tm = types.ModuleType("torchmetrics")
    tm.MeanMetric = MeanMetric
    sys.modules["torchmetrics"] = tm

    from oracle.resnet34 import create_model
    timm = types.ModuleType("timm")
    timm.create_model = create_model
    sys.modules["timm"] = timm

    dm = types.ModuleType("src.data.DownstreamDataModule")

    class DownstreamDataModule:
        pass

    dm.DownstreamDataModule = DownstreamDataModule
    sys.modules["src.data.DownstreamDataModule"] = dm

    transformers.AutoModel.from_pretrained = classmethod(
        lambda cls, *a, **k: make_bert(TEXT_DROPOUT))


def import_reference():
    _install_stubs()
    sys.path.insert(0, REF)
    cwd = os.getcwd()
    os.chdir(REF)  # the module reads logging.conf from the CWD (:23)
    try:
        import src.models.pretrain.VisionLanguageModule as ref
    finally:
        os.chdir(cwd)
    return ref


def build_reference_model(ref, seed=0):
    model = ref.VisionLanguageModule(
        image_model="resnet34", text_encoder_model="tinybert",
        optimizer=functools.partial(torch.optim.AdamW, lr=5e-5),
        deduplicate=False, masked_loss=False, image_embedding_dim=512,
        text_embedding_dim=312, embedding_dim=128)
    W.apply_recipe(model, seed)
    return model


class _Fixed(torch.nn.Module):
    def __init__(self, t):
        super().__init__()
        self.t = t

    def forward(self, *a, **k):
        return self.t


def head_case(ref, B, seed, logit_scale=None):
    """Reference forward + _compute_loss on given features (encoders bypassed)."""
    model = build_reference_model(ref, 0)
    g = torch.Generator().manual_seed(1000 + seed)
    f_img = torch.randn(B, 512, generator=g).requires_grad_()
    f_txt = torch.randn(B, 312, generator=g).requires_grad_()
    if logit_scale is not None:
        with torch.no_grad():
            model.logit_scale.fill_(logit_scale)
    model.image_encoder = _Fixed(f_img)
    model.text_encoder = _Fixed(f_txt)
    batch = {"x-ray": None, "caption_tokenized": {}}
    logits, ie, te = model(batch)
    loss, li, lt = model._compute_loss(logits, deduplicate=False, masked=False)
    loss.backward()
    small = B <= 8
    out = {
        "B": torch.tensor(B), "seed": torch.tensor(seed),
        "logit_scale": model.logit_scale.detach().clone(),
        "loss": loss.detach(), "image_loss": li.detach(), "text_loss": lt.detach(),
        "d_logit_scale": model.logit_scale.grad,
        "d_image_projection_rows16": model.image_projection.grad[:16].clone(),
        "d_text_projection_rows16": model.text_projection.grad[:16].clone(),
        "d_image_projection_norm": model.image_projection.grad.norm(),
        "d_text_projection_norm": model.text_projection.grad.norm(),
    }
    rows = slice(None) if small else slice(0, 16)
    for k, v in (("logits", logits), ("img_emb", ie), ("txt_emb", te),
                 ("d_f_img", f_img.grad), ("d_f_txt", f_txt.grad)):
        out[k + ("" if small else "_rows16")] = v.detach()[rows].clone()
    if not small:
        out["logits_norm"] = logits.detach().norm()
        out["d_f_img_norm"] = f_img.grad.norm()
        out["d_f_txt_norm"] = f_txt.grad.norm()
    return out


def direction_case(ref, B=8, seed=1):
    """Gradients of the per-direction losses (the reference returns image_loss /
    text_loss as autograd tensors, :550-552): image_loss alone, and
    0.7 * loss + 1.3 * text_loss, through the reference forward + _compute_loss."""
    out = {"B": torch.tensor(B), "seed": torch.tensor(seed)}
    for tag, wl, wi, wt in (("image_only", 0.0, 1.0, 0.0), ("mixed", 0.7, 0.0, 1.3)):
        model = build_reference_model(ref, 0)
        g = torch.Generator().manual_seed(1000 + seed)
        f_img = torch.randn(B, 512, generator=g).requires_grad_()
        f_txt = torch.randn(B, 312, generator=g).requires_grad_()
        model.image_encoder = _Fixed(f_img)
        model.text_encoder = _Fixed(f_txt)
        logits, ie, te = model({"x-ray": None, "caption_tokenized": {}})
        loss, li, lt = model._compute_loss(logits, deduplicate=False, masked=False)
        (wl * loss + wi * li + wt * lt).backward()
        out[tag] = {"weights": torch.tensor([wl, wi, wt]), "d_f_img": f_img.grad.clone(),
                    "d_f_txt": f_txt.grad.clone(), "d_logit_scale": model.logit_scale.grad.clone(),
                    "d_image_projection_rows16": model.image_projection.grad[:16].clone(),
                    "d_text_projection_rows16": model.text_projection.grad[:16].clone()}
    return out


def head_inputs(B, seed):
    """Regenerate the head-case features exactly as head_case drew them."""
    g = torch.Generator().manual_seed(1000 + seed)
    return torch.randn(B, 512, generator=g), torch.randn(B, 312, generator=g)


def gathered_case(ref, world=8, B=256, E=128, seed=7):
    """Global-batch definition: N = world*B embeddings through the reference
    _compute_loss; stored as reductions to stay small."""
    model = build_reference_model(ref, 0)
    g = torch.Generator().manual_seed(seed)
    N = world * B
    ie = torch.nn.functional.normalize(torch.randn(N, E, generator=g)).requires_grad_()
    te = torch.nn.functional.normalize(torch.randn(N, E, generator=g)).requires_grad_()
    ls = model.logit_scale
    logits = (ie @ te.T) * torch.clamp(ls.exp(), max=100)   # forward :456-459
    loss, li, lt = model._compute_loss(logits, deduplicate=False, masked=False)
    loss.backward()
    return {"world": torch.tensor(world), "B": torch.tensor(B), "E": torch.tensor(E),
            "seed": torch.tensor(seed), "loss": loss.detach(), "image_loss": li.detach(),
            "text_loss": lt.detach(), "d_logit_scale": ls.grad.clone(),
            "d_img_rows_0_8": ie.grad[:8].clone(), "d_txt_rows_0_8": te.grad[:8].clone(),
            "d_img_norm": ie.grad.norm(), "d_txt_norm": te.grad.norm()}


def step_case(ref, B=4, H=64, T=12, seed=0, data_seed=0):
    """Full training step through the reference code at a reduced shape."""
    torch.manual_seed(0)
    model = build_reference_model(ref, seed)
    batch = synth_batch(B, H, T, data_seed)
    out = {"B": torch.tensor(B), "H": torch.tensor(H), "T": torch.tensor(T),
           "seed": torch.tensor(seed), "data_seed": torch.tensor(data_seed)}
    # eval-mode linear-probe embedding (LinearProbeCallback._extract_features :92-116)
    model.eval()
    with torch.no_grad():
        out["probe_features"] = model.image_encoder(batch["x-ray"]).clone()
        lg, ie, te = model(batch)
        out["eval_loss"] = model._compute_loss(lg, deduplicate=False, masked=False)[0]
    model.train()
    model.on_train_epoch_start()
    loss = model.training_step(batch)                                       # :634-645
    with torch.no_grad():
        lg, ie, te = model(batch)  # same batch stats again (forward is deterministic w/o dropout)
    out["train_loss"] = loss.detach()
    out["logits"] = lg.detach()
    out["img_emb"] = ie.detach()
    out["txt_emb"] = te.detach()
    # reset running stats side effect of the extra forward: re-run cleanly
    model = build_reference_model(ref, seed)
    model.train()
    model.on_train_epoch_start()
    opt = model.configure_optimizers()["optimizer"]                         # :130-184
    opt.zero_grad()
    loss = model.training_step(batch)
    loss.backward()
    before = {k: v.detach().clone() for k, v in model.named_parameters()}
    grad_norm = {k: (v.grad.norm().item() if v.grad is not None else -1.0)
                 for k, v in model.named_parameters()}
    opt.step()
    names = sorted(before)
    out["param_names"] = names
    out["grad_norm"] = torch.tensor([grad_norm[k] for k in names], dtype=torch.float64)
    p = dict(model.named_parameters())
    out["delta_norm"] = torch.tensor([(p[k].detach() - before[k]).norm().item() for k in names],
                                     dtype=torch.float64)
    sd = model.state_dict()
    out["bn1_running_mean"] = sd["image_encoder.model.bn1.running_mean"].clone()
    out["bn1_running_var"] = sd["image_encoder.model.bn1.running_var"].clone()
    out["l4_bn2_running_var"] = sd["image_encoder.model.layer4.2.bn2.running_var"].clone()
    out["group_names"] = [g.get("name") for g in opt.param_groups]
    out["group_sizes"] = torch.tensor([sum(q.numel() for q in g["params"]) for g in opt.param_groups])
    return out


def known_answers(ref):
    model = build_reference_model(ref, 0)
    res = {}
    for name, m in (("nb14", [[1, .5, 1], [.5, 1, .3], [1, .3, 1]]),
                    ("asym", [[2, .1, -1], [.3, 1.5, .2], [0, -.5, .9]])):
        lg = torch.tensor(m, dtype=torch.float32)
        loss, li, lt = model._compute_loss(lg, deduplicate=False, masked=False)
        res[name] = torch.stack([loss, li, lt])
        res[name + "_logits"] = lg
    e = torch.tensor([[1, 1], [1, 1.1], [2, 1], [3, 1]], dtype=torch.float32)
    lab = torch.tensor([0, 0, 1, 1])
    res["prec_k1"] = torch.tensor(model.precision_at_k_on_image_embeddings(e, lab, ks=[1])[1])
    g = torch.Generator().manual_seed(5)
    ie, te = torch.randn(32, 16, generator=g), torch.randn(32, 16, generator=g)
    lab = torch.randint(0, 2, (32,), generator=g)
    res["retr_img"], res["retr_txt"], res["retr_lab"] = ie, te, lab
    res["prec"] = torch.tensor([model.precision_at_k_on_image_embeddings(ie, lab, ks=[3, 5, 10, 15])[k]
                                for k in (3, 5, 10, 15)])
    res["recall"] = torch.tensor([model.recall_at_k_on_image_text_retreival(ie, te, ks=[3, 5, 10, 15])[k]
                                  for k in (3, 5, 10, 15)])
    return res


def main():
    ref = import_reference()
    if sys.argv[1:] == ["directions"]:   # r5: only the per-direction fixture
        torch.save(direction_case(ref), os.path.join(HERE, "head_dir_B8_s1.pt"))
        return
    torch.save(known_answers(ref), os.path.join(HERE, "known_answers.pt"))
    for B, seed, ls in ((4, 0, None), (8, 1, None), (8, 2, math.log(150.0)), (256, 3, None)):
        tag = f"head_B{B}_s{seed}"
        torch.save(head_case(ref, B, seed, ls), os.path.join(HERE, tag + ".pt"))
    torch.save(gathered_case(ref), os.path.join(HERE, "gathered_N2048.pt"))
    torch.save(step_case(ref), os.path.join(HERE, "step_B4_H64_T12.pt"))
    print("golden vectors written to", HERE)


if __name__ == "__main__":
    main()

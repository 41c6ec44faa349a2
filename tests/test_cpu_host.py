"""CPU: the C-ABI library and the host-side mirror of the reference API.

No compute call reaches the device here: the library is loaded and its exports
are checked against include/vlp_hip.h; the module is constructed on CPU
(parameters only) to check the reference's API contract (names, parameter
count, optimizer groups, error behaviour; VisionLanguageModule.py citations).
"""
import functools
import os
import subprocess
import sys

import pytest
import torch

from tests.conftest import PKG, ROOT

LIB = os.path.join(PKG, "vlp_amd", "libvlp_hip.so")
HDR = os.path.join(ROOT, "include", "vlp_hip.h")


def _need_lib():
    if not os.path.exists(LIB):
        pytest.skip("libvlp_hip.so not built (run __graft_entry__.build())")


def test_header_parses_and_every_symbol_is_exported():
    _need_lib()
    from vlp_amd import _lib
    protos = _lib.parse_header(HDR)
    assert len(protos) >= 40
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l and l.split()[-1].startswith("vlp_")}
    missing = set(protos) - exported
    extra = exported - set(protos)
    assert not missing, f"declared but not exported: {sorted(missing)}"
    assert not extra, f"exported but not declared in include/vlp_hip.h: {sorted(extra)}"


def test_library_loads_with_typed_bindings():
    _need_lib()
    from vlp_amd import _lib
    L = _lib.lib()
    for name, p in L.protos.items():
        fn = L._fns[name]
        assert len(fn.argtypes) == len(p["args"]), name
    # pure-host entry point: no device work
    assert L._dll.vlp_abi_version() == 3


def test_every_declaration_cites_the_reference():
    text = open(HDR).read()
    # each section of the ABI names the reference call it replaces (file:line)
    sections = text.split("/* ----------------")[1:]
    assert len(sections) >= 5
    import re
    for sec in sections:
        assert re.search(r"\w+\.py:\d+", sec.split("*/")[0]), sec[:80]


def test_missing_library_fails_loudly(tmp_path):
    code = ("import sys; sys.path[:0]=[%r, %r]\n"
            "try:\n    from vlp_amd import _lib; _lib.lib()\nexcept ImportError as e:\n"
            "    print('IMPORTERROR', e)\n") % (ROOT, PKG)
    env = dict(os.environ, VLP_HIP_LIB=str(tmp_path / "nope.so"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=120)
    assert "IMPORTERROR" in r.stdout and "no CPU fallback" in r.stdout


# ---------------- host mirror of the reference module API ----------------

def _module(**kw):
    from src.models.pretrain.VisionLanguageModule import VisionLanguageModule
    args = dict(image_model="resnet34", text_encoder_model="tinybert",
                optimizer=functools.partial(torch.optim.AdamW, lr=5e-5), deduplicate=False,
                masked_loss=False, image_embedding_dim=512, text_embedding_dim=312, embedding_dim=128,
                device="cpu")
    args.update(kw)
    return VisionLanguageModule(**args)


@pytest.fixture(scope="module")
def module():
    return _module()


def test_parameter_count_and_names_match_reference(module):
    # 35 740 393 parameters incl. the unused BERT pooler
    assert sum(p.numel() for p in module.parameters()) == 35_740_393
    from oracle.clip import OracleVLP
    ref = {k: v.shape for k, v in OracleVLP(128).state_dict().items() if "num_batches_tracked" not in k}
    ours = {k: v.shape for k, v in module.state_dict().items() if "num_batches_tracked" not in k}
    assert ours.keys() == ref.keys()
    for k in ref:
        assert tuple(ours[k]) == tuple(ref[k]), k


def test_state_dict_roundtrip_with_reference_keys(module, tmp_path):
    from oracle import weights as W
    from oracle.clip import OracleVLP
    o = OracleVLP(128)
    W.apply_recipe(o, 3)
    m = _module()
    m.load_state_dict(o.state_dict(), strict=False)
    sd = m.state_dict()
    for k, v in o.state_dict().items():
        if "num_batches_tracked" in k:
            continue
        torch.testing.assert_close(sd[k].float(), v.float(), rtol=0, atol=0, msg=k)
    # parameters are views into the flat arenas: loading wrote through
    assert m.image_projection.data_ptr() == m._head.arena.view("image_projection").data_ptr()
    ck = tmp_path / "vlp.ckpt"
    torch.save({"state_dict": sd, "hyper_parameters": {
        "image_model": "resnet34", "text_encoder_model": "tinybert", "optimizer": None,
        "deduplicate": False, "masked_loss": False, "image_embedding_dim": 512,
        "text_embedding_dim": 312, "embedding_dim": 128}}, ck)
    m2 = type(m).load_from_checkpoint(str(ck), device="cpu")
    torch.testing.assert_close(m2.logit_scale, m.logit_scale)


def test_optimizer_groups_follow_reference(module):
    # VisionLanguageModule.py:130-297: groups, per-group lr, lr=0 freezes, lr<0 raises
    opt = module.configure_optimizers()["optimizer"]
    names = [g.get("name") for g in opt.param_groups]
    assert names == ["remaining_params", "projection_and_logitscale", "image_encoder", "text_encoder"]
    assert [len(g["params"]) for g in opt.param_groups][1:] == [3, 108, 71]
    m = _module(text_encoder_lr=0.0, projections_lr=1e-3)
    opt = m.configure_optimizers()["optimizer"]
    names = [g.get("name") for g in opt.param_groups]
    assert "text_encoder" not in names
    assert not any(p.requires_grad for p in m.text_encoder.parameters())
    assert [g["lr"] for g in opt.param_groups if g.get("name") == "projection_and_logitscale"] == [1e-3]
    with pytest.raises(ValueError):
        _module(image_encoder_lr=-1.0).configure_optimizers()


def test_constructor_contract():
    # :87-92 deduplicate forces masked_loss off; :46-49 unsupported text model -> ValueError
    m = _module(deduplicate=True, masked_loss=True)
    assert m.hparams["masked_loss"] is False
    with pytest.raises(ValueError):
        _module(text_encoder_model="gpt2")
    # the HIP contrastive head takes 4 <= E <= 256, E % 4 == 0 (the reference configs
    # use 32 and 128): anything else is refused at construction, not mid-step
    assert _module(embedding_dim=32)._head.embedding_dim == 32
    for bad in (30, 512):
        with pytest.raises(ValueError, match="embedding_dim"):
            _module(embedding_dim=bad)
    # bf16: the projection matmuls need E % 8 == 0 (16-B bf16 rows); fp32 keeps E % 4
    assert _module(embedding_dim=36, compute_dtype="fp32")._head.embedding_dim == 36
    with pytest.raises(ValueError, match="embedding_dim"):
        _module(embedding_dim=36, compute_dtype="bf16")


def test_validation_dataloader_index_contract(module):
    # :671-678 -> indices other than 0/1 raise ValueError; checked on the logging
    # branch by a stub forward (no device work)
    logits = torch.eye(4) * 5
    m = module

    class Stub:
        pass
    orig = type(m).forward
    try:
        type(m).forward = lambda self, b: (logits, torch.eye(4), torch.eye(4))
        m._compute_loss = lambda lg, *a, **k: (torch.tensor(0.5), torch.tensor(0.5), torch.tensor(0.5))
        batch = {"label": torch.zeros(4, dtype=torch.long), "caption": ["a"] * 4}
        m.on_validation_epoch_start()
        m.validation_step(batch, 0, 0)
        m.validation_step(batch, 0, 1)
        with pytest.raises(ValueError):
            m.validation_step(batch, 0, 2)
    finally:
        type(m).forward = orig
        del m._compute_loss


def test_retrieval_metrics_match_reference_known_answers(module):
    from tests.conftest import ROOT as R
    ka = torch.load(os.path.join(R, "tests", "golden", "known_answers.pt"), weights_only=True)
    e = torch.tensor([[1, 1], [1, 1.1], [2, 1], [3, 1]], dtype=torch.float32)
    assert module.precision_at_k_on_image_embeddings(e, torch.tensor([0, 0, 1, 1]), [1])[1] == 1.0
    p = module.precision_at_k_on_image_embeddings(ka["retr_img"], ka["retr_lab"], [3, 5, 10, 15])
    r = module.recall_at_k_on_image_text_retreival(ka["retr_img"], ka["retr_txt"], [3, 5, 10, 15])
    assert [p[k] for k in (3, 5, 10, 15)] == pytest.approx(ka["prec"].tolist(), abs=1e-7)
    assert [r[k] for k in (3, 5, 10, 15)] == pytest.approx(ka["recall"].tolist(), abs=1e-7)
    assert module.recall_at_k_on_image_text_retreival(e, e, [1, 2]) == {1: 1.0, 2: 1.0}


def test_fused_adamw_span_grouping():
    # every parameter with a gradient inside one arena collapses into ONE
    # contiguous launch span per arena (alignment gaps hold no other parameter)
    from vlp_amd.optim import FusedAdamW
    m = _module()
    opt = m.configure_optimizers()["optimizer"]
    assert isinstance(opt, FusedAdamW)
    for g in opt.param_groups:
        for p in g["params"]:
            arena, o, n = opt._loc[id(p)]
            p.grad = arena.grad[o:o + n].view_as(p)
    img = [g for g in opt.param_groups if g.get("name") == "image_encoder"][0]
    txt = [g for g in opt.param_groups if g.get("name") == "text_encoder"][0]
    assert len(opt._spans(img)) == 1
    # the BERT pooler never gets a gradient (only CLS is used): it splits the span at most once
    txt["params"][-1].grad = None
    assert len(opt._spans(txt)) <= 2
    with pytest.raises(ValueError):
        FusedAdamW([torch.nn.Parameter(torch.zeros(3))], arenas=[])


def test_augment_maps_match_oracle():
    """Host half of the device augmentation: the composed output->source maps
    equal the oracle's per-transform composition (oracle/prep.py)."""
    import torch
    import oracle.prep as op
    from vlp_amd.augment import Augmenter
    a = Augmenter(seed=3)
    prm = a.draw(64)
    assert torch.allclose(a.maps(prm), op.source_maps(prm), atol=1e-12)

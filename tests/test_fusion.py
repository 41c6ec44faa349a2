"""Late-fusion finetune (reference src/models/baseline/FusionModule.py,
src/utils/coral_loss/coral.py).

CPU: the oracle and the product CORAL / _compute_loss against golden vectors
produced by the reference's own coral() and FusionModule._compute_loss
(tests/golden/make_fusion_golden.py).
GPU: FusionModule on the HIP ResNet34 tower (fp32 parity mode) against the CPU
oracle on the same weights and batch: logits and loss |d| <= 1e-4, parameter
gradients rel-L2 <= 1e-3; bf16 throughput mode loss within 5e-2; a VLP
checkpoint's image_encoder.model.* weights load into image_network.
"""
import functools
import os
import types

import pytest
import torch

from oracle import weights as W
from oracle.fusion import OracleFusion, coral as oracle_coral
from src.utils.coral_loss.coral import coral

GOLD = torch.load(os.path.join(os.path.dirname(__file__), "golden", "fusion_loss.pt"), weights_only=True)


def _coral_cases():
    return [k for k in GOLD if k.startswith("coral_")]


@pytest.mark.parametrize("name", _coral_cases())
def test_coral_vs_reference_golden(name):
    c = GOLD[name]
    for fn in (coral, oracle_coral):
        s = c["source"].clone().requires_grad_()
        t = c["target"].clone().requires_grad_()
        loss = fn(s, t)
        assert torch.allclose(loss, c["loss"], rtol=1e-5, atol=1e-7), (name, loss.item(), c["loss"].item())
        if "grad_source" in c:
            gs, gt = torch.autograd.grad(loss, (s, t))
            assert torch.allclose(gs, c["grad_source"], rtol=1e-4, atol=1e-8)
            assert torch.allclose(gt, c["grad_target"], rtol=1e-4, atol=1e-8)
    assert torch.isnan(coral(torch.ones(1, 3), torch.randn(4, 3)))       # one-sample domain: NaN as the reference


def test_compute_loss_vs_reference_golden():
    from src.models.baseline.FusionModule import FusionModule
    for case in GOLD["compute_loss"]:
        lam = float(case["coral_lambda"])
        me = types.SimpleNamespace(label_weights=case["label_weights"],
                                   hparams=types.SimpleNamespace(coral_lambda=lam))
        o = OracleFusion(tuple(case["label_weights"].tolist()), lam)
        for fn in (lambda f, lg: FusionModule._compute_loss(me, f, lg, case["labels"], case["dataset"]),
                   lambda f, lg: o.compute_loss(f, lg, case["labels"], case["dataset"])):
            f = case["features"].clone().requires_grad_()
            lg = case["logits"].clone().requires_grad_()
            tot, cls, cor = fn(f, lg)
            assert abs(tot.item() - case["loss"].item()) < 1e-6
            assert abs(cls.item() - case["classification_loss"].item()) < 1e-6
            assert abs(float(cor.detach()) - case["coral_loss"].item()) < 1e-6
            gf, gl = torch.autograd.grad(tot, (f, lg), allow_unused=True)
            assert torch.allclose(gl, case["grad_logits"], rtol=1e-5, atol=1e-8)
            gf = torch.zeros_like(f) if gf is None else gf
            assert torch.allclose(gf, case["grad_features"], rtol=1e-4, atol=1e-9)


def _fusion_batch(B, H, seed=0):
    g = torch.Generator().manual_seed(seed)
    x_u8 = torch.randint(0, 256, (B, 1, H, H), generator=g, dtype=torch.uint8)
    x = ((x_u8.float() - 127.5) / 73.9).repeat(1, 3, 1, 1)
    site = torch.nn.functional.one_hot(torch.randint(0, 9, (B,), generator=g), 9).float()
    age = torch.nn.functional.one_hot(torch.randint(0, 4, (B,), generator=g), 4).float()
    sex = torch.nn.functional.one_hot(torch.randint(0, 2, (B,), generator=g), 2).float()
    return {"x-ray": x, "x-ray-u8": x_u8, "tumor": torch.tensor([0, 1] * (B // 2)),
            "dataset": ["INTERNAL", "INTERNAL", "BTXRD", "BTXRD", "INTERNAL", "BTXRD"][:B] if B <= 6
            else ["INTERNAL" if i % 2 else "BTXRD" for i in range(B)],
            "anatomy_site_encoded": site, "age_encoded": age, "sex_encoded": sex}


def _oracle(seed=0, lw=(0.7, 2.0), lam=0.5):
    torch.manual_seed(seed)
    o = OracleFusion(lw, lam)
    sd = o.state_dict()
    for k in sd:
        if k.startswith("image_network.trunk."):
            rk = k.replace("image_network.trunk.", "image_encoder.model.")
            sd[k] = W.value_for(rk, sd[k].shape, seed).to(sd[k].dtype)
    o.load_state_dict(sd)
    return o


def _hip(dtype, o, lw=(0.7, 2.0), lam=0.5):
    from src.models.baseline.FusionModule import FusionModule
    m = FusionModule("resnet34", functools.partial(torch.optim.AdamW, lr=1e-3), label_weights=lw,
                     coral_lambda=lam, compute_dtype=dtype)
    m.load_state_dict(o.state_dict_hip_layout(), strict=True)
    return m


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


@pytest.mark.gpu
@pytest.mark.parametrize("B,H", [(6, 64), (8, 256)])
def test_fusion_step_vs_oracle_fp32(B, H):
    """fp32 HIP step vs the CPU oracle (FusionModule.py:318-390).  Per tensor
    rel-L2 <= 1e-3 at 64 px.  At 256 px (B = 8, layer 1 at 64 x 64 on the
    generic tiles) a ReLU whose pre-activation sits within rounding of 0 flips
    between any two fp32 implementations, so there the gate is the
    fp64 envelope of the VLP parity tests: with e(.) the rel-L2 against the
    oracle run in fp64, every tensor e(HIP) <= max(4 e(oracle fp32), 2e-2) and
    the tower's 36 conv weights as one vector e(HIP) <= max(2 e(oracle fp32), 5e-3)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    batch = _fusion_batch(B, H)
    o = _oracle()
    m = _hip("fp32", o)
    o.train()
    m.train()
    lo, fo = o(batch["x-ray"], batch["age_encoded"], batch["sex_encoded"], batch["anatomy_site_encoded"])
    Lo, _, Co = o.compute_loss(fo, lo, batch["tumor"], batch["dataset"])
    Lo.backward()
    loss = m.training_step(batch)
    loss.backward()
    torch.cuda.synchronize()
    lm, _ = m(batch["x-ray"], batch["age_encoded"], batch["sex_encoded"], batch["anatomy_site_encoded"])
    assert (lm.detach().cpu() - lo.detach()).abs().max().item() < 1e-4
    assert abs(loss.item() - Lo.item()) < 1e-4, (loss.item(), Lo.item())
    assert float(m.logged["train/coral_loss"].detach()) > 0.0
    og = {k.replace("image_network.trunk.", "image_network."): p.grad for k, p in o.named_parameters()}
    ref = og
    if H > 64:   # fp64 envelope
        o64 = _oracle().double()
        o64.train()
        l64, f64 = o64(*(batch[k].double() for k in ("x-ray", "age_encoded", "sex_encoded", "anatomy_site_encoded")))
        o64.compute_loss(f64, l64, batch["tumor"], batch["dataset"])[0].backward()
        ref = {k.replace("image_network.trunk.", "image_network."): p.grad for k, p in o64.named_parameters()}
    errs, envs, convs = {}, {}, ([], [], [])
    for k, p in m.named_parameters():
        if og[k] is None or og[k].norm() < 1e-6:    # biases feeding BatchNorm1d: analytically 0
            continue
        assert p.grad is not None, k
        errs[k] = _rel(p.grad, ref[k])
        envs[k] = 1e-3 if H <= 64 else max(4 * _rel(og[k], ref[k]), 2e-2)
        if k.startswith("image_network.") and p.dim() == 4:
            convs[0].append(p.grad.double().cpu().flatten())
            convs[1].append(og[k].double().flatten())
            convs[2].append(ref[k].double().flatten())
    worst = max(errs, key=lambda k: errs[k] / envs[k])
    tower = _rel(torch.cat(convs[0]), torch.cat(convs[2]))
    tower_env = 1e-3 if H <= 64 else max(2 * _rel(torch.cat(convs[1]), torch.cat(convs[2])), 5e-3)
    print(f"fusion fp32 B={B} {H}px: loss {loss.item():.6f} vs {Lo.item():.6f}; worst tensor {worst} "
          f"{errs[worst]:.2e} (envelope {envs[worst]:.2e}); tower conv vector {tower:.2e} (envelope {tower_env:.2e})")
    assert len(convs[0]) == 36
    for k, e in errs.items():
        assert e <= envs[k], (k, e, envs[k])
    assert tower <= tower_env, (tower, tower_env)


@pytest.mark.gpu
def test_fusion_bf16_u8_and_optimizer_step(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    B, H = 6, 64
    batch = _fusion_batch(B, H, seed=1)
    o = _oracle(seed=1)
    m32 = _hip("fp32", o)
    m16 = _hip("bf16", o)
    l32 = m32.training_step(batch).item()
    b16 = {k: v for k, v in batch.items() if k != "x-ray"}          # uint8 upload path
    opt = m16.configure_optimizers()["optimizer"]
    w0 = m16.image_network.conv1.weight.detach().clone()
    loss = m16.training_step(b16)
    loss.backward()
    opt.step()
    assert abs(loss.item() - l32) < 5e-2, (loss.item(), l32)
    assert not torch.equal(w0, m16.image_network.conv1.weight.detach())
    assert all(torch.isfinite(p).all() for p in m16.parameters())
    # vision_encoder_lr groups (:144-170)
    from src.models.baseline.FusionModule import FusionModule
    mg = FusionModule("resnet34", functools.partial(torch.optim.AdamW, lr=1e-3), vision_encoder_lr=1e-5)
    groups = mg.configure_optimizers()["optimizer"].param_groups
    assert [g["name"] for g in groups] == ["image_backbone", "head_and_remaining_parameters"]
    assert groups[0]["lr"] == 1e-5 and sum(p.numel() for p in groups[0]["params"]) == 21284672
    # a VLP checkpoint's image encoder initialises image_network (:82-113)
    from src.models.pretrain.VisionLanguageModule import VisionLanguageModule
    v = VisionLanguageModule("resnet34", "tinybert", functools.partial(torch.optim.AdamW, lr=5e-5),
                             False, False, 512, 312, 128, compute_dtype="bf16")
    W.apply_recipe(v, 3)
    path = tmp_path / "vlp.ckpt"
    torch.save({"state_dict": {k: t.detach().cpu() for k, t in v.state_dict().items()}}, path)
    mp = FusionModule("resnet34", functools.partial(torch.optim.AdamW, lr=1e-3), pretrained_vlp_module=str(path))
    assert torch.equal(mp.image_network.layer3.get_submodule("1").conv2.weight.cpu(),
                       v.image_encoder.model.layer3.get_submodule("1").conv2.weight.cpu())
    with pytest.raises(ValueError):
        FusionModule("alexnet", None)
    with pytest.raises(NotImplementedError):
        FusionModule("nest_small", None)


def test_state_dict_layout_matches_reference_keys():
    """timm resnet34(num_classes=10) + tabular MLP + combination keys; construction only (no compute)."""
    from src.models.baseline.FusionModule import FusionModule
    o = _oracle()
    m = FusionModule("resnet34", functools.partial(torch.optim.AdamW, lr=1e-3), device="cpu")
    m.load_state_dict(o.state_dict_hip_layout(), strict=True)
    assert sum(p.numel() for p in m.parameters()) == 21291329      # 21 284 672 trunk + 5130 fc + 1506 + 21
    assert torch.equal(m.image_network.fc.weight, o.image_network.fc.weight)
    assert "image_network.layer4.2.bn2.running_var" in m.state_dict()


@pytest.mark.gpu
def test_fusion_all_reduce_gradients_single_rank():
    """The trainer's DP hook on FusionModule: tower gradients alias the flat arena, so the
    reduction is one RCCL call over it plus one over the head (world 1: values unchanged)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import socket
    import torch.distributed as dist
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(s.getsockname()[1]))
    s.close()
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        o = _oracle(seed=2)
        m = _hip("bf16", o)
        opt = m.configure_optimizers()["optimizer"]
        batch = _fusion_batch(6, 64, seed=2)
        for _ in range(2):          # second step: gradients accumulate into the existing p.grad
            opt.zero_grad(set_to_none=False)
            m.training_step(batch).backward()
        tower = m.image_network
        p0 = tower.conv1.weight
        assert p0.grad.data_ptr() == tower.arena.gview("conv1.weight").data_ptr()
        before = {n: p.grad.clone() for n, p in m.named_parameters()}
        m.all_reduce_gradients(1)
        torch.cuda.synchronize()
        for n, p in m.named_parameters():
            assert torch.equal(p.grad, before[n]), n
    finally:
        dist.destroy_process_group()


def _oracle_from_hip(sd, lw=(0.7, 2.0), lam=0.5):
    """OracleFusion holding a HIP FusionModule state dict (the trunk under image_network.trunk.)."""
    o = OracleFusion(lw, lam)
    o.load_state_dict({("image_network.trunk." + k[len("image_network."):]
                        if k.startswith("image_network.") and not k.startswith("image_network.fc.") else k): v
                       for k, v in sd.items()})
    return o


@pytest.mark.gpu
def test_fusion_dp2_trainer_all_reduce(tmp_path):
    """BASELINE configs[4]'s data-parallel path at world size 2:
    two ranks (torch.distributed.run, gloo, both on the one GPU; tests/_fusion_dp_worker.py)
    each run one step of src/utils/trainer.py's Trainer.fit on their 6-row shard of a
    12-row batch, fp32 parity mode.  The trainer's DDP hook (FusionModule.all_reduce_gradients:
    one SUM all-reduce over the tower's flat arena, one over the head, x 1/world) must leave
    both ranks with bit-identical gradients that equal the mean of the two ranks' own
    (collective-free) gradients to fp32 rounding, and that mean must match the mean of the
    per-shard oracle gradients (per-rank BatchNorm statistics, as DDP) inside the strict
    fp64 envelope of the VLP parity tests: per tensor e(HIP) <= max(4 e(oracle fp32), 2e-3),
    e measured against the oracle run in fp64.  Weights: the module's own seeded init (as
    tests/test_gpu_dp.py), whose fp32 gradients are well conditioned; with the name-keyed
    recipe weights (live residual branches, 2 x 2 maps at layer 4 for B = 6 at 64 px) one
    of the two shards sits 1.3 % from fp64 in every tensor below layer 4 in a SINGLE-process
    HIP step as well (tools/diag_fusion_shards.py) -- the ReLU-flip sensitivity of
    test_gpu_model.grad_envelope_check, not the all-reduce."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import subprocess
    import sys
    from tests.conftest import ROOT
    B, H = 6, 64
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1",
           "--nnodes=1", "--nproc-per-node", "2", os.path.join(ROOT, "tests", "_fusion_dp_worker.py"),
           str(tmp_path), str(B), str(H)]
    r = subprocess.run(cmd, env=dict(os.environ, OMP_NUM_THREADS="4"), timeout=300, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = [torch.load(tmp_path / f"r{k}.pt", weights_only=True) for k in range(2)]
    g0, g1 = res[0]["grads"], res[1]["grads"]
    assert g0.keys() == g1.keys() and len(g0) > 100
    for k in g0:
        assert torch.equal(g0[k], g1[k]), f"ranks disagree after the all-reduce: {k}"
        mean = (res[0]["local"][k] + res[1]["local"][k]) * 0.5
        assert torch.allclose(g0[k], mean, rtol=1e-6, atol=1e-12), k
    assert not torch.equal(res[0]["local"]["image_network.conv1.weight"], res[1]["local"]["image_network.conv1.weight"])
    init = torch.load(tmp_path / "init.pt", weights_only=True)
    full = _fusion_batch(2 * B, H)
    refs, shard64, losses = {}, [{}, {}], []
    for dt in (torch.float32, torch.float64):
        ref = refs[dt] = {}
        for rk in range(2):
            o = _oracle_from_hip(init).to(dt)
            o.train()
            sl = slice(rk * B, (rk + 1) * B)
            lo, fo = o(*(full[k][sl].to(dt) for k in ("x-ray", "age_encoded", "sex_encoded", "anatomy_site_encoded")))
            L = o.compute_loss(fo, lo, full["tumor"][sl], full["dataset"][sl])[0]
            L.backward()
            if dt == torch.float64:
                losses.append(L.item())
            for k, p in o.named_parameters():
                if p.grad is not None:
                    kk = k.replace("image_network.trunk.", "image_network.")
                    ref[kk] = ref.get(kk, 0) + p.grad.double() / 2
                    if dt == torch.float64:
                        shard64[rk][kk] = p.grad.double()
    for rk in range(2):
        assert abs(res[rk]["loss"] - losses[rk]) < 1e-4, (rk, res[rk]["loss"], losses[rk])
    checked, bad, rows = 0, [], []
    for k, g in g0.items():
        r64 = refs[torch.float64].get(k)
        if r64 is None or r64.norm() < 1e-6:
            # biases feeding BatchNorm1d, and the residual-branch convs behind timm's
            # zero-initialised last BN: analytically 0 -- HIP's must be too
            assert g.double().norm().item() <= 1e-6, (k, g.norm().item())
            continue
        e, e32 = _rel(g, r64), _rel(refs[torch.float32][k], r64)
        env = max(4 * e32, 2e-3)
        rows.append((e / env, k, e, e32, [_rel(res[rk]["local"][k], shard64[rk][k]) for rk in range(2)]))
        if not (e <= env or (g.double() - r64).norm().item() <= 1e-6):
            bad.append(k)
        checked += 1
    rows.sort(reverse=True)
    for row in rows[:12]:
        print("fusion dp2: %.2f of envelope  %s  e=%.2e e32=%.2e  per-rank local e=%s" % (row[0], row[1], row[2], row[3],
                                                                                        ["%.2e" % v for v in row[4]]))
    assert not bad, bad[:10]
    assert checked >= 50, checked     # stem, downsample convs, every BN, fc, tabular and combination layers

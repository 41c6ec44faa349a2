"""src/train.py / Hydra-config / src/data collation boundary (SURVEY §8(a) collation
row, §8(b) config boundary and loop semantics).  CPU tests: config composition,
instantiation, the synthetic data module's batch schema and normalisation
(checked against the oracle-side synth.normalize_u8 formula, PretrainDataModule.py:165-171),
and the Trainer's step order with a plain-torch stand-in module."""
import functools

import pytest
import torch

from src.data.PretrainDataModule import (DevicePrefetcher, PairCollator, PretrainDataModule,
                                         SyntheticRadiographCaptions, normalize_u8)
from src.utils.config import compose, instantiate
from src.utils.trainer import Trainer
from tests.golden import synth


def test_compose_experiment_and_overrides():
    c = compose("train", ["experiment=pretrain/pretrain_resnet34_tinybert", "data.batch_size=4",
                          "scheduler=cosine", "trainer.max_epochs=7"])
    assert c["data"]["_target_"] == "src.data.PretrainDataModule.PretrainDataModule"
    assert c["data"]["batch_size"] == 4 and c["data"]["tokenizer"] == "tinybert"
    assert c["model"]["text_encoder_model"] == "tinybert"
    assert c["model"]["embedding_dim"] == 128 and c["model"]["text_embedding_dim"] == 312
    assert c["model"]["optimizer"]["lr"] == 5e-5                  # experiment optimizer.lr
    assert c["model"]["scheduler"]["T_max"] == 7                   # ${trainer.max_epochs} after the CLI
    opt = instantiate(c["model"]["optimizer"])
    assert isinstance(opt, functools.partial) and opt.func is torch.optim.AdamW and opt.keywords["lr"] == 5e-5
    assert isinstance(instantiate(c["trainer"]), Trainer)            # lightning Trainer target, absent here


def test_compose_defaults_and_errors():
    # the reference defaults list (configs/train.yaml:5-20), group by group
    c = compose("train", [])
    assert c["seed"] == 42 and c["task_name"] == "train"
    assert c["data"]["_target_"] == "src.data.DownstreamDataModule.DownstreamDataModule"
    assert c["model"]["_target_"] == "src.models.baseline.OnlyImagingModule.OnlyImagingModule"
    assert c["model"]["model"] == "resnet50"
    assert set(c["callbacks"]) == {"lr_monitor", "checkpoint_internal", "checkpoint_btxrd", "early_stopping_internal",
                                   "early_stopping_btxrd", "snapshot_btxrd", "snapshot_internal", "snapshot_combined"}
    assert c["logger"]["wandb"]["name"] == "resnet50"                     # ${model.model}
    assert c["paths"]["output_dir"].startswith(c["paths"]["work_dir"])   # ${hydra:runtime.output_dir}
    assert c["scheduler"]["_target_"] == "torch.optim.lr_scheduler.CosineAnnealingLR"
    assert c["model"]["scheduler"]["T_max"] == c["trainer"]["max_epochs"] == 10
    with pytest.raises(NotImplementedError):
        instantiate(c["model"])                                           # baseline outside the hot path
    c = compose("train", ["experiment=pretrain/pretrain_resnet34_tinybert"])
    assert c["scheduler"] == {} and c["model"]["scheduler"] == {}       # no_scheduler
    assert set(c["callbacks"]) == {"lr_monitor", "checkpoint_combined", "early_stopping_combined",
                                   "snapshot_combined"}
    assert c["callbacks"]["checkpoint_combined"]["monitor"] == "val/combined/loss"
    assert c["model"]["downstream_datamodule"]["_target_"] == "src.data.DownstreamDataModule.DownstreamDataModule"
    assert c["logger"]["wandb"]["name"] == "resnet34_tinybert"
    vl = compose("train", ["model=vision_language"])["model"]
    assert vl["text_encoder_model"] == "distilbert" and vl["downstream_datamodule"] == "downstream"
    with pytest.raises(FileNotFoundError):
        compose("train", ["experiment=pretrain/does_not_exist"])
    with pytest.raises(ValueError):
        compose("train", ["no_equals_sign"])
    c = compose("train", ["experiment=pretrain/pretrain_resnet34_tinybert_mi355x"])
    assert (c["data"]["batch_size"], c["data"]["image_size"], c["model"]["compute_dtype"]) == (256, 512, "bf16")


def test_reference_experiment_keeps_fp32_arithmetic():
    """the reference's own experiment sets no trainer precision
    (configs/trainer/default.yaml: Lightning fp32), so its model computes in fp32;
    only the _mi355x experiment opts into bf16, and trainer.precision selects it."""
    import src.train as T
    c = compose("train", ["experiment=pretrain/pretrain_resnet34_tinybert"])
    mc = T.model_config(c, (1.0, 1.0))
    assert "precision" not in c["trainer"] and mc["compute_dtype"] == "fp32"
    mc["downstream_datamodule"] = None
    m = instantiate(mc, device="cpu")
    assert m.image_encoder.model.compute_dtype == "fp32" and m.text_encoder.model.compute_dtype == "fp32"
    assert m._head.compute_dtype == "fp32"
    c = compose("train", ["experiment=pretrain/pretrain_resnet34_tinybert", "+trainer.precision=bf16-mixed"])
    assert T.model_config(c, (1.0, 1.0))["compute_dtype"] == "bf16"
    c = compose("train", ["experiment=pretrain/pretrain_resnet34_tinybert_mi355x"])
    assert T.model_config(c, (1.0, 1.0))["compute_dtype"] == "bf16"
    with pytest.raises(ValueError):
        T.compute_dtype_for("16-mixed")
    from src.models.pretrain.VisionLanguageModule import VisionLanguageModule
    import inspect
    assert inspect.signature(VisionLanguageModule).parameters["compute_dtype"].default == "fp32"


def test_datamodule_schema_and_normalisation():
    with pytest.raises(ValueError):
        PretrainDataModule(num_channels=2)
    with pytest.raises(NotImplementedError):
        PretrainDataModule(synthetic=False)
    dm = PretrainDataModule(batch_size=4, num_workers=0, image_size=32, n_samples=10, tokenizer="tinybert")
    (fold, lw), = list(dm.get_cv_splits())
    assert fold is dm and lw == (1.0, 1.0)
    batches = list(dm.train_dataloader())
    assert len(batches) == 2                                             # drop_last on train
    b = batches[0]
    assert b["x-ray-u8"].shape == (4, 1, 32, 32) and b["x-ray-u8"].dtype == torch.uint8
    ct = b["caption_tokenized"]
    assert set(ct) == {"input_ids", "token_type_ids", "attention_mask"}
    assert ct["input_ids"].shape == (4, 40) and ct["input_ids"].dtype == torch.long
    assert (ct["input_ids"][:, 0] == 101).all()
    L = ct["attention_mask"].sum(1)
    assert ((L >= 10) & (L <= 22)).all()
    assert (ct["input_ids"].gather(1, (L - 1)[:, None]) == 102).all()
    assert (ct["input_ids"] * (1 - ct["attention_mask"]) == 0).all()
    assert all(len(b[k]) == 4 for k in ("caption", "dataset", "anatomy_site", "image_path"))
    val = dm.val_dataloader()
    assert len(val) == 2 and all(len(list(v)) == 16 for v in val)         # 64 val pairs, no drop_last
    # fp32 upload == the reference's normalised 3-channel tensor on the same bytes
    ds = SyntheticRadiographCaptions(3, 16, seed=5)
    samples = [ds[i] for i in range(3)]
    f32 = PairCollator("fp32")(samples)["x-ray"]
    u8 = PairCollator("u8")(samples)["x-ray-u8"]
    assert f32.shape == (3, 3, 16, 16) and f32.dtype == torch.float32
    assert torch.equal(f32, synth.normalize_u8(u8))
    assert torch.equal(normalize_u8(u8, 1), ((u8.float() - 127.5) / 73.9))
    # determinism and per-index independence
    assert torch.equal(ds[1]["x-ray-u8"], SyntheticRadiographCaptions(3, 16, seed=5)[1]["x-ray-u8"])
    assert not torch.equal(ds[0]["x-ray-u8"], ds[1]["x-ray-u8"])
    with pytest.raises(IndexError):
        ds[3]
    with pytest.raises(ValueError):
        PairCollator("u8")([])
    assert PretrainDataModule(num_channels=1, num_workers=0).upload == "fp32"
    assert len(PretrainDataModule(try_with_only_n_samples=5, num_workers=0).train_dataset) == 5


def test_prefetcher_cpu_passthrough():
    items = [{"a": torch.arange(3)}, {"a": torch.arange(4)}]
    out = list(DevicePrefetcher(items, "cpu"))
    assert out == items


class _Toy(torch.nn.Module):
    """Plain-torch stand-in with the hooks the Trainer drives."""

    def __init__(self):
        super().__init__()
        self.w = torch.nn.Parameter(torch.ones(3))
        self.calls = []

    @property
    def device(self):
        return self.w.device

    def configure_optimizers(self):
        return {"optimizer": torch.optim.SGD(self.parameters(), lr=0.1)}

    def on_train_epoch_start(self):
        self.calls.append("epoch_start")

    def on_train_epoch_end(self):
        self.calls.append("epoch_end")

    def training_step(self, batch, i):
        assert self.training
        self.calls.append(("step", i))
        return ((self.w * batch["x"]).sum() - 1.0) ** 2


def test_trainer_loop_semantics(tmp_path):
    m = _Toy()
    data = [{"x": torch.full((3,), float(i + 1))} for i in range(5)]
    t = Trainer(max_epochs=3, log_every_n_steps=2, max_steps=7, default_root_dir=str(tmp_path))
    t.fit(m, train_dataloaders=data)
    assert t.global_step == 7 and t.current_epoch == 1
    assert [s for s, _ in t.history] == [2, 4, 6]
    assert m.calls[0] == "epoch_start" and m.calls.count("epoch_end") == 2
    # the step really optimises: w moved away from ones by SGD
    assert not torch.allclose(m.w.detach(), torch.ones(3))
    m2 = _Toy()
    Trainer(max_epochs=1, limit_train_batches=2, default_root_dir=str(tmp_path)).fit(m2, train_dataloaders=data)
    assert [c for c in m2.calls if isinstance(c, tuple)] == [("step", 0), ("step", 1)]
    with pytest.raises(ValueError):
        Trainer(min_epochs=3, max_epochs=2)


def test_downstream_datamodule_and_fusion_config():
    from src.data.DownstreamDataModule import DownstreamDataModule
    with pytest.raises(ValueError):
        DownstreamDataModule(num_channels=2)
    with pytest.raises(NotImplementedError):
        DownstreamDataModule(synthetic=False)
    c = compose("train", ["experiment=baseline_imaging_and_clinical/baseline_imaging_and_clinical_resnet_34",
                          "data.num_workers=0", "data.image_size=16", "data.batch_size=4", "data.n_samples=40"])
    assert c["model"]["_target_"] == "src.models.baseline.FusionModule.FusionModule"
    assert c["model"]["optimizer"]["_target_"] == "torch.optim.AdamW"
    assert c["model"]["scheduler"]["_target_"] == "transformers.get_cosine_schedule_with_warmup"
    assert c["model"]["scheduler"]["num_training_steps"] == 300 and c["data"]["batch_size"] == 4
    assert "early_stopping_btxrd" in c["callbacks"] and "early_stopping_internal" not in c["callbacks"]
    dm = instantiate(c["data"])
    (fold, (w0, w1)), = list(dm.get_cv_splits())
    labels = torch.cat([b["tumor"] for b in fold.train_dataloader()])
    assert labels.numel() == 40
    n0, n1 = int((labels == 0).sum()), int((labels == 1).sum())
    assert abs(w0 - 40 / (2 * n0)) < 1e-12 and abs(w1 - 40 / (2 * n1)) < 1e-12   # DownstreamDataModule.py:330-332
    b = next(iter(fold.train_dataloader()))
    assert b["anatomy_site_encoded"].shape == (4, 9) and b["age_encoded"].shape == (4, 4)
    assert b["sex_encoded"].shape == (4, 2) and b["x-ray-u8"].dtype == torch.uint8
    assert torch.cat((b["anatomy_site_encoded"], b["age_encoded"], b["sex_encoded"]), 1).sum(1).eq(3).all()
    assert len(fold.val_dataloader()) == 2


def _dp_worker(rank, world, port, q):
    import os
    import sys
    from tests.conftest import ROOT
    sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-language-pretraining-for-bone-tumor-detection_amd")]
    import torch.distributed as dist
    from src.utils.trainer import Trainer as T
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = _Toy()
    data = [{"x": torch.tensor([1.0, 2.0, 3.0]) * (rank + 1)}]
    T(max_epochs=1).fit(m, train_dataloaders=data)
    q.put((rank, m.w.detach().tolist()))          # plain lists: no fd-shared storage
    dist.barrier()
    dist.destroy_process_group()


def test_trainer_averages_gradients_gloo_ws2():
    """World size 2 over gloo: a module without its own collectives gets DDP-mean gradients,
    so both ranks take the same SGD step, equal to one step on the mean gradient."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: torch.tensor(w) for r, w in (q.get(timeout=120) for _ in range(2))}
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    grads = []
    for r in range(2):
        w = torch.ones(3, requires_grad=True)
        x = torch.tensor([1.0, 2.0, 3.0]) * (r + 1)
        (((w * x).sum() - 1.0) ** 2).backward()
        grads.append(w.grad)
    ref = torch.ones(3) - 0.1 * (grads[0] + grads[1]) / 2
    assert torch.allclose(res[0], res[1]) and torch.allclose(res[0], ref, atol=1e-6)


def test_linear_probe_callback_host_logic():
    """LinearProbeCallback (reference LinearProbeCallback.py:17-116) with a stand-in encoder on CPU:
    the every-n-epochs gate, the concatenated validation sets and sklearn's metrics."""
    import numpy as np
    from sklearn.linear_model import LogisticRegression
    from sklearn.metrics import balanced_accuracy_score, roc_auc_score
    from src.data.DownstreamDataModule import DownstreamDataModule
    from src.utils.LinearProbeCallback import LinearProbeCallback

    dm = DownstreamDataModule(batch_size=8, num_workers=0, image_size=8, n_samples=48, n_val_samples=16)
    fold, _ = next(dm.get_cv_splits())
    cb = LinearProbeCallback(fold.train_dataloader(), fold.val_dataloader(), every_n_epochs=5)
    assert len(cb.val_dataloader.dataset) == 32

    class Enc(torch.nn.Module):
        def forward(self, x):                              # uint8 [B,1,8,8] -> 64-d features
            return x.float().flatten(1) / 255.0

    class Mod:
        image_encoder = Enc()
        device = torch.device("cpu")
        logged = {}

        def log(self, k, v, **kw):
            self.logged[k] = v

    m = Mod()
    cb.on_validation_start(types_ns(current_epoch=1), m)
    assert m.logged == {}
    cb.on_validation_start(types_ns(current_epoch=5), m)
    X = np.concatenate([b["x-ray-u8"].float().flatten(1).numpy() / 255.0 for b in fold.train_dataloader()])
    # the train loader shuffles: refit on the callback's own extraction instead
    Xt, yt = cb._extract_features(Enc(), cb.train_dataloader, torch.device("cpu"))
    Xv, yv = cb._extract_features(Enc(), cb.val_dataloader, torch.device("cpu"))
    assert Xt.shape == (48, 64) and Xv.shape == (32, 64) and X.shape == (48, 64)
    clf = LogisticRegression(max_iter=1000, solver="lbfgs").fit(Xt, yt)
    # (the fit inside the callback saw the shuffled order: lbfgs agrees to round-off)
    assert abs(m.logged["downstream_validation/linear_probe_auroc"]
               - roc_auc_score(yv, clf.predict_proba(Xv)[:, 1])) < 1e-3
    assert abs(m.logged["downstream_validation/linear_probe_balanced_accuracy"]
               - balanced_accuracy_score(yv, clf.predict(Xv))) < 0.05


def types_ns(**kw):
    import types
    return types.SimpleNamespace(sanity_checking=False, **kw)


class _ValToy(_Toy):
    """_Toy with a validation loop that logs a monitored metric."""

    def __init__(self, val_curve):
        super().__init__()
        self.val_curve, self.logged, self.hparams = list(val_curve), {}, {
            "optimizer": functools.partial(torch.optim.AdamW, lr=5e-5), "embedding_dim": 128, "obj": object()}

    def validation_step(self, batch, i, idx=0):
        pass

    def on_validation_epoch_end(self):
        self.logged["val/combined/loss"] = torch.tensor(self.val_curve.pop(0))


def test_trainer_checkpoint_and_early_stopping(tmp_path):
    """ModelCheckpoint keeps the best val/combined/loss (Lightning checkpoint dict,
    loadable with weights_only=True), EarlyStopping stops after `patience` rounds
    without improvement, LearningRateMonitor logs the group lr; validation runs
    every epoch over all batches by default (Lightning's limit_val_batches=1.0)."""
    from src.utils.trainer import EarlyStopping, LearningRateMonitor, ModelCheckpoint
    m = _ValToy([3.0, 2.0, 2.5, 2.6, 2.7, 1.0])
    ck = ModelCheckpoint(monitor="val/combined/loss", mode="min", save_top_k=1,
                         filename="combined-epoch:{epoch}-val_combined_loss:{val/combined/loss:.2f}",
                         auto_insert_metric_name=False)
    es = EarlyStopping(monitor="val/combined/loss", mode="min", patience=2)
    t = Trainer(max_epochs=6, callbacks=[ck, es, LearningRateMonitor()], default_root_dir=str(tmp_path))
    data = [{"x": torch.ones(3)}]
    t.fit(m, train_dataloaders=data, val_dataloaders=[data])
    assert t.current_epoch == 3 and t.should_stop                        # 2.5, 2.6 after best 2.0
    assert ck.best_model_score == 2.0
    assert ck.best_model_path.endswith("combined-epoch:1-val_combined_loss:2.00.ckpt")
    files = list((tmp_path / "checkpoints").iterdir())
    assert len(files) == 1                                                # save_top_k = 1
    d = torch.load(ck.best_model_path, weights_only=True)
    assert set(d) >= {"state_dict", "hyper_parameters", "epoch", "global_step"} and d["epoch"] == 1
    hp = d["hyper_parameters"]
    assert hp["optimizer"] == {"_target_": "torch.optim.adamw.AdamW", "_partial_": True, "lr": 5e-5}
    assert "obj" not in hp and hp["embedding_dim"] == 128
    opt = instantiate(hp["optimizer"])
    assert opt.func is torch.optim.AdamW and t.logged_metrics["lr-SGD/0"] == 0.1
    assert Trainer().limit_val_batches is None and Trainer().checkpoint_callback is not None


def test_vlm_checkpoint_roundtrip_cpu(tmp_path):
    """Lightning-format checkpoint of VisionLanguageModule: logit_scale exported in the
    reference's float64 (:111), hyper-parameters rebuilt (optimizer partial) by
    load_from_checkpoint with weights_only=True."""
    from src.models.pretrain.VisionLanguageModule import VisionLanguageModule
    m = VisionLanguageModule("resnet34", "tinybert", functools.partial(torch.optim.AdamW, lr=5e-5),
                             False, False, 512, 312, 128, device="cpu")
    sd = m.state_dict()
    assert sd["logit_scale"].dtype == torch.float64 and sd["image_projection"].dtype == torch.float32
    t = Trainer(enable_checkpointing=False)
    path = str(tmp_path / "m.ckpt")
    t.save_checkpoint(path, m)
    m2 = VisionLanguageModule.load_from_checkpoint(path, device="cpu")
    assert m2.hparams.optimizer.func is torch.optim.AdamW and m2.hparams.optimizer.keywords["lr"] == 5e-5
    for k, v in m2.state_dict().items():
        assert torch.equal(v, sd[k]), k


def _shard_worker(rank, world, port, q):
    import os
    import sys
    from tests.conftest import ROOT
    sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-language-pretraining-for-bone-tumor-detection_amd")]
    import torch.distributed as dist
    from src.data.DownstreamDataModule import DownstreamDataModule
    from src.data.PretrainDataModule import PretrainDataModule
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    fold, lw = next(DownstreamDataModule(num_workers=0, image_size=8, n_samples=12, batch_size=4).get_cv_splits())
    paths = [p for b in fold.train_dataloader() for p in b["image_path"]]
    pre = PretrainDataModule(num_workers=0, image_size=8, n_samples=8, batch_size=4)
    imgs = [b["x-ray-u8"].sum().item() for b in pre.train_dataloader()]
    q.put((rank, paths, lw, imgs))
    dist.barrier()
    dist.destroy_process_group()


def test_datamodules_shard_per_rank_gloo_ws2():
    """Data parallel: every rank reads different samples (the downstream set is
    split as DistributedSampler would, with the whole set's label weights; the
    pretraining stream is seeded per rank)."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_shard_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: (paths, lw, imgs) for r, paths, lw, imgs in (q.get(timeout=120) for _ in range(2))}
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    (p0, lw0, i0), (p1, lw1, i1) = res[0], res[1]
    assert len(p0) == len(p1) == 6 and not set(p0) & set(p1)
    assert sorted(p0 + p1) == sorted(f"synthetic://downstream/{i}.png" for i in range(12))
    assert lw0 == lw1
    assert i0 != i1


def test_shard_indices_pad_like_distributed_sampler():
    """ranks must get equal sample (hence batch) counts; the pad wraps."""
    from src.data.DownstreamDataModule import DownstreamDataModule as D
    for n, world in ((257, 2), (13, 4), (8, 8), (3, 8), (12, 2)):
        shards = [D.shard_indices(n, r, world) for r in range(world)]
        per = -(-n // world)
        assert all(len(s) == per for s in shards)
        flat = sorted(i for s in shards for i in s)
        assert set(flat) == set(range(n))          # every sample is read, the pad repeats the head
        assert len(flat) == per * world
    # n = 257, world = 2, bs = 128 -> 2 batches on both ranks (129 samples each)
    assert all(-(-len(D.shard_indices(257, r, 2)) // 128) == 2 for r in range(2))


def _sync_worker(rank, world, port, q, tmp):
    import os
    import sys
    from tests.conftest import ROOT
    sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-language-pretraining-for-bone-tumor-detection_amd")]
    import torch.distributed as dist
    from src.utils.trainer import EarlyStopping, ModelCheckpoint, Trainer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # rank-local validation losses disagree: rank 0 keeps improving, rank 1 stalls
    seq = [3.0, 2.0, 1.5, 1.0, 0.5] if rank == 0 else [3.0, 3.5, 3.6, 3.7, 3.8]
    m = _ValToy(seq)
    ck = ModelCheckpoint(monitor="val/combined/loss", mode="min", save_top_k=1, dirpath=tmp)
    es = EarlyStopping(monitor="val/combined/loss", mode="min", patience=2)
    t = Trainer(max_epochs=5, callbacks=[ck, es], default_root_dir=tmp)
    data = [{"x": torch.ones(3)}]
    t.fit(m, train_dataloaders=data, val_dataloaders=[data])
    q.put((rank, t.current_epoch, ck.best_model_path, ck.best_model_score, os.path.exists(ck.best_model_path)))
    dist.barrier()
    dist.destroy_process_group()


def test_trainer_decisions_agree_across_ranks_gloo_ws2(tmp_path):
    """the monitored metric is the mean over ranks, so EarlyStopping and
    ModelCheckpoint decide identically on every rank, and the best checkpoint
    exists for every rank when it reads best_model_path."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_sync_worker, args=(r, 2, port, q, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: rest for r, *rest in (q.get(timeout=180) for _ in range(2))}
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    (e0, p0, s0, x0), (e1, p1, s1, x1) = res[0], res[1]
    # means over ranks: 3.0, 2.75, 2.55, 2.35, 2.15 -> keeps improving, no early stop
    assert e0 == e1 == 4
    assert p0 == p1 and x0 and x1
    assert abs(s0 - 2.15) < 1e-6 and s0 == s1   # fp32 logged values

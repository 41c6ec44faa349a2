"""src/train.py end to end on the HIP path: composed config -> synthetic data module
-> DevicePrefetcher (side-stream H2D) -> Trainer loop -> VisionLanguageModule's fused
step.  Checks the prefetched device batch equals the pinned host batch, the API
forward on the uint8 upload equals the fp32 batch (fp32 parity mode, eval), and that
two short trainings from the same seed (train.yaml seed 42) give the same loss
history (rtol 1e-5)."""
import functools
import os

import pytest
import torch

from oracle import weights as W
from oracle.clip import OracleVLP
from src.data.PretrainDataModule import DevicePrefetcher, PairCollator, SyntheticRadiographCaptions

pytestmark = pytest.mark.gpu

_ARGS = ["experiment=pretrain/pretrain_resnet34_tinybert", "data.batch_size=4", "data.image_size=64",
         "data.n_samples=16", "data.num_workers=0", "trainer.max_epochs=1", "model.compute_dtype=fp32",
         "model.text_dropout=0.0", "downstream_data.image_size=64", "downstream_data.n_samples=32",
         "downstream_data.n_val_samples=16", "downstream_data.batch_size=8", "downstream_data.num_workers=0"]


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def test_prefetcher_delivers_identical_batches():
    ds = SyntheticRadiographCaptions(8, 32, seed=3)
    col = PairCollator("u8")
    host = [col([ds[i] for i in range(j, j + 4)]) for j in (0, 4)]
    host = [{**h, "x-ray-u8": h["x-ray-u8"].pin_memory()} for h in host]
    got = list(DevicePrefetcher(host, "cuda:0"))
    assert len(got) == 2
    for h, d in zip(host, got):
        assert d["x-ray-u8"].is_cuda and torch.equal(d["x-ray-u8"].cpu(), h["x-ray-u8"])
        for k in h["caption_tokenized"]:
            assert torch.equal(d["caption_tokenized"][k].cpu(), h["caption_tokenized"][k])
        assert d["caption"] == h["caption"]


def test_api_forward_u8_equals_fp32_eval():
    from src.models.pretrain.VisionLanguageModule import VisionLanguageModule
    ds = SyntheticRadiographCaptions(4, 64, seed=9)
    samples = [ds[i] for i in range(4)]
    bu = PairCollator("u8")(samples)
    bf = PairCollator("fp32")(samples)
    m = VisionLanguageModule("resnet34", "tinybert", functools.partial(torch.optim.AdamW, lr=5e-5),
                             False, False, 512, 312, 128, compute_dtype="fp32", text_dropout=0.0)
    W.apply_recipe(m, 0)
    m.eval()
    with torch.no_grad():
        lu, iu, tu = m(bu)
        lf, i_f, tf = m(bf)
        o = OracleVLP(128, text_dropout=0.0)
        W.apply_recipe(o, 0)
        o.eval()
        fo = o.image_encoder(bf["x-ray"]).double()
        fu = m.image_encoder(bu["x-ray-u8"].cuda()).double().cpu()
    assert torch.allclose(lu, lf, atol=1e-5, rtol=0)
    assert ((fu - fo).norm() / fo.norm()).item() < 1e-4                    # linear-probe features vs oracle


def test_train_main_runs_and_is_deterministic(tmp_path):
    """Also: validation over [lera, mura] every epoch, the reference's
    checkpoint_combined callback keeps the best val/combined/loss checkpoint, and
    the post-fit step reloads it and evaluates downstream precision@k (:189-210)."""
    from src import train as T
    from src.utils.config import compose
    hist = []
    for run in range(2):
        cfg = compose("train", _ARGS + [f"paths.output_dir={tmp_path / str(run)}"])
        metrics, objs = T.train(cfg)
        tr = objs["trainer"]
        assert tr.global_step == 4
        ck = tr.checkpoint_callback
        assert ck.monitor == "val/combined/loss" and ck.best_model_path.startswith(str(tmp_path / str(run)))
        assert "val/combined/loss" in tr.logged_metrics and "best_model" in objs
        assert any(k.startswith("downstream_entire/label_precision_at_") for k in metrics)
        hist.append([l for _, l in tr.history])
        assert all(torch.isfinite(torch.tensor(h)) for h in hist[-1])
        assert "train/loss" in metrics
        assert all(torch.isfinite(p).all() for p in objs["model"].parameters())
        # LinearProbeCallback ran at epoch 0 on the HIP encoder's eval-mode features
        lg = objs["model"].logged
        assert 0.0 <= float(lg["downstream_validation/linear_probe_auroc"]) <= 1.0
        assert 0.0 <= float(lg["downstream_validation/linear_probe_balanced_accuracy"]) <= 1.0
    assert torch.allclose(torch.tensor(hist[0]), torch.tensor(hist[1]), rtol=1e-5, atol=0)


def test_train_fusion_experiment():
    from src import train as T
    from src.utils.config import compose
    cfg = compose("train", ["experiment=baseline_imaging_and_clinical/baseline_imaging_and_clinical_resnet_34",
                            "data.batch_size=8", "data.image_size=64", "data.n_samples=24", "data.num_workers=0",
                            "trainer.max_epochs=2", "model.coral_lambda=0.5"])
    metrics, objs = T.train(cfg)
    tr = objs["trainer"]
    assert tr.global_step == 6 and len(tr.history) == 6
    assert all(torch.isfinite(torch.tensor(l)) for _, l in tr.history)
    assert objs["model"].label_weights.tolist() != [1.0, 1.0]          # set from the fold's labels
    assert "train/coral_loss" in tr.logged_metrics

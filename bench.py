#!/usr/bin/env python3
"""Benchmark: image-text pairs/s of the full CLIP pretraining step
(ResNet34 + TinyBERT forward + backward + fused global-batch InfoNCE + AdamW)
at bs=256/GPU, 512x512, T=40, bf16 (BASELINE.json configs[1]; configs[2] for
--gpus 8 via torch.distributed.run).

  python bench.py [--gpus N] [--steps K] [--warmup W]

One process per GPU (RCCL over xGMI for N > 1), W untimed warm-up steps (more,
untimed, until --warmup-seconds have passed, the same count on every rank), then
exactly K timed steps bracketed by barrier + synchronize; the max over ranks is
reported.  `value` times the K steps on a batch resident in HBM when the clock
starts (the bench contract: the PCIe-inclusive rate is never `value`).
`upload_prefetched` times the same K steps as SURVEY §8(d) writes the step,
with the batch upload inside it: the collated batch (pinned host memory, uint8
1-channel radiographs -- the data module's default -- or with --input fp32 the
reference's fp32 x-ray [B,3,H,W]; caption ids/masks [B,T] int64) goes up
through src/data's DevicePrefetcher, which copies batch i+1 on a side stream
while step i runs.

The JSON line also carries
  roofline     : the dominant kernel (by total time) timed with HIP events on
                 its launch stream during the timed steps; achieved = its
                 algorithmic FLOPs / its summed launch duration
  cpu_baseline : the CPU oracle (timm-layout ResNet34 + HF BertModel + the
                 reference head/loss + torch AdamW, fp32) on this host's cores,
                 on a bounded sample (rank 0, N=1 only)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "vision-language-pretraining-for-bone-tumor-detection_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_F32_TFLOPS = 157.3
FLOP_PER_PAIR_512 = 114.72e9  # ResNet34 113.60 + TinyBERT 1.117 + head


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--warmup-seconds", type=float, default=5.0,
                    help="after the W warm-up steps, keep stepping (untimed) until this many seconds of "
                         "warm-up have passed: r6 boxes ran the first ~2-3 s of a process's steady stepping "
                         "at a third of the rate")
    ap.add_argument("--image-model", default="resnet34", choices=["resnet34", "nest_small"],
                    help="image tower: resnet34 (BASELINE configs[1]) or nest_small (configs[3], bs=128)")
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default 256; 128 for nest_small)")
    ap.add_argument("--image-size", type=int, default=512)
    ap.add_argument("--seq-len", type=int, default=40)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--input", default="u8", choices=["fp32", "u8"],
                    help="collated image form: the uint8 1-channel upload (the data module's default) or "
                         "the reference's fp32 3-channel batch")
    ap.add_argument("--no-loss-check", dest="loss_check", action="store_false",
                    help="skip the bf16-vs-fp32-oracle loss comparison on the bench batch")
    ap.add_argument("--cpu-sample-batch", type=int, default=None,
                    help="CPU-baseline sample batch (default 32; 4 for nest_small)")
    ap.add_argument("--cpu-sample-steps", type=int, default=3)
    ap.add_argument("--no-cpu-configs0", dest="cpu_configs0", action="store_false",
                    help="skip the cpu_baseline sample at BASELINE configs[0] (bs=8, 224^2)")
    ap.add_argument("--roofline-kernel", default="auto")
    ap.add_argument("--kernel-report", default="")
    ap.add_argument("--pcie-steps", type=int, default=5,
                    help="steps timed with the batch copied from pinned host memory (0: skip)")
    ap.add_argument("--wgrad-stream", type=int, default=1, choices=[0, 1],
                    help="ResNet34 weight gradients on a side stream beside the data-gradient chain (default 1)")
    ap.add_argument("--roofline-steps", type=int, default=5,
                    help="steps of the isolated (serial-schedule) pass that times the roofline kernel")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI; gloo for CPU rehearsal)")
    ap.add_argument("--dp-rehearsal", type=int, default=1, choices=[0, 1],
                    help="N=1: also time the K steps with the data-parallel schedule on a world-1 RCCL group "
                         "(every collective issued, per-stage gradient buckets launched from the weight-gradient "
                         "stream) and report it beside `value` as `dp_schedule_1gpu`")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU work: exercise the launcher, the rendezvous and the max-over-ranks timing "
                         "and print the JSON line (CPU test of the N-rank path)")
    ap.add_argument("--master-port", type=int, default=None,
                    help="rendezvous port when bench.py launches its own ranks (default: a free port)")
    a = ap.parse_args()
    nest = a.image_model != "resnet34"
    if a.batch is None:
        a.batch = 128 if nest else 256
    if a.cpu_sample_batch is None:
        a.cpu_sample_batch = 4 if nest else 32
    return a


def flop_per_pair(args):
    """ResNet34 113.60 + TinyBERT 1.117 + head GFLOP per pair at 512^2
    (FlopCounterMode); NesT: vlp_amd.nest.nest_flops_per_image (GEMMs, convs and
    attention, backward = 2x forward) + TinyBERT."""
    if args.image_model == "resnet34":
        return FLOP_PER_PAIR_512 * (args.image_size / 512) ** 2
    from vlp_amd.nest import nest_flops_per_image
    return nest_flops_per_image(args.image_model, args.image_size) + 1.117e9


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args, argv):
    """`python bench.py --gpus N` with N > 1 and no WORLD_SIZE in the environment:
    start the N ranks as ONE child process tree (`python -m torch.distributed.run
    --nproc-per-node N ... bench.py <same args>`), one process per GPU.  This
    process has not touched the GPU (no HIP call before this point) and never
    re-execs: it waits for the child, whose rank 0 prints the JSON line on the
    inherited stdout, and returns the child's exit code."""
    import subprocess
    port = args.master_port or _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def setup_dist(args):
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws > 1:
        lr = int(os.environ.get("LOCAL_RANK", "0"))
        if args.gpus != ws:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws}")
        if args.backend == "gloo":
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(lr)
            dist.init_process_group("nccl", device_id=torch.device("cuda", lr))
        return dist.get_rank(), ws, lr
    if args.gpus != 1:
        raise SystemExit(f"bench.py: --gpus {args.gpus} needs {args.gpus} ranks (run without WORLD_SIZE "
                         "and bench.py launches them)")
    if not args.dry_run:
        torch.cuda.set_device(0)
    return 0, 1, 0


def dry_run(args, rank, world):
    """The N-rank bench path without GPU work: barrier-bracketed timed region,
    max over ranks, rank 0 prints one JSON line with the same keys as a real run."""
    def timed():
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        acc = torch.zeros(1 << 16)
        for _ in range(args.steps):
            acc.add_(1.0)
        if world > 1:
            dist.barrier()
        e = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
        if world > 1:
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
        return e.item()
    el = max(timed(), 1e-9)
    if rank == 0:
        print(json.dumps({
            "metric": f"image-text pairs/sec (fwd+bwd) at bs={args.batch}/GPU, 1/2/4/8 MI355X",
            "value": round(world * args.batch * args.steps / el, 2), "unit": "image-text pairs/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 6), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": args.dtype, "data": "dry run (no GPU work)",
            "config": {"workload": "dry run of the launcher and rank timing", "global_batch": world * args.batch,
                       "per_gpu_batch": args.batch, "parallelism": f"dp{world}"},
            "backend": args.backend if world > 1 else None}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def make_batch(B, H, T, device, seed, form="fp32"):
    """form "fp32": the reference's collated x-ray [B,3,H,W] fp32; "u8": the 1-channel
    uint8 radiograph (x-ray-u8 [B,1,H,W]) that the module normalises on the device
    (src/data/PretrainDataModule.py's default upload), same pixels."""
    from tests.golden.synth import synth_batch
    b = synth_batch(B, H, T, seed, with_u8=form == "u8")
    img = {"x-ray-u8": b["x-ray-u8"].to(device)} if form == "u8" else {"x-ray": b["x-ray"].to(device)}
    return {**img, "label": b["label"].to(device), "caption": b["caption"],
            "caption_tokenized": {k: v.to(device) for k, v in b["caption_tokenized"].items()}}


def make_host_batch(B, H, T, seed, form="u8"):
    """The collated batch as the data module hands it over: pinned host memory."""
    from tests.golden.synth import synth_batch
    b = synth_batch(B, H, T, seed, with_u8=form == "u8")
    img = {"x-ray-u8": b["x-ray-u8"].pin_memory()} if form == "u8" else {"x-ray": b["x-ray"].pin_memory()}
    return {**img, "label": b["label"].pin_memory(), "caption": b["caption"],
            "caption_tokenized": {k: v.pin_memory() for k, v in b["caption_tokenized"].items()}}


def loss_delta_vs_fp32(args, model, host):
    """The bench's own weights (after warm-up and timed steps) and batch, one
    train-mode forward (batch-statistics BN, text dropout off on both sides) in
    the bench dtype on the GPU and in fp32 in the CPU oracle: |loss delta| and
    the embeddings' rel-L2 (bf16 deviation measured and
    reported).  CPU cost: one fp32 forward of the full batch."""
    from oracle.clip import OracleVLP, compute_loss
    from tests.golden.synth import normalize_u8
    torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)))
    cfg = model.text_encoder.model.cfg
    saved = (cfg.hidden_dropout, cfg.attention_dropout)
    cfg.hidden_dropout = cfg.attention_dropout = 0.0
    sd = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    nest = args.image_model != "resnet34"
    if nest:   # no BatchNorm: eval mode keeps DropPath's random masks out of the comparison
        model.eval()
    with torch.no_grad():
        loss, li, lt, ie, te = model.training_step_outputs(host)
        loss, ie, te = loss.item(), ie.float().cpu(), te.float().cpu()
    model.train()
    cfg.hidden_dropout, cfg.attention_dropout = saved
    o = OracleVLP(128, text_dropout=0.0, image_model=args.image_model, img_size=args.image_size)
    o.load_state_dict(sd, strict=False)
    o.train(not nest)
    x = host["x-ray"] if "x-ray" in host else normalize_u8(host["x-ray-u8"])
    t0 = time.perf_counter()
    with torch.no_grad():
        lg, oie, ote = o({"x-ray": x, "caption_tokenized": host["caption_tokenized"]})
        lo = compute_loss(lg)[0].item()
    rel = lambda a, b: ((a.double() - b.double()).norm() / b.double().norm()).item()   # noqa: E731
    # eval-mode image features (the linear-probe embedding) of the first 8 images: for
    # NesT the logits can sit at the uniform ln(B) fixed point, where the loss says nothing
    xp = host["x-ray-u8"][:8] if "x-ray-u8" in host else host["x-ray"][:8]
    model.eval()
    o.eval()
    with torch.no_grad():
        f = model.image_encoder(xp.to(next(model.parameters()).device)).float().cpu()
        fo = o.image_encoder(x[:8])
    model.train()
    return {"loss": round(loss, 6), "loss_fp32_oracle": round(lo, 6), "abs_delta": abs(loss - lo),
            "img_emb_rel_l2": rel(ie, oie), "txt_emb_rel_l2": rel(te, ote),
            "probe_features_rel_l2": rel(f, fo),
            "logit_spread": round(float(lg.std()), 6),
            "note": (f"bench weights and batch, train-mode forward, text dropout off; oracle fp32 on "
                     f"{torch.get_num_threads()} CPU threads ({time.perf_counter() - t0:.1f} s)")}


def cpu_baseline(args):
    """Oracle (reference CPU fp32 path, restated) on a bounded sample of the bench
    workload, plus the same step at BASELINE configs[0] (bs=8, 224^2, the
    reference's own CPU-runnable case) beside it."""
    res = _cpu_oracle_steps(args, args.cpu_sample_batch, args.image_size, args.seq_len)
    if args.image_model == "resnet34" and args.cpu_configs0:
        c0 = _cpu_oracle_steps(args, 8, 224, args.seq_len)
        res["configs0"] = {k: c0[k] for k in ("value", "unit", "cores", "sample")}
    return res


def _cpu_oracle_steps(args, B, H, T):
    from oracle import weights as W
    from oracle.clip import OracleVLP, compute_loss
    from tests.golden.synth import synth_batch
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    torch.set_num_threads(threads)
    model = OracleVLP(128, text_dropout=0.1, image_model=args.image_model, img_size=H)
    if args.image_model == "resnet34":
        W.apply_recipe(model, 0)
    model.train()
    opt = torch.optim.AdamW(model.param_groups(), lr=5e-5)
    batch = synth_batch(B, H, T, 0)
    times = []
    for i in range(args.cpu_sample_steps + 1):
        t0 = time.perf_counter()
        opt.zero_grad()
        lg, _, _ = model(batch)
        loss = compute_loss(lg)[0]
        loss.backward()
        opt.step()
        if i > 0:
            times.append(time.perf_counter() - t0)
    times.sort()
    med = times[len(times) // 2]
    return {"value": round(B / med, 3), "unit": "image-text pairs/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"oracle fp32 CPU step (fwd+bwd+AdamW), bs={B}, {H}x{H}, T={T}, "
                      f"median of {len(times)} steps after 1 warm-up ({med:.2f} s/step)"}


def mfma_peak_measured(dev):
    """Dense bf16 MFMA ceiling of this card (vlp_mfma_peak_probe), TFLOP/s."""
    from vlp_amd._lib import lib
    blocks, iters = 2048, 2000
    out = torch.empty(blocks * 256, device=dev)
    st = torch.cuda.current_stream(dev)
    best = 0.0
    for _ in range(4):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        lib().vlp_mfma_peak_probe(blocks, iters, out.data_ptr(), st.cuda_stream)
        e1.record(st)
        e1.synchronize()
        best = max(best, blocks * 4 * iters * 8 * 16384 / (e0.elapsed_time(e1) * 1e-3) / 1e12)
    return round(best, 1)


def rank_of():
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def pcie_inclusive(args, model, opt, world, dev):
    """The SURVEY §8(d) step including the batch's H2D copy: the batch starts in
    pinned host memory each step (as the reference's pin_memory DataLoader
    hands it over) and goes up with non_blocking copies inside training_step.
    Two forms: the reference's collated fp32 3-channel images (805 MB at
    bs=256, 512^2) and the 1-channel uint8 upload (67 MB) that
    vlp_stem_prep_u8 normalises on the device.  Reported beside `value`."""
    from tests.golden.synth import synth_batch
    b = synth_batch(args.batch, args.image_size, args.seq_len, 0, with_u8=True)
    caps = {k: v.pin_memory() for k, v in b["caption_tokenized"].items()}
    out = {}
    for form, key in (("fp32_3ch", "x-ray"), ("u8_1ch", "x-ray-u8")):
        host = {key: b[key].pin_memory(), "caption_tokenized": caps, "label": b["label"], "caption": b["caption"]}

        def step():
            opt.zero_grad()
            loss = model.training_step(host)
            loss.backward()
            opt.step()
        step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.pcie_steps):
            step()
        torch.cuda.synchronize()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
        el = el.item()
        out[form] = {"value": round(world * args.batch * args.pcie_steps / el, 2),
                     "ms_per_step": round(el / args.pcie_steps * 1e3, 3),
                     "h2d_mb_per_step": round(b[key].numel() * b[key].element_size() / 1e6, 1)}
        # same upload through src/data's DevicePrefetcher: batch i+1 is copied on a
        # side stream while step i runs (the training loop's data path)
        from src.data.PretrainDataModule import DevicePrefetcher

        def steps_overlapped(n):
            for dbatch in DevicePrefetcher((host for _ in range(n)), dev):
                opt.zero_grad()
                loss = model.training_step(dbatch)
                loss.backward()
                opt.step()
        steps_overlapped(2)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        steps_overlapped(args.pcie_steps)
        torch.cuda.synchronize()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
        el = el.item()
        out[form + "_prefetched"] = {"value": round(world * args.batch * args.pcie_steps / el, 2),
                                     "ms_per_step": round(el / args.pcie_steps * 1e3, 3)}
    # the training loop's default (disable_augmentations=False): the uint8 upload
    # through the reference's augmentations on the device (PretrainDataModule.
    # device_augment -> vlp_aug_warp), which hands the step the fp32 3-channel
    # batch (independent per-channel noise), i.e. the 3-channel stem path
    from vlp_amd.augment import Augmenter
    aug = Augmenter(seed=7 + rank_of())
    host = {"x-ray-u8": b["x-ray-u8"].pin_memory(), "caption_tokenized": caps, "label": b["label"],
            "caption": b["caption"]}

    def steps_augmented(n):
        for dbatch in DevicePrefetcher((host for _ in range(n)), dev):
            xb = aug(dbatch["x-ray-u8"], channels=3, mean=127.5, std=73.9)
            opt.zero_grad()
            loss = model.training_step({"x-ray": xb, "caption_tokenized": dbatch["caption_tokenized"],
                                        "label": dbatch["label"]})
            loss.backward()
            opt.step()
    steps_augmented(2)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    steps_augmented(args.pcie_steps)
    torch.cuda.synchronize()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    el = el.item()
    out["u8_1ch_augmented_prefetched"] = {"value": round(world * args.batch * args.pcie_steps / el, 2),
                                          "ms_per_step": round(el / args.pcie_steps * 1e3, 3)}
    out["unit"] = "image-text pairs/s"
    out["steps"] = args.pcie_steps
    return out


def dp_rehearsal(args, prefetched_steps, timed, dev):
    """The world > 1 step schedule measured on one GPU: a world-1 RCCL process
    group with vlp_amd.dist.REHEARSE set, so ClipStepFn issues every collective
    of a data-parallel step (embedding all-gathers, loss all-reduce, gradient
    reduce-scatters, the head / text arenas and the four per-stage image-arena
    buckets, each launched from the stream that produced it) and the image
    tower fires its per-stage callbacks.  Same prefetched steps as `value`."""
    from vlp_amd import dist as vdist
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=dev)
    vdist.REHEARSE = True
    try:
        prefetched_steps(2)
        el, _ = timed(lambda: prefetched_steps(args.steps))
    finally:
        vdist.REHEARSE = False
        torch.cuda.synchronize()
        dist.destroy_process_group()
    return {"value": round(args.batch * args.steps / el, 2), "ms_per_step": round(el / args.steps * 1e3, 3),
            "note": "world-1 RCCL group, every data-parallel collective issued, image-arena buckets per stage "
                    "from the weight-gradient stream (the N > 1 schedule on one GPU)"}


def _traffic(family, dtype="bf16", image_model="resnet34"):
    """HBM bytes per launch of the roofline kernel from the committed PMC passes
    (profiles/roofline_traffic.json, written by tools/pmc_traffic.py from
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of this same command).  The
    table holds the default bf16 runs (ResNet34 and NesT families); any other
    dtype reports null rather than another kernel's bytes."""
    if dtype != "bf16":
        return None
    path = os.path.join(ROOT, "profiles", "roofline_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    e = d.get("families", {}).get(family)
    return round(e["traffic_bytes_per_launch"]) if e else None


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args, sys.argv[1:]))
    rank, world, local = setup_dist(args)
    if args.dry_run:
        dry_run(args, rank, world)
        return
    from src.models.pretrain.VisionLanguageModule import VisionLanguageModule
    from vlp_amd import ktimer
    import functools

    dev = torch.device("cuda", local)
    torch.manual_seed(1234 + rank)
    if args.image_model == "resnet34":
        model = VisionLanguageModule("resnet34", "tinybert", functools.partial(torch.optim.AdamW, lr=5e-5),
                                     False, False, 512, 312, 128, compute_dtype=args.dtype, device=dev)
    else:   # BASELINE configs[3]: timm nest_small at img_size = the batch resolution
        model = VisionLanguageModule(args.image_model, "tinybert", functools.partial(torch.optim.AdamW, lr=5e-5),
                                     False, False, 384, 312, 128, compute_dtype=args.dtype, device=dev,
                                     image_size=args.image_size)
    model.train()
    opt = model.configure_optimizers()["optimizer"]
    batch = make_batch(args.batch, args.image_size, args.seq_len, dev, seed=rank, form=args.input)

    def step():
        opt.zero_grad()
        loss = model.training_step(batch)
        loss.backward()   # includes the gradient all-reduce (N > 1)
        opt.step()
        return loss

    # schedule: the image tower's weight gradients run on a side stream beside
    # the data-gradient chain (vlp_amd.resnet34._USE_WG_STREAM, the default).
    # The roofline kernel is timed in a separate pass with the serial schedule,
    # where its launches do not share the CUs with the data-gradient chain.
    from vlp_amd import resnet34 as _r34
    from vlp_amd import clip_model as _cm
    from vlp_amd._lib import lib as _vlib
    resnet = args.image_model == "resnet34"
    text_stream0 = _cm._USE_TEXT_STREAM

    def set_wgrad_stream(on):
        # off = the fully serial schedule of the kernel report and the roofline pass:
        # the weight gradients AND the text tower on the main stream, so no family's
        # HIP-event time includes sharing the CUs with another stream
        if resnet:
            _r34._USE_WG_STREAM = bool(on) and args.wgrad_stream
        _cm._USE_TEXT_STREAM = text_stream0 if on else False
    set_wgrad_stream(True)

    t_w = time.perf_counter()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    def warm_more(t0, secs):
        # every rank runs the same number of extra steps (they hold collectives)
        more = torch.tensor([1.0 if time.perf_counter() - t0 < secs else 0.0], device=dev)
        if world > 1:
            dist.all_reduce(more, op=dist.ReduceOp.MAX)
        return more.item() > 0
    while warm_more(t_w, args.warmup_seconds):
        for _ in range(5):
            step()
        torch.cuda.synchronize()
    # select the dominant kernel family to time (by total time in one serial step)
    tk = args.roofline_kernel
    if tk == "auto":
        set_wgrad_stream(False)
        ktimer.enable(None)
        step()
        torch.cuda.synchronize()
        totals = ktimer.totals()
        ktimer.disable()
        set_wgrad_stream(True)
        tk = max(totals, key=lambda k: totals[k][0]) if totals else None
        if args.kernel_report and rank == 0:
            with open(args.kernel_report, "w") as f:
                json.dump({k: {"ms": v[0], "launches": v[1], "gflop": v[2] / 1e9}
                           for k, v in sorted(totals.items(), key=lambda kv: -kv[1][0])}, f, indent=1)

    def timed(run):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = run()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
        e = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
        return e.item(), out

    # `value`: K steps on the batch already resident in HBM (the W warm-up steps
    # above ran the same way).  On shared hosts the upload path picks up the
    # host's PCIe / memory contention (r6: three boxes ran the prefetched window at
    # 2.2-4.7k pairs/s while the resident window beside it held 6.4-6.7k)
    el_hbm, loss = timed(lambda: [step() for _ in range(args.steps)][-1])
    # `upload_prefetched`: the SURVEY §8(d) step, batch upload included.  The
    # batch the data module collates (pinned host memory; the uint8 1-channel
    # radiograph, its default upload) reaches HBM through src/data's
    # DevicePrefetcher: batch i+1 is copied on a side HIP stream while step i
    # runs, every batch but the first crossing PCIe inside the timed region
    from src.data.PretrainDataModule import DevicePrefetcher
    host = make_host_batch(args.batch, args.image_size, args.seq_len, seed=rank, form=args.input)

    def prefetched_steps(n):
        loss = None
        for dbatch in DevicePrefetcher((host for _ in range(n)), dev):
            opt.zero_grad()
            loss = model.training_step(dbatch)
            loss.backward()
            opt.step()
        return loss

    # warm the copy stream and the pinned buffers: at least W prefetched steps and
    # 1 s of them (r6: on some boxes the first second of uploads from freshly
    # pinned pages ran at ~0.8 GB/s while the same process's later prefetched
    # windows ran at full rate)
    t_w = time.perf_counter()
    prefetched_steps(max(2, args.warmup))
    torch.cuda.synchronize()
    while warm_more(t_w, 1.0):
        prefetched_steps(2)
        torch.cuda.synchronize()
    el, _ = timed(lambda: prefetched_steps(args.steps))
    rehearsal = None
    if world == 1 and args.dp_rehearsal:
        rehearsal = dp_rehearsal(args, prefetched_steps, timed, dev)
        # the plain schedule again right after it: the box's drift between the two
        el2, _ = timed(lambda: prefetched_steps(args.steps))
        rehearsal["value_plain_rerun"] = round(args.batch * args.steps / el2, 2)
    # isolated roofline pass: serial schedule, the dominant family timed with HIP
    # events on its launch stream; bracketed by marker dispatches so a rocprofv3
    # kernel trace of this command averages exactly these launches
    # (tools/roofline_window.py)
    set_wgrad_stream(False)
    prefetched_steps(1)
    torch.cuda.synchronize()
    _vlib().vlp_trace_marker(0, torch.cuda.current_stream(dev).cuda_stream)
    ktimer.enable(tk)
    el_serial, _ = timed(lambda: prefetched_steps(args.roofline_steps))
    ktimer.disable()
    _vlib().vlp_trace_marker(1, torch.cuda.current_stream(dev).cuda_stream)
    tot = ktimer.totals().get(tk, (0.0, 0, 0.0))
    # the same family under the default (stream) schedule, for reference
    set_wgrad_stream(True)
    shared = None
    if resnet and args.wgrad_stream and tk and tk.startswith("conv_wgrad"):
        prefetched_steps(1)
        ktimer.enable(tk)
        timed(lambda: prefetched_steps(args.roofline_steps))
        ktimer.disable()
        shared = ktimer.totals().get(tk, (0.0, 0, 0.0))
    pcie = pcie_inclusive(args, model, opt, world, dev) if args.pcie_steps > 0 else None
    ldelta = loss_delta_vs_fp32(args, model, host) if (world == 1 and args.loss_check) else None
    peak_meas = mfma_peak_measured(dev) if args.dtype == "bf16" else None
    ms_k, nl, flop_k = tot
    set_wgrad_stream(True)
    if rank == 0:
        pairs = world * args.batch * args.steps
        value = pairs / el_hbm
        peak = PEAK_BF16_TFLOPS if args.dtype == "bf16" else PEAK_F32_TFLOPS
        achieved = (flop_k / (ms_k / 1e3)) / 1e12 if ms_k > 0 else 0.0
        res = {
            # BASELINE.json's metric is quoted at bs=256 (ResNet34); other batches name theirs
            "metric": f"image-text pairs/sec (fwd+bwd) at bs={args.batch}/GPU, 1/2/4/8 MI355X",
            "value": round(value, 2),
            "unit": "image-text pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "warmup_seconds": args.warmup_seconds,
            "ms_per_step": round(el_hbm / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": ("synthetic (seeded uint8 radiographs as "
                     + ("the uint8 1-channel upload, normalised on the device"
                        if args.input == "u8" else "the reference's normalised 3-ch fp32 tensor")
                     + ", resident in HBM when the timed region starts; seeded token ids; random-init weights; "
                       "the upload-inclusive rate is upload_prefetched)"),
            "config": {"workload": ("ResNet34" if args.image_model == "resnet34" else "NesT-Small")
                       + "+TinyBERT CLIP pretrain step (fwd+bwd+global-batch InfoNCE+AdamW)",
                       "global_batch": world * args.batch, "per_gpu_batch": args.batch,
                       "image_size": args.image_size, "seq_len": args.seq_len,
                       "parallelism": f"dp{world}"},
            "model_flops_frac": round(value * flop_per_pair(args) / (world * peak * 1e12), 4),
            "roofline": {"bound": "mfma", "kernel": tk, "achieved": round(achieved, 2), "peak": peak,
                         "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
                         "avg_launch_us": round(ms_k * 1e3 / max(nl, 1), 2), "launches": nl,
                         "flop_per_launch": round(flop_k / max(nl, 1)), "peak_measured": peak_meas,
                         "frac_of_measured": round(achieved / peak_meas, 4) if peak_meas else None,
                         "traffic_unit": "HBM bytes/launch",
                         "traffic": _traffic(tk, args.dtype, args.image_model),
                         "timed_in": f"isolated pass of {args.roofline_steps} steps, serial schedule "
                                     "(bracketed by vlp_trace_marker dispatches)"},
            "loss": round(loss.item(), 5),
            "upload_prefetched": {"value": round(pairs / el, 2), "ms_per_step": round(el / args.steps * 1e3, 3),
                                  "note": "same K steps with the SURVEY 8(d) upload inside the timed region: the "
                                          "batch collated in pinned host memory, copied per step by the side-stream "
                                          "DevicePrefetcher (batch i+1 during step i)"},
        }
        ps = world * args.batch * args.roofline_steps
        res["serial_schedule"] = {"value": round(ps / el_serial, 2),
                                  "ms_per_step": round(el_serial / args.roofline_steps * 1e3, 3),
                                  "steps": args.roofline_steps,
                                  "note": "the roofline pass: same prefetched steps with the weight gradients and the "
                                          "text tower on the main stream (no CU sharing); `value` uses the side streams"}
        if shared is not None and shared[0] > 0:
            res["roofline"]["achieved_under_default_schedule"] = round((shared[2] / (shared[0] / 1e3)) / 1e12, 2)
        if rehearsal is not None:
            # the rehearsal runs prefetched steps: compared with the prefetched windows
            up = pairs / el
            rehearsal["vs_upload_prefetched"] = round(rehearsal["value"] / up, 4)
            # against the two plain runs bracketing it in time (the box drifts between runs)
            rehearsal["vs_plain_mean"] = round(rehearsal["value"] / ((up + rehearsal["value_plain_rerun"]) / 2), 4)
            res["dp_schedule_1gpu"] = rehearsal
        if ldelta is not None:
            res["loss_delta_vs_fp32"] = ldelta
        if pcie is not None:
            res["pcie_inclusive"] = pcie
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(args)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""Benchmark: images/sec of one U-Net training step (forward + BCE loss + backward
[+ RCCL all-reduce] + Adam) on synthetic 512x512 data, Base config
(UNetWithBackbone resnet34, no attention, batch 16 per GPU), BASELINE.json
configs[1] (N=1) / configs[2] (N>1, weak scaling, 16 per rank).

python bench.py --gpus N --steps K --warmup W
N>1: one process per GPU.  Under torch.distributed.run (WORLD_SIZE set) every
rank runs the step; started bare, the parent launches
`python -m torch.distributed.run --nproc-per-node N` itself (before any GPU
call) and exits with its return code.  Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

MFMA_BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 (MI355X_MICROARCH.md)
MFMA_FP8_PEAK_TFLOPS = 5000.0  # MI355X dense fp8 (block-scaled e4m3 MFMA, MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0


def config_key(backbone: str, width: int, attention: bool, fp8: bool, batch: int, size: int) -> str:
    """Workload key of a PMC profile (scripts/pmc_traffic.py --config)."""
    return f"{backbone}/w{width}/{'attention' if attention else 'plain'}/{'fp8' if fp8 else 'bf16'}/{batch}x{size}"


# files written before the config key existed profiled layer_profile.py's default workload
LEGACY_CONFIG = config_key("resnet34", 1, False, False, 16, 512)


def pmc_traffic(kernel: str, config: str):
    """(HBM bytes per launch of `kernel`, source file) from the newest committed
    rocprofv3 PMC summary OF THIS WORKLOAD (scripts/pmc_traffic.py: FETCH_SIZE
    x2 + WRITE_SIZE, MI355X_MICROARCH.md HBM section; PMC passes cannot run
    inside the timed bench), or (None, None) when no profile of this config
    holds that kernel: bytes measured on another config are never quoted."""
    import glob
    found = sorted(glob.glob(os.path.join(REPO, "profiles", "*", "*", "pmc_traffic*.json")),
                   key=lambda p: (os.path.dirname(p), p))
    # rocprof names spell out defaulted template arguments ("..., false>")
    # that the executor's kernel tag leaves off
    def canon(name: str) -> str:
        name = name.replace(" ", "")
        while name.endswith(",false>"):
            name = name[: -len(",false>")] + ">"
        return name
    want = canon(kernel)
    for path in reversed(found):  # newest profiling session of the newest round first
        with open(path) as f:
            doc = json.load(f)
        cfg, table = (doc["config"], doc["kernels"]) if "kernels" in doc else (LEGACY_CONFIG, doc)
        if cfg != config:
            continue
        for key, ent in table.items():
            if canon(key) == want:
                return ent["bytes_per_launch"], os.path.relpath(path, REPO)
        return None, None  # the newest profile of this config lacks the kernel (e.g. a renamed instance)
    return None, None


def cpu_baseline(batch: int, h: int, steps: int, threads: int, width: int = 1, attention: bool = False,
                 backbone: str = "resnet34"):
    """Time the oracle (fp32 torch-CPU restatement of the reference path) on host cores."""
    import oracle
    torch.set_num_threads(threads)
    pkg = importlib.import_module("image-segmentation-project_amd")
    xs, ms = pkg.synthetic_cells(batch, h, h, seed=1234)
    x, y = torch.from_numpy(xs), torch.from_numpy(ms)
    m = oracle.ReferenceUNet(width=width, use_attention=attention, backbone=backbone)
    m.load_state_dict(oracle.closed_form_state_dict(m))
    m.train()
    opt = oracle.make_adam(m)
    crit = oracle.get_loss_function({"loss_fn": "bce"})
    oracle.train_step(m, opt, crit, x[:2], y[:2])  # warm-up
    t0 = time.perf_counter()
    for _ in range(steps):
        oracle.train_step(m, opt, crit, x, y)
    dt = time.perf_counter() - t0
    return {"value": round(batch * steps / dt, 3), "unit": "images/sec", "cores": threads, "kind": "port",
            "sample": f"{steps} fp32 train steps (fwd+bce+bwd+Adam) of batch {batch} at {h}x{h}, "
                      f"oracle/unet_ref.py on {threads} host threads"}


def cpu_baseline_data(frames, masks, size: int, n: int):
    """The reference's per-image host preprocessing (dataset.py:30-66) as restated
    by the numpy oracle, timed on one host thread over a bounded sample."""
    import oracle.dataset_ref as dref
    t0 = time.perf_counter()
    for i in range(n):
        dref.preprocess(frames[i], masks[i], (size, size))
    dt = (time.perf_counter() - t0) / n
    return {"value": round(1.0 / dt, 2), "unit": "frames/sec", "cores": 1, "kind": "port",
            "sample": f"{n} frames through oracle/dataset_ref.py (numpy, one thread)"}


def data_bench(args):
    """--data: throughput of the on-GPU data pipeline (SURVEY.md §8(f) row 3,
    dataset.py:30-66,147-151) on decoded uint8 frames resident in HBM: resize
    (INTER_AREA / INTER_NEAREST), percentile clip + CLAHE + min-max, mask
    binarisation; and the RandomRotate90 / VerticalFlip augmentation."""
    import numpy as np
    pkg = importlib.import_module("image-segmentation-project_amd")
    rng = np.random.default_rng(0)
    n, src = args.batch, args.data_src
    frames = rng.integers(0, 256, (n, src, src), dtype=np.uint8)
    masks = (rng.random((n, src, src)) < 0.3).astype(np.uint8) * 255
    x, m = torch.from_numpy(frames).cuda(), torch.from_numpy(masks).cuda()
    aug = pkg.CellAugmenter(augmentations_per_image=1, seed=0)
    for _ in range(args.warmup):
        pkg.preprocess(x, m, (args.size, args.size))
        aug.augment_training_data(x, m)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pkg.preprocess(x, m, (args.size, args.size))
    torch.cuda.synchronize()
    dt_pre = (time.perf_counter() - t0) / args.steps
    t0 = time.perf_counter()
    for _ in range(args.steps):
        aug.augment_training_data(x, m)
    torch.cuda.synchronize()
    dt_aug = (time.perf_counter() - t0) / args.steps
    line = {"metric": f"preprocessed frames/sec (uint8 {src}x{src} -> float32 {args.size}x{args.size}, "
                      "clip+CLAHE+min-max+mask)",
            "value": round(n / dt_pre, 1), "unit": "frames/sec", "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "higher_is_better": True, "data": "synthetic uint8 frames",
            "config": {"workload": "dataset.py preprocessing on GPU", "batch": n},
            "augment_frames_per_sec": round(n / dt_aug, 1)}
    if not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline_data(frames, masks, args.size, args.cpu_frames)
    print(json.dumps(line), flush=True)


def launch_ranks(n: int) -> int:
    """Re-run this script as n ranks under torch.distributed.run (a child
    process, never an exec: the parent has not touched the GPU)."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def miou_parity(model, x, y, width: int, attention: bool, backbone: str = "resnet34", reference: bool = True):
    """North-star parity on the bench batch: foreground IoU of the HIP train-mode
    forward vs the oracle (fp32 CPU restatement of the reference) on the same
    weights and images, reference aggregation (utils.py:120-151).  Every rank
    runs the HIP forward (it moves the BN running statistics and the fp8
    delayed-amax state, so all ranks must take it before the timed steps);
    only the rank with reference=True runs the oracle."""
    pkg = importlib.import_module("image-segmentation-project_amd")
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()} if reference else None
    with torch.no_grad():
        out = model(x)
        miou = pkg.calculate_metrics_from_logits(out, y)["iou"]
    if not reference:
        return miou, None
    import oracle
    ref = oracle.ReferenceUNet(width=width, use_attention=attention, backbone=backbone)
    ref.load_state_dict(sd)
    ref.train()
    with torch.no_grad():
        rl = ref(x.cpu())
        miou_ref = oracle.calculate_metrics(torch.sigmoid(rl), y.cpu())["iou"]
    return miou, miou_ref


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=16, help="images per GPU")
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--attention", action="store_true",
                    help="use_attention=True decoder (AttentionGate + ChannelAttention, the reference default)")
    ap.add_argument("--width", type=int, default=1,
                    help="channel multiplier: 1 = Base (configs[1]), 2 = Wide 128->1024 (configs[4], bf16 here)")
    ap.add_argument("--data", action="store_true",
                    help="bench the on-GPU data pipeline instead of the training step (--batch frames)")
    ap.add_argument("--data-src", type=int, default=1024, help="--data: source frame size")
    ap.add_argument("--cpu-frames", type=int, default=8, help="--data: frames in the CPU oracle sample")
    ap.add_argument("--backbone", default="resnet34", choices=["resnet34", "resnet50"],
                    help="encoder (advanced_models.py:72-130); resnet50 = Bottleneck 256..2048")
    ap.add_argument("--fp8", action="store_true",
                    help="forward convs with >= 128 input channels in fp8 e4m3 (configs[4] Wide fp8); bwd bf16")
    ap.add_argument("--cpu-steps", type=int, default=2)
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "16")))
    ap.add_argument("--no-cpu-baseline", action="store_true", help="skip the timed CPU oracle baseline")
    ap.add_argument("--no-parity", action="store_true", help="skip the step-0 mIoU parity leg against the CPU oracle")
    ap.add_argument("--graph", dest="graph", action="store_true", default=None,
                    help="replay the step as one HIP graph (default for --gpus 1)")
    ap.add_argument("--no-graph", dest="graph", action="store_false")
    ap.add_argument("--grad-dtype", default="fp32", choices=["fp32", "bf16"],
                    help="N>1: gradient exchange dtype (bf16: opt-in compression, ddp.py)")
    ap.add_argument("--torch-adam", action="store_true",
                    help="torch.optim.Adam (foreach) instead of the fused HIP Adam (optim.py)")
    args = ap.parse_args()

    if args.data:
        return data_bench(args)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    pkg = importlib.import_module("image-segmentation-project_amd")
    ddp = importlib.import_module("image-segmentation-project_amd.ddp")

    torch.manual_seed(0)
    model = pkg.UNetWithBackbone(n_classes=1, backbone=args.backbone, pretrained=False,
                                  use_attention=args.attention, width=args.width, fp8=args.fp8).to(dev)
    if world > 1:
        ddp.enable_data_parallel(model, grad_dtype=args.grad_dtype)
    use_graph = args.graph if args.graph is not None else world == 1
    if args.torch_adam:
        opt = torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=1e-5, capturable=use_graph)
    else:
        opt = importlib.import_module("image-segmentation-project_amd.optim").Adam(
            model.parameters(), lr=1e-3, weight_decay=1e-5)
    crit = pkg.get_loss_function({"loss_fn": "bce"})
    xs, ms = pkg.synthetic_cells(args.batch, args.size, args.size, seed=1234 + rank)
    x = torch.from_numpy(xs).to(dev)
    y = torch.from_numpy(ms).to(dev)
    model.train()
    parity = None
    if not args.no_parity:  # step-0 weights; the HIP forward on every rank, the oracle on rank 0
        parity = miou_parity(model, x, y, args.width, args.attention, args.backbone, reference=rank == 0)
        if rank != 0:
            parity = None
    if world > 1:
        dist.barrier()

    def eager_step():
        out = model(x)
        loss = crit(out, y)
        opt.zero_grad()
        loss.backward()
        opt.step()
        return out, loss

    step = pkg.GraphedTrainStep(model, crit, opt, x, y) if use_graph else eager_step

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out, loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    # metric side: mIoU (reference aggregation) of the last step's pre-step logits
    miou = pkg.calculate_metrics_from_logits(out.detach(), y)["iou"]
    imgs = args.batch * args.steps * world
    flops_step = model.step_flops((args.batch, 1, args.size, args.size), training=True)
    ms_step = dt / args.steps * 1e3
    step_tflops = flops_step / (dt / args.steps) / 1e12
    # dominant kernel family (implicit-GEMM conv fwd/dgrad/wgrad): per-launch HIP
    # events around every launch of one eager step right after the timed region
    plan = model._last_plan
    torch.cuda.synchronize()
    plan.profile(True)
    eager_step()
    torch.cuda.synchronize()
    recs = plan.profile_report()
    plan.profile(False)
    conv = [r for r in recs if r[2] > 0]
    conv_ms = sum(r[1] for r in conv)
    conv_tflops = sum(r[2] for r in conv) / 1e9 / conv_ms if conv_ms > 0 else 0.0
    kernel_ms_total = sum(r[1] for r in recs)
    # dominant kernel = the conv template instance with the most event time
    by_kernel = {}
    for name, ms_, fl, kern in conv:
        k = by_kernel.setdefault(kern, [0.0, 0.0, 0])
        k[0] += ms_
        k[1] += fl
        k[2] += 1
    dom = max(by_kernel, key=lambda k: by_kernel[k][0])
    dom_ms, dom_fl, dom_n = by_kernel[dom]
    achieved_tflops = dom_fl / 1e9 / dom_ms
    dom_peak = MFMA_FP8_PEAK_TFLOPS if dom.startswith("conv_f8_kernel") else MFMA_BF16_PEAK_TFLOPS
    traffic, traffic_src = pmc_traffic(dom, config_key(args.backbone, args.width, args.attention, args.fp8,
                                                        args.batch, args.size))
    dom_us = dom_ms / dom_n * 1e3
    line = {
        "metric": "images/sec + mIoU, 512x512 U-Net bf16 at 1/2/4/8 MI355X",
        "value": round(imgs / dt, 3),
        "unit": "images/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp8-e4m3 fwd convs (C>=128) + bf16" if args.fp8 else "bf16",
        "data": "synthetic (Gaussian cells, seed 1234+rank), random-init weights",
        "miou": round(miou, 6),
        "miou_step0": None if parity is None else round(parity[0], 6),
        "miou_ref": None if parity is None else round(parity[1], 6),
        "miou_abs_diff": None if parity is None else float(f"{abs(parity[0] - parity[1]):.3e}"),
        "config": {"workload": ("Base" if args.width == 1 else f"Wide (x{args.width} channels)")
                   + f" U-Net {args.backbone} " + ("attention" if args.attention else "no-attention")
                   + " train step (fwd+bce+bwd+Adam)",
                   "global_batch": args.batch * world, "image": f"{args.size}x{args.size}",
                   "parallelism": f"dp{world}", "fp8": bool(args.fp8),
                   "grad_exchange": args.grad_dtype if world > 1 else None},
        "roofline": {"bound": "mfma", "achieved": round(achieved_tflops, 2), "peak": dom_peak,
                     "unit": "TFLOP/s", "frac": round(achieved_tflops / dom_peak, 4),
                     "traffic": traffic,
                     # PMC bytes per launch (committed profile named here) over this
                     # run's measured average launch time: the kernel's HBM rate
                     "traffic_source": traffic_src,
                     "hbm_gbs": None if traffic is None else round(traffic / dom_us / 1e3, 1),
                     "hbm_peak_gbs": HBM_PEAK_GBS,
                     "kernel": dom, "launches_per_step": dom_n,
                     "avg_launch_us": round(dom_us, 2),
                     "kernel_ms_per_step": round(dom_ms, 3),
                     "conv_family_tflops": round(conv_tflops, 2), "conv_ms_per_step": round(conv_ms, 3),
                     "all_kernels_ms_per_step": round(kernel_ms_total, 3),
                     "step_tflops": round(step_tflops, 2),
                     "step_frac": round(step_tflops / MFMA_BF16_PEAK_TFLOPS, 4)},
        "graph": bool(use_graph),
        "optimizer": "torch.optim.Adam (foreach)" if args.torch_adam else "fused HIP Adam (unet_adam_step)",
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args.batch, args.size, args.cpu_steps, args.cpu_threads, args.width,
                                            args.attention, args.backbone)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

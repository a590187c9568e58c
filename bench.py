#!/usr/bin/env python3
"""Headline benchmark: VGG-11 training throughput (images/sec, whole job) on N MI355X.

    python bench.py --gpus 1 --steps 40 --warmup 10
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Config = BASELINE.json: VGG-11 (reference architecture, random init), synthetic CIFAR-10-shaped
data (3x32x32, 10 classes, on-device crop/flip/normalise), bf16 compute with fp32 master
weights/grads, SGD(0.1, 0.9, 1e-4), part-3 strategy (bucketed DDP on RCCL, collectives issued in
stream order inside the captured step).
Default protocol = the reference's (/root/reference/part3/main.py:167): a FIXED
global batch of 256 split int(256/N) per GPU (strong scaling: 256, 128, 64, 32 images per GPU at
N = 1, 2, 4, 8; 255 in total at N = 3). ``--per-gpu-batch B`` instead fixes B images per GPU
(weak scaling, global batch B*N). Every timed step is a full training step (augment + forward +
backward + gradient all-reduce + optimizer), replayed from hipGraphs.
W untimed warm-up steps, then EXACTLY K timed steps bracketed by barrier + synchronize; the
elapsed time is the MAX over ranks; rank 0 prints one JSON line. After the timed region the
reference's own timing window is also measured and reported as an extra key: 40 iterations, each
followed by a host synchronisation (the reference's per-iteration ``loss.item()``), the wall time
of iterations 1..39 averaged (iteration 0 excluded, /root/reference/part1/main.py:86-91) and
then averaged over ranks (report printed p.4 §3) -> ``avg_ms_iter_1_39``.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

BASELINE_IMG_S = 385.5  # reference part 3 (DDP), 4 CPU nodes, Table 1


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=40)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--model", default="vgg11")
    p.add_argument("--global-batch", type=int, default=None,
                   help="strong scaling: split int(B/N) per GPU (default 256, the reference's)")
    p.add_argument("--per-gpu-batch", type=int, default=None,
                   help="weak scaling: B images per GPU (global batch B*N)")
    p.add_argument("--ref-window", type=int, default=40,
                   help="iterations of the reference timing window (0 = skip)")
    p.add_argument("--strategy", default="ddp",
                   choices=["ddp", "allreduce", "gather_scatter", "gather_broadcast"])
    # Bucket sizing for xGMI: --bucket-mb auto. The reference DDP default is
    # 25 MB (+1 MB first bucket); pass --bucket-mb 25 --first-bucket-mb 1 for that plan.
    p.add_argument("--bucket-mb", default="auto",
                   help="DDP bucket cap in MiB, or 'auto' (parallel/bucket_plan.py): one bucket "
                        "when the collectives are inline in the captured step, else sized from "
                        "the all-reduce bandwidth table (parallel/comm_tuning.json)")
    p.add_argument("--first-bucket-mb", default="auto")
    p.add_argument("--grad-comm", default="fp32", choices=["fp32", "bf16"],
                   help="DDP gradient all-reduce dtype (bf16 halves the xGMI bytes; default "
                        "fp32 = the reference's gradient precision)")
    p.add_argument("--segmented", default=None,
                   help="DDP: cut the captured step before these fused stages (comma list) and "
                        "run each bucket's all-reduce + optimizer update on the comm stream "
                        "while the earlier layers' backward runs (engine/step.py "
                        "SegmentedDDPStep); 0 = one graph, inline collectives. Default on >1 "
                        "GPUs: VGG 4, ResNet-50 8,14; on 1 GPU 0. Env DDP_AMD_SEGMENTED overrides")
    p.add_argument("--zero", action="store_true",
                   help="pipelined DDP step with the ZeRO-1 sharded update (reduce-scatter -> "
                        "SGD on 1/N of the parameters -> all-gather, parallel/zero.py)")
    p.add_argument("--update", default="auto",
                   help="pipelined DDP step, per gradient bucket: 'allreduce' = fp32 all-reduce + "
                        "replicated SGD; 'shard16' = fp32 reduce-scatter + SGD on this rank's "
                        "shard + all-gather of the bf16 operand bytes (parallel/zero.py "
                        "ShardedBf16Update: 25%% fewer wire bytes, 1/N of the SGD); 'auto' = the "
                        "cheaper of the two per bucket from the all-reduce / reduce-scatter / "
                        "all-gather timings of the start-up probe (parallel/cut_plan.py); or one "
                        "code per bucket, last layers first, e.g. s16,s16,ar")
    p.add_argument("--lr", type=float, default=None,
                   help="SGD learning rate (default: the reference's 0.1 for VGG; 0.01 for "
                        "ResNet-50, whose random-init training on the synthetic data is chaotic "
                        "at 0.1 in fp32 PyTorch as well: profiles/r2_resnet50_b256.md)")
    p.add_argument("--no-graph", action="store_true")
    p.add_argument("--train-size", type=int, default=None)
    p.add_argument("--json-out", default=None)
    p.add_argument("--attempt-timeout", type=float, default=480.0,
                   help="N > 1: kill an attempt's ranks after this many seconds and fall back "
                        "(utils/ladder.py)")
    p.add_argument("--no-fallback", action="store_true",
                   help="N > 1: run the given plan once, without the fallback ladder "
                        "(utils/ladder.py: planned -> inline captured DDP -> eager DDP)")
    p.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                   help="cpu: the same protocol on ATen + Gloo (fp32, eager; the multi-rank "
                        "launch / fallback / JSON plumbing without a GPU)")
    return p.parse_args()


def launch_or_check(args):
    """``--gpus N`` (N > 1) runs the ranks as attempts of the fallback ladder (utils/ladder.py):
    without an outer launcher this process spawns the N ranks of each attempt itself; as one
    rank of an outer launcher (torchrun) it supervises its own rank's child of each attempt.
    Either way it makes no GPU call and returns the exit code. Returns None when this process is
    a rank that should run (N = 1, an attempt's child, or --no-fallback under a launcher)."""
    from ddp_amd.utils import ladder
    from ddp_amd.utils.launch import self_launch, under_launcher, visible_devices
    attempts = ladder.default_attempts(args.strategy)
    if not under_launcher():
        if args.gpus <= 1:
            return None
        if args.device == "cuda" and visible_devices() < args.gpus:
            raise SystemExit(f"--gpus {args.gpus} but only {visible_devices()} GPU(s) visible: "
                             f"refusing to run {args.gpus} ranks on fewer devices")
        if args.no_fallback:
            return self_launch(__file__, sys.argv[1:], args.gpus, timeout_s=args.attempt_timeout,
                               require_devices=False)
        return ladder.run_self(__file__, sys.argv[1:], args.gpus, attempts,
                               timeout_s=args.attempt_timeout)
    world = int(os.environ["WORLD_SIZE"])
    if world != args.gpus:
        raise SystemExit(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report "
                         f"a {world}-rank run as {args.gpus} GPUs")
    if world > 1 and not args.no_fallback and ladder.CHILD_ENV not in os.environ:
        return ladder.run_under_launcher(__file__, sys.argv[1:], attempts,
                                         timeout_s=args.attempt_timeout)
    return None


def main():
    args = parse()
    rc = launch_or_check(args)
    if rc is not None:
        sys.exit(rc)
    if args.device == "cpu":
        sys.exit(run_cpu(args))
    sys.exit(run_gpu(args))


def run_gpu(args):
    import torch
    import torch.distributed as dist
    import ddp_amd
    from ddp_amd.data import SyntheticCIFAR10, SyntheticImageNet, DeviceLoader
    from ddp_amd.engine import TrainStep, SegmentedDDPStep, CrossEntropyLoss
    from ddp_amd.engine.step import default_cuts
    from ddp_amd.models import build
    from ddp_amd.optim import FusedSGD
    from ddp_amd.parallel import (DistributedDataParallel, RcclCommunicator, STRATEGIES,
                                  check_replicas)
    from ddp_amd.utils import Watchdog, fault_point, ladder, seed_everything

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    if ndev < min(world, args.gpus) or local_rank >= ndev:
        raise SystemExit(f"[bench] rank {rank}: {ndev} GPU(s) visible for {world} ranks "
                         f"(LOCAL_RANK {local_rank})")
    torch.cuda.set_device(local_rank)
    device = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)  # control plane (TCPStore)
    # failure tests: "bench" fires in every fallback attempt, "bench<k>" in attempt k only
    fault_point(rank, "bench")
    fault_point(rank, "bench" + os.environ.get(ladder.ATTEMPT_ENV, "0"))
    comm = RcclCommunicator(rank, world, local_rank)
    # proof of the rank count: what RCCL itself reports for the data-plane communicator
    rccl_ranks = comm.comm.count()
    if world > 1 and rccl_ranks != world:
        raise SystemExit(f"[bench] RCCL communicator has {rccl_ranks} ranks, expected {world}")
    # failure detection: on >1 ranks a watchdog thread aborts the RCCL
    # communicator and exits non-zero when no progress is reported for DDP_AMD_WATCHDOG_S
    # seconds (default 300) or RCCL reports an async error, instead of hanging on a dead peer
    watchdog = None
    wd_s = float(os.environ.get("DDP_AMD_WATCHDOG_S", "300"))
    if world > 1 and wd_s > 0:
        watchdog = Watchdog(timeout_s=wd_s, comm=comm, poll_s=min(5.0, wd_s / 4)).start()

    def beat():
        if watchdog is not None:
            watchdog.beat()

    seed_everything(ddp_amd.SEED)
    resnet = args.model.startswith("resnet")
    if args.per_gpu_batch:
        B, scaling = args.per_gpu_batch, "weak"
    elif args.global_batch or not resnet:
        B, scaling = int((args.global_batch or 256) / world), "strong"
    else:
        # ResNet-50 (the driver's large-gradient stress config, not the reference's): 256
        # images per GPU (~60 GB of activations of the 288 GB HBM; 31% more images/s than 64 per
        # GPU on one MI355X, and 4x less gradient traffic per image)
        B, scaling = 256, "weak"
    if B < 1:
        raise SystemExit(f"global batch too small for {world} ranks")
    global_batch = B * world
    ds = (SyntheticImageNet(True, n=args.train_size) if resnet
          else SyntheticCIFAR10(True, n=args.train_size))
    loader = DeviceLoader(ds, B, device, world, rank, train=True, cpad=8)
    model = build(args.model).to(device)
    criterion = CrossEntropyLoss()
    sync = None
    # Multi-GPU default: the pipelined step — each bucket's all-reduce + optimizer update runs
    # on the comm stream while the earlier layers' backward runs (one-GPU study with an
    # 8-GPU-sized stand-in collective: profiles/r2_pipelined_ddp.md); one GPU has no collective
    # to hide -> one graph.
    # On > 1 GPUs without --segmented / DDP_AMD_SEGMENTED the cuts are chosen on the node below
    # (parallel/cut_plan.py: measured stage backward times x the start-up all-reduce probe)
    cut_source = "cli" if args.segmented is not None else (
        "env" if "DDP_AMD_SEGMENTED" in os.environ else "default")
    if args.segmented is None:
        args.segmented = os.environ.get("DDP_AMD_SEGMENTED",
                                        default_cuts(args.model, B) if world > 1 else "0")
    cuts = [int(v) for v in str(args.segmented).split(",") if int(v) > 0]
    segmented = bool(cuts) and args.strategy == "ddp" and not args.no_graph
    # all-reduce bandwidth of THIS node, measured on the live communicator before the bucket
    # plan is made (DDP_AMD_COMM_PROBE=0 falls back to comm_tuning.json)
    comm_table = None
    if world > 1 and os.environ.get("DDP_AMD_COMM_PROBE", "1") != "0":
        from ddp_amd.parallel.bucket_plan import probe_table
        comm_table = probe_table(comm, world, args.grad_comm, device=device)
        beat()
    if args.strategy == "ddp":
        # captured step (``captured``): the reducer's collectives are inline in the graph (or
        # bypassed by the pipelined step) -> 'auto' plans one bucket = one collective
        model = DistributedDataParallel(model, comm, bucket_cap_mb=args.bucket_mb,
                                        first_bucket_cap_mb=args.first_bucket_mb,
                                        grad_comm_dtype=args.grad_comm,
                                        captured=not args.no_graph, comm_table=comm_table)
    else:
        fn = STRATEGIES[args.strategy]
        sync = lambda m: fn(m, comm)  # noqa: E731
    lr = args.lr if args.lr is not None else (0.01 if resnet else 0.1)
    opt = FusedSGD(model.parameters(), lr=lr, momentum=0.9, weight_decay=1e-4)
    cut_plan = None
    if (segmented and cut_source == "default" and world > 1
            and os.environ.get("DDP_AMD_CUT_PLAN", "1") != "0"):
        cut_plan = choose_cuts_on_node(model, opt, criterion, loader, args, world, comm_table)
        beat()
        if cut_plan.get("cuts"):
            cuts = cut_plan["cuts"]
            args.segmented = ",".join(str(c) for c in cuts)
            cut_source = cut_plan["source"]
    update_plan = None
    if segmented:
        emu_gbps = float(os.environ.get("DDP_AMD_EMULATE_COMM_GBPS", "0"))
        emu_world = int(os.environ.get("DDP_AMD_EMULATE_WORLD", "8"))
        update_plan = choose_update(args, model, cuts, world, comm_table, cut_plan,
                                    emu_world if (world == 1 and emu_gbps > 0) else world)
        step = SegmentedDDPStep(model, opt, criterion, loader, split=cuts,
                                emulate=int(os.environ.get("DDP_AMD_EMULATE_COMM", "0")),
                                emulate_gbps=emu_gbps, emulate_world=emu_world,
                                grad_comm=args.grad_comm, zero=args.zero,
                                update=update_plan["update"])
    elif args.zero:
        raise SystemExit("--zero needs the pipelined DDP step (--segmented with cuts, hipGraph)")
    else:
        step = TrainStep(model, opt, criterion, loader, sync=sync, use_graph=not args.no_graph)

    graph_ok = False
    nwarm = max(args.warmup, 2)
    step.warmup(min(nwarm, 2))
    if not args.no_graph:
        try:
            step.capture()
            graph_ok = True
        except Exception as e:  # fall back to eager steps, loudly
            print(f"[bench] hipGraph capture failed ({e!r}); timing eager steps", file=sys.stderr)
            step.graph = None
    arena = model.arena if hasattr(model, "arena") else opt.arena
    if graph_ok and world > 1:
        if not step.validate_distributed(arena, world):
            graph_ok = False
            print("[bench] replicas diverged under graph replay; timing eager steps",
                  file=sys.stderr)
        nwarm = max(nwarm - 1, 2)
    beat()
    for _ in range(nwarm - 2):
        step.step()
    torch.cuda.synchronize()
    warm_loss = step.pop_loss()
    beat()

    def barrier():
        if world > 1:
            dist.barrier()

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step.step()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    beat()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    loss = step.pop_loss() / max(args.steps, 1)

    # the reference's window: per-iteration wall time incl. a host sync, iterations 1..39
    ref_ms = None
    if args.ref_window > 1:
        barrier()
        tot = 0.0
        for i in range(args.ref_window):
            t = time.perf_counter()
            step.step()
            torch.cuda.synchronize()
            if i > 0:
                tot += time.perf_counter() - t
            beat()
        ref = torch.tensor([tot / (args.ref_window - 1)], dtype=torch.float64)
        if world > 1:
            dist.all_reduce(ref)
            ref /= world
        ref_ms = float(ref.item()) * 1000.0
        step.pop_loss()
    consistent = True
    if world > 1:
        if hasattr(step, "sync_masters"):
            step.sync_masters()  # sharded updates: owners' fp32 masters to every rank
        consistent = check_replicas(arena, world)
    plan = comm_plan(args, world, step, model, cuts, segmented, comm_table)
    plan["cut_source"] = cut_source if segmented else None
    if cut_plan is not None:
        plan["cut_plan"] = cut_plan
    if update_plan is not None:
        plan["update_plan"] = update_plan
    ms = elapsed / args.steps * 1000.0
    value = global_batch * args.steps / elapsed
    out = {
        "metric": "images/sec (whole node) VGG-11 CIFAR-10" if not resnet
        else "images/sec (whole node) ResNet-50 synthetic ImageNet",
        "value": round(value, 2),
        "unit": "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 4),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": round(value / BASELINE_IMG_S, 2) if not resnet else None,
        "dtype": "bf16",
        "data": "synthetic (CIFAR-10-shaped 3x32x32, 10 classes, on-device crop/flip/normalise; random-init weights)"
        if not resnet else "synthetic (ImageNet-shaped 3x224x224, 1000 classes)",
        "config": {"model": args.model, "global_batch": global_batch, "per_gpu_batch": B,
                   "seq_len": None, "parallelism": f"dp{world}",
                   "strategy": {"ddp": "part3 bucketed DDP", "allreduce": "part2b all_reduce",
                                "gather_scatter": "part2a gather/scatter",
                                "gather_broadcast": "part2a gather/broadcast"}[args.strategy],
                   "hipgraph": graph_ok,
                   "buckets": (len(step.buckets) if segmented else len(getattr(model, "buckets", []))),
                   "grad_comm": args.grad_comm,
                   "comm": (f"segmented@{args.segmented}" if segmented else "overlap-stream" if getattr(getattr(model, "reducer", None), "overlap",
                                                         lambda: False)() else "inline"),
                   "optimizer": f"SGD(lr={lr:g}, momentum=0.9, wd=1e-4) fused" +
                                (", ZeRO-1 sharded" if args.zero else "") +
                                (", sharded update + bf16 operand all-gather on buckets "
                                 + ",".join(str(j) for j, u in enumerate(update_plan["update"])
                                            if u == "s16")
                                 if update_plan and "s16" in update_plan["update"] else "")},
        "launcher": os.environ.get("DDP_AMD_LAUNCHER",
                                   "torchrun" if "TORCHELASTIC_RUN_ID" in os.environ
                                   else ("env" if world > 1 else "single-process")),
        "rccl_ranks": rccl_ranks,
        "device_count": torch.cuda.device_count(),
        "rccl_version": _version_str(native_version()),
        "gpu": torch.cuda.get_device_name(local_rank),
        "comm_plan": plan,
        "avg_ms_iter_1_39": round(ref_ms, 4) if ref_ms is not None else None,
        "img_s_iter_1_39": round(global_batch / ref_ms * 1000.0, 2) if ref_ms else None,
        "train_loss_mean": round(loss, 4),
        "warmup_loss_sum": round(warm_loss, 4),
        "replicas_consistent": consistent,
    }
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if watchdog is not None:
        watchdog.stop()
    if world > 1:
        dist.destroy_process_group()
    # a result whose replicas diverged is not reported as a success (the ladder falls back)
    return 0 if consistent else ladder.RC_REPLICAS


def run_cpu(args):
    """The benchmark protocol on the CPU (ATen kernels, Gloo, fp32, eager steps): warm-up, K
    timed steps between barriers, max over ranks, rank 0's JSON line. Exercises the multi-rank
    launch, the fallback ladder and the JSON contract without a GPU (tests/test_bench_cpu.py);
    its numbers are CPU numbers (``"device": "cpu"``)."""
    import torch
    import torch.distributed as dist
    import ddp_amd
    from ddp_amd.data import SyntheticCIFAR10
    from ddp_amd.data.loader import CPULoader
    from ddp_amd.engine import CrossEntropyLoss
    from ddp_amd.models import build
    from ddp_amd.optim import FusedSGD
    from ddp_amd.parallel import (DistributedDataParallel, STRATEGIES, TorchCommunicator,
                                  check_replicas)
    from ddp_amd.utils import Watchdog, fault_point, ladder, seed_everything

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    torch.set_num_threads(1)  # one core per rank (the CPU tests run several ranks)
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    fault_point(rank, "bench")
    fault_point(rank, "bench" + os.environ.get(ladder.ATTEMPT_ENV, "0"))
    watchdog = None
    wd_s = float(os.environ.get("DDP_AMD_WATCHDOG_S", "300"))
    if world > 1 and wd_s > 0:
        watchdog = Watchdog(timeout_s=wd_s, poll_s=min(1.0, wd_s / 4)).start()
    seed_everything(ddp_amd.SEED)
    B = args.per_gpu_batch or int((args.global_batch or 256) / world)
    scaling = "weak" if args.per_gpu_batch else "strong"
    loader = CPULoader(SyntheticCIFAR10(True, n=args.train_size), B, world, rank)
    model = build(args.model)
    comm = TorchCommunicator() if world > 1 else None
    sync = None
    if comm is not None and args.strategy == "ddp":
        model = DistributedDataParallel(model, comm, bucket_cap_mb=25, first_bucket_cap_mb=1)
    elif comm is not None:
        fn = STRATEGIES[args.strategy]
        sync = lambda m: fn(m, comm)  # noqa: E731
    lr = args.lr if args.lr is not None else 0.1
    opt = FusedSGD(model.parameters(), lr=lr, momentum=0.9, weight_decay=1e-4)
    crit = CrossEntropyLoss()
    batches = iter(())
    loss_sum = [0.0]

    def step():
        nonlocal batches
        try:
            x, y = next(batches)
        except StopIteration:
            batches = iter(loader)
            x, y = next(batches)
        opt.zero_grad()
        loss = crit(model(x), y)
        loss.backward()
        if sync is not None:
            sync(model)
        opt.step()
        loss_sum[0] += float(loss.item())
        if watchdog is not None:
            watchdog.beat()

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    loss_sum[0] = 0.0
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    arena = model.arena if hasattr(model, "arena") else opt.arena
    consistent = check_replicas(arena, world)
    ms = elapsed / max(args.steps, 1) * 1000.0
    value = B * world * args.steps / elapsed
    out = {
        "metric": "images/sec (whole node) VGG-11 CIFAR-10", "value": round(value, 2),
        "unit": "images/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": scaling,
        "vs_baseline": round(value / BASELINE_IMG_S, 2), "dtype": "fp32", "device": "cpu",
        "data": "synthetic (CIFAR-10-shaped 3x32x32, 10 classes; random-init weights)",
        "config": {"model": args.model, "global_batch": B * world, "per_gpu_batch": B,
                   "seq_len": None, "parallelism": f"dp{world}", "strategy": args.strategy,
                   "hipgraph": False, "comm": "gloo"},
        "launcher": os.environ.get("DDP_AMD_LAUNCHER", "torchrun" if "TORCHELASTIC_RUN_ID"
                                   in os.environ else ("env" if world > 1 else "single-process")),
        "train_loss_mean": round(loss_sum[0] / max(args.steps, 1), 4),
        "replicas_consistent": consistent,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if watchdog is not None:
        watchdog.stop()
    if world > 1:
        dist.destroy_process_group()
    return 0 if consistent else ladder.RC_REPLICAS


def choose_cuts_on_node(model, opt, criterion, loader, args, world, comm_table):
    """Pipelined-step cuts from THIS node's measurements (parallel/cut_plan.py): every fused
    stage's backward time at this per-GPU batch (device events on a cut-everywhere step,
    engine/step.py profile_stage_times; state rolled back) and the all-reduce curve of the
    start-up probe (or comm_tuning.json). The stage times are maxed over ranks so every rank
    picks the same cuts. Any failure keeps the fallback cuts and says why."""
    import torch
    import torch.distributed as dist
    from ddp_amd.engine.step import profile_stage_times
    from ddp_amd.parallel.bucket_plan import load_table, rows_for
    from ddp_amd.parallel.cut_plan import plan_cuts, seg_boundary_us
    inner = model.module
    n = inner.n_stages()
    arena = model.arena
    pidx = {id(p): i for i, p in enumerate(arena.params)}
    first = [pidx[id(inner.first_param_of_stage(i))] for i in range(n)] + [len(arena.params)]
    off = list(arena.offsets) + [arena.total]
    pbytes = [4 * (off[first[i + 1]] - off[first[i]]) for i in range(n)]
    ok = 1
    try:
        stage_us = profile_stage_times(model, opt, criterion, loader, n)
    except Exception as e:  # keep the fallback cuts, loudly (on every rank: see below)
        print(f"[bench] stage profiling failed ({e!r}); fallback cuts", file=sys.stderr)
        ok, stage_us = 0, [0.0] * n
    # collective decision: every rank takes part in both reductions whatever happened locally
    flag = torch.tensor([ok], dtype=torch.int64)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    t = torch.tensor(stage_us, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if int(flag.item()) == 0:
        return {"source": "fallback (stage profiling failed on a rank)", "cuts": None}
    stage_us = [float(v) for v in t]
    rows, table_src = rows_for(comm_table or load_table(), world, args.grad_comm)
    wire = 0.5 if args.grad_comm == "bf16" else 1.0
    # 'auto' may pick the sharded update for a bucket only when THIS node's reduce-scatter and
    # all-gather were measured by the start-up probe (never from the model table alone)
    upd = "auto" if (args.update == "auto" and args.grad_comm == "fp32" and not args.zero
                     and shard_columns_measured(comm_table, world)) else \
        ("shard16" if args.update == "shard16" else "allreduce")
    best, ranked = plan_cuts(stage_us, pbytes, rows, wire_scale=wire, update=upd, world=world,
                             seg_overhead_us=seg_boundary_us(loader.batch_size))
    return {"source": "probe" if comm_table is not None else "table", "comm_table": table_src,
            "cuts": best["cuts"], "stage_us": [round(v, 1) for v in stage_us],
            "stage_param_bytes": pbytes, "bucket_bytes": best["bucket_bytes"],
            "predicted_allreduce_us": [round(v, 1) for v in best["allreduce_us"]],
            "predicted_step_us": round(best["step_us"], 1),
            "predicted_exposed_us": round(best["exposed_us"], 1), "update": best["update"],
            "top5": ranked[:5]}


def choose_update(args, model, cuts, world, comm_table, cut_plan, plan_world):
    """Per-bucket update plan of the pipelined step ("ar" = all-reduce + replicated SGD, "s16" =
    reduce-scatter + shard SGD + bf16 operand all-gather). --update allreduce / shard16 force one
    plan for every bucket; auto takes the cut planner's per-bucket choice when it ran, else
    prices each bucket with parallel/cut_plan.py bucket_costs on the probe's (or the table's)
    collective timings. The sharded plan needs fp32 gradients, no --zero, and buckets that
    divide into 4-element multiples per rank (64-aligned buckets: 1, 2, 4, 8 ranks)."""
    from ddp_amd.parallel.bucket_plan import load_table, rows_for
    from ddp_amd.parallel.cut_plan import SGD_US_PER_BYTE, bucket_costs
    inner = model.module
    arena = model.arena
    pidx = {id(p): i for i, p in enumerate(arena.params)}
    first = sorted(pidx[id(inner.first_param_of_stage(c))] for c in cuts)
    bounds = [len(arena.params)] + first[::-1] + [0]
    ranges = []
    for j in range(len(bounds) - 1):
        i1, i0 = bounds[j], bounds[j + 1]
        ranges.append((arena.offsets[i0], arena.offsets[i1] if i1 < len(arena.params) else arena.total))
    nb = len(ranges)
    if args.update not in ("auto", "allreduce", "shard16"):
        codes = args.update.split(",")
        if len(codes) != nb or any(c not in ("ar", "s16") for c in codes):
            raise SystemExit(f"--update {args.update}: need {nb} codes (ar / s16) for cuts {cuts}")
        return {"update": codes, "source": "forced per bucket"}
    even = plan_world >= 1 and all((hi - lo) % plan_world == 0 and ((hi - lo) // plan_world) % 4 == 0
                                   for lo, hi in ranges)
    allowed = args.grad_comm == "fp32" and not args.zero and even
    emu_gbps = float(os.environ.get("DDP_AMD_EMULATE_COMM_GBPS", "0"))
    measured = shard_columns_measured(comm_table, world) or (world == 1 and emu_gbps > 0)
    if args.update == "allreduce" or not allowed or (plan_world <= 1 and args.update == "auto") \
            or (args.update == "auto" and not measured):
        why = ("forced" if args.update == "allreduce" else "one rank: nothing to shard"
               if plan_world <= 1 else "sharded plan not applicable (bf16 wire, --zero or "
               "uneven shards)" if not allowed else "no measured reduce-scatter / all-gather "
               "curve on this node: all-reduce")
        if args.update == "shard16" and not allowed:
            raise SystemExit("--update shard16 needs --grad-comm fp32, no --zero and buckets "
                             f"divisible by {plan_world} ranks")
        return {"update": ["ar"] * nb, "source": why}
    if args.update == "shard16":
        return {"update": ["s16"] * nb, "source": "forced"}
    if cut_plan is not None and cut_plan.get("update") and len(cut_plan["update"]) == nb:
        return {"update": list(cut_plan["update"]), "source": "cut planner"}
    if world == 1 and emu_gbps > 0:  # one-GPU stand-in study: price the stand-in itself
        from ddp_amd.parallel.cut_plan import stand_in_rows
        rows, src = stand_in_rows(plan_world, emu_gbps), f"stand-in {emu_gbps:g} GB/s"
    else:
        rows, src = rows_for(comm_table or load_table(), max(plan_world, 2), "fp32")
    sgd = (lambda b: b * SGD_US_PER_BYTE)
    out, costs = [], []
    for lo, hi in ranges:
        (t_ar, u_ar), (t_s, u_s) = bucket_costs(rows, 4 * (hi - lo), 1.0, plan_world, sgd)
        out.append("s16" if t_s + u_s < t_ar + u_ar else "ar")
        costs.append({"bytes": 4 * (hi - lo), "ar_us": round(t_ar + u_ar, 1),
                      "s16_us": round(t_s + u_s, 1)})
    return {"update": out, "source": f"priced on {src}", "bucket_costs": costs}


def shard_columns_measured(comm_table, world):
    """True when the start-up probe measured this node's reduce-scatter and bf16 all-gather
    times (parallel/bucket_plan.py probe_table): the only basis on which --update auto may
    choose the sharded update."""
    if not comm_table:
        return False
    from ddp_amd.parallel.bucket_plan import rows_for
    rows, _ = rows_for(comm_table, world, "fp32")
    return bool(rows) and all("rs_us" in r and "ag16_us" in r for r in rows)


def native_version():
    from ddp_amd.ops.common import native
    return native().RcclComm.version()


def _version_str(v):
    # NCCL_VERSION_CODE = major * 10000 + minor * 100 + patch (>= 2.9)
    return f"{v // 10000}.{v // 100 % 100}.{v % 100}" if v else None


def comm_plan(args, world, step, model, cuts, segmented, comm_table=None):
    """Which gradient-communication plan this run used: collective granularity, bucket bytes
    on the wire, wire dtype, and the all-reduce bandwidth table with its knee: measured on this
    node's communicator at start-up (world > 1), else parallel/comm_tuning.json ("model" until
    tools/comm_bench.py --write-table measured a node). With measured rows, the predicted
    all-reduce time of every bucket is reported too."""
    from ddp_amd.parallel.bucket_plan import knee_bytes, load_table, predict_us, rows_for
    wire = 2 if args.grad_comm == "bf16" else 4
    rows, source = rows_for(comm_table or load_table(), max(world, 2), args.grad_comm)
    out = {"wire": args.grad_comm, "comm_table": source,
           "comm_table_knee_bytes": knee_bytes(rows) if rows else None,
           "collectives_live": world > 1}
    if comm_table is not None:
        out["probe_busbw_GBps"] = {str(r["bytes"]): r["busbw_GBps"] for r in rows}
    if segmented:
        out.update(kind="pipelined segments (bucket all-reduce + its SGD under the earlier "
                        "layers' backward)", cuts=cuts,
                   bucket_bytes=[(hi - lo) * wire for (_, (lo, hi)) in step.buckets],
                   zero=bool(args.zero))
    elif args.strategy == "ddp":
        out.update(kind="reducer buckets, inline in the captured step" if not args.no_graph
                   else "reducer buckets, comm stream", cuts=[],
                   bucket_bytes=[int(b[3]) * wire for b in getattr(model, "buckets", [])],
                   reason=getattr(model, "bucket_plan_reason", None))
    else:
        n = sum(1 for _ in model.parameters())
        out.update(kind=f"per-parameter {args.strategy} ({n} collectives)", cuts=[],
                   bucket_bytes=None)
    if comm_table is not None and out.get("bucket_bytes"):
        out["predicted_allreduce_us"] = [round(predict_us(rows, b), 1) for b in out["bucket_bytes"]]
    return out


if __name__ == "__main__":
    main()

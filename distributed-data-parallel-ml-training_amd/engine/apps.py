"""Entry points behind part1/main.py, part2/part2a/main.py, part2/part2b/main.py, part3/main.py.

Reference parity: ``main()`` of each reference script (part1/main.py:114-130,
part2/part2a/main.py:181-207, part2/part2b/main.py:169-195, part3/main.py:159-186):
parse -> [init process group + diagnostics] -> seed (89395) -> per-rank batch int(256/ws) ->
CrossEntropyLoss -> loaders (sharded train, unsharded test) -> VGG11 -> [DDP] ->
SGD(0.1, 0.9, 1e-4) -> 1 epoch of train_model + test_model -> [destroy_process_group].

On a GPU the same program runs on the gfx950 kernels with the native RCCL communicator;
on a CPU it runs on ATen + Gloo, exactly like the reference.
"""
import functools
import os

import torch

from .. import SEED
from ..data import SyntheticCIFAR10, make_loader
from ..models import build
from ..optim import FusedSGD
from ..parallel import (DistributedDataParallel, STRATEGIES, destroy, init_distributed_setup,
                        make_communicator, test_distributed_setup)
from ..utils import MetricsSink, Watchdog, load_checkpoint, local_rank_of, parse_all, pick_device, \
    save_checkpoint, seed_everything
from .trainer import CrossEntropyLoss, test_model, train_model, train_model_graph

PART_STRATEGY = {"part1": None, "part2a": "gather_scatter", "part2b": "allreduce", "part3": "ddp"}


def main(part, argv=None):
    strategy = PART_STRATEGY[part]
    distributed = strategy is not None
    args = parse_all(argv, distributed=distributed, description=f"ddp_amd {part}")
    torch.set_num_threads(args.threads)
    world, rank = 1, 0
    if distributed:
        world, rank = args.size, args.rank
        device = pick_device(args.device, local_rank=local_rank_of(rank))
        init_distributed_setup(args.master_ip, args.master_port, rank, world, backend="gloo")
        test_distributed_setup()
    else:
        device = pick_device(args.device)

    seed_everything(SEED)
    batch_size = int(args.global_batch / world)  # batch for one node

    criterion = CrossEntropyLoss()
    train_ds = SyntheticCIFAR10(train=True, seed=SEED, n=args.train_size)
    test_ds = SyntheticCIFAR10(train=False, seed=SEED, n=args.test_size)
    train_loader = make_loader(train_ds, batch_size, device, world, rank, train=True,
                               shard=distributed, max_batches=args.max_batches)
    test_loader = make_loader(test_ds, batch_size, device, train=False, shard=False)

    model = build(args.model).to(device)
    comm = make_communicator(device) if distributed else None
    if strategy == "ddp":
        # --graph on a GPU captures the step (TrainStep: inline collectives, one bucket is
        # best) unless the pipelined segmented step takes over (its own per-segment buckets)
        captured = bool(args.graph) and torch.device(device).type == "cuda"
        model = DistributedDataParallel(model, comm, bucket_cap_mb=args.bucket_mb,
                                        first_bucket_cap_mb=args.first_bucket_mb,
                                        captured=captured)
    optimizer = FusedSGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=0.0001)
    if args.resume:
        load_checkpoint(args.resume, model, optimizer)
    sync = None
    if strategy in STRATEGIES:
        sync = functools.partial(_sync, STRATEGIES[strategy], comm)
    metrics = MetricsSink(args.metrics, rank)
    # failure detection (the reference has none, part2/part2a/main.py:58): beat
    # once per iteration; no beat for --watchdog-s seconds or an RCCL async error -> abort the
    # communicator and exit non-zero instead of hanging on a dead peer
    watchdog = None
    if distributed and args.watchdog_s > 0:
        watchdog = Watchdog(timeout_s=args.watchdog_s, comm=comm,
                            poll_s=min(5.0, args.watchdog_s / 4)).start()

    step = None
    if args.graph and torch.device(device).type == "cuda":
        # opt-in: each iteration is one replay of the captured step (the warm-up steps consume
        # the first batches of the shard, like any other iteration would)
        # the warm-up steps train on the first batches: snapshot the training state and roll
        # it back after the capture, so the epoch starts exactly where the eager loop would
        from .step import TrainStep, SegmentedDDPStep, default_cuts
        arena = model.arena if hasattr(model, "arena") else optimizer.arena
        snap = (arena.data.clone(), optimizer.momentum_buffer.clone())
        split = [int(v) for v in os.environ.get("DDP_AMD_SEGMENTED",
                                                default_cuts(args.model, batch_size)).split(",")
                 if int(v) > 0]
        if (strategy == "ddp" and world > 1 and split
                and hasattr(model.module, "forward_loss_split")):
            # each bucket's all-reduce + optimizer update on the comm stream while the earlier
            # layers' backward runs (engine/step.py SegmentedDDPStep)
            step = SegmentedDDPStep(model, optimizer, criterion, train_loader, split=split)
        else:
            step = TrainStep(model, optimizer, criterion, train_loader, sync=sync)
        step.warmup(2)
        step.capture()
        torch.cuda.synchronize()
        if world > 1 and not step.validate_distributed(arena, world):
            print("[ddp_amd] replicas diverged under graph replay; running eager steps",
                  flush=True)
        torch.cuda.synchronize()
        arena.data.copy_(snap[0])
        optimizer.momentum_buffer.copy_(snap[1])
        optimizer.repack()
        train_loader.cursor.zero_()
        del snap

    for epoch in range(args.epochs):
        if step is not None:
            if epoch > 0:
                train_loader.set_epoch(epoch)
                step.capture()  # the augmentation seed is a launch argument: new epoch, new graph
            train_model_graph(step, train_loader, epoch, metrics=metrics, watchdog=watchdog,
                              rank=rank)
        else:
            train_loader.set_epoch(epoch)
            train_model(model, train_loader, optimizer, criterion, epoch, device, sync,
                        metrics=metrics, watchdog=watchdog, rank=rank)
        if not args.no_test:
            test_model(model, test_loader, criterion, device, watchdog=watchdog)

    if args.save and rank == 0:
        save_checkpoint(args.save, model, optimizer)
    if watchdog is not None:
        watchdog.stop()
    if distributed:
        destroy()
    return model


def _sync(fn, comm, model):
    fn(model, comm)

#!/usr/bin/env python3
"""All-reduce bus-bandwidth sweep on the native RCCL communicator (one process per GPU):

    python tools/comm_bench.py --gpus 8 [--dtype fp32|bf16] [--iters 20] [--max-mb 128] \
        [--write-table [PATH]]
    (or under torchrun: python -m torch.distributed.run --nproc-per-node 8 \
        --master-addr 127.0.0.1 tools/comm_bench.py --gpus 8 ...)

``--gpus N`` without an outer launcher spawns the N ranks itself (ddp_amd/utils/launch.py).
``--device cpu`` runs the same sweep over Gloo (TorchCommunicator) — the CPU tests drive the
launcher + sweep + table write end to end that way. Rank 0 prints one JSON line per message
size (parallel/commbench.py); ``--write-table`` merges the rows into the bucket-sizing table
(default parallel/comm_tuning.json) as "measured" for this world size and dtype."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (default: WORLD_SIZE, or 1); >1 without a launcher self-spawns")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--min-kb", type=float, default=64.0)
    ap.add_argument("--max-mb", type=float, default=128.0)
    ap.add_argument("--write-table", nargs="?", const="", default=None,
                    help="merge the measured rows into the bucket-sizing table "
                         "(default parallel/comm_tuning.json) for this world size and dtype")
    ap.add_argument("--launch-timeout", type=float, default=1800.0)
    a = ap.parse_args()
    from ddp_amd.utils.launch import self_launch, under_launcher
    if not under_launcher() and (a.gpus or 1) > 1:
        sys.exit(self_launch(__file__, sys.argv[1:], a.gpus, timeout_s=a.launch_timeout,
                             require_devices=a.device == "cuda"))
    import torch
    import torch.distributed as dist
    from ddp_amd.parallel import RcclCommunicator, TorchCommunicator
    from ddp_amd.parallel.commbench import allreduce_sweep, default_sizes
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus is not None and a.gpus != world:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    if a.device == "cuda":
        torch.cuda.set_device(local)
        comm, dev = RcclCommunicator(rank, world, local), f"cuda:{local}"
    else:
        if world == 1:
            raise SystemExit("--device cpu needs >= 2 ranks (Gloo)")
        comm, dev = TorchCommunicator(), "cpu"
    dt = torch.float32 if a.dtype == "fp32" else torch.bfloat16
    sizes = default_sizes(lo=int(a.min_kb * 1024), hi=int(a.max_mb * (1 << 20)))
    rows = allreduce_sweep(comm, sizes, dt, dev, iters=a.iters)
    if rank == 0:
        for r in rows:
            print(json.dumps(dict(r, world=world, dtype=a.dtype, device=a.device)), flush=True)
        if a.write_table is not None:
            from ddp_amd.parallel.bucket_plan import TABLE_FILE, merge_rows
            merge_rows(a.write_table or TABLE_FILE, world, a.dtype, rows,
                       source="measured" if a.device == "cuda" else "measured-gloo-cpu")
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

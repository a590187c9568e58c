#!/usr/bin/env python3
"""All-reduce bus-bandwidth sweep on the native RCCL communicator (one process per GPU):

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        tools/comm_bench.py [--dtype fp32|bf16] [--iters 20] [--max-mb 128]

Rank 0 prints one JSON line per message size (parallel/commbench.py)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--max-mb", type=float, default=128.0)
    ap.add_argument("--write-table", nargs="?", const="", default=None,
                    help="merge the measured rows into the bucket-sizing table "
                         "(default parallel/comm_tuning.json) for this world size and dtype")
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    import ddp_amd  # noqa: F401
    from ddp_amd.parallel import RcclCommunicator
    from ddp_amd.parallel.commbench import allreduce_sweep, default_sizes
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = RcclCommunicator(rank, world, local)
    dt = torch.float32 if a.dtype == "fp32" else torch.bfloat16
    rows = allreduce_sweep(comm, default_sizes(hi=int(a.max_mb * (1 << 20))), dt, f"cuda:{local}",
                           iters=a.iters)
    if rank == 0:
        for r in rows:
            print(json.dumps(dict(r, world=world, dtype=a.dtype)), flush=True)
        if a.write_table is not None:
            from ddp_amd.parallel.bucket_plan import TABLE_FILE, merge_rows
            merge_rows(a.write_table or TABLE_FILE, world, a.dtype, rows)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

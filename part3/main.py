"""Part 3 — bucketed, backward-overlapped DDP (reference: part3/main.py).

Run one process per rank (per GPU on MI355X, per node/CPU process otherwise):

    python part3/main.py --num-nodes W --rank R [--master-ip IP] [--master-port P]

Same four flags and defaults as the reference; --rank falls back to $RANK, then to the
hostname digit (nodeK), then 0. Collectives run on RCCL over xGMI on GPUs, Gloo on CPUs.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ddp_amd.engine.apps import main  # noqa: E402

if __name__ == "__main__":
    main("part3")

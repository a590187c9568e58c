"""Per-stage backward times of the pipelined step on one GPU (engine/step.py profile_stage_times:
a step cut before EVERY fused stage, no collectives, device events between the segment graphs)
-> the ``stage_us`` input of parallel/cut_plan.py (tests/test_cut_plan.py STAGES).

    python tools/stage_times.py --batch 32 [--model vgg11] [--reps 8]
Prints one JSON line {"batch", "model", "stage_us": [...]}."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="vgg11")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--reps", type=int, default=8)
    a = ap.parse_args()
    import torch
    import ddp_amd
    from ddp_amd.data import SyntheticCIFAR10, SyntheticImageNet, DeviceLoader
    from ddp_amd.engine import CrossEntropyLoss
    from ddp_amd.engine.step import profile_stage_times
    from ddp_amd.models import build
    from ddp_amd.optim import FusedSGD
    from ddp_amd.parallel import DistributedDataParallel, RcclCommunicator
    torch.manual_seed(ddp_amd.SEED)
    dev = torch.device("cuda", 0)
    ds = SyntheticImageNet(True) if a.model.startswith("resnet") else SyntheticCIFAR10(True)
    loader = DeviceLoader(ds, a.batch, dev, 1, 0, train=True, cpad=8)
    model = DistributedDataParallel(build(a.model).to(dev), RcclCommunicator(0, 1, 0),
                                    bucket_cap_mb=256.0, first_bucket_cap_mb=256.0, captured=True)
    opt = FusedSGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    n = model.module.n_stages()
    runs = [profile_stage_times(model, opt, CrossEntropyLoss(), loader, n, reps=a.reps)
            for _ in range(3)]
    stage = [sorted(col)[1] for col in zip(*runs)]
    print(json.dumps({"model": a.model, "batch": a.batch,
                      "stage_us": [round(v, 1) for v in stage]}))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""In-process A/B of a native kernel switch on the captured VGG-11 training step (one MI355X).

    python tools/ab_toggle.py --setter conv_wgrad_pm_set --values 1,0 --batches 256,128,64,32
    python tools/ab_toggle.py --const ddp_amd.ops.layers:FUSE_BN_IN_POOL_MAX_BATCH --values 32,64

For each batch: one model / optimizer / loader; for every trial and every value, the switch is
set (``native().<setter>(value)``), a fresh TrainStep is captured (the launch configuration is
baked into the graph at capture) and ``--reps`` replays are timed with device events. Values
alternate within each trial, so slow drift of the box affects them alike. Prints the median
ms per step of each value and one JSON line per batch.
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--setter", default=None, help="native setter, e.g. conv_rows_pm_set")
    ap.add_argument("--const", default=None,
                    help="module constant instead, e.g. ddp_amd.ops.layers:FUSE_BN_IN_POOL_MAX_BATCH")
    ap.add_argument("--values", default="1,0")
    ap.add_argument("--batches", default="256,32")
    ap.add_argument("--model", default="vgg11")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--trials", type=int, default=7)
    a = ap.parse_args()
    import torch
    import ddp_amd
    from ddp_amd.data import DeviceLoader, SyntheticCIFAR10, SyntheticImageNet
    from ddp_amd.engine import CrossEntropyLoss, TrainStep
    from ddp_amd.models import build
    from ddp_amd.optim import FusedSGD
    n = ddp_amd.native()
    if a.const:
        import importlib
        mod_name, attr = a.const.split(":")
        mod = importlib.import_module(mod_name)
        setter = lambda v: setattr(mod, attr, v)  # noqa: E731
        a.setter = a.const
    else:
        setter = getattr(n, a.setter)
    values = [int(v) for v in a.values.split(",")]
    dev = torch.device("cuda", 0)
    for B in [int(b) for b in a.batches.split(",")]:
        torch.manual_seed(ddp_amd.SEED)
        ds = SyntheticImageNet(True, n=4 * B) if a.model == "resnet50" else SyntheticCIFAR10(True)
        loader = DeviceLoader(ds, B, dev, 1, 0, train=True, cpad=8)
        model = build(a.model).to(dev)
        opt = FusedSGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
        crit = CrossEntropyLoss()
        res = {v: [] for v in values}
        for _ in range(a.trials):
            for v in values:
                setter(v)
                st = TrainStep(model, opt, crit, loader)
                st.warmup(2)
                st.capture()
                for _ in range(3):
                    st.step()
                torch.cuda.synchronize()
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    st.step()
                e1.record()
                torch.cuda.synchronize()
                res[v].append(e0.elapsed_time(e1) / a.reps)
                del st
            torch.cuda.empty_cache()
        setter(values[0])
        med = {v: sorted(t)[len(t) // 2] for v, t in res.items()}
        print(json.dumps({"batch": B, "setter": a.setter,
                          "median_ms": {str(v): round(m, 4) for v, m in med.items()},
                          "all_ms": {str(v): [round(x, 4) for x in t] for v, t in res.items()}}),
              flush=True)
        del model, opt, loader
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

"""Host launch time vs device time per training step (is the step host-bound?).

    python tools/host_time.py [--segmented 4] [--steps 200]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--segmented", type=int, default=0)
    ap.add_argument("--steps", type=int, default=200)
    a = ap.parse_args()
    import torch
    import ddp_amd  # noqa: F401
    from ddp_amd.data import SyntheticCIFAR10, DeviceLoader
    from ddp_amd.engine import TrainStep, SegmentedDDPStep, CrossEntropyLoss
    from ddp_amd.models import build
    from ddp_amd.optim import FusedSGD
    from ddp_amd.parallel import DistributedDataParallel, RcclCommunicator
    dev = torch.device("cuda", 0)
    loader = DeviceLoader(SyntheticCIFAR10(True), 256, dev, 1, 0, train=True, cpad=8)
    model = DistributedDataParallel(build("vgg11").to(dev), RcclCommunicator(0, 1, 0),
                                    bucket_cap_mb=256.0, first_bucket_cap_mb=256.0)
    opt = FusedSGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    crit = CrossEntropyLoss()
    st = (SegmentedDDPStep(model, opt, crit, loader, split=a.segmented) if a.segmented
          else TrainStep(model, opt, crit, loader))
    st.warmup(2)
    st.capture()
    for _ in range(20):
        st.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        st.step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    # host cost of one step while the device is idle (no queue back-pressure)
    host = []
    for _ in range(20):
        torch.cuda.synchronize()
        h0 = time.perf_counter()
        st.step()
        host.append(time.perf_counter() - h0)
    torch.cuda.synchronize()
    print(f"segmented={a.segmented} launch-loop {1e3 * (t1 - t0) / a.steps:.4f} ms/step, "
          f"device {1e3 * (t2 - t0) / a.steps:.4f} ms/step, idle-host step() "
          f"{1e3 * sorted(host)[len(host) // 2]:.4f} ms", flush=True)


if __name__ == "__main__":
    main()

"""Device-side timeline of the DDP bucket collectives vs the backward, from HIP timing events
(no profiler: rocprofv3's kernel trace puts every stream of this process on one hardware queue,
which serialises exactly the concurrency under test). Live single-rank RCCL communicator:

    DDP_AMD_RCCL_SELF=1 python tools/overlap_probe.py --mode eager|pipelined [--steps 6]

eager     = part3's eager DDP step: the native Reducer launches each full bucket's
            ncclAllReduce on its comm stream from the backward's gradient-ready hooks (4 MiB
            buckets + 1 MiB first). Timeline: each bucket's [start, end] on the comm stream vs
            the gradient announcements on the compute stream.
pipelined = the captured pipelined step (engine/step.py SegmentedDDPStep): each bucket's
            all-reduce + SGD on the comm stream vs the segment graphs on the main stream.
Prints a markdown table per mode and a final JSON summary line.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def overlap(a, b):
    return max(0.0, min(a[1], b[1]) - max(a[0], b[0]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="eager", choices=["eager", "pipelined"])
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--cuts", default="3,6")
    ap.add_argument("--standin-gbps", type=float, default=0.0,
                    help="no live communicator: a timed 32-CU stand-in collective instead")
    a = ap.parse_args()
    import torch
    import ddp_amd
    from ddp_amd.models import VGG11
    from ddp_amd.optim import FusedSGD
    from ddp_amd.data import SyntheticCIFAR10, DeviceLoader
    from ddp_amd.engine import TrainStep, SegmentedDDPStep, CrossEntropyLoss
    from ddp_amd.parallel import DistributedDataParallel, RcclCommunicator
    from ddp_amd.ops.common import register_grad_ready_hook, clear_grad_ready_hooks
    torch.manual_seed(ddp_amd.SEED)
    comm = RcclCommunicator(0, 1, 0, self_comm=a.standin_gbps <= 0)
    m = DistributedDataParallel(VGG11().cuda(), comm, bucket_cap_mb=4.0, first_bucket_cap_mb=1.0)
    opt = FusedSGD(m.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    ld = DeviceLoader(SyntheticCIFAR10(True, n=4096), a.batch, "cuda", cpad=8)
    crit = CrossEntropyLoss()
    T = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    summary = {"mode": a.mode, "batch": a.batch, "live_rccl": bool(comm.live),
               "GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES"),
               "comm_priority": "high"}
    if a.mode == "eager":
        st = TrainStep(m, opt, crit, ld, use_graph=False)
        st.step()
        torch.cuda.synchronize()
        m.reducer.set_timing(True)
        ann = []

        def hook(p, stream):
            ev = T()
            ev.record(stream)
            ann.append(ev)
        h = register_grad_ready_hook(hook)
        rows = []
        for _ in range(a.steps):
            ann.clear()
            ref = T()
            ref.record()
            st.step()
            torch.cuda.synchronize()
            ta = [ref.elapsed_time(e) for e in ann]
            bw = (min(ta), max(ta))  # first .. last gradient announced on the compute stream
            rows = [(b, s, e, overlap((s, e), bw) / max(e - s, 1e-9))
                    for b, (s, e) in enumerate(m.reducer.bucket_times(ref.cuda_event))]
        clear_grad_ready_hooks(h)
        print(f"backward (first .. last gradient announced): {bw[0]:.3f} .. {bw[1]:.3f} ms; "
              f"comm stream overlap {m.reducer.overlap()}; launch log {m.reducer.launch_log()}")
        print("| bucket | start ms | end ms | fraction of the collective inside the backward |")
        print("|---|---|---|---|")
        for b, s, e, f in rows:
            print(f"| {b} | {s:.3f} | {e:.3f} | {f:.2f} |")
        summary.update(backward_ms=[round(bw[0], 4), round(bw[1], 4)],
                       buckets=[[b, round(s, 4), round(e, 4), round(f, 3)] for b, s, e, f in rows],
                       done_before_backward_end=sum(1 for _, _, e, _ in rows if e < bw[1]))
    else:
        st = SegmentedDDPStep(m, opt, crit, ld, split=[int(v) for v in a.cuts.split(",")],
                              emulate_gbps=a.standin_gbps)
        st.warmup(2)
        st.capture()
        main = torch.cuda.current_stream()
        for _ in range(a.steps):
            st.probe = []
            segs = []
            ref = T()
            ref.record()
            for j, g in enumerate(st.graphs):
                s0 = T()
                s0.record(main)
                g.replay()
                s1 = T()
                s1.record(main)
                segs.append((s0, s1))
                st._comm(j)
            torch.cuda.synchronize()
            seg_t = [(ref.elapsed_time(x), ref.elapsed_time(y)) for x, y in segs]
            com_t = [(j, ref.elapsed_time(x), ref.elapsed_time(y)) for j, x, y in st.probe]
        st.probe = None
        print("| bucket | comm start ms | comm end ms | overlap with later segments ms |")
        print("|---|---|---|---|")
        hid = tot = 0.0
        for j, s, e in com_t:
            ov = sum(overlap((s, e), seg_t[k]) for k in range(j + 1, len(seg_t)))
            hid += ov
            tot += e - s
            print(f"| {j} | {s:.3f} | {e:.3f} | {ov:.3f} |")
        print("segments (main stream):", [(round(x, 3), round(y, 3)) for x, y in seg_t])
        summary.update(segments=[[round(x, 4), round(y, 4)] for x, y in seg_t],
                       comm=[[j, round(s, 4), round(e, 4)] for j, s, e in com_t],
                       comm_ms=round(tot, 4), comm_hidden_ms=round(hid, 4),
                       step_ms=round(max(max(y for _, y in seg_t), max(e for _, _, e in com_t)), 4))
    print(json.dumps(summary))


if __name__ == "__main__":
    main()

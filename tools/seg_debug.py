"""Compare one SegmentedDDPStep update against TrainStep from the same snapshot (one GPU)."""
import copy, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import ddp_amd
from ddp_amd.models import VGG11
from ddp_amd.engine import CrossEntropyLoss, TrainStep, SegmentedDDPStep
from ddp_amd.optim import FusedSGD
from ddp_amd.data import SyntheticCIFAR10, DeviceLoader
from ddp_amd.parallel import DistributedDataParallel, RcclCommunicator

torch.manual_seed(4)
m = DistributedDataParallel(VGG11().cuda(), RcclCommunicator(0, 1, 0), bucket_cap_mb=256.0,
                            first_bucket_cap_mb=256.0)
opt = FusedSGD(m.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
ld = DeviceLoader(SyntheticCIFAR10(True, n=512), 64, "cuda")
crit = CrossEntropyLoss()
ts = TrainStep(m, opt, crit, ld)
ss = SegmentedDDPStep(m, opt, crit, ld, split=int(os.environ.get("SPLIT", "4")), emulate=0)
ts.warmup(2)
torch.cuda.synchronize()
snap = (m.arena.data.clone(), opt.momentum_buffer.clone(), ld.cursor.clone())

def restore():
    m.arena.data.copy_(snap[0]); opt.momentum_buffer.copy_(snap[1]); ld.cursor.copy_(snap[2])
    m.arena.grad.zero_()
    for sp in m.module.fused_plan():
        sp._packed_version = None
        sp.maybe_pack()
    torch.cuda.synchronize()

def run(fn):
    restore()
    fn()
    torch.cuda.synchronize()
    return m.arena.data - snap[0]

def cos(a, b):
    return float(torch.dot(a, b) / (a.norm() * b.norm() + 1e-30))

d_t1 = run(ts._body)
d_t2 = run(ts._body)
d_s = run(ss._body)
print("train vs train", cos(d_t1, d_t2), "train vs seg", cos(d_t1, d_s),
      "norm ratio", float(d_s.norm() / d_t1.norm()))
a = m.arena
for i, p in enumerate(a.params):
    o, n = a.offsets[i], a.numels[i]
    c = cos(d_t1[o:o + n], d_s[o:o + n]); c0 = cos(d_t1[o:o + n], d_t2[o:o + n])
    print(i, tuple(p.shape), f"base {c0:.4f} seg {c:.4f}")
ss.warmup(1)
ss.capture()
d_g = run(ss.step)
print("train vs seg-graph", cos(d_t1, d_g), "cursor", int(ld.cursor.item()), int(snap[2].item()))

"""Per-parameter comparison: DDP step with live single-rank RCCL vs without (same state)."""
import copy, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import ddp_amd
from ddp_amd.models import VGG11
from ddp_amd.optim import FusedSGD
from ddp_amd.data import SyntheticCIFAR10, DeviceLoader
from ddp_amd.engine import TrainStep, SegmentedDDPStep, CrossEntropyLoss
from ddp_amd.parallel import DistributedDataParallel, RcclCommunicator

torch.manual_seed(7)
base = VGG11().cuda()

def run(live, graph, seg):
    m = DistributedDataParallel(copy.deepcopy(base), RcclCommunicator(0, 1, 0, self_comm=live),
                                bucket_cap_mb=256.0, first_bucket_cap_mb=256.0)
    opt = FusedSGD(m.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    ld = DeviceLoader(SyntheticCIFAR10(True, n=512), 64, "cuda")
    cls = SegmentedDDPStep if seg else TrainStep
    st = cls(m, opt, CrossEntropyLoss(), ld, **({"split": 4} if seg else {}))
    before = m.arena.data.clone()
    if graph:
        st.capture()
        st.step()
    else:
        st._body()
    torch.cuda.synchronize()
    d = (m.arena.data - before).clone()
    offs = list(m.arena.offsets) + [m.arena.total]
    m.close()
    return d, offs

for seg in (False, True):
    for graph in (False, True):
        a, offs = run(False, graph, seg)
        a2, _ = run(False, graph, seg)
        b, _ = run(True, graph, seg)
        cos = lambda x, y: float(torch.dot(x, y) / (x.norm() * y.norm() + 1e-30))
        print(f"seg={seg} graph={graph}: base cos {cos(a, a2):.5f} live cos {cos(a, b):.5f} "
              f"norm ratio {float(b.norm() / a.norm()):.4f}", flush=True)
        worst = sorted(((cos(a[offs[i]:offs[i+1]], b[offs[i]:offs[i+1]]), i) for i in range(len(offs) - 1)))[:4]
        print("   worst params (cos, idx):", [(round(c, 4), i) for c, i in worst], flush=True)

"""Does a captured hipMemsetAsync node order before the kernel that reads its buffer?

The strided dgrad (csrc/kernels/conv_igemm.hip, zero_fill) zeroes dx with a kernel because a
round-3 ResNet-50 study saw sporadic NaN gradients in REPLAYED steps when it was a
hipMemsetAsync. This probe isolates the claim: a graph of

    kernel: fill X with 0x7f bytes  ->  hipMemsetAsync(X, 0)  ->  kernel: copy X -> Y

(and the same with the zero fill as a kernel instead of the memset node) is replayed many times;
every replay must leave Y all zero. Sizes cover the ResNet-50 b256 strided dx (411 MB).
Prints one JSON line: bad replays per (variant, size)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def run(kind, nbytes, reps, pre_bytes=0):
    import torch
    import ddp_amd
    n = ddp_amd.native()
    x = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    y = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    pre = torch.empty(max(pre_bytes, 16), dtype=torch.uint8, device="cuda")
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            st = torch.cuda.current_stream().cuda_stream
            if pre_bytes:  # an unrelated big kernel before: the memset may race ahead of X's writer
                n.fill_bytes(pre.data_ptr(), 1, pre_bytes, st)
            n.fill_bytes(x.data_ptr(), 0x7F, nbytes, st)
            if kind == "memset":
                n.memset_async(x.data_ptr(), 0, nbytes, st)
            else:
                n.fill_bytes(x.data_ptr(), 0, nbytes, st)
            n.copy_bytes(y.data_ptr(), x.data_ptr(), nbytes, st)
    torch.cuda.synchronize()
    bad = 0
    for _ in range(reps):
        y.fill_(0xAA)
        g.replay()
        torch.cuda.synchronize()
        if int(torch.count_nonzero(y)) != 0:
            bad += 1
    del g
    return bad


def main():
    out = {}
    for nbytes, reps in ((4 << 20, 300), (128 << 20, 100), (411041792, 40)):
        for kind in ("kernel", "memset"):
            for pre in (0, 256 << 20):
                out[f"{kind}/{nbytes}/pre{pre}"] = run(kind, nbytes, reps, pre)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

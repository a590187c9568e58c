#!/usr/bin/env python3
"""Link a variant of the native extension for same-session A/B runs on the GPU box:

    python tools/link_variant.py NAME kernel_obj.o [more.o ...]

replaces the same-named objects of build/native/ (e.g. a conv_igemm.hip.o compiled with other
flags, saved as /tmp/conv_x.o -> pass it as conv_igemm.hip.o=/tmp/conv_x.o) and writes
ab_so/_native_NAME.so. Load it with DDP_AMD_NATIVE_PATH=ab_so/_native_NAME.so.
"""
import glob
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    name, repl = sys.argv[1], dict(a.split("=", 1) for a in sys.argv[2:])
    objs = []
    for o in sorted(glob.glob(os.path.join(REPO, "build", "native", "*.o"))):
        objs.append(repl.pop(os.path.basename(o), o))
    if repl:
        raise SystemExit(f"no such objects in build/native: {list(repl)}")
    os.makedirs(os.path.join(REPO, "ab_so"), exist_ok=True)
    out = os.path.join(REPO, "ab_so", f"_native_{name}.so")
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", out,
           "-L/opt/rocm/lib", "-lrccl", "-lamdhip64"]
    subprocess.run(cmd, check=True)
    print(out)


if __name__ == "__main__":
    main()

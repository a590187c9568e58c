"""Build the in-tree native extension ``_native`` for gfx950 with hipcc (no JIT cache).

    python -m ddp_amd._build            # or: python distributed-data-parallel-ml-training_amd/_build.py

* every ``csrc/kernels/*.hip`` is compiled for ``--offload-arch=gfx950`` (device code),
* ``csrc/runtime/*.cpp`` (RCCL communicator + bucketed reducer) and ``csrc/bind.cpp`` (pybind11)
  are host C++ compiled by the same hipcc,
* the result is linked against HIP and RCCL into ``_native<EXT_SUFFIX>`` next to this file so it
  travels with the repository snapshot to the GPU box. At run time torch's bundled
  ``libamdhip64.so.7`` / ``librccl.so.1`` satisfy the DT_NEEDED entries (torch is imported first),
  so the process has exactly one HIP runtime.
Objects are cached in ``build/native`` and rebuilt when a source or any header changes.
"""
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_DIR)
CSRC = os.path.join(PKG_DIR, "csrc")
ARCH = os.environ.get("DDP_AMD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _hipcc():
    for c in (os.path.join(ROCM, "bin", "hipcc"), shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build ddp_amd)")


def _includes():
    import pybind11
    return ["-I" + CSRC, "-I" + os.path.join(CSRC, "kernels"), "-I" + pybind11.get_include(),
            "-I" + sysconfig.get_paths()["include"], "-I" + os.path.join(ROCM, "include")]


# build variants: name -> (module file stem, object dir, extra defines). "det" is the
# deterministic-statistics test build (csrc/kernels/api.h kStatRep; loaded by _ext.load() when
# DDP_AMD_DETERMINISTIC=1).
VARIANTS = {"release": ("_native", "native", []),
            "det": ("_native_det", "native_det", ["-DDDP_AMD_DETERMINISTIC"])}


def ext_path(variant="release"):
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(PKG_DIR, VARIANTS[variant][0] + suffix)


def _newest_header():
    hs = glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def _deps(obj):
    """Headers the object was built from (the compiler's -MMD file), or None if unknown."""
    d = obj + ".d"
    if not os.path.exists(d):
        return None
    with open(d) as f:
        text = f.read().replace("\\\n", " ")
    parts = text.split(":", 1)
    return [t for t in parts[1].split()] if len(parts) == 2 else None


def _compile(cmd, src, obj, hdr_time, verbose):
    if os.path.exists(obj):
        t = os.path.getmtime(obj)
        deps = _deps(obj)
        # a source is rebuilt when it or a header IT includes changed (all headers when the
        # dependency file is missing)
        newest = (max([os.path.getmtime(x) for x in deps if os.path.exists(x)] + [0.0])
                  if deps is not None else hdr_time)
        if deps is not None and any(not os.path.exists(x) for x in deps):
            newest = hdr_time
        if t >= os.path.getmtime(src) and t >= newest:
            return obj, False
    if verbose:
        print("[ddp_amd build]", os.path.relpath(src, PKG_DIR), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{r.stdout}\n{r.stderr}")
    return obj, True


def _sources():
    return (sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
            + sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp"))) + [os.path.join(CSRC, "bind.cpp")])


def up_to_date(variant="release"):
    """The in-tree extension is newer than every source and header. The object cache
    (build/native) does not travel with a snapshot, so this is what a GPU box checks: an
    up-to-date extension is loaded as is instead of being rebuilt there."""
    out = ext_path(variant)
    if not os.path.exists(out):
        return False
    newest = max([_newest_header()] + [os.path.getmtime(s) for s in _sources()])
    return os.path.getmtime(out) >= newest


def build(verbose=True, jobs=None, variants=("release", "det")):
    """Build every variant (release = the shipped extension, det = the deterministic-
    statistics test build); returns the release path."""
    for v in variants:
        _build_variant(v, verbose, jobs)
    return ext_path()


def _build_variant(variant, verbose=True, jobs=None):
    stem, objdir, defines = VARIANTS[variant]
    BUILD = os.path.join(REPO, "build", objdir)
    if not os.path.isdir(BUILD) and up_to_date(variant):
        return ext_path(variant)
    hipcc = _hipcc()
    os.makedirs(BUILD, exist_ok=True)
    inc = _includes()
    # DDP_AMD_DEBUG_BUILD=1: -O1 -g and the DDP_DEVICE_CHECK bounds checks (common.h)
    debug = os.environ.get("DDP_AMD_DEBUG_BUILD", "0") == "1"
    common = (["-O1", "-g", "-DDDP_AMD_DEBUG"] if debug else ["-O3"]) + \
        ["-std=c++17", "-fPIC", "-Wno-unused-result"] + defines
    hdr_time = _newest_header()
    tasks = []
    for src in sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip"))):
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        cmd = [hipcc, f"--offload-arch={ARCH}", "-x", "hip", *common, *inc, "-c", src, "-o", obj,
               "-MMD", "-MF", obj + ".d"]
        tasks.append((cmd, src, obj))
    host_srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp"))) + [os.path.join(CSRC, "bind.cpp")]
    for src in host_srcs:
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        cmd = [hipcc, "-x", "c++", "-D__HIP_PLATFORM_AMD__", *common, "-fvisibility=hidden", *inc,
               "-c", src, "-o", obj, "-MMD", "-MF", obj + ".d"]
        tasks.append((cmd, src, obj))
    jobs = jobs or min(8, os.cpu_count() or 4)
    changed = False
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = [ex.submit(_compile, c, s, o, hdr_time, verbose) for c, s, o in tasks]
        objs = []
        for f in futs:
            o, ch = f.result()
            objs.append(o)
            changed |= ch
    out = ext_path(variant)
    if changed or not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(o) for o in objs):
        tmp = out + ".tmp"
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", tmp,
               "-L" + os.path.join(ROCM, "lib"), "-lrccl", "-lamdhip64"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, out)
        if verbose:
            print("[ddp_amd build] linked", os.path.relpath(out, REPO), flush=True)
    return out


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)

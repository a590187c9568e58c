"""Loader for the in-tree native extension ``_native`` (HIP kernels + RCCL runtime).

The extension is built by ``_build.py`` (``python -m ddp_amd._build`` or
``__graft_entry__.build()``) into this package directory so that it travels with the repo
snapshot to the GPU box. There is deliberately NO silent fallback: GPU code paths call
``load()`` and fail loudly when the extension is missing or stale.
"""
import importlib.machinery
import importlib.util
import os
import sys

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
_MODNAME = "_native"
_module = None


def so_path():
    """The release build, or the deterministic-statistics test build with
    DDP_AMD_DETERMINISTIC=1 (_build.py variant "det")."""
    suffix = importlib.machinery.EXTENSION_SUFFIXES[0]
    name = _MODNAME + ("_det" if os.environ.get("DDP_AMD_DETERMINISTIC", "0") == "1" else "")
    return os.path.join(_PKG_DIR, name + suffix)


def available():
    return os.path.exists(so_path())


def load():
    """Import the extension. torch must be imported first so that the process has exactly one
    HIP runtime (torch's bundled libamdhip64.so.7 satisfies our DT_NEEDED by SONAME)."""
    global _module
    if _module is not None:
        return _module
    import torch  # noqa: F401  (load torch's HIP runtime first)
    # DDP_AMD_NATIVE_PATH: load another build of the same extension (A/B of kernel variants in
    # one GPU session, tools/gpu/ab_build.sh); the in-tree build is the default
    path = os.environ.get("DDP_AMD_NATIVE_PATH") or so_path()
    if not os.path.exists(path):
        raise RuntimeError(
            f"ddp_amd native extension not built ({path} missing). "
            "Run `python -c 'import __graft_entry__ as g; g.build()'` first.")
    spec = importlib.util.spec_from_file_location("ddp_amd._native", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    sys.modules["ddp_amd._native"] = mod
    _module = mod
    return mod

"""Import shim: exposes the package directory ``distributed-data-parallel-ml-training_amd/``
(not a valid Python identifier) under the import name ``ddp_amd``.

``import ddp_amd`` executes the package's ``__init__.py`` with ``__path__`` pointing at the
hyphenated directory, then replaces this shim in ``sys.modules`` so that
``import ddp_amd.ops.conv`` etc. resolve inside the real package.
"""
import importlib.util
import os
import sys

_PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                        "distributed-data-parallel-ml-training_amd")

_spec = importlib.util.spec_from_file_location(
    __name__, os.path.join(_PKG_DIR, "__init__.py"), submodule_search_locations=[_PKG_DIR])
_mod = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)

"""Reference-compatible model module (part1/model.py of the reference, 4 identical copies).

Exports the same names (`_cfg`, `_make_layers`, `_VGG`, `VGG11`) with the same module tree
and state_dict keys; the implementation lives in ddp_amd.models.vgg (fused gfx950 path on GPU,
ATen on CPU).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ddp_amd.models.vgg import _cfg, _make_layers, _VGG, VGG11, VGG13, VGG16, VGG19  # noqa: E402,F401

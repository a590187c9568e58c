#!/bin/bash
# round 5: the b256 trajectory test with / without the pair-master SGD (r5y follow-up)
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r5y2; mkdir -p $O
for m in 1 0 1 0; do
  DDP_AMD_SGD_PAIR_MASTER=$m timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -k "b256_trajectory" -q --timeout 240 --timeout-method thread > $O/t_$m.log 2>&1; echo "master=$m rc=$? $(tail -1 $O/t_$m.log)"; grep -E "^emu|^fp32|^gpu|cosine" $O/t_$m.log | head -4
done
python - <<'PY'
import sys; sys.path.insert(0, ".")
import torch, ddp_amd
from ddp_amd.ops.common import native
print("ok")
PY

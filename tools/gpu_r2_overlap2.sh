#!/bin/bash
# pipelined step: does the comm stream overlap the segment graphs? (HW queue assignment)
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/ovl2
p() { local tag=$1; shift; env "$@" timeout -k 10 120 python tools/overlap_probe.py --mode pipelined --batch 256 ${EXTRA:-} > gpurun_out/ovl2/$tag.md 2>&1 || { tail -20 gpurun_out/ovl2/$tag.md; exit 1; }; echo "$tag $(tail -1 gpurun_out/ovl2/$tag.md | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["comm_ms"], d["comm_hidden_ms"], d["step_ms"])')"; }
p live_default DDP_AMD_RCCL_SELF=1
p live_prio DDP_AMD_RCCL_SELF=1 DDP_AMD_COMM_PRIORITY=high
p live_q8 DDP_AMD_RCCL_SELF=1 GPU_MAX_HW_QUEUES=8
EXTRA="--standin-gbps 171" p standin_default X=1
EXTRA="--standin-gbps 171" p standin_prio DDP_AMD_COMM_PRIORITY=high

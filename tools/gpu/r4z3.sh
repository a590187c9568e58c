#!/bin/bash
# round 4: fused-sums pair path fixed -> validate, then re-measure DDP_AMD_BN_BWD_FUSE_MAX_HW
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r4z3; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -v --timeout 120 --timeout-method thread -k "fused_sums" > $O/t_fused_sums.log 2>&1 || { tail -30 $O/t_fused_sums.log; exit 1; }
grep -E "PASS|FAIL" $O/t_fused_sums.log
timeout -k 10 300 python -u tools/probes/grad_determinism.py --batch 256 --hw 16,16,64,256 > $O/grad_b256.txt 2>&1 || { tail -20 $O/grad_b256.txt; exit 1; }
grep "whole" $O/grad_b256.txt
for B in 256 128 64 32; do for hw in 16 64 256 16 64 256; do
  timeout -k 10 200 env DDP_AMD_BN_BWD_FUSE_MAX_HW=$hw python bench.py --global-batch $B --steps 60 --warmup 10 --ref-window 0 > $O/b${B}_hw${hw}.log 2>&1 || { tail -5 $O/b${B}_hw${hw}.log; exit 1; }
  echo "b$B hw$hw $(tail -1 $O/b${B}_hw${hw}.log | grep -oE '"ms_per_step": [0-9.]+')"
done; done

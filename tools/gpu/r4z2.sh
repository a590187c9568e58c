#!/bin/bash
# round 4: validate the BN-backward sums fusion on 8x8 / 16x16 dgrad outputs (MAX_HW 64 / 256)
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r4z2; mkdir -p $O
timeout -k 10 300 python -u tools/probes/grad_determinism.py --batch 256 --hw 16,16,64,256 > $O/grad_b256.txt 2>&1 || { tail -20 $O/grad_b256.txt; exit 1; }
timeout -k 10 300 python -u tools/probes/grad_determinism.py --batch 32 --hw 16,16,64,256 > $O/grad_b32.txt 2>&1 || { tail -20 $O/grad_b32.txt; exit 1; }
grep "whole" $O/grad_b256.txt $O/grad_b32.txt
timeout -k 10 900 env DDP_AMD_BN_BWD_FUSE_MAX_HW=256 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_hw256.log 2>&1 || { grep -E "FAIL|Error" $O/gpu_tests_hw256.log | head -20; tail -30 $O/gpu_tests_hw256.log; exit 1; }
tail -1 $O/gpu_tests_hw256.log
for B in 256 128 64; do for hw in 64 256 64 256; do
  timeout -k 10 200 env DDP_AMD_BN_BWD_FUSE_MAX_HW=$hw python bench.py --global-batch $B --steps 60 --warmup 10 --ref-window 0 > $O/b${B}_hw${hw}.log 2>&1 || { tail -5 $O/b${B}_hw${hw}.log; exit 1; }
  echo "b$B hw$hw $(tail -1 $O/b${B}_hw${hw}.log | grep -oE '"ms_per_step": [0-9.]+')"
done; done

cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/tr || exit 1
for P in 1 2; do
for B in 256 128 64 32; do for V in "0:x" "1:x" "2:x" "1:4096" "1:8192"; do
  T=${V%%:*}; R=${V##*:}; [ "$R" = x ] && R=1073741824
  DDP_AMD_FUSE_BN_IN=$T DDP_AMD_FUSE_BN_IN_MAX_ROWS=$R timeout -k 10 200 python bench.py --global-batch $B --steps 60 --warmup 10 --ref-window 0 > gpurun_out/tr/b.log 2>&1 || { tail -5 gpurun_out/tr/b.log; exit 1; }
  echo "p$P B=$B FUSE=$V $(python -c "import json; d=json.loads(open('gpurun_out/tr/b.log').read().strip().splitlines()[-1]); print(d['ms_per_step'])")"
done; done; done

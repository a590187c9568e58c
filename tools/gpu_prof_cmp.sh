cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/prof_cmp
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/prof_cmp -o base -- python bench.py --steps 20 --warmup 5 > gpurun_out/prof_cmp_base.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/prof_cmp -o seg -- python bench.py --steps 20 --warmup 5 --segmented 4 > gpurun_out/prof_cmp_seg.log 2>&1 || exit 1
echo ok

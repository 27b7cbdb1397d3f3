set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02g_b64prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02g_b64prof -o b64 -- python bench.py --workload batch64 --steps 2 --warmup 1 --pipeline 0 --no-cpu-baseline > gpurun_out/r02g_b64prof.log 2>&1
find gpurun_out/r02g_b64prof -name "*kernel_stats.csv" | head -3

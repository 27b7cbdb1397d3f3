set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-pb}
rm -rf gpurun_out/${TAG}_db
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_db -o pb -- python3 bench.py --workload batch64 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}.log 2>&1 || { tail gpurun_out/${TAG}.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/${TAG}_db > gpurun_out/${TAG}_stats.txt 2>&1
head -45 gpurun_out/${TAG}_stats.txt

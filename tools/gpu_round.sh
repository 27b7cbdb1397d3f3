#!/bin/bash
# One GPU-box pass: gpu parity tests, smoke, bench, rocprof kernel stats.
# Usage (from the repo root, via gpurun): bash tools/gpu_round.sh TAG [tests|bench|prof ...]
set -o pipefail
TAG=${1:-run}; shift
STEPS=${@:-tests smoke bench prof}
mkdir -p gpurun_out
export TMPDIR=/tmp
for s in $STEPS; do
  case $s in
    tests) timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
           tail -3 gpurun_out/${TAG}_tests.log ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -30 gpurun_out/${TAG}_smoke.log; exit 1; }
           tail -2 gpurun_out/${TAG}_smoke.log ;;
    bench) timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
           cat gpurun_out/${TAG}_bench.json ;;
    prof)  rm -rf gpurun_out/prof_${TAG}
           timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o bench -- python3 bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench_under_rocprof.log 2>&1 || { tail -30 gpurun_out/${TAG}_bench_under_rocprof.log; exit 1; }
           python tools/prof_summary.py gpurun_out/prof_${TAG} > gpurun_out/${TAG}_kernel_stats.txt 2>&1; head -25 gpurun_out/${TAG}_kernel_stats.txt ;;
  esac
done

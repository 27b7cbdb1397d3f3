set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r02b_tests.log 2>&1 || { tail -40 gpurun_out/r02b_tests.log; exit 1; }
tail -3 gpurun_out/r02b_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r02b_bench.json 2> gpurun_out/r02b_bench.err || { tail -30 gpurun_out/r02b_bench.err; exit 1; }
cat gpurun_out/r02b_bench.json
timeout -k 10 300 python bench.py --workload batch64 --steps 2 --warmup 1 > gpurun_out/r02b_b64.json 2> gpurun_out/r02b_b64.err || { tail -30 gpurun_out/r02b_b64.err; exit 1; }
cat gpurun_out/r02b_b64.json

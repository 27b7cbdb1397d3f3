set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_golden_gpu.py tests/test_t2s_gpu.py tests/test_api_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r02r_tests.log 2>&1 || { tail -40 gpurun_out/r02r_tests.log; exit 1; }
tail -2 gpurun_out/r02r_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r02r_bench.json 2> gpurun_out/r02r_bench.err || { tail -20 gpurun_out/r02r_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r02r_bench.json')); print(d['value'], d['phase_ms'])"

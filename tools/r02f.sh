set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r02f}
timeout -k 10 400 python -u -m pytest tests/test_batch64_gpu.py tests/test_t2s_gpu.py tests/test_api_gpu.py tests/test_persist_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python bench.py --workload batch64 --steps 2 --warmup 1 > gpurun_out/${TAG}_b64.json 2> gpurun_out/${TAG}_b64.err || { tail -30 gpurun_out/${TAG}_b64.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_b64.json'));print('utt/s',d['value'],d['ms_per_step'],d['phase_ms'])"

# decode-kernel iteration: parity tests of the persistent/golden paths, phase trace, bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r02c}
timeout -k 10 300 python -u -m pytest tests/test_persist_gpu.py tests/test_golden_gpu.py tests/test_t2s_gpu.py tests/test_api_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 120 python tools/ptrace2.py > gpurun_out/${TAG}_ptrace.txt 2>&1 || { tail -20 gpurun_out/${TAG}_ptrace.txt; exit 1; }
cat gpurun_out/${TAG}_ptrace.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print('utt/s',d['value'],'x_rt',d['x_realtime'],d['phase_ms'])"

set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r02i}
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python bench.py --workload batch64 --steps 2 --warmup 1 > gpurun_out/${TAG}_b64.json 2> gpurun_out/${TAG}_b64.err || { tail -30 gpurun_out/${TAG}_b64.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_b64.json'));print('b64 utt/s',d['value'],d['ms_per_step'],d['phase_ms'])"
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print('single utt/s',d['value'],d['x_realtime'],d['phase_ms'])"

set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_vits_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02t_tests.log 2>&1 || { tail -40 gpurun_out/r02t_tests.log; exit 1; }
tail -1 gpurun_out/r02t_tests.log
GENIE_MRF_CONCURRENT=1 timeout -k 10 400 python -u -m pytest tests/test_vits_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02t_tests2.log 2>&1 || { tail -40 gpurun_out/r02t_tests2.log; exit 1; }
tail -1 gpurun_out/r02t_tests2.log
for v in 0 1 0 1; do
GENIE_MRF_CONCURRENT=$v timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r02t_bench$v.json 2> gpurun_out/r02t_bench.err || { tail -20 gpurun_out/r02t_bench.err; exit 1; }
python -c "import json,sys; d=json.load(open('gpurun_out/r02t_bench$v.json')); print('conc=$v', round(d['value'],2), {k: round(x,3) for k,x in d['phase_ms'].items()})"
done

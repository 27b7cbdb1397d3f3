set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_vits_gpu.py tests/test_golden_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02s_tests.log 2>&1 || { tail -40 gpurun_out/r02s_tests.log; exit 1; }
tail -2 gpurun_out/r02s_tests.log
rm -rf gpurun_out/prof_r02s
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02s -o bench -- python3 bench.py --no-cpu-baseline > gpurun_out/r02s_bench.json 2> gpurun_out/r02s_bench.err || { tail -20 gpurun_out/r02s_bench.err; exit 1; }
python tools/utt_timeline.py gpurun_out/prof_r02s/bench_results.db 30 > gpurun_out/r02s_timeline.txt; head -50 gpurun_out/r02s_timeline.txt

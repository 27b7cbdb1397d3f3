set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_roberta_gpu.py tests/test_hubert_gpu.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r02q_tests.log 2>&1 || { tail -40 gpurun_out/r02q_tests.log; exit 1; }
grep -E "rms|passed|failed" gpurun_out/r02q_tests.log | tail -8

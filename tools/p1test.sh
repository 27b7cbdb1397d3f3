set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_persist_gpu.py > gpurun_out/p1_tests.log 2>&1; r=$?
tail -25 gpurun_out/p1_tests.log
[ $r -eq 0 ] || exit $r
timeout -k 10 120 python tools/ptrace1.py > gpurun_out/p1_ptrace.txt 2>&1 && cat gpurun_out/p1_ptrace.txt

set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_persist_gpu.py tests/test_golden_gpu.py tests/test_t2s_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r02m_tests.log 2>&1 || { tail -40 gpurun_out/r02m_tests.log; exit 1; }
tail -3 gpurun_out/r02m_tests.log
timeout -k 10 300 python -u tools/knob_sweep.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r02m_knobs.txt

set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_golden_gpu.py -k "bench_size" -x -v --timeout 120 --timeout-method thread > gpurun_out/r02l_tests.log 2>&1 || { tail -30 gpurun_out/r02l_tests.log; exit 1; }
tail -3 gpurun_out/r02l_tests.log
timeout -k 10 300 python -u tools/knob_sweep.py "k1=1,k0=1" "k1=1,k0=4" "k1=1,k0=0" 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r02l_knobs.txt

set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_overlap_gpu.py > gpurun_out/r02g_t5.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/r02g_bench2.json 2> gpurun_out/r02g_bench2.err

set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_vits_gpu.py tests/test_api_gpu.py tests/test_tutorial_gpu.py tests/test_overlap_gpu.py > gpurun_out/r02g_t6.log 2>&1
timeout -k 10 200 python bench.py --vocoder-cus 0 --steps 20 --no-cpu-baseline --concurrent-streams 0 > gpurun_out/r02g_seq2.json 2>> gpurun_out/r02g_b64.err
timeout -k 10 200 python bench.py --workload batch64 --steps 20 --no-cpu-baseline > gpurun_out/r02g_b64d.json 2>> gpurun_out/r02g_b64.err

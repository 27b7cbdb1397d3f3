set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_batch64_gpu.py tests/test_t2s_gpu.py > gpurun_out/r02g_t3.log 2>&1
for a in "1" "0"; do
timeout -k 10 200 python bench.py --workload batch64 --steps 8 --warmup 2 --pipeline $a --no-cpu-baseline > gpurun_out/o.json 2>> gpurun_out/r02g_b64.err
echo "pipe $a $(cat gpurun_out/o.json)" >> gpurun_out/r02g_attn.txt
done

set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_vits_gpu.py -k "async" > gpurun_out/r02g_t2.log 2>&1
for a in "0 4" "64 4" "96 4" "128 4" "64 2"; do set -- $a
timeout -k 10 200 python bench.py --workload batch64 --steps 8 --warmup 2 --batch-vocoder-cus $1 --vits-lanes $2 --no-cpu-baseline > gpurun_out/o.json 2>> gpurun_out/r02g_b64.err
echo "vcus $1 lanes $2 $(cat gpurun_out/o.json)" >> gpurun_out/r02g_cus.txt
done

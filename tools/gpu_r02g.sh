set -e
mkdir -p gpurun_out
python -c "import torch; import ctypes; h=ctypes.CDLL('libamdhip64.so'); a=ctypes.c_int(); b=ctypes.c_int(); torch.cuda.init(); print('prio range', h.hipDeviceGetStreamPriorityRange(ctypes.byref(a), ctypes.byref(b)), a.value, b.value)" > gpurun_out/r02g_prio.txt 2>&1
for a in "0 0 4" "1 -1 4" "1 0 4" "0 -1 4" "1 -1 6"; do set -- $a
timeout -k 10 200 python bench.py --workload batch64 --steps 8 --warmup 2 --pipeline 1 --lane-priority $1 --t2s-priority $2 --vits-lanes $3 --no-cpu-baseline > gpurun_out/o.json 2>> gpurun_out/r02g_b64.err
echo "lp $1 tp $2 lanes $3 $(cat gpurun_out/o.json)" >> gpurun_out/r02g_prio.txt
done

set -e
mkdir -p gpurun_out
bash tools/gpu_round.sh r02g pmc
for p in 1 0; do
timeout -k 10 400 python tools/qps_sweep.py --qps 5,20,50,100,200 --requests 120 --pipeline $p > gpurun_out/r02g_qps_p$p.json 2> gpurun_out/r02g_qps_p$p.err
done

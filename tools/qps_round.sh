set -e
mkdir -p gpurun_out
timeout -k 10 900 python tools/qps_sweep.py --qps 5,20,50,100,200 --requests 1000 > gpurun_out/${1:-r02h}_qps.json 2> gpurun_out/${1:-r02h}_qps.err

set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_server_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/r02j_tests.log 2>&1 || { tail -40 gpurun_out/r02j_tests.log; exit 1; }
tail -2 gpurun_out/r02j_tests.log
timeout -k 10 400 python tools/qps_sweep.py --qps 5,20,50,100,200 --requests 60 > gpurun_out/r02j_qps.json 2> gpurun_out/r02j_qps.err || { tail -30 gpurun_out/r02j_qps.err; exit 1; }
cat gpurun_out/r02j_qps.err | grep offered
cat gpurun_out/r02j_qps.json

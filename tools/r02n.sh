set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/knob_sweep.py "pf=1" "pf=2" "pf=3" "pf=5" 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r02n_knobs.txt

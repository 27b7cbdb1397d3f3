set -o pipefail
mkdir -p gpurun_out
for d in 0 20 40 80; do
  echo "pf_delay $d"
  GENIE_PF_DELAY=$d timeout -k 10 120 python tools/ptrace2.py > gpurun_out/pf_$d.txt 2>&1 || { tail -5 gpurun_out/pf_$d.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/pf_$d.txt
done

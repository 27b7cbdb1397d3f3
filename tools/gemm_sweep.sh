# GEMM tile-configuration sweep (tools/gemm_bench.cpp): wall time per launch and rocprof
# kernel durations, for the register-staged k_gemm_x2 (cfg 0) and k_gemm_x3 configurations.
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in ${@:-0 1 5}; do
  if [ "$c" = 0 ]; then export GENIE_GEMM_X3=0; else unset GENIE_GEMM_X3; export GENIE_GEMM_CFG=$c; fi
  rm -rf gpurun_out/gprof_$c
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/gprof_$c -o g -- ./tools/gemm_bench > gpurun_out/gemm_cfg$c.txt 2>&1 || exit 1
  echo "== cfg $c"; cut -c1-17,48-60 gpurun_out/gemm_cfg$c.txt
  find gpurun_out/gprof_$c -name "*kernel_stats.csv" -exec cut -d, -f1-8 {} \; | head -4
done

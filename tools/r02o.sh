set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_r02o_mfma
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_r02o_mfma -o pmc -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r02o_pmc_mfma.log 2>&1 || { tail -20 gpurun_out/r02o_pmc_mfma.log; exit 1; }
python tools/mfma_busy.py gpurun_out/pmc_r02o_mfma --json gpurun_out/r02o_mfma_busy.json > gpurun_out/r02o_mfma_busy.txt 2>&1; cat gpurun_out/r02o_mfma_busy.txt
timeout -k 10 400 python bench.py --workload mixed100 --steps 2 --warmup 1 > gpurun_out/r02o_mixed100.json 2> gpurun_out/r02o_mixed100.err || { tail -20 gpurun_out/r02o_mixed100.err; exit 1; }
cat gpurun_out/r02o_mixed100.json

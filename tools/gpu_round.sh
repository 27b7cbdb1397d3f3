#!/bin/bash
# One GPU-box pass: gpu parity tests, smoke, bench, rocprof kernel stats.
# Usage (from the repo root, via gpurun): bash tools/gpu_round.sh TAG [tests|bench|prof ...]
set -o pipefail
TAG=${1:-run}; shift
STEPS=${@:-tests smoke bench prof}
mkdir -p gpurun_out
export TMPDIR=/tmp
for s in $STEPS; do
  case $s in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
           tail -3 gpurun_out/${TAG}_tests.log ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -30 gpurun_out/${TAG}_smoke.log; exit 1; }
           tail -2 gpurun_out/${TAG}_smoke.log ;;
    bench) timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
           cat gpurun_out/${TAG}_bench.json ;;
    prof)  rm -rf gpurun_out/prof_${TAG}
           timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o bench -- python3 bench.py --no-cpu-baseline --concurrent-streams 0 > gpurun_out/${TAG}_bench_under_rocprof.log 2>&1 || { tail -30 gpurun_out/${TAG}_bench_under_rocprof.log; exit 1; }
           python tools/prof_summary.py gpurun_out/prof_${TAG} > gpurun_out/${TAG}_kernel_stats.txt 2>&1; head -25 gpurun_out/${TAG}_kernel_stats.txt ;;
    batched) for w in batch64 mixed100; do
             timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > gpurun_out/${TAG}_$w.json 2> gpurun_out/${TAG}_$w.err || { tail -30 gpurun_out/${TAG}_$w.err; exit 1; }
             cat gpurun_out/${TAG}_$w.json
           done ;;
    mfma)  # MFMA busy cycles per kernel (SQ_VALU_MFMA_BUSY_CYCLES; GRBM_GUI_ACTIVE sums the 8 XCDs)
           for w in bench aux; do
             if [ $w = bench ]; then cmd="python3 bench.py --no-cpu-baseline --concurrent-streams 0 --steps 3 --warmup 1"; else cmd="python3 tools/aux_models_bench.py"; fi
             rm -rf gpurun_out/pmc_${TAG}_mfma_$w
             timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_${TAG}_mfma_$w -o pmc -- $cmd > gpurun_out/${TAG}_pmc_mfma_$w.log 2>&1 || { tail -30 gpurun_out/${TAG}_pmc_mfma_$w.log; exit 1; }
             python tools/mfma_util.py gpurun_out/pmc_${TAG}_mfma_$w > gpurun_out/${TAG}_mfma_$w.txt 2>&1; head -30 gpurun_out/${TAG}_mfma_$w.txt
           done ;;
    mfmab) # the same MFMA-busy pass over one batch64 batch (k_decode_persistm, k_mrf_pair, the packed prefill)
           rm -rf gpurun_out/pmc_${TAG}_mfma_batch64
           timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_${TAG}_mfma_batch64 -o pmc -- python3 bench.py --workload batch64 --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/${TAG}_pmc_mfma_batch64.log 2>&1 || { tail -30 gpurun_out/${TAG}_pmc_mfma_batch64.log; exit 1; }
           python tools/mfma_util.py gpurun_out/pmc_${TAG}_mfma_batch64 > gpurun_out/${TAG}_mfma_batch64.txt 2>&1; head -30 gpurun_out/${TAG}_mfma_batch64.txt ;;
    pmc)   for c in FETCH_SIZE WRITE_SIZE; do
             rm -rf gpurun_out/pmc_${TAG}_$c
             timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_${TAG}_$c -o pmc -- python3 bench.py --no-cpu-baseline --concurrent-streams 0 --steps 3 --warmup 1 > gpurun_out/${TAG}_pmc_$c.log 2>&1 || { tail -30 gpurun_out/${TAG}_pmc_$c.log; exit 1; }
             python tools/pmc_summary.py gpurun_out/pmc_${TAG}_$c --gfx950-fetch-x2 --json gpurun_out/${TAG}_pmc_$c.json > gpurun_out/${TAG}_pmc_$c.txt 2>&1; grep -i "persist\|conv1d<11" gpurun_out/${TAG}_pmc_$c.txt | head -5 || true
           done ;;
  esac
done

mkdir -p gpurun_out
for c in x2 0 7 8; do
  if [ "$c" = x2 ]; then export GENIE_GEMM_X3=0; unset GENIE_GEMM_CFG; else unset GENIE_GEMM_X3; export GENIE_GEMM_CFG=$c; fi
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --concurrent-streams 0 > gpurun_out/ab_$c.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab_$c.json')); print('$c', round(d['x_realtime'],1), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['phase_ms'].items()}, round(d['sequential']['ms_per_utt'],3))"
done

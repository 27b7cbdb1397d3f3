set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in ${CFGS:-0 1 2 3}; do
  for dbg in ${DBGS:-0 1 2}; do
    rm -rf gpurun_out/cb_${cfg}_${dbg}
    GENIE_CONVH_CFG=$cfg GENIE_CONVH_DBG=$dbg timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/cb_${cfg}_${dbg} -o cb -- python3 tools/convh_bench.py --inproc > gpurun_out/cb_${cfg}_${dbg}.log 2>&1 || { tail gpurun_out/cb_${cfg}_${dbg}.log; exit 1; }
    python3 - gpurun_out/cb_${cfg}_${dbg} $cfg $dbg <<'PY'
import glob, sqlite3, sys, collections
db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
c = sqlite3.connect(db)
rows = c.execute("select name,grid_x,grid_y,workgroup_x,duration from kernels").fetchall()
agg = collections.OrderedDict()
for n, gx, gy, wx, d in rows:
    if "k_conv_h" not in n: continue
    k = (n.split("<")[1].split(">")[0], gx // wx, gy)
    agg.setdefault(k, []).append(d / 1000)
for k, v in agg.items():
    v = sorted(v)[len(v)//4:]   # drop warmup
    print(f"cfg {sys.argv[2]} dbg {sys.argv[3]} {k[0]:16s} grid {k[1]:4d}x{k[2]:2d}: {sum(v)/len(v):7.2f} us")
PY
  done
done

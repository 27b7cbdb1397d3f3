set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-vp}
timeout -k 10 120 python tools/vits_only.py 6 > gpurun_out/${TAG}_wall.txt 2>&1 || { tail gpurun_out/${TAG}_wall.txt; exit 1; }
cat gpurun_out/${TAG}_wall.txt | grep -v amdgpu.ids
rm -rf gpurun_out/${TAG}_db
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/${TAG}_db -o vp -- python3 tools/vits_only.py 6 > gpurun_out/${TAG}_prof.log 2>&1 || { tail gpurun_out/${TAG}_prof.log; exit 1; }
python3 - gpurun_out/${TAG}_db > gpurun_out/${TAG}_breakdown.txt <<'PY'
import glob, sqlite3, sys, collections
db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
c = sqlite3.connect(db)
rows = c.execute("select name,grid_x,grid_y,grid_z,workgroup_x,start,end from kernels order by start").fetchall()
N = 6
agg = collections.OrderedDict(); tot = 0.0; byname = collections.Counter()
for n, gx, gy, gz, wx, s, e in rows:
    nm = n.split("(")[0].replace("void ", "").replace("gsv::", "").replace("(anonymous namespace)::", "")
    d = (e - s) / 1000 / N
    k = (nm[:40], gx // wx, gy, gz)
    a = agg.setdefault(k, [0, 0.0]); a[0] += 1; a[1] += d; tot += d; byname[nm[:40]] += d
print(f"kernel time per utterance {tot:.1f} us, {len(rows)/N:.0f} dispatches per utterance")
for nm, d in byname.most_common(25): print(f"  {nm:40s} {d:8.1f} us")
print()
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:45]:
    print(f"{k[0]:40s} grid=({k[1]},{k[2]},{k[3]}) n/utt={v[0]/N:5.1f} us/utt={v[1]:8.1f} avg={v[1]/v[0]*N:7.1f}")
PY
head -80 gpurun_out/${TAG}_breakdown.txt

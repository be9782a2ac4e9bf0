# Summary of one tools/gpu_<tag>.sh run: GPU tests, build phases, bench lines, kernel trace means.
tag=$1
tail -1 gpurun_out/${tag}_gpu_tests.log
tail -2 gpurun_out/${tag}_phases.log
for f in gpurun_out/${tag}_bench*.log; do grep '^{' $f | python -c "
import json,sys
d=json.loads(sys.stdin.readline())
print('$(basename $f)', 'head', round(d['ms_per_step']*1e3,1), *[(k, round(d[k]['ms_per_step']*1e3,1)) for k in ('batched','c2','c4','c5','c3train') if k in d])"; done
python - $tag <<'PY'
import csv,collections,numpy as np,glob,sys
f=glob.glob(f"gpurun_out/{sys.argv[1]}_trace/**/*kernel_trace.csv",recursive=True)
if f:
    rows=list(csv.DictReader(open(f[0])))
    d=collections.defaultdict(list)
    for r in rows:
        d[r["Kernel_Name"].split("(")[0][:50]+" "+r["Grid_Size_X"]].append((int(r["End_Timestamp"])-int(r["Start_Timestamp"]))/1000)
    for k,v in sorted(d.items(),key=lambda kv:-sum(kv[1]))[:8]:
        v=np.array(v); print(f"  {k:60s} n={len(v):5d} mean={v.mean():7.2f} p50={np.median(v):7.2f} p90={np.percentile(v,90):7.2f}")
PY

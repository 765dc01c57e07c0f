"""Per-solve kernel time of the weighted partition by kernel from a rocprofv3 kernel trace of
tools/probe_wpart.py (the world-1 and world-2 segments split at the generator kernels).
Usage: python tools/wpart_kernels.py <run_kernel_trace.csv>"""
import csv, collections, re, sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
names=[r['Kernel_Name'] for r in rows]
idx=[i for i,n in enumerate(names) if 'wp_kron_count_k' in n]
segs=[(idx[0],idx[1],'world1'),(idx[1],len(rows),'world2')]
for a,b,lab in segs:
    agg=collections.defaultdict(lambda:[0,0.0])
    for r in rows[a:b]:
        n=re.sub(r'^void ','',r['Kernel_Name']).replace('pj::(anonymous namespace)::','')
        n=n.split('(')[0]
        if not (n.startswith('wp_') or 'rocclr' in n): continue
        if 'kron' in n: continue
        d=(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6
        agg[n][0]+=1; agg[n][1]+=d
    print('==',lab, 'per solve (6 solves; world 2 = both ranks summed)')
    tot=0
    for n,(c,t) in sorted(agg.items(), key=lambda x:-x[1][1]):
        tot+=t
        print(f"{n[:40]:40s} {c/6:6.1f} {t/6:8.3f} ms")
    print('total', round(tot/6,3))

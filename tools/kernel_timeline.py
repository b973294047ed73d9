"""Per-call kernel timeline of a config-1 latency run (tools/ab_batch_latency.py under
rocprofv3 --kernel-trace): median duration of each kernel per call and the gap before it,
read from rocprofv3's sqlite output. Usage: python tools/kernel_timeline.py DIR..."""
import sqlite3, glob, collections, re, statistics as st, sys
for d in sys.argv[1:]:
    db = glob.glob(d + "/**/*.db", recursive=True)[0]
    c = sqlite3.connect(db)
    rows = c.execute("select name,start,end from kernels order by start").fetchall()
    def nm(n):
        n = n.replace('(anonymous namespace)::','').replace('void ','').replace('nw::','')
        return re.sub(r'\(.*','',n)
    ks = [(nm(n), s, e) for n,s,e in rows]
    calls=[]; cur=None
    for k in ks:
        if k[0].startswith('k_pip_points'):
            cur=[]; calls.append(cur)
        if cur is not None: cur.append(k)
    calls=calls[20:]
    dur=collections.defaultdict(list); gaps=collections.defaultdict(list); tot=[]; between=[]
    for j,cl in enumerate(calls):
        for i,(n,s,e) in enumerate(cl):
            dur[n].append((e-s)/1e3)
            if i: gaps[n].append((s-cl[i-1][2])/1e3)
        tot.append((cl[-1][2]-cl[0][1])/1e3)
        if j: between.append((cl[0][1]-calls[j-1][-1][2])/1e3)
    print(d, len(calls), 'gpu span median', st.median(tot), 'idle between calls', st.median(between))
    for n in dur: print(f"  {n[:40]:40s} {st.median(dur[n]):8.1f} gap-before {st.median(gaps[n]) if gaps[n] else 0:6.1f}")

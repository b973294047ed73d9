import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l)
    sv=d.get('service_latency') or {}
    for N,v in sv.items():
        if not isinstance(v,dict): continue
        for x in v.get('loads',[]):
            print(N, *[f"{k}={x[k]:.3f}" if isinstance(x[k],float) else f"{k}={x[k]}" for k in ('offered_certs_per_s','achieved_certs_per_s','p50_ms','p99_ms','max_ms','certs_per_job','parity')])

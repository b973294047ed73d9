#!/usr/bin/env python3
"""Diagnostics (GPU box): the bench's asyncio NativeService leg (N = 50 certificates at a fixed
rate) with every mismatch listed — (request, got, expected) — and the service's hedge counts,
for one configuration (the environment: NW_SMALL_DONE ...; argv: rate, certificates, hedge
deadline in seconds, 0 = off). Prints one JSON line.

    python tools/r06/svc_py_check.py 10000 20000 0.001
"""
import asyncio
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from narwhal_amd import crypto as C, service as SV, workloads as W  # noqa: E402


def main():
    N, uniq = 50, 8192
    rate, total, hedge = float(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3])
    keys = [(bytes(pk), bytes(sd) + bytes(pk)) for sd, pk in
            zip(W.fixture_seeds(N), C.keypair_from_seed_many(W.fixture_seeds(N)))]
    s = W.certificate_stream(uniq, keys, lambda sk, m: C.sign_many(sk, m),
                             lambda d, o: C.sha512_digest32_many(d, o[:-1], np.diff(o)), seed=300)
    s, exp_st, exp_ix = W.mutate_votes(s, np.arange(50, uniq, 100), seed=N + 11)
    hb, ho, vo = s["header_bytes"].tobytes(), s["header_offsets"], s["vote_offsets"]
    rows = [SV.CertRow(hb[int(ho[i]):int(ho[i + 1])], int(s["payload_counts"][i]),
                       s["ids"][i].tobytes(), s["header_sigs"][i].tobytes(),
                       s["vote_pks"][int(vo[i]):int(vo[i + 1])].tobytes(),
                       s["vote_sigs"][int(vo[i]):int(vo[i + 1])].tobytes(),
                       int(vo[i + 1] - vo[i])) for i in range(uniq)]
    expect = [(int(a), int(b)) for a, b in zip(exp_st, exp_ix)]
    got = [None] * total

    async def run():
        svc = SV.NativeService(s["committee"], max_items=1 << 20, max_delay=0.0005,
                               max_inflight=4, hedge=hedge)
        loop = asyncio.get_running_loop()
        done = loop.create_future()
        left = [total]

        def make_cb(i):
            def cb(f):
                got[i] = f.result()
                left[0] -= 1
                if left[0] == 0:
                    done.set_result(None)
            return cb
        await asyncio.gather(*[svc.certificate_status(rows[i]) for i in range(64)])
        t0 = loop.time()
        i = 0
        while i < total:
            now = loop.time()
            while i < total and t0 + i / rate <= now:
                (lp, fut), f = svc._future()
                svc.submit_certificate(rows[i % uniq], (lp, fut))
                f.add_done_callback(make_cb(i))
                i += 1
            await asyncio.sleep(min(0.0002, max(0.0, t0 + i / rate - loop.time())))
        await done
        hs = svc.hedge_stats()
        jobs = svc.stats()[1]
        svc.close()
        return hs, jobs

    hs, jobs = asyncio.run(run())
    bad = [(i, tuple(int(x) for x in got[i]), expect[i % uniq]) for i in range(total)
           if tuple(got[i]) != expect[i % uniq]]
    print(json.dumps({"rate": rate, "certs": total, "hedge_s": hedge,
                      "small_done": os.environ.get("NW_SMALL_DONE", "default"),
                      "jobs": jobs, "hedged_hostfirst_hostonly": list(hs),
                      "mismatches": len(bad), "first": bad[:12]}), flush=True)


if __name__ == "__main__":
    main()

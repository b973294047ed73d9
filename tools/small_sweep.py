"""Job-size sweep of Certificate::verify host calls: the small-job launch (nw_small.hip,
NW_SMALL=1) against the bulk pipeline (NW_SMALL=0), blocking nw_certificates_verify_many
per job, median wall time of `reps` calls per size (the service's jobs are exactly these
calls). Prints one JSON line per (committee, certificates per job). Bench tooling."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from narwhal_amd import crypto as C  # noqa: E402
from narwhal_amd import messages as M  # noqa: E402
from narwhal_amd import workloads as W  # noqa: E402


class _Com:
    def __init__(self, p):
        self._p = p

    def packed(self):
        return self._p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--committees", default="4,50")
    ap.add_argument("--sizes", default="1,4,16,64,256,1024,4096,16384")
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--modes", default="1,0")
    args = ap.parse_args()
    sizes = [int(x) for x in args.sizes.split(",")]
    for N in [int(x) for x in args.committees.split(",")]:
        keys = [(bytes(pk), bytes(sd) + bytes(pk)) for sd, pk in
                zip(W.fixture_seeds(N), C.keypair_from_seed_many(W.fixture_seeds(N)))]
        s = W.certificate_stream(max(sizes), keys, lambda sk, m: C.sign_many(sk, m),
                                 lambda d, o: C.sha512_digest32_many(d, o[:-1], np.diff(o)),
                                 seed=N)
        com = _Com(s["committee"])
        for n in sizes:
            ho, vo = s["header_offsets"], s["vote_offsets"]
            sub = {"header_bytes": s["header_bytes"][:int(ho[n])], "header_offsets": ho[:n + 1],
                   "payload_counts": s["payload_counts"][:n], "ids": s["ids"][:n],
                   "header_sigs": s["header_sigs"][:n], "vote_offsets": vo[:n + 1],
                   "vote_pks": s["vote_pks"][:int(vo[n])], "vote_sigs": s["vote_sigs"][:int(vo[n])]}
            row = {"committee": N, "certs": n, "slots": n + int(vo[n])}
            for mode in args.modes.split(","):
                os.environ["NW_SMALL"] = mode
                os.environ["NW_SMALL_MAX_SLOTS"] = str(1 << 30)
                st, _ = M.verify_certificates_many(com, sub, None)   # warm (tables, pool)
                assert (st == 0).all()
                ts = []
                for _ in range(args.reps):
                    t0 = time.perf_counter()
                    M.verify_certificates_many(com, sub, None)
                    ts.append(time.perf_counter() - t0)
                med = float(np.median(ts))
                row[f"small{mode}_ms"] = med * 1e3
                row[f"small{mode}_certs_per_s"] = n / med
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()

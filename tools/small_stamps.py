"""Per-phase times of the small-job kernel (nw_small.hip, NW_SMALL_STAMPS=1: s_memrealtime
stamps per workgroup at the phase boundaries, printed by the library to stderr) for one-
certificate / few-certificate jobs at N = 4 and 50, next to the blocking call's wall time.
Bench tooling (GPU box)."""
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
    for N in (4, 50):
        keys = [(bytes(pk), bytes(sd) + bytes(pk)) for sd, pk in
                zip(W.fixture_seeds(N), C.keypair_from_seed_many(W.fixture_seeds(N)))]
        s = W.certificate_stream(64, keys, lambda sk, m: C.sign_many(sk, m),
                                 lambda d, o: C.sha512_digest32_many(d, o[:-1], np.diff(o)),
                                 seed=N)
        com = _Com(s["committee"])
        for n in (1, 4, 16):
            ho, vo = s["header_offsets"], s["vote_offsets"]
            sub = {"header_bytes": s["header_bytes"][:int(ho[n])], "header_offsets": ho[:n + 1],
                   "payload_counts": s["payload_counts"][:n], "ids": s["ids"][:n],
                   "header_sigs": s["header_sigs"][:n], "vote_offsets": vo[:n + 1],
                   "vote_pks": s["vote_pks"][:int(vo[n])], "vote_sigs": s["vote_sigs"][:int(vo[n])]}
            os.environ.pop("NW_SMALL_STAMPS", None)
            M.verify_certificates_many(com, sub, None)     # tables, pool
            ts = []
            for _ in range(30):
                t = time.perf_counter()
                st, _ = M.verify_certificates_many(com, sub, None)
                ts.append(time.perf_counter() - t)
            assert (st == 0).all()
            print(f"N={N} certs={n}: blocking call median {np.median(ts) * 1e3:.3f} ms", flush=True)
            os.environ["NW_SMALL_STAMPS"] = "1"
            for _ in range(3):
                M.verify_certificates_many(com, sub, None)
            sys.stderr.flush()
    os.environ.pop("NW_SMALL_STAMPS", None)


if __name__ == "__main__":
    main()

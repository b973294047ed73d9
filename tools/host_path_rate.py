#!/usr/bin/env python3
"""One core's rate of the engine's host verification path (nw_host.cpp: the service's hedge)
against the dalek-equivalent restatement (oracle/nw_dalek.c, test infrastructure), per
committee size: single Certificate::verify calls of honest certificates with a quorum of
votes, one thread. Prints one JSON line. (Runs on the CPU; on the GPU box it measures the
box's cores, the ones the hedge threads run on.)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from narwhal_amd import workloads as W  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests import cert_cases as CC  # noqa: E402
from tests.test_host_path import host_certs  # noqa: E402


def main():
    out = {}
    for N in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "4,50").split(",")]:
        keys = O.keys(N)
        s = W.certificate_stream(200, keys, CC.oracle_sign_many, CC.oracle_digest_many, seed=3,
                                 n_votes=W.quorum(N))
        s1 = W.certificate_stream(1, keys, CC.oracle_sign_many, CC.oracle_digest_many, seed=4,
                                  n_votes=W.quorum(N))
        com = s["committee"]
        host_certs(com, s1)
        t = time.perf_counter()
        host_certs(com, s1)
        tb = time.perf_counter() - t          # the committee's host tables + one certificate
        t = time.perf_counter()
        st, _ = host_certs(com, s)
        th = time.perf_counter() - t
        assert (st == 0).all()
        t = time.perf_counter()
        st2, _ = O.certificates_verify_many(com, s, nthreads=1, engine="dalek")
        td = time.perf_counter() - t
        assert (st2 == 0).all()
        out[f"N{N}"] = {"host_path_ms_per_cert": (th - tb) / 199 * 1e3,
                        "host_tables_build_ms": tb * 1e3,
                        "dalek_equivalent_ms_per_cert": td / 200 * 1e3}
    print(json.dumps(out))


if __name__ == "__main__":
    main()

"""Long seeded run of tests/test_gpu_fuzz.py's differential fuzz (GPU box): for each seed,
an honest certificate stream with about half its certificates damaged (byte xors, odd point
encodings, s + l, vote duplication / removal / swaps), verified on the small-job kernel and
on the bulk pipeline with injected coefficients; every (status, index) compared with the
oracle's. Prints one JSON summary line (test infrastructure: the oracle is the checker).
    python tools/fuzz_long.py SEED0 SEEDS"""
import collections
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

from narwhal_amd import messages as M, workloads as W  # noqa: E402
from oracle import oracle as O  # noqa: E402
from cert_cases import oracle_digest_many, oracle_sign_many  # noqa: E402
from test_gpu_fuzz import _damage  # noqa: E402
from test_gpu_messages import _Com  # noqa: E402


def main():
    s0, ns = int(sys.argv[1]), int(sys.argv[2])
    shapes = [(4, 400), (7, 300), (10, 250), (20, 120), (50, 60)]
    checked, mism, statuses = 0, [], collections.Counter()
    t0 = time.time()
    for seed in range(s0, s0 + ns):
        N, n = shapes[seed % len(shapes)]
        s = W.certificate_stream(n, O.keys(N), oracle_sign_many, oracle_digest_many,
                                 payload=seed % 3, seed=9000 + seed)
        rng = np.random.Generator(np.random.PCG64(seed))
        d = _damage(s, rng, 0.5)
        z16 = rng.integers(0, 256, size=(len(d["vote_pks"]), 16), dtype=np.uint8)
        ost, oix = O.certificates_verify_many(s["committee"], d, z16)
        statuses.update(int(x) for x in ost)
        com = _Com(s["committee"])
        for small in ("1", "0"):
            os.environ["NW_SMALL"] = small
            st, ix = M.verify_certificates_many(com, d, z16)
            bad = np.nonzero((st != ost) | (ix != oix))[0]
            checked += len(st)
            mism += [(seed, small, int(i)) for i in bad[:5]]
        print(f"seed {seed} N={N} n={n} ok={not mism} {time.time() - t0:.0f}s", file=sys.stderr,
              flush=True)
    print(json.dumps({"seeds": [s0, s0 + ns], "certificates_checked": checked,
                      "mismatches": len(mism), "first_mismatches": mism[:10],
                      "oracle_statuses": dict(sorted(statuses.items()))}))


if __name__ == "__main__":
    main()

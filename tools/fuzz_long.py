"""Long seeded run of tests/test_gpu_fuzz.py's differential fuzz (GPU box): for each seed,
an honest certificate stream with about half its certificates damaged (byte xors, odd point
encodings, s + l, vote duplication / removal / swaps), verified on the small-job kernel and
on the bulk pipeline with injected coefficients; every (status, index) compared with the
oracle's. Prints one JSON summary line (test infrastructure: the oracle is the checker).
    python tools/fuzz_long.py SEED0 SEEDS [irregular]
``irregular``: committees with mixed-order, small-order, non-canonical and undecodable
members (tests/irregular.py) plus damage on a quarter of the certificates; injected
coefficients on the small-job kernel, the bulk keyed pipeline and the per-certificate path
(every verdict == the oracle's), then random coefficients on the small-job kernel, the bulk
keyed pipeline, the merged-group and small-group policies (every verdict one the oracle
gives for some coefficient set, 64 sets)."""
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


def irregular(s0, ns):
    import irregular as I
    from test_gpu_fuzz import INJECTED_PATHS, RANDOM_PATHS, ENV_KEYS, _irregular_case
    shapes = [(4, 120), (7, 120), (10, 100), (20, 50), (50, 20), (100, 10)]
    checked, mism, statuses, zdep, kinds_seen = 0, [], collections.Counter(), 0, collections.Counter()
    t0 = time.time()

    def run(env, z16):
        for k in ENV_KEYS:
            os.environ.pop(k, None)
        os.environ.update(env)
        return M.verify_certificates_many(_Com(com), d, z16)
    for seed in range(s0, s0 + ns):
        N, n = shapes[seed % len(shapes)]
        com, d, z16, kinds = _irregular_case(N, n, 5000 + seed)
        kinds_seen.update(kinds)
        ost, oix = O.certificates_verify_many(com, d, z16)
        statuses.update(int(x) for x in ost)
        for env in INJECTED_PATHS:
            for _ in range(2):
                st, ix = run(env, z16)
                bad = np.nonzero((st != ost) | (ix != oix))[0]
                checked += len(st)
                mism += [(seed, "injected", str(env), int(i)) for i in bad[:5]]
        poss = I.possible_verdicts(com, d, 64, seed)
        zdep += sum(len(v) > 1 for v in poss)
        for env in RANDOM_PATHS:
            st, ix = run(env, None)
            checked += len(st)
            mism += [(seed, "random", str(env), i) for i, (a, x) in enumerate(zip(st, ix))
                     if (int(a), int(x)) not in poss[i]][:5]
        print(f"seed {seed} N={N} n={n} kinds={sorted(set(kinds))} ok={not mism} "
              f"{time.time() - t0:.0f}s", file=sys.stderr, flush=True)
    print(json.dumps({"mode": "irregular", "seeds": [s0, s0 + ns], "verdicts_checked": checked,
                      "mismatches": len(mism), "first_mismatches": mism[:10],
                      "coefficient_dependent_certificates": zdep,
                      "member_kinds": dict(kinds_seen),
                      "oracle_statuses_injected": dict(sorted(statuses.items()))}))


def main():
    s0, ns = int(sys.argv[1]), int(sys.argv[2])
    if len(sys.argv) > 3 and sys.argv[3] == "irregular":
        return irregular(s0, ns)
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

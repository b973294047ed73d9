"""Long seeded run of tests/test_gpu_fuzz.py's differential fuzz (GPU box): for each seed,
an honest certificate stream with about half its certificates damaged (byte xors, odd point
encodings, s + l, vote duplication / removal / swaps), verified on the small-job kernel and
on the bulk pipeline with injected coefficients; every (status, index) compared with the
oracle's. Prints one JSON summary line (test infrastructure: the oracle is the checker).
    python tools/fuzz_long.py SEED0 SEEDS [irregular|batch]
``irregular``: committees with mixed-order, small-order, non-canonical and undecodable
members (tests/irregular.py) plus damage on a quarter of the certificates; injected
coefficients on the small-job kernel, the bulk keyed pipeline and the per-certificate path
(every verdict == the oracle's), then random coefficients on the small-job kernel, the bulk
keyed pipeline, the merged-group and small-group policies (every verdict one the oracle
gives for some coefficient set: 64 sets, widened to 4,096 more for a verdict outside them).
``batch``: test_gpu_fuzz.py's irregular vote corpus (irregular signers among honest ones, byte
damage, odd R encodings, s + l, high bits) over random batch-size mixes that reach the
chunked-Straus, Pippenger and fused one-call paths; injected coefficients; every batch status
of verify_batch_many, every item's strict status and one lone batch's (status, index)
through the blocking call, against the oracle."""
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
    widened = 0   # random-z verdicts outside the 64 sampled sets, found by the wider search
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
            outside = [(i, (int(a), int(x))) for i, (a, x) in enumerate(zip(st, ix))
                       if (int(a), int(x)) not in poss[i]]
            widened += len(outside)
            mism += [(seed, "random", str(env), i, v) for i, v in outside
                     if not I.verdict_possible(com, d, i, v, seed)][:5]
        print(f"seed {seed} N={N} n={n} kinds={sorted(set(kinds))} ok={not mism} "
              f"{time.time() - t0:.0f}s", file=sys.stderr, flush=True)
    print(json.dumps({"mode": "irregular", "seeds": [s0, s0 + ns], "verdicts_checked": checked,
                      "mismatches": len(mism), "first_mismatches": mism[:10],
                      "coefficient_dependent_certificates": zdep,
                      "verdicts_found_by_widened_search": widened,
                      "member_kinds": dict(kinds_seen),
                      "oracle_statuses_injected": dict(sorted(statuses.items()))}))


def batch(s0, ns):
    from narwhal_amd import crypto as C
    from test_gpu_fuzz import DECODABLE, _irregular_vote_corpus
    kind_sets = [None, DECODABLE, ("mixed",), ("mixed", "small"), ("noncanon",)]
    checked, strict_checked, mism, statuses = 0, 0, [], collections.Counter()
    t0 = time.time()
    for seed in range(s0, s0 + ns):
        rng = np.random.Generator(np.random.PCG64([seed, 5]))
        shape = seed % 4
        if shape == 0:     # many small batches (chunked Straus)
            sizes = rng.integers(0, 400, size=int(rng.integers(1, 40)))
        elif shape == 1:   # Pippenger-size batches side by side
            sizes = rng.integers(400, 3000, size=int(rng.integers(1, 6)))
        elif shape == 2:   # one lone batch in the fused one-call range
            sizes = rng.integers(2925, 16385, size=1)
        else:              # a mix
            sizes = np.concatenate([rng.integers(0, 100, size=5), rng.integers(500, 5000, size=2)])
        kinds = kind_sets[seed % len(kind_sets)]
        # decodable members only for large batches: an undecodable key fails the batch fast
        if kinds is None and sizes.max(initial=0) > 1000:
            kinds = DECODABLE
        irr = float(rng.choice([0.0005, 0.002, 0.01, 0.08]))
        bad = float(rng.choice([0.0, 0.0005, 0.003, 0.03]))
        dig, pks, sigs, off, z16, bidx = _irregular_vote_corpus(sizes, 70000 + seed, bad, irr,
                                                                kinds)
        ost = O.verify_batch_many(dig, pks, sigs, off, z16)
        statuses.update(int(x) for x in ost)
        st = C.verify_batch_many(dig, pks, sigs, off, z16)
        checked += len(st)
        mism += [(seed, "batch", int(i)) for i in np.nonzero(st != ost)[0][:5]]
        if len(pks):
            sst, _ = C.verify_strict_many(dig[bidx], pks, sigs)
            osst = O.verify_strict_many(dig[bidx], pks, sigs)
            strict_checked += len(sst)
            mism += [(seed, "strict", int(i)) for i in np.nonzero(sst != osst)[0][:5]]
            b = int(np.argmax(np.diff(off)))
            a, e = int(off[b]), int(off[b + 1])
            votes = [(C.PublicKey(pks[i].tobytes()), C.Signature.from_bytes(sigs[i].tobytes()))
                     for i in range(a, e)]
            ost1, oix1 = O.verify_batch(dig[b].tobytes(), pks[a:e], sigs[a:e], z16[a:e])
            try:
                C.Signature.verify_batch(C.Digest(dig[b].tobytes()), votes,
                                         z16=z16[a:e].tobytes())
                got = (0, 0)
            except C.CryptoError as err:
                got = (err.code, err.index)
            if got != (ost1, oix1 if ost1 else 0):
                mism.append((seed, "lone", got, (int(ost1), int(oix1))))
        print(f"seed {seed} batches={len(sizes)} votes={int(off[-1])} ok={not mism} "
              f"{time.time() - t0:.0f}s", file=sys.stderr, flush=True)
    print(json.dumps({"mode": "batch", "seeds": [s0, s0 + ns], "batch_verdicts_checked": checked,
                      "strict_verdicts_checked": strict_checked, "mismatches": len(mism),
                      "first_mismatches": mism[:10],
                      "oracle_batch_statuses": dict(sorted(statuses.items()))}))


def main():
    s0, ns = int(sys.argv[1]), int(sys.argv[2])
    if len(sys.argv) > 3 and sys.argv[3] == "irregular":
        return irregular(s0, ns)
    if len(sys.argv) > 3 and sys.argv[3] == "batch":
        return batch(s0, ns)
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

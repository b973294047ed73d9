#!/usr/bin/env python3
"""Differential fuzz of the engine's host verification path (narwhal_amd/csrc/nw_host.cpp,
the certificate service's hedge) against the oracle, on the CPU (test infrastructure: the
oracle is the checker). Per seed:

* an irregular committee (tests/irregular.py: mixed-order, small-order, non-canonical and
  undecodable members as authors and voters) with a quarter of its certificates damaged
  (tests/test_gpu_fuzz.py _damage): nw_host_certificates_verify_many with injected
  coefficients (every (status, index) == the oracle's), headers only (==), and with fresh
  CSPRNG coefficients (every verdict one the oracle gives for some coefficient set: 64 sets,
  widened to 4,096 more for a verdict outside them);
* irregular-signer batches of ragged sizes with injected coefficients (==), and every item
  of them through nw_host_verify_strict_many (==).

    python tools/fuzz_host.py SEED0 SEEDS OUT.json
"""
import collections
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

from oracle import oracle as O  # noqa: E402
import irregular as I  # noqa: E402
from test_gpu_fuzz import _irregular_case  # noqa: E402
from test_host_path import host_batch, host_certs, host_strict  # noqa: E402
from test_dalek_restatement import _irregular_batch  # noqa: E402

SHAPES = [(4, 60), (7, 50), (10, 40), (20, 24), (50, 10), (100, 6)]


def main():
    s0, ns, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    t0 = time.time()
    checked = collections.Counter()
    mism = []
    statuses = collections.Counter()
    kinds_seen = collections.Counter()
    widened = 0
    for seed in range(s0, s0 + ns):
        N, n = SHAPES[seed % len(SHAPES)]
        com, d, z16, kinds = _irregular_case(N, n, 7000 + seed)
        kinds_seen.update(kinds)
        ost, oix = O.certificates_verify_many(com, d, z16)
        statuses.update(int(x) for x in ost)
        st, ix = host_certs(com, d, z16)
        bad = np.nonzero((st != ost) | (ix != oix))[0]
        checked["certs_injected"] += len(st)
        mism += [(seed, "certs_injected", int(i)) for i in bad[:5]]
        hst, hix = O.certificates_verify_many(com, d, headers_only=True)
        st, ix = host_certs(com, d, None, headers_only=True)
        bad = np.nonzero((st != hst) | (ix != hix))[0]
        checked["headers"] += len(st)
        mism += [(seed, "headers", int(i)) for i in bad[:5]]
        st, ix = host_certs(com, d, None)
        poss = I.possible_verdicts(com, d, 64, 7000 + seed)
        for i in range(len(st)):
            v = (int(st[i]), int(ix[i]))
            if v in poss[i]:
                continue
            if I.verdict_possible(com, d, i, v, 7000 + seed):
                widened += 1
            else:
                mism.append((seed, "certs_random", i))
        checked["certs_random"] += len(st)
        # irregular-signer batches, ragged sizes, injected z; every item strict
        rng = np.random.Generator(np.random.PCG64([seed, 11]))
        batches = [_irregular_batch(int(k), 90_000 + 16 * seed + j, bad=int(rng.integers(0, 3) == 0))
                   for j, k in enumerate(rng.integers(1, 40, 6))]
        dg = np.stack([np.frombuffer(b[0], np.uint8) for b in batches])
        pks = np.concatenate([b[1] for b in batches])
        sigs = np.concatenate([b[2] for b in batches])
        z = np.concatenate([b[3] for b in batches])
        off = np.cumsum([0] + [len(b[1]) for b in batches]).astype(np.uint64)
        bst, bfi = host_batch(dg, pks, sigs, off, z)
        for j, b in enumerate(batches):
            want = O.verify_batch(b[0], b[1], b[2], b[3])
            checked["batches"] += 1
            if (int(bst[j]), int(bfi[j])) != tuple(want):
                mism.append((seed, "batch", j))
        msgs = np.concatenate([np.repeat(dg[j:j + 1], len(b[1]), axis=0) for j, b in enumerate(batches)])
        sst = host_strict(msgs, pks, sigs)
        ost = O.verify_strict_many(msgs, pks, sigs)
        bad = np.nonzero(sst != ost)[0]
        checked["strict"] += len(sst)
        mism += [(seed, "strict", int(i)) for i in bad[:5]]
    res = {"tool": "tools/fuzz_host.py", "seeds": [s0, s0 + ns], "checked": dict(checked),
           "mismatches": len(mism), "first_mismatches": mism[:20],
           "random_z_widened": widened, "oracle_statuses": dict(sorted(statuses.items())),
           "member_kinds": dict(kinds_seen), "seconds": round(time.time() - t0, 1)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))
    return 0 if not mism else 1


if __name__ == "__main__":
    sys.exit(main())

"""Generates the golden vectors in tests/golden/ from the CPU oracle.

Run only after tests/test_oracle.py passes (the oracle is pinned to the reference's
known-answer tests and to scipy/numpy). The reference package itself is not run here
(SURVEY.md §8(c)); these are the oracle's outputs on seeded inputs:

  rdm_N.npz        X (N x D float32, seeded), rdm = compute_rdm(X)        rsa.py:59-93
  spearman_N.npz   A, B (RDMs of seeded features), scipy spearmanr of the upper
                   triangles and the exact-midrank restatement            rsa.py:96-129
  bootstrap_N.npz  model/neural RDMs, the RandomState(42) index sets, point,
                   50 bootstrap scores and the 2.5/97.5 percentiles       evals.py:341-373
  rng.npz          numpy.random.RandomState(seed).choice(n, k, replace=False) streams

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import rsa_oracle as O  # noqa: E402

SIZES = {4: 16, 16: 48, 64: 128, 256: 512}
N_BOOT = 50


def main():
    for n, d in SIZES.items():
        feats = O.synthetic_features(n, [d, d // 2 + 3], seed=1000 + n, relu=[True, False])
        x = feats[0]
        np.savez_compressed(os.path.join(HERE, f"rdm_{n}.npz"), X=x, rdm=O.compute_rdm(x))
        a, b = O.compute_rdm(feats[0]), O.compute_rdm(feats[1])
        iu = np.triu_indices(n, 1)
        np.savez_compressed(os.path.join(HERE, f"spearman_{n}.npz"), A=a, B=b,
                            scipy=np.float64(O.compute_rdm_correlation(a, b, "Spearman")),
                            exact=np.float64(O.midrank_spearman(a[iu], b[iu])),
                            pearson=np.float64(O.compute_rdm_correlation(a, b, "Pearson")))
        if n >= 16:
            point, scores, lo, hi = O.bootstrap_rsa(a, b, n_bootstrap=N_BOOT, seed=42)
            rs = np.random.RandomState(42)
            idx = np.stack([rs.choice(n, int(0.9 * n), replace=False) for _ in range(N_BOOT)])
            np.savez_compressed(os.path.join(HERE, f"bootstrap_{n}.npz"), A=a, B=b, idx=idx,
                                point=np.float64(point), scores=scores, ci=np.array([lo, hi]))
    streams = {}
    for seed, n, k, draws in [(42, 10, 9, 5), (42, 256, 230, 5), (42, 1000, 900, 3),
                              (0, 10000, 9000, 2), (7, 1854, 370, 2)]:
        rs = np.random.RandomState(seed)
        streams[f"s{seed}_n{n}_k{k}"] = np.stack([rs.choice(n, k, replace=False) for _ in range(draws)])
    streams["perm_42_1854"] = np.random.RandomState(42).permutation(1854)
    np.savez_compressed(os.path.join(HERE, "rng.npz"), **streams)
    print("golden vectors written to", HERE)


if __name__ == "__main__":
    main()

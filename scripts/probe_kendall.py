"""Kendall tau-a engine timing at configs[1]'s size (N = 10k, 1000 bootstraps of 9000):
the bench's synthetic RDM shapes, HIP events around the point-only call and the full
1001-subset call, per-kernel times from vr_ktimer where available.

  python scripts/probe_kendall.py [n] [n_boot]      (CASES=unit,point ... to run a subset;
                                                     ALT_LIB=path: another library build)
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if os.environ.get("ALT_LIB"):  # another library build (A/B)
    import visreps_amd._lib as _L  # noqa: E402

    _L.LIB_PATH = os.environ["ALT_LIB"]
from visreps_amd.analysis import rsa as R  # noqa: E402
from visreps_amd.analysis._random import bootstrap_indices  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(20260306)
    z = torch.randn(n, 64, device=dev, generator=g)
    xm = torch.relu(z @ (torch.randn(64, 4096, device=dev, generator=g) / 8)
                    + 2 * torch.randn(n, 4096, device=dev, generator=g))
    xn = z @ torch.randn(64, 2000, device=dev, generator=g) + 3 * torch.randn(n, 2000, device=dev, generator=g)
    xn2 = z @ torch.randn(64, 2000, device=dev, generator=g) + 3 * torch.randn(n, 2000, device=dev, generator=g)
    xu = torch.randn(n, 2000, device=dev, generator=g)  # independent of z: an uncorrelated RDM
    plans = {"model": R.RankPlan(R.compute_rdm(xm)), "neural": R.RankPlan(R.compute_rdm(xn)),
             "neural2": R.RankPlan(R.compute_rdm(xn2)), "noise": R.RankPlan(R.compute_rdm(xu))}
    idx = bootstrap_indices(42, n, int(0.9 * n), nb)
    out = {"n": n, "n_boot": nb}
    from visreps_amd._lib import ktimer_enable, ktimer_read
    for name, a, b, sets in (("point", "model", "neural", None), ("one_pass", "model", "neural", idx[:63]),
                             ("unit", "model", "neural", idx), ("unit_n2_n", "neural2", "neural", idx),
                             ("unit_noise_n", "noise", "neural", idx), ("unit_n_noise", "neural", "noise", idx)):
        if os.environ.get("CASES") and name not in os.environ["CASES"].split(","):
            continue
        pa, pb = plans[a], plans[b]
        R.bootstrap_kendall(pa, pb, sets if sets is None else sets[:2], full_first=True)  # warm
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t = time.perf_counter()
        ktimer_enable(True)
        e0.record()
        sc = R.bootstrap_kendall(pa, pb, sets, full_first=True)
        e1.record()
        torch.cuda.synchronize()
        kms, kl, _ = ktimer_read("k_kwalk")
        ktimer_enable(False)
        out[name] = {"ms": round(e0.elapsed_time(e1), 2), "wall_s": round(time.perf_counter() - t, 3),
                     "point": float(sc[0]), "kwalk_ms": round(kms, 2), "kwalk_launches": kl}
        print(name, out[name], file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

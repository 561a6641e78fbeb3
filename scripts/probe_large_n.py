"""Engine unit time above the two-workgroup LDS mask limit: N = 12,000 and
20,500 stimuli, 4 regions x 3 model plans, 1000 RandomState(42) bootstraps of 0.9 N.

Modes (one line each, ms per unit = HIP-event time of the calls / 12 units):
  grid     the region-fused call (bootstrap_spearman_grid; masks in LDS up to 20,352, else L2)
  region   one joined multi call per region (VISREPS_ENGINE_GRID path off: k_rankB per unit)
and every score of `grid` is compared with `region` (bit-equal). ALT_LIB=path selects another
library build (e.g. the prefetching walk with L2 masks, -DVR_XW_L2=1). SIZES=12000,20500."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

if os.environ.get("ALT_LIB"):
    import visreps_amd._lib as _L
    _L.LIB_PATH = os.environ["ALT_LIB"]
from visreps_amd import _lib
from visreps_amd.analysis import rsa as R
from visreps_amd.analysis._random import bootstrap_indices

dev = torch.device("cuda", 0)
NB = int(os.environ.get("NB", 1000))


def rdm(n, d, seed, z):
    g = torch.Generator(device=dev).manual_seed(seed)
    x = z @ torch.randn(z.size(1), d, device=dev, generator=g) / 8 + torch.randn(n, d, device=dev, generator=g)
    return R.compute_rdm(torch.relu(x) if seed % 2 else x)


def timed(fn):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    out = fn()
    b.record()
    torch.cuda.synchronize()
    return out, a.elapsed_time(b)


for n in [int(s) for s in os.environ.get("SIZES", "12000,20500").split(",")]:
    g = torch.Generator(device=dev).manual_seed(n)
    z = torch.randn(n, 64, device=dev, generator=g)
    neurals = [R.RankPlan(rdm(n, 1000 + 500 * i, 2 * i, z)) for i in range(4)]
    models = [R.RankPlan(rdm(n, 2048, 11 + 2 * j, z)) for j in range(3)]
    del z
    torch.cuda.empty_cache()
    idx = torch.from_numpy(bootstrap_indices(42, n, int(0.9 * n), NB).copy()).to(dev)
    units = len(neurals) * len(models)
    sj = R.SharedJoins(neurals)
    js = [sj.join(pm) for pm in models]  # js[m][region]
    del sj
    L = _lib.lib()
    c0 = [int(L.vr_engine_est_reruns()), int(L.vr_engine_est_predicted()), int(L.vr_engine_est1_fallbacks())]
    _lib.ktimer_enable(True)
    grid, t_grid = timed(lambda: R.bootstrap_spearman_grid(neurals, models, idx, js, full_first=True))
    gl = _lib.ktimer_read("k_rankB_grid")
    _lib.ktimer_enable(False)
    _lib.workspace.release("engine")
    torch.cuda.empty_cache()
    _lib.ktimer_enable(True)
    outs, t_reg = [], 0.0
    for i, pn in enumerate(neurals):
        o, t = timed(lambda: R.bootstrap_spearman_multi(pn, models, idx, full_first=True,
                                                        joined=[js[m][i] for m in range(len(models))]))
        outs.append(o)
        t_reg += t
    rb = _lib.ktimer_read("k_rankB_est")
    _lib.ktimer_enable(False)
    equal = all(torch.equal(grid[i], outs[i]) for i in range(len(neurals)))
    print(f"n={n} M={n * (n - 1) // 2} boots={NB}: grid {t_grid / units:.2f} ms/unit "
          f"(k_rankB_grid {gl[1]} launches, {gl[0] / max(gl[1], 1):.3f} ms each) | per-region {t_reg / units:.2f} ms/unit "
          f"(k_rankB {rb[1]} launches, {rb[0] / max(rb[1], 1):.3f} ms each) | bit-equal {equal} "
          f"| calls off EST 3 up front {int(L.vr_engine_est_predicted()) - c0[1]}, in EST 1 "
          f"{int(L.vr_engine_est1_fallbacks()) - c0[2]}, passes re-run exact {int(L.vr_engine_est_reruns()) - c0[0]}",
          flush=True)
    del neurals, models, js, grid, outs, idx
    _lib.workspace.release()
    torch.cuda.empty_cache()

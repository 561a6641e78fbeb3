"""configs[2]'s plan-free statistics at 73,000 stimuli (2.66e9 pairs): spearman_full and the
Kendall full path on two latent-structured RDMs (Spearman in its default bucketed count-table form,
then VISREPS_FULL_FORM=table and =sort), each timed twice with HIP events (the first
call also allocates its workspace). ALT_LIB=path selects another library build."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

if os.environ.get("ALT_LIB"):
    import visreps_amd._lib as _L
    _L.LIB_PATH = os.environ["ALT_LIB"]
from visreps_amd._lib import workspace
from visreps_amd.analysis import rsa as R

dev = torch.device("cuda", 0)
n = int(os.environ.get("N", 73000))
g = torch.Generator(device=dev).manual_seed(73)
z = torch.randn(n, 32, device=dev, generator=g)
a = R.compute_rdm(torch.relu(z @ torch.randn(32, 256, device=dev, generator=g) + torch.randn(n, 256, device=dev, generator=g)))
b = R.compute_rdm(z + 0.7 * torch.randn(n, 32, device=dev, generator=g))
del z
torch.cuda.synchronize()


def timed(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    v = fn()
    e1.record()
    torch.cuda.synchronize()
    return v, e0.elapsed_time(e1)


def form(name):
    def run():
        if name == "sort":  # the sort form's workspace (the default one holds the count tables)
            from visreps_amd._lib import lib
            workspace.get(dev, lib().vr_spearman_full_sort_workspace(n), "spearman_full")
        os.environ["VISREPS_FULL_FORM"] = name
        try:
            return R.spearman_full(a, b)
        finally:
            del os.environ["VISREPS_FULL_FORM"]
    return run


for name, fn, tag in (("spearman_full", lambda: R.spearman_full(a, b), "spearman_full"),
                      ("spearman_full[table form]", form("table"), "spearman_full"),
                      ("spearman_full[sort form]", form("sort"), "spearman_full"),
                      ("kendall_full", lambda: R.compute_rdm_correlation(a, b, correlation="Kendall"), "kendall_full")):
    v1, t1 = timed(fn)
    v2, t2 = timed(fn)
    assert v1 == v2
    from visreps_amd._lib import lib
    form_used = lib().vr_spearman_full_last_form() if name.startswith("spearman") else None
    print(f"{name} n={n}: {t2:.1f} ms (first call {t1:.1f} ms) value={v2!r} form={form_used}", flush=True)
    workspace.release(tag)
    torch.cuda.empty_cache()

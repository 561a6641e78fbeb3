"""RDMs at the BASELINE configs' large sizes on one MI355X (HIP-event timed), with a
fp64 spot check of sampled rows against the reference's formula (rsa.py:59-93).

  cfg3 analogue: N = 73,000 stimuli x D = 43,264 (conv5), fp32 features, full 73k x 73k RDM
  cfg5:          N = 50,000 x D = 768 (CLIP width) and x D = 151,296 (ViT-B/16 block), bf16
                 features (the reference upcasts to fp32 before centring, rsa.py:76)

Features are synthetic: relu(Z W + 2 E) with a 64-d latent, seeded.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from visreps_amd.analysis import rsa as R

dev = torch.device("cuda", 0)
CASES = [(73000, 43264, torch.float32, "cfg3: conv5 N=73k fp32"),
         (50000, 768, torch.bfloat16, "cfg5: CLIP width N=50k bf16"),
         (50000, 151296, torch.bfloat16, "cfg5: ViT-B/16 block N=50k bf16")]
if os.environ.get("CASES"):
    CASES = [CASES[int(i)] for i in os.environ["CASES"].split(",")]


def features(n, d, dtype, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    z = torch.randn(n, 64, device=dev, generator=g)
    x = torch.empty(n, d, device=dev, dtype=dtype)
    for c0 in range(0, d, 8192):
        c1 = min(d, c0 + 8192)
        w = torch.randn(64, c1 - c0, device=dev, generator=g) / 8.0
        e = torch.randn(n, c1 - c0, device=dev, generator=g)
        x[:, c0:c1] = torch.relu(z @ w + 2.0 * e).to(dtype)
    return x


def spot_check(x, rdm, rows, correction=1e-12):
    """max |RDM - RDM_fp64| over the sampled rows (fp64 centring and Gram)."""
    n, d = x.shape
    xs = x[rows].double()
    ms = xs.mean(1, keepdim=True)
    xs = xs - ms
    ss = torch.sqrt((xs * xs).mean(1) + correction)
    worst = 0.0
    for c0 in range(0, n, 4096):
        c1 = min(n, c0 + 4096)
        xc = x[c0:c1].double()
        xc = xc - xc.mean(1, keepdim=True)
        sc = torch.sqrt((xc * xc).mean(1) + correction)
        corr = (xs @ xc.T / d) / (ss[:, None] * sc[None, :] + correction)
        ref = 1.0 - corr.clamp(-1.0, 1.0)
        cols = torch.arange(c0, c1, device=dev)
        ref[rows[:, None] == cols[None, :]] = 0.0
        worst = max(worst, float((rdm[rows, c0:c1].double() - ref).abs().max()))
        del xc, corr, ref
    return worst


out = []
for i, (n, d, dtype, name) in enumerate(CASES):
    t = time.perf_counter()
    x = features(n, d, dtype, 1000 + i)
    torch.cuda.synchronize()
    rdm = R.compute_rdm(x)  # warm-up: workspace and output allocation
    torch.cuda.synchronize()
    del rdm  # its block goes back to the caching allocator: the timed calls allocate nothing
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 2
    a.record()
    for _ in range(reps):
        rdm = R.compute_rdm(x)
        if _ + 1 < reps:
            del rdm
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    rows = torch.randperm(n, device=dev, generator=torch.Generator(device=dev).manual_seed(7))[:64]
    err = spot_check(x, rdm, rows)
    sym = float((rdm[rows][:, rows] - rdm[rows][:, rows].T).abs().max())
    rec = {"case": name, "n": n, "d": d, "dtype": str(dtype).replace("torch.", ""),
           "rdm_ms": round(ms, 2), "tflops_effective": round(n * (n + 1) * d / ms / 1e9, 1),
           "max_abs_err_vs_fp64_64rows": err, "max_asym_sampled": sym,
           "peak_mem_GB": round(torch.cuda.max_memory_allocated() / 1e9, 1),
           "wall_s_incl_generation": round(time.perf_counter() - t, 1)}
    print(json.dumps(rec), flush=True)
    out.append(rec)
    assert err < 2e-5 and sym == 0.0, rec
    del x, rdm
    R.workspace.release()
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats()

"""Pipelined (global_load_lds) vs register-staged wide split Gram: bit-equality of the RDMs
and HIP-event time per RDM (VISREPS_GRAM_PIPE is read per call)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from visreps_amd.analysis import rsa as R
dev = torch.device("cuda", 0)


def timed(x, pipe, reps=3):
    os.environ["VISREPS_GRAM_PIPE"] = pipe
    out = R.compute_rdm(x)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        R.compute_rdm(x)
    b.record(); torch.cuda.synchronize()
    return out, a.elapsed_time(b) / reps


for spec in os.environ.get("CASES", "10000x43264,10000x290400,10000x4096,20000x43264,4096x8192").split(","):
    N, D = (int(v) for v in spec.split("x"))
    g = torch.Generator(device=dev).manual_seed(N + D)
    x = torch.randn(N, D, device=dev, generator=g).relu_()
    r0, t0 = timed(x, "0")
    r1, t1 = timed(x, "1")
    same = torch.equal(r0, r1)
    diff = float((r0 - r1).abs().max())
    fl = N * (N + 1) * D
    print(f"N={N} D={D}: regstage {t0:.2f} ms ({fl / t0 / 1e9:.1f} TF/s)  glds {t1:.2f} ms ({fl / t1 / 1e9:.1f} TF/s)"
          f"  bit-equal={same} max|d|={diff:.3g}", flush=True)
    del x, r0, r1

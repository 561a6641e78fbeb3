"""Split-Gram RDM time and a hash of the RDM bytes for one library build
(VISREPS_AMD_LIB selects it): two builds whose kernels sum in the same order print the
same hashes. CASES = comma-separated NxD (relu'd N(0,1) rows)."""
import hashlib, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from visreps_amd.analysis import rsa as R
dev = torch.device("cuda", 0)
for spec in os.environ.get("CASES", "10000x43264,10000x290400,10000x186624").split(","):
    N, D = (int(v) for v in spec.split("x"))
    g = torch.Generator(device=dev).manual_seed(N + D)
    x = torch.randn(N, D, device=dev, generator=g).relu_()
    r = R.compute_rdm(x)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(3):
        R.compute_rdm(x)
    b.record(); torch.cuda.synchronize()
    t = a.elapsed_time(b) / 3
    h = hashlib.sha1(r.cpu().numpy().tobytes()).hexdigest()[:16]
    print(f"N={N} D={D}: {t:.2f} ms ({N * (N + 1) * D / t / 1e9:.1f} TF/s) sha1={h}", flush=True)
    del x, r

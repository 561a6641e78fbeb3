"""Per-wave start / end clocks of one k_rankB launch (probe build -DVR_PROBE_WT=1:
bash scripts/build_alt.sh wt "-DVR_PROBE_WT=1"): a unit of random N = 10k RDMs with 1023
bootstraps (16 full 64-lane passes), the last launch's waves. Shows whether the launch
time is the waves' common work or a tail of slow waves. Usage: ALT_LIB=abl/wt.so python ..."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import visreps_amd._lib as _L

_L.LIB_PATH = os.environ["ALT_LIB"]
from visreps_amd.analysis import rsa as R
from visreps_amd.analysis._random import bootstrap_indices

dev = torch.device("cuda", 0)
n = 10000
g = torch.Generator(device=dev).manual_seed(3)
a = R.compute_rdm(torch.randn(n, 300, device=dev, generator=g))
b = R.compute_rdm(torch.relu(torch.randn(n, 200, device=dev, generator=g)))
pa, pb = R.RankPlan(a), R.RankPlan(b)
idx = torch.from_numpy(bootstrap_indices(42, n, int(0.9 * n), 1023).copy()).to(dev)
for _ in range(2):
    R.bootstrap_spearman(pa, pb, idx, full_first=True)
torch.cuda.synchronize()
L = _L.lib()
buf = np.zeros(2 * 16384, dtype=np.uint64)
assert L.vr_probe_wave_times(buf.ctypes.data_as(ctypes.c_void_p)) == 0
st, en = buf[:16384].astype(np.int64), buf[16384:].astype(np.int64)
ok = (st > 0) & (en > 0)
st, en = st[ok], en[ok]
t0 = st.min()
dur = (en - st) * 10e-3  # us (100 MHz)
end = (en - t0) * 10e-3
beg = (st - t0) * 10e-3
print(f"waves {ok.sum()}  launch span {end.max():.1f} us  starts: max {beg.max():.1f} us")
print("wave duration us: " + "  ".join(f"p{q}={np.percentile(dur, q):.1f}" for q in (0, 10, 50, 90, 99, 100)))
print("wave end us:      " + "  ".join(f"p{q}={np.percentile(end, q):.1f}" for q in (0, 10, 50, 90, 99, 100)))
print(f"mean duration / span = {dur.mean() / end.max():.3f}")
# per XCD (blockIdx round-robin over 8 XCDs: wave // 16 % 8) and per segment position
w = np.nonzero(ok)[0]
xcd = (w // 16) % 8
print("median duration per XCD: " + " ".join(f"{np.median(dur[xcd == x]):.0f}" for x in range(8)))

"""Per-layer timing of CustomCNN's feature stack at the bench batch (fp32, cudnn.benchmark /
MIOpen find as in bench.py), with two alternatives per Conv2d: NHWC (channels_last) and
im2col (F.unfold) + fp32 matmul. Prints ms per batch and per 10k-image step, and the max
|diff| of each alternative against the default conv."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
os.environ.setdefault("MIOPEN_FIND_MODE", "NORMAL")
import torch
import torch.nn.functional as F

from visreps_amd.models.custom_model import CustomCNN

torch.backends.cudnn.benchmark = True
dev = torch.device("cuda", 0)
torch.manual_seed(0)
B = int(os.environ.get("BATCH", "128"))
steps = 10000 / B
model = CustomCNN(num_classes=1000).to(dev).eval()
x = torch.randn(B, 3, 224, 224, device=dev)


def timeit(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def im2col_conv(m, inp):
    k, s, p = m.kernel_size, m.stride, m.padding
    cols = F.unfold(inp, k, padding=p, stride=s)  # (B, C k k, L)
    ho = (inp.shape[2] + 2 * p[0] - k[0]) // s[0] + 1
    wo = (inp.shape[3] + 2 * p[1] - k[1]) // s[1] + 1
    w = m.weight.reshape(m.out_channels, -1)
    return torch.matmul(w, cols).reshape(inp.shape[0], m.out_channels, ho, wo)


total = 0.0
with torch.no_grad():
    h = x
    for i, m in enumerate(model.features):
        inp = h
        t = timeit(lambda: m(inp.clone()) if isinstance(m, torch.nn.ReLU) else m(inp))
        total += t
        line = f"{i:2d} {type(m).__name__:12s} in {tuple(inp.shape)} {t:7.3f} ms/batch {t * steps:7.1f} ms/step"
        if isinstance(m, torch.nn.Conv2d):
            ref = m(inp)
            mc = torch.nn.Conv2d(m.in_channels, m.out_channels, m.kernel_size, m.stride, m.padding, bias=False).to(dev)
            mc.weight.data.copy_(m.weight.data)
            mc = mc.to(memory_format=torch.channels_last)
            inc = inp.contiguous(memory_format=torch.channels_last)
            tc = timeit(lambda: mc(inc))
            dc = (mc(inc) - ref).abs().max().item()
            ti = timeit(lambda: im2col_conv(m, inp))
            di = (im2col_conv(m, inp) - ref).abs().max().item()
            line += f" | nhwc {tc:7.3f} (d {dc:.1e}) | im2col {ti:7.3f} (d {di:.1e})"
        print(line, flush=True)
        h = m(inp) if not isinstance(m, torch.nn.ReLU) else m(inp.clone())
print(f"features total {total:.3f} ms/batch, {total * steps:.1f} ms/step")

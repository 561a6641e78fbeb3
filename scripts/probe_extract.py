"""Extraction-only timing (CustomCNN, 14 points, N=10k synthetic images, bench.py's
extract()): BATCH and BENCH=1 (torch.backends.cudnn.benchmark, MIOpen find) from the env."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch

import bench
from visreps_amd.dataloaders.synthetic import make_images
from visreps_amd.models.custom_model import CustomCNN
from visreps_amd.models.utils import FeatureExtractor

torch.backends.cudnn.benchmark = os.environ.get("BENCH", "0") == "1"
dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = CustomCNN(num_classes=1000).to(dev).eval()
ext = FeatureExtractor(model, bench.LAYERS, extract_pre_and_post=True)
images = make_images(range(10000), device=dev)
if os.environ.get("CL") == "1":  # channels_last (NHWC) convolutions
    model = model.to(memory_format=torch.channels_last)
    images = images.contiguous(memory_format=torch.channels_last)
batch = int(os.environ.get("BATCH", "128"))
with torch.no_grad():
    for it in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        f = bench.extract(ext, images, batch)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        del f
print(f"CL={os.environ.get('CL', '0')} batch={batch} cudnn.benchmark={torch.backends.cudnn.benchmark} "
      f"find={os.environ.get('MIOPEN_FIND_MODE')}: {dt * 1e3:.1f} ms", flush=True)

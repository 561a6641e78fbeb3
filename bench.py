"""Benchmark: end-to-end RSA eval seconds (extract -> RDM -> 1000-bootstrap Spearman).

Workload = BASELINE.json configs[1]: a randomly initialised CustomCNN (the AlexNet-style
network visreps evaluates; 7 layers x pre/post = 14 extraction points) over N = 10,000
synthetic 224x224 stimuli, x 4 NSD-shaped ROIs (V1/V2/V3 = 2000 voxels, hV4 = 1000),
every (point, ROI) unit = point Spearman + 1000 bootstrap subsets of int(0.9 N)
stimuli (RandomState(42) per unit, evals.py:341-373). One step = the whole eval:
extraction, 18 RDMs, 18 rank plans, 56 units. Inputs (images, responses) are resident
in HBM before timing starts.

  python bench.py [--gpus N --steps K --warmup W]   (N > 1 under torch.distributed.run)

Rank 0 prints one JSON line. `roofline` is the bootstrap engine (the dominant cost):
algorithmic bytes 8*[M(N) + 1000*M(0.9N)] per unit / engine time from HIP events;
`roofline_gram` is the Gram (MFMA). `cpu_baseline` times the CPU oracle
(oracle/rsa_oracle.py, numpy/scipy port of the reference path) on a bounded sample on
this host and extrapolates to the full workload (N=1 only).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

# MIOpen find (NORMAL) + cudnn.benchmark pick the convolution kernels by timing them during
# warm-up: CustomCNN extraction of 10k images 349 -> 239 ms against FAST's heuristic choice
# (scripts/probe_extract.py, profiles/r1_extract_ab.log).
os.environ.setdefault("MIOPEN_FIND_MODE", "NORMAL")
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import numpy as np
import torch
import torch.distributed as dist

torch.backends.cudnn.benchmark = True

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from visreps_amd.dataloaders.synthetic import NSD_ROIS_4, make_images, make_responses, shard_rows
from visreps_amd.models.custom_model import CustomCNN
from visreps_amd.models.utils import FeatureExtractor
from visreps_amd.pipeline import PrefetchedRDMs, StepTimes, all_units_rsa, distributed_rdm, engine_bytes

METRIC = "end-to-end RSA eval sec (extract→RDM→1000-bootstrap Spearman), N=10k stimuli"
LAYERS = ["conv1", "conv2", "conv3", "conv4", "conv5", "fc1", "fc2"]
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP32_MFMA_PEAK_TF = 157.3  # MI355X_MICROARCH.md: FP32 matrix 157.3 TFLOP/s spec
BF16_MFMA_PEAK_TF = 2516.6  # MI355X_MICROARCH.md / SURVEY §8(d): BF16 dense matrix peak


def log(*a):
    print(*a, file=sys.stderr, flush=True)


@torch.no_grad()
def extract(extractor: FeatureExtractor, images: torch.Tensor, batch: int):
    """Flattened points of every local stimulus, written into per-point HBM buffers."""
    n = images.size(0)
    bufs = None
    for b0 in range(0, n, batch):
        feats = extractor(images[b0:b0 + batch])
        if bufs is None:
            bufs = {k: torch.empty((n, v[0].numel()), dtype=torch.float32, device=images.device)
                    for k, v in feats.items()}
        for k, v in feats.items():
            bufs[k][b0:b0 + v.size(0)] = v.reshape(v.size(0), -1)
    return bufs


def pmc_traffic():
    """HBM bytes per unit of the engine from the committed rocprofv3 --pmc passes
    (FETCH_SIZE + WRITE_SIZE over one multi call, scripts/gpu_pmc.sh + pmc_traffic.py).
    Counted in a separate profiler run: a PMC pass cannot share this timed run."""
    path = os.path.join(ROOT, "profiles", "r1_pmc_traffic_v6.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return round(float(d["engine_unit_bytes"])), (
            "profiles/r1_pmc_traffic_v6.json: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate "
            "passes over one 14-unit engine call at N=10k, raw counters (no gfx950 x2 read "
            "correction: the engine's reads are 2-4 B/lane row gathers, not 16 B/lane streams)")
    except (OSError, KeyError, ValueError):
        return None, None


def cpu_baseline(n: int, n_boot: int, dims: dict, voxels: dict, model_rdm: torch.Tensor,
                 neural_rdm: torch.Tensor, images: torch.Tensor, model) -> dict:
    """CPU oracle (numpy/scipy port) on a bounded sample, extrapolated to the workload."""
    from oracle import rsa_oracle as O

    threads = torch.get_num_threads()
    rng = np.random.default_rng(0)
    # (a) Gram throughput of the oracle's compute_rdm at the workload's N, fc1 width
    x = rng.standard_normal((n, 4096), dtype=np.float32)
    t = time.perf_counter()
    O.compute_rdm(x)
    t_gram = time.perf_counter() - t
    gflops = n * (n + 1) * 4096 / t_gram / 1e9
    del x
    # (b) one full-triangle Spearman (scipy) on the GPU-built RDMs
    a = model_rdm.cpu().numpy()
    b = neural_rdm.cpu().numpy()
    t = time.perf_counter()
    O.compute_rdm_correlation(a, b, "Spearman")
    t_sp = time.perf_counter() - t
    # (c) one bootstrap sub-RDM gather pair, as evals.py:365-366
    idx = np.random.RandomState(42).choice(n, int(0.9 * n), replace=False)
    t = time.perf_counter()
    _ = a[idx][:, idx], b[idx][:, idx]
    t_gather = time.perf_counter() - t
    del a, b
    # (d) CPU forward of a 32-image batch
    m_cpu = model.to("cpu").eval()
    xb = images[:32].cpu()
    t = time.perf_counter()
    with torch.no_grad():
        m_cpu(xb)
    t_fwd = (time.perf_counter() - t) / 32
    model.to(images.device)
    k = int(0.9 * n)
    M, Mk = n * (n - 1) / 2, k * (k - 1) / 2
    sp_boot = t_sp * (Mk * math.log(Mk)) / (M * math.log(M))
    units = len(dims) * len(voxels)
    gram_total = sum(n * (n + 1) * d for d in list(dims.values()) + list(voxels.values())) / (gflops * 1e9)
    total = t_fwd * n + gram_total + units * (t_sp + n_boot * (sp_boot + t_gather))
    sample = (f"oracle on this host: compute_rdm N={n} D=4096 ({t_gram:.2f}s, {gflops:.0f} GFLOP/s), "
              f"one N={n} triangle spearmanr ({t_sp:.2f}s), one bootstrap sub-RDM gather pair "
              f"({t_gather:.3f}s), CustomCNN CPU forward ({1 / t_fwd:.0f} img/s); extrapolated to "
              f"{units} units x (1 + {n_boot}) Spearman (M log M scaling to k={k}), "
              f"{len(dims) + len(voxels)} Grams, {n} forwards")
    return {"value": round(total, 1), "unit": "s", "cores": threads, "kind": "port",
            "sample": sample}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=10000)
    ap.add_argument("--boot", type=int, default=1000)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    pg = None
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
        pg = dist.group.WORLD
    N = args.n
    rows = shard_rows(N, rank, world)

    torch.manual_seed(0)  # identical random-init weights on every rank
    model = CustomCNN(num_classes=1000).to(dev).eval()
    extractor = FeatureExtractor(model, LAYERS, extract_pre_and_post=True)
    points = list(extractor.return_nodes)
    images = make_images(rows, device=dev)
    responses = make_responses(images, rows, NSD_ROIS_4)
    torch.cuda.synchronize()

    dims = {}

    def step(times: StepTimes):
        feats = extract(extractor, images, args.batch)
        for p, f in feats.items():
            dims[p] = f.size(1)
        neural = {r: distributed_rdm(y, N, pg, times) for r, y in responses.items()}
        res = all_units_rsa(PrefetchedRDMs(feats, points, N, pg, times), points, neural,
                            N, n_boot=args.boot, seed=42, pg=pg, times=times)
        del feats
        return res, neural

    for w in range(args.warmup):
        t = time.perf_counter()
        step(StepTimes())
        torch.cuda.synchronize()
        log(f"[rank {rank}] warmup {w}: {time.perf_counter() - t:.2f}s")

    if pg is not None:
        dist.barrier()
    torch.cuda.synchronize()
    times = StepTimes()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res, neural = step(times)
    torch.cuda.synchronize()
    if pg is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    times.resolve()
    stats = torch.tensor([elapsed, times.engine_ms, times.engine_bytes, times.gram_ms,
                          times.gram_flops], dtype=torch.float64, device=dev)
    if pg is not None:
        mx = stats.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        elapsed = float(mx[0])
    per_step = elapsed / args.steps

    if rank == 0:
        eng_gbs = times.engine_bytes / (times.engine_ms / 1e3) / 1e9 if times.engine_ms else 0.0
        gram_tf = times.gram_flops / (times.gram_ms / 1e3) / 1e12 if times.gram_ms else 0.0
        units_per_rank = math.ceil(len(points) * len(NSD_ROIS_4) / world)
        per_launch = engine_bytes(N, args.boot)
        traffic, tsrc = pmc_traffic()
        roof = {"bound": "hbm", "achieved": round(eng_gbs, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(eng_gbs / HBM_PEAK_GBS, 4), "traffic": traffic,
                "traffic_source": tsrc,
                "kernel": ("bootstrap engine pass chain (vr_bootstrap_spearman_multi: per pass one "
                           "A-side rank walk of the neural plan + one B-side walk per unit)"),
                "algorithmic_bytes_per_call": per_launch,
                "avg_call_ms": round(times.engine_ms / max(1, times.engine_calls), 3)}
        if traffic:  # bandwidth actually drawn: PMC bytes per unit / measured time per unit
            drawn = traffic / (roof["avg_call_ms"] / 1e3) / 1e9
            roof["traffic_gbs"] = round(drawn, 1)
            roof["traffic_frac"] = round(drawn / HBM_PEAK_GBS, 4)
        if os.environ.get("VISREPS_GRAM") == "fp32":
            gpeak, gkern = FP32_MFMA_PEAK_TF, "k_gram (exact fp32, v_mfma_f32_32x32x2_f32)"
        else:  # 3 bf16 MFMA products per algorithmic FLOP: ceiling = bf16 dense peak / 3
            gpeak = round(BF16_MFMA_PEAK_TF / 3, 1)
            gkern = ("k_gram3 (centred rows split hi+lo bf16, 3 x v_mfma_f32_32x32x16_bf16 "
                     "per k-step, fp32 accumulate; peak = bf16 dense peak / 3)")
        roof_gram = {"bound": "mfma", "achieved": round(gram_tf, 2), "peak": gpeak,
                     "unit": "TFLOP/s", "frac": round(gram_tf / gpeak, 4), "kernel": gkern,
                     "algorithmic_flops": "N(N+1)D per RDM",
                     "ms_per_step": round(times.gram_ms / args.steps, 2)}
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            t = time.perf_counter()
            any_model = distributed_rdm(torch.nn.functional.relu(
                torch.randn(N, 256, device=dev)), N)  # a model-shaped RDM for the sample
            cpu = cpu_baseline(N, args.boot, dims, NSD_ROIS_4, any_model, neural["V1"], images, model)
            log(f"cpu baseline sample took {time.perf_counter() - t:.1f}s")
        first = res[(points[0], "V1")]
        line = {
            "metric": METRIC,
            "value": round(per_step, 4),
            "unit": "s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(per_step * 1e3, 2),
            "higher_is_better": False,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": ("f32 Gram" if os.environ.get("VISREPS_GRAM") == "fp32" else
                      "bf16x3-split Gram, fp32 accumulate (max |dRDM| vs fp64 <= 5e-6)")
                     + " / exact int ranks, fp64 statistic",
            "data": "synthetic (seeded images + NSD-shaped ROI responses; random-init CustomCNN)",
            "config": {"workload": "configs[1]: CustomCNN 14 points x 4 NSD ROIs, N=10k, 1000-bootstrap Spearman RSA",
                       "n_stimuli": N, "points": len(points), "rois": list(NSD_ROIS_4),
                       "units": len(points) * len(NSD_ROIS_4), "n_bootstrap": args.boot,
                       "parallelism": f"stimulus-sharded extraction + block Gram, units/{world} ranks"},
            "roofline": roof,
            "roofline_gram": roof_gram,
            "cpu_baseline": cpu,
            "check": {"unit": f"{points[0]} x V1", "score": first["score"],
                      "ci": [first["ci_low"], first["ci_high"]]},
        }
        print(json.dumps(line), flush=True)
    if pg is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

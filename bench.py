"""Benchmark: end-to-end RSA eval seconds (extract -> RDM -> 1000-bootstrap Spearman).

Workload = BASELINE.json configs[1]: a randomly initialised CustomCNN (the AlexNet-style
network visreps evaluates; 7 layers x pre/post = 14 extraction points) over N = 10,000
synthetic 224x224 stimuli, x 4 NSD-shaped ROIs (V1/V2/V3 = 2000 voxels, hV4 = 1000). One
step = the whole reference eval (visreps/evals.py:222-400):
  * extraction of the 14 points for every stimulus;
  * phase 1 (evals.py:249-287): every point's rows projected by its sparse random
    projection (k = min(4096, D), the bulk extraction's SRP), RandomState(42).choice(N, 1000)
    selection stimuli, 14 + 4 selection RDMs, 56 Spearmans, best point per ROI;
  * phase 2 + scoring (evals.py:302-373), for all 56 (point, ROI) units: 18 RDMs, 18 rank
    plans, point Spearman + 1000 bootstrap subsets of int(0.9 N) stimuli each, the
    RandomState(42) index sets drawn inside the step.
Inputs (images, responses) are resident in HBM before timing starts.

  python bench.py [--gpus N --steps K --warmup W]   (N > 1 under torch.distributed.run)

Rank 0 prints one JSON line. `roofline` is the bootstrap engine (the dominant cost): the
engine's own algorithmic HBM bytes per call (pipeline.engine_call_bytes) / its HIP-event
time; the reference-equivalent rate (both fp32 triangles read once per
Spearman) is reported beside it, not as the fraction. `roofline_gram` is the Gram (MFMA).
`cpu_baseline` runs the CPU oracle (oracle/rsa_oracle.py) to BASELINE.md's plan: configs[0]
in full, and at N = 10k one Gram, the point Spearman and 5 bootstrap Spearmans,
extrapolated linearly to the workload (N=1 only).
"""
from __future__ import annotations

import argparse
import contextlib
import ctypes
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
from visreps_amd._lib import KTIMER_KERNELS, check, ktimer_enable, ktimer_read, lib, stream_of
from visreps_amd.analysis._random import draw_bootstrap_indices
from visreps_amd.pipeline import (KERNELS, PlanPrefetch, ShardedRDMs, StepTimes, all_units_rsa, engine_bytes,
                                  engine_call_bytes, engine_pair_bytes, engine_tri, make_schedule, phase1_rows,
                                  phase1_select)

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


@torch.no_grad()
def extract_split(extractor: FeatureExtractor, images: torch.Tensor, batch: int, keep: np.ndarray,
                  correction: float = 1e-12):
    """bench.extract with the Gram prepass fused in: every batch's hooked outputs are split
    straight into per-point SplitRows (row statistics + bf16 hi/lo records,
    vr_rdm_split_rows_f32) -- no fp32 copy of the features is made -- and only the local
    rows `keep` (phase 1's selection stimuli, pipeline.phase1_rows order) are kept in fp32.
    Returns ({point: SplitRows}, {point: (len(keep), D) fp32 rows})."""
    n, dev = images.size(0), images.device
    K = KERNELS
    out = sel = None
    keep = np.asarray(keep, dtype=np.int64)
    for b0 in range(0, n, batch):
        feats = extractor(images[b0:b0 + batch])
        if out is None:
            out = {k: K.empty_split(n, v[0].numel(), dev) for k, v in feats.items()}
            sel = {k: torch.empty((len(keep), v[0].numel()), dtype=torch.float32, device=dev) for k, v in feats.items()}
        b1 = min(n, b0 + batch)
        at = np.flatnonzero((keep >= b0) & (keep < b1))  # host-side: no device sync per batch
        xs = {k: v.reshape(v.size(0), -1) for k, v in feats.items()}
        # every point of the batch in one launch (rows x points blocks: a batch's rows alone
        # would leave most CUs idle)
        K.split_rows_multi(list(xs.values()), correction, [out[k] for k in xs], b0)
        # the batch's phase-1 selection rows of every point, one launch
        K.gather_rows_multi(list(xs.values()), keep[at] - b0, at, [sel[k] for k in xs])
    return out, sel


def split_mode(n: int, dims: dict) -> bool:
    """The bench Grams all take the bf16 split kernel (n^2 d >= 1e10 for every point, or
    VISREPS_GRAM=split); then extraction writes split rows directly. VISREPS_GRAM=fp32
    keeps fp32 feature buffers for the exact-fp32 kernel."""
    mode = os.environ.get("VISREPS_GRAM")
    if mode == "fp32":
        return False
    return mode == "split" or all(float(n) * n * d >= 1e10 for d in dims.values())


PMC_PROFILE = os.path.join(ROOT, "profiles", "r6_pmc_engine_grid.json")


def pmc_traffic(n: int, est: bool):
    """HBM bytes of the engine from the committed rocprofv3 --pmc passes over the bench's own
    engine path on its RDMs (JOINED=1 GRID=1 scripts/gpu_pmc_engine.sh: shared joins + one
    region-fused grid call, 56 units): FETCH_SIZE x 2 (the gfx950
    correction, MI355X_MICROARCH.md; calibrated for these 128-B row gathers in
    profiles/r2_fetch_calibration.json) + WRITE_SIZE. A PMC pass cannot share this timed
    run, so the figures come from that separate profile -- and only when it was taken on this
    very build (library sha256), at this N and in this engine form; otherwise None."""
    from visreps_amd._lib import build_id

    try:
        with open(PMC_PROFILE) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if (d.get("build_id") != build_id() or int(d.get("n", -1)) != n or bool(d.get("est", True)) != est
            or not d.get("joined", False) or not d.get("grid", False)):
        return None
    return d


def kernel_table(kt: dict, steps: int, est: bool, tri: bool = False, regions: int = 4) -> dict:
    """Per hot kernel over the timed steps (vr_ktimer): ms and launches per step, average
    launch time, and for the engine kernels the algorithmic bytes per launch and GB/s.
    k_rankB_grid (and the full-set pass's launches, which are grid launches when the grid
    runs) count pairs x regions: per (pair, region) the A position 4 + TB row 128 and the
    B codes' 4 shared by the regions."""
    a_b, b_b, j_b = engine_pair_bytes(est, tri)
    grid_b = (engine_pair_bytes(True, tri)[1] - 4) + 4.0 / regions
    bpp = {"k_rankB_est": engine_pair_bytes(True, tri)[1], "k_rankB_full": engine_pair_bytes(True, tri)[1],
           "k_rankB_grid": grid_b,
           "k_rankB_exact": engine_pair_bytes(False)[1],
           "k_rankA": 4 + 128, "k_countA": 4, "k_join": j_b,  # k_rankA: codes 4 + TB row write 128
           "k_full_corr": 4,  # the EST 4 pass: posA stream 4 B per pair (flag words ~1 bit)
           "k_join4": 1}  # k_join4's vr_ktimer units are its algorithmic bytes (codes 4 + 16-B record + 4 per region)
    out = {}
    for k, (ms, n, units) in kt.items():
        e = {"ms_per_step": round(ms / steps, 2), "launches_per_step": round(n / steps, 2),
             "avg_us": round(1e3 * ms / n, 1) if n else None,
             "units_per_launch": units / n if n else 0.0}
        if k in bpp:
            e["bytes_per_launch"] = bpp[k] * units / n if n else 0.0
            e["gbs"] = round(bpp[k] * units / (ms / 1e3) / 1e9, 1) if ms else 0.0
        else:  # Gram kernels: tile FLOPs
            e["tflops"] = round(units / (ms / 1e3) / 1e12, 1) if ms else 0.0
        out[k] = e
    return out


def structured_est_probe(n: int, plan_b, dev) -> dict:
    """EST fallback cost on a strongly structured neural RDM (per-stimulus effects, as real
    fMRI RDMs have: d_ab = u_a + u_b + noise with heavy-tailed u; tests/test_engine_est.py's
    shape) against one of the bench's model plans, N = n, 1000 bootstraps: one unit in the
    default EST form (whatever it re-runs exact) and forced exact. Outside the timed steps."""
    from visreps_amd.analysis import rsa as R
    from visreps_amd.analysis._random import bootstrap_indices

    g = torch.Generator(device=dev).manual_seed(7)
    u = torch.empty(n, device=dev).exponential_(1.0, generator=g) ** 2
    a = u[:, None] + u[None, :] + 0.05 * torch.rand(n, n, device=dev, generator=g)
    a = torch.triu(a, 1)
    a = a + a.T
    plan_a = R.RankPlan(a)
    del a
    idx = bootstrap_indices(42, n, int(0.9 * n), 1000)
    L = lib()
    out = {}
    all_scores = {}
    for form, env in (("est", None), ("exact", "0")):
        old = os.environ.get("VISREPS_ENGINE_EST")
        if env is None:
            os.environ.pop("VISREPS_ENGINE_EST", None)
        else:
            os.environ["VISREPS_ENGINE_EST"] = env
        try:
            R.bootstrap_spearman_multi(plan_a, [plan_b], idx, full_first=True)  # warm
            torch.cuda.synchronize()
            r0, q0 = int(L.vr_engine_est_reruns()), int(L.vr_engine_est_predicted())
            f0 = int(L.vr_engine_est1_fallbacks())
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            sc = R.bootstrap_spearman_multi(plan_a, [plan_b], idx, full_first=True)
            e1.record()
            torch.cuda.synchronize()
            out[form] = {"unit_ms": round(e0.elapsed_time(e1), 2), "reruns": int(L.vr_engine_est_reruns()) - r0,
                         "predicted_off_est3": int(L.vr_engine_est_predicted()) - q0,
                         "est1_fallback": int(L.vr_engine_est1_fallbacks()) - f0, "point": float(sc[0, 0])}
            all_scores[form] = sc.cpu().numpy()
        finally:
            if old is None:
                os.environ.pop("VISREPS_ENGINE_EST", None)
            else:
                os.environ["VISREPS_ENGINE_EST"] = old
    out["passes"] = -(-1001 // 64)
    # every one of the 1001 scores (point + 1000 bootstraps), bit for bit
    out["scores_equal"] = bool(np.array_equal(all_scores["est"], all_scores["exact"]))
    out["scores_compared"] = int(all_scores["est"].size)
    out["note"] = ("neural RDM d_ab = u_a + u_b + 0.05 noise, u ~ Exp(1)^2, vs the V1 neural plan of the bench: "
                   "EST passes the A side flags are re-run exact (est.reruns); a call whose first-pass A counts "
                   "already break the EST 3 window leaves EST 3 before any EST pass (est.predicted_off_est3) and "
                   "runs EST 1, per-lane count tables (est.est1_fallback), its flagged passes exact; "
                   "exact = VISREPS_ENGINE_EST=0")
    return out


FP64_MFMA_PEAK_TF = 78.6  # MI355X spec sheet: FP64 matrix (not in MI355X_MICROARCH.md; confirm on the box)


def kendall_leg(plan_m, plan_n, n: int, n_boot: int) -> dict:
    """compare_method=kendall (rsa.py:22-40, allowed by utils.py:518) on one bench unit
    (the first point x V1 plans, N = n, the RandomState(42) subsets): point + n_boot
    bootstrap tau-a in one call, outside the timed steps. Byte model of the dominant kernel
    k_kwalk (one stream walk of one pass: an inversion level or a tie stream): 4-B pair code
    + 2 bit planes = 4.25 B per pair; it is bound by the window machinery (mask lookups,
    64x64 transposes, bit-parallel pair counts), not HBM, so `frac` is low by construction."""
    from visreps_amd.analysis import rsa as R
    from visreps_amd.analysis._random import bootstrap_indices

    idx = bootstrap_indices(42, n, int(0.9 * n), n_boot)
    R.bootstrap_kendall(plan_m, plan_n, idx[:2], full_first=True)  # warm
    torch.cuda.synchronize()
    ktimer_enable(True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    sc = R.bootstrap_kendall(plan_m, plan_n, idx, full_first=True)
    e1.record()
    torch.cuda.synchronize()
    ms, launches, pairs = ktimer_read("k_kwalk")
    ktimer_enable(False)
    gbs = 4.25 * pairs / (ms / 1e3) / 1e9 if ms else 0.0
    return {"unit_ms": round(e0.elapsed_time(e1), 2), "subsets": int(sc.numel()), "point": float(sc[0]),
            "k_kwalk": {"ms": round(ms, 2), "launches": launches, "avg_us": round(1e3 * ms / max(1, launches), 1),
                        "bytes_model": "4.25 B per pair per walk (pair code 4 + bucket-start and y-bit planes)",
                        "achieved_gbs": round(gbs, 1), "peak_gbs": HBM_PEAK_GBS,
                        "frac": round(gbs / HBM_PEAK_GBS, 4),
                        "bound": "VALU (window transposes + pair counts), not HBM"},
            "note": ("point + bootstrap tau-a of one unit (bench's first point x V1, N=%d, %d subsets of %d), "
                     "HIP events; outside the timed steps" % (n, n_boot, int(0.9 * n)))}


def configs3_leg(dev, dims: dict, n_boot: int) -> dict:
    """BASELINE configs[3] on device-resident synthetic inputs, outside the timed steps:
      * THINGS behavioural RSA (evals.py:95-155 -> compute_rsa, rsa.py:132-281): 1,854
        concepts (20 % selection / 80 % evaluation, RandomState(42).permutation), 14
        concept-mean points of the CustomCNN widths vs a 66-d embedding, layer selection +
        point + n_boot bootstraps;
      * the encoding score's cross-validated ridge (encoding_score.py:47-62, himalaya
        RidgeCV(alphas=logspace(-10, 10, 20), cv=5)) at n = 26,000 (20,800 fit, 5,200
        predicted), p = 4,096, 48 voxels, primal form: six fp64 p x p Grams X^T X on the
        fp64 MFMA (vr_gram64_f32, k_cov), rocSOLVER eigh, fp64 products.
    roofline_gram64: algorithmic FLOPs n p (p + 1) per Gram / k_cov HIP-event time / FP64
    matrix peak (78.6 TF spec)."""
    from visreps_amd.analysis.alignment import AlignmentData
    from visreps_amd.analysis.encoding_score import ridge_cv_predict_primal
    from visreps_amd.analysis.rsa import compute_rsa

    nc = 1854
    g = torch.Generator(device=dev).manual_seed(1854)
    z = torch.randn(nc, 64, device=dev, generator=g)
    acts = {p: torch.relu(z @ (torch.randn(64, d, device=dev, generator=g) / 8)
                          + 2 * torch.randn(nc, d, device=dev, generator=g)) for p, d in dims.items()}
    emb = z @ torch.randn(64, 66, device=dev, generator=g) + torch.randn(nc, 66, device=dev, generator=g)
    perm = np.random.RandomState(42).permutation(nc)
    ns = int(nc * 0.2)
    sel_t = torch.as_tensor(perm[:ns], device=dev)
    ev_t = torch.as_tensor(perm[ns:], device=dev)
    sel = AlignmentData({p: a[sel_t] for p, a in acts.items()}, emb[sel_t])
    ev = AlignmentData({p: a[ev_t] for p, a in acts.items()}, emb[ev_t])
    del acts
    with contextlib.redirect_stdout(sys.stderr):
        compute_rsa({"compare_method": "spearman"}, sel, ev, n_select=None, bootstrap=True, n_bootstrap=8)  # warm
        torch.cuda.synchronize()
        t = time.perf_counter()
        res = compute_rsa({"compare_method": "spearman"}, sel, ev, n_select=None, bootstrap=True,
                          n_bootstrap=n_boot)[0]
        torch.cuda.synchronize()
        t_rsa = time.perf_counter() - t
    del sel, ev
    # ridge at configs[3]'s size (tests/test_encoding.py::test_ridge_cv_full_size_matches_closed_form's data)
    n_fit, n_new, p, v = 20800, 5200, 4096, 48
    g = torch.Generator(device=dev).manual_seed(26000)
    Z = torch.randn(n_fit + n_new, 256, device=dev, generator=g)
    X = Z @ torch.randn(256, p, device=dev, generator=g) + 0.5 * torch.randn(n_fit + n_new, p, device=dev, generator=g)
    X = (X - X.mean(0)) / X.std(0)
    Y = (X @ (torch.randn(p, v, device=dev, generator=g) / 64.0)) * torch.logspace(1, -2, v, device=dev) \
        + torch.randn(n_fit + n_new, v, device=dev, generator=g)
    ridge_cv_predict_primal(X[:2000], Y[:2000], X[n_fit:n_fit + 10])  # warm (solver handles, kernels)
    torch.cuda.synchronize()
    ktimer_enable(True)
    t = time.perf_counter()
    pred, alphas = ridge_cv_predict_primal(X[:n_fit], Y[:n_fit], X[n_fit:])
    torch.cuda.synchronize()
    t_ridge = time.perf_counter() - t
    ms, launches, flops = ktimer_read("k_cov")
    ktimer_enable(False)
    tf = flops / (ms / 1e3) / 1e12 if ms else 0.0
    return {"things_rsa": {"s": round(t_rsa, 3), "concepts": nc, "selection": ns, "evaluation": nc - ns,
                           "points": len(dims), "n_bootstrap": n_boot, "best_layer": res["layer"],
                           "score": res["score"]},
            "ridge": {"s": round(t_ridge, 3), "n_fit": n_fit, "n_new": n_new, "p": p, "voxels": v,
                      "distinct_alphas": int(len(set(np.asarray(alphas).tolist()))), "form": "primal (p < n)"},
            "roofline_gram64": {"bound": "mfma", "kernel": "k_cov (v_mfma_f64_16x16x4_f64, fp64 X^T X tiles)",
                                "achieved": round(tf, 2), "peak": FP64_MFMA_PEAK_TF, "unit": "TFLOP/s",
                                "frac": round(tf / FP64_MFMA_PEAK_TF, 4), "launches": launches,
                                "ms": round(ms, 2), "algorithmic_flops": "n p (p + 1) per Gram (unique i <= j)",
                                "peak_source": "MI355X spec sheet FP64 matrix (not listed in MI355X_MICROARCH.md)"},
            "note": "device-resident synthetic inputs, wall time incl. eigh and host orchestration; outside the timed steps"}


def _free_device(dev):
    from visreps_amd._lib import workspace

    workspace.release()
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()


def _latent_features(dev, n: int, d: int, seed: int, dtype, relu: bool, chunk: int = 8192, zseed: int = 0):
    """Synthetic (n, d) features with shared latent structure (z W / 8 + 2 noise, as
    tests/test_benchsize.py's cfg3 data), generated in row chunks to bound the fp32 temporaries.
    Features made with the same zseed share the stimulus latents z (model vs neural)."""
    z = torch.randn(n, 64, device=dev, generator=torch.Generator(device=dev).manual_seed(zseed))
    g = torch.Generator(device=dev).manual_seed(seed)
    w = torch.randn(64, d, device=dev, generator=g) / 8
    x = torch.empty((n, d), dtype=dtype, device=dev)
    for r0 in range(0, n, chunk):
        r1 = min(n, r0 + chunk)
        t = z[r0:r1] @ w
        t += 2 * torch.randn(r1 - r0, d, device=dev, generator=g)
        if relu:
            t.relu_()
        x[r0:r1] = t.to(dtype)
        del t
    return x


def _rdm_timed(x, reps: int = 1):
    """compute_rdm(x) after one warm call (workspace allocation, kernel load): the HIP-event
    time of the whole call (prepass + Gram + epilogue) and the Gram kernels' own time (vr_ktimer
    k_gram_wide + k_gram_tile), per call."""
    from visreps_amd.analysis import rsa as R

    rdm = R.compute_rdm(x)
    del rdm
    torch.cuda.synchronize()
    ktimer_enable(True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        rdm = R.compute_rdm(x)
    e1.record()
    torch.cuda.synchronize()
    wide_ms, wide_n, _ = ktimer_read("k_gram_wide")
    tile_ms, tile_n, _ = ktimer_read("k_gram_tile")
    ktimer_enable(False)
    return rdm, e0.elapsed_time(e1) / reps, (wide_ms + tile_ms) / reps, (wide_n + tile_n) / reps


def _gram_roof(n: int, d: int, call_ms: float, gram_ms: float, products: int = 3) -> dict:
    flops = float(n) * (n + 1) * d
    split_peak = BF16_MFMA_PEAK_TF / products
    tf_call = flops / (call_ms / 1e3) / 1e12
    tf_gram = flops / (gram_ms / 1e3) / 1e12 if gram_ms else 0.0
    return {"bound": "mfma", "achieved": round(tf_call, 2), "peak": round(split_peak, 1), "unit": "TFLOP/s",
            "frac": round(tf_call / split_peak, 4), "gram_kernels_tflops": round(tf_gram, 2),
            "gram_kernels_frac": round(tf_gram / split_peak, 4),
            "frac_of_bf16_dense_peak": round(tf_call / BF16_MFMA_PEAK_TF, 4),
            "algorithmic_flops": "N(N+1)D per RDM (unique pairs i <= j, 2 FLOP per multiply-add)",
            "peak_note": ("split ceiling = bf16 dense peak 2516.6 / 3: every k-step is 3 bf16 MFMA products "
                          "(hi hi + hi lo + lo hi of the centred fp32 values, as the reference centres in fp32 "
                          "before its matmul, rsa.py:76-90); frac_of_bf16_dense_peak = algorithmic FLOPs / the bf16 dense "
                          "peak itself (MFMA busy = 3 x that)") if products == 3 else
                         ("one product per k (bf16 features: x_i x_j exact in fp32, the centring a rank-1 "
                          "correction in the epilogue): peak = the bf16 dense peak 2516.6")}


def configs4_leg(dev) -> dict:
    """BASELINE configs[4]: bf16 features at N = 50,000 -> compute_rdm (rsa.py:59-93; the
    bf16 entry point vr_rdm_pearson_bf16 widens on the fly, no fp32 copy of the features):
      * ViT-B/16 block output (197 tokens x 768 = D 151,296, the pca_labels_vit dump's block
        hook), 15.1 GB of bf16 features;
      * CLIP ViT-L/14 encode_image embedding, D = 768.
    Synthetic latent-structured bf16 features of those shapes (the forward passes are
    covered by tests/test_benchsize.py::test_cfg5_*); HIP events around compute_rdm after one
    warm call, outside the timed steps."""
    n = 50000
    out = {}
    for name, d, reps in (("vit_b16_block", 151296, 1), ("clip_vit_l14", 768, 5)):
        _free_device(dev)
        x = _latent_features(dev, n, d, seed=d, dtype=torch.bfloat16, relu=False)
        rows = torch.randperm(n, device=dev, generator=torch.Generator(device=dev).manual_seed(3))[:64]
        rdm, call_ms, gram_ms, launches = _rdm_timed(x, reps)  # default: one product per k
        ok = bool(torch.all(torch.diagonal(rdm) == 0)) and bool(torch.isfinite(rdm[:64]).all())
        sample = rdm[rows].clone()
        del rdm
        os.environ["VISREPS_GRAM_ONE"] = "0"  # the split (hi/lo, 3 products) form, for comparison
        try:
            rdm3, call3_ms, gram3_ms, _ = _rdm_timed(x, reps)
        finally:
            os.environ.pop("VISREPS_GRAM_ONE", None)
        diff = float((rdm3[rows] - sample).abs().max())
        del rdm3, x
        e = {"n": n, "d": d, "dtype": "bf16 features (rsa.py:76 widens to fp32): one bf16 product per k, centring "
                                      "as a rank-1 correction in the epilogue",
             "rdm_ms": round(call_ms, 2), "gram_ms": round(gram_ms, 2), "gram_launches": launches,
             "sane": ok, "split_form": {"rdm_ms": round(call3_ms, 2), "gram_ms": round(gram3_ms, 2),
                                        "roofline": _gram_roof(n, d, call3_ms, gram3_ms, 3),
                                        "max_abs_rdm_diff_vs_one_product_64_rows": diff}}
        e["roofline"] = _gram_roof(n, d, call_ms, gram_ms, 1)
        out[name] = e
    _free_device(dev)
    out["note"] = ("one RDM per shape after a warm call; rdm_ms = HIP events around compute_rdm (row statistics "
                   "+ prepass + Gram + epilogue), gram_ms = the Gram kernels alone (vr_ktimer); split_form = the "
                   "same RDM with VISREPS_GRAM_ONE=0 (the round-5 hi/lo kernel); outside the timed steps")
    return out


def configs2_leg(dev) -> dict:
    """BASELINE configs[2] on one GPU (the N = 1 point of its scaling curve): the NSD
    73k-stimulus full RDM -- 73,000 x 43,264 fp32 features (AlexNet conv5 width) -> split-Gram
    compute_rdm (rsa.py:59-93), a 73,000 x 2,000-voxel neural RDM, and the full-triangle
    Spearman of the two (rsa.py:96-129 at 2.66e9 pairs, vr_spearman_full_f32: midranks from
    per-key count tables of each triangle, exact integer dot). Synthetic features; HIP events
    after one warm call; outside the timed steps."""
    from visreps_amd.analysis import rsa as R

    n, d, v = 73000, 43264, 2000
    _free_device(dev)
    x = _latent_features(dev, n, d, seed=7, dtype=torch.float32, relu=True)
    rdm_m, call_ms, gram_ms, launches = _rdm_timed(x)
    del x
    _free_device(dev)
    y = _latent_features(dev, n, v, seed=8, dtype=torch.float32, relu=False)
    rdm_n = R.compute_rdm(y)
    del y
    _free_device(dev)
    R.spearman_full(rdm_m[:4096, :4096], rdm_n[:4096, :4096])  # warm (kernels, small workspace)
    # first full-size call: it also allocates the ~33 GB workspace (the pool keeps it), so its
    # time includes the device allocation; the second call is the kernels' steady state
    sf = []
    for _ in range(2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rho = R.spearman_full(rdm_m, rdm_n)
        e1.record()
        torch.cuda.synchronize()
        sf.append(e0.elapsed_time(e1))
    first_ms, sf_ms = sf
    # the bootstrap beyond the rank plans (rsa.bootstrap_full: evals.py:355-373 at n = 73k, one
    # plan-free sub-RDM Spearman per draw of 0.9 n): a few RandomState(42) draws, timed
    from visreps_amd.analysis._random import bootstrap_indices
    nd = 8
    bidx = torch.from_numpy(bootstrap_indices(42, n, int(0.9 * n), nd).copy()).to(dev)
    R.bootstrap_full(rdm_m, rdm_n, bidx[:1], full_first=False)  # warm (the subset workspace)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    bscores = R.bootstrap_full(rdm_m, rdm_n, bidx, full_first=False)
    e1.record()
    torch.cuda.synchronize()
    boot_ms = e0.elapsed_time(e1) / nd
    del bidx
    from visreps_amd._lib import workspace
    workspace.release("spearman_full")
    # compare_method=kendall on the same pair (rsa.py:22-40 at 2.66e9 elements, beyond the rank
    # plans: vr_kendall_full_f32, dense ranks + inversions one rank bit per level)
    kt = []
    for _ in range(2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        tau = R.compute_rdm_correlation(rdm_m, rdm_n, correlation="Kendall")
        e1.record()
        torch.cuda.synchronize()
        kt.append(e0.elapsed_time(e1))
    workspace.release("kendall_full")
    M = n * (n - 1) // 2
    from visreps_amd._lib import lib as _vlib
    sf_form = ["bucketed count tables", "count tables", "radix sort"][_vlib().vr_spearman_full_last_form()]
    # algorithmic bytes per pair of the bucketed count-table form (both RDMs together): key
    # range 8 (both triangles read), key offsets 8 read + 8 written, B's two keys-only LSD
    # passes 2 x 12, A's two (kA, kB) passes 2 x 20, bucket starts 8, per-key counts 8, dot 8
    # read + one 4-B random read of B's table + A's (cached) 4 -> 120 B per pair. The dot's
    # random table read costs a line each (transaction-, not byte-bound); vs_sort_model
    # restates the time on the round-5 sort pipeline's ~120 B per pair and RDM (the model
    # VERDICT r5 #6 set its 0.45 / 180 ms target on).
    bpp = 120
    gbs = bpp * M / (sf_ms / 1e3) / 1e9
    sort_model = 2 * 120 * M / (sf_ms / 1e3) / 1e9 / HBM_PEAK_GBS
    out = {"n": n, "d": d, "voxels": v, "rdm_ms": round(call_ms, 2), "gram_ms": round(gram_ms, 2),
           "gram_launches": launches, "roofline_gram": _gram_roof(n, d, call_ms, gram_ms),
           "spearman_full": {"ms": round(sf_ms, 2), "first_call_ms": round(first_ms, 2), "pairs": M, "rho": rho,
                             "form": sf_form, "pairs_per_s": round(M / (sf_ms / 1e3), 1),
                             "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                                          "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                                          "algorithmic_bytes_model": "120 B per pair, both RDMs (key range 8, key "
                                          "offsets 16, B radix 2 x 12, A radix 2 x 20, bucket starts 8, counts 8, "
                                          "dot 16 incl. one 4-B random read)",
                                          "vs_sort_model": round(sort_model, 4)}},
           "bootstrap_full": {"ms_per_draw": round(boot_ms, 2), "draws_timed": nd, "subset": int(0.9 * n),
                              "est_1000_draws_s": round(boot_ms, 2),
                              "first_scores": [round(float(v), 8) for v in bscores[:3].tolist()],
                              "note": "rsa.bootstrap_full (n > 65,535: no rank plans): one vr_spearman_full_subset_f32 "
                                      "per RandomState(42) draw on the sub-RDMs read in place; est_1000_draws_s = "
                                      "ms_per_draw x 1000 / 1000"},
           "kendall_full": {"ms": round(kt[1], 2), "first_call_ms": round(kt[0], 2), "pairs": M, "tau_a": tau,
                            "note": "vr_kendall_full_f32 (kendall_full.hip): 2 radix sorts + one inversion level per "
                                    "bit of the y dense rank"},
           "one_gpu_s": round((call_ms + sf_ms) / 1e3, 3),
           "note": ("model RDM (73k x 43,264 split Gram) + full-triangle Spearman vs a 73k x 2,000-voxel neural "
                    "RDM on one GPU; the neural RDM's own build is not in one_gpu_s (it is the same kernel at "
                    "D = 2,000); extraction of 73k images is not included")}
    del rdm_m, rdm_n
    _free_device(dev)
    return out


def _time(fn):
    t = time.perf_counter()
    out = fn()
    return time.perf_counter() - t, out


def cpu_baseline(n: int, n_boot: int, dims: dict, voxels: dict, model, images) -> dict:
    """The CPU oracle (numpy/scipy restatement of the reference path, oracle/rsa_oracle.py)
    timed to BASELINE.md's plan on this host's cores:
      * configs[0] in full: phase 1 (1000 selection stimuli, 14 points at
        k = min(4096, D), one ROI) and one unit at N = 256 (conv5 D = 43,264, V = 2000):
        RDMs, point Spearman, 1000 bootstraps, percentiles;
      * N = 10k: the conv5 Gram (its FLOP rate prices all 18 Grams), the point Spearman
        and 5 bootstrap Spearmans (RandomState(42) draws, sub-RDM gathers included),
        extrapolated linearly to 56 units x 1000 bootstraps; CustomCNN CPU forward of 32
        images, extrapolated to N."""
    from oracle import rsa_oracle as O

    cores = len(os.sched_getaffinity(0))
    threads = max(1, min(cores, int(os.environ.get("OMP_NUM_THREADS", cores))))
    torch.set_num_threads(threads)
    # configs[0] in full
    t0 = time.perf_counter()
    sel = O.synthetic_features(1000, [min(4096, d) for d in dims.values()] + [2000], seed=20260306,
                               relu=[True] * len(dims) + [False])
    rn = O.compute_rdm(sel[-1])
    sc = [O.compute_rdm_correlation(O.compute_rdm(x), rn, "Spearman") for x in sel[:-1]]
    best = int(np.argmax(sc))
    x256, y256 = O.synthetic_features(256, [43264, 2000], seed=7, relu=[True, False])
    O.bootstrap_rsa(O.compute_rdm(x256), O.compute_rdm(y256), n_bootstrap=1000, seed=42)
    t_cfg1 = time.perf_counter() - t0
    del sel, x256, y256
    # N = 10k sample
    x, y = O.synthetic_features(n, [43264, voxels[next(iter(voxels))]], relu=[True, False])
    t_gram, a = _time(lambda: O.compute_rdm(x))
    gflops = n * (n + 1) * x.shape[1] / t_gram / 1e9
    del x
    b = O.compute_rdm(y)
    t_point, _ = _time(lambda: O.compute_rdm_correlation(a, b, "Spearman"))
    rs = np.random.RandomState(42)
    k = int(0.9 * n)
    t_boot = 0.0
    nb = 5
    for _ in range(nb):
        dt, _ = _time(lambda: O.compute_rdm_correlation(*(lambda i: (a[i][:, i], b[i][:, i]))(
            rs.choice(n, k, replace=False)), "Spearman"))
        t_boot += dt
    t_boot /= nb
    del a, b
    m_cpu = model.to("cpu").eval()
    xb = images[:32].cpu()
    with torch.no_grad():
        t_fwd, _ = _time(lambda: m_cpu(xb))
    t_fwd /= 32
    model.to(images.device)
    units = len(dims) * len(voxels)
    gram_total = sum(n * (n + 1) * d for d in list(dims.values()) + list(voxels.values())) / (gflops * 1e9)
    phase1 = t_cfg1  # one ROI's phase 1 + one N=256 unit: a lower bound for 4 ROIs' phase 1
    total = t_fwd * n + gram_total + units * (t_point + n_boot * t_boot) + phase1
    sample = (f"oracle on {threads} host threads ({cores} in the affinity mask): configs[0] run in full "
              f"in {t_cfg1:.1f}s (phase 1: 1000 stimuli x 14 points + one N=256 unit with 1000 "
              f"bootstraps); N={n}: conv5 Gram {t_gram:.1f}s ({gflops:.0f} GFLOP/s), point Spearman "
              f"{t_point:.1f}s, {nb} bootstrap Spearmans {t_boot:.1f}s each (gathers included), "
              f"CustomCNN CPU forward {1 / t_fwd:.0f} img/s; extrapolated linearly to {units} units "
              f"x (1 + {n_boot}) Spearmans, {len(dims) + len(voxels)} Grams, {n} forwards")
    return {"value": round(total, 1), "unit": "s", "cores": threads, "kind": "port", "sample": sample}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", "--stimuli", dest="n", type=int, default=10000)
    ap.add_argument("--boot", type=int, default=1000)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-est-probe", action="store_true")
    ap.add_argument("--no-extra-legs", action="store_true", help="skip the Kendall and configs[2]/[3]/[4] legs")
    ap.add_argument("--no-exact-step", action="store_true", help="skip the exact-form step after the timed steps")
    ap.add_argument("--legs", default="kendall,configs3,configs4,configs2",
                    help="comma list of extra legs (outside the timed steps) to run at N = 1")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; more ranks than GPUs (the gloo rehearsal of the multi-rank path
    # on a one-GPU box) share devices round-robin
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    pg = feat_pg = None
    if world > 1:
        # RCCL (backend "nccl") over xGMI; VISREPS_DIST_BACKEND=gloo only rehearses the
        # orchestration when ranks share a GPU (RCCL refuses two ranks on one device)
        backend = os.environ.get("VISREPS_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        pg = dist.group.WORLD
        # the row exchange to the RDM owners gets its own communicator (ShardedRDMs.start)
        feat_pg = dist.new_group(list(range(world)))
    N = args.n
    rows = shard_rows(N, rank, world)

    torch.manual_seed(0)  # identical random-init weights on every rank
    model = CustomCNN(num_classes=1000).to(dev).eval()
    extractor = FeatureExtractor(model, LAYERS, extract_pre_and_post=True)
    points = list(extractor.return_nodes)
    images = make_images(rows, device=dev)
    responses = make_responses(images, rows, NSD_ROIS_4)
    torch.cuda.synchronize()

    # SRP matrices of the phase-1 projection (sklearn construction, seeded so every rank
    # holds the same ones; the reference fits them once and caches them, so they are built
    # before timing): one per distinct point width
    dims = {}
    with torch.no_grad():
        for p, f in extractor(images[:2]).items():
            dims[p] = f[0].numel()
    from visreps_amd.analysis.sparse_random_projection import SparseProjector, get_srp_transformer

    cache = os.path.join("/tmp", f"visreps_srp_cache_{os.getuid()}")
    proj_by_d = {d: SparseProjector(get_srp_transformer(D=d, k=min(4096, d), density=None, seed=0,
                                                        cache_dir=cache), dev)
                 for d in sorted(set(dims.values()))}
    projectors = {p: proj_by_d[d] for p, d in dims.items()}

    # who computes and who reads every RDM of the step (the same on every rank): owners get
    # the full rows of their RDMs, consumers the packed tiles (pipeline.make_schedule)
    regions = list(NSD_ROIS_4)
    sched = make_schedule(N, dims, points, NSD_ROIS_4, world)

    split = split_mode(N, dims)
    # VISREPS_PLAN_PREFETCH=1: rank plans on a second stream under the Grams. Measured neutral
    # (profiles/r3_bench_ab.log: the Grams' 2 x 245 VGPRs per SIMD leave no room beside them,
    # so the plan kernels only interleave: units -43 ms, Grams +33 ms); off by default.
    prefetch = os.environ.get("VISREPS_PLAN_PREFETCH", "0") == "1"
    plan_stream = torch.cuda.Stream(device=dev) if prefetch else None
    _, _, keep = phase1_rows(N, 1000, 42, rank, world)

    from concurrent.futures import ThreadPoolExecutor

    draw_pool = ThreadPoolExecutor(1)

    def step(times: StepTimes):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
        ev[0].record()
        # this step's bootstrap index sets, drawn on a host thread (the ctypes call releases
        # the GIL) while the GPU extracts; all_units_rsa takes them when its units start
        draw = draw_pool.submit(draw_bootstrap_indices, 42, N, int(0.9 * N), args.boot) if args.boot > 0 else None
        if split:  # the Gram prepass fused into extraction (bench.extract_split)
            feats, sel_rows = extract_split(extractor, images, args.batch, keep)
        else:
            feats, sel_rows = extract(extractor, images, args.batch), None
        ev[1].record()
        rows = {("m", p): feats[p] for p in points}
        rows.update({("n", r): responses[r] for r in regions})
        # N > 1: the row exchanges to the RDM owners start now, on their own communicator,
        # and stream under phase 1
        ex = ShardedRDMs(sched, rows, pg, times, exchange_pg=feat_pg)
        ex.start()
        sel = phase1_select(feats, projectors, responses, points, N, n_select=1000, seed=42,
                            pg=pg, times=times, selected_rows=sel_rows)
        ev[2].record()
        # this rank's RDMs: its pieces' Grams + the exchange of the rest; the rank plans of the
        # RDMs its units read are built on a second stream as each RDM is ready
        pf = PlanPrefetch(dev, sched.needs(rank), plan_stream) if prefetch else None
        rd = ex.finish(on_ready=pf)
        ev[3].record()
        del feats, rows, ex, sel_rows
        neural = {r: rd[("n", r)] for r in regions if ("n", r) in rd}
        res = all_units_rsa(lambda p: rd.pop(("m", p)), points, neural, N, n_boot=args.boot, seed=42, pg=pg,
                            times=times, regions=regions, plans=pf.plans() if pf else None,
                            indices=draw.result if draw is not None else None)
        ev[4].record()
        times.phases(["extract", "phase1", "rdms", "units"], ev)
        return res, neural, sel

    for w in range(args.warmup):
        t = time.perf_counter()
        step(StepTimes())
        torch.cuda.synchronize()
        log(f"[rank {rank}] warmup {w}: {time.perf_counter() - t:.2f}s")

    L = lib()
    if pg is not None:
        dist.barrier()
    torch.cuda.synchronize()
    times = StepTimes()
    reruns0, tails0 = int(L.vr_engine_est_reruns()), int(L.vr_engine_est_tail_flags())
    pred0 = int(L.vr_engine_est_predicted())
    ktimer_enable(True)  # per-launch HIP events on the launch stream of the hot kernels
    check(L.vr_trace_mark(1, 0, ctypes.c_void_p(stream_of(dev))), "vr_trace_mark")
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res, neural, sel = step(times)
    torch.cuda.synchronize()
    if pg is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    check(L.vr_trace_mark(0, 0, ctypes.c_void_p(stream_of(dev))), "vr_trace_mark")
    times.resolve()
    kt = {k: ktimer_read(k) for k in KTIMER_KERNELS}
    ktimer_enable(False)
    est_reruns = int(L.vr_engine_est_reruns()) - reruns0
    est_predicted = int(L.vr_engine_est_predicted()) - pred0
    est_tail_flags = int(L.vr_engine_est_tail_flags()) - tails0
    stats = torch.tensor([elapsed, times.engine_ms, times.engine_bytes, times.gram_ms,
                          times.gram_flops], dtype=torch.float64, device=dev)
    if pg is not None:
        mx = stats.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        elapsed = float(mx[0])
    per_step = elapsed / args.steps

    first_unit = res[(points[0], "V1")]
    # the headline for RDMs whose subsets break the EST window (structured fMRI RDMs go exact
    # up front): one more whole step with every engine pass in the exact chunk-base form
    exact_step = None
    if world == 1 and os.environ.get("VISREPS_ENGINE_EST") != "0" and not args.no_exact_step:
        os.environ["VISREPS_ENGINE_EST"] = "0"
        try:
            torch.cuda.synchronize()
            t = time.perf_counter()
            res_x, _, _ = step(StepTimes())
            torch.cuda.synchronize()
            exact_step = {"s": round(time.perf_counter() - t, 4),
                          "max_abs_diff_vs_est_step": float(max(
                              np.max(np.abs(np.asarray(res_x[u]["bootstrap_scores"] + [res_x[u]["score"]])
                                            - np.asarray(res[u]["bootstrap_scores"] + [res[u]["score"]])))
                              for u in res)),
                          "diff_note": ("the step re-extracts, and the fc GEMMs are not bit-reproducible run to run "
                                        "(4e-7); on the same RDMs the two forms are bit-equal "
                                        "(tests/test_engine_est.py, test_benchsize.py)"),
                          "note": ("one whole configs[1] step (extract -> phase 1 -> RDMs -> 56 units) with "
                                   "VISREPS_ENGINE_EST=0: every engine pass in the exact chunk-base form, the "
                                   "cost on RDMs the EST window cannot serve; after the timed steps, "
                                   "wall clock with synchronize")}
            del res_x
        finally:
            os.environ.pop("VISREPS_ENGINE_EST", None)
    if rank == 0:
        calls = max(1, times.engine_calls)
        unit_ms = times.engine_ms / calls                  # per unit (engine calls cover 14 units)
        eng_gbs = times.engine_bytes / (times.engine_ms / 1e3) / 1e9 if times.engine_ms else 0.0
        ref_gbs = times.engine_ref_bytes / (times.engine_ms / 1e3) / 1e9 if times.engine_ms else 0.0
        gram_tf = times.gram_flops / (times.gram_ms / 1e3) / 1e12 if times.gram_ms else 0.0
        est = os.environ.get("VISREPS_ENGINE_EST") != "0"
        pmc = pmc_traffic(N, est)
        tri = engine_tri(N, est)
        a_b, b_b, j_b = engine_pair_bytes(est, tri)
        kernels = kernel_table(kt, args.steps, est, tri, regions=len(NSD_ROIS_4))
        # `roofline`: the dominant kernel, k_rankB (the B-side rank walk), priced per launch:
        # its algorithmic bytes (pairs walked x B/pair) / its HIP-event launch time
        grid = est and kernels.get("k_rankB_grid", {}).get("launches_per_step", 0) > 0
        rb = kernels["k_rankB_grid" if grid else "k_rankB_est" if est else "k_rankB_exact"]
        rb_pmc = (pmc or {}).get("kernels", {}).get("k_rankB_grid" if grid else "k_rankB")
        roof = {"bound": "hbm", "achieved": rb["gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(rb["gbs"] / HBM_PEAK_GBS, 4),
                "traffic": round(rb_pmc["bytes_per_launch"]) if rb_pmc else None,
                "kernel": (("k_rankB_grid, EST 3 form: B-side rank walk of one model plan for all %d regions "
                            "(one unit per region) over one pass of 64 bootstrap subsets (the full-set pass 0 and "
                            "phase-1 launches are k_rankB_full in kernels_per_step)" % len(NSD_ROIS_4)) if grid else
                           "k_rankB, " + ("EST 5 form (triangle-order TB)" if tri else "EST 3 form" if est
                                          else "exact chunk-base form")
                           + ": B-side rank walk of one unit over one pass of %d bootstrap subsets " % (63 if tri else 64)
                           + "(the full-set pass 0 and phase-1 launches are k_rankB_full in kernels_per_step)"),
                "algorithmic_bytes_per_launch": round(rb["bytes_per_launch"]),
                "algorithmic_bytes_model": ((f"{rb['bytes_per_launch'] / max(rb['units_per_launch'], 1):.0f} B per "
                                             "pair and region: per region A position 4 (stream) + 128 B TB row gather, "
                                             "the B codes' 4 B shared by the regions") if grid else
                                            f"{b_b} B per pair: codes 4 (stream; the row is the pair's triangle "
                                            "index) + 128 B TB row gather (lane 63: the coarse A position)" if tri else
                                            f"{b_b} B per pair: codes 4 + A position 4 (streams"
                                            + (" + window low end 4" if b_b > 136 else "; the window low end is "
                                               "computed from the A position") + ") + 128 B TB row gather" if est else
                                            f"{b_b} B per pair: codes, A position, A chunk 4 each + 128 B TB "
                                            "row gather (the 256-B chunk-base rows are L2-resident)"),
                "pairs_per_launch": round(rb["units_per_launch"]),  # (grid: pairs x regions)
                "launches_per_step": rb["launches_per_step"], "avg_launch_us": rb["avg_us"],
                "timing": "HIP events around every launch on its stream (vr_ktimer), timed steps only",
                "traffic_source": ((f"{os.path.relpath(PMC_PROFILE, ROOT)}: {pmc['source']}; bytes per "
                                    "launch") if rb_pmc else
                                   "null: no PMC profile of this build/N/form (scripts/gpu_pmc_engine.sh)")}
        if rb_pmc:
            roof["traffic_over_algorithmic"] = round(rb_pmc["bytes_per_launch"] / rb["bytes_per_launch"], 3)
        j4 = kernels.get("k_join4")
        roof_join4 = None
        if j4 and j4["launches_per_step"]:
            j4_pmc = (pmc or {}).get("kernels", {}).get("k_join4")
            roof_join4 = {"bound": "hbm", "achieved": j4["gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": round(j4["gbs"] / HBM_PEAK_GBS, 4), "avg_launch_us": j4["avg_us"],
                          "launches_per_step": j4["launches_per_step"],
                          "algorithmic_bytes_per_launch": round(j4["bytes_per_launch"]),
                          "algorithmic_bytes_model": ("per model pair: codes 4 (stream) + the 16-B position "
                                                      "record of the 4 neural plans (random gather) + 4 B written "
                                                      "per region"),
                          "traffic": round(j4_pmc["bytes_per_launch"]) if j4_pmc else None}
            if j4_pmc and j4["avg_us"]:
                # each random 16-B record gather fills a whole 128-B L2 line: the kernel's own
                # line traffic per launch time against HBM peak (profiles/r6_microbench_join.log)
                roof_join4["traffic_rate_frac"] = round(
                    j4_pmc["bytes_per_launch"] / (j4["avg_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
        roof_engine = {"bound": "hbm", "achieved": round(eng_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                       "frac": round(eng_gbs / HBM_PEAK_GBS, 4),
                       "scope": ("whole engine calls (vr_bootstrap_spearman_multi[_joined]: A walks, B walks, "
                                 "tails, per-unit joins) and the shared joins before them (k_posmap4 + k_join4), "
                                 "HIP events around each"),
                       "algorithmic_bytes_per_unit": round(times.engine_bytes / calls),
                       "algorithmic_bytes_model": (f"per pair: A side {a_b} B per pass (count pre-pass codes 4, "
                                                   "rank walk codes 4 + 128 B TB row write; shared by the "
                                                   f"call's units), B walk {b_b} B per pass and unit, join "
                                                   f"{j_b} B per unit, or with shared joins per model pair codes 4 + "
                                                   "16-B record gather + 4 B per region written, and the 16-B "
                                                   "record table built once (pipeline.shared_join_bytes)"),
                       "avg_unit_ms": round(unit_ms, 3),
                       "traffic_per_unit": round(pmc["bytes_per_unit"]) if pmc else None,
                       "reference_equivalent_gbs": round(ref_gbs, 1),
                       "reference_equivalent_note": ("SURVEY §8(d) bytes (both fp32 triangles read once per "
                                                     "Spearman) / the same time: what the reference's "
                                                     "algorithm would have to stream; not a roofline")}
        if os.environ.get("VISREPS_GRAM") == "fp32":
            gpeak, gkern = FP32_MFMA_PEAK_TF, "k_gram (exact fp32, v_mfma_f32_32x32x2_f32)"
        else:  # 3 bf16 MFMA products per algorithmic FLOP: ceiling = bf16 dense peak / 3
            gpeak = round(BF16_MFMA_PEAK_TF / 3, 1)
            gkern = ("k_gram3e / k_gram3 (centred rows split hi+lo bf16 by k_stats_split, 3 x "
                     "bf16 MFMA per k-step -- v_mfma_f32_16x16x32_bf16 in the 256^2 super-tiles, "
                     "32x32x16 in the 128^2 tiles -- fp32 accumulate; peak = bf16 dense peak / 3)")
        gw = kernels["k_gram_wide"]
        roof_gram = {"bound": "mfma", "achieved": round(gram_tf, 2), "peak": gpeak,
                     "unit": "TFLOP/s", "frac": round(gram_tf / gpeak, 4), "kernel": gkern,
                     "algorithmic_flops": "N(N+1)D per RDM (phase-1 selection RDMs included)",
                     "ms_per_step": round(times.gram_ms / args.steps, 2),
                     "wide_kernel": {"name": ("k_gram3p" if os.environ.get("VISREPS_GRAM_KERNEL") == "p" else "k_gram3e") + " (256^2 super-tiles)", "ms_per_step": gw["ms_per_step"],
                                     "tflops_tile": gw["tflops"],
                                     "frac_tile": round(gw["tflops"] / gpeak, 4) if gw["tflops"] else None,
                                     "note": "tile FLOPs 2 d x 256^2 per block (diagonal super-tiles counted whole)"}}
        est_structured = None
        if world == 1 and N <= 65535 and not args.no_est_probe:
            from visreps_amd.analysis.rsa import RankPlan

            t = time.perf_counter()
            est_structured = structured_est_probe(N, RankPlan(neural["V1"]), dev)
            log(f"structured-RDM EST probe took {time.perf_counter() - t:.1f}s: {est_structured}")
        kendall = configs3 = configs4 = configs2 = None
        legs = set() if args.no_extra_legs or world != 1 or N > 65535 else set(args.legs.split(","))
        if "kendall" in legs:
            from visreps_amd.analysis.rsa import RankPlan

            t = time.perf_counter()
            kendall = kendall_leg(RankPlan(neural["V2"]), RankPlan(neural["V1"]), N, args.boot)
            kendall["note"] = kendall["note"].replace("bench's first point x V1", "the V2 x V1 neural RDMs")
            log(f"kendall leg took {time.perf_counter() - t:.1f}s: {kendall}")
        if "configs3" in legs:
            t = time.perf_counter()
            configs3 = configs3_leg(dev, dims, args.boot)
            log(f"configs[3] leg took {time.perf_counter() - t:.1f}s: {configs3}")
        # the big-memory legs run with the step's buffers and the library's scratch released;
        # a failure is reported in the line, not fatal to it
        del res
        for name, fn in (("configs4", configs4_leg), ("configs2", configs2_leg)):
            if name not in legs:
                continue
            t = time.perf_counter()
            try:
                r = fn(dev)
            except Exception as e:  # noqa: BLE001
                r = {"error": f"{type(e).__name__}: {e}"}
                _free_device(dev)
            log(f"{name} leg took {time.perf_counter() - t:.1f}s: {r}")
            if name == "configs4":
                configs4 = r
            else:
                configs2 = r
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            t = time.perf_counter()
            cpu = cpu_baseline(N, args.boot, dims, NSD_ROIS_4, model, images)
            log(f"cpu baseline sample took {time.perf_counter() - t:.1f}s")
        first = first_unit
        best = {r: b for r, (b, _) in sel.items()}
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
                      "bf16x3-split Gram, fp32 accumulate (|dSpearman| < 1e-5 vs fp64 RDMs: tests/test_benchsize.py)")
                     + " / exact int ranks, fp64 statistic",
            "data": "synthetic (seeded images + NSD-shaped ROI responses; random-init CustomCNN)",
            "config": {"workload": "configs[1]: CustomCNN 14 points x 4 NSD ROIs, N=10k, 1000-bootstrap Spearman RSA",
                       "n_stimuli": N, "points": len(points), "rois": list(NSD_ROIS_4),
                       "units": len(points) * len(NSD_ROIS_4), "n_bootstrap": args.boot,
                       "phase1": ("SRP k=min(4096,D) of every point for the 1000 selection stimuli (row-wise, so equal to "
                                  "projecting every row and selecting, as the reference does), selection RDMs, "
                                  "14x4 Spearmans"),
                       "index_draws": "RandomState(42) 1000 x choice(N, 0.9N) drawn inside every step",
                       "inputs": ("ImageNet-normalised 224x224 float32 images already resident in HBM: the "
                                  "get_transform leg (Resize/CenterCrop/Normalize, vr_transform_u8) and the "
                                  "DataLoader's per-batch H2D copy (visreps/models/utils.py:338) are outside "
                                  "the timed step"),
                       "parallelism": (f"stimulus-sharded extraction; RDMs by owner ranks (rows all_to_all to the "
                                       f"owners, packed tiles to the consumers); units/{world} ranks")},
            "roofline": roof,
            "roofline_engine": roof_engine,
            "roofline_gram": roof_gram,
            "roofline_join4": roof_join4,
            "kernels_per_step": {k: v for k, v in kernels.items() if v["launches_per_step"]},
            "est_reruns": est_reruns,
            "est_predicted_off_est3": est_predicted,
            "est_tail_flags": est_tail_flags,
            "est_structured": est_structured,
            "exact_form_step_s": exact_step,
            "kendall_unit": kendall,
            "configs3": configs3,
            "configs4": configs4,
            "configs2_1gpu": configs2,
            "timed_region": ("bracketed by k_trace_mark_begin / k_trace_mark_end dispatches (vr_trace_mark): "
                             "scripts/check_timed_kernels.py lists the kernels between them in a rocprofv3 "
                             "trace (profiles/r3_timed_kernels.json)"),
            "breakdown_ms_per_step": dict(
                {k: round(v / args.steps, 1) for k, v in times.phase_ms.items()},
                engine=round(times.engine_ms / args.steps, 1), gram=round(times.gram_ms / args.steps, 1),
                note=("HIP events on rank 0's compute stream; rdms = all Grams (model + neural) + exchanges, "
                      "units = plans + engine")),
            "cpu_baseline": cpu,
            "check": {"unit": f"{points[0]} x V1", "score": first["score"],
                      "ci": [first["ci_low"], first["ci_high"]], "phase1_best": best},
        }
        print(json.dumps(line), file=_STDOUT, flush=True)
    if pg is not None:
        dist.destroy_process_group()


_STDOUT = sys.stdout

if __name__ == "__main__":
    # the contract's one JSON line is the only stdout output: progress and library prints
    # (the SRP fitter's console lines) go to stderr
    with contextlib.redirect_stdout(sys.stderr):
        main()

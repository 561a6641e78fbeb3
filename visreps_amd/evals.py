"""`--mode eval` for the RSA hot path (reference: visreps/evals.py).

eval(cfg) -> pandas.DataFrame with the reference's result records
    {layer, compare_method, score, ci_low, ci_high, analysis, layer_selection_scores
     [, bootstrap_scores]}                                           (evals.py:380-392)

_eval_rsa mirrors evals.py:209-398 step for step:
  phase 1  per (region, subject): RandomState(42).choice(n_train, n_select) over the
           string-ordered train rows, neural RDM, one RDM + Spearman per SRP'd point,
           best = first strict maximum                                  (:249-287)
  phase 2  each unique best layer re-extracted without SRP on the int-sorted shared test
           IDs -> model RDM                                             (:302-323)
  scoring  neural test RDM, point Spearman, and with bootstrap=True a fresh
           RandomState(42) per (region, subject), 1000 x choice(n, int(0.9 n)) sub-RDM
           Spearmans and 2.5/97.5 linear percentiles                    (:333-373)
Every RDM is built by the HIP Gram kernel and every Spearman / bootstrap runs in the
rank-plan engine (one plan per RDM, reused across its units); there is no CPU path.

Datasets: neural_dataset="synthetic" runs end to end on the NSD-shaped synthetic source
(dataloaders/neural.py). nsd / tvsd / things-behavior / nsd_synthetic need the
reference's on-disk data, which this build does not read; they raise.
analysis="encoding_score" is out of scope and raises.
"""
from __future__ import annotations

import json
import os
from typing import Dict, List

import numpy as np
import pandas as pd
import torch

from .analysis.alignment import (_align_stimulus_level, compute_traintest_alignment,
                                 prepare_traintest_alignment)
from .analysis.rsa import RankPlan, bootstrap_rsa, compute_rdm, compute_rdm_correlation
from .analysis._random import LegacyRandomState
from .dataloaders.neural import _make_loader, load_synthetic_data
from .models import utils as mutils
from .utils import Config, get_seed_letter, rprint, save_results

__all__ = ["eval", "_eval_rsa"]


def _load_cfg(cfg):
    """Merge the training config of a checkpoint run under the runtime cfg (evals.py:31-41)."""
    path = f"{cfg.checkpoint_dir}/cfg{cfg.cfg_id}{get_seed_letter(cfg.seed)}/config.json"
    if not os.path.exists(path):
        if cfg.get("random_init", False):
            cfg.epoch = cfg.get("epoch", 0)
            return cfg
        raise FileNotFoundError(f"training config not found: {path}")
    with open(path) as f:
        base = Config(json.load(f))
    base.epoch = int(str(cfg.checkpoint_model).split("_")[-1].split(".")[0])
    for k in ("mode", "exp_name", "lr_scheduler", "n_classes"):
        base.pop(k, None)
    return base.merge(cfg)


def _listify(val) -> List:
    return list(val) if isinstance(val, (list, tuple)) else [val]


def eval(cfg):  # noqa: A001  (reference name)
    """Unified evaluation entry point (evals.py:67-206) for the RSA path."""
    verbose = cfg.get("verbose", False)
    if cfg.load_model_from == "checkpoint":
        cfg = _load_cfg(cfg)
    elif cfg.load_model_from == "torchvision":
        cfg.epoch = -1
        cfg.cfg_id = "pretrained" if cfg.get("pretrained_dataset") == "imagenet1k" else "untrained"
        cfg.return_nodes = mutils.TORCHVISION_RETURN_NODES[cfg.model_name]
    if not torch.cuda.is_available():
        raise RuntimeError("visreps_amd eval needs a HIP (MI355X) device")
    dev = torch.device("cuda", torch.cuda.current_device())

    dataset = str(cfg.neural_dataset).lower()
    if dataset != "synthetic":
        raise NotImplementedError(
            f"neural_dataset='{dataset}' reads the reference's on-disk data, which this build "
            "does not ship; use neural_dataset='synthetic' (NSD-shaped) or supply the arrays "
            "to visreps_amd.evals._eval_rsa directly")
    analysis = str(cfg.get("analysis", "rsa")).lower()
    if analysis not in ("rsa", "encoding_score"):
        raise ValueError(f"Unknown analysis method: {analysis}")

    subjects = _listify(cfg.subject_idx)
    regions = _listify(cfg.region)
    letter = get_seed_letter(cfg.seed) if isinstance(cfg.seed, int) else "?"
    rprint(
        f"\n  RSA eval | cfg{cfg.get('cfg_id', '?')}{letter} epoch {cfg.get('epoch', '?')} | "
        f"{dataset.upper()} | {len(subjects)} subjects x {len(regions)} regions | seed {cfg.seed}\n",
        style="info",
    )
    model = mutils.load_model(cfg, dev, verbose=verbose)
    model = mutils.configure_feature_extractor(cfg, model, verbose=verbose)

    all_data = load_synthetic_data(cfg, subjects, regions)
    stimuli = all_data["stimuli"]
    rprint(f"  {len(subjects)} subjects x {len(regions)} regions, {len(stimuli)} stimuli, "
           f"{len(all_data['shared_test_ids'])} shared test IDs", style="success")

    dl = _make_loader(stimuli, None, cfg.get("batchsize", 128), cfg.get("num_workers", 0))
    acts, ids = mutils.get_activations(model, dl, dev, keep_on_device=True,
                                       srp_seed=cfg.get("srp_seed"),
                                       srp_cache_dir=cfg.get("srp_cache_dir", "model_checkpoints/srp_cache"))
    rprint("  Activations extracted once for all subjects/regions", style="success")
    del dl
    if analysis == "encoding_score":
        results = _eval_encoding(cfg, model, acts, ids, all_data, subjects, regions, verbose)
    else:
        results = _eval_rsa(cfg, model, acts, ids, all_data, subjects, regions, dev, verbose)
    torch.cuda.empty_cache()
    return results


def _eval_rsa(cfg, model, acts, ids, all_data, subjects, regions, dev, verbose):
    """Two-phase RSA (evals.py:209-398)."""
    method = str(cfg.get("compare_method", "spearman")).lower()
    bootstrap = cfg.get("bootstrap", False)
    n_bootstrap = int(cfg.get("n_bootstrap", 1000))
    n_select = cfg.get("n_select", 1000)
    neural = all_data["neural"]
    shared_test_ids = all_data["shared_test_ids"]
    stimuli = all_data["stimuli"]

    # ---- phase 1: per-(region, subject) layer selection on SRP activations
    rprint("\n  Phase 1: Per-subject layer selection", style="info")
    per_region_layers: Dict = {}
    per_region_scores: Dict = {}
    for region in regions:
        per_region_layers[region], per_region_scores[region] = {}, {}
        for subj in subjects:
            train_acts, train_neural, _ = _align_stimulus_level(acts, neural[region][subj]["train"], ids)
            n_train_subj = train_neural.size(0)
            if n_select is not None and n_select < n_train_subj:
                sel_idx = LegacyRandomState(42).choice(n_train_subj, int(n_select), replace=False)
            else:
                sel_idx = np.arange(n_train_subj)
            sel_t = torch.as_tensor(sel_idx, dtype=torch.long)
            neural_rdm_sel = compute_rdm(train_neural.to(dev)[sel_t.to(dev)])
            plan_sel = RankPlan(neural_rdm_sel)
            best_layer, best_score, subj_scores = None, -float("inf"), []
            for layer, layer_acts in train_acts.items():
                rows = layer_acts[sel_t.to(layer_acts.device)]
                flat = rows.flatten(start_dim=1) if rows.ndim > 2 else rows
                layer_rdm = compute_rdm(flat)
                score = _compare(layer_rdm, neural_rdm_sel, plan_sel, method)
                subj_scores.append({"layer": layer, "score": score})
                if score > best_score:
                    best_score, best_layer = score, layer
            per_region_layers[region][subj] = best_layer
            per_region_scores[region][subj] = subj_scores
            if verbose:
                rprint(f"    {region} subj {subj}: {best_layer} ({best_score:.4f}), "
                       f"{len(sel_idx)} stimuli for selection", style="info")
            del train_acts, train_neural
    del acts
    torch.cuda.empty_cache()
    rprint("  Freed bulk SRP activations", style="success")

    # ---- phase 2: exact re-extraction of each unique best layer on the test stimuli
    rprint("\n  Phase 2: Test evaluation", style="info")
    test_stimuli = stimuli.subset([sid for sid in shared_test_ids if sid in stimuli])
    dl_test = _make_loader(test_stimuli, None, cfg.get("batchsize", 128), cfg.get("num_workers", 0))
    rprint(f"  Test dataloader: {len(test_stimuli)} stimuli", style="success")
    unique_layers = sorted({l for rl in per_region_layers.values() for l in rl.values()})
    model_rdms, model_plans = {}, {}
    for layer in unique_layers:
        rprint(f"  Re-extracting {layer} without SRP...", style="info")
        exact, _ = mutils.extract_single_layer(model, dl_test, dev, layer, shared_test_ids,
                                               keep_on_device=True)
        flat = exact.flatten(start_dim=1) if exact.ndim > 2 else exact
        model_rdms[layer] = compute_rdm(flat)
        del exact, flat
    del model, dl_test
    torch.cuda.empty_cache()

    # ---- per-(region, subject) scoring
    all_results = []
    for region in regions:
        rprint(f"\n  -- Region: {region} --", style="info")
        for subj in subjects:
            best_layer = per_region_layers[region][subj]
            test_neural = neural[region][subj]["test"]
            responses = [test_neural[sid] for sid in shared_test_ids if sid in test_neural]
            neural_tensor = torch.as_tensor(np.stack(responses).squeeze(), dtype=torch.float32)
            neural_rdm = compute_rdm(neural_tensor.to(dev))
            ci_low = ci_high = None
            boot_list = None
            if bootstrap and method in ("spearman", "kendall"):
                if best_layer not in model_plans:
                    model_plans[best_layer] = RankPlan(model_rdms[best_layer])
                point, scores, ci_low, ci_high = bootstrap_rsa(
                    model_plans[best_layer], RankPlan(neural_rdm), n_bootstrap=n_bootstrap, seed=42,
                    method=method)
                boot_list = scores.tolist()
            else:
                point = compute_rdm_correlation(model_rdms[best_layer], neural_rdm,
                                                correlation=method.capitalize())
                if bootstrap:  # the valid compare methods (utils.py) all have an engine
                    raise NotImplementedError(f"bootstrap with compare_method='{method}'")
            msg = f"    subj {subj} | {method.capitalize():<10}| {best_layer} = {point:.4f}"
            if bootstrap:
                msg += f"  [95% CI: {ci_low:.4f}, {ci_high:.4f}]"
            rprint(msg, style="highlight")
            result = {
                "layer": best_layer,
                "compare_method": method,
                "score": point,
                "ci_low": ci_low,
                "ci_high": ci_high,
                "analysis": "rsa",
                "layer_selection_scores": per_region_scores[region][subj],
            }
            if boot_list is not None:
                result["bootstrap_scores"] = boot_list
            if cfg.get("log_expdata"):
                save_results(pd.DataFrame([result]), cfg.merge({"subject_idx": subj, "region": region}))
            all_results.append(result)
    return pd.DataFrame(all_results)


def _compare(layer_rdm, neural_rdm, neural_plan, method: str) -> float:
    """Phase-1 comparison; Spearman reuses the neural RDM's rank plan across points."""
    if method in ("spearman", "kendall"):
        return float(bootstrap_rsa(RankPlan(layer_rdm), neural_plan, n_bootstrap=0, method=method)[0])
    return compute_rdm_correlation(layer_rdm, neural_rdm, correlation=method.capitalize())


def _eval_encoding(cfg, model, acts, ids, all_data, subjects, regions, verbose):
    """Per-(region, subject) encoding score on the SRP activations (evals.py:551-591):
    train/test alignment, then compute_traintest_alignment -> compute_encoding_score."""
    neural = all_data["neural"]
    all_results: List[dict] = []
    for region in regions:
        rprint(f"\n  -- Region: {region} --", style="info")
        for subj in subjects:
            train_data, test_data = prepare_traintest_alignment(cfg, acts, neural[region][subj], ids)
            scores = compute_traintest_alignment(cfg, train_data, test_data, verbose=verbose)
            del train_data, test_data
            if cfg.get("log_expdata"):
                save_results(pd.DataFrame(scores), cfg.merge({"subject_idx": subj, "region": region}))
            all_results.extend(scores)
    del acts, model
    torch.cuda.empty_cache()
    return pd.DataFrame(all_results)

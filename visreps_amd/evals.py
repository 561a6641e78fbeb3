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

Datasets (no on-disk data exists offline; every source is a seeded
synthetic stand-in with the reference's data contract):
  synthetic / nsd   NSD-shaped stimuli and per-subject responses (dataloaders/neural.py)
  tvsd              TVSD-shaped: V1/V4/IT MUA of 2 monkeys, ~22k train + 100 test THINGS
                    images per subject, string-sorted shared test IDs (evals.py:189-190)
  things-behavior   THINGS-shaped concepts x 66-d embeddings, images per concept; 80/20
                    concept split by RandomState(42).permutation, layer selection on 20 %,
                    re-extraction without SRP + concept averaging for the 80 % (:95-155)
  nsd_synthetic     220 test stimuli, best layers looked up in results.db from the NSD
                    run with the same identity (_lookup_nsd_best_layers, :404-548)
analysis="encoding_score" runs compute_traintest_alignment -> compute_encoding_score on
the SRP activations (:551-591); its ridge follows himalaya's published RidgeCV (parity
unpinned: himalaya is not installed).
reconstruct_from_pcs=True replaces every re-extracted layer by its rank-pca_k PCA
reconstruction (analysis/reconstruct_from_pcs.py) before the RDM, as the reference does.
"""
from __future__ import annotations

import json
import os
from typing import Dict, List

import numpy as np
import pandas as pd
import torch

import sqlite3

from .analysis.alignment import (AlignmentData, _align_stimulus_level, compute_traintest_alignment,
                                 prepare_concept_alignment, prepare_traintest_alignment)
from .analysis.reconstruct_from_pcs import reconstruct_from_pcs
from .analysis.rsa import (RankPlan, _concept_average_exact, bootstrap_rsa, compute_rdm,
                           compute_rdm_correlation)
from .analysis._random import LegacyRandomState
from .dataloaders.neural import (_make_loader, load_nsd_synthetic_test_data, load_synthetic_data,
                                 load_things_synthetic, load_tvsd_synthetic)
from .models import utils as mutils
from . import utils as U
from .utils import Config, get_seed_letter, rprint, save_results

__all__ = ["eval", "_eval_rsa", "_eval_things", "_eval_rsa_nsd_synthetic", "_lookup_nsd_best_layers"]


def _load_cfg(cfg):
    """Merge the training config of a checkpoint run under the runtime cfg (evals.py:31-41)."""
    path = f"{cfg.checkpoint_dir}/cfg{cfg.cfg_id}{get_seed_letter(cfg.seed)}/config.json"
    if not os.path.exists(path):
        if cfg.get("random_init", False):  # no training run: its config fields default
            cfg.epoch = cfg.get("epoch", 0)
            cfg.model_name = cfg.get("model_name") or "CustomCNN"
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
    analysis = str(cfg.get("analysis", "rsa")).lower()
    if analysis not in ("rsa", "encoding_score"):
        raise ValueError(f"Unknown analysis method: {analysis}")
    if dataset == "things-behavior":
        return _eval_things(cfg, dev, verbose)
    if dataset == "nsd_synthetic":
        subjects, regions = _listify(cfg.subject_idx), _listify(cfg.region)
        letter = get_seed_letter(cfg.seed) if isinstance(cfg.seed, int) else "?"
        rprint(f"\n  RSA eval (NSD Synthetic) | cfg{cfg.get('cfg_id', '?')}{letter} "
               f"epoch {cfg.get('epoch', '?')} | {len(subjects)} subjects x {len(regions)} regions | "
               f"seed {cfg.seed}\n", style="info")
        return _eval_rsa_nsd_synthetic(cfg, subjects, regions, dev, verbose)
    if dataset not in ("synthetic", "nsd", "tvsd"):
        raise NotImplementedError(
            f"neural_dataset='{dataset}' reads the reference's on-disk data, which this build "
            "does not ship; 'synthetic'/'nsd' (NSD-shaped), 'tvsd' (TVSD-shaped), "
            "'things-behavior' and 'nsd_synthetic' run on seeded synthetic stand-ins")

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

    if dataset == "tvsd":  # evals.py:189-190: the same two-phase path on TVSD's contract
        all_data = load_tvsd_synthetic(cfg, subjects, regions)
    else:
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
    unique_layers = {l for rl in per_region_layers.values() for l in rl.values()}
    model_rdms = _extract_model_rdms(cfg, model, dl_test, dev, unique_layers, shared_test_ids)
    model_plans: Dict = {}
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
            result = _score(best_layer, model_rdms, model_plans, neural_rdm, method, bootstrap,
                            n_bootstrap, subj, per_region_scores[region][subj])
            if cfg.get("log_expdata"):
                save_results(pd.DataFrame([result]), cfg.merge({"subject_idx": subj, "region": region}))
            all_results.append(result)
    return pd.DataFrame(all_results)


def _score(best_layer, model_rdms, model_plans, neural_rdm, method, bootstrap, n_bootstrap, subj,
           selection_scores) -> dict:
    """Point estimate + optional bootstrap of one (region, subject) (evals.py:346-392):
    the model RDM's rank plan is built once per layer and reused across subjects."""
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
        "layer_selection_scores": selection_scores,
    }
    if boot_list is not None:
        result["bootstrap_scores"] = boot_list
    return result


def _extract_model_rdms(cfg, model, dl, dev, layers, ids) -> Dict[str, torch.Tensor]:
    """Each layer re-extracted without SRP (rows in `ids` order), optionally replaced by
    its rank-pca_k PCA reconstruction, -> model RDM (evals.py:312-323, :474-484)."""
    rdms = {}
    for layer in sorted(layers):
        rprint(f"  Extracting {layer} without SRP...", style="info")
        exact, _ = mutils.extract_single_layer(model, dl, dev, layer, ids, keep_on_device=True)
        if cfg.get("reconstruct_from_pcs"):
            exact = reconstruct_from_pcs({layer: exact}, cfg.get("pca_k", 1))[layer]
        rdms[layer] = compute_rdm(exact.flatten(start_dim=1) if exact.ndim > 2 else exact)
        del exact
    return rdms


def _eval_things(cfg, dev, verbose):
    """THINGS-behaviour: 80/20 concept-level train/test RSA (evals.py:95-155). Concept-mean
    SRP activations, a RandomState(42) permutation of the concepts, 20 % for layer
    selection and 80 % for evaluation; the best layer is re-extracted without SRP for
    every image and concept-averaged for the evaluation concepts."""
    model = mutils.load_model(cfg, dev, verbose=verbose)
    model = mutils.configure_feature_extractor(cfg, model, verbose=verbose)
    neural_data, stimuli = load_things_synthetic(cfg)
    rprint("  THINGS data loaded", style="success")
    dl = _make_loader(stimuli, None, cfg.get("batchsize", 128), cfg.get("num_workers", 0))
    acts, ids = mutils.get_activations(model, dl, dev, keep_on_device=True,
                                       srp_seed=cfg.get("srp_seed"),
                                       srp_cache_dir=cfg.get("srp_cache_dir", "model_checkpoints/srp_cache"))
    all_concepts = prepare_concept_alignment(cfg, acts, neural_data, ids)
    del acts, neural_data, ids
    torch.cuda.empty_cache()

    perm = LegacyRandomState(42).permutation(all_concepts.neural.size(0))
    n_sel = int(all_concepts.neural.size(0) * 0.2)
    sel_idx, eval_idx = perm[:n_sel], perm[n_sel:]

    def rows(a, idx):
        return a[torch.as_tensor(idx, dtype=torch.long, device=a.device)]

    sids = all_concepts.stimulus_ids
    selection = AlignmentData(
        activations={l: rows(a, sel_idx) for l, a in all_concepts.activations.items()},
        neural=rows(all_concepts.neural, sel_idx),
        stimulus_ids=[sids[i] for i in sel_idx],
    )
    evaluation = AlignmentData(
        activations={l: rows(a, eval_idx) for l, a in all_concepts.activations.items()},
        neural=rows(all_concepts.neural, eval_idx),
        stimulus_ids=[sids[i] for i in eval_idx],
        concept_image_ids={sids[i]: all_concepts.concept_image_ids[sids[i]] for i in eval_idx},
    )
    del all_concepts
    rprint(f"  {n_sel} selection concepts, {len(eval_idx)} evaluation concepts", style="success")

    def re_extract_fn(layer, stimulus_ids=None):  # noqa: ARG001  (reference signature)
        raw_acts, raw_ids = mutils.extract_single_layer(model, dl, dev, layer, keep_on_device=True)
        if cfg.get("reconstruct_from_pcs"):
            raw_acts = reconstruct_from_pcs({layer: raw_acts}, cfg.pca_k)[layer]
            rprint(f"    Reconstructed from {cfg.pca_k} PCs", style="info")
        return _concept_average_exact(raw_acts, raw_ids, evaluation), evaluation.stimulus_ids

    scores = compute_traintest_alignment(cfg, selection, evaluation, verbose=verbose,
                                         re_extract_fn=re_extract_fn)
    del model, dl
    torch.cuda.empty_cache()
    results = pd.DataFrame(scores)
    if cfg.get("log_expdata"):
        save_results(results, cfg)
    return results


def _lookup_nsd_best_layers(cfg, subjects, regions) -> Dict:
    """Best RSA layer per (region, subject) from the NSD eval with the same identity, read
    from results.db by its run_id (evals.py:404-439)."""
    method = str(cfg.get("compare_method", "spearman")).lower()
    conn = sqlite3.connect(str(U._RESULTS_DB_PATH))
    layers: Dict = {}
    try:
        for region in regions:
            layers[region] = {}
            for subj in subjects:
                nsd_cfg = cfg.merge({"neural_dataset": "nsd", "analysis": "rsa", "subject_idx": subj,
                                     "region": region, "compare_method": method})
                run_id = U._compute_run_id(nsd_cfg)
                try:
                    row = pd.read_sql_query("SELECT layer FROM results WHERE run_id=? AND compare_method=?",
                                            conn, params=(run_id, method))
                except pd.errors.DatabaseError:
                    row = pd.DataFrame()
                if row.empty:
                    raise ValueError(
                        f"No NSD RSA result found (run_id={run_id}) for seed={cfg.seed}, "
                        f"region={region}, subj={subj}, cfg_id={cfg.get('cfg_id')}. Run NSD eval first.")
                layers[region][subj] = row.iloc[0]["layer"]
    finally:
        conn.close()
    return layers


def _eval_rsa_nsd_synthetic(cfg, subjects, regions, dev, verbose):
    """NSD Synthetic (evals.py:442-548): best layers reused from the NSD eval, extracted
    without SRP on the synthetic test stimuli, scored per (region, subject)."""
    method = str(cfg.get("compare_method", "spearman")).lower()
    bootstrap = cfg.get("bootstrap", False)
    n_bootstrap = int(cfg.get("n_bootstrap", 1000))
    best_layers = _lookup_nsd_best_layers(cfg, subjects, regions)
    if verbose:
        for region in regions:
            for subj in subjects:
                rprint(f"    {region} subj {subj}: reusing layer {best_layers[region][subj]} from NSD",
                       style="info")
    test_data = load_nsd_synthetic_test_data(cfg, subjects=subjects, regions=regions)
    test_ids, neural = test_data["test_ids"], test_data["neural"]
    rprint(f"  Loaded {len(test_ids)} synthetic test stimuli", style="success")
    model = mutils.load_model(cfg, dev, verbose=verbose)
    model = mutils.configure_feature_extractor(cfg, model, verbose=verbose)
    dl_test = _make_loader(test_data["stimuli"], None, cfg.get("batchsize", 128), cfg.get("num_workers", 0))
    unique_layers = {l for rl in best_layers.values() for l in rl.values()}
    model_rdms = _extract_model_rdms(cfg, model, dl_test, dev, unique_layers, test_ids)
    del model, dl_test
    torch.cuda.empty_cache()
    model_plans: Dict = {}
    all_results = []
    for region in regions:
        rprint(f"\n  -- Region: {region} --", style="info")
        for subj in subjects:
            best_layer = best_layers[region][subj]
            responses = [neural[region][subj][sid] for sid in test_ids]
            neural_rdm = compute_rdm(torch.as_tensor(np.stack(responses).squeeze(), dtype=torch.float32).to(dev))
            result = _score(best_layer, model_rdms, model_plans, neural_rdm, method, bootstrap,
                            n_bootstrap, subj, [])
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

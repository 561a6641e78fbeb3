"""Stimulus alignment containers (reference: visreps/analysis/alignment.py).

AlignmentData and the stimulus-ID join fix the row order every RDM is built in
(alignment.py:23-39), so they are mirrored exactly; the encoding-score dispatch is out
of scope for this build (OUT) and raises.
"""
from __future__ import annotations

import logging
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch

from .rsa import compute_rsa

logger = logging.getLogger(__name__)

__all__ = [
    "AlignmentData",
    "_align_stimulus_level",
    "prepare_traintest_alignment",
    "compute_traintest_alignment",
    "prepare_concept_alignment",
]


@dataclass
class AlignmentData:
    """Activations and neural data for one split (alignment.py:14-20)."""

    activations: Dict[str, torch.Tensor]
    neural: torch.Tensor
    stimulus_ids: Optional[List[str]] = None
    concept_image_ids: Optional[Dict[str, List[str]]] = None


def _align_stimulus_level(acts_raw, targets, keys):
    """Rows of acts_raw whose key is in targets, in the order of keys (alignment.py:23-39).
    Returns (acts, neural, matched_ids)."""
    idx = [i for i, k in enumerate(keys) if str(k) in targets]
    matched_ids = [str(keys[i]) for i in idx]
    if not matched_ids:
        neural = torch.empty(0, dtype=torch.float32)
        acts = {l: a[:0] for l, a in acts_raw.items()}
        return acts, neural, matched_ids
    neural = torch.as_tensor(np.stack([targets[sid] for sid in matched_ids]), dtype=torch.float32)
    acts = {}
    for l, a in acts_raw.items():
        acts[l] = a[torch.as_tensor(idx, dtype=torch.long, device=a.device)] if isinstance(
            a, torch.Tensor) else a[idx]
    return acts, neural, matched_ids


def prepare_traintest_alignment(cfg, acts_raw, neural_data_raw, keys) -> Tuple[AlignmentData, AlignmentData]:
    """Train and test AlignmentData from one activation dump (alignment.py:42-71)."""
    tr_a, tr_n, tr_ids = _align_stimulus_level(acts_raw, neural_data_raw["train"], keys)
    te_a, te_n, te_ids = _align_stimulus_level(acts_raw, neural_data_raw["test"], keys)
    return (AlignmentData(tr_a, tr_n, stimulus_ids=tr_ids),
            AlignmentData(te_a, te_n, stimulus_ids=te_ids))


def compute_traintest_alignment(cfg, train: AlignmentData, test: AlignmentData,
                                verbose: bool = False, re_extract_fn=None) -> List[dict]:
    """RSA dispatch (alignment.py:74-114). n_select defaults to None (all train)."""
    analysis = cfg.get("analysis", "rsa").lower()
    bootstrap = cfg.get("bootstrap", True)
    n_bootstrap = cfg.get("n_bootstrap", 1000)
    if analysis == "encoding_score" and cfg.get("neural_dataset", "").lower() == "things-behavior":
        raise ValueError(
            "Encoding score is not supported for things-behavior (behavioral embeddings "
            "have no voxels to predict). Use analysis=rsa instead."
        )
    if analysis == "rsa":
        return compute_rsa(cfg, train, test, n_select=cfg.get("n_select", None),
                           bootstrap=bootstrap, n_bootstrap=n_bootstrap, verbose=verbose,
                           re_extract_fn=re_extract_fn)
    if analysis == "encoding_score":
        from .encoding_score import compute_encoding_score

        pca_k = cfg.get("pca_k", 1) if cfg.get("reconstruct_from_pcs") else None
        return compute_encoding_score(train, test, bootstrap=bootstrap, n_bootstrap=n_bootstrap,
                                      verbose=verbose, reconstruct_pca_k=pca_k)
    raise ValueError(f"Unknown analysis method: {analysis}")


def prepare_concept_alignment(cfg, acts_raw, neural_data_raw, keys) -> AlignmentData:
    """Concept-mean activations paired with behavioural embeddings (alignment.py:117-162)."""
    key_to_idx = {k: i for i, k in enumerate(keys)}
    embeddings = neural_data_raw["embeddings"]
    image_ids = neural_data_raw["image_ids"]
    concepts, concept_image_ids = [], {}
    concept_acts = {l: [] for l in acts_raw}
    for concept, img_ids in image_ids.items():
        indices = [key_to_idx[sid] for sid in img_ids if sid in key_to_idx]
        if not indices:
            continue
        concepts.append(concept)
        concept_image_ids[concept] = [sid for sid in img_ids if sid in key_to_idx]
        for l, a in acts_raw.items():
            sel = a[torch.as_tensor(indices, dtype=torch.long, device=a.device)]
            concept_acts[l].append(sel.float().mean(0))
    acts = {l: torch.stack(vs).to(acts_raw[l].dtype) for l, vs in concept_acts.items()}
    neural = torch.as_tensor(np.stack([embeddings[c] for c in concepts], dtype=np.float32))
    logger.info("Prepared concept alignment: %d concepts.", len(concepts))
    return AlignmentData(acts, neural, stimulus_ids=concepts, concept_image_ids=concept_image_ids)

"""Stimulus alignment (reference: visreps/analysis/alignment.py).

The containers and the stimulus-ID joins fix the row order every RDM is built in, so
their semantics follow the reference exactly:

* stimulus level (alignment.py:23-39): rows of the activation dump whose key has a
  response, in dump order;
* train/test (alignment.py:42-71): the same join for each split;
* concept level (alignment.py:117-162): per THINGS concept (dict order, concepts with no
  extracted image dropped) the float mean of its images' activations, cast back to the
  layer dtype, paired with the concept's embedding (float32);
* dispatch (alignment.py:74-114): analysis=rsa -> compute_rsa, analysis=encoding_score ->
  compute_encoding_score (refused for things-behavior).
"""
from __future__ import annotations

import logging
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

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
    """One split: per-layer activations (rows = stimuli or concepts), the matching neural
    or behavioural targets, and the IDs that fix the row order (alignment.py:14-20)."""

    activations: Dict[str, torch.Tensor]
    neural: torch.Tensor
    stimulus_ids: Optional[List[str]] = None
    concept_image_ids: Optional[Dict[str, List[str]]] = None


def _take_rows(a, rows: Sequence[int]):
    """a[rows] for a tensor (on its own device) or any numpy-indexable array."""
    if isinstance(a, torch.Tensor):
        return a.index_select(0, torch.as_tensor(list(rows), dtype=torch.long, device=a.device))
    return a[list(rows)]


def _align_stimulus_level(acts_raw, targets, keys):
    """(acts, neural, ids): the dump rows whose key is in `targets`, dump order."""
    hits = [(row, str(key)) for row, key in enumerate(keys) if str(key) in targets]
    ids = [sid for _, sid in hits]
    if not hits:
        return {name: a[:0] for name, a in acts_raw.items()}, torch.empty(0, dtype=torch.float32), ids
    rows = [row for row, _ in hits]
    neural = torch.as_tensor(np.stack([targets[sid] for sid in ids]), dtype=torch.float32)
    return {name: _take_rows(a, rows) for name, a in acts_raw.items()}, neural, ids


def prepare_traintest_alignment(cfg, acts_raw, neural_data_raw, keys) -> Tuple[AlignmentData, AlignmentData]:  # noqa: ARG001
    """Train and test AlignmentData from one activation dump."""
    splits = []
    for part in ("train", "test"):
        acts, neural, ids = _align_stimulus_level(acts_raw, neural_data_raw[part], keys)
        splits.append(AlignmentData(acts, neural, stimulus_ids=ids))
    return splits[0], splits[1]


def compute_traintest_alignment(cfg, train: AlignmentData, test: AlignmentData,
                                verbose: bool = False, re_extract_fn=None) -> List[dict]:
    """Dispatch on cfg.analysis. n_select defaults to None (all train stimuli)."""
    analysis = str(cfg.get("analysis", "rsa")).lower()
    dataset = str(cfg.get("neural_dataset", "")).lower()
    common = dict(bootstrap=cfg.get("bootstrap", True), n_bootstrap=cfg.get("n_bootstrap", 1000),
                  verbose=verbose)
    if analysis == "encoding_score":
        if dataset == "things-behavior":
            raise ValueError(
                "Encoding score is not supported for things-behavior (behavioral embeddings "
                "have no voxels to predict). Use analysis=rsa instead."
            )
        from .encoding_score import compute_encoding_score

        pca_k = cfg.get("pca_k", 1) if cfg.get("reconstruct_from_pcs") else None
        return compute_encoding_score(train, test, reconstruct_pca_k=pca_k, **common)
    if analysis == "rsa":
        return compute_rsa(cfg, train, test, n_select=cfg.get("n_select", None),
                           re_extract_fn=re_extract_fn, **common)
    raise ValueError(f"Unknown analysis method: {analysis}")


def prepare_concept_alignment(cfg, acts_raw, neural_data_raw, keys) -> AlignmentData:  # noqa: ARG001
    """Concept-mean activations paired with behavioural embeddings."""
    where = {k: i for i, k in enumerate(keys)}
    groups: Dict[str, List[str]] = {}
    for concept, images in neural_data_raw["image_ids"].items():
        present = [sid for sid in images if sid in where]
        if present:  # a concept none of whose images was extracted has no row
            groups[concept] = present
    concepts = list(groups)

    def concept_means(a):
        rows = [_take_rows(a, [where[sid] for sid in groups[c]]).float().mean(0) for c in concepts]
        return torch.stack(rows).to(a.dtype)

    acts = {name: concept_means(a) for name, a in acts_raw.items()}
    emb = neural_data_raw["embeddings"]
    neural = torch.as_tensor(np.stack([emb[c] for c in concepts], dtype=np.float32))
    logger.info("Prepared concept alignment: %d concepts.", len(concepts))
    return AlignmentData(acts, neural, stimulus_ids=concepts, concept_image_ids=groups)

"""Neural-data loaders for the eval path.

The reference reads NSD / TVSD / THINGS from absolute /data paths (visreps/dataloaders/
neural.py); none of that data exists offline, so this build ships the same *contract*
with a deterministic NSD-shaped synthetic source:

  load_synthetic_data(cfg, subjects, regions) -> {
      "neural": {region: {subj: {"train": {sid: (V,) float32}, "test": {sid: (V,)}}}},
      "shared_test_ids": [sid, ...]  sorted by int (neural.py:170),
      "stimuli": {sid: row},         images generated on demand
  }
  _make_loader(stimuli, transform, batch, workers) iterates (images, ids) in the
  lexicographic ID order of the reference's _StimuliDataset (neural.py:474, :513-523).

Stimulus IDs are decimal strings without padding, so string order and int order differ
exactly as they do for NSD IDs, and phase 1 / phase 2 row orders are exercised as in
the reference. Responses follow dataloaders/synthetic.make_responses with a per-subject
noise seed.
"""
from __future__ import annotations

from typing import Dict, Iterator, List, Sequence, Tuple

import numpy as np
import torch

from . import synthetic as syn

__all__ = ["SyntheticStimuli", "load_synthetic_data", "_make_loader", "StimulusLoader"]


class SyntheticStimuli(dict):
    """sid -> stimulus row; images are generated per 64-row block on demand."""

    def __init__(self, rows: Dict[str, int], seed: int, device):
        super().__init__(rows)
        self.seed = int(seed)
        self.device = torch.device(device)

    def subset(self, sids: Sequence[str]) -> "SyntheticStimuli":
        return SyntheticStimuli({s: self[s] for s in sids if s in self}, self.seed, self.device)

    def images(self, rows: Sequence[int]) -> torch.Tensor:
        out = torch.empty((len(rows), 3, 224, 224), dtype=torch.float32, device=self.device)
        if not rows:
            return out
        rows_t = np.asarray(rows, dtype=np.int64)
        for blk in np.unique(rows_t // syn.BLOCK):
            b0 = int(blk) * syn.BLOCK
            block = syn.make_images(range(b0, b0 + syn.BLOCK), seed=self.seed, device=self.device)
            sel = np.nonzero(rows_t // syn.BLOCK == blk)[0]
            out[torch.as_tensor(sel, device=self.device)] = block[
                torch.as_tensor(rows_t[sel] - b0, device=self.device)]
        return out


class StimulusLoader:
    """Batches of (images (B,3,224,224) on the stimuli's device, ids) in string-sorted ID
    order, like DataLoader(_StimuliDataset(stimuli), shuffle=False)."""

    def __init__(self, stimuli: SyntheticStimuli, batch: int):
        self.stimuli = stimuli
        self.batch = max(1, int(batch))
        self.ids = sorted(stimuli.keys(), key=str)

    def __len__(self) -> int:
        return (len(self.ids) + self.batch - 1) // self.batch

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, List[str]]]:
        for i in range(0, len(self.ids), self.batch):
            ids = self.ids[i:i + self.batch]
            yield self.stimuli.images([self.stimuli[s] for s in ids]), ids


def _make_loader(stimuli, transform, batch, workers):  # noqa: ARG001  (tensors need no transform)
    return StimulusLoader(stimuli, batch)


def load_synthetic_data(cfg, subjects: Sequence[int], regions: Sequence[str]) -> Dict:
    """NSD-shaped synthetic data: n_test shared test stimuli + n_train train stimuli per
    subject (cfg.synthetic.n_test / n_train / voxels / seed; defaults 1000 / 1000 /
    NSD_ROIS_4 / 20260306)."""
    sc = cfg.get("synthetic", {}) or {}
    n_test = int(sc.get("n_test", 1000))
    n_train = int(sc.get("n_train", 1000))
    seed = int(sc.get("seed", 20260306))
    vox_cfg = dict(sc.get("voxels", {}) or {})
    voxels = {r: int(vox_cfg.get(r, syn.NSD_ROIS_4.get(r, 1000))) for r in regions}
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
        else torch.device("cpu")
    n_total = n_test + n_train
    rows = {str(i): i for i in range(n_total)}
    stimuli = SyntheticStimuli(rows, seed, dev)
    test_ids = [str(i) for i in range(n_test)]
    train_ids = [str(i) for i in range(n_test, n_total)]
    neural: Dict[str, Dict[int, Dict[str, Dict[str, np.ndarray]]]] = {r: {} for r in regions}
    chunk = 4096
    for subj in subjects:
        per_region = {r: np.empty((n_total, v), np.float32) for r, v in voxels.items()}
        for c0 in range(0, n_total, chunk):
            rr = range(c0, min(n_total, c0 + chunk))
            imgs = syn.make_images(rr, seed=seed, device=dev)
            resp = syn.make_responses(imgs, rr, voxels, seed=seed + 7 * (int(subj) + 1))
            for r in voxels:
                per_region[r][rr.start:rr.stop] = resp[r].cpu().numpy()
            del imgs, resp
        for r in regions:
            y = per_region[r]
            neural[r][subj] = {
                "train": {s: y[rows[s]] for s in train_ids},
                "test": {s: y[rows[s]] for s in test_ids},
            }
    return {"neural": neural, "shared_test_ids": sorted(test_ids, key=int), "stimuli": stimuli}

"""Neural-data loaders for the eval path.

The reference reads NSD / TVSD / THINGS from absolute /data paths (visreps/dataloaders/
neural.py); none of that data exists offline, so this build ships the same *contract*
with a deterministic NSD-shaped synthetic source:

  load_synthetic_data(cfg, subjects, regions) -> {
      "neural": {region: {subj: {"train": {sid: (V,) float32}, "test": {sid: (V,)}}}},
      "shared_test_ids": [sid, ...]  sorted by int (neural.py:170),
      "stimuli": {sid: row},         images generated on demand
  }
  load_tvsd_synthetic(cfg, subjects, regions) -> the load_all_tvsd_data contract
      (neural.py:393-460): V1/V4/IT, ~22k train + 100 test stimuli per subject
  load_things_synthetic(cfg) -> (targets, stimuli), the THINGS-behaviour contract
      (neural.py:313-336): targets = {"embeddings": {concept: (66,) float32},
      "image_ids": {concept: [sid, ...]}}, stimuli = {sid: image}
  load_nsd_synthetic_test_data(cfg, subjects, regions) -> {"neural": {region: {subj:
      {sid: (V,)}}}, "stimuli", "test_ids" (sorted names), "regions", "subjects"}
      (neural.py:192-241; 220 stimuli)
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

__all__ = ["SyntheticStimuli", "load_synthetic_data", "load_things_synthetic", "load_tvsd_synthetic",
           "load_nsd_synthetic_test_data", "_make_loader", "StimulusLoader"]


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


def _make_loader(stimuli, transform, batch, workers):  # noqa: ARG001
    """Synthetic stimuli are generated as normalised tensors (no transform applies); any
    other {key: path | uint8 array | PIL image} mapping is read and transformed on the
    device by dataloaders.obj_cls.ImageLoader (get_transform, vr_transform_u8)."""
    if isinstance(stimuli, SyntheticStimuli):
        return StimulusLoader(stimuli, batch)
    from .obj_cls import ImageLoader

    return ImageLoader(stimuli, transform, batch)


def _device():
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
        else torch.device("cpu")


def _responses(stimuli: SyntheticStimuli, n: int, voxels: Dict[str, int], seed: int,
               noise: float = 3.0) -> Dict[str, np.ndarray]:
    """make_responses for rows 0..n-1 of `stimuli`, in 4096-row chunks, on the host."""
    out = {r: np.empty((n, v), np.float32) for r, v in voxels.items()}
    for c0 in range(0, n, 4096):
        rr = range(c0, min(n, c0 + 4096))
        imgs = syn.make_images(rr, seed=stimuli.seed, device=stimuli.device)
        resp = syn.make_responses(imgs, rr, voxels, seed=seed, noise=noise)
        for r in voxels:
            out[r][rr.start:rr.stop] = resp[r].cpu().numpy()
        del imgs, resp
    return out


def load_things_synthetic(cfg) -> Tuple[Dict, SyntheticStimuli]:
    """THINGS-shaped behavioural data: cfg.synthetic.things_concepts concepts (default
    1854) with things_images images each (default 2); a concept's 66-d embedding is the
    non-negative (SPoSE-like) mean over its images of a response to their latent."""
    sc = cfg.get("synthetic", {}) or {}
    n_c = int(sc.get("things_concepts", 1854))
    per = int(sc.get("things_images", 2))
    seed = int(sc.get("seed", 20260306)) + 17
    concepts = [f"concept{c:04d}" for c in range(n_c)]
    rows: Dict[str, int] = {}
    image_ids: Dict[str, List[str]] = {}
    for c, name in enumerate(concepts):
        sids = [f"{name}_{j:02d}s" for j in range(per)]
        image_ids[name] = sids
        for j, sid in enumerate(sids):
            rows[sid] = c * per + j
    stimuli = SyntheticStimuli(rows, seed, _device())
    emb = _responses(stimuli, n_c * per, {"things": 66}, seed + 3, noise=1.0)["things"]
    embeddings = {name: np.maximum(emb[c * per:(c + 1) * per].mean(0), 0.0).astype(np.float32)
                  for c, name in enumerate(concepts)}
    return {"embeddings": embeddings, "image_ids": image_ids}, stimuli


def load_nsd_synthetic_test_data(cfg, subjects: Sequence[int], regions: Sequence[str]) -> Dict:
    """NSD-Synthetic-shaped test data: cfg.synthetic.nsd_synthetic_n stimuli (default 220,
    names sorted), per-subject responses with the NSD source's voxel counts."""
    sc = cfg.get("synthetic", {}) or {}
    n = int(sc.get("nsd_synthetic_n", 220))
    seed = int(sc.get("seed", 20260306)) + 29
    vox_cfg = dict(sc.get("voxels", {}) or {})
    voxels = {r: int(vox_cfg.get(r, syn.NSD_ROIS_4.get(r, 1000))) for r in regions}
    names = [f"synth{i:03d}" for i in range(n)]
    stimuli = SyntheticStimuli({s: i for i, s in enumerate(names)}, seed, _device())
    neural: Dict = {r: {} for r in regions}
    for subj in subjects:
        resp = _responses(stimuli, n, voxels, seed + 7 * (int(subj) + 1))
        for r in regions:
            neural[r][subj] = {s: resp[r][i] for i, s in enumerate(names)}
    return {"regions": list(regions), "subjects": list(subjects), "neural": neural,
            "stimuli": stimuli, "test_ids": sorted(names)}


TVSD_VOXELS = {"V1": 512, "V4": 256, "IT": 256}  # MUA sites per region (synthetic counts)


def load_tvsd_synthetic(cfg, subjects: Sequence[int], regions: Sequence[str]) -> Dict:
    """TVSD-shaped macaque MUA data with the contract of load_all_tvsd_data
    (reference neural.py:393-460): regions V1 / V4 / IT, subjects 0 (monkey F) and 1 (monkey
    N), per subject "train" (cfg.synthetic.tvsd_n_train, default 22,248 THINGS images) and
    "test" (tvsd_n_test, default 100) response dicts keyed by THINGS-style image names, and
    shared_test_ids = the test names common to every subject, sorted as strings (neural.py:453;
    NSD sorts its IDs as integers instead). Responses: dataloaders/synthetic.make_responses
    with a per-subject seed and the TVSD_VOXELS site counts (cfg.synthetic.voxels overrides)."""
    sc = cfg.get("synthetic", {}) or {}
    n_train = int(sc.get("tvsd_n_train", 22248))
    n_test = int(sc.get("tvsd_n_test", 100))
    seed = int(sc.get("seed", 20260306)) + 41
    vox_cfg = dict(sc.get("voxels", {}) or {})
    voxels = {r: int(vox_cfg.get(r, TVSD_VOXELS.get(r, 256))) for r in regions}
    # THINGS image names: 12 train images per concept (22,248 = 1,854 x 12), one test
    # image per test concept; the concept order is not the name order
    train_ids = [f"c{(c * 7919) % 1854:04d}_{j:02d}s" for c in range(-(-n_train // 12)) for j in range(12)][:n_train]
    test_ids = [f"c{(c * 104729) % 1854:04d}_99t" for c in range(n_test)]
    names = train_ids + test_ids
    if len(set(names)) != len(names):
        raise ValueError("tvsd_n_train / tvsd_n_test exceed the synthetic THINGS name space")
    stimuli = SyntheticStimuli({s: i for i, s in enumerate(names)}, seed, _device())
    neural: Dict = {r: {} for r in regions}
    for subj in subjects:
        resp = _responses(stimuli, len(names), voxels, seed + 11 * (int(subj) + 1))
        for r in regions:
            neural[r][subj] = {"train": {s: resp[r][i] for i, s in enumerate(train_ids)},
                               "test": {s: resp[r][len(train_ids) + i] for i, s in enumerate(test_ids)}}
    return {"regions": list(regions), "subjects": list(subjects), "neural": neural, "stimuli": stimuli,
            "shared_test_ids": sorted(test_ids)}


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

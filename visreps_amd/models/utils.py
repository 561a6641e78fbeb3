"""Feature extraction for the eval path (reference: visreps/models/utils.py).

  FeatureExtractor          forward hooks at conv1..conv5 / fc1..fc2 (x pre/post)  :33-260
  configure_feature_extractor                                                       :262-278
  get_activations           phase-1 bulk extraction, sparse random projection     :281-347
  extract_single_layer      exact re-extraction of one layer, reordered to ids    :350-404
  load_model                checkpoint / torchvision / custom construction        :407-471

MI355X differences (not semantics): activations can stay in HBM (keep_on_device=True)
so the RDM kernels read them in place; the SRP product runs in the HIP CSR kernel of
visreps_amd.analysis.sparse_random_projection; checkpoints are read with
torch.load(weights_only=True) — the reference pickles whole nn.Modules, which this build
will not unpickle (convert them to state_dicts once, in the reference's environment:
INTEGRATION.md, "Checkpoints: converting the reference's pickled models").
"""
from __future__ import annotations

from collections import defaultdict
from typing import Dict, Iterable, List, Optional, Tuple

import torch
import torch.nn as nn

from . import custom_model, standard_model
from .custom_model import CustomCNN, TinyCustomCNN
from .standard_model import AlexNetModule, VisionTransformer
from ..utils import get_seed_letter, rprint

TORCHVISION_RETURN_NODES = {
    "AlexNet": ["conv1", "conv2", "conv3", "conv4", "conv5", "fc1", "fc2"],
    "ViTBase": [f"block{i}" for i in range(1, 13)],
}

_ACTS = (nn.ReLU, nn.GELU, nn.LeakyReLU)
_CONVS = (nn.Conv1d, nn.Conv2d, nn.Conv3d)


class FeatureExtractor(nn.Module):
    """Hooks semantic extraction points; forward(x) returns {point: output tensor}.

    Outputs are the hooked modules' output tensors themselves (no copy), so an in-place
    ReLU right after a Conv/Linear makes `_pre` equal `_post`, exactly as in the
    reference for torchvision AlexNet; CustomCNN has BatchNorm in between, so its _pre
    is genuinely pre-BN."""

    def __init__(self, model: nn.Module, return_nodes=None, post_relu: bool = True,
                 extract_pre_and_post: bool = True):
        super().__init__()
        self.model = model
        if isinstance(return_nodes, (list, tuple)):
            return_nodes = {node: node for node in return_nodes}
        self.return_nodes = dict(return_nodes or {})
        self.post_relu = post_relu
        self.extract_pre_and_post = extract_pre_and_post
        self.features: Dict[str, torch.Tensor] = {}
        self.handles = []
        base = self._create_layer_mapping()
        if extract_pre_and_post:
            post = self._remap_to_post_relu(base)
            self.layer_mapping, self.return_nodes = self._build_pre_post_mapping(base, post)
        elif post_relu:
            self.layer_mapping = self._remap_to_post_relu(base)
        else:
            self.layer_mapping = base
        self._attach_hooks()

    def _create_layer_mapping(self) -> Dict[str, str]:
        """Semantic name -> module path (utils.py:61-154): AlexNet/VGG-style
        features+classifier containers, ViT blocks, else a generic conv/fc walk."""
        mapping: Dict[str, str] = {}
        m = self.model
        if isinstance(m, VisionTransformer):
            mapping["patch_embed"] = "conv_proj"
            for i, _ in enumerate(m.encoder.layers):
                mapping[f"block{i + 1}"] = f"encoder.layers.encoder_layer_{i}"
            mapping["head"] = "heads.head"
        elif hasattr(m, "features") and hasattr(m, "classifier"):
            convs = [n for n, mod in m.features.named_modules() if isinstance(mod, _CONVS)]
            fcs = [n for n, mod in m.classifier.named_modules() if isinstance(mod, nn.Linear)]
            mapping.update({f"conv{i + 1}": f"features.{n}" for i, n in enumerate(convs)})
            mapping.update({f"fc{i + 1}": f"classifier.{n}" for i, n in enumerate(fcs)})
        if not mapping:
            ci = fi = 1
            for name, mod in m.named_modules():
                if isinstance(mod, _CONVS) and "downsample" not in name:
                    mapping[f"conv{ci}"] = name
                    ci += 1
                elif isinstance(mod, nn.Linear):
                    mapping[f"fc{fi}"] = name
                    fi += 1
        return mapping

    def _remap_to_post_relu(self, mapping: Dict[str, str]) -> Dict[str, str]:
        """Move each requested point to the next activation in its Sequential, stopping
        at the next Conv/Linear (utils.py:156-196)."""
        requested = set(self.return_nodes or [])
        out = {}
        for name, path in mapping.items():
            out[name] = path
            if requested and name not in requested:
                continue
            parts = path.split(".")
            if len(parts) != 2:
                continue
            container = getattr(self.model, parts[0], None)
            if not isinstance(container, nn.Sequential) or not parts[1].isdigit():
                continue
            for i in range(int(parts[1]) + 1, len(container)):
                if isinstance(container[i], _ACTS):
                    out[name] = f"{parts[0]}.{i}"
                    break
                if isinstance(container[i], _CONVS + (nn.Linear,)):
                    break
        return out

    def _build_pre_post_mapping(self, base, post):
        """name_pre -> raw Conv/Linear, name_post -> its activation; points without a
        downstream activation keep a single entry (utils.py:198-230)."""
        combined, expanded = {}, {}
        for name, out_name in self.return_nodes.items():
            b, p = base.get(name), post.get(name)
            if b is None:
                print(f"Warning: {name} not found in base mapping")
                continue
            if p is not None and b != p:
                combined[f"{name}_pre"] = b
                combined[f"{name}_post"] = p
                expanded[f"{name}_pre"] = f"{name}_pre"
                expanded[f"{name}_post"] = f"{name}_post"
            else:
                combined[name] = b
                expanded[name] = out_name
        return combined, expanded

    def _attach_hooks(self):
        by_path: Dict[str, List[str]] = defaultdict(list)
        for sem in self.return_nodes:
            if sem in self.layer_mapping:
                by_path[self.layer_mapping[sem]].append(self.return_nodes[sem])
            else:
                print(f"Warning: {sem} not found in model")
        for name, module in self.model.named_modules():
            if name in by_path:
                outs = by_path[name]

                def hook(_m, _inp, output, outs=outs):
                    for o in outs:
                        self.features[o] = output

                self.handles.append(module.register_forward_hook(hook))

    def forward(self, x):
        self.features = {}
        self.model(x)
        return self.features

    def __del__(self):
        for h in getattr(self, "handles", []):
            h.remove()


def configure_feature_extractor(cfg, model, verbose=False) -> FeatureExtractor:
    rn = cfg.get("return_nodes", {})
    if hasattr(rn, "to_container"):
        rn = rn.to_container()
    if not rn:
        raise ValueError("return_nodes must be specified in config")
    rn = {n: n for n in rn} if isinstance(rn, (list, tuple)) else dict(rn)
    pre_post = cfg.get("extract_pre_and_post", True)
    model.eval()
    ex = FeatureExtractor(model, rn, extract_pre_and_post=pre_post)
    suffix = f" ({len(rn)} layers × pre/post)" if pre_post else ""
    rprint(f"  ✓ {len(ex.return_nodes)} extraction points{suffix}", style="success")
    if verbose:
        rprint(f"    Layers: {list(rn)}", style="info")
        rprint(f"    Points: {list(ex.return_nodes)}", style="info")
    return ex


@torch.no_grad()
def get_activations(model: nn.Module, dataloader: Iterable, device: torch.device,
                    keep_on_device: bool = False, srp_seed: Optional[int] = None,
                    srp_cache_dir: str = "model_checkpoints/srp_cache",
                    k_fixed: int = 4096) -> Tuple[Dict[str, torch.Tensor], List]:
    """Every point of every batch, projected to k = min(4096, D) with a sparse random
    projection (utils.py:281-347). The projection matrices come from
    get_srp_transformer (sklearn construction, cached); the reference leaves
    random_state=None, so an unseeded run is not reproducible there either."""
    from ..analysis.sparse_random_projection import SparseProjector, get_srp_transformer

    model.eval()
    acts: Dict[str, List[torch.Tensor]] = defaultdict(list)
    ids: List = []
    it = iter(dataloader)
    try:
        first = next(it)
    except StopIteration:
        return {}, []
    probe = model(first[0].to(device))
    srp = {}
    for name, out in probe.items():
        D = out.reshape(out.size(0), -1).size(1)
        comp = get_srp_transformer(D=D, k=min(k_fixed, D), density=None, seed=srp_seed,
                                   cache_dir=srp_cache_dir)
        srp[name] = SparseProjector(comp, device)
    rprint(f"  ✓ SRP transformers for {len(probe)} layers (k={k_fixed})", style="success")

    def consume(batch):
        imgs, keys = batch
        ids.extend(keys)
        feats = model(imgs.to(device, non_blocking=True))
        for name, out in feats.items():
            flat = out.reshape(out.size(0), -1).float()
            proj = srp[name](flat)
            acts[name].append(proj if keep_on_device else proj.cpu())

    consume(first)
    for batch in it:
        consume(batch)
    return {n: torch.cat(b, 0) for n, b in acts.items()}, ids


@torch.no_grad()
def extract_single_layer(model: nn.Module, dataloader: Iterable, device: torch.device,
                         layer_name: str, stimulus_ids: Optional[List[str]] = None,
                         keep_on_device: bool = False) -> Tuple[torch.Tensor, List]:
    """Exact (un-projected) activations of one point; rows reordered to stimulus_ids
    when given (utils.py:350-404)."""
    model.eval()
    chunks, all_ids = [], []
    for imgs, keys in dataloader:
        all_ids.extend(keys)
        out = model(imgs.to(device, non_blocking=True))[layer_name]
        flat = out.reshape(out.size(0), -1).float()
        chunks.append(flat if keep_on_device else flat.cpu())
    acts = torch.cat(chunks, 0)
    if stimulus_ids is not None:
        pos = {str(k): i for i, k in enumerate(all_ids)}
        keep = [pos[str(s)] for s in stimulus_ids if str(s) in pos]
        acts = acts[torch.as_tensor(keep, dtype=torch.long, device=acts.device)]
        all_ids = [all_ids[i] for i in keep]
    rprint(f"  ✓ Re-extracted {layer_name}: {tuple(acts.shape)} (exact, no SRP)", style="success")
    return acts, all_ids


def load_model(cfg, device, num_classes=None, verbose=False) -> nn.Module:
    """Checkpoint / torchvision-architecture / custom model (utils.py:407-471)."""
    if cfg.get("load_model_from") == "checkpoint":
        if cfg.get("random_init", False):
            torch.manual_seed(int(cfg.get("init_seed", 0)))
            return CustomCNN(num_classes=cfg.get("n_classes", 1000)).to(device)
        letter = get_seed_letter(cfg.seed)
        path = f"{cfg.checkpoint_dir}/cfg{cfg.cfg_id}{letter}/{cfg.checkpoint_model}"
        ckpt = torch.load(path, map_location="cpu", weights_only=True)
        state = ckpt.get("model_state_dict", ckpt.get("state_dict", ckpt))
        n_cls = next((v.shape[0] for k, v in state.items() if k.endswith("classifier.8.weight")), 1000)
        tiny = any(k.startswith("classifier.1.weight") and v.shape[1] == 512 * 16 for k, v in state.items())
        model = (TinyCustomCNN if tiny else CustomCNN)(num_classes=n_cls)
        model.load_state_dict(state, strict=True)
        rprint(f"  ✓ Loaded checkpoint (cfg{cfg.cfg_id}{letter})", style="success")
        return model.to(device)
    model_class = cfg.get("model_class", "standard_model")
    name = cfg.get("model_name", "AlexNet")
    if model_class == "custom_model":
        arch = cfg.get("arch", {}) or {}
        params = dict(num_classes=num_classes,
                      trainable_layers={"conv": arch.get("conv_trainable", "11111"),
                                        "fc": arch.get("fc_trainable", "111")},
                      dropout=arch.get("dropout", 0.5), pooling_type=arch.get("pooling_type", "max"))
        model = (TinyCustomCNN if "tiny" in name.lower() else CustomCNN)(**params)
    else:
        fn = getattr(standard_model, name, None)
        if fn is None:
            raise ValueError(f"Model '{name}' not found in standard_model.")
        model = fn(cfg.get("pretrained_dataset", "none"), num_classes)
    return model.to(device)

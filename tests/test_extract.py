"""Feature dumps (scripts/extract_representations/utils.py:31-78 and the model scripts):
loader-order concatenation, image names from dataset.samples, the name/feature mismatch
error, L2-normalised AlexNet fc2 / ViT CLS rows, and the npz layout. CPU (torch plumbing
around the forward pass; no HIP kernel involved)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from visreps_amd import extract_representations as X
from visreps_amd.models.standard_model import AlexNetModule, VisionTransformer


class _DS(torch.utils.data.Dataset):
    def __init__(self, n, size, named=True):
        g = torch.Generator().manual_seed(0)
        self.x = torch.randn(n, 3, size, size, generator=g)
        if named:
            self.samples = [(f"path/{i}", i % 3, f"img_{i:03d}") for i in range(n)]

    def __len__(self):
        return len(self.x)

    def __getitem__(self, i):
        return self.x[i], 0


def test_alexnet_fc2_rows_l2_normalised_in_loader_order(tmp_path):
    torch.manual_seed(0)
    model, fn = X.alexnet_fc2(AlexNetModule(1000))
    assert len(model.classifier) == 6
    ds = _DS(10, 64)
    loader = torch.utils.data.DataLoader(ds, batch_size=4, shuffle=False)
    feats, names = X.extract_features(model, [loader], fn, torch.device("cpu"))
    assert feats.shape == (10, 4096) and feats.dtype == np.float32
    assert names == [f"img_{i:03d}" for i in range(10)]
    np.testing.assert_allclose(np.linalg.norm(feats, axis=1), 1.0, rtol=1e-5)
    with torch.no_grad():
        ref = F.normalize(model(ds.x), p=2, dim=-1).numpy()
    np.testing.assert_allclose(feats, ref, rtol=1e-5, atol=1e-6)
    path = X.save_features(feats, names, "toy", "alexnet_features", root=str(tmp_path))
    assert path.endswith("obj_cls/toy/features_alexnet_features.npz")
    f2, n2 = X.load_features(path, "alexnet_features")
    assert np.array_equal(f2, feats) and n2 == names


def test_vit_cls_features():
    torch.manual_seed(0)
    model, fn = X.vit_cls(VisionTransformer(num_layers=2))
    ds = _DS(3, 224)
    loader = torch.utils.data.DataLoader(ds, batch_size=2, shuffle=False)
    feats, names = X.extract_features(model, [loader], fn, torch.device("cpu"))
    assert feats.shape == (3, 768) and len(names) == 3
    np.testing.assert_allclose(np.linalg.norm(feats, axis=1), 1.0, rtol=1e-5)
    with torch.no_grad():
        assert torch.allclose(model(ds.x[:1]), model.heads(model.forward_features(ds.x[:1])[:, 0]))


def test_vit_large_patch16_cls_dump():
    # vit_representations.py's default model (vit_large_patch16_224): 24 pre-norm blocks of
    # width 1024 (16 heads, MLP 4096), 197 tokens; the dump is the L2-normalised 1024-d CLS
    from visreps_amd.models.standard_model import vit_large_patch16_224

    torch.manual_seed(0)
    m = vit_large_patch16_224().eval()
    assert len(m.encoder.layers) == 24 and m.hidden_dim == 1024
    assert m.encoder.pos_embedding.shape == (1, 197, 1024)
    blk = m.encoder.layers[0]
    assert blk.self_attention.num_heads == 16 and blk.mlp[0].out_features == 4096
    assert sum(p.numel() for p in m.parameters()) > 300_000_000  # ViT-L scale (~304M with the head)
    model, fn = X.vit_cls(m)
    ds = _DS(2, 224)
    loader = torch.utils.data.DataLoader(ds, batch_size=2, shuffle=False)
    feats, names = X.extract_features(model, [loader], fn, torch.device("cpu"))
    assert feats.shape == (2, 1024) and names == ["img_000", "img_001"]
    np.testing.assert_allclose(np.linalg.norm(feats, axis=1), 1.0, rtol=1e-5)
    with torch.no_grad():
        tok = m.forward_features(ds.x)
    np.testing.assert_allclose(feats, F.normalize(tok[:, 0], dim=-1).numpy(), rtol=1e-5, atol=1e-6)


def test_name_mismatch_raises():
    model, fn = X.alexnet_fc2(AlexNetModule(1000))
    loader = torch.utils.data.DataLoader(_DS(2, 64, named=False), batch_size=2)
    with pytest.raises(ValueError, match="Mismatch"):
        X.extract_features(model, [loader], fn, torch.device("cpu"))


def test_clip_visual_structure_and_unit_rows():
    # clip/model.py VisionTransformer at a tiny width: token layout, ln_post on the class
    # token, projection, and the dump's row normalisation
    from visreps_amd.models.foundation import CLIPImageModel, CLIPVisual

    torch.manual_seed(0)
    m = CLIPImageModel(input_resolution=28, patch_size=14, width=32, layers=2, heads=4, output_dim=16).eval()
    v = m.visual
    assert v.positional_embedding.shape == (5, 32) and v.conv1.bias is None
    assert isinstance(v.transformer[0].mlp.gelu, torch.nn.Module)
    x = torch.randn(3, 3, 28, 28)
    model, fn = X.clip_image(m)
    with torch.no_grad():
        f = fn(model, x)
        # manual forward of the tower
        t = v.conv1(x).reshape(3, 32, -1).permute(0, 2, 1)
        t = torch.cat([v.class_embedding + torch.zeros(3, 1, 32), t], 1) + v.positional_embedding
        t = v.transformer(v.ln_pre(t).permute(1, 0, 2)).permute(1, 0, 2)
        ref = v.ln_post(t[:, 0]) @ v.proj
    assert torch.allclose(f, ref / ref.norm(dim=-1, keepdim=True), atol=1e-6)
    assert torch.allclose(f.norm(dim=-1), torch.ones(3), atol=1e-6)


def test_clip_vit_l14_dimensions():
    from visreps_amd.models.foundation import clip_vit_l14

    v = clip_vit_l14().visual
    assert v.conv1.weight.shape == (1024, 3, 14, 14)
    assert v.positional_embedding.shape == (257, 1024) and v.proj.shape == (1024, 768)
    assert len(v.transformer) == 24 and v.transformer[0].attn.num_heads == 16


def test_dino_structure_and_cls_rows():
    from visreps_amd.models.foundation import DINOv3ViT, _apply_rope, _rope_tables

    torch.manual_seed(0)
    m = DINOv3ViT(img_size=32, patch_size=16, embed_dim=32, depth=2, num_heads=4, num_registers=4).eval()
    x = torch.randn(2, 3, 32, 32)
    with torch.no_grad():
        tok = m.forward_features(x)
    assert tok.shape == (2, 1 + 4 + 4, 32)
    model, fn = X.dino_cls(m)
    with torch.no_grad():
        f = fn(model, x)
    assert torch.allclose(f, F.normalize(tok[:, 0], dim=-1), atol=1e-6)
    # the rotary embedding is a rotation: norms of q/k rows are preserved
    cos, sin = _rope_tables(2, 8)
    q = torch.randn(1, 1, 4, 8)
    assert torch.allclose(_apply_rope(q, cos, sin).norm(dim=-1), q.norm(dim=-1), atol=1e-5)

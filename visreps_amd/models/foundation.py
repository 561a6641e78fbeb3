"""The foundation-model feature extractors of the reference's representation dumps
(scripts/extract_representations/clip_representations.py:26-38,
dino_representations.py:24-38), rebuilt with random initialisation.

Neither clip nor timm is installed and no weights can be downloaded, so the networks are
defined here with the published architectures:

* CLIP ViT-L/14 image tower (OpenAI clip/model.py VisionTransformer): conv1 14x14/14
  without bias, class embedding, 257 learned positions, ln_pre, 24 residual blocks of
  width 1024 / 16 heads with QuickGELU MLPs, ln_post on the class token, 1024 x 768
  projection. encode_image(x) = visual(x); the dump L2-normalises it.
* DINOv3 ViT-L/16 (timm 'vit_large_patch16_dinov3'): 16x16 patches, width 1024, 24
  blocks / 16 heads, a class token and 4 register tokens, 2-D rotary position embedding
  on the patch tokens' queries and keys, LayerScale; forward_features returns the
  normed tokens [CLS, registers, patches] and the dump L2-normalises the CLS token.
  timm's exact module layout is not reproduced (no weights to load), so this is the
  architecture class, not a checkpoint-compatible copy.

Their loaders' preprocessing is get_transform's device kernel with Pillow's bicubic
filter (clip._transform: Resize(224, BICUBIC), CenterCrop(224), CLIP mean/std; timm
eval transform for the DINOv3 config: bicubic, crop_pct 1.0, ImageNet mean/std).
"""
from __future__ import annotations

import math
from collections import OrderedDict

import torch
import torch.nn as nn
import torch.nn.functional as F

__all__ = ["CLIPVisual", "CLIPImageModel", "clip_vit_l14", "DINOv3ViT", "dinov3_vit_l16",
           "CLIP_MEAN", "CLIP_STD"]

CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)


class QuickGELU(nn.Module):
    def forward(self, x):
        return x * torch.sigmoid(1.702 * x)


class _ResidualAttentionBlock(nn.Module):
    def __init__(self, d_model: int, n_head: int):
        super().__init__()
        self.attn = nn.MultiheadAttention(d_model, n_head)
        self.ln_1 = nn.LayerNorm(d_model)
        self.mlp = nn.Sequential(OrderedDict([
            ("c_fc", nn.Linear(d_model, d_model * 4)), ("gelu", QuickGELU()),
            ("c_proj", nn.Linear(d_model * 4, d_model))]))
        self.ln_2 = nn.LayerNorm(d_model)

    def forward(self, x):  # x: (L, N, D)
        h = self.ln_1(x)
        x = x + self.attn(h, h, h, need_weights=False)[0]
        return x + self.mlp(self.ln_2(x))


class CLIPVisual(nn.Module):
    """clip/model.py VisionTransformer (the image tower)."""

    def __init__(self, input_resolution=224, patch_size=14, width=1024, layers=24, heads=16,
                 output_dim=768):
        super().__init__()
        self.input_resolution = input_resolution
        self.conv1 = nn.Conv2d(3, width, kernel_size=patch_size, stride=patch_size, bias=False)
        scale = width ** -0.5
        self.class_embedding = nn.Parameter(scale * torch.randn(width))
        self.positional_embedding = nn.Parameter(
            scale * torch.randn((input_resolution // patch_size) ** 2 + 1, width))
        self.ln_pre = nn.LayerNorm(width)
        self.transformer = nn.Sequential(*[_ResidualAttentionBlock(width, heads) for _ in range(layers)])
        self.ln_post = nn.LayerNorm(width)
        self.proj = nn.Parameter(scale * torch.randn(width, output_dim))

    def forward(self, x):
        x = self.conv1(x)
        x = x.reshape(x.shape[0], x.shape[1], -1).permute(0, 2, 1)
        cls = self.class_embedding.to(x.dtype) + torch.zeros(x.shape[0], 1, x.shape[-1], dtype=x.dtype,
                                                             device=x.device)
        x = torch.cat([cls, x], dim=1) + self.positional_embedding.to(x.dtype)
        x = self.ln_pre(x).permute(1, 0, 2)
        x = self.transformer(x).permute(1, 0, 2)
        return self.ln_post(x[:, 0, :]) @ self.proj


class CLIPImageModel(nn.Module):
    """The part of clip.load's model the dump uses: .visual and encode_image."""

    def __init__(self, **kw):
        super().__init__()
        self.visual = CLIPVisual(**kw)

    @property
    def dtype(self):
        return self.visual.conv1.weight.dtype

    def encode_image(self, image):
        return self.visual(image.type(self.dtype))


def clip_vit_l14() -> CLIPImageModel:
    return CLIPImageModel()


# ----------------------------------------------------------------------------- DINOv3
def _rope_tables(grid: int, head_dim: int, base: float = 100.0, device=None):
    """cos / sin of a 2-D axial rotary embedding: half of each head's channels rotate with
    the patch row, half with the column (frequencies base^(-4i/head_dim))."""
    q = head_dim // 4
    freqs = base ** (-torch.arange(q, dtype=torch.float32, device=device) / q)
    coords = (torch.arange(grid, dtype=torch.float32, device=device) + 0.5) / grid * 2 - 1
    yy, xx = torch.meshgrid(coords, coords, indexing="ij")
    ang = torch.cat([yy.reshape(-1, 1) * freqs * math.pi, xx.reshape(-1, 1) * freqs * math.pi], dim=1)
    return ang.cos(), ang.sin()  # (P, head_dim / 2): one angle per rotated channel pair


def _apply_rope(t, cos, sin):
    """t (B, H, P, hd): rotate channel halves (rotate-half convention)."""
    h = t.shape[-1] // 2
    t1, t2 = t[..., :h], t[..., h:]
    c, s = cos.to(t.dtype), sin.to(t.dtype)
    return torch.cat([t1 * c - t2 * s, t1 * s + t2 * c], dim=-1)


class _DinoBlock(nn.Module):
    def __init__(self, dim: int, heads: int, n_prefix: int, ls_init: float = 1e-5):
        super().__init__()
        self.heads, self.n_prefix = heads, n_prefix
        self.norm1 = nn.LayerNorm(dim, eps=1e-5)
        self.qkv = nn.Linear(dim, dim * 3, bias=True)
        self.proj = nn.Linear(dim, dim)
        self.ls1 = nn.Parameter(ls_init * torch.ones(dim))
        self.norm2 = nn.LayerNorm(dim, eps=1e-5)
        self.mlp = nn.Sequential(nn.Linear(dim, 4 * dim), nn.GELU(), nn.Linear(4 * dim, dim))
        self.ls2 = nn.Parameter(ls_init * torch.ones(dim))

    def forward(self, x, cos, sin):
        B, L, D = x.shape
        qkv = self.qkv(self.norm1(x)).reshape(B, L, 3, self.heads, D // self.heads).permute(2, 0, 3, 1, 4)
        q, k, v = qkv[0], qkv[1], qkv[2]
        p = self.n_prefix
        q = torch.cat([q[:, :, :p], _apply_rope(q[:, :, p:], cos, sin)], dim=2)
        k = torch.cat([k[:, :, :p], _apply_rope(k[:, :, p:], cos, sin)], dim=2)
        a = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(B, L, D)
        x = x + self.ls1 * self.proj(a)
        return x + self.ls2 * self.mlp(self.norm2(x))


class DINOv3ViT(nn.Module):
    """ViT with a class token, register tokens, 2-D RoPE and LayerScale (DINOv3 layout)."""

    def __init__(self, img_size=224, patch_size=16, embed_dim=1024, depth=24, num_heads=16,
                 num_registers=4):
        super().__init__()
        self.grid = img_size // patch_size
        self.patch_embed = nn.Conv2d(3, embed_dim, kernel_size=patch_size, stride=patch_size)
        self.cls_token = nn.Parameter(torch.zeros(1, 1, embed_dim))
        self.reg_token = nn.Parameter(torch.zeros(1, num_registers, embed_dim))
        self.n_prefix = 1 + num_registers
        self.blocks = nn.ModuleList([_DinoBlock(embed_dim, num_heads, self.n_prefix) for _ in range(depth)])
        self.norm = nn.LayerNorm(embed_dim, eps=1e-5)
        self.head_dim = embed_dim // num_heads
        nn.init.trunc_normal_(self.cls_token, std=0.02)
        nn.init.trunc_normal_(self.reg_token, std=0.02)
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.trunc_normal_(m.weight, std=0.02)
                nn.init.zeros_(m.bias)

    def forward_features(self, x):
        B = x.shape[0]
        x = self.patch_embed(x).flatten(2).transpose(1, 2)
        x = torch.cat([self.cls_token.expand(B, -1, -1).to(x.dtype),
                       self.reg_token.expand(B, -1, -1).to(x.dtype), x], dim=1)
        cos, sin = _rope_tables(self.grid, self.head_dim, device=x.device)
        for blk in self.blocks:
            x = blk(x, cos, sin)
        return self.norm(x)

    def forward(self, x):
        return self.forward_features(x)[:, 0]


def dinov3_vit_l16() -> DINOv3ViT:
    return DINOv3ViT()

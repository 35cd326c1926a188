"""Import shims that let the reference package load in this container.

Used ONLY by make_golden.py, in the survey/build container (never on the GPU box).
The reference depends on packages that are absent here:

* timm 0.9.7 (`timm.models.vision_transformer.Block`) -- restated below from
  timm 0.9.7's published Block/Attention/Mlp semantics (pre-LN, fused SDPA,
  GELU(erf) MLP, dropout after attention probs / proj / GELU / fc2, no
  layer-scale, no drop-path).  State-dict names match timm.
* torchvision (only `save_image_grid` uses it), zarr (isinstance checks only),
  transformers CLIP (loaded by model NAME -> needs network).  These are stubbed.
"""
import sys
import types

import torch
import torch.nn as nn
import torch.nn.functional as F


class _Attention(nn.Module):
    def __init__(self, dim, num_heads=8, qkv_bias=False, attn_drop=0.0, proj_drop=0.0):
        super().__init__()
        self.num_heads = num_heads
        self.head_dim = dim // num_heads
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = nn.Linear(dim, dim)
        self.proj_drop = nn.Dropout(proj_drop)

    def forward(self, x):
        b, n, c = x.shape
        qkv = self.qkv(x).reshape(b, n, 3, self.num_heads, self.head_dim).permute(2, 0, 3, 1, 4)
        q, k, v = qkv.unbind(0)
        p = self.attn_drop.p if self.training else 0.0
        y = F.scaled_dot_product_attention(q, k, v, dropout_p=p)
        y = y.transpose(1, 2).reshape(b, n, c)
        return self.proj_drop(self.proj(y))


class _Mlp(nn.Module):
    def __init__(self, in_features, hidden_features, drop=0.0):
        super().__init__()
        self.fc1 = nn.Linear(in_features, hidden_features)
        self.act = nn.GELU()
        self.drop1 = nn.Dropout(drop)
        self.fc2 = nn.Linear(hidden_features, in_features)
        self.drop2 = nn.Dropout(drop)

    def forward(self, x):
        return self.drop2(self.fc2(self.drop1(self.act(self.fc1(x)))))


class Block(nn.Module):
    def __init__(self, dim, num_heads, mlp_ratio=4.0, qkv_bias=False, qk_norm=False,
                 proj_drop=0.0, attn_drop=0.0, init_values=None, drop_path=0.0,
                 act_layer=nn.GELU, norm_layer=nn.LayerNorm, mlp_layer=None):
        super().__init__()
        self.norm1 = norm_layer(dim)
        self.attn = _Attention(dim, num_heads, qkv_bias, attn_drop, proj_drop)
        self.norm2 = norm_layer(dim)
        self.mlp = _Mlp(dim, int(dim * mlp_ratio), proj_drop)

    def forward(self, x):
        x = x + self.attn(self.norm1(x))
        x = x + self.mlp(self.norm2(x))
        return x


def install(ref_root="/root/reference"):
    if ref_root not in sys.path:
        sys.path.insert(0, ref_root)
    timm = types.ModuleType("timm")
    timm_models = types.ModuleType("timm.models")
    vit = types.ModuleType("timm.models.vision_transformer")
    vit.Block = Block
    timm.models = timm_models
    timm_models.vision_transformer = vit
    sys.modules.setdefault("timm", timm)
    sys.modules.setdefault("timm.models", timm_models)
    sys.modules.setdefault("timm.models.vision_transformer", vit)

    tv = types.ModuleType("torchvision")
    tv.io = types.SimpleNamespace(write_video=None)
    sys.modules.setdefault("torchvision", tv)

    zarr = types.ModuleType("zarr")

    class _Array:  # isinstance() target only
        pass

    zarr.Array = _Array
    sys.modules.setdefault("zarr", zarr)

    lm = types.ModuleType("unified_video_action.utils.language_model")
    lm.get_text_model = lambda task_name, language_emb_model, model_path=None: (None, None, 30)
    lm.extract_text_features = lambda *a, **k: None
    sys.modules.setdefault("unified_video_action.utils.language_model", lm)

"""Shared building blocks for the detector models.

All models here are *inference-first*: every Conv+BatchNorm pair is a
:class:`ConvBNAct` that can fold its BatchNorm into the convolution weights
(:meth:`ConvBNAct.fuse`).  After folding, a layer is exactly
``act(conv(x, W') + b')`` which is what the hand-written MFMA convolution
kernel (``csrc/kernels/conv_mfma.hip``) consumes: NHWC bf16 activations,
[Cout][kh][kw][Cin] bf16 weights, fp32 bias, activation fused in the
epilogue.

Weights are random-initialised (there is no network access for checkpoints,
BASELINE.json: "random-init model weights"); ``seed_everything`` makes the
initialisation deterministic so that tests and benches are reproducible.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

ACT_NONE, ACT_RELU, ACT_SILU, ACT_LEAKY = 0, 1, 2, 3
_ACT_NAMES = {"none": ACT_NONE, "relu": ACT_RELU, "silu": ACT_SILU, "leaky": ACT_LEAKY}


def seed_everything(seed: int = 0) -> None:
    torch.manual_seed(seed)


def apply_act(x: torch.Tensor, act: int) -> torch.Tensor:
    if act == ACT_RELU:
        return F.relu(x)
    if act == ACT_SILU:
        return F.silu(x)
    if act == ACT_LEAKY:
        return F.leaky_relu(x, 0.1)
    return x


class ConvBNAct(nn.Module):
    """conv(k, s, p, groups=1, no bias) -> BatchNorm2d -> activation.

    ``fuse()`` replaces the BN by a conv bias (eval semantics)."""

    def __init__(self, c1: int, c2: int, k: int = 1, s: int = 1, p: Optional[int] = None,
                 act: str | int = "silu", bn: bool = True, bias: bool = False):
        super().__init__()
        if p is None:
            p = k // 2
        self.k, self.s, self.p = k, s, p
        self.conv = nn.Conv2d(c1, c2, k, s, p, bias=bias or not bn)
        self.bn = nn.BatchNorm2d(c2, eps=1e-3, momentum=0.03) if bn else None
        self.act = _ACT_NAMES[act] if isinstance(act, str) else int(act)
        self.fused = not bn

    @torch.no_grad()
    def randomize_bn(self, gen: Optional[torch.Generator] = None) -> None:
        """Give BN non-trivial running statistics so that folding is tested
        on realistic numbers (random-init weights otherwise leave BN as the
        identity)."""
        if self.bn is None:
            return
        c = self.bn.num_features
        self.bn.running_mean.copy_(torch.randn(c, generator=gen) * 0.1)
        self.bn.running_var.copy_(torch.rand(c, generator=gen) * 0.5 + 0.75)
        self.bn.weight.copy_(torch.rand(c, generator=gen) * 0.5 + 0.75)
        self.bn.bias.copy_(torch.randn(c, generator=gen) * 0.1)

    @torch.no_grad()
    def fuse(self) -> "ConvBNAct":
        if self.fused:
            return self
        bn = self.bn
        w = self.conv.weight
        scale = bn.weight / torch.sqrt(bn.running_var + bn.eps)
        b0 = self.conv.bias if self.conv.bias is not None else torch.zeros_like(bn.running_mean)
        new = nn.Conv2d(self.conv.in_channels, self.conv.out_channels, self.k, self.s, self.p, bias=True)
        new.weight.copy_(w * scale.view(-1, 1, 1, 1))
        new.bias.copy_((b0 - bn.running_mean) * scale + bn.bias)
        new = new.to(device=w.device, dtype=w.dtype)
        self.conv = new
        self.bn = None
        self.fused = True
        return self

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        y = self.conv(x)
        if self.bn is not None:
            y = self.bn(y)
        return apply_act(y, self.act)


def fuse_model(model: nn.Module) -> nn.Module:
    for m in model.modules():
        if isinstance(m, ConvBNAct):
            m.fuse()
        elif hasattr(m, "fuse_bn") and callable(m.fuse_bn):
            m.fuse_bn()
    return model


def randomize_bn(model: nn.Module, seed: int = 0) -> None:
    g = torch.Generator().manual_seed(seed)
    for m in model.modules():
        if isinstance(m, ConvBNAct):
            m.randomize_bn(g)
        elif isinstance(m, (nn.BatchNorm1d, nn.BatchNorm2d)):
            c = m.num_features
            with torch.no_grad():
                m.running_mean.copy_(torch.randn(c, generator=g) * 0.1)
                m.running_var.copy_(torch.rand(c, generator=g) * 0.5 + 0.75)
                m.weight.copy_(torch.rand(c, generator=g) * 0.5 + 0.75)
                m.bias.copy_(torch.randn(c, generator=g) * 0.1)


def kaiming_init(model: nn.Module) -> None:
    for m in model.modules():
        if isinstance(m, (nn.Conv2d, nn.ConvTranspose2d, nn.Linear)):
            nn.init.kaiming_uniform_(m.weight, a=math.sqrt(5))

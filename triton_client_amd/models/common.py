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

ACT_NONE, ACT_RELU, ACT_SILU, ACT_LEAKY, ACT_MISH = 0, 1, 2, 3, 4
_ACT_NAMES = {"none": ACT_NONE, "relu": ACT_RELU, "silu": ACT_SILU, "leaky": ACT_LEAKY, "mish": ACT_MISH,
              "linear": ACT_NONE}


def seed_everything(seed: int = 0) -> None:
    torch.manual_seed(seed)


def apply_act(x: torch.Tensor, act: int) -> torch.Tensor:
    if act == ACT_RELU:
        return F.relu(x)
    if act == ACT_SILU:
        return F.silu(x)
    if act == ACT_LEAKY:
        return F.leaky_relu(x, 0.1)
    if act == ACT_MISH:
        return F.mish(x)
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
    """He-normal (fan-in, ReLU gain) for every conv/linear.  PyTorch's default
    (kaiming_uniform, a=sqrt(5)) shrinks ReLU activations ~6x per layer, so a
    14-layer random BEV backbone collapses every anchor logit into a 0.06-wide
    band; He init keeps activations O(1) like a trained network, which makes
    the detection statistics (and hence the NMS work) realistic."""
    for m in model.modules():
        if isinstance(m, (nn.Conv2d, nn.Linear)):
            nn.init.kaiming_normal_(m.weight, mode="fan_in", nonlinearity="relu")
        elif isinstance(m, nn.ConvTranspose2d):
            # weight [Cin, Cout, k, k]; with k == stride every output pixel sums
            # exactly Cin taps, so the ReLU-preserving std is sqrt(2 / Cin).
            nn.init.normal_(m.weight, 0.0, math.sqrt(2.0 / m.weight.shape[0]))


@torch.no_grad()
def lsuv_rescale(model: nn.Module, run_forward, head_modules=(), head_std: float = 1.5, eps: float = 1e-8) -> int:
    """LSUV-style data-dependent rescaling of a random-init network.

    One forward pass with hooks: each conv's output std is measured on the
    sample data and its weight and bias are scaled so the output has unit
    std (``head_std`` for the detection heads), and the rescaled output is
    what the next layer sees.  This is what BatchNorm running statistics do
    for a trained network; without it a random detector's logits sit in a
    band far narrower than a trained model's, which makes the detection
    statistics (and hence the NMS workload) unrealistic.  Returns the number
    of layers rescaled."""
    heads = set(id(m) for m in head_modules)
    convs = [m for m in model.modules() if isinstance(m, (nn.Conv2d, nn.ConvTranspose2d))]
    seen = set()

    def hook(mod, inp, out):
        if id(mod) in seen:
            return None
        seen.add(id(mod))
        std = out.float().std().item()
        if not (std > eps):
            return None
        s = (head_std if id(mod) in heads else 1.0) / std
        mod.weight.mul_(s)
        if mod.bias is not None:
            mod.bias.mul_(s)
        return out * s

    handles = [c.register_forward_hook(hook) for c in convs]
    try:
        run_forward()
    finally:
        for h in handles:
            h.remove()
    return len(seen)


def broadcast_parameters(model: nn.Module, src: int = 0) -> None:
    """Make every rank's weights identical to rank ``src``'s (RCCL broadcast)."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    with torch.no_grad():
        for t in list(model.parameters()) + list(model.buffers()):
            dist.broadcast(t.data, src)

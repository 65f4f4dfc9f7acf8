"""Fused BEV neck + head (K15): weight permutation on the CPU, kernel vs fp32 on the GPU."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from triton_client_amd.ops.neck import chunk32_perm, permute_head_weight


def test_chunk_perm_is_the_accumulator_layout():
    p = chunk32_perm()
    assert sorted(p) == list(range(32))
    # lane group g, element e: e < 4 -> acc tile 2t (channels 4g..4g+3), else tile 2t+1 (16 + 4g..)
    for g in range(4):
        assert p[8 * g: 8 * g + 4] == [4 * g + e for e in range(4)]
        assert p[8 * g + 4: 8 * g + 8] == [16 + 4 * g + e for e in range(4)]


def test_permuted_head_contracts_to_the_same_result():
    torch.manual_seed(0)
    w = torch.randn(72, 384)
    x = torch.randn(5, 384)
    wp = permute_head_weight(w)
    assert wp.shape == (80, 384) and wp[72:].abs().sum() == 0
    # the kernel feeds x in accumulator order: position p of chunk c holds channel c*32 + perm[p]
    perm = chunk32_perm()
    idx = torch.tensor([c * 32 + perm[q] for c in range(12) for q in range(32)])
    got = x[:, idx] @ wp[:72].t()
    torch.testing.assert_close(got, x @ w.t(), rtol=1e-5, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("grid", [0, 8, 24])
def test_neck_head_kernel_vs_fp32(cuda, grid):
    from triton_client_amd.ops.conv import NHWC, FusedConv
    from triton_client_amd.ops.neck import FusedNeckHead

    torch.manual_seed(grid)
    B, H, W = 2, 72, 76  # quarter-res 18 x 19 = 342 pixels per class: a full and a partial tile
    dec = [nn.ConvTranspose2d(64, 128, 1, 1), nn.ConvTranspose2d(128, 128, 2, 2), nn.ConvTranspose2d(256, 128, 4, 4)]
    for d in dec:
        nn.init.normal_(d.weight, std=0.08)
        nn.init.normal_(d.bias, std=0.3)
    head = nn.Conv2d(384, 72, 1)
    nn.init.normal_(head.weight, std=0.05)
    ups = [FusedConv(d, act=1, device=cuda) for d in dec]
    fh = FusedConv(head, device=cuda)
    neck = FusedNeckHead(ups, [1, 2, 4], fh, cuda, grid=grid)
    x1 = torch.randn(B, H, W, 96)  # branch 1 reads channels [32, 96)
    x2 = torch.randn(B, H // 2, W // 2, 128)
    x3 = torch.randn(B, H // 4, W // 4, 256)
    xs = [NHWC(x1.to(cuda, torch.bfloat16), 32, 64), NHWC(x2.to(cuda, torch.bfloat16)),
          NHWC(x3.to(cuda, torch.bfloat16))]
    out = torch.full((B, H, W, 72), float("nan"), dtype=torch.bfloat16, device=cuda)
    neck(xs, NHWC(out))
    torch.cuda.synchronize()
    with torch.no_grad():
        ins = [x1[..., 32:], x2, x3]
        cat = torch.cat([F.relu(d(x.to(torch.bfloat16).float().permute(0, 3, 1, 2))) for d, x in zip(dec, ins)], 1)
        ref = head(cat).permute(0, 2, 3, 1)
    got = out.float().cpu()
    assert torch.isfinite(got).all()
    err = (got - ref).abs().max().item()
    assert err < 0.03 * max(1.0, ref.abs().max().item()), err

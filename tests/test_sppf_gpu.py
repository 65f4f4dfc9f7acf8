"""nhwc_ops.hip tca_sppf_pool3 (YOLOv5 SPPF's three chained 5x5 max-pools in one launch) against
three tca_maxpool_nhwc launches and against torch max_pool2d: the same clipped-window maxes, so
the same bits; channel-offset input and output slices, fp32 and bf16."""
import pytest
import torch
import torch.nn.functional as F

from triton_client_amd.ops.conv import NHWC, maxpool_nhwc, sppf_pools


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("hw", [(20, 20), (13, 17), (1, 9)])
def test_sppf_one_launch_matches_three_pools(cuda, dtype, hw):
    torch.manual_seed(hw[0])
    B, (H, W), cs = 3, hw, 64
    src = torch.randn(B, H, W, cs + 16, device=cuda).to(dtype)
    y0 = NHWC(src, 8, cs)
    one = torch.full((B, H, W, 4 * cs + 8), 7.0, device=cuda).to(dtype)
    sppf_pools(y0, one, cs, 5)
    three = torch.full_like(one, 7.0)
    y1 = maxpool_nhwc(y0, NHWC(three, cs, cs), 5)
    y2 = maxpool_nhwc(y1, NHWC(three, 2 * cs, cs), 5)
    maxpool_nhwc(y2, NHWC(three, 3 * cs, cs), 5)
    torch.cuda.synchronize()
    assert torch.equal(one[..., cs:4 * cs], three[..., cs:4 * cs])
    assert (one[..., :cs] == 7.0).all() and (one[..., 4 * cs:] == 7.0).all()
    x = src[..., 8:8 + cs].permute(0, 3, 1, 2).float()
    r = x
    for i in range(1, 4):
        r = F.max_pool2d(r, 5, 1, 2)
        assert torch.equal(one[..., i * cs:(i + 1) * cs].float(), r.permute(0, 2, 3, 1))

"""conv_wx3 (conv_hx3.hip): 3x3 stride-1 pair convolution as a Winograd F(2,3) along the
fragment axis.  CPU: the transformed weight image (ops/conv.py wx_weights) decoded and run
through the same transform equations reproduces the direct convolution.  GPU: both
orientations against fp64 (partial tiles, odd extents, channel-offset slices, a residual)."""
import copy

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from triton_client_amd.ops.conv import NHWC, FusedConv, from_pairs, to_pairs, wx_weights


def rel_l2(got, ref):
    got, ref = got.double().cpu(), ref.double().cpu()
    return ((got - ref).norm() / ref.norm().clamp_min(1e-30)).item()


def _unfrag(wf: torch.Tensor) -> torch.Tensor:
    """Inverse of frag_weights: [Kp/32][N/16][2][4][16][8] -> [N, Kp] (hi + lo, fp64)."""
    ks, g, _, fq, fr, e = wf.shape
    t = wf.double().sum(2)  # hi + lo: ks, g, fq, fr, e
    return t.permute(1, 3, 0, 2, 4).reshape(g * fr, ks * fq * e)


@pytest.mark.parametrize("cm", [False, True])
def test_wx_weights_transform_equations_cpu(cm):
    torch.manual_seed(int(cm))
    B, H, W, cin, cout = 1, 7, 10, 32, 16
    conv = nn.Conv2d(cin, cout, 3, 1, 1, bias=False).double()
    fc = FusedConv(copy.deepcopy(conv).float(), device="cpu", precision="fp32")
    U = _unfrag(wx_weights(fc.w_f32_gemm, fc.cin_p, cm)).reshape(cout, 3, 4, cin)  # n, kl, xi, ci
    x = torch.randn(B, cin, H, W, dtype=torch.float64)
    ref = conv(x)
    if cm:  # fragment axis = y: transpose so the fragment axis is the last one
        x, ref = x.transpose(2, 3), ref.transpose(2, 3)
    Hl, Wf = x.shape[2], x.shape[3]
    xp = F.pad(x, (1, 1 + Wf % 2, 1, 1))  # zero halo (+1 column for an odd extent's last pair)
    out = torch.zeros(B, cout, Hl, Wf + Wf % 2, dtype=torch.float64)
    for t in range(0, Wf, 2):  # pixel pair t, t + 1: inputs t - 1 .. t + 2 (padded index t .. t + 3)
        for kl in range(3):
            d = xp[:, :, kl:kl + Hl, t:t + 4]  # b, ci, line, k
            V = torch.stack([d[..., 0] - d[..., 2], d[..., 1] + d[..., 2], d[..., 2] - d[..., 1],
                             d[..., 1] - d[..., 3]], -1)  # b, ci, line, xi
            M = torch.einsum("bclx,nxc->bnlx", V, U[:, kl])
            out[:, :, :, t] += M[..., 0] + M[..., 1] + M[..., 2]
            out[:, :, :, t + 1] += M[..., 1] - M[..., 2] - M[..., 3]
    assert rel_l2(out[..., :Wf], ref) < 1e-5


SHAPES = [(2, 23, 31, 64, 128), (1, 21, 37, 256, 256), (3, 9, 16, 96, 128), (1, 62, 54, 128, 256), (2, 19, 50, 64, 64),
          (2, 13, 70, 32, 128), (1, 40, 33, 128, 128),
          # more tiles than CUs: persistent workgroups walk several tiles (and N tiles) each
          (5, 124, 108, 32, 128), (12, 62, 54, 32, 256), (4, 70, 100, 32, 64)]


@pytest.mark.gpu
@pytest.mark.parametrize("tile", [130, 131, 132])
@pytest.mark.parametrize("shape", SHAPES)
def test_wx3_vs_fp64(cuda, tile, shape):
    B, H, W, cin, cout = shape
    torch.manual_seed(tile + cin + cout + H)
    conv = nn.Conv2d(cin, cout, 3, 1, 1, bias=True).double()
    fc = FusedConv(copy.deepcopy(conv).float(), act=1, device=cuda, precision="fp32")
    assert fc.wx3_ok()
    buf = torch.randn(B, H, W, cin + 16, dtype=torch.float64)
    res = torch.randn(B, H, W, cout, dtype=torch.float64)
    x = NHWC(to_pairs(buf.float()).to(cuda), 8, cin, pair=True)
    r = NHWC(to_pairs(res.float()).to(cuda), pair=True)
    out = torch.full((B, H, W, cout + 16), 7.0, dtype=torch.float32, device=cuda)
    fc(x, out=NHWC(out, 8, cout, pair=True), res=r, tile=tile)
    torch.cuda.synchronize()
    assert (out[..., :8] == 7.0).all() and (out[..., 8 + cout:] == 7.0).all()
    ref = torch.relu(conv(buf[..., 8:8 + cin].permute(0, 3, 1, 2))) + from_pairs(r.t).double().cpu().permute(0, 3, 1, 2)
    got = NHWC(out, 8, cout, pair=True).nchw()
    assert rel_l2(got, ref) < 5e-5, rel_l2(got, ref)


@pytest.mark.gpu
def test_wx3_post_residual_act_no_bias(cuda):
    torch.manual_seed(3)
    B, H, W, cin, cout = 2, 17, 29, 64, 128
    conv = nn.Conv2d(cin, cout, 3, 1, 1, bias=False).double()
    fc = FusedConv(copy.deepcopy(conv).float(), act=1, device=cuda, precision="fp32", post_res=True)
    xin = torch.randn(B, H, W, cin, dtype=torch.float64)
    res = torch.randn(B, H, W, cout, dtype=torch.float64)
    for tile in (131, 132):
        out = NHWC(torch.empty(B, H, W, cout, device=cuda), pair=True)
        fc(NHWC(to_pairs(xin.float()).to(cuda), pair=True), out=out,
           res=NHWC(to_pairs(res.float()).to(cuda), pair=True), tile=tile)
        torch.cuda.synchronize()
        ref = torch.relu(conv(xin.permute(0, 3, 1, 2)) + from_pairs(to_pairs(res.float())).double().permute(0, 3, 1, 2))
        assert rel_l2(out.nchw(), ref) < 5e-5

"""conv_wino.hip: 3x3 stride-1 convolution by 1-D Winograd F(2,3) along the fragment axis
(the fp32-mode BEV backbone layers): the tap transform on the CPU (fp64 emulation of the
algorithm == the direct convolution), and the kernel against fp64 references for every tile,
pair / fp32 storage in and out, partial tiles, channel-offset slices and uniform-tile skipping."""
import copy

import numpy as np
import pytest
import torch
import torch.nn as nn

from triton_client_amd.ops.conv import NHWC, FusedConv, from_pairs, to_pairs, wino_taps, wino_tile


@pytest.fixture(autouse=True)
def _wino_all_widths(monkeypatch):
    """The kernel serves N = 64 too (the default routes only N >= 128 layers to it)."""
    from triton_client_amd.ops import conv as conv_mod
    monkeypatch.setattr(conv_mod, "WINO_MIN_N", 64)


def rel_l2(got, ref):
    got, ref = got.double().cpu(), ref.double().cpu()
    return ((got - ref).norm() / ref.norm().clamp_min(1e-30)).item()


def _wino_conv_fp64(x, V, cm):
    """x [B, Cin, H, W] fp64, V [N, 3, 4, Cin] (wino_taps) -> F(2,3) conv, fp64."""
    if cm:  # Winograd along y: run the x-axis algorithm on the transposed image
        return _wino_conv_fp64(x.transpose(2, 3), V, False).transpose(2, 3)
    B, C, H, W = x.shape
    Wp = (W + 1) // 2 * 2
    xp = torch.nn.functional.pad(x, (1, Wp - W + 1, 1, 1))  # pad 1 all round, + odd-width column
    out = torch.zeros(B, V.shape[0], H, Wp, dtype=torch.float64)
    for kl in range(3):
        rows = xp[:, :, kl:kl + H]  # input line i + kl for output line i
        d = [rows[:, :, :, j:j + Wp - 1:2] for j in range(4)]  # tile t: input 2t - 1 + j (padded index 2t + j)
        U = [d[0] - d[2], d[1] + d[2], d[2] - d[1], d[1] - d[3]]
        m = [torch.einsum("bchw,nc->bnhw", U[p], V[:, kl, p]) for p in range(4)]
        out[..., 0::2] += m[0] + m[1] + m[2]
        out[..., 1::2] += m[1] - m[2] - m[3]
    return out[..., :W]


@pytest.mark.parametrize("cm", [False, True])
def test_wino_taps_fp64_equals_direct_conv(cm):
    torch.manual_seed(1)
    conv = nn.Conv2d(16, 8, 3, 1, 1, bias=False).double()
    x = torch.randn(2, 16, 7, 9, dtype=torch.float64)
    Wg = conv.weight.detach().permute(0, 2, 3, 1).reshape(8, 9 * 16)  # (ky * 3 + kx) * cin + ci
    got = _wino_conv_fp64(x, wino_taps(Wg, 16, cm), cm)
    np.testing.assert_allclose(got.numpy(), conv(x).detach().numpy(), rtol=1e-12, atol=1e-12)


def test_wino_tile_orientation():
    assert wino_tile(248, 216, 64) == 4 and wino_tile(124, 108, 128) == 2 and wino_tile(62, 54, 256) == 2
    assert wino_tile(20, 64, 64) == 3 and wino_tile(20, 64, 128) == 1


SHAPES = [(2, 23, 31, 64, 128), (1, 21, 37, 256, 256), (2, 19, 50, 64, 64), (3, 9, 16, 96, 128),
          (2, 8, 16, 32, 64), (1, 62, 54, 128, 256), (1, 33, 65, 64, 64)]


@pytest.mark.gpu
@pytest.mark.parametrize("tile", [130, 131, 132, 133, 134])
@pytest.mark.parametrize("shape", SHAPES)
def test_wino_tiles_vs_fp64(cuda, tile, shape):
    """Pair in / out with channel-offset slices, partial tiles along both axes, odd chunk counts
    (Cin 96) and ReLU, against fp64 (the fp32-mode budget of tests/test_fp32_mode_gpu.py); the
    channels outside the output slice stay untouched; close to hx3 (tile 110)."""
    B, H, W, cin, cout = shape
    if tile in (131, 132) and cout % 128:
        pytest.skip("128-channel tiles need N % 128 == 0")
    torch.manual_seed(tile + cin + cout)
    conv = nn.Conv2d(cin, cout, 3, 1, 1, bias=True).double()
    fc = FusedConv(copy.deepcopy(conv).float(), act=1, device=cuda, precision="fp32")
    assert fc.wino_ok()
    buf = torch.relu(torch.randn(B, H, W, cin + 16, dtype=torch.float64))
    x = NHWC(to_pairs(buf.float()).to(cuda), 8, cin, pair=True)
    outs = {}
    for t in (tile, 110):
        out = torch.full((B, H, W, cout + 16), 7.0, dtype=torch.float32, device=cuda)
        fc(x, out=NHWC(out, 8, cout, pair=True), tile=t)
        torch.cuda.synchronize()
        outs[t] = out
        assert (out[..., :8] == 7.0).all() and (out[..., 8 + cout:] == 7.0).all()
    ref = torch.relu(conv(buf[..., 8:8 + cin].permute(0, 3, 1, 2)))
    got = NHWC(outs[tile], 8, cout, pair=True).nchw()
    assert rel_l2(got, ref) < 5e-5, rel_l2(got, ref)
    hx = NHWC(outs[110], 8, cout, pair=True).nchw()
    assert rel_l2(got, hx) < 5e-5, rel_l2(got, hx)


@pytest.mark.gpu
@pytest.mark.parametrize("pin,pout", [(0, 0), (0, 1), (1, 0)])
def test_wino_fp32_storage(cuda, pin, pout):
    """fp32 NHWC storage in and / or out (the backbone chain between stride-2 layers)."""
    from triton_client_amd import _native
    from triton_client_amd.ops.conv import wino_weights

    torch.manual_seed(7 + pin * 2 + pout)
    B, H, W, cin, cout = 2, 30, 27, 128, 128
    conv = nn.Conv2d(cin, cout, 3, 1, 1, bias=True).double()
    fc = FusedConv(copy.deepcopy(conv).float(), act=1, device=cuda, precision="fp32")
    xin = torch.relu(torch.randn(B, H, W, cin, dtype=torch.float64))
    xt = (to_pairs(xin.float()) if pin else xin.float()).to(cuda)
    out = torch.empty(B, H, W, cout, dtype=torch.float32, device=cuda)
    for t in (1, 2):
        wf = wino_weights(fc.w_f32_gemm, cin, t == 2).to(cuda)
        _native.call("tca_conv_wino", _native.ptr(xt), B, H, W, cin, cin, 0, pin, _native.ptr(wf),
                     _native.ptr(fc.b_gemm), cout, _native.ptr(out), cout, 0, pout, 1, None, 0, None, t,
                     _native.stream_ptr(None))
        torch.cuda.synchronize()
        got = (from_pairs(out) if pout else out).double().cpu().permute(0, 3, 1, 2)
        ref = torch.relu(conv(xin.permute(0, 3, 1, 2)))
        assert rel_l2(got, ref) < 5e-5, (t, rel_l2(got, ref))


@pytest.mark.gpu
def test_wino_uniform_tiles(cuda):
    """Uniform-tile skipping: tiles whose pixels all reach uni_min store uni_val; the rest are
    computed (the same pixels as without the depth map)."""
    torch.manual_seed(5)
    B, H, W, c = 2, 40, 36, 64
    conv = nn.Conv2d(c, c, 3, 1, 1, bias=True).double()
    fc = FusedConv(copy.deepcopy(conv).float(), act=1, device=cuda, precision="fp32")
    xin = torch.relu(torch.randn(B, H, W, c, dtype=torch.float64))
    x = NHWC(to_pairs(xin.float()).to(cuda), pair=True)
    depth = torch.zeros(B, H, W, dtype=torch.uint8)
    depth[0] = 3  # image 0: every tile uniform
    depth[1, :, 20:] = 3  # image 1: a band of uniform pixels
    val = to_pairs(torch.arange(c, dtype=torch.float32).view(1, c)).view(c).to(cuda)
    full = NHWC(torch.empty(B, H, W, c, device=cuda), pair=True)
    skip = NHWC(torch.empty(B, H, W, c, device=cuda), pair=True)
    fc(x, out=full, tile=130)
    fc(x, out=skip, tile=130, uni=(depth.to(cuda), 2, val))
    torch.cuda.synchronize()
    f, s = from_pairs(full.t).cpu(), from_pairs(skip.t).cpu()
    assert torch.equal(s[0], torch.arange(c, dtype=torch.float32).expand(H, W, c))
    # image 1: tiles that touch a non-uniform pixel are computed exactly as without the map
    computed = ~torch.isclose(s[1], torch.arange(c, dtype=torch.float32).expand(H, W, c)).all(-1)
    assert computed[:, :16].all()
    assert torch.equal(s[1][computed], f[1][computed])

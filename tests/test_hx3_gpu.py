"""conv_hx3.hip: halo-tiled 3x3 stride-1 pair convolution with register-streamed
fragment-order weights (the fp32-mode BEV backbone layers), against fp64
references, and close to the conv_mfma.hip halo kernel (same products)."""
import copy

import pytest
import torch
import torch.nn as nn

from triton_client_amd.ops.conv import NHWC, FusedConv, frag_weights, from_pairs, split_bf16, to_pairs


def rel_l2(got, ref):
    got, ref = got.double().cpu(), ref.double().cpu()
    return ((got - ref).norm() / ref.norm().clamp_min(1e-30)).item()


def test_frag_weights_layout_cpu():
    """Block (ks, g, h), lane fq * 16 + fr, element e holds W[16 g + fr, 32 ks + 8 fq + e] (hi / lo)."""
    torch.manual_seed(0)
    N, Kp = 48, 96
    W = torch.randn(N, Kp)
    wf = frag_weights(W)
    assert wf.shape == (Kp // 32, N // 16, 2, 4, 16, 8) and wf.dtype == torch.bfloat16
    hi, lo = split_bf16(W)
    for ks, g, fq, fr, e in [(0, 0, 0, 0, 0), (2, 1, 3, 15, 7), (1, 2, 1, 7, 3)]:
        n, k = 16 * g + fr, 32 * ks + 8 * fq + e
        assert wf[ks, g, 0, fq, fr, e] == hi[n, k] and wf[ks, g, 1, fq, fr, e] == lo[n, k]


SHAPES = [(2, 23, 31, 64, 128), (1, 21, 37, 256, 256), (2, 19, 50, 64, 64), (3, 9, 16, 96, 128),
          (2, 8, 16, 32, 64), (1, 62, 54, 128, 256)]


@pytest.mark.gpu
@pytest.mark.parametrize("tile", [110, 111, 112, 113, 114, 115, 116])
@pytest.mark.parametrize("shape", SHAPES)
def test_hx3_tiles_vs_fp64(cuda, tile, shape):
    """Channel-offset input / output slices, partial row and column tiles, odd
    chunk counts (Cin 96), a pair residual and ReLU, against fp64; the channels
    outside the output slice stay untouched; and agreement with the halo kernel
    of conv_mfma.hip (tile 90: the same products in another summation order)."""
    B, H, W, cin, cout = shape
    if tile in (111, 112) and cout % 128:
        pytest.skip("128-channel tiles need N % 128 == 0")
    torch.manual_seed(tile + cin + cout)
    conv = nn.Conv2d(cin, cout, 3, 1, 1, bias=True).double()
    fc = FusedConv(copy.deepcopy(conv).float(), act=1, device=cuda, precision="fp32")
    assert fc.hx3_ok()
    buf = torch.randn(B, H, W, cin + 16, dtype=torch.float64)
    res = torch.randn(B, H, W, cout, dtype=torch.float64)
    x = NHWC(to_pairs(buf.float()).to(cuda), 8, cin, pair=True)
    r = NHWC(to_pairs(res.float()).to(cuda), pair=True)
    outs = {}
    for t in (tile, 90):
        out = torch.full((B, H, W, cout + 16), 7.0, dtype=torch.float32, device=cuda)
        fc(x, out=NHWC(out, 8, cout, pair=True), res=r, tile=t)
        torch.cuda.synchronize()
        outs[t] = out
        assert (out[..., :8] == 7.0).all() and (out[..., 8 + cout:] == 7.0).all()
    ref = torch.relu(conv(buf[..., 8:8 + cin].permute(0, 3, 1, 2))) + from_pairs(r.t).double().cpu().permute(0, 3, 1, 2)
    got = NHWC(outs[tile], 8, cout, pair=True).nchw()
    assert rel_l2(got, ref) < 5e-5, rel_l2(got, ref)
    hx = NHWC(outs[90], 8, cout, pair=True).nchw()
    assert rel_l2(got, hx) < 2e-5, rel_l2(got, hx)


@pytest.mark.gpu
def test_hx3_post_residual_act_and_no_bias(cuda):
    """act(conv + residual) (the ResNet form, act flag | 16) and a bias-free conv."""
    torch.manual_seed(3)
    B, H, W, cin, cout = 2, 17, 29, 64, 128
    conv = nn.Conv2d(cin, cout, 3, 1, 1, bias=False).double()
    fc = FusedConv(copy.deepcopy(conv).float(), act=1, device=cuda, precision="fp32", post_res=True)
    xin = torch.randn(B, H, W, cin, dtype=torch.float64)
    res = torch.randn(B, H, W, cout, dtype=torch.float64)
    out = NHWC(torch.empty(B, H, W, cout, device=cuda), pair=True)
    fc(NHWC(to_pairs(xin.float()).to(cuda), pair=True), out=out, res=NHWC(to_pairs(res.float()).to(cuda), pair=True),
       tile=110)
    torch.cuda.synchronize()
    ref = torch.relu(conv(xin.permute(0, 3, 1, 2)) + from_pairs(to_pairs(res.float())).double().permute(0, 3, 1, 2))
    assert rel_l2(out.nchw(), ref) < 5e-5


@pytest.mark.gpu
def test_wino_is_the_default_for_pair_backbone_layers(cuda, monkeypatch):
    """tile 0 routes an eligible stride-1 pair conv to conv_wino.hip F(2,3) (the same bits as
    tile 130), and to hx3 (tile 110) with ops.conv.WINO off."""
    from triton_client_amd.ops import conv as conv_mod
    torch.manual_seed(5)
    B, H, W, cin, cout = 2, 20, 24, 128, 128
    fc = FusedConv(nn.Conv2d(cin, cout, 3, 1, 1), act=1, device=cuda, precision="fp32")
    x = NHWC(to_pairs(torch.randn(B, H, W, cin)).to(cuda), pair=True)
    a = NHWC(torch.empty(B, H, W, cout, device=cuda), pair=True)
    b = NHWC(torch.empty(B, H, W, cout, device=cuda), pair=True)
    fc(x, out=a, tile=0)
    fc(x, out=b, tile=130)
    torch.cuda.synchronize()
    assert torch.equal(a.t, b.t)
    monkeypatch.setattr(conv_mod, "WINO", False)
    fc(x, out=a, tile=0)
    fc(x, out=b, tile=110)
    torch.cuda.synchronize()
    assert torch.equal(a.t, b.t)


# stride 2: odd and even extents (partial tiles, the bottom / right halo past the image)
S2_SHAPES = [(2, 23, 31, 64, 128), (1, 48, 34, 64, 64), (2, 19, 50, 128, 256), (3, 16, 32, 96, 64),
             (1, 124, 108, 128, 256)]


@pytest.mark.gpu
@pytest.mark.parametrize("tile", [120, 121, 122, 123, 124])
@pytest.mark.parametrize("shape", S2_SHAPES)
def test_hx3s2_tiles_vs_fp64(cuda, tile, shape):
    """3x3 stride-2 phase kernel: channel-offset slices, a pair residual and ReLU against
    fp64, untouched channels outside the output slice, and agreement with the xb
    implicit-GEMM kernel (tile 73) on the same split products."""
    B, H, W, cin, cout = shape
    if tile in (121, 122) and cout % 128:
        pytest.skip("128-channel tiles need N % 128 == 0")
    torch.manual_seed(tile + cin + cout + H)
    conv = nn.Conv2d(cin, cout, 3, 2, 1, bias=True).double()
    fc = FusedConv(copy.deepcopy(conv).float(), act=1, device=cuda, precision="fp32")
    assert fc.hx3_ok()
    Ho, Wo = fc.out_hw(H, W)
    buf = torch.randn(B, H, W, cin + 16, dtype=torch.float64)
    res = torch.randn(B, Ho, Wo, cout, dtype=torch.float64)
    x = NHWC(to_pairs(buf.float()).to(cuda), 8, cin, pair=True)
    r = NHWC(to_pairs(res.float()).to(cuda), pair=True)
    outs = {}
    for t in (tile, 73):
        out = torch.full((B, Ho, Wo, cout + 16), 7.0, dtype=torch.float32, device=cuda)
        fc(x, out=NHWC(out, 8, cout, pair=True), res=r, tile=t)
        torch.cuda.synchronize()
        outs[t] = out
        assert (out[..., :8] == 7.0).all() and (out[..., 8 + cout:] == 7.0).all()
    ref = torch.relu(conv(buf[..., 8:8 + cin].permute(0, 3, 1, 2))) + from_pairs(r.t).double().cpu().permute(0, 3, 1, 2)
    got = NHWC(outs[tile], 8, cout, pair=True).nchw()
    assert rel_l2(got, ref) < 5e-5, rel_l2(got, ref)
    xb = NHWC(outs[73], 8, cout, pair=True).nchw()
    assert rel_l2(got, xb) < 2e-5, rel_l2(got, xb)


@pytest.mark.gpu
@pytest.mark.parametrize("tile", [120, 123, 124])
def test_hx3s2_occupancy_reads_unmarked_pixels_as_zero(cuda, tile):
    """The sparse-canvas form: garbage in the unmarked pixels, occupancy 0 there; the
    result equals the conv of the masked input (and the default route takes it)."""
    torch.manual_seed(11)
    B, H, W, cin, cout = 2, 50, 38, 64, 64
    conv = nn.Conv2d(cin, cout, 3, 2, 1, bias=True).double()
    fc = FusedConv(copy.deepcopy(conv).float(), act=1, device=cuda, precision="fp32")
    occ = (torch.rand(B, H, W) < 0.1).to(torch.uint8)
    xin = torch.randn(B, H, W, cin, dtype=torch.float64)
    garbage = torch.full_like(xin, 1e6)
    stored = torch.where(occ.bool()[..., None], xin, garbage)
    x = NHWC(to_pairs(stored.float()).to(cuda), pair=True, occ=occ.to(cuda))
    Ho, Wo = fc.out_hw(H, W)
    out = NHWC(torch.empty(B, Ho, Wo, cout, device=cuda), pair=True)
    fc(x, out=out, tile=tile)
    dflt = NHWC(torch.empty(B, Ho, Wo, cout, device=cuda), pair=True)
    fc(x, out=dflt)
    torch.cuda.synchronize()
    ref = torch.relu(conv((xin * occ[..., None].double()).permute(0, 3, 1, 2)))
    assert rel_l2(out.nchw(), ref) < 5e-5, rel_l2(out.nchw(), ref)
    assert rel_l2(dflt.nchw(), ref) < 5e-5


@pytest.mark.gpu
@pytest.mark.parametrize("tile", [120, 123, 124])
@pytest.mark.parametrize("pattern", ["random", "arcs"])
def test_hx3s2_occupancy_skips_are_exact(cuda, tile, pattern):
    """Occupancy-gated stride-2 conv (empty tiles and empty line fragments skipped) against the
    same kernel reading the zero-masked input without occupancy: bit-identical."""
    torch.manual_seed(12)
    B, H, W, cin, cout = 2, 96, 80, 64, 64
    conv = nn.Conv2d(cin, cout, 3, 2, 1, bias=True)
    fc = FusedConv(conv, act=1, device=cuda, precision="fp32")
    if pattern == "random":
        occ = (torch.rand(B, H, W) < 0.08).to(torch.uint8)
    else:  # thin rings around a corner, like a LiDAR's ground returns: most line fragments empty
        yy, xx = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
        r = ((yy - 5.0) ** 2 + (xx + 3.0) ** 2).sqrt()
        occ = ((r % 23.0) < 1.2).to(torch.uint8).expand(B, H, W).contiguous()
        occ[1, 40:, :] = 0
    xin = torch.randn(B, H, W, cin) * occ[..., None]
    stored = torch.where(occ.bool()[..., None], xin, torch.full_like(xin, 3e4))
    x_occ = NHWC(to_pairs(stored).to(cuda), pair=True, occ=occ.to(cuda))
    x_dense = NHWC(to_pairs(xin).to(cuda), pair=True)
    Ho, Wo = fc.out_hw(H, W)
    outs = []
    for x in (x_occ, x_dense):
        o = NHWC(torch.full((B, Ho, Wo, cout), float("nan"), device=cuda), pair=True)
        fc(x, out=o, tile=tile)
        outs.append(o.t)
    torch.cuda.synchronize()
    assert torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32))


@pytest.mark.gpu
@pytest.mark.parametrize("tile", [120, 121, 124])
def test_hx3s2_fp32_storage_out(cuda, tile):
    """act flag 32: the stride-2 kernel writes fp32 storage (the input of an F(2,3) layer, see
    models/fast.py _BEVBackbonePlan.out_pair): the same accumulators as the pair output, so the
    two decode to within the hi / lo split error, and the fp32 tile meets the fp64 budget."""
    torch.manual_seed(11)
    B, H, W, cin, cout = 2, 37, 29, 64, 128
    conv = nn.Conv2d(cin, cout, 3, 2, 1, bias=True).double()
    fc = FusedConv(copy.deepcopy(conv).float(), act=1, device=cuda, precision="fp32")
    x = NHWC(to_pairs(torch.randn(B, H, W, cin)).to(cuda), pair=True)
    Ho, Wo = fc.out_hw(H, W)
    op = NHWC(torch.empty(B, Ho, Wo, cout, device=cuda), pair=True)
    of = NHWC(torch.empty(B, Ho, Wo, cout, device=cuda), pair=False)
    fc(x, out=op, tile=tile)
    fc(x, out=of, tile=tile)
    torch.cuda.synchronize()
    assert rel_l2(op.nchw(), of.t.permute(0, 3, 1, 2)) < 2e-5
    ref = torch.relu(conv(from_pairs(x.t).double().cpu().permute(0, 3, 1, 2)))
    assert rel_l2(of.t.permute(0, 3, 1, 2), ref) < 5e-5


@pytest.mark.gpu
@pytest.mark.parametrize("tile", [140, 141, 142])
@pytest.mark.parametrize("cin", [32, 64])
@pytest.mark.parametrize("pattern", ["random", "arcs", "empty"])
def test_s2sp_sparse_gather_conv(cuda, tile, cin, pattern, monkeypatch):
    """conv_s2sp.hip (tiles 140-142; the route over an occupancy-marked canvas when S2SP): garbage in the
    unmarked cells; channel-offset input / output slices; partial 8 x 32 tiles; against fp64 on
    the masked input; close to the dense hx3s2 kernel (same split products, another order) and
    bit-identical to it on pixels whose window is empty; bit-reproducible run to run; fp32
    storage out (act | 32) decodes to the pair output."""
    torch.manual_seed(13 + cin)
    B, H, W, cout = 2, 70, 90, 64
    conv = nn.Conv2d(cin, cout, 3, 2, 1, bias=True).double()
    fc = FusedConv(copy.deepcopy(conv).float(), act=1, device=cuda, precision="fp32")
    assert fc.s2sp_ok()
    from triton_client_amd.ops import conv as conv_mod
    monkeypatch.setattr(conv_mod, "S2SP", True)
    if pattern == "random":
        occ = (torch.rand(B, H, W) < 0.05).to(torch.uint8)
    elif pattern == "arcs":
        yy, xx = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
        r = ((yy - 5.0) ** 2 + (xx + 3.0) ** 2).sqrt()
        occ = ((r % 17.0) < 1.5).to(torch.uint8).expand(B, H, W).contiguous()
        occ[1, :, 50:] = 0
    else:
        occ = torch.zeros(B, H, W, dtype=torch.uint8)
    xin = torch.randn(B, H, W, cin, dtype=torch.float64) * occ[..., None].double()
    stored = torch.where(occ.bool()[..., None], xin, torch.full_like(xin, 1e6))
    buf = torch.zeros(B, H, W, cin + 16)
    buf[..., 8:8 + cin] = stored.float()
    x = NHWC(to_pairs(buf).to(cuda), 8, cin, pair=True, occ=occ.to(cuda))
    Ho, Wo = fc.out_hw(H, W)
    outs = []
    for t in (tile, tile, 0 if tile == 140 else tile):
        o = torch.full((B, Ho, Wo, cout + 16), 7.0, dtype=torch.float32, device=cuda)
        fc(x, out=NHWC(o, 8, cout, pair=True), tile=t)
        outs.append(o)
    dense = torch.full((B, Ho, Wo, cout + 16), 7.0, dtype=torch.float32, device=cuda)
    fc(x, out=NHWC(dense, 8, cout, pair=True), tile=120)
    of = NHWC(torch.empty(B, Ho, Wo, cout, device=cuda), pair=False)
    fc(x, out=of, tile=tile)
    torch.cuda.synchronize()
    o = outs[0]
    assert (o[..., :8] == 7.0).all() and (o[..., 8 + cout:] == 7.0).all()
    assert torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32))  # reproducible
    assert torch.equal(outs[0].view(torch.int32), outs[2].view(torch.int32))  # the default route
    ref = torch.relu(conv(xin.permute(0, 3, 1, 2)))
    got = NHWC(o, 8, cout, pair=True).nchw()
    assert rel_l2(got, ref) < 5e-5, rel_l2(got, ref)
    dn = NHWC(dense, 8, cout, pair=True).nchw()
    assert rel_l2(got, dn) < 2e-6, rel_l2(got, dn)
    # pixels whose 3 x 3 stride-2 window holds no occupied cell: act(bias), bit for bit
    win = torch.nn.functional.max_pool2d(occ.float()[:, None], 3, 2, 1)[:, 0] > 0
    empty = (~win).to(cuda)
    assert torch.equal(o[..., 8:8 + cout][empty].view(torch.int32), dense[..., 8:8 + cout][empty].view(torch.int32))
    assert rel_l2(got, of.t.permute(0, 3, 1, 2)) < 2e-5

"""fp32 mode's pair activation storage ({hi | lo} bf16 halves per 8 channels,
read by the split-product kernels as MFMA fragments without a VALU split):
the pair conv / neck kernels vs fp64 references, and a pair-storage BEV plan
bit-identical to the plain-fp32 plan (same hi / lo operands, same tiles)."""
import copy
import dataclasses

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from triton_client_amd.ops.conv import NHWC, FusedConv, from_pairs, to_pairs

pytestmark = pytest.mark.gpu

ACTS = {0: lambda t: t, 1: torch.relu}


def rel_l2(got, ref):
    got, ref = got.double().cpu(), ref.double().cpu()
    return ((got - ref).norm() / ref.norm().clamp_min(1e-30)).item()


def test_pairs_roundtrip_cpu():
    x = torch.randn(2, 3, 5, 64)
    p = to_pairs(x)
    assert p.dtype == torch.float32 and p.shape == x.shape
    assert ((from_pairs(p) - x).abs() <= x.abs() * 2 ** -16).all()


@pytest.mark.parametrize("tile", [0, 20, 22, 24, 25, 41, 70, 71, 72])
@pytest.mark.parametrize("out_pair", [True, False])
def test_conv_pair_vs_fp64(cuda, tile, out_pair):
    torch.manual_seed(tile)
    B, H, W, cin, cout = 2, 23, 31, 64, 128
    conv = nn.Conv2d(cin, cout, 3, 1, 1, bias=True).double()
    fc = FusedConv(copy.deepcopy(conv).float(), act=1, device=cuda, precision="fp32")
    buf = torch.randn(B, H, W, cin + 16, dtype=torch.float64)
    xin = buf[..., 8:8 + cin]
    out = torch.zeros(B, H, W, cout + 16, dtype=torch.float32, device=cuda)
    fc(NHWC(to_pairs(buf.float()).to(cuda), 8, cin, pair=True), out=NHWC(out, 8, cout, pair=out_pair), tile=tile)
    torch.cuda.synchronize()
    ref = torch.relu(conv(xin.permute(0, 3, 1, 2)))
    got = NHWC(out, 8, cout, pair=out_pair).nchw()
    assert rel_l2(got, ref) < 5e-5
    assert out[..., :8].abs().sum().item() == 0 and out[..., 8 + cout:].abs().sum().item() == 0


XB_TWINS = [(70, 25), (71, 26), (72, 32), (73, 20), (74, 25), (75, 26), (76, 37), (77, 22), (78, 70), (79, 71), (68, 42), (69, 41)]


@pytest.mark.parametrize("xb,glds", XB_TWINS)
@pytest.mark.parametrize("shape", [(2, 23, 31, 64, 128, 3, 1, 1), (3, 17, 12, 32, 64, 3, 2, 1),
                                   (2, 9, 14, 128, 72, 1, 1, 0), (1, 40, 33, 96, 256, 3, 1, 1)])
def test_conv_pair_xb_bit_identical_to_glds(cuda, xb, glds, shape):
    """The buffer-descriptor kernels (zero fill by range check, periodic swizzle)
    run the glds kernels' K order and MFMA sequence: identical bits, including
    padding taps, partial M / N tiles, stride 2, 1x1 and a residual."""
    torch.manual_seed(xb)
    B, H, W, cin, cout, k, s, pad = shape
    conv = nn.Conv2d(cin, cout, k, s, pad, bias=True)
    fc = FusedConv(conv, act=1, device=cuda, precision="fp32", post_res=True)
    x = NHWC(to_pairs(torch.randn(B, H, W, cin + 8)).to(cuda), 8, cin, pair=True)
    Ho, Wo = (H + 2 * pad - k) // s + 1, (W + 2 * pad - k) // s + 1
    r = NHWC(to_pairs(torch.randn(B, Ho, Wo, cout)).to(cuda), pair=True)
    outs = []
    for t in (xb, glds):
        o = NHWC(torch.full((B, Ho, Wo, cout + 8), 7.0, device=cuda), 0, cout, pair=True)
        fc(x, out=o, res=r, tile=t)
        outs.append(o.t.clone())
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    assert (outs[0][..., cout:] == 7.0).all()


XB_F32_TWINS = [(80, 20), (81, 41), (82, 25), (83, 26), (84, 22), (85, 24), (86, 42), (87, 47)]


@pytest.mark.parametrize("xb,glds", XB_F32_TWINS)
@pytest.mark.parametrize("shape", [(2, 23, 31, 64, 128, 3, 1, 1), (3, 17, 12, 32, 64, 3, 2, 1),
                                   (2, 9, 14, 128, 72, 1, 1, 0)])
def test_conv_fp32_xb_bit_identical_to_glds(cuda, xb, glds, shape):
    """fp32-input xb kernels (split at the fragment read, the camera chain's form)
    == their glds twins, bit for bit, fp32 and SiLU with a pre-activation residual."""
    torch.manual_seed(xb)
    B, H, W, cin, cout, k, s, pad = shape
    conv = nn.Conv2d(cin, cout, k, s, pad, bias=True)
    fc = FusedConv(conv, act=2, device=cuda, precision="fp32")
    x = NHWC(torch.randn(B, H, W, cin + 8, device=cuda), 8, cin)
    Ho, Wo = (H + 2 * pad - k) // s + 1, (W + 2 * pad - k) // s + 1
    r = NHWC(torch.randn(B, Ho, Wo, cout, device=cuda))
    outs = []
    for t in (xb, glds):
        o = NHWC(torch.full((B, Ho, Wo, cout + 8), 7.0, device=cuda), 8, cout)
        fc(x, out=o, res=r, tile=t)
        outs.append(o.t.clone())
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    assert (outs[0][..., :8] == 7.0).all()


def test_conv_pair_residual_and_deconv_shuffle(cuda):
    torch.manual_seed(1)
    B, H, W = 2, 12, 10
    conv = nn.Conv2d(64, 64, 3, 1, 1).double()
    fc = FusedConv(copy.deepcopy(conv).float(), act=1, device=cuda, precision="fp32", post_res=True)
    x = torch.randn(B, H, W, 64, dtype=torch.float64)
    r = torch.randn(B, H, W, 64, dtype=torch.float64)
    out = NHWC(torch.zeros(B, H, W, 64, device=cuda), pair=True)
    fc(NHWC(to_pairs(x.float()).to(cuda), pair=True), out=out, res=NHWC(to_pairs(r.float()).to(cuda), pair=True))
    ref = torch.relu(conv(x.permute(0, 3, 1, 2)) + r.permute(0, 3, 1, 2))
    assert rel_l2(out.nchw(), ref) < 5e-5
    up = nn.ConvTranspose2d(64, 128, 2, stride=2).double()
    fu = FusedConv(copy.deepcopy(up).float(), act=1, device=cuda, precision="fp32")
    o2 = NHWC(torch.zeros(B, 2 * H, 2 * W, 128 + 64, device=cuda), 64, 128, pair=True)
    fu(NHWC(to_pairs(x.float()).to(cuda), pair=True), out=o2)
    ref2 = torch.relu(up(x.permute(0, 3, 1, 2)))
    assert rel_l2(o2.nchw(), ref2) < 5e-5


def test_bev_plan_pair_equals_fp32_plan(cuda):
    """Pair storage feeds the MFMAs the same hi / lo halves the fp32 plan splits
    at its fragment reads.  The pair plan's wide 3x3 stride-1 layers take the
    halo-tiled kernel (same products, (chunk, tap) summation order), so the two
    plans agree to fp32 rounding; a plain canvas converted on entry matches the
    pair canvas bit for bit."""
    from triton_client_amd.config.lidar import KITTI_PILLARS, PointPillarsConfig
    from triton_client_amd.models.common import fuse_model, randomize_bn
    from triton_client_amd.models.fast import FastBEV
    from triton_client_amd.models.pointpillars import build_pointpillars

    v = dataclasses.replace(KITTI_PILLARS, point_cloud_range=(0.0, -10.24, -3.0, 20.48, 10.24, 1.0))
    m = build_pointpillars(PointPillarsConfig(voxel=v))
    randomize_bn(m, 2)
    m = fuse_model(m.eval())
    nx, ny, _ = m.cfg.voxel.grid_size
    canvas = torch.zeros(2, ny, nx, 64)
    canvas[:, ::3, ::2] = torch.rand(2, (ny + 2) // 3, (nx + 1) // 2, 64)
    fp = FastBEV(m, 2, device=cuda, precision="fp32", pair=True)
    f32 = FastBEV(m, 2, device=cuda, precision="fp32", pair=False)
    assert fp.pair and not f32.pair and fp.neck is not None
    a = [o.values().clone() for o in fp.forward(NHWC(to_pairs(canvas).to(cuda), pair=True))]
    b = [o.values().clone() for o in f32.forward(NHWC(canvas.to(cuda)))]
    c = [o.values().clone() for o in fp.forward(NHWC(canvas.to(cuda)))]  # plain canvas: converted on entry
    torch.cuda.synchronize()
    for x, y, z in zip(a, b, c):
        assert torch.equal(x, z) and rel_l2(x, y) < 5e-5, rel_l2(x, y)  # measured 7.8e-6 (vs fp64: ~1e-5)
    with torch.no_grad():
        ref = m.double().bev_forward(canvas.double().permute(0, 3, 1, 2))
    m.float()
    for o, r in zip(a, ref):
        assert rel_l2(o.permute(0, 3, 1, 2), r) < 2e-4


def test_lidar_pipeline_uses_pair_canvas(cuda):
    import numpy as np

    from triton_client_amd.pipelines import LidarPipeline
    from triton_client_amd.utils.synthetic import LidarSpec, lidar_sweep

    spec = LidarSpec(rings=32, azimuth_steps=1024, sensor_height=3.23)
    lid = LidarPipeline(batch=2, max_points=32768, device=cuda, z_offset=1.5, precision="fp32")
    for b in range(2):
        c = lidar_sweep(spec, b)
        raw = torch.from_numpy(c.view(np.uint8).reshape(-1))
        lid.data[b * lid.frame_bytes: b * lid.frame_bytes + raw.numel()].copy_(raw)
        lid.frame_n[b] = c.shape[0]
    lid.calibrate_detection_density(500.0)
    r1 = lid.step()
    n1 = r1.count.clone()
    assert lid.enc.pair and lid.fast.pair
    r2 = lid.step()  # pair canvas from the scatter, cleared by cell list
    torch.cuda.synchronize()
    assert torch.equal(n1, r2.count) and int(n1.min()) > 0


@pytest.mark.parametrize("tile", [0, 77, 71, 70])
def test_conv_pair_occupancy_gated_reads(cuda, tile):
    """tca_conv_nhwc_x3p_occ: pixels marked unoccupied read as zeros through the
    descriptor range check, so (a) with zeros there the output is bit-identical to
    the plain call, (b) garbage there is never read."""
    torch.manual_seed(tile)
    B, H, W, cin, cout = 2, 40, 36, 64, 128 if tile == 70 else 64
    s = 2 if tile == 77 else 1
    conv = nn.Conv2d(cin, cout, 3, s, 1, bias=True)
    fc = FusedConv(conv, act=1, device=cuda, precision="fp32")
    occ = (torch.rand(B, H, W) < 0.1).to(torch.uint8)
    x = torch.randn(B, H, W, cin) * occ[..., None]
    xz = NHWC(to_pairs(x).to(cuda), pair=True)
    Ho, Wo = fc.out_hw(H, W)
    plain = NHWC(torch.empty(B, Ho, Wo, cout, device=cuda), pair=True)
    # auto (tile 0) at stride 1 routes an ungated call to conv_hx3 (a different summation
    # order): the ungated reference is then the gated kernel with every cell occupied
    ones = torch.ones(B, H, W, dtype=torch.uint8, device=cuda)
    fc(NHWC(xz.t, pair=True, occ=ones) if (tile == 0 and s == 1) else xz, out=plain, tile=tile)
    gated = NHWC(torch.empty(B, Ho, Wo, cout, device=cuda), pair=True)
    fc(NHWC(xz.t, pair=True, occ=occ.to(cuda)), out=gated, tile=tile)
    junk = x + torch.randn(B, H, W, cin) * (1 - occ[..., None])  # garbage in every unoccupied cell
    gj = NHWC(torch.empty(B, Ho, Wo, cout, device=cuda), pair=True)
    fc(NHWC(to_pairs(junk).to(cuda), pair=True, occ=occ.to(cuda)), out=gj, tile=tile)
    torch.cuda.synchronize()
    assert torch.equal(plain.t, gated.t) and torch.equal(plain.t, gj.t)


@pytest.mark.parametrize("s2sp", [False, True], ids=["dense_gated", "sparse_gather"])
def test_lidar_pipeline_occupancy_matches_ungated(cuda, monkeypatch, s2sp):
    """The occupancy-gated first conv against the ungated one on the whole canvas: bit-identical
    with the dense gated kernel (masked loads give the same zeros); with the sparse-gather kernel
    (conv_s2sp.hip, opt-in) the same detections to within the summation order."""
    import numpy as np

    from triton_client_amd.ops import conv as conv_mod
    from triton_client_amd.pipelines import LidarPipeline

    monkeypatch.setattr(conv_mod, "S2SP", s2sp)
    from triton_client_amd.utils.synthetic import LidarSpec, lidar_sweep

    spec = LidarSpec(rings=32, azimuth_steps=1024, sensor_height=3.23)
    lid = LidarPipeline(batch=2, max_points=32768, device=cuda, z_offset=1.5, precision="fp32")
    for b in range(2):
        c = lidar_sweep(spec, 10 + b)
        raw = torch.from_numpy(c.view(np.uint8).reshape(-1))
        lid.data[b * lid.frame_bytes: b * lid.frame_bytes + raw.numel()].copy_(raw)
        lid.frame_n[b] = c.shape[0]
    lid.calibrate_detection_density(500.0)
    r1 = lid.step()
    assert lid.enc.occ is not None
    occ_cells = int(lid.enc.occ.sum())
    n1, b1 = r1.count.clone(), r1.box.clone()
    occ, lid.enc.occ = lid.enc.occ, None  # ungated: the first conv reads the whole canvas
    r2 = lid.step()
    torch.cuda.synchronize()
    lid.enc.occ = occ
    assert occ_cells > 0 and torch.equal(n1, r2.count)
    for b in range(2):
        k = int(n1[b])
        if s2sp:  # near-equal scores may swap places in the NMS order: match boxes as a set
            d = (b1[b, :k, None, :] - r2.box[b, None, :k, :]).abs().amax(-1)
            tol = 1e-3 * (1.0 + b1[b, :k].abs().amax(-1))
            matched = (d.amin(1) <= tol).float().mean().item()
            assert matched >= 0.98, matched
        else:
            assert torch.equal(b1[b, :k], r2.box[b, :k])


@pytest.mark.parametrize("tile", [90, 91, 92, 93, 94, 95, 96, 97, 102])
@pytest.mark.parametrize("shape", [(2, 23, 31, 64, 128), (1, 21, 37, 256, 256), (2, 19, 50, 64, 64), (3, 9, 16, 96, 72)])
def test_conv_pair_halo_tiles_vs_fp64(cuda, tile, shape):
    """Halo-tiled 3x3 stride-1 pair kernels (tiles 90-93): channel-offset input
    and output slices, partial row / column tiles, N not a multiple of the tile,
    a residual, against an fp64 reference; and close to the xb kernel (same
    products, (chunk, tap) instead of (tap, chunk) summation order)."""
    torch.manual_seed(tile + shape[3])
    B, H, W, cin, cout = shape
    conv = nn.Conv2d(cin, cout, 3, 1, 1, bias=True).double()
    fc = FusedConv(copy.deepcopy(conv).float(), act=1, device=cuda, precision="fp32")
    buf = torch.randn(B, H, W, cin + 16, dtype=torch.float64)
    res = torch.randn(B, H, W, cout, dtype=torch.float64)
    xin = buf[..., 8:8 + cin]
    x = NHWC(to_pairs(buf.float()).to(cuda), 8, cin, pair=True)
    r = NHWC(to_pairs(res.float()).to(cuda), pair=True)
    outs = {}
    for t in (tile, 0):
        out = torch.zeros(B, H, W, cout + 16, dtype=torch.float32, device=cuda)
        fc(x, out=NHWC(out, 8, cout, pair=True), res=r, tile=t)
        torch.cuda.synchronize()
        outs[t] = out
        assert out[..., :8].abs().sum().item() == 0 and out[..., 8 + cout:].abs().sum().item() == 0
    ref = torch.relu(conv(xin.permute(0, 3, 1, 2))) + from_pairs(r.t).double().cpu().permute(0, 3, 1, 2)
    got = NHWC(outs[tile], 8, cout, pair=True).nchw()
    assert rel_l2(got, ref) < 5e-5, rel_l2(got, ref)
    xb = NHWC(outs[0], 8, cout, pair=True).nchw()
    assert rel_l2(got, xb) < 2e-6, rel_l2(got, xb)


@pytest.mark.parametrize("tile", [98, 99, 100, 101])
@pytest.mark.parametrize("shape", [(2, 23, 31, 64, 128), (1, 21, 37, 256, 256), (2, 19, 50, 64, 64)])
def test_conv_fp32_halo_tiles_vs_fp64(cuda, tile, shape):
    """Plain-fp32 twins of the halo tiles (split at the fragment read, fp32
    output): channel-offset slices, partial tiles, a residual, vs fp64 and
    close to the xb kernel."""
    torch.manual_seed(tile + shape[3])
    B, H, W, cin, cout = shape
    conv = nn.Conv2d(cin, cout, 3, 1, 1, bias=True).double()
    fc = FusedConv(copy.deepcopy(conv).float(), act=1, device=cuda, precision="fp32")
    buf = torch.randn(B, H, W, cin + 16, dtype=torch.float64)
    res = torch.randn(B, H, W, cout, dtype=torch.float64)
    x = NHWC(buf.float().to(cuda), 8, cin)
    r = NHWC(res.float().to(cuda))
    outs = {}
    for t in (tile, 81 if cout <= 64 else 80):
        out = torch.zeros(B, H, W, cout + 16, dtype=torch.float32, device=cuda)
        fc(x, out=NHWC(out, 8, cout), res=r, tile=t)
        torch.cuda.synchronize()
        outs[t] = out
        assert out[..., :8].abs().sum().item() == 0 and out[..., 8 + cout:].abs().sum().item() == 0
    ref = torch.relu(conv(buf[..., 8:8 + cin].permute(0, 3, 1, 2))) + res.permute(0, 3, 1, 2)
    got = NHWC(outs[tile], 8, cout).nchw()
    assert rel_l2(got, ref) < 5e-5, rel_l2(got, ref)
    assert rel_l2(got, NHWC(outs[81 if cout <= 64 else 80], 8, cout).nchw()) < 2e-6

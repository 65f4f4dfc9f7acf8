"""Uniform-tile skipping in the PointPillars first block (conv_hx3.hip tca_bev_uniform_depth /
tca_conv_hx3p_uni, models/fast.py _BEVBackbonePlan.forward_blocks).

A pixel whose receptive field holds no occupied canvas cell (and no image border) carries the
same vector after every conv of the block; tiles made only of such pixels store that vector
instead of running the K loop.  The block outputs must be bit-identical to the dense run."""
import numpy as np
import pytest
import torch

from triton_client_amd import _native


def depth_ref(occ: np.ndarray, maxd: int) -> np.ndarray:
    """The definition, directly: u(p) = the 3x3 stride-2 window of p holds no occupied cell;
    depth(p) = 1 + the largest r < maxd with every pixel within Chebyshev radius r of p inside
    the image and uniform (0 when p is not uniform)."""
    B, H, W = occ.shape
    Ho, Wo = (H + 1) // 2, (W + 1) // 2
    o = np.pad(occ != 0, ((0, 0), (1, 2), (1, 2)))
    busy = np.zeros((B, Ho, Wo), bool)
    for dy in range(3):
        for dx in range(3):
            busy |= o[:, dy:dy + 2 * Ho:2, dx:dx + 2 * Wo:2]
    u = ~busy
    d = np.zeros((B, Ho, Wo), np.uint8)
    for b in range(B):
        for y in range(Ho):
            for x in range(Wo):
                if not u[b, y, x]:
                    continue
                k = 1
                while k < maxd:
                    y0, y1, x0, x1 = y - k, y + k + 1, x - k, x + k + 1
                    if y0 < 0 or x0 < 0 or y1 > Ho or x1 > Wo or not u[b, y0:y1, x0:x1].all():
                        break
                    k += 1
                d[b, y, x] = k
    return d


@pytest.mark.gpu
@pytest.mark.parametrize("shape,maxd,dens", [((2, 60, 50), 4, 0.01), ((1, 37, 81), 6, 0.003),
                                             ((3, 33, 140), 4, 0.02), ((1, 20, 20), 1, 0.05)])
def test_uniform_depth_matches_definition(cuda, shape, maxd, dens):
    g = np.random.default_rng(sum(shape) + maxd)
    occ = (g.random(shape) < dens).astype(np.uint8)
    occ[0, : shape[1] // 3, : shape[2] // 4] = 0  # an empty region that survives erosion
    B, H, W = shape
    ot = torch.from_numpy(occ).to(cuda)
    d = torch.full((B, (H + 1) // 2, (W + 1) // 2), 255, dtype=torch.uint8, device=cuda)
    _native.call("tca_bev_uniform_depth", _native.ptr(ot), B, H, W, maxd, _native.ptr(d), _native.stream_ptr(None))
    torch.cuda.synchronize()
    want = depth_ref(occ, maxd)
    assert np.array_equal(d.cpu().numpy(), want)
    assert want.max() >= min(maxd, 3)  # deep pixels present


def _lidar(cuda, B=2):
    from triton_client_amd.pipelines import LidarPipeline
    from triton_client_amd.utils.synthetic import LidarSpec, lidar_sweep

    lid = LidarPipeline(batch=B, device=cuda, precision="fp32")
    for b in range(B):
        c = lidar_sweep(LidarSpec(), 20 + b)
        raw = torch.from_numpy(c.view(np.uint8).reshape(-1))
        lid.data[b * lid.frame_bytes: b * lid.frame_bytes + raw.numel()].copy_(raw)
        lid.frame_n[b] = c.shape[0]
    return lid


@pytest.mark.gpu
def test_first_block_uniform_skip_bit_identical(cuda, monkeypatch):
    import triton_client_amd.models.fast as fast

    lid = _lidar(cuda)
    lid.calibrate_detection_density(500.0)
    f = lid.build_fast()
    bb = f.bb
    assert bb.uni_vals is not None and len(bb.uni_vals) == len(bb.blocks[0][0])
    lid.step_pre()
    canvas = lid.enc.canvas_nhwc()
    assert canvas.occ is not None
    outs = []
    for on in (True, False):
        monkeypatch.setattr(fast, "BEV_UNIFORM", on)
        # poison the block buffers: every pixel must be written by either path
        for convs, pp, H, W in bb.blocks:
            for p in pp:
                p.t.fill_(float("nan"))
        outs.append([o.t.clone() for o in f.forward_blocks(canvas)])
        torch.cuda.synchronize()
    depth = bb.depth.clone()
    # the skip path ran: a good share of the last layer's pixels are uniform
    assert (depth >= len(bb.blocks[0][0])).float().mean().item() > 0.1
    for a, b in zip(*outs):
        assert torch.equal(a.view(torch.int32), b.view(torch.int32))
    # the uniform pixels hold the constants
    last = outs[0][0][0]
    n = len(bb.blocks[0][0])
    ys, xs = torch.nonzero(depth[0] >= n, as_tuple=True)
    assert torch.equal(last[ys, xs], bb.uni_vals[n - 1].expand(ys.numel(), -1))


@pytest.mark.gpu
def test_lidar_step_same_detections_with_uniform_skip(cuda, monkeypatch):
    import triton_client_amd.models.fast as fast

    lid = _lidar(cuda)
    lid.calibrate_detection_density(500.0)
    r1 = lid.step()
    n1, b1 = r1.count.clone(), r1.box.clone()
    monkeypatch.setattr(fast, "BEV_UNIFORM", False)
    r2 = lid.step()
    torch.cuda.synchronize()
    assert int(n1.min()) > 0 and torch.equal(n1, r2.count)
    for b in range(2):
        k = int(n1[b])
        assert torch.equal(b1[b, :k], r2.box[b, :k])

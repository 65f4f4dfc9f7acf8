"""HIP kernels vs fp32 / sequential references (MI355X only)."""
import dataclasses

import numpy as np
import pytest
import torch

from triton_client_amd.config.lidar import KITTI_PILLARS, KITTI_SECOND_VOXELS, NUSC_PILLARS, PointPillarsConfig
from triton_client_amd.ops import golden
from triton_client_amd.ops import lidar as lidar_ops
from triton_client_amd.ops.image import preprocess
from triton_client_amd.ops.lidar import (AnchorPostprocess, PillarEncoder, PointLayout, Voxelizer, pc2_unpack,
                                         pillar_features_reference, voxelize_np)
from triton_client_amd.ops.nms import Candidates, sort_and_nms, sort_and_nms_cpu
from triton_client_amd.ops._ws import Workspace
from triton_client_amd.ops.yolo import YoloPostprocess

from test_ops_cpu import synth_cloud

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", ["stretch", "letterbox"])
@pytest.mark.parametrize("layout,dtype,oc", [("NCHW", torch.float32, 3), ("NHWC", torch.bfloat16, 4),
                                             ("NCHW", torch.float16, 3)])
def test_preprocess_gpu(cuda, mode, layout, dtype, oc):
    rng = np.random.default_rng(0)
    frames = torch.from_numpy(rng.integers(0, 256, size=(3, 90, 161, 3), dtype=np.uint8))
    ref, xr = preprocess(frames, (64, 96), mode=mode, layout=layout, out_channels=oc, dtype=torch.float32,
                         swap_rb=True)
    out, xg = preprocess(frames.to(cuda), (64, 96), mode=mode, layout=layout, out_channels=oc, dtype=dtype,
                         swap_rb=True)
    torch.cuda.synchronize()
    assert xr == xg
    tol = {torch.float32: 1e-5, torch.float16: 2e-3, torch.bfloat16: 8e-3}[dtype]
    diff = (out.float().cpu() - ref.float()).abs()
    # rint ties may flip by one u8 step on a handful of pixels
    assert (diff > tol).float().mean() < 5e-3
    assert diff.max() <= 1 / 255 + tol


def _random_candidates(B, cap, n, D, rotated, seed):
    rng = np.random.default_rng(seed)
    box = np.zeros((B, cap, D), np.float32)
    score = np.zeros((B, cap), np.float32)
    cls = np.zeros((B, cap), np.int32)
    key = np.zeros((B, cap), np.uint64)
    count = np.zeros((B,), np.int32)
    for b in range(B):
        m = n[b]
        if rotated:
            box[b, :m, :2] = rng.uniform(0, 40, (m, 2))
            box[b, :m, 2] = rng.uniform(-2, 0, m)
            box[b, :m, 3:6] = rng.uniform(0.5, 4.5, (m, 3))
            box[b, :m, 6] = rng.uniform(-np.pi, np.pi, m)
        else:
            xy = rng.uniform(0, 600, (m, 2))
            wh = rng.uniform(4, 120, (m, 2))
            box[b, :m, :4] = np.concatenate([xy, xy + wh], 1)
        s = rng.random(m).astype(np.float32)
        if m:
            s[: m // 10] = s[0]  # exact score ties
        score[b, :m] = s
        cls[b, :m] = rng.integers(0, 3, m)
        idx = rng.permutation(m * 3)[:m].astype(np.uint64)  # unique anchor ids
        ordered = np.where((s.view(np.uint32) & 0x80000000) != 0, ~s.view(np.uint32), s.view(np.uint32) | 0x80000000)
        key[b, :m] = (ordered.astype(np.uint64) << np.uint64(32)) | (np.uint64(0xFFFFFFFF) - idx)
        count[b] = m
    return box, score, cls, key, count


@pytest.mark.parametrize("mode", ["letterbox", "stretch"])
def test_preprocess_s2d_gpu(cuda, mode):
    """Space-to-depth output = space_to_depth2 of the plain NHWC output, bit-exact."""
    from triton_client_amd.ops.image import space_to_depth2
    rng = np.random.default_rng(3)
    frames = torch.from_numpy(rng.integers(0, 256, size=(2, 180, 322, 3), dtype=np.uint8)).to(cuda)
    ref, _ = preprocess(frames, (96, 128), mode, "COCO", torch.bfloat16, "NHWC", 3, swap_rb=True)
    got, _ = preprocess(frames, (96, 128), mode, "COCO", torch.bfloat16, "S2D", swap_rb=True)
    torch.cuda.synchronize()
    exp = space_to_depth2(ref.permute(0, 2, 3, 1).contiguous())
    assert torch.equal(got.cpu(), exp.cpu())


def _greedy_replay(gbox, box, score, cls, tie, thr, pre_max, max_out, agnostic, eps=1e-5):
    """Replay greedy rotated NMS over the candidates in the GPU's sort order (score
    desc, tie asc), taking the GPU's keep / drop decision for each and checking it
    against the fp64 IoU with the boxes the GPU kept before it.  Returns (decisions
    that differ from fp64, decisions whose fp64 max-IoU lies within eps of the
    threshold); asserts every difference is one of the latter and that the replay
    reproduces the GPU's whole kept list in order."""
    from triton_client_amd.ops import golden

    row = {box[i].tobytes(): i for i in range(len(box))}
    gidx = [row[r.astype(np.float32).tobytes()] for r in gbox]
    gset = set(gidx)
    order = np.lexsort((tie, -score.astype(np.float64)))[:pre_max]
    kept, flips, near = [], 0, 0
    for i in order:
        if len(kept) >= max_out:
            break
        prior = [k for k in kept if agnostic or cls[k] == cls[i]]
        mx = float(golden.rotated_iou_bev(box[i].astype(np.float64), box[prior].astype(np.float64)).max()) if prior else 0.0
        borderline = abs(mx - thr) < eps
        near += borderline
        if (i in gset) != (mx <= thr):
            assert borderline, (i, mx, thr)
            flips += 1
        if i in gset:
            kept.append(int(i))
    assert kept == gidx, "the GPU kept list is not a greedy outcome in score order"
    return flips, near


@pytest.mark.parametrize("rotated,agnostic", [(False, False), (True, True), (True, False)])
@pytest.mark.parametrize("pre_max", [64, 1000, 4096])
def test_sort_nms_gpu_vs_golden(cuda, rotated, agnostic, pre_max):
    B, cap, D = 3, 6000, 7 if rotated else 4
    n = [0, 700, 5000] if pre_max > 64 else [10, 63, 200]
    box, score, cls, key, count = _random_candidates(B, cap, n, D, rotated, seed=pre_max + rotated)
    ws = Workspace(cuda)
    cand = Candidates(torch.from_numpy(box).to(cuda), torch.from_numpy(score).to(cuda),
                      torch.from_numpy(cls).to(cuda), torch.from_numpy(key.view(np.int64)).to(cuda),
                      torch.from_numpy(count).to(cuda))
    thr = 0.1 if rotated else 0.45
    max_out = 300
    res = sort_and_nms(ws, cand, int(rotated), thr, pre_max, max_out, agnostic=agnostic)
    torch.cuda.synchronize()
    got = res.per_image()
    for b in range(B):
        m = count[b]
        tie = (np.uint64(0xFFFFFFFF) - (key[b, :m] & np.uint64(0xFFFFFFFF))).astype(np.int64)
        keep = sort_and_nms_cpu(box[b, :m], score[b, :m], cls[b, :m], tie, int(rotated), thr, pre_max, max_out,
                                agnostic)
        ref_box = box[b, keep]
        g = got[b]
        if rotated:
            # the GPU's full kept list must be the greedy outcome under the fp64 rotated IoU
            # (ops/golden.py): a decision may differ from fp64 only where the fp64 IoU is
            # within 1e-5 of the threshold (fp32 polygon clipping), and those are counted
            flips, near = _greedy_replay(g["box"], box[b, :m], score[b, :m], cls[b, :m], tie, thr, pre_max,
                                         max_out, agnostic)
            assert flips <= near, (flips, near)
            if near == 0:
                np.testing.assert_array_equal(g["box"], ref_box)  # no borderline pair: the exact fp64 kept set
            np.testing.assert_array_equal(g["cls"], cls[b, keep] if flips == 0 else g["cls"])
        else:
            assert len(keep) == len(g["box"])
            np.testing.assert_allclose(g["box"], ref_box, rtol=1e-6)
            np.testing.assert_array_equal(g["cls"], cls[b, keep])


def test_yolo_postprocess_gpu_vs_cpu(cuda):
    from triton_client_amd.models.yolov5 import DEFAULT_ANCHORS
    torch.manual_seed(0)
    B, nc, na = 2, 80, 3
    hs = [torch.randn(B, na * (nc + 5), s, s) * 2 for s in (80, 40, 20)]
    for h in hs:  # sparse objectness like a trained / prior-initialised head
        h.view(B, na, nc + 5, *h.shape[2:])[:, :, 4] -= 3.0
    pp_cpu = YoloPostprocess(nc, DEFAULT_ANCHORS, conf_thres=0.3, device="cpu")
    pp_gpu = YoloPostprocess(nc, DEFAULT_ANCHORS, conf_thres=0.3, device=cuda)
    ref = pp_cpu.cpu(hs)
    for layout in ("nchw", "nhwc"):
        hg = [h.to(cuda) for h in hs]
        if layout == "nhwc":
            hg = [h.contiguous(memory_format=torch.channels_last) for h in hg]
        res, dec = pp_gpu(hg, decoded_out=True)
        torch.cuda.synchronize()
        np.testing.assert_allclose(dec.cpu().numpy(), pp_cpu.decode_cpu(hs).numpy(), rtol=1e-4, atol=1e-3)
        dec = dec.clone()
        assert torch.equal(pp_gpu.decode(hg), dec)  # decode-only kernel (served output): same formulas
        for b in range(B):
            n = int(ref.count[b])
            assert int(res.count[b]) == n and n > 0
            np.testing.assert_allclose(res.box[b, :n].cpu(), ref.box[b, :n], rtol=1e-4, atol=1e-3)
            np.testing.assert_array_equal(res.cls[b, :n].cpu(), ref.cls[b, :n])


def test_pc2_unpack_gpu(cuda):
    clouds = [synth_cloud(n, seed=s) for n, s in ((5000, 1), (1, 2), (12345, 3))]
    data = b"".join(c.tobytes() for c in clouds)
    offs = np.cumsum([0] + [c.nbytes for c in clouds[:-1]])
    ns = np.array([len(c) for c in clouds], np.int32)
    d = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    ref, rc = pc2_unpack(None, d, torch.from_numpy(offs), torch.from_numpy(ns), PointLayout.xyzi_f32(), 16384,
                         True, 1.5, out_stride=5)
    ws = Workspace(cuda)
    got, gc = pc2_unpack(ws, d.to(cuda), torch.from_numpy(offs).to(cuda), torch.from_numpy(ns).to(cuda),
                         PointLayout.xyzi_f32(), 16384, True, 1.5, out_stride=5)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(gc.cpu().numpy(), rc.numpy())
    for b in range(3):
        n = int(rc[b])
        np.testing.assert_allclose(got[b, :n].cpu().numpy(), ref[b, :n].numpy(), rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("vcfg", [KITTI_PILLARS, KITTI_SECOND_VOXELS, NUSC_PILLARS])
@pytest.mark.parametrize("hash_mode", ["auto", "1", "0"])
def test_voxelize_gpu_exact(cuda, vcfg, hash_mode, monkeypatch):
    """Order-exact vs the NumPy spconv golden, with the cell rows as the dense grid and as the
    per-frame hash table (voxelize.hip hash_slot; auto: hash for SECOND's 90 M-cell grid)."""
    if hash_mode != "auto":
        monkeypatch.setattr(lidar_ops, "VOX_HASH_FORCE", hash_mode)
    cfg = dataclasses.replace(vcfg, max_voxels=2000)
    B, N = 2, 20000
    nf = cfg.num_point_features
    pts = np.zeros((B, N, nf), np.float32)
    cnt = np.array([N, N // 3], np.int32)
    for b in range(B):
        p = synth_cloud(N, seed=10 + b, nan_frac=0.0, pcr=cfg.point_cloud_range)
        pts[b, :, :4] = p
    vox = Voxelizer(cfg, B, N, device=cuda, nfeat=nf)
    for rep in range(2):  # second run checks the self-resetting scratch
        v, c, n, vc = vox(torch.from_numpy(pts).to(cuda), torch.from_numpy(cnt).to(cuda))
        torch.cuda.synchronize()
        for b in range(B):
            rv, rcoord, rn, _ = voxelize_np(pts[b, :cnt[b]], cfg, nf)
            k = int(vc[b])
            assert k == len(rn)
            np.testing.assert_array_equal(c[b, :k, 1:].cpu().numpy(), rcoord)
            np.testing.assert_array_equal(c[b, :k, 0].cpu().numpy(), b)
            np.testing.assert_array_equal(n[b, :k].cpu().numpy(), rn)
            np.testing.assert_array_equal(v[b, :k].cpu().numpy(), rv)


@pytest.mark.parametrize("vcfg", [KITTI_PILLARS, KITTI_SECOND_VOXELS])
@pytest.mark.parametrize("hash_mode", ["auto", "1"])
def test_voxelize_gpu_dense_voxels(cuda, vcfg, hash_mode, monkeypatch):
    """Clustered clouds: voxels with 9..300 points exercise the dense-voxel
    (wave bitonic top-P) path of the CSR slot sort; slot order must still be
    the first P points in point order (spconv)."""
    if hash_mode != "auto":
        monkeypatch.setattr(lidar_ops, "VOX_HASH_FORCE", hash_mode)
    cfg = dataclasses.replace(vcfg, max_voxels=3000)
    rng = np.random.default_rng(7)
    r = np.asarray(cfg.point_cloud_range, np.float32)
    vs = np.asarray(cfg.voxel_size, np.float32)
    B, N = 2, 6000
    nf = cfg.num_point_features
    pts = np.zeros((B, N, nf), np.float32)
    for b in range(B):
        p = rng.uniform(r[:3], r[3:], size=(N, 3)).astype(np.float32)
        # pile points into a few voxels: 300, 130, 65, 20, 9 points
        start = 0
        for k, m in enumerate((300, 130, 65, 20, 9)):
            centre = r[:3] + vs * (np.array([10 + 7 * k, 12 + 3 * b, 0]) + 0.5)
            p[start:start + m] = centre + rng.uniform(-0.4, 0.4, size=(m, 3)).astype(np.float32) * vs
            start += m
        perm = rng.permutation(N)
        pts[b, :, :3] = p[perm]
        pts[b, :, 3] = rng.uniform(0, 1, N)
    cnt = np.array([N, N - 1000], np.int32)
    vox = Voxelizer(cfg, B, N, device=cuda, nfeat=nf)
    for rep in range(2):
        v, c, n, vc = vox(torch.from_numpy(pts).to(cuda), torch.from_numpy(cnt).to(cuda))
        torch.cuda.synchronize()
        for b in range(B):
            rv, rcoord, rn, _ = voxelize_np(pts[b, :cnt[b]], cfg, nf)
            k = int(vc[b])
            assert k == len(rn) and rn.max() == cfg.max_points_per_voxel
            np.testing.assert_array_equal(c[b, :k, 1:].cpu().numpy(), rcoord)
            np.testing.assert_array_equal(n[b, :k].cpu().numpy(), rn)
            np.testing.assert_array_equal(v[b, :k].cpu().numpy(), rv)


@pytest.mark.parametrize("variant", [0, 1, 2], ids=["valu_fp32", "mfma_split", "valu_fp32_two_pillars"])
def test_pillar_vfe_gpu_vs_fp32(cuda, variant):
    """The VFE kernels against the fp32 PyTorch reference: 0 = the linearity-folded fp32 VALU
    kernel (tight tolerance), 1 = the split-bf16 MFMA kernel, 2 = the VALU kernel taking two
    pillars per wave iteration."""
    from triton_client_amd import _native

    old = _native.kernels().tca_pillar_vfe_set_variant(variant)
    try:
        _pillar_vfe_check(cuda, 2e-3 if variant == 1 else 1e-4)
    finally:
        _native.kernels().tca_pillar_vfe_set_variant(old)


@pytest.mark.parametrize("pair", [False, True], ids=["fp32_canvas", "pair_canvas"])
@pytest.mark.parametrize("batch", [1, 3])
def test_pillar_vfe_two_pillar_walk_matches_one_pillar(cuda, pair, batch):
    """The two-pillars-per-iteration VALU kernel writes the one-pillar kernel's features and canvas
    within the fp32 test bound (same per-pillar expressions; the compiler contracts them into FMAs
    differently: ~1e-5 apart) and exactly its occupancy: every pillar of every frame, odd counts
    leaving a half-empty last pair."""
    from triton_client_amd import _native

    cfg = dataclasses.replace(KITTI_PILLARS, max_voxels=5000)
    N = 20000
    pts = np.stack([synth_cloud(N, seed=40 + b, nan_frac=0.0, pcr=cfg.point_cloud_range) for b in range(batch)])
    pts[..., 3] /= 255.0
    cnt = np.array([N - 977 * b for b in range(batch)], np.int32)  # frames of different pillar counts
    torch.manual_seed(1)
    W = torch.randn(64, 10) * 0.3
    bias = torch.randn(64) * 0.1
    pg, cg = torch.from_numpy(pts).to(cuda), torch.from_numpy(cnt).to(cuda)
    outs = []
    k = _native.kernels()
    old = k.tca_pillar_vfe_set_variant(0)
    try:
        for variant in (0, 2):
            k.tca_pillar_vfe_set_variant(variant)
            vox = Voxelizer(cfg, batch, N, device=cuda)
            enc = PillarEncoder(cfg, W, bias, batch, device=cuda, dtype=torch.float32)
            enc.set_pair(pair)
            feat = torch.zeros(batch, cfg.max_voxels, 64, device=cuda)
            vox.assign(pg, cg)
            enc.encode_from_slots(pg, vox, feat_out=feat)
            torch.cuda.synchronize()
            vc = vox.voxel_count.cpu()
            outs.append((vc, [feat[b, :int(vc[b])].cpu() for b in range(batch)], enc.canvas.cpu(),
                         None if enc.occ is None else enc.occ.cpu()))
    finally:
        k.tca_pillar_vfe_set_variant(old)
    (vc0, f0, c0, o0), (vc2, f2, c2, o2) = outs
    assert torch.equal(vc0, vc2) and int(vc0.min()) > 100
    tol = 1e-4 * max(1.0, max(float(a.abs().max()) for a in f0))  # the vs-fp32 test's bound
    for a, b_ in zip(f0, f2):
        torch.testing.assert_close(b_, a, rtol=0.0, atol=tol)
    if pair:
        from triton_client_amd.ops.conv import from_pairs
        c0, c2 = from_pairs(c0), from_pairs(c2)
    torch.testing.assert_close(c2, c0, rtol=0.0, atol=tol)
    if pair:
        assert torch.equal(o0, o2) and int(o0.sum()) == int(vc0.sum())


def _pillar_vfe_check(cuda, tol):
    cfg = dataclasses.replace(KITTI_PILLARS, max_voxels=6000)
    B, N = 2, 30000
    pts = np.stack([synth_cloud(N, seed=20 + b, nan_frac=0.0, pcr=cfg.point_cloud_range) for b in range(B)])
    pts[..., 3] /= 255.0
    cnt = np.array([N, N], np.int32)
    torch.manual_seed(0)
    W = torch.randn(64, 10) * 0.3
    bias = torch.randn(64) * 0.1
    vox = Voxelizer(cfg, B, N, device=cuda)
    enc = PillarEncoder(cfg, W, bias, B, device=cuda)
    pg = torch.from_numpy(pts).to(cuda)
    cg = torch.from_numpy(cnt).to(cuda)
    feat = torch.zeros(B, cfg.max_voxels, 64, device=cuda)
    vox.assign(pg, cg)
    enc.encode_from_slots(pg, vox, feat_out=feat)
    vox.finish(pg, cg, gather=True)  # materialise voxels for the reference
    torch.cuda.synchronize()
    for b in range(B):
        k = int(vox.voxel_count[b])
        ref = pillar_features_reference(vox.voxels[b, :k].cpu(), vox.num_points[b, :k].cpu(),
                                        vox.coords[b, :k].cpu(), cfg, W, bias)
        got = feat[b, :k].cpu()
        err = (got - ref).abs().max().item()
        assert err < tol * max(1.0, ref.abs().max().item()), err
        # canvas scatter: each pillar's cell holds its feature in bf16
        co = vox.coords[b, :k].cpu().long()
        cv = enc.canvas[b, co[:, 2], co[:, 3]].float().cpu()
        torch.testing.assert_close(cv, got, rtol=1e-2, atol=1e-2)
    # clear(): the cells written above go back to zero
    enc.clear(vox)
    torch.cuda.synchronize()
    assert enc.canvas.abs().sum().item() == 0


def test_anchor_postprocess_gpu_vs_cpu(cuda):
    cfg = PointPillarsConfig()
    ap_c = AnchorPostprocess(cfg, 1, device="cpu")
    ap_g = AnchorPostprocess(cfg, 1, device=cuda)
    H, W, A, C = ap_c.H, ap_c.W, ap_c.A, ap_c.C
    g = torch.Generator().manual_seed(0)
    cls = torch.randn(1, A * C, H, W, generator=g) - 3.5
    box = torch.randn(1, A * 7, H, W, generator=g) * 0.1
    dr = torch.randn(1, A * 2, H, W, generator=g)
    ref = ap_c.cpu(cls, box, dr)
    got = ap_g(cls.to(cuda).contiguous(memory_format=torch.channels_last),
               box.to(cuda).contiguous(memory_format=torch.channels_last),
               dr.to(cuda).contiguous(memory_format=torch.channels_last))
    torch.cuda.synchronize()
    n_r, n_g = int(ref.count[0]), int(got.count[0])
    assert n_r > 10 and abs(n_r - n_g) <= 2
    k = min(n_r, n_g, 50)
    np.testing.assert_allclose(got.box[0, :k].cpu().numpy(), ref.box[0, :k].numpy(), rtol=1e-4, atol=1e-4)
    np.testing.assert_array_equal(got.cls[0, :k].cpu().numpy(), ref.cls[0, :k].numpy())


def test_anchor_postprocess_merged_head_fast_path(cuda):
    """The merged fp32 NHWC head (the fused neck's output, cls / box / dir channel slices of
    one [B, H, W, 72] buffer) takes the pixel-major decode (anchors.hip
    anchor_decode_px_kernel): same candidates as the anchor-major kernel on the same data,
    and the same detections as the CPU reference."""
    from triton_client_amd.ops.conv import NHWC

    cfg = PointPillarsConfig()
    ap_c = AnchorPostprocess(cfg, 2, device="cpu")
    ap_g = AnchorPostprocess(cfg, 2, device=cuda)
    H, W, A, C = ap_c.H, ap_c.W, ap_c.A, ap_c.C
    g = torch.Generator().manual_seed(1)
    head = torch.cat([torch.randn(2, H, W, A * C, generator=g) - 3.5, torch.randn(2, H, W, A * 7, generator=g) * 0.1,
                      torch.randn(2, H, W, A * 2, generator=g)], -1)
    assert head.shape[-1] == 72
    hd = head.to(cuda)
    cb, cd = A * C, A * C + A * 7  # channel offsets of box and dir in the merged head
    views = (NHWC(hd, 0, A * C), NHWC(hd, cb, A * 7), NHWC(hd, cd, A * 2))
    fast = ap_g(*views)
    torch.cuda.synchronize()
    fast = [t.clone() for t in (fast.box, fast.score, fast.cls, fast.count)]
    # the anchor-major kernel on the same data: separate channels_last tensors (ld = A * C, no fast path)
    nchw = head.permute(0, 3, 1, 2)
    slow = ap_g(*(nchw[:, a:b].to(cuda).contiguous(memory_format=torch.channels_last)
                  for a, b in ((0, cb), (cb, cd), (cd, cd + A * 2))))
    torch.cuda.synchronize()
    for x, y in zip(fast, (slow.box, slow.score, slow.cls, slow.count)):
        assert torch.equal(x, y)
    ref = ap_c.cpu(nchw[:, :cb], nchw[:, cb:cd], nchw[:, cd:])
    for b in range(2):
        n_r, n_g = int(ref.count[b]), int(fast[3][b])
        assert n_r > 10 and abs(n_r - n_g) <= 2
        k = min(n_r, n_g, 50)
        np.testing.assert_allclose(fast[0][b, :k].cpu().numpy(), ref.box[b, :k].numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("cin,cout,k,s,p,act", [
    (16, 32, 3, 2, 1, 2), (32, 32, 3, 1, 1, 2), (64, 64, 3, 1, 1, 1), (64, 128, 3, 2, 1, 1),
    (128, 256, 1, 1, 0, 2), (24, 16, 1, 1, 0, 0), (8, 16, 6, 2, 2, 2), (256, 72, 1, 1, 0, 0)])
def test_fused_conv_vs_fp32(cuda, cin, cout, k, s, p, act):
    import torch.nn as nn
    from triton_client_amd.ops.conv import NHWC, FusedConv
    torch.manual_seed(0)
    conv = nn.Conv2d(cin, cout, k, s, p, bias=True)
    B, H, W = 2, 37, 29
    x = torch.randn(B, H, W, cin)
    fc = FusedConv(conv, act=act, device=cuda)
    xg = x.to(cuda, torch.bfloat16)
    y = fc(NHWC(xg))
    torch.cuda.synchronize()
    ref = fc(NHWC(x.to(torch.bfloat16).float()), out=NHWC(torch.empty(*y.shape, dtype=torch.float32)))
    got = y.tensor().float().cpu()
    r = ref.tensor()[..., :cout]
    err = (got[..., :cout] - r).abs().max().item()
    assert err < 0.02 * max(1.0, r.abs().max().item()), err


@pytest.mark.parametrize("tile", [1, 2, 3, 4, 5, 6, 7])
def test_fused_conv_v1_tiles(cuda, tile):
    """v1 (register-staged) tiles incl. the N=16 ones, with N / M tails and Cin % 32 != 0."""
    import torch.nn as nn
    from triton_client_amd.ops.conv import NHWC, FusedConv
    torch.manual_seed(tile)
    for cin, cout, k, s in ((16, 16, 3, 1), (24, 40, 3, 2), (16, 72, 1, 1)):
        conv = nn.Conv2d(cin, cout, k, s, k // 2, bias=True)
        fc = FusedConv(conv, act=2, device=cuda)
        x = torch.randn(2, 23, 31, cin)
        y = fc(NHWC(x.to(cuda, torch.bfloat16)), tile=tile)
        torch.cuda.synchronize()
        ref = torch.nn.functional.silu(conv(x.to(torch.bfloat16).float().permute(0, 3, 1, 2))).permute(0, 2, 3, 1)
        err = (y.tensor().float().cpu()[..., :cout] - ref).abs().max().item()
        assert err < 0.03 * max(1.0, ref.abs().max().item()), (cin, cout, err)


def test_fused_conv_slices_residual_and_transpose(cuda):
    import torch.nn as nn
    from triton_client_amd.ops.conv import NHWC, FusedConv
    torch.manual_seed(1)
    B, H, W = 2, 20, 24
    buf = torch.randn(B, H, W, 48).to(cuda, torch.bfloat16)  # read channels [16, 48)
    conv = nn.Conv2d(32, 16, 3, 1, 1)
    fc = FusedConv(conv, act=2, device=cuda)
    out = torch.zeros(B, H, W, 64, dtype=torch.bfloat16, device=cuda)
    res = torch.randn(B, H, W, 40).to(cuda, torch.bfloat16)
    fc(NHWC(buf, 16, 32), out=NHWC(out, 8, 16), res=NHWC(res, 24, 16))
    torch.cuda.synchronize()
    xin = buf[..., 16:48].float().permute(0, 3, 1, 2).cpu()
    ref = torch.nn.functional.silu(conv(xin)) + res[..., 24:40].float().permute(0, 3, 1, 2).cpu()
    got = out[..., 8:24].float().permute(0, 3, 1, 2).cpu()
    assert (got - ref).abs().max().item() < 0.05
    assert out[..., :8].abs().sum().item() == 0 and out[..., 24:].abs().sum().item() == 0
    # transpose conv k=s=2 and 4 via pixel shuffle
    for s_ in (2, 4):
        ct = nn.ConvTranspose2d(64, 32, s_, stride=s_, bias=True)
        x = torch.randn(B, 9, 7, 64)
        fct = FusedConv(ct, act=1, device=cuda)
        y = fct(NHWC(x.to(cuda, torch.bfloat16)))
        torch.cuda.synchronize()
        ref = torch.relu(ct(x.to(torch.bfloat16).float().permute(0, 3, 1, 2))).permute(0, 2, 3, 1)
        assert y.shape == (B, 9 * s_, 7 * s_, 32)
        assert (y.tensor().float().cpu() - ref).abs().max().item() < 0.05


@pytest.mark.parametrize("tile", [11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 31, 32, 33, 34, 35, 36, 37, 38, 39, 40, 41, 42, 43, 44])
def test_fused_conv_glds_tiles(cuda, tile):
    """v2 (global_load_lds, BK=64) tiles: Cin % 64 == 0 shapes with stride, channel
    slices, residual, M/N tails and a pixel-shuffle transpose conv, vs fp32."""
    import torch.nn as nn
    from triton_client_amd.ops.conv import NHWC, FusedConv
    torch.manual_seed(tile)
    B, H, W = 2, 23, 31  # M tail: 2*23*31 = 1426 (not a multiple of any BM)
    for cin, cout, k, s, act in ((64, 64, 3, 1, 1), (128, 72, 3, 2, 2), (192, 256, 1, 1, 0), (64, 128, 1, 1, 1)):
        conv = nn.Conv2d(cin, cout, k, s, k // 2, bias=True)
        fc = FusedConv(conv, act=act, device=cuda)
        buf = torch.randn(B, H, W, cin + 64).to(cuda, torch.bfloat16)
        xin = NHWC(buf, 64, cin)  # channels [64, 64+cin)
        Ho, Wo = (H + 2 * (k // 2) - k) // s + 1, (W + 2 * (k // 2) - k) // s + 1
        res = torch.randn(B, Ho, Wo, fc.N + 16).to(cuda, torch.bfloat16)
        out = torch.zeros(B, Ho, Wo, fc.N + 8, dtype=torch.bfloat16, device=cuda)
        fc(xin, out=NHWC(out, 8, fc.N), res=NHWC(res, 16, fc.N), tile=tile)
        torch.cuda.synchronize()
        x32 = buf[..., 64:64 + cin].float().permute(0, 3, 1, 2).cpu()
        acts = {0: lambda t: t, 1: torch.relu, 2: torch.nn.functional.silu}
        ref = acts[act](conv(x32)) + res[..., 16:16 + cout].float().permute(0, 3, 1, 2).cpu()
        got = out[..., 8:8 + cout].float().permute(0, 3, 1, 2).cpu()
        err = (got - ref).abs().max().item()
        assert err < 0.03 * max(1.0, ref.abs().max().item()), (cin, cout, k, s, err)
        assert out[..., :8].abs().sum().item() == 0
    ct = nn.ConvTranspose2d(128, 64, 2, stride=2, bias=True)
    fct = FusedConv(ct, act=1, device=cuda)
    x = torch.randn(B, 9, 7, 128)
    y = fct(NHWC(x.to(cuda, torch.bfloat16)), tile=tile)
    torch.cuda.synchronize()
    ref = torch.relu(ct(x.to(torch.bfloat16).float().permute(0, 3, 1, 2))).permute(0, 2, 3, 1)
    assert (y.tensor().float().cpu() - ref).abs().max().item() < 0.05


def test_fused_conv_halo_tile(cuda):
    """v3 halo kernel (tile 50: 3x3 s1, Cin = N = 64, persistent, LDS-resident
    weights + 18x18 input halo): partial edge tiles (H, W not multiples of 16),
    input/output channel slices, more tiles than CUs and fewer, vs fp32."""
    import torch.nn as nn
    from triton_client_amd.ops.conv import NHWC, FusedConv
    torch.manual_seed(50)
    conv = nn.Conv2d(64, 64, 3, 1, 1, bias=True)
    fc = FusedConv(conv, act=1, device=cuda)
    for B, H, W in ((2, 23, 31), (3, 16, 16), (16, 70, 54), (1, 5, 3)):
        buf = torch.randn(B, H, W, 96).to(cuda, torch.bfloat16)
        xin = NHWC(buf, 16, 64)  # channels [16, 80)
        out = torch.zeros(B, H, W, 80, dtype=torch.bfloat16, device=cuda)
        fc(xin, out=NHWC(out, 8, 64), tile=50)
        torch.cuda.synchronize()
        x32 = buf[..., 16:80].float().permute(0, 3, 1, 2).cpu()
        ref = torch.relu(conv(x32))
        got = out[..., 8:72].float().permute(0, 3, 1, 2).cpu()
        err = (got - ref).abs().max().item()
        assert err < 0.03 * max(1.0, ref.abs().max().item()), (B, H, W, err)
        assert out[..., :8].abs().sum().item() == 0 and out[..., 72:].abs().sum().item() == 0
    with pytest.raises(Exception):  # outside the contract (stride 2) is refused, not run
        fc2 = FusedConv(nn.Conv2d(64, 64, 3, 2, 1), act=1, device=cuda)
        fc2(NHWC(torch.randn(1, 8, 8, 64).to(cuda, torch.bfloat16)), tile=50)


@pytest.mark.parametrize("cin,cout,s", [(16, 16, 1), (16, 32, 2), (32, 32, 1), (16, 32, 1), (32, 16, 2), (16, 16, 2)])
def test_fused_conv_small_halo(cuda, cin, cout, s):
    """v4 small-halo kernel (tile 60: 3x3, Cin, N in {16, 32}, stride 1/2): edge
    tiles, channel slices, SiLU, the Bottleneck residual (both orders) vs fp32."""
    import torch.nn as nn
    from triton_client_amd.ops.conv import NHWC, FusedConv
    torch.manual_seed(60 + cin + cout + s)
    conv = nn.Conv2d(cin, cout, 3, s, 1, bias=True)
    for B, H, W in ((2, 23, 31), (1, 40, 17)):
        for post in (False, True):
            fc = FusedConv(conv, act=2, device=cuda, post_res=post)
            buf = torch.randn(B, H, W, cin + 16).to(cuda, torch.bfloat16)
            xin = NHWC(buf, 8, cin)  # channels [8, 8+cin)
            Ho, Wo = (H - 1) // s + 1, (W - 1) // s + 1
            res = torch.randn(B, Ho, Wo, cout + 8).to(cuda, torch.bfloat16)
            out = torch.zeros(B, Ho, Wo, cout + 16, dtype=torch.bfloat16, device=cuda)
            fc(xin, out=NHWC(out, 8, cout), res=NHWC(res, 8, cout), tile=60)
            torch.cuda.synchronize()
            x32 = buf[..., 8:8 + cin].float().permute(0, 3, 1, 2).cpu()
            r32 = res[..., 8:8 + cout].float().permute(0, 3, 1, 2).cpu()
            y = conv(x32)
            ref = torch.nn.functional.silu(y + r32) if post else torch.nn.functional.silu(y) + r32
            got = out[..., 8:8 + cout].float().permute(0, 3, 1, 2).cpu()
            err = (got - ref).abs().max().item()
            assert err < 0.03 * max(1.0, ref.abs().max().item()), (B, H, W, post, err)
            assert out[..., :8].abs().sum().item() == 0 and out[..., 8 + cout:].abs().sum().item() == 0


@pytest.mark.parametrize("agnostic", [False, True])
def test_yolo_merge_nms_gpu_matches_cpu(cuda, agnostic):
    """tca_nms_merge (K4m) == the NumPy merge-NMS on the same decoded heads."""
    from triton_client_amd.models.yolov5 import STRIDES
    from triton_client_amd.ops.image import frame_xform
    from triton_client_amd.ops.yolo import YoloPostprocess

    torch.manual_seed(3)
    nc, img = 6, (128, 160)
    anchors = torch.tensor([[10, 13, 16, 30, 33, 23], [30, 61, 62, 45, 59, 119], [116, 90, 156, 198, 373, 326]],
                           dtype=torch.float32).reshape(3, 3, 2)
    heads = [torch.randn(2, 3 * (5 + nc), img[0] // s, img[1] // s) * 2.0 + 0.5 for s in STRIDES]
    xf, _ = frame_xform((240, 320), img, "letterbox")
    pg = YoloPostprocess(nc, anchors, img, conf_thres=0.3, iou_thres=0.45, device=cuda, merge=True, agnostic=agnostic)
    pc = YoloPostprocess(nc, anchors, img, conf_thres=0.3, iou_thres=0.45, device="cpu", merge=True, agnostic=agnostic)
    rg = pg([h.to(cuda) for h in heads], xf).per_image()
    rc = pc.cpu(heads, xf).per_image()
    merged_any = False
    for g, c in zip(rg, rc):
        assert len(g["score"]) == len(c["score"]) and len(c["score"]) > 0
        np.testing.assert_array_equal(g["cls"], c["cls"])
        np.testing.assert_allclose(g["score"], c["score"], rtol=1e-5)
        np.testing.assert_allclose(g["box"], c["box"], rtol=1e-4, atol=2e-3)
    plain = YoloPostprocess(nc, anchors, img, conf_thres=0.3, iou_thres=0.45, device="cpu", agnostic=agnostic)
    for p, c in zip(plain.cpu(heads, xf).per_image(), rc):
        merged_any |= len(p["score"]) != len(c["score"]) or not np.allclose(p["box"][:len(c["box"])], c["box"])
    assert merged_any  # the merge changed something on these heads


@pytest.mark.gpu
def test_copy_segments_kernel(cuda):
    """csrc/kernels/copy.hip: many segments in one launch, aligned and unaligned, empty and
    multi-chunk, bytes outside the segments untouched."""
    import numpy as np

    from triton_client_amd import _native

    g = torch.Generator().manual_seed(0)
    src = torch.randint(0, 256, (3 << 20,), dtype=torch.uint8, generator=g).to(cuda)
    dst = torch.zeros_like(src)
    segs = [(0, 0, 1 << 20), (1 << 20, (1 << 20) + 3, 70001), (2 << 20, 5, 0), ((2 << 20) + 7, 11, 1),
            ((2 << 20) + 64, 4096, 200000)]
    dp = np.asarray([dst.data_ptr() + d for d, _, _ in segs], np.int64)
    sp = np.asarray([src.data_ptr() + s for _, s, _ in segs], np.int64)
    nb = np.asarray([n for _, _, n in segs], np.int64)
    _native.call("tca_copy_segments", len(segs), dp.ctypes.data, sp.ctypes.data, nb.ctypes.data,
                 _native.stream_ptr(torch.cuda.current_stream()))
    torch.cuda.synchronize()
    ref = torch.zeros_like(src)
    for d, s, n in segs:
        ref[d:d + n] = src[s:s + n]
    assert torch.equal(dst, ref)


@pytest.mark.parametrize("vcfg", [KITTI_PILLARS, KITTI_SECOND_VOXELS])
@pytest.mark.parametrize("hash_mode", ["auto", "1"])
def test_voxelize_gpu_exact_ring_order(cuda, vcfg, hash_mode, monkeypatch):
    """Points in sensor (ring / azimuth) order: long runs of consecutive points in one cell, so
    the run-aggregated atomics (voxelize.hip wave_run: one atomicMin / count / cursor reservation
    per run) carry most points.  Runs cross wave boundaries, are cut by out-of-range points, and
    the LiDAR sweep of the bench is order-exact against the spconv golden too."""
    from triton_client_amd.utils.synthetic import LidarSpec, lidar_sweep
    if hash_mode != "auto":
        monkeypatch.setattr(lidar_ops, "VOX_HASH_FORCE", hash_mode)
    cfg = dataclasses.replace(vcfg, max_voxels=20000)
    nf = cfg.num_point_features
    sweeps = []
    for b in range(2):
        p = lidar_sweep(LidarSpec(rings=32, azimuth_steps=1024, sensor_height=3.23), 20 + b)
        p = p[~np.isnan(p).any(1)]
        p[:, 2] += 1.5
        sweeps.append(p)
    rng = np.random.default_rng(3)
    r = np.asarray(cfg.point_cloud_range, np.float32)
    runs = np.repeat(rng.uniform(r[:3], r[3:], size=(300, 3)).astype(np.float32), rng.integers(1, 150, 300), 0)
    runs[::97] = r[3:] + 5  # out of range: cuts a run
    ordered = np.concatenate([runs, np.zeros((len(runs), 1), np.float32)], 1)
    sweeps.append(ordered)
    B, N = len(sweeps), max(len(p) for p in sweeps)
    pts = np.zeros((B, N, nf), np.float32)
    cnt = np.array([len(p) for p in sweeps], np.int32)
    for b, p in enumerate(sweeps):
        pts[b, :len(p), :4] = p
    vox = Voxelizer(cfg, B, N, device=cuda, nfeat=nf)
    for rep in range(2):
        v, c, n, vc = vox(torch.from_numpy(pts).to(cuda), torch.from_numpy(cnt).to(cuda))
        torch.cuda.synchronize()
        for b in range(B):
            rv, rcoord, rn, _ = voxelize_np(pts[b, :cnt[b]], cfg, nf)
            k = int(vc[b])
            assert k == len(rn) and k > 100
            np.testing.assert_array_equal(c[b, :k, 1:].cpu().numpy(), rcoord)
            np.testing.assert_array_equal(n[b, :k].cpu().numpy(), rn)
            np.testing.assert_array_equal(v[b, :k].cpu().numpy(), rv)


@pytest.mark.parametrize("shift", [0, 4, 1])
@pytest.mark.parametrize("out_stride", [4, 5])
def test_pc2_unpack_gpu_alignments(cuda, shift, out_stride):
    """The xyzi float32 fast paths (one 16-B load per point with the frame 16-B aligned, dword
    loads when 4-B aligned, byte loads otherwise) and the 16-B output store give the CPU
    unpack's points."""
    clouds = [synth_cloud(n, seed=s) for n, s in ((7000, 4), (3, 5), (20001, 6))]
    blobs, offs, o = [], [], 0
    for c in clouds:
        pad = bytes(shift)
        blobs.append(pad + c.tobytes())
        offs.append(o + shift)
        o += len(pad) + c.nbytes
    d = torch.frombuffer(bytearray(b"".join(blobs)), dtype=torch.uint8)
    ns = np.array([len(c) for c in clouds], np.int32)
    offs = np.asarray(offs, np.int64)
    ref, rc = pc2_unpack(None, d, torch.from_numpy(offs), torch.from_numpy(ns), PointLayout.xyzi_f32(), 32768,
                         True, 1.5, out_stride=out_stride)
    ws = Workspace(cuda)
    got, gc = pc2_unpack(ws, d.to(cuda), torch.from_numpy(offs).to(cuda), torch.from_numpy(ns).to(cuda),
                         PointLayout.xyzi_f32(), 32768, True, 1.5, out_stride=out_stride)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(gc.cpu().numpy(), rc.numpy())
    for b in range(3):
        n = int(rc[b])
        np.testing.assert_allclose(got[b, :n].cpu().numpy(), ref[b, :n].numpy(), rtol=1e-6, atol=1e-7)

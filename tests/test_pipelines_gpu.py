"""End-to-end device pipelines vs their CPU reference paths (MI355X only)."""
import numpy as np
import pytest
import torch

from triton_client_amd.ops.conv import NHWC
from triton_client_amd.pipelines import CameraPipeline, GraphRunner, LidarPipeline
from triton_client_amd.utils.synthetic import LidarSpec, camera_frame, lidar_sweep

pytestmark = pytest.mark.gpu


def _load_lidar(lid, spec, seeds):
    for b, s in enumerate(seeds):
        c = lidar_sweep(spec, s)
        raw = torch.from_numpy(c.view(np.uint8).reshape(-1))
        lid.data[b * lid.frame_bytes: b * lid.frame_bytes + raw.numel()].copy_(raw)
        lid.frame_n[b] = c.shape[0]


def test_lidar_pipeline_matches_cpu_postprocess(cuda):
    spec = LidarSpec(rings=32, azimuth_steps=1024, sensor_height=3.23)
    B = 2
    lid = LidarPipeline(batch=B, max_points=32768, device=cuda)
    _load_lidar(lid, spec, [1, 2])
    d = lid.calibrate_detection_density(500.0)
    assert -30 < d < 30
    res = lid.step()
    torch.cuda.synchronize()
    cand_count = lid.post.ws.get("anc_count", (B,), torch.int32).cpu()
    vc = lid.vox.voxel_count.cpu()
    assert (vc > 1000).all(), vc
    assert (cand_count > 100).all(), (cand_count, d)
    # post-process the very head outputs the pipeline used, on the CPU
    from triton_client_amd.ops.lidar import AnchorPostprocess
    if lid.fast is not None:
        cls, box, dr = (v.nchw() for v in (NHWC(lid.fast.hout.t, 0, lid.fast.n_cls),
                                          NHWC(lid.fast.hout.t, lid.fast.n_cls, lid.fast.n_box),
                                          NHWC(lid.fast.hout.t, lid.fast.n_cls + lid.fast.n_box, lid.fast.n_dir)))
    else:
        with torch.no_grad():
            cls, box, dr = lid.model.bev_forward(lid.enc.canvas_nchw())
    ref = AnchorPostprocess(lid.cfg, B, device="cpu").cpu(cls.float().cpu(), box.float().cpu(), dr.float().cpu())
    for b in range(B):
        n_r, n_g = int(ref.count[b]), int(res.count[b])
        assert n_r > 0 and abs(n_r - n_g) <= max(2, n_r // 50), (n_r, n_g)


def test_camera_pipeline_graph_replay_matches_eager(cuda):
    B = 2
    cam = CameraPipeline(batch=B, src_hw=(360, 640), device=cuda)
    for b in range(B):
        cam.frames[b].copy_(torch.from_numpy(camera_frame(360, 640, b)))
    cam.calibrate_detection_density(50.0)
    eager = cam.step()
    torch.cuda.synchronize()
    e = [t.clone() for t in (eager.box, eager.score, eager.cls, eager.count)]
    runner = GraphRunner(cam.step)
    g = runner()
    torch.cuda.synchronize()
    assert int(e[3].sum()) > 0
    # MIOpen convs are not bitwise deterministic run to run, which can reorder
    # equal-score candidates: compare the kept sets, not the order.
    from triton_client_amd.ops.golden import box_iou_np
    for b in range(B):
        n, m = int(e[3][b]), int(g.count[b])
        assert abs(n - m) <= max(1, n // 20)
        iou = box_iou_np(e[0][b, :n].cpu().numpy(), g.box[b, :m].cpu().numpy())
        assert (iou.max(1) > 0.9).mean() > 0.9


def test_lidar_graph_replay_twice_is_stable(cuda):
    """Self-resetting scratch: replaying the captured step on the same input
    must give identical results (catches stale voxel/canvas state)."""
    spec = LidarSpec(rings=32, azimuth_steps=1024, sensor_height=3.23)
    lid = LidarPipeline(batch=2, max_points=32768, device=cuda)
    _load_lidar(lid, spec, [3, 4])
    lid.calibrate_detection_density(500.0)
    runner = GraphRunner(lid.step)
    r1 = runner()
    torch.cuda.synchronize()
    a = [t.clone() for t in (r1.box, r1.score, r1.count)]
    r2 = runner()
    torch.cuda.synchronize()
    assert int(a[2].sum()) > 0
    # the fused-conv plan, voxeliser (sorted slot insertion), anchor decode
    # (key-ordered top-k) and NMS are all deterministic: replays are bitwise equal
    for b in range(2):
        n = int(a[2][b])
        assert n == int(r2.count[b])
        assert torch.equal(a[0][b, :n], r2.box[b, :n])
        assert torch.equal(a[1][b, :n], r2.score[b, :n])


@pytest.mark.parametrize("neck_back,blocks_front", [(False, None), (True, None), (True, 2)])
def test_lidar_post_split_pipelining_matches_step(cuda, neck_back, blocks_front):
    """bench.py --lidar-pipeline 2 / 3 / 4: pipeline B's front (preprocessing + network; with
    blocks_front only the first two down blocks, the third runs in the back half) on one
    stream beside pipeline A's back (neck + head / decode + rotated NMS of A's previous
    front) on another gives A exactly the detections of a plain step(); two rounds over
    swapped frames catch a canvas cell left uncleared."""
    spec = LidarSpec(rings=32, azimuth_steps=1024, sensor_height=3.23)
    la = LidarPipeline(batch=2, max_points=32768, device=cuda)
    _load_lidar(la, spec, [5, 6])
    la.calibrate_detection_density(500.0)
    lb = LidarPipeline(la.model, batch=2, max_points=32768, device=cuda)
    _load_lidar(lb, spec, [7, 8])

    def snap(r):
        return [t.clone() for t in (r.box, r.score, r.count)]

    ref = {}
    for name, lp, seeds in (("a1", la, [5, 6]), ("b1", lb, [7, 8]), ("a2", la, [7, 8]), ("b2", lb, [5, 6])):
        _load_lidar(lp, spec, seeds)
        ref[name] = snap(lp.step())
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    main = torch.cuda.current_stream()
    got = {}
    for rnd, (sa, sb) in enumerate((([5, 6], [7, 8]), ([7, 8], [5, 6])), 1):
        _load_lidar(la, spec, sa)
        _load_lidar(lb, spec, sb)
        torch.cuda.synchronize()
        la.step_front(neck_back, blocks_front)
        s1.wait_stream(main)
        s2.wait_stream(main)
        with torch.cuda.stream(s1):
            lb.step_front(neck_back, blocks_front)
        with torch.cuda.stream(s2):
            got[f"a{rnd}"] = snap(la.step_back())
        main.wait_stream(s1)
        main.wait_stream(s2)
        got[f"b{rnd}"] = snap(lb.step_back())
        torch.cuda.synchronize()
    for name in ref:
        r, g = ref[name], got[name]
        assert int(r[2].sum()) > 0, name
        for b in range(2):
            n = int(r[2][b])
            assert n == int(g[2][b]), (name, b)
            assert torch.equal(r[0][b, :n], g[0][b, :n]), (name, b)
            assert torch.equal(r[1][b, :n], g[1][b, :n]), (name, b)


@pytest.mark.parametrize("front_after", [0, 1])
def test_lidar_front_next_pipelining_matches_step(cuda, front_after):
    """bench.py --lidar-pipeline 5: pipeline A's down blocks on one stream beside pipeline B's
    neck + head + decode + NMS and then B's preprocessing of its NEXT batch on another; the two
    pipelines swap roles every step.  Every batch gets exactly the detections of a plain step()."""
    spec = LidarSpec(rings=32, azimuth_steps=1024, sensor_height=3.23)
    la = LidarPipeline(batch=2, max_points=32768, device=cuda)
    _load_lidar(la, spec, [5, 6])
    la.calibrate_detection_density(500.0)
    lb = LidarPipeline(la.model, batch=2, max_points=32768, device=cuda)

    def snap(r):
        return [t.clone() for t in (r.box, r.score, r.count)]

    seeds = {"a1": [5, 6], "b1": [7, 8], "a2": [7, 8], "b2": [5, 6]}
    ref = {}
    for name in ("a1", "b1", "a2", "b2"):
        lp = la if name[0] == "a" else lb
        _load_lidar(lp, spec, seeds[name])
        ref[name] = snap(lp.step())
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    main = torch.cuda.current_stream()
    # prologue: A's canvas (a1), B's down blocks (b1)
    _load_lidar(la, spec, seeds["a1"])
    _load_lidar(lb, spec, seeds["b1"])
    la.step_pre()
    lb.step_front(neck_back=True)
    torch.cuda.synchronize()
    got = {}
    # step k: X = blocks on s1, Y = back + next front on s2; Y's data holds its next batch
    plan = [(la, lb, "b1", "b2"), (lb, la, "a1", "a2"), (la, lb, "b2", None), (lb, la, "a2", None)]
    ev = torch.cuda.Event()
    for x, y, done, nxt in plan:
        if nxt is not None:
            _load_lidar(y, spec, seeds[nxt])
        torch.cuda.synchronize()
        s1.wait_stream(main)
        s2.wait_stream(main)
        with torch.cuda.stream(s1):  # front_after: Y's next front waits for X's first down block
            x.step_blocks(mark=(x.fast.bb.convs_before(front_after), ev) if front_after else None)
        with torch.cuda.stream(s2):
            got[done] = snap(y.step_back())
            if nxt is not None:
                if front_after:
                    s2.wait_event(ev)
                y.step_pre()
        main.wait_stream(s1)
        main.wait_stream(s2)
        torch.cuda.synchronize()
    for name in ref:
        r, g = ref[name], got[name]
        assert int(r[2].sum()) > 0, name
        for b in range(2):
            n = int(r[2][b])
            assert n == int(g[2][b]), (name, b)
            assert torch.equal(r[0][b, :n], g[0][b, :n]), (name, b)
            assert torch.equal(r[1][b, :n], g[1][b, :n]), (name, b)


@pytest.mark.parametrize("lazy", [True, False], ids=["occ_clear", "full_clear"])
def test_lidar_occupancy_only_clear_matches_fresh_pipeline(cuda, monkeypatch, lazy):
    """With the fast plan's first conv gating its canvas loads on the occupancy bytes, a frame's
    clear resets only the previous frame's occupancy (not its features): a pipeline that ran other
    sweeps first gives exactly the voxels, occupancy, (masked) dense canvas, head maps and
    detections of a fresh one -- and so does the full clear."""
    import triton_client_amd.pipelines.lidar as lidar_mod
    monkeypatch.setattr(lidar_mod, "LAZY_CANVAS_CLEAR", lazy)
    spec = LidarSpec(rings=32, azimuth_steps=1024, sensor_height=3.23)
    la = LidarPipeline(batch=2, max_points=32768, device=cuda)
    # built before the calibration too: both pipelines take the same weights
    lf = LidarPipeline(la.model, batch=2, max_points=32768, device=cuda)
    _load_lidar(la, spec, [5, 6])
    la.calibrate_detection_density(500.0)
    la.step()
    assert la.enc.occ_gated == lazy and la.enc.pair
    _load_lidar(la, spec, [7, 8])
    ra = la.step()
    _load_lidar(lf, spec, [7, 8])
    rf = lf.step()
    torch.cuda.synchronize()
    same = {}
    vc = la.vox.voxel_count
    same["voxel_count"] = torch.equal(vc, lf.vox.voxel_count)
    for b in range(2):
        k = int(vc[b])
        same[f"coords{b}"] = torch.equal(la.vox.coords[b, :k], lf.vox.coords[b, :k])
        same[f"num_points{b}"] = torch.equal(la.vox.num_points[b, :k], lf.vox.num_points[b, :k])
    same["occ"] = torch.equal(la.enc.occ, lf.enc.occ)
    same["canvas"] = torch.equal(la.enc.canvas_nchw(), lf.enc.canvas_nchw())
    occ = la.enc.occ.bool()
    same["canvas_occupied"] = torch.equal(la.enc.canvas[occ], lf.enc.canvas[occ])
    same["depth"] = torch.equal(la.fast.bb.depth, lf.fast.bb.depth) if la.fast.bb.depth is not None else True
    same["hout"] = torch.equal(la.fast.hout.t, lf.fast.hout.t)
    same["count"] = torch.equal(ra.count, rf.count)
    for b in range(2):  # rows past a frame's count are scratch (a reused pipeline keeps older ones)
        k = int(ra.count[b])
        same[f"box{b}"] = torch.equal(ra.box[b, :k], rf.box[b, :k])
        same[f"score{b}"] = torch.equal(ra.score[b, :k], rf.score[b, :k])
    assert all(same.values()), {k: v for k, v in same.items() if not v}
    assert int(ra.count.min()) > 0
    if lazy:  # the old cells of frames 5 / 6 hold stale features: only the occupancy hides them
        stale = (la.enc.occ == 0) & (la.enc.canvas.abs().amax(-1) > 0)
        assert int(stale.sum()) > 0

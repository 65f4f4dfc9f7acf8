"""JPEG ingest on MI355X: the HIP IDCT + upsample + colour kernels against the
NumPy reference of the same stage (float64 IDCT) and against libjpeg (PIL)."""
import io

import numpy as np
import pytest
import torch
from PIL import Image

from triton_client_amd.ops import jpeg as J
from triton_client_amd.utils.synthetic import camera_frame

pytestmark = pytest.mark.gpu


def _jpeg(img, **kw):
    buf = io.BytesIO()
    Image.fromarray(img).save(buf, format="JPEG", quality=kw.pop("quality", 90), **kw)
    return buf.getvalue()


@pytest.mark.parametrize("sub", [2, 1, 0])
@pytest.mark.parametrize("hw", [(720, 1280), (181, 243)])
def test_gpu_reconstruction_matches_reference(cuda, sub, hw):
    B = 3
    frames = [camera_frame(*hw, seed=s) for s in range(B)]
    jpegs = [_jpeg(f, subsampling=sub, restart_marker_rows=(1 if sub == 2 else 0)) for f in frames]
    dec = J.JpegBatchDecoder(B, cuda, threads=3)
    out = torch.zeros((B, hw[0], hw[1], 3), dtype=torch.uint8, device=cuda)
    dec.decode(jpegs, out)
    torch.cuda.synchronize()
    got = out.cpu().numpy().astype(int)
    for i, j in enumerate(jpegs):
        c, q, geo = J.decode_coefficients(j)
        ref = J.reconstruct_numpy(c, q, geo).astype(int)
        d = np.abs(got[i] - ref)  # fp32 vs fp64 IDCT: a rounding tie may flip
        assert d.max() <= 3 and (d > 0).mean() < 1e-3, (d.max(), (d > 0).mean())
        d2 = np.abs(got[i] - J.decode_pil(j).astype(int))
        assert d2.mean() < 0.1 and d2.max() <= 4, (d2.mean(), d2.max())
    assert dec.stats["fallback"] == 0


def test_gpu_decoder_fallback_and_slot_rotation(cuda):
    """A progressive frame falls back to the host decode; three batches in a
    row through two pinned slots stay frame-exact."""
    B, hw = 4, (96, 128)
    frames = [camera_frame(*hw, seed=10 + s) for s in range(3 * B)]
    dec = J.JpegBatchDecoder(B, cuda, threads=2, slots=2)
    out = torch.zeros((B, *hw, 3), dtype=torch.uint8, device=cuda)
    for b in range(3):
        chunk = frames[b * B:(b + 1) * B]
        jpegs = [_jpeg(f, progressive=(b == 1 and i == 2)) for i, f in enumerate(chunk)]
        dec.upload(dec.stage(jpegs))
        dec.reconstruct(out)
        torch.cuda.synchronize()
        got = out.cpu().numpy().astype(int)
        for i, j in enumerate(jpegs):
            ref = J.decode_pil(j).astype(int)
            d = np.abs(got[i] - ref)
            if b == 1 and i == 2:
                assert d.max() == 0  # host fallback: libjpeg's own pixels
            else:
                assert d.mean() < 0.1 and d.max() <= 4
    assert dec.stats["fallback"] == 1

"""JPEG ingest, host half (csrc/runtime/jpeg_entropy.cpp) and the NumPy
reference of the GPU half (ops/jpeg.py reconstruct_numpy), against PIL's
libjpeg decode of the same files."""
import ctypes
import io

import numpy as np
import pytest
from PIL import Image

from triton_client_amd.ops import jpeg as J
from triton_client_amd.utils.synthetic import camera_frame


def _jpeg(img, **kw):
    buf = io.BytesIO()
    im = Image.fromarray(img)
    if kw.pop("gray", False):
        im = im.convert("L")
    im.save(buf, format="JPEG", quality=kw.pop("quality", 90), **kw)
    return buf.getvalue()


CASES = {
    "420": dict(subsampling=2),
    "422": dict(subsampling=1),
    "444": dict(subsampling=0),
    "420_restart_blocks": dict(subsampling=2, restart_marker_blocks=5),
    "420_restart_rows": dict(subsampling=2, restart_marker_rows=1),
    "420_q100": dict(subsampling=2, quality=100),
    "420_q30": dict(subsampling=2, quality=30),
    "gray": dict(gray=True),
}


@pytest.mark.parametrize("case", list(CASES))
@pytest.mark.parametrize("hw", [(181, 243), (64, 64), (40, 49)])
def test_entropy_decode_and_reconstruction_match_libjpeg(case, hw):
    """Odd sizes exercise MCU padding and the upsampling edge rules.  The
    reconstruction uses a float IDCT where libjpeg uses its integer one, so
    pixels may differ by 1 level in a plane, a few after YCbCr->RGB."""
    data = _jpeg(camera_frame(*hw, seed=7), **dict(CASES[case]))
    if "restart" in case:
        assert b"\xff\xdd" in data  # DRI present: the restart path is exercised
    coef, q, geo = J.decode_coefficients(data)
    assert (geo.width, geo.height) == (hw[1], hw[0])
    got = J.reconstruct_numpy(coef, q, geo).astype(int)
    ref = J.decode_pil(data).astype(int)
    d = np.abs(got - ref)
    assert d.mean() < 0.1, d.mean()
    assert d.max() <= (1 if case == "gray" else 4), d.max()


def test_sampling_geometry():
    img = camera_frame(100, 130, seed=1)
    g = J.probe(_jpeg(img, subsampling=2))
    assert g.sampling[:1] == ((2, 2),) and g.sampling[1:] == ((1, 1), (1, 1))
    assert (g.mcux, g.mcuy) == (9, 7) and g.nblocks == 9 * 7 * 4 + 2 * 9 * 7 and g.gpu_ok
    g = J.probe(_jpeg(img, subsampling=1))
    assert g.sampling[0] == (2, 1) and (g.mcux, g.mcuy) == (9, 13)
    g = J.probe(_jpeg(img, gray=True))
    assert g.nc == 1 and g.nblocks == 17 * 13


def test_unsupported_and_corrupt_inputs_fail_cleanly():
    img = camera_frame(64, 80, seed=2)
    with pytest.raises(ValueError, match="unsupported"):
        J.decode_coefficients(_jpeg(img, progressive=True))
    with pytest.raises(ValueError, match="not a JPEG"):
        J.probe(b"\x89PNG\r\n\x1a\n" + bytes(100))
    good = _jpeg(img)
    with pytest.raises(ValueError):
        J.probe(good[:40])  # truncated inside the headers
    # fuzz: truncations and byte flips never crash the decoder; they either
    # decode (garbage pixels) or report an error
    rng = np.random.default_rng(0)
    coef = np.empty((4096, 64), np.int16)
    q = np.empty(192, np.float32)
    g = np.zeros(16, np.int32)
    rt = J._rt()
    for trial in range(300):
        b = bytearray(good)
        if trial % 2:
            b = b[: rng.integers(2, len(b))]
        for _ in range(rng.integers(1, 8)):
            b[rng.integers(0, len(b))] = rng.integers(0, 256)
        b = bytes(b)
        rc = rt.tca_jpeg_decode_coefs(b, len(b), coef.ctypes.data, 4096, q.ctypes.data, g.ctypes.data)
        assert rc in (0, -1, -2, -3, -4, -5)


def _dht_tables(data):
    """(offset of the 16 counts, nsym) of every Huffman table in every DHT segment."""
    out = []
    p = 2
    while p + 4 < len(data):
        if data[p] == 0xFF and data[p + 1] == 0xC4:
            end = p + 2 + (data[p + 2] << 8 | data[p + 3])
            t = p + 4
            while t + 17 <= end:
                nsym = sum(data[t + 1:t + 17])
                out.append((t + 1, nsym))
                t += 17 + nsym
            p = end
        else:
            p += 1
    return out


@pytest.mark.parametrize("variant", ["all_len1", "three_len1"])
def test_oversubscribed_huffman_table_is_rejected(variant):
    """A DHT whose code counts over-subscribe a length (counts[0] >= 3) must be
    rejected before the fast lookup table is filled (its index would run past
    the table).  The segment length stays consistent, so only the code-space
    check can catch it."""
    good = _jpeg(camera_frame(48, 64, seed=3))
    tables = _dht_tables(good)
    assert tables
    coef = np.empty((4096, 64), np.int16)
    q = np.empty(192, np.float32)
    g = np.zeros(16, np.int32)
    rt = J._rt()
    for off, nsym in tables:
        b = bytearray(good)
        counts = [0] * 16
        if variant == "all_len1":
            counts[0] = nsym
        else:
            last = max(i for i in range(16) if good[off + i])
            counts[0], counts[last] = 3, nsym - 3
        b[off:off + 16] = bytes(counts)
        with pytest.raises(ValueError):
            J.probe(bytes(b))
        rc = rt.tca_jpeg_decode_coefs(bytes(b), len(b), coef.ctypes.data, 4096, q.ctypes.data, g.ctypes.data)
        assert rc < 0


def test_batch_decode_threads_and_status():
    """tca_jpeg_decode_batch on 4 threads == one-by-one decode; a progressive
    frame in the batch reports its error without disturbing the others."""
    frames = [camera_frame(72, 96, seed=s) for s in range(6)]
    jpegs = [_jpeg(f) for f in frames]
    jpegs[3] = _jpeg(frames[3], progressive=True)
    geo = J.probe(jpegs[0])
    n = len(jpegs)
    coef = np.zeros((n, geo.nblocks, 64), np.int16)
    q = np.zeros((n, 192), np.float32)
    g = np.zeros((n, 16), np.int32)
    st = np.full(n, 7, np.int32)
    ptrs = (ctypes.c_char_p * n)(*jpegs)
    lens = (ctypes.c_int64 * n)(*[len(j) for j in jpegs])
    failed = J._rt().tca_jpeg_decode_batch(ptrs, lens, n, coef.ctypes.data, geo.nblocks, q.ctypes.data,
                                           g.ctypes.data, st.ctypes.data, 4)
    assert failed == 1 and st[3] == -2 and (np.delete(st, 3) == 0).all()
    for i in (0, 1, 2, 4, 5):
        c1, q1, _ = J.decode_coefficients(jpegs[i])
        np.testing.assert_array_equal(coef[i], c1)
        np.testing.assert_array_equal(q[i], q1.reshape(-1))

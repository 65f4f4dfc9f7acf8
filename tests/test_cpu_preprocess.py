"""Host preprocess (csrc/runtime/cpu_image.cpp) == the NumPy golden, bit for
bit, and the config-1 tool (single JPEG over gRPC to a CPU-only server) runs."""
import json

import numpy as np
import pytest
import torch

from triton_client_amd.ops import golden as G
from triton_client_amd.ops import image as I
from triton_client_amd.utils.synthetic import camera_frame


@pytest.mark.parametrize("mode", ["stretch", "letterbox"])
@pytest.mark.parametrize("layout", ["NCHW", "NHWC"])
@pytest.mark.parametrize("swap", [False, True])
def test_native_cpu_preprocess_matches_golden(mode, layout, swap):
    assert I._cpu_runtime() is not None  # the C++ path is the one under test
    f = torch.from_numpy(np.stack([camera_frame(181, 243, s) for s in range(2)]))
    o, _ = I.preprocess(f, (96, 128), mode, "COCO", torch.float32, layout, swap_rb=swap)
    sc, bi = I.SCALING_PRESETS["COCO"]
    ref = np.stack([G.preprocess_image(f[b].numpy(), (96, 128), mode, sc, bi, swap, 114.0, "NCHW") for b in range(2)])
    np.testing.assert_array_equal(o.contiguous().numpy(), ref)


def test_config1_tool_runs(capsys):
    from tools.config1_bench import main

    assert main(["--frames", "2", "--warmup", "1", "--cam", "240x320"]) == 0
    line = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert line["value"] > 0 and line["device"] == "cpu" and line["stages_ms"]["server_compute"] > 0

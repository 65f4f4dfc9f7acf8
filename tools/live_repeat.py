"""Run tests/test_live.py::test_live_drivers_publish_engine_results N times in one process
(the two live drivers building their engines concurrently), with a per-run progress line."""
import sys
import time

sys.path.insert(0, ".")
sys.path.insert(0, "tests")


def main():
    import torch

    import test_live
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    dev = torch.device("cuda")
    for i in range(n):
        t = time.perf_counter()
        test_live.test_live_drivers_publish_engine_results(dev)
        print(f"run {i}: ok in {time.perf_counter() - t:.1f}s", flush=True)


if __name__ == "__main__":
    main()

import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

# Run order of the suite (the driver runs `pytest -m gpu -x` under one wall-time limit): the per-row
# oracle tests first — reward stack / obs / reset / info against the reference's recorded outputs,
# the benchmarked configs' flows, K2 on the 264 reference frames, video, the emulator parity file —
# then the surface tests, and the long-horizon file last, so that a slow box cuts the most
# redundant coverage, never the only test of a §8 row.
FILE_ORDER = (
    "test_gpu_reward.py",
    "test_gpu_scale.py",
    "test_k2_frames.py",
    "test_video.py",
    "test_gpu_parity.py",
    "test_gpu_env.py",
    "test_gpu_batching.py",
    "test_bench_contract.py",
    "test_pyboy_external.py",
)
LAST = ("test_gpu_horizon.py",)


def file_rank(fname: str) -> int:
    if fname in LAST:
        return len(FILE_ORDER) + 1 + LAST.index(fname)
    if fname in FILE_ORDER:
        return FILE_ORDER.index(fname)
    return len(FILE_ORDER)          # CPU-only files: between the GPU files and the horizon


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs under gpurun)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.hookimpl(trylast=True)
def pytest_collection_modifyitems(session, config, items):
    # after pytest's own fixture-scope reordering; the sort is stable, so the order inside a file
    # (and of a module fixture's parametrisations) is kept
    items.sort(key=lambda it: file_rank(os.path.basename(str(it.fspath))))

"""The GPU suite's run order (tests/conftest.py): the driver runs `pytest -m gpu -x` under one
wall-time limit, so the per-row oracle tests (reward stack, obs, reset, info, the benchmarked
configs' flows, K2 frames, video, emulator parity) must run before the long-horizon file, and the
horizon file must hold only the launch shapes the benchmark takes."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _collected(*args):
    env = dict(os.environ)
    env.pop("PK_HORIZON_EXTENDED", None)
    out = subprocess.run([sys.executable, "-m", "pytest", "tests", "--collect-only", "-q", *args],
                         cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    return [ln.split("::")[0] for ln in out.stdout.splitlines() if "::" in ln], \
        [ln for ln in out.stdout.splitlines() if "::" in ln]


def test_gpu_suite_runs_oracle_rows_first_and_horizon_last():
    files, ids = _collected("-m", "gpu")
    first = {f: files.index(f) for f in dict.fromkeys(files)}
    order = list(first)
    # every file's tests are contiguous
    for f in order:
        k = first[f]
        assert all(x == f for x in files[k:k + files.count(f)]), f
    assert order[0] == "tests/test_gpu_reward.py"
    assert order[1] == "tests/test_gpu_scale.py"
    assert order[-1] == "tests/test_gpu_horizon.py"
    for f in ("tests/test_k2_frames.py", "tests/test_video.py", "tests/test_gpu_parity.py"):
        assert first[f] < first["tests/test_gpu_horizon.py"]
    # the horizon holds the benchmarked shapes only, parts in order within each shape
    seg = [i for i in ids if "test_horizon_10k_segments[" in i]
    shapes = list(dict.fromkeys(i.split("[")[1].rsplit("-", 1)[0] for i in seg))
    assert shapes == ["small_l32", "small_l16", "wg512_l32", "auto"], shapes
    for s in shapes:
        parts = [int(i.rsplit("-", 1)[1].rstrip("]")) for i in seg if f"[{s}-" in i]
        assert parts == sorted(parts)

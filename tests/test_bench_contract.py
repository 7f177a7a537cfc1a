"""bench.py's output contract and the evidence it cites.

CPU: every committed PMC stamp (profiles/pmc_<workload>.json, what a bench line reports as
`roofline.traffic`, `roofline.issue` and `pmc_stamp`) carries the fields the line reads, and the
rocprofv3 kernel-stats file it names as its source exists in the repo and agrees with the stamp's
K1 average.  GPU: one short `python bench.py` run prints ONE JSON line with the driver's keys, a
`roofline` object whose achieved/peak/frac are consistent, and a `value` that is the env-steps of
the timed steps over the timed span."""
import csv
import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

WORKLOADS = ("config2", "config3", "config4", "config5")


@pytest.mark.parametrize("w", WORKLOADS)
def test_pmc_stamp_fields_and_source(w):
    path = os.path.join(HERE, "profiles", f"pmc_{w}.json")
    d = json.load(open(path))
    for k in ("hbm_bytes_per_launch_k1", "hbm_bytes_per_env_step_k1", "envs_per_launch", "valu_busy_pct",
              "valu_utilization_pct", "wait_any_pct", "k1_avg_ms_rocprof_stats", "issue", "source"):
        assert k in d, k
    assert d["hbm_bytes_per_launch_k1"] == pytest.approx(d["hbm_bytes_per_env_step_k1"] * d["envs_per_launch"], rel=1e-3)
    isa = d["issue"]["isa_per_emulated_instr"]
    assert isa["total"] == pytest.approx(sum(v for k, v in isa.items() if k != "total"), abs=0.5)
    # the cited kernel-stats CSV is committed, and its K1 average is the stamp's
    files = [t for t in d["source"].split() if t.startswith("profiles/")]
    stats = [f for f in files if f.endswith("_kernel_stats.csv")]
    assert stats, d["source"]
    for f in files:
        assert os.path.exists(os.path.join(HERE, f)), f
    # the VecEnv workloads (two concurrent sub-batch launches) are counted at the timed steps'
    # occupancy, two waves per SIMD (2,048 waves on 1,024 SIMDs), and say so; the serialised
    # one-launch record sits beside it
    if w != "config2":
        assert "two waves per SIMD" in d.get("regime", ""), w
        assert d["waves_per_launch"] == 2048 and "serialised_record" in d
        assert d["serialised_record"]["waves_per_launch"] == 1024
    rows = list(csv.DictReader(open(os.path.join(HERE, stats[0]))))
    k1 = [r for r in rows if "pk_step_kernel" in r["Name"]]
    assert k1, stats[0]
    assert float(k1[0]["AverageNs"]) / 1e6 == pytest.approx(d["k1_avg_ms_rocprof_stats"], rel=1e-3)


def test_cpu_quota_parses():
    import bench
    cores, raw = bench._cpu_quota()
    assert cores is None or cores >= 1


@pytest.mark.gpu
def test_bench_line_contract():
    out = subprocess.run([sys.executable, os.path.join(HERE, "bench.py"), "--steps", "3", "--warmup", "1",
                          "--no-cpu-baseline"], capture_output=True, text=True, timeout=240, cwd=HERE)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1 and d["higher_is_better"] is True
    assert "workload" in d["config"]
    envs = d["config"]["envs_per_gpu"]
    assert d["value"] == pytest.approx(envs * 1000.0 / d["ms_per_step"], rel=0.02)
    r = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], rel=1e-2)
    assert 0 < r["k1_ms"] <= r["span_ms"] <= d["ms_per_step"] * 1.05
    # the per-GPU rate of the whole step (concurrent sub-batch launches together)
    assert r["achieved_per_step"] == pytest.approx(r["bytes_per_env_step"] * envs / (d["ms_per_step"] / 1e3) / 1e9,
                                                   rel=0.02)
    assert r["frac_per_step"] == pytest.approx(r["achieved_per_step"] / r["peak"], rel=1e-2)
    c = d["collectives"]
    assert c["fired_in_timed_steps"] == c["expected_in_timed_steps"]

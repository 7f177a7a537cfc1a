"""Multi-GPU path on CPU: env sharding, the episode-statistics all-reduce over gloo
(world_size 2), and sharded emulation == single-process emulation for the same env ids
(host-simulation build of the HIP kernels on each rank)."""
import hashlib
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pokegym_amd.dist import STAT_FIELDS, EpisodeStats, InfoStats, shard_range
from pokegym_amd.info import NFIELDS

HERE = os.path.dirname(os.path.abspath(__file__))


def test_shard_range_partitions_contiguously():
    for n in (1, 7, 64, 262144, 262145):
        for w in (1, 2, 3, 8):
            rs = [shard_range(n, w, r) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in rs]
            assert max(sizes) - min(sizes) <= 1


def test_episode_stats_accumulate():
    st = EpisodeStats(3, "cpu")
    r = torch.tensor([1.0, 2.0, 3.0], dtype=torch.float64)
    st.update(r, torch.tensor([0, 0, 0], dtype=torch.uint8))
    st.update(r, torch.tensor([1, 0, 0], dtype=torch.uint8))
    st.update(r, torch.tensor([0, 1, 1], dtype=torch.uint8))
    s = st.allreduce()
    assert s["episodes"] == 3
    assert s["episodic_return_sum"] == 2.0 + 6.0 + 9.0
    assert s["episode_length_sum"] == 2 + 3 + 3
    assert s["steps"] == 9 and s["reward_sum"] == 18.0
    assert st.ep_return.tolist() == [1.0, 0.0, 0.0]
    # the summary covers one logging interval; the open episode keeps its running return
    st.update(r, torch.tensor([1, 0, 0], dtype=torch.uint8))
    s = st.allreduce()
    assert s["episodes"] == 1 and s["episodic_return_sum"] == 2.0 and s["steps"] == 3
    assert st.allreduce(reset=False)["episodes"] == 0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir, fn):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fn(rank, world, out_dir)
    finally:
        dist.destroy_process_group()


def _stats_fn(rank, world, out_dir):
    st = EpisodeStats(4, "cpu")
    r = torch.full((4,), float(rank + 1), dtype=torch.float64)
    st.update(r, torch.tensor([1, 0, 1, 0], dtype=torch.uint8))
    s = st.allreduce()
    with open(os.path.join(out_dir, f"stats{rank}.txt"), "w") as f:
        f.write(repr([s[k] for k in STAT_FIELDS]))


def test_stats_allreduce_gloo_world2(tmp_path):
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path), _stats_fn), nprocs=2, join=True)
    got = [eval(open(tmp_path / f"stats{r}.txt").read()) for r in range(2)]
    # episodes: 2 per rank; returns: 2*1 + 2*2; lengths 4; reward sums 4*1 + 4*2; steps 8
    assert got[0] == got[1] == [6.0, 4.0, 4.0, 12.0, 8.0]


def test_info_stats_mean_of_emitted_records():
    st = InfoStats("cpu")
    info = torch.arange(NFIELDS * 3, dtype=torch.float64).reshape(NFIELDS, 3)
    st.update(info, torch.tensor([1, 0, 1], dtype=torch.uint8))
    st.update(info * 0, torch.tensor([0, 0, 0], dtype=torch.uint8))
    s = st.allreduce()
    assert s["info_records"] == 2
    assert s["stats"]["step"] == (0 + 2) / 2 and s["reward"]["has_bicycle_in_bag_reward"] == (NFIELDS - 1) * 3 + 1
    assert st.sum.abs().sum() == 0   # reset after the read


def _info_fn(rank, world, out_dir):
    st = InfoStats("cpu")
    info = torch.full((NFIELDS, 4), float(rank + 1), dtype=torch.float64)
    st.update(info, torch.tensor([1, 1, 0, rank], dtype=torch.uint8))
    s = st.allreduce()
    with open(os.path.join(out_dir, f"info{rank}.txt"), "w") as f:
        f.write(repr([s["info_records"], s["stats"]["money"], s["reward"]["delta"]]))


def test_info_stats_allreduce_gloo_world2(tmp_path):
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path), _info_fn), nprocs=2, join=True)
    got = [eval(open(tmp_path / f"info{r}.txt").read()) for r in range(2)]
    # rank 0: 2 records of 1.0, rank 1: 3 records of 2.0 -> mean 8/5
    assert got[0] == got[1] == [5.0, 1.6, 1.6]


N_ENVS, STEPS = 6, 2


def _actions():
    return np.random.default_rng(3).integers(0, 8, (STEPS, N_ENVS)).astype(np.uint8)


def _run_hostsim(env_ids, acts):
    sys.path.insert(0, os.path.join(HERE, "hostsim"))
    from sim import SimEmulator
    from pokegym_amd.testrom.game import game_rom
    emu = SimEmulator(game_rom(), len(env_ids), None, render=True)
    for t in range(STEPS):
        emu.step(acts[t, env_ids])
    out = [hashlib.sha1(emu.snapshot(i)).hexdigest() for i in range(len(env_ids))]
    emu.close()
    return out


def _shard_fn(rank, world, out_dir):
    a, b = shard_range(N_ENVS, world, rank)
    hashes = _run_hostsim(list(range(a, b)), _actions())
    allh = [None] * world
    dist.all_gather_object(allh, hashes)
    if rank == 0:
        with open(os.path.join(out_dir, "shards.txt"), "w") as f:
            f.write(repr([h for part in allh for h in part]))


@pytest.mark.slow
def test_sharded_emulation_equals_single_process(tmp_path):
    single = _run_hostsim(list(range(N_ENVS)), _actions())
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path), _shard_fn), nprocs=2, join=True)
    assert eval(open(tmp_path / "shards.txt").read()) == single


FLOW_ENVS, FLOW_STEPS, FLOW_LOG = 8, 6, 3


def _flow_fn(rank, world, out_dir):
    """bench.py's StepFlow (the timed per-step unit of configs[2]..[4]) on a host-simulated shard."""
    sys.path.insert(0, os.path.dirname(HERE))
    import bench
    from tests.hostsim.emulator import HostsimEmulator
    from pokegym_amd.env import VecEnv
    from pokegym_amd.testrom.game import game_rom
    rom = game_rom()
    acts = torch.from_numpy(np.random.default_rng(7 + rank).integers(0, 8, (FLOW_STEPS, FLOW_ENVS)).astype(np.uint8))
    out = {}
    # configs[4] (reward stack, template reload on done, 2-step episodes) and configs[3] (screen obs):
    # VecEnv recv/send with auto-reset, its logging-interval all-reduce
    for name, kw in (("c5", dict(reward=True, reload_on_reset=True)), ("c4", dict(render=True))):
        emu = HostsimEmulator(rom, FLOW_ENVS, max_episode_steps=2, **kw)
        vec = VecEnv(FLOW_ENVS, emulator=emu, log_interval=FLOW_LOG, max_episode_steps=2)
        vec.async_reset()
        f = bench.StepFlow(emu, vec, world, FLOW_LOG, "cpu")
        f.acts = acts
        for t in range(FLOW_STEPS + 1):   # the last logging record is returned by the next recv
            f.step(t % FLOW_STEPS, False)
        out[name] = [{k: (float(v) if not isinstance(v, dict) else {a: float(b) for a, b in v.items()})
                      for k, v in d.items()} for d in f.vec_logs]
        vec.close()
    with open(os.path.join(out_dir, f"flow{rank}.txt"), "w") as fh:
        fh.write(repr(out))


@pytest.mark.slow
def test_bench_flow_gloo_world2(tmp_path):
    """bench.py's per-step flow for configs[4] (VecEnv with the reward stack: step, per-env template
    reload on done, episode/info-statistics all-reduce every FLOW_LOG steps) and configs[3] (screen
    obs) on two gloo ranks, each stepping its own host-simulated shard: the collectives fire inside
    the run and every rank sees the sum over both shards."""
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path), _flow_fn), nprocs=2, join=True)
    got = [eval(open(tmp_path / f"flow{r}.txt").read(), {"nan": float("nan")}) for r in range(2)]
    for name in ("c5", "c4"):
        logs = [g[name] for g in got]
        # two logging records per rank, identical on both ranks (all-reduced); 2-step episodes end at
        # steps 2 | 4, 6 of the two intervals, on 2 x FLOW_ENVS envs
        assert len(logs[0]) == len(logs[1]) == FLOW_STEPS // FLOW_LOG
        assert repr(logs[0]) == repr(logs[1])
        assert [d["episodes"] for d in logs[0]] == [2 * FLOW_ENVS * 1, 2 * FLOW_ENVS * 2]
    # the reward flow also all-reduces the info records (one per done)
    assert [d["info_records"] for d in got[0]["c5"]] == [2 * FLOW_ENVS * 1, 2 * FLOW_ENVS * 2]

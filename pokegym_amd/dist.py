"""Multi-GPU sharding of envs (one process per GPU) and the episode-statistics all-reduce.

Envs are independent, so env.step has no data-path collective: rank g of W
owns the contiguous env-id range shard_range(N, W, g) and runs it on its own GPU.  The only
collective is the all-reduce (sum) of a few float64 episode statistics per logging interval —
over RCCL/xGMI on MI355X (backend "nccl"), or gloo on CPU.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

STAT_FIELDS = ("episodic_return_sum", "episodes", "episode_length_sum", "reward_sum", "steps")


def shard_range(num_envs: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [start, end) env ids of `rank`; sizes differ by at most one."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} not in [0, {world})")
    base, extra = divmod(num_envs, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def env_rank() -> tuple[int, int, int]:
    """(rank, world, local_rank) from the torchrun environment (1 process = 1 GPU)."""
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("LOCAL_RANK", "0"))


class EpisodeStats:
    """Device-resident per-env episode accumulators + a 5-float64 summary all-reduced over ranks.
    With sub-batches (VecEnv batch_size < num_envs, each stepped on its own stream) every
    sub-batch accumulates into its own summary row, so concurrent updates never share a tensor."""

    def __init__(self, n: int, device, nbatches: int = 1):
        self.device = torch.device(device)
        self.ep_return = torch.zeros(n, dtype=torch.float64, device=self.device)
        self.ep_length = torch.zeros(n, dtype=torch.float64, device=self.device)
        self.summary = torch.zeros((nbatches, len(STAT_FIELDS)), dtype=torch.float64, device=self.device)
        self.snap = torch.zeros_like(self.summary)   # rows taken at a deferred logging interval (snapshot)

    def update(self, rewards: torch.Tensor, done: torch.Tensor, batch: int = 0, envs: slice = slice(None)):
        """Accumulate one step of the envs `envs` (rewards/done cover exactly those envs);
        finished episodes move into the summary row `batch` (no host sync)."""
        d = done.to(torch.float64)
        ret, length = self.ep_return[envs], self.ep_length[envs]
        ret.add_(rewards.to(torch.float64))
        length.add_(1.0)
        s = self.summary[batch]
        s[0] += (ret * d).sum()
        s[1] += d.sum()
        s[2] += (length * d).sum()
        s[3] += rewards.to(torch.float64).sum()
        s[4] += float(rewards.numel())
        keep = 1.0 - d
        ret.mul_(keep)
        length.mul_(keep)

    def snapshot(self, batch: int):
        """Move sub-batch row `batch` into the snapshot and restart it, on the current stream (the
        sub-batch's own: stream-ordered after its last update, no host sync)."""
        self.snap[batch].copy_(self.summary[batch])
        self.summary[batch].zero_()

    def allreduce(self, group=None, reset: bool = True, snapshot: bool = False) -> dict:
        """Sum the summaries of all ranks (RCCL over xGMI when the tensors live on GPUs).  With
        reset (the default, like InfoStats) the summary restarts, so each call covers one logging
        interval; per-env episodes in progress keep accumulating.  snapshot=True sums the rows
        snapshot() took instead (they were restarted then)."""
        out = (self.snap if snapshot else self.summary).sum(dim=0)
        if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
            dist.all_reduce(out, op=dist.ReduceOp.SUM, group=group)
        if reset and not snapshot:
            self.summary.zero_()
        vals = out.tolist()
        res = dict(zip(STAT_FIELDS, vals))
        res["mean_episodic_return"] = vals[0] / vals[1] if vals[1] else float("nan")
        res["mean_episode_length"] = vals[2] / vals[1] if vals[1] else float("nan")
        return res

    def reset_summary(self):
        self.summary.zero_()


class InfoStats:
    """Device-side sum of the info telemetry records (pokegym_amd/info.py) of every env that emitted
    one, plus their count; all-reduced and averaged per logging interval, like PufferLib's mean over
    the info dicts its envs returned."""

    def __init__(self, device, nbatches: int = 1):
        from .info import NFIELDS
        self.device = torch.device(device)
        # one row per sub-batch (concurrent streams); last column = count
        self.sum = torch.zeros((nbatches, NFIELDS + 1), dtype=torch.float64, device=self.device)
        self.snap = torch.zeros_like(self.sum)   # rows taken at a deferred logging interval (snapshot)

    def update(self, info: torch.Tensor, flag: torch.Tensor, batch: int = 0):
        """info: f64 (NFIELDS, m) view, flag: (m,) 0/1 of the same envs — one GEMV, no host sync."""
        f = flag.to(torch.float64)
        row = self.sum[batch]
        row[:-1] += torch.mv(info, f)
        row[-1] += f.sum()

    def snapshot(self, batch: int):
        """As EpisodeStats.snapshot."""
        self.snap[batch].copy_(self.sum[batch])
        self.sum[batch].zero_()

    def allreduce(self, group=None, reset: bool = True, snapshot: bool = False) -> dict:
        from .info import REWARD_FIELDS, STATS_FIELDS
        out = (self.snap if snapshot else self.sum).sum(dim=0)
        if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
            dist.all_reduce(out, op=dist.ReduceOp.SUM, group=group)
        if reset and not snapshot:
            self.sum.zero_()
        vals = out.tolist()
        n = vals[-1]
        mean = [v / n if n else float("nan") for v in vals[:-1]]
        ns = len(STATS_FIELDS)
        return {"info_records": n, "stats": dict(zip(STATS_FIELDS, mean[:ns])),
                "reward": dict(zip(REWARD_FIELDS, mean[ns:]))}

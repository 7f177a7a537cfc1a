"""Gymnasium- and PufferLib-shaped surfaces over the batched MI355X env.step.

`Environment` is the drop-in for pokegym.environment.Environment (environment.py:436-1812): same
constructor arguments, reset(seed, options, max_episode_steps, reward_scale) -> (obs, info),
step(action) -> (obs, reward, terminated, truncated, info), close(); observation (72, 80, 4) u8,
Discrete(8) actions.  Where the reference raises inside step/reset, the same exception type is
raised here (the device reports it per env, include/pokegym_amd.h PK_ERR_*).

`VecEnv` is the PufferLib-style batch of N envs on ONE GPU (the intended way to use the device):
reset(seed) -> (obs, infos); step(actions) -> (obs, rewards, terminals, truncations, infos);
async_reset/send/recv; single_observation_space, single_action_space, num_envs.  Finished envs
are reset inside step (their returned obs is the first obs of the next episode), stream-ordered
with no host synchronisation; episode statistics are accumulated on the device and all-reduced
across ranks every `log_interval` steps (pokegym_amd.dist; with sub-batches the record is read one
env-step after the interval, from per-stream snapshots, so the pipeline never drains).  For several GPUs, run one process
per GPU and build each rank's shard with `make_sharded_vecenv`.
"""
from __future__ import annotations

import io
import os
import random
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

from . import spaces
from .dist import EpisodeStats, InfoStats, env_rank, shard_range

HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT_STATE = os.path.join(HERE, "states", "Bulbasaur.state")  # environment.py:119-120


def _session_path(env_id: int) -> Path:
    """environment.py:130-140: experiments/{running experiment name}/sessions/{env_id}."""
    name = "default_exp_name"
    try:
        with open(os.path.join("experiments", "running_experiment.txt")) as f:
            name = f.read().strip() or name
    except OSError:
        pass
    return Path("experiments") / name / "sessions" / str(env_id)


def _read(path_or_bytes):
    if path_or_bytes is None or isinstance(path_or_bytes, (bytes, bytearray)):
        return path_or_bytes
    with open(path_or_bytes, "rb") as f:
        return f.read()


class Base:
    """pokegym.environment.Base (environment.py:89-434): the emulator surface without the reward
    stack — step(action) runs the action and returns (render(), 0, False, False, {}) (:404-406),
    reset() returns the current screen without touching the game (:228-230), plus the savestate,
    screenshot and video helpers Environment inherits.  As there, the template state is kept in
    initial_states but not loaded (make_env boots the ROM, :116-122), and render() keeps its own
    visited-tile memory per map (:157-160, :256-272), here on the device."""

    _next_id = 0

    def __init__(self, rom_path="pokemon_red.gb", state_path=None, headless=True, save_video=False, quiet=False,
                 device: int = 0, **kwargs):
        state = _read(state_path if state_path is not None else DEFAULT_STATE)
        self.emu = self._emulator(_read(rom_path), state, device)
        self.observation_space = spaces.observation_space()
        self.action_space = spaces.action_space()
        self.headless = headless
        self.initial_states = [io.BytesIO(state)]   # environment.py:119-122 (the template state)
        self.pokemon_center_save_states = []
        # video / screenshots (environment.py:123, :128, :140, :200-206, :1244-1249, :1340, :1616)
        self.save_video = save_video
        self.screenshot_counter = 0
        self.reset_count = 0
        self.env_id = Base._next_id
        Base._next_id += 1
        self.s_path = Path(kwargs["s_path"]) if "s_path" in kwargs else _session_path(self.env_id)
        self._recorder = None
        if save_video:
            from .video import FrameRecorder
            self._recorder = FrameRecorder(self.emu, [0])
        self.screen_memory = {}     # map -> (255, 255) u8 device tensor (environment.py:157-160)

    def _emulator(self, rom, state, device):
        # the ROM boots; the template state only goes into initial_states (environment.py:116-122)
        from .emulator import BatchedEmulator
        return BatchedEmulator(rom, 1, state=None, device=device, render=True)

    def video(self):
        """environment.py:408-410: the current (144, 160, 3) screen."""
        from .video import to_rgb
        return to_rgb(self.emu.screen[0].cpu().numpy())

    def add_video_frame(self):
        """environment.py:621-622 (the frame stays on the device until the episode is written)."""
        self._recorder.capture()

    def save_screenshot(self, event, map_n):
        """environment.py:200-206: screenshots/{counter}_{event}_{map_n}.jpeg."""
        from .video import save_screenshot
        self.screenshot_counter += 1
        return save_screenshot(self.emu.screen[0].cpu().numpy(), event, map_n, self.screenshot_counter)

    # -- savestates (environment.py:208-227): PyBoy v9 images of the device state --------------
    def save_state(self):
        """environment.py:208-213: append the current machine state (v9 savestate) to
        pokemon_center_save_states."""
        self.pokemon_center_save_states.append(io.BytesIO(self.emu.snapshot(0)))

    def load_pokemon_center_state(self):
        return self.pokemon_center_save_states[len(self.pokemon_center_save_states) - 1]

    def load_last_state(self):
        return self.initial_states[len(self.initial_states) - 1]

    def load_first_state(self):
        return self.initial_states[0]

    def load_random_state(self):
        return self.initial_states[random.randint(0, len(self.initial_states) - 1)]

    def load_pyboy_state(self, state):
        """pyboy_binding.py:59-69 load_pyboy_state: install a v9 savestate (bytes or file object)."""
        data = state.getvalue() if hasattr(state, "getvalue") else bytes(state)
        self.emu.load_env(0, data)

    def reset(self, seed=None, options=None):
        """environment.py:228-230: the current screen, the game untouched (seeding is not supported)."""
        return self.video(), {}

    def step(self, action):
        """environment.py:404-406: run the action (the same press / release schedule as
        Environment.step, pyboy_binding.py:71-91), then (render(), 0, False, False, {})."""
        a = torch.tensor([int(action)], dtype=torch.uint8, device=self.emu.device)
        self.emu.step(a)
        return self.render(), 0, False, False, {}

    def render(self):
        """environment.py:256-272 (+ get_fixed_window :233-254): mark the player's tile in this
        map's memory, then the screen at half resolution (3 channels) beside the (72, 80) window of
        that memory centred on the player, zero-padded past the 255 x 255 edge."""
        pos = self.emu.peek(0, 0xD35E, 5)               # ram_map.position: D35E map, D361 y, D362 x
        r, c, m = pos[3], pos[4], min(pos[0], 247)
        mm = self.screen_memory.get(m)
        if mm is None:
            mm = self.screen_memory[m] = torch.zeros((255, 255), dtype=torch.uint8, device=self.emu.device)
        if r <= 254 and c <= 254:
            mm[r, c] = 255
        win = torch.zeros((72, 80), dtype=torch.uint8, device=self.emu.device)
        y0, y1, x0, x1 = max(0, r - 36), min(255, r + 36), max(0, c - 40), min(255, c + 40)
        if y0 < y1 and x0 < x1:
            win[y0 - r + 36:y1 - r + 36, x0 - c + 40:x1 - c + 40] = mm[y0:y1, x0:x1]
        half = self.emu.screen[0, ::2, ::2]
        return torch.stack((half, half, half, win), dim=2).cpu().numpy()

    def close(self):
        self.emu.close()


class Environment(Base):
    """One env (a single emulator lane) with pokegym's reward stack (environment.py:436-1812).
    Functionally the reference env; for throughput use VecEnv, which steps thousands of envs per
    kernel launch."""

    def __init__(self, rom_path="pokemon_red.gb", state_path=None, headless=True, save_video=False, quiet=False,
                 verbose=False, device: int = 0, max_episode_steps: int = 20480, reward_scale: float = 4.0, **kwargs):
        self.max_episode_steps, self.reward_scale = max_episode_steps, reward_scale
        self._default_episode = (int(max_episode_steps), float(reward_scale))   # reset()'s defaults
        super().__init__(rom_path, state_path, headless, save_video, quiet, device=device, **kwargs)
        self.screen_memory = None   # the reward stack's observation keeps it on the device (K3)

    def _emulator(self, rom, state, device):
        from .emulator import BatchedEmulator
        return BatchedEmulator(rom, 1, state=state, device=device, render=True, reward=True,
                               max_episode_steps=self.max_episode_steps, reward_scale=self.reward_scale, heatmap=True)

    def reset(self, seed=None, options=None, max_episode_steps=None, reward_scale=None):
        """environment.py:1233-1334 (seeding is not supported, as in the reference).  As there, every
        reset sets max_episode_steps / reward_scale from its arguments (:1258-1259): an argument left
        out takes its default — the constructor's value, 20480 / 4.0 unless given (the reference's
        reset defaults) — so one reset(max_episode_steps=X) does not stick to later resets."""
        mes = self._default_episode[0] if max_episode_steps is None else int(max_episode_steps)
        rsc = self._default_episode[1] if reward_scale is None else float(reward_scale)
        if (mes, rsc) != (self.max_episode_steps, self.reward_scale):
            self.emu.set_episode_params(mes, rsc)
            self.max_episode_steps, self.reward_scale = mes, rsc
        obs = self.emu.reset()
        self.emu.raise_if_failed(0)
        if self.save_video:   # a new episode file: {s_path}/reset_{k} (environment.py:1244-1249)
            self._recorder.clear()
            self._video_file = self.s_path / f"reset_{self.reset_count}"
        self.reset_count += 1
        return obs[0].cpu().numpy(), {}

    def step(self, action, fast_video=True):
        """environment.py:1336-1812; info is {} except at done / every 10000th step (:1621), where it
        holds the numeric scalars of the reference's "stats" and "reward" dicts (pokegym_amd/info.py)."""
        a = torch.tensor([int(action)], dtype=torch.uint8, device=self.emu.device)
        obs, rew, term, trunc = self.emu.step(a)
        if self.save_video:
            self.add_video_frame()
        self.emu.raise_if_failed(0)
        done = bool(term[0].item())
        if self.save_video and done:    # environment.py:1616-1617: the episode's video is closed
            self.last_video = self._recorder.write(self._video_file)
            self._recorder.clear()
        info = self.emu.info_dicts([0]).get(0, {})
        if info:   # "pokemon_exploration_map": self.counts_map (float64 in the reference)
            info["pokemon_exploration_map"] = self.emu.heatmap[0].cpu().numpy().astype(np.float64)
            info["stats"]["pokemon_exploration_map"] = info["pokemon_exploration_map"]
        return obs[0].cpu().numpy(), float(rew[0].item()), done, done, info

    def render(self):
        """Base.render's observation as the reward stack's K3 built it for the last step / reset."""
        return self.emu.obs[0].cpu().numpy()


class VecEnv:
    """N envs on one GPU with PufferLib-style batch semantics (device tensors in and out).

    batch_size < num_envs splits the envs into num_envs / batch_size sub-batches (the reference
    trains 72 envs 24 at a time, README.md:116-118): recv() returns the next sub-batch whose step
    has finished, send(actions) steps the sub-batch the last recv() returned on its own HIP stream
    (pk_step_range) and returns immediately, so the policy works on one sub-batch while the GPU
    steps the others.  batch_size must divide num_envs; a sub-batch starts on a 64-env image group
    (pk_step_range), so a batch_size that is not a multiple of 64 (the reference's 24) is laid out
    in 64-aligned slots whose padding envs are never stepped.  step(actions) steps all envs at once.
    Sub-batches overlap on the GPU while the HIP runtime has a hardware queue per stream
    (GPU_MAX_HW_QUEUES, 4 by default: the default stream plus up to 3 sub-batches; beyond that
    streams share queues and their launches serialise)."""

    def __init__(self, num_envs: int, rom_path=None, state_path=None, rom: bytes | None = None, state: bytes | None = None,
                 device: int | None = None, max_episode_steps: int = 20480, reward_scale: float = 4.0,
                 reload_on_reset: bool = False, env_offset: int = 0, log_interval: int = 128, emulator=None,
                 heatmap: bool = False, reward: bool = True, power_on: bool = False, batch_size: int | None = None):
        """reward=False: the screen-obs env of configs[3] — obs is the (144, 160) u8 screen, rewards are
        0 and episodes end at max_episode_steps.  power_on=True starts (and resets) every env from
        the cartridge's power-on state instead of a savestate."""
        self.batch_size = batch_size or num_envs
        if num_envs % self.batch_size:
            raise ValueError("batch_size must divide num_envs")
        self.num_batches = num_envs // self.batch_size
        # slot of a sub-batch in the emulator: batch_size rounded up to a 64-env group
        self.slot = (self.batch_size if self.num_batches == 1 or self.batch_size % 64 == 0
                     else -(-self.batch_size // 64) * 64)
        n_phys = self.num_batches * self.slot
        if emulator is None:
            from .emulator import BatchedEmulator
            rom = rom if rom is not None else _read(rom_path or "pokemon_red.gb")
            if power_on:
                state = None
            else:
                state = state if state is not None else _read(state_path if state_path is not None else DEFAULT_STATE)
            emulator = BatchedEmulator(rom, n_phys, state=state, device=0 if device is None else device, render=True,
                                       reward=reward, max_episode_steps=max_episode_steps, reward_scale=reward_scale,
                                       reload_on_reset=reload_on_reset, heatmap=heatmap)
        if getattr(emulator, "n", n_phys) != n_phys:
            raise ValueError(f"the emulator must hold {n_phys} envs ({self.num_batches} sub-batch slots of {self.slot})")
        self.emu = emulator
        self.device = emulator.device
        self.num_envs = self.num_agents = num_envs
        # emulator index of every env (only differs from the env index when slots are padded)
        self._padded = n_phys != num_envs
        self._phys = (torch.cat([torch.arange(b * self.slot, b * self.slot + self.batch_size)
                                 for b in range(self.num_batches)]).to(self.device) if self._padded else None)
        self.single_observation_space = (spaces.observation_space() if getattr(emulator, "reward", True)
                                         else spaces.screen_space())
        self.single_action_space = spaces.action_space()
        self.env_ids = torch.arange(env_offset, env_offset + num_envs, device=self.device)
        self.masks = torch.ones(num_envs, dtype=torch.bool, device=self.device)
        self.stats = EpisodeStats(num_envs, self.device, self.num_batches)
        self.info_stats = (InfoStats(self.device, self.num_batches) if getattr(emulator, "info", None) is not None
                           else None)
        self.log_interval = log_interval
        self.t = 0
        self._pending = None
        # first PK_ERR_* code of every env since the last check: the device clears an env's error
        # word when the env auto-resets, so the codes are kept here (no host sync) and raised at
        # the next logging interval — an exception between two checks is not lost
        errs = getattr(emulator, "errors", None)
        self.sticky_errors = torch.zeros_like(errs) if errs is not None else None
        # sub-batch pipeline (batch_size < num_envs): one stream + completion event per sub-batch,
        # FIFO of finished ones
        self._streams = [torch.cuda.Stream(self.device) for _ in range(self.num_batches)] if self.num_batches > 1 else []
        self._events = [torch.cuda.Event() for _ in range(self.num_batches)] if self.num_batches > 1 else []
        self._ready: list[int] = []
        self._current: int | None = None
        self._batch_steps = 0
        self.logs_fired = 0        # logging intervals that fired (error check + all-reduce issued)
        # deferred interval read (sub-batch pipeline): the interval's rows and error codes are
        # snapshotted on each sub-batch stream where it fires, and read by the host num_batches
        # recv()s later, when the last of those streams' steps is the one being received
        self._log_wait = 0
        self._snap_events = [torch.cuda.Event() for _ in range(self.num_batches)] if self.num_batches > 1 else []
        self._snap_err = torch.zeros_like(self.sticky_errors) if self.sticky_errors is not None else None

    def _range(self, b: int) -> slice:
        return slice(b * self.batch_size, (b + 1) * self.batch_size)

    def _prange(self, b: int) -> slice:
        """Emulator envs of sub-batch b."""
        return slice(b * self.slot, b * self.slot + self.batch_size)

    def phys(self, env: int) -> int:
        """Emulator index of env."""
        return (env // self.batch_size) * self.slot + env % self.batch_size

    def _logical(self, obs: torch.Tensor) -> torch.Tensor:
        return obs.index_select(0, self._phys) if self._padded else obs

    def _join_streams(self):
        """The current stream waits for every sub-batch stream (steps still in flight)."""
        if self._streams:
            cur = torch.cuda.current_stream(self.device)
            for st in self._streams:
                cur.wait_stream(st)

    def reset(self, seed=None, max_episode_steps=None, reward_scale=None):
        """Reset every env; max_episode_steps / reward_scale (Environment.reset's arguments,
        environment.py:1233) apply to all envs from here on, None keeps the current values.  Unlike
        the single Environment (where each reset() restores 20480 / 4.0, as the reference does), they
        are the VecEnv's configuration: its device auto-resets keep them."""
        self._join_streams()
        if max_episode_steps is not None or reward_scale is not None:
            mes = max_episode_steps if max_episode_steps is not None else getattr(self.emu, "max_episode_steps", 20480)
            rsc = reward_scale if reward_scale is not None else getattr(self.emu, "reward_scale", 4.0)
            self.emu.set_episode_params(mes, rsc)
        obs = self._logical(self.emu.reset())
        self.t = 0
        self._log_wait = 0
        if self.sticky_errors is not None:
            self.sticky_errors.zero_()
        return obs, []

    def raise_if_failed(self, codes: torch.Tensor | None = None):
        """Raise the reference's exception for the first env that hit one since the last check
        (codes: the sticky error codes, or a snapshot of them)."""
        codes = self.sticky_errors if codes is None else codes
        if codes is None:
            return
        bad = torch.nonzero(codes).flatten()
        if bad.numel():
            from ._native import ERR_EXCEPTIONS
            p = int(bad[0])
            code = int(codes[p])
            e = (p // self.slot) * self.batch_size + p % self.slot
            codes.zero_()
            raise ERR_EXCEPTIONS.get(code, RuntimeError)(
                f"env {e}: reference reward stack raises here (PK_ERR {code}); {bad.numel()} env(s) failed")

    def _step_range(self, b: int, actions: torch.Tensor):
        """Step sub-batch b (envs _range(b)) on the current stream, then book-keep and auto-reset."""
        sl, psl = self._range(b), self._prange(b)
        if self.num_batches == 1:
            obs, rew, term, trunc = self.emu.step(actions)
        else:
            obs, rew, term, trunc = self.emu.step_range(psl.start, actions)
        self.stats.update(rew, term, batch=b, envs=sl)
        if self.info_stats is not None:
            self.info_stats.update(self.emu.info[:, psl], self.emu.info_flag[psl], batch=b)
        if self.sticky_errors is not None:
            se = self.sticky_errors[psl]
            torch.where(se != 0, se, self.emu.errors[psl], out=se)
        rewards = rew.clone()
        terminals = term.to(torch.bool)
        truncations = trunc.to(torch.bool)
        # auto-reset the finished envs (no host sync); their obs is the first obs of the next episode
        if self.num_batches == 1:
            self.emu.reset(term)
        else:
            self.emu.reset_range(psl.start, self.batch_size, self.emu.terminals)
        return obs, rewards, terminals, truncations

    def _log(self, deferred: bool = False):
        infos = []
        if not (self.log_interval and self._batch_steps % (self.log_interval * self.num_batches) == 0):
            return infos
        if deferred and self._streams:
            # the sub-batch pipeline: no host sync here (it would drain every stream's queue).  Each
            # stream, after its latest step, moves its statistics rows and error codes into the
            # snapshot and restarts them; recv() reads the snapshot once the step it waits for is
            # the last of these (_read_logs)
            for b, st in enumerate(self._streams):
                with torch.cuda.stream(st):
                    self.stats.snapshot(b)
                    if self.info_stats is not None:
                        self.info_stats.snapshot(b)
                    if self.sticky_errors is not None:
                        psl = self._prange(b)
                        self._snap_err[psl].copy_(self.sticky_errors[psl])
                        self.sticky_errors[psl].zero_()
                    self._snap_events[b].record(st)
            self.logs_fired += 1
            self._log_wait = self.num_batches
            return infos
        # the sticky error codes and the statistics rows are written by the sub-batch streams:
        # wait for every one of them before reading and clearing (the next send() orders its
        # stream after these reads again through st.wait_stream(current))
        self._join_streams()
        self.raise_if_failed()
        self.logs_fired += 1
        infos = [self.stats.allreduce()]
        if self.info_stats is not None:
            infos[0].update(self.info_stats.allreduce())
        return infos

    def _read_logs(self):
        """The deferred interval's record: wait (host) for the snapshot, raise its first error code,
        all-reduce its rows."""
        cur = torch.cuda.current_stream(self.device)
        for e in self._snap_events:
            cur.wait_event(e)
        self.raise_if_failed(self._snap_err)
        infos = [self.stats.allreduce(snapshot=True)]
        if self.info_stats is not None:
            infos[0].update(self.info_stats.allreduce(snapshot=True))
        return infos

    def step(self, actions):
        """Step every env (all sub-batches) with actions of shape (num_envs,)."""
        if isinstance(actions, np.ndarray):
            actions = torch.from_numpy(actions)
        a = actions.to(device=self.device, dtype=torch.uint8).contiguous()
        self._join_streams()
        # an interval that fired on a send() and has not been read by a recv() yet
        pending = []
        if self._log_wait:
            self._log_wait = 0
            pending = self._read_logs()
        if self.num_batches == 1:
            obs, rewards, terminals, truncations = self._step_range(0, a)
        else:
            outs = [self._step_range(b, a[self._range(b)]) for b in range(self.num_batches)]
            obs = self._logical(self.emu.obs if self.emu.reward else self.emu.screen)
            rewards = torch.cat([o[1] for o in outs])
            terminals = torch.cat([o[2] for o in outs])
            truncations = torch.cat([o[3] for o in outs])
        self.t += 1
        self._batch_steps += self.num_batches
        return obs, rewards, terminals, truncations, pending + self._log()

    def save_state(self, env: int) -> bytes:
        """PyBoy v9 savestate of one env (pk_snapshot; environment.py:208-213 per env)."""
        return self.emu.snapshot(self.phys(env))

    def load_state(self, env: int, state: bytes):
        """Install a v9 savestate into one env (pk_load_env; pyboy_binding.py:59-69)."""
        self.emu.load_env(self.phys(env), state)

    def video_recorder(self, envs, capacity: int = 1024):
        """A FrameRecorder (pokegym_amd/video.py) of the given envs' screens: call .capture() after
        each step, .write(path, k) at an episode's end (the reference's save_video per env)."""
        from .video import FrameRecorder
        return FrameRecorder(self.emu, [self.phys(int(e)) for e in envs], capacity)

    def exploration_map(self, group=None) -> torch.Tensor:
        """Sum of every env's counts_map over all ranks (int64 (444, 436), RCCL all-reduce) — the
        aggregate of the reference's per-env info["pokemon_exploration_map"]; needs heatmap=True."""
        hm = getattr(self.emu, "heatmap", None)
        if hm is None:
            raise RuntimeError("VecEnv(heatmap=True) keeps the per-env counts_map")
        out = hm.sum(dim=0, dtype=torch.int64)
        if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
            dist.all_reduce(out, op=dist.ReduceOp.SUM, group=group)
        return out

    # PufferLib async API: async_reset, then repeatedly recv() -> policy -> send(actions)
    def async_reset(self, seed=None):
        obs, infos = self.reset(seed)
        if self.num_batches == 1:   # one batch: send() steps synchronously on the current stream
            z = torch.zeros(self.num_envs, device=self.device)
            f = torch.zeros(self.num_envs, dtype=torch.bool, device=self.device)
            self._pending = (obs, z, f, f, infos)
            return
        cur = torch.cuda.current_stream(self.device)
        z = torch.zeros(self.num_envs, dtype=torch.float64, device=self.device)
        f = torch.zeros(self.num_envs, dtype=torch.bool, device=self.device)
        self._pending = [(z[self._range(b)], f[self._range(b)], f[self._range(b)]) for b in range(self.num_batches)]
        for b in range(self.num_batches):
            self._events[b].record(cur)
        self._ready = list(range(self.num_batches))
        self._current = None

    def recv(self):
        """The next finished sub-batch: (obs, rewards, terminals, truncations, infos, env_ids, masks),
        device tensors over its batch_size envs; the current stream waits for its step (no host sync).
        The num_batches-th recv() after a logging interval fired reads that interval's snapshot (a
        host wait for the streams' steps of the interval — the last of which is the one received
        here): it raises the first reference exception an env hit, else returns the all-reduced
        record in infos."""
        if self.num_batches == 1:
            obs, rew, term, trunc, infos = self._pending
            return obs, rew, term, trunc, infos, self.env_ids, self.masks
        if self._current is not None:
            raise RuntimeError("recv() called twice without send()")
        if not self._ready:
            raise RuntimeError("recv() before async_reset()")
        logged = []
        if self._log_wait:
            self._log_wait -= 1
            if self._log_wait == 0:
                logged = self._read_logs()
        b = self._ready.pop(0)
        torch.cuda.current_stream(self.device).wait_event(self._events[b])
        self._current = b
        sl = self._range(b)
        rew, term, trunc = self._pending[b]
        obs = self.emu.obs if self.emu.reward else self.emu.screen
        infos, self._pending_infos = getattr(self, "_pending_infos", []) + logged, []
        return obs[self._prange(b)], rew, term, trunc, infos, self.env_ids[sl], self.masks[sl]

    def current_envs(self) -> slice:
        """Local env range of the sub-batch the last recv() returned (host-side, no sync)."""
        return self._range(self._current) if self.num_batches > 1 else slice(0, self.num_envs)

    def send(self, actions):
        """Step the sub-batch the last recv() returned, with actions (batch_size,), on its own stream."""
        if self.num_batches == 1:
            self._pending = self.step(actions)
            return
        b = self._current
        if b is None:
            raise RuntimeError("send() without a preceding recv()")
        if isinstance(actions, np.ndarray):
            actions = torch.from_numpy(actions)
        cur = torch.cuda.current_stream(self.device)
        a = actions.to(device=self.device, dtype=torch.uint8).contiguous()
        st = self._streams[b]
        st.wait_stream(cur)                       # the policy's actions (and its reads of obs)
        with torch.cuda.stream(st):
            a.record_stream(st)
            _, rew, term, trunc = self._step_range(b, a)
            self._events[b].record(st)
        self._pending[b] = (rew, term, trunc)
        self._batch_steps += 1
        if self._batch_steps % self.num_batches == 0:
            self.t += 1
        logged = self._log(deferred=True)
        if logged:
            self._pending_infos = logged
        self._ready.append(b)
        self._current = None

    def close(self):
        if self._streams:
            torch.cuda.synchronize(self.device)
        self.emu.close()


def make_sharded_vecenv(num_envs_total: int, **kwargs) -> VecEnv:
    """This rank's shard (contiguous env ids) of a num_envs_total batch; one process per GPU."""
    rank, world, local = env_rank()
    start, end = shard_range(num_envs_total, world, rank)
    kwargs.setdefault("device", local)
    return VecEnv(end - start, env_offset=start, **kwargs)

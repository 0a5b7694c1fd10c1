"""VecInventoryEnv: E copies of the reference's InventoryEnvironment resident on one MI355X.

Thin host wrapper over the C ABI of libmarlsc.so (include/marlsc.h). torch provides device
memory and the current HIP stream; all environment arithmetic runs in the HIP kernels
(csrc/env_kernels.hip). There is no CPU fallback: without the built library this raises.

Semantics per env follow `InventoryEnvironment` (src/environment/envs/multi_env.py:192-366)
with RLlib's EnvRunner loop folded in: an env whose episode truncates is reset inside the same
`step()` (its terminal observation is returned in `final_obs`), exactly as the runner calls
`reset()` after a truncation. Per-env root seeds are `SeedManager.derive_env_seed(base_seed,
worker_index, env_index)` (seed_manager.py:165-186, used by the env factory at
src/algorithms/base.py:413-419), so env `g` has the same trajectory however envs are sharded.
"""
from __future__ import annotations

import ctypes as C
from typing import Any, Dict, Optional

import numpy as np
import torch

from . import abi
from .seeding import default_train_seed
from .spec import EnvSpec


def _p(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


class VecInventoryEnv:
    def __init__(self, env_config: Any, n_envs: int, *, env_meta: Optional[Dict[str, Any]] = None,
                 device: int = 0, base_seed: Optional[int] = None, worker_index: int = 0,
                 env_index_offset: int = 0, env_seeds=None, allow_nr_ne_nw: bool = True,
                 demand_trace: Any = None, spec: Optional[EnvSpec] = None,
                 episode_ahead: Optional[int] = None, ea_mem_fraction: float = 0.0):
        self.spec = spec if spec is not None else EnvSpec.from_config(
            env_config, env_meta, allow_nr_ne_nw=allow_nr_ne_nw, demand_trace=demand_trace)
        self.n_envs = int(n_envs)
        self.env_index_offset = int(env_index_offset)  # global id of env 0 (keys the rollout noise)
        self.device = torch.device("cuda", device)
        self.base_seed = default_train_seed() if base_seed is None else int(base_seed)
        L = abi.lib()
        desc = self.spec.to_desc()
        # episode-ahead Poisson demand (msc_env_desc.episode_ahead): None automatic, 0 off (short-lived
        # envs: evaluation, observation statistics), n > 0 at most n slots; its memory is budgeted
        # against the device's free memory (ea_mem_fraction, default 0.25)
        desc.episode_ahead = -1 if episode_ahead is None else int(episode_ahead)
        desc.ea_mem_fraction = float(ea_mem_fraction)
        seeds = None
        if env_seeds is not None:
            arr = np.ascontiguousarray(env_seeds, dtype=np.uint32)
            assert arr.shape == (self.n_envs,)
            seeds = arr.ctypes.data_as(C.POINTER(C.c_uint32))
        h = C.c_void_p()
        with torch.cuda.device(self.device):
            abi.check(L.msc_env_create(C.byref(desc), device, self.n_envs, self.base_seed & 0xFFFFFFFF,
                                       worker_index, env_index_offset, seeds, C.byref(h)))
        self._h = h
        n = C.c_int64()
        W, K, R, Lo, F, lm, eas = (C.c_int32() for _ in range(7))
        abi.check(L.msc_env_dims(h, C.byref(n), C.byref(W), C.byref(K), C.byref(R), C.byref(Lo), C.byref(F), C.byref(lm),
                                 C.byref(eas)))
        self.ea_slots = eas.value
        self.W, self.K, self.R, self.L, self.F = W.value, K.value, R.value, Lo.value, F.value
        assert self.L == self.spec.local_obs_dim
        E, dev = self.n_envs, self.device
        self.obs = torch.zeros((E, self.W, self.L), dtype=torch.float32, device=dev)
        self.final_obs = torch.zeros_like(self.obs)
        self.rewards = torch.zeros((E, self.W), dtype=torch.float32, device=dev)
        self.rewards_f64 = torch.zeros((E, self.W), dtype=torch.float64, device=dev)
        self.truncated = torch.zeros(E, dtype=torch.uint8, device=dev)
        self._info = None

    # ---- properties mirroring the reference object ------------------------------------------
    @property
    def n_agents(self) -> int:
        return self.W

    @property
    def local_obs_dim(self) -> int:
        return self.L

    @property
    def global_obs_dim(self) -> int:
        return self.L * self.W

    @property
    def agents(self):
        return [f"warehouse_{i}" for i in range(self.W)]

    # ---- API ---------------------------------------------------------------------------------
    def reset(self, mask: Optional[torch.Tensor] = None, root_seeds: Optional[torch.Tensor] = None,
              eval_restart: bool = False) -> torch.Tensor:
        """Reset envs (mask: [E] u8/bool on device, None = all). root_seeds ([E] int on device)
        follows reset(seed=...) of an env built without a seed (update_root_seed)."""
        m = None if mask is None else mask.to(device=self.device, dtype=torch.uint8).contiguous()
        s = None if root_seeds is None else root_seeds.to(device=self.device, dtype=torch.int64).to(torch.int32).contiguous()
        flags = abi.RESET_EVAL_RESTART if eval_restart else 0
        abi.check(abi.lib().msc_env_reset(self._h, _p(m), _p(s), flags, _p(self.obs), _stream()))
        self._t_sync = 0 if mask is None else -1  # common timestep of every env (-1: unknown)
        return self.obs

    def step(self, actions: torch.Tensor, *, want_final_obs: bool = True, want_f64: bool = False,
             info: Optional[Dict[str, torch.Tensor]] = None, obs_out: Optional[torch.Tensor] = None,
             rewards_out: Optional[torch.Tensor] = None, truncated_out: Optional[torch.Tensor] = None):
        """actions [E, W, K] float32 on the device. Returns (obs [E,W,L], rewards [E,W],
        truncated [E] bool-as-u8, final_obs [E,W,L] or None). Returned tensors are internal
        buffers, overwritten by the next call. obs_out / rewards_out (contiguous f32 [E,W,L] / [E,W]
        on the device, e.g. a rollout buffer's row): written instead of the internal buffers, which
        then keep their previous contents (`obs` is stale until the caller copies the latest back).
        truncated_out (contiguous uint8 [E] on the device): the truncation flags, likewise."""
        for name, t, shape in (("obs_out", obs_out, (self.n_envs, self.W, self.L)), ("rewards_out", rewards_out, (self.n_envs, self.W))):
            if t is not None and (t.dtype != torch.float32 or not t.is_contiguous() or t.device != self.device
                                  or tuple(t.shape) != shape):
                raise ValueError(f"{name} must be a contiguous float32 {shape} tensor on {self.device}")
        if truncated_out is not None and (truncated_out.dtype != torch.uint8 or not truncated_out.is_contiguous()
                                          or truncated_out.device != self.device or tuple(truncated_out.shape) != (self.n_envs,)):
            raise ValueError(f"truncated_out must be a contiguous uint8 ({self.n_envs},) tensor on {self.device}")
        if actions.dtype != torch.float32 or not actions.is_contiguous() or actions.device != self.device:
            actions = actions.to(device=self.device, dtype=torch.float32).contiguous()
        if actions.shape != (self.n_envs, self.W, self.K):
            raise ValueError(f"actions must have shape {(self.n_envs, self.W, self.K)}, got {tuple(actions.shape)}")
        si = None
        if info is not None:
            s = abi.MscStepInfo()
            for k, v in info.items():
                setattr(s, k, C.cast(C.c_void_p(v.data_ptr()), C.POINTER(C.c_double if v.dtype == torch.float64 else C.c_int32)))
            si = C.byref(s)
        obs = self.obs if obs_out is None else obs_out
        rew = self.rewards if rewards_out is None else rewards_out
        tr = self.truncated if truncated_out is None else truncated_out
        abi.check(abi.lib().msc_env_step(
            self._h, _p(actions), _p(obs), _p(rew), _p(self.rewards_f64) if want_f64 else None,
            _p(tr), _p(self.final_obs) if want_final_obs else None, si, _stream()))
        ts = getattr(self, "_t_sync", -1)
        self._t_sync = -1 if ts < 0 else (0 if ts + 1 >= self.spec.episode_length else ts + 1)
        return obs, rew, tr, (self.final_obs if want_final_obs else None)

    def may_truncate(self) -> bool:
        """Whether the next step() can end an episode (host-side lockstep tracking, no sync): False
        only while every env is known to sit at the same timestep before the last one."""
        ts = getattr(self, "_t_sync", -1)
        return ts < 0 or ts + 1 >= self.spec.episode_length

    def generate_demand(self) -> None:
        """Draw the next step's demand now (see msc_env_generate_demand); overlappable."""
        abi.check(abi.lib().msc_env_generate_demand(self._h, _stream()))

    def set_pipelining(self, enabled: bool) -> None:
        """Toggle the library's automatic next-step demand pipelining (results are identical)."""
        abi.check(abi.lib().msc_env_set_pipelining(self._h, int(bool(enabled))))

    def set_chain_priority(self, enabled: bool) -> None:
        """Run the step chain's kernels ahead of the pipelined demand kernel (msc_env_set_chain_priority):
        for callers whose own work between steps (a policy forward) makes the env step their critical
        path. Results are identical either way."""
        abi.check(abi.lib().msc_env_set_chain_priority(self._h, int(bool(enabled))))

    def set_timing(self, max_steps: int) -> None:
        """Bracket the demand / step launches of the next max_steps steps with HIP events on the
        streams they run on (msc_env_set_timing); 0 turns it off."""
        abi.check(abi.lib().msc_env_set_timing(self._h, int(max_steps)))

    def read_timing(self) -> Dict[str, float]:
        """Mean device ms of the timed demand / step launches (msc_env_read_timing)."""
        import ctypes as C
        d, s, nd, ns = C.c_double(), C.c_double(), C.c_int64(), C.c_int64()
        abi.check(abi.lib().msc_env_read_timing(self._h, C.byref(d), C.byref(s), C.byref(nd), C.byref(ns)))
        return {"demand_ms": d.value, "step_ms": s.value, "n_demand": nd.value, "n_step": ns.value}

    def set_episode_ahead(self, enabled: bool) -> None:
        """msc_env_set_episode_ahead: switch episode-ahead demand off (per-step pipelined demand from the
        current step on) or back on (from the next common episode start); results are identical."""
        with torch.cuda.device(self.device):
            abi.check(abi.lib().msc_env_set_episode_ahead(self._h, 1 if enabled else 0))

    def ea_memory(self) -> Dict[str, int]:
        """Episode-ahead memory (msc_env_ea_memory): the create-time budget and the bytes allocated."""
        b, a = C.c_int64(), C.c_int64()
        abi.check(abi.lib().msc_env_ea_memory(self._h, C.byref(b), C.byref(a)))
        return {"budget": b.value, "allocated": a.value, "slots": self.ea_slots}

    STEP_C_FORM = 1  # include/marlsc.h MSC_OPT_STEP_C_FORM
    ALLOC_PRIO_SPLIT = 2  # include/marlsc.h MSC_OPT_ALLOC_PRIO_SPLIT

    def set_option(self, key: int, value: int) -> None:
        """A kernel-form option of this handle (msc_env_set_option; results are identical)."""
        abi.check(abi.lib().msc_env_set_option(self._h, int(key), int(value)))

    def kernel_choice(self) -> Dict[str, int]:
        """The kernels this handle runs (msc_env_kernel_choice), chosen at create time by shape."""
        keys = ("alloc", "alloc_sort", "fuse_a", "fuse_c", "group_tables_lds", "group_width", "ea_slots",
                "demand_impl", "demand_uni")
        buf = (C.c_int32 * len(keys))()
        n = abi.lib().msc_env_kernel_choice(self._h, buf, len(keys))
        if n < 0:
            abi.check(n)
        return {k: int(buf[i]) for i, k in enumerate(keys[:n])}

    def read_timing_ea(self) -> Dict[str, float]:
        """Episode-ahead demand (msc_env_read_timing_ea): mean device ms of the timed episode
        generation launches, their count, slots per env (0: off) and whether the current episode
        reads a generated slot."""
        ms, n, slots, act, work = C.c_double(), C.c_int64(), C.c_int32(), C.c_int32(), C.c_double()
        abi.check(abi.lib().msc_env_read_timing_ea(self._h, C.byref(ms), C.byref(n), C.byref(slots), C.byref(act),
                                                   C.byref(work)))
        return {"ea_ms": ms.value, "n_ea": n.value, "slots": slots.value, "active": bool(act.value),
                "ea_env_steps_per_launch": work.value}

    def work_counters(self) -> Dict[str, float]:
        """Demand work issued since create (msc_env_work_counters): episode-ahead generation launches
        and their env-steps, per-step demand launches, step calls."""
        la, ew, dl, st = C.c_int64(), C.c_double(), C.c_int64(), C.c_int64()
        abi.check(abi.lib().msc_env_work_counters(self._h, C.byref(la), C.byref(ew), C.byref(dl), C.byref(st)))
        return {"ea_launches": la.value, "ea_env_steps": ew.value, "demand_launches": dl.value, "steps": st.value}

    def alloc_info(self) -> Dict[str, torch.Tensor]:
        """Device buffers for msc_step_info (the reference's collect_step_info dict)."""
        E, W, K, R = self.n_envs, self.W, self.K, self.R
        shapes = {"inventory_before": (W, K), "pending_total": (W, K), "order_quantities": (W, K),
                  "demand_per_region": (R, K), "fulfilled_per_warehouse": (W, K), "unfulfilled_demands": (R, K),
                  "shipment_counts": (W, R), "shipment_quantities": (W, R), "shipment_quantities_by_sku": (W, R, K),
                  "lost_order_counts": (R,), "n_orders": (), "lost_sales": (W, K), "costs": (4, W)}
        return {k: torch.zeros((E,) + sh, dtype=torch.float64 if k in ("lost_sales", "costs") else torch.int32,
                               device=self.device) for k, sh in shapes.items()}

    def obs_flat(self, obs: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Reference layout [E, W, L*(1+W)] = local_w || concat_j local_j (multi_env.py:566-573)."""
        obs = self.obs if obs is None else obs
        if out is None:
            out = torch.empty((self.n_envs, self.W, self.L * (1 + self.W)), dtype=torch.float32, device=self.device)
        abi.check(abi.lib().msc_env_obs_flat(self._h, _p(obs), _p(out), _stream()))
        return out

    def read_state(self) -> Dict[str, np.ndarray]:
        E = self.n_envs
        inv = np.zeros((E, self.W, self.K), np.int32)
        ts = np.zeros(E, np.int32)
        ep = np.zeros(E, np.int32)
        rng = np.zeros((E, 2, 6), np.uint64)
        abi.check(abi.lib().msc_env_read_state(self._h, inv.ctypes.data_as(C.c_void_p), ts.ctypes.data_as(C.c_void_p),
                                               ep.ctypes.data_as(C.c_void_p), rng.ctypes.data_as(C.c_void_p)))
        return {"inventory": inv, "timestep": ts, "episode_counter": ep, "rng": rng}

    def save_state(self) -> bytes:
        n = abi.lib().msc_env_state_bytes(self._h)
        buf = (C.c_char * n)()
        abi.check(abi.lib().msc_env_save_state(self._h, buf))
        return bytes(buf)

    def load_state(self, blob: bytes) -> None:
        self._t_sync = -1
        n = abi.lib().msc_env_state_bytes(self._h)
        if len(blob) != n:
            raise ValueError(f"state blob has {len(blob)} bytes, expected {n}")
        buf = (C.c_char * n).from_buffer_copy(blob)
        abi.check(abi.lib().msc_env_load_state(self._h, buf))

    def set_episode_counters(self, counters) -> None:
        """SeedManager._episode_counter of every env ([E] ints >= 0; the caller-side write of
        src/algorithms/base.py:81): the next reset of env i starts episode counters[i] of its root
        seed (msc_env_set_episode_counters)."""
        arr = np.ascontiguousarray(counters, dtype=np.int32)
        if arr.shape != (self.n_envs,):
            raise ValueError(f"counters must have shape ({self.n_envs},), got {arr.shape}")
        abi.check(abi.lib().msc_env_set_episode_counters(self._h, arr.ctypes.data_as(C.c_void_p)))

    def check(self) -> None:
        abi.check(abi.lib().msc_env_check(self._h))

    def close(self) -> None:
        if getattr(self, "_h", None):
            abi.lib().msc_env_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

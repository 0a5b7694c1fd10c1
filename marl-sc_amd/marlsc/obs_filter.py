"""RLlib's running observation filter, `obs_normalization: "meanstd"` (the reference's
src/algorithms/mappo.py:170-171 / ippo.py:173-175: the `MeanStdFilter(multi_agent=True)`
env-to-module connector; evaluation applies the trained filter with update=False,
base.py:131-140, :176-177), on the device (csrc/obs_filter.hip, msc_meanstd_filter).

Model (ray.rllib.utils.filter, ray 2.52.1 -- not installed here, restated in
oracle/meanstd_ref.py, parity unpinned against RLlib itself):
* one RunningStat per agent and feature: the columns of an env's observation row [W * L];
* every observation the policy sees is pushed (Welford), then normalised with the statistics
  that include it: clip((x - mean) / (std + 1e-6), -10, 10); envs in env order, then the final
  observations of the envs whose episode was truncated at that step;
* each env runner keeps its own filter (running statistics + a buffer of its pushes since the
  last synchronisation); after every sampling round the driver folds every runner's buffer into
  its statistics (RunningStat.update, runner order) and every runner continues from them.
Here a runner is a rollout lane (one env handle) of a rank; ranks exchange their lanes' buffers
with one all_gather (RCCL on MI355X, gloo on CPU) and fold them in (rank, lane) order, so every
rank holds the same statistics.

The kernel's stream order is the caller's current stream; the observation rows are contiguous f32
[E, W * L], normalised in place unless `out` is given.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Optional

import torch
import torch.distributed as dist

from . import abi

SMALL_NUMBER = 1e-6
CLIP = 10.0


def _vp(t: Optional[torch.Tensor]):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def merge_stats(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """RunningStat.update on packed f64 [1 + 2C] (n, M[C], S[C]) rows: a (+) b (Chan et al.), in
    the reference's operation order."""
    C_ = (a.numel() - 1) // 2
    n1, n2 = float(a[0]), float(b[0])
    n = n1 + n2
    if n == 0:
        return a.clone()
    m1, s1, m2, s2 = a[1:1 + C_], a[1 + C_:], b[1:1 + C_], b[1 + C_:]
    delta = m1 - m2
    delta2 = delta * delta
    m = (n1 * m1 + n2 * m2) / n
    s = s1 + s2 + (delta2 / n) * n1 * n2
    out = torch.empty_like(a)
    out[0] = n
    out[1:1 + C_] = m
    out[1 + C_:] = s
    return out


class MeanStdObsFilter:
    """Per-lane device filters + the driver's statistics. `n_cols` = W * L (agent x feature)."""

    def __init__(self, n_cols: int, device, n_lanes: int = 1, clip: float = CLIP, eps: float = SMALL_NUMBER):
        self.C, self.clip, self.eps = int(n_cols), float(clip), float(eps)
        self.device = torch.device(device)
        # lane state: {n, buffer n, 0, 0, M[C], S[C], buffer M[C], buffer S[C]} (msc_meanstd_filter)
        self.lanes = [torch.zeros(4 + 4 * self.C, dtype=torch.float64, device=self.device) for _ in range(int(n_lanes))]
        self.driver = torch.zeros(1 + 2 * self.C, dtype=torch.float64, device=self.device)
        # filter scratch per (lane, rows): lanes run on their own HIP streams, so two lanes with the
        # same env count must not share one segment buffer
        self._scratch: Dict[tuple, torch.Tensor] = {}
        self._eval_state: Optional[torch.Tensor] = None

    # -- device calls -------------------------------------------------------------------------
    def _scratch_for(self, lane: int, rows: int) -> torch.Tensor:
        s = self._scratch.get((lane, rows))
        if s is None:
            n = int(abi.lib().msc_meanstd_scratch_doubles(rows, self.C))
            if n < 0:
                raise ValueError("bad filter shape")
            s = self._scratch[(lane, rows)] = torch.empty(n, dtype=torch.float64, device=self.device)
        return s

    def _call(self, state, x, out, mask, update, lane: int = -1):
        rows = x.shape[0]
        if x.dtype != torch.float32 or not x.is_contiguous() or x.numel() != rows * self.C:
            raise ValueError(f"observations must be contiguous f32 [rows, {self.C}]")
        if out is None:
            out = x
        if mask is not None:
            mask = mask.to(torch.uint8).contiguous()
            if mask.numel() != rows:
                raise ValueError("mask must have one entry per row")
        scratch = self._scratch_for(lane, rows) if update else None
        abi.check(abi.lib().msc_meanstd_filter(_vp(x), _vp(out), rows, self.C, _vp(mask), 1 if update else 0,
                                               _vp(state), _vp(scratch), self.clip, self.eps,
                                               C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)))
        return out

    def apply(self, lane: int, obs: torch.Tensor, mask: Optional[torch.Tensor] = None,
              out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Push the rows of obs (those with mask != 0) into lane `lane`'s filter and normalise
        them (in place unless `out`)."""
        return self._call(self.lanes[lane], obs.reshape(obs.shape[0], -1), None if out is None else out.reshape(obs.shape[0], -1),
                          mask, True, lane).view_as(obs)

    def normalize(self, obs: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """filter(obs, update=False) with the driver's statistics (evaluation)."""
        if self._eval_state is None:
            self._eval_state = self._lane_state_from_driver()
        x = obs.reshape(obs.shape[0], -1)
        if out is None:
            out = torch.empty_like(x)
        return self._call(self._eval_state, x, out.reshape(obs.shape[0], -1), None, False).view_as(obs)

    # -- synchronisation (FilterManager.synchronize) --------------------------------------------
    def _lane_state_from_driver(self) -> torch.Tensor:
        st = torch.zeros(4 + 4 * self.C, dtype=torch.float64, device=self.device)
        st[0] = self.driver[0]
        st[4:4 + 2 * self.C] = self.driver[1:]
        return st

    def lane_buffers(self) -> torch.Tensor:
        """[n_lanes, 1 + 2C] packed buffers (n, M, S) of this rank's lanes."""
        C_ = self.C
        return torch.stack([torch.cat([st[1:2], st[4 + 2 * C_:]]) for st in self.lanes])

    def sync(self, group=None) -> None:
        """Fold every lane's buffer (every rank's, in rank then lane order) into the driver's
        statistics; every lane continues from them with an empty buffer."""
        bufs = self.lane_buffers()
        if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
            parts = [torch.empty_like(bufs) for _ in range(dist.get_world_size(group))]
            dist.all_gather(parts, bufs, group=group)
            bufs = torch.cat(parts)
        d = self.driver
        for b in bufs:
            d = merge_stats(d, b)
        self.driver = d
        for st in self.lanes:
            st.copy_(self._lane_state_from_driver())
        self._eval_state = None

    # -- state ------------------------------------------------------------------------------------
    @property
    def count(self) -> int:
        return int(self.driver[0])

    @property
    def mean(self) -> torch.Tensor:
        return self.driver[1:1 + self.C]

    @property
    def std(self) -> torch.Tensor:
        n = float(self.driver[0])
        var = self.driver[1 + self.C:] / (n - 1) if n > 1 else self.mean ** 2
        return var.sqrt()

    def state_dict(self) -> Dict[str, torch.Tensor]:
        return {"driver": self.driver.detach().cpu(), "lanes": torch.stack(self.lanes).detach().cpu()}

    def load_state_dict(self, sd: Dict[str, torch.Tensor]) -> None:
        d = sd["driver"].to(self.device, torch.float64)
        if d.numel() != 1 + 2 * self.C:
            raise ValueError("filter state of another observation size")
        self.driver = d.clone()
        lanes = sd.get("lanes")
        for i, st in enumerate(self.lanes):
            if lanes is not None and i < lanes.shape[0]:
                st.copy_(lanes[i].to(self.device))
            else:
                st.copy_(self._lane_state_from_driver())
        self._eval_state = None


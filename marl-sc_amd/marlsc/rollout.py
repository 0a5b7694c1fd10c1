"""On-device rollout for IPPO / MAPPO: the actor/critic forward of the reference's RLModule in
PyTorch-ROCm over the HIP env, and GAE + advantage normalisation in HIP.

Reference structure restated (RLlib itself is not importable here, so this row is parity
unpinned against the reference and checked against the numpy GAE in oracle/gae_ref.py):
* `MLP`: `MLPArchitecture.build` (src/algorithms/models/architectures/mlp.py:14-60) -- Linear +
  activation per hidden size, output Linear, optional output activation;
* `ActorCritic`: `BaseRLModule._forward_inference/_forward_train/compute_values`
  (src/algorithms/models/rlmodules/base.py:480-715) for MLP networks without shared layers --
  actor on the local slice (or the full flat obs when actor_obs_type == "global"), free `log_std`
  clamped at `logstd_floor` (`_append_log_std`), critic on local (IPPO) or full flat obs (MAPPO);
* GAE(gamma, lambda) with truncation bootstrap V(final_obs) and RLlib's per-batch standardisation
  `(A - mean) / max(1e-4, std)`, statistics all-reduced across ranks (marlsc/dist.py).

Memory plan (288 GB HBM): the rollout stores the LOCAL observations only ([T, E, W, L] f32, 3.6 GB
at C3); the MAPPO critic's flat input (local || global of the same env) is rebuilt on the device by
`msc_env_obs_flat` when needed instead of storing [T, E, W, L(1+W)] (32 GB at C3).
"""
from __future__ import annotations

import contextlib
import ctypes as C
import os
from dataclasses import dataclass
from typing import Any, Dict, Optional

import torch
import torch.nn as nn

from . import abi
from . import mlp as mlp3
from .dist import allreduce_adv_stats
from .mlp import mlp3_forward
from .vec_env import VecInventoryEnv

_ACT = {"relu": nn.ReLU, "tanh": nn.Tanh, "elu": nn.ELU, "gelu": nn.GELU, "sigmoid": nn.Sigmoid}


def _act(name: str) -> nn.Module:
    return _ACT.get(str(name).lower(), nn.ReLU)()


class MLP(nn.Sequential):
    def __init__(self, in_dim: int, out_dim: int, config: Dict[str, Any]):
        layers, d = [], in_dim
        for h in config.get("hidden_sizes", [128, 128]):
            layers += [nn.Linear(d, h), _act(config.get("activation", "relu"))]
            d = h
        layers.append(nn.Linear(d, out_dim))
        if config.get("output_activation"):
            layers.append(_act(config["output_activation"]))
        super().__init__(*layers)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return mlp_forward(self, x)


# Inference (no autograd): a whole Linear-ReLU-Linear-ReLU-Linear MLP with hidden sizes 64 / 128 /
# 256 (both actors, the IPPO critic) runs as one f32-MFMA kernel (marlsc/mlp.py, MSC_FUSED_MLP3=0
# turns it off); any other Linear -> ReLU pair runs as one GEMM with the ReLU in the GEMM epilogue
# (torch._addmm_activation -> hipBLASLt). MSC_FUSED_MLP=0 restores the plain layer sequence.
_FUSED = os.environ.get("MSC_FUSED_MLP", "1") != "0"


def _out_rows(out: Optional[torch.Tensor], rows: int, n_out: int) -> Optional[torch.Tensor]:
    """`out` as the fused kernel's [rows, n_out] output buffer, or None when it cannot be one."""
    if out is None or not out.is_contiguous() or out.dtype != torch.float32 or out.numel() != rows * n_out:
        return None
    return out.view(rows, n_out)


def mlp_forward(layers, x: torch.Tensor, start: int = 0, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """layers[start:] applied to x (an nn.Sequential of Linear / activation modules). `out`: a
    buffer the fused kernel may write the result into (the caller checks the returned pointer)."""
    mods = list(layers)[start:]
    if not (_FUSED and x.is_cuda and not torch.is_grad_enabled()):
        for m in mods:
            x = m(x)
        return x
    if mlp3.ENABLED and x.dtype == torch.float32 and mlp3.fusable(mods):
        n_out = mods[-1].out_features
        # the whole MLP as one f32-MFMA kernel (csrc/mlp.hip)
        return mlp3_forward(mods, x, _out_rows(out, x.numel() // x.shape[-1], n_out))
    i = 0
    while i < len(mods):
        m = mods[i]
        if isinstance(m, nn.Linear) and m.bias is not None and i + 1 < len(mods) and isinstance(mods[i + 1], nn.ReLU):
            lead = x.shape[:-1]
            x = torch._addmm_activation(m.bias, x.reshape(-1, x.shape[-1]), m.weight.t()).reshape(*lead, -1)
            i += 2
        else:
            x = m(x)
            i += 1
    return x


@dataclass
class RolloutConfig:
    gamma: float = 0.99
    lam: float = 0.95
    actor_obs_type: str = "local"
    critic_obs_type: str = "global"
    logstd_init: float = -1.0
    logstd_floor: float = -3.5
    actor: Optional[Dict[str, Any]] = None
    critic: Optional[Dict[str, Any]] = None

    @classmethod
    def from_algorithm_config(cls, cfg: Dict[str, Any]) -> "RolloutConfig":
        """From a config_files/algorithms/*.yaml dict (the reference's schema)."""
        a = cfg.get("algorithm", cfg)
        s = a.get("algorithm_specific", {})
        nets = s.get("networks", {}) or {}
        if nets.get("shared_layers"):
            raise ValueError("shared_layers (GRU) networks are outside this build's rollout path")
        for k in ("actor", "critic"):
            if nets.get(k, {}).get("type", "mlp") != "mlp":
                raise ValueError(f"{k}: only mlp networks are supported")
        return cls(gamma=float(s.get("gamma", 0.99)), lam=float(s.get("lam", 0.95)),
                   actor_obs_type=s.get("actor_obs_type", "local"),
                   critic_obs_type=s.get("critic_obs_type", "global" if a.get("name") == "mappo" else "local"),
                   logstd_init=float(s.get("logstd_init", -1.0)), logstd_floor=float(s.get("logstd_floor", -3.5)),
                   actor=(nets.get("actor") or {}).get("config"), critic=(nets.get("critic") or {}).get("config"))


class ActorCritic(nn.Module):
    def __init__(self, local_obs_dim: int, global_obs_dim: int, action_dim: int, rc: RolloutConfig):
        super().__init__()
        self.local_obs_dim, self.rc = local_obs_dim, rc
        full = local_obs_dim + global_obs_dim
        self.actor = MLP(full if rc.actor_obs_type == "global" else local_obs_dim, action_dim,
                         rc.actor or {"hidden_sizes": [256, 256]})
        self.critic = MLP(full if rc.critic_obs_type == "global" else local_obs_dim, 1,
                          rc.critic or {"hidden_sizes": [64, 64]})
        self.log_std = nn.Parameter(torch.full((action_dim,), float(rc.logstd_init)))

    def dist_inputs(self, local_obs: torch.Tensor, full_obs: Optional[torch.Tensor] = None):
        """(mean, log_std) -- ACTION_DIST_INPUTS split in two."""
        mean = self.actor_mean(local_obs, full_obs)
        log_std = torch.clamp(self.log_std, min=self.rc.logstd_floor).expand_as(mean)
        return mean, log_std

    def actor_mean(self, local_obs: torch.Tensor, full_obs: Optional[torch.Tensor] = None) -> torch.Tensor:
        return self.actor(full_obs if self.rc.actor_obs_type == "global" else local_obs)

    def log_std_table(self) -> torch.Tensor:
        """[1, K] unclamped log_std for msc_gaussian_sample (the kernel applies logstd_floor)."""
        return self.log_std.detach().float().reshape(1, -1).contiguous()

    def actor_sample(self, local_obs: torch.Tensor, full_obs: Optional[torch.Tensor], sample) -> bool:
        """The actor forward with the action sampling fused into its kernel (see fused_actor_sample)."""
        return fused_actor_sample(self.actor, full_obs if self.rc.actor_obs_type == "global" else local_obs, sample)

    def values(self, local_obs: torch.Tensor, full_obs: Optional[torch.Tensor] = None,
               out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """V [..., W]; `out` (contiguous, that shape) receives it when the fused critic runs."""
        if self.rc.critic_obs_type == "global" and full_obs is None:
            return split_global_mlp(self.critic, local_obs, out=out).squeeze(-1)
        x = full_obs if self.rc.critic_obs_type == "global" else local_obs
        return mlp_forward(self.critic, x, out=out).squeeze(-1)


def split_global_mlp(mlp: nn.Sequential, local_obs: torch.Tensor, agent: Optional[int] = None,
                     out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """An MLP over the per-agent flat input local_w || (local_0 .. local_{W-1}) evaluated from the
    local observations [..., W, L] without materialising it: the first Linear's columns split into
    a local block (per agent) and a global block (once per env, shared by its W agents) --
    mathematically the same layer, ~W x fewer first-layer flops and no [E, W, L(1+W)] buffer.
    agent=None: all W agents ([..., W, out]); agent=w: agent w only ([..., out]).
    out: a contiguous buffer of the fused kernel's output (rows x outputs), used when it runs."""
    first = mlp[0]
    W, L = local_obs.shape[-2], local_obs.shape[-1]
    glob = local_obs.reshape(*local_obs.shape[:-2], W * L)
    mods = list(mlp)
    if (agent is None and _FUSED and mlp3.ENABLED and local_obs.is_cuda and local_obs.dtype == torch.float32
            and not torch.is_grad_enabled() and mlp3.fusable(mods)):
        # the whole critic as one f32-MFMA kernel over the E*W rows, with the per-env global block
        # (one GEMM over E rows) added to the first layer of each of the env's W rows
        g = torch.nn.functional.linear(glob.reshape(-1, W * L), first.weight[:, L:])  # b1: in the kernel
        o = _out_rows(out, local_obs[..., 0].numel(), mods[-1].out_features)
        return mlp3_forward(mods, local_obs, o, w1=first.weight[:, :L], pre1=g, group=W)
    g = torch.nn.functional.linear(glob, first.weight[:, L:])
    if agent is None:
        h = torch.nn.functional.linear(local_obs, first.weight[:, :L], first.bias) + g.unsqueeze(-2)
    else:
        h = torch.nn.functional.linear(local_obs[..., agent, :], first.weight[:, :L], first.bias) + g
    return mlp_forward(mlp, h, 1)


def fused_actor_sample(actor: nn.Sequential, x: torch.Tensor, sample) -> bool:
    """Run `actor` over x with msc_gaussian_sample fused into the MLP kernel's epilogue (sample =
    (log_std [P, K], logstd_floor, eps, actions, logp, clipped)); False (nothing launched) when the
    fused kernel does not apply, e.g. more than 8 outputs or a non-ReLU MLP."""
    mods = list(actor)
    if not (_FUSED and mlp3.ENABLED and x.is_cuda and x.dtype == torch.float32 and not torch.is_grad_enabled()
            and mlp3.sample_fusable(mods)):
        return False
    mlp3_forward(mods, x, None, sample=sample)
    return True


def _vp(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


def gaussian_sample(mean: torch.Tensor, log_std: torch.Tensor, logstd_floor: float, eps: torch.Tensor,
                    actions: torch.Tensor, logp: torch.Tensor) -> torch.Tensor:
    """msc_gaussian_sample: actions = mean + exp(max(log_std, floor)) * eps, logp = the diagonal
    Gaussian log-density summed over the last dim, into `actions` / `logp`; returns the [-1, 1]
    clipped actions the env receives. mean / eps / actions [..., K], logp [...] (f32 CUDA);
    log_std [K] (shared) or [P, K] repeating every P rows (e.g. [W, K]: one row per agent)."""
    K = mean.shape[-1]
    for t in (mean, eps, actions, logp):
        assert t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()
    assert actions.shape == mean.shape == eps.shape and logp.shape == mean.shape[:-1]
    ls = log_std.detach().float().reshape(-1, K).contiguous()
    assert (mean.numel() // K) % ls.shape[0] == 0
    clipped = torch.empty_like(mean)
    abi.check(abi.lib().msc_gaussian_sample(_vp(mean), _vp(ls), ls.shape[0], C.c_float(logstd_floor), _vp(eps),
                                            mean.numel() // K, K, _vp(actions), _vp(logp), _vp(clipped),
                                            C.c_void_p(torch.cuda.current_stream().cuda_stream)))
    return clipped


def gae(rewards, values, next_values, terminated, truncated, gamma, lam, adv=None, targets=None, stats=None,
        groups: int = 1):
    """msc_gae_grouped over [T, N] (values [T+1, N]); returns (adv, targets, stats [groups, 3] f64 of
    [sum, sum_sq, n] per group; sequence n belongs to group n % groups)."""
    T, N = rewards.shape
    for name, t, shape in (("rewards", rewards, (T, N)), ("values", values, (T + 1, N)),
                           ("next_values", next_values, (T, N))):
        if t.dtype != torch.float32 or not t.is_contiguous() or tuple(t.shape) != shape:
            raise ValueError(f"{name}: expected contiguous float32 {shape}")
    for name, t in (("terminated", terminated), ("truncated", truncated)):
        if t.dtype != torch.uint8 or not t.is_contiguous() or tuple(t.shape) != (T, N):
            raise ValueError(f"{name}: expected contiguous uint8 {(T, N)}")
    adv = torch.empty_like(rewards) if adv is None else adv
    targets = torch.empty_like(rewards) if targets is None else targets
    if stats is None:
        stats = torch.zeros((groups, 3), dtype=torch.float64, device=rewards.device)
    elif tuple(stats.shape) != (groups, 3) or stats.dtype != torch.float64:
        raise ValueError(f"stats: expected float64 {(groups, 3)}")
    else:
        stats.zero_()
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    abi.check(abi.lib().msc_gae_grouped(_vp(rewards), _vp(values), _vp(next_values), _vp(terminated), _vp(truncated),
                                        N, T, C.c_float(gamma), C.c_float(lam), _vp(adv), _vp(targets), int(groups),
                                        _vp(stats), st))
    return adv, targets, stats


def normalize_advantages(adv: torch.Tensor, stats: torch.Tensor) -> torch.Tensor:
    """In place (A - mean_g) / max(1e-4, std_g) with the (already all-reduced) statistics of the
    [groups, 3] table; element i of the flattened [T, N] advantages belongs to group i % groups."""
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    g = stats.numel() // 3
    abi.check(abi.lib().msc_adv_normalize_grouped(_vp(adv), adv.numel(), g, _vp(stats), st))
    return adv


NOISE_CHUNK = 16  # rollout steps whose Gaussian noise is drawn in one launch
_TORCH_NOISE = os.environ.get("MSC_NOISE", "keyed") == "torch"


def keyed_normal(shape, row0: int, seed: int, step0: int) -> torch.Tensor:
    """msc_normal_keyed: f32 standard normals of shape [n_steps, n_envs, ...] on the current stream;
    element (s, e, j) depends only on (seed, global env row0 + e, step step0 + s, flat index j)."""
    n_steps, n_rows = int(shape[0]), int(shape[1])
    row_len = 1
    for d in shape[2:]:
        row_len *= int(d)
    out = torch.empty(tuple(shape), dtype=torch.float32, device=torch.device("cuda", torch.cuda.current_device()))
    abi.check(abi.lib().msc_normal_keyed(_vp(out), n_steps, n_rows, row_len, int(row0), int(seed) & 0xFFFFFFFFFFFFFFFF,
                                         int(step0), C.c_void_p(torch.cuda.current_stream().cuda_stream)))
    return out


class _Lane:
    """One env handle of a collector: its slice [e0, e1) of the buffers' env axis and the HIP stream
    its step chain (policy forward -> sampling -> env step) is issued on (None: the caller's)."""

    def __init__(self, env: VecInventoryEnv, e0: int, stream: Optional[torch.cuda.Stream], flat: Optional[torch.Tensor]):
        self.env, self.e0, self.e1, self.stream, self.flat = env, e0, e0 + env.n_envs, stream, flat
        self.noise: Optional[torch.Tensor] = None
        self.critic_stream: Optional[torch.cuda.Stream] = None  # V(obs_t) off the step chain
        self.obs_filtered = False  # the env's current observation already went through the obs filter

    def ctx(self):
        return torch.cuda.stream(self.stream) if self.stream is not None else contextlib.nullcontext()


class RolloutCollector:
    """T steps of E envs x W agents (N = E*W sequences). Advantages are standardised per module as
    RLlib's GAE connector does: over every agent for one shared policy (adv_groups = 1), per agent
    for one policy per agent (adv_groups = W).

    `env` may be a list of env handles (lanes) covering consecutive env-id ranges, e.g. the two
    halves of a rank's envs: each lane's step chain runs on its own HIP stream, so one lane's env
    kernels (VALU-bound) overlap the other lane's policy GEMMs (MFMA-bound). The buffers' env axis
    is the concatenation of the lanes; each env's trajectory is the same as with one handle (envs
    are independent and seeded by global id), and so is its Gaussian noise (keyed by global env id)."""

    def __init__(self, env, module: ActorCritic, T: int, *, seed: int = 0, adv_groups: int = 1,
                 obs_filter: str = "off"):
        envs = list(env) if isinstance(env, (list, tuple)) else [env]
        e0 = envs[0]
        for x in envs[1:]:
            if x.spec is not e0.spec and (x.W, x.K, x.L) != (e0.W, e0.K, e0.L):
                raise ValueError("rollout lanes must share one env spec")
        self.env, self.envs, self.module, self.T = e0, envs, module, int(T)
        E = sum(x.n_envs for x in envs)
        W, K, L = e0.W, e0.K, e0.local_obs_dim
        dev = e0.device
        self.E, self.N = E, E * W
        # T + 1 observation rows: the env writes step t's result straight into row t + 1 (no copy
        # per step); `obs` is the first T rows, the last one is copied back into the env at the end
        self._obs_all = torch.empty((T + 1, E, W, L), device=dev)
        self.obs = self._obs_all[:T]
        self.actions = torch.empty((T, E, W, K), device=dev)
        self.logp = torch.empty((T, E, W), device=dev)
        self.rewards = torch.empty((T, E, W), device=dev)
        self.values = torch.empty((T + 1, E, W), device=dev)
        self.next_values = torch.zeros((T, E, W), device=dev)
        self.terminated = torch.zeros((T, E, W), dtype=torch.uint8, device=dev)
        self.truncated = torch.zeros((T, E, W), dtype=torch.uint8, device=dev)
        self._trunc_env = torch.zeros((T, E), dtype=torch.uint8, device=dev)  # the env writes these rows
        self.adv = torch.empty((T, E, W), device=dev)
        self.targets = torch.empty((T, E, W), device=dev)
        if adv_groups not in (1, W):
            raise ValueError(f"adv_groups must be 1 (shared policy) or W={W} (one policy per agent)")
        self.adv_groups = int(adv_groups)
        self.stats = torch.zeros((self.adv_groups, 3), dtype=torch.float64, device=dev)
        self._need_flat = module.rc.actor_obs_type == "global"  # the critic splits its first layer
        # The values of obs_t are read only by the GAE after the rollout: with few envs the critic runs
        # on a side stream per lane, after the step that wrote obs_t, beside the actor -> sampling ->
        # env chain (C2 IPPO rollout 136.9 -> 139.5 M agent-steps/s); on a full chip it only takes
        # issue slots from the env kernels (C3 MAPPO 224.7 -> 214.9 M), and not when it reads the
        # lane's flat buffer, which the next step rewrites. MSC_ROLLOUT_CRITIC_SIDE=0|1 forces it.
        cs = os.environ.get("MSC_ROLLOUT_CRITIC_SIDE")
        self._critic_side = (self.N <= 65536 if cs is None else cs != "0") and not self._need_flat
        # Gaussian action noise keyed by (seed, global env id, rollout step): msc_normal_keyed, so an
        # env's noise does not depend on which rank or lane steps it
        self._noise_seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.noise_step = 0  # rollout steps drawn so far (checkpointed)
        import inspect
        self._values_out = "out" in inspect.signature(module.values).parameters
        self._ls: Optional[torch.Tensor] = None
        # obs_normalization "meanstd": RLlib's running filter, one per lane (env runner), synchronised
        # after every collect (marlsc/obs_filter.py)
        self.obs_filter = None
        if obs_filter == "meanstd":
            from .obs_filter import MeanStdObsFilter
            self.obs_filter = MeanStdObsFilter(W * L, dev, n_lanes=len(envs))
        elif obs_filter not in ("off", None):
            raise ValueError(f"obs_filter must be 'off' or 'meanstd', not {obs_filter!r}")
        # Episode-ahead demand beside the policy kernels: at 4,096 envs it lifts the rollout (the
        # per-step demand chain would bound the step), at 32,768 the background generation takes the
        # MLP kernels' CU slots (C3 MAPPO rollout 1.15 -> 1.32 ms per step, profiles/r04/ab_ea_c3.txt),
        # so lanes of >= 16,384 envs step with per-step pipelined demand. MSC_ROLLOUT_EA=0|1 forces it.
        rea = os.environ.get("MSC_ROLLOUT_EA")
        for x in envs:
            if getattr(x, "ea_slots", 0) and hasattr(x, "set_episode_ahead"):
                x.set_episode_ahead(x.n_envs < 16384 if rea is None else rea != "0")
        self._lanes, off = [], 0
        for x in envs:
            st = torch.cuda.Stream(device=dev) if len(envs) > 1 else None
            flat = torch.empty((x.n_envs, W, L * (1 + W)), device=dev) if self._need_flat else None
            self._lanes.append(_Lane(x, off, st, flat))
            off += x.n_envs

    def _full(self, ln: _Lane, obs):
        return ln.env.obs_flat(obs=obs, out=ln.flat) if self._need_flat else None

    def _values_into(self, t: int, sl: slice, obs, full) -> None:
        """V(obs_t) into values[t, sl]: written by the fused critic kernel directly when the module
        takes an output buffer, copied otherwise."""
        dst = self.values[t, sl]
        v = self.module.values(obs, full, out=dst) if self._values_out else self.module.values(obs, full)
        if v.data_ptr() != dst.data_ptr():
            dst.copy_(v)

    def _critic_on_side(self, ln: _Lane, t: int, sl: slice, obs, full) -> None:
        if ln.critic_stream is None:
            ln.critic_stream = torch.cuda.Stream(device=obs.device)
        ev = torch.cuda.Event()
        ev.record()
        ln.critic_stream.wait_event(ev)
        with torch.cuda.stream(ln.critic_stream):
            self._values_into(t, sl, obs, full)

    def _noise_chunk(self, ln: _Lane) -> int:
        per_step = max(1, self.actions[0, ln.e0:ln.e1].numel() * 4)
        if os.environ.get("MSC_NOISE_CHUNK"):
            return max(1, int(os.environ["MSC_NOISE_CHUNK"]))
        return max(NOISE_CHUNK, min(self.T, (1 << 30) // per_step))

    def _step(self, ln: _Lane, t: int) -> None:
        env, m, sl = ln.env, self.module, slice(ln.e0, ln.e1)
        obs = self._obs_all[t, sl]
        full = self._full(ln, obs)
        if self._critic_side:
            self._critic_on_side(ln, t, sl, obs, full)
        # standard-normal noise for `chunk` steps of the lane at once (one launch instead of one per
        # step), keyed by global env id. The whole rollout's noise when it fits 1 GiB: a noise launch
        # between step_c and the actor lets the next demand kernel reach the CUs before the actor,
        # whose one 384-VGPR wave per SIMD then no longer fits beside the demand waves (the actor of
        # that step 378 -> 906 us, profiles/r06/trace_roll_c3_r06il.txt)
        chunk = self._noise_chunk(ln)
        if t % chunk == 0:
            n = min(chunk, self.T - t)
            if _TORCH_NOISE:  # A/B only: torch's generator (not shard-invariant)
                if not hasattr(self, "_gen"):
                    self._gen = torch.Generator(device=obs.device).manual_seed(self._noise_seed & 0x7FFFFFFF)
                ln.noise = torch.randn((n,) + tuple(self.actions[t, sl].shape), device=obs.device, generator=self._gen)
            else:
                ln.noise = keyed_normal((n,) + tuple(self.actions[t, sl].shape), ln.env.env_index_offset,
                                        self._noise_seed, self.noise_step + t)
        eps = ln.noise[t % chunk]
        a = None
        if self._ls is not None and hasattr(m, "actor_sample"):
            # actor forward + sampling + log-density + the env's clip in one kernel launch
            clipped = torch.empty_like(self.actions[t, sl])
            if m.actor_sample(obs, full, (self._ls, m.rc.logstd_floor, eps, self.actions[t, sl], self.logp[t, sl],
                                          clipped)):
                a = clipped
        if a is None:
            if self._ls is not None:  # the module's raw log_std rows, taken once per collect
                mean, ls = m.actor_mean(obs, full), self._ls
            else:
                mean, log_std = m.dist_inputs(obs, full)
                ls = log_std[0]
            # sample, log-density and the env's clip in one HIP kernel (msc_gaussian_sample)
            # (log_std rows: one shared row or one per agent, repeating every P rows)
            a = gaussian_sample(mean.contiguous(), ls, m.rc.logstd_floor, eps, self.actions[t, sl], self.logp[t, sl])
        if not self._critic_side:
            self._values_into(t, sl, obs, full)
        may_end = env.may_truncate()
        _, _, trunc, final_obs = env.step(a, obs_out=self._obs_all[t + 1, sl], rewards_out=self.rewards[t, sl],
                                          truncated_out=self._trunc_env[t, sl])
        li = self._lanes.index(ln) if self.obs_filter is not None else 0
        if self.obs_filter is not None:  # the new observations first, then the truncated envs' final ones
            self.obs_filter.apply(li, self._obs_all[t + 1, sl])
            if may_end:
                self.obs_filter.apply(li, final_obs, mask=trunc)
        # truncation bootstrap: V(final_obs) for the envs whose episode ended at this step
        # (skipped while the envs are known to be mid-episode in lockstep; next_values is zeroed
        # once per rollout)
        if may_end:
            full_f = self._full(ln, final_obs)
            self.next_values[t, sl] = torch.where(trunc.bool().unsqueeze(-1), m.values(final_obs, full_f),
                                                  torch.zeros((), device=final_obs.device))

    @torch.no_grad()
    def collect(self, normalize: bool = True) -> Dict[str, torch.Tensor]:
        m, T = self.module, self.T
        main = torch.cuda.current_stream()
        self.next_values.zero_()
        # log_std does not change during a collect: its rows go to the sampling kernel as they are
        # (the kernel clamps at logstd_floor), no clamp / broadcast launches per step
        self._ls = m.log_std_table() if hasattr(m, "log_std_table") and hasattr(m, "actor_mean") else None
        for ln in self._lanes:
            if not getattr(ln, "form_set", False) and hasattr(ln.env, "set_option"):
                # the observation kernel's spill-free form: with policy kernels between the steps it
                # is faster than the form the env stepping uses beside the demand kernel (C3 MAPPO
                # rollout 1.18 -> 1.14 ms per step, profiles/r06/ab_step_c_wpe.txt); results identical
                if os.environ.get("MSC_ROLLOUT_STEP_C_FORM", "4") == "4":
                    ln.env.set_option(ln.env.STEP_C_FORM, 4)
                # the allocation at full priority for its whole run: here the step chain, not the
                # demand kernel beside it, bounds a step (the env stepping's 12/16 split costs the C3
                # MAPPO rollout 1.14 -> 1.18 ms per step, profiles/r06/ab_alloc_prio.txt)
                ln.env.set_option(ln.env.ALLOC_PRIO_SPLIT, int(os.environ.get("MSC_ROLLOUT_AL_PRIO_SPLIT", "16")))
                ln.form_set = True
            if os.environ.get("MSC_ROLLOUT_CHAIN_PRIO", "0") != "0" and not getattr(ln, "prio_set", False):
                # A/B: step chain ahead of the next step's demand kernel (neutral: 1.234 vs 1.228 ms
                # per step; the step kernels wait for CU space, not for issue slots)
                ln.env.set_chain_priority(True)
                ln.prio_set = True
            if ln.stream is not None:
                ln.stream.wait_stream(main)
            with ln.ctx():
                self._obs_all[0, ln.e0:ln.e1].copy_(ln.env.obs)
                if self.obs_filter is not None and not ln.obs_filtered:  # the reset observation
                    self.obs_filter.apply(self._lanes.index(ln), self._obs_all[0, ln.e0:ln.e1])
                ln.obs_filtered = True
        # lanes interleaved per step on the host; each lane's chain is ordered on its own stream
        for t in range(T):
            for ln in self._lanes:
                with ln.ctx():
                    self._step(ln, t)
        for ln in self._lanes:
            with ln.ctx():
                last = self._obs_all[T, ln.e0:ln.e1]
                self.values[T, ln.e0:ln.e1] = m.values(last, self._full(ln, last))
                ln.env.obs.copy_(last)  # the env's own buffer holds the current observation again
            if ln.stream is not None:
                main.wait_stream(ln.stream)
            if ln.critic_stream is not None:
                main.wait_stream(ln.critic_stream)
        self.noise_step += T
        # the per-env truncation flags of every step to every agent's sequence (one launch)
        self.truncated.copy_(self._trunc_env.unsqueeze(-1).expand_as(self.truncated))
        if self.obs_filter is not None:
            self.obs_filter.sync()
        N = self.N
        gae(self.rewards.view(T, N), self.values.view(T + 1, N), self.next_values.view(T, N),
            self.terminated.view(T, N), self.truncated.view(T, N), m.rc.gamma, m.rc.lam,
            self.adv.view(T, N), self.targets.view(T, N), self.stats, groups=self.adv_groups)
        if normalize:
            allreduce_adv_stats(self.stats)
            normalize_advantages(self.adv, self.stats)
        return {"obs": self.obs, "actions": self.actions, "logp": self.logp, "rewards": self.rewards,
                "values": self.values, "advantages": self.adv, "value_targets": self.targets}

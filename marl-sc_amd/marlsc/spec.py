"""EnvSpec: the reference's EnvironmentConfig + env_meta flattened into plain numpy arrays, and
its packing into the C-ABI descriptor `msc_env_desc` (include/marlsc.h).

Accepts a `marlsc.config.ConfigNode`, a plain dict in the YAML `environment:` layout, or the
reference's own pydantic `EnvironmentConfig` (duck-typed), so a caller of the reference can hand
its config object over unchanged. Follows `create_environment_context`
(src/environment/context.py:146-208) and `InventoryEnvironment.__init__`
(src/environment/envs/multi_env.py:58-190).
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field
from typing import Any, Dict, Optional

import numpy as np

from . import abi
from .config import ConfigNode, FEATURE_DEFAULTS, validate_environment_config


def _g(o: Any, k: str):
    if isinstance(o, ConfigNode):
        return o[k]
    if isinstance(o, dict):
        return o[k]
    return getattr(o, k)


def _g_opt(o: Any, k: str, default=None):
    try:
        v = _g(o, k)
    except (KeyError, AttributeError):
        return default
    return default if v is None else v


def _features_dict(f) -> Dict[str, bool]:
    if f is None:
        return dict(FEATURE_DEFAULTS)
    return {k: bool(_g_opt(f, k, FEATURE_DEFAULTS[k])) for k in FEATURE_DEFAULTS}


@dataclass
class EnvSpec:
    W: int
    K: int
    R: int
    episode_length: int
    action_type: str
    action_param: np.ndarray
    init_type: str
    init_min: int
    init_max: int
    init_values: np.ndarray
    holding: np.ndarray
    holding_per_sku: bool
    penalty: np.ndarray
    penalty_per_sku: bool
    sku_weights: np.ndarray
    distances: np.ndarray
    outbound_fixed: np.ndarray
    outbound_variable: np.ndarray
    inbound_fixed: np.ndarray
    inbound_variable: np.ndarray
    demand_type: str
    lambda_orders: np.ndarray
    probability_skus: np.ndarray
    lambda_quantity: np.ndarray
    max_splits: int
    lead_type: str
    expected_lead_times: np.ndarray
    max_dev_per_sku: bool
    max_deviation: np.ndarray
    lost_type: str
    lost_alpha: float
    scope: str
    scale_factor: float
    features: Dict[str, bool]
    include_warehouse_id: bool
    obs_normalization: str
    obs_mean: Optional[np.ndarray]
    obs_std: Optional[np.ndarray]
    num_eval_episodes: int
    trace: Optional[Dict[str, np.ndarray]] = None
    _keep: list = field(default_factory=list, repr=False)

    # ---- derived -------------------------------------------------------------------------
    @property
    def max_expected_lead_time(self) -> int:
        return int(self.expected_lead_times.max())

    @property
    def feature_flags(self) -> int:
        return sum(bit for k, bit in abi.FEATURE_BITS if self.features[k])

    @property
    def n_features(self) -> int:
        """_compute_local_obs_dim without the one-hot (multi_env.py:444-502)."""
        f, K = self.features, self.K
        n = 0
        n += (K + f["inventory_aggregate"]) if f["inventory"] else 0
        n += (self.max_expected_lead_time * K + f["pipeline_aggregate"]) if f["pipeline"] else 0
        n += (K + f["incoming_demand_home_aggregate"]) if f["incoming_demand_home"] else 0
        n += K if f["units_shipped_home"] else 0
        n += (K + f["units_shipped_away_aggregate"]) if f["units_shipped_away"] else 0
        n += K if f["stockout"] else 0
        n += (K + f["rolling_demand_mean_aggregate"]) if f["rolling_demand_mean"] else 0
        n += (K + f["demand_forecast_aggregate"]) if f["demand_forecast"] else 0
        n += K * (f["days_of_supply"] + f["net_inventory_position"] + f["demand_variability"])
        n += abi.HISTORY * K if f["demand_history"] else 0
        return int(n)

    @property
    def local_obs_dim(self) -> int:
        return self.n_features + (self.W if self.include_warehouse_id else 0)

    @property
    def home_regions(self) -> np.ndarray:
        return np.argmin(self.distances, axis=1)

    @property
    def closest_warehouses(self) -> np.ndarray:
        return np.argmin(self.distances, axis=0)

    def expected_orders_per_step(self) -> float:
        if self.demand_type == "poisson":
            return float(self.lambda_orders.sum())
        off = self.trace["offsets"]
        return float(np.max(np.diff(off))) if len(off) > 1 else 0.0

    def order_capacity(self) -> int:
        """Per-env per-step order buffer: mean + 12 sigma + slack for Poisson, trace max otherwise."""
        if self.demand_type == "poisson":
            lam = float(self.lambda_orders.sum())
            return int(math.ceil(lam + 12.0 * math.sqrt(lam + 1.0) + 64))
        return int(max(1, np.max(np.diff(self.trace["offsets"]))))

    # ---- construction ----------------------------------------------------------------------
    @classmethod
    def from_config(cls, cfg: Any, env_meta: Optional[Dict[str, Any]] = None, *,
                    allow_nr_ne_nw: bool = True, demand_trace: Any = None) -> "EnvSpec":
        if isinstance(cfg, dict):
            cfg = validate_environment_config(cfg, allow_nr_ne_nw=allow_nr_ne_nw)
        meta = dict(env_meta or {})
        W, K, R = int(_g(cfg, "n_warehouses")), int(_g(cfg, "n_skus")), int(_g(cfg, "n_regions"))
        T = int(_g(cfg, "episode_length"))
        act = _g(cfg, "action_space")
        atype = _g(act, "type")
        akey = {"direct": "max_order_quantities", "demand_centered": "max_quantity_adjustment",
                "base_stock": "max_stock_level"}[atype]
        aparam = np.asarray(_g(_g(act, "params"), akey), dtype=np.float64)
        ii = _g(cfg, "initial_inventory")
        itype = _g(ii, "type")
        iparams = _g_opt(ii, "params", {}) or {}
        imin = imax = 0
        ivals = np.zeros((W, K), dtype=np.int32)
        if itype == "uniform":
            imin, imax = int(iparams["min"]), int(iparams["max"])
        elif itype == "custom":
            v = iparams["values"]
            ivals = np.full((W, K), int(v), dtype=np.int32) if np.isscalar(v) else np.asarray(v, dtype=np.int32)
        cs = _g(cfg, "cost_structure")
        hold, pen = _g(cs, "holding_cost"), _g(cs, "penalty_cost")
        sc = _g(cs, "shipment_cost")
        comp = _g(cfg, "components")
        ds = _g(comp, "demand_sampler")
        dtype_ = _g(ds, "type")
        if dtype_ == "poisson":
            p = _g(ds, "params")
            lo, ps, lq = p["lambda_orders"], p["probability_skus"], p["lambda_quantity"]
            if np.isscalar(lo):
                lo_a = np.full(R, float(lo))
                ps_a = np.full(R, float(ps))
                lq_a = np.full((R, K), float(lq))
            else:
                lo_a, ps_a, lq_a = (np.asarray(lo, np.float64), np.asarray(ps, np.float64),
                                    np.asarray(lq, np.float64))
        else:
            lo_a, ps_a, lq_a = np.zeros(R), np.zeros(R), np.zeros((R, K))
        alp = _g(_g(comp, "demand_allocator"), "params")
        ms = alp["max_splits"]
        max_splits = W - 1 if ms == "default" else int(ms)
        lt = _g(comp, "lead_time_sampler")
        ltp = _g(lt, "params")
        elt = np.asarray(_g(ltp, "expected_lead_times"), dtype=np.int32)
        md = np.zeros(1, np.int32)
        md_per = False
        if _g(lt, "type") == "stochastic":
            dev = _g(_g(ltp, "deviation"), "max_deviation")
            md_per = isinstance(dev, (list, tuple, np.ndarray))
            md = np.asarray(dev if md_per else [dev], dtype=np.int32)
        ls = _g(comp, "lost_sales_handler")
        ltype = _g(ls, "type")
        alpha = float(_g(ls, "params")["alpha"]) if ltype == "cost" else 0.0
        rcp = _g(_g(comp, "reward_calculator"), "params")
        norm = meta.get("obs_normalization", "off") or "off"
        stats = meta.get("obs_stats")
        mean = std = None
        if norm in ("meanstd_custom", "meanstd_grouped") and stats is not None:
            mean = np.ascontiguousarray(stats[0], dtype=np.float32)
            std = np.ascontiguousarray(stats[1], dtype=np.float32)
            norm_c = "meanstd"
        elif norm == "ratio":
            norm_c = "ratio"
        else:
            norm_c = "off"
        dist = _g_opt(cs, "distances")
        skw = _g_opt(cs, "sku_weights")
        spec = cls(
            W=W, K=K, R=R, episode_length=T, action_type=atype, action_param=aparam,
            init_type=itype, init_min=imin, init_max=imax, init_values=ivals,
            holding=np.atleast_1d(np.asarray(hold, np.float64)), holding_per_sku=isinstance(hold, (list, tuple)),
            penalty=np.atleast_1d(np.asarray(pen, np.float64)), penalty_per_sku=isinstance(pen, (list, tuple)),
            sku_weights=np.asarray(skw if skw is not None else np.ones(K), np.float64),
            distances=np.asarray(dist if dist is not None else np.zeros((W, R)), np.float64),
            outbound_fixed=np.asarray(_g(sc, "outbound_fixed"), np.float64),
            outbound_variable=np.asarray(_g(sc, "outbound_variable"), np.float64),
            inbound_fixed=np.asarray(_g(sc, "inbound_fixed"), np.float64),
            inbound_variable=np.asarray(_g(sc, "inbound_variable"), np.float64),
            demand_type=dtype_, lambda_orders=lo_a, probability_skus=ps_a, lambda_quantity=lq_a,
            max_splits=max_splits, lead_type=_g(lt, "type"), expected_lead_times=elt,
            max_dev_per_sku=md_per, max_deviation=md, lost_type=ltype, lost_alpha=alpha,
            scope=_g(rcp, "scope"), scale_factor=float(_g(rcp, "scale_factor")),
            features=_features_dict(_g_opt(cfg, "features")),
            include_warehouse_id=bool(meta.get("include_warehouse_id", False)),
            obs_normalization=norm_c, obs_mean=mean, obs_std=std,
            num_eval_episodes=int(meta.get("num_eval_episodes") or 0),
        )
        if dtype_ == "empirical":
            from .trace import pack_demand_trace
            src = demand_trace if demand_trace is not None else meta.get("demand_trace")
            if src is None:
                raise ValueError("EmpiricalDemandSampler requires a demand trace (env_meta['demand_trace'])")
            spec.trace = pack_demand_trace(src, K, data_mode=meta.get("data_mode", "train"))
        spec.validate()
        return spec

    def validate(self) -> None:
        if not (1 <= self.W <= abi.MAX_W and 1 <= self.K <= abi.MAX_K and 1 <= self.R <= abi.MAX_R):
            raise ValueError(f"unsupported dims W={self.W} K={self.K} R={self.R} "
                             f"(max {abi.MAX_W}/{abi.MAX_K}/{abi.MAX_R})")
        if self.demand_type == "poisson":
            # rates >= 10 take numpy's PTRS branch (demand_sampler.py:138,153 -> Generator.poisson):
            # the library's sequential sampler (csrc/demand_ab.hip, demand_seq_kernel)
            if not (np.all(self.lambda_orders > 0) and np.all(self.lambda_quantity > 0)):
                raise ValueError("Poisson rates must be positive (PositiveFloat, schema.py:191)")
            if np.any(self.lambda_orders >= 1e6) or np.any(self.lambda_quantity >= 20000):
                raise ValueError("Poisson rates out of range: lambda_orders < 1e6, lambda_quantity < 20000 "
                                 "(quantities are 16-bit record fields)")
            lam = float(self.lambda_orders.sum())
            if np.ceil(lam + 12.0 * np.sqrt(lam + 1.0) + 64.0) > abi.ORDER_CAP_MAX:
                raise ValueError(f"sum of lambda_orders {lam:g}: per-step order capacity exceeds "
                                 f"{abi.ORDER_CAP_MAX} records per env (int32 record indexing)")
        if self.obs_mean is not None and self.obs_mean.shape != (self.n_features,):
            raise ValueError(f"obs_stats must have shape ({self.n_features},), got {self.obs_mean.shape}")
        if self.demand_type == "empirical" and self.trace["n_rows"] < self.episode_length:
            raise ValueError(f"EmpiricalDemandSampler: episode_length ({self.episode_length}) > available "
                             f"timesteps ({self.trace['n_rows']})")

    # ---- C ABI -----------------------------------------------------------------------------
    def to_desc(self) -> abi.MscEnvDesc:
        keep = self._keep
        keep.clear()

        def arr(a, dt, ct):
            if a is None:
                return None
            a = np.ascontiguousarray(a, dtype=dt)
            keep.append(a)
            return a.ctypes.data_as(C.POINTER(ct))

        d = abi.MscEnvDesc()
        d.abi_version = abi.ABI_VERSION
        d.n_warehouses, d.n_skus, d.n_regions, d.episode_length = self.W, self.K, self.R, self.episode_length
        d.action_type = abi.ACTION[self.action_type]
        d.action_param = arr(self.action_param, np.float64, C.c_double)
        d.init_type = abi.INIT[self.init_type]
        d.init_min, d.init_max = self.init_min, self.init_max
        d.init_values = arr(self.init_values, np.int32, C.c_int32)
        d.holding_per_sku, d.holding_cost = int(self.holding_per_sku), arr(self.holding, np.float64, C.c_double)
        d.penalty_per_sku, d.penalty_cost = int(self.penalty_per_sku), arr(self.penalty, np.float64, C.c_double)
        d.sku_weights = arr(self.sku_weights, np.float64, C.c_double)
        d.distances = arr(self.distances, np.float64, C.c_double)
        d.outbound_fixed = arr(self.outbound_fixed, np.float64, C.c_double)
        d.outbound_variable = arr(self.outbound_variable, np.float64, C.c_double)
        d.inbound_fixed = arr(self.inbound_fixed, np.float64, C.c_double)
        d.inbound_variable = arr(self.inbound_variable, np.float64, C.c_double)
        d.demand_type = abi.DEMAND[self.demand_type]
        d.lambda_orders = arr(self.lambda_orders, np.float64, C.c_double)
        d.probability_skus = arr(self.probability_skus, np.float64, C.c_double)
        d.lambda_quantity = arr(self.lambda_quantity, np.float64, C.c_double)
        if self.trace is not None:
            d.trace_n_rows = int(self.trace["n_rows"])
            d.trace_offsets = arr(self.trace["offsets"], np.int64, C.c_int64)
            d.trace_regions = arr(self.trace["regions"], np.int32, C.c_int32)
            d.trace_quantities = arr(self.trace["quantities"], np.int32, C.c_int32)
        d.max_splits = self.max_splits
        d.lead_type = abi.LEAD[self.lead_type]
        d.expected_lead_times = arr(self.expected_lead_times, np.int32, C.c_int32)
        d.max_dev_per_sku = int(self.max_dev_per_sku)
        d.max_deviation = arr(self.max_deviation, np.int32, C.c_int32)
        d.lost_type, d.lost_alpha = abi.LOST[self.lost_type], self.lost_alpha
        d.reward_scope, d.reward_scale = abi.SCOPE[self.scope], self.scale_factor
        d.feature_flags = self.feature_flags
        d.include_warehouse_id = int(self.include_warehouse_id)
        d.obs_norm = abi.OBS_NORM[self.obs_normalization]
        d.obs_mean = arr(self.obs_mean, np.float32, C.c_float)
        d.obs_std = arr(self.obs_std, np.float32, C.c_float)
        d.num_eval_episodes = self.num_eval_episodes
        d.episode_ahead = -1  # automatic; VecInventoryEnv(episode_ahead=...) overrides
        d.ea_mem_fraction = 0.0
        return d

"""Environment config loading/validation with the reference's `config_files` schema.

Mirrors `load_environment_config` (src/config/loader.py:117-165: `environment:` key,
legacy `max_order_quantities` migration `:290-315`, `feature_config_path` indirection relative to
the CWD `:153-156`) and the shape rules of `EnvironmentConfig._shape_checks` / `_post_checks`
(src/config/schema.py:664-890): per-SKU lists of length K, (W,R) cost matrices, (W,K)
lead times, `max_splits: "default"` -> W-1 and `< W`, mandatory inventory/pipeline features,
aggregates only with their parent feature.

One deliberate relaxation: the reference forbids n_regions != n_warehouses
(schema.py:670-675) although the env arithmetic supports it and every BASELINE config needs it;
`allow_nr_ne_nw=True` lifts that single check.

The result is a `ConfigNode` tree: attribute access like the reference's pydantic models
(`cfg.components.demand_sampler.type`) and item access for `params` dicts.
"""
from __future__ import annotations

import copy
import os
from pathlib import Path
from typing import Any, Dict, Optional

import yaml

FEATURE_DEFAULTS: Dict[str, bool] = {
    # FeatureConfig defaults (schema.py:595-622)
    "inventory": True, "pipeline": True, "incoming_demand_home": True, "units_shipped_home": True,
    "units_shipped_away": True, "stockout": True, "rolling_demand_mean": True, "demand_forecast": True,
    "days_of_supply": False, "net_inventory_position": False, "demand_variability": False,
    "demand_history": False, "inventory_aggregate": True, "pipeline_aggregate": True,
    "incoming_demand_home_aggregate": True, "units_shipped_away_aggregate": True,
    "rolling_demand_mean_aggregate": True, "demand_forecast_aggregate": True,
}
AGGREGATE_PARENTS = [
    ("inventory", "inventory_aggregate"), ("pipeline", "pipeline_aggregate"),
    ("incoming_demand_home", "incoming_demand_home_aggregate"),
    ("units_shipped_away", "units_shipped_away_aggregate"),
    ("rolling_demand_mean", "rolling_demand_mean_aggregate"),
    ("demand_forecast", "demand_forecast_aggregate"),
]


class ConfigNode:
    """Read-mostly view over a validated config dict (attribute + item access)."""

    def __init__(self, data: Dict[str, Any]):
        object.__setattr__(self, "_d", data)

    def __getattr__(self, k):
        d = object.__getattribute__(self, "_d")
        if k not in d:
            raise AttributeError(k)
        v = d[k]
        return ConfigNode(v) if isinstance(v, dict) and k != "params" else v

    def __setattr__(self, k, v):
        self._d[k] = v

    def __getitem__(self, k):
        return self._d[k]

    def __contains__(self, k):
        return k in self._d

    def get(self, k, default=None):
        return self._d.get(k, default)

    def to_dict(self) -> Dict[str, Any]:
        return copy.deepcopy(self._d)

    def __repr__(self):
        return f"ConfigNode({self._d!r})"


def _is_num(x) -> bool:
    return isinstance(x, (int, float)) and not isinstance(x, bool)


def _check_len(lst, n, what):
    if not isinstance(lst, list) or len(lst) != n:
        raise ValueError(f"{what} must have length {n}, got {len(lst) if isinstance(lst, list) else lst!r}")


def _check_mat(m, rows, cols, what):
    if not isinstance(m, list) or len(m) != rows or any(not isinstance(r, list) or len(r) != cols for r in m):
        raise ValueError(f"{what} must have shape ({rows}, {cols})")


def validate_feature_config(f: Optional[Dict[str, Any]]) -> Dict[str, bool]:
    out = dict(FEATURE_DEFAULTS)
    for k, v in (f or {}).items():
        if k not in FEATURE_DEFAULTS:
            raise ValueError(f"unknown feature '{k}'")
        out[k] = bool(v)
    if not out["inventory"]:
        raise ValueError("inventory must always be enabled")
    if not out["pipeline"]:
        raise ValueError("pipeline must always be enabled")
    for parent, agg in AGGREGATE_PARENTS:
        if out[agg] and not out[parent]:
            raise ValueError(f"'{agg}' cannot be enabled when '{parent}' is disabled")
    return out


def _migrate(d: Dict[str, Any]) -> Dict[str, Any]:
    if d.get("action_space") is not None:
        return d
    mq = d.pop("max_order_quantities", None)
    if mq is None:
        return d
    k = d.get("n_skus", 1)
    d["action_space"] = {"type": "direct", "params": {
        "max_order_quantities": [int(mq)] * k if _is_num(mq) else [int(x) for x in mq]}}
    return d


def validate_environment_config(raw: Dict[str, Any], *, allow_nr_ne_nw: bool = False) -> ConfigNode:
    d = _migrate(copy.deepcopy(raw))
    W, K, R = int(d["n_warehouses"]), int(d["n_skus"]), int(d["n_regions"])
    if min(W, K, R, int(d["episode_length"])) <= 0:
        raise ValueError("n_warehouses, n_skus, n_regions, episode_length must be positive")
    if R != W and not allow_nr_ne_nw:
        raise ValueError(f"n_regions ({R}) must equal n_warehouses ({W}) (home region assumption: "
                         "each warehouse is assigned to exactly one region); pass allow_nr_ne_nw=True to relax")
    act = d["action_space"]
    key = {"direct": "max_order_quantities", "demand_centered": "max_quantity_adjustment",
           "base_stock": "max_stock_level"}.get(act["type"])
    if key is None:
        raise ValueError(f"unknown action_space type {act['type']!r}")
    _check_len(act["params"][key], K, f"action_space.params.{key}")
    _check_len(d["max_wh_capacities"], W, "max_wh_capacities")
    ii = d["initial_inventory"]
    if ii["type"] == "uniform":
        if ii["params"]["min"] > ii["params"]["max"]:
            raise ValueError("uniform params must satisfy min <= max")
    elif ii["type"] == "custom":
        v = ii["params"]["values"]
        if not _is_num(v):
            _check_mat(v, W, K, "initial_inventory.custom params.values")
    elif ii["type"] != "zero":
        raise ValueError(f"unknown initial_inventory type {ii['type']!r}")
    cs = d["cost_structure"]
    for k in ("holding_cost", "penalty_cost"):
        if isinstance(cs[k], list):
            _check_len(cs[k], K, k)
    sc = cs["shipment_cost"]
    for k in ("outbound_fixed", "outbound_variable"):
        _check_mat(sc[k], W, R, f"shipment_cost.{k}")
    for k in ("inbound_fixed", "inbound_variable"):
        _check_mat(sc[k], W, K, f"shipment_cost.{k}")
    if cs.get("sku_weights") is not None:
        _check_len(cs["sku_weights"], K, "sku_weights")
    if cs.get("distances") is not None:
        _check_mat(cs["distances"], W, R, "distances")
    comp = d["components"]
    ds = comp["demand_sampler"]
    if ds["type"] == "poisson":
        p = ds["params"]
        scal = [_is_num(p[k]) for k in ("lambda_orders", "probability_skus", "lambda_quantity")]
        if any(scal) and not all(scal):
            raise ValueError("poisson params must be either all scalars or all arrays; cannot mix scalar and array parameters")
        if not all(scal):
            _check_len(p["lambda_orders"], R, "demand_sampler.poisson params.lambda_orders")
            _check_len(p["probability_skus"], R, "demand_sampler.poisson params.probability_skus")
            _check_mat(p["lambda_quantity"], R, K, "demand_sampler.poisson params.lambda_quantity")
    elif ds["type"] != "empirical":
        raise ValueError(f"Unknown demand sampler: {ds['type']}")
    al = comp["demand_allocator"]
    if al["type"] != "greedy":
        raise ValueError(f"Unknown demand allocator: {al['type']}")
    ms = al["params"]["max_splits"]
    if ms == "default":
        al["params"]["max_splits"] = W - 1
    elif int(ms) >= W or int(ms) < 0:
        raise ValueError(f"demand_allocator.greedy max_splits must be < n_warehouses={W}")
    lt = comp["lead_time_sampler"]
    if lt["type"] not in ("fixed", "stochastic"):
        raise ValueError(f"Unknown lead time sampler: {lt['type']}")
    _check_mat(lt["params"]["expected_lead_times"], W, K, "lead_time_sampler params.expected_lead_times")
    if lt["type"] == "stochastic":
        md = lt["params"]["deviation"]["max_deviation"]
        if isinstance(md, list):
            _check_len(md, K, "lead_time_sampler deviation.max_deviation")
    ls = comp["lost_sales_handler"]
    if ls["type"] not in ("closest", "shipment", "cost"):
        raise ValueError(f"Unknown lost sales handler: {ls['type']}")
    rc = comp["reward_calculator"]
    if rc["type"] != "cost":
        raise ValueError(f"Unknown reward calculator: {rc['type']}")
    if rc["params"]["scope"] not in ("agent", "team"):
        raise ValueError("reward scope must be 'agent' or 'team'")
    d["features"] = validate_feature_config(d.get("features"))
    return ConfigNode(d)


def load_feature_config(path: str) -> Dict[str, bool]:
    with open(path) as fh:
        f = yaml.safe_load(fh)
    return validate_feature_config(f.get("features", f))


def load_environment_config(path: str, *, allow_nr_ne_nw: bool = False) -> ConfigNode:
    """`load_environment_config` of src/config/loader.py:117-165 (synthetic data_source needs the
    reference's pickled generator models, which are absent offline: rejected)."""
    with open(path) as fh:
        d = yaml.safe_load(fh)
    d = d.get("environment", d)
    d = _migrate(d)
    fpath = d.pop("feature_config_path", None)
    if fpath is not None:
        d["features"] = load_feature_config(fpath if os.path.isabs(fpath) or os.path.exists(fpath)
                                            else str(Path(path).resolve().parents[2] / fpath))
    if d.get("data_source", {}).get("type") == "synthetic":
        raise ValueError("data_source 'synthetic' needs the reference's fitted generator models (absent); "
                         "use marlsc.synthetic.make_synthetic_env_config or a 'custom' data source")
    return validate_environment_config(d, allow_nr_ne_nw=allow_nr_ne_nw)

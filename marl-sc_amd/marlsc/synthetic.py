"""Deterministic synthetic supply-chain configurations (any W warehouses x R regions x K SKUs).

The reference ships only 3-warehouse YAMLs and a closed-form cost helper
(`src/utils/cost_generator.py:87-166`) that is never called from `src/` and yields negative
distances when n_regions > n_warehouses (`_ring_distance` at `:77-80`). BASELINE.json's configs
(2x4x2, 8x64x5, 16x256x5) need n_regions != n_warehouses, so this module builds its own
tie-free, non-negative cost structure:

    t(w, r)   = ring(w, r mod W) / max(W // 2, 1)
    sf(i,j,a) = 1 + a * sin(0.9 i + 1.7 j + 0.3)
    distance  = (150 + 270 t) * sf(w, r, .06)
    out_fixed = (22 + 20 t)   * sf(w, r, .08)
    out_var   = (0.18 + 0.24 t) * sf(w, r, .06)

The returned dict has exactly the `environment:` layout of the reference YAMLs
(`config_files/environments/env_symmetric_3WH5SKU.yaml`), so it goes through the same loader.
"""
from __future__ import annotations

import math
from typing import Any, Dict, Optional

# Feature toggles of config_files/features/feature_config.yaml (the reference's default file).
FEATURE_CONFIG_YAML = {
    "inventory": True, "inventory_aggregate": True, "pipeline": True, "rolling_demand_mean": True,
    "stockout": False, "incoming_demand_home": False, "units_shipped_home": False,
    "units_shipped_away": False, "demand_forecast": False, "days_of_supply": False,
    "net_inventory_position": False, "demand_history": False, "demand_variability": False,
    "pipeline_aggregate": False, "incoming_demand_home_aggregate": False,
    "units_shipped_away_aggregate": False, "rolling_demand_mean_aggregate": False,
    "demand_forecast_aggregate": False,
}


def _sf(i: int, j: int, amp: float) -> float:
    return 1.0 + amp * math.sin(0.9 * i + 1.7 * j + 0.3)


def _ring(i: int, j: int, n: int) -> int:
    d = abs(i - j)
    return min(d, n - d)


def sku_arrays(n_skus: int) -> Dict[str, list]:
    """Per-SKU weights / penalties / inbound levels: strictly increasing, 3-decimal rounded."""
    weights, penalty, in_fixed, in_var = [], [], [], []
    for s in range(n_skus):
        x = s / max(n_skus - 1, 1)
        weights.append(round(0.5 + 9.5 * x ** 1.3 + 0.01 * math.sin(2.1 * s + 0.4), 3))
        penalty.append(round(3.0 + 4.0 * x + 0.02 * math.sin(1.3 * s + 0.7), 3))
        in_fixed.append(round(1.0 + 1.5 * x, 3))
        in_var.append(round(0.8 + 0.6 * x, 5))
    return {"sku_weights": weights, "penalty": penalty, "in_fixed": in_fixed, "in_var": in_var}


def make_synthetic_env_config(
    n_warehouses: int,
    n_regions: int,
    n_skus: int,
    *,
    episode_length: int = 100,
    lambda_orders: float = 4.0,
    probability_skus: float = 0.667,
    lambda_quantity: float = 5.0,
    lead_time: int = 3,
    initial_inventory: int = 60,
    max_quantity_adjustment: int = 20,
    features: Optional[Dict[str, bool]] = None,
    lost_sales: str = "shipment",
    scope: str = "agent",
    scale_factor: float = 0.01,
) -> Dict[str, Any]:
    """Build an `environment:` config dict (reference YAML layout) for a W x R x K instance.

    Defaults are SURVEY.md section 8's assumptions for BASELINE configs 1-5: Poisson
    lambda_o=4 / p=0.667 / lambda_q=5 per region, demand_centered +-20, fixed lead time 3,
    custom initial inventory 60, shipment lost sales, agent scope, scale 0.01 and the
    feature_config.yaml feature set.
    """
    W, R, K = n_warehouses, n_regions, n_skus
    half = max(W // 2, 1)
    dist, of, ov = [], [], []
    for w in range(W):
        drow, frow, vrow = [], [], []
        for r in range(R):
            t = _ring(w, r % W, W) / half
            drow.append(round((150.0 + 270.0 * t) * _sf(w, r, 0.06), 3))
            frow.append(round((22.0 + 20.0 * t) * _sf(w, r, 0.08), 3))
            vrow.append(round((0.18 + 0.24 * t) * _sf(w, r, 0.06), 5))
        dist.append(drow)
        of.append(frow)
        ov.append(vrow)
    sku = sku_arrays(K)
    return {
        "n_warehouses": W,
        "n_skus": K,
        "n_regions": R,
        "episode_length": episode_length,
        "max_wh_capacities": [10_000_000] * W,
        "action_space": {"type": "demand_centered",
                         "params": {"max_quantity_adjustment": [max_quantity_adjustment] * K}},
        "initial_inventory": {"type": "custom", "params": {"values": [[initial_inventory] * K for _ in range(W)]}},
        "cost_structure": {
            "holding_cost": 1.0,
            "penalty_cost": sku["penalty"],
            "shipment_cost": {
                "outbound_fixed": of,
                "outbound_variable": ov,
                "inbound_fixed": [list(sku["in_fixed"]) for _ in range(W)],
                "inbound_variable": [list(sku["in_var"]) for _ in range(W)],
            },
            "sku_weights": sku["sku_weights"],
            "distances": dist,
        },
        "components": {
            "demand_sampler": {"type": "poisson", "params": {
                "lambda_orders": [lambda_orders] * R,
                "probability_skus": [probability_skus] * R,
                "lambda_quantity": [[lambda_quantity] * K for _ in range(R)],
            }},
            "demand_allocator": {"type": "greedy", "params": {"max_splits": "default"}},
            "lead_time_sampler": {"type": "fixed", "params": {
                "expected_lead_times": [[lead_time] * K for _ in range(W)]}},
            "lost_sales_handler": ({"type": "cost", "params": {"alpha": 5.0}} if lost_sales == "cost"
                                   else {"type": lost_sales, "params": None}),
            "reward_calculator": {"type": "cost", "params": {
                "scope": scope, "scale_factor": scale_factor, "cost_weights": [0.25, 0.25, 0.25, 0.25]}},
        },
        "data_source": {"type": "custom"},
        "features": dict(features if features is not None else FEATURE_CONFIG_YAML),
    }


def make_synthetic_trace(n_regions: int, n_skus: int, n_timesteps: int = 300, orders_per_step=(200, 1000),
                         seed: int = 0) -> Dict[str, Any]:
    """A synthetic preprocessor output frame (src/data/preprocessor.py:682-696: timestep,
    region_id, order_id, sku_id, quantity; one row per order line) for the empirical sampler at
    any size (SURVEY.md 8(d), configs[4]: ~Poisson(200-1,000) orders per timestep over the
    regions). Order ids are strings, as in the real data; an order has 1..K lines with
    quantities 1..12. Returned as a dict of numpy columns (what `pack_demand_trace` and
    `env_meta['demand_trace']` accept)."""
    import numpy as np

    rng = np.random.default_rng(seed)
    lo, hi = orders_per_step
    n_t = rng.poisson(rng.uniform(lo, hi, n_timesteps)).astype(np.int64)   # orders per timestep
    n = int(n_t.sum())
    order_ts = np.repeat(np.arange(n_timesteps, dtype=np.int64), n_t)
    order_reg = rng.integers(0, n_regions, n)
    lines = rng.integers(1, n_skus + 1, n)                                  # distinct SKUs per order
    # the first `lines` SKUs of a random permutation per order
    perm = np.argsort(rng.random((n, n_skus)), axis=1)
    take = np.arange(n_skus)[None, :] < lines[:, None]
    o_idx, col = np.nonzero(take)
    sku = perm[o_idx, col]
    oid = np.char.add("o", np.char.zfill(np.arange(n).astype(str), 8))
    return {"timestep": order_ts[o_idx], "region_id": order_reg[o_idx], "order_id": oid[o_idx],
            "sku_id": sku.astype(np.int64), "quantity": rng.integers(1, 13, o_idx.size).astype(np.int64)}

"""Helpers to load the golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py)."""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np

from marlsc.spec import EnvSpec

GOLDEN = Path(__file__).resolve().parent / "golden"
ENV_FIXTURES = ["c1_2x4x2", "repo_3wh5sku", "c3_8x64x5", "c8_split", "variant_a", "variant_b", "variant_c"]


def load(name):
    d = dict(np.load(GOLDEN / f"{name}.npz"))
    meta = json.loads(str(d.pop("meta_json")))
    return d, meta


def spec_of(d, meta) -> EnvSpec:
    env_meta = dict(meta["env_meta"])
    if "obs_mean" in d:
        env_meta["obs_stats"] = (d["obs_mean"], d["obs_std"])
    return EnvSpec.from_config(meta["config"], env_meta, allow_nr_ne_nw=True)


INFO_MAP = {  # fixture key -> msc_step_info field
    "inventory": "inventory_before", "pending_total": "pending_total", "order_quantities": "order_quantities",
    "demand_per_region": "demand_per_region", "fulfilled_per_warehouse": "fulfilled_per_warehouse",
    "unfulfilled_demands": "unfulfilled_demands", "shipment_counts": "shipment_counts",
    "shipment_quantities": "shipment_quantities", "shipment_quantities_by_sku": "shipment_quantities_by_sku",
    "lost_order_counts": "lost_order_counts", "n_orders": "n_orders", "lost_sales": "lost_sales",
}
COST_KEYS = ["holding_cost", "penalty_cost", "outbound_shipment_cost", "inbound_shipment_cost"]


def f32_ulp_diff(a, b):
    a = np.asarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.asarray(b, np.float32).view(np.int32).astype(np.int64)
    a = np.where(a < 0, -(a & 0x7FFFFFFF), a)
    b = np.where(b < 0, -(b & 0x7FFFFFFF), b)
    return np.abs(a - b)

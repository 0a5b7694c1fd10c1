"""TEST INFRASTRUCTURE ONLY (imported by tests/, never by the product path): numpy restatement of
the statistics arithmetic of `compute_obs_statistics` (reference src/utils/obs_stats.py:11-169),
written from the reference's FeatureConfig flags, independently of the product's feature-group
table (marlsc/ppo.py:feature_groups), so a wrong group width or aggregate flag there shows up.
The arithmetic is the reference's own numpy calls on the same f32 sample matrix, so equal inputs
give bit-equal outputs."""
from __future__ import annotations

from typing import Dict, Tuple

import numpy as np

# the per-SKU groups of _compute_grouped_stats in their fixed order (obs_stats.py:129-145):
# (flag, width in SKU blocks: 'lt' = max expected lead time, aggregate flag or None)
_GROUPS = (("inventory", 1, "inventory_aggregate"),
           ("pipeline", "lt", "pipeline_aggregate"),
           ("incoming_demand_home", 1, "incoming_demand_home_aggregate"),
           ("units_shipped_home", 1, None),
           ("units_shipped_away", 1, "units_shipped_away_aggregate"),
           ("stockout", 1, None),
           ("rolling_demand_mean", 1, "rolling_demand_mean_aggregate"),
           ("demand_forecast", 1, "demand_forecast_aggregate"))


def obs_statistics_ref(all_obs: np.ndarray, mode: str, features: Dict[str, bool], n_skus: int,
                       max_expected_lead_time: int) -> Tuple[np.ndarray, np.ndarray]:
    x = np.array(all_obs, dtype=np.float32)                      # obs_stats.py:74
    if mode == "meanstd_grouped":                                # :77-80, :93-169
        mean = np.zeros(x.shape[1], dtype=np.float32)
        std = np.ones(x.shape[1], dtype=np.float32)
        i = 0
        for flag, width, agg in _GROUPS:
            if not features.get(flag):
                continue
            w = n_skus * (max_expected_lead_time if width == "lt" else 1)
            mean[i:i + w] = float(x[:, i:i + w].mean())          # :157-161
            std[i:i + w] = float(x[:, i:i + w].std())
            i += w
            if agg is not None and features.get(agg):            # :164-167
                mean[i] = float(x[:, i].mean())
                std[i] = float(x[:, i].std())
                i += 1
    else:
        mean = x.mean(axis=0)                                    # :82-83
        std = x.std(axis=0)
    std = np.where(std < 1e-8, 1.0, std)                         # :85
    return mean, std

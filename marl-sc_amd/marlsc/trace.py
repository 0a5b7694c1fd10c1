"""Empirical demand trace -> CSR device layout (the input side of `EmpiricalDemandSampler`).

The reference samples empirical demand from the preprocessor's output frame
(src/data/preprocessor.py:682-696: columns timestep, region_id, order_id, sku_id, quantity) by
filtering one timestep per call and grouping by (region_id, order_id) with pandas
(src/environment/components/demand_sampler.py:199-261), ~42 ms per step at 256 regions.
Here the frame is packed ONCE into CSR over the sorted available timesteps:

    offsets[i] .. offsets[i+1]  = orders of the i-th available timestep, in groupby order
    regions[j], quantities[j, :K] = region and per-SKU summed quantity of order j

so that one env step reads its orders as a contiguous slice. SKU ids outside [0, K) are dropped
like the reference (demand_sampler.py:255).
"""
from __future__ import annotations

from typing import Any, Dict

import numpy as np


def _frame_columns(src: Any):
    cols = {}
    for c in ("timestep", "region_id", "order_id", "sku_id", "quantity"):
        cols[c] = np.asarray(src[c])
    return cols


def pack_demand_trace(src: Any, n_skus: int, data_mode: str = "train") -> Dict[str, Any]:
    """src: DataFrame / dict of columns, or {"train": ..., "val": ...} (data_mode selects, as
    `context.data_mode == "val"` does at demand_sampler.py:188-192)."""
    if isinstance(src, dict) and "train" in src:
        src = src["val"] if data_mode == "val" and src.get("val") is not None else src["train"]
    c = _frame_columns(src)
    ts_unique = np.unique(c["timestep"])
    q = c["quantity"]
    if np.any(q != np.round(q)) or np.any(q < 0) or np.any(q > 65535):
        raise ValueError("trace quantities must be integers in [0, 65535]")
    # group key order: timestep, region_id, order_id (lexicographic on the order id's own type)
    oid = c["order_id"]
    oid_codes = np.unique(oid, return_inverse=True)[1]
    order = np.lexsort((oid_codes, c["region_id"], c["timestep"]))
    ts, reg, oc = c["timestep"][order], c["region_id"][order].astype(np.int64), oid_codes[order]
    sku, qty = c["sku_id"][order].astype(np.int64), q[order].astype(np.int64)
    new = np.ones(len(ts), dtype=bool)
    new[1:] = (ts[1:] != ts[:-1]) | (reg[1:] != reg[:-1]) | (oc[1:] != oc[:-1])
    gid = np.cumsum(new) - 1
    n_orders = int(gid[-1] + 1) if len(gid) else 0
    quant = np.zeros((n_orders, n_skus), dtype=np.int64)
    ok = (sku >= 0) & (sku < n_skus)
    np.add.at(quant, (gid[ok], sku[ok]), qty[ok])
    regions = reg[new].astype(np.int32)
    order_ts = ts[new]
    row = np.searchsorted(ts_unique, order_ts)
    offsets = np.zeros(len(ts_unique) + 1, dtype=np.int64)
    np.add.at(offsets, row + 1, 1)
    offsets = np.cumsum(offsets)
    if np.any(quant > 65535):
        raise ValueError("summed order quantity exceeds 65535")
    return {"n_rows": int(len(ts_unique)), "timesteps": ts_unique, "offsets": offsets,
            "regions": regions, "quantities": quant.astype(np.int32)}


def _group_mean(vals) -> float:
    """The f64 mean pandas' `groupby(...).mean()` computes for one group (its cython group_mean):
    a Kahan-compensated running sum in row order, NaNs skipped, divided by the count. A plain
    sum / len can differ in the last ulp and flip `idxmin` between near-equal regions."""
    total, comp, n = 0.0, 0.0, 0
    for v in vals:
        if v != v:
            continue
        n += 1
        y = v - comp
        t = total + y
        comp = t - total - y
        if comp != comp:
            comp = 0.0
        total = t
    return total / n if n else float("nan")


def map_excluded_regions(order_region_ids, selected_region_ids, warehouse_to_region) -> "np.ndarray":
    """`DataProcessor.map_excluded_regions` (src/data/preprocessor.py:382-441), restated on numpy
    columns: an order whose region is not selected moves to the selected region that shares
    warehouses with it and has the lowest mean `fixed_costs` over those warehouse pairs
    (`groupby('destinationregionid').mean().idxmin()`, the smallest id among equal means); with no
    warehouse pair for the excluded region, or no selected region served by its warehouses, it
    moves to selected_region_ids[0]. Region ids compare as strings, as in the reference.

    warehouse_to_region: dict / DataFrame with columns sourcenodeid, destinationregionid,
    fixed_costs. Returns the mapped region ids (elements of selected_region_ids)."""
    ids = np.asarray(order_region_ids, dtype=object)
    sel = list(selected_region_ids)
    sel_str = [str(r) for r in sel]
    sel_set = set(sel_str)
    src = np.asarray(warehouse_to_region["sourcenodeid"], dtype=object)
    dst = np.asarray(warehouse_to_region["destinationregionid"], dtype=object).astype(str)
    fc = np.asarray(warehouse_to_region["fixed_costs"], dtype=np.float64)
    ids_str = ids.astype(str)
    out = ids.copy()
    excluded = [r for r in dict.fromkeys(ids.tolist()) if str(r) not in sel_set]  # first-seen order (unique())
    for ex in excluded:
        ex_s = str(ex)
        pair = dst == ex_s
        if not pair.any():
            nearest = sel[0]
        else:
            whs = set(src[pair].tolist())
            inc = np.isin(dst, sel_str) & np.array([w in whs for w in src.tolist()], dtype=bool)
            if not inc.any():
                nearest = sel[0]
            else:
                # mean fixed cost per destination region; pandas groups and idxmin on the original
                # destinationregionid values; ties -> the first in sorted group order
                keys = np.asarray(warehouse_to_region["destinationregionid"], dtype=object)[inc]
                costs = fc[inc]
                groups = {}
                for k, v in zip(keys.tolist(), costs.tolist()):
                    groups.setdefault(k, []).append(v)
                means = {k: _group_mean(v) for k, v in groups.items()}
                # idxmin: NaN means skipped, the first minimum in sorted key order
                cand = [k for k in sorted(groups) if means[k] == means[k]] or sorted(groups)
                best_k = min(cand, key=lambda k: means[k])
                nearest = next((r for r in sel if str(r) == str(best_k)), sel[0])
        out[ids_str == ex_s] = nearest
    return out

"""TEST INFRASTRUCTURE ONLY (imported by tests/, never by the product path): pandas restatement of
`DataProcessor.map_excluded_regions` (reference src/data/preprocessor.py:382-441), written with the
same pandas operations the reference runs on the same columns -- `astype(str).isin`, `unique()` in
first-seen order, the warehouse filter, `groupby('destinationregionid')['fixed_costs'].mean()` and
`idxmin()` -- so the product's numpy restatement (marlsc/trace.py) is checked against pandas' own
group-mean arithmetic (Kahan-compensated sums) and its tie rule.
Parity note: pinned to pandas, the reference's own dependency; the reference's test of this
function (tests/test_excluded_region_mapping.py) reads data_files/raw CSVs that the reference does
not ship, so no reference-produced vector exists."""
from __future__ import annotations

import pandas as pd


def map_excluded_regions_pd(order_region_ids, selected_region_ids, w2r: pd.DataFrame) -> pd.Series:
    ids = pd.Series(order_region_ids, dtype=object)
    sel = list(selected_region_ids)
    sel_str = [str(r) for r in sel]                       # preprocessor.py:399
    out = ids.copy()                                      # :396
    dst_str = w2r["destinationregionid"].astype(str)
    for ex in ids[~ids.astype(str).isin(set(sel_str))].unique():   # :403-407
        pairs = w2r[dst_str == str(ex)]                   # :412-414
        if len(pairs) == 0:
            near = sel[0]                                 # :417-418
        else:
            inc = w2r[dst_str.isin(sel_str) & w2r["sourcenodeid"].isin(pairs["sourcenodeid"].unique())]
            if len(inc) == 0:
                near = sel[0]                             # :429-430
            else:
                best = str(inc.groupby("destinationregionid")["fixed_costs"].mean().idxmin())  # :434-435
                near = next((r for r in sel if str(r) == best), sel[0])                      # :436
        out[ids.astype(str) == str(ex)] = near            # :439
    return out

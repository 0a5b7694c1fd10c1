"""ctypes mirror of include/marlsc.h and the loader of the HIP library (libmarlsc.so).

The product path has no CPU fallback: if the HIP library is missing, `lib()` raises.
torch is imported first so that libmarlsc.so binds to the same HIP runtime instance as torch
(both carry the soname libamdhip64.so.7).
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

ABI_VERSION = 2
MAX_W, MAX_K, MAX_R, HISTORY = 32, 16, 4096, 5
ORDER_CAP_MAX = 1 << 24  # include/marlsc.h MSC_ORDER_CAP_MAX

DEMAND = {"poisson": 0, "empirical": 1}
ACTION = {"direct": 0, "demand_centered": 1, "base_stock": 2}
INIT = {"uniform": 0, "custom": 1, "zero": 2}
LEAD = {"fixed": 0, "stochastic": 1}
LOST = {"closest": 0, "shipment": 1, "cost": 2}
SCOPE = {"agent": 0, "team": 1}
OBS_NORM = {"off": 0, "ratio": 1, "meanstd": 2}
RESET_EVAL_RESTART = 1

# (feature key, bit) in _build_local_obs block order (multi_env.py:620-695)
FEATURE_BITS = [
    ("inventory", 1 << 0), ("inventory_aggregate", 1 << 1), ("pipeline", 1 << 2), ("pipeline_aggregate", 1 << 3),
    ("incoming_demand_home", 1 << 4), ("incoming_demand_home_aggregate", 1 << 5), ("units_shipped_home", 1 << 6),
    ("units_shipped_away", 1 << 7), ("units_shipped_away_aggregate", 1 << 8), ("stockout", 1 << 9),
    ("rolling_demand_mean", 1 << 10), ("rolling_demand_mean_aggregate", 1 << 11), ("demand_forecast", 1 << 12),
    ("demand_forecast_aggregate", 1 << 13), ("days_of_supply", 1 << 14), ("net_inventory_position", 1 << 15),
    ("demand_variability", 1 << 16), ("demand_history", 1 << 17),
]

P = C.POINTER
dp, ip, lp, fp = P(C.c_double), P(C.c_int32), P(C.c_int64), P(C.c_float)


class MscEnvDesc(C.Structure):
    _fields_ = [
        ("abi_version", C.c_int32),
        ("n_warehouses", C.c_int32), ("n_skus", C.c_int32), ("n_regions", C.c_int32), ("episode_length", C.c_int32),
        ("action_type", C.c_int32), ("action_param", dp),
        ("init_type", C.c_int32), ("init_min", C.c_int32), ("init_max", C.c_int32), ("init_values", ip),
        ("holding_per_sku", C.c_int32), ("holding_cost", dp),
        ("penalty_per_sku", C.c_int32), ("penalty_cost", dp),
        ("sku_weights", dp), ("distances", dp), ("outbound_fixed", dp), ("outbound_variable", dp),
        ("inbound_fixed", dp), ("inbound_variable", dp),
        ("demand_type", C.c_int32), ("lambda_orders", dp), ("probability_skus", dp), ("lambda_quantity", dp),
        ("trace_n_rows", C.c_int32), ("trace_offsets", lp), ("trace_regions", ip), ("trace_quantities", ip),
        ("max_splits", C.c_int32),
        ("lead_type", C.c_int32), ("expected_lead_times", ip), ("max_dev_per_sku", C.c_int32), ("max_deviation", ip),
        ("lost_type", C.c_int32), ("lost_alpha", C.c_double),
        ("reward_scope", C.c_int32), ("reward_scale", C.c_double),
        ("feature_flags", C.c_uint32), ("include_warehouse_id", C.c_int32),
        ("obs_norm", C.c_int32), ("obs_mean", fp), ("obs_std", fp),
        ("num_eval_episodes", C.c_int32),
        ("episode_ahead", C.c_int32), ("ea_mem_fraction", C.c_double),
    ]


I32P = P(C.c_int32)
F64P = P(C.c_double)


class MscStepInfo(C.Structure):
    _fields_ = [(n, I32P) for n in (
        "inventory_before", "pending_total", "order_quantities", "demand_per_region", "fulfilled_per_warehouse",
        "unfulfilled_demands", "shipment_counts", "shipment_quantities", "shipment_quantities_by_sku",
        "lost_order_counts", "n_orders")] + [("lost_sales", F64P), ("costs", F64P)]


INFO_FIELDS_I32 = [f for f, t in MscStepInfo._fields_ if t is I32P]

_LIB = None
# MSC_LIB_VARIANT=<name> selects an A/B or profiling build libmarlsc_<name>.so (make variant)
_VARIANT = os.environ.get("MSC_LIB_VARIANT", "")
LIB_PATH = Path(__file__).resolve().parent / "_lib" / (f"libmarlsc_{_VARIANT}.so" if _VARIANT else "libmarlsc.so")


class MscGaussianEpilogue(C.Structure):
    """msc_gaussian_epilogue (include/marlsc.h): the fused MLPs' action-sampling epilogue."""
    _fields_ = [("log_std", C.c_void_p), ("log_std_rows", C.c_int32), ("logstd_floor", C.c_float),
                ("eps", C.c_void_p), ("actions", C.c_void_p), ("logp", C.c_void_p), ("clipped", C.c_void_p)]


def lib() -> C.CDLL:
    """Load libmarlsc.so (built by __graft_entry__.build()). Raises if it is missing."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not LIB_PATH.exists():
        raise RuntimeError(f"HIP library not built: {LIB_PATH} missing (run `python __graft_entry__.py`)")
    import torch  # noqa: F401  (bind to torch's HIP runtime instance)
    L = C.CDLL(str(LIB_PATH), mode=C.RTLD_GLOBAL)
    vp = C.c_void_p
    L.msc_env_create.argtypes = [P(MscEnvDesc), C.c_int, C.c_int64, C.c_uint32, C.c_uint32, C.c_int64,
                                 P(C.c_uint32), P(vp)]
    L.msc_env_destroy.argtypes = [vp]
    L.msc_env_destroy.restype = None
    L.msc_poisson_draws.argtypes = [vp, vp, C.c_int64, C.c_int64, vp, vp]
    L.msc_normal_keyed.argtypes = [vp, C.c_int32, C.c_int64, C.c_int32, C.c_int64, C.c_uint64, C.c_uint64, vp]
    L.msc_env_set_episode_ahead.argtypes = [vp, C.c_int32]
    L.msc_env_ea_memory.argtypes = [vp, P(C.c_int64), P(C.c_int64)]
    L.msc_env_dims.argtypes = [vp, P(C.c_int64), ip, ip, ip, ip, ip, ip, ip]
    L.msc_env_kernel_choice.argtypes = [vp, ip, C.c_int32]
    L.msc_env_set_option.argtypes = [vp, C.c_int32, C.c_int32]
    L.msc_env_reset.argtypes = [vp, vp, vp, C.c_int32, vp, vp]
    L.msc_env_step.argtypes = [vp, vp, vp, vp, vp, vp, vp, P(MscStepInfo), vp]
    L.msc_env_obs_flat.argtypes = [vp, vp, vp, vp]
    L.msc_env_generate_demand.argtypes = [vp, vp]
    L.msc_env_set_pipelining.argtypes = [vp, C.c_int32]
    L.msc_env_set_chain_priority.argtypes = [vp, C.c_int32]
    L.msc_env_set_timing.argtypes = [vp, C.c_int32]
    L.msc_env_read_timing.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_int64),
                                      C.POINTER(C.c_int64)]
    L.msc_env_read_timing_ea.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_int64), C.POINTER(C.c_int32),
                                         C.POINTER(C.c_int32), C.POINTER(C.c_double)]
    L.msc_env_work_counters.argtypes = [vp, C.POINTER(C.c_int64), C.POINTER(C.c_double), C.POINTER(C.c_int64),
                                        C.POINTER(C.c_int64)]
    L.msc_env_read_state.argtypes = [vp, vp, vp, vp, vp]
    L.msc_env_state_bytes.argtypes = [vp]
    L.msc_env_state_bytes.restype = C.c_int64
    L.msc_env_save_state.argtypes = [vp, vp]
    L.msc_env_load_state.argtypes = [vp, vp]
    L.msc_env_check.argtypes = [vp]
    L.msc_gae.argtypes = [vp, vp, vp, vp, vp, C.c_int64, C.c_int32, C.c_float, C.c_float, vp, vp, vp, vp]
    L.msc_adv_normalize.argtypes = [vp, C.c_int64, vp, vp]
    L.msc_gae_grouped.argtypes = [vp, vp, vp, vp, vp, C.c_int64, C.c_int32, C.c_float, C.c_float, vp, vp, C.c_int32,
                                  vp, vp]
    L.msc_adv_normalize_grouped.argtypes = [vp, C.c_int64, C.c_int32, vp, vp]
    L.msc_env_set_episode_counters.argtypes = [vp, vp]
    L.msc_gaussian_sample.argtypes = [vp, vp, C.c_int32, C.c_float, vp, C.c_int64, C.c_int32, vp, vp, vp, vp]
    L.msc_mlp3_w3_layout.argtypes = [C.c_int32]
    L.msc_mlp3_relu_forward.argtypes = [vp, C.c_int64, C.c_int32, C.c_int32, C.c_int32, C.c_int32, vp, vp, vp, vp, vp,
                                        vp, vp, vp, C.c_int32, vp]
    L.msc_mlp2_relu_forward.argtypes = [vp, C.c_int64, C.c_int32, C.c_int32, C.c_int32, vp, vp, vp, vp, vp, vp,
                                        C.c_int32, vp]
    L.msc_mlp3_relu_forward_sampled.argtypes = [vp, C.c_int64, C.c_int32, C.c_int32, C.c_int32, C.c_int32, vp, vp, vp,
                                                vp, vp, vp, vp, vp, C.c_int32, P(MscGaussianEpilogue), vp]
    L.msc_mlp2_relu_forward_sampled.argtypes = [vp, C.c_int64, C.c_int32, C.c_int32, C.c_int32, vp, vp, vp, vp, vp,
                                                vp, C.c_int32, P(MscGaussianEpilogue), vp]
    L.msc_meanstd_scratch_doubles.argtypes = [C.c_int64, C.c_int32]
    L.msc_meanstd_scratch_doubles.restype = C.c_int64
    L.msc_meanstd_filter.argtypes = [vp, vp, C.c_int64, C.c_int32, vp, C.c_int32, vp, vp, C.c_double, C.c_double, vp]
    L.msc_seedseq_u32.argtypes = [P(C.c_uint32), C.c_int32]
    L.msc_seedseq_u32.restype = C.c_uint32
    L.msc_last_error.restype = C.c_char_p
    L.msc_abi_version.restype = C.c_int
    if L.msc_abi_version() != ABI_VERSION:
        raise RuntimeError("libmarlsc ABI version mismatch")
    _LIB = L
    return L


def check(rc: int) -> None:
    if rc != 0:
        msg = lib().msc_last_error()
        raise RuntimeError(f"libmarlsc error {rc}: {msg.decode() if msg else '?'}")


EXPORTED_SYMBOLS = [
    "msc_env_create", "msc_env_destroy", "msc_env_dims", "msc_env_kernel_choice", "msc_env_set_option", "msc_env_ea_memory", "msc_env_reset", "msc_env_step", "msc_env_generate_demand", "msc_env_set_pipelining", "msc_env_set_chain_priority", "msc_env_set_episode_ahead", "msc_env_set_timing", "msc_env_read_timing", "msc_env_read_timing_ea", "msc_env_work_counters", "msc_env_obs_flat",
    "msc_env_read_state", "msc_env_state_bytes", "msc_env_save_state", "msc_env_load_state", "msc_env_check",
    "msc_env_set_episode_counters", "msc_gae", "msc_adv_normalize", "msc_gae_grouped", "msc_adv_normalize_grouped", "msc_gaussian_sample", "msc_mlp3_w3_layout", "msc_mlp3_relu_forward", "msc_mlp2_relu_forward",
    "msc_mlp3_relu_forward_sampled", "msc_mlp2_relu_forward_sampled",
    "msc_normal_keyed", "msc_poisson_draws", "msc_meanstd_scratch_doubles", "msc_meanstd_filter", "msc_seedseq_u32", "msc_last_error", "msc_abi_version",
]

#!/usr/bin/env python
"""Benchmark of the env hot path: `InventoryEnvironment.step()` of Jakoebly/marl-sc
(src/environment/envs/multi_env.py:253-366) on MI355X through libmarlsc.

A "step" = one pass of msc_env_step over every env of the rank (demand generation kernel +
fused step kernel, including in-kernel auto-resets every episode_length steps), with synthetic
uniform[-1, 1] actions already resident in HBM. Metric: agent-steps/s = envs x agents x steps / s,
whole job. N > 1: one process per GPU (torchrun), each rank owns `--envs` envs with disjoint global
env ids (weak scaling, no data-path collective: the headline), and the line's `strong` object times
BASELINE configs[3] as stated, 32,768 envs in total split over the ranks (`--scaling`); barrier +
synchronize bracket every timed region and the max over ranks is reported.

Roofline: average device duration of each kernel measured with HIP events on the launch stream
(torch's current stream); algorithmic bytes per launch from the state layout.
cpu_baseline: the C oracle (oracle/, a scalar port of the reference) timed on the host cores on a
bounded sample of the same workload, rank 0 at N = 1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "marl-sc_amd"))
sys.path.insert(0, str(REPO / "oracle"))

BASELINE = json.loads((REPO / "BASELINE.json").read_text())
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, chip-level parameters (spec)
# VALU issue peak (MI355X_MICROARCH.md:54): a wave64 VALU instruction issues over 2 cycles on its
# SIMD-32, so the chip issues 1024 SIMDs x clock / 2 wave-instructions per second: 1228.8 G/s at the
# 2400 MHz max clock (MI355X_MICROARCH.md:34). Objects that know the kernel's effective clock under
# load (rocprofv3 GRBM_GUI_ACTIVE pass, profiles/traffic.json) also quote the peak at that clock.
CLOCK_MAX_MHZ = 2400.0


def valu_peak(clk_mhz: float = CLOCK_MAX_MHZ) -> float:
    return 1024 * clk_mhz * 1e6 / 2


VALU_PEAK_WINST = valu_peak()
# secondary, measured (tools/ubench_isa.hip, profiles/r02/ubench_isa.txt): independent v_add_u32 at
# 4 waves per SIMD retired one wave64 instruction per 1.78 ns per SIMD = 574 G/s for the chip. The
# same run's shader-cycle counter (s_memtime) reads 8.70 cycles per instruction per wave at 4 waves,
# i.e. one issue per 2.17 cycles per SIMD: the 2-cycle basis above, at an effective ~1.2 GHz over that
# run's wall time (launch ramp and clock under an all-CU load included), so the two peaks differ by
# the clock, not by the cycles per instruction; f64 mul / 64-bit mad: 1.35-1.7x a v_add_u32
VALU_UBENCH_WINST = 1024 / 1.784e-9


def issue_object(insts: float, seconds: float, clk_mhz=None, **extra) -> dict:
    """VALU issue roofline: insts wave-instructions over `seconds` against the 2-cycle peak at the
    max clock (frac) and, when known, at the kernel's effective clock (frac_at_clock)."""
    ach = insts / seconds
    o = dict(extra)
    o.update({"bound": "valu issue", "achieved": round(ach / 1e9, 2), "peak": round(VALU_PEAK_WINST / 1e9, 1),
              "unit": "G wave-instructions/s", "frac": round(ach / VALU_PEAK_WINST, 4),
              "peak_basis": "1024 SIMDs x 2400 MHz / 2 cycles per wave64 VALU instruction (MI355X_MICROARCH.md:34,54)",
              "ubench_peak": round(VALU_UBENCH_WINST / 1e9, 1),
              "ubench_basis": "tools/ubench_isa.hip: 2.17 shader cycles per v_add_u32 issue per SIMD at 4 waves "
                              "(the 2-cycle basis), 1.78 ns wall per issue (~1.2 GHz effective over the run)"})
    if clk_mhz:
        pk = valu_peak(clk_mhz)
        o.update({"clock_mhz": clk_mhz, "peak_at_clock": round(pk / 1e9, 1), "frac_at_clock": round(ach / pk, 4)})
    return o
MFMA_F32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 matrix (v_mfma_f32_32x32x2_f32), dense
DEMAND_KERNEL = "demand_v3_kernel"  # the Poisson demand kernel of the headline handle (set in main)


def demand_kernel_name(env) -> str:
    """Base name of the demand kernel a handle runs (msc_env_kernel_choice's demand entry)."""
    impl = env.kernel_choice().get("demand_impl", 0)
    return {9: "demand_v3_kernel", 8: "demand_v2_kernel", 7: "demand_ab_kernel", 5: "demand_park4_kernel"}.get(
        impl, "demand_unit_kernel")


def is_demand_kernel(name: str) -> bool:
    return name.startswith("demand_") or name in ("reset_kernel", "ea_materialize_kernel")
STEP_KERNELS = ("step_a_kernel", "alloc_lane_kernel", "step_c_kernel")
GAE_BYTES_PER_ELEM = 4 + 4 + 1 + 1 + 4 + 4  # reward, value, terminated, truncated in; advantage, target out (next value: truncated rows only)


def ensure_built():
    lib = REPO / "marl-sc_amd" / "marlsc" / "_lib" / "libmarlsc.so"
    if not lib.exists():
        subprocess.run(["make", "-s", "-C", str(REPO / "marl-sc_amd"), "-j8"], check=True)


def algorithmic_bytes(spec, mean_orders: float):
    """Minimum HBM bytes one env moves per step (see DESIGN.md section 'Roofline')."""
    W, K, L = spec.W, spec.K, spec.local_obs_dim
    WK = W * K
    ring = max(int(spec.expected_lead_times.max()) + (int(spec.max_deviation.max()) if spec.lead_type == "stochastic" else 0) + 1, 2)
    nv = (1 + K + 7) // 8
    rec = 16 * nv
    demand = 40 + 40 + 40 + 4 + rec * mean_orders  # rng state in / out / pre-generation copy, count, records
    step = (2 * WK * 4            # inventory r/w
            + WK * ring * 4       # pending ring read
            + 2 * WK * 4          # new order + arrival clear
            + WK * 4 + 4 * WK * 4  # history: new entry + 4 older entries for the rolling mean
            + 2 * WK * 4          # incoming home demand r/w
            + 2 * WK * 4          # EMA forecast r/w
            + rec * mean_orders   # order records in
            + WK * 4              # actions
            + W * L * 4           # local observations
            + W * 4 + 1 + 8)      # rewards, truncation, timestep
    return demand, step


def _mlp_traffic(tj: Path, key: str):
    """HBM bytes per launch of the fused MLP from its rocprofv3 PMC passes (tools/bench_mlp.py), if recorded."""
    if not tj.exists():
        return None
    return json.loads(tj.read_text()).get("mlp3_relu_kernel", {}).get(key, {}).get("traffic")


def bench_obs_stats(cfg, meta, n_episodes: int = 2):
    """meanstd_custom statistics (obs_stats.py:11-90) from a short random-policy run on the GPU env
    (the reference uses 100 episodes; the values only set the normalisation constants, not the work)."""
    from marlsc.ppo import compute_obs_statistics
    from marlsc.seeding import SeedManager
    return compute_obs_statistics(cfg, SeedManager(42), "meanstd_custom", n_episodes=n_episodes, env_meta=meta)


def time_env(env, pool, steps: int, warmup: int, world: int, ea: bool = False):
    """warmup untimed steps, then `steps` timed ones (barrier + synchronize on both sides); then a
    timing pass of min(steps, 50) steps with the library's per-launch HIP events."""
    import torch
    import torch.distributed as dist
    for i in range(warmup):
        env.step(pool[i % len(pool)])
    env.check()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    w0 = env.work_counters()
    t0 = time.perf_counter()
    for i in range(steps):
        env.step(pool[i % len(pool)])
    t_host = time.perf_counter() - t0  # the host's enqueue time (the device may still be busy)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    w1 = env.work_counters()
    env.check()
    # the timing pass: 50 steps, or with episode-ahead demand 2.5 episodes (a generation launch covers
    # whole episodes of every env: one or two per episode in steady state)
    kp = min(steps, 50) if not ea else int(2.5 * env.spec.episode_length)
    kp = int(os.environ.get("MSC_BENCH_TIMING_STEPS", kp))
    env.set_timing(kp)
    for i in range(kp):
        env.step(pool[i % len(pool)])
    tm = env.read_timing()
    tm.update(env.read_timing_ea())
    env.set_timing(0)
    # host enqueue cost per step: bursts of 10 steps enqueued right after a synchronize (inside the
    # long timed loop the launch queue fills once the device falls behind, and enqueue then waits
    # for the device: t_host / steps is that back-pressured figure, kept as enqueue_ms_per_step)
    tb, nb = 0.0, 0
    for _ in range(20):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for i in range(10):
            env.step(pool[i % len(pool)])
        tb += time.perf_counter() - t1
        nb += 10
    torch.cuda.synchronize()
    tm["host_ms_per_step"] = tb / nb * 1e3
    tm["enqueue_ms_per_step"] = t_host / steps * 1e3
    tm["window"] = window_work(w0, w1, env.n_envs, steps)
    env.check()
    return dt, tm


def window_work(w0: dict, w1: dict, n_envs: int, steps: int) -> dict:
    """Demand work issued (and, after the window's closing synchronize, finished) inside a timed
    window, from the library's monotonic counters (msc_env_work_counters): episode-ahead generation
    launches and the env-steps of demand they drew, per-step demand launches (E env-steps each),
    against the env-steps the window timed. In steady state the generated env-steps cover the timed
    ones (the generation runs up to S episodes ahead, so a window can also hold demand its own steps
    do not read yet)."""
    ea_l = int(w1["ea_launches"] - w0["ea_launches"])
    ea_w = int(round(w1["ea_env_steps"] - w0["ea_env_steps"]))
    dl = int(w1["demand_launches"] - w0["demand_launches"])
    if ea_l == 0 and dl == 0:
        # empirical demand: the trace is resident in HBM and the step reads it directly (no generation)
        return {"ea_launches_in_window": 0, "demand_launches_in_window": 0,
                "env_steps_timed": int(n_envs) * int(steps), "steps_in_window": int(w1["steps"] - w0["steps"]),
                "ahead_change_steps": None, "demand": "trace resident in HBM, no generation work"}
    return {"ea_launches_in_window": ea_l, "ea_env_steps_in_window": ea_w, "demand_launches_in_window": dl,
            "demand_env_steps_in_window": ea_w + dl * n_envs, "env_steps_timed": int(n_envs) * int(steps),
            "steps_in_window": int(w1["steps"] - w0["steps"]),
            # steps of demand per env generated beyond (> 0) or drawn from the buffer built before the
            # window (< 0): a window is sustained when this is not far below zero
            "ahead_change_steps": round((ea_w + dl * n_envs - int(n_envs) * int(steps)) / max(1, n_envs), 1)}


def time_rollout(envs, module, T: int, world: int, seed: int, warm: int = 1, reps: int = 1, with_window: bool = False):
    """Seconds per rollout of T steps (RolloutCollector.collect) after `warm` untimed ones."""
    import torch
    import torch.distributed as dist
    from marlsc.rollout import RolloutCollector
    col = RolloutCollector(envs, module, T, seed=seed)
    el = envs if isinstance(envs, list) else [envs]
    for _ in range(warm):
        col.collect()  # warm-up (GEMM heuristics, allocator; episode-ahead demand reaches steady state)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    w0 = [x.work_counters() for x in el]
    t0 = time.perf_counter()
    for _ in range(reps):
        col.collect()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = (time.perf_counter() - t0) / reps
    ww = [window_work(a, x.work_counters(), x.n_envs, T * reps) for a, x in zip(w0, el)]
    for x in el:
        x.check()
    if with_window:
        return dt, merge_windows(ww, [x.n_envs for x in el])
    return dt


def merge_windows(ww: list, n_envs: list) -> dict:
    """One `window` object for env handles stepped together (rollout lanes): the integer counters
    summed, `ahead_change_steps` recomputed over all their envs; the trace form when no handle had
    generation work (empirical demand)."""
    if all(w.get("ahead_change_steps") is None for w in ww):
        out = dict(ww[0])
        for k in ("env_steps_timed",):
            out[k] = sum(int(w[k]) for w in ww)
        return out
    keys = ("ea_launches_in_window", "ea_env_steps_in_window", "demand_launches_in_window",
            "demand_env_steps_in_window", "env_steps_timed")
    out = {k: sum(int(w.get(k, 0)) for w in ww) for k in keys}
    out["steps_in_window"] = max(int(w["steps_in_window"]) for w in ww)
    out["ahead_change_steps"] = round((out["demand_env_steps_in_window"] - out["env_steps_timed"]) / max(1, sum(n_envs)), 1)
    return out


def c2_line(args, rank: int):
    """BASELINE configs[1]: 8 x 64 x 5, 4,096 envs on one GPU, IPPO rollout (the reference's
    config_files/algorithms/ippo.yaml: actor / critic [256], critic on local obs, meanstd_custom)."""
    import torch
    import yaml
    from marlsc import make_synthetic_env_config
    from marlsc.rollout import ActorCritic, RolloutConfig
    from marlsc.seeding import default_train_seed
    from marlsc.spec import EnvSpec
    from marlsc.vec_env import VecInventoryEnv
    algo = yaml.safe_load(open(REPO / "config_files/algorithms/ippo.yaml"))
    norm = algo["algorithm"]["algorithm_specific"]["obs_normalization"]
    cfg = make_synthetic_env_config(8, 64, 5)
    meta = {"include_warehouse_id": True, "obs_normalization": norm}
    meta["obs_stats"] = bench_obs_stats(cfg, meta)
    spec = EnvSpec.from_config(cfg, meta)
    E = args.c2_envs
    env = VecInventoryEnv(None, E, spec=spec, device=torch.cuda.current_device(), base_seed=default_train_seed(42))
    g = torch.Generator(device="cuda").manual_seed(99)
    pool = [torch.rand((E, spec.W, spec.K), generator=g, device="cuda") * 2 - 1 for _ in range(8)]
    env.reset()
    T = spec.episode_length
    # Episode-ahead demand refills 4 slots per launch, i.e. one generation launch per 4 episodes:
    # a timed window of 1,000 steps held 2 or 3 of them depending on its phase (0.214 / 0.246 ms per
    # step in consecutive windows, tools/ab_state.py), so the window is a whole number of refill
    # periods (24 episodes = 6 periods), after a warm-up of the same length: the snapshot's first 15
    # episodes are generated in two bulk launches that keep the generation stream busy for the first
    # ~20 episodes (a 12-episode window after 12 read 162 M where 48 episodes read 175.5 M,
    # profiles/r03/ab_ea_slots.txt)
    # round 5: 96 episodes after 96 (24 refill periods each): the 24-after-24 window of round 4 held
    # generation launches for only 75 % of the env-steps it timed, a 48-episode window 92 % (one refill
    # of 4 slots x 100 steps short: a refill in flight at the window's start was launched before it);
    # the line's `window` object reports what was generated inside the window, and `value_sustained`
    # scales `value` by min(1, generated / timed) as a lower bound
    period = 4 * T
    steps = max(args.c2_episodes * T, -(-args.steps // period) * period)
    warm = args.c2_episodes * T
    dt, tm = time_env(env, pool, steps, warm, 1, ea=True)
    rc = RolloutConfig.from_algorithm_config(algo)
    torch.manual_seed(0)
    module = ActorCritic(spec.local_obs_dim, spec.local_obs_dim * spec.W, spec.K, rc).cuda()
    # eight refill periods (32 episodes = 32 rollouts) timed after two: a generation launch of one
    # refill runs beside the next few rollouts, so a window of one or two periods read 0.21-0.29 ms per
    # step depending on its phase (profiles/r04/c2_rollout_phases.txt); 16 rollouts still held
    # generation for only 62 % of their env-steps (round 5), hence the longer window
    t_roll, roll_win = time_rollout(env, module, T, 1, seed=rank, warm=8, reps=32, with_window=True) if args.rollout_T > 0 else (0.0, None)
    a_h, c_h = rc.actor["hidden_sizes"], rc.critic["hidden_sizes"]
    out = {"workload": f"InventoryEnvironment.step x {E} envs/GPU, {spec.W} agents x {spec.R} regions x {spec.K} SKUs "
                       f"(BASELINE configs[1])",
           "value": round(E * spec.W * steps / dt, 1), "unit": "agent-steps/s", "ms_per_step": round(dt / steps * 1e3, 4),
           "steps": steps, "warmup": warm, "obs_normalization": norm,
           "host_ms_per_step": round(tm["host_ms_per_step"], 4), "enqueue_ms_per_step": round(tm["enqueue_ms_per_step"], 4),
           "demand": (f"episode-ahead: future episodes drawn on a side stream ({tm['slots']} slots per env, "
                      f"generated in 50-step chunks, several slots per launch)" if tm["slots"] else "per step (pipelined)"),
           "kernels_ms": {"step_kernels": round(tm["step_ms"], 4),
                          "demand_ea_chunk": round(tm["ea_ms"], 4) if tm["n_ea"] else None,
                          "demand_per_step": round(tm["demand_ms"], 4) if tm["n_demand"] else None},
           "window": tm["window"],
           "value_sustained": round(E * spec.W * steps / dt * min(1.0, tm["window"]["demand_env_steps_in_window"]
                                                                   / max(1, tm["window"]["env_steps_timed"])), 1)}
    # the step kernels against the VALU issue peak: PMC instruction counts of the same workload
    # (scripts/gpu_profile.sh -> profiles/traffic.json) over the live step-kernel time
    tj = Path(args.traffic_json)
    if tj.exists():
        tr = json.loads(tj.read_text())
        key = f"{spec.W}x{spec.R}x{spec.K}x{E}"
        cs = tr.get("counters", {}).get(key, {})
        names = tuple(n for n in cs if not is_demand_kernel(n)) or ("step_a_kernel", "alloc_scan_kernel", "step_c_kernel")
        cn = [cs.get(n, {}).get("SQ_INSTS_VALU") for n in names]
        tb = [tr.get(key, {}).get(n) for n in names]
        if all(x is not None for x in cn) and tm["step_ms"] > 0:
            out["roofline"] = issue_object(
                sum(cn), tm["step_ms"] * 1e-3, None, kernel="step_kernels (" + " + ".join(names) + ")",
                insts_per_step=int(sum(cn)), traffic=sum(tb) if all(x is not None for x in tb) else None,
                note="VALU wave-instructions of the step kernels (PMC) over their live time per step; the scan "
                     "allocation runs one env per wave (4 waves per SIMD at 4,096 envs) and is latency-bound on "
                     "its per-order DPP / permute chain, not issue-bound (DESIGN.md section 3)")
    if args.rollout_T > 0:
        out["rollout"] = {"value": round(E * spec.W * T / t_roll, 1), "unit": "agent-steps/s",
                          "ms_per_step": round(t_roll / T * 1e3, 4), "T": T,
                          "policy": f"IPPO (config_files/algorithms/ippo.yaml): actor {spec.local_obs_dim}-"
                                    f"{'-'.join(map(str, a_h))}-{spec.K}, critic {spec.local_obs_dim}-"
                                    f"{'-'.join(map(str, c_h))}-1 on local obs, fp32, parameter sharing",
                          "includes": "env step, actor + critic forward, Gaussian sampling, buffer writes, truncation "
                                      "bootstrap, GAE kernel, adv-norm statistics + normalise",
                          "window": roll_win,
                          "value_sustained": round(E * spec.W * T / t_roll * min(1.0, roll_win["demand_env_steps_in_window"]
                                                                                  / max(1, roll_win["env_steps_timed"])), 1)}
    env.close()
    return out


def c5_line(args, rank: int):
    """BASELINE configs[4]: 16 agents x 256 regions x 5 SKUs, 8,192 envs, empirical demand traces (a
    synthetic preprocessor frame of ~200-1,000 orders per step), excluded-region mapping shape; the
    env step, then its MAPPO rollout (the line's `rollout` object)."""
    import torch
    from marlsc import make_synthetic_env_config
    from marlsc.seeding import default_train_seed
    from marlsc.spec import EnvSpec
    from marlsc.synthetic import make_synthetic_trace
    from marlsc.vec_env import VecInventoryEnv
    cfg = make_synthetic_env_config(16, 256, 5)
    cfg["components"]["demand_sampler"] = {"type": "empirical", "params": None}
    meta = {"include_warehouse_id": True, "demand_trace": make_synthetic_trace(256, 5, 300, orders_per_step=(200, 1000), seed=0)}
    if args.obs_norm != "off":
        meta["obs_normalization"] = args.obs_norm
        meta["obs_stats"] = bench_obs_stats(cfg, dict(meta))
    spec = EnvSpec.from_config(cfg, meta)
    E = args.c5_envs
    env = VecInventoryEnv(None, E, spec=spec, device=torch.cuda.current_device(), base_seed=default_train_seed(42))
    g = torch.Generator(device="cuda").manual_seed(1234 + rank)
    pool = [torch.rand((E, spec.W, spec.K), generator=g, device="cuda") * 2 - 1 for _ in range(8)]
    env.reset()
    steps = max(100, args.steps)
    dt, tm = time_env(env, pool, steps, args.warmup, 1)
    # configs[4] names a MAPPO rollout: the reference's config_files/algorithms/mappo.yaml (actor on the
    # local obs, critic on local || global, mappo.yaml:31-32) over the same envs
    t_roll, roll_win, rc = 0.0, None, None
    if args.rollout_T > 0:
        import yaml
        from marlsc.rollout import ActorCritic, RolloutConfig
        rc = RolloutConfig.from_algorithm_config(yaml.safe_load(open(REPO / "config_files/algorithms/mappo.yaml")))
        torch.manual_seed(0)
        module = ActorCritic(spec.local_obs_dim, spec.local_obs_dim * spec.W, spec.K, rc).cuda()
        t_roll, roll_win = time_rollout(env, module, args.rollout_T, 1, seed=rank, warm=1, reps=2, with_window=True)
        del module
    env.close()
    mean_orders = float(spec.trace["offsets"][-1]) / spec.trace["n_rows"]
    out = {"workload": f"InventoryEnvironment.step x {E} envs/GPU, {spec.W} agents x {spec.R} regions x {spec.K} SKUs, "
                       f"empirical demand trace ({mean_orders:.0f} orders per step on average) (BASELINE configs[4])",
           "value": round(E * spec.W * steps / dt, 1), "unit": "agent-steps/s", "ms_per_step": round(dt / steps * 1e3, 4),
           "steps": steps, "warmup": args.warmup, "obs_normalization": meta.get("obs_normalization", "off"),
           "host_ms_per_step": round(tm["host_ms_per_step"], 4), "enqueue_ms_per_step": round(tm["enqueue_ms_per_step"], 4),
           "kernels_ms": {"step_kernels": round(tm["step_ms"], 4)}, "window": tm["window"]}
    if rc is not None:
        a_h, c_h = rc.actor["hidden_sizes"], rc.critic["hidden_sizes"]
        out["rollout"] = {"value": round(E * spec.W * args.rollout_T / t_roll, 1), "unit": "agent-steps/s",
                          "ms_per_step": round(t_roll / args.rollout_T * 1e3, 4), "T": args.rollout_T, "reps": 2,
                          "policy": f"MAPPO (config_files/algorithms/mappo.yaml): actor {spec.local_obs_dim}-"
                                    f"{'-'.join(map(str, a_h))}-{spec.K}, critic {spec.local_obs_dim * (1 + spec.W)}-"
                                    f"{'-'.join(map(str, c_h))}-1 on local || global, fp32, parameter sharing, "
                                    f"obs {meta.get('obs_normalization', 'off')}",
                          "includes": "env step, actor forward + Gaussian sampling, MAPPO critic (first layer split: "
                                      "global block once per env), buffer writes, truncation bootstrap, GAE kernel, "
                                      "adv-norm statistics + normalise",
                          "window": roll_win}
    # the step kernels (no demand kernel: the trace window is read inside step_a) against the VALU
    # issue peak and their HBM bytes, from the PMC passes of this workload (profiles/traffic.json)
    tj = Path(args.traffic_json)
    if tj.exists() and tm["step_ms"] > 0:
        tr = json.loads(tj.read_text())
        key = f"{spec.W}x{spec.R}x{spec.K}x{E}"
        cs = tr.get("counters", {}).get(key, {})
        names = tuple(n for n in cs if n not in ("reset_kernel",))
        cn = [cs[n].get("SQ_INSTS_VALU") for n in names]
        tb = [tr.get(key, {}).get(n) for n in names]
        if names and all(x is not None for x in cn):
            out["roofline"] = issue_object(
                sum(cn), tm["step_ms"] * 1e-3, None, kernel="step_kernels (" + " + ".join(names) + ")",
                insts_per_step=int(sum(cn)), traffic=sum(tb) if all(x is not None for x in tb) else None,
                note="one env per 16-lane group (4 envs per wave, 2 waves per SIMD at 8,192 envs): the per-order "
                     "chain's whole instruction stream (VALU + SALU, SQ_INSTS_SALU in the PMC summary) at one wave's "
                     "issue cadence bounds it, not the VALU peak; phase C runs inside step_b (DESIGN.md section 3)")
            salu = [cs[n].get("SQ_INSTS_SALU") for n in names]
            if all(x is not None for x in salu):
                out["roofline"]["salu_insts_per_step"] = int(sum(salu))
    return out


def ea_fraction_per_rank() -> float:
    """The episode-ahead memory budget of a rank's handle (marlsc.dist.ea_mem_fraction): ranks sharing
    one card split the library's default quarter of its free memory."""
    from marlsc.dist import ea_mem_fraction
    return ea_mem_fraction()


def strong_line(args, rank: int, world: int, spec, meta: dict) -> dict:
    """BASELINE configs[3] as stated: `--strong-envs` envs in total (32,768) sharded over the N ranks,
    rank g owning global env ids [g * E / N, (g + 1) * E / N) (every env seeded from
    its global id, so the trajectories are those of the one-GPU run). Per rank the library picks its
    kernels by shard size (per-step pipelined demand + lane allocator at >= 16,384 envs, episode-ahead
    demand + scan allocator at <= 8,192), as a one-GPU run of that size would. Barrier + synchronize
    bracket the window, max over ranks; then the MAPPO rollout over the same shards (the adv-norm
    statistics all-reduced across ranks each rollout)."""
    import torch
    import torch.distributed as dist
    from marlsc.seeding import default_train_seed
    from marlsc.vec_env import VecInventoryEnv
    from marlsc.dist import shard
    E_tot = args.strong_envs
    if E_tot % world:
        raise SystemExit(f"--strong-envs {E_tot} is not divisible by {world} ranks")
    n, off = shard(E_tot, "strong", rank, world)
    env = VecInventoryEnv(None, n, spec=spec, device=torch.cuda.current_device(), base_seed=default_train_seed(42),
                          env_index_offset=off, ea_mem_fraction=ea_fraction_per_rank())
    g = torch.Generator(device="cuda").manual_seed(4321 + rank)
    pool = [torch.rand((n, spec.W, spec.K), generator=g, device="cuda") * 2 - 1 for _ in range(8)]
    env.reset()
    T = spec.episode_length
    ea = bool(env.ea_slots)
    if ea:  # whole refill periods after the generation pipeline has filled (as the c2 line)
        period = 4 * T
        steps, warm = max(6 * period, -(-args.steps // period) * period), 6 * period
    else:
        steps, warm = args.steps, args.warmup
    dt, tm = time_env(env, pool, steps, warm, world, ea=ea)
    t_roll, roll_win = 0.0, None
    if args.rollout_T > 0:
        import yaml
        from marlsc.rollout import ActorCritic, RolloutConfig
        rc = RolloutConfig.from_algorithm_config(yaml.safe_load(open(REPO / "config_files/algorithms/mappo.yaml")))
        torch.manual_seed(0)
        module = ActorCritic(spec.local_obs_dim, spec.local_obs_dim * spec.W, spec.K, rc).cuda()
        env.set_pipelining(True)
        t_roll, roll_win = time_rollout(env, module, args.rollout_T, world, seed=0, warm=4 if ea else 1,
                                        reps=8 if ea else 2, with_window=True)
    tt = torch.tensor([dt, t_roll], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    dt, t_roll = (float(x) for x in tt.tolist())
    env.close()
    out = {"workload": f"InventoryEnvironment.step x {E_tot} envs in total ({n} per GPU x {world}), {spec.W} agents x "
                       f"{spec.R} regions x {spec.K} SKUs (BASELINE configs[3])",
           "scaling": "strong", "n_envs_total": E_tot, "n_envs_per_gpu": n, "n_gpus": world,
           "value": round(E_tot * spec.W * steps / dt, 1), "unit": "agent-steps/s",
           "ms_per_step": round(dt / steps * 1e3, 4), "steps": steps, "warmup": warm,
           "env_ids": f"rank g owns global env ids [g*{n}, (g+1)*{n})",
           "demand": "episode-ahead" if ea else "per step (pipelined)",
           "kernels_ms": {"step_kernels": round(tm["step_ms"], 4),
                          "demand_per_step": round(tm["demand_ms"], 4) if tm["n_demand"] else None,
                          "demand_ea_chunk": round(tm["ea_ms"], 4) if tm["n_ea"] else None},
           "window": tm["window"]}
    if args.rollout_T > 0:
        out["rollout"] = {"value": round(E_tot * spec.W * args.rollout_T / t_roll, 1), "unit": "agent-steps/s",
                          "ms_per_step": round(t_roll / args.rollout_T * 1e3, 4), "T": args.rollout_T,
                          "policy": "MAPPO (config_files/algorithms/mappo.yaml), adv-norm statistics all-reduced over ranks",
                          "window": roll_win}
    return out


def cpu_baseline(spec, seconds: float):
    """The C oracle on the host's cores (<= 16 threads), plus a 1-core figure."""
    out = _cpu_rate(spec, seconds, max(1, min(16, os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "16")))))
    one = _cpu_rate(spec, min(5.0, seconds / 3), 1)
    out["value_1core"] = one["value"]
    return out


def _cpu_rate(spec, seconds: float, threads: int):
    import numpy as np
    import oracle as orc
    E = 64 * threads
    env = orc.OracleEnv(spec, E, base_seed=4321)
    env.reset()
    rng = np.random.default_rng(0)
    acts = [rng.uniform(-1, 1, (E, spec.W, spec.K)).astype(np.float32) for _ in range(4)]
    env.step(acts[0], n_threads=threads)  # warm-up (page-in, thread pool)
    t0 = time.perf_counter()
    for i in range(3):
        env.step(acts[(i + 1) % 4], n_threads=threads)
    one = (time.perf_counter() - t0) / 3
    steps = int(max(3, min(20000, seconds / max(one, 1e-6))))
    t0 = time.perf_counter()
    for i in range(steps):
        env.step(acts[i % 4], n_threads=threads)
    dt = time.perf_counter() - t0
    return {"value": round(E * spec.W * steps / dt, 1), "unit": "agent-steps/s", "cores": threads, "kind": "port",
            "sample": f"oracle/msc_oracle.c (scalar C port of the reference step), {E} envs x {steps} steps of "
                      f"the same {spec.W}x{spec.R}x{spec.K} workload, OpenMP over envs, {dt:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--config", choices=("c3", "c5"), default="c3",
                    help="c3: BASELINE configs[2]/[3] (8 x 64 x 5, Poisson, 32768 envs, default); c5: configs[4] "
                         "(16 x 256 x 5, empirical trace of ~200-1,000 orders per step, 8192 envs)")
    ap.add_argument("--envs", type=int, default=None, help="envs per GPU (default: 32768 for c3, 8192 for c5)")
    ap.add_argument("--agents", type=int, default=8)
    ap.add_argument("--regions", type=int, default=64)
    ap.add_argument("--skus", type=int, default=5)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=str(REPO / "profiles" / "traffic.json"))
    ap.add_argument("--rollout-T", type=int, default=100,
                    help="steps of the MAPPO rollout line (0 = skip): env + actor/critic forward + buffers + GAE")
    ap.add_argument("--rollout-warm", type=int, default=1, help="untimed rollouts before the timed ones (MAPPO line)")
    ap.add_argument("--rollout-reps", type=int, default=1, help="timed rollouts of the MAPPO line")
    ap.add_argument("--c2-episodes", type=int, default=96, help="episodes of warm-up and of the timed window of the c2 line")
    ap.add_argument("--c2-envs", type=int, default=4096, help="envs of the configs[1] line (0 = skip it)")
    ap.add_argument("--c5-envs", type=int, default=8192, help="envs of the configs[4] line (0 = skip it)")
    ap.add_argument("--no-ea-line", dest="ea_line", action="store_false",
                    help="skip the episode-ahead steady-state line of the headline envs")
    ap.add_argument("--scaling", choices=("weak", "strong", "both"), default="both",
                    help="N > 1: weak = each rank steps --envs envs (global ids [g*E, (g+1)*E)); strong = BASELINE "
                         "configs[3], --strong-envs in total split over the ranks; both (default) = the weak headline "
                         "plus a `strong` object (at N = 1 the two coincide and only the headline runs)")
    ap.add_argument("--strong-envs", type=int, default=32768, help="total envs of the strong-scaling measurement")
    ap.add_argument("--obs-norm", choices=("meanstd_custom", "off"), default="meanstd_custom",
                    help="observation normalisation of the headline env (the reference MAPPO config's is meanstd_custom)")
    ap.add_argument("--rollout-lanes", type=int, default=int(os.environ.get("MSC_ROLLOUT_LANES", "1")),
                    help="env handles the rollout's envs are split into, each stepping on its own HIP stream so one "
                         "lane's env kernels overlap another's policy GEMMs (1 = one handle, one stream)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # one process per GPU over RCCL ("nccl" on ROCm); MSC_DIST_BACKEND=gloo rehearses the
        # multi-rank path with every rank on the visible GPU(s) (ranks share a card when fewer)
        backend = os.environ.get("MSC_DIST_BACKEND", "nccl")
        dev_i = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev_i)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_i))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    if rank == 0:
        ensure_built()
    if world > 1:
        dist.barrier()

    from marlsc import make_synthetic_env_config
    from marlsc.seeding import default_train_seed
    from marlsc.spec import EnvSpec
    from marlsc.vec_env import VecInventoryEnv

    meta = {"include_warehouse_id": True}
    if args.config == "c5":
        from marlsc.synthetic import make_synthetic_trace
        args.agents, args.regions, args.skus = 16, 256, 5
        cfg = make_synthetic_env_config(16, 256, 5)
        cfg["components"]["demand_sampler"] = {"type": "empirical", "params": None}
        meta["demand_trace"] = make_synthetic_trace(256, 5, 300, orders_per_step=(200, 1000), seed=0)
    else:
        cfg = make_synthetic_env_config(args.agents, args.regions, args.skus)
    if args.obs_norm != "off":
        meta["obs_normalization"] = args.obs_norm
        meta["obs_stats"] = bench_obs_stats(cfg, dict(meta))
    spec = EnvSpec.from_config(cfg, meta)
    E = args.envs if args.envs is not None else (8192 if args.config == "c5" else 32768)
    dev = torch.cuda.current_device()
    # episode-ahead buffers (the memory budget picks the slots: 4 at 32,768 envs) for the steady-state
    # line below; the headline steps with per-step pipelined demand (EA paused)
    want_ea = world == 1 and args.config == "c3" and args.ea_line
    from marlsc.dist import shard
    env = VecInventoryEnv(None, E, spec=spec, device=dev, base_seed=default_train_seed(42),
                          env_index_offset=shard(E, "weak", rank, world)[1], ea_mem_fraction=ea_fraction_per_rank(),
                          episode_ahead=16 if want_ea else None)
    if env.ea_slots and E > 8192:
        env.set_episode_ahead(False)
    global DEMAND_KERNEL
    DEMAND_KERNEL = demand_kernel_name(env)
    g = torch.Generator(device="cuda").manual_seed(1234 + rank)
    pool = [torch.rand((E, spec.W, spec.K), generator=g, device="cuda") * 2 - 1 for _ in range(8)]
    env.reset()

    K = args.steps
    # (1) the timed run: the production step path (demand of step t+1 pipelined on the library's
    #     side stream behind the step kernel of step t, see msc_env_step), then (2) per-launch device
    #     durations for the roofline in the same regime: the library brackets each demand launch and
    #     each step launch (step_a/b/c) with HIP events on the stream it runs on (msc_env_set_timing)
    dt, tm = time_env(env, pool, K, args.warmup, world)
    t_demand, t_step = tm["demand_ms"] / 1e3, tm["step_ms"] / 1e3
    # (1b) the same envs in episode-ahead steady state: whole future episodes of
    #      every env generated on the library's side stream while earlier ones step; a generation
    #      launch refills one slot per episode, so the window is whole episodes after the pipeline
    #      has filled (6 episodes of warm-up, 8 timed); every timed step's demand is generated inside
    #      the window in steady state
    ea_line = None
    if want_ea and env.ea_slots:
        T_ep = spec.episode_length
        env.set_episode_ahead(True)
        dt_ea, tm_ea = time_env(env, pool, 8 * T_ep, 6 * T_ep, 1, ea=True)
        env.set_episode_ahead(False)
        ea_line = {"value": round(E * spec.W * 8 * T_ep / dt_ea, 1), "unit": "agent-steps/s",
                   "ms_per_step": round(dt_ea / (8 * T_ep) * 1e3, 4), "steps": 8 * T_ep, "warmup": 6 * T_ep,
                   "slots": tm_ea["slots"], "host_ms_per_step": round(tm_ea["host_ms_per_step"], 4),
                   "enqueue_ms_per_step": round(tm_ea["enqueue_ms_per_step"], 4),
                   "kernels_ms": {"step_kernels": round(tm_ea["step_ms"], 4),
                                  DEMAND_KERNEL + "_ea": round(tm_ea["ea_ms"], 3),
                                  "ea_env_steps_per_launch": int(tm_ea["ea_env_steps_per_launch"])},
                   "window": tm_ea["window"],
                   "note": "episode-ahead demand in steady state (msc_env_set_episode_ahead): one generation launch "
                           "per episode refills a slot with a whole future episode of every env; the headline "
                           "`value` is the per-step pipelined path, whose first steps the driver's short "
                           "windows measure"}
    # episode-ahead demand (the library's default): the demand work of the timed
    # steps runs as generation launches of whole episodes on a side stream; per launch its duration
    # and the env-steps it generated
    ea_regime = tm["n_ea"] > 0 and tm["ea_env_steps_per_launch"] > 0
    t_ea = tm["ea_ms"] / 1e3 if ea_regime else 0.0
    ea_work = tm["ea_env_steps_per_launch"] if ea_regime else 0.0
    # (3) MAPPO rollout (configs[2]): env step + actor/critic forward + sampling + buffer writes +
    #     GAE kernel + adv-norm statistics all-reduce, T steps per rollout
    t_roll, roll_win = 0.0, None
    if args.rollout_T > 0:
        import yaml
        from marlsc.rollout import ActorCritic, RolloutCollector, RolloutConfig
        rc = RolloutConfig.from_algorithm_config(yaml.safe_load(open(REPO / "config_files/algorithms/mappo.yaml")))
        torch.manual_seed(0)
        module = ActorCritic(spec.local_obs_dim, spec.local_obs_dim * spec.W, spec.K, rc).cuda()
        nl = max(1, args.rollout_lanes)
        if nl == 1:
            renv = env
            env.set_pipelining(True)
        else:  # the rank's envs (same global ids) as nl handles of consecutive env-id ranges
            cuts = [E * j // nl for j in range(nl + 1)]
            renv = [VecInventoryEnv(None, cuts[j + 1] - cuts[j], spec=spec, device=dev, base_seed=default_train_seed(42),
                                    env_index_offset=rank * E + cuts[j]) for j in range(nl)]
            for x in renv:
                x.set_pipelining(os.environ.get("MSC_ROLLOUT_PIPELINE", "1") != "0")
                x.reset()
        t_roll, roll_win = time_rollout(renv, module, args.rollout_T, world, seed=0, warm=args.rollout_warm,
                                        reps=args.rollout_reps, with_window=True)
    # (4) the HBM-bound kernel of the rollout: msc_gae (GAE reverse scan + advantage statistics) over
    #     one MAPPO rollout's [T, E * W] sequences, timed alone with events on its stream
    gae_line = None
    if rank == 0 and args.rollout_T > 0:
        from marlsc.rollout import gae
        T, N = args.rollout_T, E * spec.W
        gg = torch.Generator(device="cuda").manual_seed(7)
        r_ = torch.randn((T, N), generator=gg, device="cuda")
        v_ = torch.randn((T + 1, N), generator=gg, device="cuda")
        nv_ = torch.randn((T, N), generator=gg, device="cuda")
        te_ = (torch.rand((T, N), generator=gg, device="cuda") < 0.01).to(torch.uint8)
        tr_ = torch.zeros((T, N), dtype=torch.uint8, device="cuda")
        tr_[T - 1] = 1
        adv_, tgt_ = torch.empty_like(r_), torch.empty_like(r_)
        st_ = torch.zeros((1, 3), dtype=torch.float64, device="cuda")
        for _ in range(3):
            gae(r_, v_, nv_, te_, tr_, 0.99, 0.95, adv_, tgt_, st_)
        reps = 20
        ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ea.record()
        for _ in range(reps):
            gae(r_, v_, nv_, te_, tr_, 0.99, 0.95, adv_, tgt_, st_)
        eb.record()
        torch.cuda.synchronize()
        t_gae = ea.elapsed_time(eb) / 1e3 / reps
        gb = GAE_BYTES_PER_ELEM * T * N
        gae_line = {"kernel": "gae4_kernel", "bound": "hbm", "achieved": round(gb / t_gae / 1e9, 1),
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gb / t_gae / 1e9 / HBM_PEAK_GBS, 4),
                    "bytes_per_launch": int(gb), "ms": round(t_gae * 1e3, 4),
                    "shape": f"T={T} x N={N} sequences (E x W of one MAPPO rollout), {GAE_BYTES_PER_ELEM} B/element"}
        del r_, v_, nv_, te_, tr_, adv_, tgt_
    # (5) the MFMA-bound kernel of the rollout: the fused actor MLP (msc_mlp3_relu_forward) over one
    #     step's E * W rows, timed alone with events on its stream
    mlp_line = None
    if rank == 0 and args.rollout_T > 0:
        from marlsc.mlp import fusable, mlp3_forward
        mods = list(module.actor)
        if fusable(mods):
            N = E * spec.W
            xg = torch.randn((N, spec.local_obs_dim), device="cuda", generator=torch.Generator(device="cuda").manual_seed(8))
            yo = torch.empty((N, spec.K), device="cuda")
            with torch.no_grad():
                for _ in range(3):
                    mlp3_forward(mods, xg, out=yo)
                reps = 20
                ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                ea.record()
                for _ in range(reps):
                    mlp3_forward(mods, xg, out=yo)
                eb.record()
                torch.cuda.synchronize()
            t_mlp = ea.elapsed_time(eb) / 1e3 / reps
            H1, H2 = mods[0].out_features, mods[2].out_features
            fl = 2.0 * N * (spec.local_obs_dim * H1 + H1 * H2 + H2 * spec.K)
            mlp_line = {"kernel": "mlp3_relu_kernel", "bound": "mfma", "achieved": round(fl / t_mlp / 1e12, 2),
                        "peak": MFMA_F32_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": round(fl / t_mlp / 1e12 / MFMA_F32_PEAK_TFLOPS, 4),
                        "flops_per_launch": int(fl), "ms": round(t_mlp * 1e3, 4),
                        "traffic": _mlp_traffic(Path(args.traffic_json), f"{spec.local_obs_dim}x{H1}x{H2}x{spec.K}x{N}"),
                        "shape": f"actor {spec.local_obs_dim}-{H1}-{H2}-{spec.K} over N={N} rows (E x W of one rollout step), "
                                 f"f32 MFMA, timed alone"}
            del xg, yo
    # (6) N > 1: BASELINE configs[3] as stated, the same 32,768 envs split over the ranks (strong)
    strong = None
    if world > 1 and args.scaling in ("strong", "both") and args.config == "c3":
        env.close()
        strong = strong_line(args, rank, world, spec, meta)
    c2 = None
    if world == 1 and args.c2_envs > 0 and args.config == "c3":
        env.close()
        c2 = c2_line(args, rank)
    c5 = None
    if world == 1 and args.c5_envs > 0 and args.config == "c3":
        c5 = c5_line(args, rank)
    tt = torch.tensor([dt, t_roll], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    dt, t_roll = (float(x) for x in tt.tolist())

    if rank == 0:
        value = E * world * spec.W * K / dt
        mean_orders = (float(spec.trace["offsets"][-1]) / spec.trace["n_rows"] if spec.demand_type == "empirical"
                       else float(spec.lambda_orders.sum()))
        b_dem, b_step = algorithmic_bytes(spec, mean_orders)
        # per launch: (duration, algorithmic bytes, duration per step of the workload) -- the dominant
        # kernel is the one with the most device time per step
        kern = {"step_kernels": (t_step, b_step * E, t_step)}
        if ea_regime:
            kern[DEMAND_KERNEL + "_ea"] = (t_ea, b_dem * ea_work, t_ea * E / ea_work)
        if t_demand > 0:
            kern[DEMAND_KERNEL] = (t_demand, b_dem * E, t_demand)
        dom = max(kern, key=lambda k: kern[k][2])
        t_dom, bytes_dom, _ = kern[dom]
        # per-launch HBM bytes / instruction counts of the same workload from the rocprofv3 PMC
        # passes (scripts/gpu_profile.sh -> profiles/traffic.json)
        traffic = valu = None
        tj = Path(args.traffic_json)
        key = f"{spec.W}x{spec.R}x{spec.K}x{E}"
        if tj.exists():
            tr = json.loads(tj.read_text())
            # the phase kernels this workload ran (allocation: lane / group (+ order sort) / scan)
            step_names = tuple(n for n in tr.get(key, {}) if not is_demand_kernel(n))
            names = (step_names or STEP_KERNELS) if dom == "step_kernels" else (dom,)
            tb = [tr.get(key, {}).get(n) for n in names]
            traffic = sum(tb) if all(x is not None for x in tb) else None
            cn = [tr.get("counters", {}).get(key, {}).get(n, {}).get("SQ_INSTS_VALU") for n in names]
            if all(x is not None for x in cn):
                # the kernel's effective clock under load (GRBM_GUI_ACTIVE / 8 / wall, PMC pass)
                clk = [tr.get("clock_mhz", {}).get(key, {}).get(n) for n in names]
                valu = issue_object(sum(cn), t_dom, clk[0] if len(names) == 1 else None,
                                    insts_per_launch=int(sum(cn)))
        # the whole pipelined step against the same issue peak: every kernel of a step (demand of
        # t + 1 and the step kernels of t run concurrently) over the measured time per step
        step_valu = None
        if tj.exists():
            cs = tr.get("counters", {}).get(key, {})
            # per step: the step kernels, plus the demand work of one step (the per-step kernel, or an
            # episode-ahead launch's instructions scaled by E / its env-steps)
            dname = DEMAND_KERNEL + "_ea" if ea_regime else DEMAND_KERNEL
            dscale = E / ea_work if ea_regime else 1.0
            names_all = ((dname,) if dname in cs else ()) + (step_names or STEP_KERNELS)
            vals = [cs.get(n, {}).get("SQ_INSTS_VALU") for n in names_all]
            if all(x is not None for x in vals):
                tot = sum(v * (dscale if n == dname else 1.0) for n, v in zip(names_all, vals))
                step_valu = issue_object(tot, dt / K, None, insts_per_step=int(tot), kernels=list(names_all))
        achieved = bytes_dom / t_dom / 1e9
        out = {
            "metric": BASELINE["metric"],
            "value": round(value, 1),
            "unit": "agent-steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(dt / K * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "window": tm["window"],
            "dtype": "int32 state, u64 PCG64, f64 rewards, f32 obs",
            "data": ("synthetic (SURVEY.md 8(d) cost structure, Poisson demand lambda_o=4 p=0.667 lambda_q=5, uniform[-1,1] actions)"
                     if args.config == "c3" else
                     f"synthetic (SURVEY.md 8(d) cost structure; empirical demand: a synthetic preprocessor frame of 300 timesteps, "
                     f"{mean_orders:.0f} orders per step on average over 256 regions; uniform[-1,1] actions)"),
            "config": {"workload": f"InventoryEnvironment.step x {E} envs/GPU, {spec.W} agents x {spec.R} regions x "
                                   f"{spec.K} SKUs " + ("(BASELINE configs[2]; configs[3] when N>1)" if args.config == "c3"
                                                        else "(BASELINE configs[4], empirical trace)"),
                       "n_envs_per_gpu": E, "agents": spec.W, "regions": spec.R, "skus": spec.K,
                       "episode_length": spec.episode_length, "obs_dim_local": spec.local_obs_dim,
                       "obs_normalization": meta.get("obs_normalization", "off"), "parallelism": f"env-shard x{world}"},
            "kernels_ms": {DEMAND_KERNEL: round(t_demand * 1e3, 4), "step_kernels": round(t_step * 1e3, 4),
                           **({DEMAND_KERNEL + "_ea": round(t_ea * 1e3, 3), "ea_env_steps_per_launch": int(ea_work),
                               "ea_slots": tm["slots"]} if ea_regime else {})},
            "host_ms_per_step": round(tm["host_ms_per_step"], 4),
            "enqueue_ms_per_step": round(tm["enqueue_ms_per_step"], 4),
            "roofline": {"kernel": dom, "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": traffic, "bytes_per_launch": int(bytes_dom),
                         **({"launch": f"episode-ahead generation of {int(ea_work)} env-steps (whole episodes of every env) "
                                       f"on the library's side stream, {t_ea * 1e3:.1f} ms"} if dom.endswith("_ea") else {}),
                         "note": "not HBM-bound: the env step is VALU-issue-bound (PCG64 draws + the per-env parse and allocation chains); see valu_issue (measured issue peak) and DESIGN.md section 3"},
        }
        if valu is not None:
            out["roofline"]["valu_issue"] = valu
        if step_valu is not None:
            out["roofline"]["step_valu_issue"] = step_valu
        if gae_line is not None:
            out["roofline_gae"] = gae_line
        if mlp_line is not None:
            out["roofline_mlp"] = mlp_line
        if args.rollout_T > 0:
            out["rollout"] = {
                "value": round(E * world * spec.W * args.rollout_T / t_roll, 1), "unit": "agent-steps/s",
                "ms_per_step": round(t_roll / args.rollout_T * 1e3, 4), "T": args.rollout_T,
                "policy": f"MAPPO (config_files/algorithms/mappo.yaml): actor {spec.local_obs_dim}-256-256-{spec.K} (fused f32-MFMA kernel), "
                          f"critic {spec.local_obs_dim * (1 + spec.W)}-64-64-1, fp32, parameter sharing, "
                          f"obs {meta.get('obs_normalization', 'off')}",
                "lanes": max(1, args.rollout_lanes),
                "includes": "env step (envs split into `lanes` handles on their own HIP streams), actor forward, MAPPO critic on local||global (first layer split: global block once per env), Gaussian sampling, "
                            "buffer writes, truncation bootstrap, GAE kernel, adv-norm all-reduce + normalise",
                "window": roll_win}
        if ea_line is not None:
            b_dem_ea = algorithmic_bytes(spec, mean_orders)[0]
            w_ea = ea_line["kernels_ms"]["ea_env_steps_per_launch"]
            t_l = ea_line["kernels_ms"][DEMAND_KERNEL + "_ea"] / 1e3
            if w_ea > 0 and t_l > 0:
                ach = b_dem_ea * w_ea / t_l / 1e9
                ea_line["roofline"] = {"kernel": DEMAND_KERNEL + "_ea", "bound": "hbm", "achieved": round(ach, 2),
                                       "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 5),
                                       "bytes_per_launch": int(b_dem_ea * w_ea),
                                       "traffic": (json.loads(Path(args.traffic_json).read_text()).get(key, {})
                                                   .get(DEMAND_KERNEL + "_ea") if Path(args.traffic_json).exists() else None)}
                if Path(args.traffic_json).exists():
                    ci = json.loads(Path(args.traffic_json).read_text()).get("counters", {}).get(key, {}).get(
                        DEMAND_KERNEL + "_ea", {}).get("SQ_INSTS_VALU")
                    if ci:
                        ea_line["roofline"]["valu_issue"] = issue_object(ci, t_l, None, insts_per_launch=int(ci))
            out["episode_ahead"] = ea_line
        if strong is not None:
            out["strong"] = strong
            if args.scaling == "strong":  # the headline is configs[3] as stated
                out["weak"] = {"value": out["value"], "ms_per_step": out["ms_per_step"], "n_envs_per_gpu": E}
                out.update({"value": strong["value"], "ms_per_step": strong["ms_per_step"], "steps": strong["steps"],
                            "warmup": strong["warmup"], "scaling": "strong"})
                out["config"]["n_envs_per_gpu"] = strong["n_envs_per_gpu"]
                out["config"]["workload"] = strong["workload"]
        if c2 is not None:
            out["c2"] = c2
        if c5 is not None:
            out["c5"] = c5
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(spec, args.cpu_seconds)
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

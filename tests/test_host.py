"""CPU tests of the host side: the C ABI's exported surface, the 128-bit LCG algebra of rng.hpp,
the folded Bernoulli threshold, config / seeding / trace host logic, and the world_size-2
advantage-statistics all-reduce (gloo). No GPU calls."""
import ctypes as C
import os
import re
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parents[1]
HEADER = REPO / "include" / "marlsc.h"


def header_functions():
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    return sorted(set(re.findall(r"\b(msc_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_documented_entry_points():
    fns = header_functions()
    for must in ("msc_env_create", "msc_env_reset", "msc_env_step", "msc_env_obs_flat", "msc_gae",
                 "msc_adv_normalize", "msc_last_error", "msc_env_destroy"):
        assert must in fns


def test_library_loads_and_exports_every_header_symbol():
    from marlsc import abi
    L = abi.lib()  # dlopen only: no HIP call is made
    missing = [f for f in header_functions() if not hasattr(L, f)]
    assert not missing, missing
    assert sorted(abi.EXPORTED_SYMBOLS) == header_functions()
    m = re.search(r"#define\s+MSC_ABI_VERSION\s+(\d+)", HEADER.read_text())
    assert L.msc_abi_version() == int(m.group(1))


def test_seedseq_utility_matches_numpy():
    from marlsc import abi
    L = abi.lib()
    for words in ([42], [123456789, 7], [987654321, 0, 5], [1, 2, 3, 4, 5]):
        arr = (C.c_uint32 * len(words))(*words)
        got = L.msc_seedseq_u32(arr, len(words))
        want = int(np.random.SeedSequence(words).generate_state(1, dtype=np.uint32)[0])
        assert got == want


RNG_TEST = r"""
#include <initializer_list>
#include <cstdio>
#include "rng.hpp"
using namespace msc;
int main() {
  for (uint32_t root : {1u, 12345u, 4000000000u}) {
    Pcg64 a; pcg_seed_child(a, root, 2);
    for (uint64_t n : {0ull, 1ull, 2ull, 3ull, 63ull, 64ull, 1000ull, 8191ull}) {
      Pcg64 b = a, c = a;
      for (uint64_t i = 0; i < n; i++) pcg_step(b);
      pcg_advance(c, n);
      if (b.s_hi != c.s_hi || b.s_lo != c.s_lo) { printf("advance %llu\n", (unsigned long long)n); return 1; }
    }
    // G-step affine map used by the interleaved generator waves
    for (int G : {1, 2, 3}) {
      uint64_t mh, ml, ch, cl;
      pcg_jump_coeffs(G, a.i_hi, a.i_lo, mh, ml, ch, cl);
      Pcg64 b = a; uint64_t th = a.s_hi, tl = a.s_lo;
      for (int k = 0; k < 20; k++) {
        for (int j = 0; j < G; j++) pcg_step(b);
        uint64_t nh, nl; mul128(th, tl, mh, ml, nh, nl); add128(nh, nl, ch, cl);
        uint64_t qh = th, ql = tl; lcg128(qh, ql, mh, ml, ch, cl);  // the generators' form
        th = nh; tl = nl;
        if (th != b.s_hi || tl != b.s_lo || qh != th || ql != tl) { printf("jump G=%d\n", G); return 1; }
        // the generators' double: bit-identical to numpy's random() of the same output
        const double u1 = u64_to_double(pcg_output(th, tl)), u2 = pcg_output_double(th, tl);
        if (u1 != u2) { printf("double %d\n", k); return 1; }
      }
    }
  }
  puts("ok");
  return 0;
}
"""


def test_rng_jump_ahead_algebra(tmp_path):
    src = tmp_path / "t.cpp"
    src.write_text(RNG_TEST)
    exe = tmp_path / "t"
    subprocess.run(["g++", "-O1", "-std=c++17", "-I", str(REPO / "marl-sc_amd" / "csrc"), str(src), "-o", str(exe)],
                   check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stdout


def p_skip(p):
    # capi.hip: ldexp(ceil(ldexp(p, 53)), -53) - 2^-53
    return np.ldexp(np.ceil(np.ldexp(p, 53)), -53) - 2.0 ** -53


@pytest.mark.parametrize("p", [0.667, 0.1, 0.5, 1.0, 1e-9, 0.3333333333333333, 0.9999999999999999, 2.0 ** -53])
def test_folded_bernoulli_threshold(p):
    # random() returns k * 2^-53; the kernels test `U > p_skip` for "SKU not drawn" (U >= p)
    k0 = int(np.floor(p * 2.0 ** 53))
    ks = np.arange(max(0, k0 - 3), min(2 ** 53, k0 + 4), dtype=np.int64)
    U = ks.astype(np.float64) * 2.0 ** -53
    assert np.array_equal(U < p, ~(U > p_skip(p)))


def test_synthetic_config_and_spec():
    from marlsc import EnvSpec, make_synthetic_env_config, validate_environment_config
    cfg = make_synthetic_env_config(8, 64, 5)
    validate_environment_config(cfg, allow_nr_ne_nw=True)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    assert (spec.W, spec.R, spec.K) == (8, 64, 5)
    assert spec.local_obs_dim == 34  # L = (ns+1) + 3 ns + ns + nw at C3
    assert spec.local_obs_dim * (1 + spec.W) == 306


def test_config_validation_rejects_bad_values():
    from marlsc import make_synthetic_env_config, validate_environment_config
    cfg = make_synthetic_env_config(2, 4, 2)
    bad = dict(cfg)
    bad["n_warehouses"] = 0
    with pytest.raises(Exception):
        validate_environment_config(bad, allow_nr_ne_nw=True)


def test_shape_caps_agree_across_header_abi_spec():
    # include/marlsc.h caps (32 warehouses x 16 SKUs x 4,096 regions) = the Python mirror's = what the
    # spec accepts; one past them is rejected before any device call
    import re
    from marlsc import EnvSpec, abi, make_synthetic_env_config
    hdr = (REPO / "include" / "marlsc.h").read_text()
    caps = {k: int(re.search(rf"#define MSC_MAX_{k} (\d+)", hdr).group(1)) for k in ("W", "K", "R")}
    assert (caps["W"], caps["K"], caps["R"]) == (abi.MAX_W, abi.MAX_K, abi.MAX_R) == (32, 16, 4096)
    spec = EnvSpec.from_config(make_synthetic_env_config(32, 6, 16), {"include_warehouse_id": True})
    assert (spec.W, spec.K) == (32, 16)
    for W, K in ((33, 4), (4, 17)):
        with pytest.raises(ValueError):
            EnvSpec.from_config(make_synthetic_env_config(W, 6, K), {"include_warehouse_id": True})
    # per-step order capacity (int32 record indexing, capi.hip): the header's cap = the mirror's, and a
    # configuration past it (rates just under the 1e6 bound in 4,096 regions) is rejected by the spec
    assert int(eval(re.search(r"#define MSC_ORDER_CAP_MAX \(([^)]*)\)", hdr).group(1))) == abi.ORDER_CAP_MAX
    EnvSpec.from_config(make_synthetic_env_config(2, 4096, 1, lambda_orders=4000.0), {"include_warehouse_id": True})
    with pytest.raises(ValueError, match="order capacity"):
        EnvSpec.from_config(make_synthetic_env_config(2, 4096, 1, lambda_orders=9.9e5), {"include_warehouse_id": True})


def test_seed_manager_semantics():
    from marlsc import SeedManager
    sm = SeedManager(42)
    t = sm.get_seed_int("train")
    assert t == int(np.random.SeedSequence(42).spawn(6)[3].generate_state(1, dtype=np.uint32)[0])
    e = SeedManager.derive_env_seed(t, 0, 5)
    assert e == int(np.random.SeedSequence([t, 0, 5]).generate_state(1, dtype=np.uint32)[0])
    env_sm = SeedManager(e, seed_registry=("preprocessing", "inventory", "demand_sampler", "lead_time_sampler"))
    env_sm.advance_episode()
    assert env_sm.root_seed == int(np.random.SeedSequence([e, 0]).generate_state(1, dtype=np.uint32)[0])
    env_sm.advance_episode()
    assert env_sm.root_seed == int(np.random.SeedSequence([e, 1]).generate_state(1, dtype=np.uint32)[0])


def test_env_shards_have_disjoint_global_ids():
    from marlsc.dist import env_index_offset
    ids = [set(range(env_index_offset(1024, r), env_index_offset(1024, r) + 1024)) for r in range(8)]
    assert sum(len(s) for s in ids) == len(set().union(*ids)) == 8192


def _adv_worker(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, str(REPO / "marl-sc_amd"))
    from marlsc.dist import allreduce_adv_stats, mean_std
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    full = torch.from_numpy(np.random.default_rng(0).normal(3.0, 2.0, 10_000))
    part = full.chunk(world)[rank]
    st = torch.tensor([part.sum().item(), (part * part).sum().item(), float(part.numel())], dtype=torch.float64)
    allreduce_adv_stats(st)
    m, s = mean_std(st)
    normed = (part - m) / max(1e-4, s)
    np.save(Path(out_dir) / f"r{rank}.npy", normed.numpy())
    dist.destroy_process_group()


def test_adv_norm_allreduce_world2_gloo(tmp_path):
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    mp.spawn(_adv_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    got = np.concatenate([np.load(tmp_path / "r0.npy"), np.load(tmp_path / "r1.npy")])
    full = np.random.default_rng(0).normal(3.0, 2.0, 10_000)
    want = (full - full.mean()) / max(1e-4, full.std())
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-12)


def test_trace_packer_matches_pandas_groupby():
    # EmpiricalDemandSampler.sample (demand_sampler.py:214-261): rows of one timestep grouped by
    # (region_id, order_id) -- pandas sorts the group keys -- quantities summed per SKU
    import pandas as pd
    from marlsc.trace import pack_demand_trace
    rng = np.random.default_rng(3)
    n = 3000
    df = pd.DataFrame({
        "timestep": rng.integers(0, 40, n),
        "region_id": rng.integers(0, 16, n),
        "order_id": [f"o{v}" for v in rng.integers(0, 400, n)],
        "sku_id": rng.integers(0, 6, n),  # sku 5 is outside K=5 and must be dropped
        "quantity": rng.integers(1, 9, n),
    })
    K = 5
    tr = pack_demand_trace(df, K)
    assert tr["n_rows"] == df["timestep"].nunique()
    for i, t in enumerate(tr["timesteps"]):
        sub = df[df["timestep"] == t]
        want = []
        for (reg, _), g in sub.groupby(["region_id", "order_id"]):
            q = np.zeros(K, np.int64)
            for s, v in zip(g["sku_id"], g["quantity"]):
                if 0 <= s < K:
                    q[s] += v
            want.append((reg, q))
        lo, hi = tr["offsets"][i], tr["offsets"][i + 1]
        assert hi - lo == len(want)
        for j, (reg, q) in enumerate(want):
            assert tr["regions"][lo + j] == reg
            assert np.array_equal(tr["quantities"][lo + j], q)


@pytest.mark.parametrize("name,dims", [("env_c1_2wh4r2sku", (2, 4, 2, 13)), ("env_c3_8wh64r5sku", (8, 64, 5, 34)),
                                       ("env_c5_16wh256r5sku", (16, 256, 5, 42))])
def test_repo_config_files_load(name, dims):
    from marlsc import EnvSpec, load_environment_config
    cfg = load_environment_config(str(REPO / "config_files" / "environments" / f"{name}.yaml"), allow_nr_ne_nw=True)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True}, allow_nr_ne_nw=True)
    assert (spec.W, spec.R, spec.K, spec.local_obs_dim) == dims


def test_map_excluded_regions():
    # DataProcessor.map_excluded_regions (preprocessor.py:382-441): an excluded region goes to the
    # selected region that shares its warehouses with the lowest mean fixed cost (ties: smallest
    # id), else to selected_region_ids[0]
    from marlsc.trace import map_excluded_regions
    w2r = {"sourcenodeid": ["W1", "W1", "W1", "W2", "W2", "W3", "W3"],
           "destinationregionid": ["R9", "R1", "R2", "R9", "R2", "R7", "R3"],
           "fixed_costs": [5.0, 4.0, 3.0, 1.0, 5.0, 2.0, 1.0]}
    sel = ["R1", "R2", "R3"]
    orders = np.array(["R1", "R9", "R2", "R8", "R9", "R7", "R3"], dtype=object)
    got = map_excluded_regions(orders, sel, w2r)
    # R9: warehouses {W1, W2}; selected pairs R1 (4), R2 (3, 5 -> mean 4) -> tie at 4 -> R1
    # R8: no pairs -> R1; R7: warehouse W3 -> selected pair R3 (1) -> R3
    assert got.tolist() == ["R1", "R1", "R2", "R1", "R1", "R3", "R3"]


def test_synthetic_trace_packs_like_the_preprocessor_frame():
    from marlsc.synthetic import make_synthetic_trace
    from marlsc.trace import pack_demand_trace
    tr = make_synthetic_trace(32, 5, 20, orders_per_step=(10, 40), seed=2)
    n_orders = len(np.unique(tr["order_id"]))
    p = pack_demand_trace(tr, 5)
    assert p["n_rows"] == 20 and p["offsets"][-1] == n_orders
    assert int(p["quantities"].sum()) == int(tr["quantity"].sum())  # every line has a SKU in [0, 5)
    assert np.all(np.diff(p["regions"][p["offsets"][3]:p["offsets"][4]]) >= 0)  # region-major within a step


def test_mean_std_per_module_rows():
    import torch
    sys.path.insert(0, str(REPO / "marl-sc_amd"))
    from marlsc.dist import mean_std
    rng = np.random.default_rng(1)
    xs = [rng.normal(g, g + 1, 1000) for g in range(3)]
    st = torch.tensor([[x.sum(), (x * x).sum(), x.size] for x in xs], dtype=torch.float64)
    m, s = mean_std(st)
    np.testing.assert_allclose(m, [x.mean() for x in xs], rtol=1e-12)
    np.testing.assert_allclose(s, [x.std() for x in xs], rtol=1e-9)
    m0, s0 = mean_std(st[1])
    assert abs(m0 - xs[1].mean()) < 1e-12 and abs(s0 - xs[1].std()) < 1e-9


def _learner_batch(S, W, L, K, seed):
    import torch
    g = torch.Generator().manual_seed(seed)
    return {"obs": torch.randn(S, W, L, generator=g), "actions": torch.randn(S, W, K, generator=g).clamp(-1, 1),
            "logp": -torch.rand(S, W, generator=g) * 5, "advantages": torch.randn(S, W, generator=g),
            "value_targets": torch.randn(S, W, generator=g),
            "mean_old": torch.randn(S, W, K, generator=g) * 0.1, "log_std_old": torch.full((S, W, K), -1.4)}


def _learner_cfg():
    sys.path.insert(0, str(REPO / "marl-sc_amd"))
    import yaml
    from marlsc.ppo import PPOConfig
    raw = yaml.safe_load(open(REPO / "config_files/algorithms/mappo.yaml"))
    # one epoch, one minibatch = the whole (rank-local) batch: the update is then a function of the
    # mean loss over every row, so the split over ranks must not change it
    raw["algorithm"]["shared"].update(batch_size=64 * 3, num_epochs=1, num_minibatches=1)
    return PPOConfig.from_algorithm_config(raw)


def _learner_module(cfg, W, L, K):
    import torch
    from marlsc.ppo import MultiAgentActorCritic
    torch.manual_seed(5)
    return MultiAgentActorCritic(W, L, L * W, K, cfg.rollout_config(), cfg.parameter_sharing)


def _learner_worker(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from marlsc.ppo import PPOLearner, minibatch_rows
    cfg = _learner_cfg()
    W, L, K = 3, 7, 2
    module = _learner_module(cfg, W, L, K)
    batch = _learner_batch(64, W, L, K, seed=11)
    mine = {k: v.chunk(world)[rank].contiguous() for k, v in batch.items()}  # this rank's envs
    lr = PPOLearner(module, cfg, seed=rank)
    assert lr.world == world and minibatch_rows(cfg, world) == 64 * 3 // world
    stats = lr.update(mine)
    assert stats["num_minibatch_steps"] == 1
    torch.save(torch.tensor(lr.kl_coeffs, dtype=torch.float64), Path(out_dir) / f"kl{rank}.pt")
    torch.save({k: v.detach() for k, v in module.state_dict().items()}, Path(out_dir) / f"p{rank}.pt")
    dist.destroy_process_group()


def test_learner_update_world2_gloo_equals_single_rank(tmp_path):
    # 2 ranks x half the batch (gradients all-reduced, minibatch rows split by minibatch_rows(cfg,
    # world)) against 1 rank x the whole batch: the same parameters after one PPOLearner.update
    import socket
    import torch
    import torch.multiprocessing as mp
    sys.path.insert(0, str(REPO / "marl-sc_amd"))
    from marlsc.ppo import PPOLearner
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    mp.spawn(_learner_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    cfg = _learner_cfg()
    W, L, K = 3, 7, 2
    module = _learner_module(cfg, W, L, K)
    p_init = {k: v.detach().clone() for k, v in module.state_dict().items()}
    single = PPOLearner(module, cfg, seed=0)
    single.update(_learner_batch(64, W, L, K, seed=11))
    ref = module.state_dict()
    for r in range(2):  # the adaptive KL coefficient follows the all-reduced mean KL
        np.testing.assert_allclose(torch.load(tmp_path / f"kl{r}.pt").numpy(), single.kl_coeffs, rtol=1e-12)
    p0 = torch.load(tmp_path / "p0.pt", weights_only=True)
    p1 = torch.load(tmp_path / "p1.pt", weights_only=True)
    moved = 0
    for k in ref:
        torch.testing.assert_close(p0[k], p1[k], rtol=0, atol=0)  # ranks stay identical
        torch.testing.assert_close(p0[k], ref[k], rtol=1e-5, atol=2e-6)
        moved += int(not torch.equal(ref[k], p_init[k]))
    assert moved > 0


def test_checkpoint_bookkeeping_of_the_reference_runner(tmp_path):
    # experiment_utils.py:256-467: checkpoint_<N> names, training_metrics.yaml truncated to N on
    # resume with the best train return re-derived from the surviving entries
    sys.path.insert(0, str(REPO / "marl-sc_amd"))
    from marlsc.experiment import load_and_truncate_training_metrics, parse_checkpoint_iteration, save_training_metrics
    assert parse_checkpoint_iteration(tmp_path / "checkpoint_12") == 12
    assert parse_checkpoint_iteration("runs/x/checkpoint_best") is None
    assert parse_checkpoint_iteration("checkpoint_final") is None
    assert parse_checkpoint_iteration("checkpoint_000003") == 3
    m = [{"iteration": i, "train_return": r, "eval_return": None} for i, r in ((1, -5.0), (2, -3.0), (3, None), (4, -1.0))]
    save_training_metrics(tmp_path, m)
    kept, best, best_it = load_and_truncate_training_metrics(tmp_path, 3)
    assert [x["iteration"] for x in kept] == [1, 2, 3] and best == -3.0 and best_it == 2
    kept, best, best_it = load_and_truncate_training_metrics(tmp_path / "nowhere", 3)
    assert kept == [] and best == float("-inf") and best_it is None


@pytest.mark.parametrize("seed", range(6))
def test_map_excluded_regions_vs_pandas(seed):
    # marlsc.trace.map_excluded_regions against oracle/preproc_ref.py, which runs the reference's
    # own pandas operations (preprocessor.py:382-441: groupby mean = Kahan-compensated sums, idxmin
    # = first minimum in sorted key order). Costs are drawn from decimals whose group means tie or
    # differ by an ulp between a plain sum / len and pandas' compensated sum.
    import pandas as pd
    from preproc_ref import map_excluded_regions_pd
    from marlsc.trace import map_excluded_regions
    rng = np.random.default_rng(seed)
    regions = [f"R{i}" for i in range(40)] if seed % 2 else list(range(100, 140))
    sel = list(rng.choice(np.array(regions, dtype=object), 15, replace=False))
    whs = [f"W{i}" for i in range(8)]
    n = 300
    vals = np.array([0.1, 0.2, 0.3, 0.7, 1.1, 1e16, -1e16, 3.0, 0.30000000000000004])
    w2r = pd.DataFrame({"sourcenodeid": rng.choice(whs, n),
                        "destinationregionid": [regions[i] for i in rng.integers(0, 40, n)],
                        "fixed_costs": rng.choice(vals[:5] if seed < 3 else vals, n)})
    w2r = w2r[~w2r["destinationregionid"].isin(regions[35:])]  # some excluded regions have no pairs
    orders = np.array([regions[i] for i in rng.integers(0, 40, 2000)], dtype=object)
    got = map_excluded_regions(orders, sel, {c: w2r[c].tolist() for c in w2r.columns})
    want = map_excluded_regions_pd(orders, sel, w2r.reset_index(drop=True))
    assert got.tolist() == want.tolist()


def test_group_mean_is_pandas_groupby_mean():
    import pandas as pd
    from marlsc.trace import _group_mean
    rng = np.random.default_rng(7)
    for _ in range(200):
        v = rng.choice([0.1, 0.2, 0.3, 0.7, 1e16, -1e16, 2.5e-3, np.nan], rng.integers(1, 30))
        want = pd.DataFrame({"k": 0, "v": v}).groupby("k")["v"].mean().iloc[0]
        got = _group_mean(v.tolist())
        assert (got == want) or (got != got and want != want), (v, got, want)


def test_bench_window_accounting():
    """bench.window_work: per-step demand, episode-ahead refills and a resident trace (no generation)."""
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import bench

    z = {"ea_launches": 0, "ea_env_steps": 0, "demand_launches": 0, "steps": 0}
    per_step = bench.window_work(z, dict(z, demand_launches=10, steps=10), 64, 10)
    assert per_step["demand_env_steps_in_window"] == 640 and per_step["ahead_change_steps"] == 0.0
    ahead = bench.window_work(z, dict(z, ea_launches=2, ea_env_steps=64 * 100, steps=50), 64, 50)
    assert ahead["ahead_change_steps"] == 50.0
    drained = bench.window_work(z, dict(z, steps=50, ea_launches=1, ea_env_steps=64 * 20), 64, 50)
    assert drained["ahead_change_steps"] == -30.0
    trace = bench.window_work(z, dict(z, steps=7), 64, 7)
    assert trace["ahead_change_steps"] is None and trace["env_steps_timed"] == 448
    # rollout lanes: the windows of several handles merged (the trace form, whose
    # 'demand' is a string, and per-env averages that must not be added up)
    merged_trace = bench.merge_windows([trace, trace], [64, 64])
    assert merged_trace["ahead_change_steps"] is None and merged_trace["env_steps_timed"] == 896
    a = bench.window_work(z, dict(z, ea_launches=2, ea_env_steps=64 * 100, steps=50), 64, 50)  # +50 per env
    b = bench.window_work(z, dict(z, ea_launches=1, ea_env_steps=32 * 20, steps=50), 32, 50)   # -30 per env
    m = bench.merge_windows([a, b], [64, 32])
    assert m["ea_launches_in_window"] == 3 and m["env_steps_timed"] == 96 * 50
    assert m["ahead_change_steps"] == round((64 * 100 + 32 * 20 - 96 * 50) / 96, 1)


def test_dist_shard_partitions(monkeypatch):
    """marlsc.dist.shard: weak and strong env-id partitions (bench.py, BASELINE configs[2] / [3]); the
    episode-ahead budget split between ranks that share one card."""
    from marlsc import dist
    assert [dist.shard(32768, "strong", g, 4) for g in range(4)] == [(8192, g * 8192) for g in range(4)]
    assert [dist.shard(32768, "weak", g, 4) for g in range(4)] == [(32768, g * 32768) for g in range(4)]
    with pytest.raises(ValueError):
        dist.shard(32768, "strong", 0, 3)
    ids = np.concatenate([np.arange(o, o + n) for n, o in (dist.shard(32768, "strong", g, 8) for g in range(8))])
    assert np.array_equal(ids, np.arange(32768))
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "4")
    monkeypatch.setattr(dist.torch.cuda, "device_count", lambda: 1)
    assert dist.ranks_per_device() == 4 and dist.ea_mem_fraction() == 0.0625
    monkeypatch.setattr(dist.torch.cuda, "device_count", lambda: 8)
    assert dist.ranks_per_device() == 1 and dist.ea_mem_fraction() == 0.25

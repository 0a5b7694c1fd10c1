"""CPU tests of the PPO training path's host logic (marlsc/ppo.py, marlsc/experiment.py): the
algorithm-config schema, learning-rate schedules, the PPO loss against a float64 per-sample
restatement of RLlib's PPOTorchLearner loss (+ hysteretic weighting, hysteretic_learner.py:35-42),
per-agent vs shared modules, a learner update, observation statistics arithmetic
(obs_stats.py:74-169), the world_size-2 gradient all-reduce (gloo) and the CLI surface of
scripts/run_experiment.sh. RLlib is not importable here: the learner is parity unpinned."""
import math
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest
import torch
import yaml

REPO = Path(__file__).resolve().parents[1]


def _cfg(name="mappo", **over):
    from marlsc.ppo import PPOConfig
    raw = yaml.safe_load(open(REPO / f"config_files/algorithms/{name}.yaml"))
    raw["algorithm"]["algorithm_specific"].update(over)
    return PPOConfig.from_algorithm_config(raw)


def test_algorithm_configs_parse_like_the_reference_schema():
    m = _cfg("mappo")
    assert m.name == "mappo" and m.critic_obs_type == "global" and m.parameter_sharing
    # the reference's own config_files/algorithms/mappo.yaml / ippo.yaml values
    assert m.num_minibatches == 10 and m.num_epochs == 20 and m.learning_rate == 0.0007598648793612028
    assert m.vf_clip_param == 2046.8403482088547 and m.use_kl_loss is True and m.clip_param == 0.2
    assert m.obs_normalization == "meanstd_custom" and m.logstd_floor == -3.51636237623627
    assert m.networks["actor"]["config"]["hidden_sizes"] == [256, 256]
    assert m.networks["critic"]["config"]["hidden_sizes"] == [64, 64]
    i = _cfg("ippo")
    assert i.name == "ippo" and i.critic_obs_type == "local" and i.clip_param == 0.1 and i.use_kl_loss is False
    assert i.networks["actor"]["config"]["hidden_sizes"] == [256] == i.networks["critic"]["config"]["hidden_sizes"]
    assert i.obs_normalization == "meanstd_custom" and i.entropy_coeff == 0.004402763769660333
    from marlsc.ppo import PPOConfig
    with pytest.raises(ValueError):
        PPOConfig.from_algorithm_config({"algorithm": {"name": "cppo", "shared": {}, "algorithm_specific": {}}})
    with pytest.raises(ValueError):
        _cfg("mappo", hysteretic_beta=1.5)
    assert _cfg("mappo", obs_normalization="meanstd").obs_normalization == "meanstd"  # RLlib's running filter
    with pytest.raises(ValueError):
        _cfg("mappo", obs_normalization="zscore")


def test_learning_rate_schedule_is_piecewise_linear():
    from marlsc.ppo import PPOConfig
    c = PPOConfig(learning_rate=[[0, 1e-3], [1000, 1e-4], [3000, 1e-5]])
    assert c.lr_at(0) == 1e-3 and c.lr_at(-5) == 1e-3
    assert math.isclose(c.lr_at(500), 5.5e-4)
    assert math.isclose(c.lr_at(2000), 5.5e-5)
    assert c.lr_at(10 ** 6) == 1e-5
    assert PPOConfig(learning_rate=3e-4).lr_at(123) == 3e-4


def _ref_loss(cfg, a, mu, ls, v, logp_old, adv, vt, mu_old=None, ls_old=None, kl_coeff=0.0):
    """float64, one sample at a time (RLlib PPOTorchLearner.compute_loss_for_module)."""
    tot = []
    for i in range(a.shape[0]):
        A = adv[i]
        if cfg.hysteretic_beta is not None and A < 0:
            A = A * cfg.hysteretic_beta
        std = np.exp(ls[i])
        logp = float(np.sum(-((a[i] - mu[i]) ** 2) / (2 * std ** 2) - ls[i] - 0.5 * math.log(2 * math.pi)))
        r = math.exp(logp - logp_old[i])
        surr = min(A * r, A * min(max(r, 1 - cfg.clip_param), 1 + cfg.clip_param))
        ent = float(np.sum(ls[i] + 0.5 * math.log(2 * math.pi * math.e)))
        vf = min(max((v[i] - vt[i]) ** 2, 0.0), cfg.vf_clip_param)
        t = -surr + cfg.vf_loss_coeff * vf - cfg.entropy_coeff * ent
        if cfg.use_kl_loss:
            v0, v1 = np.exp(2 * ls_old[i]), np.exp(2 * ls[i])
            kl = float(np.sum(ls[i] - ls_old[i] + (v0 + (mu_old[i] - mu[i]) ** 2) / (2 * v1) - 0.5))
            t += kl_coeff * kl
        tot.append(t)
    return float(np.mean(tot))


@pytest.mark.parametrize("over", [{}, {"hysteretic_beta": 0.3}, {"use_kl_loss": True}])
def test_ppo_loss_matches_per_sample_restatement(over):
    from marlsc.ppo import ppo_loss
    cfg = _cfg("mappo", **over)
    g = np.random.default_rng(5)
    S, K = 37, 5
    a = g.normal(size=(S, K))
    mu = g.normal(size=(S, K)) * 0.5
    ls = np.tile(g.uniform(-2, 0, size=K), (S, 1))
    v = g.normal(size=S) * 4
    vt = g.normal(size=S) * 4
    adv = g.normal(size=S)
    logp_old = g.normal(size=S) - 6
    mu_old = mu + g.normal(size=(S, K)) * 0.1
    ls_old = ls + 0.05
    T = lambda x: torch.tensor(x, dtype=torch.float64)  # noqa: E731
    batch = {"actions": T(a), "logp": T(logp_old), "advantages": T(adv), "value_targets": T(vt),
             "mean_old": T(mu_old), "log_std_old": T(ls_old)}
    loss, st = ppo_loss(cfg, T(mu), T(ls), T(v), batch, kl_coeff=0.2)
    ref = _ref_loss(cfg, a, mu, ls, v, logp_old, adv, vt, mu_old, ls_old, kl_coeff=0.2)
    assert abs(float(loss) - ref) < 1e-9 * max(1.0, abs(ref))


def test_shared_and_per_agent_modules():
    from marlsc.ppo import MultiAgentActorCritic
    cfg = _cfg("mappo")
    rc = cfg.rollout_config()
    W, L, K = 3, 7, 2
    for shared in (True, False):
        torch.manual_seed(0)
        m = MultiAgentActorCritic(W, L, L * W, K, rc, shared)
        assert len(m.policies) == (1 if shared else W)
        obs = torch.randn(4, W, L)
        full = torch.cat([obs, obs.reshape(4, 1, W * L).expand(4, W, W * L)], -1)
        mean, ls = m.dist_inputs(obs, full)
        assert mean.shape == (4, W, K) and ls.shape == (4, W, K)
        assert m.values(obs, full).shape == (4, W)
        if not shared:  # agent w's outputs come from policy w alone
            p1 = m.policies[1]
            torch.testing.assert_close(mean[:, 1], p1.actor(obs[:, 1]))
            torch.testing.assert_close(m.values(obs, full)[:, 2], m.policies[2].critic(full[:, 2]).squeeze(-1))


def test_learner_update_reduces_the_loss_on_a_fixed_batch():
    from marlsc.ppo import MultiAgentActorCritic, PPOLearner, ppo_loss
    cfg = _cfg("ippo")
    cfg.num_epochs, cfg.num_minibatches, cfg.grad_clip = 20, 2, 5.0
    cfg.learning_rate = 3e-3
    rc = cfg.rollout_config()
    torch.manual_seed(1)
    W, L, K, S = 2, 6, 3, 64
    m = MultiAgentActorCritic(W, L, L * W, K, rc, True)
    obs = torch.randn(S, W, L)
    with torch.no_grad():
        mean, ls = m.dist_inputs(obs)
        a = mean + ls.exp() * torch.randn_like(mean)
        from marlsc.ppo import gaussian_logp
        logp = gaussian_logp(a, mean, ls)
    batch = {"obs": obs, "actions": a, "logp": logp, "advantages": torch.randn(S, W),
             "value_targets": torch.randn(S, W) * 3}

    def loss_now():
        with torch.no_grad():
            mu, l2 = m.dist_inputs(obs)
            return float(ppo_loss(cfg, mu, l2, m.values(obs), batch, 0.0)[0])
    before = loss_now()
    out = PPOLearner(m, cfg, seed=0).update(batch, None, timestep=0)
    assert np.isfinite(out["total_loss"]) and out["learning_rate"] == 3e-3
    assert loss_now() < before


def test_grouped_observation_statistics_arithmetic():
    from marlsc.ppo import obs_statistics_from_samples
    from marlsc import make_synthetic_env_config
    from marlsc.spec import EnvSpec
    from marlsc.synthetic import FEATURE_CONFIG_YAML
    feats = {**FEATURE_CONFIG_YAML, "inventory": True, "inventory_aggregate": True, "pipeline": True,
             "pipeline_aggregate": False, "units_shipped_home": True}
    cfg = make_synthetic_env_config(2, 3, 2, episode_length=5, features=feats)
    spec = EnvSpec.from_config(cfg, {})
    L = spec.n_features
    x = np.random.default_rng(0).uniform(0, 9, size=(50, L)).astype(np.float32)
    x[:, -1] = 3.0  # a constant column: std < 1e-8 -> 1.0 (obs_stats.py:82)
    m, s = obs_statistics_from_samples(x, "meanstd_custom")
    np.testing.assert_array_equal(m, x.mean(axis=0))
    assert s[-1] == 1.0
    mg, sg = obs_statistics_from_samples(x, "meanstd_grouped", spec)
    K, lt = spec.K, spec.max_expected_lead_time
    assert mg[0] == np.float32(float(x[:, 0:K].mean())) and mg[1] == mg[0]  # inventory SKU columns share
    assert mg[K] == np.float32(float(x[:, K].mean()))                       # the aggregate has its own
    p0 = K + 1
    assert np.all(mg[p0:p0 + lt * K] == np.float32(float(x[:, p0:p0 + lt * K].mean())))


@pytest.mark.parametrize("seed", range(8))
def test_observation_statistics_vs_oracle_restatement(seed):
    # the product's statistics (marlsc/ppo.py: feature_groups + obs_statistics_from_samples) against
    # the oracle's restatement of obs_stats.py:73-169 over random feature sets (every group, with and
    # without aggregates), bit-exact: both run the reference's numpy calls on the same f32 samples
    from obs_stats_ref import obs_statistics_ref
    from marlsc.ppo import obs_statistics_from_samples
    from marlsc import make_synthetic_env_config
    from marlsc.spec import EnvSpec
    from marlsc.synthetic import FEATURE_CONFIG_YAML
    rng = np.random.default_rng(seed)
    names = ["inventory", "pipeline", "incoming_demand_home", "units_shipped_home", "units_shipped_away",
             "stockout", "rolling_demand_mean", "demand_forecast"]
    aggs = ["inventory_aggregate", "pipeline_aggregate", "incoming_demand_home_aggregate",
            "units_shipped_away_aggregate", "rolling_demand_mean_aggregate", "demand_forecast_aggregate"]
    feats = {**FEATURE_CONFIG_YAML, **{k: bool(rng.integers(0, 2)) for k in names + aggs}}
    feats["inventory"] = feats["pipeline"] = True  # always on (schema validator)
    for parent, agg in [("inventory", "inventory_aggregate"), ("pipeline", "pipeline_aggregate"),
                        ("incoming_demand_home", "incoming_demand_home_aggregate"),
                        ("units_shipped_away", "units_shipped_away_aggregate"),
                        ("rolling_demand_mean", "rolling_demand_mean_aggregate"),
                        ("demand_forecast", "demand_forecast_aggregate")]:
        feats[agg] = feats[agg] and feats[parent]
    cfg = make_synthetic_env_config(3, 4, 1 + seed % 3, episode_length=6, features=feats)
    spec = EnvSpec.from_config(cfg, {})
    x = rng.normal(rng.uniform(-5, 5, spec.n_features), rng.uniform(0.1, 3, spec.n_features),
                   size=(257, spec.n_features)).astype(np.float32)
    x[:, rng.integers(0, spec.n_features)] = 2.5  # a constant column: std 1.0
    for mode in ("meanstd_custom", "meanstd_grouped"):
        m, s = obs_statistics_from_samples(x, mode, spec)
        m2, s2 = obs_statistics_ref(x, mode, dict(spec.features), spec.K, spec.max_expected_lead_time)
        np.testing.assert_array_equal(m, m2)
        np.testing.assert_array_equal(s, s2)


def _grad_worker(rank, world, port, out):
    import torch.distributed as dist
    from marlsc.ppo import allreduce_grads
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    p = torch.nn.Parameter(torch.zeros(5))
    q = torch.nn.Parameter(torch.zeros(2, 3))
    p.grad = torch.full((5,), float(rank + 1))
    q.grad = torch.arange(6.0).reshape(2, 3) * (rank + 1)
    allreduce_grads([p, q])
    np.save(os.path.join(out, f"g{rank}.npy"), np.concatenate([p.grad.numpy(), q.grad.numpy().ravel()]))
    dist.destroy_process_group()


def test_gradient_allreduce_world2_gloo(tmp_path):
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    mp.spawn(_grad_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    g0, g1 = np.load(tmp_path / "g0.npy"), np.load(tmp_path / "g1.npy")
    np.testing.assert_array_equal(g0, g1)
    np.testing.assert_allclose(g0[:5], 1.5)
    np.testing.assert_allclose(g0[5:], np.arange(6.0) * 1.5)


def test_cli_accepts_the_reference_arguments_and_script_is_executable():
    from marlsc.experiment import parse_args
    a = parse_args(["--mode", "single", "--env-config", "e.yaml", "--algorithm-config", "a.yaml",
                    "--storage-dir", "./x", "--experiment-name", "N", "--wandb-project", "marl-sc",
                    "--root-seed", "42"])
    assert a.mode == "single" and a.root_seed == 42 and a.experiment_name == "N"
    b = parse_args(["--mode", "evaluate", "--storage-dir", "./x", "--experiment-name", "N",
                    "--eval-episodes", "100", "--visualize", "--root-seed", "42"])
    assert b.mode == "evaluate" and b.eval_episodes == 100
    sh = REPO / "scripts" / "run_experiment.sh"
    assert os.access(sh, os.X_OK)
    assert subprocess.run(["bash", "-n", str(sh)]).returncode == 0


def test_split_first_layer_critic_equals_the_flat_input_critic():
    # the critic over local_w || (local_0..local_{W-1}) evaluated from the local observations only
    from marlsc.ppo import MultiAgentActorCritic
    cfg = _cfg("mappo")
    rc = cfg.rollout_config()
    W, L, K = 4, 9, 3
    for shared in (True, False):
        torch.manual_seed(3)
        m = MultiAgentActorCritic(W, L, L * W, K, rc, shared).double()
        obs = torch.randn(6, W, L, dtype=torch.float64)
        full = torch.cat([obs, obs.reshape(6, 1, W * L).expand(6, W, W * L)], -1)
        torch.testing.assert_close(m.values(obs), m.values(obs, full), rtol=1e-12, atol=1e-12)


def test_cyclic_minibatch_rows_cover_every_row_once_per_pass():
    # RLlib's MiniBatchCyclicIterator: minibatches wrap into the next reshuffled pass
    from marlsc.ppo import _CyclicRows
    g = torch.Generator().manual_seed(0)
    rows = torch.arange(10) * 3 + 1
    st = _CyclicRows(rows, 4, g)
    seen = []
    while st.covered < 3:
        idx = st.next()
        assert idx.numel() == 4
        seen.append(idx)
    flat = torch.cat(seen)
    assert flat.numel() == 32 and st.covered == 3  # ceil(3 passes x 10 rows / 4) minibatches
    for p in range(3):  # the first 30 rows are three permutations of the module's rows
        assert sorted(flat[10 * p:10 * (p + 1)].tolist()) == sorted(rows.tolist())


@pytest.mark.parametrize("shared", [True, False])
def test_minibatch_steps_per_epoch_follow_rllib_agent_step_sizing(shared):
    # minibatch_size = batch_size // num_minibatches AGENT steps per module (mappo.py:148): the
    # shared policy's batch holds W rows per env step, so it takes W x num_minibatches steps per
    # epoch; each per-agent policy holds one row per env step: num_minibatches steps per epoch
    from marlsc.ppo import MultiAgentActorCritic, PPOLearner
    cfg = _cfg("ippo")
    cfg.num_epochs, cfg.num_minibatches, cfg.grad_clip = 3, 4, None
    W, L, K, S = 4, 5, 2, 64
    cfg.batch_size = S  # one env step per sample
    rc = cfg.rollout_config()
    torch.manual_seed(0)
    m = MultiAgentActorCritic(W, L, L * W, K, rc, shared)
    obs = torch.randn(S, W, L)
    batch = {"obs": obs, "actions": torch.randn(S, W, K), "logp": torch.randn(S, W) - 3,
             "advantages": torch.randn(S, W), "value_targets": torch.randn(S, W)}
    out = PPOLearner(m, cfg, seed=0).update(batch)
    per_epoch = (W if shared else 1) * cfg.num_minibatches
    assert out["num_minibatch_steps"] == cfg.num_epochs * per_epoch


def test_per_agent_modules_update_independently_of_other_agents_data():
    # one policy per agent: the learner minimises the SUM of the module losses and clips each
    # module's gradients by its own norm (RLlib TorchLearner), so agent 0's policy update does not
    # depend on agent 1's batch at all -- not even through a shared gradient-norm clip (the
    # advantages of agent 1 are 1000x larger in the second run)
    from marlsc.ppo import MultiAgentActorCritic, PPOLearner
    cfg = _cfg("ippo")
    cfg.num_epochs, cfg.num_minibatches, cfg.grad_clip, cfg.batch_size = 2, 2, 0.5, 32
    W, L, K, S = 2, 6, 3, 32
    rc = cfg.rollout_config()
    g = torch.Generator().manual_seed(4)
    obs = torch.randn(S, W, L, generator=g)
    base = {"obs": obs, "actions": torch.randn(S, W, K, generator=g), "logp": torch.randn(S, W, generator=g) - 3,
            "advantages": torch.randn(S, W, generator=g), "value_targets": torch.randn(S, W, generator=g)}
    params = []
    for scale in (1.0, 1000.0):
        torch.manual_seed(9)
        m = MultiAgentActorCritic(W, L, L * W, K, rc, False)
        b = dict(base)
        adv = base["advantages"].clone()
        adv[:, 1] *= scale
        b["advantages"] = adv
        PPOLearner(m, cfg, seed=0).update(b)
        params.append([p.detach().clone() for p in m.policies[0].parameters()])
    for a, c in zip(*params):
        torch.testing.assert_close(a, c, rtol=0, atol=0)


def test_grouped_advantage_standardisation_restatement():
    # per-module standardisation of the numpy oracle (tests the checker the GPU tests use):
    # with agents' advantages on very different scales every agent ends with mean 0 / std 1
    from gae_ref import normalize_grouped
    g = np.random.default_rng(2)
    T, E, W = 30, 50, 2
    adv = g.normal(size=(T, E * W)) * np.tile([1.0, 300.0], E) + np.tile([5.0, -40.0], E)
    out = normalize_grouped(adv, W)
    for w in range(W):
        col = out[:, w::W]
        assert abs(col.mean()) < 1e-9 and abs(col.std() - 1.0) < 1e-9

"""GPU tests of the training path (marlsc/ppo.py, marlsc/experiment.py): observation statistics of
the random-policy episodes on the GPU env against the same episodes on the C oracle, short IPPO /
MAPPO training runs, checkpoint round trips and the run_experiment CLI (single + evaluate).
The learner itself is parity unpinned (RLlib absent)."""
import json
from pathlib import Path

import numpy as np
import pytest
import torch
import yaml

pytestmark = pytest.mark.gpu
REPO = Path(__file__).resolve().parents[1]


def _algo(name, **over):
    from marlsc.ppo import PPOConfig
    raw = yaml.safe_load(open(REPO / f"config_files/algorithms/{name}.yaml"))
    raw["algorithm"]["algorithm_specific"].update(over.pop("specific", {}))
    raw["algorithm"]["shared"].update(over)
    return PPOConfig.from_algorithm_config(raw)


@pytest.mark.parametrize("mode", ["meanstd_custom", "meanstd_grouped"])
def test_obs_statistics_gpu_equal_oracle_episodes(mode):
    import oracle as orc
    from marlsc import SeedManager, make_synthetic_env_config
    from marlsc.ppo import compute_obs_statistics, obs_statistics_from_samples
    from marlsc.spec import EnvSpec
    cfg = make_synthetic_env_config(3, 5, 2, episode_length=12)
    sm = SeedManager(2024)
    mean, std = compute_obs_statistics(cfg, sm, mode, n_episodes=3)
    # the same procedure on the C restatement of the reference env (obs_stats.py:48-72); a fresh
    # SeedManager: SeedSequence.spawn hands out new children on every call
    env_seed, action_seed = SeedManager(2024).spawn_child_seeds("obs_stats", 2)
    spec = EnvSpec.from_config(cfg, {"obs_normalization": "off"})
    env = orc.OracleEnv(spec, 1, env_seeds=[env_seed])
    rng = np.random.default_rng(action_seed)
    obs = env.reset()
    samples = []
    for _ in range(3):
        for _ in range(spec.episode_length):
            samples.append(obs[0])
            a = np.stack([rng.uniform(-1, 1, size=(spec.K,)).astype(np.float32) for _ in range(spec.W)])
            obs, _, _, fo = env.step(a[None], final_obs=True)
        samples.append(fo[0])
    m2, s2 = obs_statistics_from_samples(np.concatenate(samples), mode, spec)
    np.testing.assert_array_equal(mean, m2)
    np.testing.assert_array_equal(std, s2)


def _trainer(name, shared=True, E=64, T=8, **spec_over):
    from marlsc import make_synthetic_env_config
    from marlsc.ppo import PPOTrainer
    cfg = _algo(name, num_epochs=2, num_minibatches=2, num_eval_episodes=4,
                specific={"parameter_sharing": shared, **spec_over})
    env_cfg = make_synthetic_env_config(4, 8, 3, episode_length=10)
    return PPOTrainer(env_cfg, cfg, root_seed=7, n_envs=E, rollout_len=T, device=0), env_cfg, cfg


@pytest.mark.parametrize("name,shared", [("mappo", True), ("ippo", False)])
def test_short_training_run_and_checkpoint_round_trip(tmp_path, name, shared):
    from marlsc.ppo import PPOTrainer
    tr, env_cfg, cfg = _trainer(name, shared)
    p0 = [p.detach().clone() for p in tr.module.parameters()]
    for _ in range(3):
        res = tr.train_iteration()
        assert np.isfinite(res["learner/total_loss"]) and np.isfinite(res["learner/vf_loss"])
    assert res["num_env_steps_sampled_lifetime"] == 3 * 8 * 64
    assert res["train/episodes"] >= 64 * 2  # episodes of 10 steps end inside 24 steps
    assert any(not torch.equal(a, b) for a, b in zip(p0, tr.module.parameters()))
    ev = tr.evaluate()
    assert ev["eval/episodes"] == 4 and np.isfinite(ev["eval/episode_return_mean"])
    assert tr.evaluate() == ev  # deterministic policy, fixed eval seed
    ck = tr.save_checkpoint(tmp_path / "ck")
    tr2 = PPOTrainer(env_cfg, cfg, root_seed=7, n_envs=64, rollout_len=8, device=0)
    tr2.load_checkpoint(ck)
    assert tr2.iteration == 3 and tr2.timesteps == tr.timesteps
    assert tr2.evaluate() == ev


def test_kl_loss_and_hysteretic_variant_runs():
    tr, _, _ = _trainer("ippo", True, E=32, T=4, use_kl_loss=True, hysteretic_beta=0.5)
    res = tr.train_iteration()
    assert "learner/mean_kl" in res and "learner/kl_coeff" in res


def test_experiment_cli_single_then_evaluate(tmp_path):
    from marlsc.experiment import main
    env = REPO / "config_files/environments/env_c1_2wh4r2sku.yaml"
    algo = REPO / "config_files/algorithms/ippo.yaml"
    assert main(["--mode", "single", "--env-config", str(env), "--algorithm-config", str(algo),
                 "--storage-dir", str(tmp_path), "--experiment-name", "T", "--root-seed", "42",
                 "--num-iterations", "2", "--envs", "32", "--rollout-len", "4"]) == 0
    out = tmp_path / "T"
    lines = (out / "training_metrics.jsonl").read_text().strip().splitlines()
    assert len(lines) == 2 and json.loads(lines[-1])["training_iteration"] == 2
    assert (out / "checkpoints" / "checkpoint_final" / "learner_state.pt").exists()
    assert main(["--mode", "evaluate", "--storage-dir", str(tmp_path), "--experiment-name", "T",
                 "--eval-episodes", "3", "--root-seed", "42"]) == 0
    res = json.loads((out / "eval_results.json").read_text())
    assert res["eval/episodes"] == 3 and res["iteration"] == 2

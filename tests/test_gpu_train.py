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


def cfg_features(cfg):
    from marlsc.spec import EnvSpec
    return dict(EnvSpec.from_config(cfg, {}).features)


@pytest.mark.parametrize("mode", ["meanstd_custom", "meanstd_grouped"])
def test_obs_statistics_gpu_equal_oracle_episodes(mode):
    import oracle as orc
    from marlsc import SeedManager, make_synthetic_env_config
    from obs_stats_ref import obs_statistics_ref
    from marlsc.ppo import compute_obs_statistics
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
    # the statistics by the oracle's restatement of obs_stats.py (groups from the feature flags)
    m2, s2 = obs_statistics_ref(np.concatenate(samples), mode, cfg_features(cfg), spec.K, spec.max_expected_lead_time)
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
    assert (out / "checkpoint_final" / "learner_state.pt").exists()
    assert (out / "metadata.json").exists() and (out / "module_weights.pt").exists()
    assert main(["--mode", "evaluate", "--storage-dir", str(tmp_path), "--experiment-name", "T",
                 "--eval-episodes", "3", "--root-seed", "42"]) == 0
    res = json.loads((out / "eval_results.json").read_text())
    assert res["eval/episodes"] == 3 and res["iteration"] == 2


def test_run_experiment_script_drives_training_and_evaluation(tmp_path):
    # the entry the north star names: `bash scripts/run_experiment.sh` (the reference's
    # scripts/run_experiment.sh:52-68 -- `--mode single` then `--mode evaluate` with the same storage
    # dir / experiment name / root seed) on BASELINE configs[0] (2 warehouses x 4 regions x 2 SKUs,
    # the reference's IPPO config), shortened through EXTRA_ARGS
    import os
    import subprocess
    env = dict(os.environ, ENV_CONFIG="./config_files/environments/env_c1_2wh4r2sku.yaml",
               ALGO_CONFIG="./config_files/algorithms/ippo.yaml", STORAGE_DIR=str(tmp_path), EXPERIMENT_NAME="SH",
               ROOT_SEED="42", EVAL_EPISODES="2", NGPUS="1",
               EXTRA_ARGS="--num-iterations 2 --envs 16 --rollout-len 4")
    r = subprocess.run(["bash", str(REPO / "scripts" / "run_experiment.sh")], env=env, cwd=str(tmp_path),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    out = tmp_path / "SH"
    lines = (out / "training_metrics.jsonl").read_text().strip().splitlines()
    assert len(lines) == 2 and json.loads(lines[-1])["training_iteration"] == 2
    assert (out / "checkpoint_final" / "learner_state.pt").exists() and (out / "module_weights.pt").exists()
    res = json.loads((out / "eval_results.json").read_text())
    assert res["eval/episodes"] == 2 and res["iteration"] == 2


def test_experiment_resume_truncates_metrics_and_exports_module_weights(tmp_path):
    # the reference runner's run directory (runner.py:163-395): checkpoint_<N> every checkpoint_freq
    # iterations, checkpoint_best on a new best train return, checkpoint_final, module_weights.pt
    # (agent 0's policy module state dict), training_metrics.yaml; --resume-from checkpoint_<N>
    # truncates the metrics to N and continues at N + 1
    from marlsc.experiment import main
    env = REPO / "config_files/environments/env_c1_2wh4r2sku.yaml"
    raw = yaml.safe_load(open(REPO / "config_files/algorithms/mappo.yaml"))
    raw["algorithm"]["shared"].update(checkpoint_freq=1, num_epochs=1, num_minibatches=2, eval_interval=0)
    algo = tmp_path / "mappo_ck1.yaml"
    algo.write_text(yaml.safe_dump(raw))
    args = ["--mode", "single", "--env-config", str(env), "--algorithm-config", str(algo),
            "--storage-dir", str(tmp_path), "--experiment-name", "R", "--root-seed", "42",
            "--envs", "16", "--rollout-len", "60"]
    assert main(args + ["--num-iterations", "3"]) == 0
    out = tmp_path / "R"
    for n in (1, 2, 3):
        assert (out / f"checkpoint_{n}" / "learner_state.pt").exists()
    assert (out / "checkpoint_best" / "learner_state.pt").exists()
    met = yaml.safe_load((out / "training_metrics.yaml").read_text())
    assert [m["iteration"] for m in met] == [1, 2, 3] and set(met[0]) == {"iteration", "train_return", "eval_return"}
    # resume from checkpoint_2: the log restarts after entry 2 and runs to 4
    assert main(args + ["--num-iterations", "4", "--resume-from", str(out / "checkpoint_2")]) == 0
    met2 = yaml.safe_load((out / "training_metrics.yaml").read_text())
    assert [m["iteration"] for m in met2] == [1, 2, 3, 4]
    assert met2[:2] == met[:2]
    w = torch.load(out / "module_weights.pt", weights_only=True)
    keys = set(w)
    assert {"log_std", "actor.0.weight", "actor.0.bias", "critic.0.weight"} <= keys
    assert all(k.startswith(("actor.", "critic.")) or k == "log_std" for k in keys)
    with pytest.raises(ValueError):  # only checkpoint_<N> carries the iteration to resume from
        main(args + ["--num-iterations", "5", "--resume-from", str(out / "checkpoint_best")])


def test_eval_envs_replay_the_reference_eval_episodes():
    # The reference evaluates on ONE env seeded with eval_seed (no per-env derivation in 'val'
    # mode, src/algorithms/base.py:405-417), episodes one after another: reset k starts episode
    # root SeedSequence([eval_seed, k]). evaluate() runs them side by side; env k must start
    # exactly where the reference's k-th sequential reset does (checked on the C oracle env).
    import oracle as orc
    from marlsc import make_synthetic_env_config
    from marlsc.spec import EnvSpec
    from marlsc.vec_env import VecInventoryEnv
    cfg = make_synthetic_env_config(3, 6, 2, episode_length=9)
    n, eval_seed = 5, 987654321
    spec = EnvSpec.from_config(cfg, {"data_mode": "val", "num_eval_episodes": n})
    gpu = VecInventoryEnv(None, n, spec=spec, device=0, env_seeds=np.full(n, eval_seed, np.uint32))
    gpu.set_episode_counters(np.arange(n))
    obs = gpu.reset().cpu().numpy()
    sg = gpu.read_state()
    ref = orc.OracleEnv(spec, 1, env_seeds=[eval_seed])
    for k in range(n):
        o = ref.reset()
        sr = ref.read_state()
        np.testing.assert_array_equal(obs[k], o[0])
        np.testing.assert_array_equal(sg["inventory"][k], sr["inventory"][0])
        np.testing.assert_array_equal(sg["rng"][k], sr["rng"][0])
        assert sg["episode_counter"][k] == k + 1 == sr["episode_counter"][0]
    gpu.close()


def test_resume_from_checkpoint_continues_the_saved_run(tmp_path):
    # resume = the uninterrupted run: the env state (pending pre-generated demand included), the
    # observations, the rollout / learner generators and the episode-return buffers are restored,
    # so iteration k+1 after a resume samples exactly what the uninterrupted run samples
    from marlsc.ppo import PPOTrainer
    tr, env_cfg, cfg = _trainer("mappo", True, E=64, T=6)
    tr.train_iteration()
    ck = tr.save_checkpoint(tmp_path / "ck")
    res_a = tr.train_iteration()
    st_a = tr.env.read_state()
    obs_a = tr.collector.obs.clone()
    tr2 = PPOTrainer(env_cfg, cfg, root_seed=7, n_envs=64, rollout_len=6, device=0)
    tr2.load_checkpoint(ck)
    res_b = tr2.train_iteration()
    st_b = tr2.env.read_state()
    for k in ("inventory", "timestep", "episode_counter", "rng"):
        np.testing.assert_array_equal(st_a[k], st_b[k])
    assert torch.equal(obs_a, tr2.collector.obs)  # the same sampled trajectory
    assert res_a["train/episodes"] == res_b["train/episodes"]
    assert res_a["num_env_steps_sampled_lifetime"] == res_b["num_env_steps_sampled_lifetime"]
    for p, q in zip(tr.module.parameters(), tr2.module.parameters()):  # f64 atomics in the GAE
        torch.testing.assert_close(p, q, rtol=1e-4, atol=1e-5)       # statistics: last-bit noise
    # a fresh trainer WITHOUT the runtime state replays iteration 1's samples: different data
    tr3 = PPOTrainer(env_cfg, cfg, root_seed=7, n_envs=64, rollout_len=6, device=0)
    tr3.load_checkpoint(ck, runtime=False)
    tr3.train_iteration()
    assert not torch.equal(obs_a, tr3.collector.obs)


def test_train_return_is_smoothed_over_num_eval_episodes():
    # metrics_num_episodes_for_smoothing = num_eval_episodes (mappo.py:177)
    tr, _, cfg = _trainer("ippo", False, E=32, T=12)
    res = tr.train_iteration()
    assert len(tr._completed) == cfg.num_eval_episodes and res["train/episodes"] == 32
    rew = tr.collector.rewards.double().sum(-1)  # [T, E]; every env's first episode ends at t = 9
    ep = rew[:10].sum(0).cpu().numpy()
    np.testing.assert_allclose(res["train/episode_return_mean"], ep[-cfg.num_eval_episodes:].mean(), rtol=1e-12)


def test_per_agent_policies_standardise_advantages_per_agent():
    # one policy per agent: RLlib standardises every module's advantages on its own
    tr, _, _ = _trainer("ippo", False, E=64, T=10)
    tr.collector.collect(normalize=True)
    W = tr.env.W
    adv = tr.collector.adv.reshape(-1, W).double()
    assert tr.collector.stats.shape == (W, 3)
    torch.testing.assert_close(adv.mean(0), torch.zeros(W, dtype=torch.float64, device=adv.device), atol=1e-4, rtol=0)
    torch.testing.assert_close(adv.std(0, unbiased=False), torch.ones(W, dtype=torch.float64, device=adv.device),
                               atol=1e-3, rtol=0)


def test_meanstd_running_filter_training_evaluation_and_checkpoint(tmp_path):
    # obs_normalization "meanstd": RLlib's running filter on the device -- every observation the
    # policy sees is pushed once (reset observation, each step's, the final observation of every
    # truncated episode), the lanes synchronise after each rollout, evaluation applies it without
    # updating, and checkpoints carry it
    from marlsc.ppo import PPOTrainer
    E, T = 64, 8
    tr, env_cfg, cfg = _trainer("mappo", True, E=E, T=T, obs_normalization="meanstd")
    for _ in range(2):
        res = tr.train_iteration()
        assert np.isfinite(res["learner/total_loss"])
    f = tr.collector.obs_filter
    # 16 steps of 10-step episodes: E reset obs + 16 E step obs + E final obs (the truncation at step 10)
    assert f.count == E + 2 * T * E + E
    assert float(tr.collector.obs.abs().max()) <= 10.0
    assert float(f.std.min()) >= 0.0 and torch.isfinite(f.mean).all()
    ev = tr.evaluate()
    assert np.isfinite(ev["eval/episode_return_mean"]) and f.count == E + 2 * T * E + E
    assert tr.evaluate() == ev
    ck = tr.save_checkpoint(tmp_path / "ck")
    tr2 = PPOTrainer(env_cfg, cfg, root_seed=7, n_envs=E, rollout_len=T, device=0)
    tr2.load_checkpoint(ck)
    assert torch.equal(tr2.collector.obs_filter.driver, f.driver)
    assert tr2.evaluate() == ev
    tr.train_iteration()
    tr2.train_iteration()
    assert tr2.collector.obs_filter.count == tr.collector.obs_filter.count


def _dist_run_single(rank, world, port, argv, sys_path):
    # one rank of `--mode single` under torchrun-like env vars, gloo collectives, every rank on GPU 0
    import os
    import sys
    sys.path[:0] = [p for p in sys_path if p not in sys.path]
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "MSC_DIST_BACKEND": "gloo"})
    from marlsc.experiment import main
    main(argv)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def test_two_rank_training_equals_one_rank(tmp_path):
    # VERDICT r03 item 8 + ADVICE r03: a whole multi-rank run of `--mode single` (gloo, two ranks
    # sharing the GPU, each stepping half of the envs by global env id) against one rank stepping all
    # of them: the rollout noise is keyed by global env id (msc_normal_keyed), the advantage statistics
    # and gradients are all-reduced, one minibatch per update; so every iteration's train return and
    # the final weights agree to fp tolerance, and checkpoint_best -- decided on the all-reduced return
    # and agreed by broadcast -- is written on the same iterations without a hang
    import socket
    import sys
    import torch.multiprocessing as mp
    from marlsc import make_synthetic_env_config
    env_cfg = make_synthetic_env_config(2, 4, 2, episode_length=10)
    env_path = tmp_path / "env.yaml"
    env_path.write_text(yaml.safe_dump({"environment": env_cfg}))
    raw = yaml.safe_load(open(REPO / "config_files/algorithms/ippo.yaml"))
    raw["algorithm"]["shared"].update(num_minibatches=1, num_epochs=1, batch_size=10 ** 7, eval_interval=0,
                                      checkpoint_freq=0, num_eval_episodes=1000)
    algo_path = tmp_path / "ippo_1mb.yaml"
    algo_path.write_text(yaml.safe_dump(raw))
    res = {}
    for world in (1, 2):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        argv = ["--mode", "single", "--env-config", str(env_path), "--algorithm-config", str(algo_path),
                "--storage-dir", str(tmp_path / f"w{world}"), "--experiment-name", "X", "--root-seed", "5",
                "--num-iterations", "3", "--envs", str(32 // world), "--rollout-len", "15"]
        mp.spawn(_dist_run_single, args=(world, port, argv, list(sys.path)), nprocs=world, join=True)
        out = tmp_path / f"w{world}" / "X"
        res[world] = (yaml.safe_load((out / "training_metrics.yaml").read_text()),
                      torch.load(out / "checkpoint_final" / "learner_state.pt", map_location="cpu", weights_only=True))
        assert (out / "checkpoint_best" / "learner_state.pt").exists()
        assert (out / "checkpoint_best" / f"runtime_rank{world - 1}.pt").exists()
    m1, m2 = res[1][0], res[2][0]
    assert [m["iteration"] for m in m1] == [m["iteration"] for m in m2] == [1, 2, 3]
    for a, b in zip(m1, m2):
        assert (a["train_return"] is None) == (b["train_return"] is None)
        if a["train_return"] is not None:
            assert abs(a["train_return"] - b["train_return"]) <= 1e-9 * max(1.0, abs(a["train_return"]))
    assert res[1][1]["timesteps"] == res[2][1]["timesteps"]
    for k, v in res[1][1]["module"].items():
        torch.testing.assert_close(res[2][1]["module"][k], v, rtol=1e-4, atol=1e-6, msg=k)

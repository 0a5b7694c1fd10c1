"""GPU tests of the on-device rollout (marlsc/rollout.py): actor/critic forward over the HIP env,
truncation bootstrap, GAE kernel and advantage normalisation on the collected buffers.

RLlib is not importable here, so GAE / normalisation are checked against the numpy restatement
(oracle/gae_ref.py) -- parity unpinned against RLlib itself."""
import numpy as np
import pytest
import torch

from gae_ref import gae as gae_np, normalize as norm_np

pytestmark = pytest.mark.gpu


def _setup(critic_obs="global", E=256, T=20, ep_len=7):
    from marlsc import make_synthetic_env_config
    from marlsc.rollout import ActorCritic, RolloutCollector, RolloutConfig
    from marlsc.spec import EnvSpec
    from marlsc.vec_env import VecInventoryEnv
    cfg = make_synthetic_env_config(8, 64, 5, episode_length=ep_len)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    env = VecInventoryEnv(None, E, spec=spec, device=0, base_seed=77)
    env.reset()
    rc = RolloutConfig(critic_obs_type=critic_obs)
    torch.manual_seed(0)
    m = ActorCritic(env.local_obs_dim, env.local_obs_dim * env.W, env.K, rc).cuda()
    return spec, env, m, RolloutCollector(env, m, T, seed=3)


@pytest.mark.parametrize("critic_obs", ["global", "local"])
def test_rollout_buffers_gae_and_normalisation(critic_obs):
    spec, env, m, col = _setup(critic_obs)
    out = col.collect(normalize=False)
    T, N = col.T, col.N
    r = col.rewards.view(T, N).double().cpu().numpy()
    v = col.values.view(T + 1, N).double().cpu().numpy()
    nv = col.next_values.view(T, N).double().cpu().numpy()
    te = col.terminated.view(T, N).cpu().numpy()
    tr = col.truncated.view(T, N).cpu().numpy()
    assert tr.any() and tr.sum() == N * (T // 7)  # episodes of 7 steps truncate inside the rollout
    a_ref, t_ref = gae_np(r, v, nv, te, tr, 0.99, 0.95)
    np.testing.assert_allclose(col.adv.view(T, N).cpu().numpy(), a_ref, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(col.targets.view(T, N).cpu().numpy(), t_ref, rtol=1e-4, atol=1e-4)
    s = col.stats.cpu().numpy()
    assert s.shape == (1, 3) and s[0, 2] == T * N
    np.testing.assert_allclose(s[0, 0], a_ref.sum(), rtol=1e-5)
    from marlsc.rollout import normalize_advantages
    normalize_advantages(col.adv, col.stats)
    np.testing.assert_allclose(col.adv.view(T, N).cpu().numpy(), norm_np(a_ref), rtol=1e-3, atol=1e-3)
    # stored values are the critic on the stored observations
    with torch.no_grad():
        full = env.obs_flat(obs=col.obs[3].contiguous()) if critic_obs == "global" else None
        v3 = m.values(col.obs[3], full)
    torch.testing.assert_close(v3, col.values[3], rtol=1e-5, atol=1e-5)


def test_rollout_replays_bit_exact_on_a_fresh_env():
    # the env consumed exactly the clipped sampled actions: a second env with the same seeds
    # stepped with them reproduces every observation and reward bit for bit
    spec, env, m, col = _setup("global", E=128, T=16)
    col.collect()
    from marlsc.vec_env import VecInventoryEnv
    env2 = VecInventoryEnv(None, 128, spec=spec, device=0, base_seed=77)
    obs = env2.reset()
    for t in range(col.T):
        assert torch.equal(obs, col.obs[t])
        obs, rew, trunc, _ = env2.step(col.actions[t].clamp(-1.0, 1.0).contiguous())
        assert torch.equal(rew, col.rewards[t])


def test_two_lane_rollout_matches_one_env_per_lane():
    # a collector over two env handles (consecutive global env ids, one HIP stream each) fills the
    # buffers' env axis lane by lane: every env consumed exactly its sampled actions (replay on one
    # fresh handle of all envs is bit-exact), the stored values are the critic on the stored
    # observations, and GAE over the joined buffers equals the numpy restatement
    from marlsc import make_synthetic_env_config
    from marlsc.rollout import ActorCritic, RolloutCollector, RolloutConfig
    from marlsc.spec import EnvSpec
    from marlsc.vec_env import VecInventoryEnv
    cfg = make_synthetic_env_config(8, 64, 5, episode_length=7)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    E, T = 192, 16
    lanes = [VecInventoryEnv(None, 64, spec=spec, device=0, base_seed=77, env_index_offset=0),
             VecInventoryEnv(None, E - 64, spec=spec, device=0, base_seed=77, env_index_offset=64)]
    for x in lanes:
        x.reset()
    torch.manual_seed(0)
    m = ActorCritic(spec.local_obs_dim, spec.local_obs_dim * spec.W, spec.K, RolloutConfig()).cuda()
    col = RolloutCollector(lanes, m, T, seed=3)
    col.collect(normalize=False)
    torch.cuda.synchronize()
    env2 = VecInventoryEnv(None, E, spec=spec, device=0, base_seed=77)
    obs = env2.reset()
    for t in range(T):
        assert torch.equal(obs, col.obs[t])
        obs, rew, trunc, _ = env2.step(col.actions[t].clamp(-1.0, 1.0).contiguous())
        assert torch.equal(rew, col.rewards[t])
        assert torch.equal(trunc, col.truncated[t, :, 0])
    N = col.N
    r = col.rewards.view(T, N).double().cpu().numpy()
    v = col.values.view(T + 1, N).double().cpu().numpy()
    nv = col.next_values.view(T, N).double().cpu().numpy()
    a_ref, _ = gae_np(r, v, nv, col.terminated.view(T, N).cpu().numpy(), col.truncated.view(T, N).cpu().numpy(), 0.99, 0.95)
    np.testing.assert_allclose(col.adv.view(T, N).cpu().numpy(), a_ref, rtol=1e-4, atol=1e-4)
    with torch.no_grad():
        v5 = m.values(col.obs[5])
    torch.testing.assert_close(v5, col.values[5], rtol=1e-5, atol=1e-5)


def test_two_lane_meanstd_filter_on_streams_equals_serial_lanes():
    # two lanes with the same env count run their meanstd filter calls on their own HIP
    # streams; each lane has its own scratch, so the concurrent run equals the same two lanes run one
    # after the other on one stream (filter statistics and normalised observations bit-exact)
    from marlsc import make_synthetic_env_config
    from marlsc.rollout import ActorCritic, RolloutCollector, RolloutConfig
    from marlsc.spec import EnvSpec
    from marlsc.vec_env import VecInventoryEnv
    cfg = make_synthetic_env_config(8, 64, 5, episode_length=7)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    E, T = 4096, 9
    torch.manual_seed(0)
    m = ActorCritic(spec.local_obs_dim, spec.local_obs_dim * spec.W, spec.K, RolloutConfig()).cuda()

    def run(serial):
        lanes = [VecInventoryEnv(None, E // 2, spec=spec, device=0, base_seed=77, env_index_offset=j * E // 2)
                 for j in range(2)]
        for x in lanes:
            x.reset()
        col = RolloutCollector(lanes, m, T, seed=3, obs_filter="meanstd")
        if serial:
            for ln in col._lanes:
                ln.stream = None
        col.collect(normalize=False)
        col.collect(normalize=False)
        torch.cuda.synchronize()
        out = (col.obs.clone(), col.obs_filter.driver.clone(), [s.clone() for s in col.obs_filter.lanes])
        for x in lanes:
            x.close()
        return out

    o1, d1, l1 = run(False)
    o2, d2, l2 = run(True)
    assert torch.equal(o1, o2)
    assert torch.equal(d1, d2)
    assert all(torch.equal(a, b) for a, b in zip(l1, l2))


def test_fused_linear_relu_inference_matches_layer_sequence():
    # rollout inference runs Linear -> ReLU pairs as one GEMM with a ReLU epilogue; the plain layer
    # sequence (autograd path, used by the learner) must agree to GEMM rounding
    from marlsc.rollout import MLP, split_global_mlp
    torch.manual_seed(0)
    mlp = MLP(34 * 9, 1, {"hidden_sizes": [64, 64]}).cuda()
    actor = MLP(34, 5, {"hidden_sizes": [256, 256]}).cuda()
    x = torch.randn(4096, 8, 34, device="cuda")
    with torch.no_grad():
        fa = actor(x)
        fc = split_global_mlp(mlp, x)
    with torch.enable_grad():
        pa = actor(x)
        pc = split_global_mlp(mlp, x)
    torch.testing.assert_close(fa, pa.detach(), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(fc, pc.detach(), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("L,H,KO,n", [(34, 256, 5, 262144 // 64), (42, 256, 5, 1000), (34, 64, 1, 77),
                                       (306, 64, 1, 4096), (33, 128, 32, 31), (1, 256, 5, 64)])
def test_fused_mlp3_kernel_matches_torch_layers(L, H, KO, n):
    # msc_mlp3_relu_forward (one f32-MFMA kernel, hidden activations in registers) against the torch
    # fp32 layer sequence of the same MLP: ragged row counts, odd input widths, 1..32 outputs
    from marlsc.mlp import fusable, mlp3_forward
    from marlsc.rollout import MLP
    torch.manual_seed(L + H + KO)
    mlp = MLP(L, KO, {"hidden_sizes": [H, H]}).cuda()
    mods = list(mlp)
    assert fusable(mods)
    x = torch.randn(n, L, device="cuda")
    with torch.no_grad():
        ref = mods[4](torch.relu(mods[2](torch.relu(mods[0](x)))))
        got = mlp3_forward(mods, x)
    torch.testing.assert_close(got, ref, rtol=2e-5, atol=2e-5)
    # the weight pack follows in-place updates (optimizer steps bump the version counters)
    with torch.no_grad():
        mods[2].weight.mul_(0.5)
        ref = mods[4](torch.relu(mods[2](torch.relu(mods[0](x)))))
        got = mlp3_forward(mods, x)
    torch.testing.assert_close(got, ref, rtol=2e-5, atol=2e-5)


@pytest.mark.parametrize("W,L", [(8, 34), (16, 42), (3, 13)])
def test_fused_mappo_critic_matches_split_layers(W, L):
    # the MAPPO critic over local_w || global through the fused kernel (per-env global block as the
    # first layer's pre1 term, group = W agents) against the same split MLP in torch layers
    from marlsc.rollout import MLP, split_global_mlp
    torch.manual_seed(W * L)
    critic = MLP(L * (1 + W), 1, {"hidden_sizes": [64, 64]}).cuda()
    x = torch.randn(777, W, L, device="cuda")
    with torch.no_grad():
        fused = split_global_mlp(critic, x)
    with torch.enable_grad():
        ref = split_global_mlp(critic, x).detach()
        full = critic(torch.cat([x, x.reshape(777, 1, W * L).expand(777, W, W * L)], dim=-1)).detach()
    torch.testing.assert_close(fused, ref, rtol=2e-5, atol=2e-5)
    torch.testing.assert_close(fused, full, rtol=2e-5, atol=2e-5)


def test_gaussian_sample_kernel_matches_torch_formula():
    # msc_gaussian_sample against the TorchDiagGaussian restatement in torch fp32
    import math
    from marlsc.rollout import gaussian_sample
    g = torch.Generator(device="cuda").manual_seed(3)
    mean = torch.randn(5000, 8, 5, device="cuda", generator=g)
    log_std = torch.randn(8, 5, device="cuda", generator=g) - 2.0  # one row per agent
    eps = torch.randn(5000, 8, 5, device="cuda", generator=g)
    act = torch.empty_like(mean)
    logp = torch.empty(5000, 8, device="cuda")
    clipped = gaussian_sample(mean, log_std, -3.5, eps, act, logp)
    ls = torch.clamp(log_std, min=-3.5)
    std = ls.exp()
    a = mean + std * eps
    lp = (-((a - mean) ** 2) / (2 * std * std) - ls - 0.5 * math.log(2 * math.pi)).sum(-1)
    torch.testing.assert_close(act, a, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(logp, lp, rtol=1e-5, atol=1e-5)
    assert torch.equal(clipped, act.clamp(-1.0, 1.0))


@pytest.mark.parametrize("L,hidden,KO,n", [
    (34, [256], 5, 32768),        # IPPO actor (config_files/algorithms/ippo.yaml:46): one hidden layer
    (34, [256], 1, 4099),         # IPPO critic on local obs (:52)
    (306, [1024], 1, 1000),       # the MAPPO test config's [1024] critic head over the flat obs
    (42, [128], 1, 77),           # the IPPO test config's [128] critic
    (13, [96], 7, 65),            # hidden 3 tiles of 32 (one tile per group), 7 outputs
    (34, [160], 17, 300),         # 5 tiles, MFMA output layer (> 8 outputs)
    (34, [256, 128], 5, 2048),    # unequal two-layer forms
    (34, [128, 256], 1, 513),
    (34, [64, 512], 5, 700),
    (34, [512, 64], 5, 700),
    (34, [512, 512], 32, 257),
])
def test_fused_mlp_forms_match_torch_layers(L, hidden, KO, n):
    # msc_mlp2_relu_forward / msc_mlp3_relu_forward against the torch fp32 layer sequence of the
    # same MLP (tolerance 2e-5 abs / rel), and the weight pack follows in-place updates
    from marlsc.mlp import fused_layers, mlp3_forward
    from marlsc.rollout import MLP
    torch.manual_seed(L + sum(hidden) + KO)
    mlp = MLP(L, KO, {"hidden_sizes": hidden}).cuda()
    mods = list(mlp)
    assert fused_layers(mods) == len(hidden) + 1
    x = torch.randn(n, L, device="cuda")

    def ref():
        y = x
        for m in mods:
            y = m(y)
        return y
    with torch.no_grad():
        torch.testing.assert_close(mlp3_forward(mods, x), ref(), rtol=2e-5, atol=2e-5)
        mods[0].weight.mul_(-0.75)
        torch.testing.assert_close(mlp3_forward(mods, x), ref(), rtol=2e-5, atol=2e-5)


@pytest.mark.parametrize("L,hidden,KO,P,n", [
    (34, [256, 256], 5, 1, 32768),  # MAPPO actor, shared log_std row
    (34, [256], 5, 8, 4096 * 8),    # IPPO actor [256], one log_std row per agent
    (13, [64, 64], 2, 2, 1002),   # ragged last tile
    (34, [96], 8, 4, 76),
])
def test_fused_actor_sampling_equals_mlp_then_gaussian_kernel(L, hidden, KO, P, n):
    # msc_mlp{2,3}_relu_forward_sampled: the sampling epilogue is msc_gaussian_sample's arithmetic on
    # the kernel's own outputs, so actions / logp / clipped equal the two-launch path bit for bit
    from marlsc.mlp import mlp3_forward, sample_fusable
    from marlsc.rollout import MLP, gaussian_sample
    torch.manual_seed(L + KO + P)
    mods = list(MLP(L, KO, {"hidden_sizes": hidden}).cuda())
    assert sample_fusable(mods)
    g = torch.Generator(device="cuda").manual_seed(11)
    x = torch.randn(n, L, device="cuda", generator=g)
    eps = torch.randn(n, KO, device="cuda", generator=g)
    ls = (torch.randn(P, KO, device="cuda", generator=g) - 1.0).contiguous()
    with torch.no_grad():
        mean = mlp3_forward(mods, x)
        a_ref, lp_ref = torch.empty_like(mean), torch.empty(n, device="cuda")
        c_ref = gaussian_sample(mean, ls, -2.0, eps, a_ref, lp_ref)
        a, lp, c, m_out = torch.empty_like(mean), torch.empty(n, device="cuda"), torch.empty_like(mean), torch.empty_like(mean)
        mlp3_forward(mods, x, m_out, sample=(ls, -2.0, eps, a, lp, c))
        a2, lp2, c2 = torch.empty_like(mean), torch.empty(n, device="cuda"), torch.empty_like(mean)
        assert mlp3_forward(mods, x, None, sample=(ls, -2.0, eps, a2, lp2, c2)) is None  # means not written
    assert torch.equal(m_out, mean)
    for got in ((a, lp, c), (a2, lp2, c2)):
        assert torch.equal(got[0], a_ref) and torch.equal(got[1], lp_ref) and torch.equal(got[2], c_ref)


@pytest.mark.parametrize("form", ["8", "21", "4"])
def test_mlp3_pass_forms_bit_identical(monkeypatch, form):
    # msc_mlp3_relu_forward's layer-2 pass forms at 256 x 256 (MSC_MLP_P8): the default 41 (passes of
    # 4 tiles, output layer interleaved into the next pass) against 8 (one pass), 21 and 4 -- the same
    # accumulation order, so means and the fused sampling outputs are bit-identical
    from marlsc.mlp import mlp3_forward
    from marlsc.rollout import MLP
    torch.manual_seed(5)
    mods = list(MLP(34, 5, {"hidden_sizes": [256, 256]}).cuda())
    g = torch.Generator(device="cuda").manual_seed(3)
    n = 4099  # ragged last tile
    x = torch.randn(n, 34, device="cuda", generator=g)
    eps = torch.randn(n, 5, device="cuda", generator=g)
    ls = (torch.randn(1, 5, device="cuda", generator=g) - 1.0).contiguous()
    outs = []
    with torch.no_grad():
        for f in ("41", form):
            monkeypatch.setenv("MSC_MLP_P8", f)
            m = torch.empty(n, 5, device="cuda")
            a, lp, c = torch.empty(n, 5, device="cuda"), torch.empty(n, device="cuda"), torch.empty(n, 5, device="cuda")
            mlp3_forward(mods, x, m, sample=(ls, -2.0, eps, a, lp, c))
            torch.cuda.synchronize()
            outs.append((m, a, lp, c))
    for u, v in zip(*outs):
        assert torch.equal(u, v)


def test_rollout_with_fused_sampling_equals_the_two_launch_path(monkeypatch):
    # the collector's fused actor + sampling launch against its mean -> msc_gaussian_sample path on
    # the same env seeds and noise: every buffer identical
    out = []
    for fused in (True, False):
        spec, env, m, col = _setup("global", E=128, T=9, ep_len=5)
        if not fused:
            monkeypatch.setattr(type(m), "actor_sample", lambda self, *a, **k: False)
        b = col.collect()
        out.append({k: v.clone() for k, v in b.items()})
        monkeypatch.undo()
    for k in out[0]:
        assert torch.equal(out[0][k], out[1][k]), k


def test_fused_mlp_rejects_unsupported_shapes():
    from marlsc.mlp import fused_layers
    from marlsc.rollout import MLP
    assert fused_layers(list(MLP(34, 5, {"hidden_sizes": [100]}))) == 0     # not a multiple of 32
    assert fused_layers(list(MLP(34, 5, {"hidden_sizes": [96, 96]}))) == 0  # two-layer sizes: 64..512 powers of 2
    assert fused_layers(list(MLP(2000, 5, {"hidden_sizes": [256]}))) == 0   # more than 1024 inputs
    assert fused_layers(list(MLP(34, 40, {"hidden_sizes": [256]}))) == 0    # more than 32 outputs
    assert fused_layers(list(MLP(34, 5, {"hidden_sizes": [64, 64, 64]}))) == 0


def test_fused_mappo_test_critic_1024_matches_split_layers():
    # the reference's mappo_test.yaml critic [1024] over local_w || global, through the one-hidden-
    # layer kernel with the per-env global block as pre1
    from marlsc.rollout import MLP, split_global_mlp
    torch.manual_seed(5)
    W, L = 8, 34
    critic = MLP(L * (1 + W), 1, {"hidden_sizes": [1024]}).cuda()
    x = torch.randn(300, W, L, device="cuda")
    with torch.no_grad():
        fused = split_global_mlp(critic, x)
    full = critic(torch.cat([x, x.reshape(300, 1, W * L).expand(300, W, W * L)], dim=-1)).detach()
    torch.testing.assert_close(fused, full, rtol=2e-5, atol=2e-5)


def test_multi_lane_rollout_after_weight_update_uses_fresh_packs():
    # with two rollout lanes (two HIP streams) the fused-MLP pack rebuilt after a weight
    # update on one lane's stream must be ordered before the other lane's use: every stored value
    # equals the critic on the stored observation with the updated weights
    from marlsc import make_synthetic_env_config
    from marlsc.rollout import ActorCritic, RolloutCollector, RolloutConfig
    from marlsc.spec import EnvSpec
    from marlsc.vec_env import VecInventoryEnv
    cfg = make_synthetic_env_config(8, 64, 5, episode_length=9)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    lanes = [VecInventoryEnv(None, 2048, spec=spec, device=0, base_seed=7, env_index_offset=0),
             VecInventoryEnv(None, 2048, spec=spec, device=0, base_seed=7, env_index_offset=2048)]
    for x in lanes:
        x.reset()
    torch.manual_seed(1)
    rc = RolloutConfig(critic_obs_type="local", critic={"hidden_sizes": [256, 256]})
    m = ActorCritic(spec.local_obs_dim, spec.local_obs_dim * spec.W, spec.K, rc).cuda()
    col = RolloutCollector(lanes, m, 6, seed=3)
    col.collect(normalize=False)
    for it in range(3):
        with torch.no_grad():  # an optimizer step: in-place parameter updates
            for p in m.parameters():
                p.add_(0.01 * torch.randn_like(p))
        col.collect(normalize=False)
        torch.cuda.synchronize()
        with torch.enable_grad():  # torch layers (no fused kernel) as the reference
            for t in (0, 3, 5):
                ref = m.critic(col.obs[t]).squeeze(-1).detach()
                torch.testing.assert_close(col.values[t], ref, rtol=2e-5, atol=2e-5)


@pytest.mark.parametrize("E", [1, 37, 300, 5000])
def test_meanstd_filter_kernel_matches_the_oracle(E):
    # obs_normalization "meanstd" (RLlib's MeanStdFilter connector, mappo.py:170-171): the device
    # filter (segments of sequential pushes joined by Chan merges) against the numpy restatement's
    # strictly sequential pushes over several steps, a masked push (final observations) and an
    # update=False pass; f32 outputs to rounding, f64 statistics to 1e-10
    from meanstd_ref import MeanStdFilter, filter_rows
    from marlsc.obs_filter import MeanStdObsFilter
    W, L = 3, 7
    C = W * L
    rng = np.random.default_rng(E)
    dev = MeanStdObsFilter(C, "cuda", n_lanes=1)
    ref = MeanStdFilter((C,))
    scale = rng.uniform(0.1, 50.0, C)
    for step in range(4):
        x = (rng.normal(2.0, 1.0, (E, W, L)) * scale.reshape(W, L)).astype(np.float32)
        xt = torch.from_numpy(x).cuda()
        mask = None
        if step == 2:
            mask = (rng.uniform(size=E) < 0.5).astype(np.uint8)
            mask[0] = 1
        got = dev.apply(0, xt, mask=None if mask is None else torch.from_numpy(mask).cuda())
        want = filter_rows(ref, x.reshape(E, C), mask=mask)
        np.testing.assert_allclose(got.reshape(E, C).cpu().numpy(), want, rtol=1e-5, atol=1e-5)
    st = dev.lanes[0].cpu().numpy()
    assert st[0] == ref.rs.n and st[1] == ref.buffer.n
    np.testing.assert_allclose(st[4:4 + C], ref.rs.M, rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(st[4 + C:4 + 2 * C], ref.rs.S, rtol=1e-10)
    np.testing.assert_allclose(st[4 + 2 * C:4 + 3 * C], ref.buffer.M, rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(st[4 + 3 * C:], ref.buffer.S, rtol=1e-10)
    # synchronisation: the driver takes the buffer; evaluation normalises without pushing
    dev.sync()
    assert dev.count == ref.rs.n and float(dev.lanes[0][1]) == 0.0
    x = rng.normal(0, 3.0, (E, W, L)).astype(np.float32)
    got = dev.normalize(torch.from_numpy(x).cuda())
    want = filter_rows(ref, x.reshape(E, C), update=False)
    np.testing.assert_allclose(got.reshape(E, C).cpu().numpy(), want, rtol=1e-5, atol=1e-5)
    assert dev.count == ref.rs.n

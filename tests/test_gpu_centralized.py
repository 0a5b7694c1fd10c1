"""GPU tests of the centralised (CPPO) single-agent views (marlsc/single_env.py), the reference's
CentralizedEnvWrapper (src/environment/envs/single_env.py:25-267): global observation, flat action
split in agent order, agent-order reward sum -- against the multi-agent env and the C oracle."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_wrapper_matches_the_multi_agent_env():
    from marlsc import CentralizedEnvWrapper, InventoryEnvironment, make_synthetic_env_config
    cfg = make_synthetic_env_config(3, 5, 2, episode_length=6)
    meta = {"include_warehouse_id": True}
    cw = CentralizedEnvWrapper(cfg, seed=11, env_meta=meta)
    ma = InventoryEnvironment(cfg, seed=11, env_meta=meta)
    L = ma._compute_local_obs_dim()
    assert cw.observation_space.shape == (3 * L,) and cw.action_space.shape == (6,)
    g, _ = cw.reset()
    o, _ = ma.reset()
    np.testing.assert_array_equal(g, o["warehouse_0"][L:])
    rng = np.random.default_rng(0)
    for t in range(9):  # crosses an episode end (auto-reset semantics of the inner env)
        a = rng.uniform(-1, 1, size=6).astype(np.float32)
        g, r, term, trunc, _ = cw.step(a)
        o, rw, te, tr, _ = ma.step({f"warehouse_{i}": a[2 * i:2 * i + 2] for i in range(3)})
        np.testing.assert_array_equal(g, o["warehouse_1"][L:])
        assert r == rw["warehouse_0"] + rw["warehouse_1"] + rw["warehouse_2"]
        assert trunc == all(tr.values()) and term is False
        if trunc:
            g, _ = cw.reset()
            ma.reset()


def test_vectorised_view_matches_the_oracle():
    import oracle as orc
    from marlsc import VecCentralizedEnv, make_synthetic_env_config
    from marlsc.spec import EnvSpec
    from marlsc.vec_env import VecInventoryEnv
    cfg = make_synthetic_env_config(4, 8, 3, episode_length=7)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    E = 70
    venv = VecCentralizedEnv(VecInventoryEnv(None, E, spec=spec, device=0, base_seed=99))
    ref = orc.OracleEnv(spec, E, base_seed=99)
    g = venv.reset()
    np.testing.assert_array_equal(g.cpu().numpy(), ref.reset().reshape(E, -1))
    rng = np.random.default_rng(4)
    for t in range(10):
        a = rng.uniform(-1, 1, size=(E, 4 * 3)).astype(np.float32)
        g, r, tr, _ = venv.step(torch.from_numpy(a).cuda())
        o, rr, trr, _ = ref.step(a.reshape(E, 4, 3))
        np.testing.assert_array_equal(g.cpu().numpy(), o.reshape(E, -1))
        tot = rr[:, 0].copy()
        for w in range(1, 4):
            tot += rr[:, w]
        np.testing.assert_allclose(r.cpu().numpy(), tot, rtol=0, atol=1e-9)
        np.testing.assert_array_equal(tr.cpu().numpy().astype(bool), trr)

"""Pin the C oracle (oracle/msc_oracle.c) against vectors produced by the reference itself.

CPU only. The oracle is the checker for the HIP path, so it must match the reference's own
outputs (tests/golden/*.npz from tests/golden/make_golden.py): bit-exact integer state
(inventory, orders, demand, shipments, PCG64 states), bit-exact observations, and rewards to
1e-9 (the north star allows 1e-5)."""
import numpy as np
import pytest

import oracle as orc
from golden_util import ENV_FIXTURES, INFO_MAP, COST_KEYS, load, spec_of


def test_rng_known_answers():
    g = dict(np.load(orc.HERE.parent / "tests/golden/rng_streams.npz"))
    st = np.zeros(8, np.uint32)
    import ctypes as C
    out = (C.c_uint32 * 8)()
    orc.lib().orc_seedseq_state(orc.u32s([42]), 1, None, 0, out, 8)
    assert np.array_equal(np.array(out[:], np.uint32), g["ss42_u32x8"])
    w = np.array(out[:], np.uint32)
    assert np.array_equal(w.view(np.uint64), g["ss42_u64x4"])
    for i in range(4):
        orc.lib().orc_seedseq_state(orc.u32s([42]), 1, orc.u32s([i]), 1, out, 8)
        assert np.array_equal(np.array(out[:], np.uint32).view(np.uint64), g["ss42_kid_u64x4"][i])
    assert [orc.seedseq_u32([123456789, e]) for e in range(16)] == g["ss_pair_u32"].tolist()
    assert [orc.seedseq_u32([987654321, 0, e]) for e in range(16)] == g["ss_triple_u32"].tolist()
    r = orc.OracleRng([42], [2])
    assert np.array_equal(r.state(), g["pcg_init"])
    assert [r.next64() for _ in range(9)] == g["next64"].tolist()
    assert [r.random() for _ in range(13)] == g["random"].tolist()
    assert [r.poisson(4.0) for _ in range(64)] == g["poisson4"].tolist()
    assert [r.poisson(l) for l in [0.5, 9.5, 1.0, 7.25, 3.0] * 8] == g["poisson_mix"].tolist()
    assert [r.integers(-2, 3) for _ in range(7)] == g["ints_a"].tolist()
    assert [r.random() for _ in range(3)] == g["random_b"].tolist()
    assert [r.integers(0, 61) for _ in range(20)] == g["ints_b"].ravel().tolist()
    assert [r.integers(0, 1000) for _ in range(5)] == g["ints_c"].tolist()
    assert [r.integers(0, 3_000_000_000) for _ in range(9)] == g["ints_d"].tolist()
    assert np.array_equal(r.state(), g["pcg_final"])


@pytest.mark.parametrize("name", ENV_FIXTURES)
def test_oracle_matches_reference(name):
    d, meta = load(name)
    spec = spec_of(d, meta)
    E, S = meta["n_envs"], meta["n_steps"]
    env = orc.OracleEnv(spec, E, env_seeds=meta["env_seeds"])
    obs = env.reset()
    np.testing.assert_array_equal(obs, d["reset_obs"][:, 0])
    st = env.read_state()
    np.testing.assert_array_equal(st["inventory"], d["reset_inventory"][:, 0])
    np.testing.assert_array_equal(st["rng"][:, 0], d["reset_rng_demand"][:, 0])
    np.testing.assert_array_equal(st["rng"][:, 1], d["reset_rng_lead"][:, 0])
    reset_steps = d["reset_step"][0]
    for t in range(S):
        info = env.alloc_info()
        obs, rew, tr, fo = env.step(d["actions"][:, t], info=info, final_obs=True)
        for fk, ik in INFO_MAP.items():
            ref = d[fk][:, t]
            if fk == "lost_sales":
                np.testing.assert_allclose(info[ik], ref, rtol=1e-12, atol=1e-9, err_msg=f"{name} t={t} {fk}")
            else:
                np.testing.assert_array_equal(info[ik], ref, err_msg=f"{name} t={t} {fk}")
        for c, ck in enumerate(COST_KEYS):
            np.testing.assert_allclose(info["costs"][:, c], d[ck][:, t], rtol=1e-12, atol=1e-9, err_msg=f"{name} t={t} {ck}")
        np.testing.assert_allclose(rew, d["rewards"][:, t], rtol=0, atol=1e-9, err_msg=f"{name} t={t} rewards")
        assert np.array_equal(tr, d["trunc"][:, t])
        terminal = fo if tr.any() else obs
        np.testing.assert_array_equal(terminal, d["obs"][:, t], err_msg=f"{name} t={t} obs")
        if tr.any():
            k = list(reset_steps).index(t + 1) if (t + 1) in reset_steps else None
            if k is not None:
                np.testing.assert_array_equal(obs, d["reset_obs"][:, k], err_msg=f"{name} reset@{t+1}")
        else:
            st = env.read_state()
            np.testing.assert_array_equal(st["inventory"], d["inv_after"][:, t])
            np.testing.assert_array_equal(st["rng"][:, 0], d["rng_demand"][:, t], err_msg=f"{name} t={t} rng demand")
            np.testing.assert_array_equal(st["rng"][:, 1], d["rng_lead"][:, t], err_msg=f"{name} t={t} rng lead")


def test_poisson_ptrs_known_answers():
    # numpy's PTRS branch (lam >= 10): 100,000 draws per rate from
    # Generator(PCG64(SeedSequence([7, i]))).poisson and one stream cycling rates across both
    # branches (tests/golden/make_ptrs_vectors.py, numpy only); draws and final states bit-exact
    g = np.load(orc.HERE.parent / "tests/golden/poisson_ptrs.npz")
    for i, lam in enumerate(g["rates"]):
        r = orc.OracleRng.from_state(g[f"init_{i}"])
        x = r.poisson_n(lam, g[f"draws_{i}"].size)
        assert np.array_equal(x, g[f"draws_{i}"].astype(np.int64)), f"lam={lam}"
        assert np.array_equal(r.state(), g[f"final_{i}"]), f"lam={lam}"
    r = orc.OracleRng.from_state(g["init_mix"])
    x = r.poisson_n(g["mix_rates"], g["draws_mix"].size)
    assert np.array_equal(x, g["draws_mix"].astype(np.int64))
    assert np.array_equal(r.state(), g["final_mix"])

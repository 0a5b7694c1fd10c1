"""GPU parity: the HIP path (libmarlsc via VecInventoryEnv) against the reference's golden vectors
and against the C oracle on larger seeded batches. Bar: bit-exact integer state, observations and
PCG64 states; rewards within 1e-6 absolute (north star: 1e-5)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import oracle as orc  # noqa: E402
from golden_util import COST_KEYS, ENV_FIXTURES, INFO_MAP, load, spec_of  # noqa: E402
from marlsc import make_synthetic_env_config  # noqa: E402
from marlsc.synthetic import FEATURE_CONFIG_YAML  # noqa: E402
from marlsc.spec import EnvSpec  # noqa: E402

pytestmark = pytest.mark.gpu
REW_ATOL = 1e-6


def _set_alloc(monkeypatch, param):
    # "<impl>[_<opt>...]": impl lane / lane2 / lane4 (one env per lane, 1 / 2 / 4 lanes per env),
    # group (one env per lane group), scan (one env per wave, prefix scan over the cost ranking);
    # opts sorted / unsorted (group kernel's visiting order), ea0 / ea1 (episode-ahead demand off /
    # on; default: on for the scan kernel, the library's choice for group, off for lane), nofc (the
    # scan allocator without its fused phases A and C: the step_a / step_c kernels run), nofa (phase C
    # fused, phase A in step_a)
    impl, *opts = param.split("_")
    monkeypatch.setenv("MSC_ALLOC_IMPL", "lane" if impl.startswith("lane") else impl)
    monkeypatch.setenv("MSC_ALLOC_LPE", impl[4:] if impl.startswith("lane") and impl[4:] else "0")
    # group kernel: envs visited in descending order of their order count (default for empirical
    # demand), forced on ("sorted") or off ("unsorted")
    sort = [o for o in opts if o in ("sorted", "unsorted")]
    if sort:
        monkeypatch.setenv("MSC_ALLOC_SORT", "1" if sort[0] == "sorted" else "0")
    else:
        monkeypatch.delenv("MSC_ALLOC_SORT", raising=False)
    # step_a / step_c with the pending ring in registers: off with the lane kernel (as the library
    # runs at >= 16,384 envs, C3), on with the others (its default below that), so both forms of the
    # two phase kernels meet every reference
    monkeypatch.setenv("MSC_OBS_RING_REG", "0" if impl.startswith("lane") else "1")
    # step_c's observation stage: the library's choice with the lane kernel (two phases; off with
    # episode-ahead demand, as with scan), the whole block in one phase with the group kernel
    if impl == "group":
        monkeypatch.setenv("MSC_OBS_STAGE", "1")
    else:
        monkeypatch.delenv("MSC_OBS_STAGE", raising=False)
    # the scan allocator runs phase C itself (MSC_FUSE_C, default on); "nofc" keeps the step_c kernel
    if "nofc" in opts:
        monkeypatch.setenv("MSC_FUSE_C", "0")
    else:
        monkeypatch.delenv("MSC_FUSE_C", raising=False)
    if "nofa" in opts:  # phase C fused, phase A in the step_a kernel
        monkeypatch.setenv("MSC_FUSE_A", "0")
    else:
        monkeypatch.delenv("MSC_FUSE_A", raising=False)
    ea = "0" if "ea0" in opts or impl.startswith("lane") else "1" if ("ea1" in opts or impl == "scan") else None
    if ea is None:
        monkeypatch.delenv("MSC_EA", raising=False)
    else:
        monkeypatch.setenv("MSC_EA", ea)


@pytest.fixture(params=["lane", "group", "group_sorted", "group_nofc", "scan", "scan_ea0", "scan_nofc", "scan_nofa"])
def alloc_impl(request, monkeypatch):
    # every phase-B allocation kernel (one env per lane / per lane group / per wave) against the same
    # references, with and without episode-ahead demand; msc_env_create picks by shape otherwise
    _set_alloc(monkeypatch, request.param)
    return request.param


@pytest.fixture(params=["lane", "lane2", "lane4", "group", "group_sorted", "group_unsorted_ea1", "scan", "scan_ea0",
                        "scan_nofc"])
def alloc_impl_lpe(request, monkeypatch):
    # as alloc_impl, plus the lane kernel's 2 / 4 lanes-per-env forms (A/B; >= 8 warehouses)
    _set_alloc(monkeypatch, request.param)
    return request.param


def _vec(spec, E, **kw):
    from marlsc.vec_env import VecInventoryEnv
    return VecInventoryEnv(None, E, spec=spec, device=0, **kw)


def _np(t):
    return t.detach().cpu().numpy()


@pytest.mark.parametrize("name", ENV_FIXTURES)
@pytest.mark.usefixtures("alloc_impl")
def test_gpu_matches_reference_golden(name):
    d, meta = load(name)
    spec = spec_of(d, meta)
    E, S = meta["n_envs"], meta["n_steps"]
    env = _vec(spec, E, env_seeds=meta["env_seeds"])
    np.testing.assert_array_equal(_np(env.reset()), d["reset_obs"][:, 0])
    st = env.read_state()
    np.testing.assert_array_equal(st["inventory"], d["reset_inventory"][:, 0])
    np.testing.assert_array_equal(st["rng"][:, 0], d["reset_rng_demand"][:, 0])
    np.testing.assert_array_equal(st["rng"][:, 1], d["reset_rng_lead"][:, 0])
    reset_steps = list(d["reset_step"][0])
    for t in range(S):
        info = env.alloc_info()
        obs, rew, tr, fo = env.step(torch.from_numpy(d["actions"][:, t]).cuda(), want_f64=True, info=info)
        h = {k: _np(v) for k, v in info.items()}
        for fk, ik in INFO_MAP.items():
            if fk == "lost_sales":
                np.testing.assert_allclose(h[ik], d[fk][:, t], rtol=1e-9, atol=1e-9, err_msg=f"{name} t={t} {fk}")
            else:
                np.testing.assert_array_equal(h[ik], d[fk][:, t], err_msg=f"{name} t={t} {fk}")
        for c, ck in enumerate(COST_KEYS):
            np.testing.assert_allclose(h["costs"][:, c], d[ck][:, t], rtol=1e-9, atol=1e-7, err_msg=f"{name} t={t} {ck}")
        np.testing.assert_allclose(_np(env.rewards_f64), d["rewards"][:, t], rtol=0, atol=REW_ATOL)
        np.testing.assert_allclose(_np(rew), d["rewards"][:, t].astype(np.float32), rtol=1e-6, atol=1e-5)
        trn = _np(tr).astype(bool)
        assert np.array_equal(trn, d["trunc"][:, t])
        np.testing.assert_array_equal(_np(fo) if trn.any() else _np(obs), d["obs"][:, t], err_msg=f"{name} t={t} obs")
        if trn.any() and (t + 1) in reset_steps:
            np.testing.assert_array_equal(_np(obs), d["reset_obs"][:, reset_steps.index(t + 1)])
        if not trn.any():
            st = env.read_state()
            np.testing.assert_array_equal(st["inventory"], d["inv_after"][:, t])
            np.testing.assert_array_equal(st["rng"][:, 0], d["rng_demand"][:, t])
            np.testing.assert_array_equal(st["rng"][:, 1], d["rng_lead"][:, t])
    env.check()


def _lockstep(spec, E, steps, seed=0, base_seed=777, check_every=1):
    env = _vec(spec, E, base_seed=base_seed)
    ref = orc.OracleEnv(spec, E, base_seed=base_seed)
    np.testing.assert_array_equal(_np(env.reset()), ref.reset())
    rng = np.random.default_rng(seed)
    for t in range(steps):
        a = rng.uniform(-1, 1, size=(E, spec.W, spec.K)).astype(np.float32)
        og, _, tg, fg = env.step(torch.from_numpy(a).cuda(), want_f64=True)
        orr, rr, tr, fr = ref.step(a, final_obs=True, n_threads=8)
        assert np.array_equal(_np(tg).astype(bool), tr)
        np.testing.assert_allclose(_np(env.rewards_f64), rr, rtol=0, atol=REW_ATOL, err_msg=f"t={t}")
        np.testing.assert_array_equal(_np(og), orr, err_msg=f"obs t={t}")
        if tr.any():
            np.testing.assert_array_equal(_np(fg)[tr], fr[tr], err_msg=f"final obs t={t}")
        if t % check_every == 0:
            sg, sr = env.read_state(), ref.read_state()
            np.testing.assert_array_equal(sg["inventory"], sr["inventory"])
            np.testing.assert_array_equal(sg["rng"], sr["rng"])
            np.testing.assert_array_equal(sg["timestep"], sr["timestep"])
    env.check()
    return env, ref


@pytest.mark.usefixtures("alloc_impl_lpe")
def test_bench_config_vs_oracle_across_episode_boundary():
    # BASELINE configs 2-4 shape (8 x 64 x 5), 512 envs, 110 steps (one in-kernel auto-reset)
    cfg = make_synthetic_env_config(8, 64, 5)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    _lockstep(spec, 512, 110, check_every=10)


@pytest.mark.parametrize("form", ["4", "5"])
def test_step_c_forms_vs_oracle(monkeypatch, form):
    # the observation kernel's two register forms (MSC_OPT_STEP_C_FORM / MSC_STEP_C_FORM: 5 waves per
    # SIMD with spills, the env stepping default; 4, the rollout collector's), through the lane
    # allocator and the 16-wave step_c, across an episode boundary
    _set_alloc(monkeypatch, "lane")
    monkeypatch.setenv("MSC_STEP_C_FORM", form)
    cfg = make_synthetic_env_config(8, 64, 5, episode_length=20)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    _lockstep(spec, 256, 45, seed=13, check_every=5)


@pytest.mark.parametrize("split", ["1", "16"])
def test_alloc_prio_split_vs_oracle(monkeypatch, split):
    # alloc_lane's priority drop after split/16 of its orders (MSC_OPT_ALLOC_PRIO_SPLIT; default 12,
    # run by every other lane test): scheduling only, results identical
    _set_alloc(monkeypatch, "lane")
    monkeypatch.setenv("MSC_AL_PRIO_SPLIT", split)
    cfg = make_synthetic_env_config(8, 64, 5, episode_length=20)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    _lockstep(spec, 256, 25, seed=17, check_every=5)


def test_set_option_mid_run_matches_default(monkeypatch):
    # msc_env_set_option between steps (the rollout collector's step_c form 4 and whole-kernel
    # allocation priority) changes no result: two handles on the same seeds, one switched after 7
    # steps, stay bit-identical across an episode boundary; bad keys / values raise
    _set_alloc(monkeypatch, "lane")
    cfg = make_synthetic_env_config(8, 64, 5, episode_length=12)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    a, b = _vec(spec, 192, base_seed=5), _vec(spec, 192, base_seed=5)
    np.testing.assert_array_equal(_np(a.reset()), _np(b.reset()))
    rng = np.random.default_rng(3)
    for t in range(20):
        if t == 7:
            b.set_option(b.STEP_C_FORM, 4)
            b.set_option(b.ALLOC_PRIO_SPLIT, 16)
        if t == 13:
            b.set_option(b.ALLOC_PRIO_SPLIT, 3)
        act = torch.from_numpy(rng.uniform(-1, 1, size=(192, spec.W, spec.K)).astype(np.float32)).cuda()
        oa, _, ta, _ = a.step(act, want_f64=True)
        ob, _, tb, _ = b.step(act, want_f64=True)
        np.testing.assert_array_equal(_np(oa), _np(ob), err_msg=f"obs t={t}")
        np.testing.assert_array_equal(_np(a.rewards_f64), _np(b.rewards_f64), err_msg=f"rewards t={t}")
        np.testing.assert_array_equal(_np(ta), _np(tb))
    for key, val in ((b.ALLOC_PRIO_SPLIT, 0), (b.ALLOC_PRIO_SPLIT, 17), (b.STEP_C_FORM, 3), (99, 1)):
        with pytest.raises(Exception):
            b.set_option(key, val)


@pytest.mark.parametrize("gen,ea", [(1, "0"), (2, "0"), (5, "0"), (7, "0"), (5, "1"), (7, "1")])
def test_demand_generator_waves_vs_oracle(monkeypatch, gen, ea):
    # the Poisson demand kernel with 1 / 2 / 5 / 7 generator waves per 64 envs (MSC_DEMAND_GEN; every
    # other test runs the default 3), per step and episode-ahead, in lockstep with the oracle at the
    # BASELINE 8 x 64 x 5 shape across an episode boundary (5 and 7: A/B instantiations at 5 SKUs)
    monkeypatch.setenv("MSC_DEMAND_GEN", str(gen))
    monkeypatch.setenv("MSC_EA", ea)
    cfg = make_synthetic_env_config(8, 64, 5, episode_length=20)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    _lockstep(spec, 192, 45, seed=gen, check_every=5)


@pytest.mark.usefixtures("alloc_impl_lpe")
def test_c5_shape_vs_oracle():
    cfg = make_synthetic_env_config(16, 256, 5, episode_length=12)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    _lockstep(spec, 64, 15, check_every=5)


def test_c5_bench_geometry_vs_oracle_8192(monkeypatch):
    # BASELINE configs[4] at its stated size, 8,192 envs x 16 x 256 x 5 with an empirical
    # trace of ~200-1,000 orders per step and meanstd observations, through the library's own choice
    # of kernels (what bench.py's c5 line runs: the group allocator over envs sorted by order count,
    # 16-lane groups, 8-wave blocks with the cost tables in LDS, the interleaved wave mapping over 256
    # blocks, phase C inside step_b), in lockstep with the oracle; 4-step episodes put an episode
    # boundary inside steps 4 and 8 (the in-kernel reset and the trace window redraw)
    from marlsc.synthetic import make_synthetic_trace
    for k in ("MSC_ALLOC_IMPL", "MSC_ALLOC_LPE", "MSC_ALLOC_SORT", "MSC_OBS_STAGE", "MSC_OBS_RING_REG", "MSC_FUSE_C",
              "MSC_FUSE_A", "MSC_EA", "MSC_SB_GW", "MSC_SB_TAB"):
        monkeypatch.delenv(k, raising=False)
    cfg = make_synthetic_env_config(16, 256, 5, episode_length=4)
    cfg["components"]["demand_sampler"] = {"type": "empirical", "params": None}
    meta = {"include_warehouse_id": True, "demand_trace": make_synthetic_trace(256, 5, 300, orders_per_step=(200, 1000), seed=0)}
    nf = EnvSpec.from_config(cfg, meta).n_features
    g = np.random.default_rng(21)
    meta.update(obs_normalization="meanstd_custom",
                obs_stats=(g.uniform(-2, 30, nf).astype(np.float32), g.uniform(0.5, 12, nf).astype(np.float32)))
    spec = EnvSpec.from_config(cfg, meta)
    probe = _vec(spec, 8192, base_seed=777)
    kc = probe.kernel_choice()
    probe.close()
    assert kc["alloc"] == 1 and kc["alloc_sort"] == 1 and kc["fuse_c"] == 1, kc
    assert kc["group_width"] == 16 and kc["group_tables_lds"] == 1, kc
    _lockstep(spec, 8192, 11, seed=8, check_every=2)


@pytest.mark.parametrize("name", ["c8_split", "variant_a", "variant_b", "variant_c", "repo_3wh5sku"])
@pytest.mark.usefixtures("alloc_impl")
def test_variants_vs_oracle_many_envs(name):
    d, meta = load(name)
    _lockstep(spec_of(d, meta), 300, 70, seed=3, check_every=7)


def test_generate_demand_split_equals_fused():
    cfg = make_synthetic_env_config(8, 64, 5)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    a, b = _vec(spec, 256, base_seed=5), _vec(spec, 256, base_seed=5)
    a.reset(), b.reset()
    rng = np.random.default_rng(1)
    side = torch.cuda.Stream()
    for t in range(30):
        act = torch.from_numpy(rng.uniform(-1, 1, (256, 8, 5)).astype(np.float32)).cuda()
        oa = a.step(act)[0].clone()
        with torch.cuda.stream(side):
            b.generate_demand()
        torch.cuda.current_stream().wait_stream(side)
        ob = b.step(act)[0]
        assert torch.equal(oa, ob)


def test_sharding_invariance():
    # env g has the same trajectory whether it lives in one batch or in a shard (global env ids)
    cfg = make_synthetic_env_config(8, 64, 5, episode_length=15)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    full = _vec(spec, 128, base_seed=99)
    lo = _vec(spec, 64, base_seed=99, env_index_offset=0)
    hi = _vec(spec, 64, base_seed=99, env_index_offset=64)
    full.reset(), lo.reset(), hi.reset()
    rng = np.random.default_rng(2)
    for _ in range(20):
        act = torch.from_numpy(rng.uniform(-1, 1, (128, 8, 5)).astype(np.float32)).cuda()
        of = full.step(act)[0].clone()
        ol = lo.step(act[:64].contiguous())[0].clone()
        oh = hi.step(act[64:].contiguous())[0].clone()
        assert torch.equal(of, torch.cat([ol, oh]))


@pytest.mark.parametrize("n_ranks", [2, 4, 8])
def test_strong_sharding_matches_one_rank_32768(n_ranks):
    # BASELINE configs[3]: 32,768 envs in total, rank g of N owning global env ids
    # [g * E / N, (g + 1) * E / N) (bench.py --scaling strong). Each shard steps the same trajectories
    # as the one-rank handle over all 32,768 envs although the library picks other kernels per shard
    # size (lane allocator + per-step demand at >= 16,384 envs; scan allocator + episode-ahead demand
    # at <= 8,192), across two episode boundaries
    E = 32768
    cfg = make_synthetic_env_config(8, 64, 5, episode_length=15)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    full = _vec(spec, E, base_seed=77)
    n = E // n_ranks
    shards = [_vec(spec, n, base_seed=77, env_index_offset=g * n) for g in range(n_ranks)]
    of = full.reset().clone()
    for g, sh in enumerate(shards):
        assert torch.equal(sh.reset(), of[g * n:(g + 1) * n])
    gen = torch.Generator(device="cuda").manual_seed(5)
    for _ in range(40):
        act = torch.rand((E, 8, 5), generator=gen, device="cuda") * 2 - 1
        o, r = (x.clone() for x in full.step(act)[:2])
        for g, sh in enumerate(shards):
            os_, rs = sh.step(act[g * n:(g + 1) * n].contiguous())[:2]
            assert torch.equal(os_, o[g * n:(g + 1) * n]) and torch.equal(rs, r[g * n:(g + 1) * n])
    for x in [full] + shards:
        x.check()
        x.close()


def test_save_load_state_roundtrip():
    d, meta = load("variant_b")
    env = _vec(spec_of(d, meta), 64, base_seed=3)
    env.reset()
    rng = np.random.default_rng(4)
    acts = [torch.from_numpy(rng.uniform(-1, 1, (64, env.W, env.K)).astype(np.float32)).cuda() for _ in range(12)]
    for a in acts[:4]:
        env.step(a)
    blob = env.save_state()
    first = [env.step(a)[0].clone() for a in acts[4:]]
    env.load_state(blob)
    second = [env.step(a)[0].clone() for a in acts[4:]]
    for x, y in zip(first, second):
        assert torch.equal(x, y)


def test_masked_reset_and_root_seeds():
    d, meta = load("c1_2x4x2")
    spec = spec_of(d, meta)
    env = _vec(spec, 8, base_seed=11)
    ref = orc.OracleEnv(spec, 8, base_seed=11)
    env.reset(), ref.reset()
    rng = np.random.default_rng(5)
    for _ in range(3):
        a = rng.uniform(-1, 1, (8, spec.W, spec.K)).astype(np.float32)
        env.step(torch.from_numpy(a).cuda())
        ref.step(a)
    mask = np.array([1, 0, 1, 0, 0, 0, 0, 1], np.uint8)
    seeds = np.arange(8, dtype=np.uint32) * 1000 + 17
    og = _np(env.reset(mask=torch.from_numpy(mask).cuda(), root_seeds=torch.from_numpy(seeds.astype(np.int64)).cuda()))
    orr = ref.reset(mask=mask, new_root_seeds=seeds)
    np.testing.assert_array_equal(og[mask == 1], orr[mask == 1])
    for _ in range(5):
        a = rng.uniform(-1, 1, (8, spec.W, spec.K)).astype(np.float32)
        o1 = _np(env.step(torch.from_numpy(a).cuda())[0])
        o2, _, _, _ = ref.step(a)
        np.testing.assert_array_equal(o1, o2)


def test_obs_flat_layout():
    d, meta = load("c3_8x64x5")
    spec = spec_of(d, meta)
    env = _vec(spec, 3, env_seeds=meta["env_seeds"])
    env.reset()
    env.step(torch.from_numpy(d["actions"][:, 0]).cuda())
    loc = _np(env.obs)
    flat = _np(env.obs_flat())
    for w in range(spec.W):
        np.testing.assert_array_equal(flat[:, w, :spec.local_obs_dim], loc[:, w])
        np.testing.assert_array_equal(flat[:, w, spec.local_obs_dim:], loc.reshape(3, -1))


@pytest.mark.parametrize("N", [5000, 4998])  # vectorised (4 sequences per lane) and scalar kernels
def test_gae_kernel_vs_numpy(N):
    import ctypes as C
    from gae_ref import gae, normalize
    from marlsc import abi
    rng = np.random.default_rng(0)
    T = 100
    r = rng.normal(size=(T, N)).astype(np.float32)
    v = rng.normal(size=(T + 1, N)).astype(np.float32)
    nv = rng.normal(size=(T, N)).astype(np.float32)
    te = (rng.random((T, N)) < 0.01).astype(np.uint8)
    tr = np.zeros((T, N), np.uint8)
    tr[49] = 1
    dev = {k: torch.from_numpy(x).cuda() for k, x in dict(r=r, v=v, nv=nv, te=te, tr=tr).items()}
    adv = torch.empty((T, N), device="cuda")
    tgt = torch.empty((T, N), device="cuda")
    stats = torch.zeros(3, dtype=torch.float64, device="cuda")
    p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    abi.check(abi.lib().msc_gae(p(dev["r"]), p(dev["v"]), p(dev["nv"]), p(dev["te"]), p(dev["tr"]), N, T,
                                C.c_float(0.99), C.c_float(0.95), p(adv), p(tgt), p(stats), None))
    a_ref, t_ref = gae(r.astype(np.float64), v.astype(np.float64), nv.astype(np.float64), te, tr, 0.99, 0.95)
    np.testing.assert_allclose(_np(adv), a_ref, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(_np(tgt), t_ref, rtol=1e-4, atol=1e-4)
    s = _np(stats)
    assert s[2] == T * N
    np.testing.assert_allclose(s[0], a_ref.sum(), rtol=1e-5)
    abi.check(abi.lib().msc_adv_normalize(p(adv), T * N, p(stats), None))
    np.testing.assert_allclose(_np(adv), normalize(a_ref), rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("groups", [1, 8])
def test_grouped_gae_statistics_vs_numpy(groups):
    # per-module standardisation (RLlib's GAE connector, one module per agent when not sharing):
    # sequence n = env * W + agent belongs to group n % W; agents get different advantage scales
    import ctypes as C
    from gae_ref import gae, normalize_grouped
    from marlsc import abi
    rng = np.random.default_rng(1)
    T, W, E = 40, 8, 300
    N = E * W
    scale = np.tile(np.arange(1, W + 1, dtype=np.float32) ** 2, E)  # agent w's rewards x (w+1)^2
    r = (rng.normal(size=(T, N)) * scale + scale).astype(np.float32)
    v = rng.normal(size=(T + 1, N)).astype(np.float32)
    nv = rng.normal(size=(T, N)).astype(np.float32)
    te = np.zeros((T, N), np.uint8)
    tr = np.zeros((T, N), np.uint8)
    tr[17] = 1
    dev = {k: torch.from_numpy(x).cuda() for k, x in dict(r=r, v=v, nv=nv, te=te, tr=tr).items()}
    adv = torch.empty((T, N), device="cuda")
    tgt = torch.empty((T, N), device="cuda")
    stats = torch.zeros((groups, 3), dtype=torch.float64, device="cuda")
    p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    abi.check(abi.lib().msc_gae_grouped(p(dev["r"]), p(dev["v"]), p(dev["nv"]), p(dev["te"]), p(dev["tr"]), N, T,
                                        C.c_float(0.99), C.c_float(0.95), p(adv), p(tgt), groups, p(stats), None))
    a_ref, _ = gae(r.astype(np.float64), v.astype(np.float64), nv.astype(np.float64), te, tr, 0.99, 0.95)
    s = _np(stats)
    for g in range(groups):
        assert s[g, 2] == T * N // groups
        np.testing.assert_allclose(s[g, 0], a_ref[:, g::groups].sum(), rtol=1e-5)
        np.testing.assert_allclose(s[g, 1], (a_ref[:, g::groups] ** 2).sum(), rtol=1e-5)
    abi.check(abi.lib().msc_adv_normalize_grouped(p(adv), T * N, groups, p(stats), None))
    np.testing.assert_allclose(_np(adv), normalize_grouped(a_ref, groups), rtol=1e-3, atol=1e-3)
    # an n_groups that does not divide the sequence count is refused, not silently misread
    with pytest.raises(RuntimeError):
        abi.check(abi.lib().msc_gae_grouped(p(dev["r"]), p(dev["v"]), p(dev["nv"]), p(dev["te"]), p(dev["tr"]), N, T,
                                            C.c_float(0.99), C.c_float(0.95), p(adv), p(tgt), 7, p(stats), None))


def test_pettingzoo_adapter_matches_golden():
    from marlsc.env import InventoryEnvironment
    d, meta = load("repo_3wh5sku")
    env_meta = dict(meta["env_meta"])
    env = InventoryEnvironment(meta["config"], seed=meta["env_seeds"][0], env_meta=env_meta)
    env.collect_step_info = True
    obs, _ = env.reset()
    L = env._compute_local_obs_dim()
    np.testing.assert_array_equal(np.stack([obs[a][:L] for a in env.agents]), d["reset_obs"][0, 0])
    for t in range(meta["n_steps"]):
        acts = {a: d["actions"][0, t, i] for i, a in enumerate(env.agents)}
        obs, rew, term, trunc, infos = env.step(acts)
        np.testing.assert_array_equal(np.stack([obs[a][:L] for a in env.agents]), d["obs"][0, t])
        np.testing.assert_allclose([rew[a] for a in env.agents], d["rewards"][0, t], atol=REW_ATOL, rtol=0)
        np.testing.assert_array_equal(infos[env.agents[0]]["shipment_quantities_by_sku"], d["shipment_quantities_by_sku"][0, t])
        assert obs[env.agents[0]].shape == env.observation_space(env.agents[0]).shape
        if trunc[env.agents[0]]:
            obs, _ = env.reset()


def test_pipelined_equals_sequential_across_resets_and_checkpoints():
    # demand of step t+1 generated on the side stream behind step t must not change any result,
    # across episode boundaries, masked resets and save/load with pending demand
    cfg = make_synthetic_env_config(8, 64, 5, episode_length=7)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    a, b = _vec(spec, 256, base_seed=21), _vec(spec, 256, base_seed=21)
    b.set_pipelining(False)
    a.reset(), b.reset()
    rng = np.random.default_rng(9)
    acts = [torch.from_numpy(rng.uniform(-1, 1, (256, 8, 5)).astype(np.float32)).cuda() for _ in range(40)]
    for t, act in enumerate(acts):
        if t == 11:
            m = torch.zeros(256, dtype=torch.uint8, device="cuda")
            m[::3] = 1
            a.reset(mask=m), b.reset(mask=m)
        if t == 23:
            blob = a.save_state()
            oa_ref = [a.step(x)[0].clone() for x in acts[23:27]]
            a.load_state(blob)
            ob_ref = [a.step(x)[0].clone() for x in acts[23:27]]
            for x, y in zip(oa_ref, ob_ref):
                assert torch.equal(x, y)
            a.load_state(blob)
        oa = a.step(act)[0].clone()
        ob = b.step(act)[0].clone()
        assert torch.equal(oa, ob), f"step {t}"
        assert torch.equal(a.rewards, b.rewards)
    sa, sb = a.read_state(), b.read_state()
    assert np.array_equal(sa["rng"], sb["rng"])  # reported as of before the demand generated ahead
    assert np.array_equal(sa["inventory"], sb["inventory"])


def test_launch_timing_counts_and_results_unchanged(monkeypatch):
    # msc_env_set_timing (bench.py's roofline durations) only adds events: same results, one
    # demand + one step launch timed per step while enabled, nothing after max_steps (per-step
    # demand; episode-ahead generation is timed per episode launch: test_episode_ahead_...)
    monkeypatch.setenv("MSC_EA", "0")
    cfg = make_synthetic_env_config(4, 8, 3, episode_length=5)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    a, b = _vec(spec, 128, base_seed=3), _vec(spec, 128, base_seed=3)
    a.reset(), b.reset()
    a.set_timing(6)
    rng = np.random.default_rng(4)
    for t in range(9):
        act = torch.from_numpy(rng.uniform(-1, 1, (128, 4, 3)).astype(np.float32)).cuda()
        assert torch.equal(a.step(act)[0], b.step(act)[0]), f"step {t}"
        assert torch.equal(a.rewards, b.rewards)
    tm = a.read_timing()
    assert tm["n_step"] == 6 and tm["n_demand"] == 6
    assert tm["step_ms"] > 0 and tm["demand_ms"] > 0
    a.set_timing(0)
    assert a.read_timing()["n_step"] == 0


@pytest.mark.parametrize("W,R,K,lo,p,lq,lost", [
    (1, 1, 1, 0.3, 0.1, 0.2, "closest"),     # mostly empty regions and orders
    (2, 3, 8, 9.5, 0.95, 9.9, "cost"),       # max SKUs (a mask unit spans every uniform of a
                                             # round) and rates near the multiplication method's
                                             # limit: long units, many carried products
    (16, 9, 4, 6.0, 0.5, 7.5, "shipment"),   # widest group (16 warehouses per env)
    (12, 7, 3, 4.0, 0.6, 5.0, "closest"),    # masked warehouse slots (12 of 16; 3 of 4 per lane)
    (24, 11, 12, 3.0, 0.6, 4.0, "cost"),     # past the 16 x 8 shapes: 32-lane groups (24 of 32),
                                             # warehouse waves looping, the sequential sampler
    (32, 6, 16, 2.0, 0.5, 3.0, "shipment"),  # the caps: 32 warehouses, 16 SKUs
    (20, 5, 9, 1.5, 0.7, 2.0, "closest"),
])
@pytest.mark.usefixtures("alloc_impl_lpe")
def test_demand_and_allocation_edges_vs_oracle(W, R, K, lo, p, lq, lost):
    cfg = make_synthetic_env_config(W, R, K, episode_length=15, lambda_orders=lo, probability_skus=p,
                                    lambda_quantity=lq, lost_sales=lost)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    _lockstep(spec, 192, 32, seed=11, check_every=4)


@pytest.mark.parametrize("W,K,dev,scope", [(24, 12, [0, 1, 2, 3] * 3, "team"), (17, 10, 2, "agent"),
                                           (8, 5, [1, 0, 2, 1, 3], "agent")])
def test_wide_stochastic_leads_all_features_vs_oracle(W, K, dev, scope):
    # stochastic lead times past 16 warehouses (step_a's warehouse loop; every actual lead time is
    # written by the per-env RNG wave), all observation features with aggregates (K > 8: numpy's
    # 8-accumulator f32 sums), ratio normalisation, cost lost sales
    cfg = make_synthetic_env_config(W, 9, K, episode_length=14, features={k: True for k in FEATURE_CONFIG_YAML},
                                    lost_sales="cost",
                                    scope=scope)
    cfg["components"]["lead_time_sampler"] = {"type": "stochastic", "params": {
        "expected_lead_times": [[1 + (w + k) % 4 for k in range(K)] for w in range(W)],
        "deviation": {"type": "uniform", "max_deviation": dev}}}
    cfg["initial_inventory"] = {"type": "uniform", "params": {"min": 5, "max": 60}}
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True, "obs_normalization": "ratio"})
    _lockstep(spec, 130, 30, seed=21, check_every=3)


@pytest.mark.parametrize("lost", ["shipment", "closest"])
@pytest.mark.usefixtures("alloc_impl")
def test_shared_home_regions_vs_oracle(lost):
    # n_regions < n_warehouses: several warehouses share a home region (multi_env.py:144), which
    # takes the allocation kernel's LDS shipped-home path; home-region features are observed
    feats = dict(FEATURE_CONFIG_YAML, units_shipped_home=True, incoming_demand_home=True, stockout=True)
    cfg = make_synthetic_env_config(8, 4, 3, episode_length=20, features=feats, lost_sales=lost)
    homes = np.argmin(np.array(cfg["cost_structure"]["distances"]), axis=1)
    assert len(set(homes.tolist())) < len(homes), "config must share home regions"
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    _lockstep(spec, 192, 25, seed=8, check_every=4)


def test_home_features_and_group_allocator_agree(monkeypatch):
    # the lane-per-env allocator (default) and the group-per-env one (MSC_ALLOC_IMPL=group) on the
    # bench shape with every home-region feature observed, against the oracle
    feats = dict(FEATURE_CONFIG_YAML, units_shipped_home=True, incoming_demand_home=True,
                 units_shipped_away=True, stockout=True)
    cfg = make_synthetic_env_config(8, 64, 5, episode_length=30, features=feats)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    monkeypatch.setenv("MSC_ALLOC_IMPL", "lane")
    _lockstep(spec, 128, 12, seed=9, check_every=3)
    monkeypatch.setenv("MSC_ALLOC_IMPL", "group")
    _lockstep(spec, 128, 12, seed=9, check_every=3)


def test_gae_vectorised_equals_scalar():
    # the two GAE kernels do the same f32 arithmetic per element: advantages / targets bit-equal
    import ctypes as C
    import os
    from marlsc import abi
    rng = np.random.default_rng(5)
    T, N = 37, 4096
    dev = {"r": rng.normal(size=(T, N)), "v": rng.normal(size=(T + 1, N)), "nv": rng.normal(size=(T, N))}
    dev = {k: torch.from_numpy(x.astype(np.float32)).cuda() for k, x in dev.items()}
    dev["te"] = torch.from_numpy((rng.random((T, N)) < 0.05).astype(np.uint8)).cuda()
    tr = np.zeros((T, N), np.uint8)
    tr[11] = 1
    tr[20, ::3] = 1
    dev["tr"] = torch.from_numpy(tr).cuda()
    p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    outs = []
    for scalar in (False, True):
        if scalar:
            os.environ["MSC_GAE_SCALAR"] = "1"
        try:
            adv, tgt = torch.empty((T, N), device="cuda"), torch.empty((T, N), device="cuda")
            st = torch.zeros(3, dtype=torch.float64, device="cuda")
            abi.check(abi.lib().msc_gae(p(dev["r"]), p(dev["v"]), p(dev["nv"]), p(dev["te"]), p(dev["tr"]), N, T,
                                        C.c_float(0.99), C.c_float(0.95), p(adv), p(tgt), p(st), None))
            torch.cuda.synchronize()
            outs.append((adv.clone(), tgt.clone(), st.clone()))
        finally:
            os.environ.pop("MSC_GAE_SCALAR", None)
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    np.testing.assert_allclose(_np(outs[0][2]), _np(outs[1][2]), rtol=1e-12)


@pytest.mark.parametrize("W,R,lost", [(16, 256, "shipment"), (3, 5, "cost")])
@pytest.mark.usefixtures("alloc_impl_lpe")
def test_empirical_trace_demand_vs_oracle(W, R, lost):
    # EmpiricalDemandSampler (demand_sampler.py:214-261): per-episode window start drawn from the
    # demand stream, one trace timestep per step from the CSR trace, across two episode
    # boundaries; BASELINE configs[4] shape (16 x 256 x 5) with ~200-1,000 orders per step.
    # Pinned to the C oracle's restatement (no reference fixture covers this sampler: SURVEY 8(c)).
    from marlsc.synthetic import make_synthetic_trace
    cfg = make_synthetic_env_config(W, R, 5, episode_length=6, lost_sales=lost)
    cfg["components"]["demand_sampler"] = {"type": "empirical", "params": None}
    trace = make_synthetic_trace(R, 5, 25, orders_per_step=(200, 1000) if R > 64 else (2, 12), seed=W)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True, "demand_trace": trace})
    _lockstep(spec, 96, 14, seed=4, check_every=3)


@pytest.mark.parametrize("slots,batch,chunk", [(4, 1, 10), (4, 2, 2), (6, 2, 4), (16, 4, 3)])
def test_episode_ahead_equals_sequential(monkeypatch, slots, batch, chunk):
    # episode-ahead demand (whole future episodes drawn on a side stream)
    # against per-step sequential demand: identical observations, rewards and reported state
    # (PCG64 demand stream included) across episode boundaries, save/load in the middle of a
    # generated episode, a full reset mid-episode, a masked reset and episode-counter rewrites;
    # refills of `batch` slots per generation, generated in chunks of `chunk` steps (6-step episodes)
    monkeypatch.setenv("MSC_EA", "1")
    monkeypatch.setenv("MSC_EA_SLOTS", str(slots))
    monkeypatch.setenv("MSC_EA_BATCH", str(batch))
    monkeypatch.setenv("MSC_EA_CHUNK", str(chunk))
    monkeypatch.setenv("MSC_ALLOC_IMPL", "scan")
    cfg = make_synthetic_env_config(8, 64, 5, episode_length=6)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    E = 192
    a, b = _vec(spec, E, base_seed=31), _vec(spec, E, base_seed=31)
    b.set_pipelining(False)
    a.reset(), b.reset()
    rng = np.random.default_rng(12)
    acts = [torch.from_numpy(rng.uniform(-1, 1, (E, 8, 5)).astype(np.float32)).cuda() for _ in range(90)]
    a.set_timing(200)
    seen_active = False
    for t, act in enumerate(acts):
        if t == 27:  # step 3 of a generated episode
            assert a.read_timing_ea()["active"]
            blob = a.save_state()
            first = [a.step(x)[0].clone() for x in acts[27:30]]
            a.load_state(blob)
            second = [a.step(x)[0].clone() for x in acts[27:30]]
            for x, y in zip(first, second):
                assert torch.equal(x, y)
            a.load_state(blob)
        if t == 40:
            a.reset(), b.reset()
        if t == 58:
            cnt = np.arange(E, dtype=np.int32) % 3
            a.set_episode_counters(cnt), b.set_episode_counters(cnt)
        if t == 75:
            m = torch.zeros(E, dtype=torch.uint8, device="cuda")
            m[::5] = 1
            a.reset(mask=m), b.reset(mask=m)
        oa = a.step(act)[0].clone()
        ob = b.step(act)[0].clone()
        assert torch.equal(oa, ob), f"step {t}"
        assert torch.equal(a.rewards, b.rewards), f"step {t}"
        seen_active |= a.read_timing_ea()["active"]
        if t % 4 == 1:
            sa, sb = a.read_state(), b.read_state()
            for k in ("rng", "inventory", "timestep", "episode_counter"):
                assert np.array_equal(sa[k], sb[k]), f"{k} at step {t}"
    assert seen_active
    tm = a.read_timing_ea()
    assert tm["slots"] == slots and tm["n_ea"] > 0 and tm["ea_ms"] > 0
    a.check()
    b.check()


def test_episode_ahead_memory_budget_binds_and_stays_exact(monkeypatch):
    # the episode-ahead buffers take at most ea_mem_fraction of the free device
    # memory; here the budget holds ~3.5 slots, so the handle runs with 3 slots (reported by
    # msc_env_dims), allocates within the budget, and stays bit-exact with per-step demand
    monkeypatch.delenv("MSC_EA", raising=False)
    monkeypatch.delenv("MSC_EA_SLOTS", raising=False)
    monkeypatch.setenv("MSC_ALLOC_IMPL", "scan")
    cfg = make_synthetic_env_config(8, 64, 5, episode_length=6)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    E = 192
    m = float(spec.lambda_orders.sum()) * 6
    cap = int(np.ceil(m + 12.0 * np.sqrt(m + 1.0) + 64.0))
    slot_bytes = 16 * cap * E + 4 * 7 * E + 4 * 6 * E + 4 * E
    free, _ = torch.cuda.mem_get_info()
    a = _vec(spec, E, base_seed=31, ea_mem_fraction=3.5 * (slot_bytes + 1024) / free)
    b = _vec(spec, E, base_seed=31, episode_ahead=0)
    mem = a.ea_memory()
    assert b.ea_slots == 0 and b.ea_memory()["allocated"] == 0
    assert a.ea_slots in (2, 3), mem
    assert 0 < mem["allocated"] <= mem["budget"], mem
    b.set_pipelining(False)
    a.reset(), b.reset()
    rng = np.random.default_rng(5)
    seen_active = False
    for t in range(60):
        act = torch.from_numpy(rng.uniform(-1, 1, (E, 8, 5)).astype(np.float32)).cuda()
        oa = a.step(act)[0].clone()
        ob = b.step(act)[0].clone()
        assert torch.equal(oa, ob), f"step {t}"
        assert torch.equal(a.rewards, b.rewards), f"step {t}"
        seen_active |= a.read_timing_ea()["active"]
    sa, sb = a.read_state(), b.read_state()
    for k in ("rng", "inventory", "timestep", "episode_counter"):
        assert np.array_equal(sa[k], sb[k]), k
    assert seen_active
    a.check()
    b.check()


@pytest.mark.parametrize("E,W,K", [(1, 6, 4), (63, 6, 4), (1000, 6, 4), (63, 16, 5), (130, 13, 6), (70, 11, 2)])
def test_scan_allocator_vs_oracle_sizes(monkeypatch, E, W, K):
    # the scan allocator (4 envs per block; a partial last block) and episode-ahead demand at odd
    # env counts against the oracle, with max_splits limiting the warehouses per order; 9-16
    # warehouses: 16-lane SKU groups, two SKU slots per lane above 4 SKUs
    monkeypatch.setenv("MSC_ALLOC_IMPL", "scan")
    monkeypatch.setenv("MSC_EA", "1")
    cfg = make_synthetic_env_config(W, 20, K, episode_length=5)
    cfg["components"]["demand_allocator"]["params"]["max_splits"] = 1 if W < 9 else 3
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    _lockstep(spec, E, 17, seed=E, check_every=2)


def test_poisson_ptrs_device_known_answers():
    # numpy's PTRS branch (lam >= 10) on the device (msc_poisson_draws runs the env's own sampler,
    # rng.hpp poisson_any_g): 100,000 draws per rate and a stream cycling rates across both branches,
    # against Generator.poisson (tests/golden/make_ptrs_vectors.py, numpy only); draws and final
    # PCG64 states bit-exact
    import ctypes as C
    from pathlib import Path
    from marlsc import abi
    g = np.load(Path(__file__).resolve().parent / "golden" / "poisson_ptrs.npz")
    streams = [(g[f"init_{i}"], np.array([lam]), g[f"draws_{i}"], g[f"final_{i}"]) for i, lam in enumerate(g["rates"])]
    streams.append((g["init_mix"], g["mix_rates"], g["draws_mix"], g["final_mix"]))
    for init, lam, draws, final in streams:
        st = np.ascontiguousarray(init, dtype=np.uint64)
        lam = np.ascontiguousarray(lam, dtype=np.float64)
        out = np.empty(draws.size, dtype=np.int64)
        fin = np.empty(6, dtype=np.uint64)
        abi.check(abi.lib().msc_poisson_draws(st.ctypes.data_as(C.c_void_p), lam.ctypes.data_as(C.c_void_p), lam.size,
                                              out.size, out.ctypes.data_as(C.c_void_p), fin.ctypes.data_as(C.c_void_p)))
        bad = np.flatnonzero(out != draws.astype(np.int64))
        assert bad.size == 0, f"lam={lam}: first mismatch at draw {bad[:5]}"
        assert np.array_equal(fin, final)


@pytest.mark.parametrize("ea", ["0", "1"])
@pytest.mark.parametrize("lo,lq", [(4.0, 12.0), (11.0, 3.0)])
def test_ptrs_rates_env_vs_oracle(monkeypatch, ea, lo, lq):
    # Poisson rates >= 10 (numpy's PTRS branch) in the env, quantities
    # (lambda_q = 12) or order counts (lambda_o = 11), against the oracle in lockstep, with
    # per-step and episode-ahead demand (the sequential sampler, csrc/demand_ab.hip)
    monkeypatch.setenv("MSC_EA", ea)
    cfg = make_synthetic_env_config(4, 16, 3, episode_length=7, lambda_orders=lo, lambda_quantity=lq)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    _lockstep(spec, 96, 17, seed=4, check_every=2)


@pytest.mark.parametrize("ea", ["0", "1"])
def test_split_parser_demand_vs_oracle(monkeypatch, ea):
    # the split chain / bookkeeper demand parser (MSC_DEMAND_IMPL=ab, csrc/demand_ab.hip; an A/B
    # variant, measured slower than the default unit parser) against the oracle, per step and episode-ahead
    monkeypatch.setenv("MSC_DEMAND_IMPL", "ab")
    monkeypatch.setenv("MSC_EA", ea)
    cfg = make_synthetic_env_config(8, 64, 5, episode_length=9)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    _lockstep(spec, 192, 21, seed=6, check_every=4)


@pytest.mark.parametrize("impl", ["v3", "unit"])
@pytest.mark.parametrize("ea", ["0", "1"])
def test_demand_v3_vs_oracle(monkeypatch, ea, impl):
    # the short-round unit parser (csrc/demand_v3.hip, the default for equal sampler parameters) and
    # the unit parser it replaced (MSC_DEMAND_IMPL=unit: its constant-threshold form stays under test),
    # per step and episode-ahead (4-step chunks continue from the recorded stream position and record
    # count), in lockstep with the oracle
    monkeypatch.setenv("MSC_DEMAND_IMPL", impl)
    monkeypatch.setenv("MSC_EA", ea)
    monkeypatch.setenv("MSC_EA_CHUNK", "4")
    cfg = make_synthetic_env_config(8, 64, 5, episode_length=9)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    env, _ = _lockstep(spec, 192, 21, seed=9, check_every=4)
    assert env.kernel_choice()["demand_impl"] == (9 if impl == "v3" else 0)


@pytest.mark.parametrize("ea", ["0", "1"])
@pytest.mark.parametrize("band,quota", [(None, None), ("3", None), (None, "8"), (None, "40")])
def test_demand_v2_vs_oracle(monkeypatch, ea, band, quota):
    # the f32-ring demand kernel (csrc/demand_v2.hip): f32 draws with the SKU draw in the sign bit, a
    # 128-position ring, the f32 Poisson chain decided outside a band around exp(-lambda) and the exact
    # recomputation (jump-ahead + numpy's f64 chain) inside it; per step and episode-ahead, in lockstep
    # with the oracle across episode boundaries. band 2^-3 sends a large share of the Poisson rounds
    # through the exact path; quota 8 / 40 exercise the generators' top-up barrier and a full ring
    monkeypatch.setenv("MSC_DEMAND_IMPL", "v2")
    monkeypatch.setenv("MSC_EA", ea)
    if band:
        monkeypatch.setenv("MSC_V2_BAND", band)
    if quota:
        monkeypatch.setenv("MSC_V2_QUOTA", quota)
    cfg = make_synthetic_env_config(8, 64, 5, episode_length=9)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    env, _ = _lockstep(spec, 192, 21, seed=7, check_every=4)
    assert env.kernel_choice()["demand_impl"] == 8


@pytest.mark.parametrize("impl", ["v2", "v3"])
@pytest.mark.parametrize("K,lo,lq,p", [(1, 4.0, 5.0, 0.667), (3, 2.5, 9.5, 0.3), (8, 1.5, 9.9, 1.0), (6, 9.9, 0.4, 0.9)])
def test_demand_v2_shapes_and_rates_vs_oracle(monkeypatch, impl, K, lo, lq, p):
    # the f32-ring kernel (v2) at other SKU counts and rates: lambda 9.5-9.9 (units past 24 draws,
    # decided exactly), p = 1 (every SKU drawn: the integer bound ceil(p 2^53) = 2^53), tiny quantity
    # rates; the same shapes through the short-round unit parser (v3, csrc/demand_v3.hip)
    monkeypatch.setenv("MSC_DEMAND_IMPL", impl)
    cfg = make_synthetic_env_config(5, 24, K, episode_length=7, lambda_orders=lo, lambda_quantity=lq,
                                    probability_skus=p)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    env, _ = _lockstep(spec, 130, 16, seed=K, check_every=3)
    assert env.kernel_choice()["demand_impl"] == (8 if impl == "v2" else 9)


@pytest.mark.parametrize("impl", ["v2", "v3"])
@pytest.mark.usefixtures("alloc_impl")
def test_demand_v2_bench_shape_vs_oracle(monkeypatch, impl):
    # BASELINE configs[2] shape with every allocation kernel, 512 envs, 110 steps (one auto-reset)
    monkeypatch.setenv("MSC_DEMAND_IMPL", impl)
    cfg = make_synthetic_env_config(8, 64, 5)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    _lockstep(spec, 512, 110, seed=11, check_every=10)


def test_episode_ahead_runtime_switch_stays_exact(monkeypatch):
    # msc_env_set_episode_ahead: episode-ahead demand switched off mid-episode (per-step pipelined
    # demand from that step on) and back on (restarting at the next common episode start) leaves
    # every observation, reward and state bit-exact with per-step demand; the step_c staging / chain
    # priority patched on each switch change nothing either
    monkeypatch.setenv("MSC_ALLOC_IMPL", "lane")
    for k in ("MSC_EA", "MSC_EA_SLOTS", "MSC_OBS_STAGE", "MSC_OBS_RING_REG"):
        monkeypatch.delenv(k, raising=False)
    cfg = make_synthetic_env_config(8, 64, 5, episode_length=6)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    E = 160
    a = _vec(spec, E, base_seed=41, episode_ahead=4)
    b = _vec(spec, E, base_seed=41, episode_ahead=0)
    assert a.ea_slots == 4 and b.ea_slots == 0
    a.reset(), b.reset()
    rng = np.random.default_rng(9)
    on = 0
    for t in range(70):
        if t == 20:
            a.set_episode_ahead(False)
        if t == 33:
            a.set_episode_ahead(True)
        act = torch.from_numpy(rng.uniform(-1, 1, (E, 8, 5)).astype(np.float32)).cuda()
        oa = a.step(act)[0].clone()
        ob = b.step(act)[0].clone()
        assert torch.equal(oa, ob), f"step {t}"
        assert torch.equal(a.rewards, b.rewards), f"step {t}"
        on += int(a.read_timing_ea()["active"])
        if t % 5 == 2:
            sa, sb = a.read_state(), b.read_state()
            for k in ("rng", "inventory", "timestep", "episode_counter"):
                assert np.array_equal(sa[k], sb[k]), f"{k} at step {t}"
    assert on > 20
    a.check()
    b.check()


@pytest.mark.parametrize("lost", ["shipment", "cost", "closest"])
@pytest.mark.parametrize("shape", [(8, 64, 5), (3, 7, 2), (16, 64, 5), (12, 9, 6), (9, 70, 3)])
def test_scan_allocator_lost_sales_handlers_vs_oracle(monkeypatch, lost, shape):
    # the scan allocator's deferred lost-sales shares (shipment / cost softmax, flushed after the order
    # loop in region order; csrc/alloc_scan.hip flush_lost) and the inline closest handler, without
    # step info (the deferred path), against the oracle: rewards 1e-6, observations / state bit-exact;
    # low inventories so most regions lose orders, more lost regions than one flush holds at 8 x 64
    monkeypatch.setenv("MSC_ALLOC_IMPL", "scan")
    W, R, K = shape
    cfg = make_synthetic_env_config(W, R, K, episode_length=11, lost_sales=lost, initial_inventory=8)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    _lockstep(spec, 130, 24, seed=17, check_every=3)


@pytest.mark.parametrize("W,K", [(16, 5), (10, 6)])
def test_scan_allocator_wide_step_info_vs_group(monkeypatch, W, K):
    # collect_step_info through the scan kernel's instrumented epilogue at 16-lane SKU groups (two
    # slots per lane): every info key equal to the group kernel's on the same seeds (the golden
    # fixtures pin the group kernel's infos to the reference at <= 8 warehouses)
    cfg = make_synthetic_env_config(W, 12, K, episode_length=9, lost_sales="shipment", initial_inventory=15)
    spec = EnvSpec.from_config(cfg, {"include_warehouse_id": True})
    outs = []
    for impl in ("group", "scan"):
        monkeypatch.setenv("MSC_ALLOC_IMPL", impl)
        env = _vec(spec, 40, base_seed=5)
        env.reset()
        rng = np.random.default_rng(2)
        rec = []
        for t in range(12):
            a = torch.from_numpy(rng.uniform(-1, 1, (40, W, K)).astype(np.float32)).cuda()
            info = env.alloc_info()
            env.step(a, info=info, want_f64=True)
            rec.append({k: _np(v).copy() for k, v in info.items()} | {"rew": _np(env.rewards_f64).copy()})
        env.check()
        outs.append(rec)
    for t, (g, sc) in enumerate(zip(*outs)):
        for k in g:
            if k in ("lost_sales", "costs", "rew"):
                np.testing.assert_allclose(sc[k], g[k], rtol=0, atol=1e-9, err_msg=f"{k} t={t}")
            else:
                np.testing.assert_array_equal(sc[k], g[k], err_msg=f"{k} t={t}")

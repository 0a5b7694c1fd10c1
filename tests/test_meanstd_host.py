"""CPU tests of obs_normalization "meanstd" (RLlib's running MeanStdFilter connector, the reference's
src/algorithms/mappo.py:170-171): the numpy restatement (oracle/meanstd_ref.py) pinned against
numpy's own statistics, the host-side merge / synchronisation of marlsc/obs_filter.py against it,
and the world_size-2 synchronisation over gloo. RLlib itself is not installed: parity with RLlib is
unpinned; the device kernel is checked against the oracle in tests/test_gpu_rollout.py."""
import os
import socket
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "oracle"))
sys.path.insert(0, str(REPO / "marl-sc_amd"))

from meanstd_ref import MeanStdFilter, RunningStat, filter_rows, synchronize  # noqa: E402


def _rs_of(x):
    rs = RunningStat(x.shape[1:])
    for row in x:
        rs.push(row)
    return rs


def test_running_stat_matches_numpy_statistics():
    x = np.random.default_rng(0).normal(5.0, 3.0, (2000, 7))
    rs = _rs_of(x)
    np.testing.assert_allclose(rs.M, x.mean(0), rtol=1e-12)
    np.testing.assert_allclose(rs.var, x.var(0, ddof=1), rtol=1e-10)
    one = _rs_of(x[:1])
    np.testing.assert_array_equal(one.var, x[0] ** 2)  # RLlib's single-push variance: M^2


def test_running_stat_merge_equals_the_concatenation():
    x = np.random.default_rng(1).normal(-2.0, 0.5, (900, 5))
    a, b = _rs_of(x[:400]), _rs_of(x[400:])
    a.update(b)
    whole = _rs_of(x)
    assert a.n == whole.n == 900
    np.testing.assert_allclose(a.M, whole.M, rtol=1e-12)
    np.testing.assert_allclose(a.S, whole.S, rtol=1e-10)
    e = RunningStat((5,))
    e.update(RunningStat((5,)))  # empty + empty stays empty
    assert e.n == 0


def test_filter_normalises_after_its_own_push_and_clips():
    f = MeanStdFilter((3,))
    rows = np.array([[1.0, 2.0, 3.0], [3.0, 2.0, 1.0], [100.0, 2.0, -50.0]], np.float32)
    out = filter_rows(f, rows)
    # first row: mean = row, var = M^2 -> 0 / (|x| + eps)
    np.testing.assert_array_equal(out[0], np.zeros(3, np.float32))
    m2 = rows[:2].astype(np.float64).mean(0)
    sd2 = rows[:2].astype(np.float64).std(0, ddof=1)
    np.testing.assert_allclose(out[1], ((rows[1] - m2) / (sd2 + 1e-6)).astype(np.float32), rtol=1e-6)
    assert np.all(np.abs(out) <= 10.0)
    before = f.rs.n
    filter_rows(f, rows, update=False)
    assert f.rs.n == before
    filter_rows(f, rows, mask=np.array([1, 0, 1]))
    assert f.rs.n == before + 2


def test_host_merge_matches_the_oracle_update():
    import torch
    from marlsc.obs_filter import merge_stats
    rng = np.random.default_rng(2)
    a, b = _rs_of(rng.normal(0, 1, (50, 4))), _rs_of(rng.normal(3, 2, (70, 4)))
    pa = torch.from_numpy(np.concatenate([[a.n], a.M, a.S]))
    pb = torch.from_numpy(np.concatenate([[b.n], b.M, b.S]))
    got = merge_stats(pa, pb).numpy()
    a.update(b)
    np.testing.assert_array_equal(got, np.concatenate([[a.n], a.M, a.S]))


def _lane_state(rs_run, rs_buf, C):
    st = np.zeros(4 + 4 * C)
    st[0], st[1] = rs_run.n, rs_buf.n
    st[4:4 + C], st[4 + C:4 + 2 * C] = rs_run.M, rs_run.S
    st[4 + 2 * C:4 + 3 * C], st[4 + 3 * C:] = rs_buf.M, rs_buf.S
    return st


def _sync_worker(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, str(REPO / "marl-sc_amd"))
    from marlsc.obs_filter import MeanStdObsFilter
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    C = 6
    f = MeanStdObsFilter(C, "cpu", n_lanes=2)
    rng = np.random.default_rng(100 + rank)
    for li in range(2):
        buf = _rs_of(rng.normal(rank + li, 1.0 + li, (30 + 10 * li, C)))
        f.lanes[li].copy_(torch.from_numpy(_lane_state(buf, buf, C)))
    f.sync()
    np.save(Path(out_dir) / f"d{rank}.npy", f.driver.numpy())
    np.save(Path(out_dir) / f"l{rank}.npy", torch.stack(f.lanes).numpy())
    dist.destroy_process_group()


def test_filter_sync_world2_gloo_folds_buffers_in_rank_lane_order(tmp_path):
    import torch.multiprocessing as mp
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    mp.spawn(_sync_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    C = 6
    runners = []
    for rank in range(2):
        rng = np.random.default_rng(100 + rank)
        for li in range(2):
            f = MeanStdFilter((C,))
            f.buffer = _rs_of(rng.normal(rank + li, 1.0 + li, (30 + 10 * li, C)))
            runners.append(f)
    driver = synchronize(RunningStat((C,)), runners)
    want = np.concatenate([[driver.n], driver.M, driver.S])
    for rank in range(2):
        d = np.load(tmp_path / f"d{rank}.npy")
        np.testing.assert_array_equal(d, want)
        lanes = np.load(tmp_path / f"l{rank}.npy")
        for st in lanes:  # every lane continues from the driver's statistics with an empty buffer
            assert st[0] == driver.n and st[1] == 0
            np.testing.assert_array_equal(st[4:4 + 2 * C], np.concatenate([driver.M, driver.S]))
            assert not st[4 + 2 * C:].any()

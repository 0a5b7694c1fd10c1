"""TEST INFRASTRUCTURE ONLY: numpy restatement of RLlib's running observation filter, the
`obs_normalization: "meanstd"` mode of the reference (src/algorithms/mappo.py:170-171,
ippo.py:173-175: `MeanStdFilter(multi_agent=True)` env-to-module connector; evaluation calls
`filter(obs, update=False)`, base.py:131-140, :176-177).

RLlib (ray==2.52.1, reference requirements.txt:81) is neither vendored nor installed here: PARITY
UNPINNED against RLlib itself. This restates ray.rllib.utils.filter as published:
  RunningStat.push(x): n += 1; n == 1: M = x; else delta = x - M; M += delta / n;
                       S += delta * delta * (n - 1) / n               (Welford)
  RunningStat.update(other): Chan et al.'s merge of (n, M, S)
  var = S / (n - 1) if n > 1 else M^2; std = sqrt(var)
  MeanStdFilter(x, update): push x (if update), then clip((x - M) / (std + 1e-6), -10, 10)
and the connector's order of pushes per env step: every env's observation in env order, one
RunningStat per agent and feature (multi_agent=True keeps a filter per agent id). The filter also
keeps a `buffer` RunningStat of the pushes since the last synchronisation; synchronising folds every
runner's buffer into the driver's statistics (RunningStat.update, runner order) and copies them back.
The statistics themselves are pinned by tests against numpy's own mean / var (ddof=1)."""
import numpy as np

SMALL_NUMBER = 1e-6
CLIP = 10.0


class RunningStat:
    def __init__(self, shape):
        self.n = 0
        self.M = np.zeros(shape, np.float64)
        self.S = np.zeros(shape, np.float64)

    def push(self, x):
        x = np.asarray(x, np.float64)
        self.n += 1
        if self.n == 1:
            self.M[...] = x
        else:
            delta = x - self.M
            self.M[...] += delta / self.n
            self.S[...] += delta * delta * (self.n - 1) / self.n

    def update(self, other):
        n1, n2 = float(self.n), float(other.n)
        n = n1 + n2
        if n == 0:
            return
        delta = self.M - other.M
        delta2 = delta * delta
        m = (n1 * self.M + n2 * other.M) / n
        s = self.S + other.S + (delta2 / n) * n1 * n2
        self.n = int(n)
        self.M, self.S = m, s

    @property
    def var(self):
        return self.S / (self.n - 1) if self.n > 1 else np.square(self.M)

    @property
    def std(self):
        return np.sqrt(self.var)

    def copy(self):
        r = RunningStat(self.M.shape)
        r.n, r.M, r.S = self.n, self.M.copy(), self.S.copy()
        return r


class MeanStdFilter:
    """One filter over the columns of an observation row (an agent's features): rs + buffer."""

    def __init__(self, shape, clip=CLIP, eps=SMALL_NUMBER):
        self.rs, self.buffer = RunningStat(shape), RunningStat(shape)
        self.clip, self.eps = clip, eps

    def __call__(self, x, update=True):
        x = np.asarray(x)
        if update:
            self.rs.push(x)
            self.buffer.push(x)
        y = (x.astype(np.float64) - self.rs.M) / (self.rs.std + self.eps)
        if self.clip:
            y = np.clip(y, -self.clip, self.clip)
        return y.astype(np.float32)


def filter_rows(filt: MeanStdFilter, rows, mask=None, update=True):
    """The connector's pass over one step: rows [E, C] in env order (rows with mask 0 skipped when
    updating, still normalised)."""
    out = np.empty(rows.shape, np.float32)
    for e in range(rows.shape[0]):
        out[e] = filt(rows[e], update=update and (mask is None or bool(mask[e])))
    return out


def synchronize(driver: RunningStat, runner_filters):
    """FilterManager.synchronize: the driver's stats absorb every runner's buffer (in order); each
    runner then continues from the driver's stats with an empty buffer."""
    for f in runner_filters:
        driver.update(f.buffer)
    for f in runner_filters:
        f.rs = driver.copy()
        f.buffer = RunningStat(driver.M.shape)
    return driver

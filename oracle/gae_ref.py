"""TEST INFRASTRUCTURE ONLY: numpy restatement of the advantage estimation the rollout uses.

The reference delegates GAE to RLlib 2.52.1 (not vendored, not installed: parity unpinned
against RLlib itself). This restates the textbook GAE(gamma, lambda) with RLlib's conventions:
terminated -> bootstrap 0, truncated -> bootstrap V(terminal obs), value targets = A + V,
then (A - mean) / max(1e-4, std) over each module's batch: the whole batch for one shared policy,
every agent's column (sequence n % W) on its own for one policy per agent."""
import numpy as np


def gae(rewards, values, next_values, terminated, truncated, gamma, lam):
    """rewards/terminated/truncated/next_values: [T, N]; values: [T+1, N]. float64 math."""
    T, N = rewards.shape
    adv = np.zeros((T, N), np.float64)
    a = np.zeros(N, np.float64)
    v_next = values[T].astype(np.float64)
    for t in range(T - 1, -1, -1):
        te = terminated[t].astype(bool)
        tr = truncated[t].astype(bool)
        boot = np.where(tr, next_values[t], v_next)
        boot = np.where(te, 0.0, boot)
        delta = rewards[t] + gamma * boot - values[t]
        a = delta + np.where(te | tr, 0.0, gamma * lam * a)
        adv[t] = a
        v_next = values[t].astype(np.float64)
    return adv, adv + values[:T]


def normalize(adv):
    return (adv - adv.mean()) / max(1e-4, adv.std())


def normalize_grouped(adv, groups):
    """adv [T, N]; sequence n standardised with the statistics of group n % groups."""
    out = np.empty_like(adv, dtype=np.float64)
    for g in range(groups):
        out[:, g::groups] = normalize(adv[:, g::groups])
    return out

"""Replay of batched-trainer rollouts through the C oracle (test infrastructure).

The trainer records (actions, reward64, done, status) per tick when ``tr._trace`` is a
list; every sampled env's layout (as assigned, in the reference's list format) is set on
an oracle env, reset, and driven by the same actions, with the reference's reset
between attempts (environment.py:183-214: headings carry over).  Rewards are compared
as float64 bit patterns, done and status exactly.
"""
import numpy as np

from oracle import pyoracle as po

STATUS = {"running": 0, "detected": 1, "vault_reached": 2, "timeout": 3, "already_done": 4}


def oracle_envs(tr, env_ids):
    cfg = tr.config
    envs = []
    for e, lay in zip(env_ids, tr.layout_lists(env_ids)):
        budget = tr.b_meta[int(e)][1]
        o = po.OracleEnv(cfg.grid_rows, cfg.grid_cols, cfg.max_steps, cfg.start_pos, cfg.vault_pos, budget)
        o.set_layout(*lay)
        o.reset()
        envs.append(o)
    return envs


def replay(tr, env_ids, trace, envs=None):
    """Drive oracle envs through trace rows; returns the number of env-steps compared."""
    envs = envs if envs is not None else oracle_envs(tr, env_ids)
    ids = np.asarray(env_ids, np.int64)
    n = 0
    for t, (a, r64, done, status) in enumerate(trace):
        a, r64, done, status = (x.cpu().numpy() for x in (a, r64, done, status))
        for j, e in enumerate(ids):
            r, d, s = envs[j].step(int(a[e]))
            assert r64[e] == r, "env %d tick %d: reward %r != oracle %r" % (e, t, r64[e], r)
            assert bool(done[e]) == bool(d), "env %d tick %d: done" % (e, t)
            assert int(status[e]) == int(s), "env %d tick %d: status %d != %d" % (e, t, status[e], s)
            if d:
                envs[j].reset()
            n += 1
    return n

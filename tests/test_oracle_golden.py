"""Pin the CPU oracle (oracle/heist_oracle.c) against the reference's golden vectors.

The oracle is the checker the GPU path is compared with on the GPU box, so it
must first reproduce the Python reference exactly on every fixture the
reference produced here (tests/golden/make_golden.py).
"""
import numpy as np
import pytest

import golden_data as gd
from oracle import pyoracle as po

STATUS_RESET = 5


def _replay(tr):
    env = po.OracleEnv(tr["R"], tr["C"], tr["max_steps"], tr["start"], tr["vault"], tr["budget"])
    valid = env.set_layout(tr["walls"], tr["cams"], tr["guards"])
    return env, valid


@pytest.mark.parametrize("tr", list(gd.env_traces()), ids=lambda t: t["name"])
def test_env_trace_bit_exact(tr):
    env, valid = _replay(tr)
    assert valid == tr["valid"]
    np.testing.assert_array_equal(env.grid(), tr["grid"])
    inf = env.info()
    assert [inf["n_walls"], inf["n_cams"], inf["n_guards"], inf["spent"]] == tr["accepted"]
    for k, op in enumerate(tr["ops"]):
        if op == -1:
            env.reset()
            r, d, st = 0.0, bool(env.info()["done"]), STATUS_RESET
        else:
            r, d, st = env.step(op)
        inf = env.info()
        ctx = "%s op#%d" % (tr["name"], k)
        assert r == tr["reward"][k], ctx  # float64, bit-exact
        assert d == tr["done"][k], ctx
        assert st == tr["status"][k], ctx
        assert (inf["pos_r"], inf["pos_c"]) == tuple(tr["pos"][k]), ctx
        assert inf["tick"] == tr["tick"][k], ctx
        ch, gi, gh = env.headings()
        np.testing.assert_array_equal(ch, tr["cam_h"][k], err_msg=ctx)
        np.testing.assert_array_equal(gi, tr["g_idx"][k], err_msg=ctx)
        np.testing.assert_array_equal(gh, tr["g_h"][k], err_msg=ctx)
        np.testing.assert_array_equal(env.visibility().astype(bool), tr["vis"][k], err_msg=ctx)
        if k < len(tr["state"]):
            s = env.state_tensor()
            assert s.tobytes() == tr["state"][k].tobytes(), ctx


def test_cones_bit_exact():
    n = 0
    for c in gd.cones():
        kind = 1 if c["kind"] == 2 else 0
        got = po.cone(kind, c["walls"], c["row"], c["col"], c["fov"], c["heading"], c["range"])
        np.testing.assert_array_equal(got, c["tiles"], err_msg=str({k: c[k] for k in ("kind", "row", "col", "fov", "heading", "range")}))
        n += 1
    assert n >= 1000


def test_cone_order_fixture_sets_match_oracle():
    """cone_order.npz's ordered lists hold exactly the oracle's visible tiles, each once
    (the order itself is pinned on the GPU by test_cone_order_matches_reference_list)."""
    n = 0
    for c in gd.cone_orders():
        got = po.cone(c["kind"], c["walls"], c["row"], c["col"], c["fov"], c["heading"], c["range"])
        assert len(set(c["order"])) == len(c["order"])
        want = np.zeros((c["R"], c["C"]), bool)
        for r, cc in c["order"]:
            want[r, cc] = True
        np.testing.assert_array_equal(got, want)
        n += 1
    assert n == 600


def test_bfs_matches_reference():
    n = 0
    for c in gd.bfs_cases():
        assert po.bfs(c["grid"], c["start"], c["goal"]) == c["valid"]
        n += 1
    assert n >= 1000


def test_gae_matches_reference():
    z = gd.load("ppo.npz")
    for i in range(int(z["n_gae"])):
        adv = po.gae(z["gae%d_r" % i], z["gae%d_v" % i], z["gae%d_d" % i])
        np.testing.assert_allclose(adv, z["gae%d_adv" % i], rtol=0, atol=1e-5)


def test_ppo_loss_matches_reference():
    z = gd.load("ppo.npz")
    for i in range(int(z["n_loss"])):
        g = lambda k: z["loss%d_%s" % (i, k)]  # noqa: E731
        parts, dl, dv = po.ppo_loss(g("logits"), g("values"), g("actions"), g("old"), g("adv"), g("ret"))
        assert abs(parts[1] - float(g("pg"))) < 1e-4
        assert abs(parts[2] - float(g("vl"))) < 1e-4
        assert abs(parts[3] - float(g("ent"))) < 1e-4
        np.testing.assert_allclose(dl, g("dlogits"), rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(dv, g("dvalues"), rtol=1e-4, atol=1e-6)


def test_reference_kats():
    kat = gd.load_json("kat.json")
    env = po.OracleEnv(10, 10, 200, (1, 1), (8, 8), 15)
    s = kat["sanity"]
    assert env.set_layout([(3, 3), (3, 4), (3, 5)],
                          [{"row": 5, "col": 5, "fov_angle": 60, "heading": 0, "rotation_speed": 15, "vision_range": 4}],
                          [{"patrol_path": [(7, 2), (7, 3), (7, 4), (7, 5)], "speed": 1, "vision_range": 3,
                            "fov_angle": 90}]) == s["valid"]
    env.reset()
    rews = []
    for _ in range(5):
        r, d, st = env.step(4)
        rews.append(r)
        if d:
            break
    assert rews == s["rewards"]
    assert po.STATUS_NAMES[st] == s["status"]
    assert int(env.visibility().sum()) == s["surveilled"]
    env = po.OracleEnv(10, 10)
    env.set_layout([], [], [])
    env.reset()
    tot = 0.0
    for _ in range(7):
        tot += env.step(2)[0]
    assert tot == kat["fixes_down"]
    for _ in range(7):
        r, d, st = env.step(4)
        tot += r
        if d:
            break
    assert tot == kat["fixes_right"] and po.STATUS_NAMES[st] == kat["fixes_status"]
    env.reset()
    st = env.state_tensor()
    assert float(st[2].min()) == kat["pos_channel_min"] and float(st[2].max()) == kat["pos_channel_max"]

"""Loaders for the golden fixtures in tests/golden/ (data made by make_golden.py)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def load_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def env_traces():
    """Yield one dict per recorded trace (layout in the reference's list/dict form)."""
    z = load("env_traces.npz")
    cfg = z["cfg"]
    n = len(cfg)
    grid_off = 0
    op_cursor = 0
    cam_cursor = 0
    g_cursor = 0
    vis_cursor = 0
    st_cursor = 0
    n_state = int(z["n_state"])
    for t in range(n):
        R, C, ms, sr, sc, vr, vc, budget = (int(x) for x in cfg[t])
        walls = [tuple(int(v) for v in w) for w in z["walls"][z["walls_off"][t]:z["walls_off"][t + 1]]]
        cams = [dict(row=int(c[0]), col=int(c[1]), fov_angle=float(c[2]), heading=float(c[3]),
                     rotation_speed=float(c[4]), vision_range=int(c[5]))
                for c in z["cams"][z["cams_off"][t]:z["cams_off"][t + 1]]]
        guards = []
        for gi, gf in zip(z["guards_i"][z["guards_off"][t]:z["guards_off"][t + 1]],
                          z["guards_fov"][z["guards_off"][t]:z["guards_off"][t + 1]]):
            off, ln, spd, rng = (int(x) for x in gi)
            guards.append(dict(patrol_path=[tuple(int(v) for v in p) for p in z["paths"][off:off + ln]],
                               speed=spd, vision_range=rng, fov_angle=float(gf)))
        ops = z["ops"][z["ops_off"][t]:z["ops_off"][t + 1]].astype(int)
        n_ops = len(ops)
        acc = [int(x) for x in z["accepted"][t]]
        nc, ng = acc[1], acc[2]
        rc = R * C
        nbytes = (rc + 7) // 8
        vis = np.unpackbits(z["vis_bits"][vis_cursor:vis_cursor + n_ops * nbytes].reshape(n_ops, nbytes), axis=1)[:, :rc]
        ns = min(n_state, n_ops)
        state = z["state"][st_cursor:st_cursor + ns * 3 * rc].reshape(ns, 3, R, C)
        sl = slice(op_cursor, op_cursor + n_ops)
        yield dict(
            name=str(z["names"][t]), R=R, C=C, max_steps=ms, start=(sr, sc), vault=(vr, vc), budget=budget,
            walls=walls, cams=cams, guards=guards, valid=bool(z["valid"][t]),
            grid=z["grid"][grid_off:grid_off + rc].reshape(R, C), accepted=acc, ops=ops,
            reward=z["reward"][sl], done=z["done"][sl], status=z["status"][sl], pos=z["pos"][sl].astype(int),
            tick=z["tick"][sl], cam_h=z["cam_h"][cam_cursor:cam_cursor + n_ops * nc].reshape(n_ops, nc),
            g_idx=z["g_idx"][g_cursor:g_cursor + n_ops * ng].reshape(n_ops, ng),
            g_h=z["g_h"][g_cursor:g_cursor + n_ops * ng].reshape(n_ops, ng),
            vis=vis.reshape(n_ops, R, C).astype(bool), state=state)
        grid_off += rc
        op_cursor += n_ops
        cam_cursor += n_ops * nc
        g_cursor += n_ops * ng
        vis_cursor += n_ops * nbytes
        st_cursor += ns * 3 * rc


def cones():
    z = load("cones.npz")
    wcur = tcur = 0
    for (kind, R, C, r, c, rng), (fov, head) in zip(z["meta"], z["params"]):
        nb = (int(R) * int(C) + 7) // 8
        walls = np.unpackbits(z["walls"][wcur:wcur + nb])[:R * C].reshape(R, C).astype(bool)
        tiles = np.unpackbits(z["tiles"][tcur:tcur + nb])[:R * C].reshape(R, C).astype(bool)
        wcur += nb
        tcur += nb
        yield dict(kind=int(kind), R=int(R), C=int(C), row=int(r), col=int(c), range=int(rng), fov=float(fov),
                   heading=float(head), walls=walls, tiles=tiles)


def cone_orders():
    """cone_order.npz: per case the emitter, walls and the reference's ordered tile list."""
    z = load("cone_order.npz")
    wcur = ocur = 0
    for (kind, R, C, r, c, rng), (fov, head), n in zip(z["meta"], z["params"], z["lens"]):
        nb = (int(R) * int(C) + 7) // 8
        walls = np.unpackbits(z["walls"][wcur:wcur + nb])[:R * C].reshape(R, C).astype(bool)
        wcur += nb
        order = [(int(i) // int(C), int(i) % int(C)) for i in z["order"][ocur:ocur + int(n)]]
        ocur += int(n)
        yield dict(kind=int(kind), R=int(R), C=int(C), row=int(r), col=int(c), range=int(rng), fov=float(fov),
                   heading=float(head), walls=walls, order=order)


def bfs_cases():
    z = load("bfs.npz")
    cur = 0
    for (R, C, sr, sc, gr, gc), v in zip(z["meta"], z["valid"]):
        g = z["grids"][cur:cur + R * C].reshape(R, C)
        cur += R * C
        yield dict(grid=g, start=(int(sr), int(sc)), goal=(int(gr), int(gc)), valid=bool(v))

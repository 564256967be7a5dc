"""Canonical board-state records and digests -- TEST INFRASTRUCTURE ONLY.

One byte layout shared by the golden generator (which reads the reference's
board objects), the oracle and the GPU export (``td_export_state``), so that a
state can be compared bit for bit through a sha256.  Floats are packed as IEEE
binary64 (``<d``), so a digest match is a bit-exact match.
"""
import hashlib
import struct

import numpy as np


def digest(b):
    return hashlib.sha256(b).hexdigest()[:32]


def obs_digest(obs):
    a = np.ascontiguousarray(obs, dtype=np.float32)
    return digest(a.tobytes())


def state_bytes(st):
    """``st``: dict with steps, base_LP, cost_def, cost_atk, attacker_cd,
    defender_cd, enemies [(type, lv, r, c, slowdown, LP, margin)],
    towers [(type, lv, r, c, cd)], map6 (L*L ints, row-major)."""
    out = [struct.pack("<qqddqqqq", int(st["steps"]), int(st["base_LP"]), float(st["cost_def"]),
                       float(st["cost_atk"]), int(st["attacker_cd"]), int(st["defender_cd"]),
                       len(st["enemies"]), len(st["towers"]))]
    for (t, lv, r, c, slow, lp, mg) in st["enemies"]:
        out.append(struct.pack("<qqqqqdd", int(t), int(lv), int(r), int(c), int(slow), float(lp), float(mg)))
    for (t, lv, r, c, cd) in st["towers"]:
        out.append(struct.pack("<qqqqd", int(t), int(lv), int(r), int(c), float(cd)))
    out.append(np.asarray(st["map6"], dtype=np.int64).tobytes())
    return b"".join(out)


def state_digest(st):
    return digest(state_bytes(st))


def layout_bytes(map_planes, start, end):
    """Planes 0-5 of TDBoard.map plus start cells and end cell."""
    m = np.asarray(map_planes, dtype=np.int64)[0:6]
    s = np.asarray(start, dtype=np.int64).reshape(-1)
    return m.tobytes() + struct.pack("<q", len(start)) + s.tobytes() + np.asarray(end, dtype=np.int64).tobytes()


def layout_digest(map_planes, start, end):
    return digest(layout_bytes(map_planes, start, end))


def oracle_state(env):
    """Canonical state of an ``oracle.td_oracle.Env``."""
    b = env._board
    return {
        "steps": b.steps, "base_LP": b.base_LP, "cost_def": b.cost_def, "cost_atk": b.cost_atk,
        "attacker_cd": env.attacker_cd, "defender_cd": env.defender_cd,
        "enemies": [(e.type, e.lv, e.loc[0], e.loc[1], e.slowdown, e.LP, e.margin) for e in b.enemies],
        "towers": [(t.type, t.lv, t.loc[0], t.loc[1], t.cd) for t in b.towers],
        "map6": b.map[6].reshape(-1).tolist(),
    }


def fhex(x):
    return float(x).hex()

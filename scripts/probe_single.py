"""Diagnostic: wall time per step of the single-env drop-in classes (B = 1 engine)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gym-td_amd"))
import numpy as np
import gym_TD
for env_id in ("TD-def-small-v0", "TD-atk-small-v0", "TD-2p-small-v0"):
    env = gym_TD.make(env_id, seed=2)
    rng = np.random.RandomState(0)
    acts = []
    for _ in range(600):
        a = env.action_space.sample() if hasattr(env.action_space, "sample") else None
        acts.append(a)
    for a in acts[:50]:
        env.step(a)
    t = time.perf_counter()
    n = 0
    for a in acts[50:]:
        _, _, d, _ = env.step(a)
        n += 1
        if d:
            while True:
                try:
                    env.reset()
                    break
                except RuntimeError:
                    pass
    dt = (time.perf_counter() - t) / n
    print("%s: %.1f us/step" % (env_id, dt * 1e6))
    env.close()

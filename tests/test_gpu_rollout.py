"""The rollout-worker hand-off (BASELINE configs[4] feeds train/PPO's
rollout worker, train/main.py:79-176, PPO/Model.py:134-192, horizon 128 in
train/PPOConfig.json:2): a policy on the GPU reads every step's observation in place
from the engine's own buffer, samples its actions on the device and hands them back as
a device tensor; the worker keeps a rollout buffer (actions, rewards, dones, a digest of
each consumed observation).  Checked against the engine's per-step outputs: a second
engine with the same seeds, stepped with the buffer's actions, reproduces every
consumed observation, reward and done bit for bit, and the per-board episode accounting
(episode_return / episode_length at done, td_episode_records at the end) equals the
buffer's own sums in step order."""
import copy

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU too, so skip cleanly
    pytest.skip("needs a GPU", allow_module_level=True)

from gym_TD import params as P  # noqa: E402
from gym_TD.envs import TDVecEnv  # noqa: E402


def _policy(L, n_act, dev):
    g = torch.Generator(device="cpu").manual_seed(L)
    w1 = (torch.randn(45 * L * L, 64, generator=g) * 0.02).to(dev)
    w2 = (torch.randn(64, n_act, generator=g) * 0.1).to(dev)

    def act(obs, gen):
        h = torch.relu(obs.reshape(obs.shape[0], -1) @ w1)  # reads the engine's buffer, no copy
        probs = torch.softmax(h @ w2, dim=-1)
        return torch.multinomial(probs, 1, generator=gen).squeeze(1)
    return act


def _digest(obs):
    """Per-board digest of an observation (f64 sum of the f32 values times a position
    weight): any changed byte of a board's observation changes it."""
    B = obs.shape[0]
    flat = obs.reshape(B, -1).to(torch.float64)
    w = torch.arange(1, flat.shape[1] + 1, device=obs.device, dtype=torch.float64)
    return (flat * w).sum(1)


@pytest.mark.parametrize("L,B,T,base_LP", [(10, 512, 300, 1), (30, 256, 128, None)])
def test_rollout_worker_handoff(L, B, T, base_LP):
    dev = torch.device("cuda", 0)
    saved = P.config.base_LP
    if base_LP is not None:
        P.config.base_LP = base_LP  # short episodes: accounting checked over several ends
    try:
        env = TDVecEnv(L, B, mode="def", seed=77, device=dev)
        ref = TDVecEnv(L, B, mode="def", seed=77, device=dev)
    finally:
        P.config.base_LP = saved
    n_act = 6 * L * L + 1
    act = _policy(L, n_act, dev)
    gen = torch.Generator(device=dev).manual_seed(3)
    try:
        obs = env.reset()
        ref.reset()
        ptr = obs.data_ptr()
        buf_act = torch.empty((T, B), dtype=torch.int64, device=dev)
        buf_rew = torch.empty((T, B), dtype=torch.float64, device=dev)
        buf_done = torch.empty((T, B), dtype=torch.uint8, device=dev)
        buf_dig = torch.empty((T, B), dtype=torch.float64, device=dev)
        buf_ret = torch.empty((T, B), dtype=torch.float64, device=dev)
        buf_len = torch.empty((T, B), dtype=torch.int32, device=dev)
        with torch.no_grad():
            for k in range(T):
                assert obs.data_ptr() == ptr  # the engine's own buffer, consumed in place
                buf_dig[k] = _digest(obs)
                a = act(obs, gen)
                assert a.is_cuda  # device-side actions straight back into the step
                buf_act[k] = a
                obs, rew, done, infos = env.step(a)
                buf_rew[k], buf_done[k] = rew, done
                buf_ret[k], buf_len[k] = infos["episode_return"], infos["episode_length"]
        # the engine's per-step outputs for the same actions, from a second engine
        for k in range(T):
            assert torch.equal(_digest(ref.engine.obs), buf_dig[k]), k
            o, r, d, _ = ref.step(buf_act[k])
            assert torch.equal(r, buf_rew[k]) and torch.equal(d, buf_done[k]), k
        # episode accounting against the buffer's own sums, in step order (f64, bit-exact)
        rew, done = buf_rew.cpu().numpy(), buf_done.cpu().numpy().astype(bool)
        ret_at, len_at = buf_ret.cpu().numpy(), buf_len.cpu().numpy()
        run = np.zeros(B)
        ln = np.zeros(B, np.int64)
        last = (np.zeros(B), np.zeros(B, np.int64), np.zeros(B, bool))
        for k in range(T):
            run = run + rew[k]
            ln += 1
            d = done[k]
            assert np.array_equal(ret_at[k][d], run[d]) and np.array_equal(len_at[k][d], ln[d]), k
            last[0][d], last[1][d], last[2][d] = run[d], ln[d], True
            run[d], ln[d] = 0.0, 0
        assert done.sum() > 0 or base_LP is None
        r_ret, r_len, r_win = env.engine.episode_records()
        has = last[2]
        assert np.array_equal(r_ret.cpu().numpy()[has], last[0][has])
        assert np.array_equal(r_len.cpu().numpy()[has], last[1][has])
        assert (r_win.cpu().numpy()[~has] == -1).all()
        assert (env.engine.flags() == 0).all()
    finally:
        env.close()
        ref.close()

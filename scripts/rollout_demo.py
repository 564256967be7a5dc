"""Rollout-worker hand-off (BASELINE.json configs[4]'s per-GPU
share): a policy consumes every step's observation straight from the engine's device
buffer (no copy, no host round trip) and feeds its sampled actions back as a device
tensor, PPO-rollout style (train/main.py:79-176 with PPO/Model.py's actor on the GPU).

    python scripts/rollout_demo.py [--map 30] [--boards 16384] [--steps 128]

Prints env-only and env+policy env-steps/s.  The policy is a small random-init conv
actor-critic in bf16 (the trainer is out of scope; this only exercises the hand-off).
A horizon of full 30x30 observations does not fit in HBM at this batch
(128 x 16,384 x 162 KB = 340 GB), so the worker keeps per-step actions, log-probs,
values, rewards and dones (the rollout buffer) and consumes each observation in place.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gym-td_amd"))

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from gym_TD.envs import TDVecEnv  # noqa: E402


class Actor(nn.Module):
    def __init__(self, L, n_actions):
        super().__init__()
        self.body = nn.Sequential(nn.Conv2d(45, 32, 3, padding=1), nn.ReLU(),
                                  nn.Conv2d(32, 32, 3, stride=2, padding=1), nn.ReLU(),
                                  nn.AdaptiveAvgPool2d(4), nn.Flatten(), nn.Linear(32 * 16, 256), nn.ReLU())
        self.pi = nn.Linear(256, n_actions)
        self.v = nn.Linear(256, 1)

    def forward(self, x):
        h = self.body(x)
        return self.pi(h), self.v(h).squeeze(-1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--map", type=int, default=30)
    ap.add_argument("--boards", type=int, default=16384)
    ap.add_argument("--steps", type=int, default=128)
    args = ap.parse_args()
    L, B, T = args.map, args.boards, args.steps
    dev = torch.device("cuda", 0)
    env = TDVecEnv(L, B, mode="def", seed=0, device=dev)
    n_act = 6 * L * L + 1
    net = Actor(L, n_act).to(dev).to(torch.bfloat16)
    obs = env.reset()
    g = torch.Generator(device=dev).manual_seed(0)

    # env only: uniform random actions drawn on the device
    acts = torch.randint(0, n_act, (T, B), device=dev, generator=g)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(T):
        obs, rew, done, infos = env.step(acts[k])
    torch.cuda.synchronize()
    env_only = B * T / (time.perf_counter() - t0)

    # env + policy: the rollout buffer a PPO worker keeps, filled step by step
    buf = {"act": torch.empty((T, B), dtype=torch.int64, device=dev),
           "logp": torch.empty((T, B), dtype=torch.float32, device=dev),
           "val": torch.empty((T, B), dtype=torch.float32, device=dev),
           "rew": torch.empty((T, B), dtype=torch.float64, device=dev),
           "done": torch.empty((T, B), dtype=torch.uint8, device=dev)}
    ptr = obs.data_ptr()
    with torch.no_grad():  # first calls build MIOpen kernels for these shapes: keep them out of the timing
        for _ in range(3):
            torch.distributions.Categorical(logits=net(obs.to(torch.bfloat16))[0].float(), validate_args=False).sample()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.no_grad():
        for k in range(T):
            assert obs.data_ptr() == ptr  # the engine's own buffer: consumed in place
            logits, v = net(obs.to(torch.bfloat16))
            dist = torch.distributions.Categorical(logits=logits.float(), validate_args=False)
            a = dist.sample()
            buf["act"][k], buf["logp"][k], buf["val"][k] = a, dist.log_prob(a), v.float()
            obs, rew, done, infos = env.step(a)
            buf["rew"][k], buf["done"][k] = rew, done
    torch.cuda.synchronize()
    with_policy = B * T / (time.perf_counter() - t0)
    print("map %dx%d, %d boards, %d steps: env only %.1f M env-steps/s, env + policy %.1f M env-steps/s, "
          "%d episodes finished" % (L, L, B, T, env_only / 1e6, with_policy / 1e6, int(buf["done"].sum())))
    env.close()


if __name__ == "__main__":
    main()

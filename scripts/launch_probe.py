"""Where does a per-step launch go?  Host issue cost vs GPU time for ouz_step_n at 4096 envs."""
import sys
import time

import torch

sys.path.insert(0, ".")
from ouzelum_amd import QuadVecTask  # noqa: E402

task = sys.argv[1] if len(sys.argv) > 1 else "LeeLanded"
n = 4096
env = QuadVecTask(task=task, num_envs=n, sim_device="cuda:0", rl_device="cuda:0", seed=1, track_episodes=True)
ring = (torch.rand((16, n, 4), device="cuda") * 2 - 1).contiguous()
env.rollout(ring, 200)
torch.cuda.synchronize()


def wall(fn, steps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e6


S = 2000
print("A step_n only           us/step %.3f" % wall(lambda: [env.rollout(ring, 16) for _ in range(S // 16)], S))
print("B step_n + ep stats     us/step %.3f" % wall(lambda: [(env.rollout(ring, 16), env.episode_stats())
                                                           for _ in range(S // 16)], S))
print("C one call of 2000      us/step %.3f" % wall(lambda: env.rollout(ring, S), S))
# host issue cost with the GPU held busy
torch.cuda._sleep(int(3e8))
t0 = time.perf_counter()
env.rollout(ring, 400)
t1 = time.perf_counter()
torch.cuda.synchronize()
print("D host issue per launch us %.3f" % ((t1 - t0) / 400 * 1e6))
torch.cuda._sleep(int(3e8))
t0 = time.perf_counter()
for _ in range(50):
    env.episode_stats()
t1 = time.perf_counter()
torch.cuda.synchronize()
print("E host episode_stats    us %.3f" % ((t1 - t0) / 50 * 1e6))
x = torch.zeros(16, device="cuda")
torch.cuda._sleep(int(3e8))
t0 = time.perf_counter()
for _ in range(400):
    x.add_(1)
t1 = time.perf_counter()
torch.cuda.synchronize()
print("F host torch add_       us %.3f" % ((t1 - t0) / 400 * 1e6))
print("G torch add_ wall       us %.3f" % wall(lambda: [x.add_(1) for _ in range(2000)], 2000))
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda._sleep(int(2e7))
s.record()
env.rollout(ring, 400)
e.record()
torch.cuda.synchronize()
print("H spin-held kernel      us %.3f" % (s.elapsed_time(e) * 1e3 / 400))
torch.cuda._sleep(int(2e7))
s.record()
for _ in range(400):
    x.add_(1)
e.record()
torch.cuda.synchronize()
print("I spin-held add_        us %.3f" % (s.elapsed_time(e) * 1e3 / 400))

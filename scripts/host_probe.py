"""Host-side cost of one VecTask.step() call, piece by piece (GPU held busy so nothing blocks)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from ouzelum_amd import QuadVecTask  # noqa: E402
from ouzelum_amd import _lib as L  # noqa: E402

n = 4096
env = QuadVecTask(task=sys.argv[1] if len(sys.argv) > 1 else "LeeLanded", num_envs=n, sim_device="cuda:0",
                  rl_device="cuda:0", seed=1)
a = torch.rand((n, 4), device="cuda") * 2 - 1
for _ in range(100):
    env.step(a)
torch.cuda.synchronize()
R = 300


def host(label, fn):
    torch.cuda._sleep(int(3e8))
    t0 = time.perf_counter()
    for _ in range(R):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"{label:34s} {(t1 - t0) / R * 1e6:7.3f} us")


dev = env.device
host("env.step(a)", lambda: env.step(a))
host("current_stream().cuda_stream", lambda: torch.cuda.current_stream(dev).cuda_stream)
host("_cuda_getCurrentRawStream", lambda: torch._C._cuda_getCurrentRawStream(0))
host("_actions_ptr", lambda: env._actions_ptr(a))
s = env._stream()
p = a.data_ptr()
host("lib.ouz_step raw", lambda: L.lib.ouz_step(env._env, p, s))
host("env.rollout(ring,1)", lambda: env.rollout(a[None], 1))

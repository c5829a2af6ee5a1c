"""A/B of two builds of the library at the BASELINE configs: fused 16-step rollout, GPU us per step back to back
(bench.Runner) and, unless OUZ_AB_PER_STEP=0, the one-launch-per-step (VecTask.step) path; rounds interleaved
between the builds (one child process per build and round, the library chosen with OUZ_LIB), and a hash of the
state and observations after the same steps of each path (equal hashes: bitwise-equal results).

    python scripts/exp/lib_ab.py ouzelum_amd/libouzelum_prev.so ouzelum_amd/libouzelum_hip.so [rounds]
"""
import hashlib
import json
import os
import subprocess
import sys

CONFIGS = [("B", "LeeLanded", 4096), ("C", "QuadTracking", 4096), ("D", "QuadFault", 8192), ("E", "QuadMixed", 4096)]
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PER_STEP = os.environ.get("OUZ_AB_PER_STEP", "1") == "1"   # also time the one-launch-per-step path


def child():
    import ctypes

    import torch
    sys.path.insert(0, ROOT)
    import bench as B
    from ouzelum_amd import _lib as L
    from ouzelum_amd.distributed import ReturnAllReduce
    dev = torch.device("cuda", 0)
    cnt = ctypes.c_uint32(0)
    L.check(L.lib.ouz_split_timeouts(ctypes.byref(cnt), 1))
    def state_sha(run):
        torch.cuda.synchronize()
        return hashlib.sha256(run.env.fstate.cpu().numpy().tobytes() + run.env.obs_buf.cpu().numpy().tobytes()
                              ).hexdigest()[:16]

    for letter, task, n in CONFIGS:
        run = B.Runner(task, n, dev, 1234, 0, 1, ReturnAllReduce(dev, batch=1))
        run.rollouts(64)
        fused = run.back_to_back_us(fused=True, launches=40)
        h = state_sha(run)
        rec = {"lib": os.environ["OUZ_LIB"], "config": letter, "task": task, "num_envs": n,
               "fused_us_per_step": round(fused, 3), "state_sha16": h}
        if PER_STEP:   # the VecTask.step path: one quad_step_kernel launch per step, from a fresh env
            del run
            run = B.Runner(task, n, dev, 1234, 0, 1, ReturnAllReduce(dev, batch=1))
            run.rollouts(320, fused=False)   # past the estimator's 300-step convergence window
            rec["step_state_sha16"] = state_sha(run)
            rec["per_step_us"] = round(run.back_to_back_us(fused=False, launches=40), 3)
        print(json.dumps(rec), flush=True)
        del run
    L.check(L.lib.ouz_split_timeouts(ctypes.byref(cnt), 0))
    print(json.dumps({"lib": os.environ["OUZ_LIB"], "multi_wave_timeouts": cnt.value}), flush=True)


def main():
    libs = sys.argv[1:3]
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    for rnd in range(rounds):
        for lib in libs:
            env = dict(os.environ, OUZ_LIB=os.path.abspath(lib), OUZ_LIB_AB_CHILD="1")
            out = subprocess.run([sys.executable, os.path.abspath(__file__)], env=env, capture_output=True, text=True,
                                 timeout=300)
            if out.returncode:
                print(out.stdout + out.stderr, flush=True)
                sys.exit(out.returncode)
            for line in out.stdout.splitlines():
                if line.startswith("{"):
                    d = json.loads(line)
                    d["round"] = rnd
                    print(json.dumps(d), flush=True)


if __name__ == "__main__":
    child() if os.environ.get("OUZ_LIB_AB_CHILD") == "1" else main()

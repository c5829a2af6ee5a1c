"""A/B of two library builds at large N (one child process per build and round, OUZ_LIB): the fused 16-step
rollout (storage + statistics, bench.py's sweep entry) and the per-step kernel, GPU us per step back to back.
    python scripts/archive/large_n_lib_ab.py A.so B.so [rounds] [task:envs ...]
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def child(cases):
    import torch
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "scripts", "exp"))
    import bench as B
    from cls_large_ab import time_env
    dev = torch.device("cuda", 0)
    for task, n in cases:
        n = int(n)
        ring = B.action_ring(n, dev, 1234)
        st = (torch.empty((16, n, 13), device=dev), torch.empty((16, n), device=dev),
              torch.empty((16, n), dtype=torch.int64, device=dev), torch.empty((16, n), dtype=torch.bool, device=dev))
        env = B.make_env(task, n, dev, 1234, 0, n)
        roll, step = time_env(env, n, ring, st)
        print(json.dumps({"lib": os.path.basename(os.environ["OUZ_LIB"]), "task": task, "num_envs": n,
                          "rollout_us_per_step": round(roll, 2), "step_us": round(step, 2)}), flush=True)
        del env, ring, st
        torch.cuda.empty_cache()


def main():
    libs = sys.argv[1:3]
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    cases = sys.argv[4:] or ["QuadTracking:4194304"]
    for rnd in range(rounds):
        for lib in libs:
            env = dict(os.environ, OUZ_LIB=os.path.abspath(lib), OUZ_AB_CHILD="1")
            out = subprocess.run([sys.executable, os.path.abspath(__file__), *cases], env=env, capture_output=True,
                                 text=True, timeout=600)
            if out.returncode:
                print(out.stdout + out.stderr, flush=True)
                sys.exit(out.returncode)
            for line in out.stdout.splitlines():
                if line.startswith("{"):
                    d = json.loads(line)
                    d["round"] = rnd
                    print(json.dumps(d), flush=True)


if __name__ == "__main__":
    child([tuple(c.split(":")) for c in sys.argv[1:]]) if os.environ.get("OUZ_AB_CHILD") == "1" else main()

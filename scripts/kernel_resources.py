"""Register / scratch / occupancy of every kernel of the library (compiler remarks, no GPU needed).

    python scripts/kernel_resources.py [filter]
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ouzelum_amd.build import FLAGS, HIPCC  # noqa: E402


def main():
    flt = sys.argv[1] if len(sys.argv) > 1 else ""
    flags = [f for f in FLAGS if f not in ("-shared", "-fPIC")]
    cmd = [HIPCC, *flags, *os.environ.get("OUZ_EXTRA_FLAGS", "").split(), "--cuda-device-only", "-c",
           os.environ.get("OUZ_SRC") or os.path.join(ROOT, "ouzelum_amd", "csrc", "quad_kernels.hip"), "-o", "/tmp/ouz_res.o",
           "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark:\s+(.*?)(?: \[-Rpass-analysis.*)?$", line)
        if not m:
            continue
        t = m.group(1).strip()
        if t.startswith("Function Name:"):
            cur = {"name": t.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in t:
            k, v = t.split(":", 1)
            cur[k.strip()] = v.strip()
    for r in rows:
        if flt and flt not in r["name"]:
            continue
        print(f"{r['name'][:72]:72s} VGPR {r.get('VGPRs', '?'):>4} AGPR {r.get('AGPRs', '?'):>3} "
              f"SGPR {r.get('SGPRs', '?'):>3} spillS {r.get('SGPRs Spill', '?'):>3} spillV {r.get('VGPRs Spill', '?'):>3} "
              f"scratch {r.get('ScratchSize [bytes/lane]', '?'):>4} occ {r.get('Occupancy [waves/SIMD]', '?'):>2} "
              f"LDS {r.get('LDS Size [bytes/block]', '?'):>6}")


if __name__ == "__main__":
    main()

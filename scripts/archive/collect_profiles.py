"""Copy the rocprofv3 kernel stats and PMC summaries of one tagged GPU run from gpurun_out/
into profiles/<tag>/ (tracked).   python scripts/archive/collect_profiles.py r01"""
import glob
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
out = os.path.join(ROOT, "profiles", tag)
os.makedirs(out, exist_ok=True)
src = os.path.join(ROOT, "gpurun_out")
n = 0
for d in glob.glob(os.path.join(src, f"profall_{tag}_*")):
    if os.path.isdir(d):
        stats = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
        if stats:
            name = os.path.basename(d)[len(f"profall_{tag}_"):]
            shutil.copy(stats[0], os.path.join(out, f"{name}_kernel_stats.csv"))
            n += 1
for f in glob.glob(os.path.join(src, f"pmc_{tag}_*_summary.json")):
    shutil.copy(f, os.path.join(out, os.path.basename(f)))
    n += 1
print(f"{n} files -> {out}")

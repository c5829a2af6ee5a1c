"""The committed roofline / issue evidence belongs to the library the tree builds.

bench.py prices HBM traffic and the issue-bound view only from PMC summaries whose ``lib_sha16`` is the loaded
library's source id (``ouz_source_id()``: sha256 of the kernel sources and flags, ``ouzelum_amd/build.py``).  A
kernel edit without a new evidence run would leave the bench line's ``traffic`` null; this catches it on the CPU.
No GPU: the library loads without one, and the id is a string compiled into it.
"""
import glob
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench as B  # noqa: E402
from ouzelum_amd import build  # noqa: E402

HEADLINE = [("rollout", "LeeLanded", 4096), ("step", "LeeLanded", 4096)]
# every other config at its bench size, and the large-N sweep (scripts/gpu_evidence_r04.sh parts a and b)
OTHERS = [(k, t, n) for t, n in (("QuadTracking", 4096), ("QuadFault", 8192), ("QuadMixed", 4096))
          for k in ("rollout", "step")]
LARGE = [(k, t, n) for n in (4194304, 16777216) for t in ("LeeLanded", "QuadTracking", "QuadFault", "QuadMixed")
         for k in ("rollout", "step")]


def test_tree_sources_match_the_built_library():
    """The in-tree .so was built from these sources (else the evidence checks below say nothing)."""
    assert B.loaded_lib_sha16() == "src-" + build.source_id(), \
        "libouzelum_hip.so is stale: rebuild with __graft_entry__.build()"


@pytest.mark.parametrize("kernel,task,n", HEADLINE + OTHERS + LARGE)
def test_traffic_evidence_of_this_build(kernel, task, n):
    t = B.load_traffic(kernel, task, n)
    assert t is not None and t.get("bytes_per_launch"), f"no PMC summary of this build for {kernel}/{task}/{n}: {t}"
    assert t["rocprof_kernel_us_per_launch"] > 0
    assert os.path.exists(os.path.join(ROOT, t["rocprof_stats"])), t["rocprof_stats"]


@pytest.mark.parametrize("kernel,task,n", HEADLINE + OTHERS)
def test_issue_evidence_of_this_build(kernel, task, n):
    iss = B.load_issue(kernel, task, n)
    assert iss is not None, f"no VALU summary of this build for {kernel}/{task}/{n}"
    assert 0.0 < iss["valu_issue_frac"] < 1.0


def test_committed_bench_line_is_of_this_build():
    """The driver-argument bench line committed with the evidence carries traffic and the issue view."""
    lines = sorted(glob.glob(os.path.join(ROOT, "profiles", "r0*", "bench", "bench_driver_*.jsonl")))
    assert lines
    with open(lines[-1]) as fh:
        d = json.loads(fh.readline())
    assert d["roofline"]["traffic"] and d["roofline"]["issue"]
    assert d["split_timeouts"] == 0
    assert len(json.dumps(d)) < B.LINE_LIMIT


def test_entries_below_the_hbm_bar_name_their_binding():
    """A roofline entry under 0.4 of HBM peak carries the counter-derived bound."""
    e = B.roofline_entry("rollout", "LeeLanded", 4096, 1.62, B.RING)
    assert e["frac"] < 0.4 and e["binding"] == "valu-issue"
    assert B.compact_roofline(e)["binding"] == "valu-issue"
    big = B.roofline_entry("step", "LeeLanded", 4194304, 126.0)
    assert big["frac"] > 0.4 and "binding" not in big
    est = B.roofline_entry("rollout", "QuadTracking", 16777216, 1059.0, B.RING)
    assert est["frac"] < 0.4 and est["binding"] == "valu" and est["issue"]["chip_valu_frac"] > 0.5

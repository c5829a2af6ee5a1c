"""bench.py's stdout line: one compact JSON object the driver can parse (BENCH_r03's 26 KB line was not).

Built here from a full record bench.py wrote on an MI355X (``profiles/r03/bench_driver_args_r03g.json``, the
old one-line form that carried every traffic-detail dict): the compact line must stay under the limit, parse
back, keep the judged fields (headline, roofline with traffic and the rocprof-priced fraction, cpu_baseline
with cores and kind, one row per config) and name the side file that holds the rest.  No GPU.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench as B  # noqa: E402

RECORD = os.path.join(ROOT, "profiles", "r03", "bench_driver_args_r03g.json")


@pytest.fixture(scope="module")
def full():
    with open(RECORD) as fh:
        out = json.load(fh)
    out["split_timeouts"] = 0
    out["detail"] = "gpurun_out/bench_detail.json"
    return out


def test_compact_line_under_limit_and_round_trips(full):
    assert len(json.dumps(full)) > 20000          # the record that broke the driver's parser
    s = B.compact_line(full)
    assert "\n" not in s and len(s) <= B.LINE_LIMIT, len(s)
    d = json.loads(s)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert d[k] == full[k], k
    rf = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "frac_from_rocprof_avg"):
        assert rf[k] == full["roofline"][k], k
    assert rf["rocprof_stats"].startswith("profiles/")
    assert "traffic_detail" not in s
    cpu = d["cpu_baseline"]
    assert cpu["kind"] == "port" and cpu["cores"] == full["cpu_baseline"]["cores"]
    assert cpu["value"] == full["cpu_baseline"]["value"]
    assert len(cpu["by_config"]) == len(full["cpu_baseline"]["table"])
    assert [c["config"] for c in d["configs"]] == [c["config"] for c in full["configs"]]
    for c in d["configs"]:
        assert set(c) >= {"config", "value", "ms_per_step", "dtype", "frac"}
    assert d["detail"] == "gpurun_out/bench_detail.json" and d["split_timeouts"] == 0
    assert any(k.endswith("/16777216") for k in d["large_n"])


def test_cpu_baseline_headline_is_the_f32_host_step(full):
    """"GPU speedup is quoted against timing (2)", the build's own vectorised f32 CPU step -- so
    ``cpu_baseline.value`` is the f32 host row of the bench workload, and the f64 oracle is a secondary entry
    (VERDICT r04 item 3).  B and C carry N = 64 / 4096 / 8192 rows on both legs."""
    runs = B.cpu_baseline_runs("LeeLanded", 4096)
    assert {(t, s) for c, t, s, _, _ in runs if c in "BC"} == {(t, s) for t in ("LeeLanded", "QuadTracking")
                                                                for s in (64, 4096, 8192)}
    row = lambda c, t, s, v, k: {"config": c, "task": t, "num_envs": s, "value": v, "cores": 16, "sample": k}  # noqa
    f32 = [row(c, t, s, 6.6e7 + s, "f32") for c, t, s, _, _ in runs]
    table = [row(c, t, s, 5.4e6 + s, "f64") for c, t, s, _, _ in runs]
    rec = B.cpu_baseline_record("LeeLanded", 4096, 16, "test cpu", f32, table, {"value": 2.2e3})
    assert rec["value"] == 6.6e7 + 4096 and rec["leg"] == "f32_host" and rec["kind"] == "port"
    assert rec["oracle_f64"]["value"] == 5.4e6 + 4096
    d = json.loads(B.compact_line({**full, "cpu_baseline": rec}))
    cpu = d["cpu_baseline"]
    assert cpu["value"] == rec["value"] and cpu["leg"] == "f32_host"
    assert cpu["by_config"]["B/LeeLanded/4096"] == 6.6e7 + 4096 and len(cpu["by_config"]) == len(runs)
    assert cpu["oracle_f64"]["value"] == 5.4e6 + 4096 and len(cpu["oracle_f64"]["by_config"]) == len(runs)


def test_compact_line_drops_optional_parts_rather_than_overflow(full):
    big = dict(full)
    big["configs"] = full["configs"] * 40            # absurdly many rows
    s = B.compact_line(big)
    assert len(s) <= B.LINE_LIMIT
    d = json.loads(s)
    assert d["value"] == full["value"] and "roofline" in d and "cpu_baseline" in d


def test_detail_file_written(tmp_path, full):
    p = tmp_path / "sub" / "bench_detail.json"
    B.write_detail(str(p), full)
    with open(p) as fh:
        assert json.load(fh)["configs"][0]["roofline"]["traffic_detail"]


def test_estimator_dtype_label_states_precision():
    assert B.task_dtype("LeeLanded") == "f32"
    lab = B.task_dtype("QuadTracking")
    assert "EKF f64 (reference numpy f64)" in lab and "PV f64 (reference torch f32)" in lab and "f32 storage" in lab


def test_launcher_reports_failed_rank():
    """``--gpus 2`` without torchrun: bench.py starts two ranks itself; a rank that fails (here: no GPU in
    this container, so a rank cannot start its device) makes the parent exit non-zero instead of printing a
    one-GPU line."""
    env = dict(os.environ, OUZ_DIST_BACKEND="gloo", HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup",
                        "1", "--no-configs", "--no-sweep", "--no-cpu-baseline"], env=env, capture_output=True,
                       text=True, timeout=300)
    assert p.returncode != 0
    assert '"metric"' not in p.stdout

"""The committed measurements reproduce (CPU): the bench line's SpMV roofline
from the committed rocprof trace, the PMC traffic summary from the committed
FETCH_SIZE / WRITE_SIZE passes, and the round's headline line's own fields
(DESIGN.md §4 Roofline, §8)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(REPO, "profiles")


def _run(*args):
    out = subprocess.run([sys.executable] + list(args), cwd=REPO, capture_output=True, text=True, check=True)
    return out.stdout


def test_roofline_reproduces_from_trace():
    out = json.loads(_run("profiles/roofline_check.py", "profiles/r04_bench_c3_b512_under_rocprof.json",
                          "profiles/r04_c3_mixed_amg_b512_kernel_trace.csv", "C3/mixed/amg/B512"))
    assert abs(out["rel_diff"]) < 0.01, out
    assert out["rocprof_frac"] >= 0.6
    # the timed region's launches, bounded by the batches' k_gather_I launches
    # (batches 2-6 of this trace: not the host-IO leg after the clock)
    line0 = json.loads(open(os.path.join(P, "r04_bench_c3_b512_under_rocprof.json")).readline())
    assert out["rocprof_launches"] == line0["roofline"]["launches"] == 95
    assert 1860.0 < out["rocprof_us_per_launch"] < 1870.0
    # measured HBM traffic per full launch within 10 % of the kernel's own bytes
    line = json.loads(open(os.path.join(P, "r04_bench_c3_b512_under_rocprof.json")).readline())
    rl = line["roofline"]
    own = rl["kernel_bytes_per_system"] * 512 + rl["kernel_shared_bytes_per_launch"]
    assert abs(out["pmc_hbm_bytes_median_launch"] / own - 1.0) < 0.10


def test_roofline_reproduces_from_trace_b1024():
    """The default batch (1024, round 5's build): the line's SpMV roofline
    reproduced from its own rocprof trace and PMC passes (profiles/r05_*)."""
    out = json.loads(_run("profiles/roofline_check.py", "profiles/r05_bench_c3_b1024_under_rocprof.json",
                          "profiles/r05_c3_mixed_amg_b1024_kernel_trace.csv", "C3/mixed/amg/B1024"))
    assert abs(out["rel_diff"]) < 0.01, out
    assert out["rocprof_frac"] >= 0.6
    line = json.loads(open(os.path.join(P, "r05_bench_c3_b1024_under_rocprof.json")).readline())
    assert line["config"]["batch"] == 1024
    assert out["rocprof_launches"] == line["roofline"]["launches"] == 95
    assert 3575.0 < out["rocprof_us_per_launch"] < 3595.0
    rl = line["roofline"]
    own = rl["kernel_bytes_per_system"] * 1024 + rl["kernel_shared_bytes_per_launch"]
    assert abs(out["pmc_hbm_bytes_median_launch"] / own - 1.0) < 0.10


def test_roofline_reproduces_from_trace_b1536_final():
    """The shipped default (batch 1536, round 5's final build): the SpMV
    roofline reproduced from the line's own rocprof trace, the untimed
    deferred-update launches (early convergence mark) left out, and the PMC
    bytes within 10 % of the kernel's own."""
    out = json.loads(_run("profiles/roofline_check.py", "profiles/r05_bench_c3_b1536_under_rocprof.json",
                          "profiles/r05_c3_mixed_amg_b1536_kernel_trace.csv", "C3/mixed/amg/B1536"))
    assert abs(out["rel_diff"]) < 0.01, out
    line = json.loads(open(os.path.join(P, "r05_bench_c3_b1536_under_rocprof.json")).readline())
    assert line["config"]["batch"] == 1536
    assert out["rocprof_launches"] == line["roofline"]["launches"]
    assert out["untimed_x_update_launches"] >= 0
    assert out["rocprof_frac"] >= 0.65
    rl = line["roofline"]
    own = rl["kernel_bytes_per_system"] * 1536 + rl["kernel_shared_bytes_per_launch"]
    assert abs(out["pmc_hbm_bytes_median_launch"] / own - 1.0) < 0.10


def test_pmc_summary_reproduces_committed_entry_b1536(tmp_path):
    dst = tmp_path / "pmc.json"
    _run("profiles/pmc_summary.py", "profiles/r06/pmc_fetch_c3_mixed_amg_b1536.csv",
         "profiles/r06/pmc_write_c3_mixed_amg_b1536.csv", str(dst), "C3/mixed/amg/B1536", "6144")
    mine = json.load(open(dst))["C3/mixed/amg/B1536"]
    ref = json.load(open(os.path.join(P, "pmc_traffic.json")))["C3/mixed/amg/B1536"]
    assert mine["kernels"].keys() == ref["kernels"].keys()
    for k, v in ref["kernels"].items():
        assert mine["kernels"][k]["hbm_bytes_per_launch"] == pytest.approx(v["hbm_bytes_per_launch"])
    assert mine["run"]["hbm_bytes_per_timestep"] == pytest.approx(ref["run"]["hbm_bytes_per_timestep"])


def test_pmc_summary_reproduces_committed_entry_b1024(tmp_path):
    dst = tmp_path / "pmc.json"
    _run("profiles/pmc_summary.py", "profiles/r05_pmc_fetch_c3_mixed_amg_b1024.csv",
         "profiles/r05_pmc_write_c3_mixed_amg_b1024.csv", str(dst), "C3/mixed/amg/B1024", "4096")
    mine = json.load(open(dst))["C3/mixed/amg/B1024"]
    ref = json.load(open(os.path.join(P, "pmc_traffic.json")))["C3/mixed/amg/B1024"]
    assert mine["kernels"].keys() == ref["kernels"].keys()
    for k, v in ref["kernels"].items():
        assert mine["kernels"][k]["hbm_bytes_per_launch"] == pytest.approx(v["hbm_bytes_per_launch"])
    assert mine["run"]["hbm_bytes_per_timestep"] == pytest.approx(ref["run"]["hbm_bytes_per_timestep"])


def test_pmc_summary_reproduces_committed_entry(tmp_path):
    dst = tmp_path / "pmc.json"
    _run("profiles/pmc_summary.py", "profiles/r04_pmc_fetch_c3_mixed_amg_b512.csv",
         "profiles/r04_pmc_write_c3_mixed_amg_b512.csv", str(dst), "C3/mixed/amg/B512", "2048")
    mine = json.load(open(dst))["C3/mixed/amg/B512"]
    ref = json.load(open(os.path.join(P, "pmc_traffic.json")))["C3/mixed/amg/B512"]
    assert mine["kernels"].keys() == ref["kernels"].keys()
    for k, v in ref["kernels"].items():
        assert mine["kernels"][k]["hbm_bytes_per_launch"] == pytest.approx(v["hbm_bytes_per_launch"])
    assert mine["run"]["hbm_bytes_per_timestep"] == pytest.approx(ref["run"]["hbm_bytes_per_timestep"])


def test_roofline_check_reproduces_r06_line():
    """The final build's default configuration: the line's SpMV roofline
    from its own rocprof trace, within 1 %."""
    out = json.loads(_run("profiles/roofline_check.py", "profiles/r06/c3_b1536_bench_under_rocprof.json",
                          "profiles/r06/c3_mixed_amg_b1536_kernel_trace.csv", "C3/mixed/amg/B1536"))
    assert abs(out["rel_diff"]) < 0.01 and out["rocprof_frac"] >= 0.65, out


def test_kernel_rates_table():
    out = _run("profiles/kernel_rates.py", "profiles/r06/c3_mixed_amg_b1536_kernel_trace.csv",
               "profiles/r06/pmc_fetch_c3_mixed_amg_b1536.csv", "profiles/r06/pmc_write_c3_mixed_amg_b1536.csv")
    rows = [r for r in out.splitlines() if r.startswith("| `k_pcg_spmv<float, false")]
    assert rows and "31.36 GB" in rows[0]
    assert out.strip() == open(os.path.join(P, "r06", "kernel_rates_c3_b1536.md")).read().strip()


def test_r06_default_line_with_legs():
    """The round-6 default line carries the reference's mesh class as legs
    (F3, S1s, S1), each with its parity, iterations and roofline, and no
    defect."""
    lines = [l for l in open(os.path.join(P, "r06", "bench_default_final.json")) if l.startswith("{")]
    line = json.loads(lines[-1])
    assert "defect" not in line and line["solver"]["recovered"] == 0
    legs = {leg["config"]: leg for leg in line["legs"]}
    assert set(legs) == {"F3", "S1s", "S1"}
    assert legs["S1"]["solver"]["pcg_iterations_per_timestep"] <= 36
    for leg in legs.values():
        assert leg["solver"]["recovered"] == leg["solver"]["failed"] == 0
        assert leg["parity"]["max_abs_err"] < 1e-6 * max(1.0, leg["parity"]["max_abs_V"])
        assert leg["roofline"]["frac"] > 0
    assert legs["F3"]["solver"]["pcg_iterations_per_timestep"] <= 20


def test_headline_line_contract():
    line = json.loads(open(os.path.join(P, "r05_bench_C3_default.json")).readline())
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "roofline",
                "cpu_baseline", "parity", "host_io"):
        assert key in line
    assert line["parity"]["max_abs_err"] < line["parity"]["bar"] == 1e-6
    assert line["solver"]["failed"] == 0 and line["solver"]["max_rel_residual"] <= 1e-8
    # value = timed timesteps / (steps x ms_per_step)
    t = line["config"]["timesteps_timed"] / (line["steps"] * line["ms_per_step"] * 1e-3)
    assert line["value"] == pytest.approx(t, rel=1e-3)
    cb = line["cpu_baseline"]
    assert cb["cores"] >= 1 and cb["host_cpu_count"] >= cb["cores"] and cb["kind"] in ("port", "reference")


def test_sq_summary_runs(tmp_path):
    src = os.path.join(P, "r04_pmc_sq_c3_b512_after.csv")
    rows = open(src).read().splitlines()
    assert rows[0].startswith("kernel,dispatches,SQ_WAVES")
    assert any(r.startswith("k_residual_rcn<2>") for r in rows)

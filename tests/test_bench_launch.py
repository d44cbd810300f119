"""bench.py contract on the CPU: ``python bench.py --gpus N`` without a launcher starts N ranks
itself, each with its own RANK and the shared private rendezvous, exactly one
JSON line comes out (rank 0), and a failing rank fails the whole run."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent

_STUB = r"""
import json, os, sys
d = sys.argv[1]
r = int(os.environ["RANK"])
open(os.path.join(d, "rank%d" % r), "w").write(json.dumps({k: os.environ[k] for k in
    ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}))
if os.environ.get("STUB_FAIL_RANK") == str(r):
    sys.exit(3)
if r == 0:
    print(json.dumps({"metric": "stub", "n_gpus": int(os.environ["WORLD_SIZE"])}), flush=True)
"""


def _run(tmp_path, n, extra_env=None):
    stub = tmp_path / "stub.py"
    stub.write_text(_STUB)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "MASTER_PORT")}
    env["KFAMD_BENCH_RANK_ARGV"] = json.dumps([sys.executable, str(stub), str(tmp_path)])
    env.update(extra_env or {})
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(n), "--steps", "1", "--warmup", "0"],
                          cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)


def test_bench_self_launches_n_ranks(tmp_path):
    p = _run(tmp_path, 4)
    assert p.returncode == 0, p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and json.loads(lines[0])["n_gpus"] == 4
    ranks = [json.loads((tmp_path / f"rank{r}").read_text()) for r in range(4)]
    assert sorted(int(x["RANK"]) for x in ranks) == [0, 1, 2, 3]
    assert all(x["WORLD_SIZE"] == "4" and x["LOCAL_RANK"] == x["RANK"] for x in ranks)
    assert len({(x["MASTER_ADDR"], x["MASTER_PORT"]) for x in ranks}) == 1


def test_bench_rank_failure_fails_the_run(tmp_path):
    p = _run(tmp_path, 2, {"STUB_FAIL_RANK": "1"})
    assert p.returncode == 3, (p.returncode, p.stderr)


def test_launch_cli_runs_program_per_rank(tmp_path):
    stub = tmp_path / "stub.py"
    stub.write_text(_STUB)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "MASTER_PORT")}
    env.update({"LOCAL_WORLD_SIZE": "3", "MASTER_ADDR": "127.0.0.9", "MASTER_PORT": "29999"})
    p = subprocess.run([sys.executable, "-m", "kubeflow_rm_amd.parallel.launch", "--", str(stub), str(tmp_path)],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    ranks = [json.loads((tmp_path / f"rank{r}").read_text()) for r in range(3)]
    # the pod's injected rendezvous is used as is
    assert all(x["MASTER_ADDR"] == "127.0.0.9" and x["MASTER_PORT"] == "29999" for x in ranks)


def test_control_plane_latencies_measured():
    """BASELINE configs 3 / 5 (bench.py extra): Profile with GPU quota, TensorBoard, PVCViewer ready."""
    from tests.conftest import _ensure_native
    _ensure_native()
    from kubeflow_rm_amd.bench_coldstart import measure_control_plane
    r = measure_control_plane(runs=2)
    for k in ("profile_ready_p50_s", "tensorboard_ready_p50_s", "pvcviewer_ready_p50_s"):
        assert r[k] is not None and 0 < r[k] < 30, r


_HANG_STUB = r"""
import json, os, sys, time
sys.path.insert(0, sys.argv[2])
from kubeflow_rm_amd.bench_extras import Extras, print_line
r = int(os.environ["RANK"])
line = {"metric": "stub", "n_gpus": int(os.environ["WORLD_SIZE"])}
ex = Extras(float(sys.argv[3]), rank=r, grace_s=1.0, nonzero_rank_delay_s=1.0,
            emit=lambda rep: print_line({**line, **rep}))
ex.run("quick", lambda e: {"quick_value": 1}, est_s=0.1, timeout_s=5)
ex.run("broken", lambda e: 1 / 0, est_s=0.1, timeout_s=5)
ex.run("hang", lambda e: time.sleep(3600), est_s=0.1, timeout_s=2)
ex.run("never", lambda e: {"never": 1})
line.update(ex.finish())
ex.emit_once()
"""


def test_bench_extra_that_hangs_still_yields_the_line(tmp_path):
    """one extra hangs on every rank; the self-launched job still ends well inside
    the budget with exactly one JSON line, the hung extra marked ``timeout``, the finished ones kept,
    and the exit status is 124 (not the headline's 0)."""
    import time
    stub = tmp_path / "hang.py"
    stub.write_text(_HANG_STUB)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "MASTER_PORT")}
    env["KFAMD_BENCH_RANK_ARGV"] = json.dumps([sys.executable, str(stub), str(tmp_path), str(ROOT), "60"])
    t0 = time.time()
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    took = time.time() - t0
    assert p.returncode == 124, (p.returncode, p.stderr)  # a hang fails the run
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    st = d["extras_status"]
    assert st["quick"]["status"] == "ok" and d["quick_value"] == 1
    assert st["broken"]["status"] == "error" and "ZeroDivisionError" in st["broken"]["error"]
    assert st["hang"]["status"] == "timeout"
    assert "never" not in st and "never" not in d
    assert took < 40, took


def test_bench_extras_skip_what_does_not_fit_the_budget():
    from kubeflow_rm_amd.bench_extras import Extras
    ex = Extras(5.0)
    assert ex.run("fits", lambda e: {"x": 1}, est_s=1)
    assert not ex.run("too_big", lambda e: {"y": 1}, est_s=30)
    # collective extras follow the agreement, not the local view
    ex.agree = lambda ok: False
    assert not ex.run("peer_says_no", lambda e: {"z": 1}, est_s=0, collective=True)
    rep = ex.finish()
    assert rep["x"] == 1 and "y" not in rep and "z" not in rep
    assert rep["extras_status"]["too_big"]["status"] == "skipped"
    assert rep["extras_status"]["peer_says_no"]["status"] == "skipped"


def test_cold_start_failures_keep_their_count_and_diagnostics():
    """The default path's prefix is ``cold_start``: its failure COUNT (``cold_start_failures``) must
    not collide with the per-variant pod diagnostics (``cold_start_failure_diagnostics``)."""
    sys.path.insert(0, str(ROOT))
    import bench

    cs = {"runs": [0.1, 0.2], "p50_s": 0.1, "p90_s": 0.2, "failures": [{"pod": "bench/nb-3", "reason": "timeout"}]}
    out = bench._cs_keys("cold_start", cs)
    assert out["cold_start_failures"] == 1
    assert out["cold_start_failure_diagnostics"] == {"cold_start": cs["failures"]}
    out2 = bench._cs_keys("cold_start_odh", dict(cs, failures=[]))
    assert out2["cold_start_odh_failures"] == 0 and "cold_start_failure_diagnostics" not in out2

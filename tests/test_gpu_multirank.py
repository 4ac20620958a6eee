"""The N-rank bench path on the GPU box's one GPU:
bench.py --gpus 2 self-launches two ranks through torch.distributed.run;
MOF_BENCH_REHEARSE=1 puts both on GPU 0 with gloo for the timing
collectives (RCCL refuses two ranks on one device). Each rank builds its own
handle and solves its own contiguous k-range; the line sums the ranks'
timesteps over the slowest rank's time, and rank 0's parity sample must meet
the bar. Weak and strong (C4's fixed job) modes."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*argv):
    env = dict(os.environ, MOF_BENCH_REHEARSE="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *argv], env=env, capture_output=True,
                         text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.timeout(300)
def test_two_ranks_weak():
    line = _bench("--gpus", "2", "--config", "C2", "--precision", "mixed", "--steps", "2", "--warmup", "1",
                  "--batch", "64", "--no-cpu-baseline", "--host-batches", "0")
    assert line["n_gpus"] == 2 and line["scaling"] == "weak" and "defect" not in line
    assert line["config"]["timesteps_timed"] == 2 * 2 * 64
    assert line["solver"]["failed"] == line["solver"]["recovered"] == 0
    assert line["parity"]["max_abs_err"] < 1e-6 * max(1.0, line["parity"]["max_abs_V"])
    assert line["legs"] is None


@pytest.mark.timeout(300)
def test_two_ranks_strong_fixed_job():
    line = _bench("--gpus", "2", "--config", "C2", "--precision", "mixed", "--steps", "1", "--warmup", "1",
                  "--fixed-timesteps", "200", "--batch", "64", "--no-cpu-baseline", "--host-batches", "0")
    assert line["n_gpus"] == 2 and line["scaling"] == "strong" and "defect" not in line
    assert line["config"]["timesteps_timed"] == 200
    # 100 timesteps per rank in balanced batches: 2 x 50
    assert line["config"]["batch_effective"] == 50
    assert line["parity"]["max_abs_err"] < 1e-6 * max(1.0, line["parity"]["max_abs_V"])

"""The bench's real multi-rank worker path, rehearsed on one GPU: ``bench.py --gpus 2`` spawns two
ranks (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1), each runs the fused engine on its
shard of the global batch with the bucketed gradient all-reduce live, and rank 0 prints ONE JSON
line.  The backend is gloo here (two ranks on one device); the nccl (RCCL) branch differs only in
the init_process_group backend string."""
import json
import os
import subprocess
import sys

import pytest

from gpu_utils import need_gpu

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_gloo_one_line():
    need_gpu()
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "c1",
                        "--steps", "4", "--warmup", "1", "--no-extra", "--no-cpu-baseline", "--backend", "gloo"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 4 and d["warmup"] == 1
    assert d["config"]["global_batch"] == 2 * d["config"]["per_gpu_batch"]
    assert d["config"]["parallelism"] == "dp2"
    assert d["value"] > 0 and d["cpu_baseline"] is None
    for k in ("kld_loss", "recon_loss", "loss"):
        assert d["elbo"][k] == d["elbo"][k]   # finite: the summed shares of the global batch

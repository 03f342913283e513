"""The N > 1 bench path on a one-GPU box (FTHE_BENCH_REHEARSE=1: two ranks on cuda:0 over gloo): the launcher, the
barriers and max-over-ranks timing, every rank's adds, and rank 0's node-wide drop-in pass (secondary.ghpair_e2e_node:
ghpair_e2e over the run's devices in one process, here two contexts of device 0 with key replicas) -- the code the
driver's 2/4/8-GPU runs execute, at a small size."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_two_rank_rehearsal_prints_the_node_pass():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(FTHE_BENCH_REHEARSE="1", FTHE_BENCH_NODE_PAIRS="65536", FTHE_BENCH_DETAIL=os.devnull)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--pairs", "65536",
                        "--steps", "1", "--warmup", "0", "--no-cpu"], capture_output=True, text=True, env=env,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["rehearsal"]
    assert sorted(p["rank"] for p in line["per_rank"]) == [0, 1]
    node = line["secondary"]["ghpair_e2e_node"]
    assert node["ok"] is True and node["shards"] == 2 and node["pairs"] == 2 * 65536 and node["devices"] == "0,0"
    assert node["encrypts_per_s"] > 0 and node["decrypts_per_s"] > 0

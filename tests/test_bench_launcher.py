"""bench.py's multi-rank harness on the CPU: `python bench.py --gpus 2` (no torchrun) spawns
the two rank processes itself, they rendezvous over gloo on 127.0.0.1, time the steps
between barriers, gather per-rank times and rank 0 prints one line with n_gpus = 2.
--dry-run replaces the GPU step with a sleep, so nothing here touches a device."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, extra_env=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(extra_env or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       env=env, timeout=240)
    return r


def test_spawns_n_ranks():
    r = _run(["--gpus", "2", "--steps", "3", "--warmup", "1", "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout                    # rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["dry_run"]
    per = line["per_rank"]
    assert sorted(p["rank"] for p in per) == [0, 1]
    assert sorted(p["local_rank"] for p in per) == [0, 1]
    assert len({p["pid"] for p in per}) == 2             # two processes
    assert line["elapsed_max_s"] == max(p["elapsed_s"] for p in per)
    assert line["elapsed_max_s"] >= 3 * 0.02
    # the N > 1 line carries the same blocks as N = 1: roofline, rank 0's CPU baseline and every
    # rank's ciphertext adds/s with the aggregate over the slowest rank
    assert "roofline" in line and "cpu_baseline" in line and line["cpu_baseline"]["cores"] >= 1
    adds = line["ciphertext_adds"]
    assert sorted(p["rank"] for p in adds["per_rank"]) == [0, 1]
    assert all(p["adds_per_s"] > 0 for p in adds["per_rank"])
    slow = max(p["median_s"] for p in adds["per_rank"])
    assert adds["aggregate_adds_per_s"] == round(2 * adds["adds_per_rank"] / slow)


def test_single_rank_default():
    r = _run(["--steps", "1", "--warmup", "0", "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][0])
    assert line["n_gpus"] == 1 and len(line["per_rank"]) == 1


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "4", "--dry-run"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in (r.stderr + r.stdout)


def test_failing_rank_fails_the_launch():
    """Rank 1 dies before the rendezvous: the parent ends rank 0 (blocked in the rendezvous)
    and exits with rank 1's status instead of hanging."""
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--dry-run"], {"FTHE_BENCH_FAIL_RANK": "1"})
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])


def test_compact_line_fits_the_driver_record():
    """The stdout line drops prose and tool detail (written to FTHE_BENCH_DETAIL instead) and fits LINE_MAX bytes,
    so the driver's kept tail holds the whole record -- with the aggregate ciphertext adds/s, the parties'
    public-key encrypts/s and the CRT decrypts/s, checked on round 4's full 14 KB line."""
    sys.path.insert(0, ROOT)
    import bench
    full = json.loads(open(os.path.join(ROOT, "profiles", "r04ze_bench.json")).read().strip().splitlines()[-1])
    assert len(json.dumps(full)) > 12000
    text = bench.compact_line(full)
    assert len(text) <= bench.LINE_MAX
    line = json.loads(text)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert line[k] == full[k], k
    assert line["ciphertext_adds"]["aggregate_adds_per_s"] == full["ciphertext_adds"]["aggregate_adds_per_s"]
    assert line["secondary"]["public_encrypt_per_s"] == full["secondary"]["public_encrypt_per_s"]
    assert line["secondary"]["crt_decrypt_per_s"] == full["secondary"]["crt_decrypt_per_s"]
    r, fr = line["roofline"], full["roofline"]
    assert (r["bound"], r["achieved"], r["peak"], r["unit"], r["frac"]) == \
        (fr["bound"], fr["achieved"], fr["peak"], fr["unit"], fr["frac"])
    cb = line["cpu_baseline"]
    assert cb["value"] == full["cpu_baseline"]["value"] and cb["cores"] and cb["kind"] and cb["sample"]
    assert "note" not in text


def test_node_e2e_arguments_and_memory_cap(monkeypatch):
    """bench.node_e2e (N > 1, rank 0 after the timed region): ghpair_e2e over the run's devices in one child process,
    N x 10M pairs by default, capped so the batch (~2.3 KB of host memory per pair) stays within 40% of the free host
    memory; under FTHE_BENCH_REHEARSE every shard on device 0 with key replicas forced.  The child is faked here."""
    sys.path.insert(0, ROOT)
    import bench
    calls = []

    class R:
        returncode = 0
        stdout = '{"encrypts_per_s": 1.0, "decrypts_per_s": 2.0, "ok": true, "shards": 4}\n'
        stderr = ""

    def fake_run(cmd, **kw):
        calls.append((cmd, kw.get("env", {})))
        return R()
    monkeypatch.setattr(bench.subprocess, "run", fake_run)
    monkeypatch.delenv("FTHE_BENCH_NODE_PAIRS", raising=False)
    monkeypatch.setattr(bench, "host_mem_bytes", lambda: 10 ** 15)
    out = bench.node_e2e(None, 4, [3, 1, 0, 2], False)
    cmd, env = calls[-1]
    assert cmd[1:] == ["2048", str(4 * 10_000_000), "2", "0,1,2,3"] and env["FTHE_SHIM_REPLICATE"] == "0"
    assert out["ok"] and out["shards"] == 4 and out["pairs_per_device"] == 10_000_000
    assert out["encrypts_per_s_per_device"] == 0
    monkeypatch.setattr(bench, "host_mem_bytes", lambda: 10 ** 9)          # 1 GB free: 0.4 GB / 2.3 KB / 2 devices
    out = bench.node_e2e(None, 2, [0, 1], True)
    cmd, env = calls[-1]
    per = int(0.4 * 10 ** 9 / bench.E2E_HOST_BYTES_PER_PAIR / 2)
    assert out["pairs_per_device"] == per and cmd[2] == str(2 * per)
    assert cmd[4] == "0,0" and env["FTHE_SHIM_REPLICATE"] == "1"


def test_host_mem_bytes_is_positive():
    sys.path.insert(0, ROOT)
    import bench
    m = bench.host_mem_bytes()
    assert m is None or m > 0

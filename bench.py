#!/usr/bin/env python3
"""bench.py -- Paillier-2048 encrypts/s, device-resident (BASELINE.json `metric`).

Workload (BASELINE.json configs[4], per-GPU share; configs[2]'s encrypt half):
one step = encrypt 10M synthetic logistic gradient pairs (20M ciphertexts) that
already sit in HBM as float32 (g, h): device fixed-point codec + fresh uniform
randomness per ciphertext from the device ChaCha20 stream + c = g^m r^n mod n^2
(CRT over p^2, q^2: the encrypting server holds the key, server.h:113-135; r^n
mod p^2 drawn as y^p mod p^2 for uniform y, the same distribution),
output 20M x 512 B ciphertexts left in HBM.

Multi-GPU: one process per GPU, each rank encrypts its own 10M pairs --
independent units, no collective on the data path (weak scaling); the barrier
and the max-over-ranks elapsed time use torch.distributed.  Under torchrun the
ranks come from the environment (WORLD_SIZE must equal --gpus); a plain
`python bench.py --gpus N` spawns the N rank processes itself.

Printed by rank 0: one JSON line with the driver's contract fields plus
`roofline` (montprog kernel: algorithmic integer MACs per second vs the
half-rate v_mad_u64_u32 peak, per-launch HIP events on the engine stream) and
`cpu_baseline` (the reference's own Paillier_GMP encrypt / decrypt / add /
merge on the bench's key and inputs, OpenMP over bounded samples on this
host's cores, cores and CPU model stated).
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Paillier-2048 encrypts/s device-resident; ciphertext adds/s; 1/2/4/8 GPU"
SEED = 20261015
KEY_BITS = 2048
# Roofline (MI355X_MICROARCH.md: 256 CUs, 2.4 GHz, SIMD32).  v_mad_u64_u32 is
# half-rate on gfx950 (measured, profiles/r01_microbench_valu.txt): 64 lanes per
# 4 cycles per SIMD -> 16 MACs/clk/SIMD.
PEAK_MAC_S = 256 * 4 * 16 * 2.4e9          # 3.93e13 32x32->64 MACs/s
MEASURED_MAD_S = 3.45e13                   # microbenchmark, 8 chains x 16 waves/CU
# W(s) = 2 s^2 + s MACs per Montgomery product on s u32 limbs,
# 1.2 e products per e-bit exponent; CRT encrypt = 2 modexps of 2048-bit exponent
# over 2048-bit moduli (s = 64).
W64 = 2 * 64 * 64 + 64
ALG_MACS_PER_CRT_ENC = 2 * 1.2 * 2048 * W64          # 4.06e7
PMC_FILE = "r06t_pmc.json"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one process per GPU); without torchrun the bench spawns them itself")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--pairs", type=int, default=10_000_000, help="gradient pairs per GPU per step")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU-baseline threads (0: every core this process may use, see host_cpu())")
    ap.add_argument("--cpu-scale", type=float, default=1.0, help="CPU-baseline sample size multiplier")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU rehearsal of the multi-rank harness (launcher, barriers, max-over-ranks, "
                         "per-rank report): gloo, no GPU, a fixed sleep as the step; never a measurement")
    return ap.parse_args()


def launch_ranks(a):
    """`--gpus N` (N > 1) outside torchrun: start N rank processes of this script, one per GPU,
    with the torchrun environment (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR/PORT on 127.0.0.1),
    and exit with the first failing status.  The parent never touches the GPU (torch is not even
    imported) and does not re-exec itself: the ranks are children."""
    import signal
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus),
                   LOCAL_WORLD_SIZE=str(a.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        time.sleep(0.2)
        for pr in list(live):
            st = pr.poll()
            if st is None:
                continue
            live.remove(pr)
            if st != 0 and rc == 0:
                rc = st
                for other in live:                      # a rank failed: end the others (exact PIDs)
                    other.send_signal(signal.SIGTERM)
    return rc if rc >= 0 else 128 - rc


def host_cpu():
    """The host cores this process may use and what they are: affinity mask, cgroup CPU quota,
    the box's OMP_NUM_THREADS share (the GPU pool sets it to the CPU share of one GPU), nproc and
    the /proc/cpuinfo model.  The baseline runs on min(affinity, quota, OMP_NUM_THREADS) threads."""
    info = {"nproc": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)), "cgroup_quota_cpus": None,
            "omp_num_threads_env": None, "model": None}
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            info["cgroup_quota_cpus"] = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        info["omp_num_threads_env"] = int(omp)
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                info["model"] = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    use = info["affinity_cpus"]
    if info["cgroup_quota_cpus"]:
        use = min(use, max(1, int(info["cgroup_quota_cpus"])))
    if info["omp_num_threads_env"]:
        use = min(use, info["omp_num_threads_env"])
    info["threads_used"] = max(1, use)
    return info


def cpu_baseline(a, pl, p1k, m, c, dev):
    """The reference's own CPU path timed on this host, on the bench's keys and inputs:
    FedTree's Paillier_GMP (paillier_gmp.cpp, compiled from the reference sources into
    oracle/_ref) -- encrypt = PowerMod(r, n, n^2) PowerMod(g, m, n^2) (:37-73), decrypt =
    PowerMod(c, lambda, n^2) (:75-85), add = x y mod n^2 (:16-21) -- OpenMP over elements as
    Server::encrypt_gh_pairs / decrypt_gh_pairs (server.h:105-109,129-133) and the party merge
    (hist_tree_builder.cpp:1026-1037) do.  Bounded samples, ~10 s in all on 16 threads.
    Without oracle/_ref: the C/GMP restatement of paillier.cpp (oracle/paillier_oracle.c)."""
    import ctypes
    import torch
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    hc = host_cpu()
    thr = a.cpu_threads or hc["threads_used"]
    sc = a.cpu_scale
    nw = pl.n_words
    m_h = m.cpu().numpy().view(np.uint64)
    try:
        ref = pyoracle.RefGMP()
    except OSError:
        ref = None
    ops = {}

    def timed(fn):
        t0 = time.perf_counter()
        fn()
        return time.perf_counter() - t0

    if ref is not None:
        kind, what = "reference", "FedTree Paillier_GMP compiled from the reference sources (oracle/_ref)"
        h = ref.key_from_primes(pl.p, pl.q)
        ne = max(thr, int(512 * thr * sc))
        mm = np.ascontiguousarray(m_h[:ne])
        ct = np.zeros((ne, 2 * nw), np.uint32)
        dt = timed(lambda: ref.lib.ref_encrypt_batch(h, nw, mm.ctypes.data, ne, ct.ctypes.data, thr))
        ops["p2048_encrypt"] = {"per_s": ne / dt, "n": ne, "s": dt}
        n1 = max(8, int(128 * sc))
        ct1 = np.zeros((n1, 2 * nw), np.uint32)
        dt1 = timed(lambda: ref.lib.ref_encrypt_batch(h, nw, mm.ctypes.data, n1, ct1.ctypes.data, 1))
        ops["p2048_encrypt_1_thread"] = {"per_s": n1 / dt1, "n": n1, "s": dt1}
        # the CPU ciphertexts are valid under the bench's key: the engine decrypts them to m
        chk = pl.decrypt_u64(ct[:256])
        same_key_ok = bool(np.array_equal(chk, mm[:256]))
        nd = ne
        cin = np.ascontiguousarray(c[:nd].cpu().numpy().view(np.uint32))
        lo = np.zeros(nd, np.uint64)
        dt = timed(lambda: ref.lib.ref_decrypt_batch(h, nw, cin.ctypes.data, nd, lo.ctypes.data, thr))
        ops["p2048_decrypt"] = {"per_s": nd / dt, "n": nd, "s": dt, "ok": bool(np.array_equal(lo, m_h[:nd]))}
        na = max(thr, int(65536 * thr * sc))
        na = min(na, 1 << 20, c.shape[0] // 2)
        xa = np.ascontiguousarray(c[:na].cpu().numpy().view(np.uint32))
        xb = np.ascontiguousarray(c[na:2 * na].cpu().numpy().view(np.uint32))
        so = np.zeros_like(xa)
        dt = timed(lambda: ref.lib.ref_add_batch(h, nw, xa.ctypes.data, xb.ctypes.data, na, so.ctypes.data, thr))
        ops["p2048_add"] = {"per_s": na / dt, "n": na, "s": dt}
        nb, parties = max(thr, int(8192 * thr * sc)), 8
        nb = min(nb, 1 << 17, c.shape[0] // parties)
        xk = np.ascontiguousarray(c[:parties * nb].cpu().numpy().view(np.uint32))
        mo = np.zeros((nb, 2 * nw), np.uint32)
        dt = timed(lambda: ref.lib.ref_merge_batch(h, nw, xk.ctypes.data, parties, nb, mo.ctypes.data, thr))
        ops["p2048_merge_8party"] = {"adds_per_s": nb * (parties - 1) / dt, "bins": nb, "s": dt,
                                     "note": "7 Paillier_GMP::add per bin, parties serial, bins in parallel"}
        del xa, xb, so, xk, mo, cin
        ref.lib.ref_free(h)
        if p1k is not None:
            h1 = ref.key_from_primes(p1k.p, p1k.q)
            n1k = max(thr, int(4096 * thr * sc))
            m1 = np.ascontiguousarray(m_h[:n1k])
            c1 = np.zeros((n1k, 2 * p1k.n_words), np.uint32)
            dt = timed(lambda: ref.lib.ref_encrypt_batch(h1, p1k.n_words, m1.ctypes.data, n1k, c1.ctypes.data, thr))
            ops["p1024_encrypt"] = {"per_s": n1k / dt, "n": n1k, "s": dt}
            ref.lib.ref_free(h1)
    else:
        kind, what = "port", "C/GMP restatement of paillier.cpp:122-139 (oracle/paillier_oracle.c)"
        same_key_ok = None
        hw = (max(pl.p.bit_length(), pl.q.bit_length()) + 31) // 32
        key = pyoracle.COracle().key(pyoracle.to_words(pl.p, hw), pyoracle.to_words(pl.q, hw))
        ne = max(thr, int(512 * thr * sc))
        rng = np.random.default_rng(SEED)
        r = rng.integers(0, 2**32, (ne, nw), dtype=np.uint64).astype(np.uint32)
        r[:, -1] &= 0x3FFFFFFF
        dt = timed(lambda: key.encrypt_batch(m_h[:ne], r, thr))
        ops["p2048_encrypt"] = {"per_s": ne / dt, "n": ne, "s": dt}
    for v in ops.values():
        for k_ in ("per_s", "adds_per_s", "s"):
            if k_ in v:
                v[k_] = round(v[k_], 3 if k_ == "s" else 1)
    enc = ops["p2048_encrypt"]
    one = ops.get("p2048_encrypt_1_thread")
    return {"value": enc["per_s"], "unit": "encrypts/s", "cores": thr, "kind": kind,
            "sample": f"{enc['n']} Paillier-2048 encrypts of the bench's own gradients under the bench's own key "
                      f"({what}: full PowerMod, no CRT; OpenMP {thr} threads), {enc['s']:.1f} s",
            "per_thread_per_s": round(enc["per_s"] / thr, 1),
            "single_thread_per_s": one["per_s"] if one else None,
            "host": hc, "same_key_decrypts_on_gpu": same_key_ok, "ops": ops}


def _sig(x, digits=4):
    """x rounded to `digits` significant digits (floats only)."""
    if isinstance(x, float) and x == x and x not in (float("inf"), float("-inf")) and x != 0:
        from math import floor, log10
        return round(x, max(0, digits - 1 - floor(log10(abs(x)))))
    return x


def _strip(o, drop):
    if isinstance(o, dict):
        return {k: _strip(v, drop) for k, v in o.items() if not drop(k)}
    if isinstance(o, list):
        return [_strip(v, drop) for v in o]
    return _sig(o)


LINE_MAX = 7000      # the driver keeps the tail of the line (~8.7 KB): the whole record must fit


def compact_line(full):
    """The stdout line: the full record without prose (notes, sources, host details -- DESIGN.md 4 explains the
    fields) and with the tool outputs reduced to their rates, at most LINE_MAX bytes.  The full record goes to
    FTHE_BENCH_DETAIL (default gpurun_out/bench_detail.json)."""
    import re
    pat = re.compile(r"note|_source$|^source$|^what$|^per_thread_per_s$|^survey_alg|^window_operand|"
                     r"^kernel_share|^montmuls_per|^launches$|^avg_launch_ms$|_range$|^pmc_calibration$|"
                     r"^pmc_launch_ms$|^pmc_kernel$|^pmc_algorithmic|^peak_GBps$|^bound$|^products_per_add$")
    line = _strip(full, lambda k: bool(pat.search(k)))
    for k, v in full.items():                            # the contract's own fields exactly as measured
        if not isinstance(v, (dict, list)):
            line[k] = v
    line["roofline"] = _strip(full.get("roofline") or {}, lambda k: bool(re.search(r"note|^survey_alg|^window_operand", k)))
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        if k in (full.get("roofline") or {}):
            line["roofline"][k] = full["roofline"][k]
    cpu = line.get("cpu_baseline")
    if isinstance(cpu, dict):
        host = (full.get("cpu_baseline") or {}).get("host") or {}
        cpu.pop("host", None)
        cpu["value"] = full["cpu_baseline"].get("value")
        cpu["host_model"] = host.get("model")
        cpu["sample"] = (full["cpu_baseline"].get("sample") or "")[:160]
        if isinstance(cpu.get("ops"), dict):
            cpu["ops"] = {k: v.get("per_s", v.get("adds_per_s")) for k, v in cpu["ops"].items() if isinstance(v, dict)}
    sec = line.get("secondary") or {}
    hl = sec.get("histogram_loop_unchanged_callers")
    if isinstance(hl, dict):
        sec["histogram_loop_unchanged_callers"] = {
            t: ({"adds_per_s": v.get("ciphertext_adds_per_s"), "vs_reference_add": v.get("vs_reference_add"),
                 "subs_per_s": (v.get("sub") or {}).get("ciphertext_subs_per_s"),
                 "vs_reference_sub": (v.get("sub") or {}).get("vs_reference_sub"), "ok": v.get("ok")}
                if isinstance(v, dict) and "error" not in v else v) for t, v in hl.items()}
    hm = sec.get("host_marshalling_shards")
    if isinstance(hm, dict) and isinstance(hm.get("shards"), list):
        sec["host_marshalling_shards"] = {"round_trip_ok": hm.get("round_trip_ok"), "per_shards": {
            str(x.get("shards")): [x.get("encrypt_side_per_s"), x.get("decrypt_side_per_s")] for x in hm["shards"]}}
    ah = sec.get("p2048_add_hbm")
    if isinstance(ah, dict):
        sec["p2048_add_hbm"] = {k: ah[k] for k in ("algorithmic_GBps", "pmc_GBps_calibrated", "pmc_VALUBusy",
                                                   "valu_frac_executed", "valu_issue_frac", "matrix_core") if k in ah}
    for k in ("ghpair_e2e", "ghpair_e2e_sharded", "ghpair_e2e_node"):
        if isinstance(sec.get(k), dict):
            sec[k] = {x: sec[k][x] for x in ("encrypts_per_s", "decrypts_per_s", "ok", "shards", "pairs", "devices",
                                              "error") if x in sec[k]}
    if isinstance(sec.get("wire"), dict):
        sec["wire"] = {k: v for k, v in sec["wire"].items() if k.endswith("_per_s") or k.endswith("_ok")
                       or k.endswith("_host")}
    text = json.dumps(line, separators=(",", ":"))
    for k in ("wire", "host_marshalling_shards", "histogram_loop_unchanged_callers", "p1024_100k_pairs",
              "fixed_base", "ghpair_operator_add", "concurrent_decrypt_gh"):
        if len(text) <= LINE_MAX:
            break
        sec.pop(k, None)
        text = json.dumps(line, separators=(",", ":"))
    return text


def write_detail(full):
    path = os.environ.get("FTHE_BENCH_DETAIL") or os.path.join(ROOT, "gpurun_out", "bench_detail.json")
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            f.write(json.dumps(full) + "\n")
    except OSError as ex:
        print(f"[bench] detail record not written: {ex}", file=sys.stderr)


def main():
    a = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and a.gpus > 1:
        sys.exit(launch_ranks(a))
    world = int(env_world or "1")
    if world != a.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={world} but --gpus {a.gpus}: launch one rank per GPU")
    if a.dry_run:
        return dry_run(a, world)
    return run(a, world)


def dry_run(a, world):
    """The multi-rank harness with a CPU sleep as the step (tests/test_bench_launcher.py)."""
    import torch.distributed as dist
    rank = int(os.environ.get("RANK", "0"))
    if os.environ.get("FTHE_BENCH_FAIL_RANK") == str(rank):
        sys.exit(3)                                   # launcher test: a rank that dies early
    if world > 1:
        dist.init_process_group("gloo")
    times = timed_steps(lambda i: time.sleep(0.02), a, world, sync=lambda: None)
    per = gather_ranks({"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "pid": os.getpid(),
                        "elapsed_s": times}, world)
    # the per-rank add batch (a sleep standing in for the device adds) and rank 0's CPU stage, in the
    # order and with the collectives of the real run
    adds = rank_adds(lambda: time.sleep(0.01) or 0.01, 1 << 20, world, rank, sync=lambda: None)
    if rank == 0:
        cpu = {"dry_run": True, "value": None, "unit": "encrypts/s", "cores": host_cpu()["threads_used"],
               "kind": None, "sample": "dry run: no CPU baseline measured"}
        print(json.dumps({"metric": METRIC, "dry_run": True, "n_gpus": world, "steps": a.steps,
                          "warmup": a.warmup, "elapsed_max_s": max(p["elapsed_s"] for p in per),
                          "roofline": {"dry_run": True}, "cpu_baseline": cpu, "ciphertext_adds": adds,
                          "per_rank": per}), flush=True)
    if world > 1:
        dist.barrier()                                 # ranks wait for rank 0's CPU stage, as in run()
        dist.destroy_process_group()


def timed_steps(step, a, world, sync):
    """W untimed steps, then K timed ones bracketed by barrier + device sync on both sides.
    Returns this rank's elapsed seconds."""
    import torch.distributed as dist
    for i in range(a.warmup):
        step(i)
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(a.steps):
        step(a.warmup + i)
        if int(os.environ.get("RANK", "0")) == 0:
            sync()                      # progress for long runs (one host sync per ~13 s step: no measurable cost)
            print(f"[bench] step {i + 1}/{a.steps} done at {time.perf_counter() - t0:.1f} s", file=sys.stderr,
                  flush=True)
    sync()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    return t1 - t0


def gather_ranks(obj, world):
    if world == 1:
        return [obj]
    import torch.distributed as dist
    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


def rank_adds(call, count, world, rank, sync):
    """The metric's second half, "ciphertext adds/s" at N GPUs: every rank times `count` device-resident
    P-2048 adds (x y mod n^2 on its own GPU; call() runs one batch and returns its kernel seconds) --
    one untimed call, then the median of 5 -- between barriers; the aggregate is all ranks' adds over
    the slowest rank's median (weak scaling, no data-path collective)."""
    import torch.distributed as dist
    call()
    sync()
    if world > 1:
        dist.barrier()
    ts = []
    for _ in range(5):
        ts.append(call())
    sync()
    med = sorted(ts)[2]
    per = gather_ranks({"rank": rank, "adds": count, "median_s": round(med, 6),
                        "adds_per_s": round(count / med)}, world)
    slow = max(p["median_s"] for p in per)
    return {"per_rank": per, "aggregate_adds_per_s": round(world * count / slow), "adds_per_rank": count,
            "note": "device-resident P-2048 ciphertext adds (fthe_add_dev: x y on the VALU, its Barrett "
                    "reduction by n^2 on the matrix cores, fthe_addb_q152), median of 5 per rank, "
                    "aggregate = ranks x adds / slowest rank"}


def host_mem_bytes():
    """Host memory this process may still use: MemAvailable, bounded by the cgroup's limit less its usage."""
    avail = None
    try:
        for ln in open("/proc/meminfo"):
            if ln.startswith("MemAvailable:"):
                avail = int(ln.split()[1]) * 1024
    except (OSError, ValueError, IndexError):
        pass
    try:
        lim = open("/sys/fs/cgroup/memory.max").read().strip()
        if lim != "max":
            cur = int(open("/sys/fs/cgroup/memory.current").read())
            room = int(lim) - cur
            avail = room if avail is None else min(avail, room)
    except (OSError, ValueError):
        pass
    return avail


# host bytes per pair of a ghpair_e2e batch: two 4096-bit mpz (limbs + allocator), the GHPair, and the pinned
# plaintext and ciphertext rows (2 x 8 B + 2 x 512 B)
E2E_HOST_BYTES_PER_PAIR = 2300


def node_e2e(a, world, devices, rehearse):
    """ghpair_e2e over every device of the run in one process (integration/ghpair_e2e.cpp): 10M pairs per device
    (FTHE_BENCH_NODE_PAIRS overrides), fewer when the host cannot hold the batch in 40% of its free memory; best of
    two reps (the first pays the pinning, the key replicas and the mpz allocations),
    every plaintext checked.  FTHE_BENCH_REHEARSE: every shard on device 0."""
    per_dev = int(os.environ.get("FTHE_BENCH_NODE_PAIRS") or 10_000_000)
    mem = host_mem_bytes()
    if mem:
        per_dev = min(per_dev, int(0.4 * mem / E2E_HOST_BYTES_PER_PAIR / world))
    per_dev = max(per_dev, 1 << 14)
    devs = ",".join("0" for _ in devices) if rehearse else ",".join(str(d) for d in sorted(devices))
    exe = os.path.join(ROOT, "tools", "bin", "ghpair_e2e")
    out = {"devices": devs, "pairs_per_device": per_dev, "host_mem_free_bytes": mem}
    t0 = time.perf_counter()
    try:
        env = dict(os.environ, FTHE_SHIM_REPLICATE="1" if rehearse else "0")
        r = subprocess.run([exe, str(KEY_BITS), str(per_dev * world), "2", devs], capture_output=True, text=True,
                           timeout=420, env=env)
        res = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else \
            {"error": f"rc {r.returncode}: {r.stderr.strip()[-300:]}"}
    except (OSError, subprocess.TimeoutExpired, ValueError, IndexError) as ex:
        res = {"error": repr(ex)[:300]}
    out.update(res)
    out["wall_s"] = round(time.perf_counter() - t0, 1)
    if "encrypts_per_s" in out:
        out["encrypts_per_s_per_device"] = round(out["encrypts_per_s"] / world)
    return out


def run(a, world):
    import torch
    import torch.distributed as dist
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # FTHE_BENCH_REHEARSE=1: every rank on cuda:0 over gloo -- exercises the multi-rank path
    # (launcher, barriers, max-over-ranks timing, rank-0 reporting) on a one-GPU box, where
    # RCCL refuses two ranks on one device.  Never used for reported numbers.
    rehearse = os.environ.get("FTHE_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    if world > 1:
        torch.cuda.set_device(local)
        # a long timeout: the ranks wait at the final barrier while rank 0 runs its CPU baseline and the node-wide
        # drop-in pass (ghpair_e2e_node), minutes at N = 8
        from datetime import timedelta
        if rehearse:
            dist.init_process_group("gloo", timeout=timedelta(minutes=60))
        else:
            # RCCL carries only the barriers and the max-over-ranks gathers: no data-path collective
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=timedelta(minutes=60))
    # the final wait for rank 0's CPU baseline and node-wide drop-in pass on a CPU (gloo) group: an RCCL barrier would
    # keep a spinning kernel on every other GPU while the node pass runs its shards there
    cpu_group = dist.new_group(backend="gloo", timeout=timedelta(minutes=60)) if world > 1 and not rehearse else None
    from fedtree_amd.paillier import Device, Paillier
    from fedtree_amd.synth import logistic_gradients
    from fedtree_amd import _lib
    import ctypes

    dev = Device(local)
    lib = dev.lib
    if lib.fthe_ctx_device(dev.ctx) != local:
        raise SystemExit(f"rank {rank}: engine context on device {lib.fthe_ctx_device(dev.ctx)}, expected {local}")
    props = torch.cuda.get_device_properties(local)
    ident = {"rank": rank, "local_rank": local, "device": local,
             "pci": f"{getattr(props, 'pci_domain_id', 0):04x}:{getattr(props, 'pci_bus_id', 0):02x}:"
                    f"{getattr(props, 'pci_device_id', 0):02x}",
             "uuid": str(getattr(props, "uuid", ""))}
    t_kg = time.perf_counter()
    pl = Paillier(dev).keygen(KEY_BITS, seed=SEED)            # the server's key (same on every rank)
    keygen_s = time.perf_counter() - t_kg
    P = a.pairs
    g, h = logistic_gradients(P, SEED + rank)
    gh = torch.from_numpy(np.concatenate([g, h])).to(f"cuda:{local}")    # resident before timing
    m = torch.empty(2 * P, dtype=torch.int64, device=f"cuda:{local}")
    c = torch.empty((2 * P, 2 * pl.n_words), dtype=torch.int32, device=f"cuda:{local}")
    torch.cuda.synchronize()

    def step(i):
        _lib.check(lib.fthe_encode_fixed_dev(dev.ctx, ctypes.c_void_p(gh.data_ptr()), 2 * P,
                                             ctypes.c_void_p(m.data_ptr())), "encode")
        pl.encrypt_u64_dev(m, c, seed=SEED * 1000 + rank * 100 + i + 1)

    def sync():
        dev.sync()
        torch.cuda.synchronize()

    for i in range(a.warmup):
        step(i)
    sync()
    lib.fthe_prof_enable(dev.ctx, 1)
    wa = argparse.Namespace(**vars(a))
    wa.warmup = 0                                    # warm-up done above, before profiling is enabled
    elapsed_rank = timed_steps(lambda i: step(a.warmup + i), wa, world, sync)
    kms, launches, lane_mm, lanes, ems, elaunch, amacs, xmacs = (ctypes.c_double() for _ in range(8))
    _lib.check(lib.fthe_prof_exec_macs(dev.ctx, ctypes.byref(xmacs)), "prof_exec_macs")
    _lib.check(lib.fthe_prof_read(dev.ctx, ctypes.byref(kms), ctypes.byref(launches), ctypes.byref(lane_mm),
                                  ctypes.byref(lanes), ctypes.byref(ems), ctypes.byref(elaunch),
                                  ctypes.byref(amacs)))
    busy, ebusy = ctypes.c_double(), ctypes.c_double()
    _lib.check(lib.fthe_prof_busy(dev.ctx, ctypes.byref(busy), ctypes.byref(ebusy)), "prof_busy")
    lib.fthe_prof_enable(dev.ctx, 0)
    enc_rank = 2 * P * a.steps
    ident.update({"elapsed_s": round(elapsed_rank, 4), "encrypts_per_s": round(enc_rank / elapsed_rank, 1)})
    per_rank = gather_ranks(ident, world)
    if world > 1 and not rehearse:
        # one rank per GPU: every rank on its own device
        if len({p["pci"] + p["uuid"] for p in per_rank}) != world:
            raise SystemExit(f"bench.py: ranks share a device: {per_rank}")
    elapsed = max(p["elapsed_s"] for p in per_rank)
    enc_total = world * enc_rank
    value = enc_total / elapsed
    # 8M adds per call (1M-add calls of ~1.4 ms disagreed by 10%); at most P, so the operands are always the two
    # distinct halves c[:na], c[na:2na] (x = y would read half the bytes and inflate the rate)
    na_rank = min(P, 1 << 23)
    add_out = torch.empty((na_rank, 2 * pl.n_words), dtype=torch.int32, device=f"cuda:{local}")
    add_b = c[na_rank:2 * na_rank]

    def _add_call():
        pl.add_dev(c[:na_rank], add_b, add_out)
        dev.sync()
        return lib.fthe_last_kernel_ms(dev.ctx) * 1e-3

    adds = rank_adds(_add_call, na_rank, world, rank, sync)
    del add_out, add_b

    # -- roofline of the dominant kernel family (the exponentiation kernels, per-launch HIP
    # events on the engine stream, this rank).  Algorithmic work = the 32-bit MACs of the
    # executed algorithm, accumulated per launch by the engine: W(s) = 2 s^2 + s per Montgomery
    # product on s = 32-bit words of the modulus (SURVEY.md 8(d) unit), and the P-adic kernel's
    # own count per squaring / product mod P^2 (fthe.hip padic_alg: digit products + Barretts).
    # the p and q launches of a chunk run side by side on the engine's two compute streams (fthe.hip split_all):
    # kernel time is the union of the launch intervals (fthe_prof_busy), not their sum, which counts the shared
    # time twice; per launch, avg_expo_launch_ms is that union over the launches (the effective time per launch)
    # and avg_expo_launch_ms_in_flight the HIP-event duration of one launch beside its partner (what rocprof's
    # kernel trace reports per dispatch)
    alg_macs = amacs.value
    k_s = busy.value * 1e-3
    achieved = alg_macs / k_s / 1e12
    roof = {"bound": "valu", "kernel": "", "achieved": round(achieved, 3),
            "peak": round(PEAK_MAC_S / 1e12, 3), "unit": "TMAC/s", "frac": round(achieved * 1e12 / PEAK_MAC_S, 4),
            "traffic": None,
            "launches": int(launches.value), "avg_launch_ms": round(busy.value / max(1, launches.value), 3),
            "expo_launches": int(elaunch.value),
            "avg_expo_launch_ms": round(ebusy.value / max(1, elaunch.value), 3),
            "avg_expo_launch_ms_in_flight": round(ems.value / max(1, elaunch.value), 3),
            "expo_launches_overlap": round(ems.value / max(1e-9, ebusy.value), 3),
            "avg_expo_launch_ms_by_kernel": {},
            "alg_macs_per_encrypt": round(alg_macs / enc_rank),
            "survey_alg_macs_per_crt_encrypt_direct": ALG_MACS_PER_CRT_ENC,
            "montmuls_per_encrypt": round(lane_mm.value / enc_rank, 1),
            "kernel_share_of_step": round(k_s / elapsed_rank, 4)}
    # exponentiation kernels: the Montgomery program kernels and the P-adic one (pseudo-variant 1037)
    for S, kname in ((37, "fthe_montprog_s37"), (74, "fthe_montprog_s74"), (152, "fthe_montprog_s152"),
                     (1037, "fthe_padic_k37"), (1137, "fthe_padic_m37")):
        vms, vn = ctypes.c_double(), ctypes.c_double()
        lib.fthe_prof_variant(dev.ctx, S, ctypes.byref(vms), ctypes.byref(vn))
        if vn.value:
            roof["avg_expo_launch_ms_by_kernel"][kname] = round(vms.value / vn.value, 3)
    roof["kernel"] = " + ".join(roof["avg_expo_launch_ms_by_kernel"]) or "fthe_montprog"
    if "fthe_padic_m37" in roof["avg_expo_launch_ms_by_kernel"]:
        roof["kernel_note"] = ("fthe_padic_m37: the P-adic products on the VALU (v_mad_u64_u32, radix 2^28) and both "
                               "Barrett reductions of every product on the matrix cores (v_mfma_i32_32x32x32_i8, "
                               "136 per squaring per wave); still VALU-bound (VALUBusy in the PMC profile), so "
                               "achieved/frac stay in VALU MAC units; DESIGN.md 3 'Matrix-core Barrett'")
    # the metric's unit of SURVEY 8(d) (W(64) Montgomery products, 1.2 e products per e-bit exponent) for
    # the work the direct-y CRT encrypt must do -- two exponentiations mod P^2 (s = 64) by the 1024-bit P:
    # above 1 because the P-adic digits need 2.1x fewer MACs than Montgomery products mod P^2, not because
    # work is skipped (tests/test_gpu_direct_y.py pins the timed path bit-exactly)
    survey_macs_direct = 2 * 1.2 * 1024 * W64
    roof["frac_survey_unit"] = round(value / world * survey_macs_direct / PEAK_MAC_S, 4)
    roof["frac_survey_unit_textbook_crt"] = round(value / world * ALG_MACS_PER_CRT_ENC / PEAK_MAC_S, 4)
    roof["frac_survey_unit_note"] = (
        "value x 2 x 1.2 x 1024 x W(64) MACs (two Montgomery exponentiations mod P^2 by the 1024-bit P) over the "
        "39.3 T MAC/s peak; _textbook_crt charges 4.06e7 (exponent n mod P(P-1)).  Both exceed 1 because the "
        "executed P-adic algorithm needs 9.49e6 MACs per encrypt (alg_macs_per_encrypt), 2.1x fewer than the "
        "Montgomery count of the same exponentiations; frac (the algorithmic unit) and issue_frac (executed "
        "instructions) measure the hardware")
    if xmacs.value and "fthe_padic_k37" in roof["avg_expo_launch_ms_by_kernel"]:
        # the P-adic kernel in issue terms: its v_mad instructions (radix 2^28, counted per program by the
        # engine) over its own launch time, against the same 39.3 T/s issue peak
        vms, vn = ctypes.c_double(), ctypes.c_double()
        lib.fthe_prof_variant(dev.ctx, 1037, ctypes.byref(vms), ctypes.byref(vn))
        rate = xmacs.value / (vms.value * 1e-3) if vms.value else 0.0
        roof["unit_note"] = ("achieved/frac count the 32-bit MACs of the executed algorithm: the P-adic products need "
                             f"{round(alg_macs / enc_rank / 1e6, 2)}e6 per encrypt, 2.1x fewer than the Montgomery CRT's "
                             "1.98e7 (round 1), so frac falls while encrypts/s rise; padic_frac_executed_mads is the "
                             "kernel's issue efficiency (its v_mad instructions over its launch time), DESIGN.md 3")
        roof["padic_executed_mads_per_encrypt"] = round(xmacs.value / enc_rank)
        roof["padic_frac_executed_mads"] = round(rate / PEAK_MAC_S, 4)
        roof["padic_frac_of_measured_mad_peak"] = round(rate / MEASURED_MAD_S, 4)
    expo_kernel = next((kn for kn in ("fthe_padic_m37", "fthe_padic_k37") if kn in roof["avg_expo_launch_ms_by_kernel"]),
                       "fthe_montprog_s74")
    # HBM traffic per full-chunk exponentiation launch from the committed PMC passes
    # (tools/pmc_round.sh; 2*FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md HBM section)
    pmc = {}
    prof_hbm = os.path.join(ROOT, "profiles", PMC_FILE)
    if os.path.exists(prof_hbm):
        pmc = json.load(open(prof_hbm))
        roof["traffic"] = pmc.get("enc", {}).get(expo_kernel, {}).get("hbm_bytes_per_launch")
        roof["traffic_source"] = f"profiles/{PMC_FILE} ({expo_kernel} full-chunk launch)"
        ek = pmc.get("enc", {}).get(expo_kernel, {})
        # the effective time per launch (the union), as the counters are per launch over the whole chip
        kms_expo = roof["avg_expo_launch_ms"]
        simd_cycles = 1024 * 2.4e9 * kms_expo * 1e-3     # every SIMD's cycles over the live launch time
        if ek.get("SQ_INSTS_VALU") and kms_expo:
            # executed issue: the kernel's VALU wave-instructions (PMC, per launch) x 4 cycles (a wave64
            # v_mad_u64_u32, 80+% of the stream, issues once per 4 cycles per SIMD) over the SIMD cycles
            roof["issue_frac"] = round(ek["SQ_INSTS_VALU"] * 4 / simd_cycles, 4)
            roof["issue_note"] = (f"{expo_kernel}: SQ_INSTS_VALU {ek['SQ_INSTS_VALU']:.4g} wave-instructions per full-chunk "
                                  f"launch (profiles/{PMC_FILE}) x 4 cycles / (1,024 SIMDs x 2.4 GHz x {kms_expo} ms, "
                                  "this run's HIP-event launch time)")
        if ek.get("SQ_INSTS_MFMA") and kms_expo:
            # matrix cores: SQ_VALU_MFMA_BUSY_CYCLES counts 32 cycles per i8 32x32x32 MFMA; the i8 dense peak
            # is 2x the bf16 rate (MI355X_MICROARCH.md MFMA table): 32x32x32x2 ops per 32 cycles per SIMD
            i8_peak = 1024 * 2.4e9 * (32 * 32 * 32 * 2) / 32
            i8_ops = ek["SQ_INSTS_MFMA"] * 32 * 32 * 32 * 2 / (kms_expo * 1e-3)
            roof["matrix_core"] = {"mfma_per_launch": ek["SQ_INSTS_MFMA"],
                                   "mfma_busy_frac": round(ek.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / simd_cycles, 4),
                                   "i8_tops": round(i8_ops / 1e12, 1), "i8_dense_peak_tops": round(i8_peak / 1e12, 1),
                                   "frac_of_i8_peak": round(i8_ops / i8_peak, 4),
                                   "valu_busy_pct": ek.get("VALUBusy"), "source": f"profiles/{PMC_FILE}",
                                   "note": "v_mfma_i32_32x32x32_i8: both Barrett products of every P-adic product"}
    # what the traffic is: SURVEY 8(d) algorithmic bytes (772 B per encrypt, half per prime launch) vs the
    # operand reads of the one-lane design (each window multiplication reads a 296-B table entry per lane)
    # lanes per exponentiation launch of the timed path: fthe.hip enc_chunk_lanes() (2 x chunk_lanes())
    lanes = int(os.environ.get("FTHE_ENC_CHUNK") or 2 * int(os.environ.get("FTHE_CHUNK") or 393216))
    roof["lanes_per_expo_launch"] = lanes
    roof["algorithmic_bytes_per_launch"] = lanes * 772 // 2
    roof["window_operand_bytes_per_launch_model"] = int(lanes * (190 + 16 + 4) * 296)
    roof["traffic_note"] = ("HBM bytes are the per-lane window-table traffic (~180 window multiplications reading and "
                            "32 table stores writing 296 B per lane per exponentiation), ~300 GB/s = ~4% of HBM "
                            "bandwidth in a VALU-bound kernel")


    secondary = {}
    p1k_cpu = None
    if rank == 0 and world == 1 and not a.no_secondary:      # N=1 runs only: scaling runs stay lean
        # CRT decrypt of every ciphertext the step produced (configs[2]'s decrypt half: 20M at 10M pairs),
        # device-resident, one call
        nd = 2 * P
        low = torch.empty(nd, dtype=torch.int64, device=f"cuda:{local}")
        pl.decrypt_u64_dev(c[:nd], low)
        dev.sync()
        secondary["crt_decrypt_per_s"] = round(nd / (lib.fthe_last_kernel_ms(dev.ctx) * 1e-3))
        secondary["crt_decrypt_ciphertexts"] = nd
        ok = torch.equal(low, m[:nd])
        secondary["decrypt_roundtrip_ok"] = bool(ok)
        # opt-in short-plaintext decrypt (plaintext < p, true of every FedTree codec value): p half only
        pl.decrypt_u64_dev(c[:nd], low, short=True)
        dev.sync()
        secondary["crt_decrypt_short_per_s"] = round(nd / (lib.fthe_last_kernel_ms(dev.ctx) * 1e-3))
        secondary["decrypt_short_roundtrip_ok"] = bool(torch.equal(low, m[:nd]))
        # the same CRT encrypt with injected r (stage A r^Q mod P, then stage B): the path the golden,
        # random-vs-oracle and configs[1] tests pin bit-exactly; r < 2^(n_bits - 2) < n drawn by torch
        low = low[:min(2 * P, 1 << 20)]
        nr = min(2 * P, 1 << 20)
        gen = torch.Generator(device=f"cuda:{local}").manual_seed(SEED + 5)
        rinj = torch.randint(-2**31, 2**31 - 1, (nr, pl.n_words), dtype=torch.int32, device=f"cuda:{local}",
                             generator=gen)
        rinj[:, -1] &= 0x3FFFFFFF
        rinj[:, 0] |= 1
        cinj = torch.empty((nr, 2 * pl.n_words), dtype=torch.int32, device=f"cuda:{local}")
        pl.encrypt_u64_dev(m[:nr], cinj, r=rinj)
        dev.sync()
        pl.encrypt_u64_dev(m[:nr], cinj, r=rinj)
        dev.sync()
        inj_rate = nr / (lib.fthe_last_kernel_ms(dev.ctx) * 1e-3)
        pl.decrypt_u64_dev(cinj, low[:nr])
        dev.sync()
        secondary["crt_encrypt_injected_r"] = {
            "encrypts_per_s": round(inj_rate), "ciphertexts": nr, "roundtrip_ok": bool(torch.equal(low[:nr], m[:nr])),
            "vs_value": round(inj_rate / value, 3),
            "note": "two-stage CRT with caller r (r^(q mod p-1) mod p on s37, then mod p^2 on s74); the headline "
                    "draws y_P directly (one stage), pinned bit-exactly by tests/test_gpu_direct_y.py"}
        del rinj, cinj
        # public-key encrypt (a party without the factorization, party.h:118-142) and the
        # opt-in fixed-base randomizer (r = h^alpha, include/fthe.h FTHE_ENC_FIXED_BASE; not
        # the reference's uniform-r algorithm, so never the headline `value`)
        npub = min(2 * P, 393216)                        # four whole launches of 98,304 (no partial round)
        pl.encrypt_u64_dev(m[:npub], c[:npub], seed=5, public=True)
        dev.sync()
        secondary["public_encrypt_per_s"] = round(npub / (lib.fthe_last_kernel_ms(dev.ctx) * 1e-3))
        # fthe_nadic_b76's issue: its VALU wave-instructions per ciphertext (PMC, one 98,304-ciphertext launch) x 4
        # cycles at this rate over every SIMD's cycles -- the public path's counterpart of roofline.issue_frac
        pb = pmc.get("pub", {}).get("fthe_nadic_b76", {})
        if pb.get("SQ_INSTS_VALU"):
            per_ct = pb["SQ_INSTS_VALU"] / 98304
            secondary["public_encrypt_issue"] = {
                "valu_wave_instr_per_ciphertext": round(per_ct),
                "valu_issue_frac": round(per_ct * secondary["public_encrypt_per_s"] * 4 / (1024 * 2.4e9), 4),
                "valu_busy_pct": pb.get("VALUBusy"), "occupancy_pct": pb.get("OccupancyPercent"),
                "source": f"profiles/{PMC_FILE} pub"}
        t0 = time.perf_counter()
        pl.set_fixed_base(None)
        fb_build_s = time.perf_counter() - t0
        nfb = min(2 * P, 1 << 21)
        cfb = torch.empty((nfb, 2 * pl.n_words), dtype=torch.int32, device=f"cuda:{local}")
        fbr = {"table_build_s": round(fb_build_s, 3)}
        for name, pub in (("crt_encrypt_per_s", False), ("public_encrypt_per_s", True)):
            pl.encrypt_u64_dev(m[:nfb], cfb, seed=6, public=pub, fixed_base=True)
            dev.sync()
            fbr[name] = round(nfb / (lib.fthe_last_kernel_ms(dev.ctx) * 1e-3))
        lowfb = torch.empty(nfb, dtype=torch.int64, device=f"cuda:{local}")
        pl.decrypt_u64_dev(cfb, lowfb)
        dev.sync()
        fbr["decrypt_roundtrip_ok"] = bool(torch.equal(lowfb, m[:nfb]))
        fbr["note"] = ("opt-in FTHE_ENC_FIXED_BASE: c = (1+mn) hs^alpha, hs = h^n mod n^2, alpha from the device "
                       "CSPRNG; 16-bit-window tables; r = h^alpha ranges over a subgroup, not the reference's distribution")
        secondary["fixed_base"] = fbr
        # latency of one GHPair (2 ciphertexts), host in and out: decrypt_gh (server.h:69-78) per node, from
        # OpenMP threads (FLtrainer.cpp:758-764).  One lane runs each modexp serially; batches this small run the
        # mod-q half on the context's side stream beside the mod-p half, so a lone pair costs one exponentiation
        # (the short decrypt has only the p half).  Concurrent callers on their own contexts overlap.
        mh = np.array([123456, 654321], dtype=np.uint64)
        ch = pl.encrypt_u64(mh, seed=3)
        pl.decrypt_u64(ch)
        t0 = time.perf_counter()
        for _ in range(5):
            pl.decrypt_u64(ch)
        dec1_ms = (time.perf_counter() - t0) / 5 * 1e3
        t0 = time.perf_counter()
        for _ in range(5):
            pl.encrypt_u64(mh, seed=4)
        enc1_ms = (time.perf_counter() - t0) / 5 * 1e3
        secondary["single_pair_latency_ms"] = {"decrypt": round(dec1_ms, 2), "encrypt": round(enc1_ms, 2),
                                               "decrypt_short": None}
        t0 = time.perf_counter()
        for _ in range(5):
            pl.decrypt_u64(ch, short=True)
        secondary["single_pair_latency_ms"]["decrypt_short"] = round((time.perf_counter() - t0) / 5 * 1e3, 2)
        # decrypt_gh from 32 OpenMP-style threads on one key: merged by the key's coalescing queue
        import threading
        nthr, rounds = 32, 12                      # the first round has no linger history
        cts = [pl.encrypt_u64(np.array([7 * i, 11 * i], dtype=np.uint64), seed=50 + i) for i in range(nthr)]
        ok = [True] * nthr
        go = threading.Barrier(nthr + 1)

        def _dgh(i):
            go.wait()
            for _ in range(rounds):
                ok[i] &= bool(np.array_equal(pl.decrypt_u64_shared(cts[i]), [7 * i, 11 * i]))

        ths = [threading.Thread(target=_dgh, args=(i,)) for i in range(nthr)]
        for t in ths:
            t.start()
        go.wait()
        t0 = time.perf_counter()
        for t in ths:
            t.join()
        ms = (time.perf_counter() - t0) * 1e3 / rounds
        secondary["concurrent_decrypt_gh"] = {"threads": nthr, "ms_per_round": round(ms, 2),
                                              "pairs_per_s": round(nthr / ms * 1e3), "ok": all(ok),
                                              "note": "fthe_decrypt_shared: concurrent single-pair calls on one key "
                                                      "merged into one launch (group commit)"}
        # GHPair::operator+ in the USE_HIP build: one Paillier_HIP_Pub::add -> fthe_add_shared per call
        # (integration/fthe_ghpair_key.h), serially and from 32 threads on one key
        rows = pl.encrypt_u64(np.arange(1, 65, dtype=np.uint64), seed=77)
        acc = rows[:1].copy()
        pl.add_shared(acc, rows[1:2], out=acc)
        nser = 200
        t0 = time.perf_counter()
        for i in range(nser):
            pl.add_shared(acc, rows[1 + i % 63:2 + i % 63], out=acc)
        ser_us = (time.perf_counter() - t0) / nser * 1e6
        nthr, per = 32, 50
        accs = [rows[i:i + 1].copy() for i in range(nthr)]
        go = threading.Barrier(nthr + 1)

        def _adds(i):
            go.wait()
            for j in range(per):
                pl.add_shared(accs[i], rows[(i + j) % 64:(i + j) % 64 + 1], out=accs[i])

        ths = [threading.Thread(target=_adds, args=(i,)) for i in range(nthr)]
        for t in ths:
            t.start()
        go.wait()
        t0 = time.perf_counter()
        for t in ths:
            t.join()
        conc_s = time.perf_counter() - t0
        secondary["ghpair_operator_add"] = {
            "serial_us_per_add": round(ser_us, 1), "threads": nthr,
            "concurrent_adds_per_s": round(nthr * per / conc_s),
            "note": "one ciphertext add per call through the key's coalescing queue, as GHPair::operator+ / += "
                    "issue them (host rows in and out, one four-lane product launch per merged batch); the "
                    "batch entry points (merge, histogram, reduce_segments) are the throughput path; Python "
                    "threads (GIL between calls): the C++ OpenMP rate is histogram_loop_unchanged_callers"}
        # the native tools below run the drop-in on this rank's GPU only (FTHE_DEVICES defaults to every visible
        # GPU: on a multi-GPU node an N = 1 run would otherwise shard them over the whole node)
        one_gpu_env = dict(os.environ, FTHE_DEVICES=str(local))
        # the same operators from C++ OpenMP threads, as FedTree's histogram loop issues them unchanged
        # (integration/ghpair_rate.cpp, hist_tree_builder.cpp:572-591): a child process, its own context
        exe = os.path.join(ROOT, "tools", "bin", "ghpair_rate")
        hl = {"note": "integration/ghpair_rate.cpp: OpenMP over features, `dest = dest + src` per instance through "
                      "GHPair::operator+ on the USE_HIP key (2 host adds x y mod n^2 per operator; empty bins "
                      "promoted from the key's GPU-filled randomizer pool), every bin checked by decryption; "
                      "reference_add_same_threads_per_s: the reference's Paillier_GMP::add (mpz_mul + mpz_mod) on "
                      "the same threads and operands in the same run; compare cpu_baseline.ops.p2048_add too. "
                      "sub: the sibling subtraction (hist_tree_builder.cpp:672-680), OpenMP over 4,096 bins, "
                      "`dest[i] = father[i] - child[i]` through GHPair::operator- (2 x mul(x, 2^64-1) + 2 adds; a "
                      "single-element mul is a host mpz_powm, as paillier_gpu.cu:65-67), every bin decrypted; "
                      "reference_sub_same_threads_per_s: mpz_powm + mpz_mul/mpz_mod on the same threads and operands; "
                      "both legs interleaved over 7 rounds at the lease's core count, rates from the medians, "
                      "vs_reference_* the median per-round ratio"}
        # at the lease's core count only (an oversubscribed 64-thread leg on a 16-core quota measured the host
        # scheduler, 0.43-1.10x between runs); both legs interleaved, 7 rounds, the median per-round ratio
        for thr in (host_cpu()["threads_used"],):
            try:
                r = subprocess.run([exe, str(KEY_BITS), str(thr), "8192", "16", "4096", "7"], capture_output=True,
                                   text=True, timeout=240, env=one_gpu_env)
                hl[f"threads_{thr}"] = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else \
                    {"error": f"rc {r.returncode}: {r.stderr.strip()[-300:]}"}
            except (OSError, subprocess.TimeoutExpired, ValueError, IndexError) as ex:
                hl[f"threads_{thr}"] = {"error": repr(ex)[:300]}
        secondary["histogram_loop_unchanged_callers"] = hl
        # the batch boundary at FedTree's own types: Paillier_HIP::encrypt / decrypt(SyncArray<GHPair>&) with
        # mpz_t marshalling of every ciphertext (integration/ghpair_e2e.cpp; server.h:105-135)
        try:
            r = subprocess.run([os.path.join(ROOT, "tools", "bin", "ghpair_e2e"), str(KEY_BITS), "2000000", "2"],
                               capture_output=True, text=True, timeout=240, env=one_gpu_env)
            ge = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else \
                {"error": f"rc {r.returncode}: {r.stderr.strip()[-300:]}"}
        except (OSError, subprocess.TimeoutExpired, ValueError, IndexError) as ex:
            ge = {"error": repr(ex)[:300]}
        ge["note"] = ("Server::encrypt_gh_pairs / decrypt_gh_pairs through Paillier_HIP on SyncArray<GHPair> with "
                      "mpz_t fields (host in and out, PCIe, mpz import/export per ciphertext); compare "
                      "e2e_host_encrypt_per_s (numpy rows) and the device-resident value")
        secondary["ghpair_e2e"] = ge
        # the host side of an N-GPU server: the same mpz_t <-> row marshalling for 1, 2, 4, 8 concurrent
        # shards of 1,048,576 pairs, no kernels (integration/marshal_rate.cpp) -- can one host feed 8 GPUs?
        try:
            r = subprocess.run([os.path.join(ROOT, "tools", "bin", "marshal_rate"), str(KEY_BITS), "1048576", "3",
                                "1,2,4,8"], capture_output=True, text=True, timeout=240)
            mr = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else \
                {"error": f"rc {r.returncode}: {r.stderr.strip()[-300:]}"}
        except (OSError, subprocess.TimeoutExpired, ValueError, IndexError) as ex:
            mr = {"error": repr(ex)[:300]}
        mr["note"] = ("Paillier_HIP::encrypt/decrypt(SyncArray<GHPair>&)'s host marshalling alone (codec + rows <-> mpz "
                      "limbs, up to 16 threads per shard, one host thread per shard), aggregated ciphertexts/s; the "
                      "8-GPU feed needs 8 x the device rate (value) on the encrypt side")
        secondary["host_marshalling_shards"] = mr
        # key generation (homo_init; re-run every round in the vertical simulation, FLtrainer.cpp:556):
        # host prime search on up to 16 threads + device key set-up
        t0 = time.perf_counter()
        for i in range(4):
            Paillier(dev).keygen(KEY_BITS, seed=SEED + 100 + i)
        secondary["keygen_s"] = {"first": round(keygen_s, 4), "mean_of_4": round((time.perf_counter() - t0) / 4, 4),
                                 "note": "Paillier-2048 (two 1024-bit primes: sieved windows, BPSW on up to 16 host "
                                         "threads), derivation and device constants"}
        # opt-in public exact fixed-base randomizer (parties, Party::encrypt_histogram party.h:118-142):
        # the key holder publishes checked bases hs_i = t_i^n, <t_i> = Z_n^*; the party (n only) draws
        # r^n = prod hs_i^y_i with y_i below n 2^64 -- within 3 * 2^-64 of the reference's distribution
        t0 = time.perf_counter()
        party = pl.public(bases=pl.public_bases())
        dev.sync()
        pb_build_s = time.perf_counter() - t0
        party.encrypt_u64_dev(m[:nfb], cfb, seed=13, fixed_base_exact=True)
        dev.sync()
        party.encrypt_u64_dev(m[:nfb], cfb, seed=14, fixed_base_exact=True)
        dev.sync()
        pb_rate = nfb / (lib.fthe_last_kernel_ms(dev.ctx) * 1e-3)
        pl.decrypt_u64_dev(cfb, lowfb)
        dev.sync()
        secondary["public_fixed_base_exact"] = {
            "bases_and_table_build_s": round(pb_build_s, 3), "public_encrypt_per_s": round(pb_rate),
            "vs_public_default": round(pb_rate / secondary["public_encrypt_per_s"], 2),
            "decrypt_roundtrip_ok": bool(torch.equal(lowfb, m[:nfb])),
            "note": "opt-in FTHE_ENC_FIXED_BASE_EXACT on a public key: 3 published bases (checked at every prime "
                    "< 2^24 dividing p-1 or q-1, rank 2 where both), y_i uniform below 2^2112: 396 gathered "
                    "4096-bit products instead of a 2048-bit exponentiation mod n^2"}
        del party
        # opt-in exact fixed-base randomizer (key holder): three generators of G_P per prime and
        # uniform exponents -> exactly the reference's r^n distribution (include/fthe.h);
        # the table build is timed with the encryptions, as a per-step cost would be
        t0 = time.perf_counter()
        pl.set_fixed_base_exact(seed=0)
        dev.sync()
        xb_build_s = time.perf_counter() - t0
        pl.encrypt_u64_dev(m[:nfb], cfb, seed=8, fixed_base_exact=True)
        dev.sync()
        t0 = time.perf_counter()
        pl.encrypt_u64_dev(m[:nfb], cfb, seed=9, fixed_base_exact=True)
        dev.sync()
        xb_s = time.perf_counter() - t0
        pl.decrypt_u64_dev(cfb, lowfb)
        dev.sync()
        secondary["fixed_base_exact"] = {
            "table_build_s": round(xb_build_s, 3),
            "crt_encrypt_per_s": round(nfb / xb_s),
            "crt_encrypt_per_s_incl_table_build_per_20M": round(2 * P / (xb_build_s + 2 * P * xb_s / nfb)),
            "decrypt_roundtrip_ok": bool(torch.equal(lowfb, m[:nfb])),
            "note": "opt-in FTHE_ENC_FIXED_BASE_EXACT: r^n mod P^2 = prod_i gam_i^y_i, gam_1..3 generating G_P "
                    "(every prime < 2^24 dividing P-1 checked; failure < 2^-66 per key), y_i uniform in [1, P): the "
                    "reference's ciphertext distribution, 192 gathered products per prime"}
        # the same with a key whose P - 1 is factored (FTHE_KEYGEN_KNOWN_ORDER): one generator per prime
        t0 = time.perf_counter()
        pko = Paillier(dev).keygen(KEY_BITS, seed=SEED + 7, known_order=True)
        ko_keygen_s = time.perf_counter() - t0
        t0 = time.perf_counter()
        pko.set_fixed_base_exact(seed=0)
        dev.sync()
        ko_build_s = time.perf_counter() - t0
        pko.encrypt_u64_dev(m[:nfb], cfb, seed=8, fixed_base_exact=True)
        dev.sync()
        t0 = time.perf_counter()
        pko.encrypt_u64_dev(m[:nfb], cfb, seed=9, fixed_base_exact=True)
        dev.sync()
        ko_s = time.perf_counter() - t0
        pko.decrypt_u64_dev(cfb, lowfb)
        dev.sync()
        secondary["fixed_base_exact"]["known_order_key"] = {
            "keygen_s": round(ko_keygen_s, 3), "table_build_s": round(ko_build_s, 3),
            "crt_encrypt_per_s": round(nfb / ko_s), "decrypt_roundtrip_ok": bool(torch.equal(lowfb, m[:nfb])),
            "note": "FTHE_KEYGEN_KNOWN_ORDER key (p-1, q-1 factored): one verified generator per prime, 64 gathered "
                    "products per prime, exactly the reference's ciphertext distribution"}
        # parties of a known-order key: 2 published bases, the second with a 128-bit exponent
        kparty = pko.public(bases=pko.public_bases())
        kparty.encrypt_u64_dev(m[:nfb], cfb, seed=15, fixed_base_exact=True)
        dev.sync()
        kparty.encrypt_u64_dev(m[:nfb], cfb, seed=16, fixed_base_exact=True)
        dev.sync()
        kp_rate = nfb / (lib.fthe_last_kernel_ms(dev.ctx) * 1e-3)
        pko.decrypt_u64_dev(cfb, lowfb)
        dev.sync()
        secondary["public_fixed_base_exact"]["known_order_key"] = {
            "public_encrypt_per_s": round(kp_rate), "decrypt_roundtrip_ok": bool(torch.equal(lowfb, m[:nfb])),
            "note": "t_1 of order lcm(p-1, q-1) (full exponent) and t_2 generating Z_n^*/<t_1> = Z_gcd(p-1,q-1) "
                    "(128-bit exponent): 140 gathered products"}
        del cfb, lowfb, pko, kparty
        # ciphertext adds (x*y mod n^2, 4096-bit n^2 on the four-lane kernel), device-resident
        na = na_rank                                     # 8M adds per timed call, distinct halves (as ciphertext_adds)
        o = torch.empty((na, 2 * pl.n_words), dtype=torch.int32, device=f"cuda:{local}")
        pl.add_dev(c[:na], c[na:2 * na], o)
        dev.sync()
        add_ts = []
        for _ in range(5):                               # the median of 5 timed calls (one call: +-5%)
            pl.add_dev(c[:na], c[na:2 * na], o)
            dev.sync()
            add_ts.append(lib.fthe_last_kernel_ms(dev.ctx) * 1e-3)
        add_s = sorted(add_ts)[2]
        secondary["p2048_add_per_s"] = round(na / add_s)
        secondary["p2048_add_per_s_range"] = [round(na / max(add_ts)), round(na / min(add_ts))]
        prods = lib.fthe_last_montmuls(dev.ctx) / na          # 4096-bit products per add
        # the add kernel's HBM side (north star): algorithmic bytes (2 rows in, 1 out, 512 B each)
        # over the live launch time, and the PMC-measured bytes of one launch
        padd = pmc.get("add", {})
        kname = "fthe_addb_q152" if "fthe_addb_q152" in padd else "fthe_montprog_s152"
        pk = padd.get(kname, {})
        rate = na / add_s
        # fthe_addb_q152 (gen_addb.py): z = x y on the VALU by one level of Karatsuba on 76-limb halves,
        # 3 x 76 x 76 radix-2^27 v_mad_u64_u32 per add (152 x 152 in the "nokara" generator variant); both
        # Barrett products (q1 mu, q3 n^2) on the i8 matrix cores, 338 v_mfma_i32_16x16x64_i8 per 16 adds
        valu_macs = 3 * 76 * 76
        i8_macs = 338 * 16 * 16 * 64 / 16
        i8_peak = 1024 * 2.4e9 * (32 * 32 * 32 * 2) / 32
        secondary["p2048_add_hbm"] = {"algorithmic_GBps": round(na * 1536 / add_s / 1e9, 1),
                                      "pmc_GBps": pk.get("hbm_GBps"), "pmc_VALUBusy": pk.get("VALUBusy"),
                                      # the same counters calibrated on the kernel's own access pattern (x = y:
                                      # a known byte count), and the algorithmic bytes of the profiled launch
                                      "pmc_GBps_calibrated": pk.get("calibration", {}).get("hbm_GBps"),
                                      "pmc_calibration": pk.get("calibration"),
                                      "pmc_launch_ms": pk.get("launch_ms"),
                                      "pmc_algorithmic_GBps": (round(pk["algorithmic_bytes_per_launch"]
                                                                     / (pk["launch_ms"] * 1e-3) / 1e9, 1)
                                                               if pk.get("launch_ms") else None),
                                      "pmc_kernel": kname if pk else None,
                                      "pmc_source": f"profiles/{PMC_FILE}" if pk else None,
                                      "peak_GBps": 8000,
                                      "bound": "valu: x y on the VALU (one 4096-bit product per add), its Barrett "
                                               "reduction by n^2 on the i8 matrix cores (fthe_addb_q152)",
                                      # VALU roofline: executed VALU MADs per add and the survey's
                                      # unit, one W(128) = 2*128^2+128 MACs per add
                                      "products_per_add": prods,
                                      "valu_macs_per_add": valu_macs,
                                      "executed_over_algorithmic_macs": round(valu_macs / (2 * 128 * 128 + 128), 3),
                                      "valu_frac_executed": round(rate * valu_macs / PEAK_MAC_S, 4),
                                      # issue: the kernel's VALU wave-instructions per add (PMC) x 4 cycles at
                                      # this rate over every SIMD's cycles (as roofline.issue_frac)
                                      "valu_issue_frac": (round(pk["SQ_INSTS_VALU"] / pk["rows_out_per_launch"] * rate
                                                                * 4 / (1024 * 2.4e9), 4)
                                                          if pk.get("SQ_INSTS_VALU") and pk.get("rows_out_per_launch")
                                                          else None),
                                      "valu_frac_survey_unit": round(rate * (2 * 128 * 128 + 128) / PEAK_MAC_S, 4),
                                      "matrix_core": {"i8_macs_per_add": round(i8_macs),
                                                      "frac_of_i8_dense_peak": round(rate * i8_macs * 2 / i8_peak, 4)}}
        # the same adds on Montgomery-resident rows (x R mod n^2, include/fthe.h): one product per add
        # instead of two; rows converted in/out once per chain (conversion not in this rate)
        mr = torch.empty((2 * na, 2 * pl.n_words), dtype=torch.int32, device=f"cuda:{local}")
        src = c[:2 * na]
        pl.to_mont_dev(src, mr)
        pl.add_mont_dev(mr[:na], mr[na:], o)
        dev.sync()
        pl.add_mont_dev(mr[:na], mr[na:], o)
        dev.sync()
        mont_s = lib.fthe_last_kernel_ms(dev.ctx) * 1e-3
        chk = torch.empty_like(o)
        pl.from_mont_dev(o, chk)
        ref = torch.empty_like(o)
        pl.add_dev(src[:na], src[na:], ref)
        dev.sync()
        secondary["p2048_add_mont_resident"] = {
            "adds_per_s": round(na / mont_s), "vs_add": round(add_s / mont_s, 2),
            "matches_add_after_from_mont": bool(torch.equal(chk, ref)),
            "note": "fthe_add_mont_dev on x R mod n^2 rows: (aR)(bR)R^-1 = (ab)R, one 4096-bit Montgomery product "
                    "per add; to/from conversion (one product each) once per device-resident chain"}
        del o, mr, chk, ref
        # configs[1]: Paillier-1024, 100k gradient pairs (200k ciphertexts), device-resident
        p1k = Paillier(dev).keygen(1024, seed=SEED + 1)
        n1k = min(2 * P, 200_000)
        c1k = torch.empty((n1k, 2 * p1k.n_words), dtype=torch.int32, device=f"cuda:{local}")
        r1k = {}
        for name, kw in (("crt_encrypt_per_s", {}), ("public_encrypt_per_s", {"public": True}),
                         ("crt_encrypt_fixed_base_exact_per_s", {"fixed_base_exact": True})):
            p1k.encrypt_u64_dev(m[:n1k], c1k, seed=11, **kw)
            dev.sync()
            p1k.encrypt_u64_dev(m[:n1k], c1k, seed=12, **kw)
            dev.sync()
            r1k[name] = round(n1k / (lib.fthe_last_kernel_ms(dev.ctx) * 1e-3))
        low1k = torch.empty(n1k, dtype=torch.int64, device=f"cuda:{local}")
        p1k.decrypt_u64_dev(c1k, low1k)
        dev.sync()
        r1k["crt_decrypt_per_s"] = round(n1k / (lib.fthe_last_kernel_ms(dev.ctx) * 1e-3))
        r1k["roundtrip_ok"] = bool(torch.equal(low1k, m[:n1k]))
        r1k["ciphertexts"] = n1k
        secondary["p1024_100k_pairs"] = r1k
        p1k_cpu = p1k                                  # the CPU baseline's P-1024 key
        del c1k, low1k, p1k
        # configs[3]: 8-party merge of 256 x 4096 bins x {g, h} (hist_tree_builder.cpp:1015-1058)
        bins, parties = 2 * 256 * 4096, 8
        if 2 * P >= bins:
            x = c[:bins].unsqueeze(0).expand(parties, bins, 2 * pl.n_words).contiguous()
            ho = torch.empty((bins, 2 * pl.n_words), dtype=torch.int32, device=f"cuda:{local}")
            mts = []
            for _ in range(3):                           # one merge: +-5% between calls on the same box
                pl.reduce_kway_dev(x, parties, ho)
                dev.sync()
                mts.append(lib.fthe_last_kernel_ms(dev.ctx))
            ms_h = sorted(mts)[1]
            secondary["hist_merge_8party_1M_bins"] = {"ms": round(ms_h, 2), "ms_min": round(min(mts), 2),
                                                      "ms_max": round(max(mts), 2), "ciphertexts_out": bins,
                                                      "adds_per_s": round(bins * (parties - 1) / (ms_h * 1e-3)),
                                                      "note": "median of 3 calls; seven launches of fthe_addb_q152 "
                                                              "over the 2M bins (out = x0 x1, then out = out x_j)"}
            del x, ho
        # party-side node histogram on the device (hist_tree_builder.cpp:565-595): 1M instances
        # x 28 features x 255 bins, g and h planes = 55.7M member products, CSR built in HBM
        nh, ncol = min(P, 1_000_000), 28
        gen = torch.Generator(device=f"cuda:{local}").manual_seed(SEED)
        hbins = torch.randint(0, 256, (nh, ncol), dtype=torch.uint8, device=f"cuda:{local}", generator=gen)
        hcut = (np.arange(ncol + 1) * 255).astype(np.int32)
        hx = torch.cat([c[:nh], c[P:P + nh]])                          # g plane, h plane
        hout = torch.empty((2 * int(hcut[-1]), 2 * pl.n_words), dtype=torch.int32, device=f"cuda:{local}")
        pl.histogram_dev(hx[:8192], 4096, 2, hbins[:4096], hcut, 255, hout)
        dev.sync()
        t0 = time.perf_counter()
        pl.histogram_dev(hx, nh, 2, hbins, hcut, 255, hout)
        dev.sync()
        dt = time.perf_counter() - t0
        members = int((hbins != 255).sum().item()) * 2
        secondary["histogram_node_dev"] = {"instances": nh, "features": ncol, "bins": int(hcut[-1]), "planes": 2,
                                           "s": round(dt, 4), "member_adds_per_s": round(members / dt)}
        del hx, hout, hbins
        # end to end, host-resident in/out: chunked, double-buffered transfers on a copy
        # stream overlapped with the kernels (pageable caller buffers go through pinned staging)
        ne = min(2 * P, 1 << 21)
        mh = m[:ne].cpu().numpy().view(np.uint64).copy()
        pl.encrypt_u64(mh, seed=3)                       # warm: the full-size path's pinned staging and slots
        t0 = time.perf_counter()
        ch = pl.encrypt_u64(mh, seed=3)
        dt = time.perf_counter() - t0
        secondary["e2e_host_encrypt_per_s"] = round(ne / dt)
        if "encrypts_per_s" in secondary.get("ghpair_e2e", {}):
            secondary["ghpair_e2e"]["vs_e2e_host_encrypt"] = round(
                secondary["ghpair_e2e"]["encrypts_per_s"] / secondary["e2e_host_encrypt_per_s"], 3)
        secondary["e2e_note"] = (f"{ne} ciphertexts, pageable numpy in/out ({ch.nbytes / 1e6:.0f} MB out), "
                                 "pinned staging + copy stream overlapped with compute")
        # the same with page-locked caller buffers (direct DMA)
        mp = torch.from_numpy(mh).pin_memory()
        cp = torch.empty((ne, 2 * pl.n_words), dtype=torch.int32).pin_memory()
        t0 = time.perf_counter()
        _lib.check(lib.fthe_encrypt_u64(pl._key, dev.ctx, ctypes.c_void_p(mp.data_ptr()), ne, None, 0, 3,
                                        ctypes.c_void_p(cp.data_ptr()), 0), "encrypt")
        dt = time.perf_counter() - t0
        secondary["e2e_host_encrypt_pinned_per_s"] = round(ne / dt)
        secondary["e2e_pinned_same_ciphertexts"] = bool(np.array_equal(cp.numpy().view(np.uint32), ch))
        del mp, cp
        t0 = time.perf_counter()
        lo = pl.decrypt_u64(ch)
        dt = time.perf_counter() - t0
        secondary["e2e_host_decrypt_per_s"] = round(ne / dt)
        secondary["e2e_decrypt_ok"] = bool(np.array_equal(lo, mh))
        nh = ne // 2
        t0 = time.perf_counter()
        pl.add_batch(ch[:nh], ch[nh:2 * nh])
        dt = time.perf_counter() - t0
        secondary["e2e_host_add_per_s"] = round(nh / dt)
        # wire formats (host): the reference's decimal GHEncBatch strings vs the binary FTHW frame
        from fedtree_amd.paillier import ct_from_decimal, ct_to_decimal, wire_decode, wire_encode
        nw_ = min(ne, 1 << 16)
        sample = ch[:nw_]
        t0 = time.perf_counter()
        strs = ct_to_decimal(sample, threads=a.cpu_threads)
        t_enc = time.perf_counter() - t0
        t0 = time.perf_counter()
        back = ct_from_decimal(strs, sample.shape[1], threads=a.cpu_threads)
        t_dec = time.perf_counter() - t0
        t0 = time.perf_counter()
        fr = wire_encode(sample)
        g_, _ = wire_decode(fr, sample.shape[1])
        t_bin = time.perf_counter() - t0
        secondary["wire"] = {"ciphertexts": nw_, "threads": a.cpu_threads,
                             "decimal_encode_per_s": round(nw_ / t_enc), "decimal_decode_per_s": round(nw_ / t_dec),
                             "decimal_bytes_per_ct": round(sum(len(x) for x in strs) / nw_, 1),
                             "binary_roundtrip_per_s": round(nw_ / t_bin), "binary_bytes_per_ct": sample.shape[1] * 4,
                             "roundtrip_ok": bool(np.array_equal(back, sample) and np.array_equal(g_, sample))}
        # the same decimal strings computed on the device (fthe_dec.hip), 1M device-resident ciphertexts
        from fedtree_amd.paillier import ct_from_decimal_dev, ct_to_decimal_dev
        nd_ = min(2 * P, 1 << 20)
        ct_to_decimal_dev(dev, c[:4096])
        dev.sync()
        dbuf, doffs = ct_to_decimal_dev(dev, c[:nd_])
        dev.sync()
        t_denc = lib.fthe_last_kernel_ms(dev.ctx) * 1e-3
        dback = ct_from_decimal_dev(dev, dbuf, doffs, c.shape[1])
        dev.sync()
        t_ddec = lib.fthe_last_kernel_ms(dev.ctx) * 1e-3
        t0 = time.perf_counter()                                   # device ciphertexts -> host strings
        hb_, ho_ = ct_to_decimal_dev(dev, c[:nd_])
        ho_ = ho_.cpu()
        hb_ = hb_[: int(ho_[-1])].cpu()
        t_e2e = time.perf_counter() - t0
        secondary["wire"].update({
            "decimal_dev_ciphertexts": nd_, "decimal_encode_dev_per_s": round(nd_ / t_denc),
            "decimal_decode_dev_per_s": round(nd_ / t_ddec),
            "decimal_dev_to_host_strings_per_s": round(nd_ / t_e2e),
            "decimal_dev_roundtrip_ok": bool(torch.equal(dback, c[:nd_])),
            "decimal_dev_matches_host": bool(ct_to_decimal(c[:256].cpu().numpy().view(np.uint32)) == [
                bytes(hb_[int(ho_[i]):int(ho_[i + 1])].numpy()).decode() for i in range(256)])})
        del ch, strs, back, fr, g_, dbuf, doffs, dback, hb_, ho_
    cpu = None
    if rank == 0 and not a.no_cpu:                # after the timed region and its barrier, at every N
        ca = argparse.Namespace(**vars(a))
        if world > 1:
            ca.cpu_scale = a.cpu_scale / 4             # N > 1: a quarter sample keeps the scaling runs short
        cpu = cpu_baseline(ca, pl, p1k_cpu, m, c, dev)
        cpu["n_gpus_of_run"] = world

    if rank == 0 and world > 1 and not a.no_secondary:
        # configs[4] through the class FedTree calls: Server::encrypt_gh_pairs / decrypt_gh_pairs on one
        # SyncArray<GHPair> of N x (pairs per device), Paillier_HIP sharding it over every device of the run in one
        # process (ShardPool: a worker thread, context and key replica per device, host rows in and out), in a
        # fresh child while the other ranks wait at the final barrier (their own buffers stay allocated)
        secondary["ghpair_e2e_node"] = node_e2e(a, world, [p["device"] for p in per_rank], rehearse)

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "encrypts/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic logistic gradients (splitmix64 seed 20261015+rank), fresh device-CSPRNG r per ciphertext",
            "config": {"workload": "Paillier-2048 encrypt of gradient pairs, device-resident, CRT (key holder)",
                       "pairs_per_gpu": P, "ciphertexts_per_gpu_per_step": 2 * P, "key_bits": KEY_BITS,
                       "parallelism": f"independent shards x{world}"},
            "roofline": roof, "cpu_baseline": cpu, "ciphertext_adds": adds, "secondary": secondary,
            "per_rank": per_rank, "rank_time_max_s": round(elapsed, 4),
            "rank_time_min_s": round(min(p["elapsed_s"] for p in per_rank), 4),
        }
        if rehearse:
            line["rehearsal"] = "FTHE_BENCH_REHEARSE=1: all ranks on cuda:0 over gloo; not a measurement"
        if cpu:
            line["speedup_vs_cpu_baseline"] = round(value / cpu["value"], 1)
        write_detail(line)
        print(compact_line(line), flush=True)
    if world > 1:
        dist.barrier(group=cpu_group)                  # the other ranks wait for rank 0's CPU stage (gloo: no GPU)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

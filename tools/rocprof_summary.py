"""Summarise rocprofv3 outputs into profiles/ text/json.

  python tools/rocprof_summary.py trace <results.db> <out.txt>
      per-kernel stats (calls, total, average) + montprog exponentiation launches
  python tools/rocprof_summary.py pmc <dir-with-counter_collection.csv>... <out.json>
      per-dispatch counter values of fthe_montprog_s74 aggregated per launch
"""
import csv
import glob
import json
import os
import sqlite3
import sys


def trace_csv(csvfile, out):
    """kernel_trace.csv of rocprofv3 --output-format csv: per-kernel stats plus the
    exponentiation launches (> 5 ms) of each montprog variant."""
    rows = list(csv.DictReader(open(csvfile)))
    per = {}
    for r in rows:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        per.setdefault(r["Kernel_Name"], []).append(d)
    lines = ["kernel,calls,total_ms,avg_ms"]
    for name, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        lines.append(f"{name[:90]},{len(v)},{sum(v) / 1e6:.3f},{sum(v) / len(v) / 1e6:.4f}")
    lines.append("")
    for name, v in sorted(per.items()):
        if name.startswith(("fthe_montprog", "fthe_padic", "fthe_nadic")):
            heavy = [d for d in v if d > 5e6]
            if heavy:
                lines.append(f"{name} exponentiation launches (>5 ms): n={len(heavy)} "
                             f"avg_ms={sum(heavy) / len(heavy) / 1e6:.3f} min_ms={min(heavy) / 1e6:.3f} "
                             f"max_ms={max(heavy) / 1e6:.3f}")
                top = [d for d in heavy if d >= 0.9 * max(heavy)]   # the dominant (encrypt) launch type
                lines.append(f"{name} launches within 10% of the longest (encrypt programs): n={len(top)} "
                             f"avg_ms={sum(top) / len(top) / 1e6:.3f}")
    # launches of one kernel that overlap (the p and q halves of a large CRT call on two streams): the union of
    # their intervals over the launches is the effective time per launch, the figure bench.py's
    # roofline.avg_expo_launch_ms reports (its _in_flight twin is the per-dispatch average above)
    spans = {}
    for r in rows:
        spans.setdefault(r["Kernel_Name"], []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    for name, v in sorted(spans.items()):
        if not name.startswith(("fthe_padic", "fthe_nadic")):
            continue
        v.sort()
        u, a, b = 0, None, None
        for s0, s1 in v:
            if b is None or s0 > b:
                if b is not None:
                    u += b - a
                a, b = s0, s1
            else:
                b = max(b, s1)
        u += b - a
        lines.append(f"{name} union of launch intervals: {u / 1e6:.3f} ms over n={len(v)} launches = "
                     f"{u / len(v) / 1e6:.3f} ms effective per launch (overlap {sum(e - s for s, e in v) / u:.3f})")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[-5:]))


def trace(db, out):
    cur = sqlite3.connect(db).cursor()
    lines = ["kernel,calls,total_ms,avg_ms,pct"]
    for name, calls, tot, avg, pct in cur.execute("select * from top_kernels"):
        lines.append(f"{name[:90]},{calls},{tot / 1e6:.3f},{avg / 1e6:.4f},{pct:.3f}")
    durs = [d for (d,) in cur.execute("select duration from kernels where name like 'fthe_montprog%'")]
    heavy = [d for d in durs if d > 10e6]        # exponentiation launches (> 10 ms)
    lines.append("")
    lines.append(f"fthe_montprog exponentiation launches (>10 ms): n={len(heavy)} "
                 f"avg_ms={sum(heavy) / max(1, len(heavy)) / 1e6:.3f} "
                 f"min_ms={min(heavy) / 1e6 if heavy else 0:.3f} max_ms={max(heavy) / 1e6 if heavy else 0:.3f}")
    row = cur.execute("select vgpr_count, accum_vgpr_count, sgpr_count, lds_size, grid_x, workgroup_x "
                      "from kernels where name like 'fthe_montprog%' limit 1").fetchone()
    if row:
        lines.append(f"fthe_montprog resources: vgpr={row[0]} agpr={row[1]} sgpr={row[2]} lds={row[3]} "
                     f"grid_x={row[4]} wg={row[5]}")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[-3:]))


def pmc(dirs, out):
    """Per montprog variant: counters of its exponentiation dispatches (those whose
    value is >= 25% of the variant's largest, i.e. not the 1-product launches)."""
    agg = {}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                kn = r.get("Kernel_Name", "")
                if not kn.startswith(("fthe_montprog", "fthe_padic", "fthe_nadic", "fthe_addb")):
                    continue
                key = (kn, r["Dispatch_Id"], r["Counter_Name"])
                agg[key] = agg.get(key, 0.0) + float(r["Counter_Value"])
    per = {}
    for (kn, disp, name), v in agg.items():
        per.setdefault(kn, {}).setdefault(name, []).append(v)
    res = {}
    for kn, counters in per.items():
        rk = {}
        for name, v in counters.items():
            v = sorted(v, reverse=True)
            heavy = [x for x in v if x >= 0.25 * v[0]] if v[0] > 0 else v
            rk[name] = {"dispatches": len(v), "expo_dispatches": len(heavy),
                        "expo_mean": sum(heavy) / len(heavy), "all_mean": sum(v) / len(v)}
        if "FETCH_SIZE" in rk and "WRITE_SIZE" in rk:
            # FETCH_SIZE/WRITE_SIZE are KB; gfx950 FETCH_SIZE reads 1/2 of a coalesced
            # stream (MI355X_MICROARCH.md HBM): calibrated on this kernel in round 1 --
            # the 329 x 296-B slot loads per lane per launch it issues = 2.05 x FETCH_SIZE.
            f, w = rk["FETCH_SIZE"]["expo_mean"], rk["WRITE_SIZE"]["expo_mean"]
            rk["hbm_bytes_per_launch"] = (2 * f + w) * 1024
            rk["hbm_bytes_formula"] = "(2*FETCH_SIZE + WRITE_SIZE) * 1024, exponentiation launches"
        res[kn] = rk
    dom = "fthe_montprog_s74"
    if dom in res and "hbm_bytes_per_launch" in res[dom]:
        res["hbm_bytes_per_launch"] = res[dom]["hbm_bytes_per_launch"]
        res["dominant_kernel"] = dom
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))




def pmc_round(tag, out):
    """Summary of tools/pmc_round.sh TAG: per workload (enc, add, kway, pub) and montprog
    kernel, the mean counters of its dominant dispatches (>= 90% of the largest value: the
    full-chunk launches), HBM bytes per launch = 2*FETCH_SIZE + WRITE_SIZE
    (KiB; gfx950 FETCH_SIZE counts half of a 16-B/lane streaming read,
    MI355X_MICROARCH.md HBM section) and the launch duration from the ops kernel
    trace (add, kway) or the bench trace (enc) for the achieved GB/s."""
    res = {}
    for w in ("enc", "add", "addsame", "kway", "pub"):
        per = {}
        for t in ("fetch", "write", "vb", "occ", "sq", "mf", "lds"):
            for f in glob.glob(f"gpurun_out/{tag}_pmc_{w}_{t}/**/*counter_collection.csv", recursive=True):
                acc = {}
                for r in csv.DictReader(open(f)):
                    kn = r["Kernel_Name"]
                    if not kn.startswith(("fthe_montprog", "fthe_padic", "fthe_nadic", "fthe_addb")):
                        continue
                    key = (kn, r["Dispatch_Id"], r["Counter_Name"])
                    acc[key] = acc.get(key, 0.0) + float(r["Counter_Value"])
                for (kn, _, cn), v in acc.items():
                    per.setdefault(kn, {}).setdefault(cn, []).append(v)
        wr = {}
        for kn, cs in per.items():
            d = {}
            for cn, v in cs.items():
                top = max(v)
                heavy = [x for x in v if x >= 0.9 * top] if top > 0 else v     # full-size launches
                d[cn] = round(sum(heavy) / len(heavy), 3)
            if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
                d["hbm_bytes_per_launch"] = (2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024
            wr[kn] = d
        res[w] = wr
    # launch durations from the ops trace (tools/prof_ops.py --ops add,kway): fthe_addb_q152 = one add launch
    # over all rows, then the merge's launches (kk - 1 per merge, each over all rows); the s152 row-I/O
    # kernel (FTHE_ADD_NO_ADDB) = add launches first, then as many kway launches, full launches within 10%
    tr = glob.glob(f"gpurun_out/{tag}_ops_trace/*kernel_trace.csv")
    if tr:
        recs = [(r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
                for r in csv.DictReader(open(tr[0]))]
        full = lambda ds: [d for d in ds if d >= 0.9 * max(ds)] if ds else []
        ab = [d for kn, d in recs if kn == "fthe_addb_q152"]
        if ab:
            kern, add, kway = "fthe_addb_q152", ab[:1], ab[1:]
            rows = int(os.environ.get("FTHE_OPS_ROWS", "1048576"))
            ins_of = {"add": 3, "kway": 3}         # every launch: two rows in, one out per row
        else:
            durs = [d for kn, d in recs if kn == "fthe_montprog_s152"]
            h = len(durs) // 2
            kern, add, kway = "fthe_montprog_s152", full(durs[:h]), full(durs[h:])
            rows = int(os.environ.get("FTHE_ROWIO_ROWS", "393216"))    # rows per full row-I/O launch
            ins_of = {"add": 3, "kway": 9}         # add: x, y, out; kway: 8 in, 1 out
        for w, ds in (("add", add), ("kway", kway)):
            if ds and kern in res[w]:
                k = res[w][kern]
                ms = sum(ds) / len(ds)
                k["launch_ms"] = round(ms, 4)
                k["launches_timed"] = len(ds)
                k["rows_out_per_launch"] = rows
                if "hbm_bytes_per_launch" in k:
                    k["hbm_GBps"] = round(k["hbm_bytes_per_launch"] / (ms * 1e-3) / 1e9, 1)
                    k["hbm_frac_of_8TBps"] = round(k["hbm_bytes_per_launch"] / (ms * 1e-3) / 8e12, 4)
                k["algorithmic_bytes_per_launch"] = rows * 512 * ins_of[w]
        # counter calibration on this kernel's own access pattern (tools/prof_ops.py addsame: x = y, so the
        # launch must read each of its `rows` rows once -- rows * 512 B -- and write as many): bytes per
        # counted byte of FETCH_SIZE and of WRITE_SIZE, applied to the distinct-row launch
        same = res.get("addsame", {}).get(kern, {})
        k = res["add"].get(kern, {})
        if same.get("FETCH_SIZE") and same.get("WRITE_SIZE") and k.get("FETCH_SIZE") and k.get("launch_ms"):
            ff = rows * 512 / (same["FETCH_SIZE"] * 1024)
            fw = rows * 512 / (same["WRITE_SIZE"] * 1024)
            cb = (ff * k["FETCH_SIZE"] + fw * k["WRITE_SIZE"]) * 1024
            k["calibration"] = {"source": "addsame (x = y): rows * 512 B read once and written once",
                                "bytes_per_fetch_byte": round(ff, 3), "bytes_per_write_byte": round(fw, 3),
                                "hbm_bytes_per_launch": round(cb),
                                "hbm_GBps": round(cb / (k["launch_ms"] * 1e-3) / 1e9, 1),
                                "vs_algorithmic": round(cb / k["algorithmic_bytes_per_launch"], 3)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "pmcround":
        pmc_round(sys.argv[2], sys.argv[3])
    elif sys.argv[1] == "trace":
        (trace_csv if sys.argv[2].endswith(".csv") else trace)(sys.argv[2], sys.argv[3])
    else:
        pmc(sys.argv[2:-1], sys.argv[-1])

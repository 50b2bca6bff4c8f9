"""Turns one GPU session's rocprofv3 output (gpurun_out/) into the committed evidence under profiles/.

Usage: python tools/summarize_profile.py TAG [ROWS]
  reads  gpurun_out/prof_TAG/run_kernel_stats.csv          (--kernel-trace --stats pass)
         gpurun_out/pmc_fetch_TAG/run_counter_collection.csv (--pmc FETCH_SIZE pass)
         gpurun_out/pmc_write_TAG/run_counter_collection.csv (--pmc WRITE_SIZE pass)
         gpurun_out/bench_TAG.json                           (the bench line of the same session)
  writes profiles/TAG/kernel_stats.csv, profiles/TAG/dq_counters.csv (dq:: kernels only),
         profiles/TAG/summary.json, and profiles/traffic_s10.json (read by bench.py).

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are in KiB-units of 1024 B
and, on gfx950, FETCH_SIZE reports half the bytes of a wide coalesced streaming read, so it is
doubled; WRITE_SIZE is taken as is.  Values are per dispatch (averaged over the dispatches).
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _name(kernel: str) -> str:
    """'void dq::scan_mixed_kernel<200u>(...)' -> 'dq::scan_mixed_kernel<200u>'"""
    k = kernel.split("(")[0]
    return k[5:] if k.startswith("void ") else k


def per_kernel(path, counter):
    out = {}
    if not os.path.exists(path):
        return out, []
    rows = list(csv.DictReader(open(path)))
    keep = [r for r in rows if _name(r["Kernel_Name"]).startswith("dq::")]
    for r in keep:
        if r["Counter_Name"] != counter:
            continue
        name = _name(r["Kernel_Name"])
        out.setdefault(name, []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in out.items()}, keep


def main():
    tag = sys.argv[1]
    rows = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000_000
    src = os.path.join(ROOT, "gpurun_out")
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    stats_path = os.path.join(src, f"prof_{tag}", "run_kernel_stats.csv")
    shutil.copy(stats_path, os.path.join(dst, "kernel_stats.csv"))
    stats = {}
    for r in csv.DictReader(open(stats_path)):
        if _name(r["Name"]).startswith("dq::"):
            stats[_name(r["Name"])] = {"calls": int(r["Calls"]),
                                              "avg_ns": float(r["AverageNs"]),
                                              "min_ns": float(r["MinNs"]),
                                              "max_ns": float(r["MaxNs"])}
    fetch, kf = per_kernel(os.path.join(src, f"pmc_fetch_{tag}", "run_counter_collection.csv"),
                           "FETCH_SIZE")
    write, kw = per_kernel(os.path.join(src, f"pmc_write_{tag}", "run_counter_collection.csv"),
                           "WRITE_SIZE")
    if kf or kw:
        with open(os.path.join(dst, "dq_counters.csv"), "w", newline="") as fh:
            w = csv.DictWriter(fh, fieldnames=list((kf or kw)[0].keys()))
            w.writeheader()
            for r in kf + kw:
                w.writerow(r)
    bench = None
    bpath = os.path.join(src, f"bench_{tag}.json")
    if os.path.exists(bpath):
        lines = [ln for ln in open(bpath) if ln.startswith("{")]
        bench = json.loads(lines[-1]) if lines else None
    dominant = max(stats, key=lambda k: stats[k]["avg_ns"]) if stats else None
    b_alg = bench["roofline"]["algorithmic_bytes_per_launch"] if bench else None
    kernels = {}
    for k, v in stats.items():
        hbm = None
        if k in fetch:
            hbm = 2 * fetch[k] * 1024 + write.get(k, 0.0) * 1024
        kernels[k] = dict(v, fetch_kib_raw=fetch.get(k), write_kib_raw=write.get(k),
                          hbm_bytes_per_dispatch=hbm)
    summary = {"tag": tag, "rows_per_gpu": rows, "dominant_kernel": dominant, "kernels": kernels,
               "algorithmic_bytes_per_launch": b_alg, "bench": bench}
    if dominant and b_alg:
        d = kernels[dominant]
        summary["rocprof_achieved_gbps"] = b_alg / d["avg_ns"]
        if d["hbm_bytes_per_dispatch"]:
            summary["traffic_over_algorithmic"] = d["hbm_bytes_per_dispatch"] / b_alg
    json.dump(summary, open(os.path.join(dst, "summary.json"), "w"), indent=1)
    if dominant and kernels[dominant]["hbm_bytes_per_dispatch"]:
        # the code object the profiled bench ran (its own line), else this tree's build
        sha = (bench or {}).get("roofline", {}).get("scan_code_object_sha")
        if not sha:
            sys.path.insert(0, ROOT)
            from bench import scan_code_object_hash
            sha = scan_code_object_hash()
        json.dump({"tag": tag, "rows_per_gpu": rows, "kernel": dominant,
                   "scan_code_object_sha": sha,
                   "hbm_bytes_per_launch": kernels[dominant]["hbm_bytes_per_dispatch"],
                   "source": f"profiles/{tag}/dq_counters.csv (2 x FETCH_SIZE + WRITE_SIZE, KiB)"},
                  open(os.path.join(ROOT, "profiles", "traffic_s10.json"), "w"), indent=1)
    print(json.dumps({k: v for k, v in summary.items() if k != "bench"}, indent=1))


if __name__ == "__main__":
    main()

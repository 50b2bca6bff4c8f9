"""Per-kernel summary of the configs[2] / [4] PMC passes (tools/gpu_pmc_c3.sh at 1e8 rows,
tools/gpu_pmc_c5.sh; one step each), with the step's totals over every kernel but the generators.

Usage: python tools/summarize_c3_pmc.py TAG [WORKLOAD]   (WORKLOAD c3 (default) or c5)
  reads  gpurun_out/{pmcf,pmcw,pmc,pmc2}_WORKLOAD_TAG/*_counter_collection.csv
  writes profiles/TAG/WORKLOAD_counters.json: per dq:: kernel, the summed counters over its dispatches,
         HBM bytes (FETCH_SIZE KiB x 1024, reported raw and x2 per MI355X_MICROARCH.md §HBM --
         the halving is calibrated only for 16-B-per-lane streaming reads; these kernels read
         8-B records, so both are given), WRITE_SIZE bytes, and the SQ wave-state fractions.
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag = sys.argv[1]
    wl = sys.argv[2] if len(sys.argv) > 2 else "c3"
    src = os.path.join(ROOT, "gpurun_out")
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for pas in ("pmcf", "pmcw", "pmc", "pmc2"):
        for path in glob.glob(os.path.join(src, f"{pas}_{wl}_{tag}", "*_counter_collection.csv")):
            for r in csv.DictReader(open(path)):
                name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
                # every kernel of the step but the synthetic table's generation, which runs once
                # before the step in the same process: its HIP generators and the torch kernels
                # around them (at::native, and torch's bundled rocPRIM 4.0.1 for cumsum; the
                # engine's own rocPRIM is 4.2)
                if ("gen_" in name.split("(")[0] or "dq_synth" in name or "at::native" in name
                        or "ROCPRIM_400001" in name):
                    continue
                k = name.split("(")[0].replace("void ", "")
                acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add((pas, r["Dispatch_Id"]))
    out = {}
    for k, c in acc.items():
        d = {name: v for name, v in c.items()}
        if "FETCH_SIZE" in c:
            d["fetch_bytes_raw"] = c["FETCH_SIZE"] * 1024
            d["fetch_bytes_x2"] = 2 * c["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in c:
            d["write_bytes"] = c["WRITE_SIZE"] * 1024
        if c.get("SQ_WAVE_CYCLES"):
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if n in c:
                    d[n + "_frac"] = c[n] / c["SQ_WAVE_CYCLES"]
        out[k] = d
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    what = {"c3": "c3 --rows 100000000 --steps 1 --warmup 0", "c5": "c5 --steps 1 --warmup 0"}[wl]
    tot_f = sum(d.get("fetch_bytes_raw", 0.0) for d in out.values())
    tot_w = sum(d.get("write_bytes", 0.0) for d in out.values())
    totals = {"fetch_bytes_raw": tot_f, "write_bytes": tot_w,
              "fetch_x2_plus_write": 2 * tot_f + tot_w}
    print("totals (GB):", {k: round(v / 1e9, 2) for k, v in totals.items()})
    json.dump({"tag": tag, "workload": what, "totals": totals, "kernels": out},
              open(os.path.join(dst, f"{wl}_counters.json"), "w"), indent=1)
    for k in sorted(out, key=lambda k: -out[k].get("fetch_bytes_raw", 0)):
        d = out[k]
        print(k[:48].ljust(48), {x: round(d[x] / 1e9, 3) for x in ("fetch_bytes_raw", "write_bytes")
                                 if x in d},
              {x: round(d[x], 2) for x in d if x.endswith("_frac")})


if __name__ == "__main__":
    main()

"""Summarise rocprofv3 counter_collection CSVs for the bench's full-size launches.

For each kernel, keeps only the dispatches with the largest grid (the bench's
timed launches; the small check launch is dropped) and reports the mean of
each counter per dispatch, plus VGPR/SGPR/LDS of the code object and the
corrected HBM bytes (FETCH_SIZE is in KiB and counts a 128-B read as 64 B on
gfx950 -> x2; WRITE_SIZE in KiB, exact for wide stores; MI355X_MICROARCH.md
'HBM / rocprofv3').  Writes summary.json beside the CSVs.
usage: python scripts/pmc_summary.py DIR [key=value ...]
The key=value pairs (workload=c3 replicas=10000 variant=12 command=...) and the
engine build stamp (redqueen_amd._lib.build_stamp: librq.so + sources sha256) go
into summary.json's "_meta"; bench.py uses a summary only when the stamp matches
the library it has loaded.
"""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
rows = collections.defaultdict(list)
for f in glob.glob(root + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows[r["Kernel_Name"].split("(")[0].replace("void ", "")].append(r)
out = {}
for k, rs in rows.items():
    gmax = max(int(r["Grid_Size"]) for r in rs)
    big = [r for r in rs if int(r["Grid_Size"]) == gmax]
    agg = collections.defaultdict(list)
    for r in big:
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    d = {c: sum(v) / len(v) for c, v in agg.items()}
    r0 = big[0]
    info = {"grid": gmax, "wg": int(r0["Workgroup_Size"]), "vgpr": int(r0.get("VGPR_Count", 0) or 0),
            "agpr": int(r0.get("Accum_VGPR_Count", 0) or 0), "sgpr": int(r0.get("SGPR_Count", 0) or 0),
            "lds": int(r0.get("LDS_Block_Size", 0) or 0), "counters": d}
    if "FETCH_SIZE" in d:
        info["hbm_read_bytes"] = d["FETCH_SIZE"] * 1024 * 2
    if "TCC_EA0_RDREQ_sum" in d and "TCC_EA0_RDREQ_64B_sum" in d:
        # read bytes by request size (exact for any access width; FETCH_SIZE x2 is exact
        # only for whole-line reads: profiles/r04_calib_half.txt)
        n32 = d.get("TCC_EA0_RDREQ_32B_sum", 0.0)
        n64 = d.get("TCC_EA0_RDREQ_64B_sum", 0.0)
        n128 = d.get("TCC_EA0_RDREQ_128B_sum", 0.0)
        info["hbm_read_bytes_by_req"] = 32 * n32 + 64 * n64 + 128 * n128
        info["rdreq"] = {"all": d["TCC_EA0_RDREQ_sum"], "32B": n32, "64B": n64, "128B": n128}
    if "WRITE_SIZE" in d:
        info["hbm_write_bytes"] = d["WRITE_SIZE"] * 1024
    if "SQ_WAVE_CYCLES" in d and d["SQ_WAVE_CYCLES"] > 0:
        wc = d["SQ_WAVE_CYCLES"]
        info["frac_active_inst"] = d.get("SQ_ACTIVE_INST_ANY", 0) / wc
        info["frac_wait_any"] = d.get("SQ_WAIT_ANY", 0) / wc
        info["frac_wait_inst"] = d.get("SQ_WAIT_INST_ANY", 0) / wc
        # wave-slot occupancy of the launch: mean wave lifetime over the launch's duration
        # (SQ_WAVE_CYCLES in units of 4 cycles; GRBM_GUI_ACTIVE summed over the 8 XCDs)
        if d.get("SQ_WAVES", 0) > 0 and d.get("GRBM_GUI_ACTIVE", 0) > 0:
            info["wave_slot_occupancy"] = wc * 4.0 / (d["SQ_WAVES"] * d["GRBM_GUI_ACTIVE"] / 8.0)
    out[k] = info
# per-kernel average duration with every kernel serialised (AMD_SERIALIZE_KERNEL=3 kernel
# trace, scripts/gpu_pmc.sh "kts" pass): the launch alone on the chip, the time a
# serialised roofline figure divides by
for f in glob.glob(root + "/kts/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Name"].split("(")[0].replace("void ", "")
        if k in out:
            out[k]["serial_avg_ns"] = float(r["AverageNs"])
            out[k]["serial_min_ns"] = float(r["MinNs"])
meta = {}
for kv in sys.argv[2:]:
    k, v = kv.split("=", 1)
    meta[k] = int(v) if v.isdigit() else v
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
try:
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "rqlib", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                              "redqueen_amd", "_lib.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    meta.update(mod.build_stamp())
except Exception as e:  # noqa: BLE001 -- a summary without a stamp is never used by bench.py
    meta["stamp_error"] = str(e)
meta["correction"] = ("hbm_read_bytes = FETCH_SIZE KiB x1024 x2 (gfx950: 128-B reads tallied at "
                      "64 B; calibrated for 4/8/16 B per lane by scripts/micro/fetch_calib.hip); "
                      "hbm_write_bytes = WRITE_SIZE KiB x1024")
out["_meta"] = meta
json.dump(out, open(os.path.join(root, "summary.json"), "w"), indent=1)
print("_meta", json.dumps(meta))
for k, v in out.items():
    if k.startswith("rq_"):
        print(k, json.dumps({a: b for a, b in v.items() if a != "counters"}))
        for c, x in sorted(v["counters"].items()):
            print("   %-22s %.6g" % (c, x))

#!/usr/bin/env python3
"""Summarize a tools/profile.sh run into profiles/ (committed evidence).

    python tools/pmc_summary.py gpurun_out/prof_r01 r01 [--config 20:3 --groups 1048576]

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats), profiles/<tag>_pmc.json
(per-kernel counter averages + derived HBM bytes) and updates profiles/pmc_traffic.json, which bench.py
reads for the roofline "traffic" field.  HBM bytes follow MI355X_MICROARCH.md "HBM": FETCH_SIZE and
WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reads exactly half the bytes of a wide (16 B/lane) coalesced
stream, so it is doubled; WRITE_SIZE is exact for 16-B streaming stores.
"""
import argparse, collections, csv, glob, json, os, re, shutil

ap = argparse.ArgumentParser()
ap.add_argument("prof_dir"); ap.add_argument("tag")
ap.add_argument("--config", default="20:3"); ap.add_argument("--groups", type=int, default=1 << 20)
ap.add_argument("--pitch", type=int, default=0, help="shard pitch of a padded-layout run (key <config>@p<pitch>)")
args = ap.parse_args()
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = os.path.join(root, "profiles"); os.makedirs(out, exist_ok=True)
shutil.copy(os.path.join(args.prof_dir, "kt", "kt_kernel_stats.csv"), os.path.join(out, f"{args.tag}_kernel_stats.csv"))

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(args.prof_dir, "pmc_*", "pmc_counter_collection.csv")):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        agg[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
        agg[k]["duration_ns"].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
summary = {}
for k, v in agg.items():
    if "kfec" not in k:
        continue
    d = {c: sum(x) / len(x) for c, x in v.items()}
    if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
        d["hbm_read_bytes_corrected"] = d["FETCH_SIZE"] * 1024 * 2
        d["hbm_write_bytes"] = d["WRITE_SIZE"] * 1024
        d["hbm_bytes_per_launch"] = d["hbm_read_bytes_corrected"] + d["hbm_write_bytes"]
    if "GRBM_GUI_ACTIVE" in d and d.get("duration_ns"):
        d["effective_clock_GHz"] = d["GRBM_GUI_ACTIVE"] / 8 / d["duration_ns"]
    if "SQ_INSTS_VALU" in d and "GRBM_GUI_ACTIVE" in d:
        # wave64 VALU = 2 cycles on a SIMD32; 1024 SIMDs; GRBM_GUI_ACTIVE summed over 8 XCDs
        d["valu_utilization"] = d["SQ_INSTS_VALU"] * 2 / (1024 * d["GRBM_GUI_ACTIVE"] / 8)
    summary[k] = d
json.dump(summary, open(os.path.join(out, f"{args.tag}_pmc.json"), "w"), indent=1)
trf_path = os.path.join(out, "pmc_traffic.json")
trf = json.load(open(trf_path)) if os.path.exists(trf_path) else {}
# the bench line's dominant kernel: the encode MAC, or for decode-only configs the syndrome-form decode MAC
dominant = re.compile(r"syn_kernel<\d+, \d+(, \d+)?>" if args.config.endswith("dec")
                      else r"mac_kernel<\d+, \d+, false(, \d+)?>")
for k, d in summary.items():
    # (the product's kernel, not the arithmetic-free ceiling build's namesake, kfec_af::, timed in the same run)
    if dominant.search(k) and "kfec_af::" not in k and "hbm_bytes_per_launch" in d:
        key = f"{args.config}@p{args.pitch}" if args.pitch else args.config
        trf[key] = {"groups": args.groups, "kernel": k, "hbm_bytes_per_launch": int(d["hbm_bytes_per_launch"]),
                    "source": f"profiles/{args.tag}_pmc.json"}
        if args.pitch:
            trf[key]["pitch"] = args.pitch
json.dump(trf, open(trf_path, "w"), indent=1)
for k, d in summary.items():
    print(k[:60], {c: round(x, 4) if isinstance(x, float) else x for c, x in d.items()
                   if c in ("duration_ns", "hbm_bytes_per_launch", "valu_utilization", "effective_clock_GHz")})

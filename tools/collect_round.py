#!/usr/bin/env python3
"""Copy the judged summaries of a tools/gpu_round.sh run into profiles/ (tracked): bench lines, wire and seal
benches, rocprofv3 kernel stats and PMC summaries (tools/pmc_summary.py), FETCH/WRITE calibration.

    python tools/collect_round.py r01
"""
import csv, collections, glob, json, os, shutil, subprocess, sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
go = os.path.join(root, "gpurun_out")
prof = os.path.join(root, "profiles")
rnd = os.path.join(go, "round")
for name in ("bench_203.json", "bench_103dec.json", "bench_20055.json", "bench_203loss1.json", "wire.json",
             "wire_ragged.json", "seal.json", "pipeline_threads.json", "latency.json", "gtest.log", "smoke.log",
             "box.txt", "e2e.json"):
    src = os.path.join(rnd, name)
    if os.path.exists(src):
        # (the round pass's latency line goes beside the curated <tag>_latency.json, never over it)
        dst = name.replace('.log', '.txt').replace("latency.json", "latency_roundpass.json")
        shutil.copy(src, os.path.join(prof, f"{tag}_{dst}"))
for cfg, groups, ptag in (("20:3", 1 << 20, "203"), ("10:3dec", 1 << 20, "103dec"), ("200:55", 1 << 18, "20055"),
                          ("20:3loss1", 1 << 20, "203loss1")):
    d = os.path.join(go, f"prof_{tag}_{ptag}")
    if os.path.isdir(d):
        subprocess.check_call([sys.executable, os.path.join(root, "tools", "pmc_summary.py"), d, f"{tag}_{ptag}",
                               "--config", cfg, "--groups", str(groups)])
        # the bench line the traced command printed (its HIP-event times, to set beside the trace's)
        kl = os.path.join(d, "kt.log")
        lines = [ln for ln in open(kl) if ln.startswith('{"metric"')] if os.path.exists(kl) else []
        if lines:
            open(os.path.join(prof, f"{tag}_bench_{ptag}_under_rocprof.json"), "w").write(lines[-1])
for name in ("wire", "seal"):
    f = os.path.join(go, f"prof_{name}", "kt_kernel_stats.csv")
    if os.path.exists(f):
        shutil.copy(f, os.path.join(prof, f"{tag}_{name}_kernel_stats.csv"))
cal = {}
for kind in ("fetch", "write"):
    for f in glob.glob(os.path.join(go, f"cal_{kind}", "**", "p_counter_collection.csv"), recursive=True):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
        cal[kind] = {k: round(sum(v) / len(v) * 1024 / 1e9, 3) for k, v in agg.items()}
if cal:
    json.dump({"unit": "GB per launch (FETCH_SIZE / WRITE_SIZE x 1024)", "note": "tools/ceiling.hip kernels with known "
               "byte counts: read_chunk reads 30.199 GB, write_chunk / copy_chunk write 4.530 GB", **cal},
              open(os.path.join(prof, f"{tag}_counter_calibration.json"), "w"), indent=1)
print("collected into", prof)

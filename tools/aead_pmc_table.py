#!/usr/bin/env python3
"""Per-kernel SQ counter summary of tools/gpu_aead_pmc.sh (averages over the kernel's dispatches).

    python tools/aead_pmc_table.py [gpurun_out/aead_pmc]
"""
import collections, csv, glob, os, re, sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/aead_pmc"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for pas in "AB":
    for f in glob.glob(os.path.join(d, pas, "*counter_collection.csv")):
        per = collections.defaultdict(dict)
        for r in csv.DictReader(open(f)):
            m = re.search(r"(gcm_kernel<\w+>|ocb_kernel<\w+>|aead16_kernel<\w+, \w+>|aead_kernel<\w+, \w+>)", r["Kernel_Name"])
            if not m:
                continue
            per[(m.group(1), r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
            per[(m.group(1), r["Dispatch_Id"])]["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        for (k, _), c in per.items():
            for kk, vv in c.items():
                agg[k][pas + ":" + kk].append(vv)
for k, c in sorted(agg.items()):
    g = lambda x: sum(c[x]) / len(c[x]) if c.get(x) else float("nan")
    wc = g("B:SQ_WAVE_CYCLES")
    print(f"{k:28s} ns={g('A:ns'):9.0f} VALU={g('A:SQ_INSTS_VALU')/1e6:7.1f}M LDSi={g('A:SQ_INSTS_LDS')/1e6:6.1f}M "
          f"ldsact={g('A:SQ_LDS_IDX_ACTIVE')/1e6:7.1f}M conf={g('A:SQ_LDS_BANK_CONFLICT')/1e6:6.1f}M "
          f"wait={g('B:SQ_WAIT_ANY')/wc:.2f} stall={g('B:SQ_WAIT_INST_ANY')/wc:.2f} act={g('B:SQ_ACTIVE_INST_ANY')/wc:.2f} "
          f"valu={g('B:SQ_ACTIVE_INST_VALU')/wc:.2f} lds={g('B:SQ_ACTIVE_INST_LDS')/wc:.2f} waves={g('B:SQ_WAVES'):.0f}")

#!/usr/bin/env python3
"""Print the seal/open kernels' SQ counters from tools/gpu_seal_pmc.sh (one line per kernel and variant).

    python tools/seal_pmc_table.py [gpurun_out/seal_pmc]
"""
import collections, csv, glob, os, sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/seal_pmc"
for vdir in sorted(glob.glob(os.path.join(d, "*_A"))):
    v = os.path.basename(vdir)[:-2]
    rows = collections.defaultdict(dict)
    for pas in "AB":
        for f in glob.glob(os.path.join(d, f"{v}_{pas}", "*counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                if not any(x in k for x in ("seal_kernel", "open_kernel", "seal_in_place")):
                    continue
                name = next(x for x in ("seal_in_place_kernel", "seal_kernel", "open_kernel") if x in k)
                rows[(pas, r["Dispatch_Id"])]["kernel"] = name
                rows[(pas, r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
                rows[(pas, r["Dispatch_Id"])]["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    # average per kernel name per pass (the bench runs each kernel 3x: none / plain_xor / in place orders)
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    order = collections.defaultdict(int)
    for (pas, did), c in sorted(rows.items(), key=lambda x: (x[0][0], int(x[0][1]))):
        name = c["kernel"] + "#" + str(order[(pas, c["kernel"])] % (4 if "place" in c["kernel"] else 2))
        order[(pas, c["kernel"])] += 1
        for kk, vv in c.items():
            if kk != "kernel":
                agg[name][pas + ":" + kk].append(vv)
    for name, c in sorted(agg.items()):
        g = lambda k: sum(c[k]) / len(c[k]) if c.get(k) else float("nan")
        wc = g("B:SQ_WAVE_CYCLES")
        print(f"{v:12s} {name:24s} ns={g('A:ns'):9.0f} VALU={g('A:SQ_INSTS_VALU')/1e6:6.1f}M LDSi={g('A:SQ_INSTS_LDS')/1e6:5.1f}M "
              f"ldsact={g('A:SQ_LDS_IDX_ACTIVE')/1e6:6.1f}M conf={g('A:SQ_LDS_BANK_CONFLICT')/1e6:6.1f}M "
              f"wait={g('B:SQ_WAIT_ANY')/wc:.2f} stall={g('B:SQ_WAIT_INST_ANY')/wc:.2f} act={g('B:SQ_ACTIVE_INST_ANY')/wc:.2f} "
              f"valu={g('B:SQ_ACTIVE_INST_VALU')/wc:.2f} lds={g('B:SQ_ACTIVE_INST_LDS')/wc:.2f} vmem={g('B:SQ_ACTIVE_INST_VMEM')/wc:.2f} "
              f"waves={g('B:SQ_WAVES'):.0f}")

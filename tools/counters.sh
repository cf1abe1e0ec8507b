#!/bin/bash
# tools/counters.sh <tag> <prof_enc args...> : one rocprofv3 --pmc pass per counter group
set -o pipefail
tag=$1; shift
out=gpurun_out/cnt_${tag}; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
i=0
for pmc in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "TCC_EA0_RDREQ_DRAM_sum" "TCC_TAG_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum" "TCC_REQ_sum TCC_READ_sum" "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum" "TCP_TCC_READ_REQ_sum" "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $pmc --output-format csv -d $out/p$i -o p -- python3 tools/prof_enc.py "$@" > $out/p$i.log 2>&1 || echo "pass $i failed: $pmc"
done
python3 - "$out" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/p_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "kfec" in r["Kernel_Name"]:
            agg[r["Kernel_Name"][:45]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    print(k, {c: round(sum(x) / len(x)) for c, x in v.items()})
PY

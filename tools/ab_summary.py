#!/usr/bin/env python3
"""Min / median encode and decode ms per library over an ab.py output file: tools/ab_summary.py file..."""
import collections, json, statistics, sys
for path in sys.argv[1:]:
    d = collections.defaultdict(lambda: ([], []))
    for line in open(path):
        name, _, js = line.partition(" ")
        if not js.startswith("{"):
            continue
        j = json.loads(js)
        d[name][0].append(j["enc_ms"]); d[name][1].append(j["dec_ms"])
    print(path)
    for k, (e, dd) in d.items():
        print(f"  {k:22s} enc min {min(e):.3f} med {statistics.median(e):.3f}   dec min {min(dd):.3f} med {statistics.median(dd):.3f}  (n={len(e)})")
